set -e
S="python scripts/sweep.py --kernels wave --tiles rows --rounds 3 --reps 5"
for v in default noshadow rootonly; do
  if [ $v = default ]; then L=""; else L="RT_MI355X_LIB=build/variants/$v/librt_mi355x.so"; fi
  echo "== $v c3"; env $L timeout -k 10 120 $S --config c3
  echo "== $v c5"; env $L timeout -k 10 200 $S --config c5 --rounds 1 --reps 2
done
echo "== stats c3"; RT_MI355X_LIB=build/variants/stats/librt_mi355x.so timeout -k 10 120 python scripts/stats.py c3
echo "== stats c5"; RT_MI355X_LIB=build/variants/stats/librt_mi355x.so timeout -k 10 300 python scripts/stats.py c5
