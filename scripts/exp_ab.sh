# A/B of library variants: scripts/exp_ab.sh "<variants>" [configs]; variant "default" = the in-tree library
set -e
VARS=${1:-default}; CFGS=${2:-c3 c5}
for v in $VARS; do
  if [ $v = default ]; then L=""; else L="RT_MI355X_LIB=build/variants/$v/librt_mi355x.so"; fi
  for c in $CFGS; do
    if [ $c = c5 ]; then R="--rounds 1 --reps 3"; T=240; else R="--rounds 3 --reps 5"; T=120; fi
    echo "== $v $c"; env $L timeout -k 10 $T python scripts/sweep.py --kernels wave --tiles rows --config $c $R
  done
done
