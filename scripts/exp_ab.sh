# Interleaved A/B of library variants in one process per config:
#   scripts/exp_ab.sh "<variant> ..." [configs] [tiles-per-block values]; "default" = the in-tree
#   library, other names = build/variants/<name>/librt_mi355x.so (scripts/build_variant.sh)
set -e
VARS=${1:-default}; CFGS=${2:-c3 c5}; TPBS=${3:-2}
ARGS=""
for v in $VARS; do
  if [ $v = default ]; then ARGS="$ARGS default=default"; else ARGS="$ARGS $v=build/variants/$v/librt_mi355x.so"; fi
done
for tpb in $TPBS; do
  for c in $CFGS; do
    if [ $c = c5 ]; then R="--rounds 3 --reps 2"; T=300; else R="--rounds 7 --reps 5"; T=150; fi
    echo "== $c tpb=$tpb"; RT_TILES_PER_BLOCK=$tpb timeout -k 10 $T python scripts/ab_libs.py --config $c $R $ARGS
  done
done
