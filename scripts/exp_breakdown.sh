# Where the c3/c5 frame time goes: the default build against timing-only builds that skip parts
# of the work (their frames are wrong by design), one process, interleaved rounds.
set -e
A="default=default noshade=build/variants/noshade/librt_mi355x.so noshadow=build/variants/noshadow/librt_mi355x.so rootonly=build/variants/rootonly/librt_mi355x.so"
echo "== c3"; timeout -k 10 200 python scripts/ab_libs.py --no-check --config c3 --rounds 7 --reps 5 $A
echo "== c5"; timeout -k 10 300 python scripts/ab_libs.py --no-check --config c5 --rounds 2 --reps 2 $A

