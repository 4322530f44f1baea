#!/bin/bash
# The HW1 configuration's rocprofv3 passes (scripts/profile.sh) summarised on the GPU box itself
# (scripts/traffic.py), keeping only the summaries: the per-dispatch CSVs of a c2 run exceed what
# gpurun copies back.  usage: scripts/profile_hw1.sh <tag> <config>
#   -> gpurun_out/<tag>_summary/ (traffic.json with the config's entry, per-kernel PMC, kernel stats)
set -u
TAG=$1; CFG=${2:-c2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
"$ROOT/scripts/profile.sh" "$TAG" --config "$CFG" --steps 30 --warmup 5 --preroll-ms 0 || exit $?
OUT=$ROOT/gpurun_out/${TAG}_summary
mkdir -p "$OUT"
python3 "$ROOT/scripts/traffic.py" "$ROOT/gpurun_out/prof_$TAG" "$CFG" --out "$OUT" --kernel render_hw1_chunks_kernel \
    > "$OUT/traffic.log" 2>&1 || exit $?
cp "$ROOT/profiles/traffic.json" "$OUT/traffic.json"
cp "$ROOT/gpurun_out/prof_$TAG"/trace/*kernel_stats.csv "$OUT/" 2>/dev/null
cp "$ROOT/gpurun_out/prof_$TAG"/*.log "$OUT/" 2>/dev/null
rm -rf "$ROOT/gpurun_out/prof_$TAG"
ls "$OUT"
