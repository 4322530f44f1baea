#!/bin/bash
# Round-3 evidence on the GPU box (run from the repo root): traversal statistics (RT_STATS
# build), kernel traces whose render-kernel mean is checked against the same process's HIP
# events, and the c3b bench line.  Output under gpurun_out/r03/.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/r03
mkdir -p "$OUT"
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
}
for c in c3 c5; do
  RT_MI355X_LIB=$ROOT/build/variants/stats/librt_mi355x.so step stats_$c 300 python3 "$ROOT/scripts/stats.py" $c
done
cd /tmp && export TMPDIR=/tmp
for m in serial none p6; do
  step trace_c3_$m 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c3_$m" -o run -- \
      python3 "$ROOT/scripts/profile_frames.py" --config c3 --frames 50 --mode $m
done
for m in serial p6; do
  step plain_c3_$m 300 python3 "$ROOT/scripts/profile_frames.py" --config c3 --frames 200 --mode $m
done
cd "$ROOT"
step bench_c3b 400 python3 bench.py --config c3b --steps 20 --warmup 5
step ab_spill_c3 300 python3 scripts/ab_libs.py --config c3 --rounds 7 --reps 10 new=default head=build/variants/head/librt_mi355x.so
