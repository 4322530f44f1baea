#!/bin/bash
# Interleaved A/B of whole bench runs (delivered frame period) over settings, each run its own
# process (settings read once per process: env vars, variant libraries).
#   scripts/bench_env_ab.sh <rounds> <config> "name|ENV=v ENV2=w" ...
# A setting's env may name RT_MI355X_LIB=build/variants/<v>/librt_mi355x.so.
# Output: gpurun_out/bench_ab/<name>.<round>.json (one bench line each) + a summary.
set -u
ROUNDS=$1; CFG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bench_ab
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    name=${spec%%|*}; envs=${spec#*|}
    env $envs timeout -k 10 200 python3 "$ROOT/bench.py" --config "$CFG" --steps 200 --warmup 10 --no-extras \
        --no-cpu-baseline --no-parity > "$OUT/$name.$r.json" 2> "$OUT/$name.$r.err"
    rc=$?
    echo "$name round $r rc=$rc $(python3 -c "import json,sys; d=json.loads(open('$OUT/$name.$r.json').read().splitlines()[-1]); print(d['ms_per_step'], d['timing']['kernel_ms'], d['timing'].get('prepass_ms'))" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
