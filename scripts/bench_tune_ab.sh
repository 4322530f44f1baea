#!/bin/bash
# Interleaved A/B of whole bench runs over tuning knobs (bench.py --tune knob=value), each run
# its own process, in the driver's window (--steps 20 --warmup 5) unless STEPS/WARMUP say else.
#   scripts/bench_tune_ab.sh <rounds> <config> "name|--tune knob=v --tune knob2=w" ...
# Output: gpurun_out/bench_tune/<name>.<round>.json (one bench line each) + a line per run.
set -u
ROUNDS=$1; CFG=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bench_tune
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    name=${spec%%|*}; args=${spec#*|}
    # shellcheck disable=SC2086
    timeout -k 10 200 python3 "$ROOT/bench.py" --config "$CFG" --steps "${STEPS:-20}" --warmup "${WARMUP:-5}" \
        --no-extras --no-cpu-baseline --no-parity $args > "$OUT/$name.$r.json" 2> "$OUT/$name.$r.err"
    rc=$?
    echo "$name round $r rc=$rc $(python3 -c "import json; d=json.loads(open('$OUT/$name.$r.json').read().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('prepass_ms'), t.get('frame_latency_ms'))" 2>/dev/null)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
