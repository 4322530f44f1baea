#!/bin/bash
# Round-4 bench lines for every config (run from the repo root on the GPU box), each into
# gpurun_out/bench_r04/<cfg>.log, each under its own time limit; stops at the first failure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/bench_r04
mkdir -p "$OUT"
for spec in "$@"; do
  cfg=${spec%%:*}; args=${spec#*:}; [ "$args" = "$spec" ] && args=""
  timeout -k 10 400 python3 "$ROOT/bench.py" --config "$cfg" $args > "$OUT/$cfg.log" 2> "$OUT/$cfg.err"
  rc=$?
  echo "bench $cfg rc=$rc $(tail -c 300 "$OUT/$cfg.log" | head -c 0)"
  python3 -c "import json,sys; d=json.loads(open('$OUT/$cfg.log').read().strip().splitlines()[-1]); print(' ', d['value'], d['ms_per_step'], d['timing']['kernel_ms'], d.get('parity',{}).get('timed_step_ppm_identical'))" 2>/dev/null
  if [ $rc -ne 0 ]; then exit $rc; fi
done
