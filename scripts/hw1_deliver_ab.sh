#!/bin/bash
# C2 delivery A/B: bench.py --config c2 over RT_TUNE_HW1_LANES x RT_TUNE_COPY_ENGINE, interleaved,
# each run its own process.  Output: gpurun_out/hw1_ab/L<lanes>_E<engine>.<round>.json + a line each.
#   scripts/hw1_deliver_ab.sh <rounds> "<lanes...>" "<engines...>"
set -u
ROUNDS=${1:-2}; LANES=${2:-"1 2"}; ENGINES=${3:-"0 -1"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/hw1_ab
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for L in $LANES; do
    for E in $ENGINES; do
      f=$OUT/L${L}_E${E}.$r
      timeout -k 10 200 python3 "$ROOT/bench.py" --config c2 --steps "${STEPS:-200}" --warmup 10 --no-cpu-baseline \
          --tune hw1_lanes=$L --tune copy_engine=$E > "$f.json" 2> "$f.err" || exit 1
      echo "L$L E$E round $r $(python3 -c "import json; d=json.loads(open('$f.json').read().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('host_submit_ms_per_frame'), d['parity']['timed_step_ppm_identical'])")"
    done
  done
done
