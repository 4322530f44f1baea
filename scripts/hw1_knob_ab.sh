#!/bin/bash
# C2 bench A/B over one HW1 knob (bench.py --tune <knob>=<value>), interleaved, each run its own
# process.  usage: scripts/hw1_knob_ab.sh <rounds> <knob> <values...>
# Output: gpurun_out/hw1_knob/<knob>_<value>.<round>.json + a line each.
set -u
ROUNDS=$1; KNOB=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/hw1_knob
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    f=$OUT/${KNOB}_$v.$r
    timeout -k 10 200 python3 "$ROOT/bench.py" --config "${CFG:-c2}" --steps "${STEPS:-200}" --warmup 10 --no-cpu-baseline \
        --tune "$KNOB=$v" > "$f.json" 2> "$f.err" || exit 1
    echo "$KNOB=$v round $r $(python3 -c "import json; d=json.loads(open('$f.json').read().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('host_submit_ms_per_frame'), t.get('host_wait_ms_per_frame'), d['parity']['timed_step_ppm_identical'])")"
  done
done
