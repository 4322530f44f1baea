#!/bin/bash
# The driver's own bench command (python3 bench.py --gpus 1 --steps 20 --warmup 5), repeated, at
# the pipeline depths given (default 2 3) -- the setting the headline is taken with.
set -u
DEPTHS=${*:-"2 3"}
for r in 1 2 3; do for d in $DEPTHS; do
  out=$(timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-extras --depth $d \
        2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['timing']; print(d['value'], d['ms_per_step'], t['kernel_ms'], t.get('frame_latency_ms'), d['parity']['timed_step_ppm_identical'])") || exit 1
  echo "depth $d: value,ms_per_step,kernel_ms,latency_ms,ppm_identical= $out"
done; done
