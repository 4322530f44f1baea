#!/bin/bash
# The delivered c3 frame period with the P6 body copied by the HIP runtime (blit kernels) or by
# SDMA copies queued through the HSA runtime (RT_TUNE_COPY_ENGINE), at pipeline depths 2 and 3;
# two rounds, same box.  usage: scripts/engine_ab.sh [steps]
set -u
STEPS=${1:-200}
for r in 1 2; do for d in 2 3; do for e in 0 1; do
  out=$(timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --no-extras --steps "$STEPS" --warmup 20 \
        --depth $d --tune copy_engine=$e 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('deliver_ms'), t.get('frame_latency_ms'), d['config']['copy_engine'][:6])") || exit 1
  echo "depth $d engine $e: ms_per_step,kernel_ms,deliver_ms,latency_ms= $out"
done; done; done
