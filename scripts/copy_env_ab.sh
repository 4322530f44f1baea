#!/bin/bash
# The delivered c3 frame period under the HIP runtime's copy settings (the P6 body reaches pinned
# host memory through ROCclr's copy path): one bench run per setting, same box.
# usage: scripts/copy_env_ab.sh [steps]
set -u
STEPS=${1:-200}
for spec in "default:X=1" "wg8:DEBUG_CLR_LIMIT_BLIT_WG=8" "wg32:DEBUG_CLR_LIMIT_BLIT_WG=32" \
            "cpdma:GPU_CP_DMA_COPY_SIZE=16777216" "engine1:GPU_BLIT_ENGINE_TYPE=1" "default2:X=2"; do
  name=${spec%%:*}; envs=${spec#*:}
  out=$(env $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --no-extras --steps "$STEPS" \
        --warmup 20 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('deliver_ms'), t.get('frame_latency_ms'))")
  rc=$?
  echo "$name ms_per_step,kernel_ms,deliver_ms,latency_ms= $out"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
