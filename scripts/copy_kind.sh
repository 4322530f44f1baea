#!/bin/bash
# Which engine moves the delivered frames: count blit-kernel copies in a short renderer run under
# each copy setting (kernel trace only), then the un-profiled delivered frame period.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_copy
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for spec in "default:X=1" "sdma_on:HSA_ENABLE_SDMA=1" "blit2:GPU_BLIT_ENGINE_TYPE=2" "forceblit0:GPU_FORCE_BLIT_COPY_SIZE=0" "dev_kernarg:HIP_FORCE_DEV_KERNARG=1"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$name" -o run -- \
    python3 "$ROOT/bench.py" --no-cpu-baseline --no-parity --no-extras --steps 20 --warmup 2 > "$OUT/$name.log" 2>&1 || exit 1
  n=$(cat "$OUT/$name"/*kernel_trace.csv | grep -c copyBuffer || true)
  p=$(cd "$ROOT" && env $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --no-extras --steps 200 --warmup 20 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['timing']['kernel_ms'])")
  echo "$name copyBuffer_kernels=$n ms_per_step,kernel_ms=$p"
done
