#!/bin/bash
# Kernel timeline of the renderer (bench.py, c3, P6 to host): rocprofv3 --kernel-trace only.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_frames
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/$1" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --no-parity --no-extras --steps 40 --warmup 5 > "$OUT/$1.log" 2>&1
echo "rc=$?"
