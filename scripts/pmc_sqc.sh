#!/bin/bash
# Scalar data cache (K$) behaviour of the c3 render kernel: one --pmc pass (kernel trace only).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_sqc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_DCACHE_MISSES_DUPLICATE \
  --output-format csv -d "$OUT/sqc" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --no-parity --no-extras --steps 10 --warmup 3 \
  > "$OUT/sqc.log" 2>&1
echo "rc=$?"
