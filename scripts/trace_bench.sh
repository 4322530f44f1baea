#!/bin/bash
# Kernel trace of the pipelined bench loop (c3, SDMA delivery), summarised by scripts/timeline.py:
# per frame the render kernel, the gap before it and where the pre-passes ran.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_bench${TRACE_TAG:-}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --steps 60 --warmup 5 --no-extras --no-cpu-baseline --no-parity "$@" > "$OUT/bench.log" 2>&1 || exit $?
python3 "$ROOT/scripts/timeline.py" "$(ls "$OUT"/*/run_kernel_trace.csv "$OUT"/run_kernel_trace.csv 2>/dev/null | head -1)" 30
