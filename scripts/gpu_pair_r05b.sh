# Round 5: pair parity, the single-frame suites that share the pipeline code, then the c3 trace and A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_renderer.py -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/pair_tests.log 2>&1 || { tail -40 gpurun_out/pair_tests.log; exit 1; }
tail -2 gpurun_out/pair_tests.log
TRACE_TAG=_p1d bash scripts/trace_bench.sh --pair 1 --depth 6 > gpurun_out/tl_p1d.txt 2>&1 || { tail -5 gpurun_out/tl_p1d.txt; exit 1; }
tail -1 gpurun_out/tl_p1d.txt
PAIR_RUNS="${PAIR_RUNS:-0:3 1:4 1:6}" bash scripts/gpu_pair_ab.sh
