# Round 5 pair mode: the whole GPU suite, the default bench line, a kernel trace of it.
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_suite.log 2>&1 || { tail -30 gpurun_out/gpu_suite.log; exit 1; }
tail -2 gpurun_out/gpu_suite.log
timeout -k 10 400 python bench.py > gpurun_out/pair_default_bench.log 2>&1 || { tail -20 gpurun_out/pair_default_bench.log; exit 1; }
python scripts/bench_line.py gpurun_out/pair_default_bench.log
TRACE_TAG=_res1 bash scripts/trace_bench.sh > gpurun_out/tl_res1.txt 2>&1 || { tail -5 gpurun_out/tl_res1.txt; exit 1; }
tail -1 gpurun_out/tl_res1.txt
