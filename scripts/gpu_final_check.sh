# Round-end check: the whole GPU suite and smoke() on the final build.
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/final_gpu_suite.log 2>&1 || { tail -30 gpurun_out/final_gpu_suite.log; exit 1; }
tail -1 gpurun_out/final_gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 \
  || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
mkdir -p gpurun_out/final4
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final4/c3_driver.log 2>&1 || { tail -20 gpurun_out/final4/c3_driver.log; exit 1; }
echo "c3 driver: $(python scripts/bench_line.py gpurun_out/final4/c3_driver.log)"
timeout -k 10 400 python bench.py > gpurun_out/final4/c3_default.log 2>&1 || { tail -20 gpurun_out/final4/c3_default.log; exit 1; }
echo "c3 default: $(python scripts/bench_line.py gpurun_out/final4/c3_default.log)"
timeout -k 10 500 python bench.py --config c3b --no-cpu-baseline > gpurun_out/final4/c3b.log 2>&1 || { tail -20 gpurun_out/final4/c3b.log; exit 1; }
echo "c3b: $(python scripts/bench_line.py gpurun_out/final4/c3b.log)"
