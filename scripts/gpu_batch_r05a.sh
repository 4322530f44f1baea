set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_hw1.py tests/test_gpu_parity.py -k "hw1 or kat or c1 or c2 or quantised or c5" -x -v --timeout 300 --timeout-method thread > gpurun_out/t18_tests.log 2>&1
rc=$?; tail -5 gpurun_out/t18_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/t18_bench_c2.log 2>&1
rc=$?; tail -c 900 gpurun_out/t18_bench_c2.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python bench.py --config c1 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/t18_bench_c1.log 2>&1
rc=$?; tail -c 300 gpurun_out/t18_bench_c1.log
exit 0
