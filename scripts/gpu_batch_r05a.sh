set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_hw1.py tests/test_gpu_parity.py -k "hw1 or kat or c1 or c2 or quantised or c5" -x -v --timeout 300 --timeout-method thread > gpurun_out/t17_tests.log 2>&1
rc=$?; tail -5 gpurun_out/t17_tests.log; echo "tests rc=$rc"; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python scripts/ab_libs.py --config c5 --rounds 5 --reps 3 q=default noq=default@quant_records=0 > gpurun_out/t17_ab_c5.log 2>&1
rc=$?; tail -3 gpurun_out/t17_ab_c5.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/t17_bench_c2.log 2>&1
rc=$?; tail -c 600 gpurun_out/t17_bench_c2.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python scripts/ab_libs.py --config c3 --rounds 9 def=default leaffam=build/variants/leaffam/librt_mi355x.so > gpurun_out/t17_ab_c3.log 2>&1
rc=$?; tail -2 gpurun_out/t17_ab_c3.log
exit 0
