set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hw1.py tests/test_gpu_renderer.py tests/test_gpu_parity.py -k "hw1 or renderer or c3_full or heavy or culling or copy_engines or band" -x -q --timeout 120 --timeout-method thread > gpurun_out/t22_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t22_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bimodal_probe.py --trials 4 --blocks 2 --steps 200 --heavy-off-trials 0 > gpurun_out/t22_gate_on.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/t22_gate_on.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bimodal_probe.py --trials 4 --blocks 2 --steps 200 --heavy-off-trials 0 --tune prepass_gate=0 > gpurun_out/t22_gate_off.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/t22_gate_off.log | cut -c1-160; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/t22_bench.log 2>&1
rc=$?; tail -c 1500 gpurun_out/t22_bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --config c2 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/t22_bench_c2.log 2>&1
rc=$?; tail -c 400 gpurun_out/t22_bench_c2.log; exit $rc
