set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "frustum or c3_full or c5 or spine or golden_scene or quantised" -x -q --timeout 300 --timeout-method thread > gpurun_out/t25_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t25_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ab_libs.py --config c3 --rounds 11 perm=default loop=build/variants/pushloop/librt_mi355x.so > gpurun_out/t25_ab_c3.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/t25_ab_c3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ab_libs.py --config c5 --rounds 5 --reps 3 perm=default loop=build/variants/pushloop/librt_mi355x.so > gpurun_out/t25_ab_c5.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/t25_ab_c5.log; exit $rc
