set -u
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "golden_scene or c3_full or c3b_full or shipped_scene or bounce" -x -q --timeout 200 --timeout-method thread > gpurun_out/t51_tests_def.log 2>&1; tail -1 gpurun_out/t51_tests_def.log
timeout -k 10 300 python scripts/ab_libs.py --config c3 --rounds 9 fixed=default greedy4=default@wide4_greedy=1 2>/dev/null | grep -v amdgpu || exit 1
timeout -k 10 300 python scripts/ab_libs.py --config c3b --rounds 5 --reps 3 fixed=default greedy4=default@wide4_greedy=1 2>/dev/null | grep -v amdgpu || exit 1
timeout -k 10 300 python scripts/ab_libs.py --config c5 --rounds 3 --reps 3 fixed=default greedy4=default@wide4_greedy=1 2>/dev/null | grep -v amdgpu || exit 1
