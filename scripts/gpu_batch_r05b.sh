set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t19_gpu_all.log 2>&1
rc=$?; tail -4 gpurun_out/t19_gpu_all.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/driver_repeat.sh > gpurun_out/t19_driver_repeat.log 2>&1
rc=$?; cat gpurun_out/t19_driver_repeat.log | tail -6; [ $rc -ne 0 ] && exit $rc
bash scripts/prof_pmc.sh r05_c2 c2 20 > gpurun_out/t19_prof_c2.log 2>&1
rc=$?; cat gpurun_out/t19_prof_c2.log; exit $rc
