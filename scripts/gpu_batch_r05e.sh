set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_renderer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t26_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t26_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bimodal_probe.py --trials 3 --blocks 2 --steps 200 --heavy-off-trials 0 --tune overlap_frames=1 > gpurun_out/t26_ovl.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/t26_ovl.log | cut -c1-170; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/bimodal_probe.py --trials 3 --blocks 2 --steps 200 --heavy-off-trials 0 > gpurun_out/t26_def.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/t26_def.log | cut -c1-170; [ $rc -ne 0 ] && exit $rc
for t in 1 0 1 0; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --tune overlap_frames=$t 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('ovl', $t, d['value'], d['ms_per_step'], d['timing']['kernel_ms'], d['timing'].get('frame_latency_ms'), d.get('parity',{}).get('timed_step_ppm_identical'))" || exit 1; done
