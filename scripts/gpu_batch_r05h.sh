set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_renderer.py tests/test_gpu_parity.py -k "renderer or heavy or c3_full or copy_engines or band" -x -q --timeout 200 --timeout-method thread > gpurun_out/t40_tests.log 2>&1
rc=$?; tail -3 gpurun_out/t40_tests.log; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for t in "kernel_timing_every=4" "kernel_timing_every=1" "kernel_timing_every=4 --tune prepass_gate=0.5" "kernel_timing_every=1 --tune prepass_gate=0.5"; do
timeout -k 10 200 python scripts/bimodal_probe.py --trials 2 --blocks 2 --steps 200 --heavy-off-trials 0 --tune $t 2>/dev/null | cut -c1-230 || exit 1
done
for t in 4 1 4 1; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --tune kernel_timing_every=$t 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('every', $t, d['value'], d['ms_per_step'], d['timing']['kernel_ms'], d['timing'].get('frame_latency_ms'), d.get('parity',{}).get('timed_step_ppm_identical'))" || exit 1; done
