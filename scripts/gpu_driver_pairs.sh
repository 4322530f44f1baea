# The driver's command three times with pairs the default, then the bench's multi-rank tests.
set -u
mkdir -p gpurun_out/final3
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final3/c3_driver_$i.log 2>&1 \
    || { tail -20 gpurun_out/final3/c3_driver_$i.log; exit 1; }
  python - "$i" <<'PY'
import json, sys
d = json.loads([x for x in open(f"gpurun_out/final3/c3_driver_{sys.argv[1]}.log") if x.startswith('{"metric')][-1])
t = d["timing"]
print(json.dumps({"run": sys.argv[1], "value": d["value"], "ms_per_step": d["ms_per_step"], "lat": t.get("frame_latency_ms"),
                  "fps": d["config"].get("frames_per_submit"), "other": t.get("other_submission"),
                  "kernel": d["roofline"]["kernel"], "kernel_ms": d["roofline"]["kernel_ms"], "frac": d["roofline"]["frac"]}))
PY
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread -k bench > gpurun_out/final3/multi.log 2>&1 || { tail -30 gpurun_out/final3/multi.log; exit 1; }
tail -1 gpurun_out/final3/multi.log
