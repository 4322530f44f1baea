set -u
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/chk_default.log 2>&1 || { tail -20 gpurun_out/chk_default.log; exit 1; }
python - <<'PY'
import json
d = json.loads([x for x in open("gpurun_out/chk_default.log") if x.startswith('{"metric')][-1])
t = d["timing"]
print(json.dumps({"value": d["value"], "ms_per_step": d["ms_per_step"], "lat": t.get("frame_latency_ms"),
                  "other": t.get("other_submission"), "render_only": t.get("render_only_value"),
                  "kernel": d["roofline"]["kernel"], "frac": d["roofline"]["frac"]}))
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread -k bench > gpurun_out/chk_multi.log 2>&1 || { tail -30 gpurun_out/chk_multi.log; exit 1; }
tail -1 gpurun_out/chk_multi.log
