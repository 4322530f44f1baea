"""One line of the headline numbers from a bench.py log (the last JSON line in it)."""
import json
import sys

d = json.loads([x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1])
t = d.get("timing", {})
print(json.dumps({"value": d["value"], "ms_per_step": d["ms_per_step"], "warmup_frames_run": d.get("warmup_frames_run"),
                  "kernel_ms": t.get("kernel_ms"), "kernel_ms_per_frame": t.get("kernel_ms_per_frame"), "deliver_ms": t.get("deliver_ms"),
                  "frame_latency_ms": t.get("frame_latency_ms"), "traced_rays_per_s": d.get("traced_rays_per_s"),
                  "parity": (d.get("parity") or {}).get("timed_step_ppm_identical"),
                  "roofline_frac": d["roofline"].get("frac"), "cpu": (d.get("cpu_baseline") or {}).get("value")}))
