"""Device-clock timeline of consecutive frames in the renderer's pipelined loop (the bench's
frames), from the RT_FRAME_SPAN variant build (scripts/build_variant.sh framespan -DRT_FRAME_SPAN):
per frame the pre-passes' first start and last end, the render kernel's first wave start and last
wave end (wall_clock64, 100 MHz), then the gaps between consecutive render kernels on the device
against the HIP-event kernel time and the delivered period.

    RT_MI355X_LIB=build/variants/framespan/librt_mi355x.so python scripts/frame_span.py [--steps 200] [--tune k=v]
"""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.argv, _argv = [sys.argv[0]], sys.argv[1:]
import bench  # noqa: E402
import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--deliver", default="p6")
ap.add_argument("--tune", action="append", default=[])
a = ap.parse_args(_argv)
rt = bench.rt
for kv in a.tune:
    rt.set_tuning(kv.split("=")[0], float(kv.split("=")[1]))
ba = bench.parse()
ctx = bench.Ctx(ba)
cfg = bench.configs.G_CONFIGS["c3"]
hs = rt.HostScene.load_json(bench.configs.scene_path(cfg["scene"]), REPO)
cam = hs.camera(cfg["width"], cfg["height"])
opts, _j = rt.DeviceScene.make_opts(spp=16, max_depth=1, miss_color=hs.settings["miss_color"])
span = torch.zeros(256 * 4, dtype=torch.int64, device="cuda")
lib = rt._lib.lib()
lib.rt_debug_frame_span_set.argtypes = [C.c_void_p]
d = {"p6": rt.RT_DELIVER_P6, "none": rt.RT_DELIVER_NONE}[a.deliver]
r = bench.make_renderer(hs, ctx, ba, d, rt.RT_GATHER_DIRECT, 3)
bench.timed_native(r, cam, opts, 20, 5, 3, ctx, 100.0)
init = torch.tensor([2**62, 0, 2**62, 0] * 256, dtype=torch.int64, device="cuda")
span.copy_(init)
torch.cuda.synchronize()
assert lib.rt_debug_frame_span_set(C.c_void_p(span.data_ptr())) == 0
t0 = time.perf_counter()
bench.run_frames(r, cam, opts, a.steps, 3)
el = time.perf_counter() - t0
assert lib.rt_debug_frame_span_set(C.c_void_p(0)) == 0
torch.cuda.synchronize()
sp = span.cpu().numpy().reshape(256, 4)
kt = r.scene(0).kernel_times(min(a.steps, 200))
r.close()
rows = sp[(sp[:, 0] < 2**62) & (sp[:, 1] > 0)]
rows = rows[np.argsort(rows[:, 0])][-min(len(rows), a.steps) + 2:-1]
rs, re_, ps, pe = (rows[:, i].astype(np.int64) for i in range(4))
dur = (re_ - rs) / 100.0
gap = (rs[1:] - re_[:-1]) / 100.0
pre_end_vs_start = (pe[1:] - rs[1:]) / 100.0
pre_start_vs_prev_end = (ps[1:] - re_[:-1]) / 100.0
out = {"tuning": a.tune, "deliver": a.deliver, "frames": int(len(rows)), "ms_per_step": round(el / a.steps * 1e3, 4),
       "kernel_event_ms_median": round(float(np.median(kt)), 4),
       "render_span_us_median": round(float(np.median(dur)), 2),
       "device_gap_us": {p: round(float(np.percentile(gap, p)), 2) for p in (10, 50, 90)},
       "device_period_us_median": round(float(np.median(np.diff(rs))) / 100.0, 2),
       "prepass_end_minus_render_start_us": {p: round(float(np.percentile(pre_end_vs_start, p)), 2) for p in (10, 50, 90)},
       "prepass_start_minus_prev_render_end_us": {p: round(float(np.percentile(pre_start_vs_prev_end, p)), 2)
                                                  for p in (10, 50, 90)}}
print(json.dumps(out), flush=True)
