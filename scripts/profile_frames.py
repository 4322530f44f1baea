"""Frames of one config for rocprofv3 runs, with the HIP-event kernel times of the same process
printed beside them, so a committed kernel trace can be checked against the bench's clock.

    python scripts/profile_frames.py [--config c3] [--frames 50] [--mode serial|none|p6]

serial: rt_render_device into one device buffer on one stream, every frame stream-ordered
        after the previous (pre-passes, then the render kernel: nothing overlaps it);
none:   the renderer with RT_DELIVER_NONE (pre-passes of frame k+1 overlap frame k's kernel);
p6:     the renderer delivering the P6 body to pinned host memory (the bench's step).
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--frames", type=int, default=50)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--mode", default="serial", choices=["serial", "none", "p6"])
ap.add_argument("--series", action="store_true", help="also print every timed frame's render-kernel ms")
ap.add_argument("--busy-ms", type=float, default=0.0, help="keep the GPU busy (matmuls) this long first")
ap.add_argument("--pair", action="store_true",
                help="serial: two frames per render launch (rt_render_device_pair), each pair run alone")
a = ap.parse_args()

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
kw = dict(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
          diffuse_bounce=hs.settings["diffuse_bounce"])
n = a.warmup + a.frames
if a.busy_ms > 0:  # clocks: the GPU busy before the first frame
    x = torch.randn(4096, 4096, device="cuda")
    t_end = time.perf_counter() + a.busy_ms * 1e-3
    while time.perf_counter() < t_end:
        for _ in range(8):
            x = (x @ x).clamp_(-1, 1)
        torch.cuda.synchronize()
if a.mode == "serial":
    ds = rt.DeviceScene.from_host(hs)
    o, _j = ds.make_opts(**kw)
    buf = torch.empty((cam.pixel_height * cam.pixel_width * 3,), dtype=torch.uint8, device="cuda")
    buf2 = torch.empty_like(buf)
    st = torch.cuda.current_stream().cuda_stream
    for k in range(n):
        if k == a.warmup:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        if a.pair:  # frames = pairs here; nothing overlaps a pair's launches
            ds.render_device_pair(cam, cam, o, None, buf.data_ptr(), None, buf2.data_ptr(), stream=st)
            torch.cuda.synchronize()
        else:
            ds.render_device(cam, o, 0, stream=st, p6_dev_ptr=buf.data_ptr())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    sc = ds
else:
    deliver = rt.RT_DELIVER_NONE if a.mode == "none" else rt.RT_DELIVER_P6
    r = rt.Renderer.from_host(hs, devices=(0,), deliver=deliver, depth=2)
    o, _j = rt.DeviceScene.make_opts(**kw)
    pend = []
    for k in range(n):
        if k == a.warmup:
            for t in pend:
                r.wait(t)
            pend = []
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        pend.append(r.submit(cam, o))
        if len(pend) >= 2:
            r.wait(pend.pop(0))
    for t in pend:
        r.wait(t)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    sc = r.scene(0)
kt = sc.kernel_times(a.frames)
pt = sc.prepass_times(a.frames)
if a.series:
    print(json.dumps({"kernel_ms_series": [round(float(x), 4) for x in kt]}), flush=True)
print(json.dumps({"config": a.config, "mode": a.mode, "frames": a.frames,
                  "render_kernel_ms_mean": round(float(kt.mean()), 4),
                  "render_kernel_ms_median": round(float(np.median(kt)), 4),
                  "prepass_ms_mean": round(float(pt.mean()), 4),
                  "ms_per_frame": round(el / a.frames * 1e3, 4),
                  "clock": "HIP events recorded by the render kernel's own dispatch (hipExtLaunchKernel)"}),
      flush=True)
