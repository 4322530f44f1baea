"""Render-kernel time of the c3 frame per output variant, interleaved in one process.

    python scripts/frame_variants.py [--config c3] [--rounds 5] [--reps 20]

Variants: rgb (float framebuffer), rgb+p6 (fused P6 epilogue too), p6 (P6 samples only, the
renderer's payload), and the renderer itself (rt_renderer, deliver none / p6 to host).  Prints
median kernel_ms / frame_ms (HIP events) per variant as JSON lines.
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H = cam.pixel_width, cam.pixel_height
ds = rt.DeviceScene.from_host(hs)
opts, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"])
rgb = torch.zeros((H * W * 3,), dtype=torch.float32, device="cuda")
p6 = torch.zeros((H * W * 3,), dtype=torch.uint8, device="cuda")
variants = {"rgb": (rgb.data_ptr(), None), "rgb+p6": (rgb.data_ptr(), p6.data_ptr()), "p6": (0, p6.data_ptr())}
res = {k: ([], []) for k in list(variants) + ["renderer_none", "renderer_p6"]}
rend = {k: rt.Renderer.from_host(hs, deliver=d)
        for k, d in (("renderer_none", rt.RT_DELIVER_NONE), ("renderer_p6", rt.RT_DELIVER_P6))}
st = torch.cuda.current_stream().cuda_stream
for _ in range(a.rounds):
    for k, (rp, pp) in variants.items():
        for _ in range(a.reps):
            ds.render_device(cam, opts, rp, stream=st, p6_dev_ptr=pp)
        torch.cuda.synchronize()
        res[k][0].extend(ds.kernel_times(a.reps))
        res[k][1].extend(ds.frame_times(a.reps))
    for k, r in rend.items():
        ts = [r.submit(cam, opts) for _ in range(2)]
        for _ in range(a.reps):
            r.wait(ts.pop(0))
            ts.append(r.submit(cam, opts))
        for t in ts:
            r.wait(t)
        sc = r.scene(0)
        res[k][0].extend(sc.kernel_times(a.reps))
        res[k][1].extend(sc.frame_times(a.reps))
for k, (kt, ft) in res.items():
    print(json.dumps({"variant": k, "kernel_ms": round(float(np.median(kt)), 4),
                      "frame_ms": round(float(np.median(ft)), 4), "n": len(kt)}), flush=True)
for r in rend.values():
    r.close()
