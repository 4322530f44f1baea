"""Render-kernel ms of the c3 frame for several cameras and launch flags, one device scene:
per (camera, flags) the median kernel ms of back-to-back frames, the tiles the pre-passes
leave, and the camera rays actually traversed (rt_count_rays_ex).

    python scripts/camera_ab.py [--moves "0,0,0;0.004,0,0.003"] [--flags 0,1] [--frames 40]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--moves", default="0,0,0;0.004,0,0.003;0.004,0,0;0,0,0.003;0.0005,0,0")
ap.add_argument("--flags", default="0")
ap.add_argument("--frames", type=int, default=40)
ap.add_argument("--tune", action="append", default=[], help="knob=value (repeatable)")
a = ap.parse_args()
for kv in a.tune:
    rt.set_tuning(kv.split("=")[0], float(kv.split("=")[1]))
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
base = hs.camera(cfg["width"], cfg["height"])
W, H = base.pixel_width, base.pixel_height
ds = rt.DeviceScene.from_host(hs, device=0)
st = torch.cuda.current_stream().cuda_stream
p6 = torch.empty((W * H * 3,), dtype=torch.uint8, device="cuda")
for mv in a.moves.split(";"):
    off = tuple(float(v) for v in mv.split(","))
    cam = rt.Camera(tuple(np.add(base.pos, off)), base.look_at, base.up, base.focal_length_mm,
                    base.sensor_height_mm, W, H)
    for fl in (int(f) for f in a.flags.split(",")):
        o, _j = rt.DeviceScene.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"],
                                         miss_color=hs.settings["miss_color"], flags=fl)
        for _ in range(10):
            ds.render_device(cam, o, 0, stream=st, p6_dev_ptr=p6.data_ptr())
        for _ in range(a.frames):
            ds.render_device(cam, o, 0, stream=st, p6_dev_ptr=p6.data_ptr())
        torch.cuda.synchronize()
        kt = ds.kernel_times(a.frames)
        rays = ds.count_rays(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"])
        print(json.dumps({"move": off, "flags": fl, "kernel_ms": round(float(np.median(kt)), 4),
                          "live_tiles": list(ds.live_tiles()), "heavy_tiles": ds.heavy_tiles(),
                          "kernel": ds.kernel_name(), "rays": rays}), flush=True)
ds.close()
