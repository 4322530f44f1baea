"""Interleaved in-process A/B of run-time settings the library reads per call (tuning knobs,
rt_tuning_set), one device scene, frames checked bit-identical across settings.

    python scripts/env_ab.py [--config c3] [--rounds 5] [--reps 20] '{"name": {"knob": value}, ...}' | @file.json

Per setting: median render-kernel ms, device-frame ms (HIP events) and wall ms per frame of a
back-to-back loop on one stream.
"""
import argparse
import json
import os
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
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("settings")
a = ap.parse_args()
settings = json.loads(Path(a.settings[1:]).read_text() if a.settings.startswith("@") else a.settings)

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H = cam.pixel_width, cam.pixel_height
ds = rt.DeviceScene.from_host(hs)
opts, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"])
rgb = torch.zeros((H * W * 3,), dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
res = {k: {"kernel": [], "frame": [], "wall": [], "heavy": []} for k in settings}
ref = None
for _ in range(a.rounds):
    for name, knobs in settings.items():
        rt.reset_tuning()
        for k, v in knobs.items():
            rt.set_tuning(k, v)
        ds.render_device(cam, opts, rgb.data_ptr(), stream=st)  # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
        torch.cuda.synchronize()
        res[name]["wall"].append((time.perf_counter() - t0) / a.reps * 1e3)
        res[name]["kernel"].extend(ds.kernel_times(a.reps))
        res[name]["frame"].extend(ds.frame_times(a.reps))
        res[name]["heavy"].append(ds.heavy_tiles())
        img = rgb.cpu().numpy()
        if ref is None:
            ref = img
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f"{name}: frame differs"
for name, r in res.items():
    print(json.dumps({"config": a.config, "setting": name, "kernel_ms": round(float(np.median(r["kernel"])), 4),
                      "frame_ms": round(float(np.median(r["frame"])), 4),
                      "wall_ms": round(float(np.median(r["wall"])), 4),
                      "heavy_tiles": int(np.median(r["heavy"]))}), flush=True)
