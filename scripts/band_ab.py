"""Interleaved in-process A/B of library builds on band shards (the per-rank work of an N-way
split, rendered on one GPU): per build, each shard's median render-kernel and device-frame ms,
and the max over shards (what bounds an N-GPU frame).  Every shard's P6 strip must be
bit-identical across builds.

    python scripts/band_ab.py [--config c3] [--bands 8] [--rounds 5] [--reps 20] name=path.so ...
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
from raytracinginonesemester_amd import _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--bands", type=int, default=8)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("libs", nargs="+")
a = ap.parse_args()
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H = cam.pixel_width, cam.pixel_height
builds = []
for spec in a.libs:
    name, path = spec.split("=", 1)
    _lib.LIB_PATH = _lib.PKG / "lib" / "librt_mi355x.so" if path == "default" else Path(path)
    _lib._lib = None
    h = _lib.lib()
    builds.append((name, h, rt.DeviceScene.from_host(hs)))
p6 = torch.zeros((H * W * 3,), dtype=torch.uint8, device="cuda")
kt = {n: [[] for _ in range(a.bands)] for n, _, _ in builds}
ft = {n: [[] for _ in range(a.bands)] for n, _, _ in builds}
ref = {}
for _ in range(a.rounds):
    for name, h, ds in builds:
        _lib._lib = h
        for b in range(a.bands):
            o, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                                 diffuse_bounce=hs.settings["diffuse_bounce"], band_rows=8, band_index=b,
                                 band_count=a.bands)
            for _ in range(3 + a.reps):
                ds.render_device(cam, o, 0, stream=None, p6_dev_ptr=p6.data_ptr())
            torch.cuda.synchronize()
            kt[name][b] += list(ds.kernel_times(a.reps))
            ft[name][b] += list(ds.frame_times(a.reps))
            rows = h.rt_shard_rows(H, 8, b, a.bands)
            strip = p6[: rows * W * 3].cpu().numpy().tobytes()
            if b in ref:
                assert strip == ref[b], f"{name}: shard {b} differs"
            else:
                ref[b] = strip
for name, _, _ in builds:
    k = [float(np.median(x)) for x in kt[name]]
    f = [float(np.median(x)) for x in ft[name]]
    print(json.dumps({"config": a.config, "bands": a.bands, "build": name, "kernel_ms_max": round(max(k), 4),
                      "frame_ms_max": round(max(f), 4), "kernel_ms": [round(x, 4) for x in k],
                      "frame_ms": [round(x, 4) for x in f]}), flush=True)
