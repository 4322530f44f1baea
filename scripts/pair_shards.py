"""Band shards of an N-GPU c3 frame rendered on one GPU, one frame per launch against two
(rt_render_device_pair): per shard the render kernel's time per frame (HIP events; a pair
launch counts as two frames) and the frame period of back-to-back frames.  "pair_moved": pairs
whose second frame is a different camera (the position moved by (0.004, 0, 0.003), as in
tests/test_gpu_pair.py), so the two frames share no rays: whether the pairs' gain comes from
the launch (tail filled, one gap less) or from the second frame reusing the first one's cache
lines (VERDICT/ADVICE r05).

    python scripts/pair_shards.py [--bands 8] [--frames 200]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import _lib as L, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--bands", type=int, default=8)
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--modes", default="single,pair,pair_moved",
                help="of single, single_moved, single_alt (cam, moved alternating), pair, pair_moved (cam, moved), pair_mm (moved, moved)")
ap.add_argument("--tune", action="append", default=[], help="knob=value (repeatable)")
a = ap.parse_args()
for kv in a.tune:
    rt.set_tuning(kv.split("=")[0], float(kv.split("=")[1]))

cfg = configs.G_CONFIGS["c3"]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
moved = rt.Camera(tuple(np.add(cam.pos, (0.004, 0.0, 0.003))), cam.look_at, cam.up, cam.focal_length_mm,
                  cam.sensor_height_mm, cfg["width"], cfg["height"])
W, H = cam.pixel_width, cam.pixel_height
ds = rt.DeviceScene.from_host(hs, device=0)
st = torch.cuda.current_stream().cuda_stream
out = []
for idx in range(a.bands):
    o, _j = rt.DeviceScene.make_opts(spp=cfg["spp"], max_depth=1, miss_color=hs.settings["miss_color"], band_rows=8,
                                     band_index=idx, band_count=a.bands)
    rows = L.lib().rt_shard_rows(H, 8, idx, a.bands)
    bufs = [torch.empty((rows * W * 3,), dtype=torch.uint8, device="cuda") for _ in range(4)]
    row = {"band": idx, "rows": rows}
    for mode in a.modes.split(","):
        for warm in (True, False):
            n = 40 if warm else a.frames
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(0, n, 2):
                ca = moved if mode in ("single_moved", "pair_mm") else cam
                cb = moved if mode in ("pair_moved", "pair_mm", "single_alt") else ca
                if mode.startswith("pair"):
                    ds.render_device_pair(ca, cb, o, None, bufs[k % 4].data_ptr(), None, bufs[(k + 1) % 4].data_ptr(),
                                          stream=st)
                else:
                    ds.render_device(ca, o, 0, stream=st, p6_dev_ptr=bufs[k % 4].data_ptr())
                    ds.render_device(cb, o, 0, stream=st, p6_dev_ptr=bufs[(k + 1) % 4].data_ptr())
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
        launches = n // 2 if mode.startswith("pair") else n
        kt = ds.kernel_times(launches)
        per_frame = float(np.mean(kt)) / (2 if mode.startswith("pair") else 1)
        row[mode] = {"kernel_ms_per_frame": round(per_frame, 4), "ms_per_frame": round(el / n * 1e3, 4),
                     "kernel": ds.kernel_name()}
    out.append(row)
    print(json.dumps(row), flush=True)
print(json.dumps({"bands": a.bands, "tune": a.tune,
                  "max_kernel_ms_per_frame": {m: max(r[m]["kernel_ms_per_frame"] for r in out) for m in a.modes.split(",")},
                  "max_ms_per_frame": {m: max(r[m]["ms_per_frame"] for r in out) for m in a.modes.split(",")}}))
ds.close()
