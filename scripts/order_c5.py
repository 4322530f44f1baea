"""c5 (or any config): render-kernel ms per tile order (RT_TILES_ROWS / XCD_CHUNK / LINEAR),
interleaved rounds in one process, frames checked identical.

    python scripts/order_c5.py [--config c5] [--rounds 3] [--reps 3]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c5")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
ds = rt.DeviceScene.from_host(hs)
orders = {"rows": rt.RT_TILES_ROWS, "xcd_chunk": rt.RT_TILES_XCD_CHUNK, "linear": rt.RT_TILES_LINEAR}
times = {k: [] for k in orders}
ref = None
for _ in range(a.rounds):
    for name, to in orders.items():
        for _ in range(a.reps):
            img = ds.render(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                            diffuse_bounce=hs.settings["diffuse_bounce"], tile_order=to)
        times[name] += list(ds.kernel_times(a.reps))
        if ref is None:
            ref = img
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), name
for name, t in times.items():
    print(json.dumps({"config": a.config, "order": name, "median_ms": round(float(np.median(t)), 3),
                      "min_ms": round(float(np.min(t)), 3)}), flush=True)
