"""A/B sweep of kernel variants in ONE process, interleaved rounds (guide §5.4 rule 24).

    python scripts/sweep.py [--config c3] [--rounds 5] [--reps 3]

Prints per-variant median / min kernel ms (HIP events around the render kernel) and checks
every variant's frame is bit-identical to the first variant's.
"""
import argparse
import itertools
import json
import os  # noqa: F401
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401  (one HIP runtime, as in bench.py)

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--kernels", default="wave,lane")
ap.add_argument("--tiles", default="linear,xcd_chunk,rows")
ap.add_argument("--flags", default="0", help="RT_FLAG_* values to compare, e.g. 0,2,4 "
                "(1 no cull, 4 binary nodes)")
a = ap.parse_args()

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
ds = rt.DeviceScene.from_host(hs)
K = {"wave": rt.RT_KERNEL_WAVE, "lane": rt.RT_KERNEL_LANE, "wavepix": rt._lib.RT_KERNEL_WAVE_PIXELS}
T = {"linear": rt.RT_TILES_LINEAR, "xcd_chunk": rt.RT_TILES_XCD_CHUNK, "rows": rt.RT_TILES_ROWS}
variants = list(itertools.product(a.kernels.split(","), a.tiles.split(","), a.flags.split(",")))
times = {v: [] for v in variants}
ref = None
for r in range(a.rounds):
    for v in variants:
        for _ in range(a.reps):
            img = ds.render(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                            kernel=K[v[0]], tile_order=T[v[1]],
                            flags=int(v[2]))
        times[v] += list(ds.kernel_times(a.reps))
        if ref is None:
            ref = img
        assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), v
samples = cfg["width"] * cfg["height"] * cfg["spp"]
for v in variants:
    t = np.array(times[v])
    print(json.dumps({"config": a.config, "kernel": v[0], "tiles": v[1], "flags": int(v[2]),
                      "median_ms": round(float(np.median(t)), 4),
                      "min_ms": round(float(t.min()), 4), "Gsamples_s": round(float(samples / np.median(t) / 1e6), 3)}),
          flush=True)
