"""Interleaved in-process A/B of library builds (one box, one process: no cross-box clock noise).

    python scripts/ab_libs.py [--config c3] [--rounds 7] [--reps 5] name=path.so[@knob=v,knob=v] ...
    (name=default means the in-tree library; @knobs: rt_tuning_set values that build's scene is
    created and rendered under, e.g. noq=default@quant_records=0)

Each build gets its own ctypes handle and its own device scene; rounds alternate between the
builds; every build's frame must be bit-identical to the first one's.  Prints per-build median
and min render-kernel ms (HIP events around the render kernel).
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401  (one HIP runtime, as in bench.py)

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--no-check", action="store_true", help="timing experiments whose frames differ by design")
ap.add_argument("--flags", type=int, default=0, help="rt_render_opts.flags for every build (e.g. 8: RT_FLAG_NO_WAVEFRONT)")
ap.add_argument("libs", nargs="+")
a = ap.parse_args()

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
builds = []
knobs = {}


def apply_tuning(name):
    rt.reset_tuning()
    for k, v in knobs[name].items():
        rt.set_tuning(k, v)


for spec in a.libs:
    name, path = spec.split("=", 1) if "=" in spec else (spec, spec)
    path, _, kv = path.partition("@")
    knobs[name] = {k: float(v) for k, v in (x.split("=") for x in kv.split(",") if x)}
    _lib.LIB_PATH = _lib.PKG / "lib" / "librt_mi355x.so" if path == "default" else Path(path)
    _lib._lib = None
    h = _lib.lib()
    apply_tuning(name)
    builds.append((name, h, rt.DeviceScene.from_host(hs)))
times = {n: [] for n, _, _ in builds}
ftimes = {n: [] for n, _, _ in builds}
ref = None
for r in range(a.rounds):
    for name, h, ds in builds:
        _lib._lib = h
        apply_tuning(name)
        for _ in range(a.reps):
            img = ds.render(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                            diffuse_bounce=hs.settings["diffuse_bounce"], flags=a.flags)
        times[name] += list(ds.kernel_times(a.reps))
        ftimes[name] += list(ds.frame_times(a.reps))
        if ref is None:
            ref = img
        if not a.no_check:
            assert np.array_equal(img.view(np.uint32), ref.view(np.uint32)), f"{name}: frame differs"
samples = cfg["width"] * cfg["height"] * cfg["spp"]
for name, _, _ in builds:
    t = np.array(times[name])
    print(json.dumps({"config": a.config, "build": name, "median_ms": round(float(np.median(t)), 4),
                      "min_ms": round(float(t.min()), 4),
                      "frame_median_ms": round(float(np.median(ftimes[name])), 4), "tuning": knobs[name],
                      "Gsamples_s": round(float(samples / np.median(t) / 1e6), 3)}), flush=True)
