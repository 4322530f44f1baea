"""Traversal statistics from an instrumented build (scripts/build_variant.sh stats -DRT_STATS):
    RT_MI355X_LIB=build/variants/stats/librt_mi355x.so python scripts/stats.py [c3|c5] [dx,dy,dz]
(dx,dy,dz: the camera's position moved by that offset)"""
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import _lib, configs  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
cfg = configs.G_CONFIGS[name]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
if len(sys.argv) > 2:
    off = tuple(float(v) for v in sys.argv[2].split(","))
    cam = rt.Camera(tuple(np.add(cam.pos, off)), cam.look_at, cam.up, cam.focal_length_mm, cam.sensor_height_mm,
                    cfg["width"], cfg["height"])
ds = rt.DeviceScene.from_host(hs)
L = _lib.lib()
out = (C.c_ulonglong * 24)()
L.rt_debug_stats(out, 1)
ds.render(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"])
L.rt_debug_stats(out, 1)
v = list(out)
keys = ["trav_p", "trav_s", "pops_p", "pops_s", "popsm_p", "popsm_s", "retest_p", "retest_s", "inner_p",
        "inner_s", "leaf_p", "leaf_s", "ambig", "lanes_p", "lanes_s", "nohit_trav_p", "nohit_pops_p",
        "rootmiss_trav_p", "leafnext_p", "leafnext_s"]
d = dict(zip(keys, v))
d["per_trav_p"] = {k: round(d[k + "_p"] / max(1, d["trav_p"]), 2) for k in ("pops", "popsm", "retest", "inner", "leaf")}
d["per_trav_s"] = {k: round(d[k + "_s"] / max(1, d["trav_s"]), 2) for k in ("pops", "popsm", "retest", "inner", "leaf")}
d["lanes_per_trav"] = [round(d["lanes_p"] / max(1, d["trav_p"]), 1), round(d["lanes_s"] / max(1, d["trav_s"]), 1)]
d["live_tiles"] = ds.live_tiles()
print(json.dumps(d))
