"""Device time of the HW1 kernels (binned vs brute force) on configs c1 / c2, plus parity
between the two.  python scripts/hw1_time.py [--reps 5]"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401  (one HIP runtime, as in bench.py)

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
for name in ("c1", "c2"):
    c = configs.HW1_CONFIGS[name]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    W, H = c["width"], c["height"]
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    args = (mesh.positions, mesh.normals, mesh.indices, cam, c["light_pos"], c["light_color"])
    res = {}
    for brute in (False, True):
        ms = []
        for _ in range(a.reps):
            rgb, hi, ht, t = rt.render_hw1(*args, spp=c["spp"], aov=True, brute=brute, timing=True)
            ms.append(t)
        res[brute] = (rgb, hi, ht, float(np.median(ms)))
    same = all(np.array_equal(res[False][i].view(np.uint32), res[True][i].view(np.uint32)) for i in range(3))
    n = W * H * c["spp"]
    print(json.dumps({"config": name, "triangles": int(np.asarray(mesh.indices).size // 3), "rays": n,
                      "binned_ms": round(res[False][3], 4), "brute_ms": round(res[True][3], 4),
                      "binned_Mrays_s": round(n / res[False][3] / 1e3, 1),
                      "brute_Mrays_s": round(n / res[True][3] / 1e3, 1), "bit_identical": same}), flush=True)
