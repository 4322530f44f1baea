"""Render one anatomy case N times (a small driver for rocprofv3 passes).
    python scripts/render_case.py full|no_light|all_miss [reps] [--no-cull]"""
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401

import raytracinginonesemester_amd as rt  # noqa: E402

case = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
flags = rt._lib.RT_FLAG_NO_CULL if "--no-cull" in sys.argv else 0
hs = rt.HostScene.load_json(REPO / "assets" / "scenes" / "frog.json", REPO)
cam = hs.camera(1920, 1080)
if case == "all_miss":
    cam = rt.Camera((0.0, -0.2, 0.2), (0.0, -1.0, 0.2), (0.0, 0.0, 1.0), 45.0, 24.0, 1920, 1080)
lights = np.zeros(0, rt.LIGHT_DTYPE) if case == "no_light" else hs.lights
ds = rt.DeviceScene(hs.num_triangles, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials, lights)
for _ in range(reps):
    ds.render(cam, spp=16, max_depth=1, flags=flags)
print(case, np.median(ds.kernel_times(reps)))
