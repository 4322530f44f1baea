"""Where does a c3 frame's time go?  Kernel ms (HIP events, median of interleaved rounds) for:
  full      — the bench workload
  no_light  — same scene with no lights (no shadow rays; ambient only)
  all_miss  — camera turned away from the frog (every ray fails the root box test)
  prim_only — no lights and no shading work beyond the primary hit
"""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401

import raytracinginonesemester_amd as rt  # noqa: E402

hs = rt.HostScene.load_json(REPO / "assets" / "scenes" / "frog.json", REPO)
cam = hs.camera(1920, 1080)
away = rt.Camera((0.0, -0.2, 0.2), (0.0, -1.0, 0.2), (0.0, 0.0, 1.0), 45.0, 24.0, 1920, 1080)
full = rt.DeviceScene.from_host(hs)
nolt = rt.DeviceScene(hs.num_triangles, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials,
                      np.zeros(0, rt.LIGHT_DTYPE))
cases = {"full": (full, cam), "no_light": (nolt, cam), "all_miss": (full, away)}
times = {k: [] for k in cases}
frames = {k: [] for k in cases}
live = {}
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    for k, (ds, c) in cases.items():
        for _ in range(3):
            ds.render(c, spp=16, max_depth=1)
        times[k] += list(ds.kernel_times(3))
        frames[k] += list(ds.frame_times(3))
        live[k] = ds.live_tiles()
for k, t in times.items():
    print(json.dumps({"case": k, "kernel_median_ms": round(float(np.median(t)), 4), "min_ms": round(float(np.min(t)), 4),
                      "frame_median_ms": round(float(np.median(frames[k])), 4), "live_tiles": live[k]}))
