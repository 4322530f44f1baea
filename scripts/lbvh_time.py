"""Time the LBVH build: host (rt_build_bvh, the reference CPU algorithm) vs GPU
(rt_build_bvh_device, device-resident mesh), on the c3 frog and the c5 heightfield.

    python scripts/lbvh_time.py [--reps 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
for cfg in ("c3", "c5"):
    sp = configs.scene_path(configs.G_CONFIGS[cfg]["scene"])
    hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
    t0 = time.perf_counter()
    hn, ha = rt.build_bvh(hs.positions, hs.indices)
    host_s = time.perf_counter() - t0
    pos = torch.from_numpy(hs.positions).cuda()
    idx = torch.from_numpy(hs.indices.view(np.int32)).cuda()
    rt.build_bvh_device(pos, idx, tensors=True)  # warm
    ts = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gn, ga = rt.build_bvh_device(pos, idx, tensors=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    same = np.array_equal(gn.cpu().numpy().view(np.uint32), hn) and \
        np.array_equal(ga.cpu().numpy().view(np.uint32), ha.view(np.uint32))
    print(json.dumps({"config": cfg, "triangles": hs.num_triangles, "host_build_ms": round(host_s * 1e3, 2),
                      "gpu_build_ms_median": round(float(np.median(ts)) * 1e3, 3),
                      "gpu_build_ms_min": round(min(ts) * 1e3, 3), "identical": bool(same)}), flush=True)
