"""Frames of a HW1 configuration (c1 / c2) for rocprofv3 runs: rt_hw1_scene resident, frames
stream-ordered on one stream (P6 samples written on the device), each waited for; the HIP-event
time of each frame's kernels is printed beside, so a committed trace can be checked against it.

    python scripts/profile_hw1.py [--config c2] [--frames 50]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c2", choices=sorted(configs.HW1_CONFIGS))
ap.add_argument("--frames", type=int, default=50)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--mode", default="serial")  # (the interface of profile_frames.py)
a = ap.parse_args()
c = configs.HW1_CONFIGS[a.config]
mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], c["width"], c["height"], hw1=True)
sc = rt.HW1Scene(mesh.positions, mesh.normals, mesh.indices)
p6 = torch.empty(c["width"] * c["height"] * 3, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
for _ in range(a.warmup + a.frames):
    sc.render_device(cam, c["light_pos"], c["light_color"], c["spp"], p6_ptr=p6.data_ptr(), stream=st)
    torch.cuda.synchronize()
ms = sc.kernel_times(a.frames)
print(json.dumps({"config": a.config, "frames": a.frames, "kernel": sc.kernel_name(),
                  "frame_kernels_ms_median": round(float(np.median(ms)), 4),
                  "frame_kernels_ms_mean": round(float(ms.mean()), 4)}), flush=True)
