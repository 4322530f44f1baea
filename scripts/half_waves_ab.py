"""A/B of half waves (RT_TUNE_HALF_WAVES, set with rt_tuning_set / --tune half_waves=1: 32 samples per wave) against full waves on band shards of
a c3 frame, one GPU, interleaved rounds: per band count N, every shard's mean kernel and frame
ms under each setting, the max over shards (the per-rank time an N-GPU frame waits for), and a
bit-exact check of every shard's P6 and float output between the two settings.

    python scripts/half_waves_ab.py [--rounds 3] [--steps 20] [--counts 1,2,4,8]
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--counts", default="1,2,4,8")
ap.add_argument("--settings", default="0,1")
a = ap.parse_args()

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
ds = rt.DeviceScene.from_host(hs, device=0)
H, W = cam.pixel_height, cam.pixel_width
dev = torch.device("cuda", 0)
p6 = torch.zeros((H * W * 3,), dtype=torch.uint8, device=dev)
rgb = torch.zeros((H * W * 3,), dtype=torch.float32, device=dev)
res = {}
for n in [int(x) for x in a.counts.split(",")]:
    S = a.settings.split(",")
    acc = {h: [[] for _ in range(n)] for h in S}
    facc = {h: [[] for _ in range(n)] for h in S}
    outs = {}
    for _ in range(a.rounds):
        for h in S:
            rt.set_tuning("half_waves", int(h))
            for r in range(n):
                o, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"],
                                     miss_color=hs.settings["miss_color"], band_rows=8, band_index=r, band_count=n)
                for _ in range(3 + a.steps):
                    ds.render_device(cam, o, rgb.data_ptr(), stream=None, p6_dev_ptr=p6.data_ptr())
                torch.cuda.synchronize()
                acc[h][r].append(float(ds.kernel_times(a.steps).mean()))
                facc[h][r].append(float(ds.frame_times(a.steps).mean()))
                rows = rt._lib.lib().rt_shard_rows(H, 8, r, n)
                got = (p6[:rows * W * 3].cpu().numpy().tobytes(), rgb[:rows * W * 3].cpu().numpy().view(np.uint32))
                if r in outs:
                    assert got[0] == outs[r][0] and np.array_equal(got[1], outs[r][1]), f"N={n} shard {r} differs"
                else:
                    outs[r] = got
    line = {"N": n}
    for h in S:
        k = [float(np.median(v)) for v in acc[h]]
        f = [float(np.median(v)) for v in facc[h]]
        line[f"half{h}"] = {"kernel_max": round(max(k), 4), "kernel_mean": round(sum(k) / n, 4),
                            "frame_max": round(max(f), 4), "frame_mean": round(sum(f) / n, 4)}
    line["identical"] = True
    print(json.dumps(line), flush=True)
rt.set_tuning("half_waves", None)
ds.close()
