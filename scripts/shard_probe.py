"""Band shards of one frame rendered alone on this GPU: per shard, render-kernel ms, live and
heavy tiles, with heavy-first dispatch on and off (RT_TUNE_HEAVY_FRAC = 0 through rt_tuning_set), to check that a shard's
work queues get their heavy tiles first like the whole frame's.
    python scripts/shard_probe.py [--config c3b] [--n 2]"""
import argparse
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3b")
ap.add_argument("--n", type=int, default=2)
ap.add_argument("--frames", type=int, default=12)
a = ap.parse_args()
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
H, W = cam.pixel_height, cam.pixel_width
p6 = torch.zeros((H * W * 3,), dtype=torch.uint8, device="cuda")
for heavy in ("default", "0"):
    rt.set_tuning("heavy_frac", 0 if heavy == "0" else None)
    ds = rt.DeviceScene.from_host(hs, device=0)
    for r in [None] + list(range(a.n)):
        kw = {} if r is None else {"band_rows": 8, "band_index": r, "band_count": a.n}
        o, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"], **kw)
        for _ in range(a.frames):
            ds.render_device(cam, o, 0, stream=None, p6_dev_ptr=p6.data_ptr())
        torch.cuda.synchronize()
        kt = ds.kernel_times(a.frames // 2)
        print(json.dumps({"heavy": heavy, "shard": r, "n": a.n, "kernel_ms": [round(float(x), 4) for x in kt],
                          "live_tiles": list(ds.live_tiles()), "heavy_tiles": ds.heavy_tiles()}), flush=True)
    ds.close()
