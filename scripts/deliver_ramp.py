"""The SDMA copy's duration over the first seconds of a process (the first process on a fresh
box copied the 6.2 MB P6 body in 0.24 ms instead of 0.114 for a whole run; later processes on the
same box did not, profiles/r05/exp/hwq_overlap_c3.log).  Blocks of frames from the first one on,
per block the mean deliver ms and ms per step:

    python scripts/deliver_ramp.py [--blocks 40] [--steps 100]
"""
import argparse
import json
import sys
import time
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.argv, _argv = [sys.argv[0]], sys.argv[1:]
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--blocks", type=int, default=40)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--idle-ms", type=float, default=0.0, help="host sleep between blocks")
a = ap.parse_args(_argv)
rt = bench.rt
ba = bench.parse()
ctx = bench.Ctx(ba)
cfg = bench.configs.G_CONFIGS["c3"]
hs = rt.HostScene.load_json(bench.configs.scene_path(cfg["scene"]), REPO)
cam = hs.camera(cfg["width"], cfg["height"])
opts, _j = rt.DeviceScene.make_opts(spp=16, max_depth=1, miss_color=hs.settings["miss_color"])
r = bench.make_renderer(hs, ctx, ba, rt.RT_DELIVER_P6, rt.RT_GATHER_DIRECT, 3)
t_start = time.perf_counter()
for b in range(a.blocks):
    t0 = time.perf_counter()
    bench.run_frames(r, cam, opts, a.steps, 3)
    el = time.perf_counter() - t0
    d = r.times(rt.RT_TIME_DELIVER, a.steps)
    print(json.dumps({"block": b, "t_s": round(time.perf_counter() - t_start, 3), "ms_per_step": round(el / a.steps * 1e3, 4),
                      "deliver_ms": round(float(d.mean()), 4), "deliver_ms_min": round(float(d.min()), 4),
                      "kernel_ms": round(float(r.scene(0).kernel_times(a.steps).mean()), 4)}), flush=True)
    if a.idle_ms:
        time.sleep(a.idle_ms / 1e3)
r.close()
