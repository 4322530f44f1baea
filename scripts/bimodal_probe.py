"""Why the c3 render kernel measures 0.148 ms in some bench processes and 0.170 in others
(scripts/driver_repeat.sh, profiles/r05/exp/driver_repeat_*.log).  One process, the bench's own
renderer and frame loop (bench.py: make_renderer, timed_native):

    python scripts/bimodal_probe.py [--trials 6] [--blocks 4] [--steps 200]

Each trial makes a new renderer (new scene buffers), pre-rolls 100 ms, then times --blocks
blocks of --steps frames; per block: kernel ms (HIP events), ms per step, pre-pass ms, heavy
tiles.  Then the same with heavy-first dispatch off (RT_TUNE_HEAVY_FRAC = 0).  A flip between
trials with blocks steady inside each points at the instance (buffer placement, the schedule it
settles into); a flip between blocks points at the box (clocks).
"""
from __future__ import annotations

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
ap.add_argument("--config", default="c3")
ap.add_argument("--trials", type=int, default=6)
ap.add_argument("--blocks", type=int, default=4)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--heavy-off-trials", type=int, default=3)
ap.add_argument("--series", action="store_true", help="print each block's per-frame kernel ms")
ap.add_argument("--tune", action="append", default=[], help="knob=value for the default trials (repeatable)")
a = ap.parse_args(_argv)

rt = bench.rt
ba = bench.parse()
ctx = bench.Ctx(ba)
cfg = bench.configs.G_CONFIGS[a.config]
sp = bench.configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == bench.configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
opts, _j = rt.DeviceScene.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                                     diffuse_bounce=hs.settings["diffuse_bounce"])


def trial(tag, k):
    r = bench.make_renderer(hs, ctx, ba, rt.RT_DELIVER_P6, rt.RT_GATHER_DIRECT, 3)
    try:
        bench.timed_native(r, cam, opts, 20, 5, 3, ctx, 100.0)
        sc = r.scene(0)
        for b in range(a.blocks):
            t0 = time.perf_counter()
            bench.run_frames(r, cam, opts, a.steps, 3)
            el = time.perf_counter() - t0
            kt = sc.kernel_times(a.steps)
            print(json.dumps({"tag": tag, "trial": k, "block": b, "kernel_ms": round(float(kt.mean()), 4),
                              "kernel_p10": round(float(sorted(kt)[len(kt) // 10]), 4),
                              "kernel_p90": round(float(sorted(kt)[9 * len(kt) // 10]), 4),
                              "ms_per_step": round(el / a.steps * 1e3, 4),
                              "prepass_ms": round(float(sc.prepass_times(a.steps).mean()), 4),
                              "deliver_ms": round(float(r.times(rt.RT_TIME_DELIVER, a.steps).mean()), 4),
                              "heavy_tiles": sc.heavy_tiles(), "kernel": sc.kernel_name(),
                              **({"series": [round(float(x), 4) for x in kt]} if a.series else {})}), flush=True)
    finally:
        r.close()


for kv in a.tune:
    rt.set_tuning(kv.split("=")[0], float(kv.split("=")[1]))
for k in range(a.trials):
    trial(",".join(a.tune) or "default", k)
rt.reset_tuning()
rt.set_tuning("heavy_frac", 0.0)
for k in range(a.heavy_off_trials):
    trial("heavy_off", k)
rt.reset_tuning()
