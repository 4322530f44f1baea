"""In-process A/B of the frame renderer with the scene's pre-passes overlapping the previous
frame's render kernel (default) against serialised frames (RT_EXP_SERIAL_PREP=1), c3, deliver
none and p6; rounds interleaved.  Prints ms per delivered frame and median kernel/frame ms."""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402,F401

import raytracinginonesemester_amd as rt  # noqa: E402

hs = rt.HostScene.load_json(REPO / "assets" / "scenes" / "frog.json", REPO)
cam = hs.camera(1920, 1080)
opts, _j = rt.DeviceScene.make_opts(spp=16, max_depth=1, miss_color=hs.settings["miss_color"])
rs = {d: rt.Renderer.from_host(hs, deliver=v) for d, v in (("none", rt.RT_DELIVER_NONE), ("p6", rt.RT_DELIVER_P6))}
res = {}
for _ in range(6):
    for serial in (False, True):
        if serial:
            os.environ["RT_EXP_SERIAL_PREP"] = "1"
        else:
            os.environ.pop("RT_EXP_SERIAL_PREP", None)
        for d, r in rs.items():
            n = 60
            ts = []
            t0 = time.perf_counter()
            for _ in range(n):
                ts.append(r.submit(cam, opts))
                if len(ts) >= 3:
                    r.wait(ts.pop(0))
            for t in ts:
                r.wait(t)
            dt = (time.perf_counter() - t0) / n * 1e3
            sc = r.scene(0)
            key = f"{d}_{'serial' if serial else 'overlap'}"
            e = res.setdefault(key, {"wall": [], "kernel": [], "frame": []})
            e["wall"].append(dt)
            e["kernel"] += list(sc.kernel_times(n))
            e["frame"] += list(sc.frame_times(n))
for k, e in res.items():
    print(json.dumps({"case": k, "ms_per_frame": round(float(np.median(e["wall"])), 4),
                      "kernel_ms": round(float(np.median(e["kernel"])), 4),
                      "frame_ms": round(float(np.median(e["frame"])), 4)}))
