"""Where a multi-bounce wave's time goes: per work item of the c3b render kernel, the record
visits of its lanes' per-lane traversals (bounce and bounce-shadow rays), from the variant build
    scripts/build_variant.sh laneiters -DRT_WAVE_TIMES -DRT_LANE_ITERS
    RT_MI355X_LIB=build/variants/laneiters/librt_mi355x.so python scripts/lane_iters.py [--config c3b]

Per item: `wsum` = sum over the wave's traversal calls of its longest lane's visits (lanes meet
after every traversal: what the wave waits for now), `lmax` = the longest lane's total visits
over all calls (what it would wait for if each lane ran its own path to the end without
meeting the others), `lsum` = all lanes' visits.  wsum / lmax > 1 is the gain a per-lane
continuation loop could buy on that item; the longest items (wall time) bound the kernel.
"""
import argparse
import ctypes as C
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import _lib, configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3b")
ap.add_argument("--out", default=str(REPO / "gpurun_out" / "lane_iters.json"))
ap.add_argument("--band", default="", help="band shard r/n (8-row bands): only that rank's rows")
a = ap.parse_args()
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H, spp = cam.pixel_width, cam.pixel_height, cfg["spp"]
lib = _lib.lib()
lib.rt_debug_wave_times_set.argtypes = [C.c_void_p, C.c_void_p]
lib.rt_debug_lane_iters_set.argtypes = [C.c_void_p, C.c_void_p]
ds = rt.DeviceScene.from_host(hs)
kw = {}
if a.band:
    r, n = (int(v) for v in a.band.split("/"))
    kw = {"band_rows": 8, "band_index": r, "band_count": n}
opts, _j = ds.make_opts(spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"], **kw)
items = (W * H + 7) // 8 * 4  # bound for any tile shape (>= 8 pixels per tile), 4 waves per tile
times = torch.zeros(items * 2, dtype=torch.int64, device="cuda")
cuts = torch.full((items,), -1, dtype=torch.int32, device="cuda")
iters = torch.zeros(items * 4, dtype=torch.int32, device="cuda")
acc = torch.zeros(256 * 16 * 256 * 4, dtype=torch.int32, device="cuda")  # >= grid blocks x 256 threads
rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
assert lib.rt_debug_wave_times_set(C.c_void_p(times.data_ptr()), C.c_void_p(cuts.data_ptr())) == 0
assert lib.rt_debug_lane_iters_set(C.c_void_p(iters.data_ptr()), C.c_void_p(acc.data_ptr())) == 0
st = torch.cuda.current_stream().cuda_stream
for _ in range(5):  # heavy-first costs settle (each frame waited for: the threshold needs a finished one)
    ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
    torch.cuda.synchronize()
times.zero_()
iters.zero_()
ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
torch.cuda.synchronize()
kms = float(ds.kernel_times(1)[0])
t = times.cpu().numpy().reshape(-1, 2)
it = iters.cpu().numpy().reshape(-1, 4).astype(np.int64)
live = np.nonzero(t[:, 1])[0]
s, e = t[live, 0], t[live, 1]
d = (e - s) * 10e-3  # us
wsum, lmax, lsum, calls = it[live, 0], it[live, 1], it[live, 2], it[live, 3]
order = np.argsort(-d)
res = {
    "config": a.config, "band": a.band, "kernel_ms_event": kms, "heavy_tiles": ds.heavy_tiles(), "items": int(len(live)),
    "dur_us_pct": {p: round(float(np.percentile(d, p)), 1) for p in (50, 90, 99, 100)},
    "total_wsum": int(wsum.sum()), "total_lmax": int(lmax.sum()), "total_lsum": int(lsum.sum()),
    "corr_dur_wsum": round(float(np.corrcoef(d, wsum)[0, 1]), 3),
    "corr_dur_lmax": round(float(np.corrcoef(d, lmax)[0, 1]), 3),
    "us_per_wsum_visit_top100": round(float((d[order[:100]] / np.maximum(wsum[order[:100]], 1)).mean()), 4),
    "longest": [{"item": int(live[i]), "dur_us": round(float(d[i]), 1), "wsum": int(wsum[i]), "lmax": int(lmax[i]),
                 "lsum": int(lsum[i]), "calls": int(calls[i]),
                 "wsum_over_lmax": round(float(wsum[i] / max(lmax[i], 1)), 2)} for i in order[:25]],
}
top = order[: max(1, len(order) // 100)]
res["top1pct_wsum_over_lmax"] = round(float(wsum[top].sum() / max(lmax[top].sum(), 1)), 3)
Path(a.out).write_text(json.dumps(res, indent=1))
print(json.dumps({k: v for k, v in res.items() if k != "longest"}))
for r in res["longest"][:25]:
    print(json.dumps(r))
