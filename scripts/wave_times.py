"""Per-wave timeline of the c3 render kernel from the RT_WAVE_TIMES variant build
(scripts/build_variant.sh wavetimes -DRT_WAVE_TIMES): start/end of every rendering wave
(wall clock, 10 ns ticks), then the kernel span, the wave-duration distribution, the number of
waves in flight over time and the longest waves' tiles.

    RT_MI355X_LIB=build/variants/wavetimes/librt_mi355x.so python scripts/wave_times.py [--config c3]
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
ap.add_argument("--config", default="c3")
ap.add_argument("--out", default=str(REPO / "gpurun_out" / "wave_times.json"))
a = ap.parse_args()
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H, spp = cam.pixel_width, cam.pixel_height, cfg["spp"]
lib = _lib.lib()
lib.rt_debug_wave_times_set.argtypes = [C.c_void_p, C.c_void_p]
ds = rt.DeviceScene.from_host(hs)
opts, _j = ds.make_opts(spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"])
tw = 256 // spp
side = 1
while side * side < tw:
    side *= 2
th = tw // side
tiles_x = (W + side - 1) // side
tiles = tiles_x * ((H + th - 1) // th)
buf = torch.zeros(tiles * 4 * 2, dtype=torch.int64, device="cuda")
rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
cuts = torch.full((tiles,), -1, dtype=torch.int32, device="cuda")
assert lib.rt_debug_wave_times_set(C.c_void_p(buf.data_ptr()), C.c_void_p(cuts.data_ptr())) == 0
phase = torch.zeros(tiles * 4 * 2, dtype=torch.int64, device="cuda")
lib.rt_debug_wave_phase_set.argtypes = [C.c_void_p]
assert lib.rt_debug_wave_phase_set(C.c_void_p(phase.data_ptr())) == 0
st = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
torch.cuda.synchronize()
buf.zero_()
phase.zero_()
ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
torch.cuda.synchronize()
kms = float(ds.kernel_times(1)[0])
t = buf.cpu().numpy().reshape(-1, 2)
cc = cuts.cpu().numpy()
ph = phase.cpu().numpy().reshape(-1, 2)
np.savez_compressed(Path(a.out).with_suffix(".npz"), times=t, cut_counts=cc, tiles_x=tiles_x, phase=ph)
live = np.nonzero(t[:, 1])[0]
s, e = t[live, 0].astype(np.int64), t[live, 1].astype(np.int64)
t0 = s.min()
s, e = (s - t0) * 10e-3, (e - t0) * 10e-3  # us
d = e - s
order = np.argsort(-d)
grid = np.linspace(0, e.max(), 41)
inflight = [int(((s <= g) & (e > g)).sum()) for g in grid]
res = {
    "config": a.config, "kernel_ms_event": kms, "live_waves": int(len(live)),
    "span_us": float(e.max()), "last_start_us": float(s.max()),
    "dur_us_pct": {p: round(float(np.percentile(d, p)), 2) for p in (10, 50, 90, 99, 99.9, 100)},
    "mean_dur_us": float(d.mean()),
    "done_by_us": {f: round(float(np.percentile(e, f)), 1) for f in (50, 90, 99, 100)},
    "inflight_every_2.5pct": inflight,
    "longest": [{"tile": int(live[i] // 4), "wave": int(live[i] % 4),
                 "x": int((live[i] // 4) % tiles_x * side), "y": int((live[i] // 4) // tiles_x * th),
                 "start_us": round(float(s[i]), 1), "dur_us": round(float(d[i]), 1)} for i in order[:15]],
}
# tile duration (max over its waves) against its cut-box count
tdur = np.zeros(tiles)
np.maximum.at(tdur, live // 4, d)
lt = np.unique(live // 4)
c = cc[lt]
res["cut_count_vs_tile_dur_us"] = {}
for lo, hi in ((1, 1), (2, 3), (4, 7), (8, 15), (16, 31), (32, 64)):
    m = (c >= lo) & (c <= hi)
    if m.any():
        res["cut_count_vs_tile_dur_us"][f"{lo}-{hi}"] = {"tiles": int(m.sum()), "mean": round(float(tdur[lt][m].mean()), 1),
                                                        "p90": round(float(np.percentile(tdur[lt][m], 90)), 1)}
res["corr_count_dur"] = float(np.corrcoef(c, tdur[lt])[0, 1])
res["culled_by_cut"] = int(((cc == 0)).sum())
Path(a.out).write_text(json.dumps(res, indent=1))
print(json.dumps(res["cut_count_vs_tile_dur_us"]), res["corr_count_dur"], res["culled_by_cut"])
print(json.dumps({k: v for k, v in res.items() if k != "longest"}))
print(json.dumps(res["longest"][:8]))
