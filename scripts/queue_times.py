"""Timeline of the render kernel's work queues from the RT_WAVE_TIMES variant build
(scripts/build_variant.sh wavetimes -DRT_WAVE_TIMES): per item (a wave's quarter of a tile) its
start / end (wall clock, 10 ns ticks), the block and wave that ran it, the XCC it ran on and
whether it was the wave's first (static) item.  Reports the dispatch ramp (first-item starts),
the gap between a wave's consecutive items (the dequeue), items per wave, the XCC each queue ran
on and when each XCC finished.

    RT_MI355X_LIB=build/variants/wavetimes/librt_mi355x.so python scripts/queue_times.py [--config c3]
"""
import argparse
import ctypes as C
import json
import os
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
ap.add_argument("--frames", type=int, default=3)
ap.add_argument("--out", default=str(REPO / "gpurun_out" / "queue_times.json"))
ap.add_argument("--bands", type=int, default=1, help="render band shard --band of an N-way split (8-row bands)")
ap.add_argument("--band", type=int, default=0)
a = ap.parse_args()
cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H, spp = cam.pixel_width, cam.pixel_height, cfg["spp"]
lib = _lib.lib()
lib.rt_debug_wave_times_set.argtypes = [C.c_void_p, C.c_void_p]
lib.rt_debug_wave_meta_set.argtypes = [C.c_void_p]
ds = rt.DeviceScene.from_host(hs)
band_kw = dict(band_rows=8, band_index=a.band, band_count=a.bands) if a.bands > 1 else {}
opts, _j = ds.make_opts(spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"], **band_kw)
hw = rt.get_tuning("half_waves")  # the library's rule (rt_render_device), or the knob when set
half = hw == 1.0 if hw is not None else (a.bands >= 4 or cfg["max_depth"] > 1)
if a.bands > 1:
    H = _lib.lib().rt_shard_rows(H, 8, a.band, a.bands)
tw = (128 if half and spp <= 32 else 256) // spp if spp <= 256 else 1  # pixels per tile
side = 1
while side * side < tw:
    side *= 2
th = max(1, tw // side)
tiles_x = (W + side - 1) // side
tiles = tiles_x * ((H + th - 1) // th)
buf = torch.zeros(tiles * 4 * 2, dtype=torch.int64, device="cuda")
meta = torch.zeros(tiles * 4, dtype=torch.int32, device="cuda")
rgb = torch.zeros(H * W * 3, dtype=torch.float32, device="cuda")
cuts = torch.full((tiles,), -1, dtype=torch.int32, device="cuda")
assert lib.rt_debug_wave_times_set(C.c_void_p(buf.data_ptr()), C.c_void_p(cuts.data_ptr())) == 0
assert lib.rt_debug_wave_meta_set(C.c_void_p(meta.data_ptr())) == 0
st = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
torch.cuda.synchronize()
frames = []
for f in range(a.frames):
    buf.zero_()
    meta.zero_()
    ds.render_device(cam, opts, rgb.data_ptr(), stream=st)
    torch.cuda.synchronize()
    kms = float(ds.kernel_times(1)[0])
    t = buf.cpu().numpy().reshape(-1, 2)
    m = meta.cpu().numpy().view(np.uint32)
    live = np.nonzero(t[:, 1])[0]
    s, e = t[live, 0].astype(np.int64), t[live, 1].astype(np.int64)
    mm = m[live]
    t0 = s.min()
    s, e = (s - t0) * 10e-3, (e - t0) * 10e-3  # us
    block, xcc, first, wv = mm >> 8, (mm >> 4) & 15, (mm >> 2) & 1, mm & 3
    queue = block & 7
    tile_q = ((live // 4) // tiles_x) & 7
    wave = block * 4 + wv
    order = np.lexsort((s, wave))
    ws, we, wid = s[order], e[order], wave[order]
    same = wid[1:] == wid[:-1]
    gaps = (ws[1:] - we[:-1])[same]
    _, per_wave = np.unique(wave, return_counts=True)
    fin = {int(x): round(float(e[xcc == x].max()), 1) for x in np.unique(xcc)}
    wave_end = np.zeros(wave.max() + 1)
    np.maximum.at(wave_end, wave, e)
    wave_end = wave_end[np.unique(wave)]
    res = {
        "config": a.config, "kernel_ms_event": round(kms, 4), "items": int(len(live)), "waves": int(len(per_wave)),
        "blocks": int(len(np.unique(block))), "span_us": round(float(e.max()), 1),
        "first_start_us_pct": {p: round(float(np.percentile(s[first == 1], p)), 2) for p in (50, 90, 99, 100)},
        "dequeue_gap_us_pct": {p: round(float(np.percentile(gaps, p)), 2) for p in (10, 50, 90, 99)} if len(gaps) else {},
        "dequeue_gap_us_sum_per_wave": round(float(gaps.sum() / len(per_wave)), 2) if len(gaps) else 0.0,
        "item_us_pct": {p: round(float(np.percentile(e - s, p)), 2) for p in (10, 50, 90, 99, 100)},
        "items_per_wave_pct": {p: int(np.percentile(per_wave, p)) for p in (0, 10, 50, 90, 100)},
        "wave_end_us_pct": {p: round(float(np.percentile(wave_end, p)), 1) for p in (10, 50, 90, 100)},
        "queue_on_own_xcc": round(float((xcc == queue).mean()), 4),
        "block_tile_same_list": round(float((queue == tile_q).mean()), 4),
        "xcc_finish_us": fin,
        "xcc_items": {int(x): int((xcc == x).sum()) for x in np.unique(xcc)},
    }
    cont = np.zeros((8, 16), dtype=int)
    np.add.at(cont, (queue, xcc), 1)
    res["queue_xcc_mode"] = [int(np.argmax(r)) for r in cont]
    res["queue_xcc_purity"] = round(float(cont.max(axis=1).sum() / cont.sum()), 4)
    d = e - s
    top = np.argsort(-d)[:10]
    res["longest"] = [{"tile": int(live[i] // 4), "q": int(live[i] % 4), "x": int((live[i] // 4) % tiles_x * side),
                       "y": int((live[i] // 4) // tiles_x * th), "start_us": round(float(s[i]), 1),
                       "dur_us": round(float(d[i]), 1), "xcc": int(xcc[i]), "first": int(first[i])} for i in top]
    frames.append(res)
    print(json.dumps(res), flush=True)
Path(a.out).write_text(json.dumps(frames, indent=1))
