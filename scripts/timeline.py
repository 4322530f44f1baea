"""Per-frame timeline of the render loop from a rocprofv3 --kernel-trace CSV (e.g. of
`bench.py`): for the last N render kernels, the gap since the previous render kernel ended and
where the frame's pre-passes (tile_cull_kernel, tile_cut_kernel) ran relative to it (us).

    python scripts/timeline.py <run_kernel_trace.csv> [N]
"""
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda x: x[0])
ren = [k for k in ks if "render_tiles_kernel" in k[2] or "render_pair_kernel" in k[2]]
pre = [k for k in ks if "tile_cull_kernel" in k[2] or "tile_cut_kernel" in k[2]]
gaps, durs, out = [], [], []
for i in range(max(1, len(ren) - n), len(ren)):
    s, e, _ = ren[i]
    ps, pe = ren[i - 1][0], ren[i - 1][1]
    mine = [p for p in pre if pe - 400_000 <= p[0] <= s]  # pre-passes started since shortly before
    first = min((p[0] for p in mine), default=None)
    last = max((p[1] for p in mine), default=None)
    gaps.append((s - pe) / 1e3)
    durs.append((e - s) / 1e3)
    out.append({"render_us": round((e - s) / 1e3, 2), "gap_us": round((s - pe) / 1e3, 2),
                "prepass_start_vs_prev_end_us": None if first is None else round((first - pe) / 1e3, 2),
                "prepass_end_vs_start_us": None if last is None else round((last - s) / 1e3, 2)})
for o in out:
    print(o)
print({"median_render_us": float(np.median(durs)), "median_gap_us": float(np.median(gaps)),
       "median_period_us": float(np.median(np.array(durs) + np.array(gaps)))})
