"""Summarise a scripts/profile.sh run into profiles/: per-kernel PMC averages per launch and the
HBM-side traffic of the render kernel for bench.py's roofline.traffic.

    python scripts/traffic.py gpurun_out/prof_<tag> <config> [--out profiles/r01]

Units and corrections (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE and WRITE_SIZE are KiB
per dispatch; on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it is doubled.  Calibrated
here by the frame write: WRITE_SIZE of the render kernel ~= W*H*12 B.
"""
import argparse
import collections
import csv
import glob
import json
import os
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
ap = argparse.ArgumentParser()
ap.add_argument("prof")
ap.add_argument("config")
ap.add_argument("--out", default=str(REPO / "profiles" / "r01"))
ap.add_argument("--kernel", default="render_tiles_kernel")
a = ap.parse_args()


def short(name):
    for k in ("render_tiles_kernel", "render_samples_kernel", "tile_cull_kernel",
              "render_hw1_kernel", "copyBuffer", "fillBuffer", "elementwise"):
        if k in name:
            return k
    return name[:40]


pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(os.path.join(a.prof, "*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(p)):
        pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
summary = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in pmc.items()}
os.makedirs(a.out, exist_ok=True)
with open(os.path.join(a.out, f"{a.config}_pmc_per_launch.csv"), "w") as f:
    f.write("kernel,counter,mean_per_launch,launches\n")
    for k, cs in sorted(pmc.items()):
        for c, v in sorted(cs.items()):
            f.write(f"{k},{c},{sum(v) / len(v):.6g},{len(v)}\n")
for st in glob.glob(os.path.join(a.prof, "trace", "*kernel_stats.csv")):
    os.makedirs(a.out, exist_ok=True)
    Path(a.out, f"{a.config}_kernel_stats.csv").write_text(Path(st).read_text())
k = summary.get(a.kernel, {})
if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
    fetch = 2 * k["FETCH_SIZE"] * 1024
    write = k["WRITE_SIZE"] * 1024
    tf = REPO / "profiles" / "traffic.json"
    data = json.loads(tf.read_text()) if tf.exists() else {}
    data[a.config] = {"kernel": a.kernel, "bytes_per_launch": round(fetch + write),
                      "fetch_bytes": round(fetch), "write_bytes": round(write),
                      "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                f"{os.path.basename(a.prof.rstrip('/'))}; FETCH_SIZE x2 (gfx950), KiB->B"}
    tf.write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data[a.config]))
for name, cs in summary.items():
    print(name, {c: round(v, 1) for c, v in cs.items()})
