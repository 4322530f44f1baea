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
ap.add_argument("--skip", type=int, default=0,
                help="drop each kernel's first N dispatches (profile_frames.py's warmup frames: the first "
                     "frames run before the heavy-first lists exist and before the clocks rise)")
a = ap.parse_args()


def short(name):
    for k in ("render_tiles_kernel", "render_pair_kernel", "tile_cull_pair_kernel", "tile_cut_pair_kernel",
              "render_samples_kernel", "tile_cull_kernel", "tile_cut_kernel",
              "render_hw1_kernel", "render_hw1_chunks_kernel", "hw1_rect_count_kernel", "hw1_scan_chunks_kernel",
              "hw1_fill_kernel", "hw1_resolve_kernel", "copyBuffer", "fillBuffer", "elementwise"):
        if k in name:
            return k
    return name[:40]


import re

instances = collections.Counter()  # render-kernel instantiations seen in the profile (launches)
pmc = collections.defaultdict(lambda: collections.defaultdict(list))
for p in sorted(glob.glob(os.path.join(a.prof, "*", "*counter_collection.csv"))):
    per = collections.defaultdict(lambda: collections.defaultdict(float))  # (kernel, dispatch) -> counter sums
    for r in csv.DictReader(open(p)):
        per[(short(r["Kernel_Name"]), int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
        m = re.search(re.escape(a.kernel) + r"<[^>]*>", r["Kernel_Name"])
        if m:
            instances[(m.group(0), int(r["Dispatch_Id"]))] += 1
    seen = collections.Counter()
    for (kn, _d), cs in sorted(per.items(), key=lambda kv: kv[0][1]):
        seen[kn] += 1
        if seen[kn] <= a.skip:
            continue
        for c, v in cs.items():
            pmc[kn][c].append(v)
summary = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in pmc.items()}
os.makedirs(a.out, exist_ok=True)
with open(os.path.join(a.out, f"{a.config}_pmc_per_launch.csv"), "w") as f:
    f.write("kernel,counter,mean_per_launch,launches\n")
    for k, cs in sorted(pmc.items()):
        for c, v in sorted(cs.items()):
            f.write(f"{k},{c},{sum(v) / len(v):.6g},{len(v)}\n")
for st in glob.glob(os.path.join(a.prof, "trace", "*kernel_stats.csv")):
    os.makedirs(a.out, exist_ok=True)
    Path(a.out, f"{a.config}_kernel_stats_all.csv").write_text(Path(st).read_text())
for tr in glob.glob(os.path.join(a.prof, "trace", "*kernel_trace.csv")):
    # the same statistics over each kernel's dispatches after the first --skip
    by = collections.defaultdict(list)
    for r in csv.DictReader(open(tr)):
        by[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    for name, v in by.items():
        d = [x[1] for x in sorted(v)[a.skip:]] or [x[1] for x in v]
        m = sum(d) / len(d)
        sd = (sum((x - m) ** 2 for x in d) / len(d)) ** 0.5
        rows.append((name, len(d), sum(d), m, min(d), max(d), sd))
    tot = sum(r[2] for r in rows) or 1
    with open(os.path.join(a.out, f"{a.config}_kernel_stats.csv"), "w") as f:
        f.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs","StdDev"\n')
        for r in sorted(rows, key=lambda r: -r[2]):
            f.write(f'"{r[0]}",{r[1]},{r[2]},{r[3]:.6f},{100 * r[2] / tot:.4f},{r[4]},{r[5]},{r[6]:.6f}\n')
k = summary.get(a.kernel, {})

SIMDS, CUS = 1024, 256  # MI355X: 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)


def issue(c):
    """Issue-side fractions of the kernel from one launch's SQ counters (summed over the 8 XCDs
    by rocprofv3).  cycles = GRBM_GUI_ACTIVE / 8 (per-XCD busy cycles ~ the launch's duration).
    VALU: a wave64 VALU instruction holds its SIMD 2 cycles at full throughput (MI355X_MICROARCH.md,
    per-instruction cycle constants: v_fma_f32 wave64 2 cyc), so valu_issue = 2 * SQ_INSTS_VALU /
    (SIMDs * cycles).  SALU: one scalar instruction per cycle per CU.  The wave-state ratios are
    SQ_WAIT_ANY, SQ_WAIT_INST_ANY and SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (same quad-cycle unit);
    waves_per_simd = 4 * SQ_WAVE_CYCLES / (SIMDs * cycles)."""
    need = ("GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY")
    if not all(n in c for n in need):
        return None
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    out = {"cycles_per_xcd": round(cyc),
           "valu_issue": round(2 * c["SQ_INSTS_VALU"] / (SIMDS * cyc), 4),
           "salu_issue": round(c["SQ_INSTS_SALU"] / (CUS * cyc), 4),
           "wait_any": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
           "waves_per_simd": round(4 * c["SQ_WAVE_CYCLES"] / (SIMDS * cyc), 3)}
    for n, key in (("SQ_WAIT_INST_ANY", "wait_inst_any"), ("SQ_ACTIVE_INST_ANY", "active_inst_any")):
        if n in c:
            out[key] = round(c[n] / c["SQ_WAVE_CYCLES"], 4)
    if "SQ_INSTS_SMEM" in c:
        out["smem_per_wave"] = round(c["SQ_INSTS_SMEM"] / c.get("SQ_WAVES", 1), 1)
    out["counters"] = {n: c[n] for n in sorted(c) if n.startswith(("SQ_", "GRBM_"))}
    return out


def binding(i):
    """Name the resource that bounds the kernel: the largest of the pipe fractions, or latency
    when no pipe is near saturation and waves spend most cycles waiting.  The scalar unit is one
    per CU at about one instruction per cycle, and v_readlane / v_writelane run at the same
    per-CU rate (scripts/micro/issue_mix.hip, profiles/r02/issue_mix.jsonl), so the SALU
    fraction understates the scalar side of a kernel that keeps its stack in VGPR lanes."""
    pipes = {"VALU issue": i["valu_issue"], "SALU issue": i["salu_issue"]}
    name, frac = max(pipes.items(), key=lambda kv: kv[1])
    if frac >= 0.8:
        return f"{name} ({frac:.2f} of peak)"
    if not a.kernel.startswith(("render_tiles", "render_pair")):
        return (f"latency: VALU issue {i['valu_issue']:.2f}, SALU issue {i['salu_issue']:.2f}; waves waiting "
                f"{i['wait_any']:.2f} of their cycles at {i['waves_per_simd']:.1f} waves/SIMD")
    return (f"latency and scalar issue: the per-wave chain scalar node load -> box tests -> ballot -> "
            f"push/pop; the busiest pipe is the per-CU scalar unit (SALU {i['salu_issue']:.2f} of its "
            f"rate before the stack's v_readlane/v_writelane, which share it), VALU issue "
            f"{i['valu_issue']:.2f}; waves waiting {i['wait_any']:.2f} of their cycles at "
            f"{i['waves_per_simd']:.1f} waves/SIMD")
names = {n for n, _ in instances}
if len(names) > 1:
    raise SystemExit(f"{a.prof}: several {a.kernel} instantiations {sorted(names)}: profile one per run")
instance = names.pop() if names else (a.kernel if a.kernel in summary else None)  # (untemplated kernels)
if "FETCH_SIZE" in k and "WRITE_SIZE" in k:
    fetch = 2 * k["FETCH_SIZE"] * 1024
    write = k["WRITE_SIZE"] * 1024
    tf = REPO / "profiles" / "traffic.json"
    data = json.loads(tf.read_text()) if tf.exists() else {}
    key = a.config if a.kernel == "render_tiles_kernel" else f"{a.config}/{a.kernel}"  # bench.py load_traffic
    data[key] = {"kernel": a.kernel, "kernel_instance": instance, "bytes_per_launch": round(fetch + write),
                      "fetch_bytes": round(fetch), "write_bytes": round(write),
                      "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                f"{os.path.basename(a.prof.rstrip('/'))}; FETCH_SIZE x2 (gfx950), KiB->B"}
    # every kernel of the profiled frames (the HW1 path's frame is five launches)
    data[key]["per_kernel"] = {
        kn: {"bytes_per_launch": round(2 * cs["FETCH_SIZE"] * 1024 + cs["WRITE_SIZE"] * 1024)}
        for kn, cs in summary.items() if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs}
    iss = issue(k)
    if iss:
        data[key]["issue"] = iss
        data[key]["binding"] = binding(iss)
    tf.write_text(json.dumps(data, indent=1) + "\n")
    print(json.dumps(data[key]))
for name, cs in summary.items():
    print(name, {c: round(v, 1) for c, v in cs.items()})
