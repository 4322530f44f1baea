"""Per-kernel resource report of a device translation unit (gfx950 assembly, compiled here):
VGPRs, AGPRs, SGPRs, scratch bytes per lane, LDS bytes, occupancy the launch bounds ask for,
and spill instruction counts.  The product library must show 0 B of scratch for the render
kernels (kill the remaining spills).

    python scripts/isa_report.py [substring] [--src file.hip] [-DFLAG ...] [--json]
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return [n.replace("(anonymous namespace)::", "") for n in r.stdout.split("\n")[:len(names)]]


def report(src: Path, defs, want: str = ""):
    with tempfile.TemporaryDirectory() as td:
        out = Path(td) / "dev.s"
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fno-fast-math", "-mcode-object-version=5", "-Wno-unused-function", *defs,
                        f"-I{REPO}/include", f"-I{REPO}/raytracinginonesemester_amd/csrc", "--cuda-device-only",
                        "-S", str(src), "-o", str(out)], check=True, cwd=td)
        text = out.read_text()
    # kernel descriptors: .amdhsa_kernel NAME ... .end_amdhsa_kernel
    rows = []
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", text, re.S):
        name, body = m.group(1), m.group(2)

        def field(k, default=0):
            mm = re.search(r"\." + k + r" (\d+)", body)
            return int(mm.group(1)) if mm else default
        rows.append({"mangled": name, "vgpr": field("amdhsa_next_free_vgpr"),
                     "sgpr": field("amdhsa_next_free_sgpr"), "scratch_B": field("amdhsa_private_segment_fixed_size"),
                     "lds_B": field("amdhsa_group_segment_fixed_size"),
                     "accum_offset": field("amdhsa_accum_offset")})
    # spill instructions per function body
    for r in rows:
        a = text.find(f"\n{r['mangled']}:")
        b = text.find(".Lfunc_end", a)
        body = text[a:b] if a >= 0 else ""
        r["spill_stores"] = len(re.findall(r"scratch_store|buffer_store.*offen.*\n?.*Spill|; \d+-byte Folded Spill", body))
        r["spill_insts"] = body.count("Spill")
        r["reload_insts"] = body.count("Reload")
    for r, d in zip(rows, demangle([r["mangled"] for r in rows])):
        r["kernel"] = d
    return [r for r in rows if want in r["kernel"]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("want", nargs="?", default="")
    ap.add_argument("--src", default=str(REPO / "raytracinginonesemester_amd" / "csrc" / "rt_device.hip"))
    ap.add_argument("--json", action="store_true")
    a, defs = ap.parse_known_args()
    rows = report(Path(a.src), defs, a.want)
    if a.json:
        print(json.dumps(rows, indent=1))
        return
    for r in rows:
        print(f"{r['vgpr']:4d} v {r['sgpr']:4d} s {r['scratch_B']:5d} B scratch {r['lds_B']:6d} B lds "
              f"{r['spill_insts']:4d} spill {r['reload_insts']:4d} reload  {r['kernel']}")


if __name__ == "__main__":
    sys.exit(main())
