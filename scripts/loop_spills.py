"""Static check of the traversal loops: compile rt_device.hip to gfx950 assembly and count, per
loop of a kernel, the instructions by kind and the SGPR/VGPR spill traffic inside it.

    python scripts/loop_spills.py [kernel-substring] [-D...]
"""
import collections
import re
import subprocess
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
want = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-D") else "render_tiles_kernelILi1ELb1ELb1E"
defs = [a for a in sys.argv[1:] if a.startswith("-D")]
with tempfile.TemporaryDirectory() as td:
    out = Path(td) / "dev.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-fno-fast-math", "-mcode-object-version=5", "-Wno-unused-function", *defs,
                    f"-I{REPO}/include", f"-I{REPO}/raytracinginonesemester_amd/csrc", "--cuda-device-only", "-S",
                    str(REPO / "raytracinginonesemester_amd/csrc/rt_device.hip"), "-o", str(out)],
                   check=True, cwd=td)
    lines = out.read_text().split("\n")
names = [i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l)]
for i in names:
    name = lines[i][:-1]
    if want not in name:
        continue
    end = next(j for j in range(i + 1, len(lines)) if lines[j].startswith("\t.size") or lines[j].startswith(".Lfunc_end"))
    cur = None
    stats = collections.defaultdict(collections.Counter)
    for l in lines[i:end]:
        m = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", l)
        if m:
            cur = f"{m.group(1)} depth {m.group(2)}"
        t = l.strip()
        if not t or t.startswith(";") or t.endswith(":") or t.startswith("."):
            continue
        op = t.split()[0]
        if "Spill" in t or "Reload" in t:
            k = "scratch_spill"
        elif op in ("v_writelane_b32", "v_readlane_b32"):
            k = op
        elif op.startswith("s_cbranch") or op == "s_branch":
            k = "branch"
        elif op.startswith("s_load") or op.startswith("s_buffer"):
            k = "smem"
        elif op.startswith(("global_", "buffer_", "scratch_", "flat_")):
            k = "vmem"
        elif op.startswith("s_"):
            k = "salu"
        elif op.startswith("v_"):
            k = "valu"
        else:
            k = "other"
        stats[cur or "outside loops"][k] += 1
    print(name)
    for h, c in stats.items():
        print(f"  {h:20s}", dict(sorted(c.items())))
