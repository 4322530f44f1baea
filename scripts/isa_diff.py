"""Kernel-by-kernel comparison of two gfx950 device assemblies (hipcc --cuda-device-only -S):
the instruction text of every kernel, comments, debug lines and label numbers dropped.  Used to
show the round-6 split of rt_device.hip into sections and translation units changed no kernel
(profiles/r06/isa_split_identical.txt).

    python scripts/isa_diff.py before.s after.s
"""
import re, sys, json
def bodies(path):
    t = open(path).read()
    out = {}
    for m in re.finditer(r"\n(_Z\S+):\s*; @", t):
        name = m.group(1)
        b = t.find(".Lfunc_end", m.end())
        body = t[m.end():b]
        # drop comments and label numbering differences
        lines = [re.sub(r";.*", "", l).strip() for l in body.split("\n")]
        lines = [re.sub(r"\.LBB\d+_", ".LBB_", re.sub(r"\.Ltmp\d+", ".Ltmp", l)) for l in lines if l and not l.startswith(".loc") and not l.startswith(".file")]
        out[name] = lines
    return out
a, b = bodies(sys.argv[1]), bodies(sys.argv[2])
same = [k for k in a if k in b and a[k] == b[k]]
diff = [k for k in a if k in b and a[k] != b[k]]
only_a = [k for k in a if k not in b]; only_b = [k for k in b if k not in a]
print(json.dumps({"same": len(same), "diff": diff, "only_before": len(only_a), "only_after": len(only_b)}, indent=0)[:3000])
