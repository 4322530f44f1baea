"""Summarise rocprofv3 --pmc passes (pmc_case.sh output): mean per launch of every counter, per kernel.
    python scripts/pmc_sum.py gpurun_out/pmc_<tag> [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "render_tiles"
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if pat not in row["Kernel_Name"]:
            continue
        acc[row["Counter_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
for c, d in sorted(acc.items()):
    v = list(d.values())
    print(f"{c:24s} {sum(v) / len(v):14.4g}  ({len(v)} launches)")
