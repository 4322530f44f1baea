"""Device-to-host copy rate into pinned host buffers against the NUMA node their pages sit on
(the c3 step took 0.25 ms instead of 0.16 in some renderer instances: the 6.2 MB P6 copy at half
speed, profiles/r05/exp/cut_boxes_ab_c3.log).

    python scripts/pinned_numa.py [--buffers 8] [--mb 6.2]

Each buffer: hipHostMalloc (through the library's rt_debug-free path: torch's pinned allocator,
which is hipHostMalloc as well), its first page's node from get_mempolicy(MPOL_F_NODE |
MPOL_F_ADDR), the GPU's node from sysfs, and the median ms of a 6.2 MB device-to-host copy.
"""
from __future__ import annotations

import argparse
import ctypes as C
import glob
import json
import os
import time

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--buffers", type=int, default=8)
ap.add_argument("--mb", type=float, default=6.2)
a = ap.parse_args()

libc = C.CDLL("libc.so.6", use_errno=True)
SYS_get_mempolicy = 239  # x86_64
MPOL_F_NODE, MPOL_F_ADDR = 1, 2


def node_of(addr: int) -> int:
    mode = C.c_int(-1)
    r = libc.syscall(SYS_get_mempolicy, C.byref(mode), None, C.c_ulong(0), C.c_void_p(addr),
                     C.c_ulong(MPOL_F_NODE | MPOL_F_ADDR))
    return mode.value if r == 0 else -1 - C.get_errno()


def gpu_numa():
    out = {}
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            out[p.split("/")[4]] = int(open(p).read())
        except OSError:
            pass
    return out


n = int(a.mb * 1e6)
dev = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.fill_(7)
s = torch.cuda.Stream()
print(json.dumps({"gpu_numa_nodes": gpu_numa(), "cpu": os.sched_getaffinity(0).__len__(),
                  "nodes": sorted(int(p.split("node")[-1]) for p in glob.glob("/sys/devices/system/node/node[0-9]*"))}),
      flush=True)
bufs = []
for i in range(a.buffers):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h.fill_(0)
    ts = []
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(s):
            h.copy_(dev, non_blocking=True)
        s.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    bufs.append(h)
    print(json.dumps({"buffer": i, "node": node_of(h.data_ptr()), "node_last_page": node_of(h.data_ptr() + n - 1),
                      "copy_ms_median": round(ts[len(ts) // 2] * 1e3, 4), "GBps": round(n / ts[len(ts) // 2] / 1e9, 1)}),
          flush=True)
