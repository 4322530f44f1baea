"""Delivery engines for the c3 frame's P6 body: the runtime's copy
(hipMemcpyAsync device-to-pinned-host, which ROCclr runs as a blit kernel on the CUs) against an
SDMA copy issued through the HSA runtime (hsa_amd_memory_async_copy: a DMA engine, no CU
slots), with the render kernel of the next frame running beside it.

    python scripts/sdma_probe.py [--frames 200] [--modes none,blit,sdma]

none: frames rendered back to back (P6 written on the device, never copied);
blit: each frame's P6 copied to pinned host memory on a copy stream after its render event
      (what rt_renderer does today), frames 3 deep;
sdma: the render stream writes 0 into an HSA signal after the frame (hipStreamWriteValue64),
      and an SDMA copy that depends on that signal is queued at once (no host wait between);
      frames 3 deep (the host waits for copy k-3 before reusing its slot).
Every mode's last host frame is checked against the device frame.  Prints ms per frame, the
render kernel's ms (HIP events) and the copy's own ms where known.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import torch  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--frames", type=int, default=200)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--modes", default="none,blit,sdma")
a = ap.parse_args()

cfg = configs.G_CONFIGS[a.config]
sp = configs.scene_path(cfg["scene"])
hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
cam = hs.camera(cfg["width"], cfg["height"])
W, H = cam.pixel_width, cam.pixel_height
N = W * H * 3
ds = rt.DeviceScene.from_host(hs)
opts, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"])
D = 3
p6 = [torch.zeros(N, dtype=torch.uint8, device="cuda") for _ in range(D)]
host = [torch.zeros(N, dtype=torch.uint8, pin_memory=True) for _ in range(D)]
S = torch.cuda.Stream()
Cs = torch.cuda.Stream()

# ---- HSA (the runtime torch's HIP runtime already initialised) ----------------------------
TL = Path(torch.__file__).parent / "lib"
hsa = C.CDLL(str(TL / "libhsa-runtime64.so"))
hip = C.CDLL(str(TL / "libamdhip64.so"))


class Agent(C.Structure):
    _fields_ = [("handle", C.c_uint64)]


class Signal(C.Structure):
    _fields_ = [("handle", C.c_uint64)]


assert hsa.hsa_init() == 0
agents = {"cpu": [], "gpu": []}
CB = C.CFUNCTYPE(C.c_int, Agent, C.c_void_p)


def _cb(ag, _d):
    t = C.c_uint32()
    hsa.hsa_agent_get_info(ag, 17, C.byref(t))  # HSA_AGENT_INFO_DEVICE
    agents["gpu" if t.value == 1 else "cpu"].append(Agent(ag.handle))
    return 0


cb = CB(_cb)
assert hsa.hsa_iterate_agents(cb, None) == 0
# the GPU agent of torch's device 0: by PCI bus id
bus = C.c_int()
hip.hipDeviceGetAttribute(C.byref(bus), 69, 0)  # hipDeviceAttributePciBusId
gpu = None
for g in agents["gpu"]:
    bdf = C.c_uint32()
    hsa.hsa_agent_get_info(g, 0xA006, C.byref(bdf))  # HSA_AMD_AGENT_INFO_BDFID
    if (bdf.value >> 8) & 0xFF == bus.value:
        gpu = g
gpu = gpu or agents["gpu"][0]
cpu = agents["cpu"][0]
hsa.hsa_signal_create.argtypes = [C.c_int64, C.c_uint32, C.c_void_p, C.POINTER(Signal)]
hsa.hsa_signal_store_screlease.argtypes = [Signal, C.c_int64]
hsa.hsa_signal_wait_scacquire.argtypes = [Signal, C.c_int, C.c_int64, C.c_uint64, C.c_int]
hsa.hsa_signal_wait_scacquire.restype = C.c_int64
hsa.hsa_amd_signal_value_pointer.argtypes = [Signal, C.POINTER(C.c_void_p)]
hsa.hsa_amd_memory_async_copy.argtypes = [C.c_void_p, Agent, C.c_void_p, Agent, C.c_size_t, C.c_uint32,
                                          C.POINTER(Signal), Signal]
hip.hipStreamWriteValue64.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint]


hsa.hsa_amd_signal_create.argtypes = [C.c_int64, C.c_uint32, C.c_void_p, C.c_uint64, C.POINTER(Signal)]


def mk_signal(v, amd=False):
    s = Signal()
    rc = hsa.hsa_amd_signal_create(v, 0, None, 0, C.byref(s)) if amd else hsa.hsa_signal_create(v, 0, None, C.byref(s))
    assert rc == 0, rc
    return s


done = [mk_signal(0) for _ in range(D)]
dep, depptr = [], []
for amd in (False, True):
    dep, depptr = [mk_signal(1, amd) for _ in range(D)], []
    for s in dep:
        p = C.c_void_p()
        rc = hsa.hsa_amd_signal_value_pointer(s, C.byref(p))
        print(json.dumps({"signal": "hsa_amd_signal_create" if amd else "hsa_signal_create", "value_pointer_rc": rc,
                          "ptr": hex(p.value or 0)}), flush=True)
        depptr.append(p.value)
    if all(depptr):
        break
if not all(depptr):
    a.modes = ",".join(m for m in a.modes.split(",") if m != "sdma") + ",sdma_host"


def wait_done(i):
    hsa.hsa_signal_wait_scacquire(done[i], 2, 1, 2 ** 63 - 1, 1)  # until value < 1 (active wait)


import threading  # noqa: E402
import queue  # noqa: E402


def run(mode, n):
    if mode == "sdma_host":
        return run_host(n)
    ev = [torch.cuda.Event() for _ in range(D)]
    cev = [torch.cuda.Event() for _ in range(D)]
    t0 = time.perf_counter()
    for k in range(n):
        i = k % D
        if mode == "sdma" and k >= D:
            wait_done(i)
        if mode == "blit" and k >= D:
            cev[i].synchronize()
        if mode == "sdma":
            hsa.hsa_signal_store_screlease(dep[i], 1)
            hsa.hsa_signal_store_screlease(done[i], 1)
        with torch.cuda.stream(S):
            ds.render_device(cam, opts, None, stream=S.cuda_stream, p6_dev_ptr=p6[i].data_ptr())
            ev[i].record(S)
            if mode == "sdma":
                assert hip.hipStreamWriteValue64(C.c_void_p(S.cuda_stream), C.c_void_p(depptr[i]), 0, 0) == 0
        if mode == "sdma":
            rc = hsa.hsa_amd_memory_async_copy(C.c_void_p(host[i].data_ptr()), cpu, C.c_void_p(p6[i].data_ptr()), gpu,
                                               N, 1, C.byref(dep[i]), done[i])
            assert rc == 0, rc
        if mode == "blit":
            Cs.wait_event(ev[i])
            with torch.cuda.stream(Cs):
                host[i].copy_(p6[i], non_blocking=True)
                cev[i].record(Cs)
    for i in range(D):
        if mode == "sdma":
            wait_done(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def run_host(n):
    """sdma_host: a helper thread waits for each frame's render event, then queues its SDMA copy
    with no dependency (the host's wake-up sits between render and copy)."""
    ev = [torch.cuda.Event(blocking=False) for _ in range(D)]
    q = queue.Queue()

    def copier():
        while True:
            item = q.get()
            if item is None:
                return
            k, i = item
            ev[i].synchronize()
            rc = hsa.hsa_amd_memory_async_copy(C.c_void_p(host[i].data_ptr()), cpu, C.c_void_p(p6[i].data_ptr()), gpu,
                                               N, 0, None, done[i])
            assert rc == 0, rc

    th = threading.Thread(target=copier, daemon=True)
    th.start()
    t0 = time.perf_counter()
    for k in range(n):
        i = k % D
        if k >= D:
            wait_done(i)
        hsa.hsa_signal_store_screlease(done[i], 1)
        ds.render_device(cam, opts, None, stream=S.cuda_stream, p6_dev_ptr=p6[i].data_ptr())
        ev[i].record(S)
        q.put((k, i))
    q.put(None)
    th.join()
    for i in range(D):
        wait_done(i)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


ref = None
res = {m: {"ms": [], "kernel": []} for m in a.modes.split(",")}
for m in res:
    run(m, 20)  # warm
for _ in range(a.rounds):
    for m in res:
        res[m]["ms"].append(run(m, a.frames))
        res[m]["kernel"].extend(ds.kernel_times(min(a.frames, 256)))
        if m != "none":
            last = (a.frames - 1) % D
            assert torch.equal(host[last], p6[last].cpu()), f"{m}: host frame differs from the device frame"
for m, r in res.items():
    print(json.dumps({"config": a.config, "mode": m, "ms_per_frame": round(float(np.median(r["ms"])), 4),
                      "ms_runs": [round(x, 4) for x in r["ms"]],
                      "kernel_ms": round(float(np.median(r["kernel"])), 4)}), flush=True)
