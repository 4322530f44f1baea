#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (camera samples/s) of the per-pixel ray path at
1920x1080x16 spp on the frog scene (BASELINE.json configs[2]; c4 when N > 1), counting frames
that reached host memory.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c3b|c5] [--deliver p6|f32]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

A step = one full frame delivered to rank 0's host memory, as the reference's timed region
is render() plus the device-to-host copy of the frame (G/src/main.cu:369-376).  The native
frame renderer (rt_renderer, include/rt_mi355x.h) does it: every rank renders its 8-row bands
(band b -> rank b % N) with the HIP kernels, which write the strip's P6 samples themselves
(write_p6, fused epilogue), and copies them over its own PCIe link into their rows of the
host frame: pinned memory of the one process (--gpus N without a launcher: this process
drives GPUs 0..N-1), or, one process per GPU under torchrun, a host frame shared by the
processes (POSIX shm pinned in each, per-rank completion words; rank 0's wait returns when
every rank has published the frame).  Frames are pipelined 2 deep on one GPU, 3 over N.
Every timed frame is waited for in host memory before the clock stops.  At N > 1 the RCCL
strip gather over xGMI (rank 0 assembles the frame in its HBM, then copies it) is measured
after the headline and reported beside it (rccl_gather).
--deliver f32 delivers the float framebuffer (the reference's own payload, 4x the bytes).
--comm torch keeps the older torch.distributed gather (nccl or gloo) as an alternate launcher.
A failed native multi-GPU path exits non-zero; --allow-fallback permits the gloo gather.

Scene upload and BVH build are outside the timed region (as G/src/main.cu:362-378 times only
render() + copy); the LBVH build times are reported beside (lbvh_build).  Rank 0 prints one
JSON line.
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import json
import math
import os
import platform
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

HW1_CONFIG_NAMES = ("c1", "c2")  # configs.HW1_CONFIGS (checked in main; the package loads HIP, so later)


def _argv_value(argv, flag):
    for i, x in enumerate(argv):
        if x == flag and i + 1 < len(argv):
            return argv[i + 1]
        if x.startswith(flag + "="):
            return x.split("=", 1)[1]
    return None


# The HW1 delivery's frames alternate over lanes, and a lane overlaps the others only on a hardware
# queue of its own (rt_render_hw1_deliver, RT_TUNE_HW1_LANES): HIP gives a process
# GPU_MAX_HW_QUEUES of them (4 by default); 8 hold the 4 lanes hw1_main runs.  HIP reads it at its
# initialisation, so it is set here, before torch loads the runtime (--hw-queues).
HW1_HW_QUEUES, HW1_LANES = 8, 4
if _argv_value(sys.argv[1:], "--config") in HW1_CONFIG_NAMES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(int(_argv_value(sys.argv[1:], "--hw-queues") or HW1_HW_QUEUES))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before librt_mi355x: one HIP runtime in the process)
import torch.distributed as dist  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
BAND_ROWS = 8
METRIC = "Mrays/s at 1920x1080x16spp (1/2/4/8 GPU) + PPM max-abs pixel diff"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs: under torchrun one process per GPU (WORLD_SIZE must match); without a "
                         "launcher this process drives GPUs 0..N-1 itself")
    ap.add_argument("--steps", type=int, default=100)  # ~35 ms of frames: a steadier average
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--preroll-ms", type=float, default=1500.0,
                    help="untimed frames for about this much wall time before the W warmup frames (GPU "
                         "clocks, and the device-to-host copies, which run at half speed for the first "
                         "~0.45 s of sustained traffic in a process; 0: none); the frames run are reported "
                         "as warmup_frames_run")
    ap.add_argument("--config", default="c3", choices=sorted(configs.G_CONFIGS) + sorted(configs.HW1_CONFIGS),
                    help="c1 / c2: the HW1 path (HW1/src/render.cpp:72-116) on one GPU (hw1_main)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "wave", "lane"])
    ap.add_argument("--deliver", default="p6", choices=["p6", "f32"])
    ap.add_argument("--gather", default="auto", choices=["auto", "rccl", "direct", "shm"],
                    help="auto: direct (one process) / shm (one process per GPU); rccl: the strip gather "
                         "to rank 0's GPU over RCCL, then rank 0's host copy")
    ap.add_argument("--allow-fallback", action="store_true",
                    help="if the native multi-GPU path fails, fall back to the torch.distributed gather "
                         "over gloo (CPU-staged; named in config.fallback).  Off: the failure exits non-zero")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: more ranks / band shards than visible GPUs, sharing them")
    ap.add_argument("--no-rccl-leg", action="store_true", help="N > 1: skip the secondary RCCL-gather measurement")
    # frames in flight: 2 on one GPU (render k+1 while frame k's P6 is copied: 0.2170 vs 0.2233
    # ms per frame at 3, 0.328 at 6); 3 over N GPUs
    ap.add_argument("--depth", type=int, default=None)
    ap.add_argument("--pair", type=int, default=None, choices=[0, 1],
                    help="1: the frames are submitted two at a time (rt_renderer_submit_pair: one render launch "
                         "renders both where the pair kernel fits them); 0: one at a time (lower frame latency); "
                         "default 1 for the configs the pair kernel takes (depth-1 frames of a scene within "
                         "RT_TUNE_BIG_SCENE_BYTES: c3 and its band shards), else 0; the other mode is measured "
                         "beside the headline")
    ap.add_argument("--comm", default="native", choices=["native", "torch"],
                    help="native: rt_renderer (librt_mi355x); torch: torch.distributed gather (alternate launcher)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="--comm torch only. gloo: CPU-staged gather (lets N ranks share one GPU)")
    ap.add_argument("--gather-payload", default="p6", choices=["p6", "f32"], help="--comm torch only")
    ap.add_argument("--hw-queues", type=int, default=HW1_HW_QUEUES,
                    help="c1 / c2: GPU_MAX_HW_QUEUES for this process (a delivery lane per 2; set before HIP "
                         "initialises)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the secondary measurements")
    ap.add_argument("--tune", action="append", default=[], metavar="KNOB=VALUE",
                    help="library tuning knob (rt_tuning_set, include/rt_mi355x.h), e.g. peer_timeout_s=60; "
                         "named in the line's config when set")
    ap.add_argument("--traffic-file", default=str(REPO / "profiles" / "traffic.json"),
                    help="per-launch HBM bytes and issue counters measured by rocprofv3 --pmc (DESIGN.md §5)")
    return ap.parse_args()


# ---- CPU baseline -----------------------------------------------------------------------
def usable_cores() -> dict:
    """Cores this process may run on: the affinity mask, capped by a cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(-(-int(q) // int(per))))
    except Exception:
        pass
    model = platform.processor() or platform.machine()
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    usable = min(aff, quota) if quota else aff
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "usable": usable, "model": model}


def cpu_baseline(hs, cam, cfg) -> dict:
    """The oracle restatement (bit-exact to the reference build, tests/test_oracle.py) timed on
    every usable core of this host on a bounded sample of the frame, plus the HW1 C1 CPU path
    and, when present, the reference's own CPU render() built from its sources (1 thread)."""
    from oracle import pyoracle as orc

    cores = usable_cores()
    threads = cores["usable"]
    b = cam.basis()
    oc = orc.camera_from_basis(b["center"], b["pixel00_loc"], b["pixel_delta_u"], b["pixel_delta_v"],
                               cam.pixel_width, cam.pixel_height)
    H, W, spp = cam.pixel_height, cam.pixel_width, cfg["spp"]
    rows = (0, H) if cfg["scene"] == "frog.json" else (H // 2 - 32, H // 2 + 32)
    reps, t0 = 0, time.perf_counter()
    while True:  # repeat the sample until ~10 s of CPU work (at least once)
        orc.render_g(hs.num_triangles, oc, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials,
                     hs.lights, spp=spp, max_depth=cfg["max_depth"], miss=hs.settings["miss_color"], rows=rows,
                     diffuse_bounce=hs.settings["diffuse_bounce"], threads=threads)
        reps += 1
        if time.perf_counter() - t0 >= 10.0:
            break
    dt = time.perf_counter() - t0
    n = (rows[1] - rows[0]) * W * spp * reps
    out = {"value": n / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": f"oracle/rt_oracle.c (bit-exact restatement of G/ render()) rows {rows[0]}..{rows[1]} of "
                     f"{W}x{H}x{spp}, {reps} pass(es), {n} samples, {dt:.2f} s, OpenMP {threads} threads",
           "host": cores}
    # HW1 CPU path (north_star: "the HW1 CPU path timed on the same box's host cores"): C1
    try:
        c1 = configs.HW1_CONFIGS["c1"]
        mesh = rt.MeshHW1(configs.MESHES / c1["mesh"])
        hcam = orc.camera(c1["position"], c1["look_at"], c1["up"], c1["focal_mm"], c1["sensor_mm"], c1["width"],
                          c1["height"], hw1=True)
        hw1 = {}
        for th in (1, threads):
            reps1, t1 = 0, time.perf_counter()
            while True:
                orc.render_hw1(mesh.positions, mesh.normals, mesh.indices, hcam, c1["light_pos"], c1["light_color"],
                               spp=c1["spp"], threads=th)
                reps1 += 1
                if time.perf_counter() - t1 >= 2.0:
                    break
            d1 = time.perf_counter() - t1
            hw1[f"{th}_threads"] = round(c1["width"] * c1["height"] * c1["spp"] * reps1 / d1 / 1e6, 4)
        out["hw1_c1"] = {"unit": "Mrays/s", **hw1,
                         "sample": "C1: HW1 brute force (HW1/src/render.cpp:72-116), sphere 960 tris, 256x256x1spp, "
                                   "oracle restatement"}
    except Exception as e:  # pragma: no cover - reported, not fatal
        out["hw1_c1"] = {"error": repr(e)}
    ref = REPO / "oracle" / "_ref" / "ref_g"
    if ref.exists() and cfg["scene"] == "frog.json":
        with tempfile.TemporaryDirectory() as td:
            r = subprocess.run([str(ref), "scene", str(configs.SCENES / cfg["scene"]), str(REPO), td, str(W), str(H),
                                str(spp), str(cfg["max_depth"]), "-1", "0"], capture_output=True, text=True,
                               timeout=600)
            if r.returncode == 0:
                ms = json.loads((Path(td) / "meta.json").read_text())["render_ms"]
                out["reference_as_shipped"] = {
                    "value": W * H * spp / (ms / 1e3) / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "reference",
                    "sample": "G/ render() CPU branch built from /root/reference sources (oracle/_ref/ref_g), "
                              f"full frame, per-pixel jitter rebuild as shipped, {ms / 1e3:.2f} s"}
    return out


# ---- timing helpers ----------------------------------------------------------------------
def sync_all(dev, world):
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)


PAIR = {"on": False}


def PAIR_CONFIGS(a, cfg) -> bool:
    """The configs the pair kernel takes: depth-1 frames of a scene within RT_TUNE_BIG_SCENE_BYTES
    (c3 and its band shards; c5's 345 MB scene takes the big-scene kernels) and one-light
    multi-bounce frames on the paired-only bounce kernels (c3b)."""
    return a.config in ("c3", "c3b")


def run_frames(r, cam, opts, n, depth):
    """Submit n frames, waiting for every one of them (host memory on rank 0), at most depth in
    flight; with --pair 1 two at a time (rt_renderer_submit_pair), an odd last one alone."""
    pend = []
    last = None
    i = 0
    while i < n:
        two = PAIR["on"] and depth >= 2 and n - i >= 2
        while len(pend) > depth - (2 if two else 1):
            last = r.wait(pend.pop(0))
        if two:
            pend += list(r.submit_pair(cam, cam, opts))
        else:
            pend.append(r.submit(cam, opts))
        i += 2 if two else 1
    for t in pend:
        last = r.wait(t)
    return last


PREROLL = {"frames": 0}


def timed_native(r, cam, opts, steps, warmup, depth, ctx, preroll_ms=0.0):
    """W warmup frames, then K timed frames.  preroll_ms > 0: before the warmup, frames for about
    that much GPU time.  The GPU's clocks rise only under sustained load: a c3 frame's render
    kernel takes 0.22 ms in the first frames after an idle period and 0.18 ms after ~100 of them
    (`scripts/profile_frames.py --series`, profiles/r03/exp/clock_ramp_series.log), so a
    few-millisecond timed region that starts cold measures the ramp.  The device-to-host copies
    ramp too, later: the first process on a fresh box copied c3's 6.2 MB P6 body in 0.238 ms for
    its first ~0.45 s of frames, then in 0.1136 ms (scripts/deliver_ramp.py,
    profiles/r05/exp/deliver_ramp_c3.log), so the default pre-roll is 1.5 s.  The count is agreed
    over the ranks (every rank renders every frame) and reported as warmup_frames_run."""
    n_pre, chunk = 0, 2
    t0 = time.perf_counter()
    while preroll_ms > 0 and n_pre < 200000:  # chunks of ~10 ms of frames; the ranks agree on each step
        tc = time.perf_counter()
        run_frames(r, cam, opts, chunk, depth)
        n_pre += chunk
        per = (time.perf_counter() - tc) / chunk
        done, nxt = ctx.max([1.0 if time.perf_counter() - t0 >= preroll_ms * 1e-3 else 0.0,
                             float(max(1, min(64, int(0.01 / max(per, 1e-6)))))])
        if done > 0:
            break
        chunk = int(nxt)
    PREROLL["frames"] = n_pre + warmup
    run_frames(r, cam, opts, warmup, depth)
    ctx.sync()
    t0 = time.perf_counter()
    last = run_frames(r, cam, opts, steps, depth)
    ctx.sync()
    t1 = time.perf_counter()
    return t1 - t0, last


GATHERS = {"rccl": rt.RT_GATHER_RCCL, "direct": rt.RT_GATHER_DIRECT, "shm": rt.RT_GATHER_HOST_SHARED}
GATHER_NAMES = {rt.RT_GATHER_RCCL: "rccl", rt.RT_GATHER_DIRECT: "direct", rt.RT_GATHER_HOST_SHARED: "shm"}
COMM_TEXT = {
    "direct": "each GPU copies its own bands into the pinned host frame over its own PCIe link (one process)",
    "shm": "each rank copies its own bands over its own PCIe link into one host frame shared by the "
           "ranks' processes (POSIX shm pinned with hipHostRegister, per-rank completion words); no RCCL",
    "rccl": "strips to rank 0's GPU over RCCL (grouped ncclSend/ncclRecv, xGMI), then rank 0's host copy",
}


class Ctx:
    """Where this process's ranks live: one process per GPU (torchrun: WORLD_SIZE > 1) or one
    process driving every GPU (--gpus N without a launcher)."""

    def __init__(self, a):
        env_world = int(os.environ.get("WORLD_SIZE", "1"))
        ndev = torch.cuda.device_count()
        self.multiproc = env_world > 1
        if self.multiproc:
            if a.gpus != env_world:
                raise SystemExit(f"bench: --gpus {a.gpus} but WORLD_SIZE {env_world}")
            self.world = env_world
            self.rank = int(os.environ.get("RANK", "0"))
            local = int(os.environ.get("LOCAL_RANK", "0"))
            if local >= ndev and not a.share_gpu:
                raise SystemExit(f"bench: local rank {local} but only {ndev} GPU(s) visible "
                                 "(--share-gpu rehearses several ranks per GPU)")
            self.devices = (local % max(ndev, 1),)
        else:
            self.world, self.rank = a.gpus, 0
            if a.gpus < 1:
                raise SystemExit("bench: --gpus must be >= 1")
            if ndev < a.gpus and not a.share_gpu:
                raise SystemExit(f"bench: --gpus {a.gpus} but only {ndev} GPU(s) visible "
                                 "(--share-gpu rehearses several band shards per GPU)")
            self.devices = tuple(d % max(ndev, 1) for d in range(a.gpus))
        self.distinct = len(set(self.devices)) == len(self.devices) and not (self.multiproc and a.share_gpu)
        self.dev = torch.device("cuda", self.devices[0])
        torch.cuda.set_device(self.dev)
        if self.multiproc:
            # control plane (barriers, max over ranks, ids) over gloo; frames move over the
            # renderer's own paths (or torch's nccl group with --comm torch)
            if a.comm == "torch" and a.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group("gloo")

    def sync(self):
        for d in sorted(set(self.devices)):
            torch.cuda.synchronize(d)
        if self.multiproc:
            dist.barrier()
        for d in sorted(set(self.devices)):
            torch.cuda.synchronize(d)

    def bcast(self, obj):
        if not self.multiproc:
            return obj
        box = [obj if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        return box[0]

    def max(self, vals):
        t = torch.tensor(vals, dtype=torch.float64)
        if self.multiproc:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(x) for x in t.tolist()]


def make_renderer(hs, ctx, a, deliver, gather, depth):
    kw = dict(band_rows=BAND_ROWS, deliver=deliver, gather=gather, depth=depth, devices=ctx.devices)
    if ctx.multiproc:
        kw.update(world_size=ctx.world, rank0=ctx.rank)
        if gather == rt.RT_GATHER_RCCL:
            kw["unique_id"] = ctx.bcast(rt.comm_unique_id() if ctx.rank == 0 else None)
        if gather == rt.RT_GATHER_HOST_SHARED:
            kw["host_frame_name"] = ctx.bcast(f"/rt_bench_{os.getpid()}_{os.urandom(6).hex()}"
                                              if ctx.rank == 0 else None)
    return rt.Renderer.from_host(hs, **kw)


def native(a, hs, cam, cfg, ctx):
    spp = cfg["spp"]
    kernel = {"auto": rt.RT_KERNEL_AUTO, "wave": rt.RT_KERNEL_WAVE, "lane": rt.RT_KERNEL_LANE}[a.kernel]
    opts, _jit = rt.DeviceScene.make_opts(spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                                          diffuse_bounce=hs.settings["diffuse_bounce"], kernel=kernel)
    if a.gather == "auto":
        gather = rt.RT_GATHER_HOST_SHARED if ctx.multiproc else rt.RT_GATHER_DIRECT
    else:
        gather = GATHERS[a.gather]
    deliver = rt.RT_DELIVER_F32 if a.deliver == "f32" else rt.RT_DELIVER_P6
    gather_note = None
    if gather == rt.RT_GATHER_HOST_SHARED and a.gather == "auto":
        # the shared host frame needs room in /dev/shm on the node; if any rank cannot make or
        # attach it, every rank takes the RCCL strip gather instead (named in config.comm)
        r, err = None, ""
        try:
            r = make_renderer(hs, ctx, a, deliver, gather, a.depth)
        except rt.RTError as e:
            err = str(e)
        if ctx.max([1.0 if err else 0.0])[0] > 0:
            if r is not None:
                r.close()
            gather_note = f"shared host frame failed ({err or 'on another rank'}); RCCL strip gather used"
            print(f"bench: {gather_note}", file=sys.stderr, flush=True)
            gather = rt.RT_GATHER_RCCL
            r = make_renderer(hs, ctx, a, deliver, gather, a.depth)
    else:
        r = make_renderer(hs, ctx, a, deliver, gather, a.depth)
    elapsed, last = timed_native(r, cam, opts, a.steps, a.warmup, a.depth, ctx, a.preroll_ms)
    warm_run = PREROLL["frames"]
    kts, fts, pts = [], [], []
    for i in range(r.local_ranks):
        sc = r.scene(i)
        kts.append(float(sc.kernel_times(a.steps).mean()))
        fts.append(float(sc.frame_times(a.steps).mean()))
        pts.append(float(sc.prepass_times(a.steps).mean()))
    sc = r.scene(0)
    res = {"elapsed": elapsed, "kernel_ms": max(kts), "frame_ms": max(fts), "prepass_ms": max(pts),
           "kernel_ms_local": kts, "live_tiles": list(sc.live_tiles()), "heavy_tiles": sc.heavy_tiles(),
           "kernel_instance": sc.kernel_name(),
           "gather_path": GATHER_NAMES[gather], "warmup_frames_run": warm_run, "gather_note": gather_note,
           "copy_engine": r.copy_engine}
    if ctx.rank == 0:
        g, d, f = (r.times(k, a.steps) for k in (rt.RT_TIME_GATHER, rt.RT_TIME_DELIVER, rt.RT_TIME_FRAME))
        res.update(gather_ms=float(g.mean()), deliver_ms=float(d.mean()), frame_latency_ms=float(f.mean()))
        addr, n = last
        res["frame_bytes"] = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_uint8 * n).from_address(addr)).tobytes()
    r.close()
    if a.no_extras:
        return res
    # secondary: render only (strips stay in HBM), the rate the round-1 bench reported
    rn = make_renderer(hs, ctx, a, rt.RT_DELIVER_NONE, gather, a.depth)
    res["render_only_s"], _ = timed_native(rn, cam, opts, a.steps, a.warmup, a.depth, ctx, a.preroll_ms)
    # secondary: the other submission mode (two frames per render launch, or one), same frames
    # and delivery, depth 6 for pairs / 3 for single frames
    if PAIR_CONFIGS(a, cfg):
        was = PAIR["on"]
        PAIR["on"] = not was
        dp = 6 if PAIR["on"] else 3
        rp = make_renderer(hs, ctx, a, deliver, gather, dp)
        el, _ = timed_native(rp, cam, opts, a.steps, a.warmup, dp, ctx, a.preroll_ms)
        res["other_mode"] = {"pair": PAIR["on"], "s": el, "depth": dp,
                             "frame_latency_ms": (float(rp.times(rt.RT_TIME_FRAME, a.steps).mean())
                                                  if ctx.rank == 0 else None)}
        rp.close()
        PAIR["on"] = was
    rn.close()
    # secondary: the other payload (f32 = the reference's Vec3 framebuffer), also the float parity
    other = rt.RT_DELIVER_P6 if deliver == rt.RT_DELIVER_F32 else rt.RT_DELIVER_F32
    ro = make_renderer(hs, ctx, a, other, gather, a.depth)
    n_other = max(10, a.steps // 4)
    el, last_o = timed_native(ro, cam, opts, n_other, 2, a.depth, ctx)
    res["other_payload"] = {"deliver": "p6" if other == rt.RT_DELIVER_P6 else "f32", "s": el, "steps": n_other}
    if ctx.rank == 0:
        addr, n = last_o
        res["other_bytes"] = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_uint8 * n).from_address(addr)).tobytes()
    ro.close()
    return res


def rccl_leg(a, hs, cam, cfg, ctx) -> dict:
    """Secondary at N > 1 on distinct GPUs: the RCCL strip gather (north_star's xGMI gather), the
    frame assembled in rank 0's HBM (RT_DELIVER_DEVICE) and, second, also copied to rank 0's host
    memory.  Reported beside the headline, never substituted for it: an RCCL error is recorded."""
    opts, _jit = rt.DeviceScene.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"],
                                          miss_color=hs.settings["miss_color"],
                                          diffuse_bounce=hs.settings["diffuse_bounce"])
    out = {}
    for name, dl in (("device", rt.RT_DELIVER_DEVICE), ("host_p6", rt.RT_DELIVER_P6)):
        rr, err = None, ""
        try:
            rr = make_renderer(hs, ctx, a, dl, rt.RT_GATHER_RCCL, 6 if PAIR["on"] else 3)
        except rt.RTError as e:
            err = str(e)
        if ctx.max([1.0 if err else 0.0])[0] > 0:  # some rank failed: no rank runs the leg
            out[name] = {"error": err or "RCCL renderer failed on another rank"}
            if rr is not None:
                rr.close()
            continue
        el, last = timed_native(rr, cam, opts, a.steps, a.warmup, 6 if PAIR["on"] else 3, ctx)
        el = ctx.max([el])[0]
        d = {"value": round(cfg["spp"] * cam.pixel_width * cam.pixel_height * a.steps / el / 1e6, 3),
             "ms_per_step": round(el / a.steps * 1e3, 4)}
        if ctx.rank == 0:
            d["gather_ms"] = round(float(rr.times(rt.RT_TIME_GATHER, a.steps).mean()), 4)
            d["deliver_ms"] = round(float(rr.times(rt.RT_TIME_DELIVER, a.steps).mean()), 4)
            if dl == rt.RT_DELIVER_P6 and a.config in GOLDEN_FULL:
                addr, n = last
                body = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_uint8 * n).from_address(addr)).tobytes()
                d["ppm_identical"] = ppm_matches_golden(a.config, rt.p6_header(cam.pixel_width, cam.pixel_height) + body)
        rr.close()
        out[name] = d
    return out


def band_shards(hs, cam, cfg, local, steps=20):
    """Each rank's share of a frame at N = 2/4/8, rendered alone on this GPU (the per-rank
    compute a multi-GPU run will show): frame_ms (cull + cut + render) and kernel_ms, and the
    render kernel's ms per frame when the shard's frames go two per launch (the bench's default)."""
    ds = rt.DeviceScene.from_host(hs, device=local)
    H, W = cam.pixel_height, cam.pixel_width
    p6 = torch.zeros((H * W * 3,), dtype=torch.uint8, device=torch.device("cuda", local))
    p6b = torch.zeros_like(p6)
    out = {}
    for n in (2, 4, 8):
        per = []
        for r in range(n):
            o, _j = ds.make_opts(spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                                 band_rows=BAND_ROWS, band_index=r, band_count=n)
            # warm-up frames waited for one by one: heavy-first takes its threshold from a
            # finished frame of this shard, as a rank's own pipelined frames give it (submitted
            # back to back, every frame of the loop ran before any had finished: no heavy lists)
            for _ in range(4):
                ds.render_device(cam, o, 0, stream=None, p6_dev_ptr=p6.data_ptr())
                torch.cuda.synchronize()
            for _ in range(steps):
                ds.render_device(cam, o, 0, stream=None, p6_dev_ptr=p6.data_ptr())
            torch.cuda.synchronize()
            kt = float(ds.kernel_times(steps).mean())
            ft = float(ds.frame_times(steps).mean())
            # the same shard two frames per launch (rt_render_device_pair): kernel ms per frame
            for _ in range(steps // 2):
                ds.render_device_pair(cam, cam, o, None, p6.data_ptr(), None, p6b.data_ptr())
            torch.cuda.synchronize()
            kp = float(ds.kernel_times(steps // 2).mean()) / (2 if ds.kernel_name().startswith("render_pair") else 1)
            per.append((ft, kt, kp))
        fr = [p[0] for p in per]
        out[str(n)] = {"frame_ms": [round(x, 4) for x in fr], "kernel_ms": [round(p[1], 4) for p in per],
                       "kernel_ms_per_frame_pairs": [round(p[2], 4) for p in per],
                       "max_over_mean": round(max(fr) / (sum(fr) / len(fr)), 4)}
    ds.close()
    return out


# ---- the torch.distributed launcher (alternate path, round 1) ----------------------------
def torch_path(a, hs, cam, cfg, world, rank, local, dev):
    """Per step: render (fused P6) into a device strip; world > 1: torch.distributed.gather of
    the strips to rank 0 (async, two buffers), un-permute on rank 0's GPU, then the frame's
    bytes copied to host memory on rank 0."""
    W, H, spp = cam.pixel_width, cam.pixel_height, cfg["spp"]
    kernel = {"auto": rt.RT_KERNEL_AUTO, "wave": rt.RT_KERNEL_WAVE, "lane": rt.RT_KERNEL_LANE}[a.kernel]
    ds = rt.DeviceScene.from_host(hs, device=local)
    opts, _jit = ds.make_opts(spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                              band_rows=BAND_ROWS, band_index=rank, band_count=world, kernel=kernel)
    lib = rt._lib.lib()
    max_rows = max(lib.rt_shard_rows(H, BAND_ROWS, r, world) for r in range(world))
    p6 = a.gather_payload == "p6"
    rb = W * 3 * (1 if p6 else 4)
    strips = [torch.zeros((max_rows, rb), dtype=torch.uint8, device=dev) for _ in range(2)]
    gdev = dev if a.backend == "nccl" else torch.device("cpu")
    gathers = [torch.empty((world, max_rows, rb), dtype=torch.uint8, device=gdev)
               if (world > 1 and rank == 0) else None for _ in range(2)]
    frame_dev = torch.empty((H, rb), dtype=torch.uint8, device=dev) if rank == 0 else None
    host = [torch.empty((H, rb), dtype=torch.uint8).pin_memory() for _ in range(2)] if rank == 0 else None
    pending = [None, None]
    stream = torch.cuda.current_stream(dev).cuda_stream
    frames = [0]

    def finish(b):
        if pending[b] is None:
            return
        if world > 1:
            pending[b].wait()
        pending[b] = None
        if rank == 0:
            if world > 1:
                g = gathers[b] if a.backend == "nccl" else gathers[b].to(dev)
                rt.unpermute_strips_device(g.data_ptr(), max_rows, rb, H, BAND_ROWS, world, frame_dev.data_ptr(),
                                           False, stream)
                host[b].copy_(frame_dev)
            else:
                host[b].copy_(strips[b][:H])

    def step():
        b = frames[0] & 1
        frames[0] += 1
        finish(b)
        s = strips[b]
        if p6:
            ds.render_device(cam, opts, 0, stream=stream, p6_dev_ptr=s.data_ptr())
        else:
            ds.render_device(cam, opts, s.data_ptr(), stream=stream)
        if world > 1:
            src = s if a.backend == "nccl" else s.cpu()
            pending[b] = dist.gather(src, gather_list=list(gathers[b].unbind(0)) if rank == 0 else None, dst=0,
                                     async_op=True)
        else:
            pending[b] = True

    def drain():
        for b in ((frames[0]) & 1, (frames[0] + 1) & 1):
            finish(b)

    for _ in range(a.warmup):
        step()
    drain()
    sync_all(dev, world)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    sync_all(dev, world)
    t1 = time.perf_counter()
    kt, ft = ds.kernel_times(a.steps), ds.frame_times(a.steps)
    res = {"elapsed": t1 - t0, "kernel_ms": float(kt.mean()), "frame_ms": float(ft.mean()),
           "live_tiles": list(ds.live_tiles()), "gather_path": f"torch.distributed.gather ({a.backend})"}
    if rank == 0:
        res["frame_bytes"] = host[(frames[0] - 1) & 1].numpy().tobytes()
    ds.close()
    return res


def load_traffic(path: Path, config: str, instance: str):
    """The measured per-launch traffic of this config's render kernel, only if it was profiled on
    the same kernel instantiation the timed frames launched (profiles/traffic.json records the
    instantiation rocprofv3 named); otherwise None: a line never cites another kernel's bytes."""
    try:
        data = json.loads(path.read_text())
    except Exception:
        return None
    # "<config>" (render_tiles_kernel) or "<config>/<kernel>" (e.g. c3/render_pair_kernel)
    for key in [config] + sorted(k for k in data if k.startswith(config + "/")):
        tr = data.get(key)
        if tr and instance and tr.get("kernel_instance") == instance:
            return tr
    return None


def primary_hit_parity(ds, cam, cfg, hs, golden: str) -> dict:
    """Primary-hit AOVs of one frame (triangle index and t per sample) against the reference's
    own full-size outputs (sha256 in tests/golden/scenes/<golden>/meta.json): equal hashes mean
    0 index mismatches."""
    meta = json.loads((REPO / "tests" / "golden" / "scenes" / golden / "meta.json").read_text())
    _, hi, ht = ds.render(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                          diffuse_bounce=hs.settings["diffuse_bounce"], aov=True)
    idx_ok = hashlib.sha256(hi.tobytes()).hexdigest() == meta["sha256"]["hits.i32"]
    t_ok = hashlib.sha256(ht.tobytes()).hexdigest() == meta["sha256"]["hitt.f32"]
    return {"vs": f"reference hits.i32 / hitt.f32 sha256 (tests/golden/scenes/{golden})",
            "hit_index_sha256_equal": idx_ok, "hit_t_sha256_equal": t_ok,
            "hit_index_mismatches": 0 if idx_ok else "unknown (hash differs)",
            "samples_hit": int((hi >= 0).sum())}


# reference outputs of the full bench frame (sphere, sphere_single: sha256 of the outputs only)
GOLDEN_FULL = {"c3": "c3_full", "c3b": "c3b_full", "sphere": "sphere_full", "sphere_single": "sphere_single_full"}


def golden_ppm(config: str) -> bytes | None:
    p = REPO / "tests" / "golden" / "scenes" / GOLDEN_FULL[config] / "image.ppm.gz"
    return gzip.open(p).read() if p.exists() else None


def golden_ppm_sha(config: str) -> str:
    meta = json.loads((REPO / "tests" / "golden" / "scenes" / GOLDEN_FULL[config] / "meta.json").read_text())
    return meta["sha256"]["image.ppm"]


def ppm_matches_golden(config: str, ppm: bytes) -> bool:
    g = golden_ppm(config)
    return ppm == g if g is not None else hashlib.sha256(ppm).hexdigest() == golden_ppm_sha(config)


def lbvh_times(hs, device: int, reps: int = 5) -> dict:
    """The LBVH build the reference times (G/src/main.cu:281-293 GPU, :306-317 CPU): the host
    build (rt_build_bvh, the reference CPU algorithm) and the GPU build (rt_build_bvh_device,
    mesh resident in HBM), wall clock around each call as the reference measures; arrays compared."""
    hn, ha = rt.build_bvh(hs.positions, hs.indices)  # warm (page-in)
    th = []
    for _ in range(3):
        t0 = time.perf_counter()
        hn, ha = rt.build_bvh(hs.positions, hs.indices)
        th.append(time.perf_counter() - t0)
    pos = torch.from_numpy(hs.positions).to(torch.device("cuda", device))
    idx = torch.from_numpy(hs.indices.view(np.int32)).to(torch.device("cuda", device))
    gn, ga = rt.build_bvh_device(pos, idx, device=device, tensors=True)  # warm (code objects, rocPRIM)
    tg = []
    for _ in range(reps):
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        gn, ga = rt.build_bvh_device(pos, idx, device=device, tensors=True)  # synchronises its stream
        tg.append(time.perf_counter() - t0)
    same = (np.array_equal(gn.cpu().numpy().view(np.uint32), hn)
            and np.array_equal(ga.cpu().numpy().view(np.uint32), ha.view(np.uint32)))
    return {"triangles": hs.num_triangles, "host_ms": round(float(np.median(th)) * 1e3, 3),
            "gpu_ms": round(float(np.median(tg)) * 1e3, 3), "gpu_ms_min": round(min(tg) * 1e3, 3),
            "arrays_identical": bool(same),
            "note": "median wall ms of the call (host: rt_build_bvh, 1 thread; GPU: rt_build_bvh_device incl. "
                    "its stream sync), outside the timed region; the reference prints both (G/src/main.cu:293,317)"}


# ---- HW1 configurations (C1 / C2: HW1/src/render.cpp:72-116 on the device) --------------
HW1_GOLDEN = {"c1": "c1_full", "c2": "c2_full"}


def hw1_cpu_baseline(mesh, c, W, H) -> dict:
    """The HW1 brute-force loop on the host: the oracle restatement (bit-exact to the reference's
    HW1 build, tests/test_oracle.py) on every usable core over a bounded band of rows, repeated to
    ~10 s, and the reference's own HW1 loop built from its sources (oracle/_ref/ref_hw1, 1 thread)
    on a reduced-resolution sample of the same camera."""
    from oracle import pyoracle as orc

    cores = usable_cores()
    threads = cores["usable"]
    hcam = orc.camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    # the band of rows through the middle of the image, where the mesh is
    rows = (0, H) if mesh.num_triangles < 5000 else (H // 2 - 24, H // 2 + 24)
    reps, t0 = 0, time.perf_counter()
    while True:
        orc.render_hw1(mesh.positions, mesh.normals, mesh.indices, hcam, c["light_pos"], c["light_color"],
                       spp=c["spp"], threads=threads, rows=rows)
        reps += 1
        if time.perf_counter() - t0 >= 10.0:
            break
    dt = time.perf_counter() - t0
    n = (rows[1] - rows[0]) * W * c["spp"] * reps
    out = {"value": n / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": f"oracle/rt_oracle.c HW1 brute force (bit-exact restatement of HW1/src/render.cpp:72-116) "
                     f"rows {rows[0]}..{rows[1]} of {W}x{H}x{c['spp']}, {reps} pass(es), {n} rays, {dt:.2f} s, "
                     f"OpenMP {threads} threads", "host": cores}
    ref = REPO / "oracle" / "_ref" / "ref_hw1"
    if ref.exists():
        w, h = (W // 8, H // 8) if mesh.num_triangles >= 5000 else (W, H)
        with tempfile.TemporaryDirectory() as td:
            args = [str(ref), "render", str(configs.MESHES / c["mesh"]), td, str(w), str(h),
                    *map(str, c["position"]), *map(str, c["look_at"]), *map(str, c["up"]), str(c["focal_mm"]),
                    str(c["sensor_mm"]), *map(str, c["light_pos"]), *map(str, c["light_color"]), str(c["spp"])]
            t1 = time.perf_counter()
            r = subprocess.run(args, capture_output=True, text=True, timeout=300)
            d1 = time.perf_counter() - t1
            if r.returncode == 0:
                out["reference_as_shipped"] = {
                    "value": w * h * c["spp"] / d1 / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "reference",
                    "sample": f"HW1 brute-force loop built from /root/reference sources (oracle/_ref/ref_hw1), "
                              f"{w}x{h}x{c['spp']} of the same camera, {d1:.2f} s wall incl. OBJ load"}
    return out


def hw1_main(a):
    """C1 / C2 on one GPU: a step = one W x H x spp frame of the HW1 path (binning passes +
    render kernel, rt_hw1_scene resident in HBM) whose P6 body (write_p6 defaults, fused into the
    render kernel) has reached pinned host memory; rt_render_hw1_deliver copies each body on the
    scene's copy stream while the next frame renders."""
    if a.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        raise SystemExit("bench: the HW1 configurations run on one GPU (replicas only)")
    c = configs.HW1_CONFIGS[a.config]
    W, H, spp = c["width"], c["height"], c["spp"]
    queues = int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    if not any(kv.startswith("hw1_lanes=") for kv in a.tune):  # a lane per 2 hardware queues, 2..4
        rt.set_tuning("hw1_lanes", min(max(queues // 2, 2), HW1_LANES))
    lanes = int(rt.get_tuning("hw1_lanes"))
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sc = rt.HW1Scene(mesh.positions, mesh.normals, mesh.indices, device=0)
    st = torch.cuda.Stream(dev)
    # rt_render_hw1_deliver: each frame's P6 body copied to pinned host memory by a DMA engine
    # while the next frames render, the frames alternating over two lanes (the copy on the render
    # stream serialised with the frames: 0.129 ms per step against 0.096 of kernels, VERDICT r05
    # item 8; one lane with the runtime's blit-kernel copies: 0.100-0.106); host frames, every
    # frame waited for before its buffer is reused and at the end.  6 host frames: the host waits
    # for the copy of the frame 5 back, long done, so its wake-up is off the GPU's path (with 3,
    # the next frame's kernels were submitted only after the host woke from frame k-2's copy:
    # ~16 us idle between frames, profiles/r06/exp/c2_deliver_trace_summary.json)
    depth = 6
    host = [torch.empty(W * H * 3, dtype=torch.uint8, pin_memory=True) for _ in range(depth)]
    nxt = {"k": 0, "submit_s": 0.0, "wait_s": 0.0}

    def frames(n):
        pend = []
        for _ in range(n):
            k = nxt["k"]
            if len(pend) >= depth - 1:
                tw = time.perf_counter()
                sc.wait(pend.pop(0))
                nxt["wait_s"] += time.perf_counter() - tw
            ts = time.perf_counter()
            pend.append(sc.render_deliver(cam, c["light_pos"], c["light_color"], spp, host[k % depth].data_ptr(),
                                          stream=st.cuda_stream))
            nxt["submit_s"] += time.perf_counter() - ts
            nxt["k"] = k + 1
        for t in pend:
            sc.wait(t)

    t0 = time.perf_counter()
    while time.perf_counter() - t0 < a.preroll_ms * 1e-3:  # clocks up (timed_native)
        frames(16)
    frames(a.warmup)
    st.synchronize()
    t0 = time.perf_counter()
    nxt["submit_s"] = nxt["wait_s"] = 0.0
    frames(a.steps)
    st.synchronize()
    elapsed = time.perf_counter() - t0
    submit_ms = nxt["submit_s"] / a.steps * 1e3  # host time inside rt_render_hw1_deliver per frame
    last_host = host[(nxt["k"] - 1) % depth]
    kms = sc.kernel_times(min(a.steps, 64))
    kernel_ms = float(np.median(kms))
    rays = W * H * spp
    value = rays * a.steps / elapsed / 1e6
    line = {"metric": f"Mrays/s ({a.config}: HW1 path, primary rays)", "value": round(value, 3), "unit": "Mrays/s",
            "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic=false: HW1/assets/meshes/{c['mesh']} as the reference ships it",
            "config": {"workload": f"{a.config}: HW1 {c['mesh']} {W}x{H}x{spp}spp, primary rays, HW1 shade "
                                   "(HW1/include/raytracer.h:21-48), brute-force winner (first index on ties)",
                       "triangles": mesh.num_triangles,
                       "step_delivers": "the frame's P6 samples in host memory (pinned), copied by a DMA engine "
                                         "while the next frames render (rt_render_hw1_deliver), every frame "
                                         "waited for",
                       "pipeline": f"frames alternate over {lanes} lanes (binning buffers + a stream each, "
                                   f"RT_TUNE_HW1_LANES; GPU_MAX_HW_QUEUES={queues}): one frame's latency-bound "
                                   "binning passes run beside the others' render kernels; every frame runs all "
                                   "four passes",
                       "lanes": lanes, "hw_queues": queues,
                       "kernels": "hw1_rect_count_kernel + hw1_scan_chunks_kernel + hw1_fill_kernel + "
                                  "render_hw1_chunks_kernel (the resolve fused in; rt_render_hw1_device)"}}
    if a.tune:
        line["config"]["tuning"] = dict(kv.partition("=")[::2] for kv in a.tune)
    instance = sc.kernel_name()
    tr = load_traffic(Path(a.traffic_file), a.config, instance)
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": instance,
            "kernel_ms": round(kernel_ms, 4),
            "note": "kernel_ms: one frame's four launches, HIP events around them (its latency: the lanes' frames "
                    "overlap); achieved_per_step: the same bytes per ms_per_step"}
    hw1_kernels = ("hw1_rect_count_kernel", "hw1_scan_chunks_kernel", "hw1_fill_kernel", "render_hw1_chunks_kernel")
    per = (tr or {}).get("per_kernel") or {}
    if tr and all(k in per for k in hw1_kernels):
        # the frame's four launches (the live kernel_ms spans them): their measured bytes summed
        frame_bytes = sum(per[k]["bytes_per_launch"] for k in hw1_kernels)
        ach = frame_bytes / (kernel_ms / 1e3) / 1e9
        step_ach = frame_bytes / (elapsed / a.steps) / 1e9  # frames overlap over the lanes
        roof.update(achieved_per_step=round(step_ach, 2), frac_per_step=round(step_ach / HBM_PEAK_GBS, 5))
        roof.update(traffic=frame_bytes, achieved=round(ach, 2), frac=round(ach / HBM_PEAK_GBS, 5),
                    achieved_from=f"measured HBM bytes of the frame's four kernels (rocprofv3 --pmc, "
                                  f"{tr.get('source', '?')}) / live kernel_ms",
                    per_kernel={k: per[k] for k in hw1_kernels})
        for k in ("issue", "binding"):
            if tr.get(k):
                roof[f"render_kernel_{k}"] = tr[k]
    else:
        roof.update(traffic=None, achieved=None, frac=None,
                    achieved_from=f"no PMC traffic profiled for {instance} on {a.config} (profiles/traffic.json)")
    line["roofline"] = roof
    line["timing"] = {"kernel_ms": round(kernel_ms, 4), "kernel_ms_min": round(float(kms.min()), 4),
                      "host_submit_ms_per_frame": round(submit_ms, 4),
                      # host time blocked in rt_hw1_wait per frame: ~0 when the host is what limits the rate
                      "host_wait_ms_per_frame": round(nxt["wait_s"] / a.steps * 1e3, 4)}
    if not a.no_parity:
        gdir = REPO / "tests" / "golden" / "scenes" / HW1_GOLDEN[a.config]
        want = gzip.open(gdir / "image.ppm.gz").read()
        body = last_host.numpy().tobytes()
        got = rt.p6_header(W, H) + body
        wb = np.frombuffer(want[len(rt.p6_header(W, H)):], np.uint8).astype(int)
        line["parity"] = {"vs": f"reference HW1 output written by ppm_p6 (tests/golden/scenes/{HW1_GOLDEN[a.config]})",
                          "timed_step_ppm_identical": got == want,
                          "timed_step_ppm_maxabs": int(np.abs(np.frombuffer(body, np.uint8).astype(int) - wb).max())}
    if not a.no_cpu_baseline:
        line["cpu_baseline"] = hw1_cpu_baseline(mesh, c, W, H)
        line["speedup_vs_cpu_baseline"] = round(value / line["cpu_baseline"]["value"], 2)
    sc.close()
    print(json.dumps(line), flush=True)


def main():
    a = parse()
    for kv in a.tune:
        k, _, v = kv.partition("=")
        rt.set_tuning(k, float(v))
    assert set(HW1_CONFIG_NAMES) == set(configs.HW1_CONFIGS), "HW1_CONFIG_NAMES out of date"
    if a.config in configs.HW1_CONFIGS:
        return hw1_main(a)
    ctx = Ctx(a)
    world, rank = ctx.world, ctx.rank
    cfg = configs.G_CONFIGS[a.config]
    sp = configs.scene_path(cfg["scene"])
    hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
    cam = hs.camera(cfg["width"], cfg["height"])
    W, H, spp = cam.pixel_width, cam.pixel_height, cfg["spp"]
    if a.pair is None:
        # One frame per launch at N = 1; two frames per launch for the band
        # shards of an N-GPU frame, which gain most (8 shards: render kernel 0.0506 vs 0.0745 ms
        # per frame, 2 shards 0.0731 vs 0.0922, scripts/pair_shards.py,
        # profiles/r05/exp/pair_shards_c3.log).  On one GPU pairs were level with single frames in
        # the driver's 20-step window (BENCH_r05: 0.162 vs 0.1599 ms/step) and double the frame
        # latency (0.79 vs 0.42 ms), so the single-frame mode is the N = 1 headline (VERDICT r05
        # item 2); the other mode is measured beside it (timing.other_submission), --pair 1 / 0
        # chooses.  A pair renders the config's one camera twice (the workload is one fixed view).
        a.pair = 1 if PAIR_CONFIGS(a, cfg) and world > 1 else 0
    PAIR["on"] = bool(a.pair)
    if a.depth is None:  # frames in flight (N = 1: depth 3 keeps the host's waits off the critical
        # path; the driver's 20-step command: 0.171 ms/step vs 0.174-0.262 at depth 2 with SDMA copies,
        # profiles/r05/exp/driver_cmd_depth_ab.log); pairs: 6, the host two pairs ahead (at 4 the next
        # pair's submit waited for the previous pair's copies: 0.157-0.165 ms/step vs 0.151 at 6,
        # profiles/r05/exp/pair_ab_c3.log)
        a.depth = 6 if a.pair else 3

    comm = a.comm
    fallback = None
    if comm == "torch" and not ctx.multiproc and world > 1:
        raise SystemExit("bench: --comm torch needs one process per GPU (torchrun)")
    if comm == "native":
        try:
            res = native(a, hs, cam, cfg, ctx)
        except rt.RTError as e:
            if world == 1 or not ctx.multiproc or not a.allow_fallback:
                print(f"bench: native {world}-GPU path failed: {e}", file=sys.stderr, flush=True)
                raise SystemExit(2)
            # --allow-fallback: the process group is gloo (the native path's control plane)
            a.backend = "gloo"
            fallback = f"native path failed ({e}); torch.distributed gather (gloo, CPU-staged) used (--allow-fallback)"
            print(f"bench: {fallback}", file=sys.stderr, flush=True)
            comm = "torch"
    if comm == "torch":
        a.deliver = a.gather_payload
        res = torch_path(a, hs, cam, cfg, world, rank, ctx.devices[0], ctx.dev)

    elapsed = res["elapsed"]
    vals = [elapsed, res["kernel_ms"], res["frame_ms"]]
    if "render_only_s" in res:
        vals.append(res["render_only_s"])
        vals.append(res["other_payload"]["s"])
    if "other_mode" in res:
        vals.append(res["other_mode"]["s"])
    m = ctx.max(vals)
    elapsed, kernel_ms, frame_ms = m[0], m[1], m[2]
    per_rank = None
    if ctx.multiproc:  # every rank's own kernel / frame ms, to set beside the one-GPU shard estimates
        mine = {"rank": rank, "device": ctx.devices[0], "kernel_ms": round(res["kernel_ms"], 4),
                "frame_ms": round(res["frame_ms"], 4), "elapsed_s": round(res["elapsed"], 6)}
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
    shards = lbvh = None
    if world == 1 and not a.no_extras and comm == "native":
        shards = band_shards(hs, cam, cfg, ctx.devices[0])
        lbvh = lbvh_times(hs, ctx.devices[0])

    samples = W * H * spp
    value = samples * a.steps / elapsed / 1e6
    line = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "warmup_frames_run": res.get("warmup_frames_run", a.warmup),
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32+f64",
        "data": ("synthetic seeded 1,048,576-triangle heightfield" if a.config == "c5" else
                 "synthetic=false: this repo's two-light scene over the reference's cornellbox.obj"
                 if a.config == "cornell" else
                 f"synthetic=false: {cfg['scene']} as the reference ships it (meshes and scene JSON are reference assets)"),
    }
    gpath = res["gather_path"]
    line["config"] = {
        "workload": f"{a.config if world == 1 or a.config != 'c3' else 'c4'}: {cfg['scene']} {W}x{H}x{spp}spp "
                    f"max_bounces={cfg['max_depth']}"
                    + ((", diffuse bounces" if hs.settings["diffuse_bounce"] else ", mirror bounces")
                       if cfg["max_depth"] > 1 else "")
                    + f", Lambert/Blinn-Phong + 1 hard shadow ray per light ({len(hs.lights)} light(s))",
        "triangles": hs.num_triangles, "bands": f"{BAND_ROWS}-row bands round-robin over {world} GPU(s)",
        "processes": world if ctx.multiproc else 1,
        "devices": "one per process" if ctx.multiproc else list(ctx.devices),
        "step_delivers": (f"the frame's {'P6 samples (PPM body)' if a.deliver == 'p6' else 'float framebuffer'}"
                          " in rank 0's host memory, every timed frame waited for"),
        "comm": (f"native rt_renderer, gather={gpath}: {COMM_TEXT[gpath]}" if comm == "native" else gpath),
        "copy_engine": (("sdma: P6 copies queued through the HSA runtime on a DMA engine once each frame's "
                         "render event fires (no CU slots)" if res.get("copy_engine") == "sdma" else
                         "runtime: hipMemcpyAsync (blit kernels on the CUs)") if comm == "native" else None),
        "pipeline_depth": a.depth if comm == "native" else 2, "kernel": a.kernel,
        "frames_per_submit": 2 if (a.pair and comm == "native") else 1}
    if a.pair and comm == "native":
        line["config"]["pair_cameras"] = ("identical: both frames of a pair are the config's one camera "
                                          "(DESIGN.md §4.15 measures a pair of two different cameras)")
    if a.share_gpu and world > 1:
        line["config"]["rehearsal"] = "--share-gpu: ranks share GPUs (not a multi-GPU measurement)"
    if a.tune:
        line["config"]["tuning"] = dict(kv.partition("=")[::2] for kv in a.tune)
    if fallback:
        line["config"]["fallback"] = fallback
    if res.get("gather_note"):
        line["config"]["gather_note"] = res["gather_note"]
    per_gpu_samples = samples / world
    bps = configs.BYTES_PER_SAMPLE.get(a.config)
    instance = res.get("kernel_instance")
    tr = load_traffic(Path(a.traffic_file), a.config, instance) if world == 1 else None
    traffic = tr.get("bytes_per_launch") if tr else None
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "traffic": traffic,
            "kernel": instance or "render_tiles_kernel", "kernel_ms": round(kernel_ms, 4),
            "frame_ms": round(frame_ms, 4),
            # a pair kernel (rt_renderer_submit_pair) renders two frames per launch: its kernel_ms
            # and bytes per launch are both per two frames
            "frames_per_launch": 2 if (instance or "").startswith("render_pair_kernel") else 1}
    if traffic:
        ach = traffic / (kernel_ms / 1e3) / 1e9
        roof.update(achieved=round(ach, 2), frac=round(ach / HBM_PEAK_GBS, 5),
                    achieved_from="measured HBM bytes per launch (rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE, "
                                  f"{tr.get('source', '?')}) / live kernel_ms")
        if roof["frames_per_launch"] > 1:
            # a pair launch fetches about what one frame's launch does (the scene's records once),
            # so its GB/s falls while the bytes per frame halve
            roof["traffic_per_frame"] = round(traffic / roof["frames_per_launch"])
        if tr.get("compulsory_bytes_per_launch"):
            roof["compulsory_bytes_per_launch"] = tr["compulsory_bytes_per_launch"]
            roof["compulsory_GBps"] = round(tr["compulsory_bytes_per_launch"] / (kernel_ms / 1e3) / 1e9, 2)
    else:
        roof.update(achieved=None, frac=None,
                    achieved_from=f"no PMC traffic profiled for {instance} on {a.config} (profiles/traffic.json)")
    if bps:
        roof["reference_equivalent_GBps"] = round(bps * per_gpu_samples * roof["frames_per_launch"] /
                                                  (kernel_ms / 1e3) / 1e9, 2)
        roof["reference_equivalent_note"] = (f"SURVEY.md §8(d) reference-layout model, {bps:.2f} B/sample: the "
                                             "bytes the reference's per-ray traversal would fetch, not this "
                                             "kernel's traffic")
    if tr and tr.get("issue"):
        roof["issue"] = tr["issue"]
        roof["binding"] = tr.get("binding")
    line["roofline"] = roof
    if not a.no_extras and rank == 0:
        # rays: camera + shadow (+ bounce) rays of one frame, counted on the
        # device by rt_count_rays_ex outside the timed region, over the same wall time; the
        # traced rate counts only camera rays that are traversed (the culling passes prove the
        # others miss: their samples are written without a traversal)
        ds = rt.DeviceScene.from_host(hs, device=ctx.devices[0])
        try:
            rays = ds.count_rays(cam, spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                                 diffuse_bounce=hs.settings["diffuse_bounce"])
            if a.config in GOLDEN_FULL and not a.no_parity:
                line["parity_primary_hits"] = primary_hit_parity(ds, cam, cfg, hs, GOLDEN_FULL[a.config])
        finally:
            ds.close()
        total = rays["camera"] + rays["shadow"] + rays["bounce"]
        traced = rays["camera_traced"] + rays["shadow"] + rays["bounce"]
        line["rays_per_frame"] = rays
        line["total_rays_per_s"] = round(total * a.steps / elapsed / 1e6, 3)
        line["traced_rays_per_s"] = round(traced * a.steps / elapsed / 1e6, 3)
        line["culled_sample_frac"] = round(1.0 - rays["camera_traced"] / max(rays["camera"], 1), 5)
        line["rays_unit"] = ("Mrays/s: total = camera + shadow + bounce rays; traced = the same with only the "
                             "camera rays of tiles the exact culling passes leave to the render kernel")
    extra = {"kernel_ms": round(kernel_ms, 4), "frame_ms": round(frame_ms, 4)}
    if roof.get("frames_per_launch", 1) > 1:  # kernel_ms is per launch: two frames
        extra["kernel_ms_per_frame"] = round(kernel_ms / roof["frames_per_launch"], 4)
        extra["kernel_ms_note"] = "kernel_ms: one render_pair_kernel launch, two frames (DESIGN.md §4.15)"
    for k in ("gather_ms", "deliver_ms", "frame_latency_ms"):
        if k in res:
            extra[k] = round(res[k], 4)
    if len(res.get("kernel_ms_local", [])) > 1:
        extra["kernel_ms_per_local_rank"] = [round(x, 4) for x in res["kernel_ms_local"]]
    if per_rank:
        extra["per_rank"] = per_rank
    if "render_only_s" in res:
        extra["render_only_value"] = round(samples * a.steps / m[3] / 1e6, 3)
        op = res["other_payload"]
        extra[f"{op['deliver']}_host_value"] = round(samples * op["steps"] / m[4] / 1e6, 3)
    if "other_mode" in res:
        om = res["other_mode"]
        extra["other_submission"] = {
            "mode": "two frames per render launch (rt_renderer_submit_pair)" if om["pair"] else "one frame per launch",
            "depth": om["depth"], "value": round(samples * a.steps / m[5] / 1e6, 3),
            "ms_per_step": round(m[5] / a.steps * 1e3, 4),
            "frame_latency_ms": None if om["frame_latency_ms"] is None else round(om["frame_latency_ms"], 4)}
    extra["live_tiles"] = res.get("live_tiles")
    if "prepass_ms" in res:
        extra["prepass_ms"] = round(res["prepass_ms"], 4)
        extra["heavy_tiles"] = res["heavy_tiles"]
        extra["note"] = ("frame_ms = the frame's device work: cull pre-passes (prep stream, overlapping the "
                         "previous frame's render kernel) + render kernel; ms_per_step is the delivered rate")
    if shards:
        extra["band_shards_one_gpu"] = shards
    line["timing"] = extra
    if lbvh:
        line["lbvh_build"] = lbvh

    if not a.no_parity and a.config in GOLDEN_FULL and rank == 0:
        gdir = REPO / "tests" / "golden" / "scenes" / GOLDEN_FULL[a.config]
        gmeta = json.loads((gdir / "meta.json").read_text())
        ref = (np.frombuffer(gzip.open(gdir / "fb.f32.gz").read(), np.float32).reshape(H, W, 3)
               if (gdir / "fb.f32.gz").exists() else None)
        ppm_ref = golden_ppm(a.config)
        par = {"vs": f"reference CPU render() output (tests/golden/scenes/{GOLDEN_FULL[a.config]}"
                     + ("" if ref is not None else ": sha256 of the float frame and P6 file") + ")"}

        def p6_check(body: bytes, tag: str):
            if ppm_ref is not None:
                got = np.frombuffer(body, np.uint8).astype(int)
                want = np.frombuffer(ppm_ref[len(rt.p6_header(W, H)):], np.uint8).astype(int)
                par[f"{tag}ppm_maxabs"] = int(np.abs(got - want).max())
            par[f"{tag}ppm_identical"] = ppm_matches_golden(a.config, rt.p6_header(W, H) + body)

        def f32_check(body: bytes, tag: str):
            if ref is None:
                par[f"{tag}rgb_sha256_equal"] = hashlib.sha256(body).hexdigest() == gmeta["sha256"]["fb.f32"]
                return
            fr = np.frombuffer(body, np.float32).reshape(H, W, 3)
            par[f"{tag}rgb_maxabs"] = float(np.abs(fr - ref).max())
            par[f"{tag}rgb_bitexact_frac"] = float((fr.view(np.uint32) == ref.view(np.uint32)).mean())

        if a.deliver == "p6":
            p6_check(res["frame_bytes"], "timed_step_")
            if "other_bytes" in res:
                f32_check(res["other_bytes"], "")
        else:
            f32_check(res["frame_bytes"], "timed_step_")
            if "other_bytes" in res:
                p6_check(res["other_bytes"], "")
        line["parity"] = par
    if world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(hs, cam, cfg)
        line["speedup_vs_cpu_baseline"] = round(value / line["cpu_baseline"]["value"], 2)
    if world > 1 and comm == "native" and ctx.distinct and not a.no_extras and not a.no_rccl_leg \
            and res["gather_path"] != "rccl":
        # last, under a watchdog: a collective that never completes must not cost the line
        import threading

        def _expire():
            if rank == 0:
                line["rccl_gather"] = {"error": "timed out after 180 s (RCCL leg abandoned)"}
                print(json.dumps(line), flush=True)
            os._exit(0)

        wd = threading.Timer(180.0, _expire)
        wd.daemon = True
        wd.start()
        line["rccl_gather"] = rccl_leg(a, hs, cam, cfg, ctx)
        wd.cancel()
    if ctx.multiproc:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
