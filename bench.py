#!/usr/bin/env python3
"""Headline benchmark: Mrays/s (camera samples/s) of the per-pixel ray path at
1920x1080x16 spp on the frog scene (BASELINE.json configs[2]; c4 when N > 1).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c5] [--kernel wave|lane]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N ...

A step = one full frame delivered on rank 0: every rank renders its image bands (rows cut
into 8-row bands, band b -> rank b % N) with the HIP kernels into device memory, which also
write the strip's P6 samples (write_p6 semantics, fused into the render and cull kernels); the
byte strips are gathered to
rank 0 over RCCL (torch.distributed, backend "nccl") and un-permuted there on the GPU
(--gather f32 gathers the float strips instead).  With two strip buffers the gather of
frame k overlaps the render of frame k+1, and all K gathers finish inside the timed region.
Scene upload and BVH build are
outside the timed region (as G/src/main.cu:362-378 times only render()).  Inputs are
resident in HBM when timing starts.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import platform
import subprocess
import sys
import tempfile
import time
from pathlib import Path

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import before librt_mi355x: one HIP runtime in the process)
import torch.distributed as dist  # noqa: E402

import raytracinginonesemester_amd as rt  # noqa: E402
from raytracinginonesemester_amd import configs  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
BAND_ROWS = 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~35 ms of frames: a steadier average
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(configs.G_CONFIGS))
    ap.add_argument("--kernel", default="auto", choices=["auto", "wave", "lane"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: CPU-staged gather (lets N ranks share one GPU to exercise the N>1 path)")
    ap.add_argument("--gather", default="p6", choices=["p6", "f32"],
                    help="what a step delivers on rank 0: p6 = the frame's P6 samples (each rank quantises "
                         "its strip on its GPU, the bytes are gathered and un-permuted; SURVEY.md §8(f) #3), "
                         "f32 = the float framebuffer strips")
    ap.add_argument("--traffic-file", default=str(REPO / "profiles" / "traffic.json"),
                    help="per-launch HBM bytes measured by rocprofv3 --pmc (see DESIGN.md)")
    return ap.parse_args()


def cpu_baseline(hs, cam, cfg) -> dict:
    """The oracle restatement (bit-exact to the reference build, tests/test_oracle.py) timed on
    this host's cores over the full frame, plus the reference's own CPU render() built from its
    sources (oracle/_ref/ref_g, 1 thread, as shipped) when present."""
    from oracle import pyoracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    b = cam.basis()
    oc = orc.camera_from_basis(b["center"], b["pixel00_loc"], b["pixel_delta_u"], b["pixel_delta_v"],
                               cam.pixel_width, cam.pixel_height)
    # bounded sample: a band of rows through the frame centre (the frog), then all rows for c3
    H, W, spp = cam.pixel_height, cam.pixel_width, cfg["spp"]
    rows = (0, H) if cfg is configs.G_CONFIGS["c3"] else (H // 2 - 32, H // 2 + 32)
    # repeat the sample until ~10 s of CPU work (at least once), so the rate is not a blip
    reps, t0 = 0, time.perf_counter()
    while True:
        orc.render_g(hs.num_triangles, oc, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials,
                     hs.lights, spp=spp, max_depth=cfg["max_depth"], miss=hs.settings["miss_color"], rows=rows,
                     threads=threads)
        reps += 1
        if time.perf_counter() - t0 >= 10.0:
            break
    dt = time.perf_counter() - t0
    n = (rows[1] - rows[0]) * W * spp * reps
    out = {"value": n / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": f"oracle/rt_oracle.c (bit-exact restatement) rows {rows[0]}..{rows[1]} of "
                     f"{W}x{H}x{spp}, {reps} pass(es), {n} samples, {dt:.2f} s, OpenMP {threads} threads"}
    ref = REPO / "oracle" / "_ref" / "ref_g"
    if ref.exists() and cfg is configs.G_CONFIGS["c3"]:
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
    out["host_cpu"] = platform.processor() or platform.machine()
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # gloo rehearsal: several ranks may share one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    cfg = configs.G_CONFIGS[a.config]
    sp = configs.scene_path(cfg["scene"])
    hs = rt.HostScene.load_json(sp, REPO if sp.parent == configs.SCENES else sp.parent)
    cam = hs.camera(cfg["width"], cfg["height"])
    W, H, spp = cam.pixel_width, cam.pixel_height, cfg["spp"]
    kernel = {"auto": rt.RT_KERNEL_AUTO, "wave": rt.RT_KERNEL_WAVE, "lane": rt.RT_KERNEL_LANE}[a.kernel]
    ds = rt.DeviceScene.from_host(hs, device=local)
    opts, _jit = ds.make_opts(spp=spp, max_depth=cfg["max_depth"], miss_color=hs.settings["miss_color"],
                              band_rows=BAND_ROWS, band_index=rank, band_count=world, kernel=kernel)
    lib = rt._lib.lib()
    rows_of = [lib.rt_shard_rows(H, BAND_ROWS, r, world) for r in range(world)]
    max_rows = max(rows_of)
    # Two strip buffers: frame k+1 renders while frame k's strips are gathered (the collective
    # runs on its own stream; before a buffer is rendered into again, the current stream waits
    # for that buffer's previous gather — a stream dependency, the host does not block).
    strips = [torch.zeros((max_rows, W, 3), dtype=torch.float32, device=dev) for _ in range(2)]
    p6 = a.gather == "p6"
    rb = W * 3  # P6 bytes per row (maxval 255)
    qstrips = [torch.zeros((max_rows, rb), dtype=torch.uint8, device=dev) for _ in range(2)] if p6 else None
    gdev = dev if a.backend == "nccl" else torch.device("cpu")
    payload = qstrips if p6 else strips
    gathers = [torch.empty((world,) + tuple(payload[0].shape), dtype=payload[0].dtype, device=gdev)
               if (world > 1 and rank == 0) else None for _ in range(2)]
    p6_frame = torch.empty((H, rb), dtype=torch.uint8, device=dev) if (p6 and rank == 0 and world > 1) else None
    pending = [None, None]
    stream = torch.cuda.current_stream(dev).cuda_stream
    frames = [0]

    def finish(b):
        """Frame in buffer b is complete on rank 0 once its gather is: un-permute the P6 bands."""
        if pending[b] is None:
            return
        pending[b].wait()
        pending[b] = None
        if p6 and rank == 0:
            g = gathers[b] if a.backend == "nccl" else gathers[b].to(dev)
            rt.unpermute_strips_device(g.data_ptr(), max_rows, rb, H, BAND_ROWS, world, p6_frame.data_ptr(),
                                       False, stream)

    def step():
        b = frames[0] & 1
        frames[0] += 1
        finish(b)  # frame k-2 used these buffers
        # p6: the render and cull kernels write the strip's P6 samples themselves (fused epilogue)
        ds.render_device(cam, opts, strips[b].data_ptr(), stream=stream,
                         p6_dev_ptr=qstrips[b].data_ptr() if p6 else None)
        if world > 1:
            src = payload[b] if a.backend == "nccl" else payload[b].cpu()
            glist = list(gathers[b].unbind(0)) if rank == 0 else None
            pending[b] = dist.gather(src, gather_list=glist, dst=0, async_op=True)

    def drain():
        for b in ((frames[0]) & 1, (frames[0] + 1) & 1):  # oldest frame first
            finish(b)

    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=gdev)
    kt, ft = ds.kernel_times(a.steps), ds.frame_times(a.steps)
    kmean = torch.tensor([float(kt.mean()) if len(kt) else float("nan"),
                          float(ft.mean()) if len(ft) else float("nan")], dtype=torch.float64, device=gdev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        dist.all_reduce(kmean, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    kernel_ms, frame_ms = float(kmean[0].item()), float(kmean[1].item())

    # the frame epilogue on the devices: quantise every strip to P6 samples,
    # gather the bytes, un-permute on rank 0's GPU; timed once, outside the render metric
    from raytracinginonesemester_amd import dist as rdist
    last = (frames[0] - 1) & 1  # the buffers of the last frame
    strip = strips[last]
    rdist.gather_p6(strip, H, BAND_ROWS, world, rank, stream=stream)  # warm (allocations)
    torch.cuda.synchronize(dev)
    te0 = time.perf_counter()
    p6_bytes = rdist.gather_p6(strip, H, BAND_ROWS, world, rank, stream=stream)
    te1 = time.perf_counter()

    # the float frame on rank 0 (one more gather of the last frame's float strips, outside the
    # timed region) and the last timed frame's P6 samples, for the parity check
    frame = None
    fparts = None
    if world > 1:
        fl = [torch.empty_like(strip) for _ in range(world)] if rank == 0 else None
        src = strip if a.backend == "nccl" else strip.cpu()
        if a.backend == "gloo" and rank == 0:
            fl = [torch.empty(strip.shape, dtype=strip.dtype) for _ in range(world)]
        dist.gather(src, gather_list=fl, dst=0)
        fparts = fl
    if rank == 0:
        parts = fparts if world > 1 else [strip]
        frame = np.zeros((H, W, 3), np.float32)
        for r in range(world):
            ys = [y for y in range(H) if (y // BAND_ROWS) % world == r] if world > 1 else list(range(H))
            frame[ys] = parts[r][:len(ys)].cpu().numpy()
    step_p6 = None
    if p6 and rank == 0:
        body = (p6_frame if world > 1 else qstrips[last][:H]).cpu().numpy().tobytes()
        step_p6 = rt.p6_header(W, H) + body

    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return

    samples = W * H * spp
    value = samples * a.steps / elapsed / 1e6
    B = configs.BYTES_PER_SAMPLE[a.config]
    per_gpu_samples = samples / world
    achieved = B * per_gpu_samples / (kernel_ms / 1e3) / 1e9  # GB/s of the dominant kernel
    traffic = None
    tf = Path(a.traffic_file)
    if tf.exists() and world == 1:  # measured for the 1-GPU launch of this config
        try:
            traffic = json.loads(tf.read_text()).get(a.config, {}).get("bytes_per_launch")
        except Exception:
            traffic = None
    line = {
        "metric": "Mrays/s at 1920x1080x16spp (1/2/4/8 GPU) + PPM max-abs pixel diff",
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32+f64",
        "data": "synthetic=false: frog.obj scene (reference asset), camera/light from frog.json"
                if a.config == "c3" else "synthetic seeded 1,048,576-triangle heightfield",
        "config": {"workload": f"{a.config if world == 1 else 'c4'}: {cfg['scene']} {W}x{H}x{spp}spp "
                               f"max_bounces={cfg['max_depth']}, "
                               f"Lambert/Blinn-Phong + 1 hard shadow ray per light",
                   "triangles": hs.num_triangles, "bands": f"{BAND_ROWS}-row bands round-robin over {world} GPU(s)",
                   "gather": (f"{'RCCL' if a.backend == 'nccl' else 'gloo (CPU-staged)'} gather to rank 0"
                              if world > 1 else None),
                   "step_delivers": ("P6 samples of the frame on rank 0 (render kernels write them"
                                     + (" + gather of the byte strips + un-permute)" if world > 1 else ")")
                                     if a.gather == "p6" else "float framebuffer strips on rank 0"),
                   "kernel": a.kernel},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                     # measured HBM-side bytes per launch over the kernel time: the scene is
                     # L2-resident and nodes are fetched once per wave, so this sits far below
                     # the algorithmic rate (the kernel is VALU- / latency-bound)
                     "traffic_gbs": (round(traffic / (kernel_ms / 1e3) / 1e9, 2) if traffic else None),
                     "traffic_frac": (round(traffic / (kernel_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5) if traffic else None),
                     "kernel": "render_tiles_kernel", "kernel_ms": round(kernel_ms, 4),
                     "frame_ms": round(frame_ms, 4), "algorithmic_bytes_per_sample": round(B, 3)},
        "p6_epilogue_ms": round((te1 - te0) * 1e3, 3),
    }
    if not a.no_parity and a.config == "c3":
        ref = np.frombuffer(gzip.open(REPO / "tests" / "golden" / "scenes" / "c3_full" / "fb.f32.gz").read(),
                            np.float32).reshape(H, W, 3)
        ppm_ref = gzip.open(REPO / "tests" / "golden" / "scenes" / "c3_full" / "image.ppm.gz").read()
        pd = np.abs(np.frombuffer(p6_bytes[17:], np.uint8).astype(int) - np.frombuffer(ppm_ref[17:], np.uint8).astype(int))
        line["parity"] = {"vs": "reference CPU render() output (tests/golden/scenes/c3_full)",
                          "rgb_maxabs": float(np.abs(frame - ref).max()),
                          "rgb_bitexact_frac": float((frame.view(np.uint32) == ref.view(np.uint32)).mean()),
                          "ppm_maxabs": int(pd.max()), "ppm_identical": p6_bytes == ppm_ref,
                          "ppm_from": "device P6 epilogue (rt_ppm_quantize_device + gather + un-permute)"}
        if step_p6 is not None:
            line["parity"]["timed_step_ppm_identical"] = step_p6 == ppm_ref
    if world == 1 and not a.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(hs, cam, cfg)
        line["speedup_vs_cpu_baseline"] = round(value / line["cpu_baseline"]["value"], 2)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
