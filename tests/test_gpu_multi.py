"""Multi-GPU delivery paths and cross-frame hazards, on one GPU.

* bench.py's N-GPU modes end to end: one process driving N band shards (RT_GATHER_DIRECT), one
  process per rank under torchrun with the shared host frame (RT_GATHER_HOST_SHARED), and the
  refusal of a failed RCCL path unless --allow-fallback.  On a one-GPU box the ranks share the
  GPU (--share-gpu); the frames must still be the reference's c3 image bit for bit.
* The shared host frame between processes with pipelined frames whose cameras alternate (so
  the culled tiles differ between consecutive frames) and a frame-size change in the middle.
* Pipelined frames in one process with alternating cameras (depth 2 and 3), stream ordering of
  rt_render_device for a caller that reuses one buffer on one stream, and c5's 8-way band
  split reassembled on one GPU.
"""
from __future__ import annotations

import ctypes as C
import gzip
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, host_scene

import raytracinginonesemester_amd as rt

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parents[1]
W, H, SPP = 1920, 1080, 16


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(stdout: str) -> dict:
    return json.loads([ln for ln in stdout.splitlines() if ln.startswith("{")][-1])


def _bench(args, nproc=None, timeout=420):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    if nproc:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(REPO / "bench.py"), *args, "--tune", "peer_timeout_s=60"]
    else:
        cmd = [sys.executable, str(REPO / "bench.py"), *args, "--tune", "peer_timeout_s=60"]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=str(REPO), env=env)


def _moved(cam, dx=0.004, dz=0.003):
    return rt.Camera(tuple(np.add(cam.pos, (dx, 0.0, dz))), cam.look_at, cam.up, cam.focal_length_mm,
                     cam.sensor_height_mm, cam.pixel_width, cam.pixel_height)


def _p6_body(rgb) -> bytes:
    return rt.encode_p6(rgb)[len(rt.p6_header(rgb.shape[1], rgb.shape[0])):]


# ---- bench.py end to end ----------------------------------------------------------------
def test_bench_in_process_one_gpu():
    """--gpus 1 without a launcher: the in-process renderer, own strip to host."""
    r = _bench(["--gpus", "1", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-extras"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert "gather=direct" in line["config"]["comm"] and line["config"]["processes"] == 1
    assert line["parity"]["timed_step_ppm_identical"]


def test_bench_in_process_two_band_shards():
    """--gpus 2 in one process (band shards sharing GPU 0 here): every frame is the c3 image."""
    r = _bench(["--gpus", "2", "--share-gpu", "--steps", "5", "--warmup", "2", "--no-cpu-baseline", "--no-extras"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["devices"] == [0, 0]
    assert "rehearsal" in line["config"]
    assert line["parity"]["timed_step_ppm_identical"]


def test_bench_two_processes_shared_host_frame():
    """torchrun, 2 ranks (sharing the GPU): each rank copies its bands into the shared host frame;
    the timed P6 frame and the float frame of the second payload are the reference's."""
    r = _bench(["--gpus", "2", "--share-gpu", "--steps", "8", "--warmup", "2", "--no-cpu-baseline"], nproc=2)
    assert r.returncode == 0, r.stderr[-3000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["processes"] == 2
    assert "gather=shm" in line["config"]["comm"] and "fallback" not in line["config"]
    assert line["parity"]["timed_step_ppm_identical"] and line["parity"]["rgb_maxabs"] == 0.0
    assert line["timing"]["render_only_value"] > 0
    assert 0.9 < line["culled_sample_frac"] < 1.0 and line["traced_rays_per_s"] < line["total_rays_per_s"]
    assert not list(Path("/dev/shm").glob("rt_bench_*")), "shared frames left behind"


def test_bench_failed_rccl_is_not_silent():
    """--gather rccl with two ranks on one GPU: RCCL refuses the duplicate device.  Without
    --allow-fallback the bench exits non-zero with the RCCL error; with it, the gloo gather runs
    and the line says so."""
    r = _bench(["--gpus", "2", "--share-gpu", "--gather", "rccl", "--steps", "3", "--warmup", "1",
                "--no-cpu-baseline", "--no-extras"], nproc=2)
    assert r.returncode != 0
    assert "native 2-GPU path failed" in r.stderr and "RT_ERR_COMM" in r.stderr
    r = _bench(["--gpus", "2", "--share-gpu", "--gather", "rccl", "--allow-fallback", "--steps", "3", "--warmup",
                "1", "--no-cpu-baseline", "--no-extras"], nproc=2)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert "gloo" in line["config"]["fallback"] and line["parity"]["timed_step_ppm_identical"]


# ---- the shared host frame between processes ----------------------------------------------
def _shared_worker(rank, world, port, name, depth, q, others_wait=True):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rt.set_tuning("peer_timeout_s", 60)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hs = host_scene("frog.json")
        cams = [hs.camera(W, H), _moved(hs.camera(W, H)), hs.camera(320, 180)]
        seq = [0, 1, 0, 1, 0, 1, 2, 2, 0, 1, 0]  # alternating cameras, a resize and back
        r = rt.Renderer.from_host(hs, devices=(0,), world_size=world, rank0=rank, gather=rt.RT_GATHER_HOST_SHARED,
                                  host_frame_name=name, depth=depth)
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1)
        got = []
        pend = []
        for k, c in enumerate(seq):
            pend.append((k, r.submit(cams[c], o)))
            # drain at a size change (the renderer waits for frames in flight before resizing)
            last = k + 1 == len(seq) or seq[k + 1] // 2 != c // 2
            while pend and (len(pend) >= depth or last):
                kk, t = pend.pop(0)
                if rank != 0 and not others_wait:
                    continue  # rank 1 never waits: its resize and close must publish its copies
                addr, n = r.wait(t)
                if rank == 0:
                    got.append((kk, bytes((C.c_uint8 * n).from_address(addr))))
        r.close()
        if rank == 0:
            q.put(got)
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("depth,others_wait", [(2, True), (3, True), (2, False)])
def test_shared_host_frame_two_processes(depth, others_wait):
    """Two processes, one rank each, into the shared host frame.  others_wait=False: rank 1
    never calls wait (the header gives non-zero ranks nothing to wait for); its copies reach
    rank 0 through the slot reuse, the resize and close alone."""
    hs = host_scene("frog.json")
    ds = rt.DeviceScene.from_host(hs, device=0)
    cams = [hs.camera(W, H), _moved(hs.camera(W, H)), hs.camera(320, 180)]
    want = [_p6_body(ds.render(c, spp=SPP, max_depth=1)) for c in cams]
    ds.close()
    ppm = gzip.open(GOLDEN / "scenes" / "c3_full" / "image.ppm.gz").read()
    assert want[0] == ppm[17:] and want[1] != want[0]
    seq = [0, 1, 0, 1, 0, 1, 2, 2, 0, 1, 0]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    name = f"/rt_test_{os.getpid()}_{depth}_{int(others_wait)}"
    procs = [ctx.Process(target=_shared_worker, args=(rk, 2, port, name, depth, q, others_wait)) for rk in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [k for k, _ in got] == list(range(len(seq)))
    for k, body in got:
        assert body == want[seq[k]], f"frame {k} (camera {seq[k]})"
    assert not list(Path("/dev/shm").glob(name[1:] + ".g*")), "shared frames left behind"


def _shared_pair_worker(rank, world, port, name, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rt.set_tuning("peer_timeout_s", 60)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        hs = host_scene("frog.json")
        cams = [hs.camera(W, H), _moved(hs.camera(W, H))]
        r = rt.Renderer.from_host(hs, devices=(0,), world_size=world, rank0=rank, gather=rt.RT_GATHER_HOST_SHARED,
                                  host_frame_name=name, depth=4)
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1)
        got, pend = [], []
        for k, (a, b) in enumerate([(0, 1), (1, 0), (0, 0), (1, 1), (0, 1)]):
            while len(pend) > 2:
                kk, t = pend.pop(0)
                addr, n = r.wait(t)
                if rank == 0:
                    got.append((kk, bytes((C.c_uint8 * n).from_address(addr))))
            ta, tb = r.submit_pair(cams[a], cams[b], o)
            pend += [(a, ta), (b, tb)]
        for kk, t in pend:
            addr, n = r.wait(t)
            if rank == 0:
                got.append((kk, bytes((C.c_uint8 * n).from_address(addr))))
        r.close()
        if rank == 0:
            q.put(got)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shared_host_frame_pairs_two_processes():
    """rt_renderer_submit_pair in two processes (one band rank each, the pair kernel on each
    rank's shard) into the shared host frame: every frame the single-frame image."""
    hs = host_scene("frog.json")
    ds = rt.DeviceScene.from_host(hs, device=0)
    want = [_p6_body(ds.render(c, spp=SPP, max_depth=1)) for c in (hs.camera(W, H), _moved(hs.camera(W, H)))]
    ds.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    name = f"/rt_test_pair_{os.getpid()}"
    procs = [ctx.Process(target=_shared_pair_worker, args=(rk, 2, port, name, q)) for rk in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(got) == 10
    for k, body in got:
        assert body == want[k], f"camera {k}"
    assert not list(Path("/dev/shm").glob(name[1:] + ".g*")), "shared frames left behind"


def test_shared_host_frame_needs_a_name():
    hs = host_scene("frog.json")
    with pytest.raises(rt.RTError) as e:
        rt.Renderer.from_host(hs, devices=(0,), world_size=2, rank0=0, gather=rt.RT_GATHER_HOST_SHARED)
    assert e.value.code == -1
    with pytest.raises(rt.RTError) as e:
        rt.Renderer.from_host(hs, devices=(0,), world_size=2, rank0=0, gather=rt.RT_GATHER_HOST_SHARED,
                              host_frame_name="/x", deliver=rt.RT_DELIVER_DEVICE)
    assert e.value.code == -7


# ---- one process: cross-frame hazards ----------------------------------------------------
@pytest.mark.parametrize("devices", [(0,), (0, 0)])
@pytest.mark.parametrize("depth", [2, 3])
def test_pipelined_alternating_cameras(devices, depth):
    """Frames in flight whose cameras alternate: the culled tiles, heavy lists and tile costs
    differ from frame to frame, so a cross-frame hazard (pre-passes of frame k+1 over frame k's
    buffers, slot reuse) would corrupt a delivered frame."""
    hs = host_scene("frog.json")
    ds = rt.DeviceScene.from_host(hs, device=0)
    cams = [hs.camera(W, H), _moved(hs.camera(W, H), -0.006, 0.004)]
    want = [_p6_body(ds.render(c, spp=SPP, max_depth=1)) for c in cams]
    ds.close()
    r = rt.Renderer.from_host(hs, devices=devices, gather=rt.RT_GATHER_DIRECT, depth=depth)
    try:
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1)
        pend = []
        for k in range(12):
            pend.append((k, r.submit(cams[k % 2], o)))
            if len(pend) >= depth:
                kk, t = pend.pop(0)
                addr, n = r.wait(t)
                assert bytes((C.c_uint8 * n).from_address(addr)) == want[kk % 2], f"frame {kk}"
        for kk, t in pend:
            addr, n = r.wait(t)
            assert bytes((C.c_uint8 * n).from_address(addr)) == want[kk % 2], f"frame {kk}"
    finally:
        r.close()


@pytest.mark.parametrize("threads", ["0", "1"])
def test_in_process_submission_threads(threads, tune):
    """Several ranks in one process, their per-rank host work on submission threads (the default
    over distinct GPUs, forced here for band shards sharing GPU 0) or on the calling thread:
    pipelined frames with alternating cameras are the single-frame images."""
    tune(renderer_threads=int(threads))
    hs = host_scene("frog.json")
    ds = rt.DeviceScene.from_host(hs, device=0)
    cams = [hs.camera(W, H), _moved(hs.camera(W, H), 0.005, 0.001)]
    want = [_p6_body(ds.render(c, spp=SPP, max_depth=1)) for c in cams]
    ds.close()
    r = rt.Renderer.from_host(hs, devices=(0,) * 4, gather=rt.RT_GATHER_DIRECT, depth=3)
    try:
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1)
        pend = []
        for k in range(9):
            pend.append((k, r.submit(cams[k % 2], o)))
            if len(pend) >= 3:
                kk, t = pend.pop(0)
                addr, n = r.wait(t)
                assert bytes((C.c_uint8 * n).from_address(addr)) == want[kk % 2], f"frame {kk}"
        for kk, t in pend:
            addr, n = r.wait(t)
            assert bytes((C.c_uint8 * n).from_address(addr)) == want[kk % 2], f"frame {kk}"
    finally:
        r.close()


def test_render_device_is_stream_ordered():
    """One buffer reused on one stream: fill, render A, copy, render B, copy.  Frame B's culling
    pre-passes (on the scene's own stream) must not write the buffer before copy A read it, nor
    before the fill."""
    hs = host_scene("frog.json")
    ds = rt.DeviceScene.from_host(hs, device=0)
    cams = [hs.camera(W, H), _moved(hs.camera(W, H), 0.008, -0.002)]
    want = [ds.render(c, spp=SPP, max_depth=1) for c in cams]
    o, _j = ds.make_opts(spp=SPP, max_depth=1)
    st = torch.cuda.Stream()
    buf = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    outs = []
    with torch.cuda.stream(st):
        for k in range(6):
            buf.fill_(float(k + 7))
            ds.render_device(cams[k % 2], o, buf.data_ptr(), stream=st.cuda_stream)
            outs.append(buf.clone())
    torch.cuda.synchronize()
    for k, x in enumerate(outs):
        assert x.cpu().numpy().view(np.uint32).tobytes() == want[k % 2].view(np.uint32).tobytes(), f"frame {k}"
    ds.close()


def test_wait_rejects_ticket_from_before_a_resize():
    hs = host_scene("frog.json")
    r = rt.Renderer.from_host(hs, devices=(0,), depth=3)
    try:
        o, _j = rt.DeviceScene.make_opts(spp=4, max_depth=1)
        t0 = r.submit(hs.camera(64, 36), o)
        t1 = r.submit(hs.camera(96, 54), o)  # new geometry: buffers reallocated
        with pytest.raises(rt.RTError, match="change of the frame size"):
            r.wait(t0)
        addr, n = r.wait(t1)
        assert n == 96 * 54 * 3
    finally:
        r.close()


def test_borrowed_scene_is_invalidated_by_renderer_close():
    hs = host_scene("frog.json")
    r = rt.Renderer.from_host(hs, devices=(0,))
    sc = r.scene(0)
    r.render(hs.camera(64, 36), spp=4)
    assert len(sc.kernel_times(1)) == 1
    r.close()
    with pytest.raises(rt.RTError, match="closed"):
        sc.kernel_times(1)


def test_c5_eight_band_shards_reassemble():
    """c5 (1,048,576 triangles, 3840x2160x64) split 8 ways (half waves, as on 8 GPUs) on one GPU:
    the reassembled P6 frame equals the one-shard frame bit for bit."""
    hs = host_scene("heightfield_c5.json")
    cam = hs.camera(3840, 2160)
    kw = dict(spp=64, max_depth=1, miss_color=hs.settings["miss_color"])
    frames = []
    for devices in [(0,), (0,) * 8]:
        r = rt.Renderer.from_host(hs, devices=devices, gather=rt.RT_GATHER_DIRECT)
        try:
            frames.append(r.render(cam, **kw))
        finally:
            r.close()
    assert frames[0].shape == (2160, 3840, 3)
    assert np.array_equal(frames[0], frames[1])
