"""The frame renderer (rt_renderer, include/rt_mi355x.h) through the C ABI: render(scene, camera)
-> frame in host memory, sharded over band ranks, gathered over RCCL or copied per rank.

Bar: the delivered frame equals the reference's own c3 output bit for bit
(tests/golden/scenes/c3_full: the float framebuffer of G/include/query.cu:130-166 and the P6
file write_p6 made of it), for every rank count, gather path, delivery kind and pipeline depth.
On one GPU several ranks share device 0 (RT_GATHER_DIRECT); the RCCL path runs at world 1 with
rank 0's strip sent to itself (RT_RENDERER_SELF_SEND), which exercises the grouped
ncclSend/ncclRecv sequence the N-GPU job uses.
"""
from __future__ import annotations

import ctypes as C
import gzip

import numpy as np
import pytest
import torch

from conftest import GOLDEN, host_scene, oracle_camera
from oracle import pyoracle as orc

import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import _lib as L

pytestmark = pytest.mark.gpu

W, H, SPP = 1920, 1080, 16


@pytest.fixture(scope="module")
def frog():
    return host_scene("frog.json")


@pytest.fixture(scope="module")
def golden():
    fb = np.frombuffer(gzip.open(GOLDEN / "scenes" / "c3_full" / "fb.f32.gz").read(), np.float32).reshape(H, W, 3)
    ppm = gzip.open(GOLDEN / "scenes" / "c3_full" / "image.ppm.gz").read()
    return fb, np.frombuffer(ppm[17:], np.uint8).reshape(H, W, 3)


def _opts(hs, spp=SPP, max_depth=1):
    o, jit = rt.DeviceScene.make_opts(spp=spp, max_depth=max_depth, miss_color=hs.settings["miss_color"])
    return o, jit


@pytest.mark.parametrize("devices", [(0,), (0, 0), (0, 0, 0), (0, 0, 0, 0), (0,) * 8])
def test_direct_bands_reassemble_p6(frog, golden, devices):
    """Band shards for world 1/2/3/4/8 on one GPU, each rank copying its bands into the host frame."""
    r = rt.Renderer.from_host(frog, devices=devices, gather=rt.RT_GATHER_DIRECT)
    try:
        p6 = r.render(frog.camera(W, H), spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
        assert np.array_equal(p6, golden[1]), f"{len(devices)} ranks: P6 differs from the reference image"
        # each rank's share of the work, for the record
        for i in range(r.local_ranks):
            assert len(r.scene(i).frame_times(1)) == 1
    finally:
        r.close()


@pytest.mark.parametrize("devices", [(0,), (0, 0, 0)])
def test_direct_bands_reassemble_f32(frog, golden, devices):
    r = rt.Renderer.from_host(frog, devices=devices, gather=rt.RT_GATHER_DIRECT, deliver=rt.RT_DELIVER_F32)
    try:
        fb = r.render(frog.camera(W, H), spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
        assert fb.view(np.uint32).tobytes() == golden[0].view(np.uint32).tobytes()
    finally:
        r.close()


def test_rccl_self_send(frog, golden):
    """RCCL path at world 1: ncclCommInitAll, grouped send/recv of the strip to rank 0, 2-D copy out."""
    r = rt.Renderer.from_host(frog, devices=(0,), gather=rt.RT_GATHER_RCCL, flags=rt.RT_RENDERER_SELF_SEND)
    try:
        cam = frog.camera(W, H)
        for _ in range(3):
            p6 = r.render(cam, spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
            assert np.array_equal(p6, golden[1])
        g = r.times(rt.RT_TIME_GATHER, 3)
        assert len(g) == 3 and np.all(g >= 0)
    finally:
        r.close()


def test_rccl_multiprocess_id_world1(frog, golden):
    """The multi-process form (ncclCommInitRank with a shared unique id) at world 1."""
    uid = rt.comm_unique_id()
    assert len(uid) == 128
    r = rt.Renderer.from_host(frog, devices=(0,), world_size=1, rank0=0, unique_id=uid, gather=rt.RT_GATHER_RCCL,
                              flags=rt.RT_RENDERER_SELF_SEND)
    try:
        p6 = r.render(frog.camera(W, H), spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
        assert np.array_equal(p6, golden[1])
    finally:
        r.close()


def test_rccl_rejects_repeated_devices(frog):
    with pytest.raises(rt.RTError) as e:
        rt.Renderer.from_host(frog, devices=(0, 0), gather=rt.RT_GATHER_RCCL)
    assert e.value.code == -7


def test_pipelined_frames_all_identical(frog, golden):
    """depth 3: frames k+1, k+2 render while frame k is copied; every delivered frame is the image."""
    r = rt.Renderer.from_host(frog, devices=(0, 0), gather=rt.RT_GATHER_DIRECT, depth=3)
    try:
        cam = frog.camera(W, H)
        o, _j = _opts(frog)
        tickets = [r.submit(cam, o) for _ in range(2)]
        n_checked = 0
        for k in range(10):
            t = tickets.pop(0)
            addr, n = r.wait(t)
            assert n == W * H * 3
            got = np.ctypeslib.as_array((C.c_uint8 * n).from_address(addr)).reshape(H, W, 3)
            assert np.array_equal(got, golden[1]), f"frame {t}"
            n_checked += 1
            tickets.append(r.submit(cam, o))
        for t in tickets:
            r.wait(t)
        assert n_checked == 10
        d = r.times(rt.RT_TIME_DELIVER, 12)
        f = r.times(rt.RT_TIME_FRAME, 12)
        assert len(d) == 12 and len(f) == 12 and np.all(f >= d)
    finally:
        r.close()


def test_overlapped_frames_long_pipelined_run(frog, golden, tune):
    """RT_TUNE_OVERLAP_FRAMES=1 over a long pipelined run (consecutive render kernels
    overlap on different render streams, so the pre-pass gate is off; a gate word overwritten by
    a late frame would hang the prep stream within a few hundred frames): 400 frames at depth 3,
    every 50th checked against the reference's frame."""
    tune(overlap_frames=1)
    r = rt.Renderer.from_host(frog, devices=(0,), depth=3, deliver=rt.RT_DELIVER_P6)
    try:
        cam = frog.camera(W, H)
        o, _j = _opts(frog)
        want = golden[1].tobytes()
        pend, checked = [], 0
        for k in range(400):
            pend.append((k, r.submit(cam, o)))
            if len(pend) >= 3:
                kk, t = pend.pop(0)
                addr, n = r.wait(t)
                if kk % 50 == 0:
                    assert bytes((C.c_uint8 * n).from_address(addr)) == want, kk
                    checked += 1
        for kk, t in pend:
            r.wait(t)
        assert checked == 8
    finally:
        r.close()


@pytest.mark.parametrize("engine,overlap", [(None, 0), (0, 0), (1, 0), (None, 1), (0, 1)])
@pytest.mark.parametrize("depth", [2, 3])
def test_copy_engines_deliver_the_reference_frame(frog, golden, engine, overlap, depth, tune):
    """One rank delivering into host memory: by default (and with RT_TUNE_COPY_ENGINE=1) the
    frames go through SDMA copies queued through the HSA runtime, with 0 through the HIP
    runtime's copies; RT_TUNE_OVERLAP_FRAMES=1 lets consecutive render kernels overlap.
    Pipelined frames with alternating cameras are each the single-frame image (P6 and float; the
    c3 frame is the reference's), and so is a frame after a resize; the copy's own times are
    reported."""
    tune(copy_engine=engine, overlap_frames=overlap)
    base = frog.camera(W, H)
    cams = [base, rt.Camera(tuple(np.add(base.pos, (0.004, 0.0, 0.003))), base.look_at, base.up,
                            base.focal_length_mm, base.sensor_height_mm, W, H)]
    for deliver in (rt.RT_DELIVER_P6, rt.RT_DELIVER_F32):
        r = rt.Renderer.from_host(frog, devices=(0,), depth=depth, deliver=deliver)
        try:
            assert r.copy_engine == ("runtime" if engine == 0 else "sdma")
            o, _j = _opts(frog)
            want = []
            for c in cams:  # the single-frame images
                addr, n = r.wait(r.submit(c, o))
                want.append(bytes((C.c_uint8 * n).from_address(addr)))
            assert want[0] == (golden[1].tobytes() if deliver == rt.RT_DELIVER_P6 else golden[0].tobytes())
            assert want[1] != want[0]
            pend = []
            for k in [0, 1, 1, 0, 1, 0, 0, 1, 0, 1]:
                pend.append((k, r.submit(cams[k], o)))
                if len(pend) >= depth:
                    kk, t = pend.pop(0)
                    addr, n = r.wait(t)
                    assert bytes((C.c_uint8 * n).from_address(addr)) == want[kk]
            for kk, t in pend:
                addr, n = r.wait(t)
                assert bytes((C.c_uint8 * n).from_address(addr)) == want[kk]
            d = r.times(rt.RT_TIME_DELIVER, 4)
            f = r.times(rt.RT_TIME_FRAME, 4)
            assert np.all(d > 0) and np.all(f >= d)
            small = frog.camera(640, 360)  # a resize, then back
            a1 = bytes((C.c_uint8 * (640 * 360 * 3 * (4 if deliver == rt.RT_DELIVER_F32 else 1))).from_address(
                r.wait(r.submit(small, o))[0]))
            addr, n = r.wait(r.submit(base, o))
            assert bytes((C.c_uint8 * n).from_address(addr)) == want[0] and len(a1) == n // 9
        finally:
            r.close()


def test_wait_rejects_stale_ticket(frog):
    r = rt.Renderer.from_host(frog, devices=(0,), depth=2)
    try:
        cam = frog.camera(64, 36)
        o, _j = _opts(frog, spp=4)
        ts = [r.submit(cam, o) for _ in range(4)]
        with pytest.raises(rt.RTError):
            r.wait(ts[0])  # slot reused by ts[2]
        r.wait(ts[3])
    finally:
        r.close()


def test_device_delivery_and_partial_band(frog):
    """RT_DELIVER_DEVICE (frame assembled in rank 0's HBM) and an image height that is not a
    multiple of the band height (a partial last band), against the oracle."""
    cam = frog.camera(160, 37)
    o, _j = _opts(frog, spp=4)
    oc = oracle_camera(cam)
    ref, _, _ = orc.render_g(frog.num_triangles, oc, frog.nodes, frog.aabbs, frog.triangles, frog.tri_object_ids,
                             frog.materials, frog.lights, spp=4, max_depth=1, miss=frog.settings["miss_color"],
                             aov=True)
    want = orc.ppm_quantize(ref, 255, True, True).astype(np.uint8).reshape(37, 160, 3)
    for devices in [(0,), (0, 0, 0)]:
        r = rt.Renderer.from_host(frog, devices=devices, gather=rt.RT_GATHER_DIRECT, deliver=rt.RT_DELIVER_DEVICE)
        try:
            got = r.render(cam, spp=4, max_depth=1, miss_color=frog.settings["miss_color"])
            assert np.array_equal(got, want), devices
        finally:
            r.close()
        r = rt.Renderer.from_host(frog, devices=devices, gather=rt.RT_GATHER_DIRECT, deliver=rt.RT_DELIVER_F32)
        try:
            got = r.render(cam, spp=4, max_depth=1, miss_color=frog.settings["miss_color"])
            assert float(np.abs(got - ref).max()) <= 2e-6
        finally:
            r.close()


def test_reference_signature_multi_gpu(frog, golden):
    """rt_render_reference_gpus (the reference signature + n_gpus) at n_gpus 1 equals the reference."""
    cam = frog.camera(W, H)
    out = np.zeros(W * H * 3, np.float32)
    mats = frog.materials
    rt.render(frog.num_triangles, W, H, cam, frog.settings["miss_color"], 1, SPP, frog.nodes, frog.aabbs,
              frog.triangles, frog.tri_object_ids, mats, len(mats), frog.lights, len(frog.lights), True, out)
    assert out.view(np.uint32).tobytes() == golden[0].view(np.uint32).tobytes()


def test_reference_signature_distinct_gpus(frog, golden):
    """rt_render_reference_gpus over up to 8 distinct GPUs (RCCL-free direct delivery, one
    process) equals the reference frame.  Skipped, visibly, on a box with one GPU."""
    dev = rt.device_count()
    if dev < 2:
        pytest.skip("needs >= 2 GPUs (this box has %d)" % dev)
    cam = frog.camera(W, H)
    mats = frog.materials
    out = np.zeros(W * H * 3, np.float32)
    rt.render(frog.num_triangles, W, H, cam, frog.settings["miss_color"], 1, SPP, frog.nodes, frog.aabbs,
              frog.triangles, frog.tri_object_ids, mats, len(mats), frog.lights, len(frog.lights), True, out,
              n_gpus=min(dev, 8))
    assert out.view(np.uint32).tobytes() == golden[0].view(np.uint32).tobytes()


def test_rccl_gather_distinct_gpus(frog, golden):
    """The RCCL strip gather over xGMI between distinct GPUs of one process (ncclCommInitAll),
    P6 and device delivery: the reference frame.  Skipped, visibly, on a box with one GPU."""
    dev = rt.device_count()
    if dev < 2:
        pytest.skip("needs >= 2 GPUs (this box has %d)" % dev)
    cam = frog.camera(W, H)
    for deliver, want in ((rt.RT_DELIVER_F32, golden[0]), (rt.RT_DELIVER_P6, golden[1]),
                          (rt.RT_DELIVER_DEVICE, golden[1])):
        r = rt.Renderer.from_host(frog, devices=tuple(range(min(dev, 8))), gather=rt.RT_GATHER_RCCL, deliver=deliver)
        try:
            got = r.render(cam, spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
            assert np.asarray(got).tobytes() == want.tobytes(), deliver
        finally:
            r.close()


def test_scene_frames_on_two_streams(frog, golden):
    """Back-to-back frames of one scene on two streams (the scene's tile lists are reused per
    frame: the second frame must wait for the first)."""
    ds = rt.DeviceScene.from_host(frog, device=0)
    cam = frog.camera(W, H)
    o, _j = _opts(frog)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [torch.zeros((H, W, 3), dtype=torch.float32, device="cuda") for _ in range(4)]
    for k, buf in enumerate(outs):
        st = (s1 if k % 2 == 0 else s2).cuda_stream
        ds.render_device(cam, o, buf.data_ptr(), stream=st)
    torch.cuda.synchronize()
    for buf in outs:
        assert buf.cpu().numpy().view(np.uint32).tobytes() == golden[0].view(np.uint32).tobytes()
    ds.close()


def test_renderer_exports():
    lib = L.lib()
    for name in ["rt_renderer_create", "rt_renderer_submit", "rt_renderer_wait", "rt_renderer_times",
                 "rt_render_reference_gpus", "rt_comm_unique_id", "rt_scene_clone"]:
        assert hasattr(lib, name)
