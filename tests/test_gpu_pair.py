"""Two frames in one render launch (rt_render_device_pair, rt_renderer_submit_pair,
RT_TUNE_PAIR_FRAMES).

Bar: every frame of a pair is byte-for-byte the frame a single render of it gives (P6 and float
framebuffers), and the c3 frame is still the reference's own (tests/golden/scenes/c3_full), for
pairs of equal and of different cameras, consecutive pipelined pairs, band shards (full and half
waves), pairs the pair kernel cannot take (another tile cut: frame A then renders alone), the
renderer's delivery paths and depths, and with the knob off.
"""
from __future__ import annotations

import ctypes as C
import gzip

import numpy as np
import pytest
import torch

from conftest import GOLDEN, host_scene

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


def _cams(frog, w=W, h=H):
    base = frog.camera(w, h)
    moved = rt.Camera(tuple(np.add(base.pos, (0.004, 0.0, 0.003))), base.look_at, base.up, base.focal_length_mm,
                      base.sensor_height_mm, w, h)
    # far back: the frog small in the view (the tree-cut culling pass on, another tile cut)
    far = rt.Camera(tuple(np.add(base.look_at, 6.0 * np.subtract(base.pos, base.look_at))), base.look_at, base.up,
                    base.focal_length_mm, base.sensor_height_mm, w, h)
    return {"base": base, "moved": moved, "far": far}


def _bufs(n, rows, w=W):
    return [(torch.zeros((rows, w, 3), dtype=torch.float32, device="cuda"),
             torch.zeros((rows, w, 3), dtype=torch.uint8, device="cuda")) for _ in range(n)]


def _singles(ds, cams, names, o, rows, w=W):
    """The single-frame images (float bits, P6 bytes) of each camera name."""
    out = {}
    for nm in names:
        (rgb, p6), = _bufs(1, rows, w)
        ds.render_device(cams[nm], o, rgb.data_ptr(), p6_dev_ptr=p6.data_ptr())
        torch.cuda.synchronize()
        out[nm] = (rgb.cpu().numpy().view(np.uint32).tobytes(), p6.cpu().numpy().tobytes())
    return out


PAIRS = [("base", "moved"), ("moved", "base"), ("base", "base"), ("far", "base"), ("base", "far"), ("far", "far"),
         ("moved", "moved"), ("base", "moved")]


@pytest.mark.parametrize("knob", [None, 0])
def test_pairs_equal_single_frames(frog, golden, knob, tune):
    """Eight consecutive pairs queued back to back on one stream (their pre-passes overlapping
    the previous pair kernel), then one sync: each frame is its single-frame image."""
    tune(pair_frames=knob)
    ds = rt.DeviceScene.from_host(frog, device=0)
    try:
        cams = _cams(frog)
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
        want = _singles(ds, cams, ["base", "moved", "far"], o, H)
        assert want["base"][1] == golden[1].tobytes()
        assert want["base"][0] == golden[0].view(np.uint32).tobytes()
        assert want["moved"][1] != want["base"][1] and want["far"][1] != want["base"][1]
        bufs = _bufs(2 * len(PAIRS), H)
        names = []
        for i, (a, b) in enumerate(PAIRS):
            (ra, pa), (rb, pb) = bufs[2 * i], bufs[2 * i + 1]
            ds.render_device_pair(cams[a], cams[b], o, ra.data_ptr(), pa.data_ptr(), rb.data_ptr(), pb.data_ptr())
            names.append(ds.kernel_name())
        torch.cuda.synchronize()
        for i, (a, b) in enumerate(PAIRS):
            for k, nm in ((2 * i, a), (2 * i + 1, b)):
                rgb, p6 = bufs[k]
                assert p6.cpu().numpy().tobytes() == want[nm][1], f"pair {i} ({a}, {b}): frame {nm} P6 differs"
                assert rgb.cpu().numpy().view(np.uint32).tobytes() == want[nm][0], f"pair {i}: frame {nm} floats"
        if knob == 0:
            assert all(n.startswith("render_tiles_kernel<49,") for n in names), names
        else:
            # pairs of one tile cut take the pair kernel
            same = [n for (a, b), n in zip(PAIRS, names) if (a == "far") == (b == "far")]
            assert all(n.startswith("render_pair_kernel<49, true, true, 7, 0>") for n in same), names
        kt = ds.kernel_times(4)
        assert len(kt) > 0 and np.all(kt > 0)
    finally:
        ds.close()


@pytest.mark.parametrize("band_count,band_index", [(2, 1), (8, 3), (8, 7)])
def test_pair_band_shards(frog, band_count, band_index):
    """Band shards of an N-GPU frame: the pair kernel at full waves (2 shards) and half waves
    (8 shards, LS = 1), each shard frame equal to its single render."""
    ds = rt.DeviceScene.from_host(frog, device=0)
    try:
        cams = _cams(frog)
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"], band_rows=8,
                                         band_index=band_index, band_count=band_count)
        rows = L.lib().rt_shard_rows(H, 8, band_index, band_count)
        want = _singles(ds, cams, ["base", "moved"], o, rows)
        bufs = _bufs(6, rows)
        seq = [("base", "moved"), ("moved", "base"), ("base", "base")]
        for i, (a, b) in enumerate(seq):
            (ra, pa), (rb, pb) = bufs[2 * i], bufs[2 * i + 1]
            ds.render_device_pair(cams[a], cams[b], o, ra.data_ptr(), pa.data_ptr(), rb.data_ptr(), pb.data_ptr())
        torch.cuda.synchronize()
        ls = 1 if band_count >= 4 else 0
        assert ds.kernel_name() == f"render_pair_kernel<49, true, true, 7, {ls}>", ds.kernel_name()
        for i, (a, b) in enumerate(seq):
            for k, nm in ((2 * i, a), (2 * i + 1, b)):
                rgb, p6 = bufs[k]
                assert p6.cpu().numpy().tobytes() == want[nm][1], f"shard {band_index}/{band_count} pair {i}"
                assert rgb.cpu().numpy().view(np.uint32).tobytes() == want[nm][0]
    finally:
        ds.close()


def test_pair_multi_bounce(frog):
    """The paired-only bounce kernels (one light, half waves: c3b's) as a pair kernel: pipelined
    pairs of 8-bounce diffuse frames, each its single-frame image."""
    ds = rt.DeviceScene.from_host(frog, device=0)
    try:
        cams = _cams(frog, 480, 270)
        for kw in (dict(spp=16, max_depth=8), dict(spp=4, max_depth=3), dict(spp=16, max_depth=8, diffuse_bounce=False)):
            o, _j = rt.DeviceScene.make_opts(miss_color=frog.settings["miss_color"], **kw)
            want = _singles(ds, cams, ["base", "moved"], o, 270, 480)
            bufs = _bufs(6, 270, 480)
            seq = [("base", "moved"), ("moved", "base"), ("base", "base")]
            for i, (a, b) in enumerate(seq):
                (ra, pa), (rb, pb) = bufs[2 * i], bufs[2 * i + 1]
                ds.render_device_pair(cams[a], cams[b], o, ra.data_ptr(), pa.data_ptr(), rb.data_ptr(), pb.data_ptr())
            torch.cuda.synchronize()
            assert ds.kernel_name() == "render_pair_kernel<17, true, false, 4, 3>", (kw, ds.kernel_name())
            for i, (a, b) in enumerate(seq):
                for k, nm in ((2 * i, a), (2 * i + 1, b)):
                    rgb, p6 = bufs[k]
                    assert p6.cpu().numpy().tobytes() == want[nm][1], (kw, i, nm)
                    assert rgb.cpu().numpy().view(np.uint32).tobytes() == want[nm][0], (kw, i, nm)
    finally:
        ds.close()


def test_pair_c3b_full_frames(frog):
    """c3b (frog.json as shipped: 8 diffuse bounces, 1080p x 16 spp) as pairs: both frames the
    reference's own image (tests/golden/scenes/c3b_full)."""
    ppm = gzip.open(GOLDEN / "scenes" / "c3b_full" / "image.ppm.gz").read()
    ds = rt.DeviceScene.from_host(frog, device=0)
    try:
        cam = frog.camera(W, H)
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=8, miss_color=frog.settings["miss_color"])
        bufs = _bufs(4, H)
        for i in range(2):
            (ra, pa), (rb, pb) = bufs[2 * i], bufs[2 * i + 1]
            ds.render_device_pair(cam, cam, o, ra.data_ptr(), pa.data_ptr(), rb.data_ptr(), pb.data_ptr())
        torch.cuda.synchronize()
        assert ds.kernel_name().startswith("render_pair_kernel<17,"), ds.kernel_name()
        for rgb, p6 in bufs:
            assert p6.cpu().numpy().tobytes() == ppm[17:]
    finally:
        ds.close()


def test_pair_outside_the_pair_kernel(frog):
    """Frames the pair kernel is not instantiated for (small spp on another tile shape, the LANE
    kernel, 128 spp whole-block items) render as two launches with the single-frame images."""
    ds = rt.DeviceScene.from_host(frog, device=0)
    try:
        cams = _cams(frog, 320, 180)
        for kw in (dict(spp=4, max_depth=1, kernel=rt.RT_KERNEL_LANE), dict(spp=128, max_depth=1)):
            o, _j = rt.DeviceScene.make_opts(miss_color=frog.settings["miss_color"], **kw)
            want = _singles(ds, cams, ["base", "moved"], o, 180, 320)
            (ra, pa), (rb, pb) = _bufs(2, 180, 320)
            ds.render_device_pair(cams["base"], cams["moved"], o, ra.data_ptr(), pa.data_ptr(), rb.data_ptr(),
                                  pb.data_ptr())
            torch.cuda.synchronize()
            assert not ds.kernel_name().startswith("render_pair_kernel"), (kw, ds.kernel_name())
            assert pa.cpu().numpy().tobytes() == want["base"][1], kw
            assert pb.cpu().numpy().tobytes() == want["moved"][1], kw
            assert rb.cpu().numpy().view(np.uint32).tobytes() == want["moved"][0], kw
    finally:
        ds.close()


def _frame(addr, n):
    return bytes((C.c_uint8 * n).from_address(addr))


@pytest.mark.parametrize("engine", [None, 0])
@pytest.mark.parametrize("depth", [2, 3, 4])
def test_renderer_pairs_deliver_single_frames(frog, golden, engine, depth, tune):
    """rt_renderer_submit_pair, pairs and single submits interleaved, every delivered frame the
    single-frame image (P6 through SDMA or the runtime's copies, and float)."""
    tune(copy_engine=engine)
    cams = _cams(frog)
    for deliver in (rt.RT_DELIVER_P6, rt.RT_DELIVER_F32):
        r = rt.Renderer.from_host(frog, devices=(0,), depth=depth, deliver=deliver)
        try:
            o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
            want = {nm: _frame(*r.wait(r.submit(cams[nm], o))) for nm in ("base", "moved")}
            assert want["base"] == (golden[1].tobytes() if deliver == rt.RT_DELIVER_P6 else golden[0].tobytes())
            pend = []
            checked = 0

            def drain(keep):
                nonlocal checked
                while len(pend) > keep:
                    nm, t = pend.pop(0)
                    assert _frame(*r.wait(t)) == want[nm], f"depth {depth} frame {t} ({nm})"
                    checked += 1

            for a, b in [("base", "moved"), ("moved", "moved"), ("base", "base"), ("moved", "base")] * 2:
                drain(depth - 2)
                ta, tb = r.submit_pair(cams[a], cams[b], o)
                pend += [(a, ta), (b, tb)]
                drain(depth - 1)
                pend.append((b, r.submit(cams[b], o)))
            drain(0)
            assert checked == 24
            assert r.scene(0).kernel_name().startswith("render_tiles_kernel<49,")
            f = r.times(rt.RT_TIME_FRAME, 6)
            assert len(f) == 6 and np.all(f > 0)
        finally:
            r.close()


@pytest.mark.parametrize("devices,gather,flags", [((0, 0, 0, 0), rt.RT_GATHER_DIRECT, 0),
                                                  ((0,), rt.RT_GATHER_RCCL, rt.RT_RENDERER_SELF_SEND)])
def test_renderer_pairs_bands_and_rccl(frog, golden, devices, gather, flags):
    """Pairs over 4 band ranks on one GPU (half waves, per-rank copies) and over the RCCL gather
    (world 1, self-send): every frame the reference's."""
    r = rt.Renderer.from_host(frog, devices=devices, gather=gather, flags=flags, depth=4)
    try:
        cam = frog.camera(W, H)
        o, _j = rt.DeviceScene.make_opts(spp=SPP, max_depth=1, miss_color=frog.settings["miss_color"])
        pend = []
        for _ in range(4):
            while len(pend) > 2:
                assert _frame(*r.wait(pend.pop(0))) == golden[1].tobytes()
            pend += list(r.submit_pair(cam, cam, o))
        for t in pend:
            assert _frame(*r.wait(t)) == golden[1].tobytes()
        want = "render_pair_kernel<49, true, true, 7, 1>" if len(devices) >= 4 else "render_pair_kernel<49, true, true, 7, 0>"
        assert r.scene(0).kernel_name() == want
    finally:
        r.close()


def test_submit_pair_needs_two_slots(frog):
    r = rt.Renderer.from_host(frog, devices=(0,), depth=1)
    try:
        cam = frog.camera(64, 36)
        o, _j = rt.DeviceScene.make_opts(spp=4, max_depth=1, miss_color=frog.settings["miss_color"])
        with pytest.raises(rt.RTError):
            r.submit_pair(cam, cam, o)
    finally:
        r.close()
