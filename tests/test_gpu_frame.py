"""The frame epilogue on the device: P6 quantisation
(rt_ppm_quantize_device) and the band un-permute of gathered strips
(rt_unpermute_strips_device), through the C ABI.

Bar: byte-identical to write_p6 (HW1/ppm_p6_lib/src/ppm_p6.cpp:137-155, 257-301) as restated by
the oracle (orc_ppm_quantize) and as the reference itself wrote the c3 image
(tests/golden/scenes/c3_full/image.ppm.gz).
"""
from __future__ import annotations

import gzip

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from oracle import pyoracle as orc

import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import dist as rd

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _oracle_body(rgb, maxval, clamp, gamma2, flip_y):
    a = np.asarray(rgb, np.float32)
    if flip_y:
        a = a[::-1]
    q = orc.ppm_quantize(a, maxval, clamp, gamma2).reshape(-1)
    if maxval < 256:
        return q.astype(np.uint8).tobytes()
    return q.astype(">u2").tobytes()


def _device_body(rgb, maxval, clamp, gamma2, flip_y, offset=0):
    a = np.ascontiguousarray(rgb, np.float32)
    H, W = a.shape[0], a.shape[1]
    bps = 1 if maxval < 256 else 2
    src = torch.zeros(a.size + offset, dtype=torch.float32, device=DEV)
    src[offset:] = torch.from_numpy(a.reshape(-1)).to(DEV)
    out = torch.zeros(a.size * bps + offset, dtype=torch.uint8, device=DEV)
    rt.quantize_p6_device(src.data_ptr() + 4 * offset, W, H, out.data_ptr() + offset, maxval, clamp, gamma2, flip_y)
    torch.cuda.synchronize()
    return out[offset:].cpu().numpy().tobytes()


def _boundary_values(maxval):
    """Floats within 40 ulps of every rounding boundary of sqrt(x) * maxval (x = ((k+0.5)/maxval)^2)
    and of the clamp edges, plus specials."""
    k = np.arange(maxval, dtype=np.float64)
    edges = ((k + 0.5) / maxval) ** 2
    base = edges.astype(np.float32).view(np.int32)
    steps = np.arange(-40, 41, dtype=np.int32)
    vals = (base[:, None] + steps[None, :]).reshape(-1).view(np.float32)
    special = np.array([0.0, -0.0, 1.0, np.nextafter(1, 2), np.nextafter(1, 0), -1.0, 2.0, np.inf, -np.inf, np.nan,
                        1e-45, 1e-38, 3.4e38, -3.4e38, 0.5], np.float32)
    return np.concatenate([vals, special])


@pytest.mark.parametrize("flip_y", [False, True])
@pytest.mark.parametrize("maxval,clamp,gamma2", [(255, True, True), (255, False, True), (255, True, False),
                                                 (255, False, False), (65535, True, True), (65535, False, False),
                                                 (1, True, True), (1000, True, True)])
def test_quantize_matches_write_p6(maxval, clamp, gamma2, flip_y):
    rng = np.random.default_rng(maxval * 4 + clamp * 2 + gamma2)
    v = np.concatenate([_boundary_values(maxval), rng.uniform(-0.5, 1.5, 20000).astype(np.float32),
                        (rng.standard_normal(2000) * 1e20).astype(np.float32)])
    W = 37  # ragged rows: the general path when flipped, the vector path's tail otherwise
    H = -(-v.size // (3 * W))
    rgb = np.zeros(H * W * 3, np.float32)
    rgb[:v.size] = v
    rgb = rgb.reshape(H, W, 3)
    assert _device_body(rgb, maxval, clamp, gamma2, flip_y) == _oracle_body(rgb, maxval, clamp, gamma2, flip_y)


@pytest.mark.parametrize("offset", [1, 3])
def test_quantize_unaligned_buffers(offset):
    rgb = np.random.default_rng(offset).uniform(0, 1, (9, 16, 3)).astype(np.float32)
    assert _device_body(rgb, 255, True, True, False, offset) == _oracle_body(rgb, 255, True, True, False)


def test_quantize_reproduces_reference_c3_image():
    """The reference's own P6 of the c3 frame (written by its ppm_p6) from the reference's float
    framebuffer, quantised on the device."""
    d = GOLDEN / "scenes" / "c3_full"
    fb = np.frombuffer(gzip.open(d / "fb.f32.gz").read(), np.float32).reshape(1080, 1920, 3)
    ref = gzip.open(d / "image.ppm.gz").read()
    got = rt.encode_p6_device(torch.from_numpy(fb.copy()).to(DEV))
    assert got == ref
    assert rt.encode_p6(fb) == ref


@pytest.mark.parametrize("flip_y", [False, True])
@pytest.mark.parametrize("height,band_rows,world", [(1080, 8, 8), (1080, 8, 3), (37, 5, 4), (16, 8, 4), (9, 8, 1)])
def test_unpermute_strips(height, band_rows, world, flip_y):
    W = 13
    frame = np.random.default_rng(height + world).integers(0, 1 << 31, (height, W, 3), dtype=np.int64) \
        .astype(np.float32)
    max_rows = rd.max_strip_rows(height, band_rows, world)
    strips = np.zeros((world, max_rows, W, 3), np.float32)
    for r in range(world):
        ys = rd.rows_of(height, band_rows, r, world)
        assert len(ys) == rt._lib.lib().rt_shard_rows(height, band_rows, r, world)
        strips[r, :len(ys)] = frame[ys]
    s = torch.from_numpy(strips).to(DEV)
    out = torch.zeros((height, W, 3), dtype=torch.float32, device=DEV)
    rt.unpermute_strips_device(s.data_ptr(), max_rows, W * 12, height, band_rows, world, out.data_ptr(), flip_y)
    torch.cuda.synchronize()
    want = frame[::-1] if flip_y else frame
    assert np.array_equal(out.cpu().numpy(), want)


def test_unpermute_rejects_short_strips():
    s = torch.zeros(64, dtype=torch.uint8, device=DEV)
    with pytest.raises(rt.RTError):
        rt.unpermute_strips_device(s.data_ptr(), 1, 4, 16, 8, 1, s.data_ptr())


def test_gather_p6_single_rank_matches_host_encode():
    rgb = np.random.default_rng(7).uniform(-0.1, 1.1, (45, 31, 3)).astype(np.float32)
    t = torch.from_numpy(rgb).to(DEV)
    for flip in (False, True):
        got = rd.gather_p6(t, 45, 8, 1, 0, flip_y=flip)
        assert got == rt.encode_p6(rgb, flip_y=flip)


@pytest.mark.parametrize("spp,miss,kernel,bands", [
    (16, (0.0, 0.0, 0.0), rt.RT_KERNEL_AUTO, (8, 0, 1)),        # c3's shape: samples kernel, culled tiles
    (3, (0.5, 0.7, 1.0), rt.RT_KERNEL_AUTO, (8, 0, 1)),         # pixels kernel, non-black miss pixels
    (4, (0.2, 0.1, 0.05), rt.RT_KERNEL_LANE, (8, 1, 3)),        # lane kernel, a band shard
])
def test_render_device_fused_p6_matches_write_p6(spp, miss, kernel, bands):
    """rt_render_device_p6: the P6 samples the render and cull kernels write alongside the float
    pixels are write_p6's quantisation of those pixels, byte for byte (live and culled tiles)."""
    from conftest import host_scene

    hs = host_scene("frog.json")
    cam = hs.camera(160, 90)
    ds = rt.DeviceScene.from_host(hs, device=0)
    band_rows, band_index, band_count = bands
    opts, _keep = ds.make_opts(spp=spp, max_depth=1, miss_color=miss, band_rows=band_rows,
                               band_index=band_index, band_count=band_count, kernel=kernel)
    rows = rt._lib.lib().rt_shard_rows(90, band_rows, band_index, band_count)
    rgb = torch.zeros((rows, 160, 3), dtype=torch.float32, device=DEV)
    p6 = torch.full((rows, 160 * 3), 7, dtype=torch.uint8, device=DEV)
    stream = torch.cuda.current_stream(DEV).cuda_stream
    ds.render_device(cam, opts, rgb.data_ptr(), stream=stream, p6_dev_ptr=p6.data_ptr())
    torch.cuda.synchronize(DEV)
    want = rt.encode_p6(rgb.cpu().numpy())
    assert want[-p6.numel():] == p6.cpu().numpy().tobytes()
    ds.close()
