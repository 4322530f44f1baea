"""The HW1 path resident on the device (rt_hw1_scene, the C2 configuration's bench path):
frames against the reference's own HW1 outputs (tests/golden/scenes/c1_full, c2_full: the
HW1/src/render.cpp:72-116 loop built from the reference sources), the P6 samples the render
kernel writes against the reference's ppm_p6 file, and the bin list's capacity fallback (a tile
whose list does not fit takes the brute-force loop) against the brute-force kernel."""
from __future__ import annotations

import gzip

import numpy as np
import pytest

from conftest import GOLDEN, golden_array, golden_meta

import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import configs

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _frame(sc, cam, c, spp, brute=False):
    W, H = cam.pixel_width, cam.pixel_height
    rgb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    p6 = torch.zeros(W * H * 3, dtype=torch.uint8, device="cuda")
    hi = torch.zeros(W * H * spp, dtype=torch.int32, device="cuda")
    ht = torch.zeros(W * H * spp, dtype=torch.float32, device="cuda")
    sc.render_device(cam, c["light_pos"], c["light_color"], spp, rgb_ptr=rgb.data_ptr(), p6_ptr=p6.data_ptr(),
                     hit_idx_ptr=hi.data_ptr(), hit_t_ptr=ht.data_ptr(),
                     stream=torch.cuda.current_stream().cuda_stream, brute=brute)
    torch.cuda.synchronize()
    return rgb.cpu().numpy(), p6.cpu().numpy(), hi.cpu().numpy(), ht.cpu().numpy()


@pytest.mark.parametrize("name,cfg", [("c1_full", "c1"), ("c2_full", "c2")])
def test_resident_hw1_frames_match_reference(name, cfg):
    c = configs.HW1_CONFIGS[cfg]
    meta = golden_meta(name)
    W, H = meta["width"], meta["height"]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    sc = rt.HW1Scene(mesh.positions, mesh.normals, mesh.indices)
    try:
        for _ in range(3):  # frames in a row on the same buffers: the same frame
            rgb, p6, hi, ht = _frame(sc, cam, c, c["spp"])
            assert np.array_equal(rgb.view(np.uint32), golden_array(name, "fb.f32.gz", np.float32).view(np.uint32))
            assert np.array_equal(hi, golden_array(name, "hits.i32.gz", np.int32))
            assert np.array_equal(ht.view(np.uint32), golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
            want = gzip.open(GOLDEN / "scenes" / name / "image.ppm.gz").read()
            assert rt.p6_header(W, H) + p6.tobytes() == want
        assert sc.kernel_name() == "render_hw1_chunks_kernel<true>"  # (as rocprofv3 names it; the resolve fused)
        assert (sc.kernel_times(3) > 0).all()
    finally:
        sc.close()


@pytest.mark.parametrize("fuse,chunk", [(0, 64), (1, 64), (2, 64), (3, 64), (2, 16), (2, 32), (3, 128), (0, 256)])
def test_hw1_fused_passes_match_reference(fuse, chunk, tune):
    """RT_TUNE_HW1_FUSE: the scan in the count pass's last block (bit 0) and the resolve in each
    tile's last render item (bit 1), each on or off, over work items of 16 to 256 list entries
    (RT_TUNE_HW1_CHUNK): the frames equal the reference's (AOVs and P6), twice in a row on the
    same buffers (the passes leave the counters zeroed)."""
    tune(hw1_fuse=fuse, hw1_chunk=chunk)
    name, c = "c2_full", configs.HW1_CONFIGS["c2"]
    meta = golden_meta(name)
    W, H = meta["width"], meta["height"]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    sc = rt.HW1Scene(mesh.positions, mesh.normals, mesh.indices)
    want = gzip.open(GOLDEN / "scenes" / name / "image.ppm.gz").read()
    try:
        for _ in range(2):
            rgb, p6, hi, ht = _frame(sc, cam, c, c["spp"])
            assert np.array_equal(hi, golden_array(name, "hits.i32.gz", np.int32))
            assert np.array_equal(ht.view(np.uint32), golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
            assert rt.p6_header(W, H) + p6.tobytes() == want
    finally:
        sc.close()


@pytest.mark.parametrize("name,cfg,lanes,engine", [("c1_full", "c1", 2, -1), ("c2_full", "c2", 2, -1),
                                                   ("c2_full", "c2", 1, -1), ("c2_full", "c2", 2, 0),
                                                   ("c2_full", "c2", 1, 0)])
def test_delivered_hw1_frames_match_reference(name, cfg, lanes, engine, tune):
    """rt_render_hw1_deliver (the C1/C2 bench step): frames pipelined into pinned host buffers,
    alternating over the scene's lanes (RT_TUNE_HW1_LANES) and each copied by a DMA engine or on
    the scene's copy stream (RT_TUNE_COPY_ENGINE) while the next render; every delivered body is
    the reference's P6 file, including frames whose device body (8 frames back) and host buffer
    were reused, and a stale ticket is refused."""
    tune(hw1_lanes=lanes, copy_engine=engine)
    c = configs.HW1_CONFIGS[cfg]
    meta = golden_meta(name)
    W, H = meta["width"], meta["height"]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    want = gzip.open(GOLDEN / "scenes" / name / "image.ppm.gz").read()
    sc = rt.HW1Scene(mesh.positions, mesh.normals, mesh.indices)
    host = [torch.zeros(W * H * 3, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
    st = torch.cuda.Stream()
    try:
        pend = []
        for k in range(20):
            if len(pend) >= 2:
                t, b = pend.pop(0)
                sc.wait(t)
                assert rt.p6_header(W, H) + host[b].numpy().tobytes() == want, (k, t)
                host[b].zero_()
            pend.append((sc.render_deliver(cam, c["light_pos"], c["light_color"], c["spp"], host[k % 3].data_ptr(),
                                           stream=st.cuda_stream), k % 3))
        for t, b in pend:
            sc.wait(t)
            assert rt.p6_header(W, H) + host[b].numpy().tobytes() == want, t
        with pytest.raises(rt.RTError):
            sc.wait(10**6)
    finally:
        sc.close()


def _big_triangles(n=12, seed=3):
    """n large overlapping triangles in front of the camera: each covers most of a 1080p image,
    so their bin lists (~n x 32k tile entries) outgrow the first capacity (65536 entries)."""
    rng = np.random.default_rng(seed)
    pos, nrm, idx = [], [], []
    for k in range(n):
        z = -float(k) * 0.05
        c = rng.uniform(-0.2, 0.2, size=2)
        s = rng.uniform(2.0, 3.0)
        v = [(c[0] - s, c[1] - s, z), (c[0] + s, c[1] - s, z), (c[0], c[1] + s, z)]
        for j in range(3):
            pos.append(v[j])
            nrm.append((0.0, 0.0, 1.0) if k % 2 else (0.3, 0.0, 0.95))
        idx.append((3 * k, 3 * k + 1, 3 * k + 2))
    return np.array(pos, np.float32), np.array(nrm, np.float32), np.array(idx, np.uint32)


def test_bin_list_capacity_fallback_is_exact():
    """The first frame's lists outgrow the bin list (the tiles past the capacity take the
    brute-force loop); the next frame runs with the capacity grown from the first frame's total.
    Both frames equal the brute-force kernel bit for bit (AOVs included)."""
    pos, nrm, idx = _big_triangles()
    c = {"light_pos": (-3.0, 0.0, 1.0), "light_color": (1.0, 0.0, 1.0)}
    cam = rt.Camera((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, 24.0, 1920, 1080, hw1=True)
    sc = rt.HW1Scene(pos, nrm, idx)
    try:
        ref = _frame(sc, cam, c, 2, brute=True)
        cap0 = sc.list_info()[0]
        for k in range(2):
            got = _frame(sc, cam, c, 2)
            cap, total = sc.list_info()
            if k == 0:  # the first frame's lists outgrew the list: its last tiles took the brute-force loop
                assert total > cap0
            else:  # the second ran with a list grown from the first frame's total
                assert cap >= total > cap0
            for x, y in zip(got, ref):
                assert np.array_equal(x.view(np.uint8), y.view(np.uint8))
        assert (ref[2] >= 0).mean() > 0.3
    finally:
        sc.close()


def test_delivered_frames_grow_each_lane_list_and_mix_with_direct_frames(tune):
    """Delivered frames over two lanes whose lists outgrow the first capacity (each lane grows its
    own list from a finished frame's total, the overflowing tiles of the frames before take the
    brute-force loop), interleaved with direct frames on the caller's stream (lane 0 shared by
    both streams): every P6 body equals the brute-force kernel's."""
    tune(hw1_lanes=2)
    pos, nrm, idx = _big_triangles()
    c = {"light_pos": (-3.0, 0.0, 1.0), "light_color": (1.0, 0.0, 1.0)}
    W, H = 1920, 1080
    cam = rt.Camera((0.0, 0.0, 3.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 20.0, 24.0, W, H, hw1=True)
    sc = rt.HW1Scene(pos, nrm, idx)
    host = [torch.zeros(W * H * 3, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
    st = torch.cuda.Stream()
    try:
        want = _frame(sc, cam, c, 1, brute=True)[1].tobytes()
        cap0 = sc.list_info()[0]
        for rnd in range(3):
            tickets = [sc.render_deliver(cam, c["light_pos"], c["light_color"], 1, host[k].data_ptr(),
                                         stream=st.cuda_stream) for k in range(4)]
            for k, t in enumerate(tickets):
                sc.wait(t)
                assert host[k].numpy().tobytes() == want, (rnd, k)
                host[k].zero_()
            assert _frame(sc, cam, c, 1)[1].tobytes() == want, rnd  # a direct frame (lane 0)
        assert sc.list_info()[0] > cap0  # the lists grew
    finally:
        sc.close()
