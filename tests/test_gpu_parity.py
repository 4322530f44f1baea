"""Parity of the HIP path (through the C ABI) with the oracle and the reference's fixtures.

Bar:
* primary-hit triangle indices and their t: bit-exact (index work);
* float framebuffer: bit-exact.  Every float/double operation of the path is reproduced in
  the reference's order without contraction, HIP's f32 division/sqrt are correctly
  rounded like x86's, and powf is a restatement of the reference libm's powf
  (tests/test_powf.py).  RGB_TOL = 2e-6 is the stated tolerance the checks also report
  against (the bound a device-libm powf would need);
* P6 output (ppm_p6 defaults): max-abs <= 1 per 8-bit sample.
"""
from __future__ import annotations

import gzip
import hashlib
import json

import numpy as np
import pytest

from conftest import GOLDEN, G_SCENES, golden_array, golden_meta, hexv, host_scene, oracle_camera
from oracle import pyoracle as orc

import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import configs

pytestmark = pytest.mark.gpu

RGB_TOL = 2e-6
KERNELS = [rt.RT_KERNEL_WAVE, rt.RT_KERNEL_LANE]
# (flags, tile order, tiles per render block): launch shapes, all of which must give the same frame
BIN = rt._lib.RT_FLAG_BINARY
LAUNCHES = [(0, rt.RT_TILES_AUTO), (BIN, rt.RT_TILES_AUTO), (0, rt.RT_TILES_LINEAR),
            (BIN, rt.RT_TILES_ROWS), (0, rt.RT_TILES_XCD_CHUNK),
            (rt._lib.RT_FLAG_NO_CULL, rt.RT_TILES_XCD_CHUNK), (BIN | rt._lib.RT_FLAG_NO_CULL, rt.RT_TILES_LINEAR)]


def _device_scene(scene):
    key = ("ds", scene)
    cache = _device_scene.__dict__.setdefault("cache", {})
    if key not in cache:
        cache[key] = rt.DeviceScene.from_host(host_scene(scene), device=0)
    return cache[key]


def _check_fb(rgb, ref, exact_frac=1.0):
    rgb = np.asarray(rgb, np.float32).reshape(-1)
    ref = np.asarray(ref, np.float32).reshape(-1)
    assert np.isfinite(rgb).all()
    d = np.abs(rgb - ref)
    assert d.max() <= RGB_TOL, f"max-abs {d.max()}"
    assert (rgb.view(np.uint32) == ref.view(np.uint32)).mean() >= exact_frac


@pytest.mark.parametrize("flags", [0, rt._lib.RT_FLAG_BINARY])
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", ["c3_small", "frog_bounce", "sphere_single", "cornell", "c5_small", "c3b_small"])
def test_golden_scene_parity(name, kernel, flags):
    meta = golden_meta(name)
    scene = G_SCENES[name]
    hs = host_scene(scene)
    cam = hs.camera(meta["width"], meta["height"])
    ds = _device_scene(scene)
    rgb, hi, ht = ds.render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                            diffuse_bounce=bool(meta["diffuse_bounce"]), miss_color=hexv(meta["miss_color"]),
                            aov=True, kernel=kernel, flags=flags)
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))


@pytest.mark.parametrize("name", ["c3_small", "frog_bounce", "sphere_single", "cornell", "c3b_small"])
def test_ray_counts_match_oracle(name):
    """rt_count_rays (total rays/s): camera, shadow and bounce rays of a frame
    equal the oracle's counters (orc_stats.rays; shadow = IsInShadow calls that cast a ray,
    shader.h:44-62; bounce = TraceRayIterative depths > 0, query.h:156-220)."""
    meta = golden_meta(name)
    scene = G_SCENES[name]
    hs = host_scene(scene)
    cam = hs.camera(meta["width"], meta["height"])
    kw = dict(spp=meta["spp"], max_depth=meta["max_depth"], diffuse_bounce=bool(meta["diffuse_bounce"]),
              miss_color=hexv(meta["miss_color"]))
    got = _device_scene(scene).count_rays(cam, **kw)
    _, st = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                         hs.tri_object_ids, hs.materials, hs.lights, spp=kw["spp"], max_depth=kw["max_depth"],
                         diffuse_bounce=kw["diffuse_bounce"], miss=tuple(kw["miss_color"]), stats=True)
    assert [got["camera"], got["shadow"], got["bounce"]] == list(st["rays"])
    assert got["shadow"] + got["bounce"] > 0  # cornell's light casts no shadow ray; its bounces count
    if meta["max_depth"] > 1:
        assert got["bounce"] > 0


def test_ray_counts_c3_full_frame():
    """c3's full frame: 33,177,600 camera rays and 687,530 shadow rays, the oracle's count (whose
    frame is the reference's bit for bit; SURVEY.md §8(d) quotes 687,822 from its survey-time
    restatement); band shards sum to the same counts."""
    cfg = configs.G_CONFIGS["c3"]
    hs = host_scene(cfg["scene"])
    cam = hs.camera(cfg["width"], cfg["height"])
    ds = _device_scene(cfg["scene"])
    got = ds.count_rays(cam, spp=cfg["spp"], max_depth=cfg["max_depth"])
    _, st = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                         hs.tri_object_ids, hs.materials, hs.lights, spp=cfg["spp"], max_depth=cfg["max_depth"],
                         stats=True)
    assert [got["camera"], got["shadow"], got["bounce"]] == list(st["rays"])
    assert {k: got[k] for k in ("camera", "shadow", "bounce")} == {"camera": 33_177_600, "shadow": 687_530,
                                                                  "bounce": 0}
    # camera rays actually traversed (the tiles culling leaves): at least every primary hit
    # (1,064,872 samples hit, tests/golden/scenes/c3_full), whole 4x4x16 tiles
    assert 1_064_872 <= got["camera_traced"] < got["camera"] and got["camera_traced"] % 256 == 0
    parts = [ds.count_rays(cam, spp=cfg["spp"], max_depth=cfg["max_depth"], band_index=b, band_count=4)
             for b in range(4)]
    assert sum(q["shadow"] for q in parts) == got["shadow"]
    assert sum(q["camera"] for q in parts) == got["camera"]


@pytest.mark.parametrize("name", ["c3_small", "frog_bounce", "cornell", "c5_small"])
def test_half_waves_parity(name, tune):
    """Half waves (32 samples per wave, the default for 8-way band shards) forced on whole
    frames: the reference's outputs bit for bit, AOVs included."""
    tune(half_waves=1)
    meta = golden_meta(name)
    scene = G_SCENES[name]
    hs = host_scene(scene)
    cam = hs.camera(meta["width"], meta["height"])
    rgb, hi, ht = _device_scene(scene).render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                                              diffuse_bounce=bool(meta["diffuse_bounce"]),
                                              miss_color=hexv(meta["miss_color"]), aov=True)
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))


@pytest.mark.parametrize("flags,tiles", LAUNCHES)
def test_c3_full_frame_matches_reference(flags, tiles):
    """1920x1080x16 frog (config c3) against the reference's own full-size outputs, for every
    launch shape (tile orders, binary/4-ary records, culling on/off)."""
    meta = golden_meta("c3_full")
    hs = host_scene("frog.json")
    cam = hs.camera(1920, 1080)
    rgb, hi, ht = _device_scene("frog.json").render(cam, spp=16, max_depth=1, aov=True, flags=flags,
                                                    tile_order=tiles)
    assert hashlib.sha256(hi.tobytes()).hexdigest() == meta["sha256"]["hits.i32"]
    assert hashlib.sha256(ht.tobytes()).hexdigest() == meta["sha256"]["hitt.f32"]
    _check_fb(rgb, golden_array("c3_full", "fb.f32.gz", np.float32))
    ppm = gzip.open(GOLDEN / "scenes" / "c3_full" / "image.ppm.gz").read()
    mine = rt.encode_p6(rgb)
    assert len(mine) == len(ppm) and mine[:17] == ppm[:17]
    diff = np.abs(np.frombuffer(mine[17:], np.uint8).astype(int) - np.frombuffer(ppm[17:], np.uint8).astype(int))
    assert diff.max() <= 1


@pytest.mark.parametrize("name", ["c3b_small", "frog_bounce", "cornell", "sphere_single"])
@pytest.mark.parametrize("flags", [0, rt._lib.RT_FLAG_BINARY])
def test_bounce_paths_per_lane_traversal(name, flags):
    """Multi-bounce frames: camera rays and their shadow rays on the wave-shared DFS, bounce rays
    and theirs on each lane's own DFS (traverse_lane_lds over 4-ary or binary records): the
    reference's outputs bit for bit."""
    meta = golden_meta(name)
    assert meta["max_depth"] > 1
    scene = G_SCENES[name]
    hs = host_scene(scene)
    cam = hs.camera(meta["width"], meta["height"])
    rgb, hi, ht = _device_scene(scene).render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                                              diffuse_bounce=bool(meta["diffuse_bounce"]),
                                              miss_color=hexv(meta["miss_color"]), aov=True, flags=flags)
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))


@pytest.mark.parametrize("name", ["c3b_small", "frog_bounce", "sphere_single"])
@pytest.mark.parametrize("flags", [0, rt._lib.RT_FLAG_BINARY])
@pytest.mark.parametrize("half", ["0", "1"])
def test_one_light_bounce_loops_parity(name, flags, half, tune):
    """One-light multi-bounce frames through both bounce loops: half waves (the default) pair a
    path's lane with a shadow lane (paired_bounces: a depth's Lo add waits for its shadow ray's
    answer, traced beside the next bounce ray); half_waves=0 forces full waves and the
    unpaired loop.  The reference's outputs bit for bit, AOVs included."""
    tune(half_waves=int(half))
    meta = golden_meta(name)
    assert meta["max_depth"] > 1 and meta["num_lights"] == 1
    scene = G_SCENES[name]
    hs = host_scene(scene)
    cam = hs.camera(meta["width"], meta["height"])
    rgb, hi, ht = _device_scene(scene).render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                                              diffuse_bounce=bool(meta["diffuse_bounce"]),
                                              miss_color=hexv(meta["miss_color"]), aov=True, flags=flags)
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))


def test_c3b_full_frame_matches_reference():
    """c3b: frog.json as shipped (max_bounces 8, diffuse bounces) at 1920x1080x16 against the
    reference's own full-size outputs (hit AOVs by sha256, float frame, P6 file)."""
    meta = golden_meta("c3b_full")
    _c3b_full_check(meta)


def _c3b_full_check(meta):
    assert meta["max_depth"] == 8 and meta["diffuse_bounce"] == 1
    hs = host_scene("frog.json")
    cam = hs.camera(1920, 1080)
    rgb, hi, ht = _device_scene("frog.json").render(cam, spp=16, max_depth=8, aov=True)
    assert hashlib.sha256(hi.tobytes()).hexdigest() == meta["sha256"]["hits.i32"]
    assert hashlib.sha256(ht.tobytes()).hexdigest() == meta["sha256"]["hitt.f32"]
    _check_fb(rgb, golden_array("c3b_full", "fb.f32.gz", np.float32))
    assert rt.encode_p6(rgb) == gzip.open(GOLDEN / "scenes" / "c3b_full" / "image.ppm.gz").read()


@pytest.mark.parametrize("flags", [0, rt._lib.RT_FLAG_BINARY])
@pytest.mark.parametrize("kernel", KERNELS)
def test_sphere_scene_parity(kernel, flags):
    """sphere.json as shipped (G/assets/json_files/sphere.json: scaled sphere instances, mirrors
    with kr up to 0.95, shininess up to 100000, 128 spp, 4 bounces, no diffuse bounce) at 192x108
    against the reference's own render(): float frame bit for bit, hit AOVs by sha256."""
    meta = golden_meta("sphere")
    assert meta["spp"] == 128 and meta["max_depth"] == 4 and meta["diffuse_bounce"] == 0
    hs = host_scene("sphere.json")
    cam = hs.camera(meta["width"], meta["height"])
    rgb, hi, ht = _device_scene("sphere.json").render(cam, spp=128, max_depth=4, diffuse_bounce=False,
                                                      miss_color=hexv(meta["miss_color"]), aov=True,
                                                      kernel=kernel, flags=flags)
    assert hashlib.sha256(hi.tobytes()).hexdigest() == meta["sha256"]["hits.i32"]
    assert hashlib.sha256(ht.tobytes()).hexdigest() == meta["sha256"]["hitt.f32"]
    _check_fb(rgb, golden_array("sphere", "fb.f32.gz", np.float32))


@pytest.mark.parametrize("name,scene", [("sphere_full", "sphere.json"), ("sphere_single_full", "sphere_single.json")])
def test_shipped_scene_full_frames(name, scene):
    """The reference's other shipped scenes at their shipped size (1920x1080; sphere.json 128 spp
    4 mirror bounces, sphere_single.json 64 spp 4 diffuse bounces): the float frame and both
    hit AOVs equal the reference's own full-size outputs (sha256 of each)."""
    meta = golden_meta(name)
    hs = host_scene(scene)
    assert (meta["width"], meta["height"], meta["spp"]) == (1920, 1080, hs.settings["spp"])
    cam = hs.camera(1920, 1080)
    rgb, hi, ht = _device_scene(scene).render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                                              diffuse_bounce=bool(meta["diffuse_bounce"]),
                                              miss_color=hexv(meta["miss_color"]), aov=True)
    assert np.isfinite(rgb).all()
    assert hashlib.sha256(np.ascontiguousarray(rgb, np.float32).tobytes()).hexdigest() == meta["sha256"]["fb.f32"]
    assert hashlib.sha256(hi.tobytes()).hexdigest() == meta["sha256"]["hits.i32"]
    assert hashlib.sha256(ht.tobytes()).hexdigest() == meta["sha256"]["hitt.f32"]


@pytest.mark.parametrize("env", [{}, {"heavy_cap": 8}, {"heavy_frac": 0.0001}])
def test_heavy_first_dispatch_changes_nothing(env, tune):
    """Heavy-first dispatch (the previous frames' per-tile costs order the render blocks; full
    heavy lists spill into the survivor lists; a tiny threshold makes every tile heavy): frames
    after the first take the heavy path and still equal the reference's c3 frame, also after
    the camera moved (stale costs) and back."""
    tune(**env)
    meta = golden_meta("c3_full")
    hs = host_scene("frog.json")
    cam = hs.camera(1920, 1080)
    moved = rt.Camera(tuple(np.add(cam.pos, (0.05, 0.02, 0.0))), cam.look_at, cam.up, cam.focal_length_mm,
                      cam.sensor_height_mm, 1920, 1080)
    ds = rt.DeviceScene.from_host(hs, device=0)
    heavy = []
    for c in (cam, cam, moved, cam, cam):
        rgb, hi, ht = ds.render(c, spp=16, max_depth=1, aov=True)
        heavy.append(ds.heavy_tiles())
        if c is cam:
            assert hashlib.sha256(hi.tobytes()).hexdigest() == meta["sha256"]["hits.i32"]
            assert hashlib.sha256(ht.tobytes()).hexdigest() == meta["sha256"]["hitt.f32"]
            _check_fb(rgb, golden_array("c3_full", "fb.f32.gz", np.float32))
    assert heavy[0] == 0 and heavy[1] > 0 and heavy[4] > 0, heavy
    if "heavy_cap" in env:
        assert heavy[4] <= 8 * 3 * int(env["heavy_cap"])
    ds.close()


@pytest.mark.parametrize("tiles", [rt.RT_TILES_ROWS, rt.RT_TILES_LINEAR])
@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("spp,W,H", [(1, 37, 23), (3, 40, 21), (64, 9, 7), (2, 1, 1), (16, 65, 3), (128, 12, 9),
                                     (256, 7, 5)])
def test_odd_shapes_against_oracle(spp, W, H, kernel, tiles):
    """spp 128 / 256: a pixel's samples span the block's waves, and the work queues hand out
    whole tiles (one barrier per item) instead of wave quarters."""
    hs = host_scene("frog.json")
    cam = hs.camera(W, H)
    rgb, hi, ht = _device_scene("frog.json").render(cam, spp=spp, max_depth=1, aov=True, kernel=kernel,
                                                    tile_order=tiles)
    ref, rhi, rht = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                                 hs.tri_object_ids, hs.materials, hs.lights, spp=spp, max_depth=1, aov=True)
    assert np.array_equal(hi, rhi)
    assert np.array_equal(ht.view(np.uint32), rht.view(np.uint32))
    _check_fb(rgb, ref)


@pytest.mark.parametrize("spp", [128, 5])
def test_bounces_whole_tile_items_against_oracle(spp):
    """Multi-bounce frames through the work queues' whole-tile items (spp 128) and the
    pixel-loop kernel (spp 5), against the oracle."""
    hs = host_scene("frog.json")
    cam = hs.camera(10, 7)
    rgb, hi, ht = _device_scene("frog.json").render(cam, spp=spp, max_depth=4, aov=True)
    ref, rhi, rht = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                                 hs.tri_object_ids, hs.materials, hs.lights, spp=spp, max_depth=4, aov=True)
    assert np.array_equal(hi, rhi)
    assert np.array_equal(ht.view(np.uint32), rht.view(np.uint32))
    _check_fb(rgb, ref)


@pytest.mark.parametrize("kernel", KERNELS)
def test_multibounce_mirror_path_against_oracle(kernel):
    """diffuse_bounce = false: every bounce takes the mirror branch (query.h:207-212)."""
    hs = host_scene("cornell.json")
    cam = hs.camera(64, 48)
    rgb = _device_scene("cornell.json").render(cam, spp=2, max_depth=4, diffuse_bounce=False,
                                              miss_color=(0.1, 0.2, 0.3), kernel=kernel)
    ref = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                       hs.tri_object_ids, hs.materials, hs.lights, spp=2, max_depth=4, diffuse_bounce=False,
                       miss=(0.1, 0.2, 0.3))
    _check_fb(rgb, ref)


@pytest.mark.parametrize("band_count", [2, 3, 8])
def test_band_shards_reassemble_to_the_full_frame(band_count):
    hs = host_scene("frog.json")
    cam = hs.camera(192, 108)
    ds = _device_scene("frog.json")
    full = ds.render(cam, spp=16)
    out = np.zeros_like(full)
    for b in range(band_count):
        strip = ds.render(cam, spp=16, band_rows=8, band_index=b, band_count=band_count)
        rows = [y for y in range(108) if (y // 8) % band_count == b]
        assert strip.shape[0] == len(rows)
        out[rows] = strip
    assert np.array_equal(out.view(np.uint32), full.view(np.uint32))


def test_reference_signature_render():
    meta = golden_meta("c3_small")
    hs = host_scene("frog.json")
    cam = hs.camera(meta["width"], meta["height"])
    out = np.zeros(meta["width"] * meta["height"] * 3, np.float32)
    rt.render(hs.num_triangles, meta["width"], meta["height"], cam, (0, 0, 0), 1, 16, hs.nodes, hs.aabbs,
              hs.triangles, hs.tri_object_ids, hs.materials, hs.materials.shape[0], hs.lights, hs.lights.shape[0],
              True, out)
    _check_fb(out, golden_array("c3_small", "fb.f32.gz", np.float32))


def test_scene_without_materials_or_lights_uses_defaults():
    hs = host_scene("frog.json")
    cam = hs.camera(48, 27)
    ds = rt.DeviceScene(hs.num_triangles, hs.nodes, hs.aabbs, hs.triangles, None, None, None)
    rgb = ds.render(cam, spp=2)
    empty_l = np.zeros(0, rt.LIGHT_DTYPE)
    ref = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles, None, None, empty_l,
                       spp=2)
    _check_fb(rgb, ref)


def test_single_triangle_scene(tmp_path):
    obj = tmp_path / "tri.obj"
    obj.write_text("v -1 1 -1\nv 1 1 -1\nv 0 1 1\nf 1 2 3\n")
    hs = rt.HostScene.load_objs([obj])
    cam = rt.Camera((0, -2, 0), (0, 0, 0), (0, 0, 1), 35, 24, 32, 24)
    rgb, hi, _ = rt.DeviceScene.from_host(hs).render(cam, spp=4, aov=True)
    ref, rhi, _ = orc.render_g(1, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids,
                               hs.materials, hs.lights, spp=4, aov=True)
    assert np.array_equal(hi, rhi) and (hi >= 0).any()
    _check_fb(rgb, ref)


@pytest.mark.parametrize("flags", [0, rt._lib.RT_FLAG_BINARY])
def test_inverted_boxes_follow_the_reference(flags):
    """AABBs with min > max on an axis (malformed input the reference still traverses, its
    slab test swapping the two parameters): the float pre-classification is switched off for
    such a scene and every box test takes the exact path, so hits match the oracle."""
    hs = host_scene("frog.json")
    aabbs = hs.aabbs.copy()
    rng = np.random.default_rng(5)
    pick = rng.choice(np.arange(1, len(aabbs)), size=len(aabbs) // 50, replace=False)
    aabbs[pick, 0], aabbs[pick, 3] = aabbs[pick, 3].copy(), aabbs[pick, 0].copy()  # swap x min/max
    ds = rt.DeviceScene(hs.num_triangles, hs.nodes, aabbs, hs.triangles, hs.tri_object_ids, hs.materials, hs.lights)
    cam = hs.camera(160, 90)
    rgb, hi, ht = ds.render(cam, spp=4, max_depth=1, aov=True, flags=flags)
    ref, rhi, rht = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, aabbs, hs.triangles,
                                 hs.tri_object_ids, hs.materials, hs.lights, spp=4, max_depth=1, aov=True)
    assert np.array_equal(hi, rhi) and (hi >= 0).any()
    assert np.array_equal(ht.view(np.uint32), rht.view(np.uint32))
    _check_fb(rgb, ref)


def test_malformed_bvh_is_rejected():
    hs = host_scene("frog.json")
    nodes = hs.nodes.copy()
    nodes[0, 1] = 0  # root's left child -> root: a cycle
    with pytest.raises(rt.RTError, match="cycle"):
        rt.DeviceScene(hs.num_triangles, nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials, hs.lights)
    nodes = hs.nodes.copy()
    nodes[3, 2] = 10 ** 9
    with pytest.raises(rt.RTError, match="out of range"):
        rt.DeviceScene(hs.num_triangles, nodes, hs.aabbs, hs.triangles, hs.tri_object_ids, hs.materials, hs.lights)


def test_device_kat_matches_reference_answers():
    doc = json.loads((GOLDEN / "kat_hw1.json").read_text())
    tri = doc["triangle"]
    t18 = np.array(tri["v0"] + tri["v1"] + tri["v2"] + tri["n"] * 3, np.float32)
    dirs = np.array([[float.fromhex(x) for x in r["dir"]] for r in doc["rays"]], np.float32)
    want = np.array([r["hit"] for r in doc["rays"]], np.int32)
    wt = np.array([float.fromhex(r["t"]) for r in doc["rays"]], np.float32)
    hit, t = rt.intersect_rays(t18, dirs, hw1=True)
    assert np.array_equal(hit, want)  # 60 hits, 5 misses incl. the reference's sweep point 41
    assert np.array_equal(t.view(np.uint32), wt.view(np.uint32))


def test_device_intersect_g_against_oracle():
    rng = np.random.default_rng(7)
    t18 = np.concatenate([rng.normal(size=9).astype(np.float32) + np.array([0, 0, -3] * 3, np.float32),
                          np.zeros(9, np.float32)])
    dirs = rng.normal(size=(20000, 3)).astype(np.float32)
    dirs[:, 2] = -np.abs(dirs[:, 2])
    for tmin, tmax in [(0.0, 3.4e38), (1e-4, 3.0)]:
        h, t = rt.intersect_rays(t18, dirs, hw1=False, tmin=tmin, tmax=tmax)
        rh, rtt = orc.intersect_g(t18, dirs, tmin=tmin, tmax=tmax)
        assert np.array_equal(h, rh) and np.array_equal(t.view(np.uint32), rtt.view(np.uint32))
        assert 0 < h.sum() < len(h)


HW1_CASES = {"c1_full": ("c1", 256, 256), "c2_small": ("c2", 160, 120), "c2_full": ("c2", 640, 480)}


@pytest.mark.parametrize("brute", [False, True])
@pytest.mark.parametrize("name", list(HW1_CASES))
def test_hw1_brute_force_parity(name, brute):
    """HW1 path against the reference's own outputs, binned (default) and brute force."""
    cfg, W, H = HW1_CASES[name]
    c = configs.HW1_CONFIGS[cfg]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], W, H, hw1=True)
    rgb, hi, ht = rt.render_hw1(mesh.positions, mesh.normals, mesh.indices, cam, c["light_pos"], c["light_color"],
                                spp=c["spp"], aov=True, brute=brute)
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32), golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))
    if (GOLDEN / "scenes" / name / "image.ppm.gz").exists():
        ppm = gzip.open(GOLDEN / "scenes" / name / "image.ppm.gz").read()
        mine = rt.encode_p6(rgb)
        n = len(f"P6\n{W} {H}\n255\n")
        d = np.abs(np.frombuffer(mine[n:], np.uint8).astype(int) - np.frombuffer(ppm[n:], np.uint8).astype(int))
        assert d.max() <= 1


def _soup(rng, n, kind):
    """Adversarial triangle soups for the binned HW1 path: mixed sizes and orientations, edge-on
    triangles whose plane passes (nearly) through the camera, triangles straddling the camera
    plane or behind it, slivers and huge triangles."""
    cam_pos = np.array([0.3, -2.0, 0.7], np.float32)
    if kind == "mixed":
        c = rng.normal(size=(n, 1, 3)) * np.array([1.0, 1.0, 0.6])
        size = np.exp(rng.uniform(np.log(1e-3), np.log(2.0), size=(n, 1, 1)))
        v = c + rng.normal(size=(n, 3, 3)) * size
    elif kind == "edge_on":
        # planes through (or 1e-7 .. 1e-3 off) the camera centre
        a = rng.normal(size=(n, 1, 3)) * 1.5
        b = rng.normal(size=(n, 1, 3)) * 1.5
        s, t = rng.uniform(0.2, 1.5, size=(n, 3, 1)), rng.uniform(-0.5, 0.5, size=(n, 3, 1))
        v = cam_pos + s * a + t * b
        off = np.where(rng.uniform(size=(n, 1, 1)) < 0.5, 0.0, 10 ** rng.uniform(-7, -3, size=(n, 1, 1)))
        v = v + off * rng.normal(size=(n, 1, 3))
    elif kind == "around":
        # large triangles around / behind / through the camera
        v = cam_pos + rng.normal(size=(n, 3, 3)) * 3.0
    else:  # slivers
        p0 = rng.normal(size=(n, 1, 3))
        dirn = rng.normal(size=(n, 1, 3))
        v = np.concatenate([p0, p0 + dirn, p0 + dirn * rng.uniform(0.3, 0.7, size=(n, 1, 1))
                            + 1e-5 * rng.normal(size=(n, 1, 3))], axis=1)
    pos = v.reshape(-1, 3).astype(np.float32)
    nrm = rng.normal(size=pos.shape).astype(np.float32)
    idx = np.arange(len(pos), dtype=np.uint32)
    return pos, nrm, idx, cam_pos


@pytest.mark.parametrize("kind", ["mixed", "edge_on", "around", "slivers"])
@pytest.mark.parametrize("spp", [1, 4])
def test_hw1_binned_equals_brute_force_fuzz(kind, spp):
    """The binned HW1 kernel skips triangles by a conservative pixel rectangle: it must return
    the brute-force loop's winner (first index with the smallest t) bit for bit."""
    rng = np.random.default_rng({"mixed": 1, "edge_on": 2, "around": 3, "slivers": 4}[kind] * 10 + spp)
    pos, nrm, idx, cam_pos = _soup(rng, 3000, kind)
    cam = rt.Camera(tuple(cam_pos), (0.0, 0.0, 0.2), (0.0, 0.0, 1.0), 30.0, 24.0, 96, 72, hw1=True)
    args = (pos, nrm, idx, cam, (-3.0, 0.0, 1.0), (1.0, 0.0, 1.0))
    a_rgb, a_hi, a_ht = rt.render_hw1(*args, spp=spp, aov=True)
    b_rgb, b_hi, b_ht = rt.render_hw1(*args, spp=spp, aov=True, brute=True)
    assert (b_hi >= 0).mean() > {"mixed": 0.05, "around": 0.05, "edge_on": 5e-4, "slivers": 5e-4}[kind]
    assert np.array_equal(a_hi, b_hi)
    assert np.array_equal(a_ht.view(np.uint32), b_ht.view(np.uint32))
    assert np.array_equal(a_rgb.view(np.uint32), b_rgb.view(np.uint32))


def test_hw1_multisample_against_oracle():
    c = configs.HW1_CONFIGS["c2"]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], 64, 48, hw1=True)
    rgb, hi, _ = rt.render_hw1(mesh.positions, mesh.normals, mesh.indices, cam, c["light_pos"], c["light_color"],
                               spp=16, aov=True)
    ref, rhi, _ = orc.render_hw1(mesh.positions, mesh.normals, mesh.indices, oracle_camera(cam), c["light_pos"],
                                 c["light_color"], spp=16, aov=True)
    assert np.array_equal(hi, rhi)
    _check_fb(rgb, ref)


def test_full_size_c5_matches_reference():
    """BASELINE config 5 on one GPU at its full size (3840x2160x64, 1,048,576 triangles, depth 1)
    against the reference's own CPU render() of the same scene (tests/golden/scenes/c5_full:
    oracle/_ref/ref_g, 42 CPU-minutes): the float frame, the primary-hit index and t buffers
    (530,841,600 samples each) and the P6 file write_p6 makes of the frame, by sha256."""
    meta = golden_meta("c5_full")
    hs = host_scene("heightfield_c5.json")
    for k in ("nodes.bin", "aabbs.bin", "tris.bin"):  # the same scene arrays as the reference's
        assert meta["sha256"][k] == golden_meta("c5_small")["sha256"][k]
    cam = hs.camera(3840, 2160)
    ds = _device_scene("heightfield_c5.json")
    rgb, hi, ht = ds.render(cam, spp=64, max_depth=1, miss_color=hexv(meta["miss_color"]), aov=True)
    assert ds.faults() == 0
    sha = meta["sha256"]
    assert hashlib.sha256(hi.tobytes()).hexdigest() == sha["hits.i32"], f"{int((hi >= 0).sum())} hits"
    del hi
    assert hashlib.sha256(ht.tobytes()).hexdigest() == sha["hitt.f32"]
    del ht
    assert hashlib.sha256(rgb.tobytes()).hexdigest() == sha["fb.f32"]
    assert hashlib.sha256(rt.encode_p6(rgb)).hexdigest() == sha["image.ppm"]


@pytest.mark.parametrize("force_cut", [False, True])
@pytest.mark.parametrize("scene", ["frog.json", "cornell.json", "sphere_single.json"])
def test_tile_culling_changes_nothing(scene, force_cut, tune):
    """Tile culling against the root box (and, forced on for every camera, against the 64-box
    cut of the tree) is exact: random cameras (near, far, inside the box, grazing, far from
    the origin) give bit-identical frames and hit AOVs with it on and off."""
    if force_cut:
        tune(cull_coverage=1.0)
    hs = host_scene(scene)
    ds = _device_scene(scene)
    box = np.concatenate([hs.aabbs[0, :3], hs.aabbs[0, 3:]])
    ctr = (box[:3] + box[3:]) / 2
    ext = np.linalg.norm(box[3:] - box[:3])
    rng = np.random.default_rng(11)
    for k in range(12):
        dist_ = ext * rng.choice([0.3, 0.8, 2.0, 10.0, 200.0])
        pos = ctr + rng.normal(size=3) * dist_
        look = ctr + rng.normal(size=3) * ext * rng.choice([0.0, 0.5, 3.0])
        if k == 0:
            pos = ctr  # inside the box
        up = (0.0, 0.0, 1.0) if k % 2 else (0.0, 1.0, 0.0)
        cam = rt.Camera(pos, look, up, float(rng.choice([18.0, 50.0, 300.0])), 24.0, 96, 64)
        a = ds.render(cam, spp=4, max_depth=1, aov=True)
        b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_NO_CULL)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), k


@pytest.mark.parametrize("spp", [3, 16])
def test_720p_frame_rows_against_oracle(spp):
    """A 1280x720 frame for the sample-per-lane (16 spp) and pixel-per-lane (3 spp) kernels:
    rows through the frog against the oracle."""
    hs = host_scene("frog.json")
    cam = hs.camera(1280, 720)
    ds = _device_scene("frog.json")
    b = ds.render(cam, spp=spp, max_depth=1, aov=True)
    ref = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                       hs.tri_object_ids, hs.materials, hs.lights, spp=spp, max_depth=1, rows=(352, 368))
    _check_fb(b[0][352:368], ref[352:368])


@pytest.mark.parametrize("scene", ["frog.json", "cornell.json", "sphere_single.json"])
def test_cut_culling_fuzz_grazing_cameras(scene, tune):
    """The float tile bounds of both culling passes (root box and 64-box cut) against many
    cameras aimed at box faces, edges and corners from near and far, with tiny and wide fields
    of view: culled frames are bit-identical to unculled ones."""
    tune(cull_coverage=1.0)
    hs = host_scene(scene)
    ds = _device_scene(scene)
    box = np.concatenate([hs.aabbs[0, :3], hs.aabbs[0, 3:]]).astype(np.float64)
    lo, hi = box[:3], box[3:]
    ext = float(np.linalg.norm(hi - lo))
    rng = np.random.default_rng(2024)
    for k in range(40):
        # a point on a face / edge / corner of the root box or of a random sub-box
        t = rng.choice([0.0, 1.0, 0.5, rng.uniform()], size=3)
        target = lo + t * (hi - lo)
        dirn = rng.normal(size=3)
        dirn /= np.linalg.norm(dirn)
        pos = target + dirn * ext * rng.choice([0.05, 0.6, 3.0, 50.0])
        up = (0.0, 0.0, 1.0) if abs(dirn[2]) < 0.9 else (0.0, 1.0, 0.0)
        cam = rt.Camera(tuple(pos), tuple(target), up, float(rng.choice([8.0, 35.0, 600.0])), 24.0, 80, 48)
        a = ds.render(cam, spp=4, max_depth=1, aov=True)
        b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_NO_CULL)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), k


@pytest.mark.parametrize("scene", ["frog.json", "cornell.json", "sphere_single.json"])
def test_frustum_loose_axis_cameras(scene):
    """Waves whose direction interval reaches |d| < 1e-8 on an axis (the camera's axis planes cross
    the image through 2x2-pixel quads) take the frustum loop with a one-sided bound on that axis
    (traverse_frustum, LOOSE): cameras a little off the scene's symmetric positions, looking along
    and across the axes, with the planes d.x = 0 / d.y = 0 / d.z = 0 through the image; frames and
    hit AOVs bit for bit against the binary-record traversal (no frustum) and the oracle."""
    hs = host_scene(scene)
    ds = _device_scene(scene)
    box = np.concatenate([hs.aabbs[0, :3], hs.aabbs[0, 3:]]).astype(np.float64)
    ctr = (box[:3] + box[3:]) / 2
    ext = float(np.linalg.norm(box[3:] - box[:3]))
    base = hs.camera(96, 64)
    cams = [rt.Camera(tuple(np.add(base.pos, off)), base.look_at, base.up, base.focal_length_mm,
                      base.sensor_height_mm, 96, 64)
            for off in [(5e-4 * ext, 0, 0), (0, 0, 3e-3 * ext), (-2e-3 * ext, 1e-3 * ext, 0), (1e-6, 0, 0)]]
    for k, (axis, up) in enumerate([((0, 1, 0), (0, 0, 1)), ((1, 0, 0), (0, 0, 1)), ((0, 0, 1), (0, 1, 0)),
                                    ((1, 1, 0), (0, 0, 1))]):
        d = np.array(axis, np.float64) / np.linalg.norm(axis)
        for dist_ in (0.7, 2.5):
            pos = ctr - d * ext * dist_ + np.array([3e-4, -2e-4, 1e-4]) * ext * (k + 1)
            cams.append(rt.Camera(tuple(pos), tuple(pos + d), up, 20.0, 24.0, 96, 64))
    for i, cam in enumerate(cams):
        a = ds.render(cam, spp=4, max_depth=1, aov=True)
        b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_BINARY)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), i
        if i % 3 == 0:
            ref, rhi, _ = orc.render_g(hs.num_triangles, oracle_camera(cam), hs.nodes, hs.aabbs, hs.triangles,
                                       hs.tri_object_ids, hs.materials, hs.lights, spp=4, max_depth=1, aov=True)
            assert np.array_equal(a[1], rhi), i
            _check_fb(a[0], ref)


@pytest.mark.parametrize("sub", [0, 2, 16, 64])
@pytest.mark.parametrize("scene", ["frog.json", "cornell.json"])
def test_cut_sub_boxes_fuzz_grazing_cameras(scene, sub, tune):
    """The cut's second level (RT_TUNE_CUT_SUB sub-boxes below each of the 64 cut boxes,
    tile_cut_sub): cameras aimed at the faces, edges and corners of boxes of random internal
    nodes at every depth of the tree (the sub-boxes' own boxes among them), from near and far,
    narrow and wide fields of view: culled frames are bit-identical to unculled ones, and to the
    frames of a scene with one cut level."""
    tune(cull_coverage=1.0, cut_sub=sub)
    hs = host_scene(scene)
    ds = rt.DeviceScene.from_host(hs, device=0)
    try:
        internal = np.nonzero(hs.nodes[:, 3] == 0xFFFFFFFF)[0]
        rng = np.random.default_rng(77 + sub)
        for k in range(24):
            n = int(rng.choice(internal))
            lo = hs.aabbs[n, :3].astype(np.float64)
            hi = hs.aabbs[n, 3:].astype(np.float64)
            ext = max(float(np.linalg.norm(hi - lo)), 1e-3)
            t = rng.choice([0.0, 1.0, 0.5, rng.uniform()], size=3)
            target = lo + t * (hi - lo)
            dirn = rng.normal(size=3)
            dirn /= np.linalg.norm(dirn)
            pos = target + dirn * ext * rng.choice([0.3, 2.0, 20.0, 400.0])
            up = (0.0, 0.0, 1.0) if abs(dirn[2]) < 0.9 else (0.0, 1.0, 0.0)
            cam = rt.Camera(tuple(pos), tuple(target), up, float(rng.choice([8.0, 35.0, 600.0])), 24.0, 80, 48)
            a = ds.render(cam, spp=4, max_depth=1, aov=True)
            b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_NO_CULL)
            for x, y in zip(a, b):
                assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), (k, n)
    finally:
        ds.close()


def test_hw1_timing_entry_point():
    """rt_render_hw1_ex with kernel timing: a positive device time and the same image."""
    c = configs.HW1_CONFIGS["c1"]
    mesh = rt.MeshHW1(configs.MESHES / c["mesh"])
    cam = rt.Camera(c["position"], c["look_at"], c["up"], c["focal_mm"], c["sensor_mm"], 64, 64, hw1=True)
    args = (mesh.positions, mesh.normals, mesh.indices, cam, c["light_pos"], c["light_color"])
    rgb, ms = rt.render_hw1(*args, timing=True)
    rgb_b, ms_b = rt.render_hw1(*args, timing=True, brute=True)
    assert ms > 0 and ms_b > 0
    assert np.array_equal(rgb.view(np.uint32), rgb_b.view(np.uint32))


# RT_TUNE_FRUSTUM_ARITY caps the arity rt_scene_create picks (log2: 2 = the 4-ary records,
# 5 = 32-ary); None = the shipped default (32-ary where the stack bound fits: frog 91, c5 126)
ARITIES = [None, 5, 4, 3, 2]


@pytest.mark.parametrize("arity", ARITIES)
@pytest.mark.parametrize("name", ["c3_small", "frog_bounce", "sphere_single", "cornell", "c5_small", "c3b_small"])
def test_frustum_record_arity_parity(name, arity, tune):
    """The camera rays' frustum traversal over 4-, 8-, 16- and 32-ary records and the default:
    the reference's hits, t and frame bit for bit."""
    tune(frustum_arity=arity)
    meta = golden_meta(name)
    hs = host_scene(G_SCENES[name])
    cam = hs.camera(meta["width"], meta["height"])
    ds = rt.DeviceScene.from_host(hs, device=0)
    info = ds.traversal_info()
    if arity is None and name in ("c3_small", "c3b_small", "frog_bounce", "c5_small"):
        assert info["frustum_log2"] == 5 and 64 < info["frustum_bound"] <= 128, info
    rgb, hi, ht = ds.render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                            diffuse_bounce=bool(meta["diffuse_bounce"]), miss_color=hexv(meta["miss_color"]),
                            aov=True)
    assert ds.faults() == 0
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))


def _fuzz_cameras(hs, rng, n, W=96, H=64):
    """Cameras aimed at box faces, edges and corners, along the axes (direction components
    crossing zero inside a wave), from inside the scene's boxes, with tiny and wide fields of
    view."""
    lo, hi = hs.aabbs[0, :3].astype(np.float64), hs.aabbs[0, 3:].astype(np.float64)
    ext = float(np.linalg.norm(hi - lo))
    axes = [np.array(v, np.float64) for v in ((1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1))]
    for k in range(n):
        if k % 3 == 0:  # along an axis: the centre column / row has a zero direction component
            dirn = axes[k // 3 % 6]
        else:
            dirn = rng.normal(size=3)
            dirn /= np.linalg.norm(dirn)
        if k % 4 == 1:  # from inside the tree: a random internal box's centre
            m = int(rng.integers(0, len(hs.aabbs)))
            pos = (hs.aabbs[m, :3] + hs.aabbs[m, 3:]).astype(np.float64) / 2
            target = pos - dirn * ext
        else:
            t = rng.choice([0.0, 1.0, 0.5, rng.uniform()], size=3)
            target = lo + t * (hi - lo)
            pos = target + dirn * ext * rng.choice([0.05, 0.6, 3.0])
        fwd = target - pos
        up = (0.0, 0.0, 1.0) if abs(fwd[2]) < 0.9 * np.linalg.norm(fwd) else (0.0, 1.0, 0.0)
        yield k, rt.Camera(tuple(pos), tuple(target), up, float(rng.choice([8.0, 35.0, 600.0])), 24.0, W, H)


@pytest.mark.parametrize("greedy", [2, 1, 0])
@pytest.mark.parametrize("arity", [None, 5, 4, 3])
@pytest.mark.parametrize("scene", ["frog.json", "cornell.json", "sphere_single.json"])
def test_frustum_fuzz_cameras(scene, arity, greedy, tune):
    """The frustum traversal's wave-level box test must pass whenever some lane's exact test
    does (adversarial cameras, _fuzz_cameras): frames (hits, t, colour) bit-identical to the
    binary-record traversal, which tests every box for every lane.  At the shipped arity (None,
    5: 32-ary records, frog's bound 94 greedy / 91 fixed-depth) the DFS uses the stack's second
    VGPR.  Both record rules (RT_TUNE_RECORD_GREEDY)."""
    tune(frustum_arity=arity, record_greedy=greedy)
    hs = host_scene(scene)
    ds = rt.DeviceScene.from_host(hs, device=0)
    for k, cam in _fuzz_cameras(hs, np.random.default_rng(7), 36):
        a = ds.render(cam, spp=4, max_depth=1, aov=True)
        b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_BINARY)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), k
    assert ds.faults() == 0


def test_frustum_fuzz_cameras_c5():
    """The c5 heightfield (1M triangles) at its shipped 32-ary records, whose DFS bound (126)
    sits next to the 128-entry stack: grazing, axis-aligned, inside-the-tree and far cameras at
    reduced resolution against the binary-record traversal, bit for bit."""
    hs = host_scene("heightfield_c5.json")
    ds = _device_scene("heightfield_c5.json")
    info = ds.traversal_info()
    assert info["frustum_log2"] == 5 and 120 < info["frustum_bound"] <= 128, info
    rng = np.random.default_rng(55)
    cams = list(_fuzz_cameras(hs, rng, 12, 64, 48))
    # grazing: just above the surface, looking along it
    for k, (x, y) in enumerate(((-1.9, -0.9), (1.9, 0.9), (0.0, -0.95), (-1.95, 0.0))):
        cams.append((100 + k, rt.Camera((x, y, 0.12), (-x, -y, 0.05), (0.0, 0.0, 1.0), 20.0, 24.0, 64, 48)))
    for k, cam in cams:
        a = ds.render(cam, spp=4, max_depth=1, aov=True, miss_color=(0.5, 0.7, 1.0))
        b = ds.render(cam, spp=4, max_depth=1, aov=True, miss_color=(0.5, 0.7, 1.0), flags=rt._lib.RT_FLAG_BINARY)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), k
    assert ds.faults() == 0


def _spine(L):
    import spine_bvh

    a = spine_bvh.as_arrays(spine_bvh.spine_scene(L))
    ds = rt.DeviceScene(a["P"], a["nodes"], a["aabbs"], a["tris"], a["objids"], a["mats"], a["lights"])
    pos, look, up, f, s = spine_bvh.CAMERA
    return a, ds, rt.Camera(pos, look, up, f, s, 48, 32)


@pytest.mark.parametrize("L,log2", [(15, 5), (30, 4), (35, 3)])
def test_spine_trees_deep_frustum_stack(L, log2, tune):
    """Trees whose frustum DFS goes past 64 stack entries (tests/spine_bvh.py): 32-ary records
    with bound 109, and trees whose 32-ary bound exceeds the 128-entry stack, which take 16-ary
    (bound 124) or 8-ary records instead.  The centre rays reach more than 64 entries before
    their first leaf (tests/test_frustum_records.py).  Frames bit-identical to the binary-record
    traversal and to the oracle; no device fault.  (Records by the fixed-depth rule,
    RT_TUNE_RECORD_GREEDY = 0, which these trees were built to push past 64 entries.)"""
    tune(record_greedy=0)
    a, ds, cam = _spine(L)
    try:
        info = ds.traversal_info()
        assert info["frustum_log2"] == log2 and 64 < info["frustum_bound"] <= 128, info
        got = ds.render(cam, spp=4, max_depth=1, aov=True)
        ref_b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_BINARY)
        assert ds.faults() == 0
    finally:
        ds.close()
    for x, y in zip(got, ref_b):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))
    rgb, hi, ht = orc.render_g(a["P"], oracle_camera(cam), a["nodes"], a["aabbs"], a["tris"], a["objids"], a["mats"],
                               a["lights"], spp=4, max_depth=1, aov=True)
    assert np.array_equal(got[1], hi) and np.array_equal(got[2].view(np.uint32), ht.view(np.uint32))
    assert (hi >= 0).mean() > 0.3
    _check_fb(got[0], rgb)


def test_frustum_stack_overflow_guard_is_loud(tune):
    """The device guard on traverse_frustum's 128-entry stack: records built past it (the test
    hook RT_TUNE_FRUSTUM_STACK_CAP; rt_scene_create never does so by default) overflow on the
    spine tree's centre rays; the traversal drops the pushes instead of wrapping a lane index,
    raises RT_FAULT_FRUSTUM_STACK, and rt_render fails with RT_ERR_INTERNAL instead of
    returning a wrong frame."""
    tune(frustum_stack_cap=10**6, record_greedy=0)
    a, ds, cam = _spine(30)
    try:
        info = ds.traversal_info()
        assert info["frustum_log2"] == 5 and info["frustum_bound"] > 128, info
        with pytest.raises(rt.RTError) as e:
            ds.render(cam, spp=4, max_depth=1)
        assert e.value.code == -9 and "overflow" in str(e.value)
        assert ds.faults() & rt._lib.RT_FAULT_FRUSTUM_STACK
        assert ds.faults() == 0  # cleared by the previous call
        # the binary-record traversal does not use the frustum stack: a valid frame
        ds.render(cam, spp=4, max_depth=1, flags=rt._lib.RT_FLAG_BINARY)
        # the fault word belongs to the frame that raised it: a faulting frame left uncleared
        # does not fail the next, valid one
        with pytest.raises(rt.RTError):
            ds.render(cam, spp=4, max_depth=1)
        ds.render(cam, spp=4, max_depth=1, flags=rt._lib.RT_FLAG_BINARY)
        assert ds.faults() == 0
    finally:
        ds.close()


@pytest.mark.parametrize("arity", [None, 4, 3])
@pytest.mark.parametrize("name", ["c3_small", "sphere_single", "cornell", "c5_small"])
def test_quantised_records_parity(name, arity, tune):
    """The big-scene kernels' frustum traversal over the quantised records (16-bit grid steps,
    build_quant_records), forced onto small scenes (RT_TUNE_QUANT_RECORDS = 1 and a zero
    big-scene threshold): the reference's hits, t and frame bit for bit at every arity."""
    tune(frustum_arity=arity, quant_records=1, big_scene_bytes=0)
    meta = golden_meta(name)
    if meta["max_depth"] != 1:
        pytest.skip("the big-scene kernels are the depth-1 ones")
    hs = host_scene(G_SCENES[name])
    cam = hs.camera(meta["width"], meta["height"])
    ds = rt.DeviceScene.from_host(hs, device=0)
    rgb, hi, ht = ds.render(cam, spp=meta["spp"], max_depth=1, miss_color=hexv(meta["miss_color"]), aov=True)
    kn = ds.kernel_name()
    assert kn.startswith("render_tiles_kernel<433,") or kn.startswith("render_tiles_kernel<305,"), kn
    assert ds.faults() == 0
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))


@pytest.mark.parametrize("scene", ["frog.json", "cornell.json", "sphere_single.json"])
def test_quantised_records_fuzz_cameras(scene, tune):
    """Quantised records under the adversarial cameras (_fuzz_cameras): frames bit-identical to
    the binary-record traversal."""
    tune(quant_records=1, big_scene_bytes=0)
    hs = host_scene(scene)
    ds = rt.DeviceScene.from_host(hs, device=0)
    for k, cam in _fuzz_cameras(hs, np.random.default_rng(19), 24):
        a = ds.render(cam, spp=4, max_depth=1, aov=True)
        assert ",".join(ds.kernel_name().split(",")[:1]) in ("render_tiles_kernel<433", "render_tiles_kernel<305")
        b = ds.render(cam, spp=4, max_depth=1, aov=True, flags=rt._lib.RT_FLAG_BINARY)
        for x, y in zip(a, b):
            assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32)), k
    assert ds.faults() == 0


def test_c5_quantised_records_auto(tune):
    """RT_TUNE_QUANT_RECORDS = -1: the c5 heightfield (34 MB of 32-ary float records) renders
    through the quantised records' kernel, frog (0.6 MB) does not; c5 rows through it against the
    binary-record traversal, bit for bit.  The shipped default (0) keeps the float records."""
    hs = host_scene("heightfield_c5.json")
    assert _device_scene("heightfield_c5.json").render(hs.camera(64, 48), spp=1, max_depth=1) is not None
    assert _device_scene("heightfield_c5.json").kernel_name().startswith("render_tiles_kernel<177,")
    tune(quant_records=-1)
    ds = rt.DeviceScene.from_host(hs, device=0)
    cam = hs.camera(480, 270)
    a = ds.render(cam, spp=4, max_depth=1, aov=True, miss_color=(0.5, 0.7, 1.0))
    assert ds.kernel_name().startswith("render_tiles_kernel<433,"), ds.kernel_name()
    b = ds.render(cam, spp=4, max_depth=1, aov=True, miss_color=(0.5, 0.7, 1.0), flags=rt._lib.RT_FLAG_BINARY)
    for x, y in zip(a, b):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))
    assert ds.faults() == 0
    ds.close()
    fr = rt.DeviceScene.from_host(host_scene("frog.json"), device=0)
    fr.render(host_scene("frog.json").camera(64, 48), spp=1, max_depth=1)
    assert not fr.kernel_name().startswith("render_tiles_kernel<433,"), fr.kernel_name()


@pytest.mark.parametrize("wide4,frustum", [(0, 1), (1, 0), (0, 0)])
@pytest.mark.parametrize("name", ["c3_small", "frog_bounce", "sphere_single", "cornell", "c5_small", "c3b_small"])
def test_record_rules_parity(name, wide4, frustum, tune):
    """The record rules off their defaults (greedy 32-ary frustum records and greedy 4-ary
    records, RT_TUNE_RECORD_GREEDY / RT_TUNE_WIDE4_GREEDY; the fixed-depth forms): every
    combination gives the reference's hits, t and frame bit for bit (the shadow rays and the
    bounce rays walk the 4-ary records)."""
    tune(wide4_greedy=wide4, record_greedy=frustum)
    meta = golden_meta(name)
    hs = host_scene(G_SCENES[name])
    cam = hs.camera(meta["width"], meta["height"])
    ds = rt.DeviceScene.from_host(hs, device=0)
    rgb, hi, ht = ds.render(cam, spp=meta["spp"], max_depth=meta["max_depth"],
                            diffuse_bounce=bool(meta["diffuse_bounce"]), miss_color=hexv(meta["miss_color"]),
                            aov=True)
    assert ds.faults() == 0
    assert np.array_equal(hi.reshape(-1), golden_array(name, "hits.i32.gz", np.int32))
    assert np.array_equal(ht.reshape(-1).view(np.uint32),
                          golden_array(name, "hitt.f32.gz", np.float32).view(np.uint32))
    _check_fb(rgb, golden_array(name, "fb.f32.gz", np.float32))
