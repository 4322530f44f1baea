"""Host side of the boundary (CPU only): the C ABI loads and exports every declared symbol,
the loaders + CPU LBVH reproduce the reference's scene arrays byte for byte, the ppm_p6
writer reproduces the reference's P6 bytes, and the error paths behave."""
from __future__ import annotations

import ctypes as C
import gzip
import hashlib
import re

import numpy as np
import pytest

from conftest import GOLDEN, G_SCENES, REPO, golden_array, golden_meta, host_scene

import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import _lib, configs


def _declared_symbols():
    hdr = (REPO / "include" / "rt_mi355x.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", hdr)))


def test_c_abi_library_exports_every_declared_symbol():
    lib = C.CDLL(str(_lib.LIB_PATH))
    syms = _declared_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)
    assert lib.rt_abi_version() == 3


def test_struct_layouts_match_reference_pods():
    # sizes measured from the reference build (tests/golden/scenes/*/meta.json) and bvh.h/MeshOBJ.h
    meta = golden_meta("c3_small")
    assert C.sizeof(_lib.Material) == meta["sizeof_material"] == 52
    assert C.sizeof(_lib.Light) == meta["sizeof_light"] == 28
    assert C.sizeof(_lib.BVHNode) == 16 and C.sizeof(_lib.AABB) == 24 and C.sizeof(_lib.Triangle) == 72
    assert _lib.Material.emission.offset == 40 and _lib.Material.kr.offset == 36


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("name", ["c3_small", "cornell", "sphere_single", "frog_bounce", "c5_small"])
def test_scene_arrays_byte_identical_to_reference(name):
    meta = golden_meta(name)
    hs = host_scene(G_SCENES[name])
    assert hs.num_triangles == meta["num_triangles"]
    for arr, f in [(hs.nodes, "nodes.bin"), (hs.aabbs, "aabbs.bin"), (hs.triangles, "tris.bin"),
                   (hs.tri_object_ids, "triobj.bin"), (hs.materials, "mats.bin"), (hs.lights, "lights.bin")]:
        assert _sha(arr) == meta["sha256"][f], f


def test_scene_settings_follow_json():
    s = host_scene("frog.json").settings
    assert s["max_depth"] == 8 and s["spp"] == 1 and s["diffuse_bounce"] is True
    assert s["miss_color"] == (0.0, 0.0, 0.0)
    hs = host_scene("cornell.json")
    assert hs.info.num_lights == 2 and hs.info.num_materials == 10  # 'front_wall' has no faces
    assert hs.lights["intensity"].tolist() == [3, 2]  # int truncation (scene.h:314)


def test_bvh_structure_invariants_c5():
    hs = host_scene("heightfield_c5.json")
    P = hs.num_triangles
    assert P == 1 << 20
    nodes = hs.nodes
    internal = nodes[:P - 1]
    assert np.all(internal[:, 3] == 0xFFFFFFFF)
    assert sorted(nodes[P - 1:, 3].tolist()) == list(range(P))
    child = np.concatenate([internal[:, 1], internal[:, 2]])
    assert len(np.unique(child)) == 2 * P - 2 and child.max() == 2 * P - 2
    assert hs.info.bvh_max_stack <= 64


def test_build_bvh_api_matches_scene_builder():
    hs = host_scene("frog.json")
    nodes, aabbs = rt.build_bvh(hs.positions, hs.indices)
    assert np.array_equal(nodes, hs.nodes) and np.array_equal(aabbs.view(np.uint32), hs.aabbs.view(np.uint32))


def test_single_triangle_scene(tmp_path):
    obj = tmp_path / "tri.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    hs = rt.HostScene.load_objs([obj])
    assert hs.num_triangles == 1 and hs.nodes.shape == (1, 4)
    assert hs.nodes[0, 3] == 0 and hs.info.bvh_max_stack == 1


def test_obj_negative_indices_objects_and_quads(tmp_path):
    obj = tmp_path / "q.obj"
    obj.write_text("o a\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf -4 -3 -2 -1\no b\n"
                   "v 0 0 1\nv 1 0 1\nv 0 1 1\nf 5 6 7\n")
    hs = rt.HostScene.load_objs([obj])
    assert hs.num_triangles == 3
    assert hs.indices.tolist() == [[0, 1, 2], [0, 2, 3], [4, 5, 6]]
    assert hs.tri_object_ids.tolist() == [0, 0, 1]
    assert hs.info.num_materials == 2


def test_obj_errors(tmp_path):
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(rt.RTError):
        rt.MeshHW1(bad)
    with pytest.raises(rt.RTError):
        rt.HostScene.load_objs([tmp_path / "missing.obj"])  # no geometry at all


def test_scene_json_errors(tmp_path):
    p = tmp_path / "s.json"
    p.write_text('{"scene": []}')
    with pytest.raises(rt.RTError, match="no valid objects"):
        rt.HostScene.load_json(p)
    p.write_text('{"scene": [ {"path": "x.obj"} ], }')
    with pytest.raises(rt.RTError, match="PARSE"):
        rt.HostScene.load_json(p)


def test_camera_rejects_zero_size_in_hw1_mode_and_clamps_in_g_mode():
    with pytest.raises(rt.RTError):
        rt.Camera(width=0, height=10, hw1=True)
    c = rt.Camera(width=0, height=0)
    assert (c.pixel_width, c.pixel_height) == (1, 1)


def test_hw1_mesh_loader():
    m = rt.MeshHW1(configs.MESHES / "sphere.obj")
    assert m.num_triangles == 960 and m.normals is not None
    f = rt.MeshHW1(configs.MESHES / "frog.obj")
    assert f.num_triangles == 19858 and f.positions.shape == (11874, 3)


@pytest.mark.parametrize("name", ["c1_full", "c3_small", "c2_full"])
def test_p6_writer_bytes_match_reference(name, tmp_path):
    meta = golden_meta(name)
    W, H = meta["width"], meta["height"]
    fb = golden_array(name, "fb.f32.gz", np.float32).reshape(H, W, 3)
    want = gzip.open(GOLDEN / "scenes" / name / "image.ppm.gz").read()
    assert rt.encode_p6(fb) == want
    out = tmp_path / "x.ppm"
    rt.write_p6(out, fb)
    assert out.read_bytes() == want
    back = rt.read_p6(out)
    assert back.shape == (H, W, 3)
    assert np.abs(back - np.clip(np.sqrt(np.clip(fb, 0, None)), 0, 1)).max() <= 0.5 / 255 + 1e-6


def test_p6_16bit_and_flip(tmp_path):
    fb = np.linspace(0, 1, 2 * 3 * 3, dtype=np.float32).reshape(2, 3, 3)
    b = rt.encode_p6(fb, maxval=65535, gamma2=False, flip_y=True)
    assert b.startswith(b"P6\n3 2\n65535\n")
    px = np.frombuffer(b[len(b"P6\n3 2\n65535\n"):], ">u2").reshape(2, 3, 3)
    assert np.array_equal(px[0], np.round(fb[1] * 65535).astype(np.uint16))
    with pytest.raises(rt.RTError):
        rt.encode_p6(fb, maxval=0)


def test_shard_rows_partition_the_image():
    lib = _lib.lib()
    for H in (1, 7, 8, 1080, 2160):
        for n in (1, 2, 3, 4, 8):
            rows = [lib.rt_shard_rows(H, 8, i, n) for i in range(n)]
            assert sum(rows) == H


def test_render_entry_points_fail_loudly_without_device():
    # On a host with no gfx950 the HIP path must raise, never fall back to a CPU path.
    if rt.device_count() > 0:
        pytest.skip("a GPU is present")
    hs = host_scene("frog.json")
    with pytest.raises(rt.RTError, match="NODEVICE"):
        rt.DeviceScene.from_host(hs)


def test_p6_header_matches_writer_and_device_epilogue_checks_arguments():
    """rt_ppm_header is write_p6's header; the device epilogue's argument checks run on the host
    (no device touched) and return RT_ERR_ARG like write_p6's checks (ppm_p6.cpp:258-266)."""
    rgb = np.zeros((3, 5, 3), np.float32)
    assert rt.encode_p6(rgb)[:len(rt.p6_header(5, 3))] == rt.p6_header(5, 3) == b"P6\n5 3\n255\n"
    assert rt.p6_header(1920, 1080, 65535) == b"P6\n1920 1080\n65535\n"
    for bad in [(0, 3, 255), (5, -1, 255), (5, 3, 0), (5, 3, 65536)]:
        with pytest.raises(rt.RTError):
            rt.p6_header(*bad)
    with pytest.raises(rt.RTError):
        rt.quantize_p6_device(0, 5, 3, 0)
    with pytest.raises(rt.RTError):
        rt.quantize_p6_device(16, 5, 3, 16, maxval=70000)
    with pytest.raises(rt.RTError):
        rt.unpermute_strips_device(16, 2, 60, 16, 8, 4, 0)
    with pytest.raises(rt.RTError):  # 16 rows over 4 ranks of 4-row bands need 4 rows per strip
        rt.unpermute_strips_device(16, 3, 60, 16, 4, 4, 32)


def test_renderer_multiprocess_rccl_needs_unique_id():
    """A multi-process renderer that resolves to RCCL (explicitly, or AUTO without a shared host
    frame name) but has no unique_id is refused with RT_ERR_ARG before any device is touched
    (it used to read the id through a null pointer)."""
    hs = host_scene("frog.json")
    for gather in (rt.RT_GATHER_RCCL, rt.RT_GATHER_AUTO):
        with pytest.raises(rt.RTError, match="unique_id") as e:
            rt.Renderer.from_host(hs, devices=(0,), world_size=2, rank0=1, gather=gather)
        assert e.value.code == -1


def test_loaded_library_is_built_from_these_sources():
    """rt_build_id() of the loaded librt_mi355x.so is the sha256 of csrc/ + include/ + flags:
    a stale prebuilt library cannot pass for the current sources."""
    from raytracinginonesemester_amd import build as b

    lib = _lib.lib()
    assert lib.rt_build_id().decode() == b.source_build_id() == b.library_build_id()


def test_tuning_knobs_are_explicit():
    """The library reads no environment variables: knobs are set through rt_tuning_set (the
    header's rt_tune_id), read back, reset, and an unknown id is refused."""
    import raytracinginonesemester_amd as rt
    from raytracinginonesemester_amd import _lib

    so = (_lib.LIB_PATH).read_bytes()
    # (rocPRIM's headers, used by the device LBVH's sort, read their own variables)
    for src in (REPO / "raytracinginonesemester_amd" / "csrc").iterdir():
        assert "getenv" not in src.read_text(), src
    for name in (b"RT_FRUSTUM_ARITY", b"RT_HALF_WAVES", b"RT_HEAVY_FRAC", b"RT_CULL_COVERAGE", b"RT_RENDERER_SERIAL"):
        assert name not in so, name
    rt.reset_tuning()
    try:
        assert all(rt.get_tuning(k) is None for k in _lib.TUNE)
        rt.set_tuning("heavy_frac", 0.25)
        rt.set_tuning("half_waves", 1)
        assert rt.get_tuning("heavy_frac") == 0.25 and rt.get_tuning("half_waves") == 1.0
        with rt.tuning(heavy_frac=0.5, frustum_arity=3):
            assert rt.get_tuning("heavy_frac") == 0.5 and rt.get_tuning("frustum_arity") == 3.0
        assert rt.get_tuning("heavy_frac") == 0.25 and rt.get_tuning("frustum_arity") is None
        rt.set_tuning("heavy_frac", None)
        assert rt.get_tuning("heavy_frac") is None
        assert _lib.lib().rt_tuning_set(len(_lib.TUNE), 1.0) == -1
        assert _lib.lib().rt_tuning_set(-1, 1.0) == -1
    finally:
        rt.reset_tuning()
    assert all(rt.get_tuning(k) is None for k in _lib.TUNE)
    # the Python table names the header's enum, id for id
    import re

    hdr = (REPO / "include" / "rt_mi355x.h").read_text()
    ids = {m.group(1).lower(): int(m.group(2)) for m in re.finditer(r"RT_TUNE_([A-Z0-9_]+) = (\d+)", hdr)}
    ids.pop("count")
    assert ids == _lib.TUNE
