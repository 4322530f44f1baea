"""Trees deeper than the 64-entry wave stack, up to and past SearchBVH's 512-entry stack
(G/include/query.h:245-248, 279-293) and its brute-force completion (query.h:298-308).

Scenes: tests/golden/chain_bvh.py caterpillars (P = 300: ~300 DFS entries, no overflow;
P = 600: the reference's stack overflows and the brute-force pass decides the tie between two
identical triangles).  Goldens: the reference's own render() + SearchBVH on the same arrays
(tests/golden/gen_golden.py gen_chain, oracle/_ref/ref_g arrays).  Bar: bit-exact hit
indices, t and float framebuffer.
"""
from __future__ import annotations

import hashlib
import sys

import numpy as np
import pytest

from conftest import GOLDEN, golden_array, golden_meta, hexv
from oracle import pyoracle as orc

sys.path.insert(0, str(GOLDEN))
import chain_bvh  # noqa: E402

NAMES = list(chain_bvh.FIXTURES)


def chain(name):
    P, W, H, spp, depth = chain_bvh.FIXTURES[name]
    d = chain_bvh.chain_scene(P)
    meta = golden_meta(name)
    for k, a in (("nodes.bin", d["nodes"]), ("aabbs.bin", d["aabbs"]), ("tris.bin", d["tris"]),
                 ("triobj.bin", d["triobj"]), ("mats.bin", d["mats"]), ("lights.bin", d["lights"])):
        assert hashlib.sha256(a.tobytes()).hexdigest() == meta["sha256"][k], f"{name}: {k} differs from the golden's input"
    return {
        "P": P, "W": W, "H": H, "spp": spp, "depth": depth, "meta": meta,
        "nodes": d["nodes"].view(np.uint32).reshape(-1, 4), "aabbs": d["aabbs"], "tris": d["tris"],
        "objids": d["triobj"], "mats": d["mats"].view(np.float32).reshape(-1, 13), "lights": d["lights"],
        "perm": d["perm"],
    }


def goldens(name, c):
    W, H, spp = c["W"], c["H"], c["spp"]
    fb = golden_array(name, "fb.f32.gz", np.float32).reshape(H, W, 3)
    hi = golden_array(name, "hits.i32.gz", np.int32).reshape(H, W, spp)
    ht = golden_array(name, "hitt.f32.gz", np.float32).reshape(H, W, spp)
    return fb, hi, ht


def test_chain_goldens_exercise_the_deep_cases():
    """The fixtures contain what they are for: P = 300 keeps the DFS's own tie winner (level 0,
    the smaller index) on some rays; at P = 600 the rays whose DFS overflows the 512 entries end
    with the brute-force pass's (the larger index, level 3), off-centre rays that miss the far
    leaves do not overflow."""
    c3, c6 = chain("chain300"), chain("chain600")
    h3 = goldens("chain300", c3)[1]
    h6 = goldens("chain600", c6)[1]
    lo3, hi3 = int(c3["perm"][0]), int(c3["perm"][3])
    lo6, hi6 = int(c6["perm"][0]), int(c6["perm"][3])
    assert (h3 == lo3).any() and (h6 == hi6).any()
    assert (h6 == hi6).sum() > (h3 == hi3).sum() and (h6 == lo6).sum() < (h3 == lo3).sum()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference_on_deep_trees(name):
    c = chain(name)
    m = c["meta"]
    cam = orc.camera_from_basis(hexv(m["center"]), hexv(m["pixel00_loc"]), hexv(m["pixel_delta_u"]),
                                hexv(m["pixel_delta_v"]), c["W"], c["H"])
    rgb, hi, ht = orc.render_g(c["P"], cam, c["nodes"], c["aabbs"], c["tris"], c["objids"], c["mats"], c["lights"],
                               spp=c["spp"], max_depth=c["depth"], aov=True)
    fb, ghi, ght = goldens(name, c)
    assert np.array_equal(hi, ghi)
    assert np.array_equal(ht.view(np.uint32), ght.view(np.uint32))
    assert np.array_equal(rgb.view(np.uint32), fb.view(np.uint32))


def _camera(c):
    import raytracinginonesemester_amd as rt

    pos, look, up, f, s = chain_bvh.CAMERA
    cam = rt.Camera(pos, look, up, f, s, c["W"], c["H"])
    b = cam.basis()
    m = c["meta"]
    for k in ("center", "pixel00_loc", "pixel_delta_u", "pixel_delta_v"):
        assert np.array_equal(np.array(b[k], np.float32).view(np.uint32), hexv(m[k]).view(np.uint32)), k
    return cam


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_device_deep_tree_matches_reference(name):
    import raytracinginonesemester_amd as rt

    c = chain(name)
    ds = rt.DeviceScene(c["P"], c["nodes"], c["aabbs"], c["tris"], c["objids"], c["mats"], c["lights"])
    try:
        rgb, hi, ht = ds.render(_camera(c), spp=c["spp"], max_depth=c["depth"], aov=True)
    finally:
        ds.close()
    fb, ghi, ght = goldens(name, c)
    assert np.array_equal(hi, ghi), f"{int((hi != ghi).sum())} primary hits differ"
    assert np.array_equal(ht.view(np.uint32), ght.view(np.uint32))
    assert np.array_equal(rgb.view(np.uint32), fb.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_device_deep_tree_ray_counts_match_oracle(name):
    """rt_count_rays through the DEEP kernels (overflowing chains included) against the oracle's
    counters."""
    import raytracinginonesemester_amd as rt

    c = chain(name)
    m = c["meta"]
    ds = rt.DeviceScene(c["P"], c["nodes"], c["aabbs"], c["tris"], c["objids"], c["mats"], c["lights"])
    try:
        got = ds.count_rays(_camera(c), spp=c["spp"], max_depth=c["depth"])
    finally:
        ds.close()
    cam = orc.camera_from_basis(hexv(m["center"]), hexv(m["pixel00_loc"]), hexv(m["pixel_delta_u"]),
                                hexv(m["pixel_delta_v"]), c["W"], c["H"])
    _, st = orc.render_g(c["P"], cam, c["nodes"], c["aabbs"], c["tris"], c["objids"], c["mats"], c["lights"],
                         spp=c["spp"], max_depth=c["depth"], stats=True)
    assert [got["camera"], got["shadow"], got["bounce"]] == list(st["rays"])


@pytest.mark.gpu
def test_reference_signature_deep_tree():
    """The drop-in entry point (query.h:13-29) accepts the deep tree the reference accepts."""
    import raytracinginonesemester_amd as rt

    name = "chain600"
    c = chain(name)
    out = np.zeros(c["W"] * c["H"] * 3, np.float32)
    rt.render(c["P"], c["W"], c["H"], _camera(c), (0.0, 0.0, 0.0), c["depth"], c["spp"], c["nodes"], c["aabbs"],
              c["tris"], c["objids"], c["mats"], 1, c["lights"], 1, True, out)
    assert np.array_equal(out.view(np.uint32), goldens(name, c)[0].reshape(-1).view(np.uint32))
