"""Malformed-input fuzz of the host-side parsers and builders (CPU, no GPU): the scene JSON
reader (restating G/include/scene.h:57-217), the OBJ loaders (G/include/MeshOBJ.h:260-427,
HW1/src/MeshOBJ.cpp:143-281), the P6 reader (HW1/ppm_p6_lib/src/ppm_p6.cpp:303-372), the CPU
LBVH (G/include/bvh.cu:209-317) and the frustum-record builder over caller BVH arrays.

Every input is either accepted or refused with an RTError: no crash, no hang.  Seeded
mutations of valid files (truncation, byte flips, token splices: huge and non-finite numbers,
indices past either end, deep nesting, huge counts).  tests/test_sanitize.py runs this file
against the AddressSanitizer/UBSan build of the host code, where an out-of-bounds access or
undefined behaviour fails the run even when it does not crash.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import REPO

import raytracinginonesemester_amd as rt
from raytracinginonesemester_amd import _lib

N_CASES = 120

TOKENS = [b"1e400", b"-1e400", b"nan", b"inf", b"-0", b"99999999999999999999", b"-2147483649", b"0x7f",
          b"\x00", b"\xff\xfe", b"[", b"]", b"{", b"}", b",", b":", b"\"", b"\\", b"\\u0000", b"/", b"//",
          b"-", b"+", b".", b"e", b"E5", b"f", b"v", b"vn", b"vt", b"o", b"g", b"#", b"\n", b"\r\n", b"\t",
          b" ", b"-1", b"-999999", b"0", b"4294967295", b"1/2/3", b"1//3", b"//", b"P6", b"255", b"65535",
          b"65536", b"0 0", b"true", b"null", b"\"path\"", b"\"scene\"", b"\"camera\""]


def _mutations(data: bytes, seed: int, n: int = N_CASES):
    rng = np.random.default_rng(seed)
    for k in range(n):
        b = bytearray(data)
        kind = k % 4
        if kind == 0 and len(b) > 1:  # truncation
            del b[int(rng.integers(0, len(b))):]
        elif kind == 1 and b:  # byte flips
            for _ in range(int(rng.integers(1, 8))):
                i = int(rng.integers(0, len(b)))
                b[i] = int(rng.integers(0, 256))
        elif kind == 2:  # token splices
            for _ in range(int(rng.integers(1, 6))):
                i = int(rng.integers(0, len(b) + 1))
                b[i:i] = TOKENS[int(rng.integers(0, len(TOKENS)))]
        else:  # token replacement of a whole run of bytes
            if b:
                i = int(rng.integers(0, len(b)))
                j = min(len(b), i + int(rng.integers(1, 16)))
                b[i:j] = TOKENS[int(rng.integers(0, len(TOKENS)))]
        yield bytes(b)


def _try(fn):
    try:
        fn()
    except rt.RTError:
        pass


SMALL_OBJ = (b"o a\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\nf 1/1/1 2/1/1 3/1/1\nf -4 -3 -2 -1\n"
             b"o b\nv 0 0 1\nv 1 0 1\nv 0 1 1\nf 5 6 7\n")


def test_obj_loaders_survive_malformed_files(tmp_path):
    p = tmp_path / "m.obj"
    for k, data in enumerate(_mutations(SMALL_OBJ, 1)):
        p.write_bytes(data)
        _try(lambda: rt.HostScene.load_objs([p]))
        _try(lambda: rt.MeshHW1(p))


def test_obj_loaders_refuse_indices_past_either_end(tmp_path):
    p = tmp_path / "i.obj"
    for face in (b"f 1 2 4", b"f 0 1 2", b"f -4 1 2", b"f 1 2 4294967296", b"f 1 2 -4294967296",
                 b"f 1 2 99999999999999999999", b"f 1", b"f 1 2", b"f 1/9 2/9 3/9", b"f 1//9 2//9 3//9"):
        p.write_bytes(b"v 0 0 0\nv 1 0 0\nv 0 1 0\n" + face + b"\n")
        _try(lambda: rt.HostScene.load_objs([p]))
        _try(lambda: rt.MeshHW1(p))


def test_obj_loader_huge_counts(tmp_path):
    p = tmp_path / "h.obj"
    # a polygon with many vertices (fan triangulation) and many objects
    n = 4000
    verts = b"".join(b"v %d %d 0\n" % (i % 97, i // 97) for i in range(n))
    p.write_bytes(verts + b"f " + b" ".join(b"%d" % (i + 1) for i in range(n)) + b"\n" +
                  b"".join(b"o x%d\n" % i for i in range(2000)))
    _try(lambda: rt.HostScene.load_objs([p]))
    _try(lambda: rt.MeshHW1(p))


def test_scene_json_survives_malformed_files(tmp_path):
    (tmp_path / "m.obj").write_bytes(SMALL_OBJ)
    base = (REPO / "assets" / "scenes" / "frog.json").read_bytes().replace(b"./assets/meshes/frog.obj", b"m.obj")
    p = tmp_path / "s.json"
    for data in _mutations(base, 2):
        p.write_bytes(data)
        _try(lambda: rt.HostScene.load_json(p, tmp_path))


def test_scene_json_deep_nesting_and_odd_values(tmp_path):
    (tmp_path / "m.obj").write_bytes(SMALL_OBJ)
    p = tmp_path / "d.json"
    cases = [b"[" * 200000 + b"]" * 200000, b"{\"a\":" * 100000 + b"1" + b"}" * 100000, b"[" * 200000,
             b"{\"scene\": [{\"path\": \"m.obj\", \"material\": {\"albedo\": [1e400, -1e400, 0]}}]}",
             b"{\"scene\": [{\"path\": \"m.obj\"}], \"camera\": {\"pixel_width\": -5, \"pixel_height\": 99999999999}}",
             b"{\"scene\": [{\"path\": \"m.obj\"}], \"camera\": {\"position\": [1, 2]}}",
             b"{\"scene\": [{\"path\": \"m.obj\", \"transform\": {\"scale\": [0, 0, 0]}}]}",
             b"{\"scene\": [{\"path\": \"m.obj\"}], \"lights\": [" + b"{}," * 5000 + b"{}]}",
             b"{\"scene\": [{\"path\": \"\\u0000\"}]}", b"{\"scene\": [{\"path\": \"m.obj\\", b"\"", b"", b"\xef\xbb\xbf{}"]
    for data in cases:
        p.write_bytes(data)
        _try(lambda: rt.HostScene.load_json(p, tmp_path))


def test_p6_reader_survives_malformed_files(tmp_path):
    good = rt.encode_p6(np.linspace(0, 1, 5 * 3 * 3, dtype=np.float32).reshape(3, 5, 3))
    p = tmp_path / "x.ppm"
    for data in list(_mutations(good, 3)) + [b"P6\n99999 99999\n255\n", b"P6\n-1 3\n255\n", b"P6\n5 3\n0\n",
                                             b"P6\n5 3\n65535\n\x00", b"P6 #c\n5 3 255\n", b"P6\n2147483647 2\n255\n",
                                             b"P3\n1 1\n255\n0 0 0\n", b"P6", b""]:
        p.write_bytes(data)
        _try(lambda: rt.read_p6(p))


def test_bvh_builder_refuses_bad_indices():
    pos = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 1]], np.float32)
    for idx in ([[0, 1, 4]], [[0, 1, -1]], [[0, 1, 2], [1, 2, 3], [3, 3, 3]], np.zeros((0, 3))):
        _try(lambda: rt.build_bvh(pos, np.asarray(idx, np.int64).astype(np.uint32)))
    with np.errstate(invalid="ignore"):
        _try(lambda: rt.build_bvh(np.full((3, 3), np.nan, np.float32), np.array([[0, 1, 2]], np.uint32)))


def test_frustum_record_builder_refuses_malformed_trees():
    """rt_debug_frustum_records takes caller BVH arrays (as rt_scene_create does): child indices
    past the array, cycles and shared children are refused, not followed."""
    hs = rt.HostScene.load_objs([REPO / "assets" / "meshes" / "sphere.obj"])
    nodes = np.array(hs.nodes, np.uint32)
    aabbs = np.array(hs.aabbs, np.float32)
    P = hs.num_triangles
    rng = np.random.default_rng(5)
    internal = np.nonzero(nodes[:, 3] == 0xFFFFFFFF)[0]
    info = (C.c_int64 * 3)()
    refused = 0
    for k in range(60):
        bad = nodes.copy()
        n = int(rng.choice(internal))
        col = 1 + k % 2
        bad[n, col] = [len(nodes), len(nodes) + 7, 0, n, 0xFFFFFFFE, int(rng.choice(internal))][k % 6]
        rc = _lib.lib().rt_debug_frustum_records(P, bad.ctypes.data, aabbs.ctypes.data, 5, 128, info, None, 0)
        refused += rc != 0
    assert refused > 0
