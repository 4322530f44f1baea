"""Synthetic 'caterpillar' BVH scenes for the deep-tree path (TEST DATA GENERATOR).

A spine of internal nodes 0..P-2: node i has the leaf of spine level i on the left and node
i+1 on the right (the last node two leaves).  The leaf of level k holds a triangle in the
plane z = -0.01 k, all of them covering the image centre, so SearchBVH
(G/include/query.h:224-311) pushes a leaf and the next spine node at every level: the DFS
stack grows by one per level.  P = 300 needs ~300 entries (more than the 64-entry wave stack,
within the reference's 512); P = 600 overflows 512, so the reference drops the spine below
level ~511 and completes by its brute-force pass over every triangle in index order
(query.h:298-308).  The triangle of level 3 duplicates level 0's (same plane, same vertices)
with a larger index: the DFS keeps level 0's (visited last, t <= bestT), the brute-force pass
the larger index — so the overflow case's answer differs from a plain DFS.

Arrays are the reference POD layouts (BVHNode, AABB, Triangle, Material, Light), built in
float32 deterministically; gen_golden.py feeds them to the reference (oracle/_ref/ref_g
arrays) and tests/test_gpu_deep.py to the GPU.
"""
from __future__ import annotations

import numpy as np

NODE = np.dtype([("parent", "<u4"), ("left", "<u4"), ("right", "<u4"), ("object", "<u4")])
MAT = np.dtype([("albedo", "<f4", 3), ("kd", "<f4"), ("spec", "<f4", 3), ("ks", "<f4"),
                ("shininess", "<f4"), ("kr", "<f4"), ("emission", "<f4", 3)])
LIGHT = np.dtype([("position", "<f4", 3), ("color", "<f4", 3), ("intensity", "<i4")])
NONE = 0xFFFFFFFF

# camera: pos, look_at, up, focal_mm, sensor_mm (G/include/camera.h:13-28)
CAMERA = ((0.0, 0.0, 5.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 30.0, 24.0)
FIXTURES = {"chain300": (300, 48, 32, 4, 1), "chain600": (600, 48, 32, 4, 1), "chain600_d2": (600, 32, 24, 4, 2)}


def chain_scene(P: int) -> dict:
    """nodes (2P-1), aabbs (2P-1, 6), tris (P, 18), triobj (P), mats (1), lights (1)."""
    assert P >= 8
    perm = (np.arange(P, dtype=np.int64) * 7919 + 3) % P  # leaf level -> triangle index
    # level 3 repeats level 0's triangle with a larger index
    i0, i3 = int(perm[0]), int(perm[3])
    if i3 < i0:
        perm[0], perm[3] = i3, i0
    z = (-0.01 * np.arange(P)).astype(np.float32)
    z[3] = z[0]
    tris = np.zeros((P, 18), np.float32)
    for k in range(P):
        t = perm[k]
        tris[t, 0:3] = (-2.0, -2.0, z[k])
        tris[t, 3:6] = (2.0, -2.0, z[k])
        tris[t, 6:9] = (0.0, 2.0, z[k])
        tris[t, 9:18] = (0.0, 0.0, 1.0) * 3
    nn = 2 * P - 1
    nodes = np.zeros(nn, NODE)
    aabbs = np.zeros((nn, 6), np.float32)
    leaf = lambda k: P - 1 + k  # noqa: E731  leaf node of spine level k
    for k in range(P):
        n = leaf(k)
        nodes[n] = (0, NONE, NONE, perm[k])
        aabbs[n] = (-2.0, -2.0, z[k], 2.0, 2.0, z[k])
    for i in range(P - 2, -1, -1):
        right = leaf(P - 1) if i == P - 2 else i + 1
        nodes[i] = (0, leaf(i), right, NONE)
        nodes[leaf(i)]["parent"] = i
        nodes[right]["parent"] = i
        lo = np.minimum(aabbs[leaf(i), :3], aabbs[right, :3])
        hi = np.maximum(aabbs[leaf(i), 3:], aabbs[right, 3:])
        aabbs[i] = np.concatenate([lo, hi])
    nodes[0]["parent"] = NONE
    mats = np.zeros(1, MAT)
    mats[0] = ((0.8, 0.3, 0.2), 1.0, (0.04, 0.04, 0.04), 0.5, 32.0, 0.0, (0.0, 0.0, 0.0))
    lights = np.zeros(1, LIGHT)
    lights[0] = ((3.0, 3.0, 5.0), (1.0, 1.0, 1.0), 5)
    return {"nodes": nodes, "aabbs": aabbs, "tris": tris, "triobj": np.zeros(P, np.int32), "mats": mats,
            "lights": lights, "perm": perm}


def write_arrays(d: dict, out_dir) -> None:
    """The reference-layout files oracle/_ref/ref_g `arrays` reads."""
    from pathlib import Path

    o = Path(out_dir)
    d["nodes"].tofile(o / "nodes.bin")
    d["aabbs"].tofile(o / "aabbs.bin")
    d["tris"].tofile(o / "tris.bin")
    d["triobj"].tofile(o / "triobj.bin")
    d["mats"].tofile(o / "mats.bin")
    d["lights"].tofile(o / "lights.bin")
    pos, look, up, f, s = CAMERA
    vals = [*pos, *look, *up, f, s]
    (o / "camera.txt").write_text(" ".join(float(v).hex() for v in vals) + "\n")
