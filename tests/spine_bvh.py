"""Synthetic 'spine of blocks' BVH scenes for the frustum traversal's stack (TEST DATA GENERATOR).

A spine of internal nodes s_0 .. s_{L-1}: s_j has a complete binary subtree of height 4 (16
leaves) on the left and s_{j+1} on the right (s_{L-1}: a block on both sides).  A 32-ary
frustum record of s_j then holds the 16 leaves of its left block, the next spine nodes' blocks
cut at decreasing depth (8 + 4 + 2 + 1 entries) and, last, s_{j+5}: the entry the traversal
holds while the 31 before it wait on the stack.  So the records' DFS stack bound grows by ~31
per five spine levels (16-ary records: ~15 per four), and every leaf triangle covers the image
centre at its own depth, so the camera rays there pass every box until they reach the spine's
end: the traversal really goes that deep.

* ``spine_scene(15)``: 32-ary records with a bound between 64 and 128 (the traversal's second
  stack VGPR is used);
* ``spine_scene(30)``: the 32-ary bound exceeds the 128-entry stack, so rt_scene_create falls
  back to 16-ary records (bound <= 128, > 64).

Arrays are the reference POD layouts (tests/golden/chain_bvh.py dtypes), boxes the unions of
the children's, as an LBVH refit makes them (every internal box contains its children's:
the wide records' precondition).
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
from chain_bvh import LIGHT, MAT, NODE, NONE  # noqa: E402

CAMERA = ((0.0, 0.0, 5.0), (0.0, 0.0, 0.0), (0.0, 1.0, 0.0), 30.0, 24.0)
BLOCK_H = 4  # height of each spine level's left block (16 leaves)


def spine_scene(L: int, seed: int = 5) -> dict:
    """nodes (2P-1), aabbs (2P-1, 6), tris (P, 18), triobj (P), mats (1), lights (1)."""
    rng = np.random.default_rng(seed)
    per = 1 << BLOCK_H
    P = per * L + per  # the last spine node has a block on both sides
    NN = 2 * P - 1
    nodes = np.zeros(NN, NODE)
    aabbs = np.zeros((NN, 6), np.float32)
    tris = np.zeros((P, 18), np.float32)
    # leaf triangles: around the image centre, each at its own depth (z in [-1, 0)), random
    # sizes and offsets so that rays off the centre miss some of them
    perm = rng.permutation(P)
    zs = -rng.permutation(P).astype(np.float32) / np.float32(P)
    nxt = [0]  # next free internal node (internal nodes first, leaves at [P-1, 2P-1))
    leaf_next = [P - 1]
    leaves = []

    def new_internal():
        n = nxt[0]
        nxt[0] += 1
        return n

    def new_leaf():
        n = leaf_next[0]
        leaf_next[0] += 1
        k = len(leaves)
        t = int(perm[k])
        c = rng.uniform(-0.3, 0.3, size=2)
        s = rng.uniform(0.8, 2.5)
        z = zs[k]
        v = np.array([[c[0] - s, c[1] - s, z], [c[0] + s, c[1] - s, z], [c[0], c[1] + s, z]], np.float32)
        tris[t, 0:9] = v.reshape(-1)
        tris[t, 9:18] = (0.0, 0.0, 1.0) * 3
        nodes[n] = (0, NONE, NONE, t)
        aabbs[n, :3], aabbs[n, 3:] = v.min(axis=0), v.max(axis=0)
        leaves.append(n)
        return n

    def link(n, l, r):
        nodes[n]["left"], nodes[n]["right"], nodes[n]["object"] = l, r, NONE
        nodes[l]["parent"] = n
        nodes[r]["parent"] = n
        aabbs[n, :3] = np.minimum(aabbs[l, :3], aabbs[r, :3])
        aabbs[n, 3:] = np.maximum(aabbs[l, 3:], aabbs[r, 3:])

    def block(h, n=None):
        if h == 0:
            return new_leaf()
        n = new_internal() if n is None else n
        l = block(h - 1)
        r = block(h - 1)
        link(n, l, r)
        return n

    spine = [new_internal() for _ in range(L)]  # s_0 = node 0, the root
    for j in range(L - 1, -1, -1):
        left = block(BLOCK_H)
        right = spine[j + 1] if j + 1 < L else block(BLOCK_H)
        link(spine[j], left, right)
    assert nxt[0] == P - 1 and leaf_next[0] == NN
    nodes[0]["parent"] = NONE
    mats = np.zeros(1, MAT)
    mats[0] = ((0.7, 0.4, 0.3), 1.0, (0.04, 0.04, 0.04), 0.5, 32.0, 0.0, (0.0, 0.0, 0.0))
    lights = np.zeros(1, LIGHT)
    lights[0] = ((2.0, 1.0, 4.0), (1.0, 1.0, 1.0), 5)
    return {"P": P, "nodes": nodes, "aabbs": aabbs, "tris": tris, "triobj": np.zeros(P, np.int32), "mats": mats,
            "lights": lights}


def as_arrays(d: dict) -> dict:
    """The views the DeviceScene constructor and the oracle take."""
    return {"P": d["P"], "nodes": d["nodes"].view(np.uint32).reshape(-1, 4), "aabbs": d["aabbs"],
            "tris": d["tris"], "objids": d["triobj"], "mats": d["mats"].view(np.float32).reshape(-1, 13),
            "lights": d["lights"]}
