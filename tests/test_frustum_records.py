"""The camera rays' frustum records (rt_scene_create's build_frustum_records)
checked on the host through rt_debug_frustum_records: no GPU.

* the records are the expansion a Python restatement of the rule makes, boxes and refs bit for
  bit: by default (RT_TUNE_RECORD_GREEDY = 1) a record's entries grow from its node's two
  children by replacing, in place, the internal entry of largest surface area by its children
  until A entries; with 0, the descendants D levels down; in both, SearchBVH's push order,
  leaves stand for themselves and children naming no valid triangle are skipped;
* a DFS over the records that passes every box (push the entries in order, hold the last, pop)
  yields the leaves in exactly the order SearchBVH's own DFS does when every box passes
  (G/include/query.h:224-311: push left, push right, pop) -- the order the traversal's
  exactness rests on;
* the stack bound the builder reports covers that DFS and fits the stack it was asked for (the
  traversal's 128 entries; smaller caps too), and the arity is the largest one that fits.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import host_scene

from raytracinginonesemester_amd import _lib

NO_REF = 0xFFFFFFFF
LEAF_BIT = 0x80000000


def build(P, nodes, aabbs, max_log2, cap=64):
    L = _lib.lib()
    nodes = np.ascontiguousarray(nodes, np.uint32)
    aabbs = np.ascontiguousarray(aabbs, np.float32)
    info = (C.c_int64 * 3)()
    assert L.rt_debug_frustum_records(P, nodes.ctypes.data, aabbs.ctypes.data, max_log2, cap, info, None, 0) == 0
    log2, bound, nrec = (int(v) for v in info)
    A = 1 << log2
    rec = np.zeros(max(nrec, 1) * 8 * A, np.float32)
    assert L.rt_debug_frustum_records(P, nodes.ctypes.data, aabbs.ctypes.data, max_log2, cap, info,
                                      rec.ctypes.data, rec.size) == 0
    return log2, bound, nrec, rec


class Model:
    """The rule restated over the reference arrays (rt_bvh_node: parent, left, right, object)."""

    def __init__(self, P, nodes, aabbs=None, greedy=2):
        self.P, self.nodes = P, np.asarray(nodes, np.int64)
        self.aabbs = None if aabbs is None else np.asarray(aabbs, np.float32)
        self.greedy = greedy  # 0 fixed depth, 1 area, 2 area x sqrt(leaves below)
        self._leaves = {}
        NN = 2 * P - 1
        self.cid = np.full(NN, NO_REF, np.int64)
        ni = nl = 0
        for n in range(NN):
            if self.nodes[n, 3] == NO_REF:
                self.cid[n] = ni
                ni += 1
            elif self.nodes[n, 3] < P:
                self.cid[n] = LEAF_BIT | nl
                nl += 1

    def ref(self, n):
        return NO_REF if n == NO_REF else int(self.cid[n])

    def is_leaf(self, n):
        r = self.ref(n)
        return r != NO_REF and (r & LEAF_BIT) != 0

    def expand(self, n, d, out):
        if self.ref(n) == NO_REF:
            return
        if d == 0 or self.is_leaf(n):
            out.append(n)
            return
        self.expand(int(self.nodes[n, 1]), d - 1, out)
        self.expand(int(self.nodes[n, 2]), d - 1, out)

    def leaves(self, n):
        if n in self._leaves:
            return self._leaves[n]
        out, st = 0, [n]
        while st:
            v = st.pop()
            if self.ref(v) == NO_REF:
                continue
            if self.is_leaf(v):
                out += 1
                continue
            st += [c for c in (int(self.nodes[v, 1]), int(self.nodes[v, 2])) if c != NO_REF]
        self._leaves[n] = out
        return out

    def area(self, n):
        import math

        b = self.aabbs[n].astype(np.float64)
        dx, dy, dz = (max(0.0, float(b[3 + i]) - float(b[i])) for i in range(3))
        a = dx * dy + dy * dz + dz * dx
        if self.greedy == 2:
            a *= math.sqrt(float(self.leaves(n)))
        return a if np.isfinite(a) else 1e300

    def greedy_entries(self, node, A):
        kids = lambda n: [c for c in (int(self.nodes[n, 1]), int(self.nodes[n, 2])) if self.ref(c) != NO_REF]
        fr = kids(node)
        while len(fr) < A:
            best, ba = -1, -1.0
            for i, n in enumerate(fr):
                if self.is_leaf(n):
                    continue
                a = self.area(n)
                if a > ba:
                    best, ba = i, a
            if best < 0:
                break
            fr[best:best + 1] = kids(fr[best])
        return fr

    def records(self, D):
        recs, fid, ents = [0], {0: 0}, []
        r = 0
        while r < len(recs):
            e = []
            if self.greedy:
                e = self.greedy_entries(recs[r], 1 << D)
            else:
                self.expand(int(self.nodes[recs[r], 1]), D - 1, e)
                self.expand(int(self.nodes[recs[r], 2]), D - 1, e)
            for n in e:
                if not self.is_leaf(n) and n not in fid:
                    fid[n] = len(recs)
                    recs.append(n)
            ents.append(e)
            r += 1
        return recs, fid, ents

    def entry_ref(self, n, fid):
        return self.ref(n) if self.is_leaf(n) else fid[n]

    def reference_leaf_order(self):
        """SearchBVH with every box passing: the valid leaves' slots in the order it tests them."""
        out, st = [], [0]
        while st:
            n = st.pop()
            r = self.ref(n)
            if self.nodes[n, 3] != NO_REF:  # a leaf (one naming no valid triangle is skipped)
                if r != NO_REF:
                    out.append(r & ~LEAF_BIT)
                continue
            for c in (int(self.nodes[n, 1]), int(self.nodes[n, 2])):
                if c != NO_REF:
                    st.append(c)
        return out


def _greedy():
    import raytracinginonesemester_amd as rt

    v = rt.get_tuning("record_greedy")
    return 2 if v is None else int(v + 0.5)


@pytest.fixture(params=[2, 1, 0], ids=["greedy_leaf_weight", "greedy_area", "fixed_depth"], autouse=True)
def record_rule(request):
    """Every test here runs under both record rules (RT_TUNE_RECORD_GREEDY)."""
    import raytracinginonesemester_amd as rt

    rt.set_tuning("record_greedy", request.param)
    yield request.param
    rt.reset_tuning()


def records_leaf_order(log2, rec):
    """The frustum traversal's DFS over the records when every entry passes."""
    A = 1 << log2
    R = rec.reshape(-1, 8 * A)
    refs = R[:, 6 * A:7 * A].view(np.uint32)
    out, st, ref, max_sp = [], [], 0, 0
    while True:
        nxt = None
        if ref & LEAF_BIT:
            out.append(ref & ~LEAF_BIT)
        else:
            es = [int(x) for x in refs[ref] if x != NO_REF]
            if es:
                st += es[:-1]
                nxt = es[-1]
                max_sp = max(max_sp, len(st))
        if nxt is not None:
            ref = nxt
            continue
        if not st:
            break
        ref = st.pop()
    return out, max_sp


def check(P, nodes, aabbs, max_log2=4, cap=64):
    m = Model(P, nodes, aabbs, greedy=_greedy())
    log2, bound, nrec, rec = build(P, nodes, aabbs, max_log2, cap)
    if log2 == 2:
        return m, log2, bound
    A = 1 << log2
    recs, fid, ents = m.records(log2)
    assert nrec == len(recs)
    want = np.zeros((nrec, 8 * A), np.float32)
    for r, e in enumerate(ents):
        assert len(e) <= A
        for i, n in enumerate(e):
            b = np.asarray(aabbs[n], np.float32)
            want[r, 6 * i:6 * i + 6] = [b[0], b[3], b[1], b[4], b[2], b[5]]
        refs = want[r, 6 * A:7 * A].view(np.uint32)
        refs[:] = NO_REF
        for i, n in enumerate(e):
            refs[i] = m.entry_ref(n, fid)
    assert np.array_equal(rec.reshape(nrec, 8 * A).view(np.uint32), want.view(np.uint32))
    order, max_sp = records_leaf_order(log2, rec)
    assert order == m.reference_leaf_order()
    assert max_sp <= bound <= cap
    return m, log2, bound


@pytest.mark.parametrize("cap,max_log2", [(128, 5), (64, 4)])
@pytest.mark.parametrize("scene", ["frog.json", "cornell.json", "sphere_single.json", "sphere.json"])
def test_shipped_scene_records(scene, cap, max_log2):
    """(128, 5): what rt_scene_create builds (32-ary records for frog, bound 91)."""
    hs = host_scene(scene)
    _, log2, bound = check(hs.num_triangles, hs.nodes, hs.aabbs, max_log2, cap)
    assert log2 == max_log2, (log2, bound)


def test_arity_cap():
    hs = host_scene("frog.json")
    for cap, want in ((3, 3), (2, 2)):
        assert build(hs.num_triangles, hs.nodes, hs.aabbs, cap)[0] == want
    check(hs.num_triangles, hs.nodes, hs.aabbs, 3)
    # a stack too small for any wide arity: none (the traversal takes the 4-ary records)
    assert build(hs.num_triangles, hs.nodes, hs.aabbs, 4, cap=8)[0] == 2


def random_tree(rng, P, invalid_frac):
    """A random binary BVH over P leaves in the reference's array form (2P-1 nodes, root 0),
    leaves naming no valid triangle (object >= P) at random, boxes the unions of the children's."""
    NN = 2 * P - 1
    nodes = np.zeros((NN, 4), np.uint32)
    nodes[0, 0] = NO_REF
    aabbs = np.zeros((NN, 6), np.float32)
    nxt = [1]
    leaves = []

    def grow(n, k):  # subtree of node n with k leaves
        if k == 1:
            nodes[n, 1] = nodes[n, 2] = NO_REF
            leaves.append(n)
            return
        a = int(rng.integers(1, k))
        l, r = nxt[0], nxt[0] + 1
        nxt[0] += 2
        nodes[n, 1], nodes[n, 2], nodes[n, 3] = l, r, NO_REF
        nodes[l, 0] = nodes[r, 0] = n
        grow(l, a)
        grow(r, k - a)

    import sys
    sys.setrecursionlimit(10000)
    grow(0, P)
    objs = rng.permutation(P).astype(np.int64)
    for i, n in enumerate(leaves):
        nodes[n, 3] = objs[i] if rng.random() >= invalid_frac else P + int(rng.integers(0, 5))
        c = rng.normal(size=3).astype(np.float32)
        aabbs[n, :3], aabbs[n, 3:] = c - 0.01, c + 0.01
    for n in range(NN - 1, -1, -1):
        if nodes[n, 3] == NO_REF:
            l, r = nodes[n, 1], nodes[n, 2]
            aabbs[n, :3] = np.minimum(aabbs[l, :3], aabbs[r, :3])
            aabbs[n, 3:] = np.maximum(aabbs[l, 3:], aabbs[r, 3:])
    return nodes, aabbs


@pytest.mark.parametrize("seed", range(6))
def test_random_trees(seed):
    rng = np.random.default_rng(seed)
    P = int(rng.integers(2, 400))
    nodes, aabbs = random_tree(rng, P, invalid_frac=0.15 if seed % 2 else 0.0)
    for cap in (64, 128, 24):
        check(P, nodes, aabbs, 5, cap)
        check(P, nodes, aabbs, 4, cap)
        check(P, nodes, aabbs, 3, cap)


def first_leaf_depth(log2, rec):
    """Stack depth of the records' DFS when it first reaches a leaf, every entry passing: the
    depth a camera ray reaches when every box it meets before its first triangle test passes
    (the spine scenes' centre rays)."""
    A = 1 << log2
    refs = rec.reshape(-1, 8 * A)[:, 6 * A:7 * A].view(np.uint32)
    st, ref = [], 0
    while not ref & LEAF_BIT:
        es = [int(x) for x in refs[ref] if x != NO_REF]
        st += es[:-1]
        ref = es[-1]
    return len(st)


@pytest.mark.parametrize("L,want_log2", [(15, 5), (30, 4), (35, 3)])
def test_spine_trees_fall_back_to_narrower_records(L, want_log2, record_rule):
    """tests/spine_bvh.py trees, built for the fixed-depth rule: the 32-ary records' DFS bound
    grows ~31 per five spine levels.  L = 15: 32-ary, bound in (64, 128] (the traversal's second
    stack VGPR); L = 30: the 32-ary bound exceeds 128 and the builder falls back to 16-ary (bound
    in (64, 128]); L = 35: to 8-ary.  The records are the rule's, their leaf order SearchBVH's,
    and the centre rays of the scene really reach more than 64 stack entries before their first
    leaf.  (The greedy rule spends the records' entries on the spine's large boxes and keeps the
    stack shallow here: its records are checked against the rule only.)"""
    import spine_bvh

    a = spine_bvh.as_arrays(spine_bvh.spine_scene(L))
    P, nodes, aabbs = a["P"], a["nodes"], a["aabbs"]
    if record_rule >= 1:
        _, log2, bound = check(P, nodes, aabbs, 5, 128)
        assert log2 == 5 and bound <= 128
        return
    _, log2, bound = check(P, nodes, aabbs, 5, 128)
    assert log2 == want_log2 and 64 < bound <= 128
    if want_log2 < 5:  # the wider arities do not fit
        assert build(P, nodes, aabbs, want_log2 + 1, 10**6)[1] > 128
    lg, _, _, rec = build(P, nodes, aabbs, 5, 128)
    assert first_leaf_depth(lg, rec) > 64
