"""The kernels decide most AABB tests with a conservative float pre-classification and fall back
to the reference's double slab test (G/include/bvh.h:81-129) only when the float estimate is
within its error bound of the boundary.  The answer must equal the reference's on every input:
fuzzed here on the host build of the same code, with adversarial near-boundary cases (rays
through box corners/edges/faces, tmax on the entry/exit parameter, degenerate boxes, tiny and
huge coordinates, axis-parallel directions)."""
from __future__ import annotations

import numpy as np

from raytracinginonesemester_amd import _lib


def _run(rays, boxes, tmm):
    n = rays.shape[0]
    rays = np.ascontiguousarray(rays, np.float32)
    boxes = np.ascontiguousarray(boxes, np.float32)
    tmm = np.ascontiguousarray(tmm, np.float32)
    fast = np.zeros(n, np.int32)
    exact = np.zeros(n, np.int32)
    cls = np.zeros(n, np.int32)
    _lib.check(_lib.lib().rt_box_test_host(rays.ctypes.data, boxes.ctypes.data, tmm.ctypes.data, n,
                                           fast.ctypes.data, exact.ctypes.data, cls.ctypes.data))
    return fast, exact, cls


def _boxes(rng, n, scale):
    c = rng.normal(size=(n, 3)) * scale
    h = np.abs(rng.normal(size=(n, 3))) * scale * rng.choice([1.0, 1e-3, 0.0], size=(n, 1), p=[0.8, 0.15, 0.05])
    return np.concatenate([c - h, c + h], axis=1).astype(np.float32)


def test_random_rays_and_boxes():
    rng = np.random.default_rng(1)
    n = 200000
    for scale in (1e-3, 1.0, 1e3):
        boxes = _boxes(rng, n, scale)
        o = (rng.normal(size=(n, 3)) * scale * 3).astype(np.float32)
        d = rng.normal(size=(n, 3)).astype(np.float32)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        par = rng.random((n, 3)) < 0.03
        d[par] = rng.choice([0.0, 5e-9, -5e-9, 2e-8], size=par.sum())
        rays = np.concatenate([o, d], axis=1)
        tmm = np.stack([np.full(n, 1e-4), rng.choice([3.4028235e38, scale, scale * 10], size=n)], axis=1)
        fast, exact, cls = _run(rays, boxes, tmm)
        assert np.array_equal(fast, exact)
        assert 0 < exact.sum() < len(exact)  # both outcomes occur


def test_adversarial_boundaries():
    """Rays aimed exactly at box corners, edge midpoints and face points, with tmax set to the
    reference's entry/exit parameters (and their float neighbours)."""
    rng = np.random.default_rng(2)
    n = 60000
    boxes = _boxes(rng, n, 1.0)
    mn, mx = boxes[:, :3], boxes[:, 3:]
    pick = rng.integers(0, 2, size=(n, 3))
    target = np.where(pick == 0, mn, mx)
    face = rng.random(n) < 0.5  # half the rays aim at a face point instead of a corner
    ax = rng.integers(0, 3, size=n)
    interior = mn + (mx - mn) * rng.random((n, 3))
    tgt = target.copy()
    tgt[face] = interior[face]
    tgt[face, ax[face]] = target[face, ax[face]]
    o = (tgt + rng.normal(size=(n, 3)) * 2).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    d = d.astype(np.float32)
    # tmax at the exact reference exit parameter along the aimed axis, and its neighbours
    with np.errstate(divide="ignore", invalid="ignore"):
        t_aim = ((tgt - o).astype(np.float64) * (1.0 / d.astype(np.float64))).max(axis=1).astype(np.float32)
    t_aim = np.where(np.isfinite(t_aim), t_aim, 1.0).astype(np.float32)
    for tmax in (t_aim, np.nextafter(t_aim, np.float32(np.inf)), np.nextafter(t_aim, np.float32(0)),
                 np.full(n, 3.4028235e38, np.float32)):
        tmm = np.stack([np.full(n, 1e-4, np.float32), tmax], axis=1)
        fast, exact, cls = _run(np.concatenate([o, d], axis=1), boxes, tmm)
        assert np.array_equal(fast, exact)
        assert (cls == 2).any()  # the fallback is exercised


def test_extreme_magnitudes():
    rng = np.random.default_rng(3)
    n = 40000
    for scale in (1e-30, 1e-20, 1e20, 1e35):
        boxes = _boxes(rng, n, scale)
        o = (rng.normal(size=(n, 3)) * scale * 2).astype(np.float32)
        d = rng.normal(size=(n, 3)).astype(np.float32)
        tmm = np.stack([np.full(n, 1e-4), np.full(n, 3.4028235e38)], axis=1)
        fast, exact, _ = _run(np.concatenate([o, d], axis=1), boxes, tmm)
        assert np.array_equal(fast, exact)


def test_near_parallel_and_overflow_scales():
    """Directions with one tiny (but not parallel) component, and coordinates up to the top of
    the float range, where the float estimates overflow: the classification must stay sound."""
    rng = np.random.default_rng(4)
    n = 60000
    for scale in (1.0, 1e30, 1e37, 1.5e38):
        boxes = _boxes(rng, n, scale)
        o = (rng.normal(size=(n, 3)) * scale * 1.5).astype(np.float32)
        d = rng.normal(size=(n, 3)).astype(np.float32)
        ax = rng.integers(0, 3, size=n)
        d[np.arange(n), ax] = rng.choice([1.01e-8, -1.01e-8, 1e-7, 3e-6, -1e-5], size=n)
        with np.errstate(over="ignore", invalid="ignore"):
            boxes = np.where(np.isfinite(boxes), boxes, 0).astype(np.float32)
            o = np.where(np.isfinite(o), o, 0).astype(np.float32)
        tmm = np.stack([np.full(n, 1e-4), rng.choice([3.4028235e38, 1.0, 1e30], size=n)], axis=1)
        fast, exact, _ = _run(np.concatenate([o, d], axis=1), boxes, tmm)
        assert np.array_equal(fast, exact), scale
