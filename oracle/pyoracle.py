"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
parity checker / CPU baseline.  The product (raytracinginonesemester_amd) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
# RT_ORACLE_LIB: another build of the same source (tests/test_sanitize.py: the ASan/UBSan one)
LIB = Path(os.environ.get("RT_ORACLE_LIB", HERE / "liboracle.so"))
REF_DIR = HERE / "_ref"


class V3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Cam(C.Structure):
    _fields_ = [("center", V3), ("pixel00", V3), ("du", V3), ("dv", V3), ("width", C.c_int32),
                ("height", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64 * 3), ("pops", C.c_uint64 * 3), ("internal_entered", C.c_uint64 * 3),
                ("leaf_entered", C.c_uint64 * 3), ("hits", C.c_uint64 * 3), ("occluded", C.c_uint64),
                ("max_pops", C.c_uint64 * 3)]

    def as_dict(self) -> dict:
        d = {k: list(getattr(self, k)) for k in ("rays", "pops", "internal_entered", "leaf_entered", "hits",
                                                  "max_pops")}
        d["occluded"] = int(self.occluded)
        return d


_P = C.c_void_p
_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        L.orc_jitter.argtypes = [C.c_int, C.c_uint32, C.c_int, _P]
        L.orc_camera_init.argtypes = [_P, _P, _P, _P, C.c_double, C.c_double, C.c_int, C.c_int, C.c_int]
        L.orc_render_g.argtypes = [C.c_size_t, C.c_int, C.c_int, _P, V3, C.c_int, C.c_int, _P, _P, _P, _P, _P,
                                   C.c_int, _P, C.c_int, C.c_int, _P, C.c_int, C.c_int, C.c_int, C.c_int,
                                   _P, _P, _P, _P]
        L.orc_search_bvh.argtypes = [C.c_size_t, _P, _P, _P, _P, _P, _P]
        L.orc_render_hw1.argtypes = [_P, _P, _P, C.c_size_t, _P, V3, V3, C.c_int, _P, C.c_int, C.c_int, C.c_int,
                                     _P, _P, _P]
        L.orc_kat_hw1.argtypes = [_P, _P, _P, C.c_int, _P, _P]
        L.orc_intersect_g.argtypes = [_P, _P, _P, C.c_int, C.c_float, C.c_float, _P, _P]
        L.orc_ppm_quantize.argtypes = [_P, C.c_size_t, C.c_int, C.c_int, C.c_int, _P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


def jitter(spp: int, seed: int = 42, centered: bool = True) -> np.ndarray:
    out = np.zeros((spp, 2), np.float32)
    lib().orc_jitter(spp, seed, 1 if centered else 0, _p(out))
    return out


def camera(pos, look_at, up, focal_mm, sensor_mm, w, h, hw1=False) -> Cam:
    c = Cam()
    rc = lib().orc_camera_init(C.byref(c), _f3(pos), _f3(look_at), _f3(up), float(focal_mm), float(sensor_mm),
                               int(w), int(h), 1 if hw1 else 0)
    if rc != 0:
        raise ValueError("camera init failed")
    return c


def camera_from_basis(center, pixel00, du, dv, w, h) -> Cam:
    c = Cam()
    c.center, c.pixel00, c.du, c.dv = V3(*center), V3(*pixel00), V3(*du), V3(*dv)
    c.width, c.height = int(w), int(h)
    return c


def render_g(num_triangles, cam: Cam, nodes, aabbs, tris, objids, mats, lights, spp=1, max_depth=1,
             diffuse_bounce=True, miss=(0, 0, 0), jitter_tab=None, rebuild_jitter=False, rows=None,
             threads=0, aov=False, stats=False):
    """G/ render() CPU branch; returns rgb (H,W,3) [, hit_idx, hit_t (H,W,spp)] [, stats]."""
    W, H = cam.width, cam.height
    y0, y1 = (0, H) if rows is None else rows
    rgb = np.zeros((H, W, 3), np.float32)
    hi = np.full((H, W, spp), -2, np.int32) if aov else None
    ht = np.zeros((H, W, spp), np.float32) if aov else None
    nd = np.ascontiguousarray(nodes, np.uint32)
    ab = np.ascontiguousarray(aabbs, np.float32)
    tr = np.ascontiguousarray(tris, np.float32)
    ob = None if objids is None else np.ascontiguousarray(objids, np.int32)
    mt = None if mats is None else np.ascontiguousarray(mats, np.float32)
    lt = np.ascontiguousarray(lights)
    jt = None if jitter_tab is None else np.ascontiguousarray(jitter_tab, np.float32)
    st = Stats()
    rc = lib().orc_render_g(int(num_triangles), W, H, C.byref(cam), V3(*miss), int(max_depth), int(spp),
                            _p(nd), _p(ab), _p(tr), _p(ob), _p(mt), 0 if mt is None else mt.size // 13,
                            _p(lt), lt.shape[0], 1 if diffuse_bounce else 0, _p(jt), 1 if rebuild_jitter else 0,
                            int(y0), int(y1), int(threads), _p(rgb), _p(hi), _p(ht), C.byref(st))
    if rc != 0:
        raise RuntimeError(f"orc_render_g failed: {rc}")
    out = [rgb]
    if aov:
        out += [hi, ht]
    if stats:
        out.append(st.as_dict())
    return out[0] if len(out) == 1 else tuple(out)


def render_hw1(positions, normals, indices, cam: Cam, light_pos, light_color, spp=1, jitter_tab=None,
               rows=None, threads=0, aov=False):
    W, H = cam.width, cam.height
    y0, y1 = (0, H) if rows is None else rows
    rgb = np.zeros((H, W, 3), np.float32)
    hi = np.full((H, W, spp), -2, np.int32) if aov else None
    ht = np.zeros((H, W, spp), np.float32) if aov else None
    pos = np.ascontiguousarray(positions, np.float32)
    nrm = np.ascontiguousarray(normals, np.float32)
    idx = np.ascontiguousarray(indices, np.uint32)
    jt = None if jitter_tab is None else np.ascontiguousarray(jitter_tab, np.float32)
    rc = lib().orc_render_hw1(_p(pos), _p(nrm), _p(idx), idx.size // 3, C.byref(cam), V3(*light_pos),
                              V3(*light_color), int(spp), _p(jt), int(y0), int(y1), int(threads), _p(rgb),
                              _p(hi), _p(ht))
    if rc != 0:
        raise RuntimeError(f"orc_render_hw1 failed: {rc}")
    return (rgb, hi, ht) if aov else rgb


def kat_hw1(tri18, dirs, origin=(0, 0, 0)):
    t = np.ascontiguousarray(tri18, np.float32)
    d = np.ascontiguousarray(dirs, np.float32)
    n = d.size // 3
    hit = np.zeros(n, np.int32)
    tt = np.zeros(n, np.float32)
    lib().orc_kat_hw1(_p(t), _f3(origin), _p(d), n, _p(hit), _p(tt))
    return hit, tt


def intersect_g(tri18, dirs, origin=(0, 0, 0), tmin=0.0, tmax=3.4028234663852886e38):
    t = np.ascontiguousarray(tri18, np.float32)
    d = np.ascontiguousarray(dirs, np.float32)
    n = d.size // 3
    hit = np.zeros(n, np.int32)
    tt = np.zeros(n, np.float32)
    lib().orc_intersect_g(_p(t), _f3(origin), _p(d), n, float(tmin), float(tmax), _p(hit), _p(tt))
    return hit, tt


def ppm_quantize(rgb, maxval=255, clamp=True, gamma2=True) -> np.ndarray:
    a = np.ascontiguousarray(rgb, np.float32)
    out = np.zeros(a.size, np.uint16)
    lib().orc_ppm_quantize(_p(a), a.size, int(maxval), 1 if clamp else 0, 1 if gamma2 else 0, _p(out))
    return out.reshape(a.shape)


def bytes_per_ray(stats: dict, cls: int) -> float:
    """SURVEY.md §8(d) traffic model: 24*(pops + 2*internal) + 16*entered + 72*leaf, per ray."""
    r = stats["rays"][cls]
    if r == 0:
        return 0.0
    pops, it, lf = stats["pops"][cls], stats["internal_entered"][cls], stats["leaf_entered"][cls]
    return (24 * (pops + 2 * it) + 16 * (it + lf) + 72 * lf) / r
