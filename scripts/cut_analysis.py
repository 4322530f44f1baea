"""CPU analysis for the tile cut: how many c3 work items
(a wave's 2x2-pixel quarter of a 4x4 tile, 64 samples) survive the exact cut test at K cut
boxes, per tile and per quarter, against the quarters that really hit the frog (the oracle's
primary-hit AOV of the full frame).  Double-precision restatement of tile_dirs/tile_misses_box
(rt_device.hip), no float slack: an estimate of what the device's float form keeps.

    python scripts/cut_analysis.py [--ks 64,128,256,1024] [--size 1920x1080] [--spp 16]
"""
from __future__ import annotations

import argparse
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import raytracinginonesemester_amd as rt  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

NO_REF = 0xFFFFFFFF


def greedy_cut(nodes, aabbs, k):
    """rt_scene_create's cut rule: from the root, replace the internal node of largest half
    surface area by its children until k nodes."""
    leaf = nodes[:, 3] != NO_REF

    def area(n):
        b = aabbs[n].astype(np.float64)
        d = b[3:] - b[:3]
        return d[0] * d[1] + d[1] * d[2] + d[2] * d[0]

    import heapq
    heap = [(-area(0), 0)]
    done = []
    while heap and len(heap) + len(done) < k:
        a, n = heapq.heappop(heap)
        if leaf[n]:
            done.append(n)
            continue
        for c in (int(nodes[n, 1]), int(nodes[n, 2])):
            if c != NO_REF:
                if leaf[c]:
                    done.append(c)
                else:
                    heapq.heappush(heap, (-area(c), c))
    return np.array(done + [n for _, n in heap], np.int64)


def tile_bounds(basis, x0, x1, y0, y1):
    """tile_dirs (double form) for arrays of tiles: Dl, Dh (n,3), scale (n)."""
    c = np.array(basis["center"], np.float64)
    p0 = np.array(basis["pixel00_loc"], np.float64)
    du = np.array(basis["pixel_delta_u"], np.float64)
    dv = np.array(basis["pixel_delta_v"], np.float64)
    pxl, pxh = x0 - 1.0, x1 + 1.0
    pyl, pyh = y0 - 1.0, y1 + 1.0
    pxm = np.maximum(abs(pxl), abs(pxh))
    pym = np.maximum(abs(pyl), abs(pyh))
    Dl = np.zeros((len(x0), 3))
    Dh = np.zeros((len(x0), 3))
    for a in range(3):
        base = p0[a] - c[a]
        u0, u1, v0, v1 = pxl * du[a], pxh * du[a], pyl * dv[a], pyh * dv[a]
        ulp = 8.0 * 1.1920928955078125e-7 * (abs(c[a]) + abs(p0[a]) + pxm * abs(du[a]) + pym * abs(dv[a]))
        Dl[:, a] = base + np.minimum(u0, u1) + np.minimum(v0, v1) - ulp
        Dh[:, a] = base + np.maximum(u0, u1) + np.maximum(v0, v1) + ulp
    scale = np.maximum(abs(Dl), abs(Dh)).max(axis=1)
    Dl -= 1e-5 * scale[:, None]
    Dh += 1e-5 * scale[:, None]
    return c, Dl, Dh, scale


def misses(c, Dl, Dh, scale, boxes):
    """tile_misses_box for every (tile, box): bool (n, k)."""
    mn = boxes[None, :, :3].astype(np.float64)
    mx = boxes[None, :, 3:].astype(np.float64)
    n = Dl.shape[0]
    entry = np.full((n, boxes.shape[0]), -np.inf)
    exit_ = np.full((n, boxes.shape[0]), np.inf)
    for a in range(3):
        dl, dh = Dl[:, a:a + 1], Dh[:, a:a + 1]
        use = (dl > 1e-6 * scale[:, None]) | (dh < -1e-6 * scale[:, None])
        nA, xA = mn[..., a] - c[a], mx[..., a] - c[a]
        pos = dl > 0
        ne = np.where(pos, nA, xA)
        nx = np.where(pos, xA, nA)
        with np.errstate(divide="ignore", invalid="ignore"):
            e0, e1 = ne / dl, ne / dh
            f0, f1 = nx / dl, nx / dh
        en = np.where(use, np.minimum(e0, e1), -np.inf)
        ex = np.where(use, np.maximum(f0, f1), np.inf)
        entry = np.maximum(entry, en)
        exit_ = np.minimum(exit_, ex)
    inside = np.ones((1, boxes.shape[0]), bool)
    for a in range(3):
        inside &= (c[a] >= mn[..., a]) & (c[a] <= mx[..., a])
    out = (exit_ < 0) | (entry - exit_ > 1e-9 * (abs(entry) + abs(exit_)))
    return out & ~inside


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="64,128,256,512,1024,4096")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--move", default="0,0,0", help="camera position offset (x,y,z)")
    a = ap.parse_args()
    W, H = map(int, a.size.split("x"))
    hs = rt.HostScene.load_json(REPO / "assets" / "scenes" / "frog.json", REPO)
    cam = hs.camera(W, H)
    mv = tuple(float(v) for v in a.move.split(","))
    if any(mv):
        cam = rt.Camera(tuple(np.add(cam.pos, mv)), cam.look_at, cam.up, cam.focal_length_mm, cam.sensor_height_mm,
                        W, H)
    b = cam.basis()
    oc = orc.camera_from_basis(b["center"], b["pixel00_loc"], b["pixel_delta_u"], b["pixel_delta_v"], W, H)
    t0 = time.time()
    _, hi, _ = orc.render_g(hs.num_triangles, oc, hs.nodes, hs.aabbs, hs.triangles, hs.tri_object_ids,
                            hs.materials, hs.lights, spp=a.spp, max_depth=1, aov=True, threads=8)
    print(f"oracle frame {time.time() - t0:.1f} s", flush=True)
    hit_px = (hi >= 0).any(axis=2)  # (H, W)
    # quarters: 2x2 pixel squares
    qh = hit_px[: H // 2 * 2, : W // 2 * 2].reshape(H // 2, 2, W // 2, 2).any(axis=(1, 3))
    th = hit_px[: H // 4 * 4, : W // 4 * 4].reshape(H // 4, 4, W // 4, 4).any(axis=(1, 3))
    print(f"tiles 4x4 hit: {int(th.sum())}, quarters 2x2 hit: {int(qh.sum())} (waves that hit something)")
    nodes, aabbs = np.asarray(hs.nodes), np.asarray(hs.aabbs)
    root = aabbs[0:1]
    ty, tx = np.mgrid[0:H // 4, 0:W // 4]
    tx, ty = tx.ravel(), ty.ravel()
    c, Dl, Dh, sc = tile_bounds(b, tx * 4.0, tx * 4.0 + 3, ty * 4.0, ty * 4.0 + 3)
    live = ~misses(c, Dl, Dh, sc, root)[:, 0]
    print(f"root survivors: {int(live.sum())} tiles")
    ltx, lty = tx[live], ty[live]
    # quarters of the live tiles
    qx = (ltx[:, None] * 2 + np.array([0, 1, 0, 1])[None]).ravel()
    qy = (lty[:, None] * 2 + np.array([0, 0, 1, 1])[None]).ravel()
    cq, qDl, qDh, qsc = tile_bounds(b, qx * 2.0, qx * 2.0 + 1, qy * 2.0, qy * 2.0 + 1)
    for k in map(int, a.ks.split(",")):
        cut = greedy_cut(nodes, aabbs, k)
        boxes = aabbs[cut]
        tl = ~misses(c, Dl[live], Dh[live], sc[live], boxes).all(axis=1)
        ql = ~misses(cq, qDl, qDh, qsc, boxes).all(axis=1)
        ql_in_tiles = ql & np.repeat(tl, 4)
        qhit = qh[qy, qx]
        print(f"K={len(cut):5d}: tiles kept {int(tl.sum()):6d} -> items {4 * int(tl.sum()):6d} "
              f"(no-hit items {4 * int(tl.sum()) - int(qhit[np.repeat(tl, 4)].sum())}); "
              f"per-quarter items kept {int(ql_in_tiles.sum()):6d} (no-hit {int((ql_in_tiles & ~qhit).sum())})",
              flush=True)


if __name__ == "__main__":
    main()
