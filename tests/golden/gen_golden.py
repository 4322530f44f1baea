#!/usr/bin/env python3
"""Generate tests/golden/ from the reference itself (run in the build container only).

Requires /root/reference and the driver binaries built from it by ``make -C oracle ref``
(oracle/_ref/ref_g, ref_hw1, ref_ppm).  Everything written here is DATA produced by the
reference's own code: jitter tables, ray-triangle KAT answers, camera bases, scene arrays
(as sha256), per-sample primary hits, float framebuffers and P6 files.

    python tests/golden/gen_golden.py            # all fixtures
    python tests/golden/gen_golden.py --only c3_small
"""
from __future__ import annotations

import argparse
import gzip
import hashlib
import json
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))
from raytracinginonesemester_amd import configs  # noqa: E402

REF = REPO / "oracle" / "_ref"

# G/ scene fixtures: name -> (scene json, W, H, spp, max_depth, keep raw hits); keep None: sha256
# of the outputs only (full-size frames too large to commit)
G_FIXTURES = {
    "c3_small": ("frog.json", 192, 108, 16, 1, True),
    "c3_full": ("frog.json", 1920, 1080, 16, 1, False),
    "frog_bounce": ("frog.json", 96, 54, 4, 0, True),          # JSON's own max_bounces 8
    "sphere_single": ("sphere_single.json", 160, 90, 4, 0, True),
    "cornell": ("cornell.json", 160, 120, 4, 0, True),
    "c5_small": ("heightfield_c5.json", 384, 216, 4, 1, True),
    # BASELINE config 5 at its full size (3840x2160x64, depth 1): the reference's frame, hit
    # and t buffers by sha256 (reference CPU render(), single-threaded: tens of CPU-minutes)
    "c5_full": ("heightfield_c5.json", 3840, 2160, 64, 1, None),
    # c3b: frog.json's own max_bounces 8 (diffuse bounce), 16 spp (bench config c3b)
    "c3b_small": ("frog.json", 192, 108, 16, 0, True),
    "c3b_full": ("frog.json", 1920, 1080, 16, 0, False),
    # sphere.json as shipped (G/assets/json_files/sphere.json): five scaled sphere instances and a
    # plane, mirrors kr 0.35/0.95/0.5, shininess up to 100000, 128 spp (spp > 64: whole-tile
    # work items), 4 bounces, diffuse_bounce false
    "sphere": ("sphere.json", 192, 108, 128, 0, False),
    "sphere_full": ("sphere.json", 1920, 1080, 128, 0, None),
    # sphere_single.json at its shipped 1920x1080x64, 4 diffuse bounces
    "sphere_single_full": ("sphere_single.json", 1920, 1080, 64, 0, None),
}
# HW1 fixtures: name -> (config, W, H)
HW1_FIXTURES = {
    "c1_full": ("c1", 256, 256),
    "c2_small": ("c2", 160, 120),
    "c2_full": ("c2", 640, 480),
}
PPM_OF = {"c1_full", "c2_full", "c3_full", "c3_small", "c3b_full"}


def sha256(p: Path) -> str:
    return hashlib.sha256(p.read_bytes()).hexdigest()


def gz(src: Path, dst: Path) -> None:
    with open(src, "rb") as f, open(dst, "wb") as raw:
        with gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0, filename="") as g:
            shutil.copyfileobj(f, g)


def run(cmd, **kw):
    print("+", " ".join(str(c) for c in cmd), flush=True)
    return subprocess.run([str(c) for c in cmd], check=True, **kw)


def gen_jitter() -> None:
    out = {"g_seed42": {}, "hw1_seed42": {}}
    for spp in (1, 4, 16, 64):
        r = run([REF / "ref_g", "jitter", spp, 42], capture_output=True, text=True)
        out["g_seed42"][str(spp)] = [ln.split() for ln in r.stdout.strip().splitlines()]
    for spp in (1, 16):
        r = run([REF / "ref_hw1", "jitter", spp, 42], capture_output=True, text=True)
        out["hw1_seed42"][str(spp)] = [ln.split() for ln in r.stdout.strip().splitlines()]
    (HERE / "jitter.json").write_text(json.dumps(out, indent=1) + "\n")


def gen_kat() -> None:
    r = run([REF / "ref_hw1", "kat"], capture_output=True, text=True)
    rows = []
    for ln in r.stdout.strip().splitlines():
        dx, dy, dz, hit, t = ln.split()
        rows.append({"dir": [dx, dy, dz], "hit": int(hit), "t": t})
    doc = {
        "source": "HW1/test_ray_tri_inter_STANDALONE/test_ray_triangle_inter.cpp:17-126 rays, "
                  "answers from HW1/include/ray.h:67-117 (reference build)",
        "triangle": {"v0": [-5.0, -5.0, -10.0], "v1": [0.0, 5.0, -10.0], "v2": [5.0, -5.0, -10.0],
                     "n": [0.0, 0.0, 1.0]},
        "origin": [0.0, 0.0, 0.0],
        "rays": rows,
    }
    (HERE / "kat_hw1.json").write_text(json.dumps(doc, indent=1) + "\n")


def ppm(fb: Path, W: int, H: int, dst_gz: Path) -> None:
    with tempfile.TemporaryDirectory() as td:
        p = Path(td) / "out.ppm"
        run([REF / "ref_ppm", fb, W, H, p])
        gz(p, dst_gz)


def gen_g(name: str) -> None:
    scene, W, H, spp, depth, keep_hits = G_FIXTURES[name]
    dst = HERE / "scenes" / name
    dst.mkdir(parents=True, exist_ok=True)
    sp = configs.scene_path(scene)
    project = REPO if sp.parent == configs.SCENES else sp.parent
    with tempfile.TemporaryDirectory() as td:
        t = Path(td)
        run([REF / "ref_g", "scene", sp, project, t, W, H, spp, depth, -1, 1])
        meta = json.loads((t / "meta.json").read_text())
        meta["scene"] = scene
        meta["sha256"] = {k: sha256(t / k) for k in
                          ("nodes.bin", "aabbs.bin", "tris.bin", "triobj.bin", "mats.bin",
                           "lights.bin", "fb.f32", "hits.i32", "hitt.f32")}
        if keep_hits is not None:
            gz(t / "fb.f32", dst / "fb.f32.gz")
        if keep_hits:
            gz(t / "hits.i32", dst / "hits.i32.gz")
            gz(t / "hitt.f32", dst / "hitt.f32.gz")
        if name in PPM_OF:
            ppm(t / "fb.f32", meta["width"], meta["height"], dst / "image.ppm.gz")
        if keep_hits is None:  # the P6 file write_p6 makes of the frame, by sha256
            run([REF / "ref_ppm", t / "fb.f32", meta["width"], meta["height"], t / "image.ppm"])
            meta["sha256"]["image.ppm"] = sha256(t / "image.ppm")
        (dst / "meta.json").write_text(json.dumps(meta, indent=1) + "\n")


def gen_hw1(name: str) -> None:
    cfg_name, W, H = HW1_FIXTURES[name]
    c = configs.HW1_CONFIGS[cfg_name]
    dst = HERE / "scenes" / name
    dst.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        t = Path(td)
        args = [REF / "ref_hw1", "render", configs.MESHES / c["mesh"], t, W, H,
                *c["position"], *c["look_at"], *c["up"], c["focal_mm"], c["sensor_mm"],
                *c["light_pos"], *c["light_color"], c["spp"]]
        run(args)
        meta = {"config": cfg_name, "width": W, "height": H, "spp": c["spp"],
                "sha256": {k: sha256(t / k) for k in ("fb.f32", "hits.i32", "hitt.f32")}}
        gz(t / "fb.f32", dst / "fb.f32.gz")
        gz(t / "hits.i32", dst / "hits.i32.gz")
        gz(t / "hitt.f32", dst / "hitt.f32.gz")
        if name in PPM_OF:
            ppm(t / "fb.f32", W, H, dst / "image.ppm.gz")
        (dst / "meta.json").write_text(json.dumps(meta, indent=1) + "\n")


def gen_chain(name: str) -> None:
    """Caterpillar BVHs deeper than 64 / 512 DFS entries (tests/golden/chain_bvh.py) through the
    reference render() and SearchBVH (ref_g arrays)."""
    sys.path.insert(0, str(HERE))
    import chain_bvh

    P, W, H, spp, depth = chain_bvh.FIXTURES[name]
    dst = HERE / "scenes" / name
    dst.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        t = Path(td)
        chain_bvh.write_arrays(chain_bvh.chain_scene(P), t)
        run([REF / "ref_g", "arrays", t, t, W, H, spp, depth, 1])
        meta = json.loads((t / "meta.json").read_text())
        meta["generator"] = "tests/golden/chain_bvh.py chain_scene(%d)" % P
        meta["sha256"] = {k: sha256(t / k) for k in
                          ("nodes.bin", "aabbs.bin", "tris.bin", "triobj.bin", "mats.bin", "lights.bin",
                           "fb.f32", "hits.i32", "hitt.f32")}
        for k in ("fb.f32", "hits.i32", "hitt.f32"):
            gz(t / k, dst / (k + ".gz"))
        (dst / "meta.json").write_text(json.dumps(meta, indent=1) + "\n")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    a = ap.parse_args()
    if not (REF / "ref_g").exists():
        sys.exit("build the reference drivers first: make -C oracle ref")
    want = set(a.only) if a.only else None
    sys.path.insert(0, str(HERE))
    import chain_bvh

    for n in chain_bvh.FIXTURES:
        if not want or n in want:
            gen_chain(n)
    if not want or "jitter" in want:
        gen_jitter()
    if not want or "kat" in want:
        gen_kat()
    for n in G_FIXTURES:
        if not want or n in want:
            gen_g(n)
    for n in HW1_FIXTURES:
        if not want or n in want:
            gen_hw1(n)


if __name__ == "__main__":
    main()
