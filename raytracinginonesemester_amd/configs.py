"""Workload definitions shared by tests, bench.py and tests/golden/gen_golden.py.

The five configurations are BASELINE.json's ``configs`` made concrete:

* ``c1`` — HW1 brute-force path, sphere, 256x256, 1 spp (HW1/src/render.cpp:72-116 with a
  camera that sees the sphere; the hard-coded one at render.cpp:43-58 gives a flat image).
* ``c2`` — HW1 path on frog.obj, 640x480, 1 spp, primary rays + HW1 ``shade`` only.
* ``c3`` — G/ path, frog.json (HW2/HW2/GPUandCPU/assets/json_files/frog.json), 1920x1080,
  16 spp, max_bounces overridden to 1: Lambert/Blinn-Phong + one hard shadow ray.
* ``c3b`` — c3 with frog.json's own max_bounces 8 (diffuse bounces), the reference default.
* ``c4`` — c3 split over N GPUs (image bands) + RCCL gather.
* ``c5`` — seeded 1,048,576-triangle heightfield, 3840x2160, 64 spp (HBM stress).
"""
from __future__ import annotations

import os
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
ASSETS = REPO / "assets"
MESHES = ASSETS / "meshes"
SCENES = ASSETS / "scenes"
CACHE = Path(os.environ.get("RT_CACHE_DIR", REPO / "build" / "cache"))

# HW1 brute-force configurations (camera/light arguments of HW1 camera + Light).
HW1_CONFIGS = {
    "c1": dict(mesh="sphere.obj", width=256, height=256, spp=1,
               position=(0.0, -4.0, 1.0), look_at=(0.0, 0.0, 0.0), up=(0.0, 0.0, 1.0),
               focal_mm=50.0, sensor_mm=24.0,
               light_pos=(-3.0, 0.0, 1.0), light_color=(1.0, 0.0, 1.0)),
    "c2": dict(mesh="frog.obj", width=640, height=480, spp=1,
               position=(0.0, -1.0, 1.0), look_at=(0.0, 0.15, 0.0), up=(0.0, 0.0, 1.0),
               focal_mm=255.0, sensor_mm=24.0,
               light_pos=(-3.0, 0.0, 1.0), light_color=(1.0, 0.0, 1.0)),
}

# G/ scene configurations: scene JSON + overrides (None keeps the JSON's value).
G_CONFIGS = {
    "c3": dict(scene="frog.json", width=1920, height=1080, spp=16, max_depth=1),
    # frog.json as shipped (max_bounces 8, diffuse bounce on) at 1080p x 16 spp: the reference's
    # default workload (G/assets/json_files/frog.json:3, G/include/scene.h:15-19)
    "c3b": dict(scene="frog.json", width=1920, height=1080, spp=16, max_depth=8),
    "c5": dict(scene="heightfield_c5.json", width=3840, height=2160, spp=64, max_depth=1),
    # the reference's other shipped scenes at their shipped settings (G/assets/json_files/):
    # sphere.json (128 spp: whole-tile work items, 4 bounces, mirrors, no diffuse bounce) and
    # sphere_single.json (64 spp, 4 diffuse bounces)
    "sphere": dict(scene="sphere.json", width=1920, height=1080, spp=128, max_depth=4),
    "sphere_single": dict(scene="sphere_single.json", width=1920, height=1080, spp=64, max_depth=4),
    # a multi-light bounce scene (two lights: the unpaired bounce loop, G/include/shader.h:87-94)
    "cornell": dict(scene="cornell.json", width=1920, height=1080, spp=16, max_depth=3),
}

# Algorithmic bytes per camera sample (SURVEY.md §8(d) traffic model: 24 B per AABB fetched
# per pop-test and per pushed child test, 16 B per BVHNode entered, 72 B per Triangle tested),
# replayed with the oracle's counters over the reference SearchBVH order (scripts/bytes_model.py):
#   c3: whole frame, 33,177,600 samples: 300.316 B (primary 248.96 B/ray, shadow
#       2,478.4 B/ray x 0.02072 shadow rays/sample) + 12 B/pixel framebuffer / 16 spp.
#   c5: every 27th row (19,660,800 samples): 11,159.58 B (primary 8,316.3 B/ray, shadow
#       13,508.3 B/ray x 0.2105/sample) + 12 B / 64 spp.
BYTES_PER_SAMPLE = {"c3": 300.316 + 12.0 / 16, "c5": 11159.58 + 12.0 / 64}

# Heightfield generator parameters for c5.
C5_GRID = (1024, 512)          # quads in x, y -> 1,048,576 triangles
C5_SEED = 20260315


def _splitmix64(x: int) -> int:
    m = (1 << 64) - 1
    z = (x + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def heightfield_obj_text(nx: int = C5_GRID[0], ny: int = C5_GRID[1], seed: int = C5_SEED) -> str:
    """OBJ text of the seeded heightfield: (nx+1)*(ny+1) vertices on x in [-2,2], y in [-1,1],
    z = 0.1 * u(i, j) with u = splitmix64(seed ^ i*73856093 ^ j*19349663) >> 40 scaled to
    [0,1); quads (v00, v10, v11, v01), no normals.  Floats printed with %.9g so every loader
    parses the same float32 values."""
    import numpy as np

    i = np.arange(nx + 1, dtype=np.uint64)
    j = np.arange(ny + 1, dtype=np.uint64)
    ii, jj = np.meshgrid(i, j, indexing="xy")           # row = j, col = i
    key = (np.uint64(seed) ^ (ii * np.uint64(73856093)) ^ (jj * np.uint64(19349663)))
    with np.errstate(over="ignore"):
        z = key + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    xs = -2.0 + 4.0 * ii.astype(np.float64) / nx
    ys = -1.0 + 2.0 * jj.astype(np.float64) / ny
    zs = 0.1 * u
    lines = ["# seeded heightfield (raytracinginonesemester_amd.configs)", "o heightfield"]
    v = np.stack([xs.ravel(), ys.ravel(), zs.ravel()], axis=1)
    lines += ["v %.9g %.9g %.9g" % tuple(r) for r in v]
    w = nx + 1
    for jy in range(ny):
        base = jy * w
        for ix in range(nx):
            v00 = base + ix + 1
            v10 = v00 + 1
            v01 = v00 + w
            v11 = v01 + 1
            lines.append(f"f {v00} {v10} {v11} {v01}")
    return "\n".join(lines) + "\n"


C5_SCENE_JSON = """{
    "settings": { "max_bounces": 1, "spp": 64 },
    "miss_color": [0.5, 0.7, 1.0],
    "camera": {
        "focal_length_mm": 24.0, "sensor_height_mm": 24.0,
        "pixel_width": 3840, "pixel_height": 2160,
        "position": [0.0, -2.5, 1.5], "look_at": [0.0, 0.0, 0.0], "up": [0.0, 0.0, 1.0]
    },
    "light": { "position": [-2.0, -1.0, 3.0], "color": [1.0, 1.0, 1.0], "intensity": 5.0 },
    "scene": [
        { "name": "heightfield", "type": "mesh", "path": "./heightfield_c5.obj",
          "material": { "albedo": [0.6, 0.55, 0.5], "kd": 1, "ks": 0 } }
    ]
}
"""


def ensure_c5_scene(cache: Path = CACHE) -> Path:
    """Write (once) the c5 heightfield OBJ + scene JSON into the cache dir; return the JSON."""
    cache.mkdir(parents=True, exist_ok=True)
    obj = cache / "heightfield_c5.obj"
    js = cache / "heightfield_c5.json"
    if not obj.exists():
        tmp = obj.with_suffix(".tmp")
        tmp.write_text(heightfield_obj_text())
        tmp.replace(obj)
    if not js.exists() or js.read_text() != C5_SCENE_JSON:
        js.write_text(C5_SCENE_JSON)
    return js


def scene_path(name: str) -> Path:
    if name == "heightfield_c5.json":
        return ensure_c5_scene()
    return SCENES / name
