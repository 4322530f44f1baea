"""Shared fixtures.  `-m "not gpu"` runs on any CPU host; `-m gpu` needs an MI355X."""
from __future__ import annotations

import gzip
import json
import sys
from functools import lru_cache
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running case")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the in-tree native pieces exist (build() is also run by the driver)."""
    import subprocess

    so = REPO / "raytracinginonesemester_amd" / "lib" / "librt_mi355x.so"
    if not so.exists():
        from raytracinginonesemester_amd import build as b

        b.build()
    if not (REPO / "oracle" / "liboracle.so").exists():
        subprocess.run(["make", "-s", "-C", str(REPO / "oracle")], check=True)


@pytest.fixture
def tune():
    """Set library tuning knobs for one test (rt_tuning_set); every knob is reset after it."""
    import raytracinginonesemester_amd as rt

    def set_(**knobs):
        for k, v in knobs.items():
            rt.set_tuning(k, v)

    yield set_
    rt.reset_tuning()


def golden_meta(name: str) -> dict:
    return json.loads((GOLDEN / "scenes" / name / "meta.json").read_text())


def golden_array(name: str, fname: str, dtype) -> np.ndarray:
    return np.frombuffer(gzip.open(GOLDEN / "scenes" / name / fname).read(), dtype)


def hexv(a):
    return np.array([float.fromhex(x) for x in a], np.float32)


# golden G/ scene fixtures -> scene JSON (tests/golden/gen_golden.py G_FIXTURES)
G_SCENES = {
    "c3_small": "frog.json",
    "frog_bounce": "frog.json",
    "sphere_single": "sphere_single.json",
    "cornell": "cornell.json",
    "c5_small": "heightfield_c5.json",
    "c3b_small": "frog.json",
}


@lru_cache(maxsize=None)
def host_scene(scene: str):
    import raytracinginonesemester_amd as rt
    from raytracinginonesemester_amd import configs

    sp = configs.scene_path(scene)
    proj = REPO if sp.parent == configs.SCENES else sp.parent
    return rt.HostScene.load_json(sp, proj)


def oracle_camera(cam):
    from oracle import pyoracle as orc

    b = cam.basis()
    return orc.camera_from_basis(b["center"], b["pixel00_loc"], b["pixel_delta_u"], b["pixel_delta_v"],
                                 cam.pixel_width, cam.pixel_height)


def gpu_available() -> bool:
    try:
        import raytracinginonesemester_amd as rt

        return rt.device_count() > 0
    except Exception:
        return False
