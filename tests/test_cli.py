"""rt_render_cli — the reference app's role (G/src/main.cu:98-436: scene JSON in, render, P6 out)
over the C++ host API (include/rt_mi355x.hpp).

GPU: the frog scene at the C3 settings written by the CLI is the reference's own P6 file byte
for byte (tests/golden/scenes/c3_full/image.ppm.gz: the reference render() + ppm_p6 write_p6).
CPU: the binary exists, links the in-tree library and rejects bad usage without a GPU.
"""
from __future__ import annotations

import gzip
import os
import subprocess
from pathlib import Path

import pytest

from conftest import GOLDEN, REPO

# RT_MI355X_CLI: another build of the CLI (tests/test_sanitize.py: the ASan/UBSan one)
CLI = Path(os.environ.get("RT_MI355X_CLI", REPO / "raytracinginonesemester_amd" / "lib" / "rt_render_cli"))


def test_cli_usage_without_arguments():
    r = subprocess.run([str(CLI)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage:" in r.stderr


def test_cli_missing_scene_is_an_error():
    r = subprocess.run([str(CLI), str(REPO / "assets" / "scenes" / "no_such_scene.json")], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 1 and "error:" in r.stderr


@pytest.mark.gpu
def test_cli_renders_the_reference_c3_image(tmp_path):
    out = tmp_path / "frog.ppm"
    r = subprocess.run([str(CLI), str(REPO / "assets" / "scenes" / "frog.json"), "--project", str(REPO), "--spp", "16",
                        "--depth", "1", "--width", "1920", "--height", "1080", "-o", str(out)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "GPU Render Time" in r.stdout
    want = gzip.open(GOLDEN / "scenes" / "c3_full" / "image.ppm.gz").read()
    assert out.read_bytes() == want
