"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only).

build.build_sanitized() compiles rt_host.cpp, the host side of every .hip unit, rt_render_cli.cpp
and the oracle's rt_oracle.c with clang -fsanitize=address,undefined (-fno-sanitize-recover: a
UBSan finding is fatal) into build/asan/.  This test runs the CPU tests that drive that code —
the scene/OBJ/P6 parsers and their malformed-input fuzz (tests/test_host_fuzz.py), the host API,
the CLI, the oracle against the reference's fixtures, the frustum-record builder and the AABB
filter — in a child python with the clang ASan runtime preloaded and RT_MI355X_LIB /
RT_ORACLE_LIB / RT_MI355X_CLI pointing at the sanitized builds.  It passes when every one of
them passes and no sanitizer report was written.

Findings this build made and that are fixed: a JSON file of 10^5 nested '[' overflowed the C
stack (the reader's nesting is now bounded); OBJ index digits past int's range overflowed a
signed int; JSON integers past int's range were converted with undefined behaviour; a forged P6
header was reported before its samples were checked; rt_debug_frustum_records followed child
indices past the caller's arrays and passed a null pointer to memcpy.
"""
from __future__ import annotations

import os
import subprocess
import sys

import pytest

from conftest import REPO

from raytracinginonesemester_amd import build as B

FILES = ["tests/test_host_fuzz.py", "tests/test_host.py", "tests/test_cli.py", "tests/test_oracle.py",
         "tests/test_frustum_records.py", "tests/test_box_filter.py"]


def test_host_code_is_clean_under_asan_and_ubsan(tmp_path):
    if B.asan_runtime() is None:
        pytest.skip("clang's AddressSanitizer runtime is not installed")
    paths = B.build_sanitized()
    env = dict(os.environ)
    env.update(LD_PRELOAD=str(paths["runtime"]),
               ASAN_OPTIONS=f"detect_leaks=0:log_path={tmp_path / 'asan'}",
               UBSAN_OPTIONS=f"print_stacktrace=1:log_path={tmp_path / 'ubsan'}",
               RT_MI355X_LIB=str(paths["lib"]), RT_ORACLE_LIB=str(paths["oracle"]), RT_MI355X_CLI=str(paths["cli"]))
    # (the build-id check is the one test that must fail here: the sanitized library carries an
    # "asan:" id, so it can never pass for the product build)
    r = subprocess.run([sys.executable, "-m", "pytest", *FILES, "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu",
                        "-k", "not loaded_library_is_built_from_these_sources"],
                       cwd=REPO, env=env, capture_output=True, text=True, timeout=1200)
    reports = sorted(p.name for p in tmp_path.iterdir() if p.name.startswith(("asan", "ubsan")))
    detail = "".join((tmp_path / n).read_text()[:3000] for n in reports)
    assert not reports, f"sanitizer reports {reports}:\n{detail}"
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert " passed" in r.stdout and " failed" not in r.stdout, r.stdout[-2000:]
