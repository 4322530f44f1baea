"""In-tree build of the native pieces (no JIT cache: the .so files travel with the repo).

    python -m raytracinginonesemester_amd.build

* librt_mi355x.so — rt_host.cpp (g++) + the device translation units (hipcc
  --offload-arch=gfx950): rt_device.hip (scene + render), rt_frame.hip (P6 quantisation and
  strip un-permute on the device), rt_lbvh.hip (LBVH build on the device).
  Every float path is compiled with -ffp-contract=off and without fast-math; HIP's default
  correctly rounded f32 division / sqrt stay on (parity with the reference CPU build).
* rt_render_cli   — C++ CLI over the C ABI (scene JSON in, P6 out), G/src/main.cu's role.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = PKG / "csrc"
OUT = PKG / "lib"
OBJ = REPO / "build" / "obj"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
FP = ["-ffp-contract=off", "-fno-fast-math"]
DEVICE_UNITS = ["rt_device", "rt_frame", "rt_lbvh", "rt_renderer"]


def _run(cmd):
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def build(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    OBJ.mkdir(parents=True, exist_ok=True)
    hdrs = [REPO / "include" / "rt_mi355x.h", CSRC / "rt_common.hpp", CSRC / "rt_math.hpp", CSRC / "rt_ppm.hpp",
            CSRC / "rt_hip_host.hpp"]
    host_o = OBJ / "rt_host.o"
    dev_objs = []
    so = OUT / "librt_mi355x.so"
    inc = [f"-I{REPO / 'include'}", f"-I{CSRC}"]
    if force or _stale(host_o, [CSRC / "rt_host.cpp", *hdrs]):
        _run([CXX, "-std=c++17", "-O2", "-fPIC", *FP, "-Wall", "-Wextra", *inc, "-c",
              CSRC / "rt_host.cpp", "-o", host_o])
    for name in DEVICE_UNITS:
        dev_o = OBJ / f"{name}.o"
        dev_objs.append(dev_o)
        if force or _stale(dev_o, [CSRC / f"{name}.hip", *hdrs]):
            # code object v5: loadable by both the image's ROCm 7.2 runtime and the ROCm 7.0 HIP
            # runtime bundled with torch (which the process uses when torch is imported first)
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *FP, "-Wall",
                  "-mcode-object-version=5",
                  "-Wno-unused-function", *inc, "-c", CSRC / f"{name}.hip", "-o", dev_o])
    if force or _stale(so, [host_o, *dev_objs]):
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", host_o, *dev_objs, "-o", so, "-ldl"])
    cli = OUT / "rt_render_cli"
    if force or _stale(cli, [CSRC / "rt_render_cli.cpp", REPO / "include" / "rt_mi355x.hpp", so]):
        _run([CXX, "-std=c++17", "-O2", *FP, "-Wall", *inc, CSRC / "rt_render_cli.cpp", "-o", cli,
              f"-L{OUT}", "-lrt_mi355x", f"-Wl,-rpath,$ORIGIN"])
    return so


if __name__ == "__main__":
    build(force="--force" in sys.argv)
