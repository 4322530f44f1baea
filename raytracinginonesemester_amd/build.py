"""In-tree build of the native pieces (no JIT cache: the .so files travel with the repo).

    python -m raytracinginonesemester_amd.build

* librt_mi355x.so — the host units rt_host.cpp and rt_records.cpp (g++) + the device translation
  units (hipcc --offload-arch=gfx950): rt_device.hip (scene + render; its device code in the
  rt_wave/instrument/traverse/shade/prepass.hpp sections), rt_hw1.hip (the HW1 path),
  rt_frame.hip (P6 quantisation and strip un-permute on the device), rt_lbvh.hip (LBVH build on
  the device), rt_renderer.hip (the multi-GPU frame renderer).  Units compile in parallel.
  Every float path is compiled with -ffp-contract=off and without fast-math; HIP's default
  correctly rounded f32 division / sqrt stay on (parity with the reference CPU build).
* rt_render_cli   — C++ CLI over the C ABI (scene JSON in, P6 out), G/src/main.cu's role.

build_sanitized() (CPU only, build/asan/): the host code — rt_host.cpp, the host side of every
.hip unit (-Xarch_host: the device code is built as usual, without sanitizers), rt_render_cli.cpp
and the oracle's rt_oracle.c — compiled by clang with -fsanitize=address,undefined
(-fno-sanitize-recover: a UBSan finding fails the run).  tests/test_sanitize.py runs the host,
CLI, oracle and malformed-input fuzz tests against it.
"""
from __future__ import annotations

import hashlib
import os
import re
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
DEVICE_UNITS = ["rt_device", "rt_hw1", "rt_frame", "rt_lbvh", "rt_renderer"]
HOST_UNITS = ["rt_host", "rt_records"]


ID_TAG = b"RT_BUILD_ID:"
SOURCE_SUFFIXES = (".hip", ".cpp", ".hpp", ".h")


def source_build_id() -> str:
    """sha256 over csrc/ and include/ (names and bytes, sorted) and the compile flags: the id
    compiled into librt_mi355x.so as rt_build_id(), so a stale prebuilt library is detectable."""
    h = hashlib.sha256()
    files = [p for d in (CSRC, REPO / "include") for p in d.iterdir() if p.suffix in SOURCE_SUFFIXES]
    for p in sorted(files, key=lambda q: q.relative_to(REPO).as_posix()):
        h.update(p.relative_to(REPO).as_posix().encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(" ".join([ARCH, *FP, "-O3", "-mcode-object-version=5"]).encode())
    return h.hexdigest()


def library_build_id(so: Path | None = None) -> str | None:
    """The id embedded in a built librt_mi355x.so (read from its bytes, nothing is loaded)."""
    so = so or OUT / "librt_mi355x.so"
    if not so.exists():
        return None
    m = re.search(re.escape(ID_TAG) + rb"([0-9a-f]{64})", so.read_bytes())
    return m.group(1).decode() if m else None


def _run(cmd):
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True)


def _step(target: Path, deps, cmd, force: bool) -> None:
    """Run cmd unless target exists and was made by this same cmd from these same input bytes
    (a content stamp beside the target; mtimes are not trusted)."""
    h = hashlib.sha256(" ".join(str(c) for c in cmd).encode())
    for d in deps:
        h.update(Path(d).read_bytes())
    stamp = Path(str(target) + ".inputs")
    if not force and target.exists() and stamp.exists() and stamp.read_text() == h.hexdigest():
        return
    _run(cmd)
    stamp.write_text(h.hexdigest())


def _parallel(jobs, force: bool) -> None:
    """_step over (target, deps, cmd) jobs on a few threads (each job is its own process)."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), os.cpu_count() or 1, 8))) as ex:
        for f in [ex.submit(_step, o, deps, cmd, force) for o, deps, cmd in jobs]:
            f.result()


def build(force: bool = False) -> Path:
    OUT.mkdir(parents=True, exist_ok=True)
    OBJ.mkdir(parents=True, exist_ok=True)
    bid = source_build_id()
    hdrs = [REPO / "include" / "rt_mi355x.h", *sorted(CSRC.glob("*.hpp"))]
    inc = [f"-I{REPO / 'include'}", f"-I{CSRC}"]
    jobs = []
    host_objs = []
    for name in HOST_UNITS:
        o = OBJ / f"{name}.o"
        host_objs.append(o)
        jobs.append((o, [CSRC / f"{name}.cpp", *hdrs],
                     [CXX, "-std=c++17", "-O2", "-fPIC", *FP, "-Wall", "-Wextra", *inc, "-c", CSRC / f"{name}.cpp", "-o", o]))
    dev_objs = []
    so = OUT / "librt_mi355x.so"
    for name in DEVICE_UNITS:
        dev_o = OBJ / f"{name}.o"
        dev_objs.append(dev_o)
        # code object v5: loadable by both the image's ROCm 7.2 runtime and the ROCm 7.0 HIP
        # runtime bundled with torch (which the process uses when torch is imported first)
        jobs.append((dev_o, [CSRC / f"{name}.hip", *hdrs],
                     [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *FP, "-Wall",
                      "-mcode-object-version=5", "-Wno-unused-function", *inc, "-c", CSRC / f"{name}.hip", "-o", dev_o]))
    _parallel(jobs, force)
    id_c = OBJ / "rt_build_id.c"
    id_c.write_text("/* generated by build.py: sha256 of csrc/ + include/ + flags */\n"
                    f"static const char tag[] __attribute__((used)) = \"{ID_TAG.decode()}{bid}\";\n"
                    "const char* rt_build_id(void) { return tag + %d; }\n" % len(ID_TAG))
    id_o = OBJ / "rt_build_id.o"
    _step(id_o, [id_c], ["gcc", "-O2", "-fPIC", "-c", id_c, "-o", id_o], force)
    _step(so, [*host_objs, *dev_objs, id_o],
          [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *host_objs, *dev_objs, id_o, "-o", so, "-ldl"],
          force or library_build_id(so) != bid)
    if library_build_id(so) != bid:
        raise RuntimeError(f"{so}: embedded build id does not match the sources")
    cli = OUT / "rt_render_cli"
    _step(cli, [CSRC / "rt_render_cli.cpp", REPO / "include" / "rt_mi355x.hpp", so],
          [CXX, "-std=c++17", "-O2", *FP, "-Wall", *inc, CSRC / "rt_render_cli.cpp", "-o", cli,
           f"-L{OUT}", "-lrt_mi355x", "-Wl,-rpath,$ORIGIN"], force)
    return so


ASAN = REPO / "build" / "asan"
LLVM_BIN = Path("/opt/rocm/lib/llvm/bin")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer", "-g", "-O1",
       "-shared-libsan"]


def asan_runtime() -> Path | None:
    """The clang AddressSanitizer runtime the sanitized build links against (LD_PRELOAD it into
    an uninstrumented python), or None when clang or its runtime is missing."""
    clang = LLVM_BIN / "clang++"
    if not clang.exists():
        return None
    r = subprocess.run([str(clang), "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True)
    p = Path(r.stdout.strip())
    return p if r.returncode == 0 and p.is_absolute() and p.exists() else None


def build_sanitized(force: bool = False) -> dict:
    """CPU-only ASan/UBSan build of the host code (see the module docstring); returns the paths."""
    ASAN.mkdir(parents=True, exist_ok=True)
    cxx, cc = LLVM_BIN / "clang++", LLVM_BIN / "clang"
    hdrs = [REPO / "include" / "rt_mi355x.h", *sorted(CSRC.glob("*.hpp"))]
    inc = [f"-I{REPO / 'include'}", f"-I{CSRC}"]
    objs = []
    jobs = []
    for name in HOST_UNITS:
        o = ASAN / f"{name}.o"
        jobs.append((o, [CSRC / f"{name}.cpp", *hdrs],
                     [cxx, "-std=c++17", "-fPIC", *FP, *SAN, *inc, "-c", CSRC / f"{name}.cpp", "-o", o]))
        objs.append(o)
    # the .hip units whole (a host-only object would reference its missing device bundle), the
    # sanitizers on the host side only (-Xarch_host: no GPU sanitizer)
    host_san = [f for flag in SAN for f in ("-Xarch_host", flag)]
    for name in DEVICE_UNITS:
        o = ASAN / f"{name}.o"
        jobs.append((o, [CSRC / f"{name}.hip", *hdrs],
                     [HIPCC, f"--offload-arch={ARCH}", "-O1", "-std=c++17", "-fPIC", *FP, *host_san,
                      "-mcode-object-version=5", "-Wno-unused-function", *inc, "-c", CSRC / f"{name}.hip", "-o", o]))
        objs.append(o)
    _parallel(jobs, force)
    id_c = ASAN / "rt_build_id.c"
    id_c.write_text("/* the sanitized CPU-only build: never the product's id */\n"
                    f"static const char tag[] __attribute__((used)) = \"asan:{source_build_id()}\";\n"
                    "const char* rt_build_id(void) { return tag; }\n")
    id_o = ASAN / "rt_build_id.o"
    _step(id_o, [id_c], [cc, "-O1", "-fPIC", "-c", id_c, "-o", id_o], force)
    objs.append(id_o)
    so = ASAN / "librt_mi355x.so"
    _step(so, objs, [cxx, "-shared", "-fPIC", *SAN, *objs, "-o", so, "-L/opt/rocm/lib", "-lamdhip64",
                     "-Wl,-rpath,/opt/rocm/lib", "-ldl"], force)
    cli = ASAN / "rt_render_cli"
    _step(cli, [CSRC / "rt_render_cli.cpp", REPO / "include" / "rt_mi355x.hpp", so],
          [cxx, "-std=c++17", *FP, *SAN, *inc, CSRC / "rt_render_cli.cpp", "-o", cli, f"-L{ASAN}", "-lrt_mi355x",
           "-Wl,-rpath,$ORIGIN"], force)
    orc = ASAN / "liboracle.so"
    osrc = REPO / "oracle" / "rt_oracle.c"
    _step(orc, [osrc, REPO / "oracle" / "rt_oracle.h"],
          [cc, "-std=c11", "-fPIC", "-shared", *FP, *SAN, "-fopenmp", osrc, "-o", orc, "-lm",
           f"-Wl,-rpath,{LLVM_BIN.parent / 'lib'}"], force)
    return {"lib": so, "cli": cli, "oracle": orc, "runtime": asan_runtime()}


if __name__ == "__main__":
    if "--asan" in sys.argv:
        print(build_sanitized(force="--force" in sys.argv))
    else:
        build(force="--force" in sys.argv)
