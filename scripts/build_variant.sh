#!/bin/bash
# Build an experimental variant of the device library with extra compile flags:
#   scripts/build_variant.sh <name> [-DFLAG ...]  ->  build/variants/<name>/librt_mi355x.so
#   SRC=<file.hip> scripts/build_variant.sh ...   builds that device source instead (e.g. an
#   older revision exported with `git show REV:raytracinginonesemester_amd/csrc/rt_device.hip`)
# The in-tree library is left as it is (its objects are built once if missing).
# Run against it with RT_MI355X_LIB=build/variants/<name>/librt_mi355x.so.
set -eu
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/build/variants/$NAME
SRC=${SRC:-$ROOT/raytracinginonesemester_amd/csrc/rt_device.hip}
mkdir -p "$OUT"
if [ ! -f "$ROOT/build/obj/rt_host.o" ] || [ ! -f "$ROOT/build/obj/rt_hw1.o" ]; then
  python3 -c "import sys; sys.path.insert(0, '$ROOT'); from raytracinginonesemester_amd import build; build.build()" > /dev/null
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall \
    -mcode-object-version=5 -Wno-unused-function "$@" -I"$ROOT/include" -I"$ROOT/raytracinginonesemester_amd/csrc" \
    -c -x hip "$SRC" -o "$OUT/rt_device.o"
# the variant's own rt_build_id: "variant:<name>:" + sha256 of the device source and the extra
# flags, so a variant library can never pass for the product build (whose id is the sources' hash)
VID=$( (cat "$SRC"; printf '%s\0' "$@") | sha256sum | cut -c1-64)
printf 'static const char tag[] __attribute__((used)) = "variant:%s:%s";\nconst char* rt_build_id(void) { return tag; }\n' \
    "$NAME" "$VID" > "$OUT/rt_build_id.c"
gcc -O2 -fPIC -c "$OUT/rt_build_id.c" -o "$OUT/rt_build_id.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$ROOT/build/obj/rt_host.o" "$ROOT/build/obj/rt_records.o" "$OUT/rt_device.o" "$ROOT/build/obj/rt_hw1.o" \
    "$ROOT/build/obj/rt_frame.o" "$ROOT/build/obj/rt_lbvh.o" "$ROOT/build/obj/rt_renderer.o" "$OUT/rt_build_id.o" \
    -o "$OUT/librt_mi355x.so"
rm -f "$OUT/rt_device.o" "$OUT/rt_build_id.o"  # only the library travels to the GPU box
echo "$OUT/librt_mi355x.so"
