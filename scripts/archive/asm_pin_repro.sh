#!/bin/bash
# Reproducer of the round-1 golden failures fixed by 5e451d6: export the tree
# before that commit into build/old_tree, build it in-tree (CPU), then on the GPU box run
#   cd build/old_tree && python -m pytest tests/test_gpu_parity.py -k golden_scene_parity
# (4 of 20 fail: the bounce-scene WAVE kernels).  The same asm on the current source
# (scripts/build_variant.sh asmpin -DRT_EXP_ASM_PIN -DRT_RENDER_WAVES=6) passes all 20.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
rm -rf "$ROOT/build/old_tree" && mkdir -p "$ROOT/build/old_tree"
git -C "$ROOT" archive 5e451d6^ | tar -x -C "$ROOT/build/old_tree"
cd "$ROOT/build/old_tree" && python3 -c "import __graft_entry__ as g; g.build()" > /dev/null
rm -rf "$ROOT/build/old_tree/oracle/_ref"
