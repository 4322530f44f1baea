#!/bin/bash
# rocprofv3 passes over serialised frames of one config (scripts/profile_frames.py --mode serial:
# nothing overlaps the render kernel, so its traced duration is its own), run from the repo root
# on the GPU box: a kernel trace + stats, then one --pmc pass per counter group (counters never
# combined with runtime/sys tracing).  Output: gpurun_out/prof_<tag>/<pass>/...
# usage: scripts/prof_pmc.sh <tag> <config> [frames]
set -u
TAG=$1; CFG=$2; FRAMES=${3:-20}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
DRIVER=profile_frames.py
case "$CFG" in c1|c2) DRIVER=profile_hw1.py ;; esac  # the HW1 path (rt_hw1_scene)
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/$DRIVER" --config "$CFG" --frames "$FRAMES" --mode serial ${PROF_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
}
run trace --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
run sq2 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE
run tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum
