#!/bin/bash
# rocprofv3 passes over the bench workload (run from the repo root on the GPU box):
#   1 kernel trace + stats; then one --pmc pass per counter group (counters never combined
#   with runtime/sys tracing).  Output: gpurun_out/prof_<tag>/<pass>/...
# usage: scripts/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS=${*:-"--steps 20 --warmup 3"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$ROOT/bench.py" --no-cpu-baseline --no-parity $ARGS > "$OUT/$name.log" 2>&1
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
