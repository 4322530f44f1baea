#!/bin/bash
# Instruction-cache counters of the c3 render kernel (serialised frames), one small pass each.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_icache
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/profile_frames.py" --config c3 --frames 12 --mode serial > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
pass ic SQC_ICACHE_HITS SQC_ICACHE_MISSES
pass ic2 SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ
pass ifetch SQ_IFETCH SQ_WAVES
