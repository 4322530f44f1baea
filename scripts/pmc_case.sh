#!/bin/bash
# PMC passes for one render case: scripts/pmc_case.sh <tag> <case> [extra args]
set -u
TAG=$1; CASE=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/scripts/render_case.py" "$CASE" 3 "$@" > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
