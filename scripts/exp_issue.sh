#!/bin/bash
# Issue-pipe counters of the c3 render kernel (one --pmc pass): scalar ALU / SMEM / branch /
# VALU cycles, issue waits, CU busy; summarised by scripts/pmc_sum.py.
# usage: scripts/exp_issue.sh <tag> [render_case args]
set -u
TAG=${1:-issue}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/scripts/render_case.py" ${@:-full} 3 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
