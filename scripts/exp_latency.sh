#!/bin/bash
# Memory-latency counters of the c3 render kernel (one --pmc pass per group), and the
# empty-dispatch floor (all tiles culled: the render grid's blocks all leave at once).
# usage: scripts/exp_latency.sh <tag>
set -u
TAG=${1:-lat}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
timeout -k 10 120 python3 "$ROOT/scripts/render_case.py" all_miss 20 > "$OUT/all_miss.log" 2>&1 || exit $?
timeout -k 10 120 python3 "$ROOT/scripts/render_case.py" full 20 > "$OUT/full.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SmemLatency" "VmemLatency" "MeanOccupancyPerActiveCU" \
           "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_TC_DATA_READ_REQ SQC_TC_STALL SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$ROOT/scripts/render_case.py" full 3 > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
done
