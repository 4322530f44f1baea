#!/bin/bash
# Kernel-trace (no counters) each anatomy case: scripts/trace_cases.sh <tag> [cases...]
set -u
TAG=$1; shift
CASES=${*:-"full no_light all_miss"}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for c in $CASES; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$c" -o run -- \
      python3 "$ROOT/scripts/render_case.py" "$c" 10 > "$OUT/$c.log" 2>&1
  rc=$?; echo "$c rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
  find "$OUT/$c" -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | cut -c1-200
done
