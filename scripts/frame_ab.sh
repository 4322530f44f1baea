#!/bin/bash
# Interleaved whole-frame A/B (bench.py frame_ms: counter reset + cull passes + render) of
# library builds on one box:  scripts/frame_ab.sh <rounds> name=path.so ...  (default = in-tree)
set -u
R=$1; shift
for i in $(seq "$R"); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    [ "$lib" = default ] && lib=raytracinginonesemester_amd/lib/librt_mi355x.so
    RT_MI355X_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/fab.log 2>&1 || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/fab.log').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frame_ms'], d['parity']['ppm_identical'])"
  done
done
