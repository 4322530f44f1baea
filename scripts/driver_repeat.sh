#!/bin/bash
# The driver's bench command repeated (full line, then without the secondary legs), same box.
set -u
for r in 1 2 3; do
  for extra in "" "--no-extras --no-cpu-baseline"; do
    out=$(timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 $extra 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['timing']; print(d['value'], d['ms_per_step'], t['kernel_ms'], t.get('prepass_ms'), t.get('frame_latency_ms'))") || exit 1
    echo "run $r [$extra]: value,ms_per_step,kernel_ms,prepass_ms,latency_ms= $out"
  done
done
