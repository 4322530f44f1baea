set -u
for r in 1 2; do for d in 2 3 4; do
  out=$(timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --no-extras --steps 200 --warmup 20 --depth $d 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('deliver_ms'), t.get('frame_latency_ms'), t.get('render_only_value'))") || exit 1
  echo "depth $d: ms_per_step,kernel_ms,deliver_ms,latency_ms,render_only= $out"
done; done
for d in 2 3; do
  out=$(timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-parity --no-extras --steps 20 --warmup 10 --depth $d 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); t=d['timing']; print(d['ms_per_step'], t['kernel_ms'], t.get('frame_latency_ms'))") || exit 1
  echo "driver-like 20 steps depth $d: $out"
done
