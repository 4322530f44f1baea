#!/bin/bash
# Renderer A/B (bench.py, P6 to host), separate processes, interleaved: kernel events recorded by
# the dispatch (default) / by separate event records (RT_EXP_EVENT_RECORD).
run() {
  env "$@" python bench.py --no-extras --no-cpu-baseline --steps 300 --warmup 20 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$*', d['ms_per_step'], d['timing']['kernel_ms'], d['parity']['timed_step_ppm_identical'])"
}
for i in 1 2 3; do
  run X=default
  run RT_EXP_EVENT_RECORD=1
done
