set -u
mkdir -p gpurun_out/final
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/final/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -5 gpurun_out/final/$tag.log; exit 1; }
  echo "$tag $(python scripts/bench_line.py gpurun_out/final/$tag.log)"
}
run c3_driver --gpus 1 --steps 20 --warmup 5
run c3_default
run c3b --config c3b --no-cpu-baseline
run c5 --config c5 --steps 20 --no-cpu-baseline
run c2 --config c2 --steps 200 --warmup 10
run c1 --config c1 --steps 200 --warmup 10 --no-cpu-baseline
bash scripts/prof_pmc.sh r05_c3b c3b 10 > gpurun_out/final/prof_c3b.log 2>&1; cat gpurun_out/final/prof_c3b.log
