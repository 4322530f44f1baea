set -u
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 240 python bench.py ${BENCH_ARGS:-} > gpurun_out/t48_bench_$i.log 2>&1 || exit 1
  python scripts/bench_line.py gpurun_out/t48_bench_$i.log
done
