# c3 A/B of pair submission over pipeline depths: PAIR_RUNS="p:depth ..." (bench.py --no-extras).
set -u
mkdir -p gpurun_out
for i in 1 2; do
  for pd in ${PAIR_RUNS:-0:3 1:4 1:6 1:8}; do
    p=${pd%%:*}; d=${pd##*:}
    timeout -k 10 240 python bench.py --pair $p --depth $d --no-extras --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/pair_ab_p${p}_d${d}_$i.log 2>&1 || { tail -20 gpurun_out/pair_ab_p${p}_d${d}_$i.log; exit 1; }
    echo "pair=$p depth=$d run $i"; python scripts/bench_line.py gpurun_out/pair_ab_p${p}_d${d}_$i.log
  done
done
