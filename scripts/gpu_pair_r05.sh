# Round 5: two frames per render launch (rt_renderer_submit_pair) -- parity, then the c3 A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pair_tests.log 2>&1 || { tail -40 gpurun_out/pair_tests.log; exit 1; }
tail -3 gpurun_out/pair_tests.log
for i in 1 2; do
  for p in 0 1; do
    timeout -k 10 240 python bench.py --pair $p --no-extras --no-cpu-baseline ${BENCH_ARGS:-} \
      > gpurun_out/pair_ab_p${p}_$i.log 2>&1 || { tail -20 gpurun_out/pair_ab_p${p}_$i.log; exit 1; }
    echo "pair=$p run $i"; python scripts/bench_line.py gpurun_out/pair_ab_p${p}_$i.log
  done
done
