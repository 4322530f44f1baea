# Big-scene pairs: parity, then the c5 A/B.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pair_tests_c5.log 2>&1 || { tail -40 gpurun_out/pair_tests_c5.log; exit 1; }
tail -1 gpurun_out/pair_tests_c5.log
for i in 1 2; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py --config c5 --steps 20 --pair $p --no-extras --no-cpu-baseline > gpurun_out/c5_pair${p}_$i.log 2>&1 \
      || { tail -20 gpurun_out/c5_pair${p}_$i.log; exit 1; }
    echo "c5 pair=$p run $i: $(python scripts/bench_line.py gpurun_out/c5_pair${p}_$i.log)"
  done
done
