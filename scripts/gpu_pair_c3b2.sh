# Bounce pairs without reserved slots: parity, c3b A/B, then the c3b and c3 default lines.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pair.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pair_tests_c3b2.log 2>&1 || { tail -40 gpurun_out/pair_tests_c3b2.log; exit 1; }
tail -1 gpurun_out/pair_tests_c3b2.log
for i in 1 2; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py --config c3b --pair $p --no-extras --no-cpu-baseline > gpurun_out/c3b2_pair${p}_$i.log 2>&1 \
      || { tail -20 gpurun_out/c3b2_pair${p}_$i.log; exit 1; }
    echo "c3b pair=$p run $i: $(python scripts/bench_line.py gpurun_out/c3b2_pair${p}_$i.log)"
  done
done
timeout -k 10 500 python bench.py --config c3b --no-cpu-baseline > gpurun_out/c3b2_default.log 2>&1 || { tail -20 gpurun_out/c3b2_default.log; exit 1; }
echo "c3b default: $(python scripts/bench_line.py gpurun_out/c3b2_default.log)"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c3_driver_after_c3b.log 2>&1 || { tail -20 gpurun_out/c3_driver_after_c3b.log; exit 1; }
echo "c3 driver: $(python scripts/bench_line.py gpurun_out/c3_driver_after_c3b.log)"
