# c3 pair-mode knob A/B (bench.py --no-extras): VARIANTS is a list of "tag|bench args".
set -u
mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS}"
for i in 1 2; do
  for v in "${VS[@]}"; do
    tag=${v%%|*}; args=${v#*|}
    timeout -k 10 240 python bench.py --no-extras --no-cpu-baseline $args > gpurun_out/pk_${tag}_$i.log 2>&1 \
      || { tail -20 gpurun_out/pk_${tag}_$i.log; exit 1; }
    echo "$tag run $i: $(python scripts/bench_line.py gpurun_out/pk_${tag}_$i.log)"
  done
done
