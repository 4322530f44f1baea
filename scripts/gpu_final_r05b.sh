# Round 5, after pair frames: the c3 bench lines (driver command, default, single-frame) and the
# rocprofv3 kernel stats of the default c3 bench command.
set -u
mkdir -p gpurun_out/final2
run() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/final2/$tag.log 2>&1 || { echo "$tag failed rc=$?"; tail -5 gpurun_out/final2/$tag.log; exit 1; }
  echo "$tag $(python scripts/bench_line.py gpurun_out/final2/$tag.log)"
}
run c3_driver --gpus 1 --steps 20 --warmup 5
run c3_default
run c3_single --pair 0
run c3_driver_b --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/final2/prof" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-extras --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/final2/prof_bench.log" 2>&1 \
  || { echo "prof failed"; exit 1; }
echo "prof $(python3 $GRAFT_REPO_ROOT/scripts/bench_line.py $GRAFT_REPO_ROOT/gpurun_out/final2/prof_bench.log)"
