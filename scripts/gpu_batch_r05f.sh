set -u
mkdir -p gpurun_out
for t in "cull_boxes=64" "cull_boxes=32" "cull_boxes=16" "cull_coverage=0"; do
timeout -k 10 200 python scripts/bimodal_probe.py --trials 2 --blocks 2 --steps 200 --heavy-off-trials 0 --tune $t > gpurun_out/t32_$t.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/t32_$t.log | cut -c1-175
done
