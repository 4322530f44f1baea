set -u
mkdir -p gpurun_out
for t in 1.0 0.9 0.75 0.5 0.25 1.0; do
timeout -k 10 200 python scripts/bimodal_probe.py --trials 2 --blocks 2 --steps 200 --heavy-off-trials 0 --tune prepass_gate=$t > gpurun_out/t35_$t.log 2>&1 || exit 1
grep -v amdgpu gpurun_out/t35_$t.log | cut -c1-200
done
