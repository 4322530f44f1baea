set -u
for t in "heavy_frac=0.10" "heavy_frac=0.06" "heavy_frac=0.08" "heavy_frac=0.13" "heavy_frac=0.16" "heavy_frac=0.10"; do
timeout -k 10 200 python scripts/bimodal_probe.py --trials 2 --blocks 2 --steps 200 --heavy-off-trials 0 --tune $t 2>/dev/null | cut -c1-190 || exit 1
done
