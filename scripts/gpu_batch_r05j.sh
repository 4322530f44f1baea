set -u
for q in 4 8; do
for t in "overlap_frames=0" "overlap_frames=1"; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python scripts/bimodal_probe.py --trials 2 --blocks 2 --steps 200 --heavy-off-trials 0 --tune $t 2>/dev/null | sed "s/^/{\"hwq\": $q} /" | cut -c1-200 || exit 1
done; done
