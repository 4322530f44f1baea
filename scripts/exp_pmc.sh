set -e
timeout -k 10 60 build/micro/valu_rate > gpurun_out/valu_rate.log 2>&1
bash scripts/pmc_case.sh def full > gpurun_out/pmc_def.log 2>&1
RT_MI355X_LIB=$GRAFT_REPO_ROOT/build/variants/pkwl/librt_mi355x.so bash scripts/pmc_case.sh pkwl full > gpurun_out/pmc_pkwl.log 2>&1
