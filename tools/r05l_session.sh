# round-5 session L: the headline with the kernel arguments forced into
# device memory / host memory (HIP_FORCE_DEV_KERNARG), against the default
set -o pipefail
mkdir -p gpurun_out/r05_l
timeout -k 10 600 tools/ab_env.sh r05l_ab "-" "HIP_FORCE_DEV_KERNARG=1" "HIP_FORCE_DEV_KERNARG=0" \
    > gpurun_out/r05_l/ab.log 2>&1
