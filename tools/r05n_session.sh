# round-5 session N: every GPU test (eval_g's task records as kernel
# arguments, eval_g's combine lanes before the staging barrier, the slot table
# staged in LDS as a variant); the headline default / MOCOHIP_GROUPS_KR=0 /
# MOCOHIP_IV_SLOTS_LDS=1
set -o pipefail
TAG=r05_n
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 tools/ab_env.sh r05n_ab "-" "MOCOHIP_GROUPS_KR=0" "MOCOHIP_IV_SLOTS_LDS=1" > gpurun_out/$TAG/ab.log 2>&1
