# round-5 session M: every GPU test; the headline with eval_g's task records
# in the kernel arguments against the task table (MOCOHIP_GROUPS_KR=0)
set -o pipefail
TAG=r05_m
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 tools/ab_env.sh r05m_ab "-" "MOCOHIP_GROUPS_KR=0" > gpurun_out/$TAG/ab.log 2>&1
