# round-5 session P: every GPU test and the headline / configs[3] lines with
# the generated groups loading their inputs at their top (codegen), against
# the final-tree profile r05_o
set -o pipefail
TAG=r05_p
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 tools/ab_env.sh r05p_ab "-" "MOCOHIP_GROUPS_KR=0" > gpurun_out/$TAG/ab.log 2>&1 || exit $?
timeout -k 10 200 python tools/config3_ab.py 400 "MOCOHIP_IVG_BASE=1;MOCOHIP_IVG_BASE=1" \
    > gpurun_out/$TAG/config3.jsonl 2> gpurun_out/$TAG/config3.err
