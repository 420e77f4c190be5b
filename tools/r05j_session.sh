# round-5 session J: every GPU test; configs[3] with / without the XCD order
# of the split path's combine and transcription blocks; its trace and FETCH /
# WRITE passes; the headline line
set -o pipefail
TAG=r05_j
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python tools/config3_ab.py 400 "MOCOHIP_IV_XCD=1;MOCOHIP_IV_XCD=0;MOCOHIP_IV_XCD=1;MOCOHIP_IV_XCD=0" \
    > gpurun_out/$TAG/config3_ab.jsonl 2> gpurun_out/$TAG/config3_ab.err || exit $?
timeout -k 10 400 bash tools/prof_config3.sh > gpurun_out/$TAG/config3_prof.log 2>&1 || exit $?
timeout -k 10 300 tools/ab_env.sh r05j_ab "-" > gpurun_out/$TAG/ab.log 2>&1
