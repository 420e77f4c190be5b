# round-5 session K: every GPU test; configs[3] with the LDS-staged combine
# (k_combine without the quotient path compiled in) against the global-memory
# combine; its trace and FETCH / WRITE passes with the default choice
set -o pipefail
TAG=r05_k
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/config3_ab.py 400 \
    "MOCOHIP_COMBINE=lds;MOCOHIP_COMBINE=global;MOCOHIP_COMBINE=lds;MOCOHIP_COMBINE=global" \
    > gpurun_out/$TAG/config3_ab.jsonl 2> gpurun_out/$TAG/config3_ab.err || exit $?
timeout -k 10 400 bash tools/prof_config3.sh > gpurun_out/$TAG/config3_prof.log 2>&1
