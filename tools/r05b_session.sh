# round-5 session B: the split combine (every GPU test), its A/B with 1024
# eval_g threads, eval_g phase cuts
set -o pipefail
mkdir -p gpurun_out/r05_b
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05_b/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 tools/ab_env.sh r05b_ab "-" "MOCOHIP_IVG_THREADS=1024" > gpurun_out/r05_b/ab.log 2>&1 || exit $?
timeout -k 10 600 tools/ivg_cut.sh r05b > gpurun_out/r05_b/cut.log 2>&1
