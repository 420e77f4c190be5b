# round-5 session F: every GPU test (the Jacobian lanes' computed slots in
# k_interval and k_combine_global, eval_g's global-memory base-slot kernel
# by default), the headline and configs[3] with / without the computed slots
set -o pipefail
mkdir -p gpurun_out/r05_f
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05_f/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 tools/ab_env.sh r05f_ab "-" "MOCOHIP_JSLOT=0" > gpurun_out/r05_f/ab.log 2>&1 || exit $?
timeout -k 10 400 python tools/config3_ab.py 400 "MOCOHIP_JSLOT=1;MOCOHIP_JSLOT=0;MOCOHIP_JSLOT=1;MOCOHIP_JSLOT=0" \
    > gpurun_out/r05_f/config3_ab.jsonl 2> gpurun_out/r05_f/config3_ab.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > "$GRAFT_REPO_ROOT/gpurun_out/r05_f/counters.txt" 2>&1
