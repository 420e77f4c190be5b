# round-5 session C: every GPU test (k_interval's combine reverted, the
# split combine for large models, ABI v7, objective terms, sharded solve),
# configs[3] with / without the split combine, the headline with / without
# the XCD-ordered k_groups blocks, a world-1 mesh line
set -o pipefail
mkdir -p gpurun_out/r05_c
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05_c/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/config3_ab.py 400 "MOCOHIP_CSPLIT=1;MOCOHIP_CSPLIT=0;MOCOHIP_CSPLIT=1;MOCOHIP_CSPLIT=0" \
    > gpurun_out/r05_c/config3_ab.jsonl 2> gpurun_out/r05_c/config3_ab.err || exit $?
timeout -k 10 600 tools/ab_env.sh r05c_ab "-" "MOCOHIP_GROUPS_XCD=0" > gpurun_out/r05_c/ab.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --multi mesh --steps 2000 --warmup 1000 --no-cpu-baseline --sweep 8 \
    > gpurun_out/r05_c/mesh_world1.json 2> gpurun_out/r05_c/mesh_world1.err
