# round-5 session A: configs[4] detection parity, eval_g phase cuts, and the
# A/B of the XCD-ordered k_groups blocks (each step under its own limit)
set -o pipefail
mkdir -p gpurun_out/r05_a
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 300 --timeout-method thread \
    -k "sparsity_detection_agrees or config_at_full_size or (kernel_variants_bit_identical and GROUPS_XCD) or batch or pruned" \
    > gpurun_out/r05_a/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 tools/ivg_cut.sh r05a > gpurun_out/r05_a/cut.log 2>&1 || exit $?
timeout -k 10 900 tools/gxcd_ab.sh r05a_gxcd > gpurun_out/r05_a/gxcd.log 2>&1
