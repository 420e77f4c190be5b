# round-5 session E1: every GPU test (eval_g's base-slot kernel and its
# bit-identity variant), smoke, the headline with / without the base slots,
# a world-1 mesh line (the one-GPU host-inclusive reference fixed)
set -o pipefail
mkdir -p gpurun_out/r05_e
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05_e/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_e/smoke.log 2>&1 || exit $?
timeout -k 10 400 tools/ab_env.sh r05e_ab "-" "MOCOHIP_IVG_BASE=0" > gpurun_out/r05_e/ab.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --multi mesh --steps 2000 --warmup 1000 --no-cpu-baseline --sweep 8 \
    > gpurun_out/r05_e/mesh_world1.json 2> gpurun_out/r05_e/mesh_world1.err
