set -o pipefail
mkdir -p gpurun_out/r06_d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "kernel_variants or combine_variants or assembly_bit_exact or generated_excitation" > gpurun_out/r06_d/pytest_variants.log 2>&1 || exit $?
timeout -k 10 500 tools/ab_env.sh r06_d_ab "-" > gpurun_out/r06_d/ab.log 2>&1 || exit $?
timeout -k 10 300 python tools/config3_ab.py 400 "MOCOHIP_DBASE=1;MOCOHIP_DBASE=0" > gpurun_out/r06_d/config3_ab.jsonl 2> gpurun_out/r06_d/config3_ab.err || exit $?
echo done
