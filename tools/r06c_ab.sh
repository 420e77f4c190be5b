set -o pipefail
mkdir -p gpurun_out/r06_c
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "kernel_variants and (variant18 or variant19 or variant20)" > gpurun_out/r06_c/pytest_variants.log 2>&1 || exit $?
timeout -k 10 700 tools/ab_env.sh r06_c_ab "-" "MOCOHIP_DBASE=1" "MOCOHIP_NT_STORES=1" "MOCOHIP_DBASE=1 MOCOHIP_NT_STORES=1" > gpurun_out/r06_c/ab.log 2>&1 || exit $?
timeout -k 10 400 python tools/config3_ab.py 400 "MOCOHIP_DBASE=0;MOCOHIP_DBASE=1;MOCOHIP_NT_STORES=1;MOCOHIP_ASM_CHUNK=2048;MOCOHIP_ASM_CHUNK=4096;MOCOHIP_ASM_CHUNK=2048,MOCOHIP_DBASE=1,MOCOHIP_NT_STORES=1;MOCOHIP_DBASE=0" > gpurun_out/r06_c/config3_ab.jsonl 2> gpurun_out/r06_c/config3_ab.err || exit $?
echo done
