# round-5 session H: every GPU test and the headline / configs[3] lines with
# the constant pool read through the constant address space (scalar loads),
# against session G's tree (profiles/r05_g)
set -o pipefail
TAG=r05_h
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 tools/ab_env.sh r05h_ab "-" "MOCOHIP_IVG_BASE=1" > gpurun_out/$TAG/ab.log 2>&1 || exit $?
timeout -k 10 200 python tools/config3_ab.py 400 "MOCOHIP_IVG_BASE=1;MOCOHIP_IVG_BASE=1" \
    > gpurun_out/$TAG/config3.jsonl 2> gpurun_out/$TAG/config3.err || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$ROOT/gpurun_out/prof_$TAG/trace_separate" -o run \
    -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --single-mode --mode separate \
    > "$ROOT/gpurun_out/prof_$TAG/trace_separate.log" 2>&1 )
