#!/bin/bash
# One GPU-box session: GPU parity tests, smoke, the default bench line, the
# k_interval phase cut and the round profile (kernel trace + PMC passes).
# Every GPU step has its own time limit; the script stops at the first failure.
#   usage: tools/gpu_round.sh <tag> [tests] [bench] [mesh] [phases] [profile]
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
(nproc; lscpu | head -20; rocm-smi --showproductname 2>/dev/null | head -20) > "$OUT/host.txt" 2>&1 || true
for what in "$@"; do
    case $what in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
            > "$OUT/pytest_gpu.log" 2>&1 || { tail -5 "$OUT/pytest_gpu.log"; exit 1; }
        tail -2 "$OUT/pytest_gpu.log"
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
        tail -2 "$OUT/smoke.log";;
    bench)
        timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
        timeout -k 10 120 python tools/driver_bench.py 200 > "$OUT/driver.json" 2> "$OUT/driver.err" || true;;
    mesh)
        timeout -k 10 300 python bench.py --multi mesh --steps 500 --warmup 200 > "$OUT/mesh.json" 2> "$OUT/mesh.err"
        tail -1 "$OUT/mesh.json";;
    phases)
        timeout -k 10 600 bash tools/iv_phases.sh "$TAG" 200;;
    profile)
        timeout -k 10 900 bash tools/profile_gpu.sh "$TAG";;
    esac
done
echo "session $TAG done"
