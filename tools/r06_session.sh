#!/bin/bash
# Round-6 GPU session (run through gpurun from the repo root):
#   tools/r06_session.sh <tag> <step> [<step> ...]
# steps: seeds (global-seed GPU parity), bench (default line), shard (the
# multi-GPU model's shard timings), mesh1 (the --multi mesh code path at
# world 1), tests (every GPU test), smoke, profile (tools/profile_gpu.sh),
# config3 (tools/prof_config3.sh).  Every step has its own time limit; the
# session stops at the first failure.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() { echo "== $1"; }
for step in "$@"; do
    case $step in
    seeds) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "global_seed or seeds" \
               --timeout 120 --timeout-method thread > "$OUT/pytest_seeds.log" 2>&1 || exit $? ;;
    tests) timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
               > "$OUT/pytest.log" 2>&1 || exit $? ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $? ;;
    bench) timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $? ;;
    bench20) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench20.json" 2> "$OUT/bench20.err" || exit $? ;;
    shard) timeout -k 10 300 python bench.py --shard-model --steps 1000 --warmup 500 > "$OUT/shard_model.json" \
               2> "$OUT/shard_model.err" || exit $? ;;
    mesh1) timeout -k 10 300 python bench.py --multi mesh --steps 500 --warmup 200 --sweep 8 > "$OUT/mesh1.json" \
               2> "$OUT/mesh1.err" || exit $? ;;
    profile) timeout -k 10 900 bash tools/profile_gpu.sh "$TAG" > "$OUT/profile.log" 2>&1 || exit $? ;;
    config3) timeout -k 10 300 bash tools/prof_config3.sh > "$OUT/config3_prof.log" 2>&1 || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
    echo "step $step ok"
done
echo "session $TAG done"
