#!/bin/bash
# One GPU-box session (run through gpurun from the repo root): GPU parity
# tests, smoke, the default bench line, then the round profile.  Every GPU
# step has its own time limit and the steps stop at the first failure.
#   usage: tools/gpu_session.sh <tag> [tests|bench|profile|all|final]
# final: tests, smoke, the profile, then the bench line reading the PMC
# summary just collected (profiles/pmc_current.json refreshed on the box;
# tools/collect_profile.sh makes the same copy here)
set -e
TAG=${1:-r01}
WHAT=${2:-all}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
(nproc; lscpu | head -20; rocm-smi --showproductname 2>/dev/null | head -20) > "$OUT/host.txt" 2>&1 || true
if [[ $WHAT == tests || $WHAT == all || $WHAT == final ]]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
if [[ $WHAT == bench || $WHAT == all ]]; then
    timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
    timeout -k 10 120 python tools/driver_bench.py 200 > "$OUT/driver.json" 2> "$OUT/driver.err"
fi
if [[ $WHAT == profile || $WHAT == all || $WHAT == final ]]; then
    timeout -k 10 900 bash tools/profile_gpu.sh "$TAG"
fi
if [[ $WHAT == final ]]; then
    python - "$ROOT/gpurun_out/prof_$TAG/pmc.json" "$TAG" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = f"profiles/{sys.argv[2]}/pmc.json"
json.dump(d, open("profiles/pmc_current.json", "w"), indent=1)
PY
    timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
fi
echo "session $TAG done"
