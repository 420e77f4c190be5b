# round-5 session E2: every GPU test (k_groups without the role-table load
# for eval_g, the global-memory base-slot variant), the headline with / without
# MOCOHIP_IVG_GM, the round profile (kernel traces, FETCH / WRITE / SQ passes
# of the fused and separate steps) and the default bench line over the PMC
# summary just collected
set -o pipefail
TAG=${1:-r05_e}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest2.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 tools/ab_env.sh r05e2_ab "-" "MOCOHIP_IVG_GM=1" > gpurun_out/$TAG/ab2.log 2>&1 || exit $?
timeout -k 10 600 bash tools/profile_gpu.sh "$TAG" > gpurun_out/$TAG/profile.log 2>&1 || exit $?
python - "gpurun_out/prof_$TAG/pmc.json" "$TAG" <<'PY' || exit $?
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = f"profiles/{sys.argv[2]}/pmc.json"
json.dump(d, open("profiles/pmc_current.json", "w"), indent=1)
PY
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
