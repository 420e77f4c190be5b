# round-5 session Q (final tree): every GPU test, smoke, the round profile
# (traces, FETCH / WRITE / SQ passes), the default bench line over the PMC
# summary just collected, the configs[3] trace and FETCH / WRITE passes
set -o pipefail
TAG=r05_q
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$TAG gpurun_out/prof_$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || exit $?
timeout -k 10 450 bash tools/profile_gpu.sh "$TAG" > gpurun_out/$TAG/profile.log 2>&1 || exit $?
python - "gpurun_out/prof_$TAG/pmc.json" "$TAG" <<'PY' || exit $?
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = f"profiles/{sys.argv[2]}/pmc.json"
json.dump(d, open("profiles/pmc_current.json", "w"), indent=1)
PY
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit $?
timeout -k 10 250 bash tools/prof_config3.sh > gpurun_out/$TAG/config3_prof.log 2>&1
