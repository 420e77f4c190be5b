# round-5 session G: every GPU test, configs[3] over eval_g's kernel variants,
# the round profile (traces, FETCH / WRITE / SQ passes, an instruction-fetch
# pass), the default bench line over the PMC summary just collected
set -o pipefail
TAG=r05_g
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 240 python tools/config3_ab.py 400 \
    "MOCOHIP_IVG_BASE=1;MOCOHIP_IVG_BASE=0;MOCOHIP_IVG_GM=1;MOCOHIP_IVG_BASE=1;MOCOHIP_IVG_BASE=0" \
    > gpurun_out/$TAG/config3_ab.jsonl 2> gpurun_out/$TAG/config3_ab.err || exit $?
timeout -k 10 500 bash tools/profile_gpu.sh "$TAG" > gpurun_out/$TAG/profile.log 2>&1 || exit $?
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_TC_INST_REQ SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_WAVES TCC_HIT TCC_MISS \
    --output-format csv -d "$ROOT/gpurun_out/prof_$TAG/pmc_ifetch_sep" -o run \
    -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --single-mode --mode separate \
    > "$ROOT/gpurun_out/prof_$TAG/pmc_ifetch_sep.log" 2>&1 ) || exit $?
python - "gpurun_out/prof_$TAG/pmc.json" "$TAG" <<'PY' || exit $?
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = f"profiles/{sys.argv[2]}/pmc.json"
json.dump(d, open("profiles/pmc_current.json", "w"), indent=1)
PY
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
