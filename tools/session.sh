#!/bin/bash
# One GPU-box session, run through gpurun from the repo root:
#   tools/session.sh <tag> <step> [<step> ...]
# Output goes to gpurun_out/<tag>/ (profiles: gpurun_out/prof_<tag>/).  Every
# GPU step has its own time limit; the session stops at the first failed
# step (no retries: read what the step left in gpurun_out/<tag>/).
#
# steps
#   tests            every GPU test (pytest -m gpu)
#   params           the MocoParameter GPU tests alone
#   seeds            the global-seed GPU parity tests
#   parity:<expr>    tests/test_gpu_parity.py -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (bench.json)
#   bench20          bench.py --steps 20 --warmup 5
#   driver           the C++ host's calls/s (tools/driver_bench.py 200)
#   shard            bench.py --shard-model (the multi-GPU model's shard timings)
#   mesh1            bench.py --multi mesh at world 1 (the mesh path's code)
#   profile          tools/profile_gpu.sh (kernel trace + PMC passes, pmc.json)
#   pmcsrc           point pmc.json's "source" at profiles/<tag>/pmc.json
#   ifetch           instruction-fetch PMC pass of eval_g (separate mode)
#   counters         rocprofv3 --list-avail
#   config3          tools/prof_config3.sh (configs[3] kernel trace)
#   config3ab:<A;B>  tools/config3_ab.py 400 over env settings A, B, ...
#   ab:<E1,E2>       tools/ab_env.sh bench A/B over the env settings E1, E2
#   cut              tools/ivg_cut.sh (eval_g interval-kernel cuts)
#   gxcd             tools/gxcd_ab.sh (k_groups XCD mapping A/B)
# (round 5's eighteen tools/r05*_session.sh were these steps in fixed orders.)
set -o pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
PYT="python -u -m pytest --timeout 300 --timeout-method thread"
for step in "$@"; do
    echo "== $step"
    case $step in
    tests) timeout -k 10 900 $PYT tests -m gpu -q -x > "$OUT/pytest.log" 2>&1 || exit $? ;;
    params) timeout -k 10 300 $PYT tests/test_parameters.py -m gpu -v > "$OUT/pytest_params.log" 2>&1 || exit $? ;;
    seeds) timeout -k 10 300 $PYT tests/test_gpu_parity.py -x -q -k "global_seed or seeds" \
               > "$OUT/pytest_seeds.log" 2>&1 || exit $? ;;
    parity:*) timeout -k 10 900 $PYT tests/test_gpu_parity.py -v -k "${step#parity:}" \
               > "$OUT/pytest_parity.log" 2>&1 || exit $? ;;
    smoke) timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $? ;;
    bench) timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $? ;;
    bench20) timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench20.json" 2> "$OUT/bench20.err" \
               || exit $? ;;
    driver) timeout -k 10 120 python tools/driver_bench.py 200 > "$OUT/driver.json" 2> "$OUT/driver.err" || exit $? ;;
    shard) timeout -k 10 300 python bench.py --shard-model --steps 1000 --warmup 500 > "$OUT/shard_model.json" \
               2> "$OUT/shard_model.err" || exit $? ;;
    mesh1) timeout -k 10 300 python bench.py --multi mesh --steps 500 --warmup 200 --sweep 8 > "$OUT/mesh1.json" \
               2> "$OUT/mesh1.err" || exit $? ;;
    profile) timeout -k 10 900 bash tools/profile_gpu.sh "$TAG" > "$OUT/profile.log" 2>&1 || exit $? ;;
    pmcsrc) python - "gpurun_out/prof_$TAG/pmc.json" "$TAG" <<'PY' || exit $?
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = f"profiles/{sys.argv[2]}/pmc.json"
json.dump(d, open(sys.argv[1], "w"), indent=1)
PY
        ;;
    ifetch) mkdir -p "gpurun_out/prof_$TAG"
        ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_TC_INST_REQ SQC_ICACHE_MISSES \
            SQC_ICACHE_REQ SQ_WAVES TCC_HIT TCC_MISS --output-format csv -d "$ROOT/gpurun_out/prof_$TAG/pmc_ifetch_sep" \
            -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --single-mode --mode separate \
            > "$ROOT/gpurun_out/prof_$TAG/pmc_ifetch_sep.log" 2>&1 ) || exit $? ;;
    counters) ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --list-avail ) > "$OUT/counters.txt" 2>&1 \
               || exit $? ;;
    config3) timeout -k 10 400 bash tools/prof_config3.sh > "$OUT/config3_prof.log" 2>&1 || exit $? ;;
    config3ab:*) timeout -k 10 400 python tools/config3_ab.py 400 "${step#config3ab:}" > "$OUT/config3_ab.jsonl" \
               2> "$OUT/config3_ab.err" || exit $? ;;
    ab:*) IFS=, read -r -a envs <<< "${step#ab:}"
        timeout -k 10 600 tools/ab_env.sh "${TAG}_ab" "-" "${envs[@]}" > "$OUT/ab.log" 2>&1 || exit $? ;;
    cut) timeout -k 10 600 tools/ivg_cut.sh "$TAG" > "$OUT/cut.log" 2>&1 || exit $? ;;
    gxcd) timeout -k 10 900 tools/gxcd_ab.sh "${TAG}_gxcd" > "$OUT/gxcd.log" 2>&1 || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
    echo "step $step ok"
done
echo "session $TAG done"
