#!/bin/bash
# Round profile on one MI355X (run through gpurun from the repo root):
#   kernel trace + stats of the bench (fused and separate steps), then
#   separate PMC passes (TCC FETCH_SIZE / WRITE_SIZE cannot share a pass; SQ
#   counters alone), then the per-launch HBM traffic summary (pmc.json).
# Output: gpurun_out/prof_<tag>/...  tools/collect_profile.sh copies the
# summaries into profiles/.
set -e
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --steps 50 --warmup 5 --no-cpu-baseline --single-mode"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_fused" -o run \
    -- python3 $B --mode fused > "$OUT/trace_fused.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_separate" -o run \
    -- python3 $B --mode separate > "$OUT/trace_separate.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
    -- python3 $B --mode fused > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
    -- python3 $B --mode fused > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_sq" -o run \
    -- python3 $B --mode fused > "$OUT/pmc_sq.log" 2>&1
# the separate step: eval_g's own launches (k_interval<D, 256> and its
# k_groups) beside eval_jac_g's
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch_sep" -o run \
    -- python3 $B --mode separate > "$OUT/pmc_fetch_sep.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write_sep" -o run \
    -- python3 $B --mode separate > "$OUT/pmc_write_sep.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d "$OUT/pmc_sq_sep" -o run \
    -- python3 $B --mode separate > "$OUT/pmc_sq_sep.log" 2>&1
python3 "$ROOT/tools/pmc_summary.py" "$OUT" "N=200,fd=forward" "$OUT/pmc.json" > "$OUT/pmc_summary.log" 2>&1
echo "profile done: $OUT"
