#!/bin/bash
# Kernel trace of the batched path (mh_batch, 8 NLPs, fused steps) with the
# batched k_interval reading group results from global memory (gm) and
# staging them in LDS (lds), and of one NLP (single), for the per-launch
# durations of kb_groups / kb_interval against k_groups / k_interval.
set -e
TAG=${1:-batch}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py --batch-only --steps 200 --warmup 50 --mode fused"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gm" -o run \
    -- python3 $B > "$OUT/gm.log" 2>&1
MOCOHIP_BATCH_GM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/lds" -o run \
    -- python3 $B > "$OUT/lds.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/single" -o run \
    -- python3 $ROOT/bench.py --steps 200 --warmup 50 --no-cpu-baseline --single-mode --mode fused \
    > "$OUT/single.log" 2>&1
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
