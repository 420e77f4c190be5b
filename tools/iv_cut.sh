#!/bin/bash
# Diagnostic: k_interval cut after each phase (MOCOHIP_IV_DEBUG_STOP, see
# tools/iv_phases.sh) on the bench's fused step, kernel trace per cut; the
# cut runs' results are incomplete by design, only durations are read.
#   usage (from the repo root, through gpurun): tools/iv_cut.sh <tag> [N]
set -e
TAG=${1:-cut}
N=${2:-200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/cut_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for s in 0 7 1 2 4 5 6; do
    MOCOHIP_IV_DEBUG_STOP=$s timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/stop$s" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline \
        --single-mode --mode fused --intervals "$N" > "$OUT/stop$s.log" 2>&1
done
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt"
echo "cut done: $OUT"
