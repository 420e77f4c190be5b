#!/bin/bash
# Diagnostic: eval_g's k_interval<D, 256> (stride-1 lanes: staging, the
# grid points' combine, the g rows) cut after each phase
# (MOCOHIP_IV_DEBUG_STOP: 7 = the launch floor, 1 = after staging, 2 = after
# the combine, 0 = whole) on the bench's SEPARATE step, kernel trace per cut;
# the cut runs' results are incomplete by design, only durations are read.
#   usage (from the repo root, through gpurun): tools/ivg_cut.sh <tag> [N]
set -e
TAG=${1:-gcut}
N=${2:-200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ivg_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for s in 0 7 1 2; do
    MOCOHIP_IV_DEBUG_STOP=$s timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/stop$s" -o run -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline \
        --single-mode --mode separate --intervals "$N" > "$OUT/stop$s.log" 2>&1
done
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt"
echo "ivg cut done: $OUT"
