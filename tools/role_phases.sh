#!/bin/bash
# Diagnostic: where k_role's time goes.  The bench's fused step under a
# rocprofv3 kernel trace with k_role cut after staging (1), after the
# combine (2), after the quotients + exchange (3), after its g rows (4), and
# whole (0) -- MOCOHIP_IV_DEBUG_STOP; cut runs give incomplete results by
# design, only their durations are read.
#   usage (from the repo root, through gpurun): tools/role_phases.sh <tag> [N] [threads]
set -e
TAG=${1:-rphases}
N=${2:-200}
TH=${3:-256}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/rphases_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for s in 0 1 2 3 4; do
    MOCOHIP_ROLE_THREADS=$TH MOCOHIP_IV_DEBUG_STOP=$s timeout -k 10 180 rocprofv3 --kernel-trace --stats \
        --output-format csv -d "$OUT/stop$s" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 \
        --no-cpu-baseline --single-mode --mode fused --intervals "$N" > "$OUT/stop$s.log" 2>&1
done
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt"
echo "role phases done: $OUT"
