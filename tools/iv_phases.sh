#!/bin/bash
# Diagnostic: where k_interval's time goes; k_role (MOCOHIP_ROLES=1) whole
# for the A/B.  The bench's fused step under a
# rocprofv3 kernel trace with k_interval cut after staging (1), after the
# combine (2), after the quotients (3), after the g rows (4), with the
# assembly's stores alone (5) or its loads and arithmetic alone (6), and
# whole (0) -- MOCOHIP_IV_DEBUG_STOP; results of the cut runs are incomplete
# by design, only their durations are read.
#   usage (from the repo root, through gpurun): tools/iv_phases.sh <tag> [N]
set -e
TAG=${1:-phases}
N=${2:-200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/phases_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# the Jacobian through k_interval whole, without the assembly-word prefetch
MOCOHIP_IV_PF=0 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/noroles" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline \
    --single-mode --mode fused --intervals "$N" > "$OUT/noroles.log" 2>&1
for t in 256 c0; do
    (
    export MOCOHIP_ROLES=1
    if [ "$t" = c0 ]; then export MOCOHIP_ROLE_COUPLE=0; else export MOCOHIP_ROLE_THREADS=$t; fi
    timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/roles$t" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline \
        --single-mode --mode fused --intervals "$N" > "$OUT/roles$t.log" 2>&1
    )
done
for s in 0 7 1 2 3 4 5 6; do
    MOCOHIP_IV_DEBUG_STOP=$s timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$OUT/stop$s" -o run -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline \
        --single-mode --mode fused --intervals "$N" > "$OUT/stop$s.log" 2>&1
done
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt"
echo "phases done: $OUT"
