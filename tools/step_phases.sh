#!/bin/bash
# Diagnostic: the headline's separate-mode step (eval_g then eval_jac_g, gait
# N=200, forward FD) under a rocprofv3 kernel trace, whole (stop 0) and with
# both interval kernels cut after their launch (7), staging (1), combine (2)
# and g rows (4) -- MOCOHIP_IV_DEBUG_STOP; results of cut runs are incomplete
# by design, only durations are read.  tools/step_stats.py splits each
# kernel by workgroup size (eval_g's interval blocks are 256 threads, the
# Jacobian's 1024) and reports the per-step gaps.
#   usage (repo root, through gpurun): tools/step_phases.sh <tag> [N]
set -e
TAG=${1:-step}
N=${2:-200}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/step_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for s in 0 7 1 2 4; do
    MOCOHIP_IV_DEBUG_STOP=$s timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv \
        -d "$OUT/stop$s" -o run -- python3 "$ROOT/bench.py" --steps 200 --warmup 20 --no-cpu-baseline \
        --single-mode --mode separate --intervals "$N" > "$OUT/stop$s.log" 2>&1
done
python3 "$ROOT/tools/step_stats.py" "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
