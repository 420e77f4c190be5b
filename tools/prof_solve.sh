#!/bin/bash
# Kernel trace of the configs[2] solve (muscle-driven MocoTrack N=200) on the
# device linear algebra, plus a Python profile of the host side of the same
# solve.  Output: gpurun_out/<tag>/...
set -e
TAG=${1:-solve}
N=${2:-200}   # or inverse125
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_solve" -o run \
    -- python3 "$ROOT/tools/solve_track.py" "$N" device > "$OUT/trace_solve.log" 2>&1
python3 "$ROOT/tools/kstats.py" "$OUT/trace_solve" > "$OUT/trace_solve_stats.txt" 2>&1
cd "$ROOT"
timeout -k 10 300 python3 -m cProfile -s tottime tools/solve_track.py "$N" device > "$OUT/cprofile.txt" 2>&1
echo "solve profile done: $OUT"
