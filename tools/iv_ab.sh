#!/bin/bash
# A/B of k_interval variants (env at mh_create): kernel trace of the bench's
# fused step at N=200 and N=400, plus the bench headline and batch lines.
#   usage (repo root, through gpurun): tools/iv_ab.sh <tag> "<VAR=val ...>" ...
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ab_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for V in "$@"; do
    for N in 200 400; do
        env $V timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$OUT/v${i}_n$N" -o run -- python3 "$ROOT/bench.py" --steps 100 --warmup 20 --no-cpu-baseline \
            --single-mode --mode fused --intervals "$N" > "$OUT/v${i}_n$N.log" 2>&1
    done
    env $V timeout -k 10 300 python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/v${i}_bench.json" 2> "$OUT/v${i}_bench.err"
    echo "$i: $V" >> "$OUT/variants.txt"
    i=$((i+1))
done
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt" || true
echo "ab done: $OUT"
