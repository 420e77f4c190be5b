#!/bin/bash
# A/B of the batch line (8 independent NLPs per GPU, one stream + host
# thread each) under HIP queue / launch settings.  Through gpurun, repo root.
set -e
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/batch_ab
mkdir -p "$OUT"
for B in 1 8; do
  for V in "X=0" "GPU_MAX_HW_QUEUES=8" "GPU_MAX_HW_QUEUES=16" "MOCOHIP_GRAPHS=1" "GPU_MAX_HW_QUEUES=16 MOCOHIP_GRAPHS=1"; do
    env $V timeout -k 10 120 python3 bench.py --batch-only --batch $B --steps 1000 --warmup 300 >> "$OUT/lines.jsonl" 2>> "$OUT/err.log"
  done
done
echo "batch ab done"
