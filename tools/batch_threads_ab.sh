#!/bin/bash
# Batched throughput (8 NLPs, gait N=200) over k_interval workgroup size x
# group-results source (global memory / LDS).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/batch_threads
mkdir -p "$OUT"
cd "$ROOT"
for th in 1024 512 256; do
  for gm in 1 0; do
    MOCOHIP_IV_THREADS=$th MOCOHIP_BATCH_GM=$gm timeout -k 10 300 python bench.py --batch-only \
        --steps 1000 --warmup 500 --mode fused > "$OUT/t${th}_gm${gm}.json" 2>> "$OUT/err.log"
    echo "threads $th gm $gm: $(python -c "import json;d=json.load(open('$OUT/t${th}_gm${gm}.json'));print(d['value'], d['batched']['value'])")"
  done
done
