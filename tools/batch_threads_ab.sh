#!/bin/bash
# Batched throughput (8 NLPs, gait N=200, fused steps) over the k_interval
# workgroup size x group-results source (global memory / LDS), and the
# kb_groups register budget (MOCOHIP_BATCH_WAVES=3).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/batch_threads
mkdir -p "$OUT"
cd "$ROOT"
run() {  # tag, env...
    local tag=$1; shift
    env "$@" timeout -k 10 300 python bench.py --batch-only --steps 1000 --warmup 500 --mode fused \
        > "$OUT/$tag.json" 2>> "$OUT/err.log"
    echo "$tag: $(python -c "import json;d=json.load(open('$OUT/$tag.json'));print(d['value'], d['batched']['value'])")"
}
for th in 1024 512 256; do
  for gm in 1 0; do
    run "t${th}_gm${gm}" MOCOHIP_IV_THREADS=$th MOCOHIP_BATCH_GM=$gm
  done
done
run t1024_gm0_w3 MOCOHIP_IV_THREADS=1024 MOCOHIP_BATCH_GM=0 MOCOHIP_BATCH_WAVES=3
run t256_gm1_w3 MOCOHIP_IV_THREADS=256 MOCOHIP_BATCH_GM=1 MOCOHIP_BATCH_WAVES=3
