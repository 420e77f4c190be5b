#!/bin/bash
# Batch A/B on one GPU box: the batch / Rajagopal GPU tests, then the batch
# throughput with the batched k_interval reading group results from global
# memory (default) and staging them in LDS, then the configs[3] line alone.
#   usage: tools/gpu_batch_ab.sh <tag>
set -e
TAG=${1:-batch}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
    -k "batch or rajagopal or wrapped" > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 python bench.py --batch-only --steps 1000 --warmup 500 > "$OUT/batch_gm.json" 2> "$OUT/bench.err"
cat "$OUT/batch_gm.json"
MOCOHIP_BATCH_GM=0 timeout -k 10 600 python bench.py --batch-only --steps 1000 --warmup 500 \
    > "$OUT/batch_lds.json" 2>> "$OUT/bench.err"
cat "$OUT/batch_lds.json"
timeout -k 10 600 python -c "
import json, sys
sys.argv = ['bench.py']
import bench
a = bench.parse(); a.steps = 2000; a.warmup = 1000
cx = bench.Ctx(a)
print(json.dumps(bench.config3_line(cx, a)))" > "$OUT/config3.json" 2>> "$OUT/bench.err"
cat "$OUT/config3.json"
echo "batch ab $TAG done"
