#!/bin/bash
# configs[3] (Rajagopal 80, N=400, generated back end) SQ counters per
# kernel: two separate rocprofv3 --pmc passes over a short run of
# tools/config3_ab.py, summarized per kernel.
#   usage (repo root, through gpurun): tools/config3_pmc.sh <tag>
set -e
TAG=${1:-c3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/config3_pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VMEM_WR" \
         "SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_IFETCH"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc$i" -o run -- \
        python3 "$ROOT/tools/config3_ab.py" 400 "MOCOHIP_ASM_CHUNK=8192" > "$OUT/pmc$i.log" 2>&1 || echo "pass $i failed"
done
python3 "$ROOT/tools/kstats.py" "$OUT" > "$OUT/summary.txt"
echo "done $OUT"
