#!/bin/bash
# configs[3] heavy-group diagnostic: what a Rajagopal 80 mass / bias part
# waits on.  tools/group_timing.py with only group G launched (default 1,
# mass_0), under separate rocprofv3 --pmc passes (instruction fetch, issue
# and wait counters; scalar and instruction cache), plus a kernel trace.
#   usage (repo root, through gpurun): tools/raja_pmc.sh <tag> [N] [G]
set -e
TAG=${1:-raja}
N=${2:-400}
G=${3:-1}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/raja_pmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/tools/group_timing.py" rajagopal80 "$N" "$G" > "$OUT/trace.log" 2>&1
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES" \
         "SQ_IFETCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS" \
         "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" \
         "SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc$i" -o run -- \
        python3 "$ROOT/tools/group_timing.py" rajagopal80 "$N" "$G" > "$OUT/pmc$i.log" 2>&1 || echo "pass $i failed: $P"
done
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(out, "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:70]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    if "groups" not in k:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} launches {len(v):4d} mean {sum(v) / len(v):16.1f}")
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in list(csv.DictReader(open(f)))[:6]:
        print("TRACE", r["Name"][:70], r["Calls"], r["AverageNs"])
PY
