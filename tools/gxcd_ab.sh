#!/bin/bash
# A/B of the k_groups blocks in k_interval's XCD order (MOCOHIP_GROUPS_XCD,
# build_taskset groups_xcd) on the headline (gait10dof18musc N=200, forward FD):
# the bench line twice per setting, interleaved, then a FETCH_SIZE pass per
# setting (per-launch HBM reads of k_interval: the group results k_groups wrote
# on the same XCD can be served by that XCD's L2).
#   usage (repo root, through gpurun): tools/gxcd_ab.sh [tag]
set -e
TAG=${1:-gxcd}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
    for v in 0 1; do
        MOCOHIP_GROUPS_XCD=$v timeout -k 10 200 python3 "$ROOT/bench.py" --single-mode --no-cpu-baseline \
            > "$OUT/bench_xcd${v}_$rep.log" 2>&1
    done
done
for v in 0 1; do
    MOCOHIP_GROUPS_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch$v" -o run \
        -- python3 "$ROOT/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --single-mode --mode fused \
        > "$OUT/fetch$v.log" 2>&1
done
python3 - "$OUT" <<'PY' | tee "$OUT/summary.txt"
import collections, csv, glob, json, os, sys
out = sys.argv[1]
for v in (0, 1):
    for rep in (1, 2):
        d = json.loads([l for l in open(os.path.join(out, f"bench_xcd{v}_{rep}.log")) if l.startswith("{")][-1])
        r = d["roofline"]
        print(f"xcd={v} rep={rep} calls/s {d['value']:.0f} fused {d.get('value_fused', 0):.0f} "
              f"k_interval {1e3 * r['kernel_ms']:.2f} us")
for v in (0, 1):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, f"fetch{v}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row["Kernel_Name"].split("(")[0].replace("void ", "")[:40]].append(float(row["Counter_Value"]))
    for k, vals in sorted(acc.items()):
        # FETCH_SIZE is in KiB and reports half of coalesced streaming reads on gfx950 (x2)
        print(f"xcd={v} {k:40s} launches {len(vals):5d} FETCH_SIZE x2 {2 * sum(vals) / len(vals) / 1024:8.2f} MB")
PY
