#!/bin/bash
# configs[3] (Rajagopal 80, generic interpreter) profile: kernel trace and
# FETCH_SIZE / WRITE_SIZE passes over a short N=400 run of tools/config3_ab.py.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_config3
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/tools/config3_ab.py" 400 "MOCOHIP_EXC_LANES=1" \
    > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$ROOT/tools/config3_ab.py" 400 "MOCOHIP_EXC_LANES=1" \
    > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$ROOT/tools/config3_ab.py" 400 "MOCOHIP_EXC_LANES=1" \
    > "$OUT/write.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU --output-format csv -d "$OUT/sq" -o run -- python3 "$ROOT/tools/config3_ab.py" 400 "MOCOHIP_EXC_LANES=1" \
    > "$OUT/sq.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/tcc" -o run -- python3 "$ROOT/tools/config3_ab.py" 400 "MOCOHIP_EXC_LANES=1" \
    > "$OUT/tcc.log" 2>&1
python3 - "$OUT" <<'PY'
import collections, csv, glob, os, sys
out = sys.argv[1]
for cnt, d in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write"), ("SQ_WAVES", "sq"), ("SQ_WAVE_CYCLES", "sq"),
               ("SQ_BUSY_CYCLES", "sq"), ("SQ_WAIT_ANY", "sq"), ("SQ_INSTS_VALU", "sq"), ("SQ_INSTS_VMEM_RD", "sq"),
               ("SQ_INSTS_VMEM_WR", "sq"), ("SQ_INSTS_SALU", "sq"), ("TCC_HIT_sum", "tcc"), ("TCC_MISS_sum", "tcc")):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == cnt:
                acc[r["Kernel_Name"].split("(")[0][:60]].append(float(r["Counter_Value"]))
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1]))[:6]:
        print(cnt, k, "launches", len(v), "mean" + (" KiB" if cnt.endswith("SIZE") else ""), round(sum(v) / len(v), 1))
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True):
    rows = list(csv.DictReader(open(f)))[:6]
    for r in rows:
        print("TRACE", r["Name"][:60], r["Calls"], r["AverageNs"])
PY
