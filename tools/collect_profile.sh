#!/bin/bash
# Copy the judged parts of a GPU session (tools/gpu_session.sh <tag>) from
# gpurun_out/ into profiles/<dest>/: rocprofv3 kernel stats, the per-kernel
# PMC summary, the bench JSON lines and the host description.
#   usage: tools/collect_profile.sh <tag> <dest>
set -e
TAG=$1
DEST=profiles/$2
mkdir -p "$DEST"
P=gpurun_out/prof_$TAG
for d in trace_fused trace_separate; do
    [ -f "$P/$d/run_kernel_stats.csv" ] && cp "$P/$d/run_kernel_stats.csv" "$DEST/${d}_kernel_stats.csv"
done
python tools/kstats.py "$P" > "$DEST/summary.txt"
grep -h '^{' "$P"/*.log > "$DEST/bench_lines_under_profiler.jsonl" || true
[ -f "gpurun_out/$TAG/bench.json" ] && cp "gpurun_out/$TAG/bench.json" "$DEST/bench.json"
if [ -f "$P/pmc.json" ]; then
    cp "$P/pmc.json" "$DEST/pmc.json"
    python - "$DEST/pmc.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
d["source"] = sys.argv[1]
json.dump(d, open("profiles/pmc_current.json", "w"), indent=1)
PY
fi
[ -f "gpurun_out/$TAG/driver.json" ] && cp "gpurun_out/$TAG/driver.json" "$DEST/driver.json"
[ -f "gpurun_out/$TAG/host.txt" ] && head -20 "gpurun_out/$TAG/host.txt" > "$DEST/host.txt"
ls "$DEST"
