#!/bin/bash
# A/B of kernel-variant environment settings on the headline bench line
# (gait10dof18musc N=200, forward FD, separate step, --single-mode): each
# setting's line twice, interleaved on the same box.
#   usage (repo root, through gpurun): tools/ab_env.sh <tag> "<ENV=V ...>" "<ENV=V ...>" ...
#   ("-" = the defaults)
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
    i=0
    for setting in "$@"; do
        envs=()
        [ "$setting" != "-" ] && read -r -a envs <<< "$setting"
        env "${envs[@]}" timeout -k 10 200 python3 "$ROOT/bench.py" --single-mode --no-cpu-baseline \
            > "$OUT/bench_${i}_$rep.log" 2>&1
        echo "$setting" > "$OUT/setting_$i.txt"
        i=$((i + 1))
    done
done
python3 - "$OUT" <<'PY' | tee "$OUT/summary.txt"
import glob, json, os, sys
out = sys.argv[1]
for f in sorted(glob.glob(os.path.join(out, "setting_*.txt"))):
    i = f.rsplit("_", 1)[1].split(".")[0]
    s = open(f).read().strip()
    for rep in (1, 2):
        lines = [l for l in open(os.path.join(out, f"bench_{i}_{rep}.log")) if l.startswith("{")]
        if not lines:
            print(f"[{s}] rep={rep}: no line"); continue
        d = json.loads(lines[-1]); r = d["roofline"]
        print(f"[{s}] rep={rep} calls/s {d['value']:.0f} ms/step {d['ms_per_step']:.5f} "
              f"k_interval {1e3 * r['kernel_ms']:.2f} us k_groups {1e3 * r['other_kernel']['kernel_ms']:.2f} us "
              f"eval_g {r.get('eval_g_stage_ms')}")
PY
