#!/bin/bash
# eval_g through the task kernels (default) vs the one-lane generated kernel
# (MOCOHIP_G_LANE=1): the default bench line, single mode, both ways; and the
# bit-identity of the two eval_g paths on the bench workload.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/g_lane
mkdir -p "$OUT"
cd "$ROOT"
for gl in 0 1; do
    MOCOHIP_G_LANE=$gl timeout -k 10 300 python bench.py --single-mode --no-cpu-baseline \
        > "$OUT/gl$gl.json" 2>> "$OUT/err.log"
    echo "g_lane $gl: $(python -c "import json;d=json.load(open('$OUT/gl$gl.json'));print(d['value'], d['roofline'].get('eval_g_stage_ms'))")"
done
timeout -k 10 300 python - <<'PY' > "$OUT/identity.txt" 2>&1
import os, numpy as np, sys
sys.path.insert(0, "opensim-moco_amd")
from mocohip import configs
from mocohip.solver import HipNLP
st = configs.gait10dof18musc(200)
rep = st.problem.create_rep()
a = HipNLP(rep, st.solver.options())
os.environ["MOCOHIP_G_LANE"] = "1"
b = HipNLP(rep, st.solver.options())
x = a.random_iterate(np.random.default_rng(3).uniform(-1, 1, a.n))
xm = a.initial_guess_from_bounds(); x[2:2 + a.NS * a.G] = xm[2:2 + a.NS * a.G]
ga, gb = a.eval_g(x), b.eval_g(x)
g2, _ = a.eval_g_jac_g(x)
print("bit-identical task vs lane eval_g:", np.array_equal(ga, gb, equal_nan=True), "max|d|", np.nanmax(np.abs(ga - gb)))
print("fused g == task eval_g:", np.array_equal(ga, g2, equal_nan=True))
PY
cat "$OUT/identity.txt"
