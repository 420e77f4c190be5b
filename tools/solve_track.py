"""Wall-clock of the configs[2] solve (muscle-driven MocoTrack
gait10dof18musc, MocoTrack's settings) on the GPU path with the device or
host linear algebra: one JSON line per run."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "opensim-moco_amd"))
from mocohip import configs  # noqa: E402
from mocohip.ipm import IpmOptions, solve_ipm  # noqa: E402

# argv[1]: N of the configs[2] MocoTrack, or "inverse<N>" (configs[4]'s
# MocoInverse) / "raja18" (the Rajagopal-18 golden MocoInverse)
what = sys.argv[1] if len(sys.argv) > 1 else "200"
ls = sys.argv[2] if len(sys.argv) > 2 else "device"
verbose = len(sys.argv) > 3
if what.startswith("inverse"):
    N = int(what[7:] or 125)
    st = configs.gait10dof18musc_inverse(N)
elif what == "raja18":
    st = configs.rajagopal18_inverse()
    N = st.solver.num_mesh_intervals
else:
    N = int(what)
    st = configs.gait10dof18musc_track(N, muscles=True)
t0 = time.perf_counter()
nlp = st.create_nlp()
setup = time.perf_counter() - t0
x0 = st.solver.starting_point(nlp)
o = IpmOptions.from_ipopt(st.solver.ipopt_options())
o.linear_solver = ls
o.print_level = 1 if verbose else 0
r = solve_ipm(nlp, x0, o)
print(json.dumps({"problem": what, "N": N, "linear_solver": r.timings.get("linear_solver"), "status": r.status,
                  "iterations": r.iterations, "objective": r.objective, "wall_clock_s": round(r.duration, 3),
                  "evaluations_s": round(r.timings["evaluations_s"], 3),
                  "linear_algebra_s": round(r.timings["linear_algebra_s"], 3), "setup_s": round(setup, 2),
                  "evaluations": r.evaluations, "n": nlp.n, "m": nlp.m, "nnz": nlp.nnz,
                  "kkt_ops": {k: [v[0], round(v[1], 4), v[2]] for k, v in
                              (getattr(getattr(nlp, "_dkkt", None), "stats", {}) or {}).items()}}), flush=True)
