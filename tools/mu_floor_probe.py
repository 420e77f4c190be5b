"""The tol-derived barrier floor (Ipopt 3.12 MonotoneMuUpdate) on the golden
MocoInverse solve (Rajagopal 18, N = 11, testMocoInverse.cpp:118-147),
through the oracle on the CPU: the iteration logs with the floor off / on and
the RMS of the solution against the reference's golden file.

    python tools/mu_floor_probe.py [--floor on|off|both] [--print]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))
sys.path.insert(0, ROOT)

from mocohip import configs  # noqa: E402
from mocohip.ipm import IpmOptions, solve_ipm  # noqa: E402
from mocohip.solver import OracleNLP  # noqa: E402
from mocohip.trajectory import MocoTrajectory  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden", "std_testMocoInverse_subject_18musc_solution.npz")


def run(floor: bool, verbose: bool, **extra):
    st = configs.rajagopal18_inverse()
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options(), threads=8)
    opts = st.solver.ipopt_options()
    opts["linear_solver"] = "host"
    o = IpmOptions.from_ipopt(opts)
    o.mu_floor_from_tol = floor
    o.print_level = 1 if verbose else 0
    for k, v in extra.items():
        setattr(o, k, v)
    x0 = st.solver.starting_point(nlp)
    r = solve_ipm(nlp, x0, o)
    sol = MocoTrajectory.from_iterate(nlp, r.x)
    d = np.load(GOLDEN)
    labels = [str(s) for s in d["labels"]]
    col = {l: i for i, l in enumerate(labels)}
    data = d["data"]
    rs = float(np.sqrt(np.mean((data[:, [col[n] for n in sol.state_names]] - sol.states) ** 2)))
    rc = float(np.sqrt(np.mean((data[:, [col[n] for n in sol.control_names]] - sol.controls) ** 2)))
    print(f"floor={'on' if floor else 'off'} {extra}: status {r.status} iters {r.iterations} "
          f"objective {r.objective:.6f} states RMS {rs:.4f} controls RMS {rc:.4f} "
          f"final mu {r.history[-1][4]:.2e}")
    nlp.close()
    return r


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--floor", default="both")
    ap.add_argument("--print", action="store_true")
    a = ap.parse_args()
    for f in ([False, True] if a.floor == "both" else [a.floor == "on"]):
        run(f, a.print)
