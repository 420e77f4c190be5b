"""The barrier-parameter floor of Ipopt 3.12's monotone update (MonotoneMuUpdate::
CalcNewMuAndTau: mu >= min(tol, compl_inf_tol) / (barrier_tol_factor + 1)),
mocohip.ipm IpmOptions.mu_floor_from_tol, against the reference's golden
MocoInverse solution (std_testMocoInverse_subject_18musc_solution.sto,
testMocoInverse.cpp:118-147; MocoInverse's tolerances 1e-3,
MocoInverse.cpp:38-39, handed to Ipopt as tol / compl_inf_tol by
MocoCasADiSolver.cpp:234-244).

What the golden file pins (CPU, through the oracle; tools/mu_floor_probe.py):
  * the barrier parameter the golden solution sits at.  Its activations at
    their 0.01 lower bound are d = mu / z away from it; with the bound
    multipliers z of our unfloored solve (the same point to RMS 0.001) the
    golden's z * d is ~1e-6 -- the unfloored sequence's last mu (1.8e-6),
    two orders of magnitude under the 9.1e-5 floor.  A solve floored at
    9.1e-5 cannot produce that file;
  * why the floored solve ends at objective 1.126, not 1.0877: it is the
    barrier problem's solution at the floor (every finite bound's x z equals
    mu: a complementarity gap of mu per bound), so its activations sit
    mu / z off their bounds and the states / controls miss the golden by
    RMS 0.03 / 0.026, over testMocoInverse's own 1e-2.  No termination-test,
    bound_push or restoration difference is involved: the floored run
    converges (Solve_Succeeded) to the floored central path.
The default therefore leaves the floor off (mu_min alone), which reproduces
the golden objective to 5e-5."""
import numpy as np
import pytest

from mocohip import configs
from mocohip.ipm import IpmOptions, solve_ipm
from mocohip.solver import OracleNLP
from mocohip.trajectory import MocoTrajectory

import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "std_testMocoInverse_subject_18musc_solution.npz")


def _solve(floor):
    st = configs.rajagopal18_inverse()
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options(), threads=8)
    opts = st.solver.ipopt_options()
    opts["linear_solver"] = "host"
    o = IpmOptions.from_ipopt(opts)
    o.mu_floor_from_tol = floor
    r = solve_ipm(nlp, st.solver.starting_point(nlp), o)
    return nlp, o, r


@pytest.fixture(scope="module")
def golden():
    d = np.load(GOLDEN)
    labels = [str(s) for s in d["labels"]]
    return {l: i for i, l in enumerate(labels)}, d["data"], labels


def _rms(sol, col, data):
    rs = float(np.sqrt(np.mean((data[:, [col[n] for n in sol.state_names]] - sol.states) ** 2)))
    rc = float(np.sqrt(np.mean((data[:, [col[n] for n in sol.control_names]] - sol.controls) ** 2)))
    return rs, rc


def test_golden_sits_below_the_floor(golden):
    col, data, labels = golden
    nlp, o, r = _solve(False)
    assert r.success
    floor = min(o.tol, o.compl_inf_tol) / (o.kappa_eps + 1.0)
    mu_last = r.history[-1][4]
    assert mu_last < floor / 10
    sol = MocoTrajectory.from_iterate(nlp, r.x)
    rs, rc = _rms(sol, col, data)
    assert rs < 1e-2 and rc < 1e-2                     # testMocoInverse.cpp:144-146
    assert abs(r.objective - 1.087741) < 1e-3          # the golden file's objective
    # the golden's barrier parameter: z * (x - lower) over the activations at
    # their lower bound, z from this solve
    xl = nlp.bounds()[0]
    NS, G = len(sol.state_names), len(sol.time)
    est = []
    for a in (l for l in labels if l.endswith("/activation")):
        j = sol.state_names.index(a)
        for k in range(G):
            ix = 2 + k * NS + j
            d = data[k, col[a]] - xl[ix]
            if r.z_l[ix] > 1e-2 and d < 1e-3:
                est.append(r.z_l[ix] * d)
    mu_golden = float(np.median(est))
    print(f"floor {floor:.2e}; unfloored final mu {mu_last:.2e}; golden's mu ~ {mu_golden:.2e} (n = {len(est)})")
    assert len(est) > 20
    assert mu_last / 10 < mu_golden < mu_last * 10
    assert mu_golden < floor / 10
    nlp.close()


def test_floored_solve_is_the_floored_central_path(golden):
    col, data, _ = golden
    nlp, o, r = _solve(True)
    assert r.success
    floor = min(o.tol, o.compl_inf_tol) / (o.kappa_eps + 1.0)
    assert r.history[-1][4] == pytest.approx(floor)
    xl, xu = nlp.bounds()[:2]
    fl, fu = np.isfinite(xl), np.isfinite(xu)
    xz = np.concatenate([((r.x - xl) * r.z_l)[fl], ((xu - r.x) * r.z_u)[fu]])
    # every bound's complementarity at the floor (Ipopt's barrier problem
    # solved to kappa_eps mu)
    assert np.median(np.abs(xz / floor - 1.0)) < 0.1
    sol = MocoTrajectory.from_iterate(nlp, r.x)
    rs, rc = _rms(sol, col, data)
    print(f"floored: objective {r.objective:.6f}, states RMS {rs:.4f}, controls RMS {rc:.4f}")
    assert r.objective > 1.1 and (rs > 1e-2 or rc > 1e-2)
    nlp.close()
