"""End to end: MocoStudy.solve() on the GPU path (HipNLP) with the host
interior-point solver (mocohip.ipm: Ipopt's algorithm restated; Ipopt is
absent), against the reference's own known-answer and golden-solution tests
of whole solves."""
import os

import numpy as np
import pytest

from mocohip import configs
from mocohip.ipm import IpmOptions, solve_ipm
from mocohip.trajectory import MocoTrajectory

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("scheme,dynamics", [("trapezoidal", "explicit"), ("trapezoidal", "implicit"),
                                             ("hermite-simpson", "explicit")])
def test_sliding_mass_known_solution(scheme, dynamics):
    """testMocoInterface.cpp:1701-1742 ("Sliding mass"): bang-bang control,
    final time 2.0, position and speed the quadratic / triangle profiles,
    force +-10; the reference's state and control names.  Trapezoidal (the
    reference's scheme): every one of the 20 times within the reference's
    1e-2.  Also in implicit dynamics mode (testImplicit.cpp solves its
    problems in both modes) and with Hermite-Simpson, where one point is a
    documented deviation of the scheme, not of the solver: the midpoint of
    the interval holding the switch sits on the speed peak, which the cubic
    interpolant cuts by 0.026, and its control is the switch itself (0)."""
    sol = configs.sliding_mass_interface(scheme=scheme, dynamics=dynamics).solve()
    assert sol.metadata["success"] == "true", sol.metadata
    assert sol.state_names == ["/slider/position/value", "/slider/position/speed"]
    assert sol.control_names == ["/actuator"]
    t = sol.time
    assert len(t) == (20 if scheme == "trapezoidal" else 39)
    assert t[-1] == pytest.approx(2.0, abs=1e-2)
    half = 0.5 * t[-1]
    pos = np.where(t < half, 0.5 * t ** 2, -0.5 * (t - half) ** 2 + (t - half) + 0.5)
    spd = np.where(t < half, t, t[-1] - t)
    frc = np.where(t < half, 10.0, -10.0)
    assert np.abs(sol.states[:, 0] - pos).max() < 1e-2
    if scheme == "trapezoidal":
        assert np.abs(sol.states[:, 1] - spd).max() < 1e-2
        assert np.abs(sol.controls[:, 0] - frc).max() < 1e-2
    else:
        sw = int(np.argmin(np.abs(t - half)))
        assert sw % 2 == 1   # a mesh-interval midpoint
        keep = np.arange(len(t)) != sw
        assert np.abs(sol.states[keep, 1] - spd[keep]).max() < 1e-2
        assert np.abs(sol.controls[keep, 0] - frc[keep]).max() < 1e-2
        assert abs(sol.states[sw, 1] - spd[sw]) < 0.03


def _golden(name, rep, with_derivatives=False):
    d = np.load(os.path.join(GOLDEN, name))
    labels = [str(l) for l in d["labels"]]
    data = d["data"]
    col = {l: i for i, l in enumerate(labels)}
    sn, cn = list(rep.state_names), list(rep.control_names)
    tr = MocoTrajectory(data[:, 0], sn, cn, states=data[:, [col[n] for n in sn]],
                        controls=data[:, [col[n] for n in cn]])
    return tr, labels, data


def _rms(gold: MocoTrajectory, sol: MocoTrajectory):
    mine = MocoTrajectory(sol.time, list(gold.state_names), list(gold.control_names),
                          states=sol.states, controls=sol.controls)
    return (gold.compare_continuous_variables_rms(mine, states=["none"]),
            gold.compare_continuous_variables_rms(mine, controls=["none"]))


def _rajagopal_golden_x(nlp, rep, labels, data):
    col = {l: i for i, l in enumerate(labels)}
    G = nlp.G
    mult = [l for l in labels if l.startswith("lambda")]
    der = [l for l in labels if "implicitderiv" in l]
    x = [data[0, 0], data[-1, 0]]
    for names in (rep.state_names, rep.control_names, mult, der):
        x += [data[k, col[n]] for k in range(G) for n in names]
    return np.array(x)


def test_moco_inverse_rajagopal18_solution():
    """testMocoInverse.cpp:118-147 (MocoInverse Rajagopal2016, 18 muscles,
    N = 11, MocoInverse tolerances 1e-3) solved on the GPU path by
    MocoStudy.solve, checked the reference's way: controls and states RMS
    against std_testMocoInverse_subject_18musc_solution.sto < 1e-2
    (measured on CPU through the oracle: 0.0024 / 0.0011).  The objective
    at the reference's solution, evaluated by our NLP, is the file's
    1.087741 to 1e-6 (the goals agree), and ours lands on it to 1e-3
    (measured 1.087729; the file records 52 Ipopt iterations in 54.5 s)."""
    st = configs.rajagopal18_inverse()
    rep = st.problem.create_rep()
    nlp = st.create_nlp()
    try:
        gold, labels, data = _golden("std_testMocoInverse_subject_18musc_solution.npz", rep)
        xg = _rajagopal_golden_x(nlp, rep, labels, data)
        assert nlp.eval_f(xg) == pytest.approx(1.087741, abs=1e-6)
        sol = st.solve(nlp=nlp)
        assert sol.metadata["success"] == "true", sol.metadata
        assert float(sol.metadata["objective"]) == pytest.approx(1.087741, rel=1e-3)
        rc, rs = _rms(gold, sol)
        assert rc < 1e-2 and rs < 1e-2, (rc, rs)
    finally:
        nlp.close()


def test_moco_track_gait_solution():
    """testMocoTrack.cpp:46-68 (MocoTrack gait10dof18musc, torque driven,
    N = 65) solved on the GPU path.  At the reference's tolerances (1e-2,
    MocoTrack.cpp:110-111) the solve converges; tightened to 1e-5 it reaches
    the problem's optimum, whose tracking cost is far below that of the
    reference's solution evaluated by the same objective (0.0259): with
    tolerance 1e-2 Ipopt stops long before the optimum of this problem (its
    solution misses the tracked knee angles by up to 0.2 rad although every
    coordinate has an unbounded reserve), so the golden file records
    Ipopt's own early iterate, which only Ipopt's exact iterate sequence
    reproduces -- the reference's RMS < 1e-2 check is therefore not
    reachable by a different optimizer (documented deviation; measured
    through the oracle: at tolerance 1e-2 our solve stops after 20
    iterations at objective 0.203, controls / states RMS 0.22 / 0.20
    against the file; at 1e-5 it reaches 0.00109 after 125 iterations)."""
    st = configs.gait10dof18musc_track()
    rep = st.problem.create_rep()
    nlp = st.create_nlp()
    try:
        gold, labels, data = _golden("std_testMocoTrackGait10dof18musc_solution.npz", rep)
        xg = np.concatenate([[data[0, 0], data[-1, 0]], gold.states.ravel(), gold.controls.ravel()])
        f_gold = nlp.eval_f(xg)
        sol = st.solve(nlp=nlp)
        assert sol.metadata["success"] == "true", sol.metadata
        tight = dict(st.solver.ipopt_options())
        for k in ("tol", "dual_inf_tol", "compl_inf_tol", "acceptable_tol", "acceptable_dual_inf_tol",
                  "acceptable_compl_inf_tol", "constr_viol_tol", "acceptable_constr_viol_tol"):
            tight[k] = 1e-5
        r = solve_ipm(nlp, st.solver.starting_point(nlp), IpmOptions.from_ipopt(tight))
        assert r.success, r.status
        assert r.objective < 0.1 * f_gold
        assert r.constraint_violation < 1e-4
        assert len(MocoTrajectory.from_iterate(nlp, r.x).time) == 131
    finally:
        nlp.close()


def test_moco_inverse_gait_n125_converges():
    """configs[4]'s NLP (MocoInverse gait10dof18musc, N = 125, random
    sparsity, forward differences, MocoInverse tolerances 1e-3) converges on
    the GPU path."""
    st = configs.gait10dof18musc_inverse(125)
    sol = st.solve()
    assert sol.metadata["success"] == "true", sol.metadata
    # (measured 7.762 through the oracle and on the GPU path)
    assert 7.5 < float(sol.metadata["objective"]) < 8.1


def test_inverse_solve_batch():
    """configs[4] layout: MocoInverse solves of scaled subjects started
    together, one process (HIP context, stream, host IPM) each, on one GPU:
    every solve converges on the generated back end (structure-only
    specialization keeps the scaled subjects on it)."""
    from mocohip import batchsolve
    out = batchsolve.solve_batch(batchsolve.sweep(3), num_mesh_intervals=10)
    assert out["succeeded"] == 3, out
    for r in out["results"]:
        assert r["backend"].startswith("generated:"), r
        assert r["iterations"] > 0
