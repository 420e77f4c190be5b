"""MocoTrajectory .sto I/O, resampling, iterate conversion and the Ipopt
option mapping (MocoTrajectory.cpp:581-800,
MocoCasADiSolver.cpp:210-246)."""
import os

import numpy as np
import pytest

from mocohip import configs
from mocohip.problem import MocoControlGoal, MocoProblem
from mocohip.solver import MocoHipSolver, OracleNLP
from mocohip.trajectory import MocoTrajectory, transcription_grid

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _golden_track():
    """The reference's converged MocoTrack solution (converted by
    tools/convert_reference_data.py from
    Moco/Tests/std_testMocoTrackGait10dof18musc_solution.sto: 20 states, 10
    controls, HS N=65 -> 131 times)."""
    d = np.load(os.path.join(GOLDEN, "std_testMocoTrackGait10dof18musc_solution.npz"))
    labels, data = [str(s) for s in d["labels"]], d["data"]
    ns, nc = 20, 10
    return MocoTrajectory(data[:, 0], labels[1:1 + ns], labels[1 + ns:1 + ns + nc], [], [], [], [],
                          data[:, 1:1 + ns], data[:, 1 + ns:1 + ns + nc])


def _track_nlp(N):
    m = configs.gait10dof18musc_model(muscles=False)
    p = MocoProblem(m)
    p.set_time_bounds(0.01, 1.3)
    p.add_goal(MocoControlGoal(weight=0.001))
    return OracleNLP(p.create_rep(), MocoHipSolver(num_mesh_intervals=N).options())


def test_sto_round_trip_and_header(tmp_path):
    tr = _golden_track()
    tr.metadata["success"] = "true"
    path = str(tmp_path / "sol.sto")
    tr.write(path)
    with open(path) as fh:
        head = fh.read().split("endheader")[0]
    for k in ("num_states=20", "num_controls=10", "num_multipliers=0", "num_derivatives=0",
              "num_slacks=0", "num_parameters=0", "success=true"):
        assert k in head
    back = MocoTrajectory.read(path)
    assert back.labels() == tr.labels()
    assert back.is_numerically_equal(tr, 0.0)
    assert back.metadata["success"] == "true"


def test_sto_blocks_in_reference_column_order(tmp_path):
    """states, controls, multipliers, derivatives, slacks, parameters
    (convertToTable, MocoTrajectory.cpp:786-800); parameters in the first row,
    NaN below (:830-838); counts must add up to the columns (:719-731)."""
    t = np.linspace(0, 1, 6)
    rng = np.random.default_rng(0)
    tr = MocoTrajectory(t, ["s0", "s1"], ["c0"], ["lambda_cid0_p0"], ["w0", "w1"], ["gamma_cid0_p0"],
                        ["p0"], rng.normal(size=(6, 2)), rng.normal(size=(6, 1)), rng.normal(size=(6, 1)),
                        rng.normal(size=(6, 2)), rng.normal(size=(6, 1)), np.array([3.5]))
    path = str(tmp_path / "all.sto")
    tr.write(path)
    lines = open(path).read().splitlines()
    i = lines.index("endheader")
    assert lines[i + 1].split("\t") == ["time", "s0", "s1", "c0", "lambda_cid0_p0", "w0", "w1",
                                        "gamma_cid0_p0", "p0"]
    assert lines[i + 2].split("\t")[-1] == "3.5" and lines[i + 3].split("\t")[-1] == "NaN"
    back = MocoTrajectory.read(path)
    assert back.is_numerically_equal(tr, 0.0)
    assert back.parameters.tolist() == [3.5]
    bad = open(path).read().replace("num_states=2", "num_states=3")
    open(path, "w").write(bad)
    with pytest.raises(ValueError, match="number of columns"):
        MocoTrajectory.read(path)


def test_resample_interpolates_and_checks_times():
    tr = _golden_track()
    t = tr.time.copy()
    ref = tr.states.copy()
    # the interpolating GCV spline reproduces the samples at the old times
    tr2 = _golden_track().resample(t)
    assert np.allclose(tr2.states, ref, rtol=0, atol=1e-12)
    # a smooth column resampled on a finer grid stays between neighbours'
    # spline values; and on a polynomial of degree <= 2 the quintic natural
    # spline is exact up to rounding
    poly = MocoTrajectory(np.linspace(0, 2, 9), ["a"], [], [], [], [], [],
                          (1.0 + 0.5 * np.linspace(0, 2, 9) - 0.25 * np.linspace(0, 2, 9) ** 2)[:, None])
    tn = np.linspace(0, 2, 37)
    poly.resample(tn)
    assert np.allclose(poly.states[:, 0], 1.0 + 0.5 * tn - 0.25 * tn ** 2, atol=1e-12)
    with pytest.raises(ValueError, match="initial time"):
        _golden_track().resample(np.array([0.0, 0.5]))
    with pytest.raises(ValueError, match="final time"):
        _golden_track().resample(np.array([0.1, 2.0]))
    with pytest.raises(ValueError, match="non-decreasing"):
        _golden_track().resample(np.array([0.2, 0.1, 0.3]))
    with pytest.raises(ValueError, match="0 or 1"):
        MocoTrajectory(np.array([0.0]), ["a"], states=np.zeros((1, 1))).resample([0.0])
    # 3 times -> GCVSpline degree min(3 - 1, 5) = 2, which GCVSpline rejects
    with pytest.raises(ValueError, match="odd"):
        MocoTrajectory(np.array([0.0, 1, 2]), ["a"], states=np.zeros((3, 1))).resample([0.5, 1.5])
    # zero duration: broadcast of the first row
    z = MocoTrajectory(np.array([0.0, 1.0]), ["a"], states=np.array([[2.0], [3.0]])).resample([0.0, 0.0])
    assert z.states[:, 0].tolist() == [2.0, 2.0]


def test_guess_to_iterate_matches_the_golden_columns():
    """At its own grid (HS N=65) the solution's iterate is the golden data
    column for column (the layout test_golden_gait_solution_order_and_defects
    pins); on another mesh it is the resampled trajectory."""
    tr = _golden_track()
    nlp = _track_nlp(65)
    x = tr.to_iterate(nlp)
    G, NS, NC = nlp.G, nlp.NS, nlp.NC
    S = x[2:2 + NS * G].reshape(G, NS)
    assert x[0] == tr.time[0] and x[1] == tr.time[-1]
    assert np.allclose(S, tr.states, rtol=0, atol=1e-12)
    assert np.abs(nlp.eval_g(x)).max() < 1e-2          # the reference's converged solution
    back = MocoTrajectory.from_iterate(nlp, x)
    assert np.allclose(back.time, tr.time, atol=1e-14)
    # resampled onto N=40 (the guess path of CasOCTranscription.cpp:593-597)
    n40 = _track_nlp(40)
    x40 = tr.to_iterate(n40)
    grid = transcription_grid("hermite-simpson", 40)
    t40 = (tr.time[-1] - tr.time[0]) * grid + tr.time[0]
    col = tr.state_names.index("/jointset/knee_r/knee_angle_r/value")
    ref = _golden_track().resample(t40).states[:, col]
    assert np.allclose(x40[2:2 + n40.NS * n40.G].reshape(n40.G, n40.NS)[:, col], ref, atol=1e-14)


@pytest.mark.parametrize("scheme,dyn", [("hermite-simpson", "explicit"), ("trapezoidal", "implicit")])
def test_iterate_round_trip(scheme, dyn, tmp_path):
    st = configs.double_pendulum(8, scheme, dynamics=dyn)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(3).uniform(-1, 1, nlp.n))
    x[0], x[1] = 0.0, 1.7
    tr = MocoTrajectory.from_iterate(nlp, x)
    assert tr.derivatives.shape[1] == nlp.NDV
    tr.write(str(tmp_path / "x.sto"))
    st.solver.guess_file = str(tmp_path / "x.sto")
    x2 = st.solver.starting_point(nlp)
    assert np.allclose(x2, x, rtol=1e-12, atol=1e-12)
    st.solver.guess_file = ""
    assert np.array_equal(st.solver.starting_point(nlp), nlp.initial_guess_from_bounds())


def test_ipopt_option_mapping():
    """MocoCasADiSolver.cpp:218-246."""
    s = MocoHipSolver()
    assert s.ipopt_options() == {"print_user_options": "yes",
                                 "hessian_approximation": "limited-memory"}
    s.verbosity = 0
    assert s.ipopt_options()["print_level"] == 0
    s.verbosity, s.optim_ipopt_print_level = 2, 5
    assert s.ipopt_options()["print_level"] == 5
    s.optim_max_iterations, s.optim_convergence_tolerance, s.optim_constraint_tolerance = 7, 1e-3, 1e-2
    o = s.ipopt_options()
    assert o["max_iter"] == 7
    for k in ("tol", "dual_inf_tol", "compl_inf_tol", "acceptable_tol", "acceptable_dual_inf_tol",
              "acceptable_compl_inf_tol"):
        assert o[k] == 1e-3
    assert o["constr_viol_tol"] == o["acceptable_constr_viol_tol"] == 1e-2
    s.optim_convergence_tolerance = -2.0
    with pytest.raises(ValueError):
        s.ipopt_options()
    s.optim_convergence_tolerance, s.verbosity = -1, 3
    with pytest.raises(ValueError):
        s.ipopt_options()


def _rms_pair(offset, n=21, shift=0.0):
    t = np.linspace(0.0, 1.0, n)
    s = np.column_stack([np.sin(3 * t), t ** 2])
    c = np.column_stack([np.cos(t)])
    a = MocoTrajectory(t, ["q", "u"], ["e"], [], [], [], ["p"], s, c, parameters=np.array([1.0]))
    s2 = s.copy()
    s2[:, 1] += offset
    b = MocoTrajectory(t + shift, ["q", "u"], ["e"], [], [], [], ["p"], s2, c.copy(),
                       parameters=np.array([1.5]))
    return a, b


def test_compare_continuous_variables_rms():
    """compareContinuousVariablesRMS (MocoTrajectory.cpp:1131-1263): zero for
    identical trajectories, c / sqrt(columns) for a constant offset c in one
    of the compared columns (the trapezoidal rule integrates a constant
    exactly), block selection by names and "none", and the name checks."""
    a, b = _rms_pair(0.0)
    assert a.compare_continuous_variables_rms(b) == pytest.approx(0.0, abs=1e-12)
    a, b = _rms_pair(0.3)
    assert a.compare_continuous_variables_rms(b) == pytest.approx(0.3 / np.sqrt(3), rel=1e-9)
    assert a.compare_continuous_variables_rms(b, states=["u"], controls=["none"]) == \
        pytest.approx(0.3, rel=1e-9)
    assert a.compare_continuous_variables_rms(b, states=["q"]) == pytest.approx(0.0, abs=1e-12)
    assert a.compare_continuous_variables_rms(b, states=["none"], controls=["none"]) == 0.0
    with pytest.raises(ValueError):
        a.compare_continuous_variables_rms(b, states=["w"])
    c = MocoTrajectory(a.time, ["q"], ["e"], [], [], [], [], a.states[:, :1], a.controls)
    with pytest.raises(ValueError):
        a.compare_continuous_variables_rms(c)
    # disjoint halves: each is compared against 0 where the other has no data
    a, b = _rms_pair(0.0, shift=0.5)
    assert a.compare_continuous_variables_rms(b) > 0.1
    # parameters (compareParametersRMS, :1311-1340)
    assert a.compare_parameters_rms(b) == pytest.approx(0.5)
    assert a.compare_parameters_rms(a) == 0.0


def test_compare_rms_empty_name_lists_mean_all():
    """An empty name list selects every column of its block, as the
    reference's empty std::vector does (MocoTrajectory.cpp:1140-1190);
    compareParametersRMS over no parameters is the reference's
    sqrt(0 / 0) = NaN, and unknown names are rejected (checkContains)."""
    a, b = _rms_pair(0.3)
    assert a.compare_continuous_variables_rms(b, states=[], controls=[]) == \
        a.compare_continuous_variables_rms(b)
    assert a.compare_parameters_rms(b, []) == a.compare_parameters_rms(b)
    e = MocoTrajectory(a.time, list(a.state_names), list(a.control_names), [], [], [], [],
                       a.states, a.controls)
    assert np.isnan(e.compare_parameters_rms(e))
    with pytest.raises(ValueError):
        a.compare_parameters_rms(b, ["no_such_parameter"])
