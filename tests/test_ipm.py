"""The host interior-point solver (mocohip.ipm, Ipopt's algorithm restated)
on CPU: known answers of small NLPs, and whole transcriptions evaluated by
the oracle (test infrastructure) so the solver is checked without a GPU."""
import numpy as np
import pytest

from mocohip import configs
from mocohip.ipm import IpmOptions, solve_ipm
from mocohip.solver import OracleNLP


class _HS071:
    """Hock-Schittkowski problem 71, Ipopt's own example (Ipopt
    examples/hs071_cpp): min x1 x4 (x1 + x2 + x3) + x3 s.t. x1 x2 x3 x4 >= 25,
    sum x^2 = 40, 1 <= x <= 5, from (1, 5, 5, 1)."""
    n, m, nnz = 4, 2, 8

    def bounds(self):
        return np.ones(4), 5 * np.ones(4), np.array([25.0, 40.0]), np.array([np.inf, 40.0])

    def jac_structure(self):
        return np.repeat([0, 1], 4).astype(np.int32), np.tile(np.arange(4), 2).astype(np.int32)

    def eval_f(self, x):
        return x[0] * x[3] * (x[0] + x[1] + x[2]) + x[2]

    def eval_grad_f(self, x):
        return np.array([x[0] * x[3] + x[3] * (x[0] + x[1] + x[2]), x[0] * x[3],
                         x[0] * x[3] + 1, x[0] * (x[0] + x[1] + x[2])])

    def eval_g(self, x):
        return np.array([np.prod(x), x @ x])

    def eval_jac_g(self, x):
        return np.array([x[1] * x[2] * x[3], x[0] * x[2] * x[3], x[0] * x[1] * x[3], x[0] * x[1] * x[2],
                         *(2 * x)])


def test_hs071_known_solution():
    """Ipopt's documented hs071 answer: f* = 17.014017..., x* = (1, 4.743,
    3.82115, 1.37941), lambda = (-0.552294, 0.161469) (Ipopt's sign
    convention L = f + g^T lambda), upper bound multiplier of x1 zero."""
    r = solve_ipm(_HS071(), np.array([1.0, 5.0, 5.0, 1.0]))
    assert r.success and r.status == "Solve_Succeeded"
    assert r.objective == pytest.approx(17.014017145179164, rel=1e-8)
    assert np.allclose(r.x, [1.0, 4.742999643601108, 3.821149978948624, 1.379408293215359], atol=1e-6)
    assert np.allclose(r.lambda_g, [-0.5522936593964548, 0.16146856250000005], atol=1e-6)
    assert r.z_l[0] == pytest.approx(1.087871, rel=1e-4)


class _Rosenbrock:
    """Bound-constrained Rosenbrock with one linear inequality row:
    min (1 - x)^2 + 100 (y - x^2)^2, x <= 0.5, x + y >= -10; the optimum
    sits on the bound x = 0.5, y = 0.25."""
    n, m, nnz = 2, 1, 2

    def bounds(self):
        return np.array([-np.inf, -np.inf]), np.array([0.5, np.inf]), np.array([-10.0]), np.array([np.inf])

    def jac_structure(self):
        return np.array([0, 0], np.int32), np.array([0, 1], np.int32)

    def eval_f(self, x):
        return (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2

    def eval_grad_f(self, x):
        return np.array([-2 * (1 - x[0]) - 400 * x[0] * (x[1] - x[0] ** 2), 200 * (x[1] - x[0] ** 2)])

    def eval_g(self, x):
        return np.array([x[0] + x[1]])

    def eval_jac_g(self, x):
        return np.array([1.0, 1.0])


def test_rosenbrock_active_bound():
    r = solve_ipm(_Rosenbrock(), np.array([-1.2, 1.0]))
    assert r.success
    assert np.allclose(r.x, [0.5, 0.25], atol=1e-6)
    assert r.objective == pytest.approx(0.25, abs=1e-8)


@pytest.mark.parametrize("scheme,dynamics", [("trapezoidal", "explicit"), ("trapezoidal", "implicit")])
def test_sliding_mass_oracle(scheme, dynamics):
    """testMocoInterface.cpp:1701-1742 ("Sliding mass") with the interior-
    point solver over the oracle's callbacks: every one of the 20 times
    within the reference's 1e-2 (position, speed and force)."""
    st = configs.sliding_mass_interface(scheme=scheme, dynamics=dynamics)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    sol = st.solve(nlp=nlp)
    assert sol.metadata["success"] == "true", sol.metadata
    t = sol.time
    assert len(t) == 20 and t[-1] == pytest.approx(2.0, abs=1e-2)
    half = 0.5 * t[-1]
    pos = np.where(t < half, 0.5 * t ** 2, -0.5 * (t - half) ** 2 + (t - half) + 0.5)
    spd = np.where(t < half, t, t[-1] - t)
    frc = np.where(t < half, 10.0, -10.0)
    assert np.abs(sol.states[:, 0] - pos).max() < 1e-2
    assert np.abs(sol.states[:, 1] - spd).max() < 1e-2
    assert np.abs(sol.controls[:, 0] - frc).max() < 1e-2


def test_options_from_moco_tolerances():
    """MocoCasADiSolver's option mapping (MocoCasADiSolver.cpp:229-244)
    reaches the solver: optim_convergence_tolerance sets tol, dual_inf_tol,
    compl_inf_tol and their acceptable_* levels; optim_constraint_tolerance
    constr_viol_tol and acceptable_constr_viol_tol; the rest keep Ipopt's
    defaults."""
    s = configs.gait10dof18musc_track().solver
    o = IpmOptions.from_ipopt(s.ipopt_options())
    assert (o.tol, o.dual_inf_tol, o.compl_inf_tol, o.acceptable_tol) == (1e-2,) * 4
    assert (o.constr_viol_tol, o.acceptable_constr_viol_tol) == (1e-2, 1e-2)
    d = IpmOptions.from_ipopt(configs.sliding_mass_interface().solver.ipopt_options())
    assert (d.tol, d.constr_viol_tol, d.dual_inf_tol, d.max_iter) == (1e-8, 1e-4, 1.0, 3000)


def test_gait_track_problem_layout():
    """The MocoTrack golden-solution problem (testMocoTrack.cpp:46-68): 20
    states, 10 reserve controls, HS N = 65 (131 grid points like the golden
    file), the file's column order."""
    st = configs.gait10dof18musc_track()
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    assert (nlp.NS, nlp.NC, nlp.G) == (20, 10, 131)
    d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                           "std_testMocoTrackGait10dof18musc_solution.npz"))
    assert [str(l) for l in d["labels"]][1:] == rep.state_names + rep.control_names
    assert d["data"].shape[0] == nlp.G


def test_ipopt_linear_solver_option_ignored():
    """An Ipopt option dictionary's linear_solver ('mumps', the value
    MocoCasADiSolver / tropter hand Ipopt) names Ipopt's sparse
    factorization, not the Newton systems' back end here: it is ignored, and
    this option's own values still apply."""
    from mocohip.ipm import IpmOptions
    assert IpmOptions.from_ipopt({"linear_solver": "mumps", "tol": 1e-6}).linear_solver == "auto"
    assert IpmOptions.from_ipopt({"linear_solver": "ma27"}).linear_solver == "auto"
    assert IpmOptions.from_ipopt({"linear_solver": "host"}).linear_solver == "host"
    assert IpmOptions.from_ipopt({"linear_solver": "mumps", "tol": 1e-6}).tol == 1e-6
