"""The device KKT module (include/mocohip_kkt.h, csrc/kkt.hip) on the GPU
against its numpy restatement (tests/_kkt_ref.py) and a dense solve: the
Jacobian it evaluates is the context's eval_jac_g bit for bit, the products
with J and the block-cyclic-reduction solves agree to rounding; and the
interior-point solver gives the same solves with the device linear algebra
as with the host's."""
import numpy as np
import pytest

import _kkt_ref as K
from mocohip import configs
from mocohip.ipm import IpmOptions, solve_ipm
from mocohip.solver import HipNLP

pytestmark = pytest.mark.gpu

CASES = {
    "sliding_mass_hs": lambda: configs.sliding_mass(7),
    "double_pendulum_trap": lambda: configs.double_pendulum(6, "trapezoidal"),
    "gait_rigid": lambda: configs.gait10dof18musc(3),
    "gait_inverse": lambda: configs.gait10dof18musc_inverse(4, sparsity="none"),
    "coupled_pendulum": lambda: configs.double_pendulum_coupled(5),
    "coupled_pendulum_implicit": lambda: configs.double_pendulum_coupled(4, dynamics="implicit"),
    "pendulum_path": lambda: configs.pendulum_control_bound(5, "both"),
    "gait_rigid_n200": lambda: configs.gait10dof18musc(200),
}


def _setup(name, seed=0):
    st = CASES[name]()
    nlp = HipNLP(st.problem.create_rep(), st.solver.options())
    rng = np.random.default_rng(seed)
    x = nlp.random_iterate(rng.uniform(-1, 1, nlp.n))
    G, NS, NC = nlp.G, nlp.NS, nlp.NC
    x[2:2 + NS * G] = nlp.initial_guess_from_bounds()[2:2 + NS * G]
    if nlp.NAR:
        x[2:2 + NS * G] = rng.uniform(0.05, 0.5, NS * G)
        x[2 + NS * G:2 + (NS + NC) * G] = rng.uniform(0.05, 0.4, NC * G)
    return nlp, x, rng


@pytest.mark.parametrize("path", ["inverse", "substitution"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_device_kkt_matches_restatement(name, path, monkeypatch):
    """Both factorization paths of csrc/kkt.hip: blocks inverted in LDS and
    every step a GEMM (default for r <= 160), or substitution
    (MOCOHIP_KKT_INV=0; the path large blocks take)."""
    monkeypatch.setenv("MOCOHIP_KKT_INV", "1" if path == "inverse" else "0")
    nlp, x, rng = _setup(name)
    try:
        dk = nlp.device_kkt()
        bm = dk.bm
        dk.eval_jacobian(x)
        vals = dk.values()
        assert np.array_equal(vals, nlp.eval_jac_g(x))        # the context's own kernels
        rs = rng.uniform(0.5, 2.0, nlp.m)
        dk.set_row_scale(rs)
        dk.eval_jacobian(x)
        # products with J (every column, dense included)
        ir, jc = nlp.jac_structure()
        import scipy.sparse as sp
        J = sp.csr_matrix((vals * rs[ir], (ir, jc)), shape=(nlp.m, nlp.n))
        V = rng.standard_normal((nlp.n, 3))
        Y = rng.standard_normal((nlp.m, 3))
        V40 = rng.standard_normal((nlp.n, 40))                 # two passes of 32 and 8 columns
        Y40 = rng.standard_normal((nlp.m, 40))
        for got, want in ((dk.jmul(V), J @ V), (dk.jtmul(Y), J.T @ Y), (dk.jmul(V[:, 0]), J @ V[:, 0]),
                          (dk.jmul(V40), J @ V40), (dk.jtmul(Y40), J.T @ Y40)):
            assert np.abs(got - want).max() <= 1e-12 * (np.abs(want).max() + 1.0)
        cols, Jd = dk.dense_columns()
        assert np.array_equal(cols, bm.dcols)
        assert np.abs(Jd - J[:, cols].toarray()).max() == 0.0
        # factor + solve against the numpy restatement of the same algorithm
        w = rng.uniform(0.1, 10.0, nlp.n)
        w[bm.dcols] = 0.0
        dc = rng.uniform(1e-8, 1e-2, nlp.m)
        assert dk.factor(w, dc)
        A, _ = K.gather(bm, vals, rs)
        D, E = K.schur_blocks(bm, A, w, dc)
        Lf, U, Vf, levels = K.cr_factor(D, E)
        # (S's condition number reaches ~1e8 here -- J's entries span
        # orders of magnitude, dc ~ 1e-8 -- so two stable orderings of the
        # same factorization agree to ~cond * eps, and the residual below
        # is the sharp check)
        for k in (1, 5, 40):                                     # 40: two passes of 32 columns
            B = rng.standard_normal((nlp.m, k))
            Xr = K.from_blocks(bm, K.cr_solve(Lf, U, Vf, levels, K.to_blocks(bm, B)))
            Xg = dk.solve(B)
            assert np.abs(Xg - Xr).max() <= 1e-5 * np.abs(Xr).max(), k
        # and the Schur complement itself: S X = B
        B = rng.standard_normal(nlp.m)
        X = dk.solve(B)
        Jb = J.tolil()
        Jb[:, bm.dcols] = 0.0
        Jb = Jb.tocsr()
        SX = Jb @ (w * (Jb.T @ X)) + dc * X
        resid = SX - B
        # backward error: the residual against |S| |X| (componentwise scale)
        absS_absX = abs(Jb) @ (w * (abs(Jb).T @ np.abs(X))) + dc * np.abs(X) + np.abs(B)
        # (the inverse path multiplies by inv(L_i): its backward error is
        # ~cond(L_i) eps rather than substitution's ~eps)
        assert (np.abs(resid) / absS_absX).max() <= 1e-10
    finally:
        nlp.close()


def test_device_kkt_reports_indefinite():
    nlp, x, rng = _setup("gait_rigid")
    try:
        dk = nlp.device_kkt()
        dk.eval_jacobian(x)
        w = -np.ones(nlp.n)
        assert not dk.factor(w, np.full(nlp.m, 1e-8))
        with pytest.raises(RuntimeError):
            dk.solve(np.ones(nlp.m))
        assert dk.factor(np.ones(nlp.n), np.full(nlp.m, 1e-8))   # recovers
    finally:
        nlp.close()


@pytest.mark.parametrize("name", ["sliding_mass_interface", "gait_track_n20", "gait_inverse_n10"])
def test_ipm_device_linear_algebra_matches_host(name):
    """The same solve with the Newton systems factored on the device and on
    the host: the same termination, objective and solution to tolerance
    (the factorizations' rounding differs, so the iterates agree to ~1e-8
    at first and the end points to the problem's conditioning)."""
    st = {"sliding_mass_interface": lambda: configs.sliding_mass_interface(),
          "gait_track_n20": lambda: configs.gait10dof18musc_track(20, muscles=True),
          "gait_inverse_n10": lambda: configs.gait10dof18musc_inverse(10)}[name]()
    nlp = st.create_nlp()
    try:
        x0 = st.solver.starting_point(nlp)
        res = {}
        for ls in ("host", "device"):
            o = IpmOptions.from_ipopt(st.solver.ipopt_options())
            o.linear_solver = ls
            res[ls] = solve_ipm(nlp, x0, o)
        h, d = res["host"], res["device"]
        assert h.success and d.success, (h.status, d.status)
        assert d.timings["linear_solver"].startswith("device")
        # the first iterates agree closely
        k = min(5, len(h.history), len(d.history))
        for a, b in zip(h.history[:k], d.history[:k]):
            assert abs(a[1] - b[1]) <= 1e-6 * max(1.0, abs(a[1])), (a, b)
        assert abs(h.objective - d.objective) <= 1e-3 * max(1.0, abs(h.objective)), (h.objective, d.objective)
    finally:
        nlp.close()
