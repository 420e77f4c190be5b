"""Pin the CPU oracle against the reference's own known answers and golden
files.  CPU only."""
import ctypes as C
import math
import os

import numpy as np
import pytest

from mocohip import abi, configs
from mocohip.problem import MocoControlGoal, MocoProblem
from mocohip.solver import MocoHipSolver, OracleNLP
from mocohip.splines import SimmSpline, gcv_interpolating_ppoly, ppoly_eval

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

lib = abi.load_oracle()


def dgf_muscle(**kw):
    m = abi.mh_muscle()
    m.active_force_width_scale = 1.0
    m.passive_fiber_strain_at_one_norm_force = 0.6
    m.tendon_strain_at_one_norm_force = 0.049
    for k, v in kw.items():
        setattr(m, k, v)
    return m


def curve(m, which, x):
    return lib.orc_dgf_curve(C.byref(m), which, float(x))


def test_dgf_curve_known_answers():
    """Moco/Tests/testMocoActuators.cpp:199-220 ("Curve values")."""
    m = dgf_muscle()
    assert curve(m, 4, 1.0) == 0.0                                  # f_T(1) == 0
    assert curve(m, 4, 1 + 0.049) == pytest.approx(1, rel=1e-10)    # f_T(1+eps_T)
    assert curve(m, 1, 1.0) == pytest.approx(0.0182288, rel=1e-4)   # f_PE(1)
    assert curve(m, 1, 0.2) == pytest.approx(0, abs=1e-4)           # f_PE(0.2)
    assert curve(m, 1, 1 + 0.6) == pytest.approx(1, rel=1e-4)       # f_PE(1+e0)
    assert curve(m, 0, 1.0) == pytest.approx(1)                     # f_AL(1)
    assert curve(m, 2, -1.0) == 0.0 or abs(curve(m, 2, -1.0)) < 1e-15  # f_V(-1)
    assert curve(m, 2, 0.0) == pytest.approx(1)                     # f_V(0)
    assert curve(m, 2, 1.0) == pytest.approx(1.794, rel=1e-3)       # f_V(1)


def test_dgf_force_velocity_inverse():
    """testMocoActuators.cpp:1026-1039: FV inverse round trip."""
    m = dgf_muscle()
    for v in np.linspace(-1, 1, 100):
        assert curve(m, 3, curve(m, 2, v)) == pytest.approx(v, abs=1e-12)


def test_dgf_tendon_inverse_and_derivative():
    m = dgf_muscle()
    for lt in np.linspace(0.99, 1.06, 30):
        f = curve(m, 4, lt)
        assert curve(m, 5, f) == pytest.approx(lt, rel=1e-12)
        h = 1e-6
        fd = (curve(m, 4, lt + h) - curve(m, 4, lt - h)) / (2 * h)
        assert curve(m, 6, lt) == pytest.approx(fd, rel=1e-7)


def test_simmspline_restatement():
    """SimmSpline (FMM cubic): interpolates the knots, C2 inside, linear
    extrapolation outside; oracle and host restatement agree."""
    x = [-2.0944, -1.74533, -1.39626, -1.0472, -0.698132, -0.349066, -0.174533,
         0.197344, 0.337395, 0.490178, 1.52146, 2.0944]
    y = [-0.0032, 0.00179, 0.00411, 0.0041, 0.00212, -0.001, -0.0031, -0.005227,
         -0.005435, -0.005574, -0.005435, -0.00525]
    s = SimmSpline(x, y)
    for xi, yi in zip(x, y):
        assert s(xi) == pytest.approx(yi, abs=1e-15)
    for t in np.linspace(-1.9, 2.0, 37):
        h = 1e-6
        assert s(t, 1) == pytest.approx((s(t + h) - s(t - h)) / (2 * h), abs=1e-7)
    assert s(3.0) == pytest.approx(y[-1] + (3.0 - x[-1]) * s.b[-1])
    # oracle evaluation through a one-coordinate model
    from mocohip.model import Body, Coordinate, Function, Joint, Model, Axis
    m = Model("spline_probe")
    m.add_body(Body("b", 1.0, (0, 0, 0), (1, 1, 1, 0, 0, 0)))
    q = Coordinate("q")
    m.add_joint(Joint("j", "ground", "b", [q], [
        Axis(abi.MH_AXIS_ROTATION, (0, 0, 1), Function.linear("q")),
        Axis(abi.MH_AXIS_TRANSLATION, (1, 0, 0), Function.simm_spline("q", x, y, 1.14724))]))
    p = MocoProblem(m)
    nlp = OracleNLP(p.create_rep(), MocoHipSolver(num_mesh_intervals=2).options())
    out = np.zeros(3)
    for t in np.linspace(-2.5, 2.5, 23):
        lib.orc_eval_function(nlp.ctx, 1, float(t), abi.dptr(out))
        assert out[0] == pytest.approx(1.14724 * s(t), abs=1e-15)
        assert out[1] == pytest.approx(1.14724 * s(t, 1), abs=1e-13)


def test_gcv_natural_spline_interpolates():
    t = np.linspace(0, 1, 23)
    y = np.sin(3 * t)[:, None]
    for deg in (3, 5):
        br, cf = gcv_interpolating_ppoly(t, y, deg)
        assert np.allclose(ppoly_eval(br, cf, t, 0), y[:, 0], atol=1e-12)
        assert np.abs(ppoly_eval(br, cf, 0.5, 0) - np.sin(1.5)) < 1e-5


def _point_inputs(nlp, states, controls, t=0.3):
    return np.concatenate([[t], states, controls])[None, :]


def test_double_pendulum_closed_form():
    """ModelFactory::createNLinkPendulum(2) dynamics vs the closed form of
    tropter/tests/test_double_pendulum.cpp:45-74 (point masses) plus the unit
    rotational inertia of each body (Inertia(1))."""
    st = configs.double_pendulum(4)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    rng = np.random.default_rng(3)
    g = 9.80665
    for _ in range(20):
        q0, q1, u0, u1, t0, t1 = rng.uniform(-2, 2, 6)
        out = nlp.eval_dae(_point_inputs(nlp, [q0, q1, u0, u1], [t0, t1]))[0]
        L0 = L1 = m0 = m1 = 1.0
        z0 = m1 * L0 * L1 * math.cos(q1)
        M = np.array([[m0 * L0 ** 2 + m1 * (L0 ** 2 + L1 ** 2) + 2 * z0 + 2.0, m1 * L1 ** 2 + z0 + 1.0],
                      [m1 * L1 ** 2 + z0 + 1.0, m1 * L1 ** 2 + 1.0]])
        V = np.array([-u1 * (2 * u0 + u1), u0 * u0]) * m1 * L0 * L1 * math.sin(q1)
        Gv = np.array([g * ((m0 + m1) * L0 * math.cos(q0) + m1 * L1 * math.cos(q0 + q1)),
                       g * m1 * L1 * math.cos(q0 + q1)])
        udot = np.linalg.solve(M, np.array([t0, t1]) - (V + Gv))
        assert np.allclose(out, udot, rtol=1e-12, atol=1e-12)


def test_sliding_mass_dynamics():
    st = configs.sliding_mass(3)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    out = nlp.eval_dae(np.array([[0.1, 0.3, -2.0, 7.0]]))
    assert out[0, 0] == pytest.approx(7.0 / 2.0, rel=1e-15)


@pytest.mark.parametrize("name,N,n,m,nnz", [
    ("sliding_mass", 50, 305, 250, 1850),
    ("double_pendulum", 100, 1208, 1000, 10400),
])
def test_layout_sizes(name, N, n, m, nnz):
    """SURVEY.md §8 config size table."""
    st = configs.CONFIGS[name](N)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    assert (nlp.n, nlp.m, nlp.nnz) == (n, m, nnz)


def test_gait_layout_sizes():
    st = configs.gait10dof18musc(200)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    assert (nlp.NS, nlp.NC) == (38, 28)
    assert (nlp.n, nlp.m) == (26468, 20800)
    assert nlp.nnz == 9604 * 200          # ≈1.92 M


def test_sliding_mass_bounds():
    """exampleSlidingMass bounds through CasOC's column rules
    (CasOCTranscription.cpp:183-250)."""
    st = configs.sliding_mass(5)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    xl, xu, gl, gu = nlp.bounds()
    G = nlp.G
    assert (xl[0], xu[0], xl[1], xu[1]) == (0, 0, 0, 5)
    pos = lambda k: 2 + k * 2
    assert (xl[pos(0)], xu[pos(0)]) == (0, 0)
    assert (xl[pos(G - 1)], xu[pos(G - 1)]) == (1, 1)
    assert (xl[pos(3)], xu[pos(3)]) == (-5, 5)
    assert (xl[pos(3) + 1], xu[pos(3) + 1]) == (-50, 50)
    assert (xl[2 + 2 * G + 3], xu[2 + 2 * G + 3]) == (-50, 50)
    assert np.all(gl == 0) and np.all(gu == 0)
    x = nlp.initial_guess_from_bounds()
    assert x[1] == 2.5 and x[pos(0)] == 0 and x[pos(G - 1)] == 1


def test_structure_contains_true_dependencies():
    """Perturbing any variable changes only rows where the structure has a
    nonzero in that column."""
    st = configs.double_pendulum(4)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    ir, jc = nlp.jac_structure()
    S = set(zip(ir.tolist(), jc.tolist()))
    x = nlp.random_iterate(np.random.default_rng(1).uniform(-1, 1, nlp.n))
    x[1] = 2.0
    g0 = nlp.eval_g(x)
    for j in range(nlp.n):
        xp = x.copy()
        xp[j] += 1e-3
        rows = np.nonzero(nlp.eval_g(xp) != g0)[0]
        for r in rows:
            assert (int(r), j) in S


def _numjac(fun, x, cols, h=1e-4):
    out = []
    for j in cols:
        e = np.zeros_like(x)
        e[j] = 1.0
        f1, f2 = fun(x + h * e), fun(x - h * e)
        f3, f4 = fun(x + 2 * h * e), fun(x - 2 * h * e)
        out.append((8 * (f1 - f2) - (f3 - f4)) / (12 * h))
    return np.array(out).T


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
def test_jacobian_matches_numerical_derivative(scheme):
    st = configs.double_pendulum(3, scheme)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(2).uniform(-1, 1, nlp.n))
    x[1] = 1.5
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    Jn = _numjac(nlp.eval_g, x, range(nlp.n))
    # central FD at h=1e-8 carries ~eps*|f|/h rounding noise
    assert np.allclose(J, Jn, rtol=1e-5, atol=1e-6)


def test_grad_f_matches_numerical_derivative():
    st = configs.double_pendulum(3)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(4).uniform(-1, 1, nlp.n))
    x[1] = 1.5
    gn = _numjac(lambda z: np.array([nlp.eval_f(z)]), x, range(nlp.n))[0]
    assert np.allclose(nlp.eval_grad_f(x), gn, rtol=1e-6, atol=1e-7)


def _golden_iterate(nlp, rep):
    d = np.load(__import__("os").path.join(__import__("os").path.dirname(__file__),
                                           "golden", "std_testMocoTrackGait10dof18musc_solution.npz"))
    labels, data = list(d["labels"]), d["data"]
    col = {l: i for i, l in enumerate(labels)}
    G, NS, NC = nlp.G, nlp.NS, nlp.NC
    x = np.zeros(nlp.n)
    x[0], x[1] = data[0, 0], data[-1, 0]
    for k in range(G):
        for s, n in enumerate(rep.state_names):
            x[2 + k * NS + s] = data[k, col[n]]
        for j, n in enumerate(rep.control_names):
            x[2 + NS * G + k * NC + j] = data[k, col[n]]
    return x, labels


def test_golden_gait_solution_order_and_defects():
    """Moco/Tests/std_testMocoTrackGait10dof18musc_solution.sto (MocoTrack
    gait10dof18musc, reserves, GRF, HS N=65, converged with constraint
    tolerance 1e-2, MocoTrack.cpp:107-109): state/control order must equal
    the file's column order, and the reference's converged iterate must
    satisfy our defects to that tolerance (pins multibody dynamics, the knee
    CustomJoint splines, reserves and the ground reactions)."""
    m = configs.gait10dof18musc_model(muscles=False)
    p = MocoProblem(m)
    p.set_time_bounds(0.01, 1.3)
    p.add_goal(MocoControlGoal(weight=0.001))
    rep = p.create_rep()
    nlp = OracleNLP(rep, MocoHipSolver(num_mesh_intervals=65).options())
    x, labels = _golden_iterate(nlp, rep)
    assert labels[1:] == rep.state_names + rep.control_names
    g = nlp.eval_g(x)
    assert np.abs(g).max() < 1e-2
    # and a 1% heavier femur or a 1% shorter knee spline is detected
    m.bodies["femur_r"].mass *= 1.5
    p2 = MocoProblem(m)
    p2.set_time_bounds(0.01, 1.3)
    nlp2 = OracleNLP(p2.create_rep(), MocoHipSolver(num_mesh_intervals=65).options())
    assert np.abs(nlp2.eval_g(x)).max() > 1e-2


def test_muscle_geometry_matches_reference_gso_fiber_lengths():
    """Muscle path geometry (PathPoint / ConditionalPathPoint /
    MovingPathPoint with the knee SimmSplines) pinned by the
    reference's GSO golden files
    Moco/Archive/Tests/std_testGait10dof18musc_GSO_solution_norm_fiber_{length,velocity}.sto
    (tests/golden/gso_norm_fiber_length.npz, tools/make_gso_fixture.py): the
    rigid-tendon normalized fiber lengths and velocities of the 9 right-leg
    muscles GlobalStaticOptimization computed from
    testGait10dof18musc_kinematics.mot, at the reference's own tolerance 1e-5
    (testGait10dof18musc.cpp:58-98, Testing.h:47-64).  Preprocessing restated
    from InverseMuscleSolverMotionData.cpp:49-114 (_gso_preprocess).
    Residual: the fiber velocity of the two muscles with MovingPathPoints
    (rect_fem_r, vasti_r) is off by up to 3.8e-5 within 0.03 s of the final
    time; every other velocity is within 5e-7 and every length within 2.7e-6.
    tools/gso_bisect.py (profiles/r06_gso) localizes it: at the golden times
    that coincide with samples (every 0.05 s) our lengths equal the golden
    ones up to a constant per-muscle offset to 1e-9 m, and per-sample length
    perturbations ONLY at the samples from t = 1.833 s on (the last two data
    rows and the padded rows after the data end) reproduce the window's
    errors to 6e-10 m -- the residual comes from how the end of the data
    enters the length spline, not from the path geometry at the golden times;
    no restated stage variant (pad, time pad, filter step / start, spline
    degree / end conditions / smoothing, selection) reproduces it."""
    nfl_err, nfv_err, t = _gso_errors(configs.gait10dof18musc_model())
    assert nfl_err.max() <= 1e-5, nfl_err.max(0)
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "gso_norm_fiber_length.npz"))
    moving = [i for i, l in enumerate(z["nfl_labels"][1:]) if l.split("/")[-1] in ("rect_fem_r", "vasti_r")]
    other = np.setdiff1d(np.arange(nfv_err.shape[1]), moving)
    assert nfv_err[:, other].max() <= 5e-7, nfv_err.max(0)
    assert nfv_err[t < 1.77][:, moving].max() <= 1e-5, nfv_err.max(0)
    assert nfv_err.max() <= 5e-5, nfv_err.max(0)
    # sensitivity: one vasti_r path point moved by 1 mm is far outside this
    m = configs.gait10dof18musc_model()
    vi = [mu.name for mu in m.muscles].index("vasti_r")
    p0 = m.muscles[vi].points[0]
    p0.loc = tuple(np.asarray(p0.loc, float) + [0.001, 0.0, 0.0])
    assert _gso_errors(m)[0].max() > 1e-4


def _gso_pad(x, p):
    """Storage::pad / Signal::Pad: p points at each end, reflected about the
    end point and negated (odd reflection)."""
    n = len(x)
    return np.concatenate([2 * x[0] - x[p:0:-1], x, 2 * x[-1] - x[n - 2:n - 2 - p:-1]])


def _gso_lowpass(dt, fc, sig):
    """Storage::lowpassIIR -> Signal::LowpassIIR: third-order Butterworth by
    the prewarped bilinear transform, run forward then backward, the first
    three outputs of each pass set to its inputs (no steady-state start)."""
    wa = math.tan(2 * math.pi * fc * dt / 2)
    wa2, wa3 = wa * wa, wa * wa * wa
    den = 1 + 2 * wa + 2 * wa2 + wa3
    b = np.array([wa3, 3 * wa3, 3 * wa3, wa3]) / den
    a = np.array([(-3 - 2 * wa + 2 * wa2 + 3 * wa3), (3 - 2 * wa - 2 * wa2 + 3 * wa3),
                  (-1 + 2 * wa - 2 * wa2 + wa3)]) / den

    def run(s):
        f = s.copy()
        for i in range(3, len(s)):
            f[i] = (b[0] * s[i] + b[1] * s[i - 1] + b[2] * s[i - 2] + b[3] * s[i - 3]
                    - a[0] * f[i - 1] - a[1] * f[i - 2] - a[2] * f[i - 3])
        return f
    return run(run(sig)[::-1])[::-1]


def _gso_errors(m):
    """|normalized fiber length / velocity - GSO golden| per (time,
    right-leg muscle), and the golden times.  InverseMuscleSolverMotionData:
    rows within [0.58 - 0.05, 1.8 + 0.05] s (:49-59), Storage::pad(size/2) and
    lowpassIIR at 6 Hz (:62-71; on the .mot's non-uniform 8-decimal times
    after resampling to the smallest step), muscle-tendon lengths at every padded row
    (:91-111), GCVSplineSet (degree 5, zero error variance: the interpolating
    natural quintic, mocohip.splines) evaluated and differentiated at the
    solution times (:249-290), then calcRigidTendonFiberKinematics
    (DeGrooteFregly2016MuscleStandalone.h:207-231)."""
    from mocohip.splines import gcv_interpolating_ppoly
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "gso_norm_fiber_length.npz"))
    kl, kin = list(z["kin_labels"]), z["kin"]
    gl, gso, gsv = list(z["nfl_labels"]), z["nfl"], z["nfv"]
    rep = MocoProblem(m).create_rep()
    nlp = OracleNLP(rep, MocoHipSolver(num_mesh_intervals=2).options())
    qnames = [n.split("/")[-2] for n in rep.state_names[:rep.nq]]
    t = kin[:, 0]
    sel = (t >= 0.58 - 0.05) & (t <= 1.8 + 0.05)
    t = t[sel]
    Q = np.stack([np.deg2rad(kin[sel, kl.index(q)]) if q not in ("pelvis_tx", "pelvis_ty")
                  else kin[sel, kl.index(q)] for q in qnames], 1)
    p = len(t) // 2
    tp = _gso_pad(t, p)
    Q = np.stack([_gso_pad(Q[:, j], p) for j in range(Q.shape[1])], 1)
    # the .mot's times are printed to 8 decimals, so its steps alternate
    # between 0.01666667 and 0.01666666: Storage::lowpassIIR on non-uniform
    # times resamples onto the uniform grid of the smallest step (degree-5 GCV
    # spline, Storage::resample) and filters with that step.  Restated so
    # (opensim-core is absent: inferred, tools/gso_bisect.py): it takes every
    # velocity but the two knee-crossing muscles' end window from 2.3e-6 to
    # 1.9e-7 of the golden file.
    dtmin = float(np.diff(tp).min())
    tn = tp[0] + np.arange(len(tp)) * dtmin
    brk, co = gcv_interpolating_ppoly(tp, Q, 5)
    seg = np.clip(np.searchsorted(brk, tn, side="right") - 1, 0, len(brk) - 2)
    Q = sum(co[seg, :, k] * (tn - brk[seg])[:, None] ** k for k in range(co.shape[2]))
    tp = tn
    Q = np.stack([_gso_lowpass(dtmin, 6.0, Q[:, j]) for j in range(Q.shape[1])], 1)
    names = [mu.name for mu in m.muscles]
    cols = [names.index(l.split("/")[-1]) for l in gl[1:]]
    L = np.zeros((len(tp), len(cols)))
    out = np.zeros(2)
    for i, q in enumerate(Q):
        q = np.ascontiguousarray(q)
        for c, im in enumerate(cols):
            assert lib.orc_muscle_length_speed(nlp.ctx, im, abi.dptr(q), abi.dptr(np.zeros(rep.nq)),
                                               abi.dptr(out)) == 0
            L[i, c] = out[0]
    brk, co = gcv_interpolating_ppoly(tp, L, 5)
    te = gso[:, 0]
    seg = np.clip(np.searchsorted(brk, te, side="right") - 1, 0, len(brk) - 2)
    dt = (te - brk[seg])[:, None]
    Lg = sum(co[seg, :, k] * dt ** k for k in range(co.shape[2]))
    Vg = sum(k * co[seg, :, k] * dt ** (k - 1) for k in range(1, co.shape[2]))
    nfl = np.empty_like(Lg)
    nfv = np.empty_like(Lg)
    for c, im in enumerate(cols):
        mu = m.muscles[im]
        w = mu.optimal_fiber_length * math.sin(mu.pennation_angle_at_optimal)
        along = Lg[:, c] - mu.tendon_slack_length
        fl = np.sqrt(along ** 2 + w * w)
        nfl[:, c] = fl / mu.optimal_fiber_length
        nfv[:, c] = Vg[:, c] * (along / fl) / (mu.max_contraction_velocity * mu.optimal_fiber_length)
    return np.abs(nfl - gso[:, 1:]), np.abs(nfv - gsv[:, 1:]), te


# ---- implicit multibody dynamics ----------------------------

@pytest.mark.parametrize("case", ["double_pendulum", "gait_rigid", "gait_compliant"])
def test_implicit_residual_vanishes_at_explicit_accelerations(case):
    """calcMultibodySystemImplicit (MocoCasOCProblem.h:245-297): the residual
    findMotionForces returns is M w + C - f_applied, zero exactly when w is
    the forward-dynamics udot; zdot is the same as in explicit mode."""
    mk = {"double_pendulum": lambda d: configs.double_pendulum(3, dynamics=d),
          "gait_rigid": lambda d: configs.gait10dof18musc(3, dynamics=d),
          "gait_compliant": lambda d: configs.gait10dof18musc(3, tendon_compliance=True, dynamics=d)}[case]
    ex = OracleNLP(mk("explicit").problem.create_rep(), mk("explicit").solver.options())
    st = mk("implicit")
    im = OracleNLP(st.problem.create_rep(), st.solver.options())
    assert im.NDV == im.NQ and ex.NDV == 0
    xm = ex.initial_guess_from_bounds()
    rng = np.random.default_rng(11)
    NQ, NS, NC = ex.NQ, ex.NS, ex.NC
    for k in range(4):
        s_ = xm[2 + k * NS:2 + (k + 1) * NS].copy()
        s_[:2 * NQ] += rng.uniform(-0.2, 0.2, 2 * NQ)
        c_ = rng.uniform(0.05, 0.5, NC)
        P = np.concatenate([[0.3], s_, c_])[None, :]
        y = ex.eval_dae(P)[0]
        r = im.eval_dae(np.concatenate([P[0], y[:NQ]])[None, :])[0]
        scale = 1.0 + np.abs(y[:NQ]).max()
        assert np.abs(r[:NQ]).max() < 1e-9 * scale, r[:NQ]
        assert np.array_equal(r[NQ:], y[NQ:])
        w2 = y[:NQ] + 0.1
        r2 = im.eval_dae(np.concatenate([P[0], w2])[None, :])[0]
        assert np.abs(r2[:NQ]).max() > 1e-3


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
def test_implicit_layout_bounds_and_structure(scheme):
    """Derivative variables after the controls with [-1000, 1000] bounds
    (CasOCTranscription.cpp:134-135,222-226); residual rows of each interval's
    grid points before its defects and the final point's residual last
    (CasOCTranscription.h:219-313); speed defects depend on the derivative
    variables only (udot = w, :339-341)."""
    N = 4
    st = configs.double_pendulum(N, scheme, dynamics="implicit")
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    NQ, NS, NC, G = nlp.NQ, nlp.NS, nlp.NC, nlp.G
    hs = scheme == "hermite-simpson"
    assert nlp.n == 2 + (NS + NC + NQ) * G
    rpi = (2 * NQ + 2 * NS + NC) if hs else (NQ + NS)
    assert nlp.m == N * rpi + NQ
    xl, xu, gl, gu = nlp.bounds()
    d0 = 2 + (NS + NC) * G
    assert np.all(xl[d0:] == -1000) and np.all(xu[d0:] == 1000)
    ir, jc = nlp.jac_structure()
    S = set(zip(ir.tolist(), jc.tolist()))
    x = nlp.random_iterate(np.random.default_rng(1).uniform(-1, 1, nlp.n))
    x[1] = 2.0
    g0 = nlp.eval_g(x)
    for j in range(nlp.n):
        xp = x.copy()
        xp[j] += 1e-3
        for r in np.nonzero(nlp.eval_g(xp) != g0)[0]:
            assert (int(r), j) in S
    # residual rows at the final grid point depend on its inputs and the time
    tail = set(jc[ir == nlp.m - 1].tolist())
    assert {0, 1} <= tail and 2 + (G - 1) * NS in tail and d0 + (G - 1) * NQ in tail


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
def test_implicit_jacobian_matches_numerical_derivative(scheme):
    st = configs.double_pendulum(3, scheme, dynamics="implicit")
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(2).uniform(-1, 1, nlp.n))
    x[1] = 1.5
    d0 = 2 + (nlp.NS + nlp.NC) * nlp.G
    x[d0:] *= 1e-2      # accelerations of O(10): FD noise eps*|residual|/h stays < 1e-6
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    Jn = _numjac(nlp.eval_g, x, range(nlp.n))
    # h = 1e-8 differences carry ~eps*|g|/h of rounding noise (|g| ~ 1e3 here)
    noise = 100 * np.finfo(float).eps * np.abs(nlp.eval_g(x)).max() / st.solver.fd_step
    assert np.allclose(J, Jn, rtol=1e-5, atol=max(1e-6, noise))
    gf = nlp.eval_grad_f(x)
    gn = _numjac(lambda z: np.array([nlp.eval_f(z)]), x, range(nlp.n))[0]
    assert np.allclose(gf, gn, rtol=1e-6, atol=1e-7)


# --------------------------------------------------------------------------
# Path constraints: MocoControlBoundConstraint.
# --------------------------------------------------------------------------
def _bound_value(f, t):
    from mocohip.problem import Constant
    if isinstance(f, Constant):
        return np.full_like(np.asarray(t, float), f.value)
    br, cf = f.ppoly()
    return ppoly_eval(br, cf, np.asarray(t, float), 0)


@pytest.mark.parametrize("section,scheme", [("lower", "hermite-simpson"), ("upper", "trapezoidal"),
                                            ("equality", "trapezoidal"), ("both", "hermite-simpson"),
                                            ("both", "trapezoidal")])
def test_path_constraint_layout_bounds_values(section, scheme):
    """Path rows open every mesh interval and the tail (flattenConstraints,
    CasOCTranscription.h:286-311); bounds [0, inf] / [-inf, 0] / [0, 0]
    repeated per mesh point (MocoControlBoundConstraint.cpp:99-118,
    CasOCTranscription.cpp:429-432); values control - bound(t) (:130-146);
    rows block-dense over t0, tf and the mesh point's inputs."""
    N = 6
    st = configs.pendulum_control_bound(N, section, scheme)
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    pc = st.problem.path_constraints[0]
    npc = {"lower": 1, "upper": 1, "equality": 1, "both": 2}[section]
    assert rep.num_path_equations == nlp.NPC == npc
    hs = scheme == "hermite-simpson"
    NS, NC, G = nlp.NS, nlp.NC, nlp.G
    rpi = npc + (2 * NS + NC if hs else NS)
    assert nlp.m == N * rpi + npc and nlp.tail_rows == npc
    x = nlp.random_iterate(np.random.default_rng(3).uniform(-1, 1, nlp.n))
    g = nlp.eval_g(x)
    xl, xu, gl, gu = nlp.bounds()
    fns = [f for f in (pc.lower_bound, pc.upper_bound) if f is not None]
    step = 2 if hs else 1
    grid = np.arange(G) / (G - 1)
    t = (x[1] - x[0]) * grid + x[0]
    ir, jc = nlp.jac_structure()
    for i in range(N + 1):
        k = i * step
        u = x[2 + NS * G + k * NC]
        for e, f in enumerate(fns):
            r = i * rpi + e
            assert g[r] == pytest.approx(u - _bound_value(f, t[k]), abs=1e-13)
            lo, hi = ((0.0, 0.0) if pc.equality_with_lower else
                      (0.0, np.inf) if f is pc.lower_bound else (-np.inf, 0.0))
            assert (gl[r], gu[r]) == (lo, hi)
            cols = jc[ir == r].tolist()
            pts = [2 + k * NS + s for s in range(NS)] + [2 + NS * G + k * NC + j for j in range(NC)]
            assert cols == [0, 1] + pts
    # every other row is an equality
    path_rows = {i * rpi + e for i in range(N + 1) for e in range(npc)}
    others = np.array([r for r in range(nlp.m) if r not in path_rows])
    assert np.all(gl[others] == 0) and np.all(gu[others] == 0)


@pytest.mark.parametrize("section,scheme,dynamics", [("equality", "hermite-simpson", "explicit"),
                                                     ("both", "trapezoidal", "explicit"),
                                                     ("both", "hermite-simpson", "implicit")])
def test_path_constraint_jacobian_matches_numerical_derivative(section, scheme, dynamics):
    st = configs.pendulum_control_bound(4, section, scheme, dynamics)
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(2).uniform(-1, 1, nlp.n))
    if nlp.NDV:
        x[2 + (nlp.NS + nlp.NC) * nlp.G:] *= 1e-2
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    Jn = _numjac(nlp.eval_g, x, range(nlp.n))
    noise = 100 * np.finfo(float).eps * max(np.abs(nlp.eval_g(x)).max(), 1.0) / st.solver.fd_step
    assert np.allclose(J, Jn, rtol=1e-5, atol=max(1e-6, noise))


def test_path_constraint_rejections():
    """initializeOnModel checks (MocoControlBoundConstraint.cpp:53-93) and
    "Time range of bounds function is too small" (testConstraints.cpp)."""
    from mocohip.problem import GCVSpline, MocoControlBoundConstraint, Constant
    st = configs.pendulum_control_bound(4, "lower")
    p = st.problem
    p.path_constraints[0].control_paths.append("/nonexistent")
    with pytest.raises(ValueError, match="no such control"):
        p.create_rep()
    p.path_constraints[0].control_paths.pop()
    p.path_constraints[0].set_upper_bound(Constant(1.0))
    p.path_constraints[0].set_equality_with_lower(True)
    with pytest.raises(ValueError, match="upper bound function must not be set"):
        p.create_rep()
    p.path_constraints = []
    p.set_time_bounds((-31, 0), (1, 50))
    c = p.add_path_constraint(MocoControlBoundConstraint())
    c.add_control_path("/tau0")
    c.set_lower_bound(GCVSpline(5, [-30.9999, 0, 0.5, 0.7, 0.8, 0.9, 50], [0, 0, 0, 0, 0, 0, 0.319]))
    with pytest.raises(ValueError, match="must be less than or equal to the minimum"):
        p.create_rep()
    c.lower_bound = None
    c.set_upper_bound(GCVSpline(5, [-31, 0, 0.5, 0.7, 0.8, 0.9, 49.99999], [0, 0, 0, 0, 0, 0, .0319]))
    with pytest.raises(ValueError, match="must be greater than or equal to the maximum"):
        p.create_rep()
    # "Can omit both bounds": a constraint without bounds adds no rows
    c.upper_bound = None
    assert p.create_rep().num_path_equations == 0


def test_gait_path_constraints_layout():
    st = configs.gait10dof18musc(4, control_bounds=True)
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    base = OracleNLP(configs.gait10dof18musc(4).problem.create_rep(), st.solver.options())
    npc = rep.num_path_equations
    assert npc == 2 * 2 + 1
    assert nlp.m == base.m + 5 * npc and nlp.n == base.n
    assert nlp.nnz == base.nnz + 5 * npc * (2 + nlp.NS + nlp.NC)
    # the DAE is untouched: same model hash inputs, same defects
    x = base.random_iterate(np.random.default_rng(0).uniform(-1, 1, base.n))
    g, g0 = nlp.eval_g(x), base.eval_g(x)
    rpi, rpi0 = (nlp.m - npc) // 4, base.m // 4
    for i in range(4):
        assert np.array_equal(g[i * rpi + npc:(i + 1) * rpi], g0[i * rpi0:(i + 1) * rpi0])


# --------------------------------------------------------------------------
# Sparsity detection: optim_sparsity_detection.
# --------------------------------------------------------------------------
SPARSE_CASES = {
    "double_pendulum": lambda: configs.double_pendulum(3),
    "double_pendulum_trap_implicit": lambda: configs.double_pendulum(3, "trapezoidal", dynamics="implicit"),
    "gait_rigid": lambda: configs.gait10dof18musc(2),
    "gait_compliant": lambda: configs.gait10dof18musc(2, tendon_compliance=True),
    "gait_implicit_pathcon": lambda: configs.gait10dof18musc(2, dynamics="implicit", control_bounds=True),
    "pendulum_bound": lambda: configs.pendulum_control_bound(3, "both"),
}


def _grid0_inputs(nlp, x):
    G = nlp.G
    st = x[2:2 + nlp.NS]
    ct = x[2 + nlp.NS * G:2 + nlp.NS * G + nlp.NC]
    dv = x[2 + (nlp.NS + nlp.NC) * G:2 + (nlp.NS + nlp.NC) * G + nlp.NDV]
    return np.concatenate([[x[0]], st, ct, dv])


def _replicated_iterate(nlp, seed=6):
    """A random iterate whose grid points all hold grid point 0's values, so
    that detection at grid point 0 sees every grid point's dependencies."""
    x = nlp.random_iterate(np.random.default_rng(seed).uniform(-1, 1, nlp.n))
    G = nlp.G
    off = 2
    for width in (nlp.NS, nlp.NC, nlp.NDV):
        if width:
            blk = x[off:off + width * G].reshape(G, width)
            blk[:] = blk[0]
        off += width * G
    return x


@pytest.mark.parametrize("rule", ["any-change", "robust"])
@pytest.mark.parametrize("name", list(SPARSE_CASES))
def test_sparsity_detection_initial_guess(name, rule):
    """Detected rows are a subset of the block-dense rows with the same
    finite-difference values, and every dropped entry is zero to rounding
    noise at the detection iterate; with the reference's rule
    (CasOCFunction.cpp:25-71: any change) exactly zero (>= 99 %), with the
    robust rule the rounding-level couplings it drops too."""
    st = SPARSE_CASES[name]()
    st.solver.optim_finite_difference_scheme = "forward"
    st.solver.optim_sparsity_detection_rule = rule
    rep = st.problem.create_rep()
    dense = OracleNLP(rep, st.solver.options())
    x = _replicated_iterate(dense)
    st.solver.optim_sparsity_detection = "initial-guess"
    st.solver.sparsity_guess = x
    sp = OracleNLP(rep, st.solver.options())
    assert (sp.n, sp.m) == (dense.n, dense.m) and sp.nnz <= dense.nnz
    ir, jc = dense.jac_structure()
    irs, jcs = sp.jac_structure()
    where = {(int(r), int(c)): i for i, (r, c) in enumerate(zip(ir, jc))}
    idx = np.array([where[(int(r), int(c))] for r, c in zip(irs, jcs)])
    assert np.all(np.diff(idx) > 0)          # same row-major order
    J, Js = dense.eval_jac_g(x), sp.eval_jac_g(x)
    assert np.array_equal(J[idx], Js, equal_nan=True)
    dropped = np.setdiff1d(np.arange(dense.nnz), idx)
    # a dropped entry is zero up to the rounding noise a 1e-8 difference
    # quotient picks up (eps |y| / h_fd, y the DAE outputs) where the 1e-5
    # detection perturbation left the output bit-identical
    P = _grid0_inputs(dense, x)
    F = max(np.abs(dense.eval_dae(P[None, :])).max(), 1.0)
    noise = 64 * np.finfo(float).eps * F / st.solver.fd_step * max(x[1] - x[0], 1.0)
    assert np.all(np.abs(np.nan_to_num(J[dropped])) <= noise)
    if rule == "any-change":
        assert np.mean(J[dropped] == 0) > 0.99
    assert np.array_equal(sp.eval_g(x), dense.eval_g(x), equal_nan=True)
    xl, xu, gl, gu = sp.bounds()
    assert all(np.array_equal(a, b) for a, b in zip((xl, xu, gl, gu), dense.bounds()))


def test_sparsity_detection_random_is_deterministic_and_smaller():
    """"random": 3 iterates from a fixed seed (CasOCSolver.cpp:76-86), so the
    pattern is the same every time; the gait model's tree and muscle paths
    leave most of each block empty."""
    st = configs.gait10dof18musc(3)
    st.solver.optim_sparsity_detection = "random"
    rep = st.problem.create_rep()
    a, b = OracleNLP(rep, st.solver.options()), OracleNLP(rep, st.solver.options())
    assert np.array_equal(a.jac_structure()[0], b.jac_structure()[0])
    assert np.array_equal(a.jac_structure()[1], b.jac_structure()[1])
    st.solver.optim_sparsity_detection = "none"
    dense = OracleNLP(rep, st.solver.options())
    assert a.nnz < dense.nnz / 2
    with pytest.raises(ValueError):
        st.solver.optim_sparsity_detection = "bogus"
        st.solver.options()


# --------------------------------------------------------------------------
# Implicit tendon dynamics: DGF tendon_compliance_dynamics_mode
# "implicit".
# --------------------------------------------------------------------------
def _physio_point(nlp, rep):
    """[t, states, controls] at the bounds midpoint with activations 0.5 and
    normalized tendon forces 0.1 (a regular point of the DGF model)."""
    x = nlp.initial_guess_from_bounds()
    st = x[2:2 + nlp.NS].copy()
    for i, n in enumerate(rep.state_names):
        if n.endswith("/activation"):
            st[i] = 0.5
        elif n.endswith("/normalized_tendon_force"):
            st[i] = 0.1
    ct = np.random.default_rng(3).uniform(0.05, 0.3, nlp.NC)
    return np.concatenate([[0.3], st, ct])


@pytest.mark.parametrize("dynamics", ["explicit", "implicit"])
def test_implicit_tendon_residual_vanishes_at_explicit_derivative(dynamics):
    """The equilibrium residual FT - FM cos(alpha) (DeGrooteFregly2016Muscle
    .cpp:826-848) is zero when the derivative variable equals the explicit
    model's normalized tendon force derivative (.cpp:211-232), and the other
    outputs agree; a perturbed derivative gives a nonzero residual."""
    ex_st = configs.gait10dof18musc(2, tendon_compliance=True, dynamics=dynamics)
    im_st = configs.gait10dof18musc(2, tendon_compliance=True, dynamics=dynamics,
                                    tendon_dynamics="implicit")
    # the explicit form inverts the force-velocity curve without the fiber
    # damping term (.cpp:285-292), so the two agree exactly only undamped
    for s_ in (ex_st, im_st):
        for mu in s_.problem.model.muscles:
            mu.fiber_damping = 0.0
    ex_rep, im_rep = ex_st.problem.create_rep(), im_st.problem.create_rep()
    ex = OracleNLP(ex_rep, ex_st.solver.options())
    im = OracleNLP(im_rep, im_st.solver.options())
    assert im.NAR == 18 and ex.NAR == 0 and im.NDV == ex.NDV + 18
    P = _physio_point(ex, ex_rep)
    acc = np.random.default_rng(5).uniform(-1, 1, ex.NACC)
    Yx = ex.eval_dae(np.concatenate([P, acc])[None, :])[0]
    NQ, NZ = ex.NQ, ex.NS - 2 * ex.NQ
    ftn_idx = [i for i, n in enumerate(ex_rep.state_names) if n.endswith("/normalized_tendon_force")]
    dft = Yx[[i - NQ for i in ftn_idx]]          # explicit zdot of the tendon states
    Yi = im.eval_dae(np.concatenate([P, acc, dft])[None, :])[0]
    assert Yi.shape == (NQ + NZ + 18,)
    fmax = max(m.max_isometric_force for m in im_st.problem.model.muscles)
    assert np.all(np.abs(Yi[NQ + NZ:]) <= 1e-9 * fmax), np.abs(Yi[NQ + NZ:]).max()
    assert np.allclose(Yi[:NQ + NZ], Yx, rtol=1e-9, atol=1e-9)
    Yp = im.eval_dae(np.concatenate([P, acc, dft + 0.05])[None, :])[0]
    assert np.all(np.abs(Yp[NQ + NZ:]) > 1e-6)


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
def test_implicit_tendon_layout_bounds_and_jacobian(scheme):
    """Derivative variables [accelerations, tendon-force derivatives] with
    implicit_auxiliary_derivative_bounds (CasOCTranscription.cpp:222-232);
    auxiliary residual rows after the multibody residuals at every grid
    point and in the tail (CasOCTranscription.h:286-311); Jacobian vs a
    numerical derivative of eval_g at a regular iterate."""
    N = 2
    st = configs.gait10dof18musc(N, tendon_compliance=True, dynamics="implicit",
                                 tendon_dynamics="implicit")
    st.solver.transcription_scheme = scheme
    st.solver.implicit_auxiliary_derivative_bounds = (-50.0, 60.0)
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    NQ, NS, NC, G = nlp.NQ, nlp.NS, nlp.NC, nlp.G
    assert nlp.NDV == NQ + 18 and nlp.NRES == NQ + 18
    assert nlp.n == 2 + (NS + NC + NQ + 18) * G
    xl, xu, _, _ = nlp.bounds()
    d0 = 2 + (NS + NC) * G
    D = (xl[d0:].reshape(G, NQ + 18), xu[d0:].reshape(G, NQ + 18))
    assert np.all(D[0][:, :NQ] == -1000) and np.all(D[1][:, NQ:] == 60) and np.all(D[0][:, NQ:] == -50)
    hs = scheme == "hermite-simpson"
    rpi = (2 if hs else 1) * nlp.NRES + (2 * NS + NC if hs else NS)
    assert nlp.m == N * rpi + nlp.NRES
    # regular iterate: the physiological point at every grid point
    P = _physio_point(nlp, rep)
    x = nlp.initial_guess_from_bounds()
    x[2:2 + NS * G] = np.tile(P[1:1 + NS], G)
    x[2 + NS * G:2 + (NS + NC) * G] = np.tile(P[1 + NS:], G)
    x[d0:] = np.random.default_rng(8).uniform(-0.5, 0.5, (NQ + 18) * G)
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    cols = sorted(set(range(0, nlp.n, 7)) | {0, 1, d0, d0 + NQ, nlp.n - 1})
    Jn = _numjac(nlp.eval_g, x, cols, h=1e-5)
    noise = 100 * np.finfo(float).eps * np.abs(nlp.eval_g(x)).max() / st.solver.fd_step
    assert np.allclose(J[:, cols], Jn, rtol=1e-4, atol=max(1e-5, noise))


# --------------------------------------------------------------------------
# Prescribed kinematics: PositionMotion / MocoInverse.
# --------------------------------------------------------------------------
def test_prescribed_kinematics_layout_and_equivalence():
    """With a PositionMotion the coordinates are not NLP states
    (MocoProblemRep.cpp:541-555), there are no acceleration variables and
    every grid point has nq multibody residual rows (CasOCProblem.h:486-503)
    plus the implicit tendon residuals.  The callback equals the implicit
    one evaluated at q(t), dq/dt, d2q/dt2 of the same spline (PositionMotion
    .cpp:36-70), bit for bit."""
    from mocohip.splines import gcv_interpolating_ppoly
    N = 3
    inv = configs.gait10dof18musc_inverse(N, sparsity="none")
    rep = inv.problem.create_rep()
    nlp = OracleNLP(rep, inv.solver.options())
    assert all(not (n.endswith("/value") or n.endswith("/speed")) for n in rep.state_names)
    NZ, NC, G, NQ = nlp.NS, nlp.NC, nlp.G, nlp.NQ
    assert (nlp.TQ, nlp.NACC, nlp.NMB, nlp.NAR) == (0, 0, NQ, 18)
    assert nlp.n == 2 + (NZ + NC + 18) * G
    # MocoInverse: no control-midpoint interpolation rows (MocoInverse.cpp:105);
    # one initial-activation endpoint row per muscle first (MocoInverse.cpp:93)
    rpi = 2 * (NQ + 18) + 2 * NZ
    assert nlp.m == 18 + N * rpi + NQ + 18
    # the equivalent implicit problem (q, u states, accelerations)
    imp = configs.gait10dof18musc(N, tendon_compliance=True, tendon_dynamics="implicit",
                                  dynamics="implicit")
    irep = imp.problem.create_rep()
    inlp = OracleNLP(irep, imp.solver.options())
    kin = inv.problem.position_motion
    qpaths = [c.path + "/value" for c in inv.problem.model.coordinates()]
    br, cf = gcv_interpolating_ppoly(kin.times, np.stack([kin.columns[q] for q in qpaths], 1), 5)
    t = 0.731
    s = np.clip(np.searchsorted(br, t, side="right") - 1, 0, len(br) - 2)
    dt = t - br[s]
    pw = np.array([dt ** k for k in range(6)])
    q = cf[s] @ pw
    u = cf[s] @ np.array([k * dt ** (k - 1) if k else 0.0 for k in range(6)])
    w = cf[s] @ np.array([k * (k - 1) * dt ** (k - 2) if k > 1 else 0.0 for k in range(6)])
    z = np.where([n.endswith("activation") for n in rep.state_names], 0.4, 0.12)
    ctl = np.random.default_rng(1).uniform(0.0, 0.3, NC)
    dft = np.random.default_rng(2).uniform(-0.5, 0.5, 18)
    Yp = nlp.eval_dae(np.concatenate([[t], z, ctl, dft])[None, :])[0]
    Yi = inlp.eval_dae(np.concatenate([[t], q, u, z, ctl, w, dft])[None, :])[0]
    assert np.allclose(Yp, Yi, rtol=1e-10, atol=1e-8 * max(1.0, np.abs(Yi).max()))
    with pytest.raises(RuntimeError, match="requires implicit"):
        inv.solver.multibody_dynamics_mode = "explicit"
        OracleNLP(rep, inv.solver.options())


def test_prescribed_kinematics_jacobian_matches_numerical_derivative():
    inv = configs.gait10dof18musc_inverse(2, sparsity="none")
    rep = inv.problem.create_rep()
    nlp = OracleNLP(rep, inv.solver.options())
    x = nlp.initial_guess_from_bounds()
    G, NZ, NC = nlp.G, nlp.NS, nlp.NC
    S = x[2:2 + NZ * G].reshape(G, NZ)
    for i, n in enumerate(rep.state_names):
        S[:, i] = 0.5 if n.endswith("/activation") else 0.1
    x[2 + NZ * G:2 + (NZ + NC) * G] = np.random.default_rng(4).uniform(0.05, 0.3, NC * G)
    d0 = 2 + (NZ + NC) * G
    x[d0:] = np.random.default_rng(5).uniform(-0.3, 0.3, nlp.n - d0)
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    cols = sorted(set(range(0, nlp.n, 5)) | {0, 1, d0, nlp.n - 1})
    Jn = _numjac(nlp.eval_g, x, cols, h=1e-5)
    noise = 100 * np.finfo(float).eps * np.abs(nlp.eval_g(x)).max() / inv.solver.fd_step
    assert np.allclose(J[:, cols], Jn, rtol=1e-4, atol=max(1e-5, noise))


def test_implicit_auxiliary_derivatives_term():
    """minimize_implicit_auxiliary_derivatives (CasOCTranscription.cpp:534-545):
    weight * duration * sum_k quad_k * sum_j w_jk^2, here on top of the
    MocoInverse control effort; gradient vs numerical derivative."""
    inv = configs.gait10dof18musc_inverse(3, sparsity="none")
    rep = inv.problem.create_rep()
    nlp = OracleNLP(rep, inv.solver.options())
    x = nlp.initial_guess_from_bounds()
    G, NZ, NC = nlp.G, nlp.NS, nlp.NC
    x[2 + NZ * G:2 + (NZ + NC) * G] = np.random.default_rng(1).uniform(0, 0.3, NC * G)
    d0 = 2 + (NZ + NC) * G
    W = np.random.default_rng(2).uniform(-2, 2, (G, 18))
    x[d0:] = W.reshape(-1)
    f = nlp.eval_f(x)
    dur = x[1] - x[0]
    quad = np.zeros(G)
    for i in range(3):
        dm = 1.0 / 3
        quad[2 * i] += dm / 6; quad[2 * i + 1] += 2 * dm / 3; quad[2 * i + 2] += dm / 6
    U = x[2 + NZ * G:2 + (NZ + NC) * G].reshape(G, NC)
    expect = dur * quad @ (U ** 2).sum(1) + 0.01 * dur * quad @ (W ** 2).sum(1)
    assert f == pytest.approx(expect, rel=1e-12)
    gf = nlp.eval_grad_f(x)
    cols = list(range(d0, nlp.n, 7))
    gn = _numjac(lambda z: np.array([nlp.eval_f(z)]), x, cols, h=1e-5)[0]
    assert np.allclose(gf[cols], gn, rtol=1e-6, atol=1e-8)


# ---------------------------------------------------------------------------
# Endpoint constraints (MocoInitialActivationGoal, MocoInverse.cpp:93) and the
# MocoInverse layout without control-midpoint interpolation (MocoInverse.cpp:105)
# ---------------------------------------------------------------------------
def _inverse(N, sparsity="none", scheme="hermite-simpson"):
    st = configs.gait10dof18musc_inverse(N, sparsity=sparsity)
    st.solver.transcription_scheme = scheme
    rep = st.problem.create_rep()
    return st, rep, OracleNLP(rep, st.solver.options())


def _inverse_iterate(nlp, seed=0):
    r = np.random.default_rng(seed)
    x = nlp.initial_guess_from_bounds()
    G, NS, NC = nlp.G, nlp.NS, nlp.NC
    S = x[2:2 + NS * G].reshape(G, NS)
    for i, n in enumerate(nlp.rep.state_names):
        S[:, i] = r.uniform(0.2, 0.6, G) if n.endswith("/activation") else r.uniform(0.05, 0.3, G)
    x[2 + NS * G:2 + (NS + NC) * G] = r.uniform(0.05, 0.4, NC * G)
    d0 = 2 + (NS + NC) * G
    x[d0:] = r.uniform(-0.5, 0.5, nlp.n - d0)
    return x


@pytest.mark.parametrize("sparsity", ["none", "random"])
def test_initial_activation_endpoint_rows(sparsity):
    """One endpoint row per muscle with activation dynamics, ahead of every
    mesh point's rows (flattenConstraints, CasOCTranscription.h:283-285),
    bounds [0, 0] (MocoConstraintInfo.h:44-54), value initial excitation -
    initial activation (MocoInitialActivationGoal.cpp:41-58).  Without
    detection the row is dense over the Endpoint callback's inputs (t0, the
    initial point, tf, the final point; CasOCFunction.h:167-240); with it,
    exactly the two columns the function reads."""
    st, rep, nlp = _inverse(3, sparsity)
    NEP, G, NS, NC, NDV = 18, nlp.G, nlp.NS, nlp.NC, nlp.NDV
    assert nlp.NEP == NEP
    ir, jc = nlp.jac_structure()
    nhead = int((ir < NEP).sum())
    assert np.all(ir[:nhead] < NEP) and np.all(ir[nhead:] >= NEP)
    assert np.all(np.diff(ir[:nhead]) >= 0)
    sidx = {n: i for i, n in enumerate(rep.state_names)}
    cidx = {n: i for i, n in enumerate(rep.control_names)}
    muscles = [m for m in st.problem.model.muscles if not m.ignore_activation_dynamics]
    W = 1 + NS + NC + NDV

    def pt_cols(k):
        return ([2 + k * NS + s for s in range(NS)] + [2 + NS * G + k * NC + j for j in range(NC)]
                + [2 + (NS + NC) * G + k * NDV + j for j in range(NDV)])
    dense = sorted([0, 1] + pt_cols(0) + pt_cols(G - 1))
    x = _inverse_iterate(nlp)
    g, J = nlp.eval_g(x), nlp.eval_jac_g(x)
    xl, xu, gl, gu = nlp.bounds()
    for e, mu in enumerate(muscles):
        cols = jc[:nhead][ir[:nhead] == e]
        a_col = 2 + sidx[mu.path + "/activation"]
        e_col = 2 + NS * G + cidx[mu.path]
        if sparsity == "none":
            assert list(cols) == dense and len(cols) == 2 * W
        else:
            assert list(cols) == sorted([a_col, e_col])
        assert g[e] == x[e_col] - x[a_col]
        assert gl[e] == 0.0 and gu[e] == 0.0
        vals = dict(zip(cols, J[:nhead][ir[:nhead] == e]))
        assert abs(vals[e_col] - 1.0) < 1e-7 and abs(vals[a_col] + 1.0) < 1e-7
        assert all(v == 0.0 for c, v in vals.items() if c not in (a_col, e_col))


def test_initial_activation_pinned_by_reference_golden_row():
    """The reference's converged MocoInverse solution
    (Moco/Tests/std_testMocoInverse_subject_18musc_solution.sto, fixture
    tests/golden/inverse_initial_activation.npz) has initial excitation ==
    initial activation for each of its 18 muscles: the endpoint rows vanish
    there, and our MocoInverse transcription has one such row per muscle."""
    d = np.load(os.path.join(GOLDEN, "inverse_initial_activation.npz"))
    assert len(d["muscles"]) == 18
    assert np.array_equal(d["excitation"], d["activation"])
    st, rep, nlp = _inverse(2)
    x = _inverse_iterate(nlp)
    sidx = {n: i for i, n in enumerate(rep.state_names)}
    cidx = {n: i for i, n in enumerate(rep.control_names)}
    muscles = [m for m in st.problem.model.muscles if not m.ignore_activation_dynamics]
    assert len(muscles) == len(d["muscles"])
    for mu, ex, ac in zip(muscles, d["excitation"], d["activation"]):
        x[2 + sidx[mu.path + "/activation"]] = ac
        x[2 + nlp.NS * nlp.G + cidx[mu.path]] = ex
    assert np.all(nlp.eval_g(x)[:18] == 0.0)


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
def test_inverse_layout_without_interp_and_jacobian(scheme):
    """interpolate_control_midpoints = false (MocoInverse.cpp:105): no
    interp rows; the whole Jacobian (endpoint head included) matches a
    numerical derivative of eval_g."""
    st, rep, nlp = _inverse(2, scheme=scheme)
    st.solver.optim_finite_difference_scheme = "central"   # O(h^2) truncation for the check
    nlp = OracleNLP(rep, st.solver.options())
    NQ, NS, NAR, N = nlp.NQ, nlp.NS, 18, 2
    npts = 2 if scheme == "hermite-simpson" else 1
    ndef = 2 * NS if scheme == "hermite-simpson" else NS
    assert nlp.m == 18 + N * (npts * (NQ + NAR) + ndef) + NQ + NAR
    st.solver.interpolate_control_midpoints = True
    with_interp = OracleNLP(rep, st.solver.options())
    assert with_interp.m == nlp.m + (N * nlp.NC if scheme == "hermite-simpson" else 0)
    x = _inverse_iterate(nlp, 3)
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    J[ir, jc] = nlp.eval_jac_g(x)
    cols = np.unique(jc)
    Jn = _numjac(nlp.eval_g, x, cols)
    # central FD at h=1e-8: eps|f|/h rounding relative to the row's scale
    scale = np.abs(Jn).max(1, keepdims=True) + 1.0
    err = np.abs(J[:, cols] - Jn) / scale
    assert err.max() <= 1e-6, err.max()


@pytest.mark.parametrize("case", ["pendulum_hs_forward", "pendulum_trap_central", "gait_backward",
                                  "gait_implicit_pathcon", "inverse_random"])
def test_assembly_from_lanes_equals_eval_jac_g(case):
    """orc_assemble_from_lanes (the checker of the device's quotient +
    assembly arithmetic) fed with the oracle's own DAE at the lane inputs of
    mh_debug_jacobian_lanes' layout reproduces orc_eval_g / orc_eval_jac_g
    bit for bit: the lane layout, the FD quotients (CasOCFunction.h:38-44)
    and the transcription chain rule agree with the direct evaluation."""
    import _lanes
    st = {"pendulum_hs_forward": lambda: configs.double_pendulum(5),
          "pendulum_trap_central": lambda: configs.double_pendulum(4, "trapezoidal"),
          "gait_backward": lambda: configs.gait10dof18musc(2, fd_scheme="backward"),
          "gait_implicit_pathcon": lambda: configs.gait10dof18musc(2, dynamics="implicit",
                                                                  control_bounds=True),
          "inverse_random": lambda: configs.gait10dof18musc_inverse(2)}[case]()
    if case == "pendulum_hs_forward":
        st.solver.optim_finite_difference_scheme = "forward"
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options(), threads=4)
    x = (_inverse_iterate(nlp, 5) if case == "inverse_random"
         else nlp.random_iterate(np.random.default_rng(4).uniform(-1, 1, nlp.n)))
    t = _lanes.oracle_times(nlp, x)
    Y = _lanes.oracle_lanes(nlp, x, t)
    g, J = nlp.assemble_from_lanes(x, t, Y)
    assert np.array_equal(g, nlp.eval_g(x), equal_nan=True)
    assert np.array_equal(J, nlp.eval_jac_g(x), equal_nan=True)


# ------------------------------------------------ MocoMarkerFinalGoal ----
def _pendulum_tip(q0, q1):
    """/markerset/marker1 of ModelFactory::createNLinkPendulum(2) in ground:
    body i's origin sits 1 m along its x axis from its pin (ModelFactory.cpp:
    60-75), so the tip is (cos q0 + cos(q0+q1), sin q0 + sin(q0+q1), 0)."""
    return np.array([math.cos(q0) + math.cos(q0 + q1), math.sin(q0) + math.sin(q0 + q1), 0.0])


@pytest.mark.parametrize("fd", ["forward", "central", "backward"])
def test_marker_final_goal_closed_form_and_gradient(fd):
    """testImplicit.cpp:76-79: weight 1000 on |marker1(tf) - (0, 2, 0)|^2
    (MocoMarkerFinalGoal.cpp:29-34) plus the final-time goal (0.001 tf)."""
    st = configs.double_pendulum_swingup(5)
    st.solver.optim_finite_difference_scheme = fd
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    for seed in range(3):
        x = nlp.random_iterate(np.random.default_rng(seed).uniform(-1, 1, nlp.n))
        x[1] = 2.0
        kf = 2 + (nlp.G - 1) * nlp.NS
        tip = _pendulum_tip(x[kf], x[kf + 1])
        f = 1000.0 * float(np.sum((tip - np.array([0.0, 2.0, 0.0])) ** 2)) + 0.001 * x[1]
        assert nlp.eval_f(x) == pytest.approx(f, rel=1e-13, abs=1e-12)
        g = nlp.eval_grad_f(x)
        gn = _numjac(lambda z: np.array([nlp.eval_f(z)]), x, range(nlp.n))[0]
        # analytic gradient of the marker term at the final coordinates
        q0, q1 = x[kf], x[kf + 1]
        d = tip - np.array([0.0, 2.0, 0.0])
        J = np.array([[-math.sin(q0) - math.sin(q0 + q1), -math.sin(q0 + q1)],
                      [math.cos(q0) + math.cos(q0 + q1), math.cos(q0 + q1)]])
        ga = 2000.0 * d[:2] @ J
        tol = 1e-5 * np.abs(ga) + 1e-4 * max(1.0, abs(f)) * math.sqrt(st.solver.fd_step)
        assert np.all(np.abs(g[kf:kf + 2] - ga) <= tol + 2e-3)
        assert np.allclose(g, gn, rtol=1e-4, atol=2e-3)
        # only tf and the final coordinates carry gradient
        nz = set(np.flatnonzero(g))
        assert nz <= {1, kf, kf + 1}


def test_goal_term_indices_validated():
    """A term index outside its kind's range (controls, states, bodies) is
    MH_ERR_INVALID at create, in the oracle and in the library's validation
    (out-of-bounds device reads otherwise)."""
    st = configs.double_pendulum(3)
    rep = st.problem.create_rep()
    for bad in (rep.num_controls, -1, 1000):
        rep._gidx[0] = bad
        with pytest.raises(RuntimeError, match="out of range"):
            OracleNLP(rep, st.solver.options())
    rep._gidx[0] = 0
    OracleNLP(rep, st.solver.options())
    st = configs.double_pendulum_swingup(3)
    rep = st.problem.create_rep()
    rep._gidx[0] = 7      # a body that does not exist
    with pytest.raises(RuntimeError, match="out of range"):
        OracleNLP(rep, st.solver.options())


# ---- kinematic constraints --------------------------------

def _kc(N=6, scheme="hermite-simpson", dynamics="explicit", enforce=True, coupler="linear"):
    st = configs.double_pendulum_coupled(N, scheme, dynamics, enforce, coupler)
    return OracleNLP(st.problem.create_rep(), st.solver.options()), st


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
@pytest.mark.parametrize("enforce", [True, False])
@pytest.mark.parametrize("dynamics", ["explicit", "implicit"])
def test_kinematic_constraint_layout(scheme, enforce, dynamics):
    """CasOCTranscription.cpp:103-140,209-241,298-309 and flattenConstraints
    (CasOCTranscription.h:219-313): one multiplier per holonomic equation at
    every grid point (bounds multiplier_bounds, default [-1000, 1000]), with
    enforced derivatives one slack per multiplier at each mesh-interval
    midpoint (HS only; velocity_correction_bounds [-0.1, 0.1]) and
    position + velocity + acceleration error rows (else position only) at
    every mesh point, first among the mesh point's rows, bounds [0, 0]."""
    N = 5
    nlp, st = _kc(N, scheme, dynamics, enforce)
    hs = scheme == "hermite-simpson"
    G = 2 * N + 1 if hs else N + 1
    NS, NC, NM = 4, 2, 1
    NDV = 2 if dynamics == "implicit" else 0
    NSL = 1 if (enforce and hs) else 0
    NK = 3 if enforce else 1
    assert nlp.n == 2 + (NS + NC + NM + NDV) * G + NSL * N
    nres = 2 if dynamics == "implicit" else 0
    rpi = NK + (2 * NS + NC if hs else NS) + nres * (2 if hs else 1)
    assert nlp.m == N * rpi + NK + nres
    xl, xu, gl, gu = nlp.bounds()
    mult = 2 + (NS + NC) * G
    assert np.all(xl[mult:mult + G] == -1000) and np.all(xu[mult:mult + G] == 1000)
    assert np.all(xl[mult + G:mult + G + NSL * N] == -0.1) and np.all(xu[mult + G:mult + G + NSL * N] == 0.1)
    assert np.all(gl == 0) and np.all(gu == 0)
    # the kinematic rows of mesh point i read its multiplier (block-dense
    # over the point's callback inputs), never a slack
    ir, jc = nlp.jac_structure()
    for i in range(N + 1):
        k = 2 * i if hs else i
        rows = i * rpi + np.arange(NK)
        cols = jc[np.isin(ir, rows)]
        assert mult + k in cols
        assert not np.any((cols >= mult + G) & (cols < mult + G + NSL * N))
    # Simpson q-rows read the interval's slack (velocity correction)
    if NSL:
        for i in range(N):
            srow = i * rpi + NK + nres * 2 + NS          # first Simpson row
            assert mult + G + i in jc[ir == srow]


@pytest.mark.parametrize("scheme", ["hermite-simpson", "trapezoidal"])
@pytest.mark.parametrize("enforce", [True, False])
@pytest.mark.parametrize("dynamics", ["explicit", "implicit"])
def test_kinematic_constraint_jacobian_numerical(scheme, enforce, dynamics):
    """eval_jac_g (FD quotients through the transcription chain rule) against
    a central numerical derivative of eval_g, and every dependence of g
    inside the structure (SimmSpline coupler: curvature in the acceleration
    errors and the velocity correction)."""
    nlp, _ = _kc(5, scheme, dynamics, enforce, "spline")
    x = nlp.random_iterate(np.random.default_rng(3).uniform(-1, 1, nlp.n))
    J = nlp.eval_jac_g(x)
    ir, jc = nlp.jac_structure()
    inside = np.zeros((nlp.m, nlp.n), bool)
    inside[ir, jc] = True
    Jn = np.zeros((nlp.m, nlp.n))
    for c in range(nlp.n):
        e = np.zeros(nlp.n)
        e[c] = 1e-6
        Jn[:, c] = (nlp.eval_g(x + e) - nlp.eval_g(x - e)) / 2e-6
    assert np.abs(Jn[~inside]).max(initial=0.0) == 0.0
    scale = np.abs(Jn).max() + 1.0
    assert np.abs(J - Jn[ir, jc]).max() <= 1e-6 * scale


def test_kinematic_constraint_physics():
    """CoordinateCoupler q1 = -2 q0 + pi (testConstraints.cpp:629-645) on the
    DAE callback: the position and velocity errors vanish on a consistent
    state; the acceleration error is affine in the multiplier and the
    multiplier that zeroes it exists; the constraint force follows Simbody's
    M udot + G^T lambda = f (d paerr / d lambda = -G M^-1 G^T < 0); the
    implicit residual vanishes at the explicit accelerations under the same
    multiplier; the velocity correction is G^T gamma = (-2 gamma, -gamma)."""
    nlp, st = _kc(2)
    q0, u0 = 0.3, -0.7
    q = np.array([q0, -2 * q0 + math.pi])
    u = np.array([u0, -2 * u0])
    tau = np.array([1.5, -0.4])

    def row(lam, gam=0.0):   # [t, q, u, tau, lambda, gamma]
        return np.concatenate([[0.2], q, u, tau, [lam, gam]])
    y = nlp.eval_dae(np.array([row(0.0), row(1.0), row(0.0, 0.05)]))
    okc, oqc = 2, 5   # outputs: udot (2), kinematic errors (3), correction (2)
    assert abs(y[0, okc]) < 1e-15 and abs(y[0, okc + 1]) < 1e-15
    a0, a1 = y[0, okc + 2], y[1, okc + 2]
    assert a1 - a0 < 0                                  # -G M^-1 G^T
    lam = -a0 / (a1 - a0)
    ys = nlp.eval_dae(np.array([row(lam)]))[0]
    assert abs(ys[okc + 2]) < 1e-9 * (abs(a0) + 1)
    assert abs(ys[1] + 2 * ys[0]) < 1e-9 * (abs(ys[0]) + 1)   # q1dd = -2 q0dd
    np.testing.assert_allclose(y[2, oqc:oqc + 2], [-2 * 0.05, -0.05], rtol=0, atol=1e-15)
    # implicit: M w + C - f + G^T lambda = 0 at w = the explicit udot
    imp, _ = _kc(2, dynamics="implicit")
    r = imp.eval_dae(np.array([np.concatenate([[0.2], q, u, tau, ys[:2], [lam, 0.0]])]))[0]
    assert np.abs(r[:2]).max() < 1e-9 * (np.abs(tau).max() + 1)


def test_lagrange_multiplier_term():
    """minimize_lagrange_multipliers (CasOCTranscription.cpp:513-521):
    f gains weight * duration * sum_k quad_k sum_j lambda_kj^2; its gradient
    is exact (the reference differentiates the MX term with AD); without
    kinematic constraints the option is rejected (MocoCasOCProblem.cpp:
    101-107)."""
    nlp, st = _kc(6)
    off, _ = _kc(6)
    st.solver.minimize_lagrange_multipliers = False
    off = OracleNLP(st.problem.create_rep(), st.solver.options())
    x = nlp.random_iterate(np.random.default_rng(2).uniform(-1, 1, nlp.n))
    G = nlp.G
    lam = x[2 + 6 * G:2 + 7 * G]
    N = 6
    mesh = np.arange(N + 1) / N
    quad = np.zeros(G)
    for i in range(N):
        dm = mesh[i + 1] - mesh[i]
        quad[2 * i] += dm / 6
        quad[2 * i + 1] += 2 * dm / 3
        quad[2 * i + 2] += dm / 6
    extra = 10.0 * (x[1] - x[0]) * np.dot(quad, lam ** 2)
    assert nlp.eval_f(x) - off.eval_f(x) == pytest.approx(extra, rel=1e-12)
    g = nlp.eval_grad_f(x) - off.eval_grad_f(x)
    np.testing.assert_allclose(g[2 + 6 * G:2 + 7 * G], 10.0 * (x[1] - x[0]) * quad * 2 * lam, rtol=1e-12)
    assert g[1] == pytest.approx(10.0 * np.dot(quad, lam ** 2), rel=1e-9)
    st2 = configs.double_pendulum(4)
    st2.solver.minimize_lagrange_multipliers = True
    with pytest.raises(RuntimeError, match="minimize_lagrange_multipliers"):
        OracleNLP(st2.problem.create_rep(), st2.solver.options())


# ---- tropter's global-seed FD Jacobian ---------

def _color(ir, jc, m, n):
    """mh_color_jacobian (host-only entry of libmocohip: no device needed)."""
    hip = abi.load_mocohip()
    ir = np.ascontiguousarray(ir, np.int32)
    jc = np.ascontiguousarray(jc, np.int32)
    color = np.empty(n, np.int32)
    k = C.c_int32()
    assert hip.mh_color_jacobian(m, n, len(ir), abi.iptr(ir), abi.iptr(jc), abi.iptr(color), C.byref(k)) == 0
    return color, k.value


def _color_ordered(ir, jc, m, n, order, lib="hip"):
    """mh_color_jacobian_ordered (the library) or orc_color_jacobian (the
    oracle's independent restatement); host only."""
    ir = np.ascontiguousarray(ir, np.int32)
    jc = np.ascontiguousarray(jc, np.int32)
    color = np.empty(n, np.int32)
    k = C.c_int32()
    if lib == "hip":
        fn = abi.load_mocohip().mh_color_jacobian_ordered
    else:
        fn = abi.load_oracle().orc_color_jacobian
    assert fn(m, n, len(ir), abi.iptr(ir), abi.iptr(jc), order, abi.iptr(color), C.byref(k)) == 0
    return color, k.value


def _valid_coloring(ir, jc, color):
    seen = {}
    for r, c in zip(ir, jc):
        key = (int(r), int(color[c]))
        assert seen.setdefault(key, int(c)) == int(c), "two columns of one color share a row"


def test_global_seed_jacobian_pinned_by_tropter_sparse_jacobian():
    """tropter/tests/test_derivatives.cpp:410-520 ("Check derivatives with
    analytical deriv.; sparse Jacobian."): constraints c_i = sum of x_j^2 over
    j in [max(i-1, 0), min(i+1, n)), n = 4, m = 5, at x = (3.1, -1.5, -0.25,
    5.3).  Finite differences along the seeds of the column coloring
    (central, eps = sqrt(DBL_EPSILON), ProblemDecorator_double.cpp:261-291),
    recovered per nonzero, equal the analytical Jacobian 2 x_j to relative
    1e-8 (the test's Approx.epsilon)."""
    n, m = 4, 5
    x = np.array([3.1, -1.5, -0.25, 5.3])

    def cons(v):
        out = np.zeros(m)
        for i in range(m):
            for j in range(max(i - 1, 0), min(i + 1, n)):
                out[i] += v[j] * v[j]
        return out
    ir = [i for i in range(m) for j in range(max(i - 1, 0), min(i + 1, n))]
    jc = [j for i in range(m) for j in range(max(i - 1, 0), min(i + 1, n))]
    assert len(ir) == 2 * n   # num_jacobian_elem
    color, k = _color(ir, jc, m, n)
    _valid_coloring(ir, jc, color)
    assert k == 2
    eps = math.sqrt(np.finfo(float).eps)
    comp = np.stack([(cons(x + eps * (color == s)) - cons(x - eps * (color == s))) / (2 * eps)
                     for s in range(k)], 1)
    vals = np.array([comp[r, color[c]] for r, c in zip(ir, jc)])
    np.testing.assert_allclose(vals, [2 * x[j] for j in jc], rtol=1e-8)


@pytest.mark.parametrize("case", ["hs", "trap", "coupled", "gait"])
def test_global_seed_jacobian_is_columnwise_fd_of_g(case):
    """The oracle's global-seed Jacobian equals, bit for bit, the central
    difference of eval_g along each single column (each row meets one column
    of a seed), and agrees with the per-callback FD Jacobian to FD accuracy;
    the coloring is valid and far smaller than n."""
    st = {"hs": lambda: configs.double_pendulum(5),
          "trap": lambda: configs.double_pendulum(5, "trapezoidal", dynamics="implicit"),
          "coupled": lambda: configs.double_pendulum_coupled(4),
          "gait": lambda: configs.gait10dof18musc(2, muscles=False)}[case]()
    rep = st.problem.create_rep()
    cb = OracleNLP(rep, st.solver.options())
    st.solver.jacobian_mode = "global-seeds"
    gs = OracleNLP(rep, st.solver.options())
    ir, jc = gs.jac_structure()
    color, k = gs.jacobian_seeds()
    _valid_coloring(ir, jc, color)
    assert np.array_equal(color, _color_ordered(ir, jc, gs.m, gs.n, abi.MH_COLORING_SMALLEST_LAST)[0])
    assert k < gs.n
    x = gs.random_iterate(np.random.default_rng(1).uniform(-1, 1, gs.n))
    J = gs.eval_jac_g(x)
    eps = math.sqrt(np.finfo(float).eps)
    cols = sorted(set(jc.tolist()))[:: max(1, len(set(jc.tolist())) // 40)]
    for c in cols:
        e = np.zeros(gs.n)
        e[c] = eps
        d = (gs.eval_g(x + e) - gs.eval_g(x - e)) / (2 * eps)
        sel = jc == c
        assert np.array_equal(J[sel], d[ir[sel]]), c
    # the two FD schemes agree to truncation accuracy (forward 1e-8 steps of
    # the callbacks vs central sqrt(eps) steps of g; the random gait iterate
    # drives the DAE to ~1e5)
    Jc = cb.eval_jac_g(x)
    assert np.abs(J - Jc).max() <= 1e-3 * (np.abs(Jc).max() + 1.0)


# ---------------------------------------------------------------------------
# Rajagopal 2016: the reference's converged MocoInverse of the
# 18-muscle model pins multibody dynamics of the 21-coordinate CustomJoint
# model, the patellofemoral couplers' multipliers with prescribed
# kinematics, DGF implicit tendons and the muscle paths
# ---------------------------------------------------------------------------
def _rajagopal18_golden_iterate(nlp, rep):
    d = np.load(os.path.join(os.path.dirname(__file__), "golden",
                             "std_testMocoInverse_subject_18musc_solution.npz"))
    labels, data = list(d["labels"]), d["data"]
    col = {l: i for i, l in enumerate(labels)}
    G, NS, NC, NDV, NM = nlp.G, nlp.NS, nlp.NC, nlp.NDV, 2
    assert data.shape[0] == G
    mult = [l for l in labels if l.startswith("lambda")]
    der = [l for l in labels if "implicitderiv" in l]
    assert len(mult) == NM and len(der) == NDV
    blocks = [(rep.state_names, NS), (rep.control_names, NC), (mult, NM), (der, NDV)]
    x = [data[0, 0], data[-1, 0]]
    for names, w in blocks:
        x += [data[k, col[n]] for k in range(G) for n in names]
    return np.array(x), labels


def _rajagopal18_residuals(keep_path_wraps=False, shift=None):
    st = configs.rajagopal18_inverse(keep_path_wraps=keep_path_wraps)
    if shift is not None:
        mu = [m for m in st.problem.model.muscles if m.name == shift][0]
        mu.points[0].loc = tuple(np.asarray(mu.points[0].loc, float) + [0.001, 0.0, 0.0])
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    x, labels = _rajagopal18_golden_iterate(nlp, rep)
    g = nlp.eval_g(x)
    NEP, N, NQ, NAR = 18, 11, rep.nq, rep.num_aux_residuals
    rpi = 2 * (NQ + NAR) + 2 * nlp.NS
    assert len(g) == NEP + N * rpi + NQ + NAR
    gi = g[NEP:NEP + N * rpi].reshape(N, rpi)
    res = np.concatenate([gi[:, :2 * (NQ + NAR)].reshape(N, 2, NQ + NAR).reshape(-1, NQ + NAR),
                          g[NEP + N * rpi:][None, :]])
    return g[:NEP], res[:, :NQ], res[:, NQ:], gi[:, 2 * (NQ + NAR):], nlp, rep


def test_rajagopal18_inverse_layout():
    """testMocoInverse.cpp:118-147 on the Rajagopal 18-muscle model: 21
    coordinates after welding subtalar / mtp, 28 states (18 activations, 10
    implicit tendon forces), 33 controls, 10 tendon-force derivatives, 2
    coupler multipliers per grid point and no kinematic rows or slacks with
    prescribed kinematics (CasOCProblem.h:508-521), HS N = 11, 18 endpoint
    rows first (MocoInitialActivationGoal), no control interpolation."""
    st = configs.rajagopal18_inverse()
    rep = st.problem.create_rep()
    nlp = OracleNLP(rep, st.solver.options())
    assert (rep.nq, nlp.NS, nlp.NC, nlp.NDV, rep.num_kinematic_constraints) == (21, 28, 33, 10, 2)
    G = 23
    assert nlp.n == 2 + (28 + 33 + 2 + 10) * G
    assert nlp.m == 18 + 11 * (2 * (21 + 10) + 2 * 28) + (21 + 10)
    d = np.load(os.path.join(os.path.dirname(__file__), "golden",
                             "std_testMocoInverse_subject_18musc_solution.npz"))
    hdr = dict(h.split("=", 1) for h in d["header"])
    assert (int(hdr["num_states"]) - 2 * rep.nq, int(hdr["num_controls"]), int(hdr["num_multipliers"]),
            int(hdr["num_derivatives"]), int(hdr["num_slacks"])) == (28, 33, 2, 10, 0)


def test_rajagopal18_inverse_golden_solution():
    """The reference's converged iterate
    (Moco/Tests/std_testMocoInverse_subject_18musc_solution.sto, MocoInverse
    constraint tolerance 1e-3) satisfies our g: every defect and endpoint
    row, the 10 implicit tendon equilibrium residuals within 0.03 N
    (Fmax 2-10 kN), the 21 multibody residuals within 1.5 N / N m (GRFs up
    to ~1 kN; the largest are the pelvis rows, from the kinematics and GRF
    splines); the patella rows vanish with the golden multipliers.
    Sensitivity: the Millard muscles' 16 PathWraps kept (which
    DeGrooteFregly2016Muscle::replaceMuscles drops,
    DeGrooteFregly2016Muscle.cpp:1007-1020) or one path point moved by
    1 mm is far outside these bounds."""
    ep, mb, aux, defects, nlp, rep = _rajagopal18_residuals()
    assert np.abs(ep).max() == 0.0
    assert np.abs(defects).max() < 1e-3   # the solve's constraint tolerance
    assert np.abs(aux).max() < 0.03, np.abs(aux).max(0)
    assert np.abs(mb).max() < 1.5, np.abs(mb).max(0)
    qn = [c.name for c in rep.problem.model.coordinates()]
    betas = [qn.index(b) for b in ("knee_angle_r_beta", "knee_angle_l_beta")]
    assert np.abs(mb[:, betas]).max() < 1e-4
    # the multipliers' sign convention (-G^T lambda applied) is what zeroes them
    x, _ = _rajagopal18_golden_iterate(nlp, rep)
    G, NS, NC = nlp.G, nlp.NS, nlp.NC
    o = 2 + (NS + NC) * G
    x[o:o + 2 * G] *= -1.0
    g = nlp.eval_g(x)
    NQ, NAR = rep.nq, rep.num_aux_residuals
    rpi = 2 * (NQ + NAR) + 2 * NS
    gb = g[18:18 + 11 * rpi].reshape(11, rpi)[:, :NQ]
    assert np.abs(gb[:, betas]).max() > 1.0
    _, mbw, auxw, _, _, _ = _rajagopal18_residuals(keep_path_wraps=True)
    assert max(np.abs(mbw).max(), np.abs(auxw).max()) > 20.0
    _, _, auxs, _, _, _ = _rajagopal18_residuals(shift="vas_int_r")
    assert np.abs(auxs).max() > 0.3


def test_wrap_cylinder_geometry():
    """WrapCylinder on wrapped_pendulum: where the straight
    path crosses the cylinder, the current path is p1 -> r1 -> r2 -> p2 with
    r1, r2 on the surface, p1 r1 and r2 p2 tangent to it, and a length equal
    to the shortest path around the cylinder computed independently
    (tangent lengths sqrt(d^2 - R^2), the arc between the tangent points,
    the axial rise over the unrolled length); the short way unconstrained,
    the constrained side with a quadrant; no wrap where the straight path
    misses (unconstrained) or passes on the constrained side; the speed is
    the path length's time derivative (cylinder fixed with the origin)."""
    import ctypes as C
    from mocohip import abi
    lib = abi.load_oracle()
    R = 0.1

    def shortest(a, b, sigma):
        da, db = np.hypot(*a[:2]), np.hypot(*b[:2])
        ang = ((math.atan2(b[1], b[0]) - math.atan2(a[1], a[0])) * sigma) % (2 * math.pi)
        arc = ang - math.acos(R / da) - math.acos(R / db)
        Lxy = math.sqrt(da * da - R * R) + R * arc + math.sqrt(db * db - R * R)
        return math.hypot(Lxy, b[2] - a[2])

    for quad in ("all", "+y", "-y"):
        st = configs.wrapped_pendulum(quadrant=quad)
        nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
        nwrap = 0
        for q0 in np.linspace(-1.4, 1.4, 15):
            q, u = np.array([q0]), np.array([0.3])
            pts, n, out = np.zeros(40), C.c_int(), np.zeros(2)
            assert lib.orc_muscle_path(nlp.ctx, 0, abi.dptr(q), abi.dptr(u), 10, C.byref(n), abi.dptr(pts)) == 0
            assert lib.orc_muscle_length_speed(nlp.ctx, 0, abi.dptr(q), abi.dptr(u), abi.dptr(out)) == 0
            P = pts[:4 * n.value].reshape(-1, 4)
            a, b = P[0, :3], P[-1, :3]
            cr = a[0] * b[1] - a[1] * b[0]
            short = 1.0 if cr >= 0 else -1.0
            if n.value == 2:
                assert out[0] == pytest.approx(np.linalg.norm(b - a), rel=1e-14)
                continue
            nwrap += 1
            assert n.value == 4 and list(P[1:3, 3]) == [-1.0, -2.0]
            for r, p in ((P[1, :3], a), (P[2, :3], b)):
                assert np.hypot(*r[:2]) == pytest.approx(R, rel=1e-13)
                assert abs(np.dot(p[:2] - r[:2], r[:2])) < 1e-15
            sides = [short] if quad == "all" else [short, -short]
            Ls = [shortest(a, b, s) for s in sides]
            assert min(abs(out[0] - L) for L in Ls) < 1e-13
            if quad == "all":
                assert out[0] == pytest.approx(Ls[0], abs=1e-13)
            # constrained: the wrap midpoint direction lies on the quadrant's side
            mid = P[1, :2] + P[2, :2]
            if quad != "all" and np.linalg.norm(mid) > 1e-9:
                assert np.sign(mid[1]) == (1 if quad == "+y" else -1)
            h = 1e-6
            Lp, Lm = np.zeros(2), np.zeros(2)
            lib.orc_muscle_length_speed(nlp.ctx, 0, abi.dptr(q + h), abi.dptr(u), abi.dptr(Lp))
            lib.orc_muscle_length_speed(nlp.ctx, 0, abi.dptr(q - h), abi.dptr(u), abi.dptr(Lm))
            assert out[1] == pytest.approx((Lp[0] - Lm[0]) / (2 * h) * u[0], rel=1e-6, abs=1e-9)
        assert nwrap >= 6


def _structures():
    """Jacobian structures to color: tropter's sparse-Jacobian test, the
    transcriptions of a few problems, a random sparse pattern."""
    out = {}
    ir = [i for i in range(5) for j in range(max(i - 1, 0), min(i + 1, 4))]
    jc = [j for i in range(5) for j in range(max(i - 1, 0), min(i + 1, 4))]
    out["tropter_sparse"] = (np.array(ir), np.array(jc), 5, 4)
    for name, mk in (("hs", lambda: configs.double_pendulum(5)),
                     ("trap", lambda: configs.double_pendulum(5, "trapezoidal", dynamics="implicit")),
                     ("coupled", lambda: configs.double_pendulum_coupled(4)),
                     ("gait", lambda: configs.gait10dof18musc(3))):
        st = mk()
        o = OracleNLP(st.problem.create_rep(), st.solver.options())
        i, j = o.jac_structure()
        out[name] = (i, j, o.m, o.n)
        o.close()
    r = np.random.default_rng(7)
    m, n = 300, 200
    dense = r.random((m, n)) < 0.03
    i, j = np.nonzero(dense)
    out["random"] = (i, j, m, n)
    return out


def test_smallest_last_coloring_library_equals_oracle():
    """ColPack's SMALLEST_LAST column order (GraphColoring.cpp:91-94), restated
    in the library (mocohip.hip smallest_last_order) and independently in the
    oracle (oracle.c smallest_last): the same colors column for column on every
    structure, a valid partial distance-2 coloring, and -- on the
    transcriptions, whose t0 / tf columns meet every defect row -- no more seeds
    than the natural order; tropter's sparse-Jacobian test keeps its 2 seeds."""
    for name, (ir, jc, m, n) in _structures().items():
        for order in (abi.MH_COLORING_SMALLEST_LAST, abi.MH_COLORING_NATURAL):
            ch, kh = _color_ordered(ir, jc, m, n, order, "hip")
            co, ko = _color_ordered(ir, jc, m, n, order, "oracle")
            assert kh == ko and np.array_equal(ch, co), (name, order)
            _valid_coloring(ir, jc, ch)
        sl = _color_ordered(ir, jc, m, n, abi.MH_COLORING_SMALLEST_LAST)[1]
        nat = _color_ordered(ir, jc, m, n, abi.MH_COLORING_NATURAL)[1]
        assert np.array_equal(_color_ordered(ir, jc, m, n, abi.MH_COLORING_NATURAL)[0], _color(ir, jc, m, n)[0])
        if name == "tropter_sparse":
            assert sl == 2
        if name != "random":
            assert sl <= nat, (name, sl, nat)


def test_smallest_last_order_is_smallest_last():
    """The order itself on a graph small enough to follow by hand: a star
    (column 0 shares a row with each of columns 1..4) plus an isolated
    column 5.  Degrees: 0 -> 4, 1..4 -> 1, 5 -> 0.  Smallest-last removes 5
    (degree 0), then 4, 3, 2 (the last of bucket 1 each time; 0 drops to
    degree 1 after three removals and is appended behind 1), then 0, then 1;
    coloring in reverse removal order (1, 0, 2, 3, 4, 5) gives 1 -> 0, 0 -> 1,
    2, 3, 4 -> 0, 5 -> 0: two seeds."""
    ir = np.array([0, 0, 1, 1, 2, 2, 3, 3])
    jc = np.array([0, 1, 0, 2, 0, 3, 0, 4])
    for lib in ("hip", "oracle"):
        color, k = _color_ordered(ir, jc, 4, 6, abi.MH_COLORING_SMALLEST_LAST, lib)
        assert k == 2
        assert color.tolist() == [1, 0, 0, 0, 0, 0]
