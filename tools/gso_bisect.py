"""Stage-by-stage A/B of the GSO preprocessing restatement against the
reference's golden fiber lengths / velocities
(Moco/Archive/Tests/std_testGait10dof18musc_GSO_solution_norm_fiber_{length,
velocity}.sto; testGait10dof18musc.cpp:58-98 asserts 1e-5).

The pipeline (InverseMuscleSolverMotionData.cpp:49-114, 249-290): rows of
testGait10dof18musc_kinematics.mot within [t0 - 0.05, tf + 0.05], Storage::pad
(size / 2), Storage::lowpassIIR (6 Hz), muscle-tendon lengths at every
padded row, GCVSplineSet(degree 5) of the lengths, its value and first
derivative at the solution times, rigid-tendon fiber kinematics.  Each
variant replaces ONE stage; the table gives, per variant, the largest
normalized fiber length / velocity error over all 9 muscles and times, and
rect_fem_r's / vasti_r's velocity error in the window t = 1.785-1.80 where
the residual sits.  CPU only (the oracle's muscle paths).

    python tools/gso_bisect.py > profiles/r06_gso/gso_bisect.txt
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opensim-moco_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from mocohip import abi, configs  # noqa: E402
from mocohip.problem import MocoProblem  # noqa: E402
from mocohip.solver import MocoHipSolver, OracleNLP  # noqa: E402
from mocohip.splines import gcv_interpolating_ppoly  # noqa: E402

Z = np.load(os.path.join(ROOT, "tests", "golden", "gso_norm_fiber_length.npz"))


def pad(x, p, kind="odd"):
    n = len(x)
    if kind == "odd":     # reflected about the end point and negated
        return np.concatenate([2 * x[0] - x[p:0:-1], x, 2 * x[-1] - x[n - 2:n - 2 - p:-1]])
    if kind == "even":    # plain mirror
        return np.concatenate([x[p:0:-1], x, x[n - 2:n - 2 - p:-1]])
    raise ValueError(kind)


def pad_time(t, p, kind):
    if kind == "odd":
        return pad(t, p, "odd")
    dt = {"uniform_first": t[1] - t[0], "uniform_min": np.diff(t).min(),
          "uniform_avg": (t[-1] - t[0]) / (len(t) - 1)}[kind]
    return np.concatenate([t[0] - dt * np.arange(p, 0, -1), t, t[-1] + dt * np.arange(1, p + 1)])


def lowpass(dt, fc, sig, init="copy3", order=3):
    """Signal::LowpassIIR: third-order Butterworth (prewarped bilinear), forward
    then backward; init: the first three outputs of each pass = its inputs
    ("copy3"), or a zero-history start ("zero")."""
    wa = math.tan(2 * math.pi * fc * dt / 2)
    wa2, wa3 = wa * wa, wa * wa * wa
    den = 1 + 2 * wa + 2 * wa2 + wa3
    b = np.array([wa3, 3 * wa3, 3 * wa3, wa3]) / den
    a = np.array([(-3 - 2 * wa + 2 * wa2 + 3 * wa3), (3 - 2 * wa - 2 * wa2 + 3 * wa3),
                  (-1 + 2 * wa - 2 * wa2 + wa3)]) / den

    def run(s):
        f = s.copy()
        if init == "zero":
            ss = np.concatenate([np.zeros(3), s])
            ff = np.zeros(len(ss))
            for i in range(3, len(ss)):
                ff[i] = (b[0] * ss[i] + b[1] * ss[i - 1] + b[2] * ss[i - 2] + b[3] * ss[i - 3]
                         - a[0] * ff[i - 1] - a[1] * ff[i - 2] - a[2] * ff[i - 3])
            return ff[3:]
        for i in range(3, len(s)):
            f[i] = (b[0] * s[i] + b[1] * s[i - 1] + b[2] * s[i - 2] + b[3] * s[i - 3]
                    - a[0] * f[i - 1] - a[1] * f[i - 2] - a[2] * f[i - 3])
        return f
    return run(run(sig)[::-1])[::-1]


class Paths:
    def __init__(self, m):
        self.m = m
        self.rep = MocoProblem(m).create_rep()
        self.nlp = OracleNLP(self.rep, MocoHipSolver(num_mesh_intervals=2).options())
        self.lib = abi.load_oracle()
        self.qnames = [n.split("/")[-2] for n in self.rep.state_names[:self.rep.nq]]
        names = [mu.name for mu in m.muscles]
        self.cols = [names.index(l.split("/")[-1]) for l in list(Z["nfl_labels"])[1:]]

    def lengths(self, Q):
        out = np.zeros(2)
        L = np.zeros((len(Q), len(self.cols)))
        zero = np.zeros(self.rep.nq)
        for i, q in enumerate(Q):
            q = np.ascontiguousarray(q)
            for c, im in enumerate(self.cols):
                assert self.lib.orc_muscle_length_speed(self.nlp.ctx, im, abi.dptr(q), abi.dptr(zero),
                                                        abi.dptr(out)) == 0
                L[i, c] = out[0]
        return L


def spline_eval(tp, L, te, kind):
    if kind.startswith("natural"):
        deg = int(kind[len("natural"):])
        brk, co = gcv_interpolating_ppoly(tp, L, deg)
        seg = np.clip(np.searchsorted(brk, te, side="right") - 1, 0, len(brk) - 2)
        dt = (te - brk[seg])[:, None]
        Lg = sum(co[seg, :, k] * dt ** k for k in range(co.shape[2]))
        Vg = sum(k * co[seg, :, k] * dt ** (k - 1) for k in range(1, co.shape[2]))
        return Lg, Vg
    if kind.startswith("notaknot"):
        from scipy.interpolate import make_interp_spline
        deg = int(kind[len("notaknot"):])
        Lg = np.zeros((len(te), L.shape[1]))
        Vg = np.zeros_like(Lg)
        for c in range(L.shape[1]):
            s = make_interp_spline(tp, L[:, c], k=deg)
            Lg[:, c], Vg[:, c] = s(te), s.derivative()(te)
        return Lg, Vg
    if kind.startswith("smooth5:"):
        return smoothing_eval(tp, L, te, float(kind.split(":")[1]))
    raise ValueError(kind)


def smoothing_eval(tp, L, te, prel, m=3):
    """The natural smoothing spline of degree 2m - 1 (GCVSPL's model:
    minimize sum (y_i - s(x_i))^2 + p int (s^(m))^2, unit weights), in the
    B-spline basis of degree 2m - 1 with knots at the data sites (which holds
    the natural spline, the minimizer); p = prel * trace(B^T B) / trace(P).
    prel -> 0 is the interpolating natural spline of the restatement; GCVSPL
    with a prescribed error variance of 0 (GCVSpline's default) searches p
    down to its lower bound, which a positive prel stands for."""
    from scipy.interpolate import BSpline
    k = 2 * m - 1
    x = np.asarray(tp, float)
    kn = np.concatenate([[x[0]] * (k + 1), x[1:-1], [x[-1]] * (k + 1)])
    nb = len(kn) - k - 1
    B = BSpline.design_matrix(x, kn, k).toarray()
    # penalty: int B_i^(m) B_j^(m) over each interval, Gauss-Legendre exact
    gx, gw = np.polynomial.legendre.leggauss(k)
    P = np.zeros((nb, nb))
    eye = np.eye(nb)
    ders = [BSpline(kn, eye[i], k).derivative(m) for i in range(nb)]
    for a, b in zip(x[:-1], x[1:]):
        xs = 0.5 * (b - a) * gx + 0.5 * (a + b)
        D = np.stack([d(xs) for d in ders])          # nb x q
        P += (D * (0.5 * (b - a) * gw)) @ D.T
    BtB = B.T @ B
    lam = prel * np.trace(BtB) / np.trace(P)
    C = np.linalg.solve(BtB + lam * P, B.T @ L)
    Lg = np.stack([BSpline(kn, C[:, c], k)(te) for c in range(L.shape[1])], 1)
    Vg = np.stack([BSpline(kn, C[:, c], k).derivative()(te) for c in range(L.shape[1])], 1)
    return Lg, Vg


def fiber(paths, Lg, Vg):
    nfl = np.empty_like(Lg)
    nfv = np.empty_like(Lg)
    for c, im in enumerate(paths.cols):
        mu = paths.m.muscles[im]
        w = mu.optimal_fiber_length * math.sin(mu.pennation_angle_at_optimal)
        along = Lg[:, c] - mu.tendon_slack_length
        fl = np.sqrt(along ** 2 + w * w)
        nfl[:, c] = fl / mu.optimal_fiber_length
        nfv[:, c] = Vg[:, c] * (along / fl) / (mu.max_contraction_velocity * mu.optimal_fiber_length)
    return nfl, nfv


def resample(tp, Qp, degree=5):
    """Storage::resample(dtmin, 5) as the restatement assumes Storage::
    lowpassIIR does on non-uniform times: the padded rows onto the uniform
    grid t_first + k dtmin (k < the row count), the values by the degree-5
    GCV interpolant (mocohip.splines)."""
    dtmin = np.diff(tp).min()
    tn = tp[0] + np.arange(len(tp)) * dtmin
    brk, co = gcv_interpolating_ppoly(tp, Qp, degree)
    seg = np.clip(np.searchsorted(brk, tn, side="right") - 1, 0, len(brk) - 2)
    d = (tn - brk[seg])[:, None]
    return tn, sum(co[seg, :, k] * d ** k for k in range(co.shape[2])), dtmin


def run(paths, dt_mode="first", time_pad="odd", data_pad="odd", iir="copy3", spline="natural5",
        t0=0.58, tf=1.8, slop=0.05, lengths_from="filtered", resampled=False):
    kl, kin = list(Z["kin_labels"]), Z["kin"]
    t = kin[:, 0]
    sel = (t >= t0 - slop) & (t <= tf + slop)
    t = t[sel]
    Q = np.stack([np.deg2rad(kin[sel, kl.index(q)]) if q not in ("pelvis_tx", "pelvis_ty")
                  else kin[sel, kl.index(q)] for q in paths.qnames], 1)
    p = len(t) // 2
    tp = pad_time(t, p, time_pad)
    dt = {"first": t[1] - t[0], "min": np.diff(tp).min(), "nominal": 1.0 / 60.0,
          "avg": (tp[-1] - tp[0]) / (len(tp) - 1)}[dt_mode]
    Qp = np.stack([pad(Q[:, j], p, data_pad) for j in range(Q.shape[1])], 1)
    if resampled:
        tp, Qp, dt = resample(tp, Qp)
    Qp = np.stack([lowpass(dt, 6.0, Qp[:, j], iir) for j in range(Q.shape[1])], 1)
    L = paths.lengths(Qp)
    te = Z["nfl"][:, 0]
    Lg, Vg = spline_eval(tp, L, te, spline)
    nfl, nfv = fiber(paths, Lg, Vg)
    return np.abs(nfl - Z["nfl"][:, 1:]), np.abs(nfv - Z["nfv"][:, 1:]), te, nfl, nfv


VARIANTS = [
    ("restatement (odd pad of data and time, dt = t1 - t0, copy3 IIR start, natural quintic)", {}),
    ("filter dt = min step of the padded times (Storage::getMinTimeStep)", {"dt_mode": "min"}),
    ("filter dt = 1/60 s (the nominal sample interval)", {"dt_mode": "nominal"}),
    ("filter dt = average step", {"dt_mode": "avg"}),
    ("time column padded uniformly by t1 - t0 (data still odd-reflected)", {"time_pad": "uniform_first"}),
    ("time column padded uniformly by the min step", {"time_pad": "uniform_min"}),
    ("data padded by plain mirror (even reflection)", {"data_pad": "even"}),
    ("IIR passes started from zero history", {"iir": "zero"}),
    ("cubic natural spline (GCVSpline degree 3)", {"spline": "natural3"}),
    ("quintic not-a-knot interpolating spline", {"spline": "notaknot5"}),
    ("selection slop 0 (rows within [t0, tf] only)", {"slop": 0.0}),
    ("padded rows resampled onto the uniform min-step grid (quintic) and filtered with that step",
     {"resampled": True}),
] + [(f"resampled, quintic SMOOTHING spline p = {pr:.0e} trace(B^T B) / trace(P) (GCVSPL's residual smoothing)",
      {"resampled": True, "spline": f"smooth5:{pr}"}) for pr in (1e-8, 1e-6, 1e-4, 1e-3, 1e-2)]


def report(name, r, labels):
    nfl_e, nfv_e, te = r[0], r[1], r[2]
    win = (te >= 1.785 - 1e-9) & (te <= 1.8 + 1e-9)
    cr, cv = labels.index("rect_fem_r"), labels.index("vasti_r")
    other = np.delete(nfv_e, [cr, cv], 1).max()
    return (f"{nfl_e.max():9.2e} {nfv_e.max():9.2e} {other:9.2e} | {nfl_e[win][:, cr].max():9.2e} "
            f"{nfv_e[win][:, cr].max():9.2e} {nfl_e[win][:, cv].max():9.2e} {nfv_e[win][:, cv].max():9.2e} | {name}")


def localize(paths, labels, resampled=True):
    """Which length samples the window residual needs: the spline is linear
    in its data, so the golden MTU lengths' difference from ours (constant
    per-muscle offset removed) is fit by per-sample length perturbations at
    the samples in (1.55, 1.95) s (ridge-regularized least squares); printed
    per sample, with the fit's residual."""
    kl, kin = list(Z["kin_labels"]), Z["kin"]
    t = kin[:, 0]
    sel = (t >= 0.53) & (t <= 1.85)
    t = t[sel]
    Q = np.stack([np.deg2rad(kin[sel, kl.index(q)]) if q not in ("pelvis_tx", "pelvis_ty")
                  else kin[sel, kl.index(q)] for q in paths.qnames], 1)
    p = len(t) // 2
    tp = pad(t, p)
    Qp = np.stack([pad(Q[:, j], p) for j in range(Q.shape[1])], 1)
    dt = t[1] - t[0]
    if resampled:
        tp, Qp, dt = resample(tp, Qp)
    Qf = np.stack([lowpass(dt, 6.0, Qp[:, j]) for j in range(Q.shape[1])], 1)
    L = paths.lengths(Qf)
    te = Z["nfl"][:, 0]

    def ev(LL):
        brk, co = gcv_interpolating_ppoly(tp, LL, 5)
        seg = np.clip(np.searchsorted(brk, te, side="right") - 1, 0, len(brk) - 2)
        d = (te - brk[seg])[:, None]
        return sum(co[seg, :, k] * d ** k for k in range(co.shape[2]))
    Lg = ev(L)
    kq = paths.qnames.index("knee_angle_r")
    idx = [i for i in range(len(tp)) if 1.55 < tp[i] < 1.95]
    w_ = te > 1.5
    Phi = np.zeros((w_.sum(), len(idx)))
    for j, i in enumerate(idx):
        d = np.zeros_like(L)
        d[i, :] = 1.0
        Phi[:, j] = ev(d)[w_, 0]
    print("# window residual localized: per-sample MTU length perturbations (m) reproducing golden - ours")
    for name in ("rect_fem_r", "vasti_r"):
        c = labels.index(name)
        mu = paths.m.muscles[paths.cols[c]]
        w = mu.optimal_fiber_length * math.sin(mu.pennation_angle_at_optimal)
        fl = Z["nfl"][:, 1 + c] * mu.optimal_fiber_length
        Lgold = np.sqrt(fl ** 2 - w * w) + mu.tendon_slack_length
        e = Lgold - Lg[:, c]
        e -= np.median(e[te < 1.6])
        b = e[w_]
        A = np.vstack([Phi, 1e-3 * np.eye(len(idx))])
        dlt, *_ = np.linalg.lstsq(A, np.concatenate([b, np.zeros(len(idx))]), rcond=None)
        print(f"# {name}: max |golden - ours| after t = 1.5 (offset removed) {np.abs(b).max():.2e} m, fit "
              f"residual {np.abs(b - Phi @ dlt).max():.2e} m")
        for j, i in enumerate(idx):
            on = abs(tp[i] * 200 - round(tp[i] * 200)) < 1e-4
            print(f"#   t {tp[i]:.5f}  knee {Qf[i, kq]:+.5f} rad  {'(golden time)' if on else '             '}"
                  f"  {dlt[j]:+.2e}")


def main():
    labels = [l.split("/")[-1] for l in list(Z["nfl_labels"])[1:]]
    paths = Paths(configs.gait10dof18musc_model())
    print("# normalized fiber length (nfl) / velocity (nfv) errors against the GSO golden files")
    print("#  all muscles, all times: nfl, nfv, nfv of the 7 muscles without MovingPathPoints | "
          "t in [1.785, 1.80]: rect_fem_r nfl, nfv; vasti_r nfl, nfv | variant")
    base = None
    for name, kw in VARIANTS:
        r = run(paths, **kw)
        if base is None:
            base = r
        print(report(name, r, labels), flush=True)
    # how far each variant moves rect_fem_r's velocity at t = 1.80 from the restatement
    print("# change of rect_fem_r's nfv at t = 1.80 against the restatement, per variant")
    cr = labels.index("rect_fem_r")
    i = int(np.argmin(np.abs(base[2] - 1.8)))
    for name, kw in VARIANTS[1:]:
        r = run(paths, **kw)
        print(f"{r[4][i, cr] - base[4][i, cr]:+.3e}  (nfl max over muscles/times {r[0].max():.2e})  {name}")
    localize(paths, labels)


if __name__ == "__main__":
    main()
