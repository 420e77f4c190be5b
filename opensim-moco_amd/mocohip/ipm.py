"""A primal-dual interior-point NLP solver over the C ABI's TNLP callbacks.

MocoCasADiSolver hands its transcription to Ipopt 3.12.8 with a
limited-memory Hessian (MocoCasADiSolver.cpp:210-246,
MocoDirectCollocationSolver.cpp:35; tropter: IPOPTSolver.cpp:302-447).
Ipopt is not in this image, so this module restates the algorithm Ipopt
implements (Waechter & Biegler, "On the implementation of an interior-point
filter line-search algorithm for large-scale nonlinear programming", Math.
Program. 106, 2006) on the host, driving exactly the callbacks an Ipopt TNLP
drives: bounds, eval_f, eval_grad_f, eval_g, eval_jac_g with the fixed
sparse structure.  Every evaluation goes through the NLP object (HipNLP: the
GPU path); the host does only the KKT linear algebra.

What is restated (section numbers of the paper):
  * problem form: fixed variables removed (fixed_variable_treatment
    make_parameter), inequality rows of g turned into equalities with bounded
    slacks, bounds relaxed by bound_relax_factor, gradient-based NLP scaling
    (nlp_scaling_max_gradient = 100) of the objective and of each row;
  * the starting point pushed into the interior (bound_push, bound_frac),
    bound multipliers 1, constraint multipliers by least squares
    (constr_mult_init_max);
  * the primal-dual barrier system (2.4)-(2.6), its Newton step with the bound
    multipliers eliminated, inertia-free regularisation delta_c when the
    constraint Jacobian is rank deficient;
  * the limited-memory BFGS Lagrangian Hessian in compact form (Byrd, Nocedal,
    Schnabel 1994; Ipopt hessian_approximation = limited-memory, history 6,
    initialization scalar1) applied through the Sherman-Morrison-Woodbury
    identity on the sparse factorization of the KKT matrix;
  * the monotone Fiacco-McCormick barrier update (kappa_eps, kappa_mu,
    theta_mu), the fraction-to-the-boundary rule, the bound-multiplier
    safeguard kappa_Sigma;
  * the filter line search (3.3-3.5: switching condition, Armijo condition,
    filter augmentation, alpha_min), second-order corrections (max_soc 4);
  * a feasibility restoration phase (minimum-norm Gauss-Newton steps on the
    constraint violation until the filter accepts the point);
  * the convergence test (scaled optimality error <= tol together with the
    unscaled constr_viol_tol / dual_inf_tol / compl_inf_tol) and the
    "acceptable" termination.

The KKT systems are solved with SuperLU (scipy.sparse.linalg.splu) on the
reduced system [[D_x + B, J^T], [J, -Dc]], slacks eliminated.  It is a
substitute for Ipopt + MUMPS, not Ipopt: the algorithm is the same, the
linear solver, the restoration phase and many safeguards differ, so iterate
sequences are not identical; converged solutions of well-posed problems
agree to the tolerances.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp
from scipy.sparse.linalg import splu


@dataclass
class IpmOptions:
    """Ipopt option names and defaults (Ipopt 3.12 documentation)."""
    tol: float = 1e-8
    dual_inf_tol: float = 1.0
    constr_viol_tol: float = 1e-4
    compl_inf_tol: float = 1e-4
    acceptable_tol: float = 1e-6
    acceptable_iter: int = 15
    acceptable_dual_inf_tol: float = 1e10
    acceptable_constr_viol_tol: float = 1e-2
    acceptable_compl_inf_tol: float = 1e-2
    max_iter: int = 3000
    mu_init: float = 0.1
    mu_min: float = 1e-11
    # the tol-derived floor of Ipopt 3.12's monotone barrier update
    # (MonotoneMuUpdate::CalcNewMuAndTau: mu >= min(tol, compl_inf_tol) /
    # (barrier_tol_factor + 1)).  Off by default: the reference's golden
    # MocoInverse solution sits at a barrier parameter ~1e-6 (its
    # activations' distances to their bounds times this solve's bound
    # multipliers), the unfloored sequence's last mu (1.8e-6), where the
    # floor would hold mu at 9.1e-5 -- and the floored solve is exactly the
    # barrier problem's solution there (objective 1.1260, controls RMS 0.026
    # against the file, over testMocoInverse's 1e-2), not an early stop:
    # tests/test_mu_floor.py, tools/mu_floor_probe.py
    mu_floor_from_tol: bool = False
    kappa_eps: float = 10.0
    kappa_mu: float = 0.2
    theta_mu: float = 1.5
    tau_min: float = 0.99
    bound_push: float = 1e-2
    bound_frac: float = 1e-2
    bound_relax_factor: float = 1e-8
    bound_mult_init_val: float = 1.0
    constr_mult_init_max: float = 1e3
    nlp_scaling_max_gradient: float = 100.0
    nlp_scaling_min_value: float = 1e-8
    limited_memory_max_history: int = 6
    limited_memory_init_val: float = 1.0
    max_soc: int = 4
    # the Newton systems' linear algebra: "host" (scipy / LAPACK over J
    # copied to the host), "device" (include/mocohip_kkt.h: J stays in HBM,
    # the Schur complement is factored on the GPU), "auto" (device when the
    # NLP offers a device KKT module -- HipNLP --, its Jacobian has the
    # per-interval block structure and it has at least
    # device_kkt_min_constraints rows, else host: below that a banded host
    # factorization costs less than the device's per-call latency chain --
    # Rajagopal-18's MocoInverse, m = 1347, solves in 0.25 s on the host and
    # 0.65 s on the device; the gait MocoInverse at N = 125, m = 16046, in
    # 1.27 s and 0.57 s)
    linear_solver: str = "auto"
    device_kkt_min_constraints: int = 5000
    kappa_soc: float = 0.99
    # after the restoration phase (Ipopt 3.12 IpRestoMinC_1Nrm): the least-
    # squares constraint multipliers are kept only when their max-norm is at
    # most constr_mult_reset_threshold (default 0: they are set to zero), and
    # the bound multipliers are reset to 1 when their max-norm exceeds
    # bound_mult_reset_threshold
    constr_mult_reset_threshold: float = 0.0
    bound_mult_reset_threshold: float = 1000.0
    print_level: int = 0
    # filter line search constants (Waechter & Biegler 2006, Table 1)
    gamma_theta: float = 1e-5
    gamma_phi: float = 1e-8
    eta_phi: float = 1e-8
    delta: float = 1.0
    s_theta: float = 1.1
    s_phi: float = 2.3
    kappa_sigma: float = 1e10
    kappa_d: float = 1e-5
    s_max: float = 100.0

    @classmethod
    def from_ipopt(cls, opts: dict) -> "IpmOptions":
        """Options from an Ipopt option dictionary (MocoHipSolver.ipopt_options:
        tol, dual_inf_tol, compl_inf_tol, acceptable_*, constr_viol_tol,
        max_iter, print_level ...); unknown keys are ignored."""
        o = cls()
        for k, v in opts.items():
            if hasattr(o, k) and (not isinstance(v, str) or isinstance(getattr(o, k), str)):
                # Ipopt's own linear_solver names its sparse factorization
                # ('mumps', 'ma27', ... as MocoCasADiSolver / tropter pass it):
                # not this option's values (the Newton systems' back end here)
                if k == "linear_solver" and v not in ("auto", "host", "device"):
                    continue
                setattr(o, k, type(getattr(o, k))(v))
        return o


@dataclass
class IpmResult:
    x: np.ndarray
    success: bool
    status: str
    objective: float
    iterations: int
    duration: float
    constraint_violation: float
    evaluations: dict
    lambda_g: Optional[np.ndarray] = None
    z_l: Optional[np.ndarray] = None
    z_u: Optional[np.ndarray] = None
    history: list = field(default_factory=list)
    timings: dict = field(default_factory=dict)


class _LBFGS:
    """Compact limited-memory BFGS matrix B = sigma I - W M W^T,
    W = [sigma S, Y], M^{-1} = [[sigma S^T S, L], [L^T, -D]] (Byrd, Nocedal,
    Schnabel 1994, (2.17)); pairs failing the curvature test are skipped."""

    def __init__(self, n: int, k: int, sigma0: float):
        self.n, self.k = n, k
        self.S: list = []
        self.Y: list = []
        self.sigma = sigma0

    def update(self, s: np.ndarray, y: np.ndarray):
        sy = float(s @ y)
        ss = float(s @ s)
        if ss <= 0.0 or sy <= math.sqrt(np.finfo(float).eps) * math.sqrt(ss) * float(np.linalg.norm(y)):
            return False
        self.S.append(s.copy())
        self.Y.append(y.copy())
        if len(self.S) > self.k:
            self.S.pop(0)
            self.Y.pop(0)
        # scalar1 initialization, bounded like Ipopt's limited_memory_init_val_min/max
        self.sigma = min(max(sy / ss, 1e-8), 1e8)
        return True

    def compact(self):
        """(W, Minv) or None when no pair is stored."""
        if not self.S:
            return None
        S = np.array(self.S).T
        Y = np.array(self.Y).T
        SY = S.T @ Y
        L = np.tril(SY, -1)
        D = np.diag(np.diag(SY))
        Minv = np.block([[self.sigma * (S.T @ S), L], [L.T, -D]])
        W = np.hstack([self.sigma * S, Y])
        return W, Minv


class _Scaled:
    """The NLP as the interior-point method sees it: free variables x, slack
    variables s of the inequality rows, constraints C(x, s) = [c_eq(x);
    c_in(x) - s], objective and rows scaled (gradient-based scaling)."""

    def __init__(self, nlp, x0: np.ndarray, opt: IpmOptions):
        self.nlp = nlp
        self.n_full, self.m_full = int(nlp.n), int(nlp.m)
        xl, xu, gl, gu = nlp.bounds()
        xl = np.asarray(xl[:self.n_full], float).copy()
        xu = np.asarray(xu[:self.n_full], float).copy()
        gl = np.asarray(gl[:self.m_full], float).copy()
        gu = np.asarray(gu[:self.m_full], float).copy()
        # rows with both bounds infinite constrain nothing (their slack would
        # have no barrier term): left out of the problem the method sees
        self.rows = np.where(~(np.isneginf(gl) & np.isposinf(gu)))[0]
        self.m = len(self.rows)
        row_map = -np.ones(self.m_full, np.int64)
        row_map[self.rows] = np.arange(self.m)
        gl, gu = gl[self.rows], gu[self.rows]
        self.xl_full, self.xu_full = xl, xu
        self.gl, self.gu = gl, gu
        self.fixed = np.isfinite(xl) & (xl == xu)
        self.free = np.where(~self.fixed)[0]
        self.nx = len(self.free)
        self.x_full = np.clip(np.asarray(x0, float), xl, xu)
        self.x_full[self.fixed] = xl[self.fixed]
        self.eq = np.where(gl == gu)[0]
        self.ineq = np.where(gl != gu)[0]
        self.ns = len(self.ineq)
        ir, jc = nlp.jac_structure()
        ir = np.asarray(ir[:nlp.nnz], np.int64)
        jc = np.asarray(jc[:nlp.nnz], np.int64)
        col_map = -np.ones(self.n_full, np.int64)
        col_map[self.free] = np.arange(self.nx)
        keep = (col_map[jc] >= 0) & (row_map[ir] >= 0)
        self.keep = np.where(keep)[0]
        self.ir, self.jc = row_map[ir[keep]], col_map[jc[keep]]
        self._csr = None          # host CSR pattern of J_x, built on first use (host linear algebra)
        self.counts = {"f": 0, "grad_f": 0, "g": 0, "jac_g": 0}
        self.eval_time = 0.0
        # bounds of v = [x, s] (relaxed, bound_relax_factor)
        lo = np.concatenate([xl[self.free], gl[self.ineq]])
        hi = np.concatenate([xu[self.free], gu[self.ineq]])
        self.obj_scale = 1.0
        self.row_scale = np.ones(self.m)
        self._set_scaling(opt)
        lo = lo.copy()
        hi = hi.copy()
        lo[self.nx:] *= self.row_scale[self.ineq]
        hi[self.nx:] *= self.row_scale[self.ineq]
        r = opt.bound_relax_factor
        fl, fu = np.isfinite(lo), np.isfinite(hi)
        lo[fl] -= r * np.maximum(1.0, np.abs(lo[fl]))
        hi[fu] += r * np.maximum(1.0, np.abs(hi[fu]))
        self.lo, self.hi = lo, hi
        self.has_lo, self.has_hi = fl, fu

    # -- evaluations (scaled) ----------------------------------------------
    def _x(self, v):
        x = self.x_full.copy()
        x[self.free] = v[:self.nx]
        return x

    def _timed(self, name, fn, *a):
        t = time.perf_counter()
        r = fn(*a)
        self.eval_time += time.perf_counter() - t
        self.counts[name] += 1
        return r

    def f(self, v):
        return self.obj_scale * float(self._timed("f", self.nlp.eval_f, self._x(v)))

    def grad_f(self, v):
        g = np.asarray(self._timed("grad_f", self.nlp.eval_grad_f, self._x(v)), float)
        return self.obj_scale * np.concatenate([g[self.free], np.zeros(self.ns)])

    def g_raw(self, v):
        return np.asarray(self._timed("g", self.nlp.eval_g, self._x(v)), float)[self.rows]

    def C(self, v, graw=None):
        g = self.g_raw(v) if graw is None else graw
        c = np.empty(self.m)
        c[self.eq] = self.row_scale[self.eq] * (g[self.eq] - self.gl[self.eq])
        c[self.ineq] = self.row_scale[self.ineq] * g[self.ineq] - v[self.nx:]
        return c

    def jac_vals(self, v):
        vals = np.asarray(self._timed("jac_g", self.nlp.eval_jac_g, self._x(v)), float)[:self.nlp.nnz]
        return vals[self.keep]

    def Jx(self, vals):
        """Scaled J_x (m x nx, CSR) from the kept Jacobian values."""
        data = (vals * self.row_scale[self.ir])[self.order]
        return sp.csr_matrix((data, self.indices, self.indptr), shape=(self.m, self.nx))

    def _csr_pattern(self):
        """(order, indptr, indices): the CSR pattern of J_x and the
        permutation of the kept values into it (the host linear algebra's;
        the device path never builds it)."""
        if self._csr is None:
            order = np.lexsort((self.jc, self.ir))
            indptr = np.concatenate([[0], np.cumsum(np.bincount(self.ir, minlength=self.m))]).astype(np.int64)
            self._csr = (order, indptr, self.jc[order])
        return self._csr

    @property
    def order(self):
        return self._csr_pattern()[0]

    @property
    def indptr(self):
        return self._csr_pattern()[1]

    @property
    def indices(self):
        return self._csr_pattern()[2]

    def _set_scaling(self, opt: IpmOptions):
        """Gradient-based scaling at the starting point (Ipopt
        nlp_scaling_method = gradient-based)."""
        v0 = np.concatenate([self.x_full[self.free], np.zeros(self.ns)])
        gf = self.grad_f(v0)
        mx = float(np.abs(gf).max(initial=0.0))
        self.obj_scale = min(1.0, opt.nlp_scaling_max_gradient / mx) if mx > 0 else 1.0
        self.obj_scale = max(self.obj_scale, opt.nlp_scaling_min_value)
        gf *= self.obj_scale / max(self.obj_scale, 1e-300)
        if self.m:
            vals = self.jac_vals(v0)
            rmax = np.zeros(self.m)
            np.maximum.at(rmax, self.ir, np.abs(vals))
            with np.errstate(divide="ignore"):
                s = np.where(rmax > 0, opt.nlp_scaling_max_gradient / rmax, 1.0)
            self.row_scale = np.clip(np.minimum(1.0, s), opt.nlp_scaling_min_value, 1.0)

    def unscaled_violation(self, v, graw=None):
        g = self.g_raw(v) if graw is None else graw
        return float(np.max(np.concatenate([[0.0], self.gl - g, g - self.gu]))) if self.m else 0.0


def _linear_algebra(nlp, P, opt):
    """The Newton systems' back end (IpmOptions.linear_solver)."""
    want = opt.linear_solver
    if want not in ("auto", "host", "device"):
        raise ValueError("linear_solver must be 'auto', 'host' or 'device'")
    big = P.m >= opt.device_kkt_min_constraints
    if (want == "device" or (want == "auto" and big)) and P.m and hasattr(nlp, "device_kkt"):
        try:
            dk = nlp.device_kkt()
        except (ValueError, RuntimeError):
            if want == "device":
                raise
            dk = None
        if dk is not None:
            return _DevLA(P, dk)
    if want == "device":
        raise ValueError("linear_solver='device' needs an NLP with a device KKT module (HipNLP)")
    return _HostLA(P)


def _ftb(v, dv, lo, hi, tau):
    """Largest alpha in (0, 1] with v + alpha dv >= v - tau (v - lo) (and
    the same for the upper bounds): the fraction-to-the-boundary rule."""
    a = 1.0
    m = np.isfinite(lo) & (dv < 0)
    if m.any():
        a = min(a, float(np.min(-tau * (v[m] - lo[m]) / dv[m])))
    m = np.isfinite(hi) & (dv > 0)
    if m.any():
        a = min(a, float(np.min(tau * (hi[m] - v[m]) / dv[m])))
    return max(a, 0.0)


def _ftb_pos(z, dz, tau):
    a = 1.0
    m = dz < 0
    if m.any():
        a = min(a, float(np.min(-tau * z[m] / dz[m])))
    return max(a, 0.0)


class _KKTBase:
    """Solves with K = [[D_x + B, J^T], [J, -Dc]] (slacks eliminated) through
    the Schur complement S = J D_x^-1 J^T + Dc of K0 (B = 0); the dense
    columns (free initial / final time) are taken out of S and put back with
    Sherman-Morrison-Woodbury, as is the limited-memory term B = -W M W^T.
    Subclasses provide S0^-1 (_s0) and the products with J (_mv, _rmv)."""

    def _lowrank(self, Dx, dense, Jd, lbfgs_compact):
        self.Sd = None
        if len(dense):
            Zd = self._s0(Jd)
            Td = np.diag(Dx[dense]) + Jd.T @ Zd
            self.Sd = (Jd, Zd, np.linalg.inv(Td))
        self.low = None
        if lbfgs_compact is not None:
            W, Minv = lbfgs_compact
            P = np.zeros((self.nx + self.m, W.shape[1]))
            P[:self.nx] = W
            Z = self._solve0_once(P)
            T = Minv - P.T @ Z
            self.low = (P, Z, np.linalg.inv(T))

    def _ssolve(self, t):
        u = self._s0(t)
        if self.Sd is not None:
            Jd, Zd, Tinv = self.Sd
            u = u - Zd @ (Tinv @ (Jd.T @ u))
        return u

    def _solve0_once(self, b):
        nx = self.nx
        rx, rc = b[:nx], b[nx:]
        Dx = self.Dx if b.ndim == 1 else self.Dx[:, None]
        dy = self._ssolve(self._mv(rx / Dx) - rc)
        dx = (rx - self._rmv(dy)) / Dx
        return np.concatenate([dx, dy]) if b.ndim == 1 else np.vstack([dx, dy])

    def _K0(self, u):
        nx = self.nx
        ux, uy = u[:nx], u[nx:]
        Dx = self.Dx if u.ndim == 1 else self.Dx[:, None]
        dc = self.dc if u.ndim == 1 else self.dc[:, None]
        top = Dx * ux + self._rmv(uy)
        bot = self._mv(ux) - dc * uy
        return np.concatenate([top, bot]) if u.ndim == 1 else np.vstack([top, bot])

    def _solve0(self, b):
        u = self._solve0_once(b)
        return u + self._solve0_once(b - self._K0(u))   # one step of iterative refinement

    def solve(self, rx, rs, rc):
        """Solve [[B + D_x, 0, J_x^T], [0, D_s, -E^T], [J_x, -E, -delta_c]]
        [dx; ds; dy] = [rx; rs; rc]; E selects the inequality rows."""
        rc2 = rc.copy()
        # ds = (rs + dy_in) / Ds  ->  row block: J dx - (1/Ds) dy_in - dc dy = rc + rs / Ds
        rc2[self.Js_idx] += rs / self.Ds
        b = np.concatenate([rx, rc2])
        u = self._solve0(b)
        if self.low is not None:
            P, Z, Tinv = self.low
            u = u + Z @ (Tinv @ (P.T @ u))
        dx, dy = u[:self.nx], u[self.nx:]
        ds = (rs + dy[self.Js_idx]) / self.Ds
        return dx, ds, dy


class _KKT(_KKTBase):
    """Host linear algebra: S is banded for a transcription (rows and
    columns ordered by mesh interval) and is factored by LAPACK's banded
    Cholesky, or by SuperLU in its natural order (MMD) when the band is
    wide."""

    def __init__(self, Jx, Js_idx, Dx, Ds, delta_c, lbfgs_compact, m):
        Jx = Jx.csr if isinstance(Jx, _HostJ) else Jx
        self.nx = Jx.shape[1]
        self.m = m
        self.J = Jx
        self.JT = Jx.T.tocsr()
        self.Js_idx = Js_idx
        self.Ds = Ds
        self.Dx = Dx
        dc = np.full(m, float(delta_c))
        dc[Js_idx] += 1.0 / Ds
        self.dc = dc
        # dense columns (t0 / tf) out of the banded part
        colnnz = np.diff(Jx.tocsc().indptr)
        thresh = max(64, 8 * int(np.median(colnnz)) if len(colnnz) else 64)
        dense = np.where(colnnz > thresh)[0] if m > 256 else np.zeros(0, int)
        self.dense = dense
        keep = np.ones(self.nx, bool)
        keep[dense] = False
        Jb = Jx[:, np.where(keep)[0]]
        S = (Jb @ sp.diags(1.0 / Dx[keep]) @ Jb.T + sp.diags(dc)).tocsr().tocoo()   # canonical
        band = int(np.abs(S.row - S.col).max(initial=0))
        self.band = None
        if m and band * 4 < m:
            # banded Cholesky (LAPACK pbtrf): S is symmetric positive
            # definite unless J is rank deficient (then delta_c > 0 is retried);
            # S is canonical (no duplicate entries), so its lower band is
            # scattered by plain assignment
            low = S.row >= S.col
            ab = np.zeros((band + 1, m))
            ab[S.row[low] - S.col[low], S.col[low]] = S.data[low]
            try:
                self.band = sla.cholesky_banded(ab, lower=True, check_finite=False)
            except np.linalg.LinAlgError as e:
                raise RuntimeError(str(e))
        else:
            self.lu = splu(S.tocsc(), permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=0.1,
                           options={"SymmetricMode": True})
        self._lowrank(Dx, dense, Jx[:, dense].toarray() if len(dense) else None, lbfgs_compact)

    def _mv(self, d):
        return self.J @ d

    def _rmv(self, y):
        return self.JT @ y

    def _s0(self, t):
        if self.band is not None:
            return sla.cho_solve_banded((self.band, True), t, check_finite=False)
        return self.lu.solve(t)


class _HostJ:
    """J_x (scaled, free columns) as a host CSR matrix."""

    def __init__(self, csr):
        self.csr = csr
        self._t = None

    def mv(self, d):
        return self.csr @ d

    def rmv(self, y):
        if self._t is None:
            self._t = self.csr.T.tocsr()
        return self._t @ y


class _HostLA:
    """The host linear algebra: J's values copied to the host every
    iteration, scipy / LAPACK factorizations."""
    name = "host (scipy: banded LAPACK Cholesky / SuperLU)"

    def __init__(self, P):
        self.P = P

    def jac(self, v):
        P = self.P
        if not P.m:
            return _HostJ(sp.csr_matrix((0, P.nx)))
        return _HostJ(P.Jx(P.jac_vals(v)))

    def kkt(self, J, Js_idx, Dx, Ds, delta_c, lbfgs_compact, m):
        return _KKT(J, Js_idx, Dx, Ds, delta_c, lbfgs_compact, m)


class _DevJ:
    """J_x (scaled, free columns) resident on the device (mocohip.kkt
    DeviceKKT's blocks): products cross the bus as vectors."""

    def __init__(self, la):
        self.la = la

    def mv(self, d):
        P, dk = self.la.P, self.la.dk
        full = np.zeros((P.n_full,) + d.shape[1:])
        full[P.free] = d
        return dk.jmul(full)[P.rows]

    def rmv(self, y):
        P, dk = self.la.P, self.la.dk
        full = np.zeros((P.m_full,) + y.shape[1:])
        full[P.rows] = y
        return dk.jtmul(full)[P.free]


class _DevLA:
    """The device linear algebra (include/mocohip_kkt.h): J evaluated into
    device memory by the context's own kernels and never copied back; the
    Schur complement over the block columns formed and factored on the
    device by block cyclic reduction (csrc/kkt.hip); the dense columns (t0,
    tf) and the limited-memory term through Sherman-Morrison-Woodbury on the
    host, as in the host path."""
    name = "device (mh_kkt: block cyclic reduction of the Schur complement on the GPU)"

    def __init__(self, P, dk):
        self.P, self.dk = P, dk
        rs = np.zeros(P.m_full)
        rs[P.rows] = P.row_scale
        dk.set_row_scale(rs)
        col_map = -np.ones(P.n_full, np.int64)
        col_map[P.free] = np.arange(P.nx)
        d = col_map[dk.bm.dcols]
        self.dense_nx = d[d >= 0]                 # dense free columns, in the free-column index
        self.dense_sel = np.where(d >= 0)[0]      # their position among the dense columns
        self.dense_free = dk.bm.dcols[d >= 0]     # their global index

    def jac(self, v):
        P = self.P
        t = time.perf_counter()
        self.dk.eval_jacobian(P._x(v))
        P.eval_time += time.perf_counter() - t
        P.counts["jac_g"] += 1
        return _DevJ(self)

    def kkt(self, J, Js_idx, Dx, Ds, delta_c, lbfgs_compact, m):
        return _DevKKT(self, Js_idx, Dx, Ds, delta_c, lbfgs_compact, m)


class _DevKKT(_KKTBase):
    def __init__(self, la, Js_idx, Dx, Ds, delta_c, lbfgs_compact, m):
        P, dk = la.P, la.dk
        self.la, self.P, self.dk = la, P, dk
        self.nx, self.m = P.nx, m
        self.Js_idx, self.Ds, self.Dx = Js_idx, Ds, Dx
        dc = np.full(m, float(delta_c))
        dc[Js_idx] += 1.0 / Ds
        self.dc = dc
        w = np.zeros(P.n_full)
        w[P.free] = 1.0 / Dx
        w[dk.bm.dcols] = 0.0
        dcf = np.ones(P.m_full)              # rows the method leaves out: unit pivots, zero rows of J
        dcf[P.rows] = dc
        if not dk.factor(w, dcf):
            raise RuntimeError("device KKT factorization: non-positive pivot")
        self._J = _DevJ(la)
        Jd = None
        if len(la.dense_nx):
            _, Jd_all = dk.dense_columns()
            Jd = Jd_all[P.rows][:, la.dense_sel]
        self._lowrank(Dx, la.dense_nx, Jd, lbfgs_compact)

    def _mv(self, d):
        return self._J.mv(d)

    def _rmv(self, y):
        return self._J.rmv(y)

    def _s0(self, t):
        P = self.P
        full = np.zeros((P.m_full,) + t.shape[1:])
        full[P.rows] = t
        return self.dk.solve(full)[P.rows]


def solve_ipm(nlp, x0: np.ndarray, options: Optional[IpmOptions] = None) -> IpmResult:
    """Minimize nlp.eval_f subject to nlp's bounds and g bounds from x0.

    The host linear algebra runs with single-threaded BLAS: the banded
    Cholesky (LAPACK pbtrf) of a transcription's Schur complement is a chain
    of small blocks, on which OpenBLAS's threads cost ~100x (gait MocoInverse
    N=125: m = 16,046, band 164: 4.8 s threaded against 0.057 s on one
    thread, measured on this repository's host)."""
    try:
        from threadpoolctl import threadpool_limits
    except ImportError:   # pragma: no cover - threadpoolctl ships with scikit-learn
        return _solve_ipm(nlp, x0, options)
    with threadpool_limits(1, user_api="blas"):
        return _solve_ipm(nlp, x0, options)


def _solve_ipm(nlp, x0: np.ndarray, options: Optional[IpmOptions] = None) -> IpmResult:
    opt = options or IpmOptions()
    t_start = time.perf_counter()
    P = _Scaled(nlp, x0, opt)
    nx, ns, m = P.nx, P.ns, P.m
    nv = nx + ns
    lo, hi, hl, hu = P.lo, P.hi, P.has_lo, P.has_hi
    t_lin = 0.0

    # ---- starting point (Ipopt's push into the interior) ----------------
    v = np.concatenate([P.x_full[P.free], np.zeros(ns)])
    graw = P.g_raw(v)
    v[nx:] = P.row_scale[P.ineq] * graw[P.ineq]
    both = hl & hu
    pl = np.where(hl, opt.bound_push * np.maximum(1.0, np.abs(lo)), 0.0)
    pu = np.where(hu, opt.bound_push * np.maximum(1.0, np.abs(hi)), 0.0)
    with np.errstate(invalid="ignore"):
        pl = np.where(both, np.minimum(pl, opt.bound_frac * (hi - lo)), pl)
        pu = np.where(both, np.minimum(pu, opt.bound_frac * (hi - lo)), pu)
    v = np.where(hl, np.maximum(v, lo + pl), v)
    v = np.where(hu, np.minimum(v, hi - pu), v)
    zl = np.where(hl, opt.bound_mult_init_val, 0.0)
    zu = np.where(hu, opt.bound_mult_init_val, 0.0)
    only_lo = hl & ~hu
    only_hi = hu & ~hl

    mu = opt.mu_init
    tau = max(opt.tau_min, 1.0 - mu)
    lb = _LBFGS(nx, opt.limited_memory_max_history, opt.limited_memory_init_val)

    def barrier(v_, f_):
        with np.errstate(divide="ignore", invalid="ignore"):
            r = f_ - mu * (np.sum(np.log(v_[hl] - lo[hl])) + np.sum(np.log(hi[hu] - v_[hu])))
        r += opt.kappa_d * mu * (np.sum(v_[only_lo] - lo[only_lo]) + np.sum(hi[only_hi] - v_[only_hi]))
        return r if np.isfinite(r) else np.inf

    def barrier_grad(v_, gf_):
        gb = gf_.copy()
        gb[hl] -= mu / (v_[hl] - lo[hl])
        gb[hu] += mu / (hi[hu] - v_[hu])
        gb[only_lo] += opt.kappa_d * mu
        gb[only_hi] -= opt.kappa_d * mu
        return gb

    def JT(Jx, y):
        r = np.empty(nv)
        r[:nx] = Jx.rmv(y)
        r[nx:] = -y[P.ineq]
        return r

    la = _linear_algebra(nlp, P, opt)
    f = P.f(v)
    c = P.C(v, graw)
    gf = P.grad_f(v)
    Jx = la.jac(v)
    # least-squares constraint multipliers (constr_mult_init_max)
    y = np.zeros(m)
    if m:
        try:
            kk = la.kkt(Jx, P.ineq, np.ones(nx), np.ones(ns), 0.0, None, m)
            _, _, y = kk.solve(-(gf[:nx] - zl[:nx] + zu[:nx]), -(gf[nx:] - zl[nx:] + zu[nx:]), np.zeros(m))
            if not np.all(np.isfinite(y)) or np.abs(y).max(initial=0) > opt.constr_mult_init_max:
                y = np.zeros(m)
        except (RuntimeError, np.linalg.LinAlgError):
            y = np.zeros(m)

    theta = float(np.abs(c).sum())
    theta_max = 1e4 * max(1.0, theta)
    theta_min = 1e-4 * max(1.0, theta)
    filt: list = []
    history = []
    acceptable_count = 0
    status = "Maximum_Iterations_Exceeded"
    success = False
    it = 0
    delta_c_last = 0.0
    prev = None      # (x part, gradient of the Lagrangian parts) for the BFGS pair

    def errors(v_, gf_, Jx_, c_, y_, zl_, zu_, mu_):
        gL = gf_ + JT(Jx_, y_) - zl_ + zu_
        dual = float(np.abs(gL).max(initial=0.0))
        primal = float(np.abs(c_).max(initial=0.0))
        with np.errstate(invalid="ignore"):
            cl = np.where(hl, (v_ - lo) * zl_ - mu_, 0.0)
            cu = np.where(hu, (hi - v_) * zu_ - mu_, 0.0)
        compl = float(max(np.abs(cl).max(initial=0.0), np.abs(cu).max(initial=0.0)))
        nb = int(hl.sum() + hu.sum())
        zsum = float(np.abs(zl_).sum() + np.abs(zu_).sum())
        sd = max(opt.s_max, (float(np.abs(y_).sum()) + zsum) / max(1, m + nb)) / opt.s_max
        sc = max(opt.s_max, zsum / max(1, nb)) / opt.s_max
        return dual, primal, compl, sd, sc

    while True:
        dual, primal, compl0, sd, sc = errors(v, gf, Jx, c, y, zl, zu, 0.0)
        E0 = max(dual / sd, primal, compl0 / sc)
        viol_u = P.unscaled_violation(v, graw)
        dual_u = dual / P.obj_scale
        compl_u = compl0 / P.obj_scale
        history.append((it, f / P.obj_scale, viol_u, dual_u, mu))
        if opt.print_level:
            print(f"iter {it:4d} f {f / P.obj_scale: .8e} inf_pr {viol_u:.2e} inf_du {dual_u:.2e} "
                  f"mu {mu:.1e} E0 {E0:.2e}")
        if (E0 <= opt.tol and viol_u <= opt.constr_viol_tol and dual_u <= opt.dual_inf_tol
                and compl_u <= opt.compl_inf_tol):
            status, success = "Solve_Succeeded", True
            break
        if (E0 <= opt.acceptable_tol and viol_u <= opt.acceptable_constr_viol_tol
                and dual_u <= opt.acceptable_dual_inf_tol and compl_u <= opt.acceptable_compl_inf_tol):
            acceptable_count += 1
            if acceptable_count >= opt.acceptable_iter:
                status, success = "Solved_To_Acceptable_Level", True
                break
        else:
            acceptable_count = 0
        if it >= opt.max_iter:
            break
        # ---- barrier parameter (monotone Fiacco-McCormick) -----------------
        while True:
            d_, p_, cm, sd_, sc_ = errors(v, gf, Jx, c, y, zl, zu, mu)
            Emu = max(d_ / sd_, p_, cm / sc_)
            if Emu > opt.kappa_eps * mu:
                break
            # Ipopt's MonotoneMuUpdate::CalcNewMuAndTau: the superlinear
            # decrease, bounded below by min(tol, compl_inf_tol) /
            # (barrier_tol_factor + 1) and by mu_min
            mu_new = min(opt.kappa_mu * mu, mu ** opt.theta_mu)
            if opt.mu_floor_from_tol:
                mu_new = max(mu_new, min(opt.tol, opt.compl_inf_tol) / (opt.kappa_eps + 1.0))
            mu_new = max(opt.mu_min, mu_new)
            if mu_new >= mu:
                break
            mu = mu_new
            tau = max(opt.tau_min, 1.0 - mu)
            filt = []
        # ---- Newton direction --------------------------------------------
        sig_l = np.where(hl, zl / np.where(hl, v - lo, 1.0), 0.0)
        sig_u = np.where(hu, zu / np.where(hu, hi - v, 1.0), 0.0)
        Sig = sig_l + sig_u
        comp = lb.compact()
        Dx = Sig[:nx] + lb.sigma
        Ds = Sig[nx:].copy()
        gb = barrier_grad(v, gf)
        rhs_v = -(gb + JT(Jx, y))
        t0 = time.perf_counter()
        kkt = None
        delta_c = 0.0
        for attempt in range(6):
            try:
                kkt = la.kkt(Jx, P.ineq, Dx, Ds, delta_c, comp, m)
                dx, ds, dy = kkt.solve(rhs_v[:nx], rhs_v[nx:], -c)
                if np.all(np.isfinite(dx)) and np.all(np.isfinite(dy)):
                    break
            except (RuntimeError, np.linalg.LinAlgError):
                pass
            delta_c = 1e-8 * mu ** 0.25 if delta_c == 0.0 else delta_c * 100.0
            kkt = None
        t_lin += time.perf_counter() - t0
        if kkt is None:
            status = "Error_In_Step_Computation"
            break
        delta_c_last = delta_c
        dv = np.concatenate([dx, ds])
        dzl = np.where(hl, mu / np.where(hl, v - lo, 1.0) - zl - sig_l * dv, 0.0)
        dzu = np.where(hu, mu / np.where(hu, hi - v, 1.0) - zu + sig_u * dv, 0.0)
        a_max = _ftb(v, dv, lo, hi, tau)
        a_z = min(_ftb_pos(zl[hl], dzl[hl], tau), _ftb_pos(zu[hu], dzu[hu], tau))
        # ---- filter line search -------------------------------------------
        phi = barrier(v, f)
        gphi_d = float(gb @ dv)
        theta = float(np.abs(c).sum())
        if gphi_d < 0:
            a_min = 0.05 * min(opt.gamma_theta, opt.gamma_phi * theta / -gphi_d,
                               opt.delta * theta ** opt.s_theta / (-gphi_d) ** opt.s_phi
                               if theta <= theta_min else np.inf)
        else:
            a_min = 0.05 * opt.gamma_theta
        a_min = max(a_min, 1e-16)

        def acceptable(theta_t, phi_t, alpha):
            if not np.isfinite(phi_t) or theta_t > theta_max:
                return False, False
            switching = gphi_d < 0 and alpha * (-gphi_d) ** opt.s_phi > opt.delta * theta ** opt.s_theta
            if switching and theta <= theta_min:
                ok = phi_t <= phi + opt.eta_phi * alpha * gphi_d
                ftype = True
            else:
                ok = theta_t <= (1 - opt.gamma_theta) * theta or phi_t <= phi - opt.gamma_phi * theta
                ftype = False
            if ok:
                for (tj, pj) in filt:
                    if not (theta_t <= tj or phi_t <= pj):
                        return False, ftype
            return ok, ftype

        alpha = a_max
        accepted = False
        ftype = False
        vt = ft = ct = gt = None
        first = True
        while alpha >= a_min:
            vt = v + alpha * dv
            ft = P.f(vt)
            gt = P.g_raw(vt)
            ct = P.C(vt, gt)
            theta_t = float(np.abs(ct).sum())
            phi_t = barrier(vt, ft)
            ok, ftype = acceptable(theta_t, phi_t, alpha)
            if ok:
                accepted = True
                break
            if first and theta_t >= theta and m:
                # second-order corrections
                c_soc = alpha * c + ct
                theta_old = theta
                for _ in range(opt.max_soc):
                    dx2, ds2, dy2 = kkt.solve(rhs_v[:nx], rhs_v[nx:], -c_soc)
                    dv2 = np.concatenate([dx2, ds2])
                    a2 = _ftb(v, dv2, lo, hi, tau)
                    vs = v + a2 * dv2
                    fs = P.f(vs)
                    gs = P.g_raw(vs)
                    cs = P.C(vs, gs)
                    th_s = float(np.abs(cs).sum())
                    ph_s = barrier(vs, fs)
                    ok, ftype = acceptable(th_s, ph_s, alpha)
                    if ok:
                        vt, ft, gt, ct, dv, alpha = vs, fs, gs, cs, dv2, a2
                        dy = dy2
                        dzl = np.where(hl, mu / np.where(hl, v - lo, 1.0) - zl - sig_l * dv, 0.0)
                        dzu = np.where(hu, mu / np.where(hu, hi - v, 1.0) - zu + sig_u * dv, 0.0)
                        a_z = min(_ftb_pos(zl[hl], dzl[hl], tau), _ftb_pos(zu[hu], dzu[hu], tau))
                        accepted = True
                        break
                    if th_s > opt.kappa_soc * theta_old:
                        break
                    theta_old = th_s
                    c_soc = a2 * c_soc + cs
                if accepted:
                    break
            first = False
            alpha *= 0.5
        if not accepted:
            # ---- feasibility restoration --------------------------------
            r = _restore(P, la, v, c, Jx, lo, hi, hl, hu, Sig, tau, filt, theta, phi, barrier, opt, m, nx)
            if r is None:
                status = "Restoration_Failed"
                break
            vt, ft, gt, ct = r
            filt.append(((1 - opt.gamma_theta) * theta, phi - opt.gamma_phi * theta))
            # reset the multipliers: least squares for y, bound multipliers kept
            v_old_x = v[:nx].copy()
            v = vt
            f, graw, c = ft, gt, ct
            gf = P.grad_f(v)
            Jx = la.jac(v)
            if max(float(np.abs(zl).max(initial=0.0)), float(np.abs(zu).max(initial=0.0))) \
                    > opt.bound_mult_reset_threshold:
                zl = np.where(hl, 1.0, 0.0)
                zu = np.where(hu, 1.0, 0.0)
            y = np.zeros(m)
            if opt.constr_mult_reset_threshold > 0:
                try:
                    kk = la.kkt(Jx, P.ineq, np.ones(nx), np.ones(ns), 0.0, None, m)
                    _, _, y = kk.solve(-(gf[:nx] - zl[:nx] + zu[:nx]), -(gf[nx:] - zl[nx:] + zu[nx:]),
                                       np.zeros(m))
                    if not np.all(np.isfinite(y)) or np.abs(y).max(initial=0) > opt.constr_mult_reset_threshold:
                        y = np.zeros(m)
                except (RuntimeError, np.linalg.LinAlgError):
                    y = np.zeros(m)
            lb = _LBFGS(nx, opt.limited_memory_max_history, opt.limited_memory_init_val)
            prev = None
            it += 1
            continue
        if not ftype or not (ft is not None and barrier(vt, ft) <= phi + opt.eta_phi * alpha * gphi_d):
            filt.append(((1 - opt.gamma_theta) * theta, phi - opt.gamma_phi * theta))
        # ---- accept -----------------------------------------------------
        x_old = v[:nx].copy()
        gf_old = gf[:nx].copy()
        v = vt
        y = y + alpha * dy
        # grad_x L(x, y+) with the Jacobian at x, before J moves to x+ (the
        # device keeps one Jacobian)
        gL_old = gf_old + Jx.rmv(y)
        zl = zl + a_z * dzl
        zu = zu + a_z * dzu
        # kappa_Sigma safeguard of the bound multipliers
        with np.errstate(divide="ignore", invalid="ignore"):
            dl = np.where(hl, v - lo, 1.0)
            du = np.where(hu, hi - v, 1.0)
            zl = np.where(hl, np.clip(zl, mu / (opt.kappa_sigma * dl), opt.kappa_sigma * mu / dl), 0.0)
            zu = np.where(hu, np.clip(zu, mu / (opt.kappa_sigma * du), opt.kappa_sigma * mu / du), 0.0)
        f, graw, c = ft, gt, ct
        gf = P.grad_f(v)
        Jx = la.jac(v)
        # BFGS pair: s = dx, y = grad_x L(x+, y+) - grad_x L(x, y+)
        s_k = v[:nx] - x_old
        y_k = (gf[:nx] + Jx.rmv(y)) - gL_old
        lb.update(s_k, y_k)
        it += 1

    x_full = P._x(v)
    viol = P.unscaled_violation(v, graw)
    # multipliers of the original NLP (unscaled, Ipopt's lambda = y * row scale / obj scale)
    lam = np.zeros(P.m_full)
    if m:
        lam[P.rows] = y * P.row_scale / P.obj_scale
    z_l = np.zeros(P.n_full)
    z_u = np.zeros(P.n_full)
    z_l[P.free] = zl[:nx] / P.obj_scale
    z_u[P.free] = zu[:nx] / P.obj_scale
    dur = time.perf_counter() - t_start
    return IpmResult(x_full, success, status, f / P.obj_scale, it, dur, viol, dict(P.counts),
                     lam, z_l, z_u, history,
                     {"evaluations_s": P.eval_time, "linear_algebra_s": t_lin,
                      "delta_c": delta_c_last, "linear_solver": la.name})


def _restore(P, la, v, c, Jx, lo, hi, hl, hu, Sig, tau, filt, theta, phi, barrier, opt, m, nx, iters=30):
    """Feasibility restoration: Gauss-Newton steps on the constraint
    violation (minimum-norm in the barrier metric), each kept inside the
    bounds by the fraction-to-the-boundary rule and backtracked until
    ||C||_1 decreases, until the point is acceptable to the filter augmented
    with the current iterate.  Returns (v, f, g_raw, C) or None."""
    filt2 = filt + [((1 - opt.gamma_theta) * theta, phi - opt.gamma_phi * theta)]
    vr, cr, Jr = v.copy(), c.copy(), Jx
    th = float(np.abs(cr).sum())
    for _ in range(iters):
        zeta = max(1e-8, math.sqrt(th / max(1.0, m)))
        Dx = Sig[:nx] + zeta
        Ds = Sig[nx:] + zeta
        try:
            kk = la.kkt(Jr, P.ineq, Dx, Ds, 1e-10, None, m)
            dx, ds, _ = kk.solve(np.zeros(nx), np.zeros(len(Ds)), -cr)
        except (RuntimeError, np.linalg.LinAlgError):
            return None
        d = np.concatenate([dx, ds])
        a = _ftb(vr, d, lo, hi, tau)
        ok = False
        while a > 1e-10:
            vt = vr + a * d
            gt = P.g_raw(vt)
            ct = P.C(vt, gt)
            tht = float(np.abs(ct).sum())
            if tht < (1 - 1e-4 * a) * th:
                ok = True
                break
            a *= 0.5
        if not ok:
            return None
        vr, cr, th = vt, ct, tht
        fr = P.f(vr)
        ph = barrier(vr, fr)
        if all(th <= tj or ph <= pj for (tj, pj) in filt2) and th <= (1 - opt.gamma_theta) * theta:
            return vr, fr, gt, cr
        Jr = la.jac(vr)
    return None


def kkt_residuals(nlp, x: np.ndarray, options: Optional[IpmOptions] = None,
                  x_scaling: Optional[np.ndarray] = None) -> dict:
    """Ipopt's termination quantities at a given iterate x, with least-squares
    constraint multipliers (no active variable bounds assumed beyond the
    fixed ones): the unscaled constraint violation, the unscaled dual
    infeasibility ||grad f + J^T lambda||_inf over the free variables, and
    the scaled optimality error E0 = max(dual / s_d, primal) that Ipopt's
    ``tol`` tests, under the gradient-based scaling computed at
    ``x_scaling`` (Ipopt's starting point; default x).  Used to check a
    reference solution file against this NLP's own termination test."""
    from scipy.sparse.linalg import lsqr
    opt = options or IpmOptions()
    P = _Scaled(nlp, x if x_scaling is None else x_scaling, opt)
    x = np.asarray(x, float)
    g = np.asarray(nlp.eval_g(x), float)[P.rows]
    gf = np.asarray(nlp.eval_grad_f(x), float)
    vals = np.asarray(nlp.eval_jac_g(x), float)[:nlp.nnz][P.keep]
    J = P.Jx(vals)                                   # row-scaled, free columns
    b = -P.obj_scale * gf[P.free]
    y = lsqr(J.T.tocsr(), b, atol=1e-14, btol=1e-14, iter_lim=50000)[0]
    r = J.T @ y - b
    viol = float(np.max(np.concatenate([[0.0], P.gl - g, g - P.gu]))) if P.m else 0.0
    primal = float(np.abs(np.where(P.gl == P.gu, P.row_scale * (g - P.gl),
                                   P.row_scale * np.maximum(0.0, np.maximum(P.gl - g, g - P.gu))))
                   .max(initial=0.0))
    sd = max(opt.s_max, float(np.abs(y).sum()) / max(1, P.m)) / opt.s_max
    dual = float(np.abs(r).max(initial=0.0))
    return {"objective": float(nlp.eval_f(x)), "constraint_violation": viol,
            "dual_infeasibility": dual / P.obj_scale, "scaled_primal": primal, "s_d": sd,
            "E0": max(dual / sd, primal), "lambda_max": float(np.abs(y).max(initial=0.0))}
