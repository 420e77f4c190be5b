"""Model-specialized DAE code generator (the "model compiler" back end).

Given a compiled model tape (the same mh_model arrays the C ABI receives),
emit straight-line HIP C++ for the explicit per-point DAE
(MocoCasOCProblem::calcMultibodySystemExplicit semantics, same algorithm as
csrc/dae_device.hpp) with every structural constant folded at generation
time (joint axes and frame orientations, path-point layout,
conditional/moving point logic, actuator wiring) and every model parameter
read from a per-model constant pool.  Zero terms of the 3-D
spatial algebra vanish (planar models lose most of them), all per-lane
state is scalar temporaries (VGPRs instead of scratch), and the mass matrix
is factored with Featherstone's fill-free L^T L scheme on the coordinate
tree.

The generated struct is compiled into libmocohip.so together with two host
functions: <Name>_match(m), the model structure the code assumes (which
mh_create checks to select it), and <Name>_fill(m, K), the model's constant
pool -- every non-structural number the code reads (see "Structure-only
specialization" below).  Models of no generated structure run the generic
device interpreter.
"""
from __future__ import annotations

import math
import re
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi

# generated task decompositions of at most this many groups load each
# group's inputs at the top of the group (see generate(): gait 42-45 groups
# yes, Rajagopal 80's 170 no)
HOIST_MAX_GROUPS = 64


def lit(v: float) -> str:
    """Exact C++ literal of a double (Python repr round-trips exactly)."""
    v = float(v)
    if math.isinf(v):
        return "(-INFINITY)" if v < 0 else "INFINITY"
    if math.isnan(v):
        return "NAN"
    r = repr(v)
    return r if ("e" in r or "." in r) else r + ".0"


class S:
    """A scalar: a folded constant (c), a named temporary (n) or a model
    parameter (p: an entry of the model's constant pool K, loaded at run
    time; v its value for the model the code was generated from)."""
    __slots__ = ("c", "n", "p", "v")

    def __init__(self, c=None, n=None, p=None, v=None):
        self.c = c
        self.n = n
        self.p = p
        self.v = v

    def is_c(self, v=None):
        return self.c is not None and (v is None or self.c == v)

    def is_k(self):
        """Known before run time: a literal or a pool entry."""
        return self.c is not None or self.p is not None

    def host(self) -> str:
        """Its expression in the host pool filler."""
        return lit(self.c) if self.c is not None else f"K[{self.p}]"

    def value(self) -> float:
        return self.c if self.c is not None else self.v

    def __str__(self):
        if self.c is not None:
            return lit(self.c)
        return f"K[{self.p}]" if self.p is not None else self.n


# ---------------------------------------------------------------------------
# Structure-only specialization.  A generated back end is compiled for a model
# STRUCTURE: topology, joint axes and frame orientations, function kinds and
# knot abscissae, path-point kinds and bodies, wrap and constraint wiring, and
# which parameters are exactly zero.  Every other number (masses, inertias,
# frame offsets, path-point locations, muscle properties, time constants,
# actuator strengths, scale factors ...) is a model PARAMETER: the code reads
# it, or a constant folded from parameters, from the model's constant pool K
# (DevModel::pool), which the generated host function fill() computes from
# the mh_model at mh_create.  The generated host function match() checks the
# structure the code assumes, so any model of that structure (a scaled
# subject, a heavier femur, another trial's data) runs the specialized
# kernels.
# ---------------------------------------------------------------------------
class PF(float):
    """A parametric model value: a float that knows its mh_model path."""
    __slots__ = ("path",)

    def __new__(cls, v, path):
        o = float.__new__(cls, v)
        o.path = path
        return o


class _Ctx:
    """Per-generation record: the pool (host expression, value) entries and
    the structural conditions of match()."""

    def __init__(self):
        self.pool: List[Tuple[str, float]] = []
        self.index: Dict[str, int] = {}
        self.checks: Dict[str, None] = {}

    def entry(self, expr: str, value: float) -> "S":
        i = self.index.get(expr)
        if i is None:
            i = len(self.pool)
            self.pool.append((expr, float(value)))
            self.index[expr] = i
        return S(p=i, v=self.pool[i][1])

    def check(self, cond: str):
        self.checks[cond] = None


_CTX: Optional[_Ctx] = None

# mh_* double fields that are model parameters (the rest are structure)
_PARAM_FIELDS = {
    "mh_body": {"mass", "com", "inertia", "p_PF", "p_BM"},
    "mh_function": {"a", "b", "scale"},
    "mh_path_point": {"loc", "range"},
    "mh_muscle": {"max_isometric_force", "optimal_fiber_length", "tendon_slack_length",
                  "pennation_angle_at_optimal", "max_contraction_velocity",
                  "activation_time_constant", "deactivation_time_constant", "fiber_damping",
                  "passive_fiber_strain_at_one_norm_force", "tendon_strain_at_one_norm_force",
                  "active_force_width_scale"},
    "mh_actuator": {"optimal_force"},
    "mh_constraint": {"scale"},
    "mh_wrap_object": {"p_BW", "radius", "length"},
}
# fields read at run time from the device tables (data, not structure)
_RUNTIME_FIELDS = {"mh_table": {"nseg", "break_begin", "coef_begin"}}


def _cond_lit(v) -> str:
    return str(int(v)) if isinstance(v, int) else lit(v)


class _Rec:
    """Recording view of one tape struct (path: its C++ expression on the
    mh_model m): structural reads add a match() condition, parametric reads
    return PF values."""
    __slots__ = ("_s", "_path")

    def __init__(self, s, path):
        object.__setattr__(self, "_s", s)
        object.__setattr__(self, "_path", path)

    def __getattr__(self, name):
        s, path = self._s, self._path
        v = getattr(s, name)
        tname = type(s).__name__
        fpath = f"{path}.{name}"
        if name in _RUNTIME_FIELDS.get(tname, ()):
            return v
        if name in _PARAM_FIELDS.get(tname, ()):
            if hasattr(v, "__len__"):
                return [PF(float(v[i]), f"{fpath}[{i}]") for i in range(len(v))]
            return PF(float(v), fpath)
        if hasattr(v, "__len__"):
            vals = [float(v[i]) for i in range(len(v))]
            for i, x in enumerate(vals):
                _CTX.check(f"{fpath}[{i}] == {lit(x)}")
            return vals
        _CTX.check(f"{fpath} == {_cond_lit(v)}")
        return v


class _RecArr:
    """Recording view of a double array of the tape (knot abscissae)."""

    def __init__(self, arr, path):
        self.arr, self.path = arr, path

    def __getitem__(self, i):
        v = float(self.arr[i])
        _CTX.check(f"{self.path}[{i}] == {lit(v)}")
        return v


class Gen:
    def __init__(self):
        self.lines: List[str] = []
        self.k = 0
        self.flops = {"add": 0, "mul": 0, "div": 0, "fn": 0}

    # -- emission -----------------------------------------------------------
    def tmp(self, expr: str, kind: Optional[str] = None) -> S:
        self.k += 1
        name = f"t{self.k}"
        self.lines.append(f"    const double {name} = {expr};")
        if kind:
            self.flops[kind] += 1
        return S(n=name)

    def var(self, init: S) -> str:
        """A mutable double (for accumulators updated in loops)."""
        self.k += 1
        name = f"v{self.k}"
        self.lines.append(f"    double {name} = {init};")
        return name

    def raw(self, line: str):
        self.lines.append("    " + line)

    @staticmethod
    def const(v: float) -> S:
        return S(c=float(v))

    # -- arithmetic with folding -----------------------------------------------
    # Literal (c) operands fold in Python; parameter (p) operands fold into a
    # new pool entry (the host filler computes it once per model); the
    # identities 0 / 1 / -1 apply to literals only.
    @staticmethod
    def _kfold(a: S, b: S, op: str, value: float) -> S:
        return _CTX.entry(f"({a.host()} {op} {b.host()})", value)

    def add(self, a: S, b: S) -> S:
        if a.is_c() and b.is_c():
            return S(c=a.c + b.c)
        if a.is_c(0.0):
            return b
        if b.is_c(0.0):
            return a
        if a.is_k() and b.is_k():
            return self._kfold(a, b, "+", a.value() + b.value())
        return self.tmp(f"{a} + {b}", "add")

    def sub(self, a: S, b: S) -> S:
        if a.is_c() and b.is_c():
            return S(c=a.c - b.c)
        if b.is_c(0.0):
            return a
        if a.is_c(0.0):
            return self.neg(b)
        if a.is_k() and b.is_k():
            return self._kfold(a, b, "-", a.value() - b.value())
        return self.tmp(f"{a} - {b}", "add")

    def neg(self, a: S) -> S:
        if a.is_c():
            return S(c=-a.c)
        if a.p is not None:
            return _CTX.entry(f"(-{a.host()})", -a.v)
        return self.tmp(f"-{a}")

    def mul(self, a: S, b: S) -> S:
        if a.is_c() and b.is_c():
            return S(c=a.c * b.c)
        if a.is_c(0.0) or b.is_c(0.0):
            return S(c=0.0)
        if a.is_c(1.0):
            return b
        if b.is_c(1.0):
            return a
        if a.is_c(-1.0):
            return self.neg(b)
        if b.is_c(-1.0):
            return self.neg(a)
        if a.is_k() and b.is_k():
            return self._kfold(a, b, "*", a.value() * b.value())
        return self.tmp(f"{a} * {b}", "mul")

    def div(self, a: S, b: S) -> S:
        if a.is_c() and b.is_c():
            return S(c=a.c / b.c)
        if a.is_c(0.0):
            return S(c=0.0)
        if b.is_c(1.0):
            return a
        if a.is_k() and b.is_k():
            return self._kfold(a, b, "/", a.value() / b.value())
        return self.tmp(f"{a} / {b}", "div")

    def fn(self, name: str, a: S) -> S:
        if a.is_c():
            return S(c=getattr(math, name)(a.c))
        if a.p is not None:
            return _CTX.entry(f"std::{name}({a.host()})", getattr(math, name)(a.v))
        return self.tmp(f"{name}({a})", "fn")

    def sel(self, cond: str, a: S, b: S) -> S:
        return self.tmp(f"({cond}) ? {a} : {b}")

    def dot(self, a: Sequence[S], b: Sequence[S]) -> S:
        acc = S(c=0.0)
        for x, y in zip(a, b):
            acc = self.add(acc, self.mul(x, y))
        return acc

    # -- 3-vectors / 3x3 (row-major lists) ---------------------------------------
    def mm(self, A, B):
        return [self.dot([A[3 * i], A[3 * i + 1], A[3 * i + 2]], [B[j], B[3 + j], B[6 + j]])
                for i in range(3) for j in range(3)]

    def mmt(self, A, B):  # A B^T
        return [self.dot([A[3 * i], A[3 * i + 1], A[3 * i + 2]],
                         [B[3 * j], B[3 * j + 1], B[3 * j + 2]]) for i in range(3) for j in range(3)]

    def mv(self, A, x):
        return [self.dot([A[3 * i], A[3 * i + 1], A[3 * i + 2]], x) for i in range(3)]

    def vadd(self, a, b):
        return [self.add(x, y) for x, y in zip(a, b)]

    def vsub(self, a, b):
        return [self.sub(x, y) for x, y in zip(a, b)]

    def vscale(self, a, s):
        return [self.mul(x, s) for x in a]

    def cross(self, a, b):
        return [self.sub(self.mul(a[1], b[2]), self.mul(a[2], b[1])),
                self.sub(self.mul(a[2], b[0]), self.mul(a[0], b[2])),
                self.sub(self.mul(a[0], b[1]), self.mul(a[1], b[0]))]

    # spatial (w, v) pairs of 3-lists
    def crm(self, a, b):
        w = self.cross(a[0], b[0])
        v = self.vadd(self.cross(a[0], b[1]), self.cross(a[1], b[0]))
        return (w, v)

    def crf(self, a, f):
        w = self.vadd(self.cross(a[0], f[0]), self.cross(a[1], f[1]))
        v = self.cross(a[0], f[1])
        return (w, v)

    def svdot(self, m, f):
        return self.add(self.dot(m[0], f[0]), self.dot(m[1], f[1]))

    def svadd(self, a, b):
        return (self.vadd(a[0], b[0]), self.vadd(a[1], b[1]))

    def svscale(self, a, s):
        return (self.vscale(a[0], s), self.vscale(a[1], s))

    def rbi_mul(self, I, x):
        m, h, II = I
        w = [self.dot([II[0], II[3], II[4]], x[0]),
             self.dot([II[3], II[1], II[5]], x[0]),
             self.dot([II[4], II[5], II[2]], x[0])]
        w = self.vadd(w, self.cross(h, x[1]))
        v = self.vsub(self.vscale(x[1], m), self.cross(h, x[0]))
        return (w, v)

    def materialize(self, a: S) -> S:
        """Force a named temporary (used for accumulators that are read many
        times, to keep the generated expression graph shallow)."""
        return a


def _c(v):
    """A constant of the generated code: a literal, or -- for a model
    parameter (PF) -- its pool entry, unless it is exactly zero (a
    structural zero: folded, and checked by match())."""
    if isinstance(v, PF):
        if float(v) == 0.0:
            _CTX.check(f"{v.path} == 0.0")
            return S(c=0.0)
        return _CTX.entry(v.path, float(v))
    return S(c=float(v))


def _vec(vals):
    return [_c(v) for v in vals]


def _unit(v: PF) -> S:
    """A scale factor: exactly 1.0 is structure (folded, checked), anything
    else a pool entry."""
    if float(v) == 1.0:
        _CTX.check(f"{v.path} == 1.0")
        return S(c=1.0)
    return _c(v)


class ModelView:
    """Recording access to the tape arrays of a CompiledModel (structure
    checked by match(), parameters through the pool)."""

    def __init__(self, cm):
        st = cm.struct
        self.cm = cm
        self.nq = st.nq
        self.nb = st.nbodies
        for f in ("nq", "nbodies", "naxes", "nfunctions", "nmuscles", "npoints", "nactuators",
                  "nexternal", "nconstraints", "nwraps", "npathwraps"):
            _CTX.check(f"m.{f} == {int(getattr(st, f))}")
        self.bodies = [_Rec(cm._bodies[i], f"m.bodies[{i}]") for i in range(st.nbodies)]
        self.axes = [_Rec(cm._axes[i], f"m.axes[{i}]") for i in range(st.naxes)]
        self.funcs = [_Rec(cm._funcs[i], f"m.functions[{i}]") for i in range(st.nfunctions)]
        self.kx = _RecArr(cm._kx, "m.knot_x")
        self.muscles = [_Rec(cm._muscles[i], f"m.muscles[{i}]") for i in range(st.nmuscles)]
        self.points = [_Rec(cm._points[i], f"m.points[{i}]") for i in range(st.npoints)]
        self.acts = [_Rec(cm._acts[i], f"m.actuators[{i}]") for i in range(st.nactuators)]
        self.tables = [_Rec(cm._tables[i], f"m.tables[{i}]") for i in range(st.ntables)]
        self.ext = [_Rec(cm._ext[i], f"m.external[{i}]") for i in range(st.nexternal)]
        self.breaks = [st.table_breaks[i] for i in range(st.nbreaks)]
        self.gravity = [PF(float(st.gravity[i]), f"m.gravity[{i}]") for i in range(3)]
        nkc = int(st.nconstraints)
        self.kcs = [_Rec(st.constraints[i], f"m.constraints[{i}]") for i in range(nkc)]
        self.wraps = [_Rec(st.wraps[i], f"m.wraps[{i}]") for i in range(int(st.nwraps))]
        self.pathwraps = [_Rec(st.pathwraps[i], f"m.pathwraps[{i}]") for i in range(int(st.npathwraps))]


def _uniform_guess(br):
    """1/spacing if floor((t - br[0]) / spacing) is within one segment of the
    right one for every t in range (so a single +-1 correction step finds
    it), else None."""
    n = len(br) - 1
    if n < 2:
        return None
    inv = n / (br[-1] - br[0])
    if not math.isfinite(inv) or inv <= 0:
        return None
    for i in range(n):
        lo = math.floor((br[i] - br[0]) * inv)
        hi = math.floor((np.nextafter(br[i + 1], -np.inf) - br[0]) * inv)
        if lo < i - 1 or hi > i + 1:
            return None
    return inv


class _Layout:
    def __init__(self, M: ModelView, implicit: bool = False, prescribed: bool = False,
                 kc_enforce: bool = True, kc_slacks: bool = False):
        NQ = M.nq
        z = 2 * NQ
        self.act_state, self.ftn_state = [], []
        self.mus_control = [-1] * len(M.muscles)
        self.tau_act = self.tau_deact = None
        # prescribed kinematics: q, u, udot from the PositionMotion table
        # (implicit mode only); the NLP states are the auxiliary states
        self.prescribed = prescribed
        implicit = implicit or prescribed
        self.NACC = NQ if implicit and not prescribed else 0
        self.ider = [-1] * len(M.muscles)   # implicit tendon: derivative input after the controls
        nar = 0
        for im, mu in enumerate(M.muscles):
            if mu.tendon_dynamics_implicit and not mu.ignore_tendon_compliance:
                self.ider[im] = self.NACC + nar
                nar += 1
            self.act_state.append(-1 if mu.ignore_activation_dynamics else z)
            z += 0 if mu.ignore_activation_dynamics else 1
            self.ftn_state.append(-1 if mu.ignore_tendon_compliance else z)
            z += 0 if mu.ignore_tendon_compliance else 1
            if not mu.ignore_activation_dynamics and self.tau_act is None:
                self.tau_act = mu.activation_time_constant
                self.tau_deact = mu.deactivation_time_constant
        self.NQ, self.NC = NQ, len(M.acts)
        self.NZ = z - 2 * NQ
        self.NS = self.NZ if prescribed else z          # NLP states
        self.NAR = nar
        self.NO = NQ + self.NZ + nar
        # implicit multibody dynamics: the generalized accelerations are
        # point inputs after the controls, then the implicit auxiliary
        # derivatives; outputs [residual, zdot, auxiliary residuals]
        self.implicit = implicit
        self.NDV = self.NACC + nar
        # kinematic constraints (mh_create's layout, mocohip.hip
        # validate_and_layout): one multiplier per CoordinateCoupler at every
        # grid point (inputs after the derivatives); with prescribed
        # kinematics no kinematic rows and no slacks (CasOCProblem.h:508-521);
        # else the position errors, with enforced derivatives also the
        # velocity and acceleration errors (outputs OKC..), and -- Hermite-
        # Simpson -- one velocity-correction slack per multiplier (inputs after
        # the multipliers; outputs OQC.., the correction G^T gamma per
        # coordinate)
        nkc = len(M.kcs)
        self.NKC = self.NM = nkc
        self.enforce = bool(kc_enforce)
        self.NK = 0 if prescribed else (3 * nkc if kc_enforce else nkc)
        self.NSL = nkc if (nkc and not prescribed and kc_enforce and kc_slacks) else 0
        self.OKC = NQ + self.NZ + nar
        self.OQC = self.OKC + self.NK
        self.NO = self.OQC + (NQ if self.NSL else 0)
        self.IM = self.NS + self.NC + self.NDV
        self.IL = self.IM + self.NM
        self.NI = self.IL + self.NSL
        for ia, a in enumerate(M.acts):
            if a.kind == abi.MH_ACT_MUSCLE:
                self.mus_control[a.target] = ia

    def sin(self, s_full: int) -> int:
        """Point-input index of full-state index s_full ([q, u, z])."""
        return s_full - 2 * self.NQ if self.prescribed else s_full


class _Emitter:
    """Emits one device function body (a fresh Gen) for a model."""

    def __init__(self, M: ModelView, Lo: _Layout):
        self.M, self.Lo = M, Lo
        self.g = Gen()
        self.inp = [S(n=f"in[{i}]") for i in range(Lo.NI)]
        if Lo.prescribed:
            # the motion's q, dq/dt, d2q/dt2 (declared by _presc_prelude)
            self.q = [S(n=f"pq{j}") for j in range(Lo.NQ)]
            self.u = [S(n=f"pu{j}") for j in range(Lo.NQ)]
            self.wacc = [S(n=f"pw{j}") for j in range(Lo.NQ)]
        else:
            self.q = self.inp[:Lo.NQ]
            self.u = self.inp[Lo.NQ:2 * Lo.NQ]
            self.wacc = self.inp[Lo.NS + Lo.NC:Lo.NS + Lo.NC + Lo.NACC] if Lo.implicit else None
        self.ctrl = self.inp[Lo.NS:Lo.NS + Lo.NC]
        self.lam = self.inp[Lo.IM:Lo.IM + Lo.NM]
        self.gam = self.inp[Lo.IL:Lo.IL + Lo.NSL]
        self.fcache: Dict[int, Tuple[S, S, S]] = {}
        self.touched = set()

    # functions of one coordinate
    def fn_eval(self, fi: int):
        g, M = self.g, self.M
        if fi in self.fcache:
            return self.fcache[fi]
        F = M.funcs[fi]
        if F.kind == abi.MH_FN_CONSTANT:
            r = (_c(F.a), _c(0.0), _c(0.0))
        elif F.kind == abi.MH_FN_LINEAR:
            sc, a = _unit(F.scale), _unit(F.a)
            r = (g.mul(sc, g.add(g.mul(a, self.q[F.coord]), _c(F.b))),
                 g.mul(sc, a), _c(0.0))
        else:
            g.k += 1
            base = f"f{g.k}"
            g.raw(f"double {base}v, {base}d1, {base}d2;")
            # interval from the literal knots (no load on the dependency
            # chain), then one round trip for the coefficients
            N = F.knot_count
            xk = [float(M.kx[F.knot_begin + i]) for i in range(N)]
            qv = self.q[F.coord]
            if N > 1:
                cnt = " + ".join(f"({qv} >= {lit(xk[i])})" for i in range(1, N - 1)) or "0"
                g.raw(f"int {base}k = {cnt};")
                g.raw(f"if (fabs({qv} - {lit(xk[0])}) <= 2e-13) {base}k = 0; "
                      f"else if (fabs({qv} - {lit(xk[N - 1])}) <= 2e-13) {base}k = {N - 1};")
                g.raw(f"mh::simm_eval_k<{N}>(M, {F.knot_begin}, {qv}, {base}k, {lit(xk[0])}, "
                      f"{lit(xk[N - 1])}, {base}v, {base}d1, {base}d2);")
            else:
                g.raw(f"mh::simm_eval_n<1>(M, {F.knot_begin}, {qv}, {base}v, {base}d1, {base}d2);")
            g.flops["add"] += 6
            g.flops["mul"] += 8
            v, d1, d2 = S(n=f"{base}v"), S(n=f"{base}d1"), S(n=f"{base}d2")
            sc = _unit(F.scale)
            if not sc.is_c(1.0):
                v, d1, d2 = g.mul(sc, v), g.mul(sc, d1), g.mul(sc, d2)
            r = (v, d1, d2)
        self.fcache[fi] = r
        return r

    def closure(self, bodies):
        """Bodies plus all their ancestors, in model (topological) order."""
        need = set()
        for b in bodies:
            while b >= 0 and b not in need:
                need.add(b)
                b = self.M.bodies[b].parent
        return sorted(need)

    def kinematics(self, bodies: Sequence[int], accel: bool, vel: bool = True):
        """Poses, spatial velocities (if vel), bias accelerations (if accel)
        and motion subspaces for the given bodies (must be ancestor-closed)."""
        accel = accel and vel
        g, M, q, u = self.g, self.M, self.q, self.u
        I3 = _vec([1, 0, 0, 0, 1, 0, 0, 0, 1])
        Z3 = _vec([0, 0, 0])
        R, P, V, A = {-1: I3}, {-1: Z3}, {-1: (Z3, Z3)}, {}
        if accel:
            A[-1] = (Z3, [g.neg(x) for x in _vec(M.gravity)])
        Sj = {}
        coord_body = {}
        for b in bodies:
            B = M.bodies[b]
            p = B.parent
            RGF = g.mm(R[p], _vec(B.R_PF))
            pGF = g.vadd(P[p], g.mv(R[p], _vec(B.p_PF)))
            Vb, Vpar = V[p], V[p]
            Ab = A[p] if accel else None
            axes = M.axes[B.axis_begin:B.axis_begin + B.axis_count]
            fvals = [self.fn_eval(ax.func) for ax in axes]
            pFM = Z3
            for ax, fv in zip(axes, fvals):
                if ax.type == abi.MH_AXIS_TRANSLATION:
                    pFM = g.vadd(pFM, g.vscale(_vec(ax.dir), fv[0]))
            oM = g.vadd(pGF, g.mv(RGF, pFM))

            def motion(s, Vframe, fv, j):
                nonlocal Vb, Ab
                coord_body[j] = b
                if not vel:
                    Sj[j] = g.svadd(Sj.get(j, (Z3, Z3)), g.svscale(s, fv[1]))
                    return
                thd = g.mul(fv[1], u[j])
                Vb = g.svadd(Vb, g.svscale(s, thd))
                if accel:
                    sd = g.crm(Vframe, s)
                    thdd = g.mul(fv[2], g.mul(u[j], u[j]))
                    if self.wacc is not None:   # implicit: RNEA with udot = w
                        thdd = g.add(thdd, g.mul(fv[1], self.wacc[j]))
                    Ab = g.svadd(Ab, g.svadd(g.svscale(sd, thd), g.svscale(s, thdd)))
                Sj[j] = g.svadd(Sj.get(j, (Z3, Z3)), g.svscale(s, fv[1]))
            for ax, fv in zip(axes, fvals):
                F = M.funcs[ax.func]
                if ax.type != abi.MH_AXIS_TRANSLATION or F.kind == abi.MH_FN_CONSTANT:
                    continue
                motion((Z3, g.mv(RGF, _vec(ax.dir))), Vpar, fv, F.coord)
            Rcur = I3
            for ax, fv in zip(axes, fvals):
                if ax.type != abi.MH_AXIS_ROTATION:
                    continue
                F = M.funcs[ax.func]
                if F.kind != abi.MH_FN_CONSTANT:
                    w = g.mv(g.mm(RGF, Rcur), _vec(ax.dir))
                    motion((w, g.cross(oM, w)), Vb, fv, F.coord)
                a0, a1, a2 = ax.dir
                if fv[0].is_k():
                    cs, sn = g.fn("cos", fv[0]), g.fn("sin", fv[0])
                else:
                    g.k += 1
                    nm = f"sc{g.k}"
                    g.raw(f"double {nm}s, {nm}c; sincos({fv[0]}, &{nm}s, &{nm}c);")
                    g.flops["fn"] += 2
                    cs, sn = S(n=f"{nm}c"), S(n=f"{nm}s")
                kk = g.sub(_c(1.0), cs)
                Rk = [g.add(cs, g.mul(kk, _c(a0 * a0))), g.sub(g.mul(kk, _c(a0 * a1)), g.mul(sn, _c(a2))),
                      g.add(g.mul(kk, _c(a0 * a2)), g.mul(sn, _c(a1))),
                      g.add(g.mul(kk, _c(a1 * a0)), g.mul(sn, _c(a2))), g.add(cs, g.mul(kk, _c(a1 * a1))),
                      g.sub(g.mul(kk, _c(a1 * a2)), g.mul(sn, _c(a0))),
                      g.sub(g.mul(kk, _c(a2 * a0)), g.mul(sn, _c(a1))),
                      g.add(g.mul(kk, _c(a2 * a1)), g.mul(sn, _c(a0))), g.add(cs, g.mul(kk, _c(a2 * a2)))]
                Rcur = g.mm(Rcur, Rk)
            RGM = g.mm(RGF, Rcur)
            RB = g.mmt(RGM, _vec(B.R_BM))
            R[b], P[b], V[b] = RB, g.vsub(oM, g.mv(RB, _vec(B.p_BM))), Vb
            if accel:
                A[b] = Ab
        return R, P, V, A, Sj, coord_body

    def inertia(self, b, R, P):
        g, B = self.g, self.M.bodies[b]
        cw = g.vadd(P[b], g.mv(R[b], _vec(B.com)))
        In = B.inertia
        Ib = _vec([In[0], In[3], In[4], In[3], In[1], In[5], In[4], In[5], In[2]])
        Ig = g.mmt(g.mm(R[b], Ib), R[b])
        m = _c(B.mass)
        c2 = g.dot(cw, cw)
        II = [g.add(Ig[0], g.mul(m, g.sub(c2, g.mul(cw[0], cw[0])))),
              g.add(Ig[4], g.mul(m, g.sub(c2, g.mul(cw[1], cw[1])))),
              g.add(Ig[8], g.mul(m, g.sub(c2, g.mul(cw[2], cw[2])))),
              g.sub(Ig[1], g.mul(m, g.mul(cw[0], cw[1]))),
              g.sub(Ig[2], g.mul(m, g.mul(cw[0], cw[2]))),
              g.sub(Ig[5], g.mul(m, g.mul(cw[1], cw[2])))]
        return (m, g.vscale(cw, m), II)

    def acc(self, name: str, val: S, sign: float = 1.0):
        if val.is_c(0.0):
            return
        self.touched.add(name)
        self.g.raw(f"{name} {'+=' if sign > 0 else '-='} {val};")
        self.g.flops["add"] += 1

    def muscle(self, im, R, P, V, Facc, tau, zdot_sink, with_adot: bool = True, resid_sink=None):
        """Path geometry, DGF and tension point forces of muscle im.  Point
        forces are subtracted into the body accumulators Facc (RNEA sign
        convention), MovingPathPoint terms added into tau; zdot values are
        handed to zdot_sink(state_index, S)."""
        g, M, Lo, u, q = self.g, self.M, self.Lo, self.u, self.q
        Z3 = _vec([0, 0, 0])
        mu = M.muscles[im]
        g.raw(f"// muscle {im}")
        pts = M.points[mu.point_begin:mu.point_begin + mu.point_count]
        pos, vel, act, dl_funcs = [], [], [], []
        for pt in pts:
            loc = _vec(pt.loc)
            dloc = list(Z3)
            mov = []
            if pt.kind == abi.MH_PP_CONDITIONAL:
                qv = q[pt.coord]
                rg = _vec(pt.range)
                act.append(f"({qv} >= {rg[0]} && {qv} <= {rg[1]})")
            else:
                act.append(None)
            if pt.kind == abi.MH_PP_MOVING:
                loc = list(loc)
                for d, fi in enumerate((pt.fx, pt.fy, pt.fz)):
                    if fi < 0:
                        continue
                    fv = self.fn_eval(fi)
                    loc[d] = fv[0]
                    F = M.funcs[fi]
                    if F.kind != abi.MH_FN_CONSTANT:
                        dloc[d] = g.mul(fv[1], u[F.coord])
                        mov.append((d, F.coord, fv[1]))
            b = pt.body
            Pw = g.vadd(P[b], g.mv(R[b], loc))
            Vw = g.vadd(g.vadd(V[b][1], g.cross(V[b][0], Pw)), g.mv(R[b], dloc))
            pos.append(Pw)
            vel.append(Vw)
            dl_funcs.append(mov)
        pws = self.path_wraps(im)
        if pws:
            self.wrapped_muscle(im, mu, pts, pos, vel, act, dl_funcs, pws, R, P, V, Facc, tau, zdot_sink,
                                with_adot, resid_sink)
            return
        segs = []
        for i in range(len(pts)):
            for j in range(i - 1, -1, -1):
                conds = [c for c in (act[j], act[i]) if c]
                conds += [f"!{act[k]}" for k in range(j + 1, i)]
                segs.append((j, i, " && ".join(conds) if conds else None))
                if act[j] is None:
                    break
        L, Sp = _c(0.0), _c(0.0)
        seginfo = []
        for (j, i, cond) in segs:
            d = g.vsub(pos[i], pos[j])
            l = g.fn("sqrt", g.dot(d, d))
            sp = g.div(g.dot(d, g.vsub(vel[i], vel[j])), l)
            ind = g.sel(cond, _c(1.0), _c(0.0)) if cond else None
            L = g.add(L, l if ind is None else g.mul(ind, l))
            Sp = g.add(Sp, sp if ind is None else g.mul(ind, sp))
            seginfo.append((j, i, d, l, ind))
        T = self.muscle_force(im, mu, L, Sp, zdot_sink, with_adot, resid_sink)
        for (j, i, d, l, ind) in seginfo:
            Tl = g.div(T, l) if ind is None else g.mul(ind, g.div(T, l))
            Fv = g.vscale(d, Tl)
            for kk, sgn in ((j, 1.0), (i, -1.0)):
                pt = pts[kk]
                if pt.body < 0:
                    continue
                f = Fv if sgn > 0 else [g.neg(x) for x in Fv]
                nrm = g.cross(pos[kk], f)
                fa = Facc[pt.body]
                for c in range(3):
                    self.acc(fa[c], nrm[c], -1.0)
                    self.acc(fa[3 + c], f[c], -1.0)
                for (dd, coord, d1) in dl_funcs[kk]:
                    Rb = R[pt.body]
                    self.acc(tau[coord], g.mul(g.dot([Rb[dd], Rb[3 + dd], Rb[6 + dd]], f), d1))

    def muscle_force(self, im, mu, L: S, Sp: S, zdot_sink, with_adot, resid_sink) -> S:
        """DeGroote-Fregly tension of muscle im at path length L and
        lengthening speed Sp; the activation / tendon-force derivatives and
        the implicit-tendon residual go to their sinks."""
        g, Lo = self.g, self.Lo
        exc = self.ctrl[Lo.mus_control[im]]
        sa, sf = Lo.act_state[im], Lo.ftn_state[im]
        a_ = self.inp[Lo.sin(sa)] if sa >= 0 else exc
        ftn = self.inp[Lo.sin(sf)] if sf >= 0 else None
        idv = Lo.ider[im]
        dft = self.inp[Lo.NS + Lo.NC + idv] if idv >= 0 else None
        T, adot, ftdot, resid = _dgf(g, mu, L, Sp, a_, exc, sa >= 0 and with_adot, ftn, sf >= 0,
                                     Lo.tau_act, Lo.tau_deact, dft)
        if sa >= 0 and with_adot:
            zdot_sink(sa, adot)
        if sf >= 0:
            zdot_sink(sf, ftdot)
        if resid is not None and resid_sink is not None:
            resid_sink(idv - Lo.NACC, resid)
        return T

    def path_wraps(self, im):
        """Muscle im's PathWrap entries [(entry, wrap object, wrap body)]:
        structure (their count, objects and bodies are match() conditions;
        the cylinders' geometry and the ranges are read at run time)."""
        out = []
        for k, pw in enumerate(self.M.pathwraps):
            if pw.muscle != im:
                continue
            w = pw.wrap
            out.append((k, w, self.M.wraps[w].body))
        return out

    def muscle_bodies(self, im):
        """Bodies whose pose muscle im's path reads: its path points' and
        its wrap surfaces' (ground excluded)."""
        mu = self.M.muscles[im]
        bs = {self.M.points[i].body for i in range(mu.point_begin, mu.point_begin + mu.point_count)}
        bs |= {wb for (_, _, wb) in self.path_wraps(im)}
        return sorted(b for b in bs if b >= 0)

    def wrapped_muscle(self, im, mu, pts, pos, vel, act, dl_funcs, pws, R, P, V, Facc, tau, zdot_sink,
                       with_adot, resid_sink):
        """A muscle whose path wraps over cylinders (GeometryPath::
        applyWrapObjects): the path is data-dependent (tangent points come
        and go with the pose), so it is built at run time -- the active path
        points from the generated positions and velocities, then the
        interpreter's own wrapping (dae_device.hpp dev_apply_wraps), path
        length and speed (mh::gen_wrap_path) -- and the tension's point
        forces come back per original path point and per wrap surface
        (mh::gen_wrap_forces), to be applied to the bodies known here."""
        g = self.g
        npt, nw = len(pts), len(pws)
        MP = npt + 2 * nw
        g.k += 1
        k = g.k
        C = f"cp{k}"
        g.raw(f"mh::CPath<{MP}> {C}; {C}.n = 0;")
        for kk, pt in enumerate(pts):
            st = " ".join(f"{C}.P[{C}.n][{d}] = {pos[kk][d]}; {C}.V[{C}.n][{d}] = {vel[kk][d]};"
                          for d in range(3))
            st += (f" {C}.pt[{C}.n] = {mu.point_begin + kk}; {C}.pwi[{C}.n] = -1; "
                   f"{C}.body[{C}.n] = {pt.body}; {C}.wlen[{C}.n] = 0.0; ++{C}.n;")
            g.raw(f"if ({act[kk]}) {{ {st} }}" if act[kk] else f"{{ {st} }}")
        wbs = sorted({wb for (_, _, wb) in pws})
        poses = ", ".join("{{" + ", ".join(str(x) for x in R[b]) + "}, {" + ", ".join(str(x) for x in P[b]) + "}}"
                          for b in wbs)
        vels = ", ".join("{" + ", ".join(str(x) for x in list(V[b][0]) + list(V[b][1])) + "}" for b in wbs)
        nb = len(wbs)
        g.raw(f"const mh::Pose xp{k}[{nb}] = {{{poses}}};")
        g.raw(f"const mh::SV xv{k}[{nb}] = {{{vels}}};")
        g.raw(f"const int xb{k}[{nb}] = {{{', '.join(str(b + 1) for b in wbs)}}};")
        g.raw(f"double L{k}, S{k}; mh::gen_wrap_path<{MP}, {nb}>(M, {im}, xp{k}, xv{k}, xb{k}, {C}, L{k}, S{k});")
        g.flops["fn"] += 40 * nw + 12 * npt
        T = self.muscle_force(im, mu, S(n=f"L{k}"), S(n=f"S{k}"), zdot_sink, with_adot, resid_sink)
        g.raw(f"double fp{k}[{npt}][3], np{k}[{npt}][3], fw{k}[{nw}][3], nw{k}[{nw}][3];")
        g.raw(f"mh::gen_wrap_forces<{MP}, {npt}, {nw}>(M, {im}, {C}, {T}, fp{k}, np{k}, fw{k}, nw{k});")
        g.flops["add"] += 12 * (npt + 2 * nw)
        g.flops["mul"] += 12 * (npt + 2 * nw)

        def apply(b, f, n):
            fa = Facc[b]
            for c in range(3):
                self.acc(fa[c], n[c], -1.0)
                self.acc(fa[3 + c], f[c], -1.0)
        for kk, pt in enumerate(pts):
            if pt.body < 0:
                continue
            f = [S(n=f"fp{k}[{kk}][{c}]") for c in range(3)]
            apply(pt.body, f, [S(n=f"np{k}[{kk}][{c}]") for c in range(3)])
            for (dd, coord, d1) in dl_funcs[kk]:
                Rb = R[pt.body]
                self.acc(tau[coord], g.mul(g.dot([Rb[dd], Rb[3 + dd], Rb[6 + dd]], f), d1))
        for s, (_, _, wb) in enumerate(pws):
            if wb >= 0:
                apply(wb, [S(n=f"fw{k}[{s}][{c}]") for c in range(3)],
                      [S(n=f"nw{k}[{s}][{c}]") for c in range(3)])

    def body_force_vars(self, bodies, init):
        out = {}
        for b in bodies:
            vals = init(b) if init else [_c(0.0)] * 6
            out[b] = [self.g.var(x) for x in vals]
            for name, x in zip(out[b], vals):
                if not x.is_c(0.0):
                    self.touched.add(name)
        return out

    def backward(self, bodies, Facc, Sj, coord_body, tau):
        """F_parent += F_child over `bodies` (descending), then
        tau_j -= S_j . F_body(j).  Accumulators never touched are structural
        zeros and are skipped."""
        g, M = self.g, self.M
        bset = set(bodies)
        for b in sorted(bodies, reverse=True):
            p = M.bodies[b].parent
            if p >= 0 and p in bset:
                for c in range(6):
                    if Facc[b][c] in self.touched:
                        g.raw(f"{Facc[p][c]} += {Facc[b][c]};")
                        g.flops["add"] += 1
                        self.touched.add(Facc[p][c])
        for j, b in sorted(coord_body.items()):
            if b not in Facc:
                continue
            fa = [S(n=n) if n in self.touched else _c(0.0) for n in Facc[b]]
            self.acc(tau[j], g.svdot(Sj[j], (fa[:3], fa[3:])), -1.0)

    def mass_matrix_factor(self, Ibody, Sj, coord_body):
        """CRBA composite inertias + Featherstone L^T L on the coordinate
        tree.  Returns (lam, H) with H the factor entries."""
        NQ = self.Lo.NQ
        lam, H = self.crba(Ibody, Sj, {j: coord_body[j] for j in range(NQ)})
        factor_columns(self.g, H, lam, range(NQ))
        return lam, H

    def crba(self, Ibody, Sj, coord_body):
        """Mass-matrix entries H[(i, j)] = S_j . (Ic_body(i) S_i) for every
        coordinate i of `coord_body` and its ancestor coordinates j, with the
        composite inertias Ic built from the bodies of `Ibody` only (the
        mass matrix is linear in the bodies' inertias: a subset gives that
        subset's share).  coord_body must be ancestor-closed."""
        g, M = self.g, self.M
        Ic = dict(Ibody)
        for b in range(M.nb - 1, -1, -1):
            p = M.bodies[b].parent
            if p >= 0 and b in Ic:
                if p in Ic:
                    mp, hp, Ip = Ic[p]
                    mb, hb, Ibb = Ic[b]
                    Ic[p] = (g.add(mp, mb), g.vadd(hp, hb), [g.add(x, y) for x, y in zip(Ip, Ibb)])
                else:
                    Ic[p] = Ic[b]
        lam = coordinate_tree(M, coord_body, self.Lo.NQ)
        H: Dict[Tuple[int, int], S] = {}
        for i in sorted(coord_body):
            Fi = g.rbi_mul(Ic[coord_body[i]], Sj[i])
            j = i
            while j >= 0:
                H[(i, j)] = g.svdot(Sj[j], Fi)
                j = lam[j]
        return lam, H

    def solve(self, lam, H, bvec):
        g, NQ = self.g, self.Lo.NQ
        bvec = list(bvec)
        xs = [None] * NQ
        for i in range(NQ - 1, -1, -1):
            xs[i] = g.mul(bvec[i], H[(i, i)])
            j = lam[i]
            while j >= 0:
                bvec[j] = g.sub(bvec[j], g.mul(H[(i, j)], xs[i]))
                j = lam[j]
        for i in range(NQ):
            j = lam[i]
            xi = xs[i]
            while j >= 0:
                xi = g.sub(xi, g.mul(H[(i, j)], xs[j]))
                j = lam[j]
            xs[i] = g.mul(xi, H[(i, i)])
        return xs

    def external_forces(self, P, Facc, only=None):
        """ExternalForce point forces from their data tables.  The table's
        degree and column count are structure; its segments and breakpoints
        are run-time data (another trial's GRF fits the same code).  Where the
        breakpoints are near-uniform (every t's direct-index guess within one
        segment of the right one, mh_table_uniform_inv > 0 -- a match()
        condition) the segment is found by direct index plus one correction
        step (two dependent loads instead of a binary search), the guess's
        origin and 1 / spacing coming from the pool."""
        g, M = self.g, self.M
        Z3 = _vec([0, 0, 0])
        for ie, e in enumerate(M.ext):
            if only is not None and ie not in only:
                continue
            b = e.body
            ti = e.table
            g.k += 1
            seg = f"seg{g.k}"
            T = M.tables[ti]
            deg, ncol = T.degree, T.ncol
            br = M.breaks[T.break_begin:T.break_begin + T.nseg + 1]
            g.raw(f"const mh_table tb{g.k} = M.tabs[{ti}];")
            tb = f"tb{g.k}"
            if _uniform_guess(br) is not None:
                _CTX.check(f"mh_table_uniform_inv(m, {ti}) > 0.0")
                b0 = _CTX.entry(f"m.table_breaks[m.tables[{ti}].break_begin]", br[0])
                inv = _CTX.entry(f"mh_table_uniform_inv(m, {ti})", _uniform_guess(br))
                g.raw(f"const int {seg} = mh::table_segment_ur(M.brk + {tb}.break_begin, {tb}.nseg, t, "
                      f"{b0}, {inv});")
            else:
                g.raw(f"const int {seg} = mh::table_segment(M, {ti}, t);")

            def col(cidx):
                return g.tmp(f"mh::table_value_c<{deg}, {ncol}>(M.coef + {tb}.coef_begin, "
                             f"M.brk + {tb}.break_begin, {seg}, {cidx}, t)")
            Fv = [col(e.force_col + d) for d in range(3)] if e.force_col >= 0 else Z3
            Pp = [col(e.point_col + d) for d in range(3)] if e.point_col >= 0 else P[b]
            Tq = [col(e.torque_col + d) for d in range(3)] if e.torque_col >= 0 else Z3
            nrm = g.vadd(g.cross(Pp, Fv), Tq)
            for c in range(3):
                self.acc(Facc[b][c], nrm[c], -1.0)
                self.acc(Facc[b][3 + c], Fv[c], -1.0)

    def kc(self, tau, errors: bool):
        """CoordinateCoupler constraints (MocoCasOCProblem.h:643-732; the
        interpreter's dae_eval / kc_outputs, operation for operation): the
        multiplier forces -G^T lambda into tau (tau[indep] -= (scale f')
        lambda, tau[dep] -= -lambda), and with ``errors`` the per-constraint
        position error scale f(q_i) - q_d, and (enforced derivatives) the
        velocity error G u, G = scale f'(q_i), and the velocity-product part
        scale f''(q_i) u_i u_i of the acceleration error.  Returns
        [(i, indep, dep, epos, evel, G, c2)]."""
        g, M, Lo = self.g, self.M, self.Lo
        out = []
        for i, K in enumerate(M.kcs):
            F = M.funcs[K.func]
            ci, d = F.coord, K.dependent
            v, d1, d2 = self.fn_eval(K.func)
            sc = _unit(K.scale)
            gi = g.mul(sc, d1)
            if Lo.NM:
                self.acc(tau[ci], g.mul(gi, self.lam[i]), -1.0)
                self.acc(tau[d], g.neg(self.lam[i]), -1.0)
            if errors and Lo.NK:
                epos = g.sub(g.mul(sc, v), self.q[d])
                evel = c2 = None
                if Lo.enforce:
                    evel = g.sub(g.mul(gi, self.u[ci]), self.u[d])
                    c2 = g.mul(g.mul(g.mul(sc, d2), self.u[ci]), self.u[ci])
                out.append((i, ci, d, epos, evel, gi, c2))
        return out

    def kc_outputs(self, info, udot, gbase=None):
        """The kinematic-constraint callback outputs (the interpreter's
        kc_outputs): position errors at OKC, then velocity and acceleration
        errors ((G udot_i - udot_d) + c2), then the velocity correction
        G^T gamma per coordinate at OQC.  ``info`` as kc() returns it (or
        group-field accessors), udot the accelerations."""
        g, Lo = self.g, self.Lo
        n = Lo.NKC
        lines = []
        for (i, ci, d, epos, evel, gi, c2) in info:
            lines.append((Lo.OKC + i, epos))
            if Lo.enforce:
                lines.append((Lo.OKC + n + i, evel))
                lines.append((Lo.OKC + 2 * n + i, g.add(g.sub(g.mul(gi, udot[ci]), udot[d]), c2)))
        if Lo.NSL:
            corr = [S(c=0.0) for _ in range(Lo.NQ)]
            for (i, ci, d, epos, evel, gi, c2) in info:
                corr[ci] = g.add(corr[ci], g.mul(gi, self.gam[i]))
                corr[d] = g.sub(corr[d], self.gam[i])
            for j in range(Lo.NQ):
                lines.append((Lo.OQC + j, corr[j]))
        for o, v in lines:
            g.raw(f"out[{o}] = {v};")

    def actuators(self, tau):
        for ia, a in enumerate(self.M.acts):
            if a.kind == abi.MH_ACT_COORDINATE:
                self.acc(tau[a.target], self.g.mul(self.ctrl[ia], _c(a.optimal_force)))


def coordinate_tree(M: ModelView, coord_body: Dict[int, int], NQ: int) -> List[int]:
    """lam[j]: the parent coordinate of coordinate j on the coordinate tree
    (the previous coordinate of the same body, else the last coordinate of
    the nearest ancestor body that has one; -1 at the root); -1 for the
    coordinates absent from coord_body."""
    body_coords: Dict[int, List[int]] = {}
    for j in sorted(coord_body):
        body_coords.setdefault(coord_body[j], []).append(j)

    def anc_coord(b):
        p = M.bodies[b].parent
        while p >= 0:
            if p in body_coords:
                return body_coords[p][-1]
            p = M.bodies[p].parent
        return -1
    lam = [-1] * NQ
    for b, cs in body_coords.items():
        for idx, j in enumerate(cs):
            lam[j] = cs[idx - 1] if idx > 0 else anc_coord(b)
    for j in coord_body:
        if lam[j] >= j:
            raise ValueError("coordinates must be ordered parents-first")
    return lam


def factor_columns(g: Gen, H: Dict[Tuple[int, int], S], lam: List[int], cols) -> None:
    """Featherstone's fill-free L^T L factorization of the columns `cols`
    (processed from the last coordinate down), in place on H: column k
    scales its row by 1/L_kk (kept on the diagonal: one division per column
    here, multiplications in the solves) and updates the entries (i, j) of
    k's ancestor coordinates.  Columns of disjoint subtrees touch disjoint
    entries except their common ancestors'."""
    for k in sorted(cols, reverse=True):
        a = g.div(_c(1.0), g.fn("sqrt", H[(k, k)]))
        H[(k, k)] = a
        i = lam[k]
        while i >= 0:
            H[(k, i)] = g.mul(H[(k, i)], a)
            i = lam[i]
        i = lam[k]
        while i >= 0:
            j = i
            while j >= 0:
                H[(i, j)] = g.sub(H[(i, j)], g.mul(H[(k, i)], H[(k, j)]))
                j = lam[j]
            i = lam[i]


def branch_parts(M: ModelView) -> Optional[Tuple[List[int], List[List[int]]]]:
    """The tree split of the heavy multibody groups: (root chain, parts).
    The root chain is the bodies from the ground down to the first body
    with more than one child (gait models: the pelvis); the parts are the
    subtrees below it (legs, torso), the root chain's bodies added to the
    smallest.  None when the tree does not branch (chains: no split)."""
    children: Dict[int, List[int]] = {b: [] for b in range(-1, M.nb)}
    for b in range(M.nb):
        children[M.bodies[b].parent].append(b)
    root, cur = [], -1
    while len(children[cur]) == 1:
        cur = children[cur][0]
        root.append(cur)
    if len(children[cur]) < 2:
        return None

    def subtree(b):
        out = [b]
        for c in children[b]:
            out += subtree(c)
        return out
    parts = [sorted(subtree(c)) for c in children[cur]]
    small = min(range(len(parts)), key=lambda i: (len(parts[i]), i))
    parts[small] = sorted(parts[small] + root)
    return root, parts


def _multibody_front(E: _Emitter, with_muscles: bool):
    """Kinematics, RNEA (bias + external + coordinate actuators [+ muscles]),
    CRBA and the L^T L factor.  Returns (tau vars, lam, H)."""
    g, M, Lo = E.g, E.M, E.Lo
    allb = list(range(M.nb))
    R, P, V, A, Sj, coord_body = E.kinematics(allb, accel=True)
    Ibody = {b: E.inertia(b, R, P) for b in allb}

    def init(b):
        Ia = g.rbi_mul(Ibody[b], A[b])
        hV = g.rbi_mul(Ibody[b], V[b])
        w, v = g.svadd(Ia, g.crf(V[b], hV))
        return list(w) + list(v)
    Facc = E.body_force_vars(allb, init)
    tau = [g.var(_c(0.0)) for _ in range(Lo.NQ)]
    E.actuators(tau)
    E.kcinfo = E.kc(tau, errors=True)
    zd = {}
    E.resid = {}
    if with_muscles:
        for im in range(len(M.muscles)):
            E.muscle(im, R, P, V, Facc, tau, lambda s, v: zd.__setitem__(s, v),
                     resid_sink=lambda k, v: E.resid.__setitem__(k, v))
    E.external_forces(P, Facc)
    E.backward(allb, Facc, Sj, coord_body, tau)
    if Lo.implicit:
        return tau, None, None, zd
    lam, H = E.mass_matrix_factor(Ibody, Sj, [coord_body[j] for j in range(Lo.NQ)])
    return tau, lam, H, zd


_PRESC_RE = re.compile(r"\bp[quw](\d+)\b")


def _presc_prelude(lines):
    """Declarations of the prescribed q_j, u_j, udot_j the lines use: one
    spline evaluation (value, first and second derivative) per coordinate."""
    used = sorted({int(m) for l in lines for m in _PRESC_RE.findall(l)})
    return [f"double pq{j}, pu{j}, pw{j}; mh::table_eval_d(M, M.kin_table, M.kin_col[{j}], t, "
            f"pq{j}, pu{j}, pw{j});" for j in used]


def generate(cm, struct_name: str, implicit: bool = False, prescribed: bool = False,
             kc_enforce: bool = True, kc_slacks: bool = False) -> Tuple[str, Dict]:
    """Return (C++ source of `struct <struct_name>`, info dict).

    The struct has
      eval()     the whole DAE in one lane (k_eval; also the FLOP reference);
      group(g)   one independent piece of the DAE (see _emit_groups) for the
                 task kernel k_groups, which evaluates only the groups a
                 finite-difference direction perturbs;
      combine()  the per-lane reduction of the group results into udot, zdot
                 (k_combine),
    plus the group metadata (fields, inputs read, time dependence, FP64 op
    counts) the host uses to build the task tables."""
    global _CTX
    _CTX = _Ctx()
    M = ModelView(cm)
    Lo = _Layout(M, implicit, prescribed, kc_enforce, kc_slacks)
    implicit = Lo.implicit
    NQ, NZ = Lo.NQ, Lo.NZ
    parts = []
    info = {"NQ": NQ, "NS": Lo.NS, "NC": Lo.NC, "implicit": implicit, "prescribed": prescribed,
            "NM": Lo.NM, "NSL": Lo.NSL, "NK": Lo.NK}

    # ---- single-lane eval ---------------------------------------------------
    E = _Emitter(M, Lo)
    tau, lam, H, zd = _multibody_front(E, with_muscles=True)
    if implicit:
        # residual = M w + C - f_applied = -(tau of the RNEA with udot = w)
        xs = [E.g.neg(S(n=t)) for t in tau]
    else:
        xs = E.solve(lam, H, [S(n=t) for t in tau])
    for i in range(NQ):
        E.g.raw(f"out[{i}] = {xs[i]};")
    for zi in range(NZ):
        E.g.raw(f"out[{NQ + zi}] = {zd.get(2 * NQ + zi, _c(0.0))};")
    for k in range(Lo.NAR):
        E.g.raw(f"out[{NQ + NZ + k}] = {E.resid[k]};")
    if E.kcinfo:
        E.kc_outputs(E.kcinfo, E.wacc if implicit else xs)
    fl = dict(E.g.flops)
    fl["total"] = sum(fl.values())
    info["flops"] = fl
    info["lines"] = len(E.g.lines)
    parts.append(("eval", "const mh::DevModel& M, const double t, const double* __restrict__ in, "
                          "double* __restrict__ out", _presc_prelude(E.g.lines) + E.g.lines))

    # ---- task decomposition ------------------------------------------------
    groups = _emit_groups(M, Lo)
    comb, comb_flops = _emit_combine(M, Lo, groups)
    info["groups"] = [(gr.name, gr.nf, sorted(gr.reads), gr.time, gr.flops) for gr in groups]
    info["combine_flops"] = comb_flops
    NG = len(groups)
    NF = max([gr.nf for gr in groups[1:]] + [1])
    NST = max(groups[0].nf, 1)
    # the leading heavy groups: mass (or its placeholder), its parts and the
    # bias parts (k_groups gives them issue priority; k_groups_part CLS 1)
    NHEAVY = 1 + sum(1 for gr in groups[1:] if gr.name.startswith(("mass", "bias")))
    RW = (Lo.NI + 63) // 64
    reads = []
    for gr in groups:
        words = [0] * RW
        for i in gr.reads:
            words[i // 64] |= 1 << (i % 64)
        reads.append("{" + ", ".join(f"0x{w:x}ULL" for w in words) + "}")
    body = ["        switch (g) {"]
    rin = re.compile(r"\bin\[(\d+)\]")
    # the group's inputs loaded at its top, all at once (one memory round trip
    # before the arithmetic instead of loads spread through it, each waited
    # on where first used): gait's task kernels 7.15 -> 6.76 us (eval_g) and
    # ~9.2 -> 8.5 us (Jacobian), headline 24.6 k -> 25.3 k calls/s
    # (profiles/r05_p).  Not for the large models, whose group kernels run at
    # the register cap (Rajagopal 80: 254 VGPRs; its DAE stage 0.38 -> 0.46 ms
    # with the inputs hoisted).
    hoist = len(groups) <= HOIST_MAX_GROUPS
    for gi, gr in enumerate(groups):
        body.append(f"        case {gi}: {{  // {gr.name}")
        if hoist:
            used = sorted({int(m) for l in gr.lines for m in rin.findall(l)})
            body.extend(f"            const double in_{i} = in[{i}];" for i in used)
            body.extend("    " + rin.sub(lambda m: f"in_{m.group(1)}", l) for l in gr.lines)
        else:
            body.extend("    " + l for l in gr.lines)
        body.append("        } break;")
    body += ["        default: break;", "        }"]
    parts.append(("group", "const int g, const mh::DevModel& M, const double t, "
                           "const double* __restrict__ in, double* __restrict__ out", body))
    parts.append(("combine", "const mh::DevModel& M, const double t, const double* __restrict__ in, "
                             "const TL& T, OUT out", comb))
    # the same combine in two steps (core.hpp interval_body's split combine):
    # its independent sums one at a time, then the rest from the sums
    nsum, sums_body, consts, sum_flops = _emit_combine_sums(M, Lo, groups)
    fin, fin_flops = _emit_combine_finish(M, Lo, groups, consts)
    parts.append(("combine_sum", "const int q, const mh::DevModel& M, const double t, "
                                 "const double* __restrict__ in, const TL& T", sums_body))
    parts.append(("combine_finish", "const mh::DevModel& M, const double t, const double* __restrict__ in, "
                                    "const TL& T, const SUMS& S, OUT out", fin))
    info["nsum"] = nsum
    info["combine_split_flops"] = (sum_flops, fin_flops)

    fns = []
    for name, args, lines in parts:
        tpl = ""
        if name in ("group", "combine", "combine_sum", "combine_finish"):
            # inputs through an accessor (loaded where used, not held in VGPRs)
            # combine: outputs through a writer (OUT: a pointer, or a strided
            # Y / LDS writer -- each output is stored as it is produced
            # instead of living in registers until the end)
            tpl = {"group": "template <class IN> ", "combine": "template <class IN, class TL, class OUT> ",
                   "combine_sum": "template <class IN, class TL> ",
                   "combine_finish": "template <class IN, class TL, class SUMS, class OUT> "}[name]
            args = args.replace("const double* __restrict__ in", "const IN& in")
        # the pool through the constant address space (dae_device.hpp kpool:
        # scalar loads)
        pre = ["    const mh::kconst* __restrict__ K = mh::kpool(M);", "    (void)K;"]
        ret = "double" if name == "combine_sum" else "void"
        fns.append(f"    {tpl}__device__ __forceinline__ static {ret} {name}({args}) {{\n"
                   + "\n".join(pre + lines) + "\n    }")
    lst = lambda v: "{" + ", ".join(str(x) for x in v) + "}"
    src = f"""struct {struct_name} {{
    static constexpr int NQ = {NQ}, NZ = {NZ}, NS = {Lo.NS}, NC = {Lo.NC}, NO = {Lo.NO}, NI = {Lo.NI};
    // kinematic constraints: multipliers, slack inputs per point
    static constexpr int NM = {Lo.NM}, NSL = {Lo.NSL};
    static constexpr bool IMPLICIT = {"true" if implicit else "false"};
    static constexpr bool PRESCRIBED = {"true" if prescribed else "false"};
    static constexpr bool EXC_LANES = false;   // k_exc_lanes is the generic interpreter's
    static constexpr int MI = NI, MO = NO;
    static constexpr double FLOPS_PER_EVAL = {float(fl['total'])};
    // task decomposition: group 0 = mass matrix factor (NST values; a
    // placeholder where the mass matrix is split into parts), groups 1.. =
    // mass-matrix parts and force groups (NF values: factor entries and
    // root-chain shares, nonzero generalized forces, z output)
    static constexpr int NG = {NG}, NST = {NST}, NF = {NF}, RW = {RW}, NHEAVY = {NHEAVY};
    static constexpr int GROUP_NF[NG] = {lst([gr.nf for gr in groups])};
    static constexpr unsigned long long GROUP_READS[NG][RW] = {{{", ".join(reads)}}};
    static constexpr unsigned char GROUP_TIME[NG] = {lst([int(gr.time) for gr in groups])};
    static constexpr double GROUP_FLOPS[NG] = {lst([float(gr.flops) for gr in groups])};
    static constexpr double COMBINE_FLOPS = {float(comb_flops)};
    // the combine's independent sums (combine_sum / combine_finish)
    static constexpr int NSUM = {nsum};
    // the model's constant pool (DevModel::pool, filled by fill())
    static constexpr int NPOOL = {max(1, len(_CTX.pool))};
{chr(10).join(fns)}
}};
"""
    conds = list(_CTX.checks)
    match = [f"// the structure {struct_name} was generated for ({len(conds)} conditions)",
             f"static bool {struct_name}_match(const mh_model& m) {{"]
    match += [f"    if (!({c})) return false;" for c in conds]
    match += ["    return true;", "}"]
    fill = [f"// its constant pool for model m ({len(_CTX.pool)} entries)",
            f"static void {struct_name}_fill(const mh_model& m, double* K) {{",
            "#pragma clang fp contract(off)", "    (void)m;"]
    fill += [f"    K[{i}] = {e};" for i, (e, _) in enumerate(_CTX.pool)]
    fill += ["}"]
    src += "\n".join(match + fill) + "\n"
    info["npool"] = len(_CTX.pool)
    info["nchecks"] = len(conds)
    _CTX = None
    return src, info


class _Group:
    def __init__(self, name, lines, fields, reads, time, flops):
        self.name, self.lines, self.fields = name, lines, fields
        self.nf = len(fields)
        self.reads, self.time, self.flops = reads, time, flops


_IN_RE = re.compile(r"\bin\[(\d+)\]")


def _reads_of(lines):
    reads = set()
    time = False
    for l in lines:
        reads.update(int(m) for m in _IN_RE.findall(l))
        if "mh::table_" in l:
            time = True
    return reads, time


def _emit_groups(M: ModelView, Lo: _Layout) -> List[_Group]:
    """Independent pieces of one DAE evaluation.  Each reads a subset of the
    point inputs (found from the emitted code) so a finite-difference
    direction only re-evaluates the groups that read the perturbed input:
      mass      position kinematics, CRBA mass matrix, L^T L factor (q only)
      bias      RNEA inertial + gravity generalized forces (q, u)
      ext_e     external load e (q along the body chain, time)
      muscle_m  path, DeGroote-Fregly force, tendon point forces -> tau, and
                the normalized tendon force derivative if compliant
      activation_m  DeGroote-Fregly activation dynamics (a_m, e_m)
    Coordinate actuators are evaluated per lane in the combine step."""
    NQ = Lo.NQ
    allb = list(range(M.nb))
    out = []
    split = branch_parts(M)

    # mass (implicit mode: the residual needs no mass matrix -- the group is
    # an empty placeholder so group 0 keeps its role in the task tables; the
    # same where the tree splits: the mass-matrix parts below carry it)
    E = _Emitter(M, Lo)
    if Lo.implicit or split:
        E.g.raw("out[0] = 0.0;")
        g0 = _Group("mass", E.g.lines, [("H", (0, 0))], set(), False, 0)
        g0.lam = None
        out.append(g0)
    else:
        R, P, _, _, Sj, cb = E.kinematics(allb, accel=False, vel=False)
        Ib = {b: E.inertia(b, R, P) for b in allb}
        lam, H = E.mass_matrix_factor(Ib, Sj, [cb[j] for j in range(NQ)])
        keys = sorted(H.keys())
        for f, k in enumerate(keys):
            E.g.raw(f"out[{f}] = {H[k]};")
        r, t = _reads_of(E.g.lines)
        g0 = _Group("mass", E.g.lines, [("H", k) for k in keys], r, t, sum(E.g.flops.values()))
        g0.lam = lam
        out.append(g0)

    def finish(Eg, name, tv, zf=None, rf=None, extra=()):
        fields = []
        for j in range(NQ):
            if tv[j] in Eg.touched:
                Eg.g.raw(f"out[{len(fields)}] = {tv[j]};")
                fields.append(("tau", j))
        for kind, key, val in extra:
            Eg.g.raw(f"out[{len(fields)}] = {val};")
            fields.append((kind, key))
        if zf is not None:
            Eg.g.raw(f"out[{len(fields)}] = {zf[1]};")
            fields.append(("z", zf[0]))
        if rf is not None:     # implicit tendon: the equilibrium residual
            Eg.g.raw(f"out[{len(fields)}] = {rf[1]};")
            fields.append(("r", rf[0]))
        lines = _presc_prelude(Eg.g.lines) + Eg.g.lines
        r, t = _reads_of(lines)
        out.append(_Group(name, lines, fields, r, t, sum(Eg.g.flops.values())))

    # Where the tree branches, the two heavy groups are split by subtree so
    # that no single task carries the whole multibody system (a task is one
    # wave's instruction stream: its length is the stage's critical path),
    # and a perturbed coordinate re-evaluates only its own subtree's part.
    # Mass-matrix part p: the CRBA entries of its bodies' inertias (the mass
    # matrix is linear in them), its own coordinates' columns factored
    # (they touch only its own entries and the root chain's), and its share
    # of the root-chain block after those columns' updates ("HR"); the
    # combine sums the shares and factors the root columns.
    if split and not Lo.implicit:
        root, parts = split
        for ip, bodies in enumerate(parts):
            E = _Emitter(M, Lo)
            cl = E.closure(bodies)
            R, P, _, _, Sj, cb = E.kinematics(cl, accel=False, vel=False)
            Ib = {b: E.inertia(b, R, P) for b in bodies}
            lam, H = E.crba(Ib, Sj, cb)
            own = [j for j in cb if cb[j] not in root]
            factor_columns(E.g, H, lam, own)
            fields = []
            for k in sorted(H):
                kind = "HR" if cb[k[0]] in root else "H"
                E.g.raw(f"out[{len(fields)}] = {H[k]};")
                fields.append((kind, k))
            r, t = _reads_of(E.g.lines)
            out.append(_Group(f"mass_{ip}", E.g.lines, fields, r, t, sum(E.g.flops.values())))

    # bias (RNEA inertial + gravity forces); split: part p applies its own
    # bodies' forces only and runs the backward pass over their closure --
    # the generalized forces are linear in the body forces, and the combine
    # sums the parts' tau like any other force group
    bias_parts = split[1] if split else [allb]
    for ip, bodies in enumerate(bias_parts):
        E = _Emitter(M, Lo)
        cl = E.closure(bodies) if split else allb
        R, P, V, A, Sj, cb = E.kinematics(cl, accel=True)
        Ib = {b: E.inertia(b, R, P) for b in bodies}

        def init(b):
            if b not in Ib:
                return [_c(0.0)] * 6
            Ia = E.g.rbi_mul(Ib[b], A[b])
            hV = E.g.rbi_mul(Ib[b], V[b])
            w, v = E.g.svadd(Ia, E.g.crf(V[b], hV))
            return list(w) + list(v)
        Facc = E.body_force_vars(cl, init)
        tv = [E.g.var(_c(0.0)) for _ in range(NQ)]
        E.backward(cl, Facc, Sj, cb, tv)
        finish(E, f"bias_{ip}" if split else "bias", tv)

    # external loads
    for ie, e in enumerate(M.ext):
        E = _Emitter(M, Lo)
        cl = E.closure([e.body])
        R, P, _, _, Sj, cb = E.kinematics(cl, accel=False, vel=False)
        Facc = E.body_force_vars(cl, None)
        tv = [E.g.var(_c(0.0)) for _ in range(NQ)]
        E.external_forces(P, Facc, only=[ie])
        E.backward(cl, Facc, Sj, cb, tv)
        finish(E, f"ext_{ie}", tv)

    # kinematic constraints: the multiplier forces and the parts of the
    # constraint errors that do not need the accelerations
    if Lo.NKC:
        E = _Emitter(M, Lo)
        tv = [E.g.var(_c(0.0)) for _ in range(NQ)]
        info = E.kc(tv, errors=True)
        extra = []
        for (i, ci, d, epos, evel, gi, c2) in info:
            extra.append(("kpos", i, epos))
            if Lo.enforce:
                extra += [("kvel", i, evel), ("kg", i, gi), ("kc2", i, c2)]
            elif Lo.NSL:
                extra.append(("kg", i, gi))
        finish(E, "constraints", tv, extra=extra)

    # activation dynamics (reads the muscle's activation and excitation only)
    for im in range(len(M.muscles)):
        sa = Lo.act_state[im]
        if sa < 0:
            continue
        E = _Emitter(M, Lo)
        adot = _activation_dot(E.g, E.inp[Lo.sin(sa)], E.ctrl[Lo.mus_control[im]], Lo.tau_act,
                               Lo.tau_deact)
        E.g.raw(f"out[0] = {adot};")
        r, t = _reads_of(E.g.lines)
        out.append(_Group(f"activation_{im}", E.g.lines, [("z", sa - 2 * NQ)], r, t,
                          sum(E.g.flops.values())))

    # muscles
    for im, mu in enumerate(M.muscles):
        E = _Emitter(M, Lo)
        cl = E.closure(E.muscle_bodies(im))
        R, P, V, _, Sj, cb = E.kinematics(cl, accel=False)
        Facc = E.body_force_vars(cl, None)
        tv = [E.g.var(_c(0.0)) for _ in range(NQ)]
        zs, rs = {}, {}
        E.muscle(im, R, P, V, Facc, tv, lambda si, v: zs.__setitem__(si, v), with_adot=False,
                 resid_sink=lambda k, v: rs.__setitem__(k, v))
        E.backward(cl, Facc, Sj, cb, tv)
        zf = None
        if Lo.ftn_state[im] >= 0:
            zf = (Lo.ftn_state[im] - 2 * NQ, zs[Lo.ftn_state[im]])
        rf = next(iter(rs.items()), None)
        finish(E, f"muscle_{im}", tv, zf, rf)
    return out


def _emit_combine(M: ModelView, Lo: _Layout, groups: List[_Group]):
    """Per-lane combine: generalized forces summed over the groups in a fixed
    order (so re-using a group's unperturbed result is bit-identical to
    re-evaluating it), coordinate actuators, the two triangular solves with
    the mass-matrix factor, and the z outputs of the groups."""
    NQ = Lo.NQ
    E = _Emitter(M, Lo)
    g = E.g
    terms = [[] for _ in range(NQ)]
    for gi, gr in enumerate(groups[1:], start=1):
        for f, (kind, j) in enumerate(gr.fields):
            if kind == "tau":
                terms[j].append(S(n=f"T({gi}, {f})"))
    for ia, a in enumerate(M.acts):
        if a.kind == abi.MH_ACT_COORDINATE:
            terms[a.target].append(g.mul(E.ctrl[ia], _c(a.optimal_force)))

    def tree(ts):
        if not ts:
            return _c(0.0)
        while len(ts) > 1:
            ts = [g.add(ts[i], ts[i + 1]) if i + 1 < len(ts) else ts[i] for i in range(0, len(ts), 2)]
        return ts[0]
    bvec = [tree(t) for t in terms]
    if Lo.implicit:
        xs = [g.neg(b) for b in bvec]     # residual = -(applied - bias with udot = w)
    elif groups[0].lam is not None:
        keys = [k for _, k in groups[0].fields]
        Hs = {k: S(n=f"T.h({f})") for f, k in enumerate(keys)}
        xs = E.solve(groups[0].lam, Hs, bvec)
    else:
        # the mass matrix in parts (_emit_groups): the parts' factored
        # columns as they are, the root-chain block summed over the parts
        # (fixed order) and factored here
        Hs, shares = {}, {}
        for gi, gr in enumerate(groups):
            for f, (kind, k) in enumerate(gr.fields):
                if kind == "H" and gi > 0:
                    Hs[k] = S(n=f"T({gi}, {f})")
                elif kind == "HR":
                    shares.setdefault(k, []).append(S(n=f"T({gi}, {f})"))
        for k in sorted(shares):
            Hs[k] = tree(shares[k])
        R0, _, _, _, _, cb = _Emitter(M, Lo).kinematics(list(range(M.nb)), accel=False, vel=False)
        lam = coordinate_tree(M, cb, NQ)
        factor_columns(g, Hs, lam, sorted({k[0] for k in shares}))
        xs = E.solve(lam, Hs, bvec)
    kcf = {}
    copies = []
    for gi, gr in enumerate(groups[1:], start=1):
        for f, (kind, zi) in enumerate(gr.fields):
            if kind == "z":
                copies.append((NQ + zi, gi, f))
            elif kind == "r":
                copies.append((NQ + Lo.NZ + zi, gi, f))
            elif kind in ("kpos", "kvel", "kg", "kc2"):
                kcf[(kind, zi)] = S(n=f"T({gi}, {f})")
    _emit_outputs(g, xs, copies)
    if Lo.NK:
        info = []
        for i, K in enumerate(M.kcs):
            F = M.funcs[K.func]
            info.append((i, F.coord, K.dependent, kcf[("kpos", i)], kcf.get(("kvel", i)),
                         kcf.get(("kg", i)), kcf.get(("kc2", i))))
        udot = [E.inp[Lo.NS + Lo.NC + j] for j in range(NQ)] if Lo.implicit else xs
        E.kc_outputs(info, udot)
    return g.lines, sum(g.flops.values())


OUT_BATCH = 24   # group-result copies loaded together before their stores


def _emit_outputs(g: Gen, xs, copies):
    """The combine's outputs: the NQ solved values, then the outputs that
    copy a group result (z, auxiliary residuals).  A copy is a load of T and
    a store to out; emitted one after the other, every load waited for the
    store before it (one counter covers a wave's loads and stores on CDNA,
    and the compiler cannot move a T load above an out store), one memory
    round trip per output -- for Rajagopal 80's 86 copies the combine's
    longest chain.  So the copies are loaded in batches of OUT_BATCH, the
    first before the solved values are stored, each batch's stores after
    its loads: a round trip per batch.  The same values (copies), bit for
    bit."""
    batches = [copies[i:i + OUT_BATCH] for i in range(0, len(copies), OUT_BATCH)]

    def load(b):
        for o, gi, f in b:
            g.raw(f"const double zo_{o} = T({gi}, {f});")

    def store(b):
        for o, _, _ in b:
            g.raw(f"out[{o}] = zo_{o};")
    if batches:
        load(batches[0])
    for i in range(len(xs)):
        g.raw(f"out[{i}] = {xs[i]};")
    for k, b in enumerate(batches):
        if k:
            load(b)
        store(b)


def _tree(g: Gen, ts):
    """The combine's fixed-order pairwise sum of a term list."""
    if not ts:
        return _c(0.0)
    while len(ts) > 1:
        ts = [g.add(ts[i], ts[i + 1]) if i + 1 < len(ts) else ts[i] for i in range(0, len(ts), 2)]
    return ts[0]


def _sum_terms(M: ModelView, Lo: _Layout, groups: List[_Group]):
    """The combine's independent sums, in _emit_combine's order: sum j < NQ
    is coordinate j's generalized force (the groups' tau fields in group
    order, then the coordinate actuators' control x optimal force), sum NQ +
    i the i-th root-chain mass-matrix entry (sorted keys) summed over the
    mass-matrix parts.  Returns (number of sums, terms(q, g, E) -> the term
    list of sum q built in Gen g, the share keys)."""
    NQ = Lo.NQ
    taus = [[] for _ in range(NQ)]
    for gi, gr in enumerate(groups[1:], start=1):
        for f, (kind, j) in enumerate(gr.fields):
            if kind == "tau":
                taus[j].append((gi, f))
    acts = [[] for _ in range(NQ)]
    for ia, a in enumerate(M.acts):
        if a.kind == abi.MH_ACT_COORDINATE:
            acts[a.target].append((ia, a.optimal_force))
    shares: Dict = {}
    if not Lo.implicit and groups[0].lam is None:
        for gi, gr in enumerate(groups):
            for f, (kind, k) in enumerate(gr.fields):
                if kind == "HR":
                    shares.setdefault(k, []).append((gi, f))
    keys = sorted(shares)

    def terms(q, g, E):
        if q < NQ:
            return ([S(n=f"T({gi}, {f})") for gi, f in taus[q]] +
                    [g.mul(E.ctrl[ia], _c(of)) for ia, of in acts[q]])
        return [S(n=f"T({gi}, {f})") for gi, f in shares[keys[q - NQ]]]
    return NQ + len(keys), terms, keys


def _emit_combine_sums(M: ModelView, Lo: _Layout, groups: List[_Group]):
    """combine_sum(q): sum q of _sum_terms alone (the same tree, so the same
    value bit for bit as inside combine()), so that a lane role's sums can
    be spread over the threads of a workgroup.  Returns (NSUM, switch body,
    per sum its constant value when it has no terms, else None)."""
    nsum, terms_of, _ = _sum_terms(M, Lo, groups)
    body = ["        switch (q) {"]
    consts = []
    flops = 0
    for q in range(nsum):
        E = _Emitter(M, Lo)
        v = _tree(E.g, terms_of(q, E.g, E))
        consts.append(v if v.is_k() else None)
        flops += sum(E.g.flops.values())
        body.append(f"        case {q}: {{")
        body.extend("    " + l for l in E.g.lines)
        body.append(f"            return {v};")
        body.append("        }")
    body += ["        default: return 0.0;", "        }"]
    return nsum, body, consts, flops


def _emit_combine_finish(M: ModelView, Lo: _Layout, groups: List[_Group], consts):
    """combine_finish(): _emit_combine's arithmetic after the sums, which it
    reads through the accessor S (S(q) = combine_sum(q) of the same lane
    role; a sum without terms stays the literal it folds to)."""
    NQ = Lo.NQ
    nsum, _, keys = _sum_terms(M, Lo, groups)
    E = _Emitter(M, Lo)
    g = E.g
    vals = [consts[q] if consts[q] is not None else S(n=f"S({q})") for q in range(nsum)]
    bvec = vals[:NQ]
    if Lo.implicit:
        xs = [g.neg(b) for b in bvec]
    elif groups[0].lam is not None:
        fkeys = [k for _, k in groups[0].fields]
        Hs = {k: S(n=f"T.h({f})") for f, k in enumerate(fkeys)}
        xs = E.solve(groups[0].lam, Hs, bvec)
    else:
        Hs = {}
        for gi, gr in enumerate(groups):
            for f, (kind, k) in enumerate(gr.fields):
                if kind == "H" and gi > 0:
                    Hs[k] = S(n=f"T({gi}, {f})")
        for i, k in enumerate(keys):
            Hs[k] = vals[NQ + i]
        R0, _, _, _, _, cb = _Emitter(M, Lo).kinematics(list(range(M.nb)), accel=False, vel=False)
        lam = coordinate_tree(M, cb, NQ)
        factor_columns(g, Hs, lam, sorted({k[0] for k in keys}))
        xs = E.solve(lam, Hs, bvec)
    kcf = {}
    copies = []
    for gi, gr in enumerate(groups[1:], start=1):
        for f, (kind, zi) in enumerate(gr.fields):
            if kind == "z":
                copies.append((NQ + zi, gi, f))
            elif kind == "r":
                copies.append((NQ + Lo.NZ + zi, gi, f))
            elif kind in ("kpos", "kvel", "kg", "kc2"):
                kcf[(kind, zi)] = S(n=f"T({gi}, {f})")
    _emit_outputs(g, xs, copies)
    if Lo.NK:
        info = []
        for i, K in enumerate(M.kcs):
            F = M.funcs[K.func]
            info.append((i, F.coord, K.dependent, kcf[("kpos", i)], kcf.get(("kvel", i)),
                         kcf.get(("kg", i)), kcf.get(("kc2", i))))
        udot = [E.inp[Lo.NS + Lo.NC + j] for j in range(NQ)] if Lo.implicit else xs
        E.kc_outputs(info, udot)
    return g.lines, sum(g.flops.values())


def _activation_dot(g: Gen, act: S, exc: S, tau_act, tau_deact) -> S:
    """DeGrooteFregly2016Muscle::calcActivationDerivative
    (DeGrooteFregly2016Muscle.cpp:189-209; the time constants are the static
    ones of the first muscle evaluated, :194-195)."""
    C = _c
    tcf = g.add(C(0.5), g.mul(C(1.5), act))
    tempAct = g.div(C(1.0), g.mul(C(tau_act), tcf))
    tempDeact = g.div(tcf, C(tau_deact))
    f = g.mul(C(0.5), g.fn("tanh", g.mul(C(0.1), g.sub(exc, act))))
    tc = g.add(g.mul(tempAct, g.add(f, C(0.5))), g.mul(tempDeact, g.add(g.neg(f), C(0.5))))
    return g.mul(tc, g.sub(exc, act))


def _dgf(g: Gen, mu, LMT: S, VMT: S, act: S, exc: S, has_act: bool, ftn: Optional[S],
         compliant: bool, tau_act, tau_deact, dft: Optional[S] = None):
    """DeGrooteFregly2016Muscle (DeGrooteFregly2016Muscle.cpp:186-425).  dft:
    the normalized tendon force derivative input of implicit tendon dynamics
    (returns the equilibrium residual FT - FM cos(alpha), .cpp:826-848)."""
    c1, c2, c3 = 0.2, 1.0, 0.2
    d1, d2, d3, d4 = -0.3211346127989808, -8.149, -0.374, 0.8825327733249912
    C = _c
    # the muscle's parameters and the constants DeGrooteFregly2016Muscle
    # derives from them (extendFinalizeFromProperties, .cpp:130-147): pool
    # entries computed on the host, as mh_create does for the interpreter
    lopt, lts, Fmax = C(mu.optimal_fiber_length), C(mu.tendon_slack_length), C(mu.max_isometric_force)
    fiberWidth = g.mul(lopt, g.fn("sin", C(mu.pennation_angle_at_optimal)))
    sqW = g.mul(fiberWidth, fiberWidth)
    vmax = g.mul(C(mu.max_contraction_velocity), lopt)
    kT = g.div(C(math.log((1.0 + c3) / c1)), g.sub(g.add(C(1.0), C(mu.tendon_strain_at_one_norm_force)), C(c2)))
    e0 = C(mu.passive_fiber_strain_at_one_norm_force)
    peOffset = g.fn("exp", g.div(C(4.0 * (0.2 - 1.0)), e0))
    peDenom = g.sub(C(math.exp(4.0)), peOffset)
    c1kT = g.mul(C(c1), kT)
    if compliant:
        ntl = g.add(g.div(g.fn("log", g.mul(C(1.0 / c1), g.add(ftn, C(c3)))), kT), C(c2))
    else:
        ntl = C(1.0)
    tendonLength = g.mul(lts, ntl)
    flat = g.sub(LMT, tendonLength)
    fiberLength = g.fn("sqrt", g.add(g.mul(flat, flat), sqW))
    nfl = g.div(fiberLength, lopt)
    cosP = g.div(flat, fiberLength)
    if mu.ignore_passive_fiber_force:
        fPE = C(0.0)
    else:
        fPE = g.div(g.sub(g.fn("exp", g.div(g.mul(C(4.0), g.sub(nfl, C(1.0))), e0)), peOffset),
                    peDenom)
    x = g.add(g.div(g.sub(nfl, C(1.0)), C(mu.active_force_width_scale)), C(1.0))

    def gl(b1, b2, b3, b4):
        num = g.mul(g.sub(x, C(b2)), g.sub(x, C(b2)))
        dd = g.add(C(b3), g.mul(C(b4), x))
        den = g.mul(dd, dd)
        return g.mul(C(b1), g.fn("exp", g.mul(C(-0.5), g.div(num, den))))
    fAL = g.add(g.add(gl(0.8150671134243542, 1.055033428970575, 0.162384573599574, 0.063303448465465),
                      gl(0.433004984392647, 0.716775413397760, -0.029947116970696, 0.200356847296188)),
                gl(0.1, 1.0, 0.353553390593274, 0.0))
    if compliant and dft is None:
        nff = g.div(ftn, cosP)
        fV = g.div(g.sub(nff, fPE), g.mul(act, fAL))
        nfv = g.div(g.sub(g.fn("sinh", g.mul(C(1.0 / d1), g.sub(fV, C(d4)))), C(d3)), C(d2))
        fiberVelocity = g.mul(nfv, vmax)
        fvat = g.div(fiberVelocity, cosP)
        tendonVelocity = g.sub(VMT, fvat)
        ntv = g.div(tendonVelocity, lts)
    else:
        if dft is not None:
            # calcTendonForceLengthInverseCurveDerivative (.h:471-476)
            ntv = g.div(dft, g.mul(c1kT, g.fn("exp", g.mul(kT, g.sub(ntl, C(c2))))))
            fvat = g.sub(VMT, g.mul(lts, ntv))
        else:
            ntv = C(0.0)
            fvat = VMT
        fiberVelocity = g.mul(fvat, cosP)
        nfv = g.div(fiberVelocity, vmax)
        tv = g.add(g.mul(C(d2), nfv), C(d3))
        arg = g.add(tv, g.fn("sqrt", g.add(g.mul(tv, tv), C(1.0))))
        fV = g.add(g.mul(C(d1), g.fn("log", arg)), C(d4))
    activeF = g.mul(Fmax, g.mul(g.mul(act, fAL), fV))
    conPass = g.mul(Fmax, fPE)
    nonCon = g.mul(g.mul(Fmax, C(mu.fiber_damping)), nfv)
    total = g.add(g.add(activeF, conPass), nonCon)
    T = g.mul(Fmax, ftn) if compliant else g.mul(total, cosP)
    adot = ftdot = C(0.0)
    if has_act:
        adot = _activation_dot(g, act, exc, tau_act, tau_deact)
    resid = None
    if compliant and dft is not None:
        ftdot = dft
        resid = g.sub(T, g.mul(total, cosP))
    elif compliant:
        ftdot = g.mul(ntv, g.mul(c1kT, g.fn("exp", g.mul(kT, g.sub(ntl, C(c2))))))
    return T, adot, ftdot, resid
