"""MocoSolver plugin mirror and NLP wrappers over the C ABI.

``MocoHipSolver`` mirrors the property surface of MocoDirectCollocationSolver
/ MocoCasADiSolver that the hot path consumes
(Moco/Moco/MocoDirectCollocationSolver.h:90-153,
 Moco/Moco/MocoCasADiSolver/MocoCasADiSolver.h:115-159; defaults at
 MocoDirectCollocationSolver.cpp:23-43 and MocoCasADiSolver.cpp:37-49).

``HipNLP`` is the IPOPT-facing NLP (the methods of tropter's
IPOPTSolver::TNLP, IPOPTSolver.cpp:302-447) backed by libmocohip.so.
``OracleNLP`` is the same interface backed by the CPU oracle; it exists for
tests and for bench.py's cpu_baseline leg only.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import abi
from .problem import MocoProblem, ProblemRep

_SCHEMES = {"hermite-simpson": abi.MH_HERMITE_SIMPSON,
            "trapezoidal": abi.MH_TRAPEZOIDAL}
_FD = {"central": abi.MH_FD_CENTRAL, "forward": abi.MH_FD_FORWARD,
       "backward": abi.MH_FD_BACKWARD}
_SPARSITY = {"none": abi.MH_SPARSITY_NONE, "random": abi.MH_SPARSITY_RANDOM,
             "initial-guess": abi.MH_SPARSITY_INITIAL_GUESS,
             "given": abi.MH_SPARSITY_GIVEN}


@dataclass
class MocoHipSolver:
    num_mesh_intervals: int = 100
    transcription_scheme: str = "hermite-simpson"
    interpolate_control_midpoints: bool = True
    multibody_dynamics_mode: str = "explicit"
    optim_finite_difference_scheme: str = "central"
    # "none" (block-dense), "random" (3 iterates, CasOCSolver.cpp:70-92) or
    # "initial-guess" (sparsity_guess, default the bounds-midpoint guess)
    optim_sparsity_detection: str = "none"
    optim_sparsity_detection_random_count: int = 3
    # how a detection probe decides a coupling (include/mocohip.h
    # mh_sparsity_rule): "any-change" (default: the reference's rule,
    # CasOCFunction.cpp:44-61 -- any nonzero change or NaN; couplings that
    # cancel to rounding level are then detected or not depending on the
    # order of floating-point operations, so the device's pattern can be a
    # strict superset or subset of another implementation's on those
    # entries, whose values are rounding noise) or "robust" (opt-in: changes
    # below 1e-12 of the callback's output magnitude count as noise -- the
    # pattern is then the model's, the same in every implementation, at the
    # price of dropping real couplings smaller than that)
    optim_sparsity_detection_rule: str = "any-change"
    sparsity_guess: Optional[np.ndarray] = None
    # "given": the callback sparsity itself (HipNLP.callback_sparsity()),
    # e.g. detected once and shared by every shard / replica
    sparsity_pattern: Optional[np.ndarray] = None
    fd_step: float = 1e-8
    device: int = 0
    # MocoDirectCollocationSolver implicit_multibody_acceleration_bounds
    # (default [-1000, 1000], MocoDirectCollocationSolver.cpp:39-40)
    implicit_multibody_acceleration_bounds: tuple = (-1000.0, 1000.0)
    # implicit_auxiliary_derivative_bounds (MocoDirectCollocationSolver.cpp:41)
    implicit_auxiliary_derivative_bounds: tuple = (-1000.0, 1000.0)
    # kinematic constraints (MocoDirectCollocationSolver.cpp:29-42)
    enforce_constraint_derivatives: bool = True
    velocity_correction_bounds: tuple = (-0.1, 0.1)
    minimize_lagrange_multipliers: bool = False
    lagrange_multiplier_weight: float = 1.0
    # "callback-fd" (MocoCasADiSolver: FD of each per-point callback) or
    # "global-seeds" (tropter: central FD of g along colored seed columns,
    # ProblemDecorator_double.cpp:261-291)
    jacobian_mode: str = "callback-fd"
    # the column order of the global-seed coloring: "smallest-last" (ColPack's
    # SMALLEST_LAST, as tropter requests it, GraphColoring.cpp:91-94) or
    # "natural" (index order; ABI <= 7)
    coloring_order: str = "smallest-last"
    # the optimizer settings (MocoDirectCollocationSolver.cpp:23-42), mapped
    # to Ipopt options by ipopt_options()
    verbosity: int = 2
    optim_solver: str = "ipopt"
    optim_max_iterations: int = -1
    optim_convergence_tolerance: float = -1.0
    optim_constraint_tolerance: float = -1.0
    optim_hessian_approximation: str = "limited-memory"
    optim_ipopt_print_level: int = -1
    # guess: a MocoTrajectory (or a .sto path, guess_file), resampled onto
    # the transcription grid (CasOCTranscription.cpp:593-597); default the
    # bounds-midpoint guess
    guess_file: str = ""

    def ipopt_options(self) -> dict:
        """The Ipopt options MocoCasADiSolver sets from these properties
        (MocoCasADiSolver.cpp:210-246, incl. its range checks), for a host
        Ipopt driving the C ABI (csrc/host/mh_ipopt_tnlp.hpp
        applies the same mapping)."""
        if self.optim_max_iterations < 0 and self.optim_max_iterations != -1:
            raise ValueError("optim_max_iterations must be >= 0 or -1")
        for name in ("optim_convergence_tolerance", "optim_constraint_tolerance"):
            v = getattr(self, name)
            if v < 0 and v != -1:
                raise ValueError(f"{name} must be >= 0 or -1")
        if self.verbosity not in (0, 1, 2):
            raise ValueError("verbosity must be 0, 1 or 2")
        opts: dict = {}
        if self.optim_solver != "ipopt":
            return opts
        opts["print_user_options"] = "yes"
        if self.verbosity < 2:
            opts["print_level"] = 0
        elif self.optim_ipopt_print_level != -1:
            opts["print_level"] = int(self.optim_ipopt_print_level)
        opts["hessian_approximation"] = self.optim_hessian_approximation
        if self.optim_max_iterations != -1:
            opts["max_iter"] = int(self.optim_max_iterations)
        if self.optim_convergence_tolerance != -1:
            tol = float(self.optim_convergence_tolerance)
            for k in ("tol", "dual_inf_tol", "compl_inf_tol", "acceptable_tol",
                      "acceptable_dual_inf_tol", "acceptable_compl_inf_tol"):
                opts[k] = tol
        if self.optim_constraint_tolerance != -1:
            tol = float(self.optim_constraint_tolerance)
            opts["constr_viol_tol"] = tol
            opts["acceptable_constr_viol_tol"] = tol
        return opts

    def starting_point(self, nlp, guess=None) -> np.ndarray:
        """IPOPT's starting point for ``nlp``: ``guess`` (a MocoTrajectory),
        else ``guess_file`` (.sto), resampled onto the grid; else the
        bounds-midpoint guess (CasOCTranscription.cpp:1123-1149)."""
        from .trajectory import MocoTrajectory
        if guess is None and self.guess_file:
            guess = MocoTrajectory.read(self.guess_file)
        if guess is None:
            return nlp.initial_guess_from_bounds()
        return guess.to_iterate(nlp)

    def options(self, interval_begin: int = 0, interval_end: int = 0) -> abi.mh_options:
        if self.transcription_scheme not in _SCHEMES:
            raise ValueError(f"transcription_scheme {self.transcription_scheme!r} "
                             "not in {'trapezoidal', 'hermite-simpson'}")
        if self.optim_finite_difference_scheme not in _FD:
            raise ValueError("optim_finite_difference_scheme must be one of "
                             "central, forward, backward")
        if self.multibody_dynamics_mode not in ("explicit", "implicit"):
            raise ValueError("multibody_dynamics_mode must be 'explicit' or 'implicit'")
        if self.optim_sparsity_detection not in _SPARSITY:
            raise ValueError("optim_sparsity_detection must be one of none, random, "
                             "initial-guess")   # MocoCasADiSolver.cpp:248-249
        o = abi.mh_options()
        o.num_mesh_intervals = int(self.num_mesh_intervals)
        o.transcription = _SCHEMES[self.transcription_scheme]
        o.interpolate_control_midpoints = int(bool(self.interpolate_control_midpoints))
        o.finite_difference_scheme = _FD[self.optim_finite_difference_scheme]
        o.fd_step = float(self.fd_step)
        o.interval_begin = int(interval_begin)
        o.interval_end = int(interval_end)
        o.device = int(self.device)
        o.multibody_dynamics_mode = (abi.MH_DYNAMICS_IMPLICIT if self.multibody_dynamics_mode == "implicit"
                                     else abi.MH_DYNAMICS_EXPLICIT)
        lo, hi = self.implicit_multibody_acceleration_bounds
        o.implicit_accel_bounds[0] = float(lo)
        o.implicit_accel_bounds[1] = float(hi)
        lo, hi = self.implicit_auxiliary_derivative_bounds
        o.implicit_aux_bounds[0] = float(lo)
        o.implicit_aux_bounds[1] = float(hi)
        o.ignore_constraint_derivatives = 0 if self.enforce_constraint_derivatives else 1
        o.minimize_lagrange_multipliers = int(bool(self.minimize_lagrange_multipliers))
        o.lagrange_multiplier_weight = float(self.lagrange_multiplier_weight)
        modes = {"callback-fd": abi.MH_JACOBIAN_CALLBACK_FD, "global-seeds": abi.MH_JACOBIAN_GLOBAL_SEEDS}
        if self.jacobian_mode not in modes:
            raise ValueError("jacobian_mode must be 'callback-fd' or 'global-seeds'")
        o.jacobian_mode = modes[self.jacobian_mode]
        orders = {"smallest-last": abi.MH_COLORING_SMALLEST_LAST, "natural": abi.MH_COLORING_NATURAL}
        if self.coloring_order not in orders:
            raise ValueError("coloring_order must be 'smallest-last' or 'natural'")
        o.coloring_order = orders[self.coloring_order]
        lo, hi = self.velocity_correction_bounds
        o.velocity_correction_bounds[0] = float(lo)
        o.velocity_correction_bounds[1] = float(hi)
        o.sparsity_detection = _SPARSITY[self.optim_sparsity_detection]
        o.sparsity_random_count = int(self.optim_sparsity_detection_random_count)
        rules = {"robust": abi.MH_SPARSITY_RULE_ROBUST, "any-change": abi.MH_SPARSITY_RULE_ANY_CHANGE}
        if self.optim_sparsity_detection_rule not in rules:
            raise ValueError("optim_sparsity_detection_rule must be 'robust' or 'any-change'")
        o.sparsity_rule = rules[self.optim_sparsity_detection_rule]
        if self.sparsity_guess is not None:
            if self.optim_sparsity_detection != "initial-guess":
                raise ValueError("sparsity_guess needs optim_sparsity_detection='initial-guess'")
            self._guess = np.ascontiguousarray(self.sparsity_guess, float).reshape(-1)
            o.sparsity_guess = abi.dptr(self._guess)
            o._guess_size = self._guess.size   # checked against n by check_guess_size
        if (self.sparsity_pattern is not None) != (self.optim_sparsity_detection == "given"):
            raise ValueError("optim_sparsity_detection='given' goes with sparsity_pattern")
        if self.sparsity_pattern is not None:
            self._pattern = np.ascontiguousarray(self.sparsity_pattern, np.uint8)
            o.sparsity_pattern = self._pattern.ctypes.data_as(C.POINTER(C.c_uint8))
        return o


class _NLPBase:
    prefix = ""

    def __init__(self, rep: ProblemRep, opts: abi.mh_options):
        self.rep = rep
        self.opts = opts
        self.ctx = C.c_void_p()
        self._create()
        info = abi.mh_nlp_info()
        self._check(self._fn("get_nlp_info")(self.ctx, C.byref(info)))
        self.info = info
        self.n, self.m, self.nnz = int(info.n), int(info.m), int(info.nnz_jac_g)
        self.G = int(info.num_grid_points)
        self.NS, self.NC = int(info.num_states), int(info.num_controls)
        self.NQ = rep.nq
        self.row_begin, self.row_end = int(info.row_begin), int(info.row_end)
        self.nnz_begin, self.nnz_end = int(info.nnz_begin), int(info.nnz_end)

    # -- plumbing
    def _fn(self, name):
        return getattr(self.lib, self.prefix + name)

    def _check(self, rc):
        if rc != 0:
            err = self._fn("last_error")()
            raise RuntimeError(f"{self.prefix}: error {rc}: {err.decode() if err else ''}")

    def _create(self):
        self._check(self._fn("create")(C.byref(self.rep.struct), C.byref(self.opts),
                                       C.byref(self.ctx)))

    def close(self):
        if self.ctx:
            self._fn("destroy")(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- TNLP surface
    def bounds(self):
        xl, xu = np.empty(self.n), np.empty(self.n)
        gl, gu = np.empty(max(self.m, 1)), np.empty(max(self.m, 1))
        self._check(self._fn("get_bounds")(self.ctx, abi.dptr(xl), abi.dptr(xu),
                                           abi.dptr(gl), abi.dptr(gu)))
        return xl, xu, gl[:self.m], gu[:self.m]

    def initial_guess_from_bounds(self):
        x = np.empty(self.n)
        self._check(self._fn("get_initial_guess_from_bounds")(self.ctx, abi.dptr(x)))
        return x

    def random_iterate(self, rand: np.ndarray):
        rand = np.ascontiguousarray(rand, float)
        assert rand.shape == (self.n,)
        x = np.empty(self.n)
        self._check(self._fn("get_random_iterate")(self.ctx, abi.dptr(rand), abi.dptr(x)))
        return x

    def jac_structure(self):
        ir = np.empty(max(self.nnz, 1), np.int32)
        jc = np.empty(max(self.nnz, 1), np.int32)
        self._check(self._fn("get_jac_structure")(self.ctx, abi.iptr(ir), abi.iptr(jc)))
        return ir[:self.nnz], jc[:self.nnz]

    @property
    def prescribed(self) -> bool:
        """Prescribed kinematics (PositionMotion): q, u not NLP states."""
        return bool(getattr(self.rep, "prescribed_kinematics", False))

    @property
    def TQ(self) -> int:
        """Coordinates among the NLP states (0 with prescribed kinematics)."""
        return 0 if self.prescribed else self.NQ

    @property
    def NZ(self) -> int:
        return self.NS - 2 * self.TQ

    @property
    def SO(self) -> int:
        """Callback output of state s's derivative: s + SO (s >= TQ)."""
        return self.NQ if self.prescribed else -self.NQ

    @property
    def implicit(self) -> bool:
        return self.opts.multibody_dynamics_mode == abi.MH_DYNAMICS_IMPLICIT

    @property
    def NACC(self) -> int:
        """Acceleration variables per grid point (implicit mode: NQ; none
        with prescribed kinematics)."""
        return self.NQ if self.implicit and not self.prescribed else 0

    @property
    def NMB(self) -> int:
        """Multibody residual rows per grid point."""
        return self.NQ if self.implicit else 0

    @property
    def NAR(self) -> int:
        """Implicit auxiliary derivatives / residuals per grid point."""
        return self.rep.num_aux_residuals

    @property
    def NDV(self) -> int:
        """Derivative variables per grid point: accelerations, then the
        implicit auxiliary derivatives."""
        return self.NACC + self.NAR

    @property
    def NKC(self) -> int:
        """Kinematic constraints (CoordinateCouplers) of the model."""
        return getattr(self.rep, "num_kinematic_constraints", 0)

    @property
    def NM(self) -> int:
        """Lagrange multipliers per grid point."""
        return self.NKC

    @property
    def NK(self) -> int:
        """Kinematic-constraint rows per mesh point (position, velocity and
        acceleration errors when enforcing constraint derivatives); none with
        prescribed kinematics (CasOCProblem.h:508-521)."""
        if getattr(self.rep, "prescribed_kinematics", False):
            return 0
        return self.NKC * (1 if self.opts.ignore_constraint_derivatives else 3)

    @property
    def NSL(self) -> int:
        """Velocity-correction slacks per mesh interval (Hermite-Simpson,
        enforcing derivatives)."""
        return (self.NKC if not self.opts.ignore_constraint_derivatives
                and self.opts.transcription == abi.MH_HERMITE_SIMPSON
                and not getattr(self.rep, "prescribed_kinematics", False) else 0)

    @property
    def NI(self) -> int:
        """Per-point inputs: states, controls, derivatives, multipliers,
        slacks."""
        return self.NS + self.NC + self.NDV + self.NM + self.NSL

    @property
    def NPAR(self) -> int:
        """MocoParameters: the last NPAR variables of x."""
        return int(self.rep.struct.nparameters)

    @property
    def NO(self) -> int:
        """DAE callback outputs: udot or multibody residual, zdot, auxiliary
        residuals, kinematic errors, velocity correction (with slacks)."""
        return self.NQ + self.NZ + self.NAR + self.NK + (self.NQ if self.NSL else 0)

    def point_inputs(self, x: np.ndarray) -> np.ndarray:
        """[G, NI] per grid point inputs from iterate x (the column layout of
        include/mocohip.h: t0, tf, states, controls, multipliers, slacks,
        derivatives; a grid point's slacks are its interval's at a
        mesh-interval midpoint, 0 elsewhere)."""
        G, NS, NC, NDV, NM, NSL = self.G, self.NS, self.NC, self.NDV, self.NM, self.NSL
        N = self.opts.num_mesh_intervals
        o = 2
        S = x[o:o + NS * G].reshape(G, NS); o += NS * G
        U = x[o:o + NC * G].reshape(G, NC); o += NC * G
        M = x[o:o + NM * G].reshape(G, NM); o += NM * G
        L = x[o:o + NSL * N].reshape(N, NSL); o += NSL * N
        W = x[o:o + NDV * G].reshape(G, NDV)
        Lg = np.zeros((G, NSL))
        if NSL:
            Lg[1::2] = L
        return np.concatenate([S, U, W, M, Lg], 1)

    @property
    def NRES(self) -> int:
        """Residual rows per grid point (multibody, then auxiliary)."""
        return self.NMB + self.NAR

    @property
    def NEP(self) -> int:
        """Endpoint-constraint equations (rows 0 .. NEP of g)."""
        return getattr(self.rep, "num_endpoint_equations", 0)

    def callback_sparsity(self) -> np.ndarray:
        """The callback sparsity behind the Jacobian structure: the NO DAE
        outputs then the path equations, rows of W = [time, inputs] flags,
        then the endpoint equations, rows of 2 W flags."""
        W = 1 + self.NI
        buf = np.zeros((self.NO + self.NPC + 2 * self.NEP) * W, np.uint8)
        self._check(self._fn("get_callback_sparsity")(
            self.ctx, buf.ctypes.data_as(C.POINTER(C.c_uint8)), buf.size))
        return buf

    @property
    def NPC(self) -> int:
        """Path-constraint equations per mesh point."""
        return self.rep.num_path_equations

    @property
    def tail_rows(self) -> int:
        """Rows after the last interval's own: the final mesh point's path
        rows and the final grid point's residuals."""
        return self.NK + self.NPC + self.NRES

    def jacobian_seeds(self):
        """(color per x column, seed count) of the global-seed Jacobian
        (jacobian_mode "global-seeds")."""
        color = np.empty(self.n, np.int32)
        k = C.c_int32()
        self._check(self._fn("get_jacobian_seeds")(self.ctx, abi.iptr(color), C.byref(k)))
        return color, int(k.value)

    def eval_f_partial(self, x) -> float:
        """This shard's objective partial (mh_eval_f_partial): the partials
        of all shards sum to eval_f."""
        x = np.ascontiguousarray(x, float)
        f = np.zeros(1)
        self._check(self._fn("eval_f_partial")(self.ctx, abi.dptr(x), abi.dptr(f)))
        return float(f[0])

    def eval_grad_f_partial(self, x) -> np.ndarray:
        """This shard's gradient partial (n doubles; the sum over the shards
        is eval_grad_f)."""
        x = np.ascontiguousarray(x, float)
        g = np.empty(self.n)
        self._check(self._fn("eval_grad_f_partial")(self.ctx, abi.dptr(x), abi.dptr(g)))
        return g

    def eval_dae(self, inputs: np.ndarray) -> np.ndarray:
        """Per-point DAE: rows [t, states, controls, derivatives] ->
        [udot or multibody residual, zdot, auxiliary residuals]."""
        inputs = np.ascontiguousarray(inputs, float)
        npts = inputs.shape[0]
        assert inputs.shape[1] == 1 + self.NI
        out = np.empty((npts, self.NO))
        self._check(self._fn("eval_dae")(self.ctx, npts, abi.dptr(inputs), abi.dptr(out)))
        return out

class HipBatch:
    """mh_batch: structurally identical HipNLPs evaluated by one launch per
    kernel (include/mocohip.h mh_batch_*).  Calls take one device pointer
    per NLP and run on the first NLP's stream."""

    def __init__(self, nlps, group_results_global: bool | None = None):
        self.nlps = list(nlps)
        self.lib = self.nlps[0].lib
        arr = (C.c_void_p * len(self.nlps))(*[n.ctx.value for n in self.nlps])
        self.batch = C.c_void_p()
        rc = self.lib.mh_batch_create(arr, len(self.nlps), C.byref(self.batch))
        if rc:
            raise RuntimeError(f"mh_batch_create: error {rc}: {self.lib.mh_last_error().decode()}")
        if group_results_global is not None:
            self._check(self.lib.mh_batch_set_group_results_global(self.batch, int(bool(group_results_global))))

    def _check(self, rc):
        if rc:
            raise RuntimeError(f"mh_batch: error {rc}: {self.lib.mh_last_error().decode()}")

    @staticmethod
    def _ptrs(ptrs):
        return (C.c_void_p * len(ptrs))(*[C.c_void_p(p) for p in ptrs])

    def eval_g_device(self, xs, gs):
        self._check(self.lib.mh_batch_eval_g_device(self.batch, self._ptrs(xs), self._ptrs(gs)))

    def eval_jac_g_device(self, xs, vs):
        self._check(self.lib.mh_batch_eval_jac_g_device(self.batch, self._ptrs(xs), self._ptrs(vs)))

    def eval_g_jac_g_device(self, xs, gs, vs):
        self._check(self.lib.mh_batch_eval_g_jac_g_device(self.batch, self._ptrs(xs), self._ptrs(gs),
                                                          self._ptrs(vs)))

    def close(self):
        if self.batch:
            self.lib.mh_batch_destroy(self.batch)
            self.batch = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def check_guess_size(rep: ProblemRep, opts: abi.mh_options, lib=None) -> None:
    """mh_create reads n doubles from mh_options.sparsity_guess: refuse a
    guess of another size before it does (n from mh_get_nlp_info_for, the
    host-only layout query)."""
    size = getattr(opts, "_guess_size", None)
    if not opts.sparsity_guess or size is None:
        return
    lib = lib or abi.load_mocohip()
    info = abi.mh_nlp_info()
    if lib.mh_get_nlp_info_for(C.byref(rep.struct), C.byref(opts), C.byref(info)) != 0:
        raise ValueError(lib.mh_last_error().decode())
    if size != int(info.n):
        raise ValueError(f"sparsity_guess has {size} values, the problem has n = {int(info.n)}")


class HipNLP(_NLPBase):
    """NLP backed by libmocohip.so (the product path)."""
    prefix = "mh_"

    def __init__(self, rep: ProblemRep, opts: abi.mh_options, lib=None):
        self.lib = lib or abi.load_mocohip()
        check_guess_size(rep, opts, self.lib)
        super().__init__(rep, opts)

    def device_kkt(self, warm: bool = False):
        """The device KKT module over this context (include/mocohip_kkt.h,
        mocohip.kkt.DeviceKKT; created once): the host optimizer's Newton
        systems factored next to the Jacobian.  Raises ValueError when the
        Jacobian lacks the per-interval block structure, RuntimeError on a
        sharded context.  warm=True (set-up ahead of a timed region, e.g. a
        sweep's workers) also runs DeviceKKT.warm at creation: the first
        kernel launches and graph captures, at the bounds-midpoint guess;
        otherwise they happen in the first solve."""
        if getattr(self, "_dkkt", None) is None:
            from .kkt import DeviceKKT
            dk = DeviceKKT(self)
            if warm:
                try:
                    dk.warm(self.initial_guess_from_bounds())
                except Exception:
                    dk.close()
                    raise
            self._dkkt = dk
        return self._dkkt

    def close(self):
        k = getattr(self, "_dkkt", None)
        if k is not None:
            k.close()
            self._dkkt = None
        super().close()

    def eval_f(self, x, new_x=True):
        x = np.ascontiguousarray(x, float)
        f = np.zeros(1)
        self._check(self.lib.mh_eval_f(self.ctx, abi.dptr(x), int(new_x), abi.dptr(f)))
        return float(f[0])

    def eval_grad_f(self, x, new_x=True):
        x = np.ascontiguousarray(x, float)
        g = np.empty(self.n)
        self._check(self.lib.mh_eval_grad_f(self.ctx, abi.dptr(x), int(new_x), abi.dptr(g)))
        return g

    def objective_terms(self, x) -> np.ndarray:
        """The objective's weighted terms at x, one per goal of the problem
        (mh_eval_objective_terms; their sum in goal order is eval_f)."""
        x = np.ascontiguousarray(x, float)
        k = C.c_int32(0)
        self.lib.mh_eval_objective_terms(self.ctx, abi.dptr(x), abi.dptr(np.zeros(1)), C.byref(k))
        out = np.zeros(max(int(k.value), 1))
        k = C.c_int32(len(out))
        self._check(self.lib.mh_eval_objective_terms(self.ctx, abi.dptr(x), abi.dptr(out), C.byref(k)))
        return out[:int(k.value)]

    def eval_g(self, x, new_x=True):
        x = np.ascontiguousarray(x, float)
        g = np.empty(max(self.row_end - self.row_begin, 1))
        self._check(self.lib.mh_eval_g(self.ctx, abi.dptr(x), int(new_x), abi.dptr(g)))
        return g[:self.row_end - self.row_begin]

    def eval_jac_g(self, x, new_x=True):
        x = np.ascontiguousarray(x, float)
        v = np.empty(max(self.nnz_end - self.nnz_begin, 1))
        self._check(self.lib.mh_eval_jac_g(self.ctx, abi.dptr(x), int(new_x), abi.dptr(v)))
        return v[:self.nnz_end - self.nnz_begin]

    def eval_g_jac_g(self, x):
        x = np.ascontiguousarray(x, float)
        g = np.empty(max(self.row_end - self.row_begin, 1))
        v = np.empty(max(self.nnz_end - self.nnz_begin, 1))
        self._check(self.lib.mh_eval_g_jac_g(self.ctx, abi.dptr(x), abi.dptr(g), abi.dptr(v)))
        return g[:self.row_end - self.row_begin], v[:self.nnz_end - self.nnz_begin]

    def eval_g_jac_g_device(self, x_ptr: int, g_ptr: int, v_ptr: int):
        self._check(self.lib.mh_eval_g_jac_g_device(self.ctx, C.c_void_p(x_ptr), C.c_void_p(g_ptr),
                                                    C.c_void_p(v_ptr)))

    def eval_g_device(self, x_ptr: int, g_ptr: int):
        self._check(self.lib.mh_eval_g_device(self.ctx, C.c_void_p(x_ptr), C.c_void_p(g_ptr)))

    def eval_jac_g_device(self, x_ptr: int, v_ptr: int):
        self._check(self.lib.mh_eval_jac_g_device(self.ctx, C.c_void_p(x_ptr), C.c_void_p(v_ptr)))

    def tnlp_eval_g_device(self, x_ptr: int, new_x: bool, g_ptr: int):
        """TNLP::eval_g on device pointers with IPOPT's new_x."""
        self._check(self.lib.mh_tnlp_eval_g_device(self.ctx, C.c_void_p(x_ptr), int(bool(new_x)),
                                                   C.c_void_p(g_ptr)))

    def tnlp_eval_jac_g_device(self, x_ptr: int, new_x: bool, v_ptr: int):
        """TNLP::eval_jac_g on device pointers with IPOPT's new_x: new_x =
        False (x unchanged since the last tnlp_eval_g_device) lets the
        Jacobian run beside that eval_g on the context's auxiliary stream."""
        self._check(self.lib.mh_tnlp_eval_jac_g_device(self.ctx, C.c_void_p(x_ptr), int(bool(new_x)),
                                                       C.c_void_p(v_ptr)))

    def lane_stride(self) -> int:
        """Finite-difference lanes per grid point (mh_debug_jacobian_lanes)."""
        ND = 2 + self.NI + self.NPAR   # t0, tf, the point inputs, the parameters
        return 2 * ND + 1 if self.opts.finite_difference_scheme == abi.MH_FD_CENTRAL else ND + 1

    def jacobian_lanes(self, x):
        """(times[G], Y[G, NO, S]): the raw lane outputs behind eval_jac_g(x)
        (mh_debug_jacobian_lanes; parity tests)."""
        x = np.ascontiguousarray(x, float)
        S = self.lane_stride()
        t = np.empty(self.G)
        Y = np.empty(self.G * self.NO * S)
        self._check(self.lib.mh_debug_jacobian_lanes(self.ctx, abi.dptr(x), abi.dptr(t), abi.dptr(Y)))
        return t, Y.reshape(self.G, self.NO, S)

    def time_stages(self, x_ptr: int, kind: int = 1, reps: int = 50):
        """(DAE stage ms, transcription stage ms): average device duration
        over ``reps`` back-to-back launches of each stage alone at the device
        iterate ``x_ptr`` (mh_debug_time_stages; bench roofline)."""
        ms = np.zeros(2)
        self._check(self.lib.mh_debug_time_stages(self.ctx, C.c_void_p(x_ptr), int(kind), int(reps),
                                                  abi.dptr(ms)))
        return float(ms[0]), float(ms[1])

    def backend(self):
        """(back-end name, FP64 ops per generated DAE eval, model hash)."""
        buf = C.create_string_buffer(128)
        fl = C.c_double()
        h = C.c_uint64()
        self._check(self.lib.mh_get_backend(self.ctx, buf, 128, C.byref(fl), C.byref(h)))
        return buf.value.decode(), fl.value, h.value

    def work(self):
        """FP64 ops per eval_jac_g / eval_g DAE stage, group evaluations per
        eval_jac_g, full-DAE-equivalent lanes per eval_jac_g (mh_get_work)."""
        w = np.zeros(4)
        self._check(self.lib.mh_get_work(self.ctx, abi.dptr(w)))
        return w

    def uses_interval_kernel(self) -> bool:
        """True when eval_jac_g runs the fused k_interval transcription
        (group results combined in LDS) rather than k_combine + k_transcribe."""
        return "interval" in self.backend_flags()

    def backend_flags(self) -> str:
        buf = C.create_string_buffer(256)
        self._check(self.lib.mh_get_backend_flags(self.ctx, buf, 256))
        return buf.value.decode()

    def set_stream(self, stream: int | None):
        """Order this context's work on a HIP stream (e.g.
        torch.cuda.current_stream().cuda_stream); None = its own stream."""
        self._check(self.lib.mh_set_stream(self.ctx, C.c_void_p(stream or 0)))

    def set_async(self, on: bool):
        """*_device entries return once enqueued (mh_set_async)."""
        self._check(self.lib.mh_set_async(self.ctx, int(bool(on))))

    def synchronize(self):
        self._check(self.lib.mh_synchronize(self.ctx))

    def set_timing(self, on: bool):
        """Record stage events on every evaluation (mh_set_timing)."""
        self._check(self.lib.mh_set_timing(self.ctx, int(bool(on))))

    def last_timings(self):
        """[whole, DAE stage, transcription stage, k_groups] of the last
        evaluation in ms (needs set_timing(True))."""
        t = np.zeros(4)
        self._check(self.lib.mh_last_timings(self.ctx, abi.dptr(t)))
        return t


class OracleNLP(_NLPBase):
    """NLP backed by the CPU oracle — TEST INFRASTRUCTURE / CPU BASELINE."""
    prefix = "orc_"

    def __init__(self, rep: ProblemRep, opts: abi.mh_options, threads: int = 1):
        self.lib = abi.load_oracle()
        super().__init__(rep, opts)
        self.lib.orc_set_threads(self.ctx, int(threads))

    def eval_dae_params(self, inputs: np.ndarray, x: np.ndarray, moved: int = -1,
                        step: float = 0.0) -> np.ndarray:
        """eval_dae on the model with iterate x's MocoParameters applied,
        parameter ``moved`` (-1: none) moved by ``step``."""
        inputs = np.ascontiguousarray(inputs, float)
        x = np.ascontiguousarray(x, float)
        npts = inputs.shape[0]
        assert inputs.shape[1] == 1 + self.NI and x.size == self.n
        out = np.empty((npts, self.NO))
        self._check(self.lib.orc_eval_dae_params(self.ctx, abi.dptr(x), int(moved), float(step), npts,
                                                 abi.dptr(inputs), abi.dptr(out)))
        return out

    def eval_f(self, x, new_x=True):
        x = np.ascontiguousarray(x, float)
        f = np.zeros(1)
        self._check(self.lib.orc_eval_f(self.ctx, abi.dptr(x), abi.dptr(f)))
        return float(f[0])

    def eval_grad_f(self, x, new_x=True):
        x = np.ascontiguousarray(x, float)
        g = np.empty(self.n)
        self._check(self.lib.orc_eval_grad_f(self.ctx, abi.dptr(x), abi.dptr(g)))
        return g

    def eval_g(self, x, new_x=True):
        """This context's rows (all of g unless it is a shard)."""
        x = np.ascontiguousarray(x, float)
        nr = self.row_end - self.row_begin
        g = np.empty(max(nr, 1))
        self._check(self.lib.orc_eval_g(self.ctx, abi.dptr(x), abi.dptr(g)))
        return g[:nr]

    def eval_jac_g(self, x, new_x=True):
        """This context's nonzeros (all of them unless it is a shard)."""
        x = np.ascontiguousarray(x, float)
        nz = self.nnz_end - self.nnz_begin
        v = np.empty(max(nz, 1))
        self._check(self.lib.orc_eval_jac_g(self.ctx, abi.dptr(x), abi.dptr(v)))
        return v[:nz]


def _oracle_assemble(self, x, times, Y):
    """(g, J) re-derived by the oracle from raw lanes (orc_assemble_from_lanes)."""
    x = np.ascontiguousarray(x, float)
    times = np.ascontiguousarray(times, float)
    Y = np.ascontiguousarray(Y, float)
    g = np.empty(max(self.m, 1))
    v = np.empty(max(self.nnz, 1))
    self._check(self.lib.orc_assemble_from_lanes(self.ctx, abi.dptr(x), abi.dptr(times), abi.dptr(Y),
                                                 abi.dptr(g), abi.dptr(v)))
    return g[:self.m], v[:self.nnz]


OracleNLP.assemble_from_lanes = _oracle_assemble


class MocoStudy:
    """MocoStudy mirror: owns a problem and a solver; ``create_nlp`` builds
    the transcription on the HIP path (MocoStudy.cpp:79-101)."""

    def __init__(self, problem: Optional[MocoProblem] = None,
                 solver: Optional[MocoHipSolver] = None):
        self.problem = problem or MocoProblem()
        self.solver = solver or MocoHipSolver()

    def init_solver(self) -> MocoHipSolver:
        self.solver = MocoHipSolver()
        return self.solver

    def create_nlp(self, interval_begin: int = 0, interval_end: int = 0) -> HipNLP:
        rep = self.problem.create_rep()
        return HipNLP(rep, self.solver.options(interval_begin, interval_end))

    def solve(self, guess=None, nlp=None, method: str = "ipm", linear_solver: str = "auto"):
        """MocoStudy::solve (MocoStudy.cpp:79-101): transcribe on the HIP
        path, optimize from the solver's starting point, return the
        solution as a MocoTrajectory with the solve statistics in its
        metadata (success, objective, num_iterations, solver_duration,
        status; MocoSolver::setSolutionStats, MocoSolver.h:97-102).  The
        optimizer is mocohip.nlpsolve (Ipopt is absent here; default the
        interior-point restatement mocohip.ipm) with the Ipopt options
        MocoCasADiSolver sets from optim_convergence_tolerance /
        optim_constraint_tolerance / optim_max_iterations
        (MocoHipSolver.ipopt_options; Ipopt's defaults where unset).
        linear_solver: the Newton systems' back end (mocohip.ipm
        IpmOptions.linear_solver: "auto" = on the device next to the
        Jacobian when the NLP offers it)."""
        from .nlpsolve import solve_nlp
        from .trajectory import MocoTrajectory
        own = nlp is None
        nlp = nlp or self.create_nlp()
        try:
            x0 = self.solver.starting_point(nlp, guess)
            s = self.solver
            tol = s.optim_convergence_tolerance if s.optim_convergence_tolerance > 0 else 1e-8
            ctol = s.optim_constraint_tolerance if s.optim_constraint_tolerance > 0 else 1e-8
            it = s.optim_max_iterations if s.optim_max_iterations > 0 else 5000
            opts = s.ipopt_options() if method == "ipm" else None
            if opts is not None:
                opts["linear_solver"] = linear_solver
            r = solve_nlp(nlp, x0, tol, ctol, it, method=method, ipopt_options=opts)
            sol = MocoTrajectory.from_iterate(nlp, r.x)
            # the objective's breakdown at the solution (setSolutionStats'
            # objectiveBreakdown, MocoSolver.h:97-102): one term per goal
            r.objective_breakdown = None
            if hasattr(nlp, "objective_terms"):
                terms = nlp.objective_terms(r.x)
                names = list(getattr(nlp.rep, "goal_names", []))
                r.objective_breakdown = [(names[i] if i < len(names) else f"goal_{i}", float(v))
                                         for i, v in enumerate(terms)]
        finally:
            if own:
                nlp.close()
        sol.metadata.update({"success": "true" if r.success else "false", "objective": repr(r.objective),
                             "num_iterations": str(r.iterations), "solver_duration": repr(r.duration),
                             "status": r.status, "optimizer": r.optimizer + " over the C ABI"})
        sol.stats = r
        return sol
