"""MocoTrajectory: the solver's guess / solution container, its ``.sto``
file format and its resampling, plus the conversion to and from the NLP
iterate x the C ABI consumes.

Reference behaviour restated here:
  * columns = states, controls, multipliers, derivatives, slacks, parameters,
    in that order (MocoTrajectory::convertToTable, MocoTrajectory.cpp:
    786-800); parameters fill the first row, NaN below (:830-838);
  * header keys num_states / num_controls / num_multipliers /
    num_derivatives / num_slacks / num_parameters (read back by the file
    constructor, MocoTrajectory.cpp:662-700, and required to add up to the
    column count, :719-731);
  * resample(time) (:581-660): slack NaNs are first filled by linear
    interpolation, then every column is re-evaluated from a GCVSplineSet of
    degree min(#times - 1, 5) (zero error variance: the interpolating natural
    spline of ``splines.gcv_interpolating_ppoly``); new times must lie within
    the old ones and be non-decreasing; a zero-duration trajectory is
    broadcast from its first row;
  * the guess handed to the transcription is the trajectory resampled at the
    grid times t0 + (tf - t0) grid (CasOCTranscription.cpp:593-597).

The ``.sto`` writer prints 17 significant digits (a lossless round trip);
the reference's TimeSeriesTable writer prints fewer, which any reader
(this one included) parses the same way.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from .splines import gcv_interpolating_ppoly, ppoly_eval

_BLOCKS = ("states", "controls", "multipliers", "derivatives", "slacks", "parameters")


def variable_names(nlp):
    """(derivative, multiplier, slack) names of ``nlp``'s iterate in the
    reference's convention (problem.ProblemRep: accelerations <coordinate>/
    accel then <muscle>/implicitderiv_normalized_tendon_force, CasOCProblem.h:
    363-377; lambda_cid<c>_p0 / gamma_cid<c>_p0, MocoProblemRep.cpp:202-230);
    generic names where the rep does not carry them."""
    rep = nlp.rep
    ndv, nm, nsl = nlp.NDV, getattr(nlp, "NM", 0), getattr(nlp, "NSL", 0)
    nacc = getattr(nlp, "NACC", 0)
    acc = list(getattr(rep, "accel_names_all", []))
    aux = list(getattr(rep, "aux_derivative_names", []))
    dn = (acc[:nacc] if len(acc) >= nacc else [f"accel_{j}" for j in range(nacc)]) + \
         (aux if len(aux) == ndv - nacc else [f"derivative_{j}" for j in range(nacc, ndv)])
    mult = list(getattr(rep, "multiplier_names", []))
    mn = mult if len(mult) == nm else [f"lambda_{j}" for j in range(nm)]
    slk = list(getattr(rep, "slack_names_all", []))
    sn = slk[:nsl] if len(slk) >= nsl else [f"gamma_{j}" for j in range(nsl)]
    return dn, mn, sn


@dataclass
class MocoTrajectory:
    time: np.ndarray
    state_names: List[str] = field(default_factory=list)
    control_names: List[str] = field(default_factory=list)
    multiplier_names: List[str] = field(default_factory=list)
    derivative_names: List[str] = field(default_factory=list)
    slack_names: List[str] = field(default_factory=list)
    parameter_names: List[str] = field(default_factory=list)
    states: Optional[np.ndarray] = None        # [ntime, nstates]
    controls: Optional[np.ndarray] = None
    multipliers: Optional[np.ndarray] = None
    derivatives: Optional[np.ndarray] = None
    slacks: Optional[np.ndarray] = None
    parameters: Optional[np.ndarray] = None    # [nparameters]
    metadata: Dict[str, str] = field(default_factory=dict)

    def __post_init__(self):
        self.time = np.asarray(self.time, float)
        nt = len(self.time)
        for b in _BLOCKS[:-1]:
            names = getattr(self, b[:-1] + "_names")
            arr = getattr(self, b)
            arr = np.zeros((nt, len(names))) if arr is None else np.asarray(arr, float).reshape(nt, len(names))
            setattr(self, b, arr)
        p = np.zeros(len(self.parameter_names)) if self.parameters is None else self.parameters
        self.parameters = np.asarray(p, float).reshape(len(self.parameter_names))

    # -------------------------------------------------------------- access
    @property
    def num_times(self) -> int:
        return len(self.time)

    def labels(self) -> List[str]:
        return (self.state_names + self.control_names + self.multiplier_names +
                self.derivative_names + self.slack_names + self.parameter_names)

    def get_state(self, name: str) -> np.ndarray:
        return self.states[:, self.state_names.index(name)]

    def get_parameter(self, name: str) -> float:
        """MocoTrajectory::getParameter."""
        return float(self.parameters[self.parameter_names.index(name)])

    def get_control(self, name: str) -> np.ndarray:
        return self.controls[:, self.control_names.index(name)]

    def set_state(self, name: str, values: Sequence[float]):
        self.states[:, self.state_names.index(name)] = np.asarray(values, float)

    def set_control(self, name: str, values: Sequence[float]):
        self.controls[:, self.control_names.index(name)] = np.asarray(values, float)

    def table(self) -> np.ndarray:
        """convertToTable's data block [ntime, ncolumns] (parameters in the
        first row, NaN below)."""
        nt = self.num_times
        par = np.full((nt, len(self.parameter_names)), np.nan)
        if nt and len(self.parameter_names):
            par[0] = self.parameters
        return np.hstack([self.states, self.controls, self.multipliers, self.derivatives,
                          self.slacks, par]) if nt else np.zeros((0, len(self.labels())))

    # -------------------------------------------------------------- .sto I/O
    def write(self, path: str, name: str = "MocoTrajectory"):
        counts = {"num_states": len(self.state_names), "num_controls": len(self.control_names),
                  "num_multipliers": len(self.multiplier_names),
                  "num_derivatives": len(self.derivative_names),
                  "num_slacks": len(self.slack_names), "num_parameters": len(self.parameter_names)}
        meta = dict(self.metadata)
        for k, v in counts.items():
            meta[k] = str(v)
        lines = [name]
        for k in sorted(meta):
            lines.append(f"{k}={meta[k]}")
        lines += ["DataType=double", "version=3", "endheader", "\t".join(["time"] + self.labels())]
        data = self.table()
        for i in range(self.num_times):
            lines.append("\t".join(_num(v) for v in [self.time[i]] + list(data[i])))
        with open(path, "w") as fh:
            fh.write("\n".join(lines) + "\n")

    @staticmethod
    def read(path: str) -> "MocoTrajectory":
        header: Dict[str, str] = {}
        with open(path) as fh:
            lines = fh.read().splitlines()
        i = 0
        while i < len(lines) and lines[i].strip().lower() != "endheader":
            if "=" in lines[i]:
                k, v = lines[i].split("=", 1)
                header[k.strip()] = v.strip()
            i += 1
        if i >= len(lines):
            raise ValueError(f"{path}: no endheader")
        labels = [s.strip() for s in lines[i + 1].split("\t") if s.strip() != ""]
        if not labels or labels[0] != "time":
            raise ValueError(f"{path}: first column must be time")
        labels = labels[1:]
        rows = [[float(v) for v in ln.split()] for ln in lines[i + 2:] if ln.strip()]
        data = np.array(rows, float).reshape(len(rows), len(labels) + 1)
        counts = []
        for key in ("num_states", "num_controls", "num_multipliers", "num_derivatives",
                    "num_slacks", "num_parameters"):
            if key not in header:
                raise ValueError(f"{path}: header has no {key}")
            v = int(header[key])
            if v < 0:
                raise ValueError(f"Invalid {key}.")
            counts.append(v)
        if sum(counts) != len(labels):
            raise ValueError("Expected num_states + num_controls + num_multipliers + num_derivatives "
                             "+ num_slacks + num_parameters = number of columns, but "
                             f"{counts} sum to {sum(counts)} != {len(labels)}.")
        names, blocks, off = [], [], 0
        for n in counts:
            names.append(labels[off:off + n])
            blocks.append(data[:, 1 + off:1 + off + n])
            off += n
        meta = {k: v for k, v in header.items()
                if not k.startswith("num_") and k not in ("DataType", "version")}
        return MocoTrajectory(data[:, 0], *names, *blocks[:5],
                              parameters=blocks[5][0] if len(data) else np.zeros(counts[5]),
                              metadata=meta)

    # -------------------------------------------------------------- resample
    def resample(self, time: Sequence[float]) -> "MocoTrajectory":
        """MocoTrajectory::resample (MocoTrajectory.cpp:581-660); in place,
        returns self."""
        time = np.asarray(time, float)
        if self.num_times < 2:
            raise ValueError("Cannot resample if number of times is 0 or 1.")
        if time[0] < self.time[0]:
            raise ValueError(f"New initial time ({time[0]}) cannot be less than existing initial "
                             f"time ({self.time[0]})")
        if time[-1] > self.time[-1]:
            raise ValueError(f"New final time ({time[-1]}) cannot be less than existing final time "
                             f"({self.time[-1]})")
        if np.any(np.diff(time) < 0):
            raise ValueError("New times must be non-decreasing.")
        # slack NaNs: linear interpolation over the valid samples (:606-610)
        for c in range(self.slacks.shape[1]):
            col = self.slacks[:, c]
            ok = ~np.isnan(col)
            if ok.any() and not ok.all():
                self.slacks[:, c] = np.interp(self.time, self.time[ok], col[ok])
        data = np.hstack([self.states, self.controls, self.multipliers, self.derivatives,
                          self.slacks])
        nt = len(time)
        if time[-1] == time[0]:
            new = np.repeat(data[:1], nt, axis=0)
        else:
            degree = min(self.num_times - 1, 5)
            if degree % 2 == 0:
                # GCVSplineSet(table, {}, min(n - 1, 5)) hands GCVSpline an
                # even degree here, which it rejects (odd degrees only)
                raise ValueError(f"GCVSpline degree must be odd (got {degree} for "
                                 f"{self.num_times} times)")
            new = np.zeros((nt, data.shape[1]))
            if data.shape[1]:
                br, co = gcv_interpolating_ppoly(self.time, data, degree)
                for c in range(data.shape[1]):
                    new[:, c] = ppoly_eval(br, co, time, c)
        self.time = time
        off = 0
        for b in _BLOCKS[:-1]:
            n = getattr(self, b).shape[1]
            setattr(self, b, new[:, off:off + n].copy())
            off += n
        return self

    def resample_with_num_times(self, num_times: int) -> "MocoTrajectory":
        """resampleWithNumTimes: uniformly spaced over the current span."""
        return self.resample(np.linspace(self.time[0], self.time[-1], int(num_times)))

    # -------------------------------------------------------------- NLP iterate
    def to_iterate(self, nlp) -> np.ndarray:
        """The iterate x of ``nlp`` (HipNLP / OracleNLP: its problem's state
        and control names, derivative count and transcription grid): t0 / tf
        from the trajectory's first and last times, every block resampled at
        the grid times (CasOCTranscription.cpp:593-597; columns matched by
        name as convertToCasOCIterate does).  Derivative variables are taken
        in order; missing ones are zero."""
        rep = nlp.rep
        grid = nlp_grid(nlp)
        t0, tf = float(self.time[0]), float(self.time[-1])
        times = (tf - t0) * grid + t0
        r = MocoTrajectory(self.time.copy(), list(self.state_names), list(self.control_names),
                           list(self.multiplier_names), list(self.derivative_names),
                           list(self.slack_names), list(self.parameter_names),
                           self.states.copy(), self.controls.copy(), self.multipliers.copy(),
                           self.derivatives.copy(), self.slacks.copy(), self.parameters.copy())
        r.resample(times)
        G, ndv = len(grid), nlp.NDV
        S = np.zeros((G, nlp.NS))
        for i, n in enumerate(rep.state_names):
            if n not in self.state_names:
                raise ValueError(f"guess has no state '{n}'")
            S[:, i] = r.states[:, self.state_names.index(n)]
        Cm = np.zeros((G, nlp.NC))
        for j, n in enumerate(rep.control_names):
            if n not in self.control_names:
                raise ValueError(f"guess has no control '{n}'")
            Cm[:, j] = r.controls[:, self.control_names.index(n)]
        dn, mn, sn = variable_names(nlp)
        nm, nsl = len(mn), len(sn)
        N = nlp.opts.num_mesh_intervals

        def by_name(want, have, data):
            # columns matched by name (convertToCasOCIterate); where the guess
            # names none of them, its columns are taken in order; missing: 0
            out = np.zeros((G, len(want)))
            named = [n for n in want if n in have]
            for j, n in enumerate(want):
                if n in have:
                    out[:, j] = data[:, have.index(n)]
                elif not named and j < data.shape[1]:
                    out[:, j] = data[:, j]
            return out
        D = by_name(dn, list(self.derivative_names), r.derivatives)
        Mu = by_name(mn, list(self.multiplier_names), r.multipliers)
        Lg = by_name(sn, list(self.slack_names), r.slacks)
        L = Lg[1::2][:N] if nsl else np.zeros((N, 0))   # the slacks at the mesh-interval midpoints
        # parameters by name (the guess's value; missing: the bounds midpoint)
        pn = list(getattr(rep, "parameter_names", []))
        P = nlp.initial_guess_from_bounds()[nlp.n - len(pn):] if pn else np.zeros(0)
        for q, n in enumerate(pn):
            if n in self.parameter_names:
                P[q] = self.parameters[self.parameter_names.index(n)]
        return np.concatenate([[t0, tf], S.ravel(), Cm.ravel(), Mu.ravel(), L.ravel(), D.ravel(), P])

    @staticmethod
    def from_iterate(nlp, x: np.ndarray) -> "MocoTrajectory":
        """The trajectory an iterate x of ``nlp`` describes (times
        t0 + (tf - t0) grid)."""
        rep = nlp.rep
        grid = nlp_grid(nlp)
        G, ns, nc, ndv = len(grid), nlp.NS, nlp.NC, nlp.NDV
        nm, nsl = getattr(nlp, "NM", 0), getattr(nlp, "NSL", 0)
        N = nlp.opts.num_mesh_intervals
        x = np.asarray(x, float)
        pn = list(getattr(rep, "parameter_names", []))
        if len(x) != 2 + (ns + nc + nm + ndv) * G + nsl * N + len(pn):
            raise ValueError("iterate size does not match the problem and grid")
        t0, tf = x[0], x[1]
        o = 2
        S = x[o:o + ns * G].reshape(G, ns); o += ns * G
        Cm = x[o:o + nc * G].reshape(G, nc); o += nc * G
        Mu = x[o:o + nm * G].reshape(G, nm); o += nm * G
        L = x[o:o + nsl * N].reshape(N, nsl); o += nsl * N
        D = x[o:o + ndv * G].reshape(G, ndv)
        # slacks live at the mesh-interval midpoints (HS): NaN elsewhere,
        # as MocoTrajectory holds them
        Lg = np.full((G, nsl), np.nan)
        if nsl:
            Lg[1::2] = L
        dn, mn, sn = variable_names(nlp)
        P = x[len(x) - len(pn):] if pn else np.zeros(0)
        return MocoTrajectory((tf - t0) * grid + t0, list(rep.state_names), list(rep.control_names),
                              mn, dn, sn, pn, S, Cm, Mu, D, Lg, P.copy())

    # -------------------------------------------------------------- comparison
    def compare_continuous_variables_rms(self, other: "MocoTrajectory", states=None, controls=None,
                                         multipliers=None, derivatives=None) -> float:
        """compareContinuousVariablesRMS (MocoTrajectory.cpp:1131-1263): per
        block, the given names (None or []: all, which both trajectories must share;
        ["none"]: skip the block); each column through an interpolating
        GCV spline of degree min(n - 1, 5) per trajectory (0 outside its time
        range), the summed squared error integrated by the trapezoidal rule on
        max(n_self, n_other) uniform times over the union of both ranges;
        sqrt(integral / duration / number of columns)."""
        blocks = (("state", states), ("control", controls), ("multiplier", multipliers),
                  ("derivative", derivatives))
        chosen = []
        for kind, names in blocks:
            mine, theirs = getattr(self, kind + "_names"), getattr(other, kind + "_names")
            if names is None or len(names) == 0:   # empty = all (MocoTrajectory.cpp:1140-1150)
                if sorted(mine) != sorted(theirs):
                    raise ValueError(f"Expected both trajectories to have the same {kind} names; "
                                     f"consider specifying the {kind}s to compare.")
                names = list(mine)
            elif list(names) == ["none"]:
                names = []
            else:
                for n in names:
                    if n not in mine or n not in theirs:
                        raise ValueError(f"Expected '{n}' to be a {kind} in both trajectories.")
            chosen.append((kind + "s", list(names)))
        ncols = sum(len(n) for _, n in chosen)
        if ncols == 0:
            return 0.0
        t0 = min(self.time[0], other.time[0])
        tf = max(self.time[-1], other.time[-1])
        nt = max(self.num_times, other.num_times)
        tt = np.linspace(t0, tf, nt)
        dt = tt[1] - tt[0]

        def sampled(traj, block, names):
            labels = getattr(traj, block[:-1] + "_names")
            data = getattr(traj, block)[:, [labels.index(n) for n in names]]
            degree = min(traj.num_times - 1, 5)
            if degree % 2 == 0:
                raise ValueError(f"GCVSpline degree must be odd (got {degree} for {traj.num_times} times)")
            br, co = gcv_interpolating_ppoly(traj.time, data, degree)
            inside = (traj.time[0] <= tt) & (tt <= traj.time[-1])
            out = np.zeros((nt, len(names)))
            for c in range(len(names)):
                out[inside, c] = ppoly_eval(br, co, tt[inside], c)
            return out

        sse = np.zeros(nt)
        for block, names in chosen:
            if names:
                sse += ((sampled(self, block, names) - sampled(other, block, names)) ** 2).sum(axis=1)
        integral = dt / 2.0 * (sse.sum() + sse[1:nt - 1].sum())
        return float(np.sqrt(integral / (tf - t0) / ncols))

    def compare_parameters_rms(self, other: "MocoTrajectory", names=None) -> float:
        """compareParametersRMS (MocoTrajectory.cpp:1311-1340): None or an
        empty list compares all parameters (NaN when there are none, as the
        reference's sqrt(0 / 0))."""
        if names is None or len(names) == 0:
            if sorted(self.parameter_names) != sorted(other.parameter_names):
                raise ValueError("Expected both trajectories to have the same parameter names; "
                                 "consider specifying the parameters to compare.")
            names = list(self.parameter_names)
        else:
            for n in names:
                if n not in self.parameter_names or n not in other.parameter_names:
                    raise ValueError(f"Expected '{n}' to be a parameter in both trajectories.")
        if not names:
            return float("nan")
        err = [(self.parameters[self.parameter_names.index(n)]
                - other.parameters[other.parameter_names.index(n)]) ** 2 for n in names]
        return float(np.sqrt(sum(err) / len(names)))

    def is_numerically_equal(self, other: "MocoTrajectory", tol: float = 1e-12) -> bool:
        if self.labels() != other.labels() or self.num_times != other.num_times:
            return False
        a, b = self.table(), other.table()
        return bool(np.allclose(self.time, other.time, rtol=0, atol=tol) and
                    np.allclose(a, b, rtol=0, atol=tol, equal_nan=True))


def nlp_grid(nlp) -> np.ndarray:
    from . import abi
    scheme = "hermite-simpson" if nlp.opts.transcription == abi.MH_HERMITE_SIMPSON else "trapezoidal"
    return transcription_grid(scheme, nlp.opts.num_mesh_intervals)


def transcription_grid(scheme: str, num_mesh_intervals: int) -> np.ndarray:
    """Normalized grid of the transcription (uniform mesh, CasOCSolver.h:
    38-42; Hermite-Simpson adds the interval midpoints, CasOCHermiteSimpson.h:
    45-68)."""
    N = int(num_mesh_intervals)
    mesh = np.array([i / N for i in range(N + 1)])
    if scheme == "trapezoidal":
        return mesh
    g = np.zeros(2 * N + 1)
    g[0::2] = mesh
    g[1::2] = 0.5 * (mesh[:-1] + mesh[1:])
    return g


def _num(v: float) -> str:
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Inf" if v > 0 else "-Inf"
    return repr(float(v))
