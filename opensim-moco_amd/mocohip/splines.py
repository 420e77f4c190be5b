"""Data splines used by the hot path.

OpenSim evaluates tabulated data (ExternalForce ground reactions, MocoTrack
/ MocoStateTrackingGoal references) through ``GCVSpline`` (Woltring's
GCVSPL) with zero error variance (MocoStateTrackingGoal.cpp:29,
GCVSplineSet defaults).  With zero error variance GCVSPL returns the
interpolating *natural* spline of odd degree 2m-1 (the minimiser of
int (f^(m))^2 through the data).  We restate it here as that natural spline,
built once on the host, and hand the device a piecewise polynomial table
(mh_table).  GCVSPL itself is third-party (opensim-core) and absent from
/root/reference: parity with its exact floating-point solve is unpinned.
"""
from __future__ import annotations

import math

import numpy as np


def gcv_interpolating_ppoly(t: np.ndarray, Y: np.ndarray, degree: int = 3):
    """Natural interpolating spline of odd ``degree`` through (t, Y[:, c]).

    Returns (breaks[nseg+1], coefs[nseg, ncol, degree+1]) with coefficients
    in ascending powers of (time - breaks[s]).
    """
    t = np.asarray(t, float)
    Y = np.asarray(Y, float)
    if Y.ndim == 1:
        Y = Y[:, None]
    order = np.argsort(t, kind="stable")
    t = t[order]
    Y = Y[order]
    keep = np.concatenate([[True], np.diff(t) > 0])
    t, Y = t[keep], Y[keep]
    n, ncol = Y.shape
    if degree % 2 != 1 or degree < 1:
        raise ValueError("GCVSpline degree must be odd")
    if n < 2:
        raise ValueError("need at least two samples")
    deg = min(degree, n - 1 if (n - 1) % 2 == 1 else n - 2)
    deg = max(deg, 1)
    nseg = n - 1
    coefs = np.zeros((nseg, ncol, deg + 1))
    if deg == 1:
        slope = np.diff(Y, axis=0) / np.diff(t)[:, None]
        coefs[:, :, 0] = Y[:-1]
        coefs[:, :, 1] = slope
        return t, coefs
    from scipy.interpolate import make_interp_spline
    m = (deg + 1) // 2
    # natural end conditions: derivatives m..2m-2 vanish at both ends
    bc = [(k, 0.0) for k in range(m, 2 * m - 1)]
    for c in range(ncol):
        spl = make_interp_spline(t, Y[:, c], k=deg, bc_type=(bc, bc))
        for k in range(deg + 1):
            d = spl if k == 0 else spl.derivative(k)
            coefs[:, c, k] = d(t[:-1]) / math.factorial(k)
    return t, coefs


def ppoly_eval(breaks, coefs, time, col):
    """Evaluate one column of a piecewise polynomial table (host helper)."""
    nseg = len(breaks) - 1
    s = np.clip(np.searchsorted(breaks, time, side="right") - 1, 0, nseg - 1)
    dt = time - breaks[s]
    c = coefs[s, col]
    v = np.zeros_like(np.asarray(dt, float))
    for k in range(c.shape[-1] - 1, -1, -1):
        v = v * dt + c[..., k]
    return v


class SimmSpline:
    """Host restatement of OpenSim's SimmSpline (Forsythe-Malcolm-Moler
    cubic with third-derivative end conditions), for tooling and tests."""

    def __init__(self, x, y):
        self.x = np.asarray(x, float)
        self.y = np.asarray(y, float)
        n = len(self.x)
        b = np.zeros(n)
        c = np.zeros(n)
        d = np.zeros(n)
        x, y = self.x, self.y
        if n < 2:
            pass
        elif n < 3:
            t = (y[1] - y[0]) / (x[1] - x[0])
            b[:] = t
        else:
            nm1 = n - 1
            d[0] = x[1] - x[0]
            c[1] = (y[1] - y[0]) / d[0]
            for i in range(1, nm1):
                d[i] = x[i + 1] - x[i]
                b[i] = 2.0 * (d[i - 1] + d[i])
                c[i + 1] = (y[i + 1] - y[i]) / d[i]
                c[i] = c[i + 1] - c[i]
            b[0] = -d[0]
            b[nm1] = -d[n - 2]
            c[0] = 0.0
            c[nm1] = 0.0
            if n > 3:
                d1 = c[2] / (x[3] - x[1]) - c[1] / (x[2] - x[0])
                d2 = c[nm1 - 1] / (x[nm1] - x[n - 3]) - c[n - 3] / (x[nm1 - 1] - x[n - 4])
                c[0] = d1 * d[0] * d[0] / (x[3] - x[0])
                c[nm1] = -(d2 * d[n - 2] * d[n - 2]) / (x[nm1] - x[n - 4])
            for i in range(1, n):
                t = d[i - 1] / b[i - 1]
                b[i] -= t * d[i - 1]
                c[i] -= t * c[i - 1]
            c[nm1] /= b[nm1]
            for j in range(nm1):
                i = nm1 - j - 1
                c[i] = (c[i] - d[i] * c[i + 1]) / b[i]
            b[nm1] = (y[nm1] - y[n - 2]) / d[n - 2] + d[n - 2] * (c[n - 2] + 2.0 * c[nm1])
            for i in range(nm1):
                b[i] = (y[i + 1] - y[i]) / d[i] - d[i] * (c[i + 1] + 2.0 * c[i])
                d[i] = (c[i + 1] - c[i]) / d[i]
                c[i] *= 3.0
            c[nm1] *= 3.0
            d[nm1] = d[n - 2]
        self.b, self.c, self.d = b, c, d

    def __call__(self, t, deriv=0):
        x, y, b, c, d = self.x, self.y, self.b, self.c, self.d
        n = len(x)
        if t < x[0]:
            return [y[0] + (t - x[0]) * b[0], b[0], 0.0][deriv]
        if t > x[-1]:
            return [y[-1] + (t - x[-1]) * b[-1], b[-1], 0.0][deriv]
        k = min(max(np.searchsorted(x, t, side="right") - 1, 0), n - 1)
        dx = t - x[k]
        if deriv == 0:
            return y[k] + dx * (b[k] + dx * (c[k] + dx * d[k]))
        if deriv == 1:
            return b[k] + dx * (2.0 * c[k] + 3.0 * dx * d[k])
        return 2.0 * c[k] + 6.0 * dx * d[k]


def pad_odd(x: np.ndarray, p: int) -> np.ndarray:
    """Signal::Pad (TableUtilities::pad / Storage::pad): p samples at each
    end, reflected about the end sample and negated (odd reflection)."""
    x = np.asarray(x, float)
    n = len(x)
    return np.concatenate([2 * x[0] - x[p:0:-1], x, 2 * x[-1] - x[n - 2:n - 2 - p:-1]])


def lowpass_iir(dt: float, fc: float, sig: np.ndarray) -> np.ndarray:
    """Signal::LowpassIIR: third-order Butterworth (prewarped bilinear
    transform) run forward then backward, the first three outputs of each
    pass set to its inputs."""
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
    return run(run(np.asarray(sig, float))[::-1])[::-1]


def filter_lowpass_table(times, columns: dict, fc: float):
    """TableUtilities::filterLowpass(table, fc, padData=true) (TabOpLowPassFilter):
    pad nrows/2 samples at both ends (times extended by the same odd
    reflection, i.e. uniformly), then LowpassIIR with the sampling interval;
    the padded rows stay in the table."""
    t = np.asarray(times, float)
    p = len(t) // 2
    tp = pad_odd(t, p)
    dt = t[1] - t[0]
    return tp, {k: lowpass_iir(dt, fc, pad_odd(np.asarray(v, float), p)) for k, v in columns.items()}
