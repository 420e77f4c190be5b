"""Finite-difference lane inputs in the layout of mh_debug_jacobian_lanes
(include/mocohip.h), rebuilt on the host with the same IEEE operations the
lanes use (test helper)."""
import numpy as np

from mocohip import abi


def grid(nlp):
    N = nlp.opts.num_mesh_intervals
    mesh = np.arange(N + 1) / N
    if nlp.opts.transcription == abi.MH_HERMITE_SIMPSON:
        return np.array([mesh[k // 2] if k % 2 == 0 else 0.5 * (mesh[k // 2] + mesh[k // 2 + 1])
                         for k in range(nlp.G)])
    return mesh


def point_inputs(nlp, x):
    """[G, NI]: each grid point's inputs (states, controls, derivatives,
    multipliers, slacks)."""
    return nlp.point_inputs(x)


def lane_steps(nlp):
    """Per lane r: (direction d, signed step) -- lane d < ND moves direction
    d by +h (backward: -h); central adds the -h lanes ND..2ND-1; the last
    lane is unperturbed (d = -1)."""
    h = nlp.opts.fd_step if nlp.opts.fd_step > 0 else 1e-8
    fd = nlp.opts.finite_difference_scheme
    ND = 2 + nlp.NI + nlp.NPAR
    S = 2 * ND + 1 if fd == abi.MH_FD_CENTRAL else ND + 1
    out = []
    for r in range(S - 1):
        step = -h if fd == abi.MH_FD_BACKWARD else h
        d = r
        if fd == abi.MH_FD_CENTRAL and r >= ND:
            d, step = r - ND, -h
        out.append((d, step))
    return out + [(-1, 0.0)]


def lane_rows(nlp, x, times):
    """[G, S, 1 + NI] DAE inputs [time, inputs] of every lane: lane d < ND
    moves direction d (0 = t0 seed 1 - g, 1 = tf seed g, 2 + j = input j,
    2 + NI + p = MocoParameter p, which moves the model, not the inputs) by
    +h (backward: -h); central adds the -h lanes ND..2ND-1; the last lane is
    unperturbed."""
    h = nlp.opts.fd_step if nlp.opts.fd_step > 0 else 1e-8
    fd = nlp.opts.finite_difference_scheme
    P = point_inputs(nlp, x)
    g = grid(nlp)
    G, NI = P.shape
    ND = 2 + NI + nlp.NPAR
    S = 2 * ND + 1 if fd == abi.MH_FD_CENTRAL else ND + 1
    rows = np.empty((G, S, 1 + NI))
    rows[:, :, 0] = times[:, None]
    rows[:, :, 1:] = P[:, None, :]
    for r in range(S - 1):
        step = -h if fd == abi.MH_FD_BACKWARD else h
        d = r
        if fd == abi.MH_FD_CENTRAL and r >= ND:
            d, step = r - ND, -h
        if d == 0:
            rows[:, r, 0] = times + step * (1.0 - g)
        elif d == 1:
            rows[:, r, 0] = times + step * g
        elif d < 2 + NI:
            rows[:, r, 1 + d - 2] = P[:, d - 2] + step
    return rows


def oracle_lanes(ref, x, times):
    """Y[G, NO, S] evaluated by the oracle's DAE at exactly the lane inputs
    (with MocoParameters: every lane on the model with x's parameters
    applied, a parameter lane's parameter moved by its step)."""
    rows = lane_rows(ref, x, times)
    G, S, W = rows.shape
    if not ref.NPAR:
        out = ref.eval_dae(rows.reshape(G * S, W))
        return out.reshape(G, S, ref.NO).transpose(0, 2, 1).copy()
    Y = np.empty((G, S, ref.NO))
    pdir = 2 + ref.NI
    for r, (d, step) in enumerate(lane_steps(ref)):
        moved = d - pdir if d >= pdir else -1
        Y[:, r] = ref.eval_dae_params(np.ascontiguousarray(rows[:, r]), x, moved, step if moved >= 0 else 0.0)
    return Y.transpose(0, 2, 1).copy()


def oracle_times(nlp, x):
    return (x[1] - x[0]) * grid(nlp) + x[0]
