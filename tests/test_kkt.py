"""The device KKT module's symbolic block map (mocohip.kkt.block_map) and
its numeric algorithm (restated in numpy, tests/_kkt_ref.py) on CPU, over
real transcription structures evaluated by the oracle: every Jacobian
nonzero lands in exactly one block entry or dense column, the Schur
complement over the block columns is block tridiagonal with exactly the
blocks the map predicts, and block cyclic reduction solves it to rounding."""
import numpy as np
import pytest

import _kkt_ref as K
from mocohip import configs
from mocohip.kkt import block_map
from mocohip.solver import OracleNLP

CASES = {
    "sliding_mass_hs": lambda: configs.sliding_mass(7),
    "double_pendulum_trap": lambda: configs.double_pendulum(6, "trapezoidal"),
    "gait_rigid": lambda: configs.gait10dof18musc(3),
    "gait_inverse": lambda: configs.gait10dof18musc_inverse(4, sparsity="none"),
    "coupled_pendulum": lambda: configs.double_pendulum_coupled(5),
    "coupled_pendulum_implicit": lambda: configs.double_pendulum_coupled(4, dynamics="implicit"),
    "pendulum_path": lambda: configs.pendulum_control_bound(5, "both"),
}


def _setup(name, seed=0):
    st = CASES[name]()
    nlp = OracleNLP(st.problem.create_rep(), st.solver.options())
    rng = np.random.default_rng(seed)
    x = nlp.random_iterate(rng.uniform(-1, 1, nlp.n))
    if nlp.NAR:
        G, NS, NC = nlp.G, nlp.NS, nlp.NC
        x[2:2 + NS * G] = rng.uniform(0.05, 0.5, NS * G)
        x[2 + NS * G:2 + (NS + NC) * G] = rng.uniform(0.05, 0.4, NC * G)
    return nlp, x, rng


@pytest.mark.parametrize("name", sorted(CASES))
def test_block_map_covers_the_jacobian(name):
    nlp, x, rng = _setup(name)
    bm = block_map(nlp)
    src = np.concatenate([bm.a_src[bm.a_src >= 0], bm.d_src[bm.d_src >= 0]])
    assert np.array_equal(np.sort(src), np.arange(nlp.nnz))       # every nonzero exactly once
    vals = nlp.eval_jac_g(x)
    rs = rng.uniform(0.5, 2.0, nlp.m)
    A, Jd = K.gather(bm, vals, rs)
    ir, jc = nlp.jac_structure()
    J = np.zeros((nlp.m, nlp.n))
    np.add.at(J, (ir, jc), vals)
    J *= rs[:, None]
    R = np.zeros_like(J)
    for b in range(bm.nb):
        for i in np.where(bm.rowmap[b] >= 0)[0]:
            cc = bm.colmap[b] >= 0
            R[bm.rowmap[b, i], bm.colmap[b, cc]] += A[b, i, cc]
    R[:, bm.dcols] += Jd
    assert np.array_equal(R, J)
    # t0 / tf are always dense (every defect row reads them through h)
    assert {0, 1} <= set(bm.dcols.tolist())
    # the shared grid point's columns are the same global columns
    P = bm.nshare
    for b in range(bm.nb - 1):
        assert np.array_equal(bm.colmap[b, bm.rshare[b]:bm.rshare[b] + P],
                              bm.colmap[b + 1, bm.lshare[b + 1]:bm.lshare[b + 1] + P])


@pytest.mark.parametrize("name", sorted(CASES))
def test_block_cyclic_reduction_solves_the_schur_complement(name):
    nlp, x, rng = _setup(name, 1)
    bm = block_map(nlp)
    vals = nlp.eval_jac_g(x)
    rs = rng.uniform(0.5, 2.0, nlp.m)
    w = rng.uniform(0.1, 10.0, nlp.n)
    w[bm.dcols] = 0.0
    dc = rng.uniform(1e-8, 1e-2, nlp.m)
    S, _ = K.dense_schur(bm, vals, rs, w, dc)
    A, _ = K.gather(bm, vals, rs)
    D, E = K.schur_blocks(bm, A, w, dc)
    # S is block tridiagonal and its blocks are D / E
    blk = -np.ones(nlp.m, int)
    loc = -np.ones(nlp.m, int)
    for b in range(bm.nb):
        ok = bm.rowmap[b] >= 0
        blk[bm.rowmap[b, ok]] = b
        loc[bm.rowmap[b, ok]] = np.where(ok)[0]
    far = np.abs(blk[:, None] - blk[None, :]) > 1
    assert not S[far].any()
    for b in range(bm.nb):
        rr = bm.rowmap[b][bm.rowmap[b] >= 0]
        np.testing.assert_allclose(D[b][np.ix_(loc[rr], loc[rr])], S[np.ix_(rr, rr)], rtol=1e-13, atol=1e-13)
        if b + 1 < bm.nb:
            r2 = bm.rowmap[b + 1][bm.rowmap[b + 1] >= 0]
            np.testing.assert_allclose(E[b][np.ix_(loc[r2], loc[rr])], S[np.ix_(r2, rr)],
                                       rtol=1e-13, atol=1e-13)
    Lf, U, V, levels = K.cr_factor(D, E)
    B = rng.standard_normal((nlp.m, 3))
    X = K.from_blocks(bm, K.cr_solve(Lf, U, V, levels, K.to_blocks(bm, B)))
    Xd = np.linalg.solve(S, B)
    assert np.abs(X - Xd).max() <= 1e-8 * np.abs(Xd).max()
