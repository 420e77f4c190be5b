"""TEST INFRASTRUCTURE: a numpy restatement of the device KKT module's
numeric algorithm (csrc/kkt.hip, include/mocohip.h mh_kkt_*) over the block
map of mocohip.kkt.block_map -- the gather of J into the blocks A_b, the
block-tridiagonal Schur complement, its block cyclic reduction and the
solves -- so the device kernels are checked against the same algorithm and
the algorithm against a dense solve."""
import numpy as np


def gather(bm, vals, row_scale):
    """(A [nb, r, c], Jd [m, nd]) from the raw Jacobian values."""
    v = np.concatenate([np.asarray(vals, float), [0.0]])
    A = v[bm.a_src]                                   # -1 -> the appended 0
    rs = np.concatenate([np.asarray(row_scale, float), [0.0]])
    A = A * rs[bm.rowmap][:, :, None]
    Jd = v[bm.d_src] * np.asarray(row_scale, float)[:, None] if bm.nd else np.zeros((bm.m, 0))
    return A, Jd


def schur_blocks(bm, A, w, dc):
    """D [nb, r, r] (padding rows: 1 on the diagonal), E [nb - 1, r, r]."""
    wl = np.concatenate([np.asarray(w, float), [0.0]])[bm.colmap]        # [nb, c]
    dcl = np.concatenate([np.asarray(dc, float), [1.0]])[bm.rowmap]      # padding rows -> 1
    D = np.einsum("bik,bk,bjk->bij", A, wl, A)
    D[:, np.arange(bm.r), np.arange(bm.r)] += dcl
    P = bm.nshare
    E = np.zeros((max(bm.nb - 1, 0), bm.r, bm.r))
    for b in range(bm.nb - 1):
        lo, ro = bm.lshare[b + 1], bm.rshare[b]
        E[b] = (A[b + 1][:, lo:lo + P] * wl[b][ro:ro + P]) @ A[b][:, ro:ro + P].T
    return D, E


def cr_factor(D, E):
    """Block cyclic reduction of the SPD block-tridiagonal matrix with
    diagonal blocks D and sub-diagonal blocks E (E[b] = S[b+1, b]).  Returns
    the per-block factors (L, U, V) and the level schedule: at level l the
    active blocks are every 2^l-th, the odd ones among them are eliminated:
    L_i L_i^T = D_i, U_i = L_i^-1 S[i, left], V_i = L_i^-1 S[i, right]; the
    even ones are updated D_j -= U^T U + V^T V and coupled by -V^T U."""
    D = D.copy()
    E = E.copy()
    nb = len(D)
    L = np.zeros_like(D)
    U = np.zeros_like(D)
    V = np.zeros_like(D)
    levels = []
    active = list(range(nb))
    while True:
        if len(active) == 1:
            i = active[0]
            L[i] = np.linalg.cholesky(D[i])
            levels.append(([i], {i: (None, None)}))
            break
        odd = active[1::2]
        nbr = {}
        for k in range(1, len(active), 2):
            i = active[k]
            left = active[k - 1]
            right = active[k + 1] if k + 1 < len(active) else None
            nbr[i] = (left, right)
            L[i] = np.linalg.cholesky(D[i])
            U[i] = np.linalg.solve(L[i], E[left])             # S[i, left] = E[left]
            if right is not None:
                V[i] = np.linalg.solve(L[i], E[i].T)          # S[i, right] = E[i]^T
        for k in range(0, len(active), 2):
            j = active[k]
            if k - 1 >= 0:
                i = active[k - 1]
                D[j] -= V[i].T @ V[i]
            if k + 1 < len(active):
                i = active[k + 1]
                D[j] -= U[i].T @ U[i]
                if k + 2 < len(active):
                    E[j] = -V[i].T @ U[i]                    # new S[j2, j]
        levels.append((odd, nbr))
        active = active[0::2]
    return L, U, V, levels


def cr_solve(L, U, V, levels, B):
    """S^-1 B, B [nb, r, k]."""
    X = B.copy()
    for odd, nbr in levels:                                  # forward
        for i in odd:
            X[i] = np.linalg.solve(L[i], X[i])
            left, right = nbr[i]
            if left is not None:
                X[left] -= U[i].T @ X[i]
            if right is not None:
                X[right] -= V[i].T @ X[i]
    for odd, nbr in reversed(levels):                        # backward
        for i in odd:
            left, right = nbr[i]
            y = X[i].copy()
            if left is not None:
                y -= U[i] @ X[left]
            if right is not None:
                y -= V[i] @ X[right]
            X[i] = np.linalg.solve(L[i].T, y)
    return X


def to_blocks(bm, b):
    """[m, k] -> [nb, r, k] (padding rows 0)."""
    b = np.asarray(b, float).reshape(bm.m, -1)
    ext = np.concatenate([b, np.zeros((1, b.shape[1]))])
    return ext[bm.rowmap]


def from_blocks(bm, X):
    out = np.zeros((bm.m, X.shape[2]))
    msk = bm.rowmap >= 0
    out[bm.rowmap[msk]] = X[msk]
    return out


def dense_schur(bm, vals, row_scale, w, dc):
    """S over the block columns, assembled densely from the values (check)."""
    import scipy.sparse as sp
    A, _ = gather(bm, vals, row_scale)
    J = np.zeros((bm.m, bm.n))
    for b in range(bm.nb):
        rr = bm.rowmap[b]
        cc = bm.colmap[b]
        for i in np.where(rr >= 0)[0]:
            for j in np.where(cc >= 0)[0]:
                if bm.a_src[b, i, j] >= 0:
                    J[rr[i], cc[j]] = A[b, i, j]
    del sp
    return J @ np.diag(w) @ J.T + np.diag(dc), J
