"""The host optimizer's KKT linear algebra on the device (include/mocohip.h
mh_kkt_*), next to the Jacobian it factors.

Ipopt solves each Newton system of the collocation NLP with MUMPS on the
host (MocoCasADiSolver -> Ipopt 3.12.8, IpPDFullSpaceSolver); the interior-
point restatement here (mocohip.ipm) eliminates the bound multipliers and
slacks and solves through the Schur complement

    S = R J W J^T R + diag(dc),   W = diag(1 / D_x) on the block columns,

whose factorization, on the host, dominated every solve (SuperLU / banded
LAPACK over J crossing PCIe each iteration: 86 % of the wall-clock).  The
collocation Jacobian has a fixed block structure that this module finds once
(``block_map``) and the device exploits on every factorization:

  * rows are contiguous per mesh interval (CasOCTranscription.h:219-313:
    flattenConstraints) -- one BLOCK per interval, plus a head block for the
    endpoint-constraint rows and a tail block for the final mesh point's
    rows when the problem has them;
  * a block's rows read only its own grid points' variables (HS: the
    interval's three points; trapezoidal: two) and its own slacks, so every
    block's Jacobian rows are a small dense matrix A_b (r x c) over LOCAL
    columns, and consecutive blocks share exactly one grid point's columns;
  * columns read by rows outside that pattern -- the initial / final time
    (every defect row reads them through h = t_f - t_0) and anything an
    endpoint constraint reads beyond grid point 0 -- are DENSE columns, kept
    out of S and put back by the optimizer with Sherman-Morrison-Woodbury
    (as the host path does).

So S is block tridiagonal: D_b = A_b W_b A_b^T + diag(dc_b) (a dense FP64
GEMM per block) and E_b = A_{b+1}[:, shared] W A_b[:, shared]^T, factored on
the device by block cyclic reduction (log2(blocks) levels of batched dense
Cholesky / triangular solves / GEMMs, every block of a level in parallel;
csrc/kkt.hip) and solved the same way.  The host keeps the optimizer's
logic and its vectors; J never leaves the device.
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass

import numpy as np


@dataclass
class BlockMap:
    """The block decomposition of one transcription's Jacobian structure.

    nb blocks of at most ``r`` rows and ``c`` local columns (padded);
    ``a_src[b, i, j]`` = index of the Jacobian nonzero that is entry (i, j) of
    A_b, -1 for a structural zero or padding; ``rowmap[b, i]`` /
    ``colmap[b, j]`` = the global row / column (-1: padding);
    ``lshare[b]`` / ``rshare[b]`` = local offset of the columns block b
    shares with block b - 1 / b + 1, ``nshare`` their count (one grid
    point's variables); ``dcols`` = the dense columns, ``d_src[i, d]`` = the
    nonzero feeding row i of dense column d (-1: zero); ``col2[j]`` = the (up
    to two) flat A positions b * c + local column of global column j."""
    nb: int
    r: int
    c: int
    nshare: int
    m: int
    n: int
    nnz: int
    a_src: np.ndarray
    rowmap: np.ndarray
    colmap: np.ndarray
    lshare: np.ndarray
    rshare: np.ndarray
    dcols: np.ndarray
    d_src: np.ndarray
    col2: np.ndarray

    @property
    def nd(self) -> int:
        return len(self.dcols)


def _point_columns(nlp, p: int) -> np.ndarray:
    """Global x columns of grid point p's per-point variables (states,
    controls, multipliers, derivatives: the CasOC layout,
    CasOCIterate.h:27-44, include/mocohip.h)."""
    G, NS, NC, NM, NDV, NSL = nlp.G, nlp.NS, nlp.NC, nlp.NM, nlp.NDV, nlp.NSL
    N = nlp.opts.num_mesh_intervals
    s = 2 + p * NS + np.arange(NS)
    u = 2 + G * NS + p * NC + np.arange(NC)
    mu = 2 + G * (NS + NC) + p * NM + np.arange(NM)
    d = 2 + G * (NS + NC + NM) + N * NSL + p * NDV + np.arange(NDV)
    return np.concatenate([s, u, mu, d]).astype(np.int64)


def block_map(nlp) -> BlockMap:
    """Symbolic analysis of ``nlp``'s Jacobian structure (an unsharded
    context: rows 0..m, nonzeros 0..nnz).  Raises ValueError when the rows
    do not have the per-interval layout."""
    n, m, nnz = int(nlp.n), int(nlp.m), int(nlp.nnz)
    if nlp.row_begin != 0 or nlp.row_end != m:
        raise ValueError("block_map needs an unsharded context")
    N = int(nlp.opts.num_mesh_intervals)
    G = int(nlp.G)
    if G == 2 * N + 1:
        q, step = 3, 2          # Hermite-Simpson: points 2i, 2i+1, 2i+2
    elif G == N + 1:
        q, step = 2, 1          # trapezoidal: points i, i+1
    else:
        raise ValueError(f"unexpected grid: G={G}, N={N}")
    NSL = nlp.NSL
    nep = int(nlp.NEP)
    ntail = int(nlp.tail_rows)
    body = m - nep - ntail
    if body <= 0 or body % N:
        raise ValueError("rows are not contiguous per mesh interval")
    rpi = body // N
    P = len(_point_columns(nlp, 0))
    # blocks: (first row, row count, grid points, slack interval or -1)
    blocks = []
    if nep:
        blocks.append((0, nep, [0], -1))
    for i in range(N):
        blocks.append((nep + i * rpi, rpi, [step * i + k for k in range(q)], i))
    if ntail:
        blocks.append((nep + N * rpi, ntail, [G - 1], -1))
    nb = len(blocks)
    r = max(b[1] for b in blocks)
    c = max(len(b[2]) * P + (NSL if b[3] >= 0 else 0) for b in blocks)
    slack0 = 2 + G * (nlp.NS + nlp.NC + nlp.NM)
    # per global column: (grid point, variable) or (slack interval, l)
    col_point = -np.ones(n, np.int64)
    col_var = -np.ones(n, np.int64)
    for p in range(G):
        cols = _point_columns(nlp, p)
        col_point[cols] = p
        col_var[cols] = np.arange(P)
    col_slk = -np.ones(n, np.int64)
    if NSL:
        for i in range(N):
            cols = slack0 + i * NSL + np.arange(NSL)
            col_slk[cols] = i
            col_var[cols] = np.arange(NSL)
    row_block = np.empty(m, np.int64)
    row_local = np.empty(m, np.int64)
    first_point = np.empty(nb, np.int64)
    npts = np.empty(nb, np.int64)
    slk = np.empty(nb, np.int64)
    rowmap = -np.ones((nb, r), np.int32)
    for b, (r0, nr, pts, si) in enumerate(blocks):
        row_block[r0:r0 + nr] = b
        row_local[r0:r0 + nr] = np.arange(nr)
        rowmap[b, :nr] = np.arange(r0, r0 + nr)
        first_point[b] = pts[0]
        npts[b] = len(pts)
        slk[b] = si
    ir, jc = nlp.jac_structure()
    ir = np.asarray(ir[:nnz], np.int64)
    jc = np.asarray(jc[:nnz], np.int64)
    rb = row_block[ir]
    pp = col_point[jc]
    rel = pp - first_point[rb]
    local = np.where((pp >= 0) & (rel >= 0) & (rel < npts[rb]), rel * P + col_var[jc], -1)
    sl = col_slk[jc]
    local = np.where((sl >= 0) & (sl == slk[rb]), npts[rb] * P + col_var[jc], local)
    dense = np.zeros(n, bool)
    dense[jc[local < 0]] = True
    dcols = np.where(dense)[0].astype(np.int32)
    inblock = ~dense[jc]
    a_src = -np.ones((nb, r, c), np.int32)
    k = np.where(inblock)[0]
    a_src[rb[k], row_local[ir[k]], local[k]] = k
    dpos = -np.ones(n, np.int64)
    dpos[dcols] = np.arange(len(dcols))
    d_src = -np.ones((m, max(len(dcols), 1)), np.int32)
    k = np.where(~inblock)[0]
    d_src[ir[k], dpos[jc[k]]] = k
    d_src = d_src[:, :len(dcols)]
    colmap = -np.ones((nb, c), np.int32)
    col2 = -np.ones((n, 2), np.int32)
    for b, (r0, nr, pts, si) in enumerate(blocks):
        cols = np.concatenate([_point_columns(nlp, p) for p in pts] +
                              ([slack0 + si * NSL + np.arange(NSL)] if si >= 0 and NSL else []))
        colmap[b, :len(cols)] = cols
        pos = b * c + np.arange(len(cols))
        first = col2[cols, 0] < 0
        col2[cols[first], 0] = pos[first]
        col2[cols[~first], 1] = pos[~first]
    col2[dcols] = -1            # dense columns: products through the dense part only
    lshare = np.zeros(nb, np.int32)
    rshare = np.zeros(nb, np.int32)
    for b in range(nb):
        rshare[b] = (npts[b] - 1) * P       # the block's last grid point
    return BlockMap(nb, r, c, P, m, n, nnz, a_src, rowmap, colmap, lshare, rshare, dcols, d_src, col2)


class mh_kkt_layout(C.Structure):
    """include/mocohip.h mh_kkt_layout."""
    _fields_ = [("nblocks", C.c_int32), ("r", C.c_int32), ("c", C.c_int32), ("nd", C.c_int32),
                ("nshare", C.c_int32), ("reserved", C.c_int32),
                ("m", C.c_int64), ("n", C.c_int64), ("nnz", C.c_int64),
                ("a_src", C.POINTER(C.c_int32)), ("rowmap", C.POINTER(C.c_int32)),
                ("colmap", C.POINTER(C.c_int32)), ("lshare", C.POINTER(C.c_int32)),
                ("rshare", C.POINTER(C.c_int32)), ("dcols", C.POINTER(C.c_int32)),
                ("d_src", C.POINTER(C.c_int32)), ("col2", C.POINTER(C.c_int32))]


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int32))


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class DeviceKKT:
    """mh_kkt over a HipNLP context: the Jacobian evaluated into device
    memory, gathered into the blocks A_b (row-scaled), the Schur complement
    formed and factored by block cyclic reduction, solves and products with
    J -- all on the context's device and stream.  Vectors cross the bus;
    J does not."""

    def __init__(self, nlp, bm: BlockMap | None = None):
        self.nlp = nlp
        self.lib = nlp.lib
        self.bm = bm or block_map(nlp)
        b = self.bm
        self._keep = [np.ascontiguousarray(a, np.int32) for a in
                      (b.a_src, b.rowmap, b.colmap, b.lshare, b.rshare, b.dcols,
                       b.d_src if b.nd else np.zeros(1, np.int32), b.col2)]
        L = mh_kkt_layout(b.nb, b.r, b.c, b.nd, b.nshare, 0, b.m, b.n, b.nnz, *[_ip(a) for a in self._keep])
        self.h = C.c_void_p()
        self._check(self.lib.mh_kkt_create(nlp.ctx, C.byref(L), C.byref(self.h)))
        self.m, self.n, self.nd = b.m, b.n, b.nd
        self.stats = {}          # op -> [calls, seconds, columns] (host wall clock per C-ABI call)

    def _tick(self, op, t0, k=1):
        s = self.stats.setdefault(op, [0, 0.0, 0])
        s[0] += 1
        s[1] += time.perf_counter() - t0
        s[2] += k

    def _check(self, rc):
        if rc:
            raise RuntimeError(f"mh_kkt: error {rc}: {self.lib.mh_last_error().decode()}")

    def set_row_scale(self, rs):
        rs = np.ascontiguousarray(rs, float)
        assert rs.shape == (self.m,)
        self._check(self.lib.mh_kkt_set_row_scale(self.h, _dp(rs)))

    def eval_jacobian(self, x):
        """J(x) evaluated on the device (the context's eval_jac_g kernels)
        into the module's own buffer and gathered into the blocks."""
        x = np.ascontiguousarray(x, float)
        t0 = time.perf_counter()
        self._check(self.lib.mh_kkt_eval_jacobian(self.h, _dp(x)))
        self._tick("eval_jacobian", t0)

    def dense_columns(self):
        """(global column indices, row-scaled values m x nd)."""
        out = np.empty((self.m, max(self.nd, 1)))
        self._check(self.lib.mh_kkt_get_dense(self.h, _dp(out)))
        return self.bm.dcols.astype(np.int64), out[:, :self.nd]

    def values(self):
        """The raw Jacobian values of the last eval_jacobian (host copy)."""
        v = np.empty(max(self.bm.nnz, 1))
        self._check(self.lib.mh_kkt_get_values(self.h, _dp(v)))
        return v[:self.bm.nnz]

    def factor(self, w, dc) -> bool:
        """S = R J W J^T R + diag(dc) over the block columns (w: n weights,
        0 for dense / fixed columns); False when S is not numerically positive
        definite."""
        w = np.ascontiguousarray(w, float)
        dc = np.ascontiguousarray(dc, float)
        ok = C.c_int32()
        t0 = time.perf_counter()
        self._check(self.lib.mh_kkt_factor(self.h, _dp(w), _dp(dc), C.byref(ok)))
        self._tick("factor", t0)
        return bool(ok.value)

    def _k(self, a, rows):
        a = np.ascontiguousarray(a, float)
        k = 1 if a.ndim == 1 else a.shape[1]
        assert a.shape[0] == rows
        return a, k

    def solve(self, b):
        """S^-1 b (b: m or m x k)."""
        b, k = self._k(b, self.m)
        out = np.empty_like(b)
        t0 = time.perf_counter()
        self._check(self.lib.mh_kkt_solve(self.h, k, _dp(b), _dp(out)))
        self._tick("solve", t0, k)
        return out

    def jmul(self, v):
        """R J v (v: n or n x k; every column, dense ones included)."""
        v, k = self._k(v, self.n)
        out = np.empty((self.m,) + v.shape[1:])
        t0 = time.perf_counter()
        self._check(self.lib.mh_kkt_jmul(self.h, k, _dp(v), _dp(out)))
        self._tick("jmul", t0, k)
        return out

    def jtmul(self, y):
        """J^T R y (y: m or m x k)."""
        y, k = self._k(y, self.m)
        out = np.empty((self.n,) + y.shape[1:])
        t0 = time.perf_counter()
        self._check(self.lib.mh_kkt_jtmul(self.h, k, _dp(y), _dp(out)))
        self._tick("jtmul", t0, k)
        return out

    def warm(self, x, widths=tuple(range(1, 13))):
        """One-time setup of the module's device work at iterate ``x``: the
        first launch of each kernel (code objects load then) and the HIP
        graphs of the factorization and of each solve width (captured on
        first use) -- a Jacobian, a factorization of J J^T + I and solves of
        ``widths`` (plus the dense columns' width) right-hand sides, results
        discarded; the per-op statistics are reset afterwards."""
        self.eval_jacobian(x)
        w = np.ones(self.n)
        w[self.bm.dcols] = 0.0
        if self.factor(w, np.ones(self.m)):
            for k in sorted(set(widths) | ({self.nd} if self.nd else set())):
                self.solve(np.ones(self.m) if k == 1 else np.ones((self.m, k)))
        self.jmul(np.zeros(self.n))
        self.jtmul(np.zeros(self.m))
        self.stats.clear()

    def close(self):
        if self.h:
            self.lib.mh_kkt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedDeviceKKT(DeviceKKT):
    """DeviceKKT on rank 0 of a mocohip.distributed.ShardedNLP: ONE NLP
    sharded by mesh interval over the ranks, its Newton systems factored on
    rank 0's GPU over the WHOLE Jacobian (the slices
    reassembled on the GPU that feeds the optimizer).  The module is created
    over rank 0's shard context with the whole NLP's block map; its Jacobian
    buffer is a torch tensor bound to it (mh_kkt_bind_values), so that the
    other ranks' slices can be received straight into their offsets -- RCCL
    point to point over xGMI (transport "device") or through host memory
    (transport "host", gloo) -- and mh_kkt_assemble then gathers the blocks.
    Everything else (factor, solve, products with J) is the module's own
    work on rank 0's GPU, as for an unsharded context."""

    def __init__(self, snlp):
        torch = snlp.torch
        self.snlp = snlp
        shard = snlp.shard
        # the shard context's own GPU (mh_options.device), which its kernels
        # write the Jacobian slice on, for both transports
        dev = torch.device("cuda", int(shard.opts.device))
        if snlp.transport == "device" and snlp.device != dev:
            raise ValueError(f"ShardedNLP device {snlp.device} is not the shard context's {dev}")
        self.dev = dev
        # the shard context's kernels, the received slices and the module's
        # kernels ordered on one dedicated stream (not torch's default one,
        # handle 0, which mh_set_stream reads as the context's own stream)
        self.stream = torch.cuda.Stream(device=dev)
        shard.set_stream(self.stream.cuda_stream)
        super().__init__(shard, block_map(snlp))
        self.vals = torch.zeros(max(1, self.bm.nnz), dtype=torch.float64, device=dev)
        self._check(self.lib.mh_kkt_bind_values(self.h, C.c_void_p(self.vals.data_ptr())))
        b, e = C.c_int64(), C.c_int64()
        self._check(self.lib.mh_kkt_shard_range(self.h, C.byref(b), C.byref(e)))
        assert (b.value, e.value) == snlp.ranges[0][2:4]

    def eval_jacobian(self, x):
        """J(x) of the whole NLP in rank 0's HBM: the request to every rank,
        rank 0's slice by its own kernels, the others' slices received into
        their offsets of the bound buffer, then the blocks gathered."""
        from .distributed import OP_JAC_DEV
        snlp, torch = self.snlp, self.snlp.torch
        x = np.ascontiguousarray(x, float)
        t0 = time.perf_counter()
        snlp._request(OP_JAC_DEV, x)
        with torch.cuda.stream(self.stream):
            self._check(self.lib.mh_kkt_eval_jacobian(self.h, _dp(x)))
            # the other ranks' slices: one grouped batch of receives (the
            # peers' transfers run concurrently, each over its own link)
            ops, staged = [], []
            for r in range(1, snlp.world):
                b, e = snlp.ranges[r][2], snlp.ranges[r][3]
                if e <= b:
                    continue
                if snlp.transport == "device":
                    ops.append(snlp.dist.P2POp(snlp.dist.irecv, self.vals[b:e], r))
                else:
                    buf = torch.empty(e - b, dtype=torch.float64)
                    ops.append(snlp.dist.P2POp(snlp.dist.irecv, buf, r))
                    staged.append((b, e, buf))
            for q in (snlp.dist.batch_isend_irecv(ops) if ops else []):
                q.wait()
            for b, e, buf in staged:
                self.vals[b:e].copy_(buf)
            self._check(self.lib.mh_kkt_assemble(self.h))
        self._tick("eval_jacobian", t0)
