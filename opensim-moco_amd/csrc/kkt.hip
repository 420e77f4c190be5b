// kkt.hip — the host optimizer's Newton-system linear algebra on the device
// (include/mocohip.h mh_kkt_*), next to the Jacobian it factors.
//
// Ipopt (MocoCasADiSolver -> Ipopt 3.12.8) factors each Newton system with
// MUMPS on the host.  The interior-point restatement here (mocohip/ipm.py)
// solves through the Schur complement S = R J W J^T R + diag(dc) of the
// bound-multiplier-eliminated system.  A collocation Jacobian's rows are
// contiguous per mesh interval and read only their interval's grid points
// (CasOCTranscription.h:219-313), so with the host's symbolic block map
// (mocohip/kkt.py block_map: one block per interval, a head block for the
// endpoint rows, a tail block for the final point's rows, dense columns t0 /
// tf kept out) S is block tridiagonal:
//
//   D_b = A_b W_b A_b^T + diag(dc_b),  E_b = A_{b+1}[:, shared] W A_b[:, shared]^T
//
// with A_b the block's rows over its local columns (a small dense matrix).
// Everything below is batched over blocks, one workgroup (or a few) per
// block, FP64:
//   k_kkt_gather   J's values (the context's own eval_jac_g kernels wrote
//                  them into this module's buffer) -> A_b, row-scaled, and
//                  the dense columns Jd;
//   k_kkt_gemm     C = alpha P diag(w) Q^T + beta C over strided operands,
//                  64 x 64 output tiles staged through LDS: forms D_b and E_b
//                  and every update of the cyclic reduction;
//   k_kkt_potrf    in-place Cholesky of one block per workgroup (in LDS when
//                  it fits: r <= 143);
//   k_kkt_trsm     L^-1 B / L^-T B, blocked by 16 rows in LDS (diagonal blocks one lane per column, the rest by the workgroup);
// and block cyclic reduction over them: at level l the active blocks are
// every 2^l-th, the odd ones are eliminated in parallel (L_i L_i^T = D_i,
// U_i = L_i^-1 S[i, left], V_i = L_i^-1 S[i, right]) and the even ones
// updated (D_j -= V^T V + U^T U, new coupling -V^T U): ceil(log2 blocks)
// levels of a handful of launches each instead of a sequential banded
// factorization.  tests/_kkt_ref.py restates the same algorithm in numpy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <functional>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mocohip_kkt.h"

// the context interface of mocohip.hip this module uses
struct mh_ctx;
int mh_internal_error(int code, const char* msg);
hipStream_t mh_internal_stream(const mh_ctx* c);
int mh_internal_device(const mh_ctx* c);
int mh_internal_shape(const mh_ctx* c, int64_t* n, int64_t* m, int64_t* nnz, int* unsharded);
int mh_internal_jac_device(mh_ctx* c, const double* x_dev, double* v_dev);
int mh_internal_shard(const mh_ctx* c, int64_t* m_full, int64_t* nnz_full, int64_t* nnz_begin, int64_t* nnz_end);

#define KCHK(expr)                                                                       \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess)                                                            \
            return mh_internal_error(MH_ERR_HIP, (std::string(#expr " failed: ") +       \
                                                  hipGetErrorString(e_)).c_str());       \
    } while (0)

namespace {

constexpr int KMAX = 32;              // right-hand sides per solve pass
constexpr int INV_RMAX_SK = 160;      // the skinny products' largest K (= INV_RMAX)
constexpr int LDS_MAX = 160 * 1024;   // gfx950 LDS per workgroup

// C = alpha (P diag(w) Q^T + P2 Q2^T) + beta C (P2 null: the first product only)
struct KTask { const double* P; const double* Q; const double* w; double* C; const double* P2; const double* Q2; };
struct KTri { const double* L; const double* B; double* X; };

// ------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------
// n doubles global -> LDS with U loads in flight per thread before the
// first store (a plain loop waits for each load's round trip in turn)
template <int U>
__device__ __forceinline__ void stage(double* __restrict__ dst, const double* __restrict__ src, int n) {
    for (int b = 0; b < n; b += U * (int)blockDim.x) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * (int)blockDim.x + (int)threadIdx.x;
            v[u] = src[i < n ? i : n - 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * (int)blockDim.x + (int)threadIdx.x;
            if (i < n) dst[i] = v[u];
        }
    }
}

__global__ void k_kkt_gather(int64_t na, int c, const int32_t* __restrict__ src, const int32_t* __restrict__ rowmap,
                             const double* __restrict__ vals, const double* __restrict__ rs,
                             double* __restrict__ A) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= na) return;
    const int s = src[e];
    double v = 0.0;
    if (s >= 0) {
        const int row = rowmap[e / c];
        v = vals[s] * rs[row];
    }
    A[e] = v;
}

__global__ void k_kkt_gather_dense(int64_t nj, int nd, const int32_t* __restrict__ src,
                                   const double* __restrict__ vals, const double* __restrict__ rs,
                                   double* __restrict__ Jd) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nj) return;
    const int s = src[e];
    Jd[e] = s >= 0 ? vals[s] * rs[e / nd] : 0.0;
}

// local weights wl[b][j] = w[colmap] (0 on padding), local diagonal shifts
// dcl[b][i] = dc[rowmap] (1 on padding rows: S stays positive definite and
// their unknowns stay 0)
__global__ void k_kkt_local(int nbc, int nbr, const int32_t* __restrict__ colmap, const int32_t* __restrict__ rowmap,
                            const double* __restrict__ w, const double* __restrict__ dc,
                            double* __restrict__ wl, double* __restrict__ dcl) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nbc) {
        const int j = colmap[e];
        wl[e] = j >= 0 ? w[j] : 0.0;
    }
    if (e < nbr) {
        const int i = rowmap[e];
        dcl[e] = i >= 0 ? dc[i] : 1.0;
    }
}

__global__ void k_kkt_add_diag(int r, const double* __restrict__ dcl, double* __restrict__ D) {
    const int b = blockIdx.x;
    for (int i = threadIdx.x; i < r; i += blockDim.x) D[((int64_t)b * r + i) * r + i] += dcl[(int64_t)b * r + i];
}

// C = alpha * P diag(w) Q^T + beta * C for one task per blockIdx.z, one 64 x
// 64 output tile per workgroup; P(i, k) = P[i psi + k psk], Q(j, k) =
// Q[j qsi + k qsk], C(i, j) = C[i ldc + j].  The tile's products run on the
// FP64 matrix cores (a fixed k order per output: deterministic); the
// operands stream through LDS in 32-deep K tiles.
__global__ __launch_bounds__(256) void k_kkt_gemm(const KTask* __restrict__ tasks, int M, int N, int K,
                                                  int psi, int psk, int qsi, int qsk, int ldc,
                                                  double alpha, double beta) {
    constexpr int TM = 64, TN = 64, TK = 32;    // K = 128: 4 load rounds per product
    constexpr int PL = TM * TK / 256, QL = TN * TK / 256;   // elements per thread per tile
    __shared__ double Ps[TK][TM + 1];
    __shared__ double Qs[TK][TN + 1];
    const KTask t = tasks[blockIdx.z];
    const int i0 = blockIdx.y * TM, j0 = blockIdx.x * TN;
    const int tid = threadIdx.x;
    // four waves, each a 32 x 32 quarter of the tile as 2 x 2 FP64 MFMA
    // tiles (v_mfma_f64_16x16x4_f64: A[i][k] from lane (i + 16 k), B[k][j]
    // from lane (j + 16 k); D element (row (lane >> 4) + 4 reg, col lane & 15))
    const int wave = tid >> 6, lane = tid & 63;
    const int wr = (wave >> 1) * 32, wcol = (wave & 1) * 32;
    typedef double f64x4 __attribute__((ext_vector_type(4)));
    f64x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = f64x4{0.0, 0.0, 0.0, 0.0};
    // thread -> tile element maps (coalesced along the operand's contiguous dimension)
    int pii[PL], pkk[PL], qjj[QL], qkk[QL];
#pragma unroll
    for (int u = 0; u < PL; ++u) {
        const int e = tid + u * 256;
        if (psk == 1) { pii[u] = e / TK; pkk[u] = e % TK; } else { pkk[u] = e / TM; pii[u] = e % TM; }
    }
#pragma unroll
    for (int u = 0; u < QL; ++u) {
        const int e = tid + u * 256;
        if (qsk == 1) { qjj[u] = e / TK; qkk[u] = e % TK; } else { qkk[u] = e / TN; qjj[u] = e % TN; }
    }
    const int npair = t.P2 ? 2 : 1;
    const int nk = (K + TK - 1) / TK;
    const int nsteps = npair * nk;
    auto load = [&](int step, double* pv, double* qv) {
        const int pr = step / nk, k0 = (step % nk) * TK;
        const double* __restrict__ Pp = pr ? t.P2 : t.P;
        const double* __restrict__ Qp = pr ? t.Q2 : t.Q;
        const double* __restrict__ wp = pr ? nullptr : t.w;
#pragma unroll
        for (int u = 0; u < PL; ++u) {
            const int gi = i0 + pii[u], gk = k0 + pkk[u];
            double v = 0.0;
            if (gi < M && gk < K) {
                v = Pp[(int64_t)gi * psi + (int64_t)gk * psk];
                if (wp) v *= wp[gk];
            }
            pv[u] = v;
        }
#pragma unroll
        for (int u = 0; u < QL; ++u) {
            const int gj = j0 + qjj[u], gk = k0 + qkk[u];
            qv[u] = (gj < N && gk < K) ? Qp[(int64_t)gj * qsi + (int64_t)gk * qsk] : 0.0;
        }
    };
    double pv[PL], qv[QL];
    load(0, pv, qv);
    for (int step = 0; step < nsteps; ++step) {
#pragma unroll
        for (int u = 0; u < PL; ++u) Ps[pkk[u]][pii[u]] = pv[u];
#pragma unroll
        for (int u = 0; u < QL; ++u) Qs[qkk[u]][qjj[u]] = qv[u];
        __syncthreads();
        if (step + 1 < nsteps) load(step + 1, pv, qv);     // in flight while this tile is multiplied
#pragma unroll
        for (int kk = 0; kk < TK; kk += 4) {
            const int kr = kk + (lane >> 4), lc = lane & 15;
            double pa[2], qb[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) pa[t] = Ps[kr][wr + 16 * t + lc];
#pragma unroll
            for (int t = 0; t < 2; ++t) qb[t] = Qs[kr][wcol + 16 * t + lc];
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[a], qb[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int gi = i0 + wr + 16 * a + (lane >> 4) + 4 * g, gj = j0 + wcol + 16 * b + (lane & 15);
                if (gi < M && gj < N) {
                    double* cp = t.C + (int64_t)gi * ldc + gj;
                    *cp = beta == 0.0 ? alpha * acc[a][b][g] : alpha * acc[a][b][g] + beta * *cp;
                }
            }
}

// The solves' products, C = alpha (P diag(w) Q^T + P2 Q2^T) + beta C with few
// columns (N <= NT <= KMAX right-hand sides): one workgroup per (task, 32
// rows).  Q (and Q2) are staged whole in LDS in one round of loads; each row
// is 8 threads' fixed-stride partial sums (k = s, s + 8, ...), their P loads
// all in flight at once, combined by a fixed butterfly: deterministic.  In
// place of k_kkt_gemm's 64 x 64 tiles, whose K loop of dependent load rounds
// set the latency of every solve step.
constexpr int SK_ROWS = 32;
constexpr int SK_KPT = INV_RMAX_SK / 8;               // P values per thread and product
template <int NT>
__global__ __launch_bounds__(256) void k_kkt_gemm_skinny(const KTask* __restrict__ tasks, int M, int N, int K,
                                                         int psi, int psk, int qsi, int qsk, int ldc,
                                                         double alpha, double beta) {
    extern __shared__ double qs[];                    // [npair][K][NP]
    constexpr int NP = NT == 1 ? 1 : NT + 1;          // padded rows: the 8 sub-lanes' k rows hit distinct banks
    const KTask t = tasks[blockIdx.y];
    const int npair = t.P2 ? 2 : 1;
    const int tid = threadIdx.x;
    const int i = blockIdx.x * SK_ROWS + (tid >> 3), sl = tid & 7;
    const int ic = min(i, M - 1);
    // this thread's P values first (independent of the staging: in flight
    // beside it), k = sl, sl + 8, ...
    double pv[2][SK_KPT];
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
        const double* __restrict__ Pp = pr ? t.P2 : t.P;
        const double* __restrict__ wp = pr ? nullptr : t.w;
#pragma unroll
        for (int u = 0; u < SK_KPT; ++u) {
            const int k = 8 * u + sl;
            pv[pr][u] = (pr < npair && k < K) ? Pp[(int64_t)ic * psi + (int64_t)k * psk] * (wp ? wp[k] : 1.0) : 0.0;
        }
    }
    for (int e = tid; e < npair * K * NT; e += 256) {
        const int pr = e / (K * NT), rem = e - pr * K * NT, k = rem / NT, j = rem - k * NT;
        const double* __restrict__ Qp = pr ? t.Q2 : t.Q;
        qs[(pr * K + k) * NP + j] = j < N ? Qp[(int64_t)j * qsi + (int64_t)k * qsk] : 0.0;
    }
    double acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = 0.0;
    __syncthreads();
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
        if (pr >= npair) break;
        const double* qp = qs + (size_t)pr * K * NP;
#pragma unroll
        for (int u = 0; u < SK_KPT; ++u) {
            const int k = 8 * u + sl;
            if (k < K) {
#pragma unroll
                for (int j = 0; j < NT; ++j) acc[j] = fma(pv[pr][u], qp[k * NP + j], acc[j]);
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        acc[j] += __shfl_xor(acc[j], 4, 8);
        acc[j] += __shfl_xor(acc[j], 2, 8);
        acc[j] += __shfl_xor(acc[j], 1, 8);
    }
    if (i < M) {
#pragma unroll
        for (int j = 0; j < NT; ++j)
            if (j % 8 == sl && j < N) {
                double* cp = t.C + (int64_t)i * ldc + j;
                *cp = beta == 0.0 ? alpha * acc[j] : alpha * acc[j] + beta * *cp;
            }
    }
}

// In-place lower Cholesky of one r x r block per workgroup (right-looking:
// pivot, column scale, trailing update, one barrier each), in dynamic LDS
// when use_lds.  A non-positive or non-finite pivot sets *status (the caller
// regularizes and refactors, as Ipopt does on a wrong inertia).
__global__ __launch_bounds__(256) void k_kkt_potrf(double* const* __restrict__ mats, int r, int use_lds,
                                                   int* __restrict__ status) {
    extern __shared__ double lds[];
    __shared__ int bad;
    double* a = mats[blockIdx.x];
    double* s = use_lds ? lds : a;
    const int tid = threadIdx.x, nt = blockDim.x;
    if (use_lds) stage<8>(s, a, r * r);
    if (tid == 0) bad = 0;
    for (int j = 0; j < r; ++j) {
        __syncthreads();
        if (tid == 0) {
            double d = s[j * r + j];
            if (!(d > 0.0) || !isfinite(d)) {
                bad = 1;
                d = 1.0;
            }
            s[j * r + j] = sqrt(d);
        }
        __syncthreads();
        const double djj = s[j * r + j];
        for (int i = j + 1 + tid; i < r; i += nt) s[i * r + j] /= djj;
        __syncthreads();
        // trailing update of the lower triangle, threads as a 16 x (nt/16) grid
        const int tx = tid & 15, ty = tid >> 4, ny = nt >> 4;
        for (int i = j + 1 + ty; i < r; i += ny) {
            const double lij = s[i * r + j];
            for (int k = j + 1 + tx; k <= i; k += 16) s[i * r + k] -= lij * s[k * r + j];
        }
    }
    __syncthreads();
    if (use_lds)
        for (int e = tid; e < r * r; e += nt) a[e] = s[e];
    if (tid == 0 && bad) *status = 1;
}

// X = L^-1 B (trans = 0) or L^-T B (trans = 1) for the JW columns j0.. of
// one task per workgroup (blockIdx.x: column chunk, blockIdx.y: task);
// B(i, j) = B[i bsi + j bsj], X(i, j) = X[i ldx + j] (in place when B == X
// with the same strides).  Blocked by TB rows: the chunk of X is staged in
// LDS, each diagonal TB x TB block is solved by one lane per column, and the
// rows below (above, for L^T) are updated by the whole workgroup with the
// block's TB columns of L -- r / TB barriers instead of a sequential
// r^2 / 2 chain per lane.  L is staged in LDS as well when use_lds.
constexpr int TRSM_TB = 16;
__global__ __launch_bounds__(256) void k_kkt_trsm(const KTri* __restrict__ tasks, int r, int ncols, int bsi, int bsj,
                                                  int ldx, int trans, int use_lds, int JW) {
    extern __shared__ double lds[];
    const KTri t = tasks[blockIdx.y];
    const int tid = threadIdx.x, nt = blockDim.x;
    const int j0 = blockIdx.x * JW;
    const int jw = min(JW, ncols - j0);
    double* Xs = lds;                                   // [r][JW]
    const double* L = t.L;
    if (use_lds) {
        double* Ls = lds + (size_t)r * JW;
        stage<8>(Ls, t.L, r * r);
        L = Ls;
    }
    for (int e0 = 0; e0 < r * jw; e0 += 4 * nt) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = min(e0 + u * nt + tid, r * jw - 1);
            const int i = e / jw, j = e - i * jw;
            v[u] = t.B[(int64_t)i * bsi + (int64_t)(j0 + j) * bsj];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + u * nt + tid;
            if (e < r * jw) {
                const int i = e / jw, j = e - i * jw;
                Xs[i * JW + j] = v[u];
            }
        }
    }
    __syncthreads();
    const int ntile = (r + TRSM_TB - 1) / TRSM_TB;
    for (int q = 0; q < ntile; ++q) {
        const int tt = trans ? ntile - 1 - q : q;
        const int a = tt * TRSM_TB, b = min(r, a + TRSM_TB);
        // the diagonal block, one lane per column
        if (tid < jw) {
            double* x = Xs + tid;
            if (!trans) {
                for (int i = a; i < b; ++i) {
                    double s = x[i * JW];
                    for (int k = a; k < i; ++k) s -= L[(int64_t)i * r + k] * x[k * JW];
                    x[i * JW] = s / L[(int64_t)i * r + i];
                }
            } else {
                for (int i = b - 1; i >= a; --i) {
                    double s = x[i * JW];
                    for (int k = i + 1; k < b; ++k) s -= L[(int64_t)k * r + i] * x[k * JW];
                    x[i * JW] = s / L[(int64_t)i * r + i];
                }
            }
        }
        __syncthreads();
        // the remaining rows: below the block (L), above it (L^T)
        const int lo = trans ? 0 : b, hi = trans ? a : r;
        const int nrow = hi - lo;
        for (int e = tid; e < nrow * jw; e += nt) {
            const int i = lo + e / jw, j = e % jw;
            double s = Xs[i * JW + j];
            if (!trans)
                for (int k = a; k < b; ++k) s -= L[(int64_t)i * r + k] * Xs[k * JW + j];
            else
                for (int k = a; k < b; ++k) s -= L[(int64_t)k * r + i] * Xs[k * JW + j];
            Xs[i * JW + j] = s;
        }
        __syncthreads();
    }
    for (int e = tid; e < r * jw; e += nt) {
        const int i = e / jw, j = e - i * jw;
        t.X[(int64_t)i * ldx + j0 + j] = Xs[i * JW + j];
    }
}

// D_i -> L_i^-1, one block per workgroup, in registers (the inverse path:
// r <= INV_RMAX).  Every later product of the reduction and of its solves is
// then a GEMM with inv(L) (k_kkt_gemm) instead of a substitution chain: the
// batched-inverse form GPU solvers use for small blocks; the solves'
// rounding is that of a product with the inverse (~cond(L) eps), which the
// optimizer's iterative refinement absorbs.
constexpr int INV_T = 10;                 // register tile edge: r <= 16 INV_T
constexpr int INV_RMAX = 16 * INV_T;
static_assert(INV_RMAX == INV_RMAX_SK, "skinny product K bound");
// In-place inverse Cholesky in registers.  Z starts as A; step k reads row k
// of Z (w) and, for every row i > k,
//     Z[i, c] <- (c == k ? 0 : Z[i, c]) - w[i] (c == k ? 1 : w[c]) / w[k],
// and row k becomes w[c] / sqrt(w[k]) (c < k) and 1 / sqrt(w[k]) (c = k) --
// applied once after the last step, since no later step reads row k.
// Columns c > k of rows > k carry the trailing Schur complement (right-looking
// Cholesky, kept symmetric, so row k also holds column k); columns c <= k
// accumulate inv(L) (the identity eliminated by the same row operations).
// After step r - 1 the lower triangle of Z is inv(L).  Thread (ty, tx) of a
// 16 x 16 grid holds the T x T tile of rows ty T + a and columns tx T + b;
// the steps run in unrolled runs of T, so step k = k0 + ii's row and column
// are register (.., ii) of the threads with ty (tx) = k0 / T -- no dynamic
// register index, no selects over the tile -- and a thread whose rows are
// all done (ty < k0 / T) skips its update.  One barrier per two steps;
// LDS holds 4 rows.
template <int T>
__global__ __launch_bounds__(256) void k_kkt_potri(double* const* __restrict__ mats, int r, int* __restrict__ status) {
    __shared__ double wbuf[4][16 * INV_T];
    __shared__ double piv[16 * INV_T];
    __shared__ int bad;
    double* a = mats[blockIdx.x];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int row0 = ty * T, col0 = tx * T;
    double z[T][T];
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int row = row0 + i, col = col0 + j;
            const double v = a[(size_t)min(row, r - 1) * r + min(col, r - 1)];
            z[i][j] = (row < r && col < r) ? v : 0.0;
        }
    // entries >= r of w stay 0 (rows and columns past r then never change);
    // every LDS read below is unconditional, so none waits inside a branch
    for (int e = tid; e < 4 * 16 * INV_T; e += 256) (&wbuf[0][0])[e] = 0.0;
    if (tid == 0) bad = 0;
    __syncthreads();                                 // zeros in before step 0's row
    // step kk with row kk of Z in w (its owners' tile row / column ii_)
    auto step = [&](int ii_, int kk, int tk, const double* w) {
        const double p = w[kk];
        const double pp = (p > 0.0 && isfinite(p)) ? p : 1.0;
        if (tid == 0) {
            if (pp != p) bad = 1;
            piv[kk] = pp;
        }
        if (ty < tk) return;                         // every row of this thread done
        const int ic = ii_ < T ? ii_ : T - 1;
        const double pinv = 1.0 / pp;
        double wc[T], f[T];
#pragma unroll
        for (int j = 0; j < T; ++j) wc[j] = w[col0 + j];
#pragma unroll
        for (int i = 0; i < T; ++i) f[i] = w[row0 + i] * (row0 + i > kk ? pinv : 0.0);
        if (tx == tk) {                              // column kk of rows > kk: restart at 0, w = 1
            wc[ic] = 1.0;
#pragma unroll
            for (int i = 0; i < T; ++i) z[i][ic] = row0 + i > kk ? 0.0 : z[i][ic];
        }
#pragma unroll
        for (int i = 0; i < T; ++i)
#pragma unroll
            for (int j = 0; j < T; ++j) z[i][j] = fma(-f[i], wc[j], z[i][j]);
    };
    // steps in pairs per barrier: the owners (one 16-lane segment of a wave)
    // also broadcast row k + 1 as step k leaves it, formed privately by the
    // same operations every thread then applies (pivot and coupling from the
    // column owner's lane), so step k + 1 needs no barrier of its own;
    // buffers alternate by pair (a fast owner never overwrites a row being read)
    int bs = 0;
    for (int k0 = 0; k0 < r; k0 += T) {
        const int tk = k0 / T;                       // the owners' ty (row) and tx (column)
#pragma unroll
        for (int ii = 0; ii < T; ii += 2) {
            const int k = k0 + ii;
            if (k >= r) break;                       // uniform
            const int i1 = ii + 1 < T ? ii + 1 : T - 1;
            const bool two = ii + 1 < T && k + 1 < r;
            double* w0 = wbuf[(bs & 1) * 2];
            double* w1 = wbuf[(bs & 1) * 2 + 1];
            ++bs;
            if (ty == tk) {
#pragma unroll
                for (int j = 0; j < T; ++j) w0[col0 + j] = z[ii][j];   // 0 past r
                if (two) {
                    const double pk = __shfl(z[ii][ii], tk, 16);
                    const double ak = __shfl(z[ii][i1], tk, 16);
                    const double ppk = (pk > 0.0 && isfinite(pk)) ? pk : 1.0;
                    const double fk = ak * (1.0 / ppk);
#pragma unroll
                    for (int j = 0; j < T; ++j) {
                        const bool ck = tx == tk && j == ii;
                        w1[col0 + j] = fma(-fk, ck ? 1.0 : z[ii][j], ck ? 0.0 : z[i1][j]);
                    }
                }
            }
            __syncthreads();
            step(ii, k, tk, w0);
            if (two) step(ii + 1, k + 1, tk, w1);
        }
    }
    __syncthreads();
    // row i of inv(L): its unscaled row over columns < i, times 1 / sqrt(p_i),
    // and 1 / sqrt(p_i) on the diagonal (row i is never read after step i,
    // so the scaling waits until here)
#pragma unroll
    for (int i = 0; i < T; ++i) {
        const int row = row0 + i;
        const double dinv = 1.0 / sqrt(row < r ? piv[row] : 1.0);
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int col = col0 + j;
            z[i][j] = col < row ? z[i][j] * dinv : (col == row ? dinv : z[i][j]);
        }
    }
    // out, the upper triangle as zeros: the GEMMs read the full block
#pragma unroll
    for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j < T; ++j) {
            const int row = row0 + i, col = col0 + j;
            if (row < r && col < r) a[(size_t)row * r + col] = col <= row ? z[i][j] : 0.0;
        }
    if (tid == 0 && bad) *status = 1;
}

using potri_fn = void (*)(double* const*, int, int*);
static potri_fn potri_kernel(int r) {
    switch ((r + 15) / 16) {
        case 1: return k_kkt_potri<1>;
        case 2: return k_kkt_potri<2>;
        case 3: return k_kkt_potri<3>;
        case 4: return k_kkt_potri<4>;
        case 5: return k_kkt_potri<5>;
        case 6: return k_kkt_potri<6>;
        case 7: return k_kkt_potri<7>;
        case 8: return k_kkt_potri<8>;
        case 9: return k_kkt_potri<9>;
        default: return k_kkt_potri<10>;
    }
}

// [m, kc] (row-major) -> X [nb][r][KMAX] (padding rows 0), and back
__global__ void k_kkt_to_blocks(int64_t nbr, int kc, const int32_t* __restrict__ rowmap,
                                const double* __restrict__ b, double* __restrict__ X) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nbr * kc) return;
    const int64_t bi = e / kc;
    const int k = (int)(e % kc);
    const int row = rowmap[bi];
    X[bi * KMAX + k] = row >= 0 ? b[(int64_t)row * kc + k] : 0.0;
}
__global__ void k_kkt_from_blocks(int64_t nbr, int kc, const int32_t* __restrict__ rowmap,
                                  const double* __restrict__ X, double* __restrict__ b) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nbr * kc) return;
    const int64_t bi = e / kc;
    const int k = (int)(e % kc);
    const int row = rowmap[bi];
    if (row >= 0) b[(int64_t)row * kc + k] = X[bi * KMAX + k];
}

// R J's values in CSR order (cv[p] = vals[src[p]] rs[row[p]]): the
// products with J and J^T read them from here
__global__ void k_kkt_csr_vals(int64_t nnz, const int32_t* __restrict__ src, const int32_t* __restrict__ row,
                               const double* __restrict__ vals, const double* __restrict__ rs,
                               double* __restrict__ cv) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < nnz) cv[p] = vals[src[p]] * rs[row[p]];
}

// out[i][k] = sum_p val[pos ? pos[p] : p] x[idx[p]][k] over p in
// [ptr[i], ptr[i + 1]): y = R J v over the CSR rows, or (pos the CSC -> CSR
// permutation) v = J^T R y over the CSC columns.  G lanes per (i, k), summed
// by a fixed butterfly: deterministic.
template <int G>
__global__ __launch_bounds__(256) void k_kkt_spmv(int64_t nout, int kc, const int32_t* __restrict__ ptr,
                                                  const int32_t* __restrict__ idx, const int32_t* __restrict__ pos,
                                                  const double* __restrict__ val, const double* __restrict__ x,
                                                  double* __restrict__ out) {
    const int64_t item = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
    const int lane = (int)(threadIdx.x % G);
    double acc = 0.0;
    if (item < nout * kc) {
        const int64_t i = item / kc;
        const int k = (int)(item - i * kc);
        const int p1 = ptr[i + 1];
        for (int p = ptr[i] + lane; p < p1; p += G)
            acc += val[pos ? pos[p] : p] * x[(int64_t)idx[p] * kc + k];
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, G);
    if (item < nout * kc && lane == 0) out[item] = acc;
}

// the dense columns of J^T R y (their CSC ranges are empty): one workgroup
// per (column, right-hand side)
__global__ __launch_bounds__(256) void k_kkt_jtmul_dense(int64_t m, int nd, int kc, const double* __restrict__ Jd,
                                                         const int32_t* __restrict__ dcols,
                                                         const double* __restrict__ y, double* __restrict__ out) {
    __shared__ double red[256];
    const int d = blockIdx.x, k = blockIdx.y;
    // 8 independent partial sums per thread (8 loads in flight), combined in
    // a fixed order: deterministic
    double p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = 0.0;
    for (int64_t i0 = threadIdx.x; i0 < m; i0 += 8 * (int64_t)blockDim.x) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t i = i0 + u * (int64_t)blockDim.x;
            const int64_t ic = i < m ? i : m - 1;
            p[u] = fma(i < m ? Jd[ic * nd + d] : 0.0, y[ic * kc + k], p[u]);
        }
    }
    const double s = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[(int64_t)dcols[d] * kc + k] = red[0];
}

inline unsigned nblk(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

// ------------------------------------------------------------------------
// the module object
// ------------------------------------------------------------------------
struct KLevel {
    // factor
    KTask* gemm_d = nullptr;   int n_d = 0;    // even j: D_j -= V_{j-1}^T V_{j-1} + U_{j+1}^T U_{j+1}
    KTask* gemm_e = nullptr;   int n_e = 0;    // even j: E_j = -V_{j+1}^T U_{j+1} (the new coupling j+2 -> j)
    double** potrf = nullptr;  int n_odd = 0;
    KTri* tri_u = nullptr;     int n_u = 0;    // U = L^-1 E[left] (every odd block but the last level's)
    KTri* tri_v = nullptr;     int n_v = 0;    // V = L^-1 E[i]^T
    // solve
    KTri* sol = nullptr;                       // X_i in place
    KTask* fwd = nullptr;                      // even j: X_j -= V_{j-1}^T X_{j-1} + U_{j+1}^T X_{j+1}  (n_d)
    KTask* bwd = nullptr;                      // odd i: X_i -= U_i X[left] + V_i X[right]            (n_u)
    // the inverse path (D_i -> inv(L_i) by k_kkt_potri; every step a GEMM)
    KTask* inv_u = nullptr;                    // U_i = inv(L_i) E[left]        (n_u)
    KTask* inv_v = nullptr;                    // V_i = inv(L_i) E[i]^T         (n_v)
    KTask* inv_y = nullptr;                    // Y_i = inv(L_i) X_i            (n_odd)
    KTask* inv_fwd = nullptr;                  // even j: X_j -= V^T Y_{j-1} + U^T Y_{j+1}  (n_d)
    KTask* inv_bwd = nullptr;                  // odd i: Y_i -= U_i X[left] + V_i X[right]  (n_u)
    KTask* inv_x = nullptr;                    // X_i = inv(L_i)^T Y_i          (n_odd)
};

struct mh_kkt {
    mh_ctx* ctx = nullptr;
    int device = 0;
    int nb = 0, r = 0, c = 0, nd = 0, P = 0;
    int64_t m = 0, n = 0, nnz = 0;
    std::vector<int32_t> lshare, rshare;
    // device
    int32_t *a_src = nullptr, *rowmap = nullptr, *colmap = nullptr, *d_src = nullptr,
            *dcols = nullptr;
    double *vals = nullptr, *A = nullptr, *Jd = nullptr, *rs = nullptr, *w = nullptr, *dc = nullptr,
           *wl = nullptr, *dcl = nullptr, *D = nullptr, *E = nullptr, *U = nullptr, *V = nullptr,
           *x = nullptr, *X = nullptr, *Y = nullptr, *bm = nullptr, *bn = nullptr;
    int* status = nullptr;
    // J in CSR (every nonzero) and CSC (the block columns; the dense columns'
    // products are k_kkt_jtmul_dense's)
    int32_t *csr_ptr = nullptr, *csr_col = nullptr, *csr_src = nullptr, *csr_row = nullptr, *csc_ptr = nullptr,
            *csc_row = nullptr, *csc_pos = nullptr;
    double* cv = nullptr;
    // pinned staging for the host vectors each call exchanges
    double *hm = nullptr, *hn = nullptr;
    KTask *t_schur = nullptr, *t_e = nullptr;
    std::vector<KLevel> levels;      // the last level holds the single remaining block
    std::vector<void*> allocs;
    bool factored = false;
    // a module over a SHARD context (the whole NLP's Jacobian on this GPU,
    // mh_kkt_eval_jacobian writing only the shard's slice [nz0, nz1), the
    // caller filling the rest of the bound buffer, then mh_kkt_assemble)
    bool sharded = false;
    int64_t nz0 = 0, nz1 = 0;
    // the factorization's and each solve width's kernel sequences as HIP
    // graphs (captured on first use; every pointer they take is fixed at
    // create): one launch per call instead of ~50 (MOCOHIP_KKT_GRAPHS=0: off)
    bool graphs = true;
    bool inv_path = true;            // r <= INV_RMAX (160) and not MOCOHIP_KKT_INV=0
    hipGraphExec_t g_factor = nullptr;
    hipGraphExec_t g_solve[KMAX + 1] = {};
};

template <typename T>
static int kalloc(mh_kkt* h, T** p, size_t count) {
    void* q = nullptr;
    KCHK(hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T)));
    h->allocs.push_back(q);
    *p = (T*)q;
    return MH_OK;
}
template <typename T>
static int kupload(mh_kkt* h, T** p, const std::vector<T>& v) {
    int rc = kalloc(h, p, v.size());
    if (rc) return rc;
    if (!v.empty()) KCHK(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return MH_OK;
}
template <typename T>
static int kupload(mh_kkt* h, T** p, const T* src, size_t count) {
    int rc = kalloc(h, p, count);
    if (rc) return rc;
    if (count) KCHK(hipMemcpy(*p, src, count * sizeof(T), hipMemcpyHostToDevice));
    return MH_OK;
}

extern "C" void mh_kkt_destroy(mh_kkt* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    if (h->g_factor) (void)hipGraphExecDestroy(h->g_factor);
    for (auto& g : h->g_solve)
        if (g) (void)hipGraphExecDestroy(g);
    for (void* p : h->allocs) (void)hipFree(p);
    if (h->hm) (void)hipHostFree(h->hm);
    if (h->hn) (void)hipHostFree(h->hn);
    delete h;
}

static int build_levels(mh_kkt* h) {
    const int r = h->r;
    const size_t rr = (size_t)r * r;
    std::vector<int> active(h->nb);
    for (int i = 0; i < h->nb; ++i) active[i] = i;
    auto Dp = [&](int i) { return h->D + rr * i; };
    auto Ep = [&](int i) { return h->E + rr * i; };
    auto Up = [&](int i) { return h->U + rr * i; };
    auto Vp = [&](int i) { return h->V + rr * i; };
    auto Xp = [&](int i) { return h->X + (size_t)r * KMAX * i; };
    auto Yp = [&](int i) { return h->Y + (size_t)r * KMAX * i; };
    while (true) {
        KLevel L;
        std::vector<double*> potrf;
        std::vector<KTri> tu, tv, sol;
        std::vector<KTask> dd, ee, fw, bw, iu, iv, iy, ifw, ibw, ix;
        const int na = (int)active.size();
        if (na == 1) {
            const int i = active[0];
            potrf.push_back(Dp(i));
            sol.push_back({Dp(i), Xp(i), Xp(i)});
            iy.push_back({Dp(i), Xp(i), nullptr, Yp(i), nullptr, nullptr});
            ix.push_back({Dp(i), Yp(i), nullptr, Xp(i), nullptr, nullptr});
        } else {
            // odd positions: eliminated (their factors, U, V)
            for (int k = 1; k < na; k += 2) {
                const int i = active[k], left = active[k - 1];
                const int right = k + 1 < na ? active[k + 1] : -1;
                potrf.push_back(Dp(i));
                sol.push_back({Dp(i), Xp(i), Xp(i)});
                tu.push_back({Dp(i), Ep(left), Up(i)});
                iu.push_back({Dp(i), Ep(left), nullptr, Up(i), nullptr, nullptr});
                iy.push_back({Dp(i), Xp(i), nullptr, Yp(i), nullptr, nullptr});
                ix.push_back({Dp(i), Yp(i), nullptr, Xp(i), nullptr, nullptr});
                if (right >= 0) {
                    tv.push_back({Dp(i), Ep(i), Vp(i)});
                    iv.push_back({Dp(i), Ep(i), nullptr, Vp(i), nullptr, nullptr});
                    bw.push_back({Up(i), Xp(left), nullptr, Xp(i), Vp(i), Xp(right)});
                    ibw.push_back({Up(i), Xp(left), nullptr, Yp(i), Vp(i), Xp(right)});
                } else {
                    bw.push_back({Up(i), Xp(left), nullptr, Xp(i), nullptr, nullptr});
                    ibw.push_back({Up(i), Xp(left), nullptr, Yp(i), nullptr, nullptr});
                }
            }
            // even positions: updated from the odd neighbours, the left one's
            // V first, then the right one's U (one output tile per thread,
            // fixed order: deterministic)
            for (int k = 0; k < na; k += 2) {
                const int j = active[k];
                const int il = k - 1 >= 0 ? active[k - 1] : -1, ir = k + 1 < na ? active[k + 1] : -1;
                if (il >= 0 && ir >= 0) {
                    dd.push_back({Vp(il), Vp(il), nullptr, Dp(j), Up(ir), Up(ir)});
                    fw.push_back({Vp(il), Xp(il), nullptr, Xp(j), Up(ir), Xp(ir)});
                    ifw.push_back({Vp(il), Yp(il), nullptr, Xp(j), Up(ir), Yp(ir)});
                } else if (il >= 0) {
                    dd.push_back({Vp(il), Vp(il), nullptr, Dp(j), nullptr, nullptr});
                    fw.push_back({Vp(il), Xp(il), nullptr, Xp(j), nullptr, nullptr});
                    ifw.push_back({Vp(il), Yp(il), nullptr, Xp(j), nullptr, nullptr});
                } else if (ir >= 0) {
                    dd.push_back({Up(ir), Up(ir), nullptr, Dp(j), nullptr, nullptr});
                    fw.push_back({Up(ir), Xp(ir), nullptr, Xp(j), nullptr, nullptr});
                    ifw.push_back({Up(ir), Yp(ir), nullptr, Xp(j), nullptr, nullptr});
                }
                if (ir >= 0 && k + 2 < na) ee.push_back({Vp(ir), Up(ir), nullptr, Ep(j), nullptr, nullptr});
            }
        }
        int rc = 0;
        L.n_odd = (int)potrf.size();
        L.n_u = (int)tu.size();
        L.n_v = (int)tv.size();
        L.n_d = (int)dd.size();
        L.n_e = (int)ee.size();
        if ((rc = kupload(h, &L.potrf, potrf)) || (rc = kupload(h, &L.sol, sol)) ||
            (rc = kupload(h, &L.tri_u, tu)) || (rc = kupload(h, &L.tri_v, tv)) ||
            (rc = kupload(h, &L.gemm_d, dd)) || (rc = kupload(h, &L.gemm_e, ee)) ||
            (rc = kupload(h, &L.fwd, fw)) || (rc = kupload(h, &L.bwd, bw)) ||
            (rc = kupload(h, &L.inv_u, iu)) || (rc = kupload(h, &L.inv_v, iv)) ||
            (rc = kupload(h, &L.inv_y, iy)) || (rc = kupload(h, &L.inv_fwd, ifw)) ||
            (rc = kupload(h, &L.inv_bwd, ibw)) || (rc = kupload(h, &L.inv_x, ix)))
            return rc;
        h->levels.push_back(L);
        if (na == 1) break;
        std::vector<int> next;
        for (int k = 0; k < na; k += 2) next.push_back(active[k]);
        active.swap(next);
    }
    return MH_OK;
}

extern "C" int mh_kkt_create(mh_ctx* ctx, const mh_kkt_layout* L, mh_kkt** out) {
    if (!ctx || !L || !out) return mh_internal_error(MH_ERR_INVALID, "null argument");
    *out = nullptr;
    int64_t n = 0, m = 0, nnz = 0;
    int unsharded = 0;
    int rc = mh_internal_shape(ctx, &n, &m, &nnz, &unsharded);
    if (rc) return rc;
    // a shard context: the layout is the WHOLE NLP's (the module factors the
    // whole Jacobian; the context evaluates its own slice of it)
    int64_t nz0 = 0, nz1 = nnz;
    if (!unsharded && (rc = mh_internal_shard(ctx, &m, &nnz, &nz0, &nz1))) return rc;
    if (L->n != n || L->m != m || L->nnz != nnz)
        return mh_internal_error(MH_ERR_INVALID, "mh_kkt_layout does not match the context's NLP (n, m, nnz)");
    if (L->nblocks < 1 || L->r < 1 || L->c < 1 || L->nd < 0 || L->nshare < 0 || L->nshare > L->c || !L->a_src ||
            !L->rowmap || !L->colmap || !L->lshare || !L->rshare || !L->col2 || (L->nd > 0 && (!L->dcols || !L->d_src)))
        return mh_internal_error(MH_ERR_INVALID, "bad mh_kkt_layout");
    // host-side checks of every index the kernels follow
    const int64_t na = (int64_t)L->nblocks * L->r * L->c;
    for (int64_t e = 0; e < na; ++e)
        if (L->a_src[e] < -1 || L->a_src[e] >= nnz) return mh_internal_error(MH_ERR_INVALID, "a_src out of range");
    for (int64_t e = 0; e < (int64_t)L->nblocks * L->r; ++e)
        if (L->rowmap[e] < -1 || L->rowmap[e] >= m) return mh_internal_error(MH_ERR_INVALID, "rowmap out of range");
    for (int64_t e = 0; e < (int64_t)L->nblocks * L->c; ++e)
        if (L->colmap[e] < -1 || L->colmap[e] >= n) return mh_internal_error(MH_ERR_INVALID, "colmap out of range");
    for (int64_t e = 0; e < 2 * n; ++e)
        if (L->col2[e] < -1 || L->col2[e] >= L->nblocks * L->c)
            return mh_internal_error(MH_ERR_INVALID, "col2 out of range");
    for (int b = 0; b < L->nblocks; ++b)
        if (L->lshare[b] < 0 || L->rshare[b] < 0 || L->lshare[b] + L->nshare > L->c || L->rshare[b] + L->nshare > L->c)
            return mh_internal_error(MH_ERR_INVALID, "shared column range out of the block");
    for (int d = 0; d < L->nd; ++d)
        if (L->dcols[d] < 0 || L->dcols[d] >= n) return mh_internal_error(MH_ERR_INVALID, "dcols out of range");
    for (int64_t e = 0; e < m * L->nd; ++e)
        if (L->d_src[e] < -1 || L->d_src[e] >= nnz) return mh_internal_error(MH_ERR_INVALID, "d_src out of range");
    auto* h = new mh_kkt;
    h->ctx = ctx;
    h->device = mh_internal_device(ctx);
    h->nb = L->nblocks; h->r = L->r; h->c = L->c; h->nd = L->nd; h->P = L->nshare;
    h->m = m; h->n = n; h->nnz = nnz;
    h->sharded = !unsharded;
    h->nz0 = nz0; h->nz1 = nz1;
    h->lshare.assign(L->lshare, L->lshare + h->nb);
    if (const char* eg = std::getenv("MOCOHIP_KKT_GRAPHS")) h->graphs = std::atoi(eg) != 0;
    h->inv_path = L->r <= INV_RMAX;
    if (const char* ei = std::getenv("MOCOHIP_KKT_INV")) h->inv_path = h->inv_path && std::atoi(ei) != 0;
    h->rshare.assign(L->rshare, L->rshare + h->nb);
    auto fail = [&](int code) { mh_kkt_destroy(h); return code; };
    if (hipSetDevice(h->device) != hipSuccess) return fail(mh_internal_error(MH_ERR_HIP, "hipSetDevice failed"));
    const size_t rr = (size_t)h->r * h->r;
    if ((rc = kupload(h, &h->a_src, L->a_src, (size_t)na)) ||
        (rc = kupload(h, &h->rowmap, L->rowmap, (size_t)h->nb * h->r)) ||
        (rc = kupload(h, &h->colmap, L->colmap, (size_t)h->nb * h->c)) ||
        (rc = kupload(h, &h->dcols, L->dcols, (size_t)h->nd)) ||
        (rc = kupload(h, &h->d_src, L->d_src, (size_t)(m * h->nd))) ||
        (rc = kalloc(h, &h->vals, (size_t)nnz)) || (rc = kalloc(h, &h->A, (size_t)na)) ||
        (rc = kalloc(h, &h->Jd, (size_t)(m * h->nd))) || (rc = kalloc(h, &h->rs, (size_t)m)) ||
        (rc = kalloc(h, &h->w, (size_t)n)) || (rc = kalloc(h, &h->dc, (size_t)m)) ||
        (rc = kalloc(h, &h->wl, (size_t)h->nb * h->c)) || (rc = kalloc(h, &h->dcl, (size_t)h->nb * h->r)) ||
        (rc = kalloc(h, &h->D, rr * h->nb)) || (rc = kalloc(h, &h->E, rr * h->nb)) ||
        (rc = kalloc(h, &h->U, rr * h->nb)) || (rc = kalloc(h, &h->V, rr * h->nb)) ||
        (rc = kalloc(h, &h->x, (size_t)n)) || (rc = kalloc(h, &h->X, (size_t)h->nb * h->r * KMAX)) ||
        (rc = kalloc(h, &h->Y, (size_t)h->nb * h->r * KMAX)) ||
        (rc = kalloc(h, &h->bm, (size_t)m * KMAX)) || (rc = kalloc(h, &h->bn, (size_t)n * KMAX)) ||
        (rc = kalloc(h, &h->status, 1)))
        return fail(rc);
    {
        // every nonzero sits in exactly one block entry or dense-column slot
        std::vector<int32_t> row_of((size_t)nnz, -1), col_of((size_t)nnz, -1);
        auto place = [&](int32_t sidx, int64_t row, int64_t col) {
            if (sidx < 0) return true;
            if (row < 0 || col < 0 || row_of[sidx] >= 0) return false;
            row_of[sidx] = (int32_t)row;
            col_of[sidx] = (int32_t)col;
            return true;
        };
        for (int bb = 0; bb < h->nb; ++bb)
            for (int i = 0; i < h->r; ++i)
                for (int j = 0; j < h->c; ++j)
                    if (!place(L->a_src[((int64_t)bb * h->r + i) * h->c + j], L->rowmap[(int64_t)bb * h->r + i],
                               L->colmap[(int64_t)bb * h->c + j]))
                        return fail(mh_internal_error(MH_ERR_INVALID, "a_src places a nonzero twice or off the map"));
        for (int64_t i = 0; i < m; ++i)
            for (int d = 0; d < h->nd; ++d)
                if (!place(L->d_src[i * h->nd + d], i, L->dcols[d]))
                    return fail(mh_internal_error(MH_ERR_INVALID, "d_src places a nonzero twice"));
        std::vector<char> dense((size_t)n, 0);
        for (int d = 0; d < h->nd; ++d) dense[L->dcols[d]] = 1;
        std::vector<int32_t> rptr((size_t)m + 1, 0), cptr((size_t)n + 1, 0);
        for (int64_t sidx = 0; sidx < nnz; ++sidx) {
            if (row_of[sidx] < 0) return fail(mh_internal_error(MH_ERR_INVALID, "a nonzero outside the block map"));
            ++rptr[row_of[sidx] + 1];
            if (!dense[col_of[sidx]]) ++cptr[col_of[sidx] + 1];
        }
        for (int64_t i = 0; i < m; ++i) rptr[i + 1] += rptr[i];
        for (int64_t j = 0; j < n; ++j) cptr[j + 1] += cptr[j];
        std::vector<int32_t> ccol((size_t)nnz), csrc((size_t)nnz), crow((size_t)nnz), fill(rptr.begin(), rptr.end() - 1);
        for (int64_t sidx = 0; sidx < nnz; ++sidx) {   // rows in nonzero order: columns ascending within a row
            const int32_t p = fill[row_of[sidx]]++;
            ccol[p] = col_of[sidx];
            csrc[p] = (int32_t)sidx;
            crow[p] = row_of[sidx];
        }
        std::vector<int32_t> kr((size_t)cptr[n]), kp((size_t)cptr[n]), cfill(cptr.begin(), cptr.end() - 1);
        for (int64_t p = 0; p < nnz; ++p)              // CSR order: rows ascending within a column
            if (!dense[ccol[p]]) {
                const int32_t q = cfill[ccol[p]]++;
                kr[q] = crow[p];
                kp[q] = (int32_t)p;
            }
        if ((rc = kupload(h, &h->csr_ptr, rptr)) || (rc = kupload(h, &h->csr_col, ccol)) ||
            (rc = kupload(h, &h->csr_src, csrc)) || (rc = kupload(h, &h->csr_row, crow)) ||
            (rc = kupload(h, &h->csc_ptr, cptr)) || (rc = kupload(h, &h->csc_row, kr)) ||
            (rc = kupload(h, &h->csc_pos, kp)) || (rc = kalloc(h, &h->cv, (size_t)nnz)))
            return fail(rc);
    }
    // the 32-column skinny product's pair of staged operands exceeds the
    // default 64 KB of dynamic LDS at K = INV_RMAX
    if (hipFuncSetAttribute((const void*)k_kkt_gemm_skinny<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)(sizeof(double) * 2 * INV_RMAX * 33)) != hipSuccess)
        return fail(mh_internal_error(MH_ERR_HIP, "hipFuncSetAttribute (skinny product LDS) failed"));
    if (hipHostMalloc((void**)&h->hm, sizeof(double) * std::max<int64_t>(m, 1) * KMAX) != hipSuccess ||
        hipHostMalloc((void**)&h->hn, sizeof(double) * std::max<int64_t>(n, 1) * KMAX) != hipSuccess)
        return fail(mh_internal_error(MH_ERR_HIP, "pinned staging allocation failed"));
    std::vector<double> ones((size_t)m, 1.0);
    if (hipMemcpy(h->rs, ones.data(), sizeof(double) * m, hipMemcpyHostToDevice) != hipSuccess)
        return fail(mh_internal_error(MH_ERR_HIP, "upload failed"));
    std::vector<KTask> ts, te;
    for (int b = 0; b < h->nb; ++b) ts.push_back({h->A + (size_t)b * h->r * h->c, h->A + (size_t)b * h->r * h->c,
                                                 h->wl + (size_t)b * h->c, h->D + rr * b, nullptr, nullptr});
    for (int b = 0; b + 1 < h->nb; ++b)
        te.push_back({h->A + (size_t)(b + 1) * h->r * h->c + h->lshare[b + 1],
                      h->A + (size_t)b * h->r * h->c + h->rshare[b], h->wl + (size_t)b * h->c + h->rshare[b],
                      h->E + rr * b, nullptr, nullptr});
    if ((rc = kupload(h, &h->t_schur, ts)) || (rc = kupload(h, &h->t_e, te)) || (rc = build_levels(h)))
        return fail(rc);
    *out = h;
    return MH_OK;
}

extern "C" int mh_kkt_set_row_scale(mh_kkt* h, const double* rs) {
    if (!h || !rs) return mh_internal_error(MH_ERR_INVALID, "null argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    KCHK(hipMemcpyAsync(h->rs, rs, sizeof(double) * h->m, hipMemcpyHostToDevice, s));
    KCHK(hipStreamSynchronize(s));
    return MH_OK;
}

static int gather(mh_kkt* h, hipStream_t s) {
    const int64_t na = (int64_t)h->nb * h->r * h->c;
    hipLaunchKernelGGL(k_kkt_gather, dim3(nblk(na, 256)), dim3(256), 0, s, na, h->c, h->a_src, h->rowmap, h->vals,
                       h->rs, h->A);
    if (h->nd) {
        const int64_t nj = h->m * h->nd;
        hipLaunchKernelGGL(k_kkt_gather_dense, dim3(nblk(nj, 256)), dim3(256), 0, s, nj, h->nd, h->d_src, h->vals,
                           h->rs, h->Jd);
    }
    hipLaunchKernelGGL(k_kkt_csr_vals, dim3(nblk(h->nnz, 256)), dim3(256), 0, s, h->nnz, h->csr_src, h->csr_row,
                       h->vals, h->rs, h->cv);
    KCHK(hipGetLastError());
    return MH_OK;
}

extern "C" int mh_kkt_eval_jacobian(mh_kkt* h, const double* x) {
    if (!h || !x) return mh_internal_error(MH_ERR_INVALID, "null argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    KCHK(hipMemcpyAsync(h->x, x, sizeof(double) * h->n, hipMemcpyHostToDevice, s));
    int rc = mh_internal_jac_device(h->ctx, h->x, h->vals + h->nz0);
    if (rc) return rc;
    h->factored = false;
    if (h->sharded) {   // the other slices come from the other ranks, then mh_kkt_assemble
        KCHK(hipStreamSynchronize(s));
        return MH_OK;
    }
    if ((rc = gather(h, s))) return rc;
    KCHK(hipStreamSynchronize(s));
    return MH_OK;
}

extern "C" int mh_kkt_assemble(mh_kkt* h) {
    if (!h) return mh_internal_error(MH_ERR_INVALID, "null argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    int rc = gather(h, s);
    if (rc) return rc;
    h->factored = false;
    KCHK(hipStreamSynchronize(s));
    return MH_OK;
}

extern "C" int mh_kkt_bind_values(mh_kkt* h, double* values_dev) {
    if (!h || !values_dev) return mh_internal_error(MH_ERR_INVALID, "null argument");
    h->vals = values_dev;   // the module's own buffer stays allocated (freed with it)
    h->factored = false;
    return MH_OK;
}

extern "C" int mh_kkt_shard_range(const mh_kkt* h, int64_t* nnz_begin, int64_t* nnz_end) {
    if (!h || !nnz_begin || !nnz_end) return mh_internal_error(MH_ERR_INVALID, "null argument");
    *nnz_begin = h->nz0;
    *nnz_end = h->nz1;
    return MH_OK;
}

extern "C" int mh_kkt_get_values(mh_kkt* h, double* v) {
    if (!h || !v) return mh_internal_error(MH_ERR_INVALID, "null argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    KCHK(hipMemcpyAsync(v, h->vals, sizeof(double) * h->nnz, hipMemcpyDeviceToHost, s));
    KCHK(hipStreamSynchronize(s));
    return MH_OK;
}

extern "C" int mh_kkt_get_dense(mh_kkt* h, double* Jd) {
    if (!h || !Jd) return mh_internal_error(MH_ERR_INVALID, "null argument");
    if (!h->nd) return MH_OK;
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    KCHK(hipMemcpyAsync(Jd, h->Jd, sizeof(double) * h->m * h->nd, hipMemcpyDeviceToHost, s));
    KCHK(hipStreamSynchronize(s));
    return MH_OK;
}

template <int NT>
static void launch_skinny(hipStream_t s, const KTask* tasks, int ntasks, int M, int N, int K, int psi, int psk,
                          int qsi, int qsk, int ldc, double alpha, double beta) {
    // LDS for a pair of operands (the tasks of one launch share their shape;
    // single-product tasks use half)
    const size_t lds = sizeof(double) * 2 * (size_t)K * (NT == 1 ? 1 : NT + 1);
    hipLaunchKernelGGL(k_kkt_gemm_skinny<NT>, dim3(nblk(M, SK_ROWS), (unsigned)ntasks), dim3(256), lds, s, tasks, M,
                       N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
}
static void launch_gemm(hipStream_t s, const KTask* tasks, int ntasks, int M, int N, int K, int psi, int psk,
                        int qsi, int qsk, int ldc, double alpha, double beta) {
    if (ntasks <= 0) return;
    if (N <= KMAX && K <= INV_RMAX) {           // the solves: a few right-hand sides
        if (N <= 1) return launch_skinny<1>(s, tasks, ntasks, M, N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
        if (N <= 2) return launch_skinny<2>(s, tasks, ntasks, M, N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
        if (N <= 4) return launch_skinny<4>(s, tasks, ntasks, M, N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
        if (N <= 8) return launch_skinny<8>(s, tasks, ntasks, M, N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
        if (N <= 16) return launch_skinny<16>(s, tasks, ntasks, M, N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
        return launch_skinny<32>(s, tasks, ntasks, M, N, K, psi, psk, qsi, qsk, ldc, alpha, beta);
    }
    hipLaunchKernelGGL(k_kkt_gemm, dim3(nblk(N, 64), nblk(M, 64), (unsigned)ntasks), dim3(256), 0, s, tasks, M, N,
                       K, psi, psk, qsi, qsk, ldc, alpha, beta);
}

// LDS plan of k_kkt_trsm for blocks of r rows: (use_lds, JW, bytes)
static void trsm_plan(int r, int& use_lds, int& JW, size_t& bytes) {
    const size_t cap = (size_t)LDS_MAX - 1024;
    for (int jw : {64, 32, 16, 8}) {
        if (sizeof(double) * ((size_t)r * r + (size_t)r * jw) <= cap) {
            use_lds = 1; JW = jw; bytes = sizeof(double) * ((size_t)r * r + (size_t)r * jw);
            return;
        }
    }
    use_lds = 0;
    JW = 64;
    while (JW > 8 && sizeof(double) * (size_t)r * JW > cap) JW /= 2;
    bytes = sizeof(double) * (size_t)r * JW;
}

static void launch_trsm(hipStream_t s, const KTri* tasks, int ntasks, int r, int ncols, int bsi, int bsj, int ldx,
                        int trans) {
    if (ntasks <= 0) return;
    int use, JW;
    size_t lds;
    trsm_plan(r, use, JW, lds);
    hipLaunchKernelGGL(k_kkt_trsm, dim3(nblk(ncols, JW), (unsigned)ntasks), dim3(256), lds, s, tasks, r, ncols,
                       bsi, bsj, ldx, trans, use, JW);
}

// Run a fixed kernel sequence on s: replayed from its HIP graph, captured
// from the sequence itself on first use.
static int run_sequence(mh_kkt* h, hipStream_t s, hipGraphExec_t& exec, const std::function<void()>& enqueue) {
    if (!h->graphs) {
        enqueue();
        KCHK(hipGetLastError());
        return MH_OK;
    }
    if (!exec) {
        (void)hipGetLastError();
        KCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        enqueue();
        hipGraph_t g = nullptr;
        const hipError_t le = hipGetLastError();
        KCHK(hipStreamEndCapture(s, &g));
        KCHK(le);
        const hipError_t ei = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        KCHK(ei);
    }
    KCHK(hipGraphLaunch(exec, s));
    return MH_OK;
}

extern "C" int mh_kkt_factor(mh_kkt* h, const double* w, const double* dc, int32_t* ok) {
    if (!h || !w || !dc || !ok) return mh_internal_error(MH_ERR_INVALID, "null argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    const int r = h->r;
    std::memcpy(h->hn, w, sizeof(double) * h->n);
    std::memcpy(h->hm, dc, sizeof(double) * h->m);
    KCHK(hipMemcpyAsync(h->w, h->hn, sizeof(double) * h->n, hipMemcpyHostToDevice, s));
    KCHK(hipMemcpyAsync(h->dc, h->hm, sizeof(double) * h->m, hipMemcpyHostToDevice, s));
    KCHK(hipMemsetAsync(h->status, 0, sizeof(int), s));
    const size_t lds = sizeof(double) * r * r;
    const int use_lds = lds + 64 <= (size_t)LDS_MAX ? 1 : 0;
    // the blocks' own LDS sizes (the attribute's maximum is the device's LDS
    // minus the kernel's static LDS); a refused request would resurface as
    // the next launch check's error, so it is checked here
    if (use_lds && lds > 65536)
        KCHK(hipFuncSetAttribute((const void*)k_kkt_potrf, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    {
        int tu, tj;
        size_t tl;
        trsm_plan(r, tu, tj, tl);
        if (tl > 65536)
            KCHK(hipFuncSetAttribute((const void*)k_kkt_trsm, hipFuncAttributeMaxDynamicSharedMemorySize, (int)tl));
    }
    const potri_fn potri = potri_kernel(r);
    const int nbc = h->nb * h->c, nbr = h->nb * r;
    int rc = run_sequence(h, s, h->g_factor, [&]() {
        hipLaunchKernelGGL(k_kkt_local, dim3(nblk(std::max(nbc, nbr), 256)), dim3(256), 0, s, nbc, nbr, h->colmap,
                           h->rowmap, h->w, h->dc, h->wl, h->dcl);
        // D_b = A_b W_b A_b^T + diag(dc_b); E_b = A_{b+1}[:, shared] W A_b[:, shared]^T
        launch_gemm(s, h->t_schur, h->nb, r, r, h->c, h->c, 1, h->c, 1, r, 1.0, 0.0);
        hipLaunchKernelGGL(k_kkt_add_diag, dim3(h->nb), dim3(256), 0, s, r, h->dcl, h->D);
        launch_gemm(s, h->t_e, h->nb - 1, r, r, h->P, h->c, 1, h->c, 1, r, 1.0, 0.0);
        for (const KLevel& L : h->levels) {
            if (h->inv_path) {
                // D_i -> inv(L_i); U, V, the even updates: GEMMs
                hipLaunchKernelGGL(potri, dim3((unsigned)L.n_odd), dim3(256), 0, s, L.potrf, r, h->status);
                launch_gemm(s, L.inv_u, L.n_u, r, r, r, r, 1, 1, r, r, 1.0, 0.0);
                launch_gemm(s, L.inv_v, L.n_v, r, r, r, r, 1, r, 1, r, 1.0, 0.0);
                launch_gemm(s, L.gemm_d, L.n_d, r, r, r, 1, r, 1, r, r, -1.0, 1.0);
                launch_gemm(s, L.gemm_e, L.n_e, r, r, r, 1, r, 1, r, r, -1.0, 0.0);
                continue;
            }
            hipLaunchKernelGGL(k_kkt_potrf, dim3((unsigned)L.n_odd), dim3(256), use_lds ? lds : 0, s, L.potrf, r,
                               use_lds, h->status);
            // U = L^-1 E[left] (row-major B), V = L^-1 E[i]^T (transposed B)
            launch_trsm(s, L.tri_u, L.n_u, r, r, r, 1, r, 0);
            launch_trsm(s, L.tri_v, L.n_v, r, r, 1, r, r, 0);
            // even j: D_j -= V_{j-1}^T V_{j-1} + U_{j+1}^T U_{j+1}; E_j = -V_{j+1}^T U_{j+1}
            launch_gemm(s, L.gemm_d, L.n_d, r, r, r, 1, r, 1, r, r, -1.0, 1.0);
            launch_gemm(s, L.gemm_e, L.n_e, r, r, r, 1, r, 1, r, r, -1.0, 0.0);
        }
    });
    if (rc) return rc;
    int st = 0;
    KCHK(hipMemcpyAsync(&st, h->status, sizeof(int), hipMemcpyDeviceToHost, s));
    KCHK(hipStreamSynchronize(s));
    *ok = st ? 0 : 1;
    h->factored = st == 0;
    return MH_OK;
}

extern "C" int mh_kkt_solve(mh_kkt* h, int32_t k, const double* b, double* xout) {
    if (!h || !b || !xout || k < 1) return mh_internal_error(MH_ERR_INVALID, "bad argument");
    if (!h->factored) return mh_internal_error(MH_ERR_INVALID, "mh_kkt_solve before a successful mh_kkt_factor");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    const int r = h->r;
    const int64_t nbr = (int64_t)h->nb * r;
    for (int k0 = 0; k0 < k; k0 += KMAX) {
        const int kc = std::min(KMAX, k - k0);
        // the chunk's columns, row-major [m][kc]
        double* in = h->hm;
        if (kc == k) std::memcpy(in, b, sizeof(double) * h->m * kc);
        else
            for (int64_t i = 0; i < h->m; ++i)
                std::memcpy(in + (size_t)i * kc, b + (size_t)i * k + k0, sizeof(double) * kc);
        KCHK(hipMemcpyAsync(h->bm, in, sizeof(double) * h->m * kc, hipMemcpyHostToDevice, s));
        int rc = run_sequence(h, s, h->g_solve[kc], [&]() {
            hipLaunchKernelGGL(k_kkt_to_blocks, dim3(nblk(nbr * kc, 256)), dim3(256), 0, s, nbr, kc, h->rowmap,
                               h->bm, h->X);
            if (h->inv_path) {
                for (size_t l = 0; l < h->levels.size(); ++l) {             // forward: Y = inv(L) X, updates
                    const KLevel& L = h->levels[l];
                    launch_gemm(s, L.inv_y, L.n_odd, r, kc, r, r, 1, 1, KMAX, KMAX, 1.0, 0.0);
                    launch_gemm(s, L.inv_fwd, L.n_d, r, kc, r, 1, r, 1, KMAX, KMAX, -1.0, 1.0);
                }
                for (size_t l = h->levels.size(); l-- > 0;) {               // backward: X = inv(L)^T (Y - U X_l - V X_r)
                    const KLevel& L = h->levels[l];
                    launch_gemm(s, L.inv_bwd, L.n_u, r, kc, r, r, 1, 1, KMAX, KMAX, -1.0, 1.0);
                    launch_gemm(s, L.inv_x, L.n_odd, r, kc, r, 1, r, 1, KMAX, KMAX, 1.0, 0.0);
                }
            } else {
                for (size_t l = 0; l < h->levels.size(); ++l) {             // forward
                    const KLevel& L = h->levels[l];
                    launch_trsm(s, L.sol, L.n_odd, r, kc, KMAX, 1, KMAX, 0);
                    launch_gemm(s, L.fwd, L.n_d, r, kc, r, 1, r, 1, KMAX, KMAX, -1.0, 1.0);
                }
                for (size_t l = h->levels.size(); l-- > 0;) {               // backward
                    const KLevel& L = h->levels[l];
                    launch_gemm(s, L.bwd, L.n_u, r, kc, r, r, 1, 1, KMAX, KMAX, -1.0, 1.0);
                    launch_trsm(s, L.sol, L.n_odd, r, kc, KMAX, 1, KMAX, 1);
                }
            }
            hipLaunchKernelGGL(k_kkt_from_blocks, dim3(nblk(nbr * kc, 256)), dim3(256), 0, s, nbr, kc, h->rowmap,
                               h->X, h->bm);
        });
        if (rc) return rc;
        KCHK(hipMemcpyAsync(in, h->bm, sizeof(double) * h->m * kc, hipMemcpyDeviceToHost, s));
        KCHK(hipStreamSynchronize(s));
        if (kc == k) std::memcpy(xout, in, sizeof(double) * h->m * kc);
        else
            for (int64_t i = 0; i < h->m; ++i)
                std::memcpy(xout + (size_t)i * k + k0, in + (size_t)i * kc, sizeof(double) * kc);
    }
    return MH_OK;
}

// a host [rows][k] matrix's columns k0 .. k0 + kc -> pinned [rows][kc], and back
static void pack(double* dst, const double* src, int64_t rows, int k, int k0, int kc) {
    if (kc == k) std::memcpy(dst, src, sizeof(double) * rows * kc);
    else
        for (int64_t i = 0; i < rows; ++i) std::memcpy(dst + (size_t)i * kc, src + (size_t)i * k + k0, sizeof(double) * kc);
}
static void unpack(double* dst, const double* src, int64_t rows, int k, int k0, int kc) {
    if (kc == k) std::memcpy(dst, src, sizeof(double) * rows * kc);
    else
        for (int64_t i = 0; i < rows; ++i) std::memcpy(dst + (size_t)i * k + k0, src + (size_t)i * kc, sizeof(double) * kc);
}
constexpr int SPMV_G = 8;

extern "C" int mh_kkt_jmul(mh_kkt* h, int32_t k, const double* v, double* y) {
    if (!h || !v || !y || k < 1) return mh_internal_error(MH_ERR_INVALID, "bad argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    for (int k0 = 0; k0 < k; k0 += KMAX) {
        const int kc = std::min(KMAX, k - k0);
        pack(h->hn, v, h->n, k, k0, kc);
        KCHK(hipMemcpyAsync(h->bn, h->hn, sizeof(double) * h->n * kc, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_kkt_spmv<SPMV_G>, dim3(nblk(h->m * kc * SPMV_G, 256)), dim3(256), 0, s, h->m, kc,
                           h->csr_ptr, h->csr_col, (const int32_t*)nullptr, h->cv, h->bn, h->bm);
        KCHK(hipGetLastError());
        KCHK(hipMemcpyAsync(h->hm, h->bm, sizeof(double) * h->m * kc, hipMemcpyDeviceToHost, s));
        KCHK(hipStreamSynchronize(s));
        unpack(y, h->hm, h->m, k, k0, kc);
    }
    return MH_OK;
}

extern "C" int mh_kkt_jtmul(mh_kkt* h, int32_t k, const double* y, double* v) {
    if (!h || !v || !y || k < 1) return mh_internal_error(MH_ERR_INVALID, "bad argument");
    KCHK(hipSetDevice(h->device));
    hipStream_t s = mh_internal_stream(h->ctx);
    for (int k0 = 0; k0 < k; k0 += KMAX) {
        const int kc = std::min(KMAX, k - k0);
        pack(h->hm, y, h->m, k, k0, kc);
        KCHK(hipMemcpyAsync(h->bm, h->hm, sizeof(double) * h->m * kc, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_kkt_spmv<SPMV_G>, dim3(nblk(h->n * kc * SPMV_G, 256)), dim3(256), 0, s, h->n, kc,
                           h->csc_ptr, h->csc_row, h->csc_pos, h->cv, h->bm, h->bn);
        if (h->nd)
            hipLaunchKernelGGL(k_kkt_jtmul_dense, dim3(h->nd, kc), dim3(256), 0, s, h->m, h->nd, kc, h->Jd, h->dcols,
                               h->bm, h->bn);
        KCHK(hipGetLastError());
        KCHK(hipMemcpyAsync(h->hn, h->bn, sizeof(double) * h->n * kc, hipMemcpyDeviceToHost, s));
        KCHK(hipStreamSynchronize(s));
        unpack(v, h->hn, h->n, k, k0, kc);
    }
    return MH_OK;
}
