/* mocohip_kkt.h — the host optimizer's Newton-system linear algebra on the
 * device, next to the Jacobian (libmocohip.so, csrc/kkt.hip).
 *
 * What it replaces: the reference hands each Newton system of the
 * transcription to Ipopt 3.12.8's linear solver (MUMPS) on the host
 * (MocoCasADiSolver.cpp:210-246 selects Ipopt; IpPDFullSpaceSolver /
 * IpStdAugSystemSolver factor [[W + Sigma, J^T], [J, -delta]]); tropter's
 * IPOPTSolver.cpp:302-447 hands Ipopt the same structure.  Here the
 * interior-point driver (mocohip/ipm.py) eliminates the bound multipliers
 * and slacks and factors the Schur complement
 *
 *     S = R J W J^T R + diag(dc),  W = diag(w) over the block columns,
 *
 * which for a collocation Jacobian is block tridiagonal over mesh intervals.
 * The host computes the block map once (mocohip/kkt.py block_map); every
 * numeric step runs on the context's device and stream.  Plain C ABI:
 * int status + the error text of mh_last_error, host pointers for vectors (row-major
 * [rows][k] for k right-hand sides), 0-based indices. */
#ifndef MOCOHIP_KKT_H
#define MOCOHIP_KKT_H

#include "mocohip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mh_kkt mh_kkt;

/* The symbolic block map (see mocohip/kkt.py BlockMap).  nblocks blocks of
 * at most r rows and c local columns; per block b:
 *   a_src[(b r + i) c + j]  Jacobian nonzero feeding entry (i, j) of A_b, -1: 0
 *   rowmap[b r + i]         global row of local row i, -1: padding
 *   colmap[b c + j]         global column of local column j, -1: padding
 *   lshare[b], rshare[b]    local offset of the nshare columns block b shares
 *                           with block b - 1 / b + 1 (one grid point's)
 * dense columns (read outside the block pattern: t0, tf, ...):
 *   dcols[d], d_src[i nd + d]  nonzero feeding row i of dense column d
 * col2[2 j + {0, 1}]        the flat A positions b c + local column of global
 *                           column j (two for a shared grid point), -1: none
 * Every index is range-checked on the host at create. */
typedef struct {
    int32_t nblocks, r, c, nd, nshare, reserved;
    int64_t m, n, nnz;
    const int32_t* a_src;
    const int32_t* rowmap;
    const int32_t* colmap;
    const int32_t* lshare;
    const int32_t* rshare;
    const int32_t* dcols;
    const int32_t* d_src;
    const int32_t* col2;
} mh_kkt_layout;

/* A KKT module over a context; the context must outlive it.  The layout is
 * the whole NLP's (n, m, nnz of mh_get_nlp_info).  Over a SHARD context
 * (mh_options interval_begin / interval_end: one rank of an NLP sharded by
 * mesh interval) the module still factors the whole
 * Jacobian on this GPU: mh_kkt_eval_jacobian writes only the shard's slice
 * [nnz_begin, nnz_end) of the values buffer, the caller receives the other
 * ranks' slices into their offsets (e.g. RCCL over xGMI into a buffer bound
 * with mh_kkt_bind_values), then calls mh_kkt_assemble. */
int mh_kkt_create(mh_ctx* ctx, const mh_kkt_layout* layout, mh_kkt** out);
void mh_kkt_destroy(mh_kkt* kkt);
/* R (m doubles, default 1): the optimizer's constraint row scaling. */
int mh_kkt_set_row_scale(mh_kkt* kkt, const double* row_scale);
/* J(x) by the context's own eval_jac_g kernels into the module's device
 * buffer, gathered into the blocks A_b and the dense columns (row-scaled).
 * Replaces the eval_jac_g a host Ipopt would make at this iterate. */
int mh_kkt_eval_jacobian(mh_kkt* kkt, const double* x);
/* Sharded module: the blocks and dense columns from the whole values buffer
 * once every slice is in it (the gather mh_kkt_eval_jacobian does itself on
 * an unsharded context); synchronous. */
int mh_kkt_assemble(mh_kkt* kkt);
/* The Jacobian values buffer: nnz doubles of device memory on the module's
 * GPU owned by the caller, used from now on instead of the module's own
 * (which stays allocated); the caller keeps it alive. */
int mh_kkt_bind_values(mh_kkt* kkt, double* values_device);
/* This module's own slice [*nnz_begin, *nnz_end) of the values (the whole
 * range on an unsharded context). */
int mh_kkt_shard_range(const mh_kkt* kkt, int64_t* nnz_begin, int64_t* nnz_end);
/* The raw values of the last mh_kkt_eval_jacobian (nnz doubles). */
int mh_kkt_get_values(mh_kkt* kkt, double* values);
/* The row-scaled dense columns, [m][nd]. */
int mh_kkt_get_dense(mh_kkt* kkt, double* jd);
/* Form S with weights w (n doubles; only block columns are read, dense
 * columns belong to the caller's low-rank update) and dc (m doubles) and
 * factor it by block cyclic reduction.  *ok = 0 when a pivot is not
 * positive (the caller regularizes, Ipopt's delta_c). */
int mh_kkt_factor(mh_kkt* kkt, const double* w, const double* dc, int32_t* ok);
/* x = S^-1 b, b and x [m][k]. */
int mh_kkt_solve(mh_kkt* kkt, int32_t k, const double* b, double* x);
/* y = R J v (v [n][k], every column including the dense ones; y [m][k]). */
int mh_kkt_jmul(mh_kkt* kkt, int32_t k, const double* v, double* y);
/* v = J^T R y (y [m][k], v [n][k]). */
int mh_kkt_jtmul(mh_kkt* kkt, int32_t k, const double* y, double* v);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* MOCOHIP_KKT_H */
