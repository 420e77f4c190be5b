/* oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE).
 *
 * This is the parity oracle for the MI355X path.  It is NOT part of the
 * product: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it, and only as the checker / CPU baseline.  The product
 * library (libmocohip.so) never links or calls it.
 *
 * It restates, in plain C99 and independently of the HIP kernels:
 *   - CasOC transcription layout, bounds, defects, quadrature, constraint
 *     flattening and block-dense Jacobian structure
 *     (Moco/Moco/MocoCasADiSolver/CasOCTranscription.{h,cpp},
 *      CasOCHermiteSimpson.cpp, CasOCTrapezoidal.cpp);
 *   - the per-grid-point explicit DAE of MocoCasOCProblem
 *     (MocoCasOCProblem.h:203-244) on a Simbody-equivalent multibody model;
 *   - DeGrooteFregly2016Muscle (Moco/Moco/Components/DeGrooteFregly2016Muscle.*);
 *   - goal integrands (MocoControlGoal.cpp:120-131,
 *     MocoStateTrackingGoal.cpp:103-117, MocoGoal.h:387-400);
 *   - finite-difference derivatives of the per-point callbacks
 *     (CasOCFunction.h:38-44: enable_fd, fd_method central|forward|backward).
 * Parity status of each piece is documented in DESIGN.md §Oracle.
 */
#ifndef MOCO_ORACLE_H
#define MOCO_ORACLE_H

#include "../include/mocohip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_ctx orc_ctx;

const char* orc_last_error(void);
int orc_create(const mh_problem* problem, const mh_options* options,
        orc_ctx** ctx);
void orc_destroy(orc_ctx* ctx);
/* Worker threads used for per-grid-point work (1 = serial). */
void orc_set_threads(orc_ctx* ctx, int nthreads);

int orc_get_nlp_info(const orc_ctx* ctx, mh_nlp_info* info);
int orc_get_bounds(const orc_ctx* ctx, double* x_l, double* x_u, double* g_l,
        double* g_u);
int orc_get_initial_guess_from_bounds(const orc_ctx* ctx, double* x);
int orc_get_random_iterate(const orc_ctx* ctx, const double* rand, double* x);
int orc_get_jac_structure(const orc_ctx* ctx, int32_t* iRow, int32_t* jCol);

int orc_eval_f(orc_ctx* ctx, const double* x, double* f);
int orc_eval_grad_f(orc_ctx* ctx, const double* x, double* grad_f);
/* mh_eval_f_partial / mh_eval_grad_f_partial: the shard's own mesh
 * intervals' quadrature, endpoint goals on the shard owning the final point. */
int orc_eval_f_partial(orc_ctx* ctx, const double* x, double* f);
int orc_eval_grad_f_partial(orc_ctx* ctx, const double* x, double* grad_f);
int orc_eval_g(orc_ctx* ctx, const double* x, double* g);
int orc_eval_jac_g(orc_ctx* ctx, const double* x, double* values);

/* g (m) and Jacobian values (nnz) re-derived from raw finite-difference
 * lane outputs Y and grid times in the layout of mh_debug_jacobian_lanes
 * (include/mocohip.h): the checker of the device's quotient and assembly
 * arithmetic.  g or values may be NULL. */
int orc_assemble_from_lanes(orc_ctx* ctx, const double* x, const double* times,
        const double* Y, double* g, double* values);

/* inputs per point: [time, states(NS), controls(NC)];
 * outputs per point: [udot(NQ), zdot(NZ)]. */
int orc_eval_dae(orc_ctx* ctx, int32_t npoints, const double* inputs,
        double* outputs);
/* the same on the model with iterate x's MocoParameters applied, parameter
 * `moved` (-1: none) moved by `step` */
int orc_eval_dae_params(orc_ctx* ctx, const double* x, int32_t moved, double step, int32_t npoints,
        const double* inputs, double* outputs);

/* Muscle-level probes for the DGF known-answer tests
 * (Moco/Tests/testMocoActuators.cpp:199-220,1026-1039). which:
 *  0 active force-length f_AL(x)      1 passive force-length f_PE(x)
 *  2 force-velocity f_V(x)            3 force-velocity inverse
 *  4 tendon force-length f_T(x)       5 tendon force-length inverse
 *  6 tendon f_T'(x)                                                   */
double orc_dgf_curve(const mh_muscle* muscle, int which, double x);

/* Muscle-tendon length / lengthening speed and generalized-coordinate
 * probes at a state (q,u): out = [length, speed] for muscle im. */
int orc_muscle_length_speed(orc_ctx* ctx, int im, const double* q,
        const double* u, double* out);
/* The muscle's current path (points and wrap tangent points) in ground:
 * *n entries of [x, y, z, kind], kind = path point index or -1 / -2. */
int orc_muscle_path(orc_ctx* ctx, int im, const double* q, const double* u, int cap, int* n,
        double* pts);
/* Evaluate a model function (joint axis / moving point) and derivatives. */
int orc_eval_function(orc_ctx* ctx, int ifn, double q, double* out3);
/* The callback sparsity behind the structure (mh_get_callback_sparsity). */
int orc_get_callback_sparsity(const orc_ctx* ctx, uint8_t* pattern, int64_t len);
int orc_get_jacobian_seeds(const orc_ctx* c, int32_t* color, int32_t* nseeds);
/* mh_color_jacobian_ordered restated (host, no context). */
int orc_color_jacobian(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow, const int32_t* jCol,
        int32_t order, int32_t* color, int32_t* ncolors);

#ifdef __cplusplus
}
#endif

#endif
