/* oracle.c — CPU restatement of the Moco direct-collocation hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C99, serial reference
 * arithmetic, optional OpenMP fan-out over grid points mirroring CasADi's
 * map(N, "thread", T) (CasOCTranscription.cpp:1179-1184).
 *
 * Each function cites the reference file:line it restates.  Third-party
 * arithmetic that is not in /root/reference (Simbody forward dynamics,
 * OpenSim GeometryPath / SimmSpline, CasADi FiniteDiff) is restated from the
 * published algorithms; see DESIGN.md §Oracle for the parity status of each.
 */
#include "oracle.h"

#include <float.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* Scalar type of the model evaluation.  The FLOP-counting build
 * (oracle/flopcount.cpp) compiles this file as C++ with a counting type. */
#ifndef ORACLE_REAL
typedef double real;
#else
typedef ORACLE_REAL real;
#endif

static __thread char g_err[512];
const char* orc_last_error(void) { return g_err; }
static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

/* ======================================================================== */
/* Small 3-vector / 3x3 helpers (row-major matrices).                        */
/* ======================================================================== */
typedef struct { real w[3], v[3]; } sv6; /* spatial vector about ground origin */

static void mat_mul(const real* A, const real* B, real* C) {
    real T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] +
                           A[3 * i + 2] * B[6 + j];
    memcpy(C, T, sizeof T);
}
static void mat_mul_bt(const real* A, const real* B, real* C) { /* A*B^T */
    real T[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            T[3 * i + j] = A[3 * i] * B[3 * j] + A[3 * i + 1] * B[3 * j + 1] +
                           A[3 * i + 2] * B[3 * j + 2];
    memcpy(C, T, sizeof T);
}
static void mat_vec(const real* A, const real* x, real* y) {
    real t0 = A[0] * x[0] + A[1] * x[1] + A[2] * x[2];
    real t1 = A[3] * x[0] + A[4] * x[1] + A[5] * x[2];
    real t2 = A[6] * x[0] + A[7] * x[1] + A[8] * x[2];
    y[0] = t0; y[1] = t1; y[2] = t2;
}
static void cross(const real* a, const real* b, real* c) {
    real t0 = a[1] * b[2] - a[2] * b[1];
    real t1 = a[2] * b[0] - a[0] * b[2];
    real t2 = a[0] * b[1] - a[1] * b[0];
    c[0] = t0; c[1] = t1; c[2] = t2;
}
static real dot3(const real* a, const real* b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}
/* Rodrigues rotation about unit axis a by angle t. */
static void axis_rotation(const real* a, real t, real* R) {
    real c = cos(t), s = sin(t), k = 1.0 - c;
    R[0] = c + k * a[0] * a[0];
    R[1] = k * a[0] * a[1] - s * a[2];
    R[2] = k * a[0] * a[2] + s * a[1];
    R[3] = k * a[1] * a[0] + s * a[2];
    R[4] = c + k * a[1] * a[1];
    R[5] = k * a[1] * a[2] - s * a[0];
    R[6] = k * a[2] * a[0] - s * a[1];
    R[7] = k * a[2] * a[1] + s * a[0];
    R[8] = c + k * a[2] * a[2];
}
/* Spatial motion cross product (w,v) x_m (w2,v2). */
static sv6 cross_m(sv6 a, sv6 b) {
    sv6 r;
    real t[3];
    cross(a.w, b.w, r.w);
    cross(a.w, b.v, r.v);
    cross(a.v, b.w, t);
    for (int i = 0; i < 3; ++i) r.v[i] += t[i];
    return r;
}
/* Spatial force cross product (w,v) x_f (n,f). */
static sv6 cross_f(sv6 a, sv6 f) {
    sv6 r;
    real t[3];
    cross(a.w, f.w, r.w);
    cross(a.v, f.v, t);
    for (int i = 0; i < 3; ++i) r.w[i] += t[i];
    cross(a.w, f.v, r.v);
    return r;
}
static real sv_dot(sv6 m, sv6 f) { return dot3(m.w, f.w) + dot3(m.v, f.v); }

/* Rigid-body inertia about the ground origin: mass, first moment h = m c,
 * rotational inertia about the origin I_O (sym: xx yy zz xy xz yz). */
typedef struct { real m, h[3], I[6]; } rbi;
static sv6 rbi_apply(const rbi* I, sv6 x) {
    /* (I_O w + h x u, m u - h x w) */
    sv6 r;
    real t[3];
    r.w[0] = I->I[0] * x.w[0] + I->I[3] * x.w[1] + I->I[4] * x.w[2];
    r.w[1] = I->I[3] * x.w[0] + I->I[1] * x.w[1] + I->I[5] * x.w[2];
    r.w[2] = I->I[4] * x.w[0] + I->I[5] * x.w[1] + I->I[2] * x.w[2];
    cross(I->h, x.v, t);
    for (int i = 0; i < 3; ++i) r.w[i] += t[i];
    cross(I->h, x.w, t);
    for (int i = 0; i < 3; ++i) r.v[i] = I->m * x.v[i] - t[i];
    return r;
}

/* ======================================================================== */
/* Functions of a coordinate.                                                */
/* ======================================================================== */
/* SimmSpline coefficients: the Forsythe–Malcolm–Moler cubic spline with
 * third-derivative end conditions, as in opensim-core SimmSpline
 * (SimmSpline::calcCoefficients; third-party, absent from /root/reference).
 * b,c,d have n entries each. */
static void simm_coefficients(int n, const double* x, const double* y,
        double* b, double* c, double* d) {
    if (n < 2) {
        if (n == 1) { b[0] = c[0] = d[0] = 0.0; }
        return;
    }
    if (n < 3) {
        double t = (y[1] - y[0]) / (x[1] - x[0]);
        b[0] = b[1] = t;
        c[0] = c[1] = 0.0;
        d[0] = d[1] = 0.0;
        return;
    }
    int nm1 = n - 1;
    d[0] = x[1] - x[0];
    c[1] = (y[1] - y[0]) / d[0];
    for (int i = 1; i < nm1; ++i) {
        d[i] = x[i + 1] - x[i];
        b[i] = 2.0 * (d[i - 1] + d[i]);
        c[i + 1] = (y[i + 1] - y[i]) / d[i];
        c[i] = c[i + 1] - c[i];
    }
    b[0] = -d[0];
    b[nm1] = -d[n - 2];
    c[0] = 0.0;
    c[nm1] = 0.0;
    if (n > 3) {
        double d1 = c[2] / (x[3] - x[1]) - c[1] / (x[2] - x[0]);
        double d2 = c[nm1 - 1] / (x[nm1] - x[n - 3]) -
                    c[n - 3] / (x[nm1 - 1] - x[n - 4]);
        double d31 = x[3] - x[0];
        double d32 = x[nm1] - x[n - 4];
        /* d(1)**2 and d(n-1)**2 of the FMM routine (SimmSpline.cpp
         * calcCoefficients: _c[0] * _d[0] * _d[0] / d30) */
        c[0] = d1 * d[0] * d[0] / d31;
        c[nm1] = -(d2 * d[n - 2] * d[n - 2]) / d32;
    }
    for (int i = 1; i < n; ++i) {
        double t = d[i - 1] / b[i - 1];
        b[i] -= t * d[i - 1];
        c[i] -= t * c[i - 1];
    }
    c[nm1] /= b[nm1];
    for (int j = 0; j < nm1; ++j) {
        int i = nm1 - j - 1;
        c[i] = (c[i] - d[i] * c[i + 1]) / b[i];
    }
    b[nm1] = (y[nm1] - y[n - 2]) / d[n - 2] + d[n - 2] * (c[n - 2] + 2.0 * c[nm1]);
    for (int i = 0; i < nm1; ++i) {
        b[i] = (y[i + 1] - y[i]) / d[i] - d[i] * (c[i + 1] + 2.0 * c[i]);
        d[i] = (c[i + 1] - c[i]) / d[i];
        c[i] *= 3.0;
    }
    c[nm1] *= 3.0;
    d[nm1] = d[n - 2];
}

/* SimmSpline::interpolate (value, first, second derivative), with linear
 * extrapolation outside the knots. */
static void simm_eval(int n, const double* x, const double* y, const double* b,
        const double* c, const double* d, real t, real* out) {
    if (n == 1) { out[0] = y[0]; out[1] = out[2] = 0.0; return; }
    if (t < x[0]) {
        out[0] = y[0] + (t - x[0]) * b[0]; out[1] = b[0]; out[2] = 0.0; return;
    }
    if (t > x[n - 1]) {
        out[0] = y[n - 1] + (t - x[n - 1]) * b[n - 1];
        out[1] = b[n - 1]; out[2] = 0.0; return;
    }
    int k;
    const double tol = 2e-13; /* SIMM ROUNDOFF_ERROR */
    if (fabs(t - x[0]) <= tol) k = 0;
    else if (fabs(t - x[n - 1]) <= tol) k = n - 1;
    else {
        int i = 0, j = n;
        for (;;) {
            k = (i + j) / 2;
            if (t < x[k]) j = k;
            else if (t > x[k + 1]) i = k;
            else break;
        }
    }
    real dx = t - x[k];
    out[0] = y[k] + dx * (b[k] + dx * (c[k] + dx * d[k]));
    out[1] = b[k] + dx * (2.0 * c[k] + 3.0 * dx * d[k]);
    out[2] = 2.0 * c[k] + 6.0 * dx * d[k];
}

/* ======================================================================== */
/* Context.                                                                  */
/* ======================================================================== */
struct orc_ctx {
    mh_problem P;      /* shallow copy; arrays are deep-copied below       */
    mh_options O;
    int nthreads;
    /* model copies */
    mh_body* bodies; mh_axis* axes; mh_function* funcs; double *kx, *ky;
    double *kb, *kc, *kd;          /* spline coefficients (per knot)       */
    mh_muscle* mus; mh_path_point* pts; mh_actuator* acts; mh_table* tabs;
    double *brk, *coef; mh_external_force* ext;
    mh_variable_info *sinfo, *cinfo; mh_goal* goals; int32_t *gidx, *gcol;
    double* gw;
    int NPC;                /* path-constraint equations per mesh point  */
    mh_path_equation* pc;
    int NEP;                /* endpoint-constraint equations (rows 0..NEP) */
    mh_endpoint_equation* ep;
    uint8_t* sp_ep;         /* detected endpoint sparsity [eq][2 (1 + NP)] */
    /* detected callback sparsity (NULL: block-dense): [output][1 + input],
     * column 0 = time; DAE outputs (NQ + NZ) and path equations */
    uint8_t *sp, *sp_pc;
    /* derived sizes */
    int NQ, NZ, NS, NC, NP; /* NP = per-point inputs excluding time */
    int implicit;           /* MH_DYNAMICS_IMPLICIT                     */
    int NDV;                /* derivative variables per grid point      */
    double acc_lo, acc_hi;  /* implicit multibody acceleration bounds   */
    int NACC;               /* acceleration variables per point (implicit) */
    int NAR;                /* implicit auxiliary residuals per point      */
    int* mus_ider;          /* muscle -> its tendon-force derivative's index
                             * in the derivative block (-1: explicit)     */
    double aux_lo, aux_hi;  /* implicit auxiliary derivative bounds      */
    /* prescribed kinematics (PositionMotion): q, u, udot from a table; the
     * NLP states are the auxiliary states only */
    int presc, kin_table;
    int32_t* kin_col;
    int TQ;                 /* coordinates among the NLP states (0 if prescribed) */
    int NMB;                /* multibody residual rows per point          */
    int SO;                 /* callback output of state s's derivative: s + SO */
    int* mus_act_state;     /* state index of activation (-1)          */
    int* mus_ftn_state;     /* state index of normalized tendon force   */
    int* mus_control;       /* control index of excitation (-1)        */
    int* coord_body;        /* owning body of coordinate               */
    double tau_act, tau_deact; /* DGF static time constants quirk      */
    /* transcription */
    int scheme, N, G, nmesh, interp;
    double* grid;   /* G */
    double* quad;   /* G quadrature coefficients */
    int64_t n, m, nnz;
    int32_t *iRow, *jCol;
    /* mesh-interval shard [ib, ie) (mh_options interval_begin/end): its grid
     * points gk0..gk1 are the only ones evaluated, and g / values receive its
     * rows [row_begin, row_end) / nonzeros [nnz_begin, nnz_end) */
    int ib, ie, gk0, gk1;
    int64_t row_begin, row_end, nnz_begin, nnz_end;
    int fd; double h;
    /* kinematic constraints (CoordinateCouplerConstraint):
     * NKC couplers, NM = NKC multipliers per grid point, NK kinematic rows
     * per mesh point (3 NKC enforcing constraint derivatives, else NKC),
     * NSL = NKC slacks per mesh interval (Hermite-Simpson, enforcing
     * derivatives), OKC / OQC: callback outputs of the kinematic errors /
     * the velocity correction G^T gamma (NQ, when NSL) */
    int NKC, NM, NK, NSL, OKC, OQC, enforce;
    mh_constraint* kcs;
    double mult_lo, mult_hi, kc_lo, kc_hi, vc_lo, vc_hi;
    int NPD;               /* callback inputs per point: NS + NC + NDV + NM */
    /* MH_JACOBIAN_GLOBAL_SEEDS: the seed (color) of every x column */
    int jac_seeds, nseeds;
    int32_t* seed_color;
    /* muscle wrapping (ABI v5): wrap surfaces, PathWrap entries grouped by
     * muscle, each muscle's first entry and count, and the current-path
     * capacity (points + 2 per PathWrap) */
    int NWR, NPW;
    mh_wrap_object* wr;
    mh_path_wrap* pw;
    int *mus_pw_begin, *mus_pw_count;
    int maxcp;
    /* SpringGeneralizedForce elements (ABI v8) */
    int NSPR;
    mh_spring* spr;
    /* MocoParameters (ABI v8): NPAR variables at x[XP..] (the last block,
     * CasOCIterate.h:27-44), bounds, the properties they write
     * (applyParametersToModelProperties, MocoCasOCProblem.h:309,508-515) */
    int NPAR, NPT;
    int64_t XP;
    mh_bounds* par_bounds;
    mh_parameter_target* par_targets;
    int owns_model;   /* 0 for the parameter copies (param_ctx): arrays shared but the parameterized ones */
};

static double* dup_d(const double* p, size_t n) {
    if (!n) return NULL;
    double* r = (double*)malloc(n * sizeof(double));
    memcpy(r, p, n * sizeof(double));
    return r;
}
#define DUP(T, p, n) ((n) ? (T*)memcpy(malloc((size_t)(n) * sizeof(T)), (p), (size_t)(n) * sizeof(T)) : NULL)

void orc_set_threads(orc_ctx* c, int nthreads) { c->nthreads = nthreads < 1 ? 1 : nthreads; }

/* ------------------------------------------------------------------------ */
/* Jacobian structure (block-dense CasOC rule).         */
/* Columns of x: [t0, tf, states(NS x G grid-major), controls(NC x G)].      */
/* ------------------------------------------------------------------------ */
/* MocoParameters applied (applyParametersToModelProperties,
 * MocoCasOCProblem.h:309,508-515): a shallow copy of the context whose
 * parameterized arrays (bodies, actuators, muscles, springs) are its own,
 * every target property set to its parameter's value in x -- parameter
 * `moved` (>= 0) moved by `step` (the finite-difference lanes along a
 * parameter).  Without parameters: the context itself. */
static orc_ctx* param_ctx(const orc_ctx* c, const double* x, int moved, double step) {
    if (c->NPAR <= 0) return (orc_ctx*)c;
    const mh_model* M = &c->P.model;
    orc_ctx* q = (orc_ctx*)malloc(sizeof(orc_ctx));
    *q = *c;
    q->owns_model = 0;
    q->bodies = DUP(mh_body, c->bodies, M->nbodies);
    q->acts = DUP(mh_actuator, c->acts, M->nactuators);
    q->mus = DUP(mh_muscle, c->mus, M->nmuscles);
    q->spr = DUP(mh_spring, c->spr, c->NSPR);
    for (int t = 0; t < c->NPT; ++t) {
        const mh_parameter_target* T = &c->par_targets[t];
        double v = x[c->XP + T->parameter];
        if (T->parameter == moved) v = v + step;
        switch (T->kind) {
        case MH_PARAM_BODY_MASS: q->bodies[T->index].mass = v; break;
        case MH_PARAM_BODY_MASS_CENTER: q->bodies[T->index].com[T->element] = v; break;
        case MH_PARAM_BODY_INERTIA: q->bodies[T->index].inertia[T->element] = v; break;
        case MH_PARAM_SPRING_STIFFNESS: q->spr[T->index].stiffness = v; break;
        case MH_PARAM_SPRING_REST_LENGTH: q->spr[T->index].rest_length = v; break;
        case MH_PARAM_SPRING_VISCOSITY: q->spr[T->index].viscosity = v; break;
        case MH_PARAM_ACTUATOR_OPTIMAL_FORCE: q->acts[T->index].optimal_force = v; break;
        case MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE: q->mus[T->index].max_isometric_force = v; break;
        default: break;
        }
    }
    return q;
}
static void param_ctx_free(const orc_ctx* c, orc_ctx* q) {
    if (q == c || !q) return;
    free(q->bodies); free(q->acts); free(q->mus); free(q->spr);
    free(q);
}
/* finite-difference directions: t0, tf, the NP point inputs, the parameters */
static int ndir(const orc_ctx* c) { return c->NP + 2 + c->NPAR; }

static int64_t col_state(const orc_ctx* c, int k, int s) { return 2 + (int64_t)k * c->NS + s; }
static int64_t col_control(const orc_ctx* c, int k, int j) {
    return 2 + (int64_t)c->NS * c->G + (int64_t)k * c->NC + j;
}
/* Lagrange multipliers (NM x G) and slacks (NSL x mesh-interval midpoints)
 * after the controls, then the "derivatives" variables (implicit mode:
 * generalized accelerations, implicit auxiliary derivatives) -- the sorted
 * key order of CasOCIterate.h:27-44 */
static int64_t col_mult(const orc_ctx* c, int k, int j) {
    return 2 + (int64_t)(c->NS + c->NC) * c->G + (int64_t)k * c->NM + j;
}
static int64_t col_slack(const orc_ctx* c, int i, int l) {
    return 2 + (int64_t)(c->NS + c->NC + c->NM) * c->G + (int64_t)i * c->NSL + l;
}
static int64_t col_deriv(const orc_ctx* c, int k, int j) {
    return 2 + (int64_t)(c->NS + c->NC + c->NM) * c->G + (int64_t)c->NSL * c->N + (int64_t)k * c->NDV + j;
}
/* Column of per-point input j of grid point k: [states, controls,
 * derivatives, multipliers, slacks]; a slack is an input of the mesh
 * interval midpoints only (-1 elsewhere). */
static int64_t col_input(const orc_ctx* c, int k, int j) {
    if (j < c->NS) return col_state(c, k, j);
    j -= c->NS;
    if (j < c->NC) return col_control(c, k, j);
    j -= c->NC;
    if (j < c->NDV) return col_deriv(c, k, j);
    j -= c->NDV;
    if (j < c->NM) return col_mult(c, k, j);
    j -= c->NM;
    if (c->scheme != MH_HERMITE_SIMPSON || k % 2 == 0) return -1;
    return col_slack(c, (k - 1) / 2, j);
}
/* is grid point k a mesh-interval midpoint carrying slacks? */
static int vc_point(const orc_ctx* c, int k) { return c->NSL && c->scheme == MH_HERMITE_SIMPSON && k % 2; }
/* DAE callback outputs: [udot or multibody residual (NQ), zdot (NZ),
 * auxiliary residuals (NAR), kinematic errors (NK)] (CasOCFunction.cpp:
 * 208-230), then the velocity correction (NQ, the VelocityCorrection
 * function of CasOCFunction.cpp:250-291, when there are slacks) */
static int nout(const orc_ctx* c) { return c->NQ + c->NZ + c->NAR + c->NK + (c->NSL ? c->NQ : 0); }
/* residual rows per grid point: multibody residuals (implicit mode), then
 * auxiliary residuals (flattenConstraints, CasOCTranscription.h:290-296) */
static int nres(const orc_ctx* c) { return c->NMB + c->NAR; }
/* callback output behind residual row r of a grid point */
static int res_out(const orc_ctx* c, int r) { return r < c->NMB ? r : c->NQ + c->NZ + (r - c->NMB); }
/* the mesh point that opens interval i (and closes interval i-1) */
static int mesh_point(const orc_ctx* c, int i) { return c->scheme == MH_HERMITE_SIMPSON ? 2 * i : i; }

static int cmp64(const void* a, const void* b) {
    int64_t x = *(const int64_t*)a, y = *(const int64_t*)b;
    return x < y ? -1 : x > y;
}

/* Does callback output o (DAE: sp, path equation: sp_pc) read input j
 * (-1 = time)?  Block-dense (no detection): always. */
static int dep(const uint8_t* sp, int NP, int o, int j) { return !sp || sp[(int64_t)o * (1 + NP) + 1 + j]; }
/* Columns of grid point k that callback output o reads, plus (if s >= 0)
 * the point's own state s (the defects' identity terms), ascending. */
static int point_cols_dep(const orc_ctx* c, const uint8_t* sp, int o, int k, int s, int64_t* out) {
    int n = 0;
    for (int j = 0; j < c->NPD; ++j) {   /* callback inputs (no slacks) */
        if (!(dep(sp, c->NP, o, j) || j == s)) continue;
        out[n++] = col_input(c, k, j);
    }
    return n;
}

/* Emits the sorted column set of every row of interval i, in row order.
 * emit(row_local, cols, ncols). Returns rows per interval. */
typedef void (*row_fn)(void* ud, int64_t row, const int64_t* cols, int ncols);
/* The parameters are inputs of every callback (ContinuousInput.parameters,
 * CasOCProblem.h:132-165): a row that reads a callback output gets the NPAR
 * parameter columns, the last of x, after its sorted columns. */
static int add_param_cols(const orc_ctx* c, int64_t* cols, int n) {
    for (int q = 0; q < c->NPAR; ++q) cols[n++] = c->XP + q;
    return n;
}
/* Multibody residual rows of grid point k (implicit mode): the callback
 * output depends on every input of the point and on the time. */
static int64_t residual_rows(const orc_ctx* c, int k, int64_t row, row_fn emit, void* ud,
        int64_t* cols) {
    for (int r = 0; r < nres(c); ++r) {
        int n = 0, o = res_out(c, r);
        if (dep(c->sp, c->NP, o, -1)) { cols[n++] = 0; cols[n++] = 1; }
        n += point_cols_dep(c, c->sp, o, k, -1, cols + n);
        qsort(cols, (size_t)n, sizeof(int64_t), cmp64);   /* multipliers precede derivatives in x */
        n = add_param_cols(c, cols, n);
        emit(ud, row++, cols, n);
    }
    return row;
}
/* Path-constraint rows of mesh grid point k: like the residuals, one
 * block-dense row per equation over time and the point's inputs (the path
 * function's Jacobian with sparsity detection "none", CasOCFunction.cpp:
 * 25-105), evaluated at mesh points only (CasOCTranscription.cpp:419-433). */
static int64_t path_rows(const orc_ctx* c, int k, int64_t row, row_fn emit, void* ud,
        int64_t* cols) {
    for (int e = 0; e < c->NPC; ++e) {
        int n = 0;
        if (dep(c->sp_pc, c->NP, e, -1)) { cols[n++] = 0; cols[n++] = 1; }
        n += point_cols_dep(c, c->sp_pc, e, k, -1, cols + n);
        qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
        n = add_param_cols(c, cols, n);
        emit(ud, row++, cols, n);
    }
    return row;
}
/* Kinematic-constraint rows of mesh grid point k (CasOCTranscription.cpp:
 * 298-309, 355-363/388-394: the errors are outputs of the mesh points'
 * multibody callback): block-dense over time and the point's callback
 * inputs; placed before the path rows (flattenConstraints,
 * CasOCTranscription.h:283-289). */
static int64_t kc_rows(const orc_ctx* c, int k, int64_t row, row_fn emit, void* ud, int64_t* cols) {
    for (int r = 0; r < c->NK; ++r) {
        int n = 0;
        cols[n++] = 0; cols[n++] = 1;
        n += point_cols_dep(c, NULL, 0, k, -1, cols + n);
        qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
        n = add_param_cols(c, cols, n);
        emit(ud, row++, cols, n);
    }
    return row;
}
/* Implicit mode: the speed rows (NQ <= s < 2NQ) have udot = the derivative
 * variable, a direct MX expression (CasOCTranscription.cpp:339-341), so they
 * depend on the point's own state s and derivative s - NQ only. */
static int speed_row_sparse(const orc_ctx* c, int s) { return c->NACC && s >= c->TQ && s < 2 * c->TQ; }

static void interval_rows(const orc_ctx* c, int i, int64_t row0, row_fn emit, void* ud) {
    int NQ = c->TQ, NS = c->NS, NC = c->NC;   /* NQ: coordinates among the states */
    int64_t* cols = (int64_t*)malloc(sizeof(int64_t) * (size_t)(3 * c->NP + 8 + c->NPAR));
    int64_t row = row0;
    if (c->scheme == MH_HERMITE_SIMPSON) {
        int ki = 2 * i, km = 2 * i + 1, kp = 2 * i + 2;
        /* flattenConstraints: the mesh point's kinematic and path rows, then
         * the residuals of the interval's grid points, then its defects
         * (CasOCTranscription.h:283-300) */
        row = kc_rows(c, ki, row, emit, ud, cols);
        row = path_rows(c, ki, row, emit, ud, cols);
        row = residual_rows(c, ki, row, emit, ud, cols);
        row = residual_rows(c, km, row, emit, ud, cols);
        /* Hermite rows, then Simpson rows (CasOCHermiteSimpson.cpp:79-84). */
        for (int pass = 0; pass < 2; ++pass) {
            for (int s = 0; s < NS; ++s) {
                int n = 0;
                cols[n++] = 0; cols[n++] = 1;
                if (s < NQ) {
                    /* qdot = u is not a callback output: exact dependence. */
                    if (pass == 0) {
                        cols[n++] = col_state(c, km, s);
                        cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                        cols[n++] = col_state(c, ki, NQ + s); cols[n++] = col_state(c, kp, NQ + s);
                    } else if (c->NSL) {
                        /* qdot at the midpoint = u + G^T gamma: the velocity
                         * correction function reads the midpoint's q, u, the
                         * interval's slacks and the parameters (block-dense,
                         * CasOCTranscription.cpp:316-333) */
                        cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                        cols[n++] = col_state(c, ki, NQ + s); cols[n++] = col_state(c, kp, NQ + s);
                        for (int j = 0; j < 2 * NQ; ++j) cols[n++] = col_state(c, km, j);
                        for (int l = 0; l < c->NSL; ++l) cols[n++] = col_slack(c, i, l);
                        qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
                        n = add_param_cols(c, cols, n);
                        emit(ud, row++, cols, n);
                        continue;
                    } else {
                        cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                        cols[n++] = col_state(c, ki, NQ + s); cols[n++] = col_state(c, km, NQ + s);
                        cols[n++] = col_state(c, kp, NQ + s);
                    }
                } else if (speed_row_sparse(c, s)) {
                    int j = s - NQ;
                    if (pass == 0) {
                        cols[n++] = col_state(c, km, s);
                        cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                        cols[n++] = col_deriv(c, ki, j); cols[n++] = col_deriv(c, kp, j);
                    } else {
                        cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                        cols[n++] = col_deriv(c, ki, j); cols[n++] = col_deriv(c, km, j);
                        cols[n++] = col_deriv(c, kp, j);
                    }
                } else {
                    /* callback output s + SO (explicit: udot / zdot;
                     * implicit / prescribed: zdot after the NQ residuals) */
                    int o = s + c->SO;
                    if (pass == 0) {
                        cols[n++] = col_state(c, km, s);
                        n += point_cols_dep(c, c->sp, o, ki, s, cols + n);
                        n += point_cols_dep(c, c->sp, o, kp, s, cols + n);
                    } else {
                        n += point_cols_dep(c, c->sp, o, ki, s, cols + n);
                        n += point_cols_dep(c, c->sp, o, km, -1, cols + n);
                        n += point_cols_dep(c, c->sp, o, kp, s, cols + n);
                    }
                    qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
                    n = add_param_cols(c, cols, n);
                    emit(ud, row++, cols, n);
                    continue;
                }
                qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
                emit(ud, row++, cols, n);
            }
        }
        if (c->interp) {
            for (int j = 0; j < NC; ++j) {
                cols[0] = col_control(c, ki, j); cols[1] = col_control(c, km, j);
                cols[2] = col_control(c, kp, j);
                emit(ud, row++, cols, 3);
            }
        }
    } else { /* trapezoidal (CasOCTrapezoidal.cpp:43-59) */
        int ki = i, kp = i + 1;
        row = kc_rows(c, ki, row, emit, ud, cols);
        row = path_rows(c, ki, row, emit, ud, cols);
        row = residual_rows(c, ki, row, emit, ud, cols);
        for (int s = 0; s < NS; ++s) {
            int n = 0;
            cols[n++] = 0; cols[n++] = 1;
            if (s < NQ) {
                cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                cols[n++] = col_state(c, ki, NQ + s); cols[n++] = col_state(c, kp, NQ + s);
            } else if (speed_row_sparse(c, s)) {
                cols[n++] = col_state(c, ki, s); cols[n++] = col_state(c, kp, s);
                cols[n++] = col_deriv(c, ki, s - NQ); cols[n++] = col_deriv(c, kp, s - NQ);
            } else {
                n += point_cols_dep(c, c->sp, s + c->SO, ki, s, cols + n);
                n += point_cols_dep(c, c->sp, s + c->SO, kp, s, cols + n);
                qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
                n = add_param_cols(c, cols, n);
                emit(ud, row++, cols, n);
                continue;
            }
            qsort(cols, (size_t)n, sizeof(int64_t), cmp64);
            emit(ud, row++, cols, n);
        }
    }
    free(cols);
}

typedef struct { int64_t count; int32_t *ir, *jc; } emit_state;
static void emit_count(void* ud, int64_t row, const int64_t* cols, int n) {
    (void)row; (void)cols;
    ((emit_state*)ud)->count += n;
}
static void emit_fill(void* ud, int64_t row, const int64_t* cols, int n) {
    emit_state* e = (emit_state*)ud;
    for (int k = 0; k < n; ++k) {
        e->ir[e->count] = (int32_t)row;
        e->jc[e->count] = (int32_t)cols[k];
        ++e->count;
    }
}
static int rows_per_interval(const orc_ctx* c) {
    return c->NK + c->NPC + 2 * c->NS * (c->scheme == MH_HERMITE_SIMPSON) + c->NS * (c->scheme == MH_TRAPEZOIDAL) +
           (c->scheme == MH_HERMITE_SIMPSON && c->interp ? c->NC : 0) +
           nres(c) * (c->scheme == MH_HERMITE_SIMPSON ? 2 : 1);
}
/* after all intervals: the final mesh point's path rows (the last pass of
 * the mesh loop), then the final grid point's residual rows
 * (CasOCTranscription.h:286-308) */
static int ntail(const orc_ctx* c) { return c->NK + c->NPC + nres(c); }
static void tail_rows(const orc_ctx* c, int64_t row0, row_fn emit, void* ud) {
    int64_t* cols = (int64_t*)malloc(sizeof(int64_t) * (size_t)(c->NP + 4 + c->NPAR));
    row0 = kc_rows(c, c->G - 1, row0, emit, ud, cols);
    row0 = path_rows(c, c->G - 1, row0, emit, ud, cols);
    residual_rows(c, c->G - 1, row0, emit, ud, cols);
    free(cols);
}

/* Endpoint-constraint rows (CasOCTranscription.h:283-285: first in g).  The
 * Endpoint callback's inputs (CasOCFunction.h:167-240) are [initial_time,
 * initial point inputs, final_time, final point inputs] (the point inputs
 * in this build's lane order: states, controls, derivatives, multipliers;
 * no parameters here; the integral input is a constant NaN when the goal has
 * no integrand, CasOCTranscription.cpp:562-564).  Subset index si of that
 * vector -> NLP column. */
static int ep_width(const orc_ctx* c) { return 2 * (1 + c->NP); }
/* ... and then the parameters (inputs 2 W + q; the Endpoint callback's
 * `parameters` input, CasOCTranscription.cpp:574-580) */
static int64_t ep_col(const orc_ctx* c, int si) {
    if (si >= ep_width(c)) return c->XP + (si - ep_width(c));
    int W = 1 + c->NP;
    int pt = si / W, j = si % W - 1;
    if (j < 0) return pt;                 /* initial_time: 0, final_time: 1 */
    int k = pt ? c->G - 1 : 0;
    if (j < c->NS) return col_state(c, k, j);
    if (j < c->NS + c->NC) return col_control(c, k, j - c->NS);
    if (j < c->NS + c->NC + c->NDV) return col_deriv(c, k, j - c->NS - c->NC);
    return col_mult(c, k, j - c->NS - c->NC - c->NDV);
}
/* Columns of endpoint row e, ascending: every input (block-dense) or the
 * detected ones; si[] receives the matching subset indices. */
static int ep_row_cols(const orc_ctx* c, int e, int64_t* cols, int* si) {
    int WE = ep_width(c), n = 0;
    for (int i = 0; i < WE; ++i)
        if (!c->sp_ep || c->sp_ep[(int64_t)e * WE + i]) { cols[n] = ep_col(c, i); si[n] = i; ++n; }
    for (int q = 0; q < c->NPAR; ++q) { cols[n] = ep_col(c, WE + q); si[n] = WE + q; ++n; }
    /* insertion sort by column (the initial point's block and the final
     * point's interleave per variable kind) */
    for (int a = 1; a < n; ++a) {
        int64_t cv = cols[a]; int sv = si[a]; int b = a - 1;
        while (b >= 0 && cols[b] > cv) { cols[b + 1] = cols[b]; si[b + 1] = si[b]; --b; }
        cols[b + 1] = cv; si[b + 1] = sv;
    }
    return n;
}
static void endpoint_rows(const orc_ctx* c, row_fn emit, void* ud) {
    int64_t* cols = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ep_width(c) + 1 + c->NPAR));
    int* si = (int*)malloc(sizeof(int) * (size_t)(ep_width(c) + 1 + c->NPAR));
    for (int e = 0; e < c->NEP; ++e) emit(ud, e, cols, ep_row_cols(c, e, cols, si));
    free(cols); free(si);
}
/* The endpoint subset vector of iterate x. */
static void ep_gather(const orc_ctx* c, const double* x, double* in) {
    int W = 1 + c->NP;
    for (int pt = 0; pt < 2; ++pt)
        for (int i = 0; i < W; ++i) in[pt * W + i] = x[ep_col(c, pt * W + i)];
    for (int q = 0; q < c->NPAR; ++q) in[2 * W + q] = x[c->XP + q];   /* the parameters */
}
/* MocoInitialActivationGoal::calcGoalImpl in endpoint-constraint mode
 * (MocoInitialActivationGoal.cpp:41-58): initial excitation - initial
 * activation. */
static double endpoint_value(const orc_ctx* c, int e, const double* in) {
    const mh_endpoint_equation* E = &c->ep[e];
    return in[1 + c->NS + E->index_a] - in[1 + E->index_b];
}

#ifndef ORACLE_COUNTING
static int detect_sparsity(orc_ctx* c, const mh_options* o);
#endif
static int sharded(const orc_ctx* c);

/* ColPack's SMALLEST_LAST column ordering as tropter requests it
 * (GraphColoring.cpp:91-94: GenerateSeedJacobian_unmanaged(..., "SMALLEST_LAST",
 * "COLUMN_PARTIAL_DISTANCE_TWO")), restated from Matula & Beck's published
 * smallest-last algorithm on the column intersection graph (ColPack itself is
 * not in the reference tree; its tie-breaking is this restatement's, the rule
 * include/mocohip.h gives for mh_color_jacobian_ordered):
 *   adjacency  columns a != b sharing a row; deg = distinct adjacent columns;
 *   buckets    one list per degree, columns appended in index order;
 *   step       the last column of the lowest non-empty bucket is removed and
 *              written at the last free slot of the order; every adjacent
 *              column still present (rows of the removed column in nonzero
 *              order, each row's columns in nonzero order, each column once)
 *              leaves its bucket -- the bucket's last column moves into its
 *              slot -- and is appended to the bucket one degree lower.
 * ord[n] receives the coloring order. */
static void smallest_last(int64_t ncols, const int64_t* roff, const int64_t* coff, const int32_t* rcol,
        const int32_t* crow, int32_t* ord) {
    int64_t* deg = (int64_t*)calloc((size_t)ncols + 1, sizeof(int64_t));
    int64_t* seen = (int64_t*)malloc(sizeof(int64_t) * ((size_t)ncols + 1));
    int64_t* slot = (int64_t*)malloc(sizeof(int64_t) * ((size_t)ncols + 1));
    char* gone = (char*)calloc((size_t)ncols + 1, 1);
    int64_t maxd = 0;
    for (int64_t v = 0; v < ncols; ++v) seen[v] = -1;
    for (int64_t v = 0; v < ncols; ++v) {
        seen[v] = v;
        for (int64_t q = coff[v]; q < coff[v + 1]; ++q) {
            const int32_t r = crow[q];
            for (int64_t t = roff[r]; t < roff[r + 1]; ++t)
                if (seen[rcol[t]] != v) { seen[rcol[t]] = v; deg[v]++; }
        }
        if (deg[v] > maxd) maxd = deg[v];
    }
    /* bucket d: the columns of current degree d, list[bstart[d] .. + bsize[d]) of a
     * per-degree array sized by how many columns start at or above d */
    int64_t** list = (int64_t**)calloc((size_t)maxd + 1, sizeof(int64_t*));
    int64_t* bsize = (int64_t*)calloc((size_t)maxd + 1, sizeof(int64_t));
    int64_t* cap = (int64_t*)calloc((size_t)maxd + 2, sizeof(int64_t));
    for (int64_t v = 0; v < ncols; ++v) cap[deg[v]]++;
    for (int64_t d = maxd; d > 0; --d) cap[d - 1] += cap[d];   /* a column only moves down */
    for (int64_t d = 0; d <= maxd; ++d) list[d] = (int64_t*)malloc(sizeof(int64_t) * (size_t)(cap[d] + 1));
    for (int64_t v = 0; v < ncols; ++v) { slot[v] = bsize[deg[v]]; list[deg[v]][bsize[deg[v]]++] = v; }
    for (int64_t v = 0; v < ncols; ++v) seen[v] = -1;
    int64_t low = 0;
    for (int64_t i = 0; i < ncols; ++i) {
        while (bsize[low] == 0) ++low;
        const int64_t u = list[low][--bsize[low]];
        gone[u] = 1;
        ord[ncols - 1 - i] = (int32_t)u;
        seen[u] = u;
        for (int64_t q = coff[u]; q < coff[u + 1]; ++q) {
            const int32_t r = crow[q];
            for (int64_t t = roff[r]; t < roff[r + 1]; ++t) {
                const int64_t w = rcol[t];
                if (gone[w] || seen[w] == u) continue;
                seen[w] = u;
                const int64_t d = deg[w];
                const int64_t moved = list[d][bsize[d] - 1];
                list[d][slot[w]] = moved;
                slot[moved] = slot[w];
                bsize[d]--;
                deg[w] = d - 1;
                slot[w] = bsize[d - 1];
                list[d - 1][bsize[d - 1]++] = w;
            }
        }
        if (low > 0) low--;
    }
    for (int64_t d = 0; d <= maxd; ++d) free(list[d]);
    free(list); free(bsize); free(cap); free(deg); free(seen); free(slot); free(gone);
}

/* Column partial distance-2 coloring: the smallest color no column sharing
 * a row already has (ColPack's COLUMN_PARTIAL_DISTANCE_TWO, GraphColoring.cpp:
 * 91-94), the columns visited in natural order (MH_COLORING_NATURAL) or in
 * the SMALLEST_LAST order above.  Returns the color count. */
static int color_columns(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow,
        const int32_t* jCol, int32_t* color, int order) {
    int64_t* roff = (int64_t*)calloc((size_t)nrows + 1, sizeof(int64_t));
    int64_t* coff = (int64_t*)calloc((size_t)ncols + 1, sizeof(int64_t));
    int32_t* rcol = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz + 1));
    int32_t* crow = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz + 1));
    int64_t* rp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nrows + 1));
    int64_t* cp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncols + 1));
    int64_t* stamp = (int64_t*)malloc(sizeof(int64_t) * (size_t)(ncols + 1));
    for (int64_t e = 0; e < nnz; ++e) { ++roff[iRow[e] + 1]; ++coff[jCol[e] + 1]; }
    for (int64_t r = 0; r < nrows; ++r) roff[r + 1] += roff[r];
    for (int64_t j = 0; j < ncols; ++j) coff[j + 1] += coff[j];
    memcpy(rp, roff, sizeof(int64_t) * (size_t)nrows);
    memcpy(cp, coff, sizeof(int64_t) * (size_t)ncols);
    for (int64_t e = 0; e < nnz; ++e) { rcol[rp[iRow[e]]++] = jCol[e]; crow[cp[jCol[e]]++] = iRow[e]; }
    int32_t* ord = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ncols + 1));
    for (int64_t j = 0; j < ncols; ++j) ord[j] = (int32_t)j;
    if (order == MH_COLORING_SMALLEST_LAST) smallest_last(ncols, roff, coff, rcol, crow, ord);
    int ncolors = 0;
    for (int64_t j = 0; j < ncols; ++j) color[j] = -1;
    for (int64_t jj = 0; jj < ncols; ++jj) {
        const int64_t j = ord[jj];
        for (int64_t q = coff[j]; q < coff[j + 1]; ++q)
            for (int64_t t = roff[crow[q]]; t < roff[crow[q] + 1]; ++t)
                if (color[rcol[t]] >= 0) stamp[color[rcol[t]]] = j;
        int k = 0;
        while (k < ncolors && stamp[k] == j) ++k;
        if (k == ncolors) stamp[ncolors++] = -1;
        color[j] = k;
    }
    free(roff); free(coff); free(rcol); free(crow); free(rp); free(cp); free(stamp); free(ord);
    return ncolors;
}

int orc_color_jacobian(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow, const int32_t* jCol,
        int32_t order, int32_t* color, int32_t* ncolors) {
    for (int64_t e = 0; e < nnz; ++e)
        if (iRow[e] < 0 || iRow[e] >= nrows || jCol[e] < 0 || jCol[e] >= ncols)
            return fail(MH_ERR_INVALID, "index out of range");
    if (order != MH_COLORING_SMALLEST_LAST && order != MH_COLORING_NATURAL)
        return fail(MH_ERR_INVALID, "unknown coloring order %d", order);
    *ncolors = color_columns(nrows, ncols, nnz, iRow, jCol, color, order);
    return MH_OK;
}

int orc_create(const mh_problem* p, const mh_options* o, orc_ctx** out) {
    if (!p || !o || !out) return fail(MH_ERR_INVALID, "null argument");
    const mh_model* M = &p->model;
    if (M->nq <= 0 && M->nmuscles <= 0) return fail(MH_ERR_INVALID, "empty model");
    if (o->num_mesh_intervals < 1) return fail(MH_ERR_INVALID, "num_mesh_intervals must be >= 1");
    orc_ctx* c = (orc_ctx*)calloc(1, sizeof(orc_ctx));
    c->P = *p;
    c->O = *o;
    c->nthreads = 1;
    c->bodies = DUP(mh_body, M->bodies, M->nbodies);
    c->axes = DUP(mh_axis, M->axes, M->naxes);
    c->funcs = DUP(mh_function, M->functions, M->nfunctions);
    c->kx = dup_d(M->knot_x, (size_t)M->nknots);
    c->ky = dup_d(M->knot_y, (size_t)M->nknots);
    c->mus = DUP(mh_muscle, M->muscles, M->nmuscles);
    c->pts = DUP(mh_path_point, M->points, M->npoints);
    c->acts = DUP(mh_actuator, M->actuators, M->nactuators);
    c->tabs = DUP(mh_table, M->tables, M->ntables);
    c->brk = dup_d(M->table_breaks, (size_t)M->nbreaks);
    c->coef = dup_d(M->table_coefs, (size_t)M->ncoefs);
    c->ext = DUP(mh_external_force, M->external, M->nexternal);
    /* SpringGeneralizedForce elements and MocoParameters (ABI v8) */
    c->NSPR = M->nsprings;
    c->spr = DUP(mh_spring, M->springs, M->nsprings);
    c->NPAR = p->nparameters;
    c->NPT = p->nparameter_targets;
    c->par_bounds = DUP(mh_bounds, p->parameter_bounds, p->nparameters);
    c->par_targets = DUP(mh_parameter_target, p->parameter_targets, p->nparameter_targets);
    c->owns_model = 1;
    if (c->NSPR < 0 || (c->NSPR > 0 && !M->springs) || c->NPAR < 0 || c->NPT < 0 ||
            (c->NPAR > 0 && !p->parameter_bounds) || (c->NPT > 0 && !p->parameter_targets)) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "bad springs / parameters");
    }
    for (int i = 0; i < c->NSPR; ++i)
        if (c->spr[i].coord < 0 || c->spr[i].coord >= M->nq) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "spring %d: bad coordinate", i);
        }
    for (int t = 0; t < c->NPT; ++t) {
        const mh_parameter_target* T = &c->par_targets[t];
        int count = 0, elems = 1;
        switch (T->kind) {
        case MH_PARAM_BODY_MASS: count = M->nbodies; break;
        case MH_PARAM_BODY_MASS_CENTER: count = M->nbodies; elems = 3; break;
        case MH_PARAM_BODY_INERTIA: count = M->nbodies; elems = 6; break;
        case MH_PARAM_SPRING_STIFFNESS: case MH_PARAM_SPRING_REST_LENGTH: case MH_PARAM_SPRING_VISCOSITY:
            count = M->nsprings; break;
        case MH_PARAM_ACTUATOR_OPTIMAL_FORCE: count = M->nactuators; break;
        case MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE: count = M->nmuscles; break;
        default: orc_destroy(c); return fail(MH_ERR_UNSUPPORTED, "parameter target %d: kind %d", t, T->kind);
        }
        if (T->parameter < 0 || T->parameter >= c->NPAR || T->index < 0 || T->index >= count ||
                T->element < 0 || T->element >= elems ||
                (T->kind == MH_PARAM_ACTUATOR_OPTIMAL_FORCE && M->actuators[T->index].kind != MH_ACT_COORDINATE)) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "parameter target %d: bad parameter / index / element", t);
        }
    }
    c->goals = DUP(mh_goal, p->goals, p->ngoals);
    c->gidx = DUP(int32_t, p->goal_index, p->nterms);
    c->gcol = DUP(int32_t, p->goal_column, p->nterms);
    c->gw = dup_d(p->goal_weight, (size_t)p->nterms);
    c->NPC = p->npath;
    c->pc = DUP(mh_path_equation, p->path, p->npath);
    if (p->npath < 0 || (p->npath > 0 && !p->path)) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "bad path constraints");
    }
    c->NEP = p->nendpoint;
    if (p->nendpoint < 0 || (p->nendpoint > 0 && !p->endpoint)) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "bad endpoint constraints");
    }
    c->ep = DUP(mh_endpoint_equation, p->endpoint, p->nendpoint);

    /* spline coefficients */
    c->kb = (double*)calloc((size_t)M->nknots + 1, sizeof(double));
    c->kc = (double*)calloc((size_t)M->nknots + 1, sizeof(double));
    c->kd = (double*)calloc((size_t)M->nknots + 1, sizeof(double));
    for (int f = 0; f < M->nfunctions; ++f) {
        const mh_function* F = &c->funcs[f];
        if (F->kind == MH_FN_SIMMSPLINE) {
            if (F->knot_count < 1 || F->knot_begin < 0 || F->knot_begin + F->knot_count > M->nknots) {
                orc_destroy(c);
                return fail(MH_ERR_INVALID, "function %d: bad knots", f);
            }
            int b0 = F->knot_begin;
            simm_coefficients(F->knot_count, c->kx + b0, c->ky + b0, c->kb + b0, c->kc + b0, c->kd + b0);
        }
    }

    /* state layout (Simbody Y order, MocoUtilities.cpp:495-528) */
    c->NQ = M->nq;
    c->mus_act_state = (int*)malloc(sizeof(int) * (size_t)(M->nmuscles + 1));
    c->mus_ftn_state = (int*)malloc(sizeof(int) * (size_t)(M->nmuscles + 1));
    c->mus_control = (int*)malloc(sizeof(int) * (size_t)(M->nmuscles + 1));
    int z = 2 * c->NQ;
    c->tau_act = c->tau_deact = NAN;
    for (int im = 0; im < M->nmuscles; ++im) {
        const mh_muscle* mu = &c->mus[im];
        c->mus_act_state[im] = mu->ignore_activation_dynamics ? -1 : z++;
        c->mus_ftn_state[im] = mu->ignore_tendon_compliance ? -1 : z++;
        c->mus_control[im] = -1;
        /* DeGrooteFregly2016Muscle.cpp:194-195: the activation time constants
         * are function-level statics, fixed by the first muscle evaluated. */
        if (!mu->ignore_activation_dynamics && isnan(c->tau_act)) {
            c->tau_act = mu->activation_time_constant;
            c->tau_deact = mu->deactivation_time_constant;
        }
    }
    c->NZ = z - 2 * c->NQ;
    c->presc = p->prescribed_kinematics != 0;
    c->kin_table = p->kinematics_table;
    c->NS = c->presc ? c->NZ : z;       /* NLP states */
    c->TQ = c->presc ? 0 : c->NQ;
    c->SO = c->presc ? c->NQ : -c->NQ;
    c->NC = M->nactuators;
    c->implicit = o->multibody_dynamics_mode == MH_DYNAMICS_IMPLICIT;
    if (o->multibody_dynamics_mode != MH_DYNAMICS_EXPLICIT && !c->implicit) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "unknown multibody dynamics mode %d", o->multibody_dynamics_mode);
    }
    /* derivative variables: accelerations, then the implicit auxiliary
     * derivatives in component order (MocoCasOCProblem.cpp:85-94,
     * MocoCasOCProblem.h:605-620) */
    if (c->presc && !c->implicit) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "Prescribed kinematics (PositionMotion) requires implicit dynamics mode.");
    }
    c->NACC = c->implicit && !c->presc ? c->NQ : 0;
    c->NMB = c->implicit ? c->NQ : 0;
    if (c->presc) {
        if (p->kinematics_table < 0 || p->kinematics_table >= M->ntables || !p->kinematics_column) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "bad kinematics table");
        }
        c->kin_col = DUP(int32_t, p->kinematics_column, c->NQ);
        for (int j = 0; j < c->NQ; ++j)
            if (c->kin_col[j] < 0 || c->kin_col[j] >= c->tabs[c->kin_table].ncol) {
                orc_destroy(c);
                return fail(MH_ERR_INVALID, "kinematics column %d out of range", j);
            }
    }
    c->mus_ider = (int*)malloc(sizeof(int) * (size_t)(M->nmuscles + 1));
    c->NAR = 0;
    for (int im = 0; im < M->nmuscles; ++im) {
        const mh_muscle* mu = &c->mus[im];
        c->mus_ider[im] = (mu->tendon_dynamics_implicit && !mu->ignore_tendon_compliance)
                ? c->NACC + c->NAR++ : -1;
    }
    c->NDV = c->NACC + c->NAR;
    c->aux_lo = -1000.0; c->aux_hi = 1000.0;
    if (o->implicit_aux_bounds[0] != 0.0 || o->implicit_aux_bounds[1] != 0.0) {
        c->aux_lo = o->implicit_aux_bounds[0];
        c->aux_hi = o->implicit_aux_bounds[1];
    }
    c->acc_lo = -1000.0; c->acc_hi = 1000.0;
    if (o->implicit_accel_bounds[0] != 0.0 || o->implicit_accel_bounds[1] != 0.0) {
        c->acc_lo = o->implicit_accel_bounds[0];
        c->acc_hi = o->implicit_accel_bounds[1];
    }
    /* kinematic constraints (MocoCasOCProblem.cpp:96-215: one multiplier per
     * holonomic equation and, enforcing derivatives, one slack "gamma" per
     * multiplier; MocoProblemRep.cpp:150-215 for the bounds) */
    c->NKC = M->nconstraints;
    if (c->NKC < 0 || (c->NKC > 0 && !M->constraints)) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "bad kinematic constraints");
    }
    c->kcs = DUP(mh_constraint, M->constraints, c->NKC);
    /* wrap surfaces and PathWraps (grouped by muscle, in path order) */
    c->NWR = M->nwraps;
    c->NPW = M->npathwraps;
    if (c->NWR < 0 || c->NPW < 0 || (c->NWR > 0 && !M->wraps) || (c->NPW > 0 && !M->pathwraps)) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "bad wrap objects");
    }
    c->wr = DUP(mh_wrap_object, M->wraps, c->NWR);
    c->pw = DUP(mh_path_wrap, M->pathwraps, c->NPW);
    c->mus_pw_begin = (int*)calloc((size_t)M->nmuscles + 1, sizeof(int));
    c->mus_pw_count = (int*)calloc((size_t)M->nmuscles + 1, sizeof(int));
    for (int i = 0; i < c->NWR; ++i) {
        const mh_wrap_object* W = &c->wr[i];
        if (W->kind != MH_WRAP_CYLINDER || W->body < -1 || W->body >= M->nbodies || !(W->radius > 0.0) ||
                W->wrap_axis < 0 || W->wrap_axis > 1 || W->wrap_sign < -1 || W->wrap_sign > 1) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "wrap object %d: bad kind/body/radius/quadrant", i);
        }
    }
    for (int k = 0; k < c->NPW; ++k) {
        const mh_path_wrap* W = &c->pw[k];
        if (W->muscle < 0 || W->muscle >= M->nmuscles || W->wrap < 0 || W->wrap >= c->NWR ||
                (k > 0 && W->muscle < c->pw[k - 1].muscle)) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "path wrap %d: bad muscle/wrap or not grouped by muscle", k);
        }
        if (c->mus_pw_count[W->muscle]++ == 0) c->mus_pw_begin[W->muscle] = k;
        if (c->mus_pw_count[W->muscle] > 8) {   /* as the device (mh_create) */
            orc_destroy(c);
            return fail(MH_ERR_UNSUPPORTED, "muscle %d: more than 8 PathWraps", W->muscle);
        }
    }
    c->maxcp = 1;
    for (int im = 0; im < M->nmuscles; ++im) {
        int cap = M->muscles[im].point_count + 2 * c->mus_pw_count[im];
        if (cap > c->maxcp) c->maxcp = cap;
    }
    for (int i = 0; i < c->NKC; ++i) {
        const mh_constraint* K = &c->kcs[i];
        int f = K->func;
        if (K->kind != MH_KC_COORDINATE_COUPLER || f < 0 || f >= M->nfunctions ||
                c->funcs[f].kind == MH_FN_CONSTANT || c->funcs[f].coord < 0 || c->funcs[f].coord >= c->NQ ||
                K->dependent < 0 || K->dependent >= c->NQ || K->dependent == c->funcs[f].coord) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "kinematic constraint %d: bad kind/function/coordinate", i);
        }
    }
    /* with prescribed kinematics the constraints keep their multipliers
     * (constraint forces in the residual) but no kinematic rows and no
     * slacks: the motion is assumed to obey them (CasOCProblem.h:508-521,
     * MocoCasOCProblem.h:664-676, CasOCTranscription.cpp:316-318) */
    if (c->NKC && !c->presc && (p->nendpoint > 0 || o->sparsity_detection != MH_SPARSITY_NONE)) {
        orc_destroy(c);
        return fail(MH_ERR_UNSUPPORTED, "kinematic constraints (without prescribed kinematics) with "
                    "endpoint constraints or sparsity detection");
    }
    if (o->minimize_lagrange_multipliers && !c->NKC) {   /* MocoCasOCProblem.cpp:101-107 */
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "Solver property 'minimize_lagrange_multipliers' was enabled but no "
                    "enabled kinematic constraints exist in the model.");
    }
    if (o->minimize_lagrange_multipliers) {
        /* the multiplier term (CasOCTranscription.cpp:513-521) as one more
         * goal, one term per multiplier */
        int ng = c->P.ngoals, nt = c->P.nterms;
        c->goals = (mh_goal*)realloc(c->goals, sizeof(mh_goal) * (size_t)(ng + 1));
        c->gidx = (int32_t*)realloc(c->gidx, sizeof(int32_t) * (size_t)(nt + c->NKC));
        c->gcol = (int32_t*)realloc(c->gcol, sizeof(int32_t) * (size_t)(nt + c->NKC));
        c->gw = (double*)realloc(c->gw, sizeof(double) * (size_t)(nt + c->NKC));
        mh_goal G;
        memset(&G, 0, sizeof G);
        G.kind = MH_GOAL_LAGRANGE_MULTIPLIERS;
        G.term_begin = nt;
        G.term_count = c->NKC;
        G.weight = o->lagrange_multiplier_weight != 0.0 ? o->lagrange_multiplier_weight : 1.0;
        c->goals[ng] = G;
        for (int j = 0; j < c->NKC; ++j) { c->gidx[nt + j] = j; c->gcol[nt + j] = 0; c->gw[nt + j] = 1.0; }
        c->P.ngoals = ng + 1;
        c->P.nterms = nt + c->NKC;
    }
    c->enforce = !o->ignore_constraint_derivatives;
    c->NM = c->NKC;
    c->NK = c->presc ? 0 : (c->enforce ? 3 * c->NKC : c->NKC);
    c->NSL = !c->presc && c->enforce && o->transcription == MH_HERMITE_SIMPSON ? c->NKC : 0;
    c->OKC = c->NQ + c->NZ + c->NAR;
    c->OQC = c->OKC + c->NK;
    c->mult_lo = -1000.0; c->mult_hi = 1000.0;
    if (!isnan(p->multiplier_bounds.lower) || !isnan(p->multiplier_bounds.upper)) {
        c->mult_lo = p->multiplier_bounds.lower; c->mult_hi = p->multiplier_bounds.upper;
    }
    c->kc_lo = 0.0; c->kc_hi = 0.0;
    if (!isnan(p->kinematic_constraint_bounds.lower) || !isnan(p->kinematic_constraint_bounds.upper)) {
        c->kc_lo = p->kinematic_constraint_bounds.lower; c->kc_hi = p->kinematic_constraint_bounds.upper;
    }
    c->vc_lo = -0.1; c->vc_hi = 0.1;
    if (o->velocity_correction_bounds[0] != 0.0 || o->velocity_correction_bounds[1] != 0.0) {
        c->vc_lo = o->velocity_correction_bounds[0]; c->vc_hi = o->velocity_correction_bounds[1];
    }
    c->NPD = c->NS + c->NC + c->NDV + c->NM;
    c->NP = c->NPD + c->NSL;
    for (int e = 0; e < c->NPC; ++e) {
        const mh_path_equation* E = &c->pc[e];
        if (E->kind != MH_PATH_CONTROL_BOUND || E->index < 0 || E->index >= c->NC ||
                E->table < -1 || E->table >= M->ntables ||
                (E->table >= 0 && (E->column < 0 || E->column >= c->tabs[E->table].ncol))) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "path equation %d: bad control/table", e);
        }
    }
    /* goals: kind, term range, and every term index within its kind's range
     * (controls, states, implicit auxiliary derivatives, bodies) */
    for (int g = 0; g < p->ngoals; ++g) {
        const mh_goal* G = &c->goals[g];
        if (G->kind < MH_GOAL_CONTROL || G->kind > MH_GOAL_MARKER_FINAL) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "goal %d: unknown kind %d", g, G->kind);
        }
        if (G->term_begin < 0 || G->term_count < 0 || G->term_begin + G->term_count > p->nterms ||
                (G->kind == MH_GOAL_MARKER_FINAL && G->term_count != 6)) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "goal %d: bad terms", g);
        }
        if (G->kind == MH_GOAL_STATE_TRACKING && (G->table < 0 || G->table >= M->ntables)) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "goal %d: bad table", g);
        }
        if (G->kind == MH_GOAL_MARKER_FINAL && c->presc) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "goal %d: marker goal with prescribed kinematics", g);
        }
        for (int k = G->term_begin; k < G->term_begin + G->term_count; ++k) {
            int idx = c->gidx[k], hi;
            switch (G->kind) {
            case MH_GOAL_CONTROL: hi = c->NC; break;
            case MH_GOAL_STATE_TRACKING: case MH_GOAL_SUM_SQUARED_STATE: hi = c->NS; break;
            case MH_GOAL_AUX_DERIVATIVES: hi = c->NAR; break;
            case MH_GOAL_MARKER_FINAL: hi = M->nbodies; if (idx == -1) continue; break;
            default: hi = 0x7fffffff; break;   /* final time: no terms read */
            }
            if (idx < 0 || idx >= hi) {
                orc_destroy(c);
                return fail(MH_ERR_INVALID, "goal %d: term %d index %d out of range", g, k, idx);
            }
            if (G->kind == MH_GOAL_STATE_TRACKING &&
                    (c->gcol[k] < 0 || c->gcol[k] >= c->tabs[G->table].ncol)) {
                orc_destroy(c);
                return fail(MH_ERR_INVALID, "goal %d: term %d column out of range", g, k);
            }
        }
    }
    for (int e = 0; e < c->NEP; ++e) {
        const mh_endpoint_equation* E = &c->ep[e];
        if (E->kind != MH_ENDPOINT_INITIAL_ACTIVATION || E->index_a < 0 || E->index_a >= c->NC ||
                E->index_b < 0 || E->index_b >= c->NS) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "endpoint equation %d: bad kind/control/state", e);
        }
    }
    for (int ia = 0; ia < M->nactuators; ++ia) {
        if (c->acts[ia].kind == MH_ACT_MUSCLE) {
            int t = c->acts[ia].target;
            if (t < 0 || t >= M->nmuscles) { orc_destroy(c); return fail(MH_ERR_INVALID, "actuator %d: bad muscle", ia); }
            c->mus_control[t] = ia;
        }
    }
    for (int im = 0; im < M->nmuscles; ++im)
        if (c->mus_control[im] < 0) { orc_destroy(c); return fail(MH_ERR_INVALID, "muscle %d has no actuator", im); }
    /* coordinate -> body */
    c->coord_body = (int*)malloc(sizeof(int) * (size_t)(c->NQ + 1));
    for (int j = 0; j < c->NQ; ++j) c->coord_body[j] = -1;
    for (int b = 0; b < M->nbodies; ++b) {
        const mh_body* B = &c->bodies[b];
        if (B->parent >= b) { orc_destroy(c); return fail(MH_ERR_INVALID, "body %d not topologically ordered", b); }
        for (int a = B->axis_begin; a < B->axis_begin + B->axis_count; ++a) {
            int f = c->axes[a].func;
            if (f < 0 || f >= M->nfunctions) { orc_destroy(c); return fail(MH_ERR_INVALID, "axis %d: bad function", a); }
            int q = c->funcs[f].coord;
            if (c->funcs[f].kind == MH_FN_CONSTANT) continue;
            if (q < 0 || q >= c->NQ) { orc_destroy(c); return fail(MH_ERR_INVALID, "axis %d: bad coordinate", a); }
            if (c->coord_body[q] >= 0 && c->coord_body[q] != b) {
                orc_destroy(c);
                return fail(MH_ERR_UNSUPPORTED, "coordinate %d drives axes of two bodies", q);
            }
            c->coord_body[q] = b;
        }
    }
    for (int j = 0; j < c->NQ; ++j)
        if (c->coord_body[j] < 0) { orc_destroy(c); return fail(MH_ERR_INVALID, "coordinate %d drives no axis", j); }

    c->sinfo = DUP(mh_variable_info, p->state_infos, c->NS);
    c->cinfo = DUP(mh_variable_info, p->control_infos, c->NC);

    /* transcription grid (CasOCHermiteSimpson.h:45-68, CasOCSolver.h:38-42) */
    c->scheme = o->transcription;
    c->N = o->num_mesh_intervals;
    c->nmesh = c->N + 1;
    c->interp = o->interpolate_control_midpoints && c->NC > 0;
    c->G = c->scheme == MH_HERMITE_SIMPSON ? 2 * c->N + 1 : c->N + 1;
    c->grid = (double*)malloc(sizeof(double) * (size_t)c->G);
    c->quad = (double*)calloc((size_t)c->G, sizeof(double));
    double* mesh = (double*)malloc(sizeof(double) * (size_t)c->nmesh);
    for (int i = 0; i < c->nmesh; ++i) mesh[i] = i / (double)c->N;
    if (c->scheme == MH_HERMITE_SIMPSON) {
        for (int k = 0; k < c->G; ++k)
            c->grid[k] = (k % 2 == 0) ? mesh[k / 2] : .5 * (mesh[k / 2] + mesh[k / 2 + 1]);
        /* CasOCHermiteSimpson.cpp:26-45 */
        for (int i = 0; i < c->N; ++i) {
            double dm = mesh[i + 1] - mesh[i];
            c->quad[2 * i] += (1.0 / 6.0) * dm;
            c->quad[2 * i + 1] += (2.0 / 3.0) * dm;
            c->quad[2 * i + 2] += (1.0 / 6.0) * dm;
        }
    } else {
        for (int k = 0; k < c->G; ++k) c->grid[k] = mesh[k];
        /* CasOCTrapezoidal.cpp:26-41 */
        for (int i = 0; i < c->N; ++i) {
            double dm = mesh[i + 1] - mesh[i];
            c->quad[i] += 0.5 * dm;
            c->quad[i + 1] += 0.5 * dm;
        }
    }
    free(mesh);
    c->n = 2 + (int64_t)(c->NS + c->NC + c->NDV + c->NM) * c->G + (int64_t)c->NSL * c->N;
    c->XP = c->n;             /* the parameters: the last block of x */
    c->n += c->NPAR;
    c->m = c->NEP + (int64_t)rows_per_interval(c) * c->N + ntail(c);
    c->fd = o->finite_difference_scheme;
    c->h = o->fd_step > 0 ? o->fd_step : 1e-8;
    if (o->sparsity_detection != MH_SPARSITY_NONE && c->NPAR > 0) {
        orc_destroy(c);
        return fail(MH_ERR_UNSUPPORTED, "MocoParameters with sparsity detection");
    }
    if (o->sparsity_detection != MH_SPARSITY_NONE) {
#ifndef ORACLE_COUNTING
        int rc = detect_sparsity(c, o);
        if (rc) { orc_destroy(c); return rc; }
#else
        orc_destroy(c);
        return fail(MH_ERR_UNSUPPORTED, "sparsity detection");
#endif
    }
    /* structure */
    emit_state e = {0, NULL, NULL};
    endpoint_rows(c, emit_count, &e);
    for (int i = 0; i < c->N; ++i) interval_rows(c, i, 0, emit_count, &e);
    tail_rows(c, 0, emit_count, &e);
    c->nnz = e.count;
    c->iRow = (int32_t*)malloc(sizeof(int32_t) * (size_t)(c->nnz + 1));
    c->jCol = (int32_t*)malloc(sizeof(int32_t) * (size_t)(c->nnz + 1));
    e.count = 0; e.ir = c->iRow; e.jc = c->jCol;
    int rpi = rows_per_interval(c);
    endpoint_rows(c, emit_fill, &e);
    for (int i = 0; i < c->N; ++i) interval_rows(c, i, c->NEP + (int64_t)i * rpi, emit_fill, &e);
    tail_rows(c, c->NEP + (int64_t)c->N * rpi, emit_fill, &e);
    /* shard (the head belongs to the first shard, the tail to the last) */
    c->ib = o->interval_begin > 0 ? o->interval_begin : 0;
    c->ie = o->interval_end > 0 && o->interval_end < c->N ? o->interval_end : c->N;
    if (c->ib >= c->ie) { orc_destroy(c); return fail(MH_ERR_INVALID, "empty interval shard"); }
    c->gk0 = mesh_point(c, c->ib);
    c->gk1 = mesh_point(c, c->ie);
    c->row_begin = c->ib == 0 ? 0 : c->NEP + (int64_t)c->ib * rpi;
    c->row_end = c->NEP + (int64_t)c->ie * rpi + (c->ie == c->N ? ntail(c) : 0);
    c->nnz_begin = 0;
    while (c->nnz_begin < c->nnz && c->iRow[c->nnz_begin] < c->row_begin) ++c->nnz_begin;
    c->nnz_end = c->nnz_begin;
    while (c->nnz_end < c->nnz && c->iRow[c->nnz_end] < c->row_end) ++c->nnz_end;
    /* tropter's global-seed Jacobian (ProblemDecorator_double.cpp:261-291):
     * column partial distance-2 coloring of the structure (ColPack's
     * SMALLEST_LAST order unless mh_options.coloring_order says natural) */
    c->jac_seeds = o->jacobian_mode == MH_JACOBIAN_GLOBAL_SEEDS;
    if (o->jacobian_mode != MH_JACOBIAN_CALLBACK_FD && !c->jac_seeds) {
        orc_destroy(c);
        return fail(MH_ERR_INVALID, "unknown jacobian_mode %d", o->jacobian_mode);
    }
    if (c->jac_seeds) {
        if (sharded(c) || o->sparsity_detection != MH_SPARSITY_NONE) {
            orc_destroy(c);
            return fail(MH_ERR_UNSUPPORTED, "MH_JACOBIAN_GLOBAL_SEEDS needs an unsharded context and the "
                        "block-dense structure");
        }
        c->seed_color = (int32_t*)malloc(sizeof(int32_t) * (size_t)(c->n + 1));
        if (o->coloring_order != MH_COLORING_SMALLEST_LAST && o->coloring_order != MH_COLORING_NATURAL) {
            orc_destroy(c);
            return fail(MH_ERR_INVALID, "unknown coloring_order %d", o->coloring_order);
        }
        c->nseeds = color_columns(c->m, c->n, c->nnz, c->iRow, c->jCol, c->seed_color, o->coloring_order);
    }
    *out = c;
    return MH_OK;
}

int orc_get_jacobian_seeds(const orc_ctx* c, int32_t* color, int32_t* nseeds) {
    if (!c->jac_seeds) return fail(MH_ERR_INVALID, "context not in MH_JACOBIAN_GLOBAL_SEEDS mode");
    memcpy(color, c->seed_color, sizeof(int32_t) * (size_t)c->n);
    *nseeds = c->nseeds;
    return MH_OK;
}

void orc_destroy(orc_ctx* c) {
    if (!c) return;
    void* ptrs[] = {c->bodies, c->axes, c->funcs, c->kx, c->ky, c->kb, c->kc, c->kd,
            c->mus, c->pts, c->acts, c->tabs, c->brk, c->coef, c->ext, c->sinfo, c->cinfo,
            c->goals, c->gidx, c->gcol, c->gw, c->pc, c->sp, c->sp_pc, c->mus_ider, c->kin_col,
            c->ep, c->sp_ep, c->kcs, c->seed_color, c->wr, c->pw, c->mus_pw_begin, c->mus_pw_count,
            c->mus_act_state, c->mus_ftn_state,
            c->mus_control, c->coord_body, c->grid, c->quad, c->iRow, c->jCol,
            c->spr, c->par_bounds, c->par_targets};
    for (size_t i = 0; i < sizeof ptrs / sizeof ptrs[0]; ++i) free(ptrs[i]);
    free(c);
}

int orc_get_nlp_info(const orc_ctx* c, mh_nlp_info* info) {
    memset(info, 0, sizeof *info);
    info->n = c->n; info->m = c->m; info->nnz_jac_g = c->nnz; info->nnz_h_lag = 0;
    info->num_grid_points = c->G; info->num_states = c->NS; info->num_controls = c->NC;
    info->row_begin = c->row_begin; info->row_end = c->row_end;
    info->nnz_begin = c->nnz_begin; info->nnz_end = c->nnz_end;
    return MH_OK;
}

int orc_get_jac_structure(const orc_ctx* c, int32_t* iRow, int32_t* jCol) {
    memcpy(iRow, c->iRow, sizeof(int32_t) * (size_t)c->nnz);
    memcpy(jCol, c->jCol, sizeof(int32_t) * (size_t)c->nnz);
    return MH_OK;
}

/* CasOC::Problem::clipEndpointBounds (CasOCProblem.h:603-606) with the
 * exact std::max / std::min NaN semantics. */
static mh_bounds clip_endpoint(mh_bounds b, mh_bounds e) {
    mh_bounds r;
    r.lower = (b.lower < e.lower) ? e.lower : b.lower;
    r.upper = (e.upper < b.upper) ? e.upper : b.upper;
    return r;
}
static void set_bounds(mh_bounds b, double* lo, double* up) {
    /* Transcription::setVariableBounds (CasOCTranscription.h:82-95) */
    if (!isnan(b.lower) && !isnan(b.upper)) { *lo = b.lower; *up = b.upper; }
    else { *lo = -INFINITY; *up = INFINITY; }
}

int orc_get_bounds(const orc_ctx* c, double* xl, double* xu, double* gl, double* gu) {
    /* CasOCTranscription.cpp:183-250 */
    set_bounds(c->P.time_initial, &xl[0], &xu[0]);
    set_bounds(c->P.time_final, &xl[1], &xu[1]);
    for (int s = 0; s < c->NS; ++s) {
        mh_variable_info vi = c->sinfo[s];
        mh_bounds ib = clip_endpoint(vi.bounds, vi.initial);
        mh_bounds fb = clip_endpoint(vi.bounds, vi.final);
        for (int k = 1; k < c->G - 1; ++k) set_bounds(vi.bounds, &xl[col_state(c, k, s)], &xu[col_state(c, k, s)]);
        set_bounds(ib, &xl[col_state(c, 0, s)], &xu[col_state(c, 0, s)]);
        set_bounds(fb, &xl[col_state(c, c->G - 1, s)], &xu[col_state(c, c->G - 1, s)]);
    }
    for (int j = 0; j < c->NC; ++j) {
        mh_variable_info vi = c->cinfo[j];
        mh_bounds ib = clip_endpoint(vi.bounds, vi.initial);
        mh_bounds fb = clip_endpoint(vi.bounds, vi.final);
        for (int k = 1; k < c->G - 1; ++k) set_bounds(vi.bounds, &xl[col_control(c, k, j)], &xu[col_control(c, k, j)]);
        set_bounds(ib, &xl[col_control(c, 0, j)], &xu[col_control(c, 0, j)]);
        set_bounds(fb, &xl[col_control(c, c->G - 1, j)], &xu[col_control(c, c->G - 1, j)]);
    }
    /* implicit: accelerations at every grid point (CasOCTranscription.cpp:222-226) */
    for (int j = 0; j < c->NDV; ++j)
        for (int k = 0; k < c->G; ++k) {
            int aux = j >= c->NACC;   /* CasOCTranscription.cpp:228-232 */
            xl[col_deriv(c, k, j)] = aux ? c->aux_lo : c->acc_lo;
            xu[col_deriv(c, k, j)] = aux ? c->aux_hi : c->acc_hi;
        }
    /* multipliers: multiplier_bounds at every grid point, initial and final
     * alike (CasOCTranscription.cpp:209-219); slacks: velocity_correction_
     * bounds (:235-241) */
    for (int j = 0; j < c->NM; ++j)
        for (int k = 0; k < c->G; ++k) { xl[col_mult(c, k, j)] = c->mult_lo; xu[col_mult(c, k, j)] = c->mult_hi; }
    for (int l = 0; l < c->NSL; ++l)
        for (int i = 0; i < c->N; ++i) { xl[col_slack(c, i, l)] = c->vc_lo; xu[col_slack(c, i, l)] = c->vc_hi; }
    /* defects, residuals and interpolating-control rows: equality to 0
     * (CasOCTranscription.cpp:275-278, 440-443) */
    /* parameters: the MocoParameter's bounds (CasOCTranscription.cpp:243-248) */
    for (int q = 0; q < c->NPAR; ++q) set_bounds(c->par_bounds[q], &xl[c->XP + q], &xu[c->XP + q]);
    if (gl) for (int64_t r = 0; r < c->m; ++r) { gl[r] = 0.0; gu[r] = 0.0; }
    /* kinematic rows: kinematic_constraint_bounds at every mesh point
     * (CasOCTranscription.cpp:303-309) */
    if (gl && c->NK) {
        int rpi = rows_per_interval(c);
        for (int i = 0; i <= c->N; ++i) {
            int64_t r0 = c->NEP + (int64_t)i * rpi;
            for (int r = 0; r < c->NK; ++r) { gl[r0 + r] = c->kc_lo; gu[r0 + r] = c->kc_hi; }
        }
    }
    /* path rows: the equation's bounds repeated at every mesh point
     * (CasOCTranscription.cpp:429-432) */
    /* endpoint rows: the constraint info's bounds (CasOCTranscription.cpp:
     * 582-583) */
    if (gl) for (int e = 0; e < c->NEP; ++e) { gl[e] = c->ep[e].g.lower; gu[e] = c->ep[e].g.upper; }
    if (gl && c->NPC) {
        int rpi = rows_per_interval(c);
        for (int i = 0; i <= c->N; ++i) {
            int64_t r0 = c->NEP + (int64_t)i * rpi + c->NK;
            for (int e = 0; e < c->NPC; ++e) { gl[r0 + e] = c->pc[e].g.lower; gu[r0 + e] = c->pc[e].g.upper; }
        }
    }
    return MH_OK;
}

int orc_get_initial_guess_from_bounds(const orc_ctx* c, double* x) {
    /* CasOCTranscription.cpp:1123-1149 */
    double* lo = (double*)malloc(sizeof(double) * (size_t)c->n);
    double* up = (double*)malloc(sizeof(double) * (size_t)c->n);
    orc_get_bounds(c, lo, up, NULL, NULL);
    for (int64_t i = 0; i < c->n; ++i) {
        double l = lo[i], u = up[i];
        if (!isinf(l) && !isinf(u)) x[i] = 0.5 * (u + l);
        else if (!isinf(l)) x[i] = l;
        else if (!isinf(u)) x[i] = u;
        else x[i] = 0;
    }
    free(lo); free(up);
    return MH_OK;
}

int orc_get_random_iterate(const orc_ctx* c, const double* rnd, double* x) {
    /* CasOCTranscription.cpp:1151-1177 */
    double* lo = (double*)malloc(sizeof(double) * (size_t)c->n);
    double* up = (double*)malloc(sizeof(double) * (size_t)c->n);
    orc_get_bounds(c, lo, up, NULL, NULL);
    for (int64_t i = 0; i < c->n; ++i) {
        double l = lo[i], u = up[i], r = rnd[i];
        double v = 0.5 * (r + 1.0) * (u - l) + l;
        if (isnan(v)) v = r < l ? l : (r > u ? u : r); /* SimTK::clamp */
        x[i] = v;
    }
    free(lo); free(up);
    return MH_OK;
}

/* ======================================================================== */
/* Model evaluation.                                                         */
/* ======================================================================== */
static void eval_function(const orc_ctx* c, int f, const real* q, real* out) {
    const mh_function* F = &c->funcs[f];
    switch (F->kind) {
    case MH_FN_CONSTANT: out[0] = F->a; out[1] = out[2] = 0.0; return;
    case MH_FN_LINEAR: {
        real s = F->scale;
        out[0] = s * (F->a * q[F->coord] + F->b);
        out[1] = s * F->a; out[2] = 0.0; return;
    }
    default: {
        int b0 = F->knot_begin;
        simm_eval(F->knot_count, c->kx + b0, c->ky + b0, c->kb + b0, c->kc + b0, c->kd + b0,
                q[F->coord], out);
        out[0] *= F->scale; out[1] *= F->scale; out[2] *= F->scale;
    }
    }
}

#ifndef ORACLE_COUNTING
int orc_eval_function(orc_ctx* c, int f, double qv, double* out3) {
    if (f < 0 || f >= c->P.model.nfunctions) return fail(MH_ERR_INVALID, "bad function");
    real* q = (real*)calloc((size_t)c->NQ + 1, sizeof(real));
    int crd = c->funcs[f].coord;
    if (crd >= 0) q[crd] = qv;
    eval_function(c, f, q, out3);
    free(q);
    return MH_OK;
}
#endif

/* Piecewise-polynomial data table (GCVSpline restated as its piecewise
 * polynomial). Column value at t. */
static real table_eval(const orc_ctx* c, int ti, int col, real t) {
    const mh_table* T = &c->tabs[ti];
    const double* br = c->brk + T->break_begin;
    int s;
    if (t <= br[0]) s = 0;
    else if (t >= br[T->nseg]) s = T->nseg - 1;
    else {
        int lo = 0, hi = T->nseg; /* br[lo] <= t < br[hi] */
        while (hi - lo > 1) {
            int mid = (lo + hi) / 2;
            if (t < br[mid]) hi = mid; else lo = mid;
        }
        s = lo;
    }
    const double* cf = c->coef + T->coef_begin + ((int64_t)s * T->ncol + col) * (T->degree + 1);
    real dt = t - br[s];
    real v = cf[T->degree];
    for (int k = T->degree - 1; k >= 0; --k) v = v * dt + cf[k];
    return v;
}

/* ---- DeGrooteFregly2016Muscle curves (DeGrooteFregly2016Muscle.h:332-476,
 *      constants :769-817) ---- */
static const double DGF_b11 = 0.8150671134243542, DGF_b21 = 1.055033428970575,
                    DGF_b31 = 0.162384573599574, DGF_b41 = 0.063303448465465,
                    DGF_b12 = 0.433004984392647, DGF_b22 = 0.716775413397760,
                    DGF_b32 = -0.029947116970696, DGF_b42 = 0.200356847296188,
                    DGF_b13 = 0.1, DGF_b23 = 1.0, DGF_b33 = 0.353553390593274,
                    DGF_b43 = 0.0;
static const double DGF_kPE = 4.0, DGF_c1 = 0.200, DGF_c2 = 1.0, DGF_c3 = 0.200;
static const double DGF_d1 = -0.3211346127989808, DGF_d2 = -8.149, DGF_d3 = -0.374,
                    DGF_d4 = 0.8825327733249912;
static const double DGF_minNormFiberLength = 0.2;

static real gaussian_like(real x, double b1, double b2, double b3, double b4) {
    real num = (x - b2) * (x - b2);
    real den = (b3 + b4 * x) * (b3 + b4 * x);
    return b1 * exp(-0.5 * num / den);
}
static real dgf_fal(const mh_muscle* mu, real l) {
    real scale = mu->active_force_width_scale;
    real x = (l - 1.0) / scale + 1.0;
    return gaussian_like(x, DGF_b11, DGF_b21, DGF_b31, DGF_b41) +
           gaussian_like(x, DGF_b12, DGF_b22, DGF_b32, DGF_b42) +
           gaussian_like(x, DGF_b13, DGF_b23, DGF_b33, DGF_b43);
}
static real dgf_fv(real v) {
    real tv = DGF_d2 * v + DGF_d3;
    real arg = tv + sqrt(tv * tv + 1.0);
    return DGF_d1 * log(arg) + DGF_d4;
}
static real dgf_fv_inv(real fv) {
    return (sinh(1.0 / DGF_d1 * (fv - DGF_d4)) - DGF_d3) / DGF_d2;
}
static real dgf_fpe(const mh_muscle* mu, real l) {
    if (mu->ignore_passive_fiber_force) return 0.0;
    real e0 = mu->passive_fiber_strain_at_one_norm_force;
    real offset = exp(DGF_kPE * (DGF_minNormFiberLength - 1.0) / e0);
    real denom = exp(DGF_kPE) - offset;
    return (exp(DGF_kPE * (l - 1.0) / e0) - offset) / denom;
}
static double dgf_kT(const mh_muscle* mu) {
    return log((1.0 + DGF_c3) / DGF_c1) / (1.0 + mu->tendon_strain_at_one_norm_force - DGF_c2);
}
static real dgf_ft(const mh_muscle* mu, real l) {
    return DGF_c1 * exp(dgf_kT(mu) * (l - DGF_c2)) - DGF_c3;
}
static real dgf_ft_deriv(const mh_muscle* mu, real l) {
    double kT = dgf_kT(mu);
    return DGF_c1 * kT * exp(kT * (l - DGF_c2));
}
static real dgf_ft_inv(const mh_muscle* mu, real f) {
    return log((1.0 / DGF_c1) * (f + DGF_c3)) / dgf_kT(mu) + DGF_c2;
}

#ifndef ORACLE_COUNTING
double orc_dgf_curve(const mh_muscle* mu, int which, double x) {
    switch (which) {
    case 0: return dgf_fal(mu, x);
    case 1: return dgf_fpe(mu, x);
    case 2: return dgf_fv(x);
    case 3: return dgf_fv_inv(x);
    case 4: return dgf_ft(mu, x);
    case 5: return dgf_ft_inv(mu, x);
    case 6: return dgf_ft_deriv(mu, x);
    default: return NAN;
    }
}
#endif

/* Tendon force and auxiliary derivatives of one DGF muscle
 * (DeGrooteFregly2016Muscle.cpp:186-233, 240-425). */
static void dgf_muscle(const orc_ctx* c, const mh_muscle* mu, real LMT, real VMT,
        real activation, real excitation, int has_act, real normTendonForce,
        int compliant, int implicit_tendon, real normTendonForceDerivative,
        real* tendonForce, real* adot, real* ftdot, real* residual) {
    /* calcMuscleLengthInfoHelper (:240-275) */
    real normTendonLength = compliant ? dgf_ft_inv(mu, normTendonForce) : 1.0;
    real tendonLength = mu->tendon_slack_length * normTendonLength;
    real fiberWidth = mu->optimal_fiber_length * sin(mu->pennation_angle_at_optimal);
    real squareFiberWidth = fiberWidth * fiberWidth;
    real fiberLengthAlongTendon = LMT - tendonLength;
    real fiberLength = sqrt(fiberLengthAlongTendon * fiberLengthAlongTendon + squareFiberWidth);
    real normFiberLength = fiberLength / mu->optimal_fiber_length;
    real cosPenn = fiberLengthAlongTendon / fiberLength;
    real fPE = dgf_fpe(mu, normFiberLength);
    real fAL = dgf_fal(mu, normFiberLength);
    real vmax = mu->max_contraction_velocity * mu->optimal_fiber_length;
    /* calcFiberVelocityInfoHelper (:277-323) */
    real normFiberVelocity, fV, normTendonVelocity;
    if (compliant && !implicit_tendon) {
        real normFiberForce = normTendonForce / cosPenn;
        fV = (normFiberForce - fPE) / (activation * fAL);
        normFiberVelocity = dgf_fv_inv(fV);
        real fiberVelocity = normFiberVelocity * vmax;
        real fiberVelocityAlongTendon = fiberVelocity / cosPenn;
        real tendonVelocity = VMT - fiberVelocityAlongTendon;
        normTendonVelocity = tendonVelocity / mu->tendon_slack_length;
    } else {
        /* rigid, or implicit tendon dynamics: the tendon velocity from the
         * normalized tendon force derivative (calcTendonForceLengthInverse-
         * CurveDerivative, DeGrooteFregly2016Muscle.h:471-476) */
        normTendonVelocity = compliant
                ? normTendonForceDerivative /
                  (DGF_c1 * dgf_kT(mu) * exp(dgf_kT(mu) * (normTendonLength - DGF_c2)))
                : 0.0;
        real tendonVelocity = mu->tendon_slack_length * normTendonVelocity;
        real fiberVelocityAlongTendon = VMT - tendonVelocity;
        real fiberVelocity = fiberVelocityAlongTendon * cosPenn;
        normFiberVelocity = fiberVelocity / vmax;
        fV = dgf_fv(normFiberVelocity);
    }
    /* calcMuscleDynamicsInfoHelper (:325-425) via calcFiberForce (.h:482-503) */
    real Fmax = mu->max_isometric_force;
    real activeFiberForce = Fmax * (activation * fAL * fV);
    real conPassive = Fmax * fPE;
    real nonConPassive = Fmax * mu->fiber_damping * normFiberVelocity;
    real totalFiberForce = activeFiberForce + conPassive + nonConPassive;
    if (compliant) *tendonForce = Fmax * normTendonForce;
    else *tendonForce = totalFiberForce * cosPenn;
    /* getEquilibriumResidual = tendon force - fiber force along the tendon
     * (.cpp:826-848, .h:638-642) */
    if (implicit_tendon) *residual = *tendonForce - totalFiberForce * cosPenn;
    /* computeStateVariableDerivatives (:186-233) */
    if (has_act) {
        real timeConstFactor = 0.5 + 1.5 * activation;
        real tempAct = 1.0 / (c->tau_act * timeConstFactor);
        real tempDeact = timeConstFactor / c->tau_deact;
        real f = 0.5 * tanh(0.1 * (excitation - activation));
        real timeConst = tempAct * (f + 0.5) + tempDeact * (-f + 0.5);
        *adot = timeConst * (excitation - activation);
    }
    if (compliant) {
        /* implicit: the derivative variable itself (.cpp:215-229) */
        if (implicit_tendon) *ftdot = normTendonForceDerivative;
        else *ftdot = normTendonVelocity * dgf_ft_deriv(mu, normTendonLength);
    }
}

/* An entry of a muscle's current path (OpenSim GeometryPath::getCurrentPath):
 * an active path point (pt >= 0) or a PathWrapPoint of PathWrap entry pwi
 * (pt < 0; wp = 1 / 2 for the wrap's first / second tangent point, on the
 * wrap object's body at body-frame location loc; wlen = the length over the
 * surface from the first tangent point, stored on the second). */
typedef struct {
    int pt, pwi, wp, body;
    real loc[3];
    real wlen;
    real P[3], V[3];
} cpoint;

/* Workspace for one DAE evaluation. */
typedef struct {
    real *R, *p;    /* body pose (world): 9, 3 per body                  */
    sv6 *V, *A, *F;   /* velocity, bias acceleration, net force per body   */
    sv6* S;           /* motion subspace per coordinate                    */
    rbi* I;           /* world inertia per body; then composite            */
    real* M;        /* NQ x NQ mass matrix                               */
    real* tau;      /* generalized forces                                */
    real* ppos;     /* path point world positions (3 per point)          */
    real* pvel;
    int* pact;
    real* fvals;    /* function value/d1/d2 per axis (3 per axis)        */
    real* xfull;    /* prescribed kinematics: [q, u, z]                  */
    real* udot;     /* prescribed kinematics: udot                       */
    cpoint* cp;     /* one muscle's current path (points + wrap points)  */
} dae_ws;

static void ws_alloc(const orc_ctx* c, dae_ws* w) {
    const mh_model* M = &c->P.model;
    int nb = M->nbodies + 1;
    w->R = (real*)malloc(sizeof(real) * 9 * (size_t)nb);
    w->p = (real*)malloc(sizeof(real) * 3 * (size_t)nb);
    w->V = (sv6*)malloc(sizeof(sv6) * (size_t)nb);
    w->A = (sv6*)malloc(sizeof(sv6) * (size_t)nb);
    w->F = (sv6*)malloc(sizeof(sv6) * (size_t)nb);
    w->S = (sv6*)malloc(sizeof(sv6) * (size_t)(c->NQ + 1));
    w->I = (rbi*)malloc(sizeof(rbi) * (size_t)nb);
    w->M = (real*)malloc(sizeof(real) * (size_t)(c->NQ * c->NQ + 1));
    w->tau = (real*)malloc(sizeof(real) * (size_t)(c->NQ + 1));
    w->ppos = (real*)malloc(sizeof(real) * 3 * (size_t)(M->npoints + 1));
    w->pvel = (real*)malloc(sizeof(real) * 3 * (size_t)(M->npoints + 1));
    w->pact = (int*)malloc(sizeof(int) * (size_t)(M->npoints + 1));
    w->fvals = (real*)malloc(sizeof(real) * 3 * (size_t)(M->naxes + 1));
    w->xfull = (real*)malloc(sizeof(real) * (size_t)(2 * c->NQ + c->NZ + 1));
    w->udot = (real*)malloc(sizeof(real) * (size_t)(c->NQ + 1));
    w->cp = (cpoint*)malloc(sizeof(cpoint) * (size_t)(c->maxcp + 1));
}
static void ws_free(dae_ws* w) {
    free(w->R); free(w->p); free(w->V); free(w->A); free(w->F); free(w->S); free(w->I);
    free(w->M); free(w->tau); free(w->ppos); free(w->pvel); free(w->pact); free(w->fvals);
    free(w->xfull); free(w->udot); free(w->cp);
}

/* Forward kinematics, velocities and velocity-product accelerations in the
 * ground frame (Simbody realizePosition/Velocity for FunctionBased
 * mobilizers; restated).  Body index b is stored at b+1; slot 0 = ground. */
/* wacc: generalized accelerations (implicit mode) or NULL (bias only). */
static void kinematics(const orc_ctx* c, const real* q, const real* u, const real* wacc, dae_ws* w) {
    const mh_model* Mo = &c->P.model;
    static const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    memcpy(w->R, I3, sizeof I3);
    w->p[0] = w->p[1] = w->p[2] = 0.0;
    memset(&w->V[0], 0, sizeof(sv6));
    memset(&w->A[0], 0, sizeof(sv6));
    /* gravity via base acceleration -g */
    for (int i = 0; i < 3; ++i) w->A[0].v[i] = -Mo->gravity[i];
    for (int j = 0; j < c->NQ; ++j) memset(&w->S[j], 0, sizeof(sv6));
    for (int b = 0; b < Mo->nbodies; ++b) {
        const mh_body* B = &c->bodies[b];
        int ps = B->parent + 1, bs = b + 1;
        const real* Rp = w->R + 9 * ps;
        const real* pp = w->p + 3 * ps;
        real RGF[9], pGF[3], t[3];
        real RPF[9], pPF[3], RBM[9], pBM[3];
        for (int i = 0; i < 9; ++i) { RPF[i] = B->R_PF[i]; RBM[i] = B->R_BM[i]; }
        for (int i = 0; i < 3; ++i) { pPF[i] = B->p_PF[i]; pBM[i] = B->p_BM[i]; }
        mat_mul(Rp, RPF, RGF);
        mat_vec(Rp, pPF, t);
        for (int i = 0; i < 3; ++i) pGF[i] = pp[i] + t[i];
        sv6 V = w->V[ps];
        sv6 Vpar = w->V[ps];
        sv6 A = w->A[ps];
        /* translations (axes fixed in F) */
        real pFM[3] = {0, 0, 0};
        for (int a = B->axis_begin; a < B->axis_begin + B->axis_count; ++a) {
            const mh_axis* X = &c->axes[a];
            real* fv = w->fvals + 3 * a;
            eval_function(c, X->func, q, fv);
            if (X->type != MH_AXIS_TRANSLATION) continue;
            for (int i = 0; i < 3; ++i) pFM[i] += fv[0] * X->dir[i];
        }
        real oM[3];
        mat_vec(RGF, pFM, t);
        for (int i = 0; i < 3; ++i) oM[i] = pGF[i] + t[i];
        for (int a = B->axis_begin; a < B->axis_begin + B->axis_count; ++a) {
            const mh_axis* X = &c->axes[a];
            if (X->type != MH_AXIS_TRANSLATION) continue;
            const mh_function* F = &c->funcs[X->func];
            if (F->kind == MH_FN_CONSTANT) continue;
            const real* fv = w->fvals + 3 * a;
            real uj = u[F->coord];
            sv6 s;
            s.w[0] = s.w[1] = s.w[2] = 0.0;
            real dir[3] = {X->dir[0], X->dir[1], X->dir[2]};
            mat_vec(RGF, dir, s.v);
            sv6 sd = cross_m(Vpar, s);
            real thd = fv[1] * uj, thdd = fv[2] * uj * uj;
            if (wacc) thdd += fv[1] * wacc[F->coord];
            for (int i = 0; i < 3; ++i) {
                V.w[i] += s.w[i] * thd; V.v[i] += s.v[i] * thd;
                A.w[i] += sd.w[i] * thd + s.w[i] * thdd;
                A.v[i] += sd.v[i] * thd + s.v[i] * thdd;
                w->S[F->coord].w[i] += fv[1] * s.w[i];
                w->S[F->coord].v[i] += fv[1] * s.v[i];
            }
        }
        /* rotations (body-fixed sequence about the M origin) */
        real Rcur[9];
        memcpy(Rcur, I3, sizeof I3);
        for (int a = B->axis_begin; a < B->axis_begin + B->axis_count; ++a) {
            const mh_axis* X = &c->axes[a];
            if (X->type != MH_AXIS_ROTATION) continue;
            const mh_function* F = &c->funcs[X->func];
            const real* fv = w->fvals + 3 * a;
            if (F->kind != MH_FN_CONSTANT) {
                real RGc[9];
                mat_mul(RGF, Rcur, RGc);
                sv6 s;
                real dir[3] = {X->dir[0], X->dir[1], X->dir[2]};
                mat_vec(RGc, dir, s.w);
                cross(oM, s.w, s.v);
                sv6 sd = cross_m(V, s);
                real uj = u[F->coord];
                real thd = fv[1] * uj, thdd = fv[2] * uj * uj;
                if (wacc) thdd += fv[1] * wacc[F->coord];
                for (int i = 0; i < 3; ++i) {
                    V.w[i] += s.w[i] * thd; V.v[i] += s.v[i] * thd;
                    A.w[i] += sd.w[i] * thd + s.w[i] * thdd;
                    A.v[i] += sd.v[i] * thd + s.v[i] * thdd;
                    w->S[F->coord].w[i] += fv[1] * s.w[i];
                    w->S[F->coord].v[i] += fv[1] * s.v[i];
                }
            }
            real Rk[9];
            real adir[3] = {X->dir[0], X->dir[1], X->dir[2]};
            axis_rotation(adir, fv[0], Rk);
            mat_mul(Rcur, Rk, Rcur);
        }
        real RGM[9];
        mat_mul(RGF, Rcur, RGM);
        real* RB = w->R + 9 * bs;
        real* pB = w->p + 3 * bs;
        mat_mul_bt(RGM, RBM, RB);       /* R_GB = R_GM R_BM^T */
        mat_vec(RB, pBM, t);
        for (int i = 0; i < 3; ++i) pB[i] = oM[i] - t[i];
        w->V[bs] = V;
        w->A[bs] = A;
    }
}

/* Path point world positions and velocities (OpenSim GeometryPath current
 * path: inactive ConditionalPathPoints are skipped). */
static void path_points(const orc_ctx* c, const real* q, const real* u, dae_ws* w) {
    const mh_model* Mo = &c->P.model;
    for (int i = 0; i < Mo->npoints; ++i) {
        const mh_path_point* pt = &c->pts[i];
        real loc[3] = {pt->loc[0], pt->loc[1], pt->loc[2]};
        real dloc[3] = {0, 0, 0};
        w->pact[i] = 1;
        if (pt->kind == MH_PP_CONDITIONAL) {
            real qv = q[pt->coord];
            w->pact[i] = (qv >= pt->range[0] && qv <= pt->range[1]);
        } else if (pt->kind == MH_PP_MOVING) {
            int fs[3] = {pt->fx, pt->fy, pt->fz};
            for (int d = 0; d < 3; ++d) {
                if (fs[d] < 0) continue;
                real o[3];
                eval_function(c, fs[d], q, o);
                loc[d] = o[0];
                const mh_function* F = &c->funcs[fs[d]];
                if (F->kind != MH_FN_CONSTANT) dloc[d] = o[1] * u[F->coord];
            }
        }
        int bs = pt->body + 1;
        const real* R = w->R + 9 * bs;
        const real* p = w->p + 3 * bs;
        real* P = w->ppos + 3 * i;
        real* Vp = w->pvel + 3 * i;
        real t[3], t2[3];
        mat_vec(R, loc, t);
        for (int d = 0; d < 3; ++d) P[d] = p[d] + t[d];
        /* v = v_O + w x P + R dloc */
        cross(w->V[bs].w, P, t);
        mat_vec(R, dloc, t2);
        for (int d = 0; d < 3; ++d) Vp[d] = w->V[bs].v[d] + t[d] + t2[d];
    }
}

/* ------------------------------------------------------------------------
 * Muscle wrapping over cylinders (opensim-core @b0222c2, third-party and
 * absent here: GeometryPath::applyWrapObjects / calcPathLengthChange,
 * WrapObject::wrapPathSegment, WrapCylinder::wrapLine; restated from their
 * documented algorithm: the shortest path around the cylinder).  Parity
 * with opensim-core's WrapCylinder is unpinned: no reference fixture holds
 * a wrapped path, because DeGrooteFregly2016Muscle::replaceMuscles
 * (DeGrooteFregly2016Muscle.cpp:1007-1020) copies only the PathPointSet, so
 * every reference problem that converts muscles to DGF (MocoInverse,
 * example3DWalking) runs without its PathWraps -- which the reference's
 * converged Rajagopal 18-muscle MocoInverse confirms (tests/test_oracle.py
 * test_rajagopal18_inverse_golden_solution).  Native DGF muscles with a
 * PathWrapSet wrap here.
 * ------------------------------------------------------------------------ */
enum { WRAP_NONE = 0, WRAP_INSIDE = 1, WRAP_WRAPPED = 2 };

/* Ground position of body-frame station loc of body b (-1 = ground) and the
 * velocity of that body-fixed point. */
static void body_station(const dae_ws* w, int body, const real* loc, real* P, real* V) {
    int bs = body + 1;
    const real* R = w->R + 9 * bs;
    const real* p = w->p + 3 * bs;
    real t[3];
    mat_vec(R, loc, t);
    for (int d = 0; d < 3; ++d) P[d] = p[d] + t[d];
    if (V) {
        cross(w->V[bs].w, P, t);
        for (int d = 0; d < 3; ++d) V[d] = w->V[bs].v[d] + t[d];
    }
}

/* WrapCylinder::wrapLine in the cylinder frame (axis z, radius R): the
 * shortest path from a to b that stays outside the cylinder.  Its
 * projection on the xy plane is tangent - arc - tangent; along the axis it
 * rises linearly with the projected length (the unrolled cylinder makes the
 * path straight), so the surface part is a helix of length
 * sqrt((R dtheta)^2 + dz^2).  No wrap when a point lies inside the radius
 * (insideRadius) or when the segment's projection misses the circle; a
 * quadrant constraint (wrap_sign != 0) forces the wrap onto its half-space:
 * a segment passing on the other side wraps around the constrained side. */
static int wrap_cylinder(const mh_wrap_object* W, const real* a, const real* b, real* r1, real* r2,
        real* wlen) {
    real R = W->radius, R2 = R * R;
    real a2 = a[0] * a[0] + a[1] * a[1], b2 = b[0] * b[0] + b[1] * b[1];
    if (a2 < R2 || b2 < R2) return WRAP_INSIDE;
    real d0 = b[0] - a[0], d1 = b[1] - a[1];
    real dd = d0 * d0 + d1 * d1;
    real t = dd > 0.0 ? -(a[0] * d0 + a[1] * d1) / dd : 0.0;
    real n0 = a[0] + t * d0, n1 = a[1] + t * d1;
    int hits = (n0 * n0 + n1 * n1 < R2) && t > 0.0 && t < 1.0;
    real cr = a[0] * b[1] - a[1] * b[0];
    real sshort = cr < 0.0 ? -1.0 : 1.0;
    real sigma = sshort;
    if (W->wrap_sign != 0) {
        real nk = W->wrap_axis == 0 ? n0 : n1;
        if (nk * (real)W->wrap_sign >= 0.0) {
            if (!hits) return WRAP_NONE;
        } else {
            sigma = -sshort;   /* around the constrained side */
        }
    } else if (!hits) {
        return WRAP_NONE;
    }
    real ra = sqrt(a2), rb = sqrt(b2);
    real th1 = atan2(a[1], a[0]) + sigma * acos(R / ra);
    real th2 = atan2(b[1], b[0]) - sigma * acos(R / rb);
    real dth = sigma * (th2 - th1);
    const real twopi = 6.283185307179586;
    while (dth < 0.0) dth = dth + twopi;
    while (dth >= twopi) dth = dth - twopi;
    real l1 = sqrt(a2 - R2), l2 = sqrt(b2 - R2), arc = R * dth;
    real Lxy = l1 + arc + l2;
    real dz = b[2] - a[2];
    real z1 = a[2] + dz * (l1 / Lxy), z2 = a[2] + dz * ((l1 + arc) / Lxy);
    r1[0] = R * cos(th1); r1[1] = R * sin(th1); r1[2] = z1;
    r2[0] = R * cos(th2); r2[1] = R * sin(th2); r2[2] = z2;
    real zz = z2 - z1;
    *wlen = sqrt(arc * arc + zz * zz);
    return WRAP_WRAPPED;
}

/* WrapObject::wrapPathSegment: the segment's ends in the wrap object's
 * frame (ground -> body -> cylinder), wrapLine, tangent points back to the
 * body frame. */
static int wrap_segment(const orc_ctx* c, const dae_ws* w, const mh_wrap_object* W, const cpoint* A,
        const cpoint* B, real* r1B, real* r2B, real* wlen) {
    int bs = W->body + 1;
    const real* R = w->R + 9 * bs;
    const real* p = w->p + 3 * bs;
    real pw[2][3];
    const cpoint* E[2] = {A, B};
    for (int e = 0; e < 2; ++e) {
        real g[3] = {E[e]->P[0] - p[0], E[e]->P[1] - p[1], E[e]->P[2] - p[2]};
        real sb[3];
        for (int i = 0; i < 3; ++i) sb[i] = R[i] * g[0] + R[3 + i] * g[1] + R[6 + i] * g[2];   /* R^T g */
        for (int i = 0; i < 3; ++i) sb[i] = sb[i] - W->p_BW[i];
        for (int i = 0; i < 3; ++i)
            pw[e][i] = W->R_BW[i] * sb[0] + W->R_BW[3 + i] * sb[1] + W->R_BW[6 + i] * sb[2];
    }
    real r1[3], r2[3];
    int res = wrap_cylinder(W, pw[0], pw[1], r1, r2, wlen);
    (void)c;
    if (res != WRAP_WRAPPED) return res;
    for (int i = 0; i < 3; ++i) {
        r1B[i] = W->R_BW[3 * i] * r1[0] + W->R_BW[3 * i + 1] * r1[1] + W->R_BW[3 * i + 2] * r1[2] + W->p_BW[i];
        r2B[i] = W->R_BW[3 * i] * r2[0] + W->R_BW[3 * i + 1] * r2[1] + W->R_BW[3 * i + 2] * r2[2] + W->p_BW[i];
    }
    return res;
}

static real dist3(const real* a, const real* b) {
    real d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
    return sqrt(dot3(d, d));
}

/* Length of a current path: straight segments, except between the two
 * tangent points of one wrap (the stored surface length). */
static real cpath_length(const cpoint* cp, int n) {
    real L = 0.0;
    for (int k = 1; k < n; ++k) {
        if (cp[k].pt < 0 && cp[k - 1].pt < 0 && cp[k].pwi == cp[k - 1].pwi) L += cp[k].wlen;
        else L += dist3(cp[k - 1].P, cp[k].P);
    }
    return L;
}

/* GeometryPath::applyWrapObjects: each PathWrap (in order) removes its
 * tangent points, tries every segment of its point range (the first and
 * last ACTIVE original points of [range_begin, range_end]) that is not the
 * surface part of one wrap, keeps the wrapped segment with the smallest
 * length change (|p1 r1| + surface + |r2 p2| - |p1 p2|) and inserts its two
 * tangent points there.  Two or more PathWraps iterate (at most 8 passes)
 * until the path length changes by less than 0.0005; after the first pass,
 * a no-wrap first object and an inside-radius second one swap order. */
static int apply_wraps(const orc_ctx* c, const dae_ws* w, int im, cpoint* cp, int n) {
    const mh_muscle* mu = &c->mus[im];
    int nw = c->mus_pw_count[im], pb = c->mus_pw_begin[im];
    int order[64], result[64];
    if (nw > 64) nw = 64;
    for (int i = 0; i < nw; ++i) { order[i] = i; result[i] = WRAP_NONE; }
    int maxit = nw < 2 ? 1 : 8;
    real last = INFINITY;
    for (int kk = 0; kk < maxit; ++kk) {
        for (int i = 0; i < nw; ++i) {
            result[i] = WRAP_NONE;
            int pwi = pb + order[i];
            const mh_path_wrap* PW = &c->pw[pwi];
            const mh_wrap_object* W = &c->wr[PW->wrap];
            for (int j = 0; j < n; ++j)
                if (cp[j].pt < 0 && cp[j].pwi == pwi) {
                    for (int k = j; k + 2 < n; ++k) cp[k] = cp[k + 2];
                    n -= 2;
                    break;
                }
            int ws = PW->range_begin < 1 ? 0 : PW->range_begin - 1;
            int we = PW->range_end < 1 ? mu->point_count - 1 : PW->range_end - 1;
            int jf = ws, jr = we;
            while (jf <= we && !w->pact[mu->point_begin + jf]) ++jf;
            if (jf > we) return n;
            while (jr >= ws && !w->pact[mu->point_begin + jr]) --jr;
            if (jr < ws) return n;
            int start = -1, end = -1;
            for (int j = 0; j < n; ++j) {
                if (cp[j].pt == mu->point_begin + jf) start = j;
                if (cp[j].pt == mu->point_begin + jr) end = j;
            }
            if (start < 0 || end < 0) return n;
            int best = -1;
            real bestc = INFINITY, br1[3] = {0, 0, 0}, br2[3] = {0, 0, 0}, bl = 0.0;
            for (int k = start; k < end; ++k) {
                if (cp[k].pt < 0 && cp[k + 1].pt < 0 && cp[k].pwi == cp[k + 1].pwi) continue;
                real r1[3], r2[3], wl;
                result[i] = wrap_segment(c, w, W, &cp[k], &cp[k + 1], r1, r2, &wl);
                if (result[i] != WRAP_WRAPPED) continue;
                real g1[3], g2[3];
                body_station(w, W->body, r1, g1, NULL);
                body_station(w, W->body, r2, g2, NULL);
                real chg = dist3(cp[k].P, g1) + wl + dist3(g2, cp[k + 1].P) - dist3(cp[k].P, cp[k + 1].P);
                if (chg < bestc) {
                    bestc = chg; best = k; bl = wl;
                    for (int d = 0; d < 3; ++d) { br1[d] = r1[d]; br2[d] = r2[d]; }
                }
            }
            if (best >= 0) {
                for (int k = n - 1; k > best; --k) cp[k + 2] = cp[k];
                n += 2;
                for (int e = 0; e < 2; ++e) {
                    cpoint* q = &cp[best + 1 + e];
                    q->pt = -1; q->pwi = pwi; q->wp = e + 1; q->body = W->body;
                    for (int d = 0; d < 3; ++d) q->loc[d] = e ? br2[d] : br1[d];
                    q->wlen = e ? bl : 0.0;
                    body_station(w, W->body, q->loc, q->P, q->V);
                }
            }
        }
        real L = cpath_length(cp, n);
        if (fabs(L - last) < 0.0005) break;
        last = L;
        if (kk == 0 && nw > 1 && result[0] == WRAP_NONE && result[1] == WRAP_INSIDE) {
            int t = order[0]; order[0] = order[1]; order[1] = t;
        }
    }
    return n;
}

/* The muscle's current path: its active points, then the wraps. */
static int current_path(const orc_ctx* c, const dae_ws* w, int im, cpoint* cp) {
    const mh_muscle* mu = &c->mus[im];
    int n = 0;
    for (int i = mu->point_begin; i < mu->point_begin + mu->point_count; ++i) {
        if (!w->pact[i]) continue;
        cp[n].pt = i; cp[n].pwi = -1; cp[n].wp = 0; cp[n].body = c->pts[i].body; cp[n].wlen = 0.0;
        for (int d = 0; d < 3; ++d) { cp[n].P[d] = w->ppos[3 * i + d]; cp[n].V[d] = w->pvel[3 * i + d]; }
        ++n;
    }
    if (c->mus_pw_count[im] > 0) n = apply_wraps(c, w, im, cp, n);
    return n;
}

/* GeometryPath length and lengthening speed over the current path: the
 * speed sums the relative velocity of consecutive points along their chord,
 * tangent points included (PathPoint::calcSpeedBetween on every segment). */
static void muscle_length_speed(const orc_ctx* c, const dae_ws* w, const cpoint* cp, int n, real* len,
        real* spd) {
    (void)c; (void)w;
    real L = 0.0, S = 0.0;
    for (int k = 1; k < n; ++k) {
        const real* a = cp[k - 1].P;
        const real* b = cp[k].P;
        real d[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
        real l = sqrt(dot3(d, d));
        if (cp[k].pt < 0 && cp[k - 1].pt < 0 && cp[k].pwi == cp[k - 1].pwi) L += cp[k].wlen;
        else L += l;
        const real* va = cp[k - 1].V;
        const real* vb = cp[k].V;
        real dv[3] = {vb[0] - va[0], vb[1] - va[1], vb[2] - va[2]};
        S += dot3(d, dv) / l;
    }
    *len = L;
    *spd = S;
}

/* Apply point force Fp (world) at path point i to its body, including the
 * MovingPathPoint generalized-force term tau_j += Fp . (R dloc/dq_j). */
static void apply_point_force(const orc_ctx* c, dae_ws* w, const real* q, int i, const real* Fp) {
    const mh_path_point* pt = &c->pts[i];
    int bs = pt->body + 1;
    if (pt->body >= 0) {
        real t[3];
        cross(w->ppos + 3 * i, Fp, t);
        for (int d = 0; d < 3; ++d) { w->F[bs].w[d] -= t[d]; w->F[bs].v[d] -= Fp[d]; }
        /* F[] holds (I a + v x* I v - f_ext): external forces subtract. */
    }
    if (pt->kind == MH_PP_MOVING && pt->body >= 0) {
        int fs[3] = {pt->fx, pt->fy, pt->fz};
        const real* R = w->R + 9 * bs;
        for (int d = 0; d < 3; ++d) {
            if (fs[d] < 0) continue;
            const mh_function* F = &c->funcs[fs[d]];
            if (F->kind == MH_FN_CONSTANT) continue;
            real o[3];
            eval_function(c, fs[d], q, o);
            /* R * (e_d * o[1]) dotted with Fp */
            real g = (R[0 + d] * Fp[0] + R[3 + d] * Fp[1] + R[6 + d] * Fp[2]) * o[1];
            w->tau[F->coord] += g;
        }
    }
}

/* Point force at a current-path entry: a path point as above, a tangent
 * point as a force at that station of the wrap object's body. */
static void apply_cpoint_force(const orc_ctx* c, dae_ws* w, const real* q, const cpoint* A, const real* Fp) {
    if (A->pt >= 0) {
        apply_point_force(c, w, q, A->pt, Fp);
        return;
    }
    if (A->body < 0) return;
    int bs = A->body + 1;
    real t[3];
    cross(A->P, Fp, t);
    for (int d = 0; d < 3; ++d) { w->F[bs].w[d] -= t[d]; w->F[bs].v[d] -= Fp[d]; }
}

/* The explicit per-point DAE (MocoCasOCProblem::calcMultibodySystemExplicit,
 * MocoCasOCProblem.h:203-244): time, states, controls -> udot, zdot. */
/* One grid point: inputs x (states), ctrl (controls) and, in implicit mode,
 * the generalized accelerations ctrl + NC.  Outputs [udot, zdot] (explicit,
 * MocoCasOCProblem.h:203-244) or [residual, zdot] (implicit,
 * MocoCasOCProblem.h:245-297: residual = the mobility forces
 * findMotionForces needs for udot = w, i.e. M w + C - f_applied, computed by
 * RNEA with the accelerations included). */
/* Value and first / second derivative of a table column (the prescribed
 * q(t), u = dq/dt, udot = d2q/dt2 of PositionMotion, PositionMotion.cpp:
 * 36-70: calcValue and calcDerivative of the same spline). */
static void table_eval_d(const orc_ctx* c, int ti, int col, real t, real* v, real* d1, real* d2) {
    const mh_table* T = &c->tabs[ti];
    const double* br = c->brk + T->break_begin;
    int s;
    if (t <= br[0]) s = 0;
    else if (t >= br[T->nseg]) s = T->nseg - 1;
    else {
        int lo = 0, hi = T->nseg;
        while (hi - lo > 1) {
            int mid = (lo + hi) / 2;
            if (t < br[mid]) hi = mid; else lo = mid;
        }
        s = lo;
    }
    const double* cf = c->coef + T->coef_begin + ((int64_t)s * T->ncol + col) * (T->degree + 1);
    real dt = t - br[s];
    real p = cf[T->degree], dp = 0.0, ddp = 0.0;
    for (int k = T->degree - 1; k >= 0; --k) {
        ddp = ddp * dt + 2.0 * dp;
        dp = dp * dt + p;
        p = p * dt + cf[k];
    }
    *v = p; *d1 = dp; *d2 = ddp;
}

static void eval_dae_full(const orc_ctx* c, dae_ws* w, real time, const real* x,
        const real* ctrl, const real* wacc, real* out);

/* Kinematic-constraint outputs of the DAE callback: the errors of each
 * CoordinateCoupler phi = scale f(q_i) - q_d (Simbody position, velocity and
 * acceleration errors; MocoCasOCProblem.h:664-732 copies qerr, uerr, udoterr
 * in that order: all position errors, then all velocity errors, then all
 * acceleration errors, the last two only when enforcing derivatives), and
 * the velocity correction G^T gamma (MocoCasOCProblem.h:298-332) from the
 * slack inputs.  udot: the callback's accelerations (explicit: the forward
 * dynamics result; implicit: the acceleration variables). */
static void kc_outputs(const orc_ctx* c, const real* q, const real* u, const real* udot,
        const real* ctrl, real* out) {
    int NKC = c->NKC;
    if (!c->NK && !c->NSL) return;   /* prescribed kinematics: multipliers only */
    real* e = out + c->OKC;
    const real* gam = ctrl + c->NC + c->NDV + c->NM;
    real* qc = c->NSL ? out + c->OQC : NULL;
    if (qc) for (int j = 0; j < c->NQ; ++j) qc[j] = 0.0;
    for (int i = 0; i < NKC; ++i) {
        const mh_constraint* K = &c->kcs[i];
        int ci = c->funcs[K->func].coord, d = K->dependent;
        real fv[3];
        eval_function(c, K->func, q, fv);
        real gi = K->scale * fv[1];
        e[i] = K->scale * fv[0] - q[d];
        if (c->enforce) {
            e[NKC + i] = gi * u[ci] - u[d];
            e[2 * NKC + i] = (gi * udot[ci] - udot[d]) + K->scale * fv[2] * u[ci] * u[ci];
        }
        if (qc) {
            qc[ci] += gi * gam[i];
            qc[d] -= gam[i];
        }
    }
}

/* The DAE callback on NLP inputs: explicit / implicit mode pass through;
 * prescribed kinematics assemble [q, u, z] and udot from the motion. */
static void eval_dae_point(const orc_ctx* c, dae_ws* w, real time, const real* x,
        const real* ctrl, real* out) {
    if (!c->presc) {
        eval_dae_full(c, w, time, x, ctrl, c->implicit ? ctrl + c->NC : NULL, out);
        return;
    }
    int NQ = c->NQ;
    for (int j = 0; j < NQ; ++j)
        table_eval_d(c, c->kin_table, c->kin_col[j], time, &w->xfull[j], &w->xfull[NQ + j], &w->udot[j]);
    for (int k = 0; k < c->NZ; ++k) w->xfull[2 * NQ + k] = x[k];
    eval_dae_full(c, w, time, w->xfull, ctrl, w->udot, out);
}

static void eval_dae_full(const orc_ctx* c, dae_ws* w, real time, const real* x,
        const real* ctrl, const real* wacc, real* out) {
    const mh_model* Mo = &c->P.model;
    int NQ = c->NQ;
    const real* q = x;
    const real* u = x + NQ;
    kinematics(c, q, u, wacc, w);
    path_points(c, q, u, w);
    /* Body inertias in ground about the origin; RNEA body forces. */
    for (int b = 0; b < Mo->nbodies; ++b) {
        const mh_body* B = &c->bodies[b];
        int bs = b + 1;
        const real* R = w->R + 9 * bs;
        const real* p = w->p + 3 * bs;
        real cw[3], t[3];
        real com[3] = {B->com[0], B->com[1], B->com[2]};
        mat_vec(R, com, t);
        for (int i = 0; i < 3; ++i) cw[i] = p[i] + t[i];
        /* I_c in ground: R Ib R^T */
        real Ib[9] = {B->inertia[0], B->inertia[3], B->inertia[4],
                        B->inertia[3], B->inertia[1], B->inertia[5],
                        B->inertia[4], B->inertia[5], B->inertia[2]};
        real T1[9], Ig[9];
        mat_mul(R, Ib, T1);
        mat_mul_bt(T1, R, Ig);
        rbi* I = &w->I[bs];
        real m = B->mass;
        I->m = m;
        for (int i = 0; i < 3; ++i) I->h[i] = m * cw[i];
        real c2 = dot3(cw, cw);
        I->I[0] = Ig[0] + m * (c2 - cw[0] * cw[0]);
        I->I[1] = Ig[4] + m * (c2 - cw[1] * cw[1]);
        I->I[2] = Ig[8] + m * (c2 - cw[2] * cw[2]);
        I->I[3] = Ig[1] - m * cw[0] * cw[1];
        I->I[4] = Ig[2] - m * cw[0] * cw[2];
        I->I[5] = Ig[5] - m * cw[1] * cw[2];
        sv6 Ia = rbi_apply(I, w->A[bs]);
        sv6 h = rbi_apply(I, w->V[bs]);
        sv6 vxh = cross_f(w->V[bs], h);
        for (int i = 0; i < 3; ++i) {
            w->F[bs].w[i] = Ia.w[i] + vxh.w[i];
            w->F[bs].v[i] = Ia.v[i] + vxh.v[i];
        }
    }
    for (int j = 0; j < NQ; ++j) w->tau[j] = 0.0;
    /* Coordinate actuators and muscles (controls in actuator order). */
    real* zdot = out + NQ;
    for (int ia = 0; ia < Mo->nactuators; ++ia) {
        const mh_actuator* A = &c->acts[ia];
        if (A->kind == MH_ACT_COORDINATE) {
            w->tau[A->target] += ctrl[ia] * A->optimal_force;
        }
    }
    /* SpringGeneralizedForce (OpenSim, third-party): the generalized force
     * -stiffness (q - rest_length) - viscosity u on its coordinate */
    for (int is = 0; is < c->NSPR; ++is) {
        const mh_spring* S = &c->spr[is];
        real f = -S->stiffness * (q[S->coord] - S->rest_length) - S->viscosity * u[S->coord];
        w->tau[S->coord] += f;
    }
    /* Kinematic constraint forces from the multipliers, applied like applied
     * forces: -G^T lambda (MocoCasOCProblem.h:643-662) */
    const real* lam = ctrl + c->NC + c->NDV;
    for (int i = 0; i < c->NKC; ++i) {
        const mh_constraint* K = &c->kcs[i];
        real fv[3];
        eval_function(c, K->func, q, fv);
        real gi = K->scale * fv[1];
        w->tau[c->funcs[K->func].coord] -= gi * lam[i];
        w->tau[K->dependent] -= -lam[i];
    }
    for (int im = 0; im < Mo->nmuscles; ++im) {
        const mh_muscle* mu = &c->mus[im];
        real L, V;
        int ncp = current_path(c, w, im, w->cp);
        muscle_length_speed(c, w, w->cp, ncp, &L, &V);
        (void)mu;
        real e = ctrl[c->mus_control[im]];
        int sa = c->mus_act_state[im], sf = c->mus_ftn_state[im];
        real a = sa >= 0 ? x[sa] : e;
        real ftn = sf >= 0 ? x[sf] : NAN;
        real T, adot = 0, ftdot = 0, resid = 0;
        int id = c->mus_ider[im];
        real dft = id >= 0 ? ctrl[c->NC + id] : 0.0;
        dgf_muscle(c, mu, L, V, a, e, sa >= 0, ftn, sf >= 0, id >= 0, dft, &T, &adot, &ftdot, &resid);
        if (sa >= 0) zdot[sa - 2 * NQ] = adot;
        if (sf >= 0) zdot[sf - 2 * NQ] = ftdot;
        if (id >= 0) out[NQ + c->NZ + (id - c->NACC)] = resid;
        /* Tension along each segment of the current path
         * (GeometryPath::addInEquivalentForces); the surface part of a wrap
         * joins two points of one body and applies nothing. */
        for (int k = 1; k < ncp; ++k) {
            const cpoint* A = &w->cp[k - 1];
            const cpoint* B = &w->cp[k];
            if (A->pt < 0 && B->pt < 0 && A->pwi == B->pwi) continue;
            real d[3] = {B->P[0] - A->P[0], B->P[1] - A->P[1], B->P[2] - A->P[2]};
            real l = sqrt(dot3(d, d));
            real Fa[3], Fb[3];
            for (int j = 0; j < 3; ++j) { Fa[j] = T * d[j] / l; Fb[j] = -Fa[j]; }
            apply_cpoint_force(c, w, q, A, Fa);
            apply_cpoint_force(c, w, q, B, Fb);
        }
    }
    /* External forces (ExternalForce, ground-expressed force and point). */
    for (int ie = 0; ie < Mo->nexternal; ++ie) {
        const mh_external_force* E = &c->ext[ie];
        real Fv[3] = {0, 0, 0}, P[3], Tq[3] = {0, 0, 0};
        int bs = E->body + 1;
        for (int d = 0; d < 3; ++d) {
            if (E->force_col >= 0) Fv[d] = table_eval(c, E->table, E->force_col + d, time);
            P[d] = E->point_col >= 0 ? table_eval(c, E->table, E->point_col + d, time) : w->p[3 * bs + d];
            if (E->torque_col >= 0) Tq[d] = table_eval(c, E->table, E->torque_col + d, time);
        }
        real t[3];
        cross(P, Fv, t);
        for (int d = 0; d < 3; ++d) { w->F[bs].w[d] -= t[d] + Tq[d]; w->F[bs].v[d] -= Fv[d]; }
    }
    /* RNEA backward pass: tau_applied - bias. */
    for (int b = Mo->nbodies - 1; b >= 0; --b) {
        int bs = b + 1;
        int ps = c->bodies[b].parent + 1;
        if (ps > 0) {
            for (int i = 0; i < 3; ++i) { w->F[ps].w[i] += w->F[bs].w[i]; w->F[ps].v[i] += w->F[bs].v[i]; }
        }
    }
    for (int j = 0; j < NQ; ++j) w->tau[j] -= sv_dot(w->S[j], w->F[c->coord_body[j] + 1]);
    if (wacc) {
        for (int j = 0; j < NQ; ++j) out[j] = -w->tau[j];
        kc_outputs(c, q, u, wacc, ctrl, out);
        return;
    }
    /* CRBA mass matrix. */
    for (int b = Mo->nbodies - 1; b >= 0; --b) {
        int bs = b + 1, ps = c->bodies[b].parent + 1;
        if (ps > 0) {
            rbi* P = &w->I[ps];
            rbi* C = &w->I[bs];
            P->m += C->m;
            for (int i = 0; i < 3; ++i) P->h[i] += C->h[i];
            for (int i = 0; i < 6; ++i) P->I[i] += C->I[i];
        }
    }
    for (int i = 0; i < NQ; ++i) {
        int b = c->coord_body[i];
        sv6 Fi = rbi_apply(&w->I[b + 1], w->S[i]);
        for (int j = 0; j < NQ; ++j) {
            /* dof j on body b or an ancestor of b */
            int bj = c->coord_body[j];
            int anc = b;
            while (anc >= 0 && anc != bj) anc = c->bodies[anc].parent;
            if (anc == bj) {
                real v = sv_dot(w->S[j], Fi);
                w->M[i * NQ + j] = v;
                w->M[j * NQ + i] = v;
            } else {
                int anc2 = bj;
                while (anc2 >= 0 && anc2 != b) anc2 = c->bodies[anc2].parent;
                if (anc2 < 0) { w->M[i * NQ + j] = 0.0; w->M[j * NQ + i] = 0.0; }
            }
        }
    }
    /* Cholesky M = L L^T (in place, lower) and solve. */
    real* L = w->M;
    for (int j = 0; j < NQ; ++j) {
        real s = L[j * NQ + j];
        for (int k = 0; k < j; ++k) s -= L[j * NQ + k] * L[j * NQ + k];
        real d = sqrt(s);
        L[j * NQ + j] = d;
        for (int i = j + 1; i < NQ; ++i) {
            real t = L[i * NQ + j];
            for (int k = 0; k < j; ++k) t -= L[i * NQ + k] * L[j * NQ + k];
            L[i * NQ + j] = t / d;
        }
    }
    real* y = out; /* udot */
    for (int i = 0; i < NQ; ++i) {
        real t = w->tau[i];
        for (int k = 0; k < i; ++k) t -= L[i * NQ + k] * y[k];
        y[i] = t / L[i * NQ + i];
    }
    for (int i = NQ - 1; i >= 0; --i) {
        real t = y[i];
        for (int k = i + 1; k < NQ; ++k) t -= L[k * NQ + i] * y[k];
        y[i] = t / L[i * NQ + i];
    }
    kc_outputs(c, q, u, y, ctrl, out);
}

#ifndef ORACLE_COUNTING
int orc_muscle_length_speed(orc_ctx* c, int im, const double* q, const double* u, double* out) {
    if (im < 0 || im >= c->P.model.nmuscles) return fail(MH_ERR_INVALID, "bad muscle");
    dae_ws w;
    ws_alloc(c, &w);
    kinematics(c, q, u, NULL, &w);
    path_points(c, q, u, &w);
    int n = current_path(c, &w, im, w.cp);
    muscle_length_speed(c, &w, w.cp, n, &out[0], &out[1]);
    ws_free(&w);
    return MH_OK;
}

/* The current path of muscle im at (q, u): *n entries of [x, y, z, kind]
 * in ground (kind: path point index >= 0, or -1 / -2 for a wrap's first /
 * second tangent point); at most cap entries are written. */
int orc_muscle_path(orc_ctx* c, int im, const double* q, const double* u, int cap, int* n, double* pts) {
    if (im < 0 || im >= c->P.model.nmuscles) return fail(MH_ERR_INVALID, "bad muscle");
    dae_ws w;
    ws_alloc(c, &w);
    kinematics(c, q, u, NULL, &w);
    path_points(c, q, u, &w);
    int m = current_path(c, &w, im, w.cp);
    *n = m;
    for (int k = 0; k < m && k < cap; ++k) {
        for (int d = 0; d < 3; ++d) pts[4 * k + d] = w.cp[k].P[d];
        pts[4 * k + 3] = w.cp[k].pt >= 0 ? (double)w.cp[k].pt : -(double)w.cp[k].wp;
    }
    ws_free(&w);
    return MH_OK;
}

int orc_eval_dae(orc_ctx* c, int32_t np, const double* in, double* out) {
    int NI = 1 + c->NP, NO = nout(c);
#pragma omp parallel num_threads(c->nthreads)
    {
        dae_ws w;
        ws_alloc(c, &w);
#pragma omp for schedule(static)
        for (int k = 0; k < np; ++k) {
            const real* p = in + (int64_t)k * NI;
            eval_dae_point(c, &w, p[0], p + 1, p + 1 + c->NS, out + (int64_t)k * NO);
        }
        ws_free(&w);
    }
    return MH_OK;
}

/* The DAE on the model with the iterate x's parameters applied, parameter
 * `moved` (>= 0) moved by `step`: the device's parameter lanes (test use:
 * tests/_lanes.py checks every lane output, parameter lanes included). */
int orc_eval_dae_params(orc_ctx* c0, const double* x, int32_t moved, double step, int32_t np,
        const double* in, double* out) {
    if (moved >= c0->NPAR) return MH_ERR_INVALID;
    orc_ctx* c = param_ctx(c0, x, moved, step);
    int rc = orc_eval_dae(c, np, in, out);
    param_ctx_free(c0, c);
    return rc;
}

/* ======================================================================== */
/* Transcription evaluation.                                                 */
/* ======================================================================== */
static void times_of(const orc_ctx* c, const double* x, double* t) {
    /* Transcription::createTimes (CasOCTranscription.h:40-43) */
    double t0 = x[0], tf = x[1];
    for (int k = 0; k < c->G; ++k) t[k] = (tf - t0) * c->grid[k] + t0;
}

/* st: states; ct: controls, the derivative variables (implicit), the
 * multipliers, then the slacks (the interval's at a mesh-interval midpoint,
 * 0 elsewhere) */
static void gather_point(const orc_ctx* c, const double* x, int k, double* st, double* ct) {
    memcpy(st, x + col_state(c, k, 0), sizeof(double) * (size_t)c->NS);
    if (c->NC) memcpy(ct, x + col_control(c, k, 0), sizeof(double) * (size_t)c->NC);
    if (c->NDV) memcpy(ct + c->NC, x + col_deriv(c, k, 0), sizeof(double) * (size_t)c->NDV);
    if (c->NM) memcpy(ct + c->NC + c->NDV, x + col_mult(c, k, 0), sizeof(double) * (size_t)c->NM);
    for (int l = 0; l < c->NSL; ++l)
        ct[c->NC + c->NDV + c->NM + l] = vc_point(c, k) ? x[col_slack(c, (k - 1) / 2, l)] : 0.0;
}

/* xdot at all grid points: qdot = u (CasOCTranscription.cpp:313-314),
 * udot = the derivative variables in implicit mode (:339-341), callback
 * outputs for the rest. xd: NS x G (grid-major); res: NQ x G multibody
 * residuals (implicit mode, else unused). */
static void all_xdot(orc_ctx* c, const double* x, const double* times, double* xd, double* res,
        double* kce) {
    int NS = c->NS, NC = c->NC, NO = nout(c), NR = nres(c);
#pragma omp parallel num_threads(c->nthreads)
    {
        dae_ws w;
        ws_alloc(c, &w);
        double* st = (double*)malloc(sizeof(double) * (size_t)(c->NP + NO + 1));
        double* ct = st + NS;
        double* y = ct + (c->NP - NS);
#pragma omp for schedule(static)
        for (int k = c->gk0; k <= c->gk1; ++k) {
            gather_point(c, x, k, st, ct);
            double* o = xd + (int64_t)k * NS;
            int TQ = c->TQ;
            eval_dae_point(c, &w, times[k], st, ct, y);
            for (int s = 0; s < NS; ++s) {
                if (s < TQ) {                                           /* qdot = u */
                    o[s] = st[TQ + s];
                    /* + the velocity correction at a mesh-interval midpoint
                     * (CasOCTranscription.cpp:316-333) */
                    if (vc_point(c, k)) o[s] = st[TQ + s] + y[c->OQC + s];
                }
                else if (c->NACC && s < 2 * TQ) o[s] = ct[NC + s - TQ];  /* udot = w */
                else o[s] = y[s + c->SO];                               /* callback */
            }
            for (int r = 0; r < NR; ++r) res[(int64_t)k * NR + r] = y[res_out(c, r)];
            for (int r = 0; r < c->NK; ++r) kce[(int64_t)k * c->NK + r] = y[c->OKC + r];
        }
        free(st);
        ws_free(&w);
    }
}

/* MocoControlBoundConstraint::calcPathConstraintErrorsImpl
 * (MocoControlBoundConstraint.cpp:130-146): error = control - bound(t). */
static double path_value(const orc_ctx* c, int e, double t, const double* ct) {
    const mh_path_equation* E = &c->pc[e];
    double b = E->table < 0 ? E->value : table_eval(c, E->table, E->column, t);
    return ct[E->index] - b;
}

/* splitmix64 uniform(-1, 1) stream, seed 0 (include/mocohip.h
 * mh_options.sparsity_detection; stands in for SimTK::Random::Uniform). */
static double splitmix_uniform(uint64_t* st) {
    uint64_t z = (*st += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

/* A detection probe's coupling test (include/mocohip.h mh_sparsity_rule):
 * ANY_CHANGE is the reference's (CasOCFunction.cpp:44-61: nonzero or NaN);
 * ROBUST ignores changes below MH_SPARSITY_ROBUST_TOL of the output's
 * magnitude (rounding noise of couplings that cancel mathematically). */
static int sparsity_coupled(int rule, double d, double scale) {
    if (isnan(d)) return 1;
    if (rule == MH_SPARSITY_RULE_ANY_CHANGE) return d != 0;
    return fabs(d) > MH_SPARSITY_ROBUST_TOL * scale;
}
/* the callback's magnitude at the detection point: max(1, max |output|) */
static double sparsity_scale(const double* y0, int n) {
    double s = 1.0;
    for (int k = 0; k < n; ++k)
        if (isfinite(y0[k]) && fabs(y0[k]) > s) s = fabs(y0[k]);
    return s;
}

/* calcJacobianSparsityWithPerturbation (CasOCFunction.cpp:25-71) for the
 * DAE callback and each path equation, at getSubsetPoint of every
 * detection iterate (CasOCFunction.h:72-86: time = initial_time, the first
 * grid point's variables); iterates per CasOCSolver.cpp:70-92. */
static int detect_sparsity(orc_ctx* c, const mh_options* o) {
    int NS = c->NS, NP = c->NP, NO = nout(c), W = 1 + NP, NPC = c->NPC;
    int npts = 1;
    double* pts;
    const int rule = o->sparsity_rule;
    if (rule != MH_SPARSITY_RULE_ROBUST && rule != MH_SPARSITY_RULE_ANY_CHANGE)
        return fail(MH_ERR_INVALID, "unknown sparsity rule %d", rule);
    if (o->sparsity_detection == MH_SPARSITY_RANDOM) {
        npts = o->sparsity_random_count > 0 ? o->sparsity_random_count : 3;
        pts = (double*)malloc(sizeof(double) * (size_t)c->n * (size_t)npts);
        double* r = (double*)malloc(sizeof(double) * (size_t)c->n);
        uint64_t st = 0;
        for (int q = 0; q < npts; ++q) {
            for (int64_t i = 0; i < c->n; ++i) r[i] = splitmix_uniform(&st);
            orc_get_random_iterate(c, r, pts + (int64_t)q * c->n);
        }
        free(r);
    } else if (o->sparsity_detection == MH_SPARSITY_INITIAL_GUESS) {
        pts = (double*)malloc(sizeof(double) * (size_t)c->n);
        if (o->sparsity_guess) memcpy(pts, o->sparsity_guess, sizeof(double) * (size_t)c->n);
        else orc_get_initial_guess_from_bounds(c, pts);   /* the default "bounds" guess */
    } else if (o->sparsity_detection == MH_SPARSITY_GIVEN) {
        if (!o->sparsity_pattern) return fail(MH_ERR_INVALID, "GIVEN sparsity needs sparsity_pattern");
        c->sp = (uint8_t*)malloc((size_t)NO * W + 1);
        c->sp_pc = (uint8_t*)malloc((size_t)NPC * W + 1);
        c->sp_ep = (uint8_t*)malloc((size_t)c->NEP * 2 * W + 1);
        memcpy(c->sp, o->sparsity_pattern, (size_t)NO * W);
        memcpy(c->sp_pc, o->sparsity_pattern + (size_t)NO * W, (size_t)NPC * W);
        memcpy(c->sp_ep, o->sparsity_pattern + (size_t)(NO + NPC) * W, (size_t)c->NEP * 2 * W);
        return MH_OK;
    } else {
        return fail(MH_ERR_INVALID, "unknown sparsity detection %d", o->sparsity_detection);
    }
    c->sp = (uint8_t*)calloc((size_t)NO * W + 1, 1);
    c->sp_pc = (uint8_t*)calloc((size_t)NPC * W + 1, 1);
    c->sp_ep = (uint8_t*)calloc((size_t)c->NEP * 2 * W + 1, 1);
    dae_ws w;
    ws_alloc(c, &w);
    double* in = (double*)malloc(sizeof(double) * (size_t)(W + 2 * NO + 2 * NPC + 2));
    double *y0 = in + W, *y = y0 + NO, *p0 = y + NO, *pv = p0 + NPC;
    const double eps = 1e-5;
    for (int q = 0; q < npts; ++q) {
        const double* x = pts + (int64_t)q * c->n;
        in[0] = x[0];
        gather_point(c, x, 0, in + 1, in + 1 + NS);
        eval_dae_point(c, &w, in[0], in + 1, in + 1 + NS, y0);
        for (int e = 0; e < NPC; ++e) p0[e] = path_value(c, e, in[0], in + 1 + NS);
        const double sd = sparsity_scale(y0, NO), sp = sparsity_scale(p0, NPC);
        for (int j = 0; j < W; ++j) {
            double sv = in[j];
            in[j] = sv + eps;
            eval_dae_point(c, &w, in[0], in + 1, in + 1 + NS, y);
            for (int e = 0; e < NPC; ++e) pv[e] = path_value(c, e, in[0], in + 1 + NS);
            in[j] = sv;
            for (int k = 0; k < NO; ++k) {
                double d = y[k] - y0[k];
                if (sparsity_coupled(rule, d, sd)) c->sp[(int64_t)k * W + j] = 1;
            }
            for (int e = 0; e < NPC; ++e) {
                double d = pv[e] - p0[e];
                if (sparsity_coupled(rule, d, sp)) c->sp_pc[(int64_t)e * W + j] = 1;
            }
        }
        /* the endpoint functions at their subset point (Endpoint::
         * getSubsetPoint, CasOCFunction.h:214-237; the integral input is 0
         * there and, being no NLP variable, adds no column) */
        if (c->NEP) {
            double* ein = (double*)malloc(sizeof(double) * (size_t)(2 * W));
            ep_gather(c, x, ein);
            double se = 1.0;
            for (int e = 0; e < c->NEP; ++e) {
                double v0 = endpoint_value(c, e, ein);
                if (isfinite(v0) && fabs(v0) > se) se = fabs(v0);
            }
            for (int j = 0; j < 2 * W; ++j) {
                double sv = ein[j];
                for (int e = 0; e < c->NEP; ++e) {
                    double v0 = endpoint_value(c, e, ein);
                    ein[j] = sv + eps;
                    double d = endpoint_value(c, e, ein) - v0;
                    ein[j] = sv;
                    if (sparsity_coupled(rule, d, se)) c->sp_ep[(int64_t)e * 2 * W + j] = 1;
                }
            }
            free(ein);
        }
    }
    free(in);
    free(pts);
    ws_free(&w);
    return MH_OK;
}

int orc_get_callback_sparsity(const orc_ctx* c, uint8_t* pattern, int64_t len) {
    int64_t W = 1 + c->NP, nd = (int64_t)nout(c) * W, np = nd + (int64_t)c->NPC * W;
    int64_t need = np + (int64_t)c->NEP * 2 * W;
    if (!pattern || len < need) return fail(MH_ERR_INVALID, "pattern needs %lld bytes", (long long)need);
    for (int64_t i = 0; i < need; ++i)
        pattern[i] = i < nd ? (c->sp ? c->sp[i] : 1)
                   : i < np ? (c->sp_pc ? c->sp_pc[i - nd] : 1) : (c->sp_ep ? c->sp_ep[i - np] : 1);
    return MH_OK;
}

/* g from the grid times, xdot (xd: NS per point) and residual outputs
 * (res: nres per point) at every grid point (flattenConstraints order). */
static void g_assemble(const orc_ctx* c, const double* x, const double* times, const double* xd,
        const double* res, const double* kce, double* g) {
    int NS = c->NS, NC = c->NC, NR = nres(c);
    int rpi = rows_per_interval(c);
    /* endpoint rows first */
    if (c->NEP) {
        double* ein = (double*)malloc(sizeof(double) * (size_t)(ep_width(c) + c->NPAR));
        ep_gather(c, x, ein);
        for (int e = 0; e < c->NEP; ++e) g[e] = endpoint_value(c, e, ein);
        free(ein);
    }
    g += c->NEP;
    double* pin = (double*)malloc(sizeof(double) * (size_t)(c->NP + 1));
    /* kinematic and path rows of every mesh point: interval i opens with
     * mesh point i's, the tail with the final mesh point's */
    for (int i = 0; i <= c->N; ++i) {
        int k = mesh_point(c, i);
        for (int r = 0; r < c->NK; ++r) g[(int64_t)i * rpi + r] = kce[(int64_t)k * c->NK + r];
        if (!c->NPC) continue;
        gather_point(c, x, k, pin, pin + NS);
        for (int e = 0; e < c->NPC; ++e) g[(int64_t)i * rpi + c->NK + e] = path_value(c, e, times[k], pin + NS);
    }
    free(pin);
    for (int i = 0; i < c->N; ++i) {
        double* gi = g + (int64_t)i * rpi + c->NK + c->NPC;
        /* residual rows of the interval's grid points first */
        int npts = c->scheme == MH_HERMITE_SIMPSON ? 2 : 1;
        int k0 = c->scheme == MH_HERMITE_SIMPSON ? 2 * i : i;
        for (int p = 0; p < npts; ++p)
            for (int o = 0; o < NR; ++o) gi[p * NR + o] = res[(int64_t)(k0 + p) * NR + o];
        gi += npts * NR;
        if (c->scheme == MH_HERMITE_SIMPSON) {
            int ki = 2 * i, km = 2 * i + 1, kp = 2 * i + 2;
            double h = times[kp] - times[ki];
            const double *xi = x + col_state(c, ki, 0), *xm = x + col_state(c, km, 0),
                         *xp = x + col_state(c, kp, 0);
            const double *fi = xd + (int64_t)ki * NS, *fm = xd + (int64_t)km * NS,
                         *fp = xd + (int64_t)kp * NS;
            /* CasOCHermiteSimpson.cpp:79-84 */
            for (int s = 0; s < NS; ++s)
                gi[s] = xm[s] - 0.5 * (xp[s] + xi[s]) - (h / 8.0) * (fi[s] - fp[s]);
            for (int s = 0; s < NS; ++s)
                gi[NS + s] = xp[s] - xi[s] - (h / 6.0) * (fp[s] + 4.0 * fm[s] + fi[s]);
            if (c->interp) {
                const double *ci = x + col_control(c, ki, 0), *cm = x + col_control(c, km, 0),
                             *cp = x + col_control(c, kp, 0);
                /* CasOCHermiteSimpson.cpp:102 */
                for (int j = 0; j < NC; ++j) gi[2 * NS + j] = cm[j] - 0.5 * (cp[j] + ci[j]);
            }
        } else {
            int ki = i, kp = i + 1;
            double h = times[kp] - times[ki];
            const double *xi = x + col_state(c, ki, 0), *xp = x + col_state(c, kp, 0);
            const double *fi = xd + (int64_t)ki * NS, *fp = xd + (int64_t)kp * NS;
            /* CasOCTrapezoidal.cpp:52-56 */
            for (int s = 0; s < NS; ++s) gi[s] = xp[s] - (xi[s] + 0.5 * h * (fp[s] + fi[s]));
        }
    }
    for (int o = 0; o < NR; ++o) g[(int64_t)c->N * rpi + c->NK + c->NPC + o] = res[(int64_t)(c->G - 1) * NR + o];
}

/* A shard context evaluates its grid points only and returns its rows /
 * nonzeros: the full-layout assembly goes through a scratch vector. */
static int sharded(const orc_ctx* c) { return c->ib != 0 || c->ie != c->N; }

int orc_eval_g(orc_ctx* c0, const double* x, double* g) {
    orc_ctx* c = param_ctx(c0, x, -1, 0.0);   /* the iterate's parameters applied */
    int NS = c->NS, NR = nres(c);
    double* times = (double*)malloc(sizeof(double) * (size_t)c->G);
    double* xd = (double*)calloc((size_t)c->G * (size_t)NS + 1, sizeof(double));
    double* res = (double*)calloc((size_t)c->G * (size_t)NR + 1, sizeof(double));
    double* kce = (double*)calloc((size_t)c->G * (size_t)c->NK + 1, sizeof(double));
    times_of(c, x, times);
    all_xdot(c, x, times, xd, res, kce);
    if (sharded(c)) {
        double* full = (double*)calloc((size_t)c->m + 1, sizeof(double));
        g_assemble(c, x, times, xd, res, kce, full);
        memcpy(g, full + c->row_begin, sizeof(double) * (size_t)(c->row_end - c->row_begin));
        free(full);
    } else {
        g_assemble(c, x, times, xd, res, kce, g);
    }
    free(times);
    free(xd);
    free(res);
    free(kce);
    param_ctx_free(c0, c);
    return MH_OK;
}

/* FD derivative blocks of the DAE at every grid point.
 * D[k][d][o]: derivative of callback output o (udot, zdot) along direction
 * d in {t0, tf, input 0..NP-1}.  CasADi FiniteDiff with enable_fd
 * (CasOCFunction.h:38-44); time seeds are d(time_k)/d(t0) = 1-grid_k and
 * d(time_k)/d(tf) = grid_k (CasOCTranscription.cpp:126-127,1189). */
static void fd_blocks(orc_ctx* c, const double* x, const double* times, double* D) {
    int NS = c->NS, NP = c->NP, NO = nout(c);
    int ND = ndir(c);
    double h = c->h;
    /* c: the iterate's parameters applied; along parameter p the callbacks
     * run over the model with that parameter moved by +h / -h */
    orc_ctx** pplus = (orc_ctx**)calloc((size_t)c->NPAR + 1, sizeof(orc_ctx*));
    orc_ctx** pminus = (orc_ctx**)calloc((size_t)c->NPAR + 1, sizeof(orc_ctx*));
    for (int q = 0; q < c->NPAR; ++q) {
        if (c->fd != MH_FD_BACKWARD) pplus[q] = param_ctx(c, x, q, h);
        if (c->fd != MH_FD_FORWARD) pminus[q] = param_ctx(c, x, q, -h);
    }
#pragma omp parallel num_threads(c->nthreads)
    {
        dae_ws w;
        ws_alloc(c, &w);
        double* in = (double*)malloc(sizeof(double) * (size_t)(NP + 1));
        double* yp = (double*)malloc(sizeof(double) * (size_t)(3 * NO + 1));
        double* ym = yp + NO;
        double* y0 = ym + NO;
#pragma omp for schedule(static)
        for (int k = c->gk0; k <= c->gk1; ++k) {
            gather_point(c, x, k, in, in + NS);
            double t = times[k];
            if (c->fd != MH_FD_CENTRAL) eval_dae_point(c, &w, t, in, in + NS, y0);
            for (int d = 0; d < ND; ++d) {
                double seed;
                int idx = -1;
                double* Dk = D + ((int64_t)k * ND + d) * NO;
                if (d >= 2 + NP) {   /* parameter d - 2 - NP */
                    int q = d - 2 - NP;
                    if (c->fd != MH_FD_BACKWARD) eval_dae_point(pplus[q], &w, t, in, in + NS, yp);
                    if (c->fd != MH_FD_FORWARD) eval_dae_point(pminus[q], &w, t, in, in + NS, ym);
                    for (int o = 0; o < NO; ++o) {
                        if (c->fd == MH_FD_CENTRAL) Dk[o] = (yp[o] - ym[o]) / (2.0 * h);
                        else if (c->fd == MH_FD_FORWARD) Dk[o] = (yp[o] - y0[o]) / h;
                        else Dk[o] = (y0[o] - ym[o]) / h;
                    }
                    continue;
                }
                if (d == 0) seed = 1.0 - c->grid[k];
                else if (d == 1) seed = c->grid[k];
                else { seed = 1.0; idx = d - 2; }
                if (c->fd != MH_FD_BACKWARD) {
                    if (idx < 0) eval_dae_point(c, &w, t + h * seed, in, in + NS, yp);
                    else {
                        double s = in[idx];
                        in[idx] = s + h * seed;
                        eval_dae_point(c, &w, t, in, in + NS, yp);
                        in[idx] = s;
                    }
                }
                if (c->fd != MH_FD_FORWARD) {
                    if (idx < 0) eval_dae_point(c, &w, t - h * seed, in, in + NS, ym);
                    else {
                        double s = in[idx];
                        in[idx] = s - h * seed;
                        eval_dae_point(c, &w, t, in, in + NS, ym);
                        in[idx] = s;
                    }
                }
                for (int o = 0; o < NO; ++o) {
                    if (c->fd == MH_FD_CENTRAL) Dk[o] = (yp[o] - ym[o]) / (2.0 * h);
                    else if (c->fd == MH_FD_FORWARD) Dk[o] = (yp[o] - y0[o]) / h;
                    else Dk[o] = (y0[o] - ym[o]) / h;
                }
            }
        }
        free(in);
        free(yp);
        ws_free(&w);
    }
    for (int q = 0; q < c->NPAR; ++q) { param_ctx_free(c, pplus[q]); param_ctx_free(c, pminus[q]); }
    free(pplus); free(pminus);
}

/* FD blocks of the path-constraint equations at every mesh point:
 * Dp[(i * ND + d) * NPC + e], directions and seeds as in fd_blocks (the
 * path function has its own FiniteDiff, CasOCTranscription.cpp:424-428). */
static void path_blocks(const orc_ctx* c, const double* x, const double* times, double* Dp) {
    int NS = c->NS, NP = c->NP, NPC = c->NPC, ND = ndir(c);
    double h = c->h;
    double* in = (double*)malloc(sizeof(double) * (size_t)(NP + 1));
    for (int i = c->ib; i <= c->ie; ++i) {
        int k = mesh_point(c, i);
        gather_point(c, x, k, in, in + NS);
        double t = times[k];
        for (int d = 0; d < ND; ++d) {
            double seed;
            int idx = -1;
            if (d >= 2 + NP) {   /* a parameter: the control bound reads no model property */
                for (int e = 0; e < NPC; ++e) Dp[((int64_t)i * ND + d) * NPC + e] = 0.0;
                continue;
            }
            if (d == 0) seed = 1.0 - c->grid[k];
            else if (d == 1) seed = c->grid[k];
            else { seed = 1.0; idx = d - 2; }
            for (int e = 0; e < NPC; ++e) {
                double vp = 0.0, vm = 0.0, v0 = 0.0;
                if (c->fd != MH_FD_CENTRAL) v0 = path_value(c, e, t, in + NS);
                if (c->fd != MH_FD_BACKWARD) {
                    if (idx < 0) vp = path_value(c, e, t + h * seed, in + NS);
                    else {
                        double sv = in[idx];
                        in[idx] = sv + h * seed;
                        vp = path_value(c, e, t, in + NS);
                        in[idx] = sv;
                    }
                }
                if (c->fd != MH_FD_FORWARD) {
                    if (idx < 0) vm = path_value(c, e, t - h * seed, in + NS);
                    else {
                        double sv = in[idx];
                        in[idx] = sv - h * seed;
                        vm = path_value(c, e, t, in + NS);
                        in[idx] = sv;
                    }
                }
                double q;
                if (c->fd == MH_FD_CENTRAL) q = (vp - vm) / (2.0 * h);
                else if (c->fd == MH_FD_FORWARD) q = (vp - v0) / h;
                else q = (v0 - vm) / h;
                Dp[((int64_t)i * ND + d) * NPC + e] = q;
            }
        }
    }
    free(in);
}

/* Derivative of xdot[s] at grid point k along direction d (0=t0, 1=tf,
 * 2+j = input j).  For s < NQ, qdot = u exactly. */
static double xdot_deriv(const orc_ctx* c, const double* D, int k, int s, int d) {
    int NQ = c->TQ, NO = nout(c), ND = ndir(c);
    if (s < NQ) {
        double v = (d == 2 + NQ + s) ? 1.0 : 0.0;
        /* midpoint: + the velocity correction's FD quotient */
        if (vc_point(c, k)) v = v + D[((int64_t)k * ND + d) * NO + (c->OQC + s)];
        return v;
    }
    if (c->NACC && s < 2 * NQ) return (d == 2 + c->NS + c->NC + (s - NQ)) ? 1.0 : 0.0;
    return D[((int64_t)k * ND + d) * NO + (s + c->SO)];
}

/* Map a Jacobian column to (grid point, direction) for an interval row. */
static int col_to_dir(const orc_ctx* c, int64_t col, int* k) {
    if (col < 2) { *k = -1; return (int)col; }
    if (col >= c->XP) { *k = -1; return 2 + c->NP + (int)(col - c->XP); }   /* parameter */
    int64_t sblock = (int64_t)c->NS * c->G;
    if (col < 2 + sblock) {
        int64_t r = col - 2;
        *k = (int)(r / c->NS);
        return 2 + (int)(r % c->NS);
    }
    int64_t r = col - 2 - sblock;
    int64_t cblock = (int64_t)c->NC * c->G;
    if (r < cblock) {
        *k = (int)(r / c->NC);
        return 2 + c->NS + (int)(r % c->NC);
    }
    r -= cblock;
    int64_t mblock = (int64_t)c->NM * c->G;
    if (r < mblock) {
        *k = (int)(r / c->NM);
        return 2 + c->NS + c->NC + c->NDV + (int)(r % c->NM);
    }
    r -= mblock;
    int64_t lblock = (int64_t)c->NSL * c->N;
    if (r < lblock) {   /* slack l of interval i: an input of the midpoint */
        *k = 2 * (int)(r / c->NSL) + 1;
        return 2 + c->NPD + (int)(r % c->NSL);
    }
    r -= lblock;
    *k = (int)(r / c->NDV);
    return 2 + c->NS + c->NC + (int)(r % c->NDV);
}

/* Jacobian values from the grid times, xdot at every grid point (xd), the
 * DAE FD blocks (D) and the path-constraint FD blocks (Dp): the chain rule
 * through the defect formulas (CasOCHermiteSimpson.cpp:53-105,
 * CasOCTrapezoidal.cpp:43-59), in structure order.  Written without fused
 * operations (the build uses -ffp-contract=off) so that the same inputs give
 * the same bits as the device's assembly. */
static void jac_assemble(const orc_ctx* c, const double* x, const double* times, const double* xd,
        const double* D, const double* Dp, double* values) {
    int NS = c->NS, NQ = c->NQ;
    int NO = nout(c), ND = ndir(c);
    int NR = nres(c);
    int PD = 2 + c->NP;   /* direction of parameter 0 */
    int NPC = c->NPC;
    int rpi = rows_per_interval(c);
    int npts_res = c->scheme == MH_HERMITE_SIMPSON ? 2 : 1;
    /* endpoint rows: FD quotients of the endpoint function along each of its
     * structural columns (the Endpoint callback's FiniteDiff, step h) */
    int64_t e0 = 0;
    if (c->NEP) {
        int WE = ep_width(c);
        double* ein = (double*)malloc(sizeof(double) * (size_t)(WE + c->NPAR));
        int64_t* cols = (int64_t*)malloc(sizeof(int64_t) * (size_t)(WE + 1 + c->NPAR));
        int* si = (int*)malloc(sizeof(int) * (size_t)(WE + 1 + c->NPAR));
        ep_gather(c, x, ein);
        for (int r = 0; r < c->NEP; ++r) {
            int nc = ep_row_cols(c, r, cols, si);
            double v0 = endpoint_value(c, r, ein);
            for (int q = 0; q < nc; ++q) {
                double sv = ein[si[q]], vp = 0.0, vm = 0.0;
                if (c->fd != MH_FD_BACKWARD) { ein[si[q]] = sv + c->h; vp = endpoint_value(c, r, ein); }
                if (c->fd != MH_FD_FORWARD) { ein[si[q]] = sv - c->h; vm = endpoint_value(c, r, ein); }
                ein[si[q]] = sv;
                values[e0++] = c->fd == MH_FD_CENTRAL ? (vp - vm) / (2.0 * c->h)
                             : (c->fd == MH_FD_FORWARD ? (vp - v0) / c->h : (v0 - vm) / c->h);
            }
        }
        free(ein); free(cols); free(si);
    }
    for (int64_t e = e0; e < c->nnz; ++e) {
        int64_t row = c->iRow[e] - c->NEP, col = c->jCol[e];
        int i = (int)(row / rpi);
        int rl = (int)(row % rpi);
        double v = 0.0;
        int kc;
        int dir = col_to_dir(c, col, &kc);
        if (row >= (int64_t)c->N * rpi) {   /* final mesh point: kinematic and path rows, then residuals */
            int rt = (int)(row - (int64_t)c->N * rpi);
            if (rt < c->NK) { values[e] = D[((int64_t)(c->G - 1) * ND + dir) * NO + c->OKC + rt]; continue; }
            rt -= c->NK;
            if (rt < NPC) values[e] = Dp[((int64_t)c->N * ND + dir) * NPC + rt];
            else values[e] = D[((int64_t)(c->G - 1) * ND + dir) * NO + res_out(c, rt - NPC)];
            continue;
        }
        if (rl < c->NK) {                   /* kinematic rows of the interval's mesh point */
            values[e] = D[((int64_t)mesh_point(c, i) * ND + dir) * NO + c->OKC + rl];
            continue;
        }
        rl -= c->NK;
        if (rl < NPC) {                     /* path rows of the interval's mesh point */
            values[e] = Dp[((int64_t)i * ND + dir) * NPC + rl];
            continue;
        }
        rl -= NPC;
        if (rl < npts_res * NR) {           /* residual rows of the interval's points */
            int kr = (c->scheme == MH_HERMITE_SIMPSON ? 2 * i : i) + rl / NR;
            values[e] = D[((int64_t)kr * ND + dir) * NO + res_out(c, rl % NR)];
            continue;
        }
        rl -= npts_res * NR;
        if (c->scheme == MH_HERMITE_SIMPSON) {
            int ki = 2 * i, km = 2 * i + 1, kp = 2 * i + 2;
            double gi = c->grid[ki], gp = c->grid[kp];
            double h = times[kp] - times[ki];
            /* dh/dt0 = -(g_p - g_i), dh/dtf = (g_p - g_i) */
            double dh0 = -(gp - gi), dhf = (gp - gi);
            if (rl < NS) { /* Hermite: x_mid - .5(x_p + x_i) - h/8 (f_i - f_p) */
                int s = rl;
                const double* fi = xd + (int64_t)ki * NS;
                const double* fp = xd + (int64_t)kp * NS;
                if (dir >= PD) {   /* a parameter moves no time: the callbacks' quotients */
                    v = 0.0 - (h / 8.0) * (xdot_deriv(c, D, ki, s, dir) - xdot_deriv(c, D, kp, s, dir));
                } else if (dir < 2) {
                    double dh = dir == 0 ? dh0 : dhf;
                    v = -(dh / 8.0) * (fi[s] - fp[s]) -
                        (h / 8.0) * (xdot_deriv(c, D, ki, s, dir) - xdot_deriv(c, D, kp, s, dir));
                } else {
                    if (kc == km && dir == 2 + s) v += 1.0;
                    if (kc == ki) {
                        if (dir == 2 + s) v += -0.5;
                        v += -(h / 8.0) * xdot_deriv(c, D, ki, s, dir);
                    }
                    if (kc == kp) {
                        if (dir == 2 + s) v += -0.5;
                        v += (h / 8.0) * xdot_deriv(c, D, kp, s, dir);
                    }
                }
            } else if (rl < 2 * NS) { /* Simpson: x_p - x_i - h/6 (f_p + 4 f_m + f_i) */
                int s = rl - NS;
                const double* fi = xd + (int64_t)ki * NS;
                const double* fm = xd + (int64_t)km * NS;
                const double* fp = xd + (int64_t)kp * NS;
                if (dir >= PD) {
                    v = 0.0 - (h / 6.0) * (xdot_deriv(c, D, kp, s, dir) + 4.0 * xdot_deriv(c, D, km, s, dir) +
                                           xdot_deriv(c, D, ki, s, dir));
                } else if (dir < 2) {
                    double dh = dir == 0 ? dh0 : dhf;
                    v = -(dh / 6.0) * (fp[s] + 4.0 * fm[s] + fi[s]) -
                        (h / 6.0) * (xdot_deriv(c, D, kp, s, dir) + 4.0 * xdot_deriv(c, D, km, s, dir) +
                                     xdot_deriv(c, D, ki, s, dir));
                } else {
                    if (kc == kp) {
                        if (dir == 2 + s) v += 1.0;
                        v += -(h / 6.0) * xdot_deriv(c, D, kp, s, dir);
                    }
                    if (kc == ki) {
                        if (dir == 2 + s) v += -1.0;
                        v += -(h / 6.0) * xdot_deriv(c, D, ki, s, dir);
                    }
                    if (kc == km) v += -(h / 6.0) * 4.0 * xdot_deriv(c, D, km, s, dir);
                }
            } else { /* interpolating controls */
                v = (kc == km) ? 1.0 : -0.5;
            }
        } else {
            int ki = i, kp = i + 1;
            double gi = c->grid[ki], gp = c->grid[kp];
            double h = times[kp] - times[ki];
            double dh0 = -(gp - gi), dhf = (gp - gi);
            int s = rl;
            const double* fi = xd + (int64_t)ki * NS;
            const double* fp = xd + (int64_t)kp * NS;
            if (dir >= PD) {
                v = 0.0 - (0.5 * h) * (xdot_deriv(c, D, kp, s, dir) + xdot_deriv(c, D, ki, s, dir));
            } else if (dir < 2) {
                double dh = dir == 0 ? dh0 : dhf;
                v = -0.5 * dh * (fp[s] + fi[s]) -
                    0.5 * h * (xdot_deriv(c, D, kp, s, dir) + xdot_deriv(c, D, ki, s, dir));
            } else {
                if (kc == kp) {
                    if (dir == 2 + s) v += 1.0;
                    v += -0.5 * h * xdot_deriv(c, D, kp, s, dir);
                }
                if (kc == ki) {
                    if (dir == 2 + s) v += -1.0;
                    v += -0.5 * h * xdot_deriv(c, D, ki, s, dir);
                }
            }
        }
        values[e] = v;
    }
    (void)NQ;
}

/* tropter's calc_jacobian (ProblemDecorator_double.cpp:261-291): per seed,
 * g at x +- eps * seed (eps = sqrt(DBL_EPSILON)), central quotient,
 * recovered into the seed's nonzeros. */
static int jac_global_seeds(orc_ctx* c, const double* x, double* values) {
    double eps = sqrt(DBL_EPSILON), two_eps = 2 * eps;
    double* xp = (double*)malloc(sizeof(double) * (size_t)c->n);
    double* xm = (double*)malloc(sizeof(double) * (size_t)c->n);
    double* gp = (double*)malloc(sizeof(double) * (size_t)(c->m + 1));
    double* gm = (double*)malloc(sizeof(double) * (size_t)(c->m + 1));
    for (int k = 0; k < c->nseeds; ++k) {
        for (int64_t j = 0; j < c->n; ++j) {
            xp[j] = c->seed_color[j] == k ? x[j] + eps : x[j];
            xm[j] = c->seed_color[j] == k ? x[j] - eps : x[j];
        }
        orc_eval_g(c, xp, gp);
        orc_eval_g(c, xm, gm);
        for (int64_t e = 0; e < c->nnz; ++e)
            if (c->seed_color[c->jCol[e]] == k) values[e] = (gp[c->iRow[e]] - gm[c->iRow[e]]) / two_eps;
    }
    free(xp); free(xm); free(gp); free(gm);
    return MH_OK;
}

int orc_eval_jac_g(orc_ctx* c0, const double* x, double* values) {
    if (c0->jac_seeds) return jac_global_seeds(c0, x, values);
    orc_ctx* c = param_ctx(c0, x, -1, 0.0);   /* the iterate's parameters applied */
    int NS = c->NS, NO = nout(c), ND = ndir(c), NR = nres(c), NPC = c->NPC;
    double* times = (double*)malloc(sizeof(double) * (size_t)c->G);
    double* xd = (double*)calloc((size_t)c->G * (size_t)NS + 1, sizeof(double));
    double* D = (double*)calloc((size_t)c->G * (size_t)ND * (size_t)NO + 1, sizeof(double));
    double* res = (double*)calloc((size_t)c->G * (size_t)NR + 1, sizeof(double));
    double* Dp = (double*)calloc((size_t)(c->N + 1) * (size_t)ND * (size_t)NPC + 1, sizeof(double));
    double* kce = (double*)calloc((size_t)c->G * (size_t)c->NK + 1, sizeof(double));
    times_of(c, x, times);
    all_xdot(c, x, times, xd, res, kce);
    free(kce);
    fd_blocks(c, x, times, D);
    if (NPC) path_blocks(c, x, times, Dp);
    if (sharded(c)) {
        double* full = (double*)calloc((size_t)c->nnz + 1, sizeof(double));
        jac_assemble(c, x, times, xd, D, Dp, full);
        memcpy(values, full + c->nnz_begin, sizeof(double) * (size_t)(c->nnz_end - c->nnz_begin));
        free(full);
    } else {
        jac_assemble(c, x, times, xd, D, Dp, values);
    }
    free(Dp);
    free(times);
    free(xd);
    free(D);
    free(res);
    param_ctx_free(c0, c);
    return MH_OK;
}

/* g and the Jacobian values from given raw lane outputs (the layout of
 * mh_debug_jacobian_lanes): CasADi's FiniteDiff quotients of the lanes
 * (CasOCFunction.h:38-44) then g_assemble / jac_assemble.  The checker for
 * the device's quotient + assembly arithmetic. */
int orc_assemble_from_lanes(orc_ctx* c, const double* x, const double* times, const double* Y,
        double* g, double* values) {
    int NS = c->NS, NO = nout(c), ND = ndir(c), NR = nres(c), NPC = c->NPC, TQ = c->TQ;
    int S = c->fd == MH_FD_CENTRAL ? 2 * ND + 1 : ND + 1, base = S - 1;
    double h = c->h;
    double* xd = (double*)malloc(sizeof(double) * (size_t)c->G * (size_t)NS);
    double* D = (double*)malloc(sizeof(double) * (size_t)c->G * (size_t)ND * (size_t)NO);
    double* res = (double*)malloc(sizeof(double) * ((size_t)c->G * (size_t)NR + 1));
    double* kce = (double*)malloc(sizeof(double) * ((size_t)c->G * (size_t)c->NK + 1));
    double* Dp = (double*)malloc(sizeof(double) * ((size_t)(c->N + 1) * (size_t)ND * (size_t)NPC + 1));
    for (int k = 0; k < c->G; ++k) {
        const double* Yk = Y + (int64_t)k * NO * S;
        for (int r = 0; r < c->NK; ++r) kce[(int64_t)k * c->NK + r] = Yk[(int64_t)(c->OKC + r) * S + base];
        for (int s = 0; s < NS; ++s) {
            double v;
            if (s < TQ) {                                                   /* qdot = u */
                v = x[col_state(c, k, TQ + s)];
                if (vc_point(c, k)) v = v + Yk[(int64_t)(c->OQC + s) * S + base];
            }
            else if (c->NACC && s < 2 * TQ) v = x[col_deriv(c, k, s - TQ)];  /* udot = w */
            else v = Yk[(int64_t)(s + c->SO) * S + base];
            xd[(int64_t)k * NS + s] = v;
        }
        for (int r = 0; r < NR; ++r) res[(int64_t)k * NR + r] = Yk[(int64_t)res_out(c, r) * S + base];
        for (int d = 0; d < ND; ++d)
            for (int o = 0; o < NO; ++o) {
                const double* y = Yk + (int64_t)o * S;
                double q;
                if (c->fd == MH_FD_CENTRAL) q = (y[d] - y[ND + d]) / (2.0 * h);
                else if (c->fd == MH_FD_FORWARD) q = (y[d] - y[base]) / h;
                else q = (y[base] - y[d]) / h;
                D[((int64_t)k * ND + d) * NO + o] = q;
            }
    }
    if (NPC) path_blocks(c, x, times, Dp);
    if (g) g_assemble(c, x, times, xd, res, kce, g);
    if (values) jac_assemble(c, x, times, xd, D, Dp, values);
    free(kce);
    free(Dp);
    free(xd);
    free(D);
    free(res);
    return MH_OK;
}

/* ======================================================================== */
/* Objective.                                                                */
/* ======================================================================== */
/* Integrand of goal g at one point (MocoControlGoal.cpp:120-131,
 * MocoStateTrackingGoal.cpp:103-117). */
static double goal_integrand(const orc_ctx* c, const mh_goal* G, double t, const double* st,
        const double* ct) {
    double L = 0.0;
    for (int k = G->term_begin; k < G->term_begin + G->term_count; ++k) {
        int idx = c->gidx[k];
        double w = c->gw[k];
        if (G->kind == MH_GOAL_CONTROL) {
            double v = ct[idx];
            /* MocoControlGoal.cpp:98-107: x*x for exponent 2 */
            L += w * (G->exponent == 2 ? v * v : pow(fabs(v), G->exponent));
        } else if (G->kind == MH_GOAL_STATE_TRACKING) {
            double ref = table_eval(c, G->table, c->gcol[k], t);
            double d = st[idx] - ref;
            L += w * (d * d);
        } else if (G->kind == MH_GOAL_SUM_SQUARED_STATE) {
            double v = st[idx];
            L += w * (v * v);
        } else if (G->kind == MH_GOAL_AUX_DERIVATIVES) {
            double v = ct[c->NC + c->NACC + idx];   /* derivatives follow the controls */
            L += w * (v * v);
        } else if (G->kind == MH_GOAL_LAGRANGE_MULTIPLIERS) {
            double v = ct[c->NC + c->NDV + idx];    /* multipliers follow the derivatives */
            L += w * (v * v);
        }
    }
    return L;
}
static int goal_has_integral(const mh_goal* G) {
    return G->kind != MH_GOAL_FINAL_TIME && G->kind != MH_GOAL_MARKER_FINAL;
}

/* MocoMarkerFinalGoal::calcGoalImpl (MocoMarkerFinalGoal.cpp:29-34):
 * realizePosition at the final state, |location in ground - reference|^2
 * (SimTK normSqr: x*x + y*y + z*z).  st: the final grid point's states. */
static double marker_cost(const orc_ctx* c, const mh_goal* G, const double* st, dae_ws* w) {
    int k0 = G->term_begin, b = c->gidx[k0];
    kinematics(c, st, st + c->NQ, NULL, w);
    const real* R = w->R + 9 * (b + 1);
    const real* p = w->p + 3 * (b + 1);
    real loc[3] = {c->gw[k0], c->gw[k0 + 1], c->gw[k0 + 2]}, y[3];
    mat_vec(R, loc, y);
    double s = 0.0;
    for (int i = 0; i < 3; ++i) {
        double d = (p[i] + y[i]) - c->gw[k0 + 3 + i];
        s += d * d;
    }
    return s;
}

/* The shard's own quadrature (mh_eval_f_partial): the intervals [ib, ie)
 * accumulated as c->quad is, so an unsharded context's partial is its
 * objective bit for bit. */
static double* shard_quad(const orc_ctx* c) {
    double* q = (double*)calloc((size_t)c->G, sizeof(double));
    for (int i = c->ib; i < c->ie; ++i) {
        double dm = (i + 1) / (double)c->N - i / (double)c->N;
        if (c->scheme == MH_HERMITE_SIMPSON) {
            q[2 * i] += (1.0 / 6.0) * dm;
            q[2 * i + 1] += (2.0 / 3.0) * dm;
            q[2 * i + 2] += (1.0 / 6.0) * dm;
        } else {
            q[i] += 0.5 * dm;
            q[i + 1] += 0.5 * dm;
        }
    }
    return q;
}

static int eval_f_impl(orc_ctx* c, const double* x, double* f, const double* quad, int endpoint);
static int eval_grad_f_impl(orc_ctx* c, const double* x, double* grad, const double* quad, int endpoint);

int orc_eval_f(orc_ctx* c, const double* x, double* f) { return eval_f_impl(c, x, f, c->quad, 1); }
int orc_eval_grad_f(orc_ctx* c, const double* x, double* grad) {
    return eval_grad_f_impl(c, x, grad, c->quad, 1);
}
int orc_eval_f_partial(orc_ctx* c, const double* x, double* f) {
    double* q = shard_quad(c);
    int rc = eval_f_impl(c, x, f, q, c->ie == c->N);
    free(q);
    return rc;
}
int orc_eval_grad_f_partial(orc_ctx* c, const double* x, double* grad) {
    double* q = shard_quad(c);
    int rc = eval_grad_f_impl(c, x, grad, q, c->ie == c->N);
    free(q);
    return rc;
}

static int eval_f_impl(orc_ctx* c, const double* x, double* f, const double* quad, int endpoint) {
    double* times = (double*)malloc(sizeof(double) * (size_t)c->G);
    double* st = (double*)malloc(sizeof(double) * (size_t)(c->NP + 1));
    double* ct = st + c->NS;
    times_of(c, x, times);
    double total = 0.0;
    /* CasOCTranscription.cpp:478-511: cost = weight * (tf-t0) * dot(quad, L) */
    for (int g = 0; g < c->P.ngoals; ++g) {
        const mh_goal* G = &c->goals[g];
        double cost;
        if (G->kind == MH_GOAL_MARKER_FINAL) {
            if (!endpoint) continue;
            dae_ws w;
            ws_alloc(c, &w);
            gather_point(c, x, c->G - 1, st, ct);
            cost = G->weight * marker_cost(c, G, st, &w);
            ws_free(&w);
        } else if (goal_has_integral(G)) {
            double acc = 0.0;
            for (int k = 0; k < c->G; ++k) {
                gather_point(c, x, k, st, ct);
                acc += quad[k] * goal_integrand(c, G, times[k], st, ct);
            }
            double integral = (x[1] - x[0]) * acc;
            cost = G->weight * integral;
        } else {
            if (!endpoint) continue;
            cost = G->weight * x[1];
        }
        total += cost;
    }
    *f = total;
    free(times);
    free(st);
    return MH_OK;
}

static int eval_grad_f_impl(orc_ctx* c, const double* x, double* grad, const double* quad, int endpoint) {
    int NS = c->NS, NP = c->NP;
    double h = c->h;
    double* times = (double*)malloc(sizeof(double) * (size_t)c->G);
    double* in = (double*)malloc(sizeof(double) * (size_t)(NP + 1));
    times_of(c, x, times);
    for (int64_t i = 0; i < c->n; ++i) grad[i] = 0.0;
    double dur = x[1] - x[0];
    for (int g = 0; g < c->P.ngoals; ++g) {
        const mh_goal* G = &c->goals[g];
        if (G->kind == MH_GOAL_MARKER_FINAL) {
            if (!endpoint) continue;
            /* FD of the cost over the final coordinates (the other final
             * states do not change a Position-stage cost: exactly 0) */
            dae_ws w;
            ws_alloc(c, &w);
            gather_point(c, x, c->G - 1, in, in + NS);
            double c0 = marker_cost(c, G, in, &w);
            for (int s = 0; s < c->NQ; ++s) {
                double v = in[s], cp = 0.0, cm = 0.0;
                if (c->fd != MH_FD_BACKWARD) { in[s] = v + h; cp = marker_cost(c, G, in, &w); }
                if (c->fd != MH_FD_FORWARD) { in[s] = v - h; cm = marker_cost(c, G, in, &w); }
                in[s] = v;
                double d = c->fd == MH_FD_CENTRAL ? (cp - cm) / (2.0 * h)
                         : (c->fd == MH_FD_FORWARD ? (cp - c0) / h : (c0 - cm) / h);
                grad[col_state(c, c->G - 1, s)] += G->weight * d;
            }
            ws_free(&w);
            continue;
        }
        if (!goal_has_integral(G)) { if (endpoint) grad[1] += G->weight; continue; }
        double acc = 0.0;
        for (int k = 0; k < c->G; ++k) {
            gather_point(c, x, k, in, in + NS);
            double t = times[k];
            double L0 = goal_integrand(c, G, t, in, in + NS);
            acc += quad[k] * L0;
            double wq = G->weight * dur * quad[k];
            for (int d = 0; d < c->NPD + 2; ++d) {   /* the goal callback's inputs */
                double seed = d == 0 ? 1.0 - c->grid[k] : (d == 1 ? c->grid[k] : 1.0);
                double lp = 0, lm = 0;
                int idx = d - 2;
                if (c->fd != MH_FD_BACKWARD) {
                    if (idx < 0) lp = goal_integrand(c, G, t + h * seed, in, in + NS);
                    else { double s = in[idx]; in[idx] = s + h; lp = goal_integrand(c, G, t, in, in + NS); in[idx] = s; }
                }
                if (c->fd != MH_FD_FORWARD) {
                    if (idx < 0) lm = goal_integrand(c, G, t - h * seed, in, in + NS);
                    else { double s = in[idx]; in[idx] = s - h; lm = goal_integrand(c, G, t, in, in + NS); in[idx] = s; }
                }
                double dL = c->fd == MH_FD_CENTRAL ? (lp - lm) / (2.0 * h)
                          : (c->fd == MH_FD_FORWARD ? (lp - L0) / h : (L0 - lm) / h);
                if (G->kind == MH_GOAL_LAGRANGE_MULTIPLIERS) {
                    /* exact (the reference differentiates this MX term with
                     * AD): d(w lambda^2)/d lambda = w 2 lambda */
                    int j = idx - (NS + c->NC + c->NDV);
                    dL = (idx >= 0 && j >= 0 && j < c->NM) ? c->gw[G->term_begin + j] * (2.0 * in[idx]) : 0.0;
                }
                int64_t col;
                if (d == 0) col = 0;
                else if (d == 1) col = 1;
                else col = col_input(c, k, idx);
                grad[col] += wq * dL;
            }
        }
        /* d/dt0 and d/dtf of the duration factor */
        grad[0] += -G->weight * acc;
        grad[1] += G->weight * acc;
    }
    free(times);
    free(in);
    return MH_OK;
}
#endif /* ORACLE_COUNTING */
