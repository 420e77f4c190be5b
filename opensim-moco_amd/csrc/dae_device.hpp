// dae_device.hpp — per-grid-point explicit DAE on gfx950 (one lane = one
// evaluation).  Replaces CasOC::Problem::calcMultibodySystemExplicit
// (Moco/Moco/MocoCasADiSolver/MocoCasOCProblem.h:203-244) and the Simbody /
// OpenSim realize chain behind it for the model class of include/mocohip.h:
//   * FunctionBased mobilizers (Pin/Slider/Planar/Custom joints), ground-frame
//     spatial algebra, RNEA bias forces, CRBA mass matrix, dense Cholesky;
//   * GeometryPath with Conditional/Moving path points; tension applied as
//     point forces; MovingPathPoint generalized-force terms;
//   * DeGrooteFregly2016Muscle (DeGrooteFregly2016Muscle.cpp:186-425);
//   * ExternalForce from piecewise-polynomial tables; CoordinateActuators.
// All arithmetic is FP64 VALU.  Size classes (template parameters) bound the
// per-lane arrays so that small models stay in VGPRs and large ones spill to
// scratch with a lane-interleaved (coalesced) layout.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/mocohip.h"

namespace mh {

struct DevModel {
    int nq, nb, nmus, nact, next, ns, nz, nc, no, np;
    int implicit;   // MH_DYNAMICS_IMPLICIT: inputs carry udot after the controls
    int nacc;       // acceleration inputs after the controls (implicit: nq)
    const int* mus_ider;  // muscle -> implicit tendon-force derivative input
                          // (index after the controls), -1 = explicit
    int presc;            // prescribed kinematics: q, u, udot from kin_table
    int kin_table;
    const int* kin_col;   // [nq] table column of each coordinate
    double gravity[3];
    double tau_act, tau_deact;
    const mh_body* bodies;
    const mh_axis* axes;
    const mh_function* funcs;
    const double* kx;
    const double* ky;
    const double* kb;
    const double* kc;
    const double* kd;
    const mh_muscle* mus;
    const mh_path_point* pts;
    const mh_actuator* acts;
    const mh_table* tabs;
    const double* brk;
    const double* coef;
    const mh_external_force* ext;
    const int* coord_body;
    const int* mus_act_state;
    const int* mus_ftn_state;
    const int* mus_control;
    const double* mus_derived;   // per muscle: fiberWidth, squareFiberWidth, vmax, kT, e0 offset, passive denom
    // kinematic constraints (CoordinateCoupler, include/mocohip.h
    // mh_constraint): count, table, callback output of the first error and
    // of the velocity correction (-1: none), derivative levels enforced,
    // offset of the multipliers after the controls pointer (the slacks
    // follow them)
    int nkc;
    const mh_constraint* kcs;
    int okc, oqc, enforce, mult;
    // muscle wrapping (ABI v5): wrap surfaces, PathWrap entries grouped by
    // muscle, each muscle's first entry and count
    const mh_wrap_object* wr;
    const mh_path_wrap* pw;
    const int* mus_pw_begin;
    const int* mus_pw_count;
    // generated back ends: the model's constant pool (codegen.py
    // "Structure-only specialization"; <Name>_fill at mh_create), else null
    const double* pool;
    // SpringGeneralizedForce elements (ABI v8)
    int nsp;
    const mh_spring* sp;
};
// The generated code reads the constant pool through the constant address
// space: the pool does not change during a launch, so its wave-uniform reads
// compile to scalar loads (SMEM through the scalar cache, into SGPRs) instead
// of vector loads that share the lanes' input loads' queue and wait counter.
typedef __attribute__((address_space(4))) const double kconst;
__device__ __forceinline__ const kconst* kpool(const DevModel& M) { return (const kconst*)M.pool; }
constexpr int MUS_DERIVED = 6;

struct SV { double w0, w1, w2, v0, v1, v2; };

__device__ __forceinline__ SV sv_zero() { return SV{0, 0, 0, 0, 0, 0}; }
__device__ __forceinline__ void cross3(double a0, double a1, double a2, double b0, double b1,
        double b2, double& c0, double& c1, double& c2) {
    c0 = a1 * b2 - a2 * b1;
    c1 = a2 * b0 - a0 * b2;
    c2 = a0 * b1 - a1 * b0;
}
// motion cross product a x_m b
__device__ __forceinline__ SV crm(const SV& a, const SV& b) {
    SV r;
    cross3(a.w0, a.w1, a.w2, b.w0, b.w1, b.w2, r.w0, r.w1, r.w2);
    double t0, t1, t2;
    cross3(a.w0, a.w1, a.w2, b.v0, b.v1, b.v2, r.v0, r.v1, r.v2);
    cross3(a.v0, a.v1, a.v2, b.w0, b.w1, b.w2, t0, t1, t2);
    r.v0 += t0; r.v1 += t1; r.v2 += t2;
    return r;
}
// force cross product a x_f f
__device__ __forceinline__ SV crf(const SV& a, const SV& f) {
    SV r;
    double t0, t1, t2;
    cross3(a.w0, a.w1, a.w2, f.w0, f.w1, f.w2, r.w0, r.w1, r.w2);
    cross3(a.v0, a.v1, a.v2, f.v0, f.v1, f.v2, t0, t1, t2);
    r.w0 += t0; r.w1 += t1; r.w2 += t2;
    cross3(a.w0, a.w1, a.w2, f.v0, f.v1, f.v2, r.v0, r.v1, r.v2);
    return r;
}
__device__ __forceinline__ double svdot(const SV& m, const SV& f) {
    return m.w0 * f.w0 + m.w1 * f.w1 + m.w2 * f.w2 + m.v0 * f.v0 + m.v1 * f.v1 + m.v2 * f.v2;
}

// Rigid-body inertia about the ground origin.
struct RBI { double m, h0, h1, h2, I0, I1, I2, I3, I4, I5; };
__device__ __forceinline__ SV rbi_mul(const RBI& I, const SV& x) {
    SV r;
    double t0, t1, t2;
    r.w0 = I.I0 * x.w0 + I.I3 * x.w1 + I.I4 * x.w2;
    r.w1 = I.I3 * x.w0 + I.I1 * x.w1 + I.I5 * x.w2;
    r.w2 = I.I4 * x.w0 + I.I5 * x.w1 + I.I2 * x.w2;
    cross3(I.h0, I.h1, I.h2, x.v0, x.v1, x.v2, t0, t1, t2);
    r.w0 += t0; r.w1 += t1; r.w2 += t2;
    cross3(I.h0, I.h1, I.h2, x.w0, x.w1, x.w2, t0, t1, t2);
    r.v0 = I.m * x.v0 - t0;
    r.v1 = I.m * x.v1 - t1;
    r.v2 = I.m * x.v2 - t2;
    return r;
}

struct Pose { double R[9]; double p[3]; };

__device__ __forceinline__ void mm3(const double* A, const double* B, double* C) {
    double T[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            T[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
    for (int i = 0; i < 9; ++i) C[i] = T[i];
}
__device__ __forceinline__ void mv3(const double* A, double x0, double x1, double x2, double& y0,
        double& y1, double& y2) {
    y0 = A[0] * x0 + A[1] * x1 + A[2] * x2;
    y1 = A[3] * x0 + A[4] * x1 + A[5] * x2;
    y2 = A[6] * x0 + A[7] * x1 + A[8] * x2;
}
__device__ __forceinline__ void axis_rot(double a0, double a1, double a2, double t, double* R) {
    double s, c;
    sincos(t, &s, &c);
    double k = 1.0 - c;
    R[0] = c + k * a0 * a0;
    R[1] = k * a0 * a1 - s * a2;
    R[2] = k * a0 * a2 + s * a1;
    R[3] = k * a1 * a0 + s * a2;
    R[4] = c + k * a1 * a1;
    R[5] = k * a1 * a2 - s * a0;
    R[6] = k * a2 * a0 - s * a1;
    R[7] = k * a2 * a1 + s * a0;
    R[8] = c + k * a2 * a2;
}

// OpenSim SimmSpline evaluation (value, d/dq, d2/dq2) with linear
// extrapolation; binary search over the knots.
__device__ __forceinline__ void simm_eval(const DevModel& M, const mh_function& F, double t,
        double& v, double& d1, double& d2) {
    const int n = F.knot_count;
    const double* x = M.kx + F.knot_begin;
    const double* y = M.ky + F.knot_begin;
    const double* b = M.kb + F.knot_begin;
    const double* c = M.kc + F.knot_begin;
    const double* d = M.kd + F.knot_begin;
    if (n == 1) { v = y[0]; d1 = 0; d2 = 0; return; }
    if (t < x[0]) { v = y[0] + (t - x[0]) * b[0]; d1 = b[0]; d2 = 0.0; return; }
    if (t > x[n - 1]) { v = y[n - 1] + (t - x[n - 1]) * b[n - 1]; d1 = b[n - 1]; d2 = 0.0; return; }
    int k;
    if (fabs(t - x[0]) <= 2e-13) k = 0;
    else if (fabs(t - x[n - 1]) <= 2e-13) k = n - 1;
    else {
        int lo = 0, hi = n;
        for (;;) {
            k = (lo + hi) >> 1;
            if (t < x[k]) hi = k;
            else if (t > x[k + 1]) lo = k;
            else break;
        }
    }
    double dx = t - x[k];
    v = y[k] + dx * (b[k] + dx * (c[k] + dx * d[k]));
    d1 = b[k] + dx * (2.0 * c[k] + 3.0 * dx * d[k]);
    d2 = 2.0 * c[k] + 6.0 * dx * d[k];
}

__device__ __forceinline__ void fn_eval(const DevModel& M, int f, const double* q, double& v,
        double& d1, double& d2) {
    const mh_function F = M.funcs[f];
    if (F.kind == MH_FN_CONSTANT) { v = F.a; d1 = 0; d2 = 0; return; }
    if (F.kind == MH_FN_LINEAR) {
        v = F.scale * (F.a * q[F.coord] + F.b);
        d1 = F.scale * F.a;
        d2 = 0.0;
        return;
    }
    simm_eval(M, F, q[F.coord], v, d1, d2);
    v *= F.scale; d1 *= F.scale; d2 *= F.scale;
}

// Value, first and second derivative of a table column (PositionMotion:
// q, u = dq/dt, udot = d2q/dt2 of one spline, PositionMotion.cpp:36-70).
__device__ __forceinline__ void table_eval_d(const DevModel& M, int ti, int col, double t, double& v,
        double& d1, double& d2) {
    const mh_table T = M.tabs[ti];
    const double* br = M.brk + T.break_begin;
    int s;
    if (t <= br[0]) s = 0;
    else if (t >= br[T.nseg]) s = T.nseg - 1;
    else {
        int lo = 0, hi = T.nseg;
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (t < br[mid]) hi = mid; else lo = mid;
        }
        s = lo;
    }
    const double* cf = M.coef + T.coef_begin + ((long)s * T.ncol + col) * (T.degree + 1);
    const double dt = t - br[s];
    double p = cf[T.degree], dp = 0.0, ddp = 0.0;
    for (int k = T.degree - 1; k >= 0; --k) {
        ddp = ddp * dt + 2.0 * dp;
        dp = dp * dt + p;
        p = p * dt + cf[k];
    }
    v = p; d1 = dp; d2 = ddp;
}

__device__ __forceinline__ double table_eval(const DevModel& M, int ti, int col, double t) {
    const mh_table T = M.tabs[ti];
    const double* br = M.brk + T.break_begin;
    int s;
    if (t <= br[0]) s = 0;
    else if (t >= br[T.nseg]) s = T.nseg - 1;
    else {
        int lo = 0, hi = T.nseg;
        while (hi - lo > 1) {
            int mid = (lo + hi) >> 1;
            if (t < br[mid]) hi = mid; else lo = mid;
        }
        s = lo;
    }
    const double* cf = M.coef + T.coef_begin + ((long)s * T.ncol + col) * (T.degree + 1);
    double dt = t - br[s];
    double v = cf[T.degree];
    for (int k = T.degree - 1; k >= 0; --k) v = v * dt + cf[k];
    return v;
}

// ---- DeGrooteFregly2016 curves (DeGrooteFregly2016Muscle.h:332-476) ----
__device__ __forceinline__ double gauss_like(double x, double b1, double b2, double b3, double b4) {
    double num = (x - b2) * (x - b2);
    double den = (b3 + b4 * x) * (b3 + b4 * x);
    return b1 * exp(-0.5 * num / den);
}
__device__ __forceinline__ double dgf_fal(double scale, double l) {
    double x = (l - 1.0) / scale + 1.0;
    return gauss_like(x, 0.8150671134243542, 1.055033428970575, 0.162384573599574,
                   0.063303448465465) +
           gauss_like(x, 0.433004984392647, 0.716775413397760, -0.029947116970696,
                   0.200356847296188) +
           gauss_like(x, 0.1, 1.0, 0.353553390593274, 0.0);
}
constexpr double DGF_d1 = -0.3211346127989808, DGF_d2 = -8.149, DGF_d3 = -0.374,
                 DGF_d4 = 0.8825327733249912, DGF_c1 = 0.2, DGF_c2 = 1.0, DGF_c3 = 0.2;
__device__ __forceinline__ double dgf_fv(double v) {
    double tv = DGF_d2 * v + DGF_d3;
    double arg = tv + sqrt(tv * tv + 1.0);
    return DGF_d1 * log(arg) + DGF_d4;
}
__device__ __forceinline__ double dgf_fv_inv(double fv) {
    return (sinh(1.0 / DGF_d1 * (fv - DGF_d4)) - DGF_d3) / DGF_d2;
}

// DeGroote-Fregly activation dynamics (DeGrooteFregly2016Muscle.cpp:186-233,
// computeStateVariableDerivatives; oracle/oracle.c dgf).  Without contraction, so the generic
// interpreter's excitation lanes (k_exc_lanes) reproduce the full
// evaluation's value bit for bit.
__device__ __forceinline__ double dgf_adot(const DevModel& M, double act, double exc) {
#pragma clang fp contract(off)
    double tcf = 0.5 + 1.5 * act;
    double tempAct = 1.0 / (M.tau_act * tcf);
    double tempDeact = tcf / M.tau_deact;
    double f = 0.5 * tanh(0.1 * (exc - act));
    double timeConst = tempAct * (f + 0.5) + tempDeact * (-f + 0.5);
    return timeConst * (exc - act);
}

// Muscle tendon force and auxiliary derivatives.
// implicit_tendon: tendon_compliance_dynamics_mode "implicit" with the
// normalized tendon force derivative dft as input; resid = the equilibrium
// residual FT - FM cos(alpha) (DeGrooteFregly2016Muscle.cpp:826-848).
__device__ __forceinline__ void dgf_eval(const DevModel& M, int im, double LMT, double VMT,
        double act, double exc, bool has_act, double ftn, bool compliant, double& T,
        double& adot, double& ftdot, bool implicit_tendon = false, double dft = 0.0,
        double* resid = nullptr) {
    const mh_muscle& mu = M.mus[im];
    const double* dv = M.mus_derived + (long)im * MUS_DERIVED;
    const double fiberWidth = dv[0], sqW = dv[1], vmax = dv[2], kT = dv[3];
    const double peOffset = dv[4], peDenom = dv[5];
    const double lopt = mu.optimal_fiber_length, lts = mu.tendon_slack_length;
    double normTendonLength = 1.0;
    if (compliant) normTendonLength = log((1.0 / DGF_c1) * (ftn + DGF_c3)) / kT + DGF_c2;
    double tendonLength = lts * normTendonLength;
    double flat = LMT - tendonLength;
    double fiberLength = sqrt(flat * flat + sqW);
    double nfl = fiberLength / lopt;
    double cosPenn = flat / fiberLength;
    double fPE = 0.0;
    if (!mu.ignore_passive_fiber_force) {
        const double e0 = mu.passive_fiber_strain_at_one_norm_force;
        fPE = (exp(4.0 * (nfl - 1.0) / e0) - peOffset) / peDenom;
    }
    double fAL = dgf_fal(mu.active_force_width_scale, nfl);
    double nfv, fV, ntv;
    if (compliant && !implicit_tendon) {
        double nff = ftn / cosPenn;
        fV = (nff - fPE) / (act * fAL);
        nfv = dgf_fv_inv(fV);
        double fiberVelocity = nfv * vmax;
        double fvat = fiberVelocity / cosPenn;
        double tendonVelocity = VMT - fvat;
        ntv = tendonVelocity / lts;
    } else {
        // rigid, or implicit: tendon velocity from the force derivative
        // (calcTendonForceLengthInverseCurveDerivative, .h:471-476)
        ntv = compliant ? dft / (DGF_c1 * kT * exp(kT * (normTendonLength - DGF_c2))) : 0.0;
        double tendonVelocity = lts * ntv;
        double fvat = VMT - tendonVelocity;
        double fiberVelocity = fvat * cosPenn;
        nfv = fiberVelocity / vmax;
        fV = dgf_fv(nfv);
    }
    const double Fmax = mu.max_isometric_force;
    double activeF = Fmax * (act * fAL * fV);
    double conPass = Fmax * fPE;
    double nonCon = Fmax * mu.fiber_damping * nfv;
    double total = activeF + conPass + nonCon;
    T = compliant ? Fmax * ftn : total * cosPenn;
    if (implicit_tendon) *resid = T - total * cosPenn;
    if (has_act) adot = dgf_adot(M, act, exc);
    if (compliant)
        ftdot = implicit_tendon ? dft : ntv * (DGF_c1 * kT * exp(kT * (normTendonLength - DGF_c2)));
    (void)fiberWidth;
}

// ---- muscle wrapping over cylinders -------------------------------------
// The oracle's wrap_cylinder / wrap_segment / apply_wraps (oracle/oracle.c:
// GeometryPath::applyWrapObjects, WrapObject::wrapPathSegment,
// WrapCylinder::wrapLine restated), operation for operation.
enum { DW_NONE = 0, DW_INSIDE = 1, DW_WRAPPED = 2 };
__device__ inline int dev_wrap_cylinder(const mh_wrap_object& W, const double* a, const double* b,
        double* r1, double* r2, double& wlen) {
#pragma clang fp contract(off)
    const double R = W.radius, R2 = R * R;
    const double a2 = a[0] * a[0] + a[1] * a[1], b2 = b[0] * b[0] + b[1] * b[1];
    if (a2 < R2 || b2 < R2) return DW_INSIDE;
    const double d0 = b[0] - a[0], d1 = b[1] - a[1];
    const double dd = d0 * d0 + d1 * d1;
    const double t = dd > 0.0 ? -(a[0] * d0 + a[1] * d1) / dd : 0.0;
    const double n0 = a[0] + t * d0, n1 = a[1] + t * d1;
    const bool hits = (n0 * n0 + n1 * n1 < R2) && t > 0.0 && t < 1.0;
    const double cr = a[0] * b[1] - a[1] * b[0];
    const double sshort = cr < 0.0 ? -1.0 : 1.0;
    double sigma = sshort;
    if (W.wrap_sign != 0) {
        const double nk = W.wrap_axis == 0 ? n0 : n1;
        if (nk * (double)W.wrap_sign >= 0.0) {
            if (!hits) return DW_NONE;
        } else {
            sigma = -sshort;
        }
    } else if (!hits) {
        return DW_NONE;
    }
    const double ra = sqrt(a2), rb = sqrt(b2);
    const double th1 = atan2(a[1], a[0]) + sigma * acos(R / ra);
    const double th2 = atan2(b[1], b[0]) - sigma * acos(R / rb);
    double dth = sigma * (th2 - th1);
    const double twopi = 6.283185307179586;
    while (dth < 0.0) dth = dth + twopi;
    while (dth >= twopi) dth = dth - twopi;
    const double l1 = sqrt(a2 - R2), l2 = sqrt(b2 - R2), arc = R * dth;
    const double Lxy = l1 + arc + l2;
    const double dz = b[2] - a[2];
    const double z1 = a[2] + dz * (l1 / Lxy), z2 = a[2] + dz * ((l1 + arc) / Lxy);
    r1[0] = R * cos(th1); r1[1] = R * sin(th1); r1[2] = z1;
    r2[0] = R * cos(th2); r2[1] = R * sin(th2); r2[2] = z2;
    const double zz = z2 - z1;
    wlen = sqrt(arc * arc + zz * zz);
    return DW_WRAPPED;
}

// A muscle's current path on the device: ground positions / velocities,
// the path point (>= 0) or -1 for a tangent point, its PathWrap entry, the
// body it is on, the surface length stored on a wrap's second point.
template <int MP>
struct CPath {
    double P[MP][3], V[MP][3];
    int pt[MP], pwi[MP], body[MP];
    double wlen[MP];
    int n;
    __device__ __forceinline__ bool arc(int k) const {   // segment k-1 -> k over a surface
        return pt[k] < 0 && pt[k - 1] < 0 && pwi[k] == pwi[k - 1];
    }
    __device__ __forceinline__ void move(int dst, int src) {
        for (int d = 0; d < 3; ++d) { P[dst][d] = P[src][d]; V[dst][d] = V[src][d]; }
        pt[dst] = pt[src]; pwi[dst] = pwi[src]; body[dst] = body[src]; wlen[dst] = wlen[src];
    }
};

__device__ __forceinline__ double dev_dist3(const double* a, const double* b) {
#pragma clang fp contract(off)
    const double d0 = b[0] - a[0], d1 = b[1] - a[1], d2 = b[2] - a[2];
    return sqrt(d0 * d0 + d1 * d1 + d2 * d2);
}

template <int MP>
__device__ inline double dev_cpath_length(const CPath<MP>& C) {
#pragma clang fp contract(off)
    double L = 0.0;
    for (int k = 1; k < C.n; ++k) L += C.arc(k) ? C.wlen[k] : dev_dist3(C.P[k - 1], C.P[k]);
    return L;
}

template <class POSE, class VEL>
__device__ inline void dev_body_station(const POSE& Pb, const VEL& Vb, const double* loc, double* P, double* V) {
#pragma clang fp contract(off)
    double t0, t1, t2;
    t0 = Pb.R[0] * loc[0] + Pb.R[1] * loc[1] + Pb.R[2] * loc[2];
    t1 = Pb.R[3] * loc[0] + Pb.R[4] * loc[1] + Pb.R[5] * loc[2];
    t2 = Pb.R[6] * loc[0] + Pb.R[7] * loc[1] + Pb.R[8] * loc[2];
    P[0] = Pb.p[0] + t0; P[1] = Pb.p[1] + t1; P[2] = Pb.p[2] + t2;
    if (V) {
        cross3(Vb.w0, Vb.w1, Vb.w2, P[0], P[1], P[2], t0, t1, t2);
        V[0] = Vb.v0 + t0; V[1] = Vb.v1 + t1; V[2] = Vb.v2 + t2;
    }
}

// WrapObject::wrapPathSegment: ends to the cylinder frame, wrapLine, tangent
// points back to the body frame.
template <class POSE>
__device__ inline int dev_wrap_segment(const mh_wrap_object& W, const POSE& Pb, const double* A,
        const double* B, double* r1B, double* r2B, double& wlen) {
#pragma clang fp contract(off)
    double pw[2][3];
    const double* E[2] = {A, B};
    for (int e = 0; e < 2; ++e) {
        const double g0 = E[e][0] - Pb.p[0], g1 = E[e][1] - Pb.p[1], g2 = E[e][2] - Pb.p[2];
        double sb[3];
        for (int i = 0; i < 3; ++i) sb[i] = Pb.R[i] * g0 + Pb.R[3 + i] * g1 + Pb.R[6 + i] * g2;
        for (int i = 0; i < 3; ++i) sb[i] = sb[i] - W.p_BW[i];
        for (int i = 0; i < 3; ++i) pw[e][i] = W.R_BW[i] * sb[0] + W.R_BW[3 + i] * sb[1] + W.R_BW[6 + i] * sb[2];
    }
    double r1[3], r2[3];
    const int res = dev_wrap_cylinder(W, pw[0], pw[1], r1, r2, wlen);
    if (res != DW_WRAPPED) return res;
    for (int i = 0; i < 3; ++i) {
        r1B[i] = W.R_BW[3 * i] * r1[0] + W.R_BW[3 * i + 1] * r1[1] + W.R_BW[3 * i + 2] * r1[2] + W.p_BW[i];
        r2B[i] = W.R_BW[3 * i] * r2[0] + W.R_BW[3 * i + 1] * r2[1] + W.R_BW[3 * i + 2] * r2[2] + W.p_BW[i];
    }
    return res;
}

// GeometryPath::applyWrapObjects on the current path C of muscle im
// (pact(i): whether original path point i is active).
template <int MP, class POSES, class VELS, class ACTIVE>
__device__ inline void dev_apply_wraps(const DevModel& M, int im, const POSES& X, const VELS& Vs,
        const ACTIVE& pact, CPath<MP>& C) {
#pragma clang fp contract(off)
    const mh_muscle& mu = M.mus[im];
    int nw = M.mus_pw_count[im];
    const int pb = M.mus_pw_begin[im];
    int order[8], result[8];
    if (nw > 8) nw = 8;
    for (int i = 0; i < nw; ++i) { order[i] = i; result[i] = DW_NONE; }
    const int maxit = nw < 2 ? 1 : 8;
    double last = __builtin_inf();
    for (int kk = 0; kk < maxit; ++kk) {
        for (int i = 0; i < nw; ++i) {
            result[i] = DW_NONE;
            const int pwi = pb + order[i];
            const mh_path_wrap PW = M.pw[pwi];
            const mh_wrap_object& W = M.wr[PW.wrap];
            for (int j = 0; j < C.n; ++j)
                if (C.pt[j] < 0 && C.pwi[j] == pwi) {
                    for (int k = j; k + 2 < C.n; ++k) C.move(k, k + 2);
                    C.n -= 2;
                    break;
                }
            const int ws = PW.range_begin < 1 ? 0 : PW.range_begin - 1;
            const int we = PW.range_end < 1 ? mu.point_count - 1 : PW.range_end - 1;
            int jf = ws, jr = we;
            while (jf <= we && !pact(mu.point_begin + jf)) ++jf;
            if (jf > we) return;
            while (jr >= ws && !pact(mu.point_begin + jr)) --jr;
            if (jr < ws) return;
            int start = -1, end = -1;
            for (int j = 0; j < C.n; ++j) {
                if (C.pt[j] == mu.point_begin + jf) start = j;
                if (C.pt[j] == mu.point_begin + jr) end = j;
            }
            if (start < 0 || end < 0) return;
            const int bs = W.body + 1;
            int best = -1;
            double bestc = __builtin_inf(), br1[3] = {0, 0, 0}, br2[3] = {0, 0, 0}, bl = 0.0;
            for (int k = start; k < end; ++k) {
                if (C.arc(k + 1)) continue;
                double r1[3], r2[3], wl;
                result[i] = dev_wrap_segment(W, X[bs], C.P[k], C.P[k + 1], r1, r2, wl);
                if (result[i] != DW_WRAPPED) continue;
                double g1[3], g2[3];
                dev_body_station(X[bs], Vs[bs], r1, g1, (double*)nullptr);
                dev_body_station(X[bs], Vs[bs], r2, g2, (double*)nullptr);
                const double chg = dev_dist3(C.P[k], g1) + wl + dev_dist3(g2, C.P[k + 1]) -
                                   dev_dist3(C.P[k], C.P[k + 1]);
                if (chg < bestc) {
                    bestc = chg; best = k; bl = wl;
                    for (int d = 0; d < 3; ++d) { br1[d] = r1[d]; br2[d] = r2[d]; }
                }
            }
            if (best >= 0 && C.n + 2 <= MP) {
                for (int k = C.n - 1; k > best; --k) C.move(k + 2, k);
                C.n += 2;
                for (int e = 0; e < 2; ++e) {
                    const int q = best + 1 + e;
                    C.pt[q] = -1; C.pwi[q] = pwi; C.body[q] = W.body;
                    C.wlen[q] = e ? bl : 0.0;
                    dev_body_station(X[bs], Vs[bs], e ? br2 : br1, C.P[q], C.V[q]);
                }
            }
        }
        const double L = dev_cpath_length(C);
        if (fabs(L - last) < 0.0005) break;
        last = L;
        if (kk == 0 && nw > 1 && result[0] == DW_NONE && result[1] == DW_INSIDE) {
            const int t = order[0]; order[0] = order[1]; order[1] = t;
        }
    }
}

// ---- wrapped muscles in generated back ends (codegen.py wrapped_muscle) ----
// The generated code builds the active path points (positions, velocities)
// of a wrapped muscle in straight-line code, then hands the data-dependent
// part -- GeometryPath::applyWrapObjects (dev_apply_wraps above, the
// interpreter's own), the path length and lengthening speed, and the point
// forces of the tension -- to these two helpers.  Poses / velocities of the
// wrap bodies come from the generated kinematics (xb: pose index = body + 1).
template <int NWB>
struct GenWrapPoses {
    const Pose* p;
    const int* b;
    __device__ __forceinline__ const Pose& operator[](int bs) const {
        for (int i = 0; i + 1 < NWB; ++i)
            if (b[i] == bs) return p[i];
        return p[NWB - 1];
    }
};
template <int NWB>
struct GenWrapVels {
    const SV* v;
    const int* b;
    __device__ __forceinline__ const SV& operator[](int bs) const {
        for (int i = 0; i + 1 < NWB; ++i)
            if (b[i] == bs) return v[i];
        return v[NWB - 1];
    }
};

template <int MP, int NWB>
__device__ __noinline__ void gen_wrap_path(const DevModel& M, int im, const Pose* xp, const SV* xv,
        const int* xb, CPath<MP>& C, double& L, double& S) {
#pragma clang fp contract(off)
    const GenWrapPoses<NWB> X{xp, xb};
    const GenWrapVels<NWB> V{xv, xb};
    auto active = [&](int i) {
        for (int k = 0; k < C.n; ++k)
            if (C.pt[k] == i) return true;
        return false;
    };
    dev_apply_wraps<MP>(M, im, X, V, active, C);
    // the interpreter's length / speed loop (dae_eval), operation for operation
    L = 0.0;
    S = 0.0;
    for (int k = 1; k < C.n; ++k) {
        const double d0 = C.P[k][0] - C.P[k - 1][0], d1 = C.P[k][1] - C.P[k - 1][1],
                     d2 = C.P[k][2] - C.P[k - 1][2];
        const double l = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        if (C.arc(k)) L += C.wlen[k];
        else L += l;
        const double e0 = C.V[k][0] - C.V[k - 1][0], e1 = C.V[k][1] - C.V[k - 1][1],
                     e2 = C.V[k][2] - C.V[k - 1][2];
        S += (d0 * e0 + d1 * e1 + d2 * e2) / l;
    }
}

// Point forces of tension T along the wrapped path: per original path point
// (index within the muscle) and per PathWrap entry of the muscle (its
// tangent points, on the wrap body), force f and moment P x f summed; zero
// for inactive points and untouched surfaces.
template <int MP, int NPT, int NW>
__device__ __noinline__ void gen_wrap_forces(const DevModel& M, int im, const CPath<MP>& C, double T,
        double (*fp)[3], double (*np)[3], double (*fw)[3], double (*nw)[3]) {
#pragma clang fp contract(off)
    for (int i = 0; i < NPT; ++i)
        for (int d = 0; d < 3; ++d) { fp[i][d] = 0.0; np[i][d] = 0.0; }
    for (int i = 0; i < NW; ++i)
        for (int d = 0; d < 3; ++d) { fw[i][d] = 0.0; nw[i][d] = 0.0; }
    const int pb = M.mus[im].point_begin, wb = M.mus_pw_begin[im];
    for (int k = 1; k < C.n; ++k) {
        if (C.arc(k)) continue;   // a wrap's surface part: both ends on one body
        const double d0 = C.P[k][0] - C.P[k - 1][0], d1 = C.P[k][1] - C.P[k - 1][1],
                     d2 = C.P[k][2] - C.P[k - 1][2];
        const double l = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
        const double F0 = T * d0 / l, F1 = T * d1 / l, F2 = T * d2 / l;
        for (int side = 0; side < 2; ++side) {
            const int kk = side == 0 ? k - 1 : k;
            const double sg = side == 0 ? 1.0 : -1.0;
            const double f0 = sg * F0, f1 = sg * F1, f2 = sg * F2;
            double n0, n1, n2;
            cross3(C.P[kk][0], C.P[kk][1], C.P[kk][2], f0, f1, f2, n0, n1, n2);
            double* fa;
            double* na;
            if (C.pt[kk] < 0) {
                if (C.body[kk] < 0) continue;
                const int s = C.pwi[kk] - wb;
                if (s < 0 || s >= NW) continue;
                fa = fw[s]; na = nw[s];
            } else {
                const int i = C.pt[kk] - pb;
                if (i < 0 || i >= NPT) continue;
                fa = fp[i]; na = np[i];
            }
            fa[0] += f0; fa[1] += f1; fa[2] += f2;
            na[0] += n0; na[1] += n1; na[2] += n2;
        }
    }
}

// Per-lane workspace.  MB = max bodies (excluding ground), MQ = max
// coordinates, MP = max path points per muscle.
template <int MB, int MQ, int MP>
struct Work {
    Pose X[MB + 1];
    SV V[MB + 1];
    SV F[MB + 1];
    SV S[MQ];
    double tau[MQ];
    double Mm[MQ * (MQ + 1) / 2];  // packed lower triangle
};

__device__ __forceinline__ int tri(int i, int j) { return i * (i + 1) / 2 + j; }  // i >= j

// Full DAE.  q,u,z packed in x (NS); controls in c (NC), followed in
// implicit mode by the generalized accelerations (NQ).  Outputs
// [udot(NQ), zdot(NZ)] (explicit) or [residual(NQ), zdot(NZ)] (implicit:
// residual = M udot + C - f_applied by RNEA with the accelerations, the
// mobility forces Simbody's findMotionForces returns,
// MocoCasOCProblem.h:245-297).
// Kinematic-constraint outputs (MocoCasOCProblem.h:664-732): per
// CoordinateCoupler phi = scale f(q_i) - q_d the position errors, then (when
// enforced) the velocity and acceleration errors; the velocity correction
// G^T gamma from the slack inputs (MocoCasOCProblem.h:298-332).  The
// oracle's kc_outputs (oracle/oracle.c), operation for operation.
__device__ inline void kc_outputs(const DevModel& M, const double* q, const double* u,
        const double* udot, const double* c, double* out) {
#pragma clang fp contract(off)
    const int n = M.nkc;
    if (M.okc < 0 && M.oqc < 0) return;   // prescribed kinematics: multipliers only
    double* e = out + M.okc;
    const double* lam = c + M.mult;
    const double* gam = lam + n;
    if (M.oqc >= 0)
        for (int j = 0; j < M.nq; ++j) out[M.oqc + j] = 0.0;
    for (int i = 0; i < n; ++i) {
        const mh_constraint K = M.kcs[i];
        const int ci = M.funcs[K.func].coord, d = K.dependent;
        double v, d1, d2;
        fn_eval(M, K.func, q, v, d1, d2);
        const double gi = K.scale * d1;
        e[i] = K.scale * v - q[d];
        if (M.enforce) {
            e[n + i] = gi * u[ci] - u[d];
            e[2 * n + i] = (gi * udot[ci] - udot[d]) + K.scale * d2 * u[ci] * u[ci];
        }
        if (M.oqc >= 0) {
            out[M.oqc + ci] += gi * gam[i];
            out[M.oqc + d] -= gam[i];
        }
    }
}

template <int MB, int MQ, int MP>
__device__ void dae_eval(const DevModel& M, Work<MB, MQ, MP>& w, double time, const double* x,
        const double* c, double* out, const double* wacc_presc = nullptr) {
    const int NQ = M.nq;
    const double* q = x;
    const double* u = x + NQ;
    // implicit: the acceleration inputs; prescribed kinematics: the motion's
    // udot (both give the multibody residual outputs)
    const double* wacc = wacc_presc ? wacc_presc : (M.implicit ? c + M.nc : nullptr);
    // ---- kinematics + RNEA forward pass --------------------------------
    w.X[0] = Pose{{1, 0, 0, 0, 1, 0, 0, 0, 1}, {0, 0, 0}};
    w.V[0] = sv_zero();
    SV A0 = sv_zero();
    A0.v0 = -M.gravity[0]; A0.v1 = -M.gravity[1]; A0.v2 = -M.gravity[2];
    // bias accelerations kept only transiently: store body A in F slot then
    // convert to force immediately.
    SV Aacc[MB + 1];
    Aacc[0] = A0;
    for (int j = 0; j < NQ; ++j) { w.S[j] = sv_zero(); w.tau[j] = 0.0; }
    for (int b = 0; b < M.nb; ++b) {
        const mh_body& B = M.bodies[b];
        const int ps = B.parent + 1, bs = b + 1;
        const Pose& Pp = w.X[ps];
        double RGF[9], pGF0, pGF1, pGF2, t0, t1, t2;
        mm3(Pp.R, B.R_PF, RGF);
        mv3(Pp.R, B.p_PF[0], B.p_PF[1], B.p_PF[2], t0, t1, t2);
        pGF0 = Pp.p[0] + t0; pGF1 = Pp.p[1] + t1; pGF2 = Pp.p[2] + t2;
        SV V = w.V[ps];
        const SV Vpar = w.V[ps];
        SV A = Aacc[ps];
        double pFM0 = 0, pFM1 = 0, pFM2 = 0;
        for (int a = B.axis_begin; a < B.axis_begin + B.axis_count; ++a) {
            const mh_axis X = M.axes[a];
            if (X.type != MH_AXIS_TRANSLATION) continue;
            double v, d1, d2;
            fn_eval(M, X.func, q, v, d1, d2);
            pFM0 += v * X.dir[0]; pFM1 += v * X.dir[1]; pFM2 += v * X.dir[2];
        }
        double oM0, oM1, oM2;
        mv3(RGF, pFM0, pFM1, pFM2, t0, t1, t2);
        oM0 = pGF0 + t0; oM1 = pGF1 + t1; oM2 = pGF2 + t2;
        for (int a = B.axis_begin; a < B.axis_begin + B.axis_count; ++a) {
            const mh_axis X = M.axes[a];
            if (X.type != MH_AXIS_TRANSLATION) continue;
            const mh_function F = M.funcs[X.func];
            if (F.kind == MH_FN_CONSTANT) continue;
            double v, d1, d2;
            fn_eval(M, X.func, q, v, d1, d2);
            const double uj = u[F.coord];
            SV s = sv_zero();
            mv3(RGF, X.dir[0], X.dir[1], X.dir[2], s.v0, s.v1, s.v2);
            SV sd = crm(Vpar, s);
            const double thd = d1 * uj;
            double thdd = d2 * uj * uj;
            if (wacc) thdd += d1 * wacc[F.coord];
            V.v0 += s.v0 * thd; V.v1 += s.v1 * thd; V.v2 += s.v2 * thd;
            A.w0 += sd.w0 * thd; A.w1 += sd.w1 * thd; A.w2 += sd.w2 * thd;
            A.v0 += sd.v0 * thd + s.v0 * thdd; A.v1 += sd.v1 * thd + s.v1 * thdd;
            A.v2 += sd.v2 * thd + s.v2 * thdd;
            SV& Sj = w.S[F.coord];
            Sj.v0 += d1 * s.v0; Sj.v1 += d1 * s.v1; Sj.v2 += d1 * s.v2;
        }
        double Rcur[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        for (int a = B.axis_begin; a < B.axis_begin + B.axis_count; ++a) {
            const mh_axis X = M.axes[a];
            if (X.type != MH_AXIS_ROTATION) continue;
            const mh_function F = M.funcs[X.func];
            double v, d1, d2;
            fn_eval(M, X.func, q, v, d1, d2);
            if (F.kind != MH_FN_CONSTANT) {
                double RGc[9];
                mm3(RGF, Rcur, RGc);
                SV s;
                mv3(RGc, X.dir[0], X.dir[1], X.dir[2], s.w0, s.w1, s.w2);
                cross3(oM0, oM1, oM2, s.w0, s.w1, s.w2, s.v0, s.v1, s.v2);
                SV sd = crm(V, s);
                const double uj = u[F.coord];
                const double thd = d1 * uj;
                double thdd = d2 * uj * uj;
                if (wacc) thdd += d1 * wacc[F.coord];
                V.w0 += s.w0 * thd; V.w1 += s.w1 * thd; V.w2 += s.w2 * thd;
                V.v0 += s.v0 * thd; V.v1 += s.v1 * thd; V.v2 += s.v2 * thd;
                A.w0 += sd.w0 * thd + s.w0 * thdd; A.w1 += sd.w1 * thd + s.w1 * thdd;
                A.w2 += sd.w2 * thd + s.w2 * thdd;
                A.v0 += sd.v0 * thd + s.v0 * thdd; A.v1 += sd.v1 * thd + s.v1 * thdd;
                A.v2 += sd.v2 * thd + s.v2 * thdd;
                SV& Sj = w.S[F.coord];
                Sj.w0 += d1 * s.w0; Sj.w1 += d1 * s.w1; Sj.w2 += d1 * s.w2;
                Sj.v0 += d1 * s.v0; Sj.v1 += d1 * s.v1; Sj.v2 += d1 * s.v2;
            }
            double Rk[9];
            axis_rot(X.dir[0], X.dir[1], X.dir[2], v, Rk);
            mm3(Rcur, Rk, Rcur);
        }
        double RGM[9];
        mm3(RGF, Rcur, RGM);
        Pose& Pb = w.X[bs];
        // R_GB = R_GM * R_BM^T
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Pb.R[3 * i + j] = RGM[3 * i] * B.R_BM[3 * j] + RGM[3 * i + 1] * B.R_BM[3 * j + 1] +
                                  RGM[3 * i + 2] * B.R_BM[3 * j + 2];
        mv3(Pb.R, B.p_BM[0], B.p_BM[1], B.p_BM[2], t0, t1, t2);
        Pb.p[0] = oM0 - t0; Pb.p[1] = oM1 - t1; Pb.p[2] = oM2 - t2;
        w.V[bs] = V;
        Aacc[bs] = A;
        // inertia in ground about origin, and I a + v x* I v
        double cw0, cw1, cw2;
        mv3(Pb.R, B.com[0], B.com[1], B.com[2], t0, t1, t2);
        cw0 = Pb.p[0] + t0; cw1 = Pb.p[1] + t1; cw2 = Pb.p[2] + t2;
        const double Ib[9] = {B.inertia[0], B.inertia[3], B.inertia[4], B.inertia[3],
                B.inertia[1], B.inertia[5], B.inertia[4], B.inertia[5], B.inertia[2]};
        double T1[9], Ig[9];
        mm3(Pb.R, Ib, T1);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Ig[3 * i + j] = T1[3 * i] * Pb.R[3 * j] + T1[3 * i + 1] * Pb.R[3 * j + 1] +
                                T1[3 * i + 2] * Pb.R[3 * j + 2];
        const double m = B.mass;
        const double c2 = cw0 * cw0 + cw1 * cw1 + cw2 * cw2;
        RBI I{m, m * cw0, m * cw1, m * cw2, Ig[0] + m * (c2 - cw0 * cw0),
                Ig[4] + m * (c2 - cw1 * cw1), Ig[8] + m * (c2 - cw2 * cw2),
                Ig[1] - m * cw0 * cw1, Ig[2] - m * cw0 * cw2, Ig[5] - m * cw1 * cw2};
        SV Ia = rbi_mul(I, A);
        SV h = rbi_mul(I, V);
        SV vxh = crf(V, h);
        w.F[bs] = SV{Ia.w0 + vxh.w0, Ia.w1 + vxh.w1, Ia.w2 + vxh.w2, Ia.v0 + vxh.v0,
                Ia.v1 + vxh.v1, Ia.v2 + vxh.v2};
    }
    // ---- actuators -------------------------------------------------------
    double* zdot = out + NQ;
    for (int ia = 0; ia < M.nact; ++ia) {
        const mh_actuator A = M.acts[ia];
        if (A.kind == MH_ACT_COORDINATE) w.tau[A.target] += c[ia] * A.optimal_force;
    }
    // ---- SpringGeneralizedForce: -stiffness (q - rest_length) - viscosity u
    for (int is = 0; is < M.nsp; ++is) {
        const mh_spring S = M.sp[is];
        const double f = -S.stiffness * (q[S.coord] - S.rest_length) - S.viscosity * u[S.coord];
        w.tau[S.coord] += f;
    }
    // ---- kinematic constraint forces -G^T lambda (MocoCasOCProblem.h:643-662)
    for (int i = 0; i < M.nkc; ++i) {
        const mh_constraint K = M.kcs[i];
        double v, d1, d2;
        fn_eval(M, K.func, q, v, d1, d2);
        const double lam = c[M.mult + i];
        w.tau[M.funcs[K.func].coord] -= (K.scale * d1) * lam;
        w.tau[K.dependent] -= -lam;
    }
    // ---- muscles: path geometry, DGF, tension as point forces -------------
    for (int im = 0; im < M.nmus; ++im) {
        const mh_muscle& mu = M.mus[im];
        CPath<MP> C;
        double (&P)[MP][3] = C.P;
        double (&Vp)[MP][3] = C.V;
        int (&pidx)[MP] = C.pt;
        int np = 0;
        for (int i = mu.point_begin; i < mu.point_begin + mu.point_count && np < MP; ++i) {
            const mh_path_point pt = M.pts[i];
            double l0 = pt.loc[0], l1 = pt.loc[1], l2 = pt.loc[2];
            double dl0 = 0, dl1 = 0, dl2 = 0;
            if (pt.kind == MH_PP_CONDITIONAL) {
                const double qv = q[pt.coord];
                if (!(qv >= pt.range[0] && qv <= pt.range[1])) continue;
            } else if (pt.kind == MH_PP_MOVING) {
                double v, d1, d2;
                if (pt.fx >= 0) {
                    fn_eval(M, pt.fx, q, v, d1, d2); l0 = v;
                    const mh_function F = M.funcs[pt.fx];
                    if (F.kind != MH_FN_CONSTANT) dl0 = d1 * u[F.coord];
                }
                if (pt.fy >= 0) {
                    fn_eval(M, pt.fy, q, v, d1, d2); l1 = v;
                    const mh_function F = M.funcs[pt.fy];
                    if (F.kind != MH_FN_CONSTANT) dl1 = d1 * u[F.coord];
                }
                if (pt.fz >= 0) {
                    fn_eval(M, pt.fz, q, v, d1, d2); l2 = v;
                    const mh_function F = M.funcs[pt.fz];
                    if (F.kind != MH_FN_CONSTANT) dl2 = d1 * u[F.coord];
                }
            }
            const int bs = pt.body + 1;
            const Pose& Pb = w.X[bs];
            double t0, t1, t2, r0, r1, r2;
            mv3(Pb.R, l0, l1, l2, t0, t1, t2);
            P[np][0] = Pb.p[0] + t0; P[np][1] = Pb.p[1] + t1; P[np][2] = Pb.p[2] + t2;
            const SV& Vb = w.V[bs];
            cross3(Vb.w0, Vb.w1, Vb.w2, P[np][0], P[np][1], P[np][2], t0, t1, t2);
            mv3(Pb.R, dl0, dl1, dl2, r0, r1, r2);
            Vp[np][0] = Vb.v0 + t0 + r0; Vp[np][1] = Vb.v1 + t1 + r1; Vp[np][2] = Vb.v2 + t2 + r2;
            pidx[np] = i;
            C.pwi[np] = -1;
            C.body[np] = pt.body;
            C.wlen[np] = 0.0;
            ++np;
        }
        C.n = np;
        if (M.mus_pw_count && M.mus_pw_count[im] > 0) {
            const int pb0 = mu.point_begin, pc0 = mu.point_count;
            auto active = [&](int i) {
                for (int k = 0; k < C.n; ++k)
                    if (C.pt[k] == i) return true;
                (void)pb0; (void)pc0;
                return false;
            };
            dev_apply_wraps<MP>(M, im, w.X, w.V, active, C);
            np = C.n;
        }
        double L = 0.0, S = 0.0;
        for (int k = 1; k < np; ++k) {
            double d0 = P[k][0] - P[k - 1][0], d1 = P[k][1] - P[k - 1][1], d2 = P[k][2] - P[k - 1][2];
            double l = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
            if (C.arc(k)) L += C.wlen[k];
            else L += l;
            double e0 = Vp[k][0] - Vp[k - 1][0], e1 = Vp[k][1] - Vp[k - 1][1], e2 = Vp[k][2] - Vp[k - 1][2];
            S += (d0 * e0 + d1 * e1 + d2 * e2) / l;
        }
        const double exc = c[M.mus_control[im]];
        const int sa = M.mus_act_state[im], sf = M.mus_ftn_state[im];
        const double act = sa >= 0 ? x[sa] : exc;
        const double ftn = sf >= 0 ? x[sf] : 0.0;
        double T, adot = 0, ftdot = 0, resid = 0;
        const int id = M.mus_ider[im];
        dgf_eval(M, im, L, S, act, exc, sa >= 0, ftn, sf >= 0, T, adot, ftdot, id >= 0,
                id >= 0 ? c[M.nc + id] : 0.0, &resid);
        if (sa >= 0) zdot[sa - 2 * NQ] = adot;
        if (sf >= 0) zdot[sf - 2 * NQ] = ftdot;
        // auxiliary residual outputs after zdot (CasOCFunction.cpp:208-230)
        if (id >= 0) out[NQ + M.nz + (id - M.nacc)] = resid;
        for (int k = 1; k < np; ++k) {
            if (C.arc(k)) continue;   // a wrap's surface part: both ends on one body
            double d0 = P[k][0] - P[k - 1][0], d1 = P[k][1] - P[k - 1][1], d2 = P[k][2] - P[k - 1][2];
            double l = sqrt(d0 * d0 + d1 * d1 + d2 * d2);
            double F0 = T * d0 / l, F1 = T * d1 / l, F2 = T * d2 / l;
            // +F at point k-1, -F at point k
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                const int kk = side == 0 ? k - 1 : k;
                const double sg = side == 0 ? 1.0 : -1.0;
                const double f0 = sg * F0, f1 = sg * F1, f2 = sg * F2;
                if (pidx[kk] < 0) {   // tangent point: a force at that station of the wrap body
                    if (C.body[kk] < 0) continue;
                    double n0, n1, n2;
                    cross3(P[kk][0], P[kk][1], P[kk][2], f0, f1, f2, n0, n1, n2);
                    SV& Fw = w.F[C.body[kk] + 1];
                    Fw.w0 -= n0; Fw.w1 -= n1; Fw.w2 -= n2;
                    Fw.v0 -= f0; Fw.v1 -= f1; Fw.v2 -= f2;
                    continue;
                }
                const mh_path_point pt = M.pts[pidx[kk]];
                if (pt.body < 0) continue;
                const int bs = pt.body + 1;
                double n0, n1, n2;
                cross3(P[kk][0], P[kk][1], P[kk][2], f0, f1, f2, n0, n1, n2);
                SV& Fb = w.F[bs];
                Fb.w0 -= n0; Fb.w1 -= n1; Fb.w2 -= n2;
                Fb.v0 -= f0; Fb.v1 -= f1; Fb.v2 -= f2;
                if (pt.kind == MH_PP_MOVING) {
                    const Pose& Pb = w.X[bs];
                    const int fs[3] = {pt.fx, pt.fy, pt.fz};
#pragma unroll
                    for (int dd = 0; dd < 3; ++dd) {
                        if (fs[dd] < 0) continue;
                        const mh_function F = M.funcs[fs[dd]];
                        if (F.kind == MH_FN_CONSTANT) continue;
                        double v, g1, g2;
                        fn_eval(M, fs[dd], q, v, g1, g2);
                        const double g = (Pb.R[dd] * f0 + Pb.R[3 + dd] * f1 + Pb.R[6 + dd] * f2) * g1;
                        w.tau[F.coord] += g;
                    }
                }
            }
        }
    }
    // ---- external forces ---------------------------------------------------
    for (int ie = 0; ie < M.next; ++ie) {
        const mh_external_force E = M.ext[ie];
        const int bs = E.body + 1;
        double F0 = 0, F1 = 0, F2 = 0, T0 = 0, T1 = 0, T2 = 0;
        double P0 = w.X[bs].p[0], P1 = w.X[bs].p[1], P2 = w.X[bs].p[2];
        if (E.force_col >= 0) {
            F0 = table_eval(M, E.table, E.force_col, time);
            F1 = table_eval(M, E.table, E.force_col + 1, time);
            F2 = table_eval(M, E.table, E.force_col + 2, time);
        }
        if (E.point_col >= 0) {
            P0 = table_eval(M, E.table, E.point_col, time);
            P1 = table_eval(M, E.table, E.point_col + 1, time);
            P2 = table_eval(M, E.table, E.point_col + 2, time);
        }
        if (E.torque_col >= 0) {
            T0 = table_eval(M, E.table, E.torque_col, time);
            T1 = table_eval(M, E.table, E.torque_col + 1, time);
            T2 = table_eval(M, E.table, E.torque_col + 2, time);
        }
        double n0, n1, n2;
        cross3(P0, P1, P2, F0, F1, F2, n0, n1, n2);
        SV& Fb = w.F[bs];
        Fb.w0 -= n0 + T0; Fb.w1 -= n1 + T1; Fb.w2 -= n2 + T2;
        Fb.v0 -= F0; Fb.v1 -= F1; Fb.v2 -= F2;
    }
    // ---- RNEA backward pass -------------------------------------------------
    for (int b = M.nb - 1; b >= 0; --b) {
        const int ps = M.bodies[b].parent + 1;
        if (ps > 0) {
            SV& Fp = w.F[ps];
            const SV& Fb = w.F[b + 1];
            Fp.w0 += Fb.w0; Fp.w1 += Fb.w1; Fp.w2 += Fb.w2;
            Fp.v0 += Fb.v0; Fp.v1 += Fb.v1; Fp.v2 += Fb.v2;
        }
    }
    for (int j = 0; j < NQ; ++j) w.tau[j] -= svdot(w.S[j], w.F[M.coord_body[j] + 1]);
    if (wacc) {
        for (int j = 0; j < NQ; ++j) out[j] = -w.tau[j];
        if (M.nkc) kc_outputs(M, q, u, wacc, c, out);
        return;
    }
    // ---- CRBA: composite inertias re-derived per body (reuse F slots is not
    //      possible; recompute the ground-frame inertia from the stored pose).
    RBI Ic[MB + 1];
    for (int b = 0; b < M.nb; ++b) {
        const mh_body& B = M.bodies[b];
        const Pose& Pb = w.X[b + 1];
        double t0, t1, t2;
        mv3(Pb.R, B.com[0], B.com[1], B.com[2], t0, t1, t2);
        const double cw0 = Pb.p[0] + t0, cw1 = Pb.p[1] + t1, cw2 = Pb.p[2] + t2;
        const double Ib[9] = {B.inertia[0], B.inertia[3], B.inertia[4], B.inertia[3],
                B.inertia[1], B.inertia[5], B.inertia[4], B.inertia[5], B.inertia[2]};
        double T1[9], Ig[9];
        mm3(Pb.R, Ib, T1);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j)
                Ig[3 * i + j] = T1[3 * i] * Pb.R[3 * j] + T1[3 * i + 1] * Pb.R[3 * j + 1] +
                                T1[3 * i + 2] * Pb.R[3 * j + 2];
        const double m = B.mass;
        const double c2 = cw0 * cw0 + cw1 * cw1 + cw2 * cw2;
        Ic[b + 1] = RBI{m, m * cw0, m * cw1, m * cw2, Ig[0] + m * (c2 - cw0 * cw0),
                Ig[4] + m * (c2 - cw1 * cw1), Ig[8] + m * (c2 - cw2 * cw2),
                Ig[1] - m * cw0 * cw1, Ig[2] - m * cw0 * cw2, Ig[5] - m * cw1 * cw2};
    }
    for (int b = M.nb - 1; b >= 0; --b) {
        const int ps = M.bodies[b].parent + 1;
        if (ps > 0) {
            RBI& P = Ic[ps];
            const RBI& C = Ic[b + 1];
            P.m += C.m; P.h0 += C.h0; P.h1 += C.h1; P.h2 += C.h2;
            P.I0 += C.I0; P.I1 += C.I1; P.I2 += C.I2; P.I3 += C.I3; P.I4 += C.I4; P.I5 += C.I5;
        }
    }
    for (int i = 0; i < NQ * (NQ + 1) / 2; ++i) w.Mm[i] = 0.0;
    for (int i = 0; i < NQ; ++i) {
        const int b = M.coord_body[i];
        const SV Fi = rbi_mul(Ic[b + 1], w.S[i]);
        for (int j = 0; j < NQ; ++j) {
            const int bj = M.coord_body[j];
            int anc = b;
            while (anc >= 0 && anc != bj) anc = M.bodies[anc].parent;
            if (anc == bj) {
                const double v = svdot(w.S[j], Fi);
                if (i >= j) w.Mm[tri(i, j)] = v; else w.Mm[tri(j, i)] = v;
            }
        }
    }
    // ---- Cholesky (packed lower) and solve ----------------------------------
    for (int j = 0; j < NQ; ++j) {
        double s = w.Mm[tri(j, j)];
        for (int k = 0; k < j; ++k) s -= w.Mm[tri(j, k)] * w.Mm[tri(j, k)];
        const double d = sqrt(s);
        w.Mm[tri(j, j)] = d;
        for (int i = j + 1; i < NQ; ++i) {
            double t = w.Mm[tri(i, j)];
            for (int k = 0; k < j; ++k) t -= w.Mm[tri(i, k)] * w.Mm[tri(j, k)];
            w.Mm[tri(i, j)] = t / d;
        }
    }
    double* y = out;
    for (int i = 0; i < NQ; ++i) {
        double t = w.tau[i];
        for (int k = 0; k < i; ++k) t -= w.Mm[tri(i, k)] * y[k];
        y[i] = t / w.Mm[tri(i, i)];
    }
    for (int i = NQ - 1; i >= 0; --i) {
        double t = y[i];
        for (int k = i + 1; k < NQ; ++k) t -= w.Mm[tri(k, i)] * y[k];
        y[i] = t / w.Mm[tri(i, i)];
    }
    if (M.nkc) kc_outputs(M, q, u, y, c, out);
}

}  // namespace mh

namespace mh {
// ---- helpers used by generated (model-specialized) DAE code ---------------
// SimmSpline with a compile-time knot count: interval by an unrolled scan
// (no data-dependent loop), SIMM end handling and linear extrapolation.
template <int N>
__device__ __forceinline__ void simm_eval_n(const DevModel& M, int kb, double t, double& v,
        double& d1, double& d2) {
    const double* __restrict__ x = M.kx + kb;
    const double* __restrict__ y = M.ky + kb;
    const double* __restrict__ b = M.kb + kb;
    const double* __restrict__ c = M.kc + kb;
    const double* __restrict__ d = M.kd + kb;
    if (N == 1) { v = y[0]; d1 = 0.0; d2 = 0.0; return; }
    int k = 0;
#pragma unroll
    for (int i = 1; i < N - 1; ++i) k += (t >= x[i]) ? 1 : 0;
    if (fabs(t - x[0]) <= 2e-13) k = 0;
    else if (fabs(t - x[N - 1]) <= 2e-13) k = N - 1;
    const double dx = t - x[k];
    const double bk = b[k], ck = c[k], dk = d[k];
    v = y[k] + dx * (bk + dx * (ck + dx * dk));
    d1 = bk + dx * (2.0 * ck + 3.0 * dx * dk);
    d2 = 2.0 * ck + 6.0 * dx * dk;
    if (t < x[0]) { v = y[0] + (t - x[0]) * b[0]; d1 = b[0]; d2 = 0.0; }
    if (t > x[N - 1]) { v = y[N - 1] + (t - x[N - 1]) * b[N - 1]; d1 = b[N - 1]; d2 = 0.0; }
}

__device__ __forceinline__ int table_segment(const DevModel& M, int ti, double t) {
    const mh_table T = M.tabs[ti];
    const double* br = M.brk + T.break_begin;
    if (t <= br[0]) return 0;
    if (t >= br[T.nseg]) return T.nseg - 1;
    int lo = 0, hi = T.nseg;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (t < br[mid]) hi = mid; else lo = mid;
    }
    return lo;
}

__device__ __forceinline__ double table_value(const DevModel& M, int ti, int s, int col, double t) {
    const mh_table T = M.tabs[ti];
    const double* cf = M.coef + T.coef_begin + ((long)s * T.ncol + col) * (T.degree + 1);
    const double dt = t - M.brk[T.break_begin + s];
    double v = cf[T.degree];
    for (int k = T.degree - 1; k >= 0; --k) v = v * dt + cf[k];
    return v;
}
}  // namespace mh

namespace mh {
// Segment of a table whose breakpoints are near-uniform (checked by the
// generator: the uniform guess is within one segment for every t): direct
// index, one correction step.  Same result as table_segment.
template <int NSEG>
__device__ __forceinline__ int table_segment_u(const double* __restrict__ br, double t, double b0,
        double inv) {
    if (t <= br[0]) return 0;
    if (t >= br[NSEG]) return NSEG - 1;
    if (t != t) return NSEG - 1;
    int s = (int)((t - b0) * inv);
    s = s < 0 ? 0 : (s > NSEG - 1 ? NSEG - 1 : s);
    const double lo = br[s], hi = br[s + 1 <= NSEG ? s + 1 : NSEG];
    if (t < lo) s -= 1;
    else if (t >= hi && s < NSEG - 1) s += 1;
    return s;
}

// Same with the segment count read at run time (the table's data, not the
// model structure: another trial's table of another length fits the same
// generated code); b0 / inv from the model's constant pool.
__device__ __forceinline__ int table_segment_ur(const double* __restrict__ br, int nseg, double t, double b0,
        double inv) {
    if (t <= br[0]) return 0;
    if (t >= br[nseg]) return nseg - 1;
    if (t != t) return nseg - 1;
    int s = (int)((t - b0) * inv);
    s = s < 0 ? 0 : (s > nseg - 1 ? nseg - 1 : s);
    const double lo = br[s], hi = br[s + 1 <= nseg ? s + 1 : nseg];
    if (t < lo) s -= 1;
    else if (t >= hi && s < nseg - 1) s += 1;
    return s;
}

// Piecewise-polynomial value with compile-time degree and column count.
template <int DEG, int NCOL>
__device__ __forceinline__ double table_value_c(const double* __restrict__ coef,
        const double* __restrict__ br, int s, int col, double t) {
    const double* cf = coef + ((long)s * NCOL + col) * (DEG + 1);
    const double dt = t - br[s];
    double v = cf[DEG];
#pragma unroll
    for (int k = DEG - 1; k >= 0; --k) v = v * dt + cf[k];
    return v;
}
}  // namespace mh

namespace mh {
// SimmSpline evaluation with the interval k already found (by the generated
// code, from literal knots): every load below is independent of the others.
template <int N>
__device__ __forceinline__ void simm_eval_k(const DevModel& M, int kb, double t, int k, double x0,
        double xn, double& v, double& d1, double& d2) {
    const double* __restrict__ x = M.kx + kb;
    const double* __restrict__ y = M.ky + kb;
    const double* __restrict__ b = M.kb + kb;
    const double* __restrict__ c = M.kc + kb;
    const double* __restrict__ d = M.kd + kb;
    const double dx = t - x[k];
    const double bk = b[k], ck = c[k], dk = d[k];
    v = y[k] + dx * (bk + dx * (ck + dx * dk));
    d1 = bk + dx * (2.0 * ck + 3.0 * dx * dk);
    d2 = 2.0 * ck + 6.0 * dx * dk;
    if (t < x0) { v = y[0] + (t - x0) * b[0]; d1 = b[0]; d2 = 0.0; }
    if (t > xn) { v = y[N - 1] + (t - xn) * b[N - 1]; d1 = b[N - 1]; d2 = 0.0; }
}
}  // namespace mh
