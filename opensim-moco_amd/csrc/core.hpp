// core.hpp — device kernels (templates over the DAE back end), the
// context struct and the back-end launchers shared by every translation
// unit of libmocohip.so: mocohip.hip (C ABI, host side, non-template
// kernels), generic.hip (device interpreter back ends) and one
// generated/gen_<model>.hip per model-specialized back end, so that the
// model back ends compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/mocohip.h"
#include "dae_device.hpp"

using namespace mh;

constexpr size_t kMaxLds = 160 * 1024;   // gfx950 LDS per workgroup

// LDS-qualified views of dynamic shared memory.  Kept in address space 3 so
// that a load that may come from LDS or from global memory (e.g. xdot_at) is
// never merged into one flat load: flat loads wait on vmcnt, i.e. on every
// outstanding global store of the thread.
typedef __attribute__((address_space(3))) double lds_double;
typedef __attribute__((address_space(3))) int lds_int;
__device__ __forceinline__ lds_double* lds(double* p) { return (lds_double*)p; }

// ------------------------------------------------------------------------
// Jacobian template (per mesh interval; identical for every interval).
// ------------------------------------------------------------------------
enum TplKind : uint8_t {
    T_HERM_T = 0, T_SIMP_T = 1, T_HERM_X = 2, T_SIMP_X = 3, T_INTERP = 4,
    T_TRAP_T = 5, T_TRAP_X = 6,
    T_RES = 7,     // implicit multibody residual output s at point pt
    T_PATH = 8,    // path-constraint equation s at mesh point pt
    T_EP = 9       // endpoint equation row along endpoint input dir (EndpointEqs)
};
struct TplEntry {
    int16_t row;   // row within the interval
    uint8_t kind;
    uint8_t pt;    // 0 = first point of interval, 1 = mid (HS), 2 = last (HS) / 1 last (trap)
    int16_t dir;   // 0 = t0, 1 = tf, 2 + j = point input j
    int16_t s;     // state index of the row (defects) / control index (interp)
};

// ------------------------------------------------------------------------
// DAE back ends.  Generic: the interpreter of dae_device.hpp with size-class
// bounded per-lane arrays.  Generated: a model-specialized straight-line
// struct from mocohip/codegen.py (see generated/models.inc), selected by
// model hash at mh_create.
// ------------------------------------------------------------------------
struct SzSmall { static constexpr int MB = 4, MQ = 4, MP = 4, MI = 24, MO = 12; };
struct SzMedium { static constexpr int MB = 16, MQ = 16, MP = 8, MI = 128, MO = 64; };
// full-body gait models (Rajagopal 2016: 14 bodies, 18-21 coordinates, up
// to 8 points + 2 wraps per path): a third of SzLarge's per-lane workspace
struct SzBody { static constexpr int MB = 16, MQ = 24, MP = 12, MI = 256, MO = 128; };
struct SzLarge { static constexpr int MB = 32, MQ = 40, MP = 12, MI = 384, MO = 192; };

template <class Z>
struct GenericDae {
    static constexpr int MI = Z::MI, MO = Z::MO;
    static constexpr bool SPLIT = false;
    static constexpr bool EXC_LANES = true;   // k_exc_lanes reproduces its excitation lanes
    using W = Work<Z::MB, Z::MQ, Z::MP>;      // per-lane multibody workspace
    __device__ __forceinline__ static void eval(const DevModel& M, double t, const double* in,
            double* out) {
        W w;
        eval_w(M, t, in, out, w);
    }
    // the same with the workspace where the caller puts it (k_eval_lds: LDS)
    __device__ __forceinline__ static void eval_w(const DevModel& M, double t, const double* in,
            double* out, W& w) {
        // one dae_eval call site, so that it can be inlined where w lives in
        // LDS (k_eval_lds): the workspace accesses then compile to ds_*
        // instructions instead of flat accesses through a generic pointer
        double xf[2 * Z::MQ + Z::MI], ud[Z::MQ];
        const double* xs = in;
        const double* wp = nullptr;
        if (M.presc) {
            // prescribed kinematics: [q, u] and udot from the motion, the
            // NLP states are the auxiliary states
            for (int j = 0; j < M.nq; ++j)
                table_eval_d(M, M.kin_table, M.kin_col[j], t, xf[j], xf[M.nq + j], ud[j]);
            for (int k = 0; k < M.nz; ++k) xf[2 * M.nq + k] = in[k];
            xs = xf;
            wp = ud;
        }
        dae_eval<Z::MB, Z::MQ, Z::MP>(M, w, t, xs, in + M.ns, out, wp);
    }
};

struct Layout {
    int NS, NC, NQ, NO, NI;  // NI = NS + NC + NDV + NM + NSL (per-point inputs)
    int G;                   // grid points (full problem)
    int k0;                  // first grid point of this shard
    int nk;                  // grid points in this shard
    int NDV;                 // derivative variables per grid point: accelerations, aux derivatives
    int NACC;                // acceleration variables per grid point (implicit multibody: NQ)
    int SO;                  // callback output of state s's derivative: s + SO (s >= NQ)
    // kinematic constraints: NM multipliers per grid point, NSL slacks per
    // mesh interval (inputs of its midpoint only; NSL > 0 only with
    // Hermite-Simpson); OQC = callback output of the velocity correction
    int NM, NSL, OQC;
    long XM, XL, DB;         // x index of the multipliers, slacks, derivatives
    // the slack inputs of grid point k (global index): the interval's at a
    // mesh-interval midpoint (odd k), none elsewhere
    __host__ __device__ __forceinline__ bool vc(int k) const { return NSL > 0 && (k & 1); }
};

// Per grid point the evaluation lanes are laid out as
//   forward/backward: [dir 0 .. ND-1 perturbed, ND = unperturbed base]
//   central:          [dir 0 .. ND-1 at +h, ND .. 2ND-1 at -h, 2ND = base]
// (dir 0 = t0 seed, dir 1 = tf seed, dir 2+j = point input j) and raw DAE
// outputs are stored Y[(kl*NO + o)*stride + lane]; eval_g uses stride 1
// with the base lane only.
struct Lanes {
    int fd;       // MH_FD_*
    int ND;       // directions
    int stride;   // lanes per grid point
    int base;     // index of the base lane
    double h;     // FD step
};

template <class D>
__device__ __forceinline__ void load_point(const double* __restrict__ x, const Layout& L, int k,
        double (&in)[D::MI]) {
    const double* xs = x + 2 + (long)k * L.NS;
    const double* xc = x + 2 + (long)L.NS * L.G + (long)k * L.NC;
    const double* xd = x + L.DB + (long)k * L.NDV;
    const double* xm = x + L.XM + (long)k * L.NM;
    const double* xl = x + L.XL + (long)((k - 1) >> 1) * L.NSL;
    const int id = L.NS + L.NC + L.NDV, im = id + L.NM;
#pragma unroll
    for (int i = 0; i < D::MI; ++i) {
        double v = 0.0;
        if (i < L.NS) v = xs[i];
        else if (i < L.NS + L.NC) v = xc[i - L.NS];
        else if (i < id) v = xd[i - L.NS - L.NC];
        else if (i < im) v = xm[i - id];
        else if (i < L.NI && L.vc(k)) v = xl[i - im];
        in[i] = v;
    }
}

// Time and inputs of evaluation lane r of grid point k (Lanes layout above).
template <class D>
__device__ __forceinline__ double lane_inputs(const Layout& L, const Lanes& Ln,
        const double* __restrict__ x, double g, int k, int r, double (&in)[D::MI]) {
#pragma clang fp contract(off)
    const double t0 = x[0], tf = x[1];
    double t = (tf - t0) * g + t0;
    load_point<D>(x, L, k, in);
    if (r != Ln.base) {
        int dir = r;
        double step = Ln.fd == MH_FD_BACKWARD ? -Ln.h : Ln.h;
        if (Ln.fd == MH_FD_CENTRAL && r >= Ln.ND) { dir = r - Ln.ND; step = -Ln.h; }
        if (dir == 0) t = t + step * (1.0 - g);
        else if (dir == 1) t = t + step * g;
        const int pi = dir - 2;
#pragma unroll
        for (int i = 0; i < D::MI; ++i) in[i] = (i == pi) ? in[i] + step : in[i];
    }
    return t;
}

// One lane = one DAE evaluation (grid point kl, lane role r).  With a lane
// map, thread j of a grid point evaluates lane map[j] of nmap (the lanes
// k_exc_lanes does not stand in for, packed so no wave idles); without,
// every lane.
template <class D>
__device__ __forceinline__ void eval_lane(const DevModel& M, const Layout& L, const Lanes& Ln,
        const double* __restrict__ x, const double* __restrict__ grid, double* __restrict__ times,
        double* __restrict__ Y, const int* __restrict__ map, int nmap) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const int per = map ? nmap : Ln.stride;
    if (gid >= (long)L.nk * per) return;
    const int kl = (int)(gid / per);
    const int j = (int)(gid - (long)kl * per);
    const int r = map ? map[j] : j;
    const int k = L.k0 + kl;
    double in[D::MI];
    double out[D::MO];
    const double t = lane_inputs<D>(L, Ln, x, grid[k], k, r, in);
    if (r == Ln.base) times[kl] = t;
    D::eval(M, t, in, out);
    double* Yk = Y + (long)kl * L.NO * Ln.stride + r;
#pragma unroll
    for (int o = 0; o < D::MO; ++o)
        if (o < L.NO) Yk[(long)o * Ln.stride] = out[o];
}
template <class D>
__global__ void __launch_bounds__(64) k_eval(DevModel M, Layout L, Lanes Ln,
        const double* __restrict__ x, const double* __restrict__ grid,
        double* __restrict__ times, double* __restrict__ Y, const int* __restrict__ map = nullptr,
        int nmap = 0) {
    eval_lane<D>(M, L, Ln, x, grid, times, Y, map, nmap);
}
// The generic interpreter's lanes with their multibody workspace (D::W:
// poses, velocities, body forces, motion subspaces, tau, mass matrix) in LDS
// instead of scratch: one slot per thread of the workgroup (blockDim.x <=
// 16 lanes, launched with blockDim.x * (sizeof(W) + 16 guard_words) bytes of
// dynamic LDS).  A thread past the last lane returns before it touches LDS,
// so every slot address stays inside the allocation.  Same arithmetic as
// k_eval, bit for bit (tests/test_gpu_parity.py::
// test_eval_g_lds_workspace_bit_identical).
// guard_words > 0 (MOCOHIP_G_LDS_GUARD, a check of the workspace's own
// indexing): each slot sits between two guard bands of guard_words doubles
// filled with a canary bit pattern, the slot itself is filled with NaN
// before the evaluation (a read of a word the evaluation did not write
// first then poisons the outputs, which the bit-identity test sees), and
// after it each thread compares its two bands and sets *status on any
// change (a workspace store outside its slot).
constexpr unsigned long long kLdsCanary = 0x7ff4deadbeefcafeull;
template <class D>
__global__ void __launch_bounds__(16) k_eval_lds(DevModel M, Layout L, Lanes Ln,
        const double* __restrict__ x, const double* __restrict__ grid,
        double* __restrict__ times, double* __restrict__ Y, int guard_words, int* __restrict__ status) {
    static_assert(sizeof(typename D::W) % sizeof(double) == 0, "workspace slots are whole doubles");
    constexpr int WW = (int)(sizeof(typename D::W) / sizeof(double));
    extern __shared__ double smem[];
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)L.nk * Ln.stride) return;
    double* band = smem + (long)threadIdx.x * (WW + 2 * guard_words);
    typename D::W* ws = reinterpret_cast<typename D::W*>(band + guard_words);
    if (guard_words) {
        for (int i = 0; i < guard_words; ++i) {
            band[i] = __longlong_as_double((long long)kLdsCanary);
            band[guard_words + WW + i] = __longlong_as_double((long long)kLdsCanary);
        }
        for (int i = 0; i < WW; ++i) band[guard_words + i] = __longlong_as_double(0x7ff8000000000badll);
    }
    const int kl = (int)(gid / Ln.stride);
    const int r = (int)(gid - (long)kl * Ln.stride);
    const int k = L.k0 + kl;
    double in[D::MI];
    double out[D::MO];
    const double t = lane_inputs<D>(L, Ln, x, grid[k], k, r, in);
    if (r == Ln.base) times[kl] = t;
    D::eval_w(M, t, in, out, *ws);
    if (guard_words) {
        bool ok = true;
        for (int i = 0; i < guard_words; ++i)
            ok = ok && (unsigned long long)__double_as_longlong(band[i]) == kLdsCanary &&
                 (unsigned long long)__double_as_longlong(band[guard_words + WW + i]) == kLdsCanary;
        if (!ok) status[0] = 1;
    }
    double* Yk = Y + (long)kl * L.NO * Ln.stride + r;
#pragma unroll
    for (int o = 0; o < D::MO; ++o)
        if (o < L.NO) Yk[(long)o * Ln.stride] = out[o];
}
// Excitation lanes of the generic interpreter.  A lane that perturbs the
// excitation of a muscle with activation dynamics changes one DAE output,
// that muscle's activation derivative: excitation enters the DAE only there
// (dae_eval: the force uses the activation state).  After k_eval has written
// the base lane, such a lane copies the base lane's outputs and re-evaluates
// dgf_adot at the perturbed excitation -- the value the full evaluation
// computes, bit for bit (tests/test_gpu_parity.py test_excitation_lanes).
// exc[r] = the muscle lane r perturbs, or -1 (built in mh_create).
template <class D>
__global__ void __launch_bounds__(64) k_exc_lanes(DevModel M, Layout L, Lanes Ln,
        const double* __restrict__ x, double* __restrict__ Y, const int* __restrict__ exc) {
#pragma clang fp contract(off)
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)L.nk * Ln.stride) return;
    const int kl = (int)(gid / Ln.stride);
    const int r = (int)(gid - (long)kl * Ln.stride);
    const int m = exc[r];
    if (m < 0) return;
    const int k = L.k0 + kl;
    double* Yk = Y + (long)kl * L.NO * Ln.stride;
    for (int o = 0; o < L.NO; ++o) Yk[(long)o * Ln.stride + r] = Yk[(long)o * Ln.stride + Ln.base];
    const int sa = M.mus_act_state[m];
    const double act = x[2 + (long)k * L.NS + (M.presc ? sa - 2 * M.nq : sa)];
    double step = Ln.fd == MH_FD_BACKWARD ? -Ln.h : Ln.h;
    if (Ln.fd == MH_FD_CENTRAL && r >= Ln.ND) step = -Ln.h;
    const double e = x[2 + (long)L.NS * L.G + (long)k * L.NC + M.mus_control[m]] + step;
    Yk[(long)(sa - M.nq) * Ln.stride + r] = dgf_adot(M, act, e);
}

// ------------------------------------------------------------------------
// Task-decomposed evaluation for generated models.
//
// A DAE evaluation is split into independent groups (mocohip/codegen.py
// _emit_groups): the mass-matrix factor, the RNEA bias forces, one group per
// external load and one per muscle.  Each group reads a known subset of the
// point inputs, so a finite-difference lane only re-evaluates the groups
// that read its perturbed input and takes every other group's result from
// the unperturbed (base) lane of the same grid point:
//
//   k_groups   one wave = one group for 64 (grid point, lane role) tasks;
//              results to T (force groups) / H (mass factor) in HBM.
//   k_combine  one lane = one (grid point, lane role): sums the generalized
//              forces of all groups in a fixed order, adds the coordinate
//              actuators, solves with the mass factor, evaluates activation
//              dynamics, writes the raw outputs Y.
//
// The fixed summation order makes a reused group result bit-identical to
// re-evaluating it, so the Jacobian equals that of full re-evaluation per
// direction (tests/test_gpu_parity.py::test_pruned_tasks_bit_identical).
// ------------------------------------------------------------------------

// Inputs of one evaluation lane read where used (L1/L2-resident x) instead
// of held in VGPRs.
// Point inputs are [states NS, controls NC, derivatives NDV, multipliers
// NM, slacks NSL] (mh_create's layout); the slacks are the interval's at a
// mesh-interval midpoint (Hermite-Simpson with enforced constraint
// derivatives) and 0 elsewhere (xl null).
template <class D>
__device__ __forceinline__ double point_input(const double* __restrict__ xs, const double* __restrict__ xc,
        const double* __restrict__ xd, const double* __restrict__ xm, const double* __restrict__ xl, int i) {
    constexpr int NDV = D::NI - D::NS - D::NC - D::NM - D::NSL;
    if (i < D::NS) return xs[i];
    if (i < D::NS + D::NC) return xc[i - D::NS];
    if (i < D::NS + D::NC + NDV) return xd[i - D::NS - D::NC];
    if (i < D::NS + D::NC + NDV + D::NM) return xm[i - D::NS - D::NC - NDV];
    return xl ? xl[i - D::NS - D::NC - NDV - D::NM] : 0.0;
}
template <class D>
struct LaneIn {
    const double* __restrict__ xs;
    const double* __restrict__ xc;
    const double* __restrict__ xd;   // implicit: accelerations (inputs NS + NC ..)
    int pi;
    double step;
    const double* __restrict__ xm;   // kinematic-constraint multipliers
    const double* __restrict__ xl;   // velocity-correction slacks (null: none at this point)
    __device__ __forceinline__ double operator[](int i) const {
        const double v = point_input<D>(xs, xc, xd, xm, xl, i);
        return i == pi ? v + step : v;
    }
};

// Where lane inputs come from: the NLP iterate x (grid times) or explicit
// points [t, point inputs] (mh_eval_dae).  XM / XL / DB: x index of the
// multipliers, slacks and derivative variables (make_layout).
struct Src {
    const double* x;
    const double* grid;
    const double* pts;   // non-null: explicit points
    int G, k0;
    long XM, XL, DB;
};

// Same, reading a grid point's inputs staged in LDS (k_interval).
template <class D>
struct LaneInL {
    const lds_double* xs;
    const lds_double* xc;
    const lds_double* xd;
    int pi;
    double step;
    const lds_double* xm;
    const lds_double* xl;   // null: no slacks at this point
    __device__ __forceinline__ double operator[](int i) const {
        constexpr int NDV = D::NI - D::NS - D::NC - D::NM - D::NSL;
        double v;
        if (i < D::NS) v = xs[i];
        else if (i < D::NS + D::NC) v = xc[i - D::NS];
        else if (i < D::NS + D::NC + NDV) v = xd[i - D::NS - D::NC];
        else if (i < D::NS + D::NC + NDV + D::NM) v = xm[i - D::NS - D::NC - NDV];
        else v = xl ? xl[i - D::NS - D::NC - NDV - D::NM] : 0.0;
        return i == pi ? v + step : v;
    }
};

// Time, perturbed input and step of evaluation lane r at normalized grid
// time g (Lanes layout above).  The single definition of the lane
// arithmetic: every kernel that evaluates lanes goes through it.
__device__ __forceinline__ double lane_time(const Lanes& Ln, double g, double t0, double tf, int r,
        int& pi, double& step) {
#pragma clang fp contract(off)
    double t = (tf - t0) * g + t0;
    pi = -1;
    step = 0.0;
    if (r != Ln.base) {
        int dir = r;
        step = Ln.fd == MH_FD_BACKWARD ? -Ln.h : Ln.h;
        if (Ln.fd == MH_FD_CENTRAL && r >= Ln.ND) { dir = r - Ln.ND; step = -Ln.h; }
        if (dir == 0) t = t + step * (1.0 - g);
        else if (dir == 1) t = t + step * g;
        pi = dir - 2;
    }
    return t;
}

template <class D>
__device__ __forceinline__ LaneIn<D> lane_input(const Src& S, const Lanes& Ln, int kl, int r,
        double& t) {
    constexpr int NDV = D::NI - D::NS - D::NC - D::NM - D::NSL;
    if (S.pts) {
        const double* p = S.pts + (long)kl * (1 + D::NI);
        t = p[0];
        const double* pm = p + 1 + D::NS + D::NC + NDV;
        return LaneIn<D>{p + 1, p + 1 + D::NS, p + 1 + D::NS + D::NC, -1, 0.0, pm, pm + D::NM};
    }
    const int k = S.k0 + kl;
    LaneIn<D> in{S.x + 2 + (long)k * D::NS, S.x + 2 + (long)D::NS * S.G + (long)k * D::NC,
                 S.x + S.DB + (long)k * NDV, -1, 0.0, S.x + S.XM + (long)k * D::NM,
                 (D::NSL > 0 && (k & 1)) ? S.x + S.XL + (long)((k - 1) >> 1) * D::NSL : nullptr};
    t = lane_time(Ln, S.grid[k], S.x[0], S.x[1], r, in.pi, in.step);
    return in;
}

// Device task tables (built on the host per lane configuration).
struct Tasks {
    int ng, stride, tdoubles, nmass, nk;   // tdoubles: T doubles per grid point
    const int* dlen;     // [ng] tasks per grid point of group g
    const int* off;      // [ng] slot offset of force group g within a grid point
    const int* roles;    // [ng][stride] j -> lane role
    const int* jd;       // [stride][ng] lane role -> slot of group g within the grid
                         // point (g = 0: index of the mass factor; base = first)
    const int4* blk;     // [nblocks] (group, first task, tasks per grid point, 1/n as float bits)
};

#define MH_IV_STAMP(i)

// CLS: 0 = every group; 1 = the heavy groups only (mass matrix and bias, or
// their parts: groups 0 .. D::NHEAVY - 1 of every generated model); 2 = the
// others.  A kernel
// compiled for one class allocates registers for that class's code alone
// (k_groups_part: a large model's heavy groups no longer set the register
// budget, hence the occupancy, of its many light ones).
template <class D, int CLS = 0>
__device__ __forceinline__ void groups_body_rec(const DevModel& M, const Src& S, const Lanes& Ln, const Tasks& TK,
        double* __restrict__ T, double* __restrict__ H, const int4 rec) {
    const int lane = threadIdx.x;
    // (group | live tasks << 16, first task, tasks per grid point, 1 / that)
    const int gx = __builtin_amdgcn_readfirstlane(rec.x);
    const int g = gx & 0xffff, cnt = gx >> 16;
    if (cnt == 0) return;           // a padding block of the XCD arrangement
    if constexpr (CLS == 1) __builtin_assume(g < D::NHEAVY);
    if constexpr (CLS == 2) __builtin_assume(g >= D::NHEAVY);
    const int first = __builtin_amdgcn_readfirstlane(rec.y);
    const int n = __builtin_amdgcn_readfirstlane(rec.z);
    const float inv = __int_as_float(__builtin_amdgcn_readfirstlane(rec.w));
    const int task = first + lane;
    const bool live = lane < cnt;
    const int tc = live ? task : 0;
    // tc / n through the float reciprocal, corrected to the exact quotient
    int kl = (int)((float)tc * inv);
    kl += (kl + 1) * n <= tc ? 1 : 0;
    kl -= kl * n > tc ? 1 : 0;
    const int j = tc - kl * n;
    // stride-1 lanes (eval_g): every task is the base role -- no dependent
    // load of the role table in front of the group's input loads
    const int r = TK.stride == 1 ? Ln.base : TK.roles[g * TK.stride + j];
    double t;
    const LaneIn<D> in = lane_input<D>(S, Ln, kl, r, t);
    constexpr int NOUT = D::NST > D::NF ? D::NST : D::NF;
    double out[NOUT];
    // the mass-matrix and bias groups are the longest tasks: give them issue
    // priority over the short muscle tasks sharing their SIMD
    if (g < D::NHEAVY) __builtin_amdgcn_s_setprio(2);
    D::group(g, M, t, in, out);
    if (!live) return;
    if (g == 0) {
        double* dst = H + ((long)kl * TK.nmass + j) * D::NST;
#pragma unroll
        for (int f = 0; f < D::NST; ++f) dst[f] = out[f];
    } else {
        // compact slab: group g's slots hold exactly its GROUP_NF[g] fields
        const int nf = D::GROUP_NF[g];
        double* dst = T + (long)kl * TK.tdoubles + TK.off[g] + j * nf;
#pragma unroll
        for (int f = 0; f < D::NF; ++f)
            if (f < nf) dst[f] = out[f];
    }
}

template <class D, int CLS = 0>
__device__ __forceinline__ void groups_body(const DevModel& M, const Src& S, const Lanes& Ln, const Tasks& TK,
        double* __restrict__ T, double* __restrict__ H, int blk) {
    groups_body_rec<D, CLS>(M, S, Ln, TK, T, H, TK.blk[blk]);   // one scalar load of the block's record
}

template <class D>
__global__ void __launch_bounds__(64) k_groups(DevModel M, Src S, Lanes Ln, Tasks TK,
        double* __restrict__ T, double* __restrict__ H) {
    groups_body<D>(M, S, Ln, TK, T, H, blockIdx.x);
}

// Variants measured no faster than the default path (round 5: k_groups_kr,
// k_combine_split, the slot table staged in LDS by k_interval) are compiled
// only with MOCOHIP_AB_VARIANTS=1 (make AB_VARIANTS=1), for A/B runs; the
// default build instantiates none of them and ignores their environment
// switches (profiles/r05_b, r05_n keep the measurements).
#ifndef MOCOHIP_AB_VARIANTS
#define MOCOHIP_AB_VARIANTS 0
#endif

// eval_g's task records in the kernel arguments.  With stride-1 lanes a
// block's record is (group | live tasks << 16, first task) -- one task per
// grid point and group -- and up to KR_MAX of them fit beside the other
// arguments: the record then arrives with the launch's arguments instead of
// one load of the task table after them (a dependent round trip at the head
// of every task wave's chain).  Opt-in (MOCOHIP_GROUPS_KR=1): measured no
// faster than the table's one scalar load (profiles/r05_n).
constexpr int KR_MAX = 384;
struct KRecs {
    int2 r[KR_MAX];
};
#if MOCOHIP_AB_VARIANTS
template <class D>
__global__ void __launch_bounds__(64) k_groups_kr(DevModel M, Src S, Lanes Ln, Tasks TK,
        double* __restrict__ T, double* __restrict__ H, KRecs KR) {
    const int2 rr = KR.r[blockIdx.x];
    groups_body_rec<D>(M, S, Ln, TK, T, H, make_int4(rr.x, rr.y, 1, __float_as_int(1.0f)));
}
#endif
// One class of groups (groups_body CLS), blocks blk0.. of the task table.
template <class D, int CLS>
__global__ void __launch_bounds__(64) k_groups_part(DevModel M, Src S, Lanes Ln, Tasks TK,
        double* __restrict__ T, double* __restrict__ H, int blk0) {
    groups_body<D, CLS>(M, S, Ln, TK, T, H, blk0 + (int)blockIdx.x);
}

// Output writers of a lane's combine: output o goes straight to its Y / LDS
// slot when the generated code produces it (no NO-long array held in
// registers until the end; the large models' combine spilled on it).
struct StridedOut {
    double* p;
    long s;
    __device__ __forceinline__ double& operator[](int o) const { return p[(long)o * s]; }
};
struct LdsOut {
    lds_double* p;
    int s;
    __device__ __forceinline__ lds_double& operator[](int o) const { return p[o * s]; }
};
// A lane role's combine sums (D::combine_sum) as D::combine_finish reads
// them: sum q at p[q * s] (LDS, [q][role]).
struct SumsLds {
    const lds_double* p;
    int s;
    __device__ __forceinline__ double operator()(int q) const { return p[q * s]; }
};

// Combine: one workgroup per grid point.  The grid point's group results
// (contiguous in T and H) are staged in LDS with coalesced loads; each lane
// (one lane role) then reads the slots it needs from LDS.
template <class D, class SP = const int* __restrict__>
struct TaskLoadLds {
    const lds_double* sT;
    const lds_double* sH;
    SP slot;                        // [stride][ng]: slot of group g for this role
    int r;
    __device__ __forceinline__ double operator()(int g, int f) const {
        return sT[slot[r * D::NG + g] + f];
    }
    __device__ __forceinline__ double h(int f) const {
        return sH[slot[r * D::NG] * D::NST + f];
    }
};

// Same arithmetic reading T/H straight from global memory: used when the
// grid point's slots do not fit in LDS (e.g. MOCOHIP_TASKS=all with central
// differences).
template <class D>
struct TaskLoadGlobal {
    const double* __restrict__ sT;
    const double* __restrict__ sH;
    const int* __restrict__ slot;
    int r;
    __device__ __forceinline__ double operator()(int g, int f) const {
        return sT[slot[r * D::NG + g] + f];
    }
    __device__ __forceinline__ double h(int f) const {
        return sH[slot[r * D::NG] * D::NST + f];
    }
};

// eval_g's lanes (stride 1: the base role only).  Every group then has one
// slot, so build_taskset puts group g (g > 0) at the prefix sum of GROUP_NF
// over groups 1 .. g - 1 and the mass factor at 0 -- offsets known at
// compile time.  Reading them as constants makes the combine's group-result
// reads plain loads at immediate offsets instead of each waiting on a scalar
// load of the slot table (the same values, bit for bit; the table path is
// MOCOHIP_IVG_BASE=0).
template <class D>
struct BaseSlots {
    int off[D::NG];
    constexpr BaseSlots() : off{} {
        int s = 0;
        for (int g = 0; g < D::NG; ++g) {
            off[g] = g > 0 ? s : 0;
            if (g > 0) s += D::GROUP_NF[g];
        }
    }
};
template <class D, class P>
struct TaskLoadBase {
    P sT;
    P sH;
    __device__ __forceinline__ double operator()(int g, int f) const {
        constexpr BaseSlots<D> B{};
        return sT[B.off[g] + f];
    }
    __device__ __forceinline__ double h(int f) const { return sH[f]; }
};

// The hardware dispatches a launch's workgroups to the 8 XCDs round-robin
// (workgroup b -> XCD b % 8), each XCD with its own L2.  Hermite-Simpson
// neighbours share a grid point, whose group results both intervals stage,
// so with I.xcd workgroup b takes interval c * q + min(c, rem) + b / 8
// (c = b % 8, q / rem = nb / 8, nb % 8): XCD c gets one contiguous run of
// intervals and the shared point's second read can hit that XCD's L2.  A
// bijection of 0 .. nb - 1 for every nb.
__device__ __forceinline__ int xcd_interval(int b, int nb) {
    const int c = b & 7, s = b >> 3, q = nb >> 3, rem = nb & 7;
    return c * q + (c < rem ? c : rem) + s;
}

// cmap (nmap roles per grid point): the lanes to combine, the others being
// excitation lanes k_exc_fill writes (null: every lane).
template <class D>
__global__ void __launch_bounds__(64) k_combine_global(DevModel M, Src S, Lanes Ln, Tasks TK,
        const double* __restrict__ T, const double* __restrict__ H, double* __restrict__ times,
        double* __restrict__ Y, long ystride_pt, const int* __restrict__ cmap, int nmap, int xcd) {
    // xcd: the blocks of one grid point's lanes on one XCD (xcd_interval over
    // the lane blocks): the lanes of a point gather from the same group
    // results, which then cross the XCD's L2 once instead of once per XCD
    const int blk = xcd ? xcd_interval((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const long gid = (long)blk * blockDim.x + threadIdx.x;
    const int per = cmap ? nmap : Ln.stride;
    if (gid >= (long)TK.nk * per) return;
    const int kl = (int)(gid / per);
    const int j = (int)(gid - (long)kl * per);
    const int r = cmap ? cmap[j] : j;
    double t;
    const LaneIn<D> in = lane_input<D>(S, Ln, kl, r, t);
    if (r == Ln.base && times) times[kl] = t;
    const TaskLoadGlobal<D> TL{T + (long)kl * TK.tdoubles, H + (long)kl * TK.nmass * D::NST,
                               TK.jd, r};
    D::combine(M, t, in, TL, StridedOut{Y + (long)kl * ystride_pt + r, (long)Ln.stride});
}

#if MOCOHIP_AB_VARIANTS
// k_combine_global with the combine in two steps (D::combine_sum /
// D::combine_finish, the arithmetic of D::combine bit for bit): a
// 256-thread workgroup takes 64 lane roles; its 4 waves compute the roles'
// NSUM independent sums -- wave w the sums w, w + 4, ... (q uniform over the
// wave), lanes over the roles -- into LDS [q][lane], then the first wave
// runs each role's factorization, solves and outputs from those sums.  A
// large model's sums are long chains of dependent group-result loads (each
// coordinate's generalized force over 80 muscles: Rajagopal 80), which one
// thread per role walked one after the other.
template <class D>
__global__ void __launch_bounds__(256) k_combine_split(DevModel M, Src S, Lanes Ln, Tasks TK,
        const double* __restrict__ T, const double* __restrict__ H, double* __restrict__ times,
        double* __restrict__ Y, long ystride_pt, const int* __restrict__ cmap, int nmap) {
    __shared__ double sS[(D::NSUM > 0 ? D::NSUM : 1) * 64];
    const int per = cmap ? nmap : Ln.stride;
    const int ln = (int)threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const long gid = (long)blockIdx.x * 64 + ln;
    const bool live = gid < (long)TK.nk * per;
    const long g = live ? gid : 0;
    const int kl = (int)(g / per);
    const int j = (int)(g - (long)kl * per);
    const int r = cmap ? cmap[j] : j;
    double t;
    const LaneIn<D> in = lane_input<D>(S, Ln, kl, r, t);
    const TaskLoadGlobal<D> TL{T + (long)kl * TK.tdoubles, H + (long)kl * TK.nmass * D::NST, TK.jd, r};
    for (int q = wv; q < D::NSUM; q += 4) {
        const double v = D::combine_sum(q, M, t, in, TL);
        if (live) sS[q * 64 + ln] = v;
    }
    __syncthreads();
    if (wv != 0 || !live) return;
    if (r == Ln.base && times) times[kl] = t;
    D::combine_finish(M, t, in, TL, SumsLds{lds(sS + ln), 64},
                      StridedOut{Y + (long)kl * ystride_pt + r, (long)Ln.stride});
}
#endif

// Excitation lanes of a generated back end (mocohip.hip k_exc_fill, launched
// through this host entry so that the fill kernel lives in one unit).
int mh_launch_exc_fill(const mh_ctx* c, int nk, int NO, int stride, int base, int tdoubles, const double* T,
                       double* Y);

// Copy n doubles to LDS with U loads in flight per thread before the first
// store (a plain strided loop serializes one memory round trip per pass).
template <int U>
__device__ __forceinline__ void stage_lds(double* __restrict__ dst, const double* __restrict__ src,
        int n) {
    for (int b = 0; b < n; b += U * (int)blockDim.x) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * (int)blockDim.x + (int)threadIdx.x;
            v[u] = src[i < n ? i : n - 1];   // unconditional: no branch per load
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = b + u * (int)blockDim.x + (int)threadIdx.x;
            if (i < n) dst[i] = v[u];
        }
    }
}

// With quot != 0 (Jacobian lanes) the kernel writes, per output o, the
// finite-difference quotient of direction r into Y slot r instead of the raw
// lane value (CasADi FiniteDiff formulas (f+ - f-)/2h, (f+ - f0)/h,
// (f0 - f-)/h; the base slot keeps the raw base value): one division per
// (grid point, output, direction) instead of one per Jacobian nonzero that
// reads it.  The lanes exchange their raw values through LDS.
// MAXT: the launch bound.  A grid point of up to 256 lane roles launches the
// 256-thread instantiation, whose lanes may keep up to 512 VGPRs: a large
// model's combine (Rajagopal 80: ~120 outputs, an 18-coordinate L^T L solve)
// then runs without the scratch spills the 1024-thread bound (128 VGPRs)
// forces on it.
// QUOT: the quotient mode compiled in (its per-lane out[NO] array sets the
// register budget; raw-value launches take the instantiation without it, so
// that a large model's combine does not spill for the quotient path it does
// not run: Rajagopal 80's 256-thread kernel carried 8.6 KB of scratch).
template <class D, int MAXT = 1024, bool QUOT = false>
__global__ void __launch_bounds__(MAXT) k_combine(DevModel M, Src S, Lanes Ln, Tasks TK,
        const double* __restrict__ T, const double* __restrict__ H, double* __restrict__ times,
        double* __restrict__ Y, long ystride_pt, int quot) {
    extern __shared__ double smem[];
    const int kl = blockIdx.x;
    const int nt = TK.tdoubles, nh = TK.nmass * D::NST;
    double* sT = smem;
    double* sH = smem + nt;
    const double* Tk = T + (long)kl * nt;
    const double* Hk = H + (long)kl * nh;
    if (nt > 0) stage_lds<16>(sT, Tk, nt);
    if (nh > 0) stage_lds<8>(sH, Hk, nh);
    __syncthreads();
    const int r = threadIdx.x;
    const bool act = r < Ln.stride;
    // Y[(kl*NO + o)*stride + r]  (ystride_pt = NO*stride; explicit points:
    // stride 1 -> out[p*NO + o])
    double* Yk = Y + (long)kl * ystride_pt + r;
    if constexpr (!QUOT) {   // raw lane values: each output straight to Y
        (void)quot;
        if (act) {
            double t;
            const LaneIn<D> in = lane_input<D>(S, Ln, kl, r, t);
            if (r == Ln.base && times) times[kl] = t;
            const TaskLoadLds<D> TL{lds(sT), lds(sH), TK.jd, r};
            D::combine(M, t, in, TL, StridedOut{Yk, (long)Ln.stride});
        }
        return;
    } else {
    double out[D::NO];
    if (act) {
        double t;
        const LaneIn<D> in = lane_input<D>(S, Ln, kl, r, t);
        if (r == Ln.base && times) times[kl] = t;
        const TaskLoadLds<D> TL{lds(sT), lds(sH), TK.jd, r};
        D::combine(M, t, in, TL, out);
    }
    __syncthreads();                 // every lane is done reading sT / sH
    double* sY = smem;               // [NO][stride] raw lane values
    if (act) {
#pragma unroll
        for (int o = 0; o < D::NO; ++o) sY[o * Ln.stride + r] = out[o];
    }
    __syncthreads();
    if (!act) return;
#pragma unroll
    for (int o = 0; o < D::NO; ++o) {
        const double* y = sY + o * Ln.stride;
        double v;
        if (r == Ln.base) v = out[o];
        else if (Ln.fd == MH_FD_CENTRAL) v = r < Ln.ND ? (out[o] - y[Ln.ND + r]) / (2.0 * Ln.h) : 0.0;
        else if (Ln.fd == MH_FD_FORWARD) v = (out[o] - y[Ln.base]) / Ln.h;
        else v = (y[Ln.base] - out[o]) / Ln.h;
        Yk[(long)o * Ln.stride] = v;
    }
    }
}

// Path-constraint equations (include/mocohip.h mh_path_equation) and the
// tables / grid their bound functions and time seeds read.
struct PathEqs {
    int npc;         // equations per mesh point
    const mh_path_equation* __restrict__ eq;
    const mh_table* __restrict__ tabs;
    const double* __restrict__ brk;
    const double* __restrict__ coef;
    const double* __restrict__ grid;
};

// Endpoint-constraint equations (include/mocohip.h mh_endpoint_equation):
// rows 0..nep of g and Jacobian entries 0..nnz of the shard that owns the
// first mesh interval.  The Endpoint callback's input vector (CasOCFunction.h:
// 167-240) is [initial_time, initial point inputs (NI), final_time, final
// point inputs]; W = 1 + NI per point.  Template entry: row = equation,
// dir = index into that vector.
struct EndpointEqs {
    int nep, nnz, W;
    const mh_endpoint_equation* __restrict__ eq;
    const TplEntry* __restrict__ tpl;
};

// Compiled Jacobian template (k_interval's assembly): one word per template
// entry of the Jacobian lane layout.  A value is base + coef * q, with q one
// double in the interval's LDS (a finite-difference quotient of sY, or the
// constant 0 / 1 of dxdot's exact qdot = u rows), or q itself (raw: residual
// rows); entries along t0 / tf (several f and dxdot terms) take the general
// jac_entry path, path-constraint entries their own loop.  Same operations in
// the same order as jac_entry, so the two agree bit for bit
// (test_kernel_variants_bit_identical, MOCOHIP_CTPL=0).
enum : uint32_t {
    CT_OFF = 0xFFFFFu,          // bits 0-19: LDS offset of q relative to sY
    CT_RAW = 1u << 26,
    CT_GEN = 1u << 27,
    CT_PATH = 1u << 28
};
__device__ __host__ __forceinline__ uint32_t ct_word(uint32_t off, uint32_t coef, uint32_t base) {
    return off | (coef << 20) | (base << 23);
}

// a / b rounded to nearest from y = 1 / b (itself rounded to nearest, formed
// once by the division): q = a y, then two residual corrections q += (a - b q)
// y with the residual exact in one fma.  A faithful q and y = RN(1/b) make
// q + (a - b q) y round to RN(a / b) (Markstein's theorem), and the first
// correction makes a y (within 1.5 ulp) faithful; tests/test_div_rn.py.  Valid while no product
// over- or underflows: |a| in [2^-900, 2^900] for b, y in [2^-60, 2^60];
// outside it (and for infinities) the division itself; a zero keeps its sign
// (a y).  The same bits as a / b at about half its instructions (no
// div_scale / rcp / div_fmas / div_fixup chain).
__device__ __forceinline__ double div_rn(double a, double b, double y) {
    double q = a * y;
    double r = __builtin_fma(-q, b, a);
    q = __builtin_fma(r, y, q);
    r = __builtin_fma(-q, b, a);
    q = __builtin_fma(r, y, q);
    const double m = __builtin_fabs(a);
    if (!(m >= 0x1p-900 && m <= 0x1p+900) && m != 0.0 && m == m) q = a / b;
    return m == 0.0 ? a * y : q;
}

struct Interval {
    int scheme;      // MH_HERMITE_SIMPSON / MH_TRAPEZOIDAL
    int interp;
    int ib;          // first interval of shard
    int rpi;         // rows per interval
    int nnz_int;     // nonzeros per interval
    int nres;        // residual rows per grid point: multibody (implicit: NQ), then auxiliary
    int nacc;        // multibody residual rows per grid point
    int oaux;        // callback output of the first auxiliary residual (NQ + NZ)
    // callback output behind residual row r of a grid point
    __device__ __forceinline__ int rout(int r) const { return r < nacc ? r : oaux + (r - nacc); }
    int N;           // mesh intervals of the whole problem
    int nnz_tail;    // nonzeros of the tail rows
    int ntail;       // tail rows: final mesh point's path rows + final residuals
    int npe;         // path-constraint entries per mesh point (lead the interval / tail)
    int nkr;         // kinematic-constraint rows per mesh point (first in the interval / tail)
    int okc;         // callback output of the first kinematic error
    PathEqs P;
    // the head (endpoint rows), written by the first interval's block when
    // this shard owns it: gh / vh = the shard's g / values (null otherwise)
    EndpointEqs E;
    double* gh;
    double* vh;
    int dbg_stop;    // diagnostic timing build only: return after phase n (0: full)
    int pf;          // k_interval prefetches its first IV_PF assembly words per thread
    int qfuse;       // k_interval forms each finite-difference quotient in the assembly
                     // (no in-place quotient pass)
    int xcd;         // k_interval: contiguous interval runs per XCD (xcd_interval)
    // k_transcribe's base-lane offsets: read from the table after the words
    // (0) or derived from the word's offset (1: off / stride * stride + base,
    // the division as a multiply-high by smagic, exact below 2^20 / stride;
    // the host checks it against the table once).  k_interval reads the
    // table: its words are prefetched with their offsets, and the derivation
    // measured slower there (17.7 -> 19.8 us, profiles/r06_c)
    int dbase;
    uint32_t smagic, sstride, sbase;
    int qdiv;        // k_transcribe's quotients by div_rn (1, MOCOHIP_QDIV=1) or the division (0)
    __device__ __forceinline__ uint32_t base_of(uint32_t w, uint32_t nyall) const {
        const uint32_t off = w & CT_OFF;
        const bool lane = !(w & (CT_GEN | CT_PATH)) && off < nyall;
        return lane ? __umulhi(off, smagic) * sstride + sbase : 0u;
    }
    // Every interval opens with its mesh point's path rows.  The interval
    // N-1 also owns the tail (flattenConstraints, CasOCTranscription.h:
    // 286-308): the final mesh point's path rows, then the final grid
    // point's residual rows, as rows rpi..rpi+ntail after its own and
    // template entries nnz_int..nnz_int+nnz_tail.
    __device__ __forceinline__ int rows(int i) const { return rpi + (i == N - 1 ? ntail : 0); }
    __device__ __forceinline__ int entries(int i) const { return nnz_int + (i == N - 1 ? nnz_tail : 0); }
};

// Path-constraint arithmetic, evaluated in order without contraction so
// that the finite-difference quotients see the same roundings as the CPU
// restatement (the perturbed time t + h*seed, the Horner steps).
__device__ __forceinline__ double path_bound(const PathEqs& P, const mh_path_equation& E, double t) {
#pragma clang fp contract(off)
    if (E.table < 0) return E.value;
    const mh_table T = P.tabs[E.table];
    const double* br = P.brk + T.break_begin;
    int s;
    if (t <= br[0]) s = 0;
    else if (t >= br[T.nseg]) s = T.nseg - 1;
    else {
        int lo = 0, hi = T.nseg;
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (t < br[mid]) hi = mid; else lo = mid;
        }
        s = lo;
    }
    const double* cf = P.coef + T.coef_begin + ((long)s * T.ncol + E.column) * (T.degree + 1);
    const double dt = t - br[s];
    double v = cf[T.degree];
    for (int k = T.degree - 1; k >= 0; --k) v = v * dt + cf[k];
    return v;
}
// MocoControlBoundConstraint::calcPathConstraintErrorsImpl
// (MocoControlBoundConstraint.cpp:130-146): control - bound(t).
__device__ __forceinline__ double path_value(const PathEqs& P, int e, double t, double control) {
    const mh_path_equation E = P.eq[e];
    return control - path_bound(P, E, t);
}
// FD quotient of equation e at grid point k along direction dir (0 = t0,
// 1 = tf, 2 + j = point input j), CasADi FiniteDiff as for the DAE lanes.
// The equation reads only its control and the time: along any other input
// the perturbed and base values are equal and the quotient is exactly 0.
__device__ __forceinline__ double path_quot(const PathEqs& P, const Lanes& Ln, int NS, int e, int k,
        double t, double control, int dir) {
#pragma clang fp contract(off)
    const mh_path_equation E = P.eq[e];
    if (dir >= 2 && dir != 2 + NS + E.index) return 0.0;
    const double h = Ln.h;
    double tp = t, tm = t, cp = control, cm = control;
    if (dir < 2) {
        const double g = P.grid[k];
        const double seed = dir == 0 ? 1.0 - g : g;
        tp = t + h * seed;
        tm = t - h * seed;
    } else {
        cp = control + h;
        cm = control - h;
    }
    if (Ln.fd == MH_FD_CENTRAL)
        return ((cp - path_bound(P, E, tp)) - (cm - path_bound(P, E, tm))) / (2.0 * h);
    const double v0 = control - path_bound(P, E, t);
    if (Ln.fd == MH_FD_FORWARD) return ((cp - path_bound(P, E, tp)) - v0) / h;
    return (v0 - (cm - path_bound(P, E, tm))) / h;
}

// x index of endpoint input si (initial / final grid point, see EndpointEqs).
__device__ __forceinline__ long ep_xindex(const Layout& L, int W, int si) {
    const int pt = si >= W ? 1 : 0, j = si - pt * W - 1;
    if (j < 0) return pt;   // initial_time = x[0], final_time = x[1]
    const long k = pt ? L.G - 1 : 0;
    if (j < L.NS) return 2 + k * L.NS + j;
    if (j < L.NS + L.NC) return 2 + (long)L.NS * L.G + k * L.NC + (j - L.NS);
    return L.DB + k * L.NDV + (j - L.NS - L.NC);
}
// An endpoint equation on its input vector (accessor in(si)).
// MH_ENDPOINT_INITIAL_ACTIVATION: MocoInitialActivationGoal::calcGoalImpl in
// endpoint-constraint mode (MocoInitialActivationGoal.cpp:41-58).
template <class A>
__device__ __forceinline__ double ep_eval(const mh_endpoint_equation& Q, int NS, const A& in) {
    return in(1 + NS + Q.index_a) - in(1 + Q.index_b);
}
// Value of equation e at iterate x with input pi perturbed by step (-1: none).
__device__ __forceinline__ double ep_value(const Layout& L, const EndpointEqs& E, const double* __restrict__ x,
        int e, int pi, double step) {
    const mh_endpoint_equation Q = E.eq[e];
    return ep_eval(Q, L.NS, [&](int si) {
        const double v = x[ep_xindex(L, E.W, si)];
        return si == pi ? v + step : v;
    });
}
// The head: endpoint rows of g and their Jacobian entries (CasADi
// FiniteDiff quotients along each structural column, as for the DAE lanes).
__device__ __forceinline__ void endpoint_head(const Layout& L, const Lanes& Ln, const EndpointEqs& E,
        const double* __restrict__ x, double* __restrict__ g, double* __restrict__ v, int tid, int nthr) {
#pragma clang fp contract(off)
    if (g)
        for (int r = tid; r < E.nep; r += nthr) g[r] = ep_value(L, E, x, r, -1, 0.0);
    if (v)
        for (int q = tid; q < E.nnz; q += nthr) {
            const TplEntry T = E.tpl[q];
            const double h = Ln.h;
            double d;
            if (Ln.fd == MH_FD_CENTRAL)
                d = (ep_value(L, E, x, T.row, T.dir, h) - ep_value(L, E, x, T.row, T.dir, -h)) / (2.0 * h);
            else if (Ln.fd == MH_FD_FORWARD)
                d = (ep_value(L, E, x, T.row, T.dir, h) - ep_value(L, E, x, T.row, -1, 0.0)) / h;
            else
                d = (ep_value(L, E, x, T.row, -1, 0.0) - ep_value(L, E, x, T.row, T.dir, -h)) / h;
            v[q] = d;
        }
}

__device__ __forceinline__ int grid_of(const Interval& I, int i, int pt) {
    return I.scheme == MH_HERMITE_SIMPSON ? 2 * i + pt : i + pt;
}

// Raw DAE outputs of a grid point's lanes and the grid point's time, as
// read by the transcription arithmetic.  YG: Y and the base-lane times in
// HBM (written by k_combine, indexed by local grid point k - k0).  YS: the
// same values staged in LDS by k_interval for the interval's own points
// (indexed by k - kf, kf = the interval's first grid point).
struct YG {
    const double* __restrict__ Y;
    const double* __restrict__ times;
    int NO, stride, k0;
    int q;   // Y holds finite-difference quotients (k_combine quot mode)
    const double* __restrict__ x;
    int NS, NC, G;
    // state s / control j of grid point k from the iterate
    __device__ __forceinline__ double xs(int k, int s) const { return x[2 + (long)k * NS + s]; }
    __device__ __forceinline__ double xc(int k, int j) const {
        return x[2 + (long)NS * G + (long)k * NC + j];
    }
    int NDV;
    long DB;
    __device__ __forceinline__ double xd(int k, int j) const { return x[DB + (long)k * NDV + j]; }
    __device__ __forceinline__ const double* row(int k, int o) const {
        return Y + ((long)(k - k0) * NO + o) * stride;
    }
    __device__ __forceinline__ double t(int k) const { return times[k - k0]; }
};
struct YS {
    const lds_double* Y;
    const lds_double* times;
    int NO, stride, kf;
    int q;
    // the interval's states / controls staged in LDS ([point][NS], [point][NC])
    const lds_double* sxs;
    const lds_double* sxc;
    int NS, NC;
    __device__ __forceinline__ double xs(int k, int s) const { return sxs[(k - kf) * NS + s]; }
    __device__ __forceinline__ double xc(int k, int j) const { return sxc[(k - kf) * NC + j]; }
    const lds_double* sxd;
    int NDV;
    __device__ __forceinline__ double xd(int k, int j) const { return sxd[(k - kf) * NDV + j]; }
    __device__ __forceinline__ const lds_double* row(int k, int o) const {
        return Y + ((k - kf) * NO + o) * stride;
    }
    __device__ __forceinline__ double t(int k) const { return times[k - kf]; }
};

// xdot[s] at grid point k.
template <class YV>
__device__ __forceinline__ double xdot_at(const Layout& L, const Lanes& Ln,
        const double* __restrict__ x, const YV& Y, int k, int s) {
#pragma clang fp contract(off)
    if (s < L.NQ) {
        // qdot = u, plus the velocity correction G^T gamma at a mesh-interval
        // midpoint (CasOCTranscription.cpp:316-333)
        if (L.vc(k)) return Y.xs(k, L.NQ + s) + Y.row(k, L.OQC + s)[Ln.base];
        return Y.xs(k, L.NQ + s);
    }
    if (L.NACC && s < 2 * L.NQ) return Y.xd(k, s - L.NQ);   // implicit: udot = w
    return Y.row(k, s + L.SO)[Ln.base];
}

template <class YV>
__device__ __forceinline__ double defect_row(const Layout& L, const Interval& I, const Lanes& Ln,
        const double* __restrict__ x, const YV& Y, int i, int r) {
#pragma clang fp contract(off)
    const int NS = L.NS;
    // residual rows: the interval's grid points (HS: 2, trapezoidal: 1), and
    // for the last interval the final grid point after all its other rows
    const int npres = I.scheme == MH_HERMITE_SIMPSON ? 2 : 1;
    const int k_first = I.scheme == MH_HERMITE_SIMPSON ? 2 * i : i;
    const int npc = I.P.npc;
    if (r >= I.rpi) {   // tail: final mesh point's kinematic and path rows, then its residuals
        int rt = r - I.rpi;
        const int kl = k_first + npres;
        if (rt < I.nkr) return Y.row(kl, I.okc + rt)[Ln.base];
        rt -= I.nkr;
        if (rt < npc) return path_value(I.P, rt, Y.t(kl), Y.xc(kl, I.P.eq[rt].index));
        return Y.row(kl, I.rout(rt - npc))[Ln.base];
    }
    // the mesh point's kinematic-constraint rows (callback outputs okc..)
    if (r < I.nkr) return Y.row(k_first, I.okc + r)[Ln.base];
    r -= I.nkr;
    if (r < npc) return path_value(I.P, r, Y.t(k_first), Y.xc(k_first, I.P.eq[r].index));
    r -= npc;
    if (r < npres * I.nres) return Y.row(k_first + r / I.nres, I.rout(r % I.nres))[Ln.base];
    r -= npres * I.nres;
    if (I.scheme == MH_HERMITE_SIMPSON) {
        const int ki = 2 * i, km = ki + 1, kp = ki + 2;
        const double h = Y.t(kp) - Y.t(ki);
        if (r < NS) {
            const int s = r;
            const double xi = Y.xs(ki, s), xm = Y.xs(km, s), xp = Y.xs(kp, s);
            const double fi = xdot_at(L, Ln, x, Y, ki, s), fp = xdot_at(L, Ln, x, Y, kp, s);
            return xm - 0.5 * (xp + xi) - (h / 8.0) * (fi - fp);
        }
        if (r < 2 * NS) {
            const int s = r - NS;
            const double xi = Y.xs(ki, s), xp = Y.xs(kp, s);
            const double fi = xdot_at(L, Ln, x, Y, ki, s), fm = xdot_at(L, Ln, x, Y, km, s),
                         fp = xdot_at(L, Ln, x, Y, kp, s);
            return xp - xi - (h / 6.0) * (fp + 4.0 * fm + fi);
        }
        const int j = r - 2 * NS;
        return Y.xc(km, j) - 0.5 * (Y.xc(kp, j) + Y.xc(ki, j));
    }
    const int ki = i, kp = i + 1;
    const double h = Y.t(kp) - Y.t(ki);
    const int s = r;
    const double xi = Y.xs(ki, s), xp = Y.xs(kp, s);
    const double fi = xdot_at(L, Ln, x, Y, ki, s), fp = xdot_at(L, Ln, x, Y, kp, s);
    return xp - (xi + 0.5 * h * (fp + fi));
}

// d (DAE output o) / d dir at grid point k (the finite-difference quotient).
template <class YV>
__device__ __forceinline__ double dout(const Lanes& Ln, const YV& Y, int k, int o, int dir) {
#pragma clang fp contract(off)
    const auto y = Y.row(k, o);
    if (Y.q) return y[dir];
    if (Ln.fd == MH_FD_CENTRAL) return (y[dir] - y[Ln.ND + dir]) / (2.0 * Ln.h);
    if (Ln.fd == MH_FD_FORWARD) return (y[dir] - y[Ln.base]) / Ln.h;
    return (y[Ln.base] - y[dir]) / Ln.h;
}

// d xdot[s] / d dir at grid point k from the raw lane outputs
// (CasADi FiniteDiff formulas: (f+ - f-)/2h, (f+ - f0)/h, (f0 - f-)/h).
template <class YV>
__device__ __forceinline__ double dxdot(const Layout& L, const Lanes& Ln, const YV& Y, int k, int s,
        int dir) {
#pragma clang fp contract(off)
    if (s < L.NQ) {
        const double v = dir == 2 + L.NQ + s ? 1.0 : 0.0;
        if (L.vc(k)) return v + dout(Ln, Y, k, L.OQC + s, dir);   // + the correction's quotient
        return v;
    }
    if (L.NACC && s < 2 * L.NQ) return dir == 2 + L.NS + L.NC + (s - L.NQ) ? 1.0 : 0.0;
    return dout(Ln, Y, k, s + L.SO, dir);
}


constexpr int ASM_CHUNK = 1024;   // nonzeros per assembly workgroup

// Per-interval constants of the Jacobian formulas (computed once per
// interval; exactly the subexpressions the formulas would form per entry).
struct IvC { double h8, h6, hh, g8, g6, gh; };
__device__ __forceinline__ IvC iv_const(double h, double dgap) {
#pragma clang fp contract(off)
    return IvC{h / 8.0, h / 6.0, 0.5 * h, dgap / 8.0, dgap / 6.0, 0.5 * dgap};
}

// Jacobian value of template entry T of the interval whose first grid point
// is k_first (HS: d/d[t0,tf] of -(h/8)(f_i - f_p) with dh/dt0 = -dgap,
// dh/dtf = dgap, etc.).
// WITH_PATH = false compiles the path-constraint case out (k_interval
// evaluates those entries in a loop of their own, off the hot loop).
template <bool WITH_PATH = true, class YV>
__device__ __forceinline__ double jac_entry(const Layout& L, const Lanes& Ln, const PathEqs& P,
        const double* __restrict__ x, const YV& Y, const TplEntry T, int k_first, const IvC& C) {
    // no contraction anywhere in the Jacobian / defect arithmetic: every
    // product and sum rounds on its own, exactly as the checker's (oracle)
    // restatement of the same formulas does (tests/test_gpu_parity.py
    // test_jacobian_assembly_bit_exact_from_device_lanes)
#pragma clang fp contract(off)
    const int s = T.s, dir = T.dir;
    double v = 0.0;
    switch (T.kind) {
    // t0 / tf columns, and (dir >= 2) the parameter columns of a row: a
    // parameter moves no time, so only the callbacks' quotients remain
    case T_HERM_T: {
        const int ki = k_first, kp = k_first + 2;
        if (dir >= 2) {
            v = 0.0 - C.h8 * (dxdot(L, Ln, Y, ki, s, dir) - dxdot(L, Ln, Y, kp, s, dir));
            break;
        }
        const double fi = xdot_at(L, Ln, x, Y, ki, s), fp = xdot_at(L, Ln, x, Y, kp, s);
        v = (dir == 0 ? C.g8 : -C.g8) * (fi - fp) -
            C.h8 * (dxdot(L, Ln, Y, ki, s, dir) - dxdot(L, Ln, Y, kp, s, dir));
        break;
    }
    case T_SIMP_T: {
        const int ki = k_first, km = k_first + 1, kp = k_first + 2;
        if (dir >= 2) {
            v = 0.0 - C.h6 * (dxdot(L, Ln, Y, kp, s, dir) + 4.0 * dxdot(L, Ln, Y, km, s, dir) +
                              dxdot(L, Ln, Y, ki, s, dir));
            break;
        }
        const double fi = xdot_at(L, Ln, x, Y, ki, s), fm = xdot_at(L, Ln, x, Y, km, s),
                     fp = xdot_at(L, Ln, x, Y, kp, s);
        v = (dir == 0 ? C.g6 : -C.g6) * (fp + 4.0 * fm + fi) -
            C.h6 * (dxdot(L, Ln, Y, kp, s, dir) + 4.0 * dxdot(L, Ln, Y, km, s, dir) +
                    dxdot(L, Ln, Y, ki, s, dir));
        break;
    }
    case T_HERM_X: {
        const int k = k_first + T.pt;
        const bool ident = dir == 2 + s;
        if (T.pt == 1) { v = ident ? 1.0 : 0.0; break; }
        if (ident) v += -0.5;
        const double dv = dxdot(L, Ln, Y, k, s, dir);
        v += (T.pt == 0 ? -C.h8 : C.h8) * dv;
        break;
    }
    case T_SIMP_X: {
        const int k = k_first + T.pt;
        const bool ident = dir == 2 + s;
        const double dv = dxdot(L, Ln, Y, k, s, dir);
        if (T.pt == 2) { if (ident) v += 1.0; v += -C.h6 * dv; }
        else if (T.pt == 0) { if (ident) v += -1.0; v += -C.h6 * dv; }
        else v += -C.h6 * 4.0 * dv;
        break;
    }
    case T_INTERP:
        v = T.pt == 1 ? 1.0 : -0.5;
        break;
    case T_RES:
        v = dout(Ln, Y, k_first + T.pt, s, dir);
        break;
    case T_PATH:
        if constexpr (WITH_PATH) {
            const int k = k_first + T.pt;
            v = path_quot(P, Ln, L.NS, s, k, Y.t(k), Y.xc(k, P.eq[s].index), dir);
        }
        break;
    case T_TRAP_T: {
        const int ki = k_first, kp = k_first + 1;
        if (dir >= 2) {
            v = 0.0 - C.hh * (dxdot(L, Ln, Y, kp, s, dir) + dxdot(L, Ln, Y, ki, s, dir));
            break;
        }
        const double fi = xdot_at(L, Ln, x, Y, ki, s), fp = xdot_at(L, Ln, x, Y, kp, s);
        v = (dir == 0 ? C.gh : -C.gh) * (fp + fi) -
            C.hh * (dxdot(L, Ln, Y, kp, s, dir) + dxdot(L, Ln, Y, ki, s, dir));
        break;
    }
    case T_TRAP_X: {
        const int k = k_first + T.pt;
        const bool ident = dir == 2 + s;
        const double dv = dxdot(L, Ln, Y, k, s, dir);
        if (T.pt == 1) { if (ident) v += 1.0; v += -C.hh * dv; }
        else { if (ident) v += -1.0; v += -C.hh * dv; }
        break;
    }
    }
    return v;
}

__device__ __forceinline__ void interval_span(const Interval& I, int i, int& k_first, int& k_last) {
    k_first = grid_of(I, i, 0);
    k_last = k_first + (I.scheme == MH_HERMITE_SIMPSON ? 2 : 1);
}

// Fused combine + transcription: one workgroup per mesh interval.  The
// group results (T, H) of the interval's 2-3 grid points are staged in LDS
// together, every (grid point, lane role) is combined in parallel into
// LDS-resident raw outputs, and the whole workgroup then writes the
// interval's g rows and Jacobian values from LDS.  Same arithmetic as
// k_combine + k_transcribe (bit-identical results) with Y never touching
// HBM and one kernel less per evaluation.  Launched when the LDS budget
// allows (interval_lds), otherwise the split path runs.
constexpr int IV_UNROLL = 4;
constexpr int IV_PF = 12;   // k_interval: assembly words per thread prefetched before the quotients
// LDS constants after the times: [0] 0.0, [1] 1.0, [2..7] the interval's
// coefficients {0, -h/8, h/8, -h/6, (-h/6) 4, -h/2}, [8..11] the bases {0,
// -1/2, 1, -1} (a word's coefficient / base selectors index them).  After
// the words (entries(N - 1) of them) the compiled template holds one more
// word per entry: the LDS offset of the entry's row's base lane.
constexpr int CT_CONST = 4;      // offset of the constants after sTimes
constexpr int CT_NCONST = 12;

// GM: the combine reads the group results straight from global memory (T,
// H) instead of staging them in LDS -- a third of the LDS, so that several
// interval blocks share a CU (the batched launches, where many blocks queue);
// the same arithmetic in the same order, bit for bit.
// BASE: eval_g's kernel (stride-1 lanes, no Jacobian values): the combine
// reads the group results at their compile-time base slots (TaskLoadBase)
// and the assembly is compiled out.
// SLDS: the role -> slot table staged in LDS with the group results (the
// Jacobian lanes' combine then reads its slots from LDS instead of global
// memory after the barrier; MOCOHIP_IV_SLOTS_LDS=1).
template <class D, bool GM, bool BASE = false, bool SLDS = false>
__device__ __forceinline__ void interval_body(const DevModel& M, const Src& S, const Lanes& Ln, const Tasks& TK,
        const Layout& L, const Interval& I, const TplEntry* __restrict__ tpl, const uint32_t* __restrict__ ctpl,
        const int* __restrict__ ctgen, int nctgen,
        const double* __restrict__ T, const double* __restrict__ H, double* __restrict__ g,
        double* __restrict__ values, int il) {
    extern __shared__ double smem[];
    if constexpr (BASE) values = nullptr;
    const int i = I.ib + il;
    int k_first, k_last;
    interval_span(I, i, k_first, k_last);
    const int npts = k_last - k_first + 1;
    const int nt = TK.tdoubles, nh = TK.nmass * D::NST;
    const int ny = D::NO * Ln.stride;
    double* sY = smem;                       // [npts][NO][stride]
    double* sTimes = sY + npts * ny;         // [npts] (+ pad)
    double* sK = sTimes + CT_CONST;          // compiled-template constants
    double* sT = sK + CT_NCONST;             // [npts][nt] (GM: none)
    double* sH = sT + (GM ? 0 : npts * nt);  // [npts][nh] (GM: none)
    double* sXs = sH + (GM ? 0 : npts * nh); // [npts][NS] states, [npts][NC] controls,
    double* sXc = sXs + npts * L.NS;         // [npts][NDV] accelerations (implicit),
    double* sXd = sXc + npts * L.NC;         // [npts][NM] multipliers, [NSL] the
    double* sXm = sXd + npts * L.NDV;        // interval's slacks (HS midpoint)
    double* sXl = sXm + npts * L.NM;
    int* sSl = (int*)(sXl + L.NSL);          // SLDS: [stride][NG] slots
    // the interval's points are consecutive local grid points: their T (and
    // H) slabs are one contiguous run each
    const int kl0 = k_first - S.k0;
    if (I.dbg_stop == 7) return;   // diagnostic: the launch floor
    if constexpr (BASE && GM) {
        // eval_g's combine lanes (one per grid point, the base role) start at
        // once: their inputs from global memory, the group results at their
        // base slots, while the other threads stage the states the g rows
        // read -- one memory round trip after the arguments instead of the
        // staging's round trip and barrier first (the same values: the LDS
        // path, MOCOHIP_IVG_GM=0, compares bit for bit)
        if ((int)threadIdx.x < npts) {
            const int p = threadIdx.x;
            double t;
            const LaneIn<D> in = lane_input<D>(S, Ln, kl0 + p, Ln.base, t);
            sTimes[p] = t;
            const TaskLoadBase<D, const double*> TL{T + (long)(kl0 + p) * nt, H + (long)(kl0 + p) * nh};
            D::combine(M, t, in, TL, LdsOut{lds(sY + p * ny + Ln.base), Ln.stride});
        }
    }
    if (!GM && nt > 0) stage_lds<16>(sT, T + (long)kl0 * nt, npts * nt);
    if (!GM && nh > 0) stage_lds<8>(sH, H + (long)kl0 * nh, npts * nh);
    stage_lds<1>(sXs, S.x + 2 + (long)k_first * L.NS, npts * L.NS);
    if (L.NC > 0) stage_lds<1>(sXc, S.x + 2 + (long)L.NS * L.G + (long)k_first * L.NC, npts * L.NC);
    if (L.NDV > 0)
        stage_lds<1>(sXd, S.x + L.DB + (long)k_first * L.NDV, npts * L.NDV);
    if (L.NM > 0) stage_lds<1>(sXm, S.x + L.XM + (long)k_first * L.NM, npts * L.NM);
    if (L.NSL > 0) stage_lds<1>(sXl, S.x + L.XL + (long)i * L.NSL, L.NSL);
    if constexpr (SLDS)
        for (int q = threadIdx.x; q < Ln.stride * D::NG; q += blockDim.x) sSl[q] = TK.jd[q];
    const double t0 = S.x[0], tf = S.x[1];
    if (threadIdx.x < 2) sK[threadIdx.x] = threadIdx.x ? 1.0 : 0.0;
    __syncthreads();
    if (I.dbg_stop == 1) return;
    // eval_g's lanes (stride 1: every lane is the base role 0, written as a
    // constant so that the role -> slot reads have uniform addresses and
    // compile to scalar loads off the combine's critical path)
    auto combine_lane = [&](int p, int r) {
        LaneInL<D> in{lds(sXs + p * L.NS), lds(sXc + p * L.NC), lds(sXd + p * L.NDV), -1, 0.0,
                      lds(sXm + p * L.NM), L.vc(k_first + p) ? lds(sXl) : nullptr};
        const double t = lane_time(Ln, S.grid[k_first + p], t0, tf, r, in.pi, in.step);
        if (r == Ln.base) sTimes[p] = t;
        const LdsOut out{lds(sY + p * ny + r), Ln.stride};
        if constexpr (BASE) {   // (BASE && GM combined before the staging, above)
            const TaskLoadBase<D, const lds_double*> TL{lds(sT + p * nt), lds(sH + p * nh)};
            D::combine(M, t, in, TL, out);
        } else if constexpr (GM) {
            const TaskLoadGlobal<D> TL{T + (long)(kl0 + p) * nt, H + (long)(kl0 + p) * nh, TK.jd, r};
            D::combine(M, t, in, TL, out);
        } else if constexpr (SLDS) {
            const TaskLoadLds<D, const lds_int*> TL{lds(sT + p * nt), lds(sH + p * nh), (const lds_int*)sSl, r};
            D::combine(M, t, in, TL, out);
        } else {
            const TaskLoadLds<D> TL{lds(sT + p * nt), lds(sH + p * nh), TK.jd, r};
            D::combine(M, t, in, TL, out);
        }
    };
    // (one thread per lane role: the combine split over the waves --
    // D::combine_sum into LDS, then D::combine_finish -- measured slower:
    // k_interval 17.6 -> 19.7 us, eval_g's 9.9 -> 10.6 us, profiles/r05_b;
    // the combine is not bound by its sums' load-and-add chains)
    if constexpr (BASE && GM) {
    } else if (BASE || Ln.stride == 1) {
        if ((int)threadIdx.x < npts) combine_lane((int)threadIdx.x, 0);
    } else {
        for (int w = threadIdx.x; w < npts * Ln.stride; w += blockDim.x) {
            const int p = w / Ln.stride, r = w - p * Ln.stride;
            combine_lane(p, r);
        }
    }
    // the compiled words of this thread's first IV_PF assembly entries,
    // loaded now: their latency hides behind the quotients and the g rows
    // (on CDNA a wave's loads and stores share one counter -- loaded after
    // the g rows' stores, they would wait for those to complete)
    const int ne_iv = values ? I.entries(i) : 0;
    uint32_t pw[IV_PF];
#pragma unroll
    for (int u = 0; u < IV_PF; ++u) {
        const int e = threadIdx.x + u * blockDim.x;
        pw[u] = I.pf && ctpl && e < ne_iv ? ctpl[e] : CT_GEN;
    }
    const uint32_t* __restrict__ cbase = ctpl ? ctpl + I.nnz_int + I.nnz_tail : nullptr;
    uint32_t pb[IV_PF];
#pragma unroll
    for (int u = 0; u < IV_PF; ++u) {
        const int e = threadIdx.x + u * blockDim.x;
        pb[u] = I.pf && ctpl && e < ne_iv ? cbase[e] : 0u;
    }
    // likewise the template entry of this thread's first t0 / tf entry
    int eg0 = -1;
    TplEntry tg0{};
    if (I.pf && ctpl && values && (int)threadIdx.x < nctgen) {
        eg0 = ctgen[threadIdx.x];
        tg0 = tpl[eg0];
    }
    __syncthreads();
    if (values && ctpl && threadIdx.x == 0) {
        // the coefficient / base tables the words select from (the same
        // doubles the general path computes)
        const IvC C0 = iv_const(sTimes[npts - 1] - sTimes[0], S.grid[k_last] - S.grid[k_first]);
        sK[2] = 0.0; sK[3] = -C0.h8; sK[4] = C0.h8; sK[5] = -C0.h6; sK[6] = -C0.h6 * 4.0; sK[7] = -C0.hh;
        sK[8] = 0.0; sK[9] = -0.5; sK[10] = 1.0; sK[11] = -1.0;
    }
    // finite-difference quotients in place (CasADi FiniteDiff formulas), once
    // per (point, output, direction) instead of once per Jacobian entry that
    // reads them; the base slot keeps the raw value for the defect rows
    if (I.dbg_stop == 2) return;
    const int quot = values && Ln.stride > 1 && !I.qfuse;
    if (quot) {
#pragma clang fp contract(off)
        // one (point, output) row of lanes per wave: lanes = directions
        const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, nwave = blockDim.x >> 6;
        const double h = Ln.h, h2 = 2.0 * Ln.h;
        for (int po = wave; po < npts * D::NO; po += nwave) {
            lds_double* y = lds(sY + po * Ln.stride);
            const double yb = y[Ln.base];
            for (int d = lane; d < Ln.ND; d += 64) {
                double q;
                if (Ln.fd == MH_FD_CENTRAL) q = (y[d] - y[Ln.ND + d]) / h2;
                else if (Ln.fd == MH_FD_FORWARD) q = (y[d] - yb) / h;
                else q = (yb - y[d]) / h;
                y[d] = q;
            }
        }
        __syncthreads();
    }
    const YS YV{lds(sY), lds(sTimes), D::NO, Ln.stride, k_first, quot, lds(sXs), lds(sXc), L.NS, L.NC,
                lds(sXd), L.NDV};
    if (I.dbg_stop == 3) return;
    if (I.dbg_stop >= 5 && values) {
        // diagnostic: the assembly's stores alone (5) / its template loads,
        // LDS reads and arithmetic alone (6)
        double* vi = values + (long)il * I.nnz_int;
        const int ne = I.entries(i);
        double acc = 0.0;
        for (int e = threadIdx.x; e < ne; e += blockDim.x) {
            if (I.dbg_stop == 5) vi[e] = 0.0;
            else {
                const uint32_t wu = ctpl ? ctpl[e] : 0u;
                acc += sY[wu & CT_OFF] * (double)(wu >> 20);
            }
        }
        if (I.dbg_stop == 6 && acc == 12345.678) vi[threadIdx.x] = acc;
        return;
    }
    if (g) {
        double* gi = g + (long)il * I.rpi;
        for (int r = threadIdx.x; r < I.rows(i); r += blockDim.x) gi[r] = defect_row(L, I, Ln, S.x, YV, i, r);
    }
    if (I.dbg_stop == 4) return;
    if (values && ctpl) __syncthreads();   // the coefficient / base tables in sK
    if (values) {
        const IvC C = iv_const(YV.t(k_last) - YV.t(k_first), S.grid[k_last] - S.grid[k_first]);
        double* vi = values + (long)il * I.nnz_int;
        const int ne = I.entries(i);
        const int B = blockDim.x;
        int e = threadIdx.x;
        // path-constraint entries (the first npe of the interval and of
        // the tail) are written by their own loop below
        if (ctpl) {
#pragma clang fp contract(off)
            const lds_double* q0 = lds(sY);
            // coefficient / base of a word: LDS tables (sK, filled above)
            const lds_double* kc = lds(sK + 2);
            const lds_double* kb = lds(sK + 8);
            // I.qfuse: the word's LDS offset names the raw value of the
            // perturbed lane; the quotient (CasADi FiniteDiff) is formed here
            // from it and its row's base (forward / backward: the base-lane
            // offset stored after the words) or mirror (central) lane -- the
            // quotient pass's arithmetic, bit for bit
            const int nyall = npts * ny;
            const int fuse = values && Ln.stride > 1 && I.qfuse;
            const double h1 = Ln.h, h2 = 2.0 * Ln.h;
            auto value = [&](uint32_t wu, double q) {
                const double coef = kc[(wu >> 20) & 7], base = kb[(wu >> 23) & 7];
                return (wu & CT_RAW) ? q : base + coef * q;
            };
            // one instantiation per (finite-difference formula, fused
            // quotient): the per-entry quotient is branch-free (its other
            // operand is read unconditionally -- the mirror lane, or the
            // row's base lane, 0 where unused -- and selected away for the
            // LDS constants past the lanes)
            auto bulk = [&](auto fdc, auto fusec) {
                constexpr int FD = decltype(fdc)::value;
                constexpr bool FUSE = decltype(fusec)::value;
                auto qat = [&](uint32_t off, uint32_t boff) -> double {
                    const double y = q0[off];
                    if constexpr (!FUSE) {
                        return y;
                    } else {
                        const bool lane = (int)off < nyall;
                        const double ym = FD == MH_FD_CENTRAL ? q0[lane ? off + Ln.ND : off] : q0[boff];
                        const double qd = FD == MH_FD_CENTRAL ? (y - ym) / h2
                                        : FD == MH_FD_FORWARD ? (y - ym) / h1 : (ym - y) / h1;
                        return lane ? qd : y;
                    }
                };
                // the bulk: one LDS value, a product and a sum per entry; the
                // t0 / tf columns of the defect rows (CT_GEN) and the path
                // entries are written by the loops below
#pragma unroll
                for (int u = 0; u < IV_PF; ++u)
                    if (!(pw[u] & (CT_GEN | CT_PATH))) vi[e + u * B] = value(pw[u], qat(pw[u] & CT_OFF, pb[u]));
                if (I.pf) e += IV_PF * B;
                for (; e + (IV_UNROLL - 1) * B < ne; e += IV_UNROLL * B) {
                    uint32_t w[IV_UNROLL], wb[IV_UNROLL];
                    double q[IV_UNROLL];
#pragma unroll
                    for (int u = 0; u < IV_UNROLL; ++u) {
                        w[u] = ctpl[e + u * B];
                        wb[u] = cbase[e + u * B];
                    }
#pragma unroll
                    for (int u = 0; u < IV_UNROLL; ++u) q[u] = qat(w[u] & CT_OFF, wb[u]);
#pragma unroll
                    for (int u = 0; u < IV_UNROLL; ++u)
                        if (!(w[u] & (CT_GEN | CT_PATH))) vi[e + u * B] = value(w[u], q[u]);
                }
                for (; e < ne; e += B) {
                    const uint32_t wu = ctpl[e];
                    if (!(wu & (CT_GEN | CT_PATH))) vi[e] = value(wu, qat(wu & CT_OFF, cbase[e]));
                }
            };
            using FF = std::integral_constant<int, MH_FD_FORWARD>;
            using FB = std::integral_constant<int, MH_FD_BACKWARD>;
            using FC = std::integral_constant<int, MH_FD_CENTRAL>;
            if (!fuse) bulk(FF{}, std::false_type{});
            else if (Ln.fd == MH_FD_FORWARD) bulk(FF{}, std::true_type{});
            else if (Ln.fd == MH_FD_BACKWARD) bulk(FB{}, std::true_type{});
            else bulk(FC{}, std::true_type{});
            if (eg0 >= 0) vi[eg0] = jac_entry<false>(L, Ln, I.P, S.x, YV, tg0, k_first, C);
            for (int j = threadIdx.x + (I.pf ? B : 0); j < nctgen; j += B) {
                const int eg = ctgen[j];
                vi[eg] = jac_entry<false>(L, Ln, I.P, S.x, YV, tpl[eg], k_first, C);
            }
            e = ne;
        }
        // template entries for IV_UNROLL iterations are loaded before any is
        // evaluated (independent loads in flight, then LDS reads + stores)
        for (; e + (IV_UNROLL - 1) * B < ne; e += IV_UNROLL * B) {
            TplEntry te[IV_UNROLL];
#pragma unroll
            for (int u = 0; u < IV_UNROLL; ++u) te[u] = tpl[e + u * B];
#pragma unroll
            for (int u = 0; u < IV_UNROLL; ++u)
                if (te[u].kind != T_PATH) vi[e + u * B] = jac_entry<false>(L, Ln, I.P, S.x, YV, te[u], k_first, C);
        }
        for (; e < ne; e += B) {
            const TplEntry te = tpl[e];
            if (te.kind != T_PATH) vi[e] = jac_entry<false>(L, Ln, I.P, S.x, YV, te, k_first, C);
        }
        if (I.npe > 0) {
            const int npe = I.npe;
            const int nw = i == I.N - 1 ? 2 * npe : npe;
            for (int w = threadIdx.x; w < nw; w += B) {
                const int ep = w < npe ? w : I.nnz_int + (w - npe);
                vi[ep] = jac_entry<true>(L, Ln, I.P, S.x, YV, tpl[ep], k_first, C);
            }
        }
    }
    if (i == 0 && (I.gh || I.vh))
        endpoint_head(L, Ln, I.E, S.x, g ? I.gh : nullptr, values ? I.vh : nullptr, threadIdx.x, blockDim.x);
}


// MAXT: the launch bound.  eval_g's launches (stride-1 lanes, c->ivg_threads
// = 256) take the 256-thread instantiation: its combine lanes may keep up to
// 512 VGPRs, where the 1024-thread bound (128) made a large model's combine
// spill (Rajagopal 80: 2.9 KB of scratch per lane, ~150 us per eval_g).
template <class D, int MAXT = 1024, bool BASE = false, bool GM = false, bool SLDS = false>
__global__ void __launch_bounds__(MAXT) k_interval(DevModel M, Src S, Lanes Ln, Tasks TK, Layout L,
        Interval I, const TplEntry* __restrict__ tpl, const uint32_t* __restrict__ ctpl,
        const int* __restrict__ ctgen, int nctgen,
        const double* __restrict__ T, const double* __restrict__ H, double* __restrict__ g,
        double* __restrict__ values, int il0) {
    // il0: the first interval of this launch within the shard (a chunked
    // assembly, whose chunks are copied to the host while the next runs)
    const int b = (int)blockIdx.x;
    interval_body<D, GM, BASE, SLDS>(M, S, Ln, TK, L, I, tpl, ctpl, ctgen, nctgen, T, H, g, values,
                                     il0 + (I.xcd ? xcd_interval(b, (int)gridDim.x) : b));
}

// ------------------------------------------------------------------------
// Batched launches (mh_batch): B structurally identical NLPs (same model
// structure, problem layout and template; their own model data, iterate,
// group-result buffers and outputs) evaluated by ONE k_groups and ONE
// k_interval launch, blockIdx.y = the NLP.  The per-NLP constants (device
// model, group-result slabs, path / endpoint tables, grid) live in device
// memory; the per-call pointers travel as kernel arguments.
// ------------------------------------------------------------------------
constexpr int MH_BATCH_MAX = 16;
struct BatchItem {
    DevModel M;
    double* T;
    double* H;
    PathEqs P;
    EndpointEqs E;
    const double* grid;
};
struct BatchPtrs {
    const double* x[MH_BATCH_MAX];
    double* g[MH_BATCH_MAX];
    double* v[MH_BATCH_MAX];
};

// W > 0: at least W waves per SIMD (the register budget shrinks to 512 / W
// VGPRs; more waves hide the transcendental latency of a batch's many tasks)
template <class D, int W>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W > 0 ? W : 1)))
kb_groups(const BatchItem* __restrict__ items, BatchPtrs BP, Lanes Ln, Tasks TK, Layout L) {
    const int b = blockIdx.y;
    const BatchItem& it = items[b];
    const Src S{BP.x[b], it.grid, nullptr, L.G, L.k0, L.XM, L.XL, L.DB};
    groups_body<D>(it.M, S, Ln, TK, it.T, it.H, blockIdx.x);
}

template <class D, bool GM, bool BASE = false>
__global__ void __launch_bounds__(BASE ? 256 : 1024) kb_interval(const BatchItem* __restrict__ items, BatchPtrs BP, Lanes Ln,
        Tasks TK, Layout L, Interval I0, const TplEntry* __restrict__ tpl, const uint32_t* __restrict__ ctpl,
        const int* __restrict__ ctgen, int nctgen, int with_g, int with_v, int nep, int nnz_ep) {
    // XCD-contiguous order over the whole (interval, NLP) grid (xcd_interval
    // on the linear workgroup id, x fastest)
    int b = (int)blockIdx.y, il = (int)blockIdx.x;
    if (I0.xcd) {
        const int nb = (int)gridDim.x;
        const int lin = xcd_interval(b * nb + il, nb * (int)gridDim.y);
        b = lin / nb;
        il = lin - b * nb;
    }
    const BatchItem& it = items[b];
    const Src S{BP.x[b], it.grid, nullptr, L.G, L.k0, L.XM, L.XL, L.DB};
    Interval I = I0;
    I.P = it.P;
    I.E = it.E;
    double* g = with_g ? BP.g[b] : nullptr;
    double* v = with_v ? BP.v[b] : nullptr;
    // the head (endpoint rows) precedes the intervals' rows (make_interval)
    I.gh = I.vh = nullptr;
    if (I.ib == 0 && nep > 0) {
        I.gh = g;
        I.vh = v;
        if (g) g += nep;
        if (v) v += nnz_ep;
    }
    interval_body<D, GM, BASE>(it.M, S, Ln, TK, L, I, tpl, ctpl, ctgen, nctgen, it.T, it.H, g, v, il);
}

// ------------------------------------------------------------------------
// k_role: the Jacobian transcription with one workgroup per (mesh interval,
// grid point of the interval) -- 3 per Hermite-Simpson interval, 2 per
// trapezoidal one.  Each block stages and combines only ITS point's group
// results (all of its lanes), forms that point's finite-difference
// quotients, and writes the Jacobian entries of the interval that read that
// point (the point's columns of every defect row, its residual and path
// rows).  The entries that couple the points -- the t0 / tf columns of the
// defect rows -- and the defect / interpolation rows of g need, of every
// point, only the t0 / tf quotients and the unperturbed outputs: each block
// publishes those (3 x NO doubles) to the interval's exchange slot and
// k_couple, launched next on the stream, writes them.  (Handing them to the
// interval's last-arriving block in the same launch needs an agent-scope
// release per block; on gfx950, whose XCDs' L2s are not coherent, that is an
// L2 write-back per block -- measured 9x slower than the extra launch.)
// Against k_interval: a third of the staging, combine and stores per block,
// three times the blocks (several per CU, overlapping their phases) and no
// idle waves at a 1024-thread barrier; the same arithmetic, bit for bit
// (test_kernel_variants_bit_identical, MOCOHIP_ROLES=0).
// ------------------------------------------------------------------------
struct RowX {   // a point's exchanged row: lanes 0 / 1 (t0 / tf quotients), full_base -> 2
    const lds_double* p;
    int full_base;
    __device__ __forceinline__ double operator[](int r) const { return p[r == full_base ? 2 : r]; }
};
// The interval's grid points as k_role sees them: OWN = true -- only the
// block's own point, all lanes (row ignores k); OWN = false -- every point,
// the exchanged columns [R][NO][XCH_W].
template <bool OWN>
struct YR {
    const lds_double* Y;
    int stride, full_base, NO, kf, q;
    const lds_double* times;
    const lds_double* sxs;
    const lds_double* sxc;
    const lds_double* sxd;
    int NS, NC, NDV;
    __device__ __forceinline__ double xs(int k, int s) const { return sxs[(k - kf) * NS + s]; }
    __device__ __forceinline__ double xc(int k, int j) const { return sxc[(k - kf) * NC + j]; }
    __device__ __forceinline__ double xd(int k, int j) const { return sxd[(k - kf) * NDV + j]; }
    __device__ __forceinline__ double t(int k) const { return times[k - kf]; }
    __device__ __forceinline__ auto row(int k, int o) const {
        if constexpr (OWN) return Y + o * stride;
        else return RowX{Y + ((k - kf) * NO + o) * stride, full_base};
    }
};
// Per role: the (entry, compiled word) lists (own-point LDS offsets), and the
// tail's list for the last role of the last interval.
struct RoleLists {
    const int* __restrict__ e;
    const uint32_t* __restrict__ w;
    int off[4];        // role r: [off[r], off[r + 1])
    int tail0, tail1;  // the tail's entries
    int couple;        // 1: the time role writes the coupling rows / entries; 0: k_couple does
};
// Exchanged columns of a point's rows: t0 quotient, tf quotient, unperturbed
// output ([point][NO][XCH_W]; k_couple's input in global memory, the time
// role's in LDS).
constexpr int XCH_W = 3;
constexpr int NB_MAX = 5;   // lanes of a neighbor point the time role combines (central)
constexpr int ROLE_PF = 16; // assembly entries per thread whose words are prefetched
__device__ __forceinline__ int nb_lanes(const Lanes& Ln) { return Ln.fd == MH_FD_CENTRAL ? 5 : 3; }
// lane of neighbor column j: t0, tf, (central: t0-, tf-), unperturbed
__device__ __forceinline__ int nb_lane(const Lanes& Ln, int j) {
    const int NL = nb_lanes(Ln);
    return j == NL - 1 ? Ln.base : (j < 2 ? j : Ln.ND + (j - 2));
}
// LDS doubles before k_role's constants (sK): own rows, neighbor lanes,
// exchanged columns, times.
__host__ __device__ __forceinline__ int role_kconst(int NO, int S, int R) {
    return NO * S + (R - 1) * NO * NB_MAX + R * NO * XCH_W + CT_CONST;
}

template <class D>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) k_role(DevModel M, Src S, Lanes Ln, Tasks TK, Layout L,
        Interval I, const TplEntry* __restrict__ tpl, RoleLists RL, double* __restrict__ xch,
        const int* __restrict__ ctgen, int nctgen, const double* __restrict__ T, const double* __restrict__ H,
        double* __restrict__ g, double* __restrict__ values) {
#pragma clang fp contract(off)
    extern __shared__ double smem[];
    const bool hs = I.scheme == MH_HERMITE_SIMPSON;
    const int R = hs ? 3 : 2, TR = hs ? 1 : 0;
    const int il = blockIdx.x / R, role = blockIdx.x - il * R;
    const int i = I.ib + il;
    int k_first, k_last;
    interval_span(I, i, k_first, k_last);
    const int S_ = Ln.stride, NO = D::NO, NL = nb_lanes(Ln), B = blockDim.x;
    const bool tr = RL.couple && role == TR;   // this block writes the coupling rows / entries
    const int nt = TK.tdoubles, nh = TK.nmass * D::NST;
    double* sY = smem;                          // own point [NO][S]
    double* sYn = sY + NO * S_;                 // neighbor lanes [R - 1][NO][NB_MAX] (time role)
    double* sYx = sYn + (R - 1) * NO * NB_MAX;  // exchanged columns [R][NO][XCH_W]
    double* sTimes = sYx + R * NO * XCH_W;      // [R] (+ pad)
    double* sK = sTimes + CT_CONST;             // 0.0, 1.0
    double* sT = sK + 2;                        // own [nt]
    double* sH = sT + nt;                       // own [nh]
    double* sXs = sH + nh;                      // [R][NS], [R][NC], [R][NDV]
    double* sXc = sXs + R * L.NS;
    double* sXd = sXc + R * L.NC;
    const int kown = k_first + role;
    const int klo = kown - S.k0;
    if (nt > 0) stage_lds<8>(sT, T + (long)klo * nt, nt);
    if (nh > 0) stage_lds<4>(sH, H + (long)klo * nh, nh);
    stage_lds<1>(sXs, S.x + 2 + (long)k_first * L.NS, R * L.NS);
    if (L.NC > 0) stage_lds<1>(sXc, S.x + 2 + (long)L.NS * L.G + (long)k_first * L.NC, R * L.NC);
    if (L.NDV > 0)
        stage_lds<1>(sXd, S.x + L.DB + (long)k_first * L.NDV, R * L.NDV);
    if (threadIdx.x < 2) sK[threadIdx.x] = threadIdx.x ? 1.0 : 0.0;
    const double t0 = S.x[0], tf = S.x[1];
    if (threadIdx.x < R) {   // every block's formulas use the interval's base times
        int pi;
        double st;
        sTimes[threadIdx.x] = lane_time(Ln, S.grid[k_first + threadIdx.x], t0, tf, Ln.base, pi, st);
    }
    __syncthreads();
    if (I.dbg_stop == 1) return;
    // own lanes: combine the point's group results from LDS; the time role
    // also the neighbor points' t0 / tf / unperturbed lanes, from theirs in
    // global memory (few lanes, on threads of their own)
    const int nnb = tr ? (R - 1) * NL : 0;
    for (int w = threadIdx.x; w < S_ + nnb; w += B) {
        int p = role, r = w;
        lds_double* Yp;
        int ys;
        if (w < S_) {
            Yp = lds(sY + r);
            ys = S_;
        } else {
            const int q = (w - S_) / NL, j = (w - S_) - q * NL;
            p = q < TR ? q : q + 1;
            r = nb_lane(Ln, j);
            Yp = lds(sYn + q * NO * NB_MAX + j);
            ys = NB_MAX;
        }
        LaneInL<D> in{lds(sXs + p * L.NS), lds(sXc + p * L.NC), lds(sXd + p * L.NDV), -1, 0.0};
        const double t = lane_time(Ln, S.grid[k_first + p], t0, tf, r, in.pi, in.step);
        double out[D::NO];
        if (w < S_) {
            const TaskLoadLds<D> TL{lds(sT), lds(sH), TK.jd, r};
            D::combine(M, t, in, TL, out);
        } else {
            const int kl = k_first + p - S.k0;
            const TaskLoadGlobal<D> TG{T + (long)kl * nt, H + (long)kl * nh, TK.jd, r};
            D::combine(M, t, in, TG, out);
        }
#pragma unroll
        for (int o = 0; o < D::NO; ++o) Yp[o * ys] = out[o];
    }
    // the assembly's compiled words: prefetched now, consumed after the quotients
    const int ra = role == 0 ? RL.off[0] : role == 1 ? RL.off[1] : RL.off[2];
    const int rb = role == 0 ? RL.off[1] : role == 1 ? RL.off[2] : RL.off[3];
    uint32_t pw[ROLE_PF];
    int pe[ROLE_PF];
    if (values) {
#pragma unroll
        for (int u = 0; u < ROLE_PF; ++u) {
            const int e = ra + threadIdx.x + u * B;
            pw[u] = e < rb ? RL.w[e] : 0u;
            pe[u] = e < rb ? RL.e[e] : -1;
        }
    }
    __syncthreads();
    if (I.dbg_stop == 2) return;
    // finite-difference quotients in place (own: every direction; neighbors:
    // t0 / tf), then the exchanged columns
    {
        const double h = Ln.h, h2 = 2.0 * Ln.h;
        const int nq = NO * Ln.ND;
        for (int w = threadIdx.x; w < nq; w += B) {
            const int o = w / Ln.ND, d = w - o * Ln.ND;
            lds_double* y = lds(sY + o * S_);
            double q;
            if (Ln.fd == MH_FD_CENTRAL) q = (y[d] - y[Ln.ND + d]) / h2;
            else if (Ln.fd == MH_FD_FORWARD) q = (y[d] - y[Ln.base]) / h;
            else q = (y[Ln.base] - y[d]) / h;
            y[d] = q;
        }
        for (int w = threadIdx.x; w < (tr ? (R - 1) * NO * 2 : 0); w += B) {
            const int qo = w >> 1, d = w & 1;
            lds_double* y = lds(sYn + qo * NB_MAX);
            double q;
            if (Ln.fd == MH_FD_CENTRAL) q = (y[d] - y[2 + d]) / h2;
            else if (Ln.fd == MH_FD_FORWARD) q = (y[d] - y[NL - 1]) / h;
            else q = (y[NL - 1] - y[d]) / h;
            y[d] = q;
        }
        __syncthreads();
    }
    if (RL.couple) {
        if (tr)
            for (int w = threadIdx.x; w < R * NO * XCH_W; w += B) {
                const int p = w / (NO * XCH_W), rem = w - p * NO * XCH_W;
                const int o = rem / XCH_W, j = rem - o * XCH_W;
                if (p == role) {
                    sYx[w] = sY[o * S_ + (j < 2 ? j : Ln.base)];
                } else {
                    const int q = p < role ? p : p - 1;
                    sYx[w] = sYn[(q * NO + o) * NB_MAX + (j < 2 ? j : NL - 1)];
                }
            }
    } else {
        // publish this point's columns for k_couple
        double* xo = xch + ((long)il * R + role) * NO * XCH_W;
        for (int w = threadIdx.x; w < NO * XCH_W; w += B) {
            const int o = w / XCH_W, j = w - o * XCH_W;
            xo[w] = sY[o * S_ + (j < 2 ? j : Ln.base)];
        }
    }
    if (I.dbg_stop == 3) return;
    const YR<true> YV{lds(sY), S_, Ln.base, NO, k_first, 1, lds(sTimes), lds(sXs), lds(sXc), lds(sXd),
                      L.NS, L.NC, L.NDV};
    const int npres = hs ? 2 : 1;
    const int npc = I.P.npc;
    double* gi = g ? g + (long)il * I.rpi : nullptr;
    // this point's rows of g: path rows (first point), its residual rows, the
    // tail (last point of the last interval)
    if (g)
        for (int r = threadIdx.x; r < I.rows(i); r += B) {
            int owner;
            if (r >= I.rpi) owner = R - 1;
            else if (r < npc) owner = 0;
            else if (r < npc + npres * I.nres) owner = (r - npc) / I.nres;
            else owner = -1;
            if (owner == role) gi[r] = defect_row(L, I, Ln, S.x, YV, i, r);
        }
    if (I.dbg_stop == 4) return;
    const IvC C = iv_const(YV.t(k_last) - YV.t(k_first), S.grid[k_last] - S.grid[k_first]);
    double* vi = values ? values + (long)il * I.nnz_int : nullptr;
    if (values) {
        const lds_double* q0 = lds(sY);
        const double c1 = -C.h8, c2 = C.h8, c3 = -C.h6, c4 = -C.h6 * 4.0, c5 = -C.hh;
        auto value = [&](uint32_t wu, double q) {
            const uint32_t ks = (wu >> 20) & 7, bs = (wu >> 23) & 7;
            const double coef = ks == 1 ? c1 : ks == 2 ? c2 : ks == 3 ? c3 : ks == 4 ? c4 : ks == 5 ? c5 : 0.0;
            const double base = bs == 1 ? -0.5 : bs == 2 ? 1.0 : bs == 3 ? -1.0 : 0.0;
            return (wu & CT_RAW) ? q : base + coef * q;
        };
#pragma unroll
        for (int u = 0; u < ROLE_PF; ++u)
            if (pe[u] >= 0) vi[pe[u]] = value(pw[u], q0[pw[u] & CT_OFF]);
        for (int e = ra + ROLE_PF * B + threadIdx.x; e < rb; e += B) {
            const uint32_t wu = RL.w[e];
            vi[RL.e[e]] = value(wu, q0[wu & CT_OFF]);
        }
        if (i == I.N - 1 && role == R - 1)
            for (int e = RL.tail0 + threadIdx.x; e < RL.tail1; e += B) {
                const uint32_t wu = RL.w[e];
                vi[RL.e[e]] = value(wu, q0[wu & CT_OFF]);
            }
        // path-constraint entries at the mesh point (first point) and, in the
        // tail, at the final mesh point (last point of the last interval)
        if (I.npe > 0 && (role == 0 || (role == R - 1 && i == I.N - 1))) {
            const int npe = I.npe;
            for (int w = threadIdx.x; w < npe; w += B) {
                const int ep = role == 0 ? w : I.nnz_int + w;
                vi[ep] = jac_entry<true>(L, Ln, I.P, S.x, YV, tpl[ep], k_first, C);
            }
        }
    }
    if (i == 0 && role == 0 && (I.gh || I.vh))
        endpoint_head(L, Ln, I.E, S.x, g ? I.gh : nullptr, values ? I.vh : nullptr, threadIdx.x, blockDim.x);
    if (tr) {
        // the coupling rows of g and t0 / tf entries of the defect rows
        __syncthreads();
        const YR<false> YA{lds(sYx), XCH_W, Ln.base, NO, k_first, 1, lds(sTimes), lds(sXs), lds(sXc), lds(sXd),
                           L.NS, L.NC, L.NDV};
        if (g)
            for (int r = npc + npres * I.nres + threadIdx.x; r < I.rpi; r += B)
                gi[r] = defect_row(L, I, Ln, S.x, YA, i, r);
        if (values)
            for (int j = threadIdx.x; j < nctgen; j += B) {
                const int eg = ctgen[j];
                vi[eg] = jac_entry<false>(L, Ln, I.P, S.x, YA, tpl[eg], k_first, C);
            }
    }
}

// The coupling rows of g (defects, interpolation) and the t0 / tf entries of
// the defect rows, per mesh interval from k_role's exchange.
template <class D>
__global__ void __launch_bounds__(256) k_couple(Src S, Lanes Ln, Layout L, Interval I,
        const TplEntry* __restrict__ tpl, const int* __restrict__ ctgen, int nctgen,
        const double* __restrict__ xch, double* __restrict__ g, double* __restrict__ values) {
#pragma clang fp contract(off)
    extern __shared__ double smem[];
    const bool hs = I.scheme == MH_HERMITE_SIMPSON;
    const int R = hs ? 3 : 2, NO = D::NO, B = blockDim.x;
    const int il = blockIdx.x, i = I.ib + il;
    int k_first, k_last;
    interval_span(I, i, k_first, k_last);
    double* sYx = smem;                         // [R][NO][XCH_W]
    double* sTimes = sYx + R * NO * XCH_W;      // [R]
    double* sXs = sTimes + 4;                   // [R][NS], [R][NC], [R][NDV]
    double* sXc = sXs + R * L.NS;
    double* sXd = sXc + R * L.NC;
    stage_lds<1>(sYx, xch + (long)il * R * NO * XCH_W, R * NO * XCH_W);
    stage_lds<1>(sXs, S.x + 2 + (long)k_first * L.NS, R * L.NS);
    if (L.NC > 0) stage_lds<1>(sXc, S.x + 2 + (long)L.NS * L.G + (long)k_first * L.NC, R * L.NC);
    if (L.NDV > 0)
        stage_lds<1>(sXd, S.x + L.DB + (long)k_first * L.NDV, R * L.NDV);
    if (threadIdx.x < R) {
        int pi;
        double st;
        sTimes[threadIdx.x] = lane_time(Ln, S.grid[k_first + threadIdx.x], S.x[0], S.x[1], Ln.base, pi, st);
    }
    __syncthreads();
    const YR<false> YA{lds(sYx), XCH_W, Ln.base, NO, k_first, 1, lds(sTimes), lds(sXs), lds(sXc), lds(sXd),
                       L.NS, L.NC, L.NDV};
    const int npres = hs ? 2 : 1;
    if (g) {
        double* gi = g + (long)il * I.rpi;
        for (int r = I.P.npc + npres * I.nres + threadIdx.x; r < I.rpi; r += B)
            gi[r] = defect_row(L, I, Ln, S.x, YA, i, r);
    }
    if (values) {
        const IvC C = iv_const(YA.t(k_last) - YA.t(k_first), S.grid[k_last] - S.grid[k_first]);
        double* vi = values + (long)il * I.nnz_int;
        for (int j = threadIdx.x; j < nctgen; j += B) {
            const int eg = ctgen[j];
            vi[eg] = jac_entry<false>(L, Ln, I.P, S.x, YA, tpl[eg], k_first, C);
        }
    }
}

// ---- objective -------------------------------------------------------------
__device__ __forceinline__ void gather_inputs(const double* __restrict__ x, const Layout& L,
        int k, double* in, int NI) {
    const double* xs = x + 2 + (long)k * L.NS;
    const double* xc = x + 2 + (long)L.NS * L.G + (long)k * L.NC;
    const double* xd = x + L.DB + (long)k * L.NDV;
    const double* xm = x + L.XM + (long)k * L.NM;
    for (int s = 0; s < L.NS; ++s) in[s] = xs[s];
    for (int j = 0; j < L.NC; ++j) in[L.NS + j] = xc[j];
    for (int j = 0; j < L.NDV; ++j) in[L.NS + L.NC + j] = xd[j];
    for (int j = 0; j < L.NM; ++j) in[L.NS + L.NC + L.NDV + j] = xm[j];
    for (int j = L.NS + L.NC + L.NDV + L.NM; j < NI; ++j) in[j] = 0.0;   // slacks: no goal reads them
}

// Goals with an integral (quadrature of an integrand): all but the endpoint
// costs (final time, final marker).
__host__ __device__ __forceinline__ bool goal_integral(int kind) {
    return kind != MH_GOAL_FINAL_TIME && kind != MH_GOAL_MARKER_FINAL;
}
constexpr int MH_MARKER_MAX_Q = 64;   // coordinates a marker goal's kernel holds per lane

struct GoalSet {
    int ngoals;
    int nc, nacc;   // controls; accelerations before the auxiliary derivatives
    int ndv;        // derivative variables (the multipliers follow them)
    const mh_goal* goals;
    const int* gidx;
    const int* gcol;
    const double* gw;
};

__device__ double goal_integrand(const DevModel& M, const GoalSet& GS, int g, double t,
        const double* st, const double* ct) {
    const mh_goal G = GS.goals[g];
    double L = 0.0;
    for (int k = G.term_begin; k < G.term_begin + G.term_count; ++k) {
        const int idx = GS.gidx[k];
        const double w = GS.gw[k];
        if (G.kind == MH_GOAL_CONTROL) {
            const double v = ct[idx];
            L += w * (G.exponent == 2 ? v * v : pow(fabs(v), (double)G.exponent));
        } else if (G.kind == MH_GOAL_STATE_TRACKING) {
            const double d = st[idx] - table_eval(M, G.table, GS.gcol[k], t);
            L += w * (d * d);
        } else if (G.kind == MH_GOAL_SUM_SQUARED_STATE) {
            const double v = st[idx];
            L += w * (v * v);
        } else if (G.kind == MH_GOAL_AUX_DERIVATIVES) {
            const double v = ct[GS.nc + GS.nacc + idx];   // derivatives follow the controls
            L += w * (v * v);
        } else if (G.kind == MH_GOAL_LAGRANGE_MULTIPLIERS) {
            const double v = ct[GS.nc + GS.ndv + idx];    // multipliers follow the derivatives
            L += w * (v * v);
        }
    }
    return L;
}

// Per-point quad-weighted integrands: C[k*ngoals + g] = quad_k * L_g(k).
template <class Z>
__global__ void __launch_bounds__(64) k_integrand(DevModel M, Layout L, GoalSet GS,
        const double* __restrict__ x, const double* __restrict__ grid,
        const double* __restrict__ quad, double* __restrict__ C) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= L.G) return;
    const double t = (x[1] - x[0]) * grid[k] + x[0];
    double in[Z::MI];
    gather_inputs(x, L, k, in, L.NI);
    for (int g = 0; g < GS.ngoals; ++g) {
        const bool integral = goal_integral(GS.goals[g].kind);
        C[(long)k * GS.ngoals + g] =
                integral ? quad[k] * goal_integrand(M, GS, g, t, in, in + L.NS) : 0.0;
    }
}

// Gradient of the integral terms: one lane per (grid point, direction).
template <class Z>
__global__ void __launch_bounds__(64) k_grad(DevModel M, Layout L, GoalSet GS, int fd, double h,
        const double* __restrict__ x, const double* __restrict__ grid,
        const double* __restrict__ quad, double* __restrict__ grad, double* __restrict__ tpart) {
    const int ND = L.NI - L.NSL + 2;   // the goal callback's inputs: no slacks
    const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (long)L.G * ND) return;
    const int k = (int)(tid / ND), d = (int)(tid % ND);
    const double g = grid[k];
    const double dur = x[1] - x[0];
    const double t = dur * g + x[0];
    double in[Z::MI];
    gather_inputs(x, L, k, in, L.NI);
    double acc = 0.0;
    for (int gi = 0; gi < GS.ngoals; ++gi) {
        const mh_goal G = GS.goals[gi];
        if (!goal_integral(G.kind)) continue;
        const double seed = d == 0 ? 1.0 - g : (d == 1 ? g : 1.0);
        double lp = 0.0, lm = 0.0, l0 = 0.0;
        if (fd != MH_FD_CENTRAL) l0 = goal_integrand(M, GS, gi, t, in, in + L.NS);
        if (fd != MH_FD_BACKWARD) {
            if (d < 2) lp = goal_integrand(M, GS, gi, t + h * seed, in, in + L.NS);
            else {
                const double s = in[d - 2];
                in[d - 2] = s + h;
                lp = goal_integrand(M, GS, gi, t, in, in + L.NS);
                in[d - 2] = s;
            }
        }
        if (fd != MH_FD_FORWARD) {
            if (d < 2) lm = goal_integrand(M, GS, gi, t - h * seed, in, in + L.NS);
            else {
                const double s = in[d - 2];
                in[d - 2] = s - h;
                lm = goal_integrand(M, GS, gi, t, in, in + L.NS);
                in[d - 2] = s;
            }
        }
        double dL = fd == MH_FD_CENTRAL ? (lp - lm) / (2.0 * h)
                  : (fd == MH_FD_FORWARD ? (lp - l0) / h : (l0 - lm) / h);
        if (G.kind == MH_GOAL_LAGRANGE_MULTIPLIERS) {
            // exact, like the reference's AD of this MX term: w 2 lambda
            const int j = d - 2 - (L.NS + L.NC + L.NDV);
            dL = (d >= 2 && j >= 0 && j < L.NM) ? GS.gw[G.term_begin + j] * (2.0 * in[d - 2]) : 0.0;
        }
        acc += G.weight * dur * quad[k] * dL;
    }
    if (d < 2) tpart[(long)k * 2 + d] = acc;
    else if (d - 2 < L.NS) grad[2 + (long)k * L.NS + (d - 2)] = acc;
    else if (d - 2 < L.NS + L.NC) grad[2 + (long)L.NS * L.G + (long)k * L.NC + (d - 2 - L.NS)] = acc;
    else if (d - 2 < L.NS + L.NC + L.NDV) grad[L.DB + (long)k * L.NDV + (d - 2 - L.NS - L.NC)] = acc;
    else grad[L.XM + (long)k * L.NM + (d - 2 - L.NS - L.NC - L.NDV)] = acc;
}


// DAE probe: one lane per input row [time, states, controls].
template <class D>
__global__ void __launch_bounds__(64) k_dae_probe(DevModel M, Layout L, int npts,
        const double* __restrict__ in, double* __restrict__ outp) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npts) return;
    const double* r = in + (long)p * (1 + L.NI);
    double v[D::MI];
    double out[D::MO];
#pragma unroll
    for (int i = 0; i < D::MI; ++i) v[i] = i < L.NI ? r[1 + i] : 0.0;
    D::eval(M, r[0], v, out);
#pragma unroll
    for (int o = 0; o < D::MO; ++o)
        if (o < L.NO) outp[(long)p * L.NO + o] = out[o];
}

// ------------------------------------------------------------------------
// Host-side structures shared by the translation units.
// ------------------------------------------------------------------------
// Static description of a task-decomposed generated model (codegen.py).
struct TaskInfo {
    int ng, nst, nf, rw, nheavy;
    const int* group_nf;
    const unsigned long long* reads;   // [ng][rw] bit i = group reads point input i
    const unsigned char* time;         // [ng] group reads the time
    const double* gflops;              // [ng] FP64 ops per group evaluation
    double combine_flops;
};

// Task tables for one lane configuration (host copy + device view).
struct TaskSet {
    Tasks dev{};
    int nblocks = 0;
    int nheavy = -1;        // leading blocks of the heavy groups (< NHEAVY); -1: not contiguous
    double flops = 0.0;     // FP64 ops per launch (groups + combine)
    double ntasks = 0.0;    // group evaluations per launch
    std::vector<int> dlen, off, roles, jd, blk;
    size_t t_doubles = 0, h_doubles = 0;
};
struct Backend;
struct GenEntry;

struct mh_ctx {
    // problem
    int NQ = 0, NZ = 0, NS = 0, NC = 0, NO = 0, NI = 0;
    int scheme = 0, N = 0, G = 0, interp = 0, rpi = 0, nnz_int = 0;
    int NDV = 0, nnz_tail = 0;     // implicit: accelerations per point, tail nonzeros
    int npc = 0, ntail = 0;        // path equations per mesh point; tail rows (npc + residuals)
    int NACC = 0, NAR = 0;         // accelerations (implicit multibody), implicit aux residuals per point
    int NMB = 0;                   // multibody residual rows per point (implicit / prescribed: NQ)
    int TQ = 0;                    // coordinates among the NLP states (0: prescribed kinematics)
    int SO = 0;                    // callback output of state s's derivative: s + SO
    int presc = 0, kin_table = -1;
    std::vector<int> kin_col;
    // kinematic constraints (mh_constraint): couplers, multipliers per grid
    // point, kinematic rows per mesh point, slacks per mesh interval, the
    // callback outputs of the errors / velocity correction, bounds
    int NKC = 0, NM = 0, NK = 0, NSL = 0, OKC = 0, OQC = 0, enforce = 1;
    std::vector<mh_constraint> kcs;
    // muscle wrapping: per muscle the first PathWrap entry and their count
    std::vector<int> mus_pw_begin, mus_pw_count;
    double mult_lo = -1000.0, mult_hi = 1000.0, kc_lo = 0.0, kc_hi = 0.0, vc_lo = -0.1, vc_hi = 0.1;
    std::vector<int> mus_ider;     // muscle -> aux derivative index after the controls (-1)
    double aux_lo = -1000.0, aux_hi = 1000.0;
    int npe = 0;                   // path-constraint template entries per mesh point
    std::vector<uint8_t> sp, sp_pc;  // detected sparsity [output][time, inputs] (empty: dense)
    std::vector<mh_path_equation> pc;
    PathEqs P{};
    // goals as uploaded: the problem's, then the internal multiplier term
    std::vector<mh_goal> goals;
    std::vector<int32_t> gidx, gcol;
    std::vector<double> gw;
    // endpoint constraints: the head of g (rows 0..nep) and of the Jacobian
    // (entries 0..nnz_ep), owned by the shard with interval 0
    int nep = 0, nnz_ep = 0;
    // MocoParameters (mh_problem.parameter_*): NPAR NLP variables at x[XP..];
    // the device model's parameterized arrays (bodies, actuators, muscles,
    // springs) exist in NCOPY copies: copy 0 with the iterate's parameter
    // values, copy 1 + p (and 1 + NPAR + p for central differences) with
    // parameter p moved by the finite-difference step; k_apply_params writes
    // them from the pristine arrays before every evaluation.  Each parameter
    // direction's lanes run as their own k_eval launch over its copy (Mp).
    int NPAR = 0, NCOPY = 1;
    int64_t XP = 0;
    std::vector<mh_bounds> par_bounds;
    std::vector<mh_parameter_target> par_targets;
    mh_parameter_target* d_par_targets = nullptr;
    std::vector<DevModel> Mp;          // [NCOPY]: Mp[0] = M
    DevModel M0{};                     // the pristine model (mh_eval_dae)
    int* d_lane_main = nullptr;        // Jacobian lanes that are not parameter lanes
    int n_lane_main = 0;
    int* d_par_lanes = nullptr;        // the lane of copy cp (cp >= 1) at [cp - 1]
    int nsprings = 0;
    std::vector<mh_endpoint_equation> ep;
    std::vector<TplEntry> eptpl;       // row = equation, dir = endpoint input index
    std::vector<uint8_t> sp_ep;        // detected [equation][2 (1 + NI)] (empty: dense)
    EndpointEqs E{};
    double acc_lo = -1000.0, acc_hi = 1000.0;
    int ib = 0, ie = 0, k0 = 0, nk = 0;
    int fd = 0;
    double h = 1e-8;
    int size_class = 0;
    const struct Backend* be = nullptr;
    const struct GenEntry* gen = nullptr;   // the generated back end's entry (match / fill), if any
    Lanes lanes_jac{}, lanes_g{};
    uint64_t model_hash = 0;
    int64_t n = 0, m = 0, nnz = 0;
    std::vector<double> grid, quad;
    std::vector<TplEntry> tpl;
    std::vector<int> tpl_col_pt;   // template column: point (0..2) or -1 for t0/tf
    std::vector<int64_t> tpl_col_off;  // template column offset within point block
    std::vector<mh_variable_info> sinfo, cinfo;
    mh_bounds t_init{}, t_final{};
    int ngoals = 0;
    // device
    int device = 0;
    hipStream_t stream = nullptr;      // the stream all work is ordered on
    hipStream_t own_stream = nullptr;  // the context's own (mh_set_stream(NULL))
    bool async = false;                // *_device entries return once enqueued
    int iv_dbg_stop = 0;               // diagnostic: k_interval stops after phase n
    int iv_pf = 1;                     // MOCOHIP_IV_PF=0: no assembly-word prefetch (A/B)
    int iv_dbase = 0;                  // k_transcribe derives base-lane offsets (MOCOHIP_DBASE=0: the table)
    std::vector<int> exc_xs;           // excitation lanes of k_exc_fill: [lane, slot, output] per lane
    bool exc_redirected = false;       // the template reads their copied outputs at the base lane
    bool exc_full = false;             // mh_debug_jacobian_lanes: fill every output
    uint32_t iv_smagic = 0, iv_sstride = 1, iv_sbase = 0;
    int iv_qdiv = 0;                   // k_transcribe: quotients by div_rn (MOCOHIP_QDIV=1; no faster)
    int iv_xcd = 1;                    // XCD-contiguous interval order (MOCOHIP_IV_XCD=0: off, A/B)
    int iv_qfuse = 1;                  // MOCOHIP_IV_QFUSE=0: in-place quotient pass (A/B)
    hipEvent_t ev[5] = {};         // stage boundaries (+ ev[4] after k_groups)
    // host entries: the Jacobian values go to the host in interval chunks on
    // copy_stream while the next chunk's k_interval runs (MOCOHIP_D2H_CHUNKS)
    static constexpr int kMaxD2hChunks = 16;
    // default 1 (one copy after the call): measured on MI355X, every chunked
    // variant was slower (gait N=200, page-locked buffers: 2,561 calls/s with
    // one copy, 2,244 / 2,097 / 1,942 with 2 / 4 / 8 chunks;
    // profiles/r03_h/d2h.txt) -- the PCIe transfer, not the assembly, is
    // the call, and each extra copy + cross-stream event costs more than the
    // ~18 us of k_interval it hides
    int d2h_chunks = 1;
    hipStream_t copy_stream = nullptr;
    hipEvent_t ev_chunk[kMaxD2hChunks] = {};
    hipEvent_t ev_copied = nullptr;
    char* dmem = nullptr;
    DevModel M{};
    GoalSet GS{};
    // d_quadp: the quadrature of this shard's own mesh intervals only (its
    // objective partial: the partials of the shards sum to the objective)
    double* d_quadp = nullptr;
    std::vector<double> quadp;
    double *d_x = nullptr, *d_grid = nullptr, *d_quad = nullptr, *d_times = nullptr, *d_Y = nullptr,
           *d_Yg = nullptr, *d_g = nullptr, *d_vals = nullptr, *d_C = nullptr, *d_grad = nullptr,
           *d_tpart = nullptr, *d_f = nullptr;
    TplEntry* d_tpl = nullptr;
    // generic interpreter: per Jacobian lane, the muscle whose excitation it
    // perturbs when k_exc_lanes stands in for the evaluation, else -1; null
    // when no lane qualifies (or MOCOHIP_EXC_LANES=0)
    int* d_exc = nullptr;
    int* d_lane_map = nullptr;     // the other lanes, in order (k_eval's lane map)
    int n_exc_lanes = 0;
    // generated back ends: per excitation lane (role, slot, output) that
    // k_exc_fill writes instead of k_combine_global, and the lanes left to
    // combine (null / 0: none qualifies, or MOCOHIP_EXC_LANES=0)
    int* d_exc_slot = nullptr;
    int* d_cmb_map = nullptr;
    int n_exc_gen = 0;
    int g_block = 4;               // generic interpreter, eval_g: k_eval workgroup size (A/B: profiles/r02_l)
    bool g_lds = false;            // generic interpreter, eval_g: workspace in LDS (k_eval_lds)
    int g_lds_guard = 0;           // k_eval_lds guard band per slot side, doubles (MOCOHIP_G_LDS_GUARD)
    int* d_lds_status = nullptr;   // set by k_eval_lds when a guard band changed
    int groups_split = -1;         // task back ends: heavy / light group kernels (-1: by occupancy)
    int combine_mode = -1;         // split path combine: 0 LDS-staged, 1 global memory (-1: by spills)
    uint32_t* d_ctpl = nullptr;    // compiled template of the Jacobian lanes (k_interval)
    std::vector<uint32_t> ctpl;
    int* d_ctgen = nullptr;        // the entries it leaves to jac_entry (t0 / tf of defect rows)
    std::vector<int> ctgen;
    // k_role: per role (grid point of the interval) the entries it writes
    // and their words compiled against the role's own-point LDS layout
    std::vector<int> rl_e;
    std::vector<uint32_t> rl_w;
    int rl_off[4] = {0, 0, 0, 0}, rl_tail[2] = {0, 0};
    int* d_rl_e = nullptr;
    uint32_t* d_rl_w = nullptr;
    double* d_xch = nullptr;       // k_role -> k_couple exchange [interval][point][NO][3]
    double* d_ep = nullptr;        // endpoint-cost values per goal (k_marker_final)
    bool has_marker = false;
    bool use_roles = false;        // MOCOHIP_ROLES=1: k_role (+ k_couple) for the Jacobian lanes
    int role_threads = 256;        // k_role workgroup size (MOCOHIP_ROLE_THREADS: 64..512)
    int iv_threads = 1024;         // k_interval workgroup size, Jacobian lanes (MOCOHIP_IV_THREADS: 256..1024)
    int ivg_threads = 256;         // k_interval workgroup size, eval_g lanes (MOCOHIP_IVG_THREADS: 64..1024)
    int csplit = 0;                // large models' combine as k_combine_split (opt-in, MOCOHIP_CSPLIT=1)
    // eval_g's k_interval reads group results at compile-time base slots
    // (MOCOHIP_IVG_BASE, default 1), from global memory (MOCOHIP_IVG_GM;
    // -1: by the grid point's result count, kIvgGmMaxDoubles)
    int ivg_base = 1;
    int ivg_gm = -1;
    int iv_slots_lds = 0;          // k_interval stages the slot table in LDS (MOCOHIP_IV_SLOTS_LDS=1)
    bool role_couple = true;       // coupling in k_role's time role (MOCOHIP_ROLE_COUPLE=0: k_couple)
    bool use_ctpl = true;          // MOCOHIP_CTPL=0: k_interval assembles through jac_entry
    float timings[4] = {0, 0, 0, 0};
    // task-decomposed back ends
    TaskSet ts_jac, ts_g, ts_probe;
    // eval_g's task records as kernel arguments (k_groups_kr; MOCOHIP_GROUPS_KR)
    bool krec_ok = false;
    KRecs krec_g{};
    double *d_T = nullptr, *d_H = nullptr;     // group results of the Jacobian lanes
    double *d_Tg = nullptr, *d_Hg = nullptr;   // of the eval_g lanes (their own: the two
                                               // evaluations may run concurrently)
    // IPOPT's new_x on the device entries (mh_tnlp_eval_*_device): ev_x is
    // recorded on the caller's stream where an evaluation at a new iterate
    // x_last starts; an eval_jac_g with new_x = 0 at the same x then runs on
    // aux_stream from that point -- concurrently with what the caller queued
    // since (its eval_g) -- and the caller's stream waits for it (ev_aux)
    hipStream_t aux_stream = nullptr;
    hipEvent_t ev_x = nullptr, ev_aux = nullptr;
    const double* x_last = nullptr;
    bool overlap = false;          // MOCOHIP_OVERLAP=1 (measured slower: DESIGN.md section 4)
    char* probe_mem = nullptr;     // tables + T/H of the last mh_eval_dae size
    double *d_pT = nullptr, *d_pH = nullptr;
    int probe_np = -1;
    // captured launch sequences, keyed by (kind, x, out pointers)
    struct GraphEntry { int kind; const void *x, *a, *b; hipGraphExec_t exec; };
    std::vector<GraphEntry> graphs;
    bool use_graphs = false;
    bool spin_wait = false;
    // per lane configuration (0: eval_g lanes, 1: Jacobian lanes): combine
    // and transcription fused in k_interval (LDS-resident raw outputs)
    bool use_interval[2] = {false, false};
    int nsimd = 1024;              // SIMDs of the device (4 per CU)
    bool asm_grid_stride = false;  // k_transcribe_gs (MOCOHIP_ASM=gs) instead of k_transcribe
    bool asm_ctpl = true;          // k_transcribe on the compiled template (MOCOHIP_ASM_CTPL=0: jac_entry)
    int asm_chunk_ct = 8192;       // ... its nonzeros per workgroup (MOCOHIP_ASM_CHUNK)
    bool quot = false;             // k_combine writes FD quotients (MOCOHIP_QUOT=1)
    const Backend* be_lane = nullptr;   // the generated model's one-lane back end (if any)
    bool g_lane = false;           // eval_g alone through be_lane + the split transcription
    int yq[2] = {0, 0};            // per lane configuration: Y of the last evaluation holds quotients
    bool timing = false;           // stage events for mh_last_timings (mh_set_timing)
    bool groups_timed = false;     // the last evaluation recorded ev[4]
    // MH_JACOBIAN_GLOBAL_SEEDS (tropter): column coloring, per seed its
    // columns and its (nonzero, row) pairs, perturbed iterates and g's
    int jac_seeds = 0, nseeds = 0;
    int coloring_order = MH_COLORING_SMALLEST_LAST;   // mh_options.coloring_order
    std::vector<int32_t> seed_color;           // [n]
    std::vector<int32_t> seed_col_off, seed_cols, seed_ent_off, seed_ents, seed_rows;
    int32_t *d_seed_cols = nullptr, *d_seed_ents = nullptr, *d_seed_rows = nullptr;
    double *d_xp = nullptr, *d_xm = nullptr, *d_gp = nullptr, *d_gm = nullptr;
};

// The per-call layout view of the context (grid points [k0, k0 + nk)).
inline Layout make_layout(const mh_ctx* c, int k0, int nk) {
    Layout L{c->NS, c->NC, c->TQ, c->NO, c->NI, c->G, k0, nk, c->NDV, c->NACC, c->SO,
             c->NM, c->NSL, c->OQC, 0, 0, 0};
    L.XM = 2 + (long)(c->NS + c->NC) * c->G;
    L.XL = L.XM + (long)c->NM * c->G;
    L.DB = L.XL + (long)c->NSL * c->N;
    return L;
}

// The transcription's per-call view of the context.  g / v (this shard's
// rows / nonzeros) are advanced past the head, which the first interval's
// block writes through I.gh / I.vh when this shard owns it.
inline Interval make_interval(const mh_ctx* c, double*& g, double*& v) {
    Interval I{c->scheme, c->interp, c->ib, c->rpi, c->nnz_int, c->NMB + c->NAR, c->NMB, c->NQ + c->NZ,
               c->N, c->nnz_tail, c->ntail, c->npe, c->NK, c->OKC, c->P, c->E, nullptr, nullptr, c->iv_dbg_stop, c->iv_pf, c->iv_qfuse,
               c->iv_xcd, c->iv_dbase, c->iv_smagic, c->iv_sstride, c->iv_sbase,
               c->iv_qdiv};
    if (c->ib == 0 && c->nep > 0) {
        I.gh = g;
        I.vh = v;
        if (g) g += c->nep;
        if (v) v += c->nnz_ep;
    }
    return I;
}

// Lane inputs from the iterate x (device pointer).
inline Src src_of(const mh_ctx* c, const double* x) {
    const Layout L = make_layout(c, c->k0, c->nk);
    return Src{x, c->d_grid, nullptr, c->G, c->k0, L.XM, L.XL, L.DB};
}

// Task tables and T/H buffers for an mh_eval_dae call (mocohip.hip).
int probe_tasks(mh_ctx* c, const TaskInfo& ti, const Lanes& ln, int np);

// A batch of structurally identical contexts evaluated together (mh_batch_*,
// include/mocohip.h); built by mh_batch_create (mocohip.hip).
struct mh_batch {
    std::vector<mh_ctx*> ctx;
    int B = 0;
    BatchItem* d_items = nullptr;   // [B] per-NLP constants
    bool gm = true;                 // kb_interval reads group results from global memory
    int waves = 3;                  // kb_groups: 0 = the compiler's register budget, 3 = >= 3 waves/SIMD
    int threads = 512;              // kb_interval workgroup (Jacobian lanes)
};

struct Backend {
    const char* name;
    // one evaluation stage: raw DAE outputs of every lane of c->lanes_g
    // (mode 0) or c->lanes_jac (mode 1) into Y, base-lane times into d_times
    void (*eval)(mh_ctx*, const double* x, int mode, double* Y);
    void (*integrand)(mh_ctx*, const double* x);
    void (*grad)(mh_ctx*, const double* x);
    void (*probe)(mh_ctx*, int np, const double* in, double* out);
    double flops_per_eval;   // generated back ends: emitted FP64 ops per DAE
    const TaskInfo* tasks;   // task-decomposed back ends (else one lane per DAE)
    // task back ends: fused combine + transcription (k_interval) for lanes
    // of mode 0/1 writing g and/or values; null for one-lane back ends
    // (intervals [i0, i1) of the shard; i1 < 0: all)
    void (*interval)(mh_ctx*, const double* x, int mode, double* g, double* v, int i0, int i1);
    size_t (*interval_bytes)(const mh_ctx*, int mode);   // its LDS need
    // raw outputs of every Jacobian lane into Y ([point][output][lane]) and
    // the base-lane times into d_times, whatever path eval_jac_g takes
    // (mh_debug_jacobian_lanes)
    void (*lanes)(mh_ctx*, const double* x, double* Y);
    // task back ends: one k_groups + one k_interval launch for every NLP of
    // a batch (lanes of mode 0/1; g and / or values written per NLP)
    void (*batch)(mh_batch*, int mode, const BatchPtrs& P, int with_g, int with_v);
};

template <class D>
static void be_eval_lane(mh_ctx* c, const double* x, int mode, double* Y) {
    Layout L = make_layout(c, c->k0, c->nk);
    const Lanes& ln = mode ? c->lanes_jac : c->lanes_g;
    const long lanes = (long)c->nk * ln.stride;
    const bool exc = mode && c->d_exc && D::EXC_LANES;
    if (mode && c->NPAR > 0) {
        // MocoParameters: the lanes that perturb no parameter over the
        // iterate's model copy (c->M), then each parameter lane over its own
        // copy (Mp[cp]), one lane per grid point -- the kernels as they are
        const long nm = (long)c->nk * c->n_lane_main;
        hipLaunchKernelGGL(k_eval<D>, dim3((unsigned)((nm + 63) / 64)), dim3(64), 0, c->stream, c->M, L, ln, x,
                c->d_grid, c->d_times, Y, c->d_lane_main, c->n_lane_main);
        if (exc)
            hipLaunchKernelGGL(k_exc_lanes<D>, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, c->stream, c->M,
                    L, ln, x, Y, c->d_exc);
        for (int cp = 1; cp < c->NCOPY; ++cp)
            hipLaunchKernelGGL(k_eval<D>, dim3((unsigned)((c->nk + 63) / 64)), dim3(64), 0, c->stream, c->Mp[cp],
                    L, ln, x, c->d_grid, c->d_times, Y, c->d_par_lanes + (cp - 1), 1);
        return;
    }
    if (!exc) {
        // eval_g of the generic interpreter: fewer lanes per workgroup (one
        // wave each) keep a wave's scratch within its CU's L1
        // (MOCOHIP_G_BLOCK; k_eval indexes by blockDim, any size <= 64 works)
        const int tb = (mode == 0 && D::EXC_LANES) ? c->g_block : 64;
        if constexpr (D::EXC_LANES) {   // the generic interpreter (GenericDae)
            if (mode == 0 && c->g_lds) {
                // MOCOHIP_G_LDS: the workspace in LDS, tb <= 16 slots per workgroup
                const size_t slot = sizeof(typename D::W) + 2 * sizeof(double) * (size_t)c->g_lds_guard;
                const int tl = std::max(1, std::min({tb, 16, (int)(65536 / slot)}));
                const size_t lds = slot * (size_t)tl;
                hipLaunchKernelGGL(k_eval_lds<D>, dim3((unsigned)((lanes + tl - 1) / tl)), dim3(tl), lds,
                        c->stream, c->M, L, ln, x, c->d_grid, c->d_times, Y, c->g_lds_guard, c->d_lds_status);
                return;
            }
        }
        hipLaunchKernelGGL(k_eval<D>, dim3((unsigned)((lanes + tb - 1) / tb)), dim3(tb), 0, c->stream, c->M, L,
                ln, x, c->d_grid, c->d_times, Y, nullptr, 0);
        return;
    }
    const int nmap = ln.stride - c->n_exc_lanes;
    const long full = (long)c->nk * nmap;
    hipLaunchKernelGGL(k_eval<D>, dim3((unsigned)((full + 63) / 64)), dim3(64), 0, c->stream, c->M, L,
            ln, x, c->d_grid, c->d_times, Y, c->d_lane_map, nmap);
    hipLaunchKernelGGL(k_exc_lanes<D>, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0, c->stream, c->M,
            L, ln, x, Y, c->d_exc);
}
// The group tasks of a task set: one k_groups launch, or -- when the model's
// group code needs so many registers that k_groups runs fewer waves per SIMD
// than the light groups' own kernel would (large models: Rajagopal) -- the
// heavy groups' blocks and then the light groups' blocks as two launches of
// k_groups_part, each with its own register budget (MOCOHIP_GROUPS_SPLIT=0/1
// overrides; same arithmetic, bit for bit).
template <class D>
static bool split_groups(const mh_ctx* c) {
    static int decided = -1;   // per model struct: the kernels' occupancy is a property of the code
    if (c->groups_split >= 0) return c->groups_split != 0;
    if (decided < 0) {
        int whole = 0, light = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&whole, k_groups<D>, 64, 0) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&light, k_groups_part<D, 2>, 64, 0) != hipSuccess)
            whole = light = 0;
        // only where the whole kernel is down to one wave per SIMD: otherwise
        // the heavy groups' latency hides behind the light ones in one launch
        // (gait: 11.2 us as one launch vs 8.3 + 6.9 us for the two classes
        // alone, tools/group_timing.py)
        decided = (whole > 0 && whole <= 4 && light > whole) ? 1 : 0;
    }
    return decided != 0;
}
template <class D>
static void launch_groups(mh_ctx* c, const Src& S, const Lanes& ln, const TaskSet& ts, double* T, double* H) {
    if (ts.nheavy > 0 && ts.nheavy < ts.nblocks && split_groups<D>(c)) {
        hipLaunchKernelGGL((k_groups_part<D, 1>), dim3((unsigned)ts.nheavy), dim3(64), 0, c->stream, c->M, S, ln,
                ts.dev, T, H, 0);
        hipLaunchKernelGGL((k_groups_part<D, 2>), dim3((unsigned)(ts.nblocks - ts.nheavy)), dim3(64), 0,
                c->stream, c->M, S, ln, ts.dev, T, H, ts.nheavy);
        return;
    }
#if MOCOHIP_AB_VARIANTS
    if (&ts == &c->ts_g && c->krec_ok) {
        static_assert(sizeof(DevModel) + sizeof(Src) + sizeof(Lanes) + sizeof(Tasks) + 2 * sizeof(double*) +
                      sizeof(KRecs) <= 4096, "k_groups_kr: kernel arguments over 4 KB");
        hipLaunchKernelGGL(k_groups_kr<D>, dim3((unsigned)ts.nblocks), dim3(64), 0, c->stream, c->M, S, ln, ts.dev,
                T, H, c->krec_g);
        return;
    }
#endif
    hipLaunchKernelGGL(k_groups<D>, dim3((unsigned)ts.nblocks), dim3(64), 0, c->stream, c->M, S, ln, ts.dev, T, H);
}

// Raw-value combine of a large model: k_combine_global (64-thread blocks,
// group results read from global memory) when the LDS-staged k_combine would
// keep its lanes' loads in scratch -- measured on the compiled kernels
// (Rajagopal 80: 8.2 KB of scratch per lane for the LDS-staged kernel at 512
// VGPRs, 56 B for the global-memory one; gait: neither spills, LDS staging
// stays).  MOCOHIP_COMBINE=lds / global overrides.
template <class D>
static bool combine_from_global(const mh_ctx* c, unsigned threads) {
    if (c->combine_mode >= 0) return c->combine_mode == 1;
    static int decided = -1;
    if (decided < 0) {
        hipFuncAttributes a{}, b{};
        const void* kl = threads <= 256 ? (const void*)k_combine<D, 256> : (const void*)k_combine<D, 1024>;
        decided = (hipFuncGetAttributes(&a, kl) == hipSuccess &&
                   hipFuncGetAttributes(&b, (const void*)k_combine_global<D>) == hipSuccess &&
                   a.localSizeBytes > 1024 && b.localSizeBytes < a.localSizeBytes / 4) ? 1 : 0;
    }
    return decided != 0;
}

template <class D>
// Returns 1 when Y holds finite-difference quotients (k_combine quot mode,
// Jacobian lanes staged in LDS), 0 when it holds raw lane values.
static int launch_tasks(mh_ctx* c, const Src& S, const Lanes& ln, const TaskSet& ts, double* T,
        double* H, double* times, double* Y, bool quot) {
    launch_groups<D>(c, S, ln, ts, T, H);
    if (c->timing && times) (void)hipEventRecord(c->ev[4], c->stream);
    const unsigned threads = (unsigned)((ln.stride + 63) / 64 * 64);
    quot = quot && ln.stride > 1;
    size_t lds = sizeof(double) * ((size_t)ts.dev.tdoubles + (size_t)ts.dev.nmass * D::NST);
    if (quot) lds = std::max(lds, sizeof(double) * (size_t)D::NO * ln.stride);
    if (threads <= 1024 && lds <= kMaxLds && !(!quot && combine_from_global<D>(c, threads))) {
        auto kern = quot ? (threads <= 256 ? k_combine<D, 256, true> : k_combine<D, 1024, true>)
                         : (threads <= 256 ? k_combine<D, 256> : k_combine<D, 1024>);
        if (lds > 65536)
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(kern, dim3((unsigned)ts.dev.nk), dim3(threads), lds, c->stream, c->M,
                S, ln, ts.dev, T, H, times, Y, (long)D::NO * ln.stride, quot ? 1 : 0);
        return quot ? 1 : 0;
    } else {
        // excitation lanes (Jacobian lanes, raw values): filled after the
        // other lanes' combine instead of combined
        const bool xs = c->d_exc_slot && &ts == &c->ts_jac;
        const int per = xs ? ln.stride - c->n_exc_gen : ln.stride;
        const long lanes = (long)ts.dev.nk * per;
#if MOCOHIP_AB_VARIANTS
        // the sums over the waves (k_combine_split, MOCOHIP_CSPLIT=1; slower)
        if (c->csplit && D::NSUM > 0)
            hipLaunchKernelGGL(k_combine_split<D>, dim3((unsigned)((lanes + 63) / 64)), dim3(256), 0,
                    c->stream, c->M, S, ln, ts.dev, T, H, times, Y, (long)D::NO * ln.stride,
                    xs ? (const int*)c->d_cmb_map : nullptr, per);
        else
#endif
            hipLaunchKernelGGL(k_combine_global<D>, dim3((unsigned)((lanes + 63) / 64)), dim3(64), 0,
                    c->stream, c->M, S, ln, ts.dev, T, H, times, Y, (long)D::NO * ln.stride,
                    xs ? (const int*)c->d_cmb_map : nullptr, per, c->iv_xcd);
        if (xs) (void)mh_launch_exc_fill(c, ts.dev.nk, D::NO, ln.stride, ln.base, ts.dev.tdoubles, T, Y);
    }
    return 0;
}
template <class D>
static void be_eval_tasks(mh_ctx* c, const double* x, int mode, double* Y) {
    const Src S = src_of(c, x);
    const Lanes& ln = mode ? c->lanes_jac : c->lanes_g;
    const TaskSet& ts = mode ? c->ts_jac : c->ts_g;
    double* T = mode ? c->d_T : c->d_Tg;
    double* H = mode ? c->d_H : c->d_Hg;
    if (c->use_interval[mode]) {   // combine happens inside k_interval
        launch_groups<D>(c, S, ln, ts, T, H);
        return;
    }
    c->yq[mode] = launch_tasks<D>(c, S, ln, ts, T, H, c->d_times, Y, mode == 1 && c->quot);
}
// LDS bytes of k_interval for one lane configuration (0: does not apply).
template <class D>
static size_t interval_lds(const mh_ctx* c, const Lanes& ln, const TaskSet& ts) {
    const size_t npts = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
    return sizeof(double) * (npts * D::NO * ln.stride + CT_CONST + CT_NCONST +
                             npts * (size_t)(c->NS + c->NC + c->NDV + c->NM) + (size_t)c->NSL +
                             npts * ((size_t)ts.dev.tdoubles + (size_t)ts.dev.nmass * D::NST)) +
           (c->iv_slots_lds && ln.stride > 1 ? sizeof(int) * (size_t)ln.stride * D::NG : 0);
}
// LDS bytes of k_role (Jacobian lanes).
template <class D>
static size_t role_lds(const mh_ctx* c) {
    const size_t R = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
    const TaskSet& ts = c->ts_jac;
    return sizeof(double) * ((size_t)role_kconst(D::NO, c->lanes_jac.stride, (int)R) + 2 +
                             (size_t)ts.dev.tdoubles + (size_t)ts.dev.nmass * D::NST +
                             R * (size_t)(c->NS + c->NC + c->NDV));
}
template <class D>
static size_t be_interval_bytes(const mh_ctx* c, int mode) {
    if (mode == 1 && c->use_roles && role_lds<D>(c) <= kMaxLds) return role_lds<D>(c);
    return interval_lds<D>(c, mode ? c->lanes_jac : c->lanes_g, mode ? c->ts_jac : c->ts_g);
}
// LDS bytes of k_interval reading the group results from global memory.
// eval_g's base-slot kernel reads the group results from global memory up
// to this many doubles per grid point, stages them in LDS above
constexpr int kIvgGmMaxDoubles = 512;
template <class D>
static size_t interval_lds_gm(const mh_ctx* c, const Lanes& ln) {
    const size_t npts = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
    return sizeof(double) * (npts * D::NO * ln.stride + CT_CONST + CT_NCONST +
                             npts * (size_t)(c->NS + c->NC + c->NDV + c->NM) + (size_t)c->NSL);
}
template <class D>
static void be_batch(mh_batch* bt, int mode, const BatchPtrs& BP, int with_g, int with_v) {
    mh_ctx* c = bt->ctx[0];
    const Lanes& ln = mode ? c->lanes_jac : c->lanes_g;
    const TaskSet& ts = mode ? c->ts_jac : c->ts_g;
    const unsigned B = (unsigned)bt->B;
    auto kg = bt->waves == 3 ? kb_groups<D, 3> : kb_groups<D, 0>;
    Layout L = make_layout(c, c->k0, c->nk);
    hipLaunchKernelGGL(kg, dim3((unsigned)ts.nblocks, B), dim3(64), 0, c->stream, bt->d_items, BP, ln,
            ts.dev, L);
    double *g0 = nullptr, *v0 = nullptr;
    const Interval I = make_interval(c, g0, v0);
    const size_t lds = bt->gm ? interval_lds_gm<D>(c, ln) : interval_lds<D>(c, ln, ts);
    // eval_g (stride-1 lanes, no values, 256 threads): the base-slot kernel
    const bool base = !with_v && ln.stride == 1 && c->ivg_base;
    auto kern = bt->gm ? (base ? kb_interval<D, true, true> : kb_interval<D, true>)
                       : (base ? kb_interval<D, false, true> : kb_interval<D, false>);
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const unsigned threads = with_v ? (unsigned)bt->threads : 256u;
    hipLaunchKernelGGL(kern, dim3((unsigned)(c->ie - c->ib), B), dim3(threads), lds, c->stream, bt->d_items, BP,
            ln, ts.dev, L, I, c->d_tpl, (mode == 1 && c->use_ctpl) ? c->d_ctpl : nullptr, c->d_ctgen,
            (int)c->ctgen.size(), with_g, with_v, c->nep, c->nnz_ep);
}
template <class D>
static void be_interval(mh_ctx* c, const double* x, int mode, double* g, double* v, int i0, int i1) {
    const Src S = src_of(c, x);
    const Lanes& ln = mode ? c->lanes_jac : c->lanes_g;
    const TaskSet& ts = mode ? c->ts_jac : c->ts_g;
    Layout L = make_layout(c, c->k0, c->nk);
    const Interval I = make_interval(c, g, v);
    // (a failed hipFuncSetAttribute would surface as the launch's error:
    // only the launched kernel's attribute is set, and only when it fits)
    if (mode == 1 && c->use_roles && role_lds<D>(c) <= kMaxLds) {
        const size_t rl = role_lds<D>(c);
        if (rl > 65536)
            (void)hipFuncSetAttribute((const void*)k_role<D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)rl);
        const unsigned R = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
        RoleLists RL{c->d_rl_e, c->d_rl_w, {c->rl_off[0], c->rl_off[1], c->rl_off[2], c->rl_off[3]},
                     c->rl_tail[0], c->rl_tail[1], c->role_couple ? 1 : 0};
        const unsigned nint = (unsigned)(c->ie - c->ib);
        hipLaunchKernelGGL(k_role<D>, dim3(R * nint), dim3((unsigned)c->role_threads), rl, c->stream, c->M, S,
                ln, ts.dev, L, I, c->d_tpl, RL, c->d_xch, c->d_ctgen, (int)c->ctgen.size(), c->d_T, c->d_H, g, v);
        if (c->role_couple) return;
        const size_t cl = sizeof(double) * (R * (size_t)D::NO * XCH_W + 4 + R * (size_t)(c->NS + c->NC + c->NDV));
        hipLaunchKernelGGL(k_couple<D>, dim3(nint), dim3(256), cl, c->stream, S, ln, L, I, c->d_tpl,
                c->d_ctgen, (int)c->ctgen.size(), c->d_xch, g, v);
        return;
    }
    size_t lds = interval_lds<D>(c, ln, ts);
    const unsigned threads = v ? (unsigned)c->iv_threads : (unsigned)c->ivg_threads;
    auto kern = threads <= 256 ? k_interval<D, 256> : k_interval<D, 1024>;
    // eval_g's launches: the base-slot kernel (MOCOHIP_IVG_BASE=0: the
    // slot-table path, bit-identical), its three combine lanes reading the
    // group results from global memory at their constant offsets when a grid
    // point's results are few (gait: 190 doubles; k_interval 8.2 -> 5.7 us
    // against a staging pass through LDS first, profiles/r05_e/ab_ivg_gm.txt),
    // staged in LDS when they are many (Rajagopal 80: 1,111 doubles, where the
    // global-memory reads made eval_g slower, profiles/r05_f); MOCOHIP_IVG_GM
    // = 0 / 1 forces either
#if MOCOHIP_AB_VARIANTS
    if (v && threads > 256 && c->iv_slots_lds && ln.stride > 1) kern = k_interval<D, 1024, false, false, true>;
#endif
    if (!v && ln.stride == 1 && threads <= 256 && c->ivg_base) {
        const bool gm = c->ivg_gm < 0 ? ts.dev.tdoubles <= kIvgGmMaxDoubles : c->ivg_gm != 0;
        kern = gm ? k_interval<D, 256, true, true> : k_interval<D, 256, true>;
        if (gm) lds = interval_lds_gm<D>(c, ln);
    }
    if (lds > 65536)
        (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (i1 < 0) { i0 = 0; i1 = c->ie - c->ib; }
    if (i1 <= i0) return;
    hipLaunchKernelGGL(kern, dim3((unsigned)(i1 - i0)), dim3(threads), lds, c->stream, c->M,
            S, ln, ts.dev, L, I, c->d_tpl, (mode == 1 && c->use_ctpl) ? c->d_ctpl : nullptr, c->d_ctgen,
            (int)c->ctgen.size(), mode ? c->d_T : c->d_Tg, mode ? c->d_H : c->d_Hg, g, v, i0);
}
template <class D>
static void be_integrand(mh_ctx* c, const double* x) {
    Layout L = make_layout(c, 0, c->G);
    hipLaunchKernelGGL(k_integrand<D>, dim3((c->G + 63) / 64), dim3(64), 0, c->stream, c->M, L,
            c->GS, x, c->d_grid, c->d_quad, c->d_C);
}
template <class D>
static void be_grad(mh_ctx* c, const double* x) {
    Layout L = make_layout(c, 0, c->G);
    const long tot = (long)c->G * (c->NI + 2);
    hipLaunchKernelGGL(k_grad<D>, dim3((unsigned)((tot + 63) / 64)), dim3(64), 0, c->stream, c->M, L,
            c->GS, c->fd, c->h, x, c->d_grid, c->d_quad, c->d_grad, c->d_tpart);
}
template <class D>
static void be_probe_lane(mh_ctx* c, int np, const double* in, double* out) {
    Layout L = make_layout(c, 0, 0);
    // the pristine model: a probe point carries no parameter values
    hipLaunchKernelGGL(k_dae_probe<D>, dim3((np + 63) / 64), dim3(64), 0, c->stream, c->M0, L, np, in,
            out);
}
// mh_eval_dae through the task kernels: explicit points, base lanes only.
template <class D>
static void be_probe_tasks(mh_ctx* c, int np, const double* in, double* out) {
    const Lanes ln{c->fd, c->NI + 2, 1, 0, c->h};
    if (probe_tasks(c, *c->be->tasks, ln, np) != MH_OK) return;
    const Src S{nullptr, nullptr, in, 0, 0, 0, 0, 0};
    (void)launch_tasks<D>(c, S, ln, c->ts_probe, c->d_pT, c->d_pH, nullptr, out, false);
}
template <class D>
static void be_lanes_lane(mh_ctx* c, const double* x, double* Y) { be_eval_lane<D>(c, x, 1, Y); }
template <class D>
static void be_lanes_tasks(mh_ctx* c, const double* x, double* Y) {
    const Src S = src_of(c, x);
    (void)launch_tasks<D>(c, S, c->lanes_jac, c->ts_jac, c->d_T, c->d_H, c->d_times, Y, false);
}
template <class D>
static constexpr Backend make_backend_lane(const char* name, double flops) {
    return Backend{name, &be_eval_lane<D>, &be_integrand<D>, &be_grad<D>, &be_probe_lane<D>, flops,
                   nullptr, nullptr, nullptr, &be_lanes_lane<D>, nullptr};
}
template <class D>
struct TaskInfoOf {
    static constexpr TaskInfo value{D::NG, D::NST, D::NF, D::RW, D::NHEAVY, D::GROUP_NF, &D::GROUP_READS[0][0],
                                    D::GROUP_TIME, D::GROUP_FLOPS, D::COMBINE_FLOPS};
};
template <class D>
static constexpr Backend make_backend_tasks(const char* name, double flops) {
    return Backend{name, &be_eval_tasks<D>, &be_integrand<D>, &be_grad<D>, &be_probe_tasks<D>, flops,
                   &TaskInfoOf<D>::value, &be_interval<D>, &be_interval_bytes<D>, &be_lanes_tasks<D>,
                   &be_batch<D>};
}

// Generic device-interpreter back ends (generic.hip), one per size class.
const Backend* generic_backends();
// A model-specialized back end (generated/gen_<model>.hip): the task kernels
// (default) and the one-lane-per-DAE kernel (MOCOHIP_BACKEND=lane), for the
// model structure match() accepts (multibody dynamics mode and prescribed
// kinematics included); fill() computes a model's constant pool.
struct GenEntry {
    bool (*match)(const mh_model&);
    void (*fill)(const mh_model&, double*);
    int npool;
    bool implicit, prescribed;
    // kinematic constraints: derivatives enforced, velocity-correction slacks
    bool kc_enforce, kc_slacks;
    const char* label;
    Backend tasks, lane;
};
#define MH_GEN_ENTRY(T, IMPLICIT, PRESCRIBED, KC_ENFORCE, KC_SLACKS, NAME)                     \
    GenEntry{&T##_match, &T##_fill, T::NPOOL, IMPLICIT, PRESCRIBED, KC_ENFORCE, KC_SLACKS, NAME, \
             make_backend_tasks<T>("generated:" NAME, T::FLOPS_PER_EVAL),                   \
             make_backend_lane<T>("generated-lane:" NAME, T::FLOPS_PER_EVAL)}

// 1 / spacing of table ti's breakpoints when a direct-index guess lands
// within one segment of the right one for every time (codegen.py
// _uniform_guess, the same arithmetic), else 0.  Host only.
inline double mh_table_uniform_inv(const mh_model& m, int ti) {
    if (ti < 0 || ti >= m.ntables) return 0.0;
    const mh_table& T = m.tables[ti];
    const int n = T.nseg;
    if (n < 2) return 0.0;
    const double* br = m.table_breaks + T.break_begin;
    const double inv = n / (br[n] - br[0]);
    if (!std::isfinite(inv) || inv <= 0.0) return 0.0;
    for (int i = 0; i < n; ++i) {
        const double lo = std::floor((br[i] - br[0]) * inv);
        const double hi = std::floor((std::nextafter(br[i + 1], -INFINITY) - br[0]) * inv);
        if (lo < i - 1 || hi > i + 1) return 0.0;
    }
    return inv;
}
