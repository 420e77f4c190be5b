// mocohip.hip — MI355X (gfx950) implementation of the C ABI in
// include/mocohip.h: the direct-collocation NLP hot path of Moco's
// MocoCasADiSolver (CasOCTranscription / CasOCHermiteSimpson /
// CasOCTrapezoidal) with its per-grid-point DAE and finite-difference
// Jacobian, re-designed for CDNA4.  One evaluation is two stages:
//
//   DAE stage (model-specialized back ends from mocohip/codegen.py)
//     k_groups    one wave = one independent piece of the DAE (mass matrix,
//                 bias forces, an external load, a muscle, an activation) for
//                 64 (grid point, lane role) tasks; a finite-difference lane
//                 only re-evaluates the pieces that read its perturbed input.
//     k_combine   one workgroup per grid point: stages the pieces in LDS, sums
//                 the generalized forces in a fixed order, solves with the
//                 mass-matrix factor -> raw outputs Y of every lane.
//   (generic interpreter / one-lane kernels: k_eval, one lane per DAE.)
//
//   transcription stage
//     k_transcribe  one workgroup per (mesh interval, nonzero chunk): the
//                 Jacobian values of a fixed per-interval template, chained
//                 through the Hermite-Simpson / trapezoidal defect formulas
//                 and CasADi's finite-difference quotients; plus one block
//                 per interval for the defect / interpolation rows of g.
//   k_integrand / k_grad / k_reduce_obj : objective and its gradient.
//
// There is no CPU fallback anywhere in this file.
#include "core.hpp"

#include <cstdarg>
#include <limits>

// ------------------------------------------------------------------------
// error handling
// ------------------------------------------------------------------------
static thread_local std::string g_err;
static int set_err(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(expr)                                                              \
    do {                                                                          \
        hipError_t e_ = (expr);                                                   \
        if (e_ != hipSuccess)                                                     \
            return set_err(MH_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

extern "C" int mh_abi_version(void) { return MH_ABI_VERSION; }
#ifndef MH_BUILD_ID
#define MH_BUILD_ID "unknown"
#endif
extern "C" const char* mh_build_id(void) { return MH_BUILD_ID; }
extern "C" const char* mh_last_error(void) { return g_err.c_str(); }

// Excitation lanes of a generated back end: a direction that perturbs the
// excitation of one muscle with activation dynamics re-evaluates only that
// muscle's activation group, whose one field is the activation derivative
// output; every other output of its combine reads base-lane slots only, so
// it equals the base lane's.  One thread per (grid point, output, such lane):
// xs[3 e] = the lane, xs[3 e + 1] = the group's slot, xs[3 e + 2] = the
// output.  Bit-identical to combining the lane
// (test_generated_excitation_fill_bit_identical, MOCOHIP_EXC_LANES=0).
__global__ void __launch_bounds__(256) k_exc_fill(int nk, int NO, int stride, int base, int tdoubles, int nx,
        const int* __restrict__ xs, const double* __restrict__ T, double* __restrict__ Y) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)nk * NO * nx) return;
    const int e = (int)(gid % nx);
    const long ko = gid / nx;
    const int o = (int)(ko % NO);
    const int kl = (int)(ko / NO);
    double* Yo = Y + ((long)kl * NO + o) * stride;
    Yo[xs[3 * e]] = o == xs[3 * e + 2] ? T[(long)kl * tdoubles + xs[3 * e + 1]] : Yo[base];
}
// The activation-derivative output of each excitation lane only (one thread
// per (grid point, lane)): when the compiled template reads every other
// output of those lanes at the base lane (redirect_exc_words), the copies
// k_exc_fill writes are never read
__global__ void __launch_bounds__(256) k_exc_fill_adot(int nk, int NO, int stride, int tdoubles, int nx,
        const int* __restrict__ xs, const double* __restrict__ T, double* __restrict__ Y) {
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)nk * nx) return;
    const int e = (int)(gid % nx);
    const int kl = (int)(gid / nx);
    Y[((long)kl * NO + xs[3 * e + 2]) * stride + xs[3 * e]] = T[(long)kl * tdoubles + xs[3 * e + 1]];
}
int mh_launch_exc_fill(const mh_ctx* c, int nk, int NO, int stride, int base, int tdoubles, const double* T,
                       double* Y) {
    // (the redirected words are the compiled template's: the TplEntry
    // assembly, MOCOHIP_CTPL=0 / MOCOHIP_ASM_CTPL=0 / MOCOHIP_ASM=gs, reads
    // every copy)
    if (c->exc_redirected && !c->exc_full && c->use_ctpl && c->asm_ctpl && !c->asm_grid_stride) {
        const long all = (long)nk * c->n_exc_gen;
        hipLaunchKernelGGL(k_exc_fill_adot, dim3((unsigned)((all + 255) / 256)), dim3(256), 0, c->stream, nk, NO,
                           stride, tdoubles, c->n_exc_gen, (const int*)c->d_exc_slot, T, Y);
        return MH_OK;
    }
    const long all = (long)nk * NO * c->n_exc_gen;
    hipLaunchKernelGGL(k_exc_fill, dim3((unsigned)((all + 255) / 256)), dim3(256), 0, c->stream, nk, NO, stride,
                       base, tdoubles, c->n_exc_gen, (const int*)c->d_exc_slot, T, Y);
    return MH_OK;
}

// MocoParameters (applyParametersToModelProperties before every
// evaluation, MocoCasOCProblem.h:309,508-515): every model copy starts as
// the pristine arrays (copied as 8-byte words), then each target property
// gets its parameter's value -- copy 0 the iterate's, copy cp >= 1 the
// iterate's moved by the finite-difference step along parameter (cp - 1) mod
// NPAR (+h; -h for backward differences and for central's second half).
// One workgroup: a few KB per copy.
struct ParamCopies {
    const mh_body* b0; const mh_actuator* a0; const mh_muscle* m0; const mh_spring* s0;
    mh_body* b; mh_actuator* a; mh_muscle* m; mh_spring* s;
    int nb, na, nm, ns, ncopy, npar;
};
__global__ void __launch_bounds__(256) k_apply_params(ParamCopies P, const mh_parameter_target* __restrict__ tg,
        int nt, const double* __restrict__ xp, double h, int fd) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x, nthr = blockDim.x;
    auto copy = [&](const void* src, void* dst, size_t bytes) {
        const long words = (long)(bytes / 8);
        const unsigned long long* s = (const unsigned long long*)src;
        unsigned long long* d = (unsigned long long*)dst;
        for (long w = tid; w < words * P.ncopy; w += nthr) d[w] = s[w % words];
    };
    copy(P.b0, P.b, sizeof(mh_body) * (size_t)P.nb);
    copy(P.a0, P.a, sizeof(mh_actuator) * (size_t)P.na);
    copy(P.m0, P.m, sizeof(mh_muscle) * (size_t)P.nm);
    copy(P.s0, P.s, sizeof(mh_spring) * (size_t)P.ns);
    __syncthreads();
    for (int k = tid; k < nt * P.ncopy; k += nthr) {
        const int t = k / P.ncopy, cp = k - t * P.ncopy;
        const mh_parameter_target T = tg[t];
        double v = xp[T.parameter];
        if (cp >= 1 && (cp - 1) % P.npar == T.parameter) {
            const bool minus = fd == MH_FD_BACKWARD || (fd == MH_FD_CENTRAL && cp > P.npar);
            v = minus ? v - h : v + h;
        }
        switch (T.kind) {
        case MH_PARAM_BODY_MASS: P.b[(size_t)cp * P.nb + T.index].mass = v; break;
        case MH_PARAM_BODY_MASS_CENTER: P.b[(size_t)cp * P.nb + T.index].com[T.element] = v; break;
        case MH_PARAM_BODY_INERTIA: P.b[(size_t)cp * P.nb + T.index].inertia[T.element] = v; break;
        case MH_PARAM_SPRING_STIFFNESS: P.s[(size_t)cp * P.ns + T.index].stiffness = v; break;
        case MH_PARAM_SPRING_REST_LENGTH: P.s[(size_t)cp * P.ns + T.index].rest_length = v; break;
        case MH_PARAM_SPRING_VISCOSITY: P.s[(size_t)cp * P.ns + T.index].viscosity = v; break;
        case MH_PARAM_ACTUATOR_OPTIMAL_FORCE: P.a[(size_t)cp * P.na + T.index].optimal_force = v; break;
        case MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE: P.m[(size_t)cp * P.nm + T.index].max_isometric_force = v; break;
        default: break;
        }
    }
}
// Writes the model copies for iterate x (device pointer) on the context stream.
static void apply_params(mh_ctx* c, const double* x) {
    if (c->NPAR <= 0) return;
    const DevModel& B = c->M0;
    const DevModel& Q = c->Mp[0];
    ParamCopies P{B.bodies, B.acts, B.mus, B.sp, (mh_body*)Q.bodies, (mh_actuator*)Q.acts, (mh_muscle*)Q.mus,
                  (mh_spring*)Q.sp, B.nb, B.nact, B.nmus, B.nsp, c->NCOPY, c->NPAR};
    hipLaunchKernelGGL(k_apply_params, dim3(1), dim3(256), 0, c->stream, P, c->d_par_targets,
            (int)c->par_targets.size(), x + c->XP, c->h, c->fd);
}

// Transcription stage of the split path, one launch: blockIdx.y = mesh
// interval; blockIdx.x < nchunks streams Jacobian nonzeros (values != null),
// the last x-block (when g != null) writes the interval's defect /
// interpolation rows.
//
// ctpl (the compiled template of k_interval, core.hpp CT_*): a nonzero is
// base + coef q with q one quotient of the interval's Y run -- the interval's
// grid points are consecutive, so their Y rows form the [point][NO][stride]
// run the words' offsets index -- read with one 4-byte word (and its row's
// base-lane offset) instead of a TplEntry and the formula's branches; t0 / tf
// (CT_GEN) and path (CT_PATH) entries take jac_entry.  The same operations in
// the same order as jac_entry: bit-identical (MOCOHIP_CTPL=0 compares).
__global__ void __launch_bounds__(256) k_transcribe(Layout L, Interval I, Lanes Ln,
        const TplEntry* __restrict__ tpl, const uint32_t* __restrict__ ctpl, const int* __restrict__ ctgen,
        int nctgen, const double* __restrict__ x,
        const double* __restrict__ grid, const double* __restrict__ times,
        const double* __restrict__ Y, double* __restrict__ g, double* __restrict__ values,
        int nchunks, int yq, int chunk) {
    // I.xcd: the chunks of one interval on one XCD (xcd_interval over the
    // linear block id): an interval's chunks gather from the same Y run,
    // which then crosses the XCD's L2 once instead of once per XCD
    int il = (int)blockIdx.y, bx = (int)blockIdx.x;
    if (I.xcd) {
        const int gx = (int)gridDim.x;
        const int lin = xcd_interval(il * gx + bx, gx * (int)gridDim.y);
        il = lin / gx;
        bx = lin - il * gx;
    }
    const int i = I.ib + il;
    const YG YV{Y, times, L.NO, Ln.stride, L.k0, yq, x, L.NS, L.NC, L.G, L.NDV, L.DB};
    if (bx < nchunks) {
        int k_first, k_last;
        interval_span(I, i, k_first, k_last);
        const IvC C = iv_const(YV.t(k_last) - YV.t(k_first), grid[k_last] - grid[k_first]);
        double* vi = values + (long)il * I.nnz_int;
        const int e_end = min(I.entries(i), (bx + 1) * chunk);
        if (ctpl) {   // chunks of asm_chunk_ct entries
#pragma clang fp contract(off)
            // the coefficient / base tables the words select from (the same
            // doubles jac_entry forms)
            __shared__ double kc[8], kb[8];
            if (threadIdx.x < 8) {
                const int t = threadIdx.x;
                kc[t] = t == 1 ? -C.h8 : t == 2 ? C.h8 : t == 3 ? -C.h6 : t == 4 ? -C.h6 * 4.0 : t == 5 ? -C.hh : 0.0;
                kb[t] = t == 1 ? -0.5 : t == 2 ? 1.0 : t == 3 ? -1.0 : 0.0;
            }
            __syncthreads();
            const int npts = k_last - k_first + 1;
            const uint32_t nyall = (uint32_t)(npts * L.NO * Ln.stride);
            const uint32_t kone = nyall + CT_CONST + 1;
            const double* __restrict__ Yi = Y + (long)(k_first - L.k0) * L.NO * Ln.stride;
            const uint32_t* __restrict__ cbase = ctpl + I.nnz_int + I.nnz_tail;
            const int eb = bx * chunk, ee = min(I.entries(i), eb + chunk);
            // the bulk, branch-free per entry: CT_U entries per thread and
            // pass (their words, then their Y values, then their stores);
            // t0 / tf (CT_GEN) and path (CT_PATH) entries are skipped here and
            // written by the two loops below.  One instantiation per
            // finite-difference formula (no per-entry scalar branches).
            auto bulk = [&](auto fdc, auto qdc) {
                constexpr int FD = decltype(fdc)::value;
                constexpr bool QD = decltype(qdc)::value;
                const double hq = FD == MH_FD_CENTRAL ? 2.0 * Ln.h : Ln.h;
                const double rq = 1.0 / hq;
                constexpr int CT_U = 8;
                for (int e0 = eb + (int)threadIdx.x; e0 < ee; e0 += CT_U * (int)blockDim.x) {
                    uint32_t w[CT_U], wb[CT_U];
#pragma unroll
                    for (int u = 0; u < CT_U; ++u) {
                        const int e = min(e0 + u * (int)blockDim.x, ee - 1);
                        w[u] = ctpl[e];
                        if (!I.dbase) wb[u] = FD == MH_FD_CENTRAL ? 0u : cbase[e];
                    }
                    if (I.dbase) {
#pragma unroll
                        for (int u = 0; u < CT_U; ++u) wb[u] = FD == MH_FD_CENTRAL ? 0u : I.base_of(w[u], nyall);
                    }
                    double ya[CT_U], yb[CT_U];
#pragma unroll
                    for (int u = 0; u < CT_U; ++u) {
                        const uint32_t off = w[u] & CT_OFF;
                        const uint32_t oy = off < nyall ? off : 0u;
                        ya[u] = Yi[oy];
                        yb[u] = FD == MH_FD_CENTRAL ? Yi[off < nyall ? off + Ln.ND : 0u] : Yi[wb[u] < nyall ? wb[u] : 0u];
                    }
#pragma unroll
                    for (int u = 0; u < CT_U; ++u) {
                        const int e = e0 + u * (int)blockDim.x;
                        const uint32_t off = w[u] & CT_OFF;
                        const double dy = FD == MH_FD_BACKWARD ? yb[u] - ya[u] : ya[u] - yb[u];
                        const double qd = QD ? div_rn(dy, hq, rq) : dy / hq;
                        const double q = off >= nyall ? (off == kone ? 1.0 : 0.0) : (yq ? ya[u] : qd);
                        const double v = (w[u] & CT_RAW) ? q : kb[(w[u] >> 23) & 7] + kc[(w[u] >> 20) & 7] * q;
                        if (e < ee && !(w[u] & (CT_GEN | CT_PATH))) vi[e] = v;
                    }
                }
            };
            // (div_rn: the step within [2^-60, 2^60], checked on the host)
            auto bulk_fd = [&](auto qdc) {
                if (Ln.fd == MH_FD_FORWARD) bulk(std::integral_constant<int, MH_FD_FORWARD>{}, qdc);
                else if (Ln.fd == MH_FD_BACKWARD) bulk(std::integral_constant<int, MH_FD_BACKWARD>{}, qdc);
                else bulk(std::integral_constant<int, MH_FD_CENTRAL>{}, qdc);
            };
            if (I.qdiv) bulk_fd(std::true_type{});
            else bulk_fd(std::false_type{});
            // t0 / tf entries of this chunk
            for (int j = threadIdx.x; j < nctgen; j += blockDim.x) {
                const int e = ctgen[j];
                if (e >= eb && e < ee) vi[e] = jac_entry<false>(L, Ln, I.P, x, YV, tpl[e], k_first, C);
            }
            // path entries (the first npe of the interval and of the tail)
            const int nw = i == I.N - 1 ? 2 * I.npe : I.npe;
            for (int w = threadIdx.x; w < nw; w += blockDim.x) {
                const int ep = w < I.npe ? w : I.nnz_int + (w - I.npe);
                if (ep >= eb && ep < ee) vi[ep] = jac_entry<true>(L, Ln, I.P, x, YV, tpl[ep], k_first, C);
            }
        } else {
            for (int e = bx * chunk + threadIdx.x; e < e_end; e += blockDim.x)
                vi[e] = jac_entry(L, Ln, I.P, x, YV, tpl[e], k_first, C);
        }
    } else {
        double* gi = g + (long)il * I.rpi;
        for (int r = threadIdx.x; r < I.rows(i); r += blockDim.x) gi[r] = defect_row(L, I, Ln, x, YV, i, r);
    }
    if (i == 0 && bx == 0 && (I.gh || I.vh))
        endpoint_head(L, Ln, I.E, x, g ? I.gh : nullptr, values ? I.vh : nullptr, threadIdx.x, blockDim.x);
}

// Transcription stage of the split path as a grid-stride loop over the
// shard's (interval, nonzero) and (interval, row) pairs: a few long-lived
// waves per SIMD instead of thousands of short workgroups (whose dispatch,
// not their memory traffic, bounded the chunked form).
__device__ __forceinline__ int div_exact(int w, int n, double inv) {
    int q = (int)((double)w * inv);
    q += (q + 1) * n <= w ? 1 : 0;
    q -= q * n > w ? 1 : 0;
    return q;
}
__global__ void __launch_bounds__(256) k_transcribe_gs(Layout L, Interval I, Lanes Ln,
        const TplEntry* __restrict__ tpl, const double* __restrict__ x,
        const double* __restrict__ grid, const double* __restrict__ times,
        const double* __restrict__ Y, double* __restrict__ g, double* __restrict__ values,
        int nint, int yq) {
    const YG YV{Y, times, L.NO, Ln.stride, L.k0, yq, x, L.NS, L.NC, L.G, L.NDV, L.DB};
    const int nthreads = gridDim.x * blockDim.x;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (values) {
        const int total = nint * I.nnz_int;
        const double inv = 1.0 / I.nnz_int;
        for (int w = tid; w < total; w += nthreads) {
            const int il = div_exact(w, I.nnz_int, inv);
            const int e = w - il * I.nnz_int;
            const int i = I.ib + il;
            int k_first, k_last;
            interval_span(I, i, k_first, k_last);
            const IvC C = iv_const(YV.t(k_last) - YV.t(k_first), grid[k_last] - grid[k_first]);
            values[w] = jac_entry(L, Ln, I.P, x, YV, tpl[e], k_first, C);
        }
    }
    if (g) {
        const int total = nint * I.rpi;
        const double inv = 1.0 / I.rpi;
        for (int w = tid; w < total; w += nthreads) {
            const int il = div_exact(w, I.rpi, inv);
            g[w] = defect_row(L, I, Ln, x, YV, I.ib + il, w - il * I.rpi);
        }
    }
    // the final grid point's residual rows (implicit mode), owned by the
    // shard holding the last interval
    if (I.ib + nint == I.N && (I.ntail > 0)) {
        const int i = I.N - 1, il = nint - 1;
        int k_first, k_last;
        interval_span(I, i, k_first, k_last);
        if (values) {
            const IvC C = iv_const(YV.t(k_last) - YV.t(k_first), grid[k_last] - grid[k_first]);
            for (int e = I.nnz_int + tid; e < I.entries(i); e += nthreads)
                values[(long)il * I.nnz_int + e] = jac_entry(L, Ln, I.P, x, YV, tpl[e], k_first, C);
        }
        if (g)
            for (int r = I.rpi + tid; r < I.rows(i); r += nthreads)
                g[(long)il * I.rpi + r] = defect_row(L, I, Ln, x, YV, i, r);
    }
    if (I.ib == 0 && (I.gh || I.vh))
        endpoint_head(L, Ln, I.E, x, g ? I.gh : nullptr, values ? I.vh : nullptr, tid, nthreads);
}

// Single-workgroup deterministic reduction of the objective (mode 0) or of
// the t0/tf gradient entries (mode 1).
__global__ void __launch_bounds__(256) k_reduce_obj(Layout L, GoalSet GS, int mode, int endpoint,
        const double* __restrict__ x, const double* __restrict__ C,
        const double* __restrict__ tpart, const double* __restrict__ ep, double* __restrict__ out) {
    __shared__ double red[256];
    const int ng = GS.ngoals;
    double total = 0.0, g0 = 0.0, g1 = 0.0;
    for (int gi = 0; gi < ng; ++gi) {
        double s = 0.0;
        for (int k = threadIdx.x; k < L.G; k += blockDim.x) s += C[(long)k * ng + gi];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int w = blockDim.x / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        const double acc = red[0];
        __syncthreads();
        const mh_goal G = GS.goals[gi];
        double term = 0.0;
        if (G.kind == MH_GOAL_FINAL_TIME) {
            if (endpoint) {
                term = G.weight * x[1];
                total += term;
                g1 += G.weight;
            }
        } else if (G.kind == MH_GOAL_MARKER_FINAL) {
            if (endpoint) {
                term = G.weight * ep[gi];   // its gradient: k_marker_final
                total += term;
            }
        } else {
            term = G.weight * ((x[1] - x[0]) * acc);
            total += term;
            g0 += -G.weight * acc;
            g1 += G.weight * acc;
        }
        // mode 2: the objective's terms, one per goal (mh_eval_objective_terms)
        if (mode == 2 && threadIdx.x == 0) out[gi] = term;
    }
    if (mode == 2) return;
    if (mode == 0) {
        if (threadIdx.x == 0) out[0] = total;
        return;
    }
    for (int c = 0; c < 2; ++c) {
        double s = 0.0;
        for (int k = threadIdx.x; k < L.G; k += blockDim.x) s += tpart[(long)k * 2 + c];
        red[threadIdx.x] = s;
        __syncthreads();
        for (int w = blockDim.x / 2; w > 0; w >>= 1) {
            if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
            __syncthreads();
        }
        if (threadIdx.x == 0) out[c] = red[0] + (c == 0 ? g0 : g1);
        __syncthreads();
    }
}

// Pose of body b in ground at coordinates q (the position part of dae_eval's
// forward pass, dae_device.hpp: parent pose x joint frames x coordinate
// functions), walking b's ancestors from the ground.
__device__ void body_pose(const DevModel& M, const double* q, int b, double* R, double* p) {
    int chain[MH_MARKER_MAX_Q + 1];
    int n = 0;
    for (int x = b; x >= 0 && n <= MH_MARKER_MAX_Q; x = M.bodies[x].parent) chain[n++] = x;
    double Rp[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, pp[3] = {0, 0, 0};
    for (int ci = n - 1; ci >= 0; --ci) {
        const mh_body& B = M.bodies[chain[ci]];
        double RGF[9], t0, t1, t2;
        mm3(Rp, B.R_PF, RGF);
        mv3(Rp, B.p_PF[0], B.p_PF[1], B.p_PF[2], t0, t1, t2);
        const double pGF0 = pp[0] + t0, pGF1 = pp[1] + t1, pGF2 = pp[2] + t2;
        double pFM0 = 0, pFM1 = 0, pFM2 = 0;
        for (int a = B.axis_begin; a < B.axis_begin + B.axis_count; ++a) {
            const mh_axis X = M.axes[a];
            if (X.type != MH_AXIS_TRANSLATION) continue;
            double v, d1, d2;
            fn_eval(M, X.func, q, v, d1, d2);
            pFM0 += v * X.dir[0]; pFM1 += v * X.dir[1]; pFM2 += v * X.dir[2];
        }
        mv3(RGF, pFM0, pFM1, pFM2, t0, t1, t2);
        const double oM0 = pGF0 + t0, oM1 = pGF1 + t1, oM2 = pGF2 + t2;
        double Rcur[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        for (int a = B.axis_begin; a < B.axis_begin + B.axis_count; ++a) {
            const mh_axis X = M.axes[a];
            if (X.type != MH_AXIS_ROTATION) continue;
            double v, d1, d2;
            fn_eval(M, X.func, q, v, d1, d2);
            double Rk[9];
            axis_rot(X.dir[0], X.dir[1], X.dir[2], v, Rk);
            mm3(Rcur, Rk, Rcur);
        }
        double RGM[9];
        mm3(RGF, Rcur, RGM);
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j)
                Rp[3 * i + j] = RGM[3 * i] * B.R_BM[3 * j] + RGM[3 * i + 1] * B.R_BM[3 * j + 1] +
                                RGM[3 * i + 2] * B.R_BM[3 * j + 2];
        mv3(Rp, B.p_BM[0], B.p_BM[1], B.p_BM[2], t0, t1, t2);
        pp[0] = oM0 - t0; pp[1] = oM1 - t1; pp[2] = oM2 - t2;
    }
    for (int i = 0; i < 9; ++i) R[i] = Rp[i];
    for (int i = 0; i < 3; ++i) p[i] = pp[i];
}

// MocoMarkerFinalGoal (MocoMarkerFinalGoal.cpp:29-34): |p_G(q(tf)) - r|^2
// of a body-fixed point; block gi = goal gi.  Lane 0: the final grid
// point's coordinates; mode 1 (gradient): lane 1 + s perturbs coordinate s by
// +h (backward: -h), central also lane 1 + NQ + s by -h, and lane 0 adds
// weight * the FD quotient to grad's final-state entries (after k_grad).
__global__ void __launch_bounds__(128) k_marker_final(DevModel M, Layout L, GoalSet GS, int fd, double h,
        int mode, const double* __restrict__ x, double* __restrict__ ep, double* __restrict__ grad) {
    const int gi = blockIdx.x;
    const mh_goal G = GS.goals[gi];
    if (G.kind != MH_GOAL_MARKER_FINAL) return;
    __shared__ double cost[2 * MH_MARKER_MAX_Q + 1];
    const int NQ = L.NQ;
    const int nl = 1 + (mode ? (fd == MH_FD_CENTRAL ? 2 * NQ : NQ) : 0);
    const double* xs = x + 2 + (long)(L.G - 1) * L.NS;
    const int k0 = G.term_begin;
    const int b = GS.gidx[k0];
    for (int j = threadIdx.x; j < nl; j += blockDim.x) {
        double q[MH_MARKER_MAX_Q];
        for (int s = 0; s < NQ; ++s) q[s] = xs[s];
        if (j > 0) {
            const int s = (j - 1) % NQ;
            const bool minus = fd == MH_FD_BACKWARD || j > NQ;
            q[s] = minus ? xs[s] - h : xs[s] + h;
        }
        double R[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, p[3] = {0, 0, 0};
        if (b >= 0) body_pose(M, q, b, R, p);
        double y0, y1, y2;
        mv3(R, GS.gw[k0], GS.gw[k0 + 1], GS.gw[k0 + 2], y0, y1, y2);
        const double d0 = (p[0] + y0) - GS.gw[k0 + 3], d1 = (p[1] + y1) - GS.gw[k0 + 4],
                     d2 = (p[2] + y2) - GS.gw[k0 + 5];
        double s2 = 0.0;
        s2 += d0 * d0;
        s2 += d1 * d1;
        s2 += d2 * d2;
        cost[j] = s2;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    ep[gi] = cost[0];
    if (!mode) return;
    for (int s = 0; s < NQ; ++s) {
        const double d = fd == MH_FD_CENTRAL ? (cost[1 + s] - cost[1 + NQ + s]) / (2.0 * h)
                       : (fd == MH_FD_FORWARD ? (cost[1 + s] - cost[0]) / h : (cost[0] - cost[1 + s]) / h);
        grad[2 + (long)(L.G - 1) * L.NS + s] += G.weight * d;
    }
}

// ------------------------------------------------------------------------
// Host side.
// ------------------------------------------------------------------------
namespace {

// SimmSpline coefficients (Forsythe–Malcolm–Moler with third-derivative end
// conditions; opensim-core SimmSpline::calcCoefficients, third-party).
void simm_coefficients(int n, const double* x, const double* y, double* b, double* c, double* d) {
    if (n < 2) { if (n == 1) b[0] = c[0] = d[0] = 0.0; return; }
    if (n < 3) {
        const double t = (y[1] - y[0]) / (x[1] - x[0]);
        b[0] = b[1] = t; c[0] = c[1] = d[0] = d[1] = 0.0;
        return;
    }
    const int nm1 = n - 1;
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
        const double d1 = c[2] / (x[3] - x[1]) - c[1] / (x[2] - x[0]);
        const double d2 = c[nm1 - 1] / (x[nm1] - x[n - 3]) - c[n - 3] / (x[nm1 - 1] - x[n - 4]);
        // third-derivative end conditions, d(1)**2 and d(n-1)**2 (FMM spline)
        c[0] = d1 * d[0] * d[0] / (x[3] - x[0]);
        c[nm1] = -(d2 * d[n - 2] * d[n - 2]) / (x[nm1] - x[n - 4]);
    }
    for (int i = 1; i < n; ++i) {
        const double t = d[i - 1] / b[i - 1];
        b[i] -= t * d[i - 1];
        c[i] -= t * c[i - 1];
    }
    c[nm1] /= b[nm1];
    for (int j = 0; j < nm1; ++j) {
        const int i = nm1 - j - 1;
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

// Device arena: one allocation per context, carved into aligned pieces.
struct Arena {
    char* base = nullptr;
    size_t size = 0, used = 0;
    std::vector<std::pair<size_t, std::vector<char>>> uploads;
    size_t reserve(size_t bytes) {
        size_t off = (used + 255) & ~size_t(255);
        used = off + bytes;
        return off;
    }
    template <class T>
    size_t put(const T* p, size_t n) {
        size_t off = reserve(sizeof(T) * std::max<size_t>(n, 1));
        std::vector<char> blob(sizeof(T) * std::max<size_t>(n, 1), 0);
        if (n) std::memcpy(blob.data(), p, sizeof(T) * n);
        uploads.emplace_back(off, std::move(blob));
        return off;
    }
};


// Which groups a lane role re-evaluates: the base lane all of them, a
// perturbed lane those that read its perturbed input (or the time, for the
// t0/tf directions).  MOCOHIP_TASKS=all disables the pruning (every group
// for every lane; the reference for the bit-identity test).
// nint > 0: the k_groups blocks are arranged for the XCDs (groups_xcd below):
// the tasks of the grid points whose intervals k_interval hands to XCD c
// (xcd_interval: one contiguous run of nint intervals per XCD; pts_per = 2
// Hermite-Simpson, 1 trapezoidal) run in blocks b with b % 8 = c.
// Stride-1 task sets put every group at its base slot, the prefix sum of
// GROUP_NF (the mass factor at 0): what eval_g's base-slot kernel
// (core.hpp TaskLoadBase) assumes at compile time.  Checked once per context.
static bool base_slots_match(const TaskInfo& ti, const TaskSet& ts) {
    int s = 0;
    for (int g = 0; g < ti.ng; ++g) {
        if (ts.jd[(size_t)g] != (g > 0 ? s : 0)) return false;
        if (g > 0) s += ti.group_nf[g];
    }
    return true;
}
static void build_taskset(const TaskInfo& ti, const Lanes& ln, int nk, int nsimd, TaskSet& ts,
        int nint = 0, int pts_per = 2) {
    const char* env = std::getenv("MOCOHIP_TASKS");
    const bool all = env && std::strcmp(env, "all") == 0;
    const int ng = ti.ng, S = ln.stride;
    ts.dlen.assign(ng, 0);
    ts.off.assign(ng, 0);
    ts.roles.assign((size_t)ng * S, 0);
    ts.jd.assign((size_t)ng * S + 1, 0);   // +1: whole doubles when staged to LDS
    int tdoubles = 0;
    for (int g = 0; g < ng; ++g) {
        std::vector<int> D{ln.base};
        for (int r = 0; r < S; ++r) {
            if (r == ln.base) continue;
            const int dir = (ln.fd == MH_FD_CENTRAL && r >= ln.ND) ? r - ln.ND : r;
            bool hit;
            if (dir < 2) hit = ti.time[g] != 0;
            else {
                const int i = dir - 2;
                hit = (ti.reads[(size_t)g * ti.rw + i / 64] >> (i % 64)) & 1ULL;
            }
            if (hit || all) D.push_back(r);
        }
        ts.dlen[g] = (int)D.size();
        // g > 0: T slab offset (doubles) of the group's slot j; g = 0: j of
        // the mass factor
        const int nf = g > 0 ? ti.group_nf[g] : 1;
        if (g > 0) ts.off[g] = tdoubles;
        // roles that do not re-evaluate g read its base-lane slot (j = 0)
        for (int r = 0; r < S; ++r) ts.jd[(size_t)r * ng + g] = g > 0 ? ts.off[g] : 0;
        for (size_t j = 0; j < D.size(); ++j) {
            ts.roles[(size_t)g * S + j] = D[j];
            ts.jd[(size_t)D[j] * ng + g] = (g > 0 ? ts.off[g] : 0) + (int)j * nf;
        }
        if (g > 0) tdoubles += (int)D.size() * nf;
    }
    // expensive groups first so they start before the cheap ones fill in
    std::vector<int> order(ng);
    for (int g = 0; g < ng; ++g) order[g] = g;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return ti.gflops[a] > ti.gflops[b];
    });
    ts.blk.clear();
    ts.flops = 0.0;
    ts.ntasks = 0.0;
    // timing diagnostic only (results invalid): launch group G's blocks alone
    const char* dg = std::getenv("MOCOHIP_DEBUG_GROUP");
    const int only = dg ? std::atoi(dg) : -1;
    // A block record is (group | live tasks << 16, first task, tasks per
    // grid point, 1 / tasks per grid point as float bits); its live tasks
    // are first .. first + live - 1 (live = 0: an empty padding block).
    auto push = [&](std::vector<int>& v, int g, long f, long cnt) {
        const float inv = 1.0f / (float)ts.dlen[g];
        int inv_bits;
        std::memcpy(&inv_bits, &inv, sizeof inv);
        v.push_back(g | (int)(cnt << 16)); v.push_back((int)f);
        v.push_back(ts.dlen[g]); v.push_back(inv_bits);
    };
    // groups_xcd: XCD c's grid points are [P[c], P[c + 1]) -- the points of
    // the intervals xcd_interval gives XCD c, a shared mesh point going to
    // the later run -- so XCD c's task waves read one contiguous run of x
    // (k_groups FETCH 6.55 -> 5.14 MB per launch, profiles/r05_ab).  The
    // group results do not stay in the writing XCD's L2 for k_interval:
    // its FETCH is the same in either order (7.48 MB), each launch starts
    // cold.  Per XCD the heavy groups' blocks lead, in the
    // same heaviest-first order; the lists are padded to equal heavy and
    // light lengths and interleaved (block b -> XCD b % 8 under the
    // hardware's round-robin dispatch; placement is speed only).
    const char* ex = std::getenv("MOCOHIP_GROUPS_XCD");
    const bool xcd = nint > 0 && only < 0 && !(ex && std::atoi(ex) == 0);
    std::vector<long> P(9, 0);
    if (xcd) {
        const int q = nint / 8, rem = nint % 8;
        for (int c = 0; c < 8; ++c) P[c] = (long)pts_per * (c * q + std::min(c, rem));
        P[8] = nk;
    }
    std::vector<int> lists[2][8];   // [heavy / light][XCD]
    for (int g : order) {
        if (only >= 0 && g != only) continue;
        const long n = (long)nk * ts.dlen[g];
        if (!xcd) {
            for (long f = 0; f < n; f += 64) push(ts.blk, g, f, std::min(64L, n - f));
        } else {
            for (int c = 0; c < 8; ++c) {
                const long a = P[c] * ts.dlen[g], e = P[c + 1] * ts.dlen[g];
                for (long f = a; f < e; f += 64) push(lists[g < ti.nheavy ? 0 : 1][c], g, f, std::min(64L, e - f));
            }
        }
        ts.flops += (double)n * ti.gflops[g];
        ts.ntasks += (double)n;
    }
    if (xcd) {
        for (int h = 0; h < 2; ++h) {
            size_t len = 0;
            for (int c = 0; c < 8; ++c) len = std::max(len, lists[h][c].size() / 4);
            const int gpad = h == 0 ? 0 : ti.ng - 1;   // a group of the class (heavy: 0)
            for (size_t s = 0; s < len; ++s)
                for (int c = 0; c < 8; ++c) {
                    if (s < lists[h][c].size() / 4)
                        ts.blk.insert(ts.blk.end(), lists[h][c].begin() + 4 * s, lists[h][c].begin() + 4 * s + 4);
                    else
                        push(ts.blk, gpad, 0, 0);
                }
        }
    }
    ts.flops += (double)nk * S * ti.combine_flops;
    ts.nblocks = (int)(ts.blk.size() / 4);
    // When the launch fits in two waves per SIMD, blocks p and p + nsimd
    // share a SIMD: order the second round ascending so the heaviest block
    // shares its SIMD with the lightest (MOCOHIP_ORDER=desc keeps plain
    // longest-first order).
    const char* eo = std::getenv("MOCOHIP_ORDER");
    const bool pair = !(eo && std::strcmp(eo, "desc") == 0) && !xcd;
    if (pair && ts.nblocks > nsimd && ts.nblocks <= 2 * nsimd) {
        for (int a = nsimd, b = ts.nblocks - 1; a < b; ++a, --b)
            for (int w = 0; w < 4; ++w) std::swap(ts.blk[4 * (size_t)a + w], ts.blk[4 * (size_t)b + w]);
    }
    // the heavy groups' blocks (groups < NHEAVY) as one leading run (k_groups_part)
    ts.nheavy = 0;
    while (ts.nheavy < ts.nblocks && (ts.blk[4 * (size_t)ts.nheavy] & 0xffff) < ti.nheavy) ++ts.nheavy;
    for (int b = ts.nheavy; b < ts.nblocks; ++b)
        if ((ts.blk[4 * (size_t)b] & 0xffff) < ti.nheavy) { ts.nheavy = -1; break; }
    ts.dev.ng = ng;
    ts.dev.stride = S;
    ts.dev.tdoubles = tdoubles;
    ts.dev.nmass = ts.dlen[0];
    ts.dev.nk = nk;
    ts.t_doubles = (size_t)nk * std::max(tdoubles, 1);
    ts.h_doubles = (size_t)nk * ts.dlen[0] * ti.nst;
}

struct TaskOffsets { size_t dlen, off, roles, jd, blk; };
static TaskOffsets put_taskset(Arena& A, const TaskSet& ts) {
    TaskOffsets o;
    o.dlen = A.put(ts.dlen.data(), ts.dlen.size());
    o.off = A.put(ts.off.data(), ts.off.size());
    o.roles = A.put(ts.roles.data(), ts.roles.size());
    o.jd = A.put(ts.jd.data(), ts.jd.size());
    o.blk = A.put(ts.blk.data(), ts.blk.size());
    return o;
}
static void bind_taskset(char* base, const TaskOffsets& o, TaskSet& ts) {
    ts.dev.dlen = (const int*)(base + o.dlen);
    ts.dev.off = (const int*)(base + o.off);
    ts.dev.roles = (const int*)(base + o.roles);
    ts.dev.jd = (const int*)(base + o.jd);
    ts.dev.blk = (const int4*)(base + o.blk);
}

}  // namespace


// Task tables and T/H buffers for an mh_eval_dae call of np points (kept
// until the next call with a different np).
int probe_tasks(mh_ctx* c, const TaskInfo& ti, const Lanes& ln, int np) {
    if (np == c->probe_np) return MH_OK;
    if (c->probe_mem) { (void)hipFree(c->probe_mem); c->probe_mem = nullptr; }
    c->probe_np = -1;
    build_taskset(ti, ln, np, c->nsimd, c->ts_probe);
    Arena A;
    const TaskOffsets to = put_taskset(A, c->ts_probe);
    const size_t oT = A.reserve(sizeof(double) * c->ts_probe.t_doubles);
    const size_t oH = A.reserve(sizeof(double) * c->ts_probe.h_doubles);
    HIPCHK(hipMalloc(&c->probe_mem, A.used));
    for (auto& up : A.uploads)
        HIPCHK(hipMemcpy(c->probe_mem + up.first, up.second.data(), up.second.size(),
                hipMemcpyHostToDevice));
    bind_taskset(c->probe_mem, to, c->ts_probe);
    c->d_pT = (double*)(c->probe_mem + oT);
    c->d_pH = (double*)(c->probe_mem + oH);
    c->probe_np = np;
    return MH_OK;
}

static int64_t col_state(const mh_ctx* c, int64_t k, int s) { return 2 + k * c->NS + s; }
static int64_t col_control(const mh_ctx* c, int64_t k, int j) {
    return 2 + (int64_t)c->NS * c->G + k * c->NC + j;
}
// Lagrange multipliers (NM x G) and slacks (NSL x mesh-interval midpoints)
// after the controls, then the "derivatives" (implicit mode: accelerations,
// implicit auxiliary derivatives) -- CasOCIterate.h:27-44 key order
static int64_t col_mult(const mh_ctx* c, int64_t k, int j) {
    return 2 + (int64_t)(c->NS + c->NC) * c->G + k * c->NM + j;
}
static int64_t col_slack(const mh_ctx* c, int64_t i, int l) {
    return 2 + (int64_t)(c->NS + c->NC + c->NM) * c->G + i * c->NSL + l;
}
static int64_t col_deriv(const mh_ctx* c, int64_t k, int j) {
    return 2 + (int64_t)(c->NS + c->NC + c->NM) * c->G + (int64_t)c->NSL * c->N + k * c->NDV + j;
}
// x column of per-point input j of grid point k: [states, controls,
// derivatives, multipliers, slacks (mesh-interval midpoints: the interval's)]
static int64_t col_input(const mh_ctx* c, int64_t k, int j) {
    if (j < c->NS) return col_state(c, k, j);
    j -= c->NS;
    if (j < c->NC) return col_control(c, k, j);
    j -= c->NC;
    if (j < c->NDV) return col_deriv(c, k, j);
    j -= c->NDV;
    if (j < c->NM) return col_mult(c, k, j);
    return col_slack(c, (k - 1) / 2, j - c->NM);
}

// x column of endpoint input si: [initial_time, initial point inputs,
// final_time, final point inputs] (EndpointEqs, CasOCFunction.h:167-240).
static int64_t ep_col(const mh_ctx* c, int si) {
    if (si >= 2 * (1 + c->NI)) return c->XP + (si - 2 * (1 + c->NI));   // parameter
    const int W = 1 + c->NI, pt = si / W, j = si % W - 1;
    if (j < 0) return pt;
    const int64_t k = pt ? c->G - 1 : 0;
    if (j < c->NS) return col_state(c, k, j);
    if (j < c->NS + c->NC) return col_control(c, k, j - c->NS);
    if (j < c->NS + c->NC + c->NDV) return col_deriv(c, k, j - c->NS - c->NC);
    return col_mult(c, k, j - c->NS - c->NC - c->NDV);
}

// Build the per-interval template in CasOC row order with columns sorted
// ascending (the block-dense structural rule), then
// (implicit mode) the tail template: the final grid point's residual rows,
// evaluated by the last interval.
static void build_template(mh_ctx* c) {
    const int NS = c->NS, NQ = c->TQ, NC = c->NC, NDV = c->NDV;   // NQ: coordinates among the states
    const bool implicit = c->NACC > 0;
    struct Col { int pt; int dir; };  // dir: 0/1 time, 2+input, 2+NI+p parameter p
    const int pdir = 2 + c->NI;       // direction of parameter 0
    auto key = [&](const Col& col) -> int64_t {
        // column index for interval 0
        if (col.dir < 2) return col.dir;
        if (col.dir >= pdir) return c->XP + (col.dir - pdir);
        return col_input(c, col.pt, col.dir - 2);
    };
    // time and parameter columns carry pt_time (the residual rows' grid
    // point; 0 otherwise) and the row's general (t0 / tf) kind: like a time
    // column, a parameter column reads the callbacks of every point of the row
    auto emit_row = [&](int row, uint8_t kind_t, uint8_t kind_x, int s, std::vector<Col> cols,
            int pt_time = 0) {
        std::sort(cols.begin(), cols.end(), [&](const Col& a, const Col& b) { return key(a) < key(b); });
        for (const auto& col : cols) {
            TplEntry e{};
            const bool gen = col.dir < 2 || col.dir >= pdir;
            e.row = (int16_t)row;
            e.kind = gen ? kind_t : kind_x;
            e.pt = (uint8_t)(gen ? pt_time : col.pt);
            e.dir = (int16_t)col.dir;
            e.s = (int16_t)s;
            c->tpl.push_back(e);
            c->tpl_col_pt.push_back(gen ? -1 : col.pt);
        }
    };
    // the parameters are inputs of every callback (ContinuousInput.parameters,
    // CasOCProblem.h:132-165): dense columns of each row that reads one
    auto param_dep = [&](std::vector<Col>& v) {
        for (int q = 0; q < c->NPAR; ++q) v.push_back({0, pdir + q});
    };
    // Inputs of point pt that callback output o reads: all of them without
    // sparsity detection (block-dense, CasOCFunction.cpp:25-105 "none"),
    // else the detected ones (sp: [output][time, inputs]); plus the point's
    // own state s_ident (the defects' identity terms).
    const int W = 1 + c->NI;                 // detected pattern: [time, every input]
    const int NPD = NS + NC + NDV + c->NM;   // callback inputs (no slacks)
    auto point_dep = [&](const std::vector<uint8_t>& sp, int o, int pt, int s_ident, std::vector<Col>& v) {
        for (int j = 0; j < NPD; ++j)
            if (sp.empty() || sp[(size_t)o * W + 1 + j] || j == s_ident) v.push_back({pt, 2 + j});
    };
    auto time_dep = [&](const std::vector<uint8_t>& sp, int o) { return sp.empty() || sp[(size_t)o * W] != 0; };
    // residual rows of point pt (multibody residuals in implicit mode, then
    // the implicit auxiliary residuals): the point's inputs + time; the
    // entry's s is the callback output
    auto residual_rows = [&](int& row, int pt) {
        for (int r = 0; r < c->NMB + c->NAR; ++r) {
            const int o = r < c->NMB ? r : c->NQ + c->NZ + (r - c->NMB);
            std::vector<Col> v;
            if (time_dep(c->sp, o)) { v.push_back({pt, 0}); v.push_back({pt, 1}); }
            point_dep(c->sp, o, pt, -1, v);
            param_dep(v);
            emit_row(row++, T_RES, T_RES, o, v, pt);
        }
    };
    // path-constraint rows of mesh point pt, like the residuals
    // (CasOCTranscription.cpp:419-433)
    auto path_rows = [&](int& row, int pt) {
        for (int e = 0; e < c->npc; ++e) {
            std::vector<Col> v;
            if (time_dep(c->sp_pc, e)) { v.push_back({pt, 0}); v.push_back({pt, 1}); }
            point_dep(c->sp_pc, e, pt, -1, v);
            param_dep(v);
            emit_row(row++, T_PATH, T_PATH, e, v, pt);
        }
    };
    // kinematic-constraint rows of mesh point pt (outputs OKC.. of the
    // multibody callback; block-dense over time and the point's inputs),
    // first among the mesh point's rows (CasOCTranscription.h:283-289)
    auto kc_rows = [&](int& row, int pt) {
        for (int r = 0; r < c->NK; ++r) {
            std::vector<Col> v{{pt, 0}, {pt, 1}};
            point_dep({}, 0, pt, -1, v);
            param_dep(v);
            emit_row(row++, T_RES, T_RES, c->OKC + r, v, pt);
        }
    };
    // implicit speed rows: udot = the acceleration variable (direct MX
    // expression, CasOCTranscription.cpp:339-341): own state + acceleration
    auto speed_sparse = [&](int s) { return implicit && s >= NQ && s < 2 * NQ; };
    const int adir = 2 + NS + NC;   // direction of acceleration 0
    int row = 0;
    if (c->scheme == MH_HERMITE_SIMPSON) {
        kc_rows(row, 0);
        path_rows(row, 0);
        residual_rows(row, 0);
        residual_rows(row, 1);
        for (int s = 0; s < NS; ++s) {
            std::vector<Col> v{{0, 0}, {0, 1}};
            if (s < NQ) {
                v.push_back({1, 2 + s}); v.push_back({0, 2 + s}); v.push_back({2, 2 + s});
                v.push_back({0, 2 + NQ + s}); v.push_back({2, 2 + NQ + s});
            } else if (speed_sparse(s)) {
                v.push_back({1, 2 + s}); v.push_back({0, 2 + s}); v.push_back({2, 2 + s});
                v.push_back({0, adir + s - NQ}); v.push_back({2, adir + s - NQ});
            } else {
                // callback output s + SO (explicit: udot / zdot; implicit /
                // prescribed: zdot after the NQ residuals)
                v.push_back({1, 2 + s});
                point_dep(c->sp, s + c->SO, 0, s, v); point_dep(c->sp, s + c->SO, 2, s, v);
                param_dep(v);
            }
            emit_row(row++, T_HERM_T, T_HERM_X, s, v);
        }
        for (int s = 0; s < NS; ++s) {
            std::vector<Col> v{{0, 0}, {0, 1}};
            if (s < NQ && c->NSL) {
                // qdot at the midpoint = u + G^T gamma: the velocity
                // correction reads the midpoint's q, u and the interval's
                // slacks (block-dense, CasOCTranscription.cpp:316-333)
                v.push_back({0, 2 + s}); v.push_back({2, 2 + s});
                v.push_back({0, 2 + NQ + s}); v.push_back({2, 2 + NQ + s});
                for (int j = 0; j < 2 * NQ; ++j) v.push_back({1, 2 + j});
                for (int l = 0; l < c->NSL; ++l) v.push_back({1, 2 + NPD + l});
                param_dep(v);
            } else if (s < NQ) {
                v.push_back({0, 2 + s}); v.push_back({2, 2 + s});
                v.push_back({0, 2 + NQ + s}); v.push_back({1, 2 + NQ + s}); v.push_back({2, 2 + NQ + s});
            } else if (speed_sparse(s)) {
                v.push_back({0, 2 + s}); v.push_back({2, 2 + s});
                v.push_back({0, adir + s - NQ}); v.push_back({1, adir + s - NQ}); v.push_back({2, adir + s - NQ});
            } else {
                point_dep(c->sp, s + c->SO, 0, s, v); point_dep(c->sp, s + c->SO, 1, -1, v);
                point_dep(c->sp, s + c->SO, 2, s, v);
                param_dep(v);
            }
            emit_row(row++, T_SIMP_T, T_SIMP_X, s, v);
        }
        if (c->interp) {
            for (int j = 0; j < NC; ++j) {
                std::vector<Col> v{{0, 2 + NS + j}, {1, 2 + NS + j}, {2, 2 + NS + j}};
                emit_row(row++, T_INTERP, T_INTERP, j, v);
            }
        }
    } else {
        kc_rows(row, 0);
        path_rows(row, 0);
        residual_rows(row, 0);
        for (int s = 0; s < NS; ++s) {
            std::vector<Col> v{{0, 0}, {0, 1}};
            if (s < NQ) {
                v.push_back({0, 2 + s}); v.push_back({1, 2 + s});
                v.push_back({0, 2 + NQ + s}); v.push_back({1, 2 + NQ + s});
            } else if (speed_sparse(s)) {
                v.push_back({0, 2 + s}); v.push_back({1, 2 + s});
                v.push_back({0, adir + s - NQ}); v.push_back({1, adir + s - NQ});
            } else {
                point_dep(c->sp, s + c->SO, 0, s, v); point_dep(c->sp, s + c->SO, 1, s, v);
                param_dep(v);
            }
            emit_row(row++, T_TRAP_T, T_TRAP_X, s, v);
        }
    }
    c->rpi = row;
    c->nnz_int = (int)c->tpl.size();
    // tail: path rows of the final mesh point, then residual rows of the
    // last grid point (point 2 of the HS interval, 1 of the trapezoidal one),
    // rows rpi.. relative to the last interval
    kc_rows(row, c->scheme == MH_HERMITE_SIMPSON ? 2 : 1);
    path_rows(row, c->scheme == MH_HERMITE_SIMPSON ? 2 : 1);
    residual_rows(row, c->scheme == MH_HERMITE_SIMPSON ? 2 : 1);
    c->nnz_tail = (int)c->tpl.size() - c->nnz_int;
    c->ntail = row - c->rpi;
    c->npe = 0;
    for (int e = 0; e < c->nnz_int; ++e) c->npe += c->tpl[e].kind == T_PATH;
    // the head: each endpoint equation's row over its inputs (all of them
    // without detection, Endpoint callback dense Jacobian; else the detected
    // ones), columns ascending (the initial and the final point's blocks
    // interleave per variable kind)
    c->eptpl.clear();
    const int WE = 2 * W;
    for (int e = 0; e < c->nep; ++e) {
        std::vector<std::pair<int64_t, int>> cols;
        for (int si = 0; si < WE; ++si)
            if (c->sp_ep.empty() || c->sp_ep[(size_t)e * WE + si]) cols.push_back({ep_col(c, si), si});
        for (int q = 0; q < c->NPAR; ++q) cols.push_back({ep_col(c, WE + q), WE + q});   // the parameters
        std::sort(cols.begin(), cols.end());
        for (const auto& cs : cols) {
            TplEntry t{};
            t.row = (int16_t)e;
            t.kind = T_EP;
            t.dir = (int16_t)cs.second;
            t.s = (int16_t)e;
            c->eptpl.push_back(t);
        }
    }
    c->nnz_ep = (int)c->eptpl.size();
}

// k_interval writes the path-constraint entries in a loop of their own over
// the first npc * (2 + NI) entries of the interval and of the tail.
static bool path_entries_lead(const mh_ctx* c) {
    const int npe = c->npe;
    if (npe > c->nnz_int || npe > c->nnz_tail) return c->npc == 0;
    for (int e = 0; e < (int)c->tpl.size(); ++e) {
        const bool lead = e < npe || (e >= c->nnz_int && e < c->nnz_int + npe);
        if ((c->tpl[e].kind == T_PATH) != lead) return false;
    }
    return true;
}

// k_transcribe's base-lane offsets derived from the words instead of read
// from the table after them (default; MOCOHIP_DBASE=0 reads the table),
// enabled only where the derivation equals the table entry for entry:
// configs[3] 1,605 -> 1,628 calls/s (profiles/r06_c; the table read shares
// the word's dependency chain).  (Non-temporal value stores were measured
// too: no difference.)  Called again after a detected template replaces the
// block-dense one.
static void setup_assembly_variants(mh_ctx* c) {
    const char* ed = std::getenv("MOCOHIP_DBASE");
    const uint32_t stride = (uint32_t)c->lanes_jac.stride;
    c->iv_sstride = stride;
    c->iv_sbase = (uint32_t)c->lanes_jac.base;
    c->iv_smagic = (uint32_t)(0xFFFFFFFFull / stride + 1);
    c->iv_dbase = 0;
    // k_transcribe's quotients by div_rn, opt-in (MOCOHIP_QDIV=1): the same
    // bits as the division, measured no faster (configs[3] 1,720 vs 1,729
    // calls/s, profiles/r06_n -- the kernel waits on memory, not on the
    // division); its range: the step (and twice it) within [2^-60, 2^60]
    const char* eq = std::getenv("MOCOHIP_QDIV");
    const double hs = c->lanes_jac.h;
    c->iv_qdiv = eq && std::strcmp(eq, "1") == 0 && hs >= 0x1p-60 && hs <= 0x1p+59;
    if (!(ed && std::strcmp(ed, "0") == 0) && !c->ctpl.empty() && c->lanes_jac.fd != MH_FD_CENTRAL) {
        const size_t nw = (size_t)c->nnz_int + (size_t)c->nnz_tail;
        const int npts = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
        const uint32_t nyall = (uint32_t)(npts * c->NO) * stride;
        bool ok = c->ctpl.size() >= 2 * nw && nyall < (1u << 20);
        for (size_t e = 0; ok && e < nw; ++e) {
            const uint32_t w = c->ctpl[e], off = w & CT_OFF;
            const bool lane = !(w & (CT_GEN | CT_PATH)) && off < nyall;
            const uint32_t d = lane ? (uint32_t)(((uint64_t)off * c->iv_smagic) >> 32) * stride + c->iv_sbase : 0u;
            ok = d == c->ctpl[nw + e];
        }
        c->iv_dbase = ok ? 1 : 0;
    }
}

// Excitation lanes filled by k_exc_fill (c->exc_xs: [lane, slot, output]
// triplets): every output of such a lane but its activation derivative is a
// copy of the base lane's, so a template word that reads one of them reads
// the base lane instead -- the quotient (y_base - y_base) / h is the same
// bits (+0, or NaN where y_base is not finite) -- and the fill then writes
// the activation derivatives only (k_exc_fill_adot).  Forward / backward
// differences (a central word also reads its mirror lane at off + ND);
// MOCOHIP_EXC_REDIRECT=0 turns it off.  Returns the words changed (the
// caller uploads them).
static long redirect_exc_words(mh_ctx* c) {
    c->exc_redirected = false;
    const char* e = std::getenv("MOCOHIP_EXC_REDIRECT");
    if (c->exc_xs.empty() || c->lanes_jac.fd == MH_FD_CENTRAL || (e && std::strcmp(e, "0") == 0)) return 0;
    // quotients formed in place (k_combine's MOCOHIP_QUOT=1, k_interval's
    // MOCOHIP_IV_QFUSE=0) leave the base lane raw: its slot is no quotient
    if (c->quot || !c->iv_qfuse) return 0;
    const uint32_t stride = (uint32_t)c->lanes_jac.stride, base = (uint32_t)c->lanes_jac.base;
    const int npts = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
    const uint32_t nyall = (uint32_t)(npts * c->NO) * stride;
    std::vector<int> adot(stride, -2);   // lane -> its filled output (-2: not an excitation lane)
    for (size_t k = 0; k + 2 < c->exc_xs.size(); k += 3) adot[c->exc_xs[k]] = c->exc_xs[k + 2];
    const size_t nw = (size_t)c->nnz_int + (size_t)c->nnz_tail;
    long changed = 0;
    for (size_t i = 0; i < nw && i < c->ctpl.size(); ++i) {
        uint32_t& w = c->ctpl[i];
        const uint32_t off = w & CT_OFF;
        if ((w & (CT_GEN | CT_PATH)) || off >= nyall) continue;
        const uint32_t lane = off % stride;
        const int o = (int)((off / stride) % (uint32_t)c->NO);
        if (adot[lane] == -2 || adot[lane] == o) continue;
        w = (w & ~(uint32_t)CT_OFF) | (off - lane + base);
        ++changed;
    }
    c->exc_redirected = true;
    return changed;
}

// The compiled template (core.hpp CT_*) of c->tpl for the Jacobian lane
// layout: per entry the LDS offset of the quotient (or constant) it scales,
// its coefficient and base -- the operations jac_entry performs for it.
static bool compile_template(mh_ctx* c) {
    const int NS = c->NS, NQ = c->TQ, NC = c->NC, NO = c->NO;
    const int ND = c->NI + 2 + c->NPAR;   // directions: t0, tf, point inputs, parameters
    const int stride = c->fd == MH_FD_CENTRAL ? 2 * ND + 1 : ND + 1;
    const int npts = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
    const uint32_t kconst = (uint32_t)(npts * NO * stride + CT_CONST);   // sK relative to sY
    if ((size_t)kconst + CT_NCONST > CT_OFF) return false;
    // LDS offset of dxdot[s] along direction dir at point pt (jac_entry's
    // dxdot: exact 0 / 1 for qdot = u and implicit udot = w)
    auto dx = [&](int pt, int s, int dir) -> uint32_t {
        if (s < NQ) return kconst + (dir == 2 + NQ + s ? 1u : 0u);
        if (c->NACC && s < 2 * NQ) return kconst + (dir == 2 + NS + NC + (s - NQ) ? 1u : 0u);
        return (uint32_t)((pt * NO + s + c->SO) * stride + dir);
    };
    c->ctpl.clear();
    for (const TplEntry& T : c->tpl) {
        const int s = T.s, dir = T.dir, pt = T.pt;
        const bool ident = dir == 2 + s;
        uint32_t w;
        switch (T.kind) {
        case T_HERM_X:
            if (pt == 1) w = ct_word(kconst, 0, ident ? 2 : 0);
            else w = ct_word(dx(pt, s, dir), pt == 0 ? 1 : 2, ident ? 1 : 0);
            break;
        case T_SIMP_X:
            if (pt == 2) w = ct_word(dx(pt, s, dir), 3, ident ? 2 : 0);
            else if (pt == 0) w = ct_word(dx(pt, s, dir), 3, ident ? 3 : 0);
            else if (s < NQ && c->NSL > 0) {
                // the midpoint's qdot = u + G^T gamma (velocity correction,
                // CasOCTranscription.cpp:316-333): dxdot = [dir is u_s] +
                // the correction output's quotient; with the exact 1 it takes
                // the general path
                if (dir == 2 + NQ + s) w = CT_GEN;
                else w = ct_word((uint32_t)((pt * NO + c->OQC + s) * stride + dir), 4, 0);
            } else w = ct_word(dx(pt, s, dir), 4, 0);
            break;
        case T_TRAP_X:
            w = ct_word(dx(pt, s, dir), 5, ident ? (pt == 1 ? 2 : 3) : 0);
            break;
        case T_INTERP:
            w = ct_word(kconst, 0, pt == 1 ? 2 : 1);
            break;
        case T_RES:
            w = (uint32_t)((pt * NO + s) * stride + dir) | CT_RAW;
            break;
        case T_PATH:
            w = CT_PATH;
            break;
        default:   // along t0 / tf (HERM_T, SIMP_T, TRAP_T)
            w = CT_GEN;
        }
        c->ctpl.push_back(w);
    }
    c->ctgen.clear();
    for (int e = 0; e < c->nnz_int + c->nnz_tail; ++e)
        if (c->ctpl[e] & CT_GEN) c->ctgen.push_back(e);
    // after the words, per entry the LDS offset of its row's base lane (the
    // forward / backward quotient's y(x) in the assembly; 0 where unused):
    // read with the word instead of dividing the offset by the stride
    const size_t nw = c->ctpl.size();
    if (nw != (size_t)c->nnz_int + (size_t)c->nnz_tail) return false;
    const uint32_t nyall = (uint32_t)(npts * NO * stride);
    const int base = stride - 1;   // the base lane closes a point's lanes (Lanes, mh_create)
    for (size_t e = 0; e < nw; ++e) {
        const uint32_t w = c->ctpl[e];
        const uint32_t off = w & CT_OFF;
        const bool lane = !(w & (CT_GEN | CT_PATH)) && off < nyall;
        c->ctpl.push_back(lane ? off / (uint32_t)stride * (uint32_t)stride + (uint32_t)base : 0u);
    }
    // k_role lists: entry e goes to the role of its point, its word against
    // that role's own-point layout (q at o * stride + dir)
    const int R = npts;
    const uint32_t rconst = (uint32_t)role_kconst(NO, stride, R);
    auto rdx = [&](int s, int dir) -> uint32_t {
        if (s < NQ) return rconst + (dir == 2 + NQ + s ? 1u : 0u);
        if (c->NACC && s < 2 * NQ) return rconst + (dir == 2 + NS + NC + (s - NQ) ? 1u : 0u);
        return (uint32_t)((s + c->SO) * stride + dir);
    };
    auto rword = [&](const TplEntry& T) -> uint32_t {
        const int s = T.s, dir = T.dir, pt = T.pt;
        const bool ident = dir == 2 + s;
        switch (T.kind) {
        case T_HERM_X:
            if (pt == 1) return ct_word(rconst, 0, ident ? 2 : 0);
            return ct_word(rdx(s, dir), pt == 0 ? 1 : 2, ident ? 1 : 0);
        case T_SIMP_X:
            if (pt == 2) return ct_word(rdx(s, dir), 3, ident ? 2 : 0);
            if (pt == 0) return ct_word(rdx(s, dir), 3, ident ? 3 : 0);
            return ct_word(rdx(s, dir), 4, 0);
        case T_TRAP_X: return ct_word(rdx(s, dir), 5, ident ? (pt == 1 ? 2 : 3) : 0);
        case T_INTERP: return ct_word(rconst, 0, pt == 1 ? 2 : 1);
        case T_RES: return (uint32_t)(s * stride + dir) | CT_RAW;
        default: return CT_GEN;
        }
    };
    if ((size_t)rconst + 2 > CT_OFF) return false;
    c->rl_e.clear();
    c->rl_w.clear();
    for (int r = 0; r < R; ++r) {
        c->rl_off[r] = (int)c->rl_e.size();
        for (int e = 0; e < c->nnz_int; ++e) {
            const TplEntry& T = c->tpl[e];
            if (T.kind == T_PATH || T.pt != r) continue;
            const uint32_t w = rword(T);
            if (w & CT_GEN) continue;   // t0 / tf columns: the time role's jac_entry loop
            c->rl_e.push_back(e);
            c->rl_w.push_back(w);
        }
    }
    c->rl_off[R] = (int)c->rl_e.size();
    for (int r = R + 1; r < 4; ++r) c->rl_off[r] = c->rl_off[R];
    c->rl_tail[0] = (int)c->rl_e.size();
    for (int e = c->nnz_int; e < c->nnz_int + c->nnz_tail; ++e) {
        const TplEntry& T = c->tpl[e];
        if (T.kind == T_PATH) continue;
        if (T.pt != R - 1) return false;
        c->rl_e.push_back(e);
        c->rl_w.push_back(rword(T));
    }
    c->rl_tail[1] = (int)c->rl_e.size();
    return true;
}

static const int kZeroInt = 0;

// The objective partial of a shard (mh_eval_f_partial): the quadrature
// weights of the shard's own mesh intervals, accumulated exactly as the
// whole problem's are (CasOCHermiteSimpson.cpp:36-43, CasOCTrapezoidal.cpp:
// 26-37), so an unsharded context's partial IS its objective, bit for bit,
// and the shards' partials sum to it.
static void shard_quadrature(mh_ctx* c) {
    c->quadp.assign(c->G, 0.0);
    for (int i = c->ib; i < c->ie; ++i) {
        const double dm = (i + 1) / (double)c->N - i / (double)c->N;
        if (c->scheme == MH_HERMITE_SIMPSON) {
            c->quadp[2 * i] += (1.0 / 6.0) * dm;
            c->quadp[2 * i + 1] += (2.0 / 3.0) * dm;
            c->quadp[2 * i + 2] += (1.0 / 6.0) * dm;
        } else {
            c->quadp[i] += 0.5 * dm;
            c->quadp[i + 1] += 0.5 * dm;
        }
    }
}

static int validate_and_layout(mh_ctx* c, const mh_problem* p, const mh_options* o,
        std::vector<int>& coord_body, std::vector<int>& act_state, std::vector<int>& ftn_state,
        std::vector<int>& mus_control, double& tau_act, double& tau_deact) {
    const mh_model& M = p->model;
    if (M.nq < 0 || M.nbodies < 0 || M.nmuscles < 0 || M.nactuators < 0)
        return set_err(MH_ERR_INVALID, "negative model counts");
    if (o->num_mesh_intervals < 1) return set_err(MH_ERR_INVALID, "num_mesh_intervals must be >= 1");
    if (o->transcription != MH_HERMITE_SIMPSON && o->transcription != MH_TRAPEZOIDAL)
        return set_err(MH_ERR_INVALID, "unknown transcription scheme %d", o->transcription);
    if (o->finite_difference_scheme < 0 || o->finite_difference_scheme > 2)
        return set_err(MH_ERR_INVALID, "unknown finite difference scheme");
    c->NQ = M.nq;
    int z = 2 * M.nq;
    tau_act = tau_deact = NAN;
    act_state.resize(M.nmuscles);
    ftn_state.resize(M.nmuscles);
    mus_control.assign(M.nmuscles, -1);
    for (int im = 0; im < M.nmuscles; ++im) {
        const mh_muscle& mu = M.muscles[im];
        if (mu.point_begin < 0 || mu.point_begin + mu.point_count > M.npoints)
            return set_err(MH_ERR_INVALID, "muscle %d: bad path point range", im);
        act_state[im] = mu.ignore_activation_dynamics ? -1 : z++;
        ftn_state[im] = mu.ignore_tendon_compliance ? -1 : z++;
        // DeGrooteFregly2016Muscle.cpp:194-195 static time constants.
        if (!mu.ignore_activation_dynamics && std::isnan(tau_act)) {
            tau_act = mu.activation_time_constant;
            tau_deact = mu.deactivation_time_constant;
        }
    }
    c->NS = z;
    c->NZ = z - 2 * M.nq;
    c->NC = M.nactuators;
    c->NO = c->NQ + c->NZ;
    if (o->multibody_dynamics_mode != MH_DYNAMICS_EXPLICIT && o->multibody_dynamics_mode != MH_DYNAMICS_IMPLICIT)
        return set_err(MH_ERR_INVALID, "unknown multibody dynamics mode %d", o->multibody_dynamics_mode);
    // derivative variables: accelerations, then the implicit auxiliary
    // derivatives in component order (MocoCasOCProblem.cpp:85-94)
    // prescribed kinematics (PositionMotion): q, u not NLP states, no
    // acceleration variables, nq multibody residual rows per point
    c->presc = p->prescribed_kinematics ? 1 : 0;
    if (c->presc) {
        if (o->multibody_dynamics_mode != MH_DYNAMICS_IMPLICIT)
            return set_err(MH_ERR_INVALID, "Prescribed kinematics (PositionMotion) requires implicit dynamics mode.");
        if (p->kinematics_table < 0 || p->kinematics_table >= M.ntables || !p->kinematics_column)
            return set_err(MH_ERR_INVALID, "bad kinematics table");
        c->kin_table = p->kinematics_table;
        c->kin_col.assign(p->kinematics_column, p->kinematics_column + M.nq);
        for (int j = 0; j < M.nq; ++j)
            if (c->kin_col[j] < 0 || c->kin_col[j] >= M.tables[c->kin_table].ncol)
                return set_err(MH_ERR_INVALID, "kinematics column %d out of range", j);
        c->NS = c->NZ;
    }
    c->TQ = c->presc ? 0 : c->NQ;
    c->SO = c->presc ? c->NQ : -c->NQ;
    c->NACC = o->multibody_dynamics_mode == MH_DYNAMICS_IMPLICIT && !c->presc ? c->NQ : 0;
    c->NMB = o->multibody_dynamics_mode == MH_DYNAMICS_IMPLICIT ? c->NQ : 0;
    c->NAR = 0;
    c->mus_ider.assign(M.nmuscles, -1);
    for (int im = 0; im < M.nmuscles; ++im)
        if (M.muscles[im].tendon_dynamics_implicit && !M.muscles[im].ignore_tendon_compliance)
            c->mus_ider[im] = c->NACC + c->NAR++;
    c->NDV = c->NACC + c->NAR;
    c->NO = c->NQ + c->NZ + c->NAR;
    if (o->implicit_aux_bounds[0] != 0.0 || o->implicit_aux_bounds[1] != 0.0) {
        c->aux_lo = o->implicit_aux_bounds[0];
        c->aux_hi = o->implicit_aux_bounds[1];
    }
    if (o->implicit_accel_bounds[0] != 0.0 || o->implicit_accel_bounds[1] != 0.0) {
        c->acc_lo = o->implicit_accel_bounds[0];
        c->acc_hi = o->implicit_accel_bounds[1];
    }
    // kinematic constraints (MocoCasOCProblem.cpp:96-215)
    const int NKC = M.nconstraints;
    if (NKC < 0 || (NKC > 0 && !M.constraints)) return set_err(MH_ERR_INVALID, "bad kinematic constraints");
    c->kcs.assign(M.constraints, M.constraints + NKC);
    for (int i = 0; i < NKC; ++i) {
        const mh_constraint& K = c->kcs[i];
        const int f = K.func;
        if (K.kind != MH_KC_COORDINATE_COUPLER || f < 0 || f >= M.nfunctions ||
                M.functions[f].kind == MH_FN_CONSTANT || M.functions[f].coord < 0 ||
                M.functions[f].coord >= M.nq || K.dependent < 0 || K.dependent >= M.nq ||
                K.dependent == M.functions[f].coord)
            return set_err(MH_ERR_INVALID, "kinematic constraint %d: bad kind/function/coordinate", i);
    }
    // prescribed kinematics: multipliers (constraint forces in the residual),
    // no kinematic rows, no slacks (CasOCProblem.h:508-521)
    if (NKC && !c->presc && (p->nendpoint > 0 || o->sparsity_detection != MH_SPARSITY_NONE))
        return set_err(MH_ERR_UNSUPPORTED, "kinematic constraints (without prescribed kinematics) with "
                       "endpoint constraints or sparsity detection");
    if (o->minimize_lagrange_multipliers && !NKC)   // MocoCasOCProblem.cpp:101-107
        return set_err(MH_ERR_INVALID, "Solver property 'minimize_lagrange_multipliers' was enabled but no "
                       "enabled kinematic constraints exist in the model.");
    // the goals as the device sees them: the problem's, then (minimize_
    // lagrange_multipliers, CasOCTranscription.cpp:513-521) the multiplier term
    c->goals.assign(p->goals, p->goals + p->ngoals);
    c->gidx.assign(p->goal_index, p->goal_index + p->nterms);
    c->gcol.assign(p->goal_column, p->goal_column + p->nterms);
    c->gw.assign(p->goal_weight, p->goal_weight + p->nterms);
    if (o->minimize_lagrange_multipliers) {
        mh_goal G{};
        G.kind = MH_GOAL_LAGRANGE_MULTIPLIERS;
        G.term_begin = p->nterms;
        G.term_count = NKC;
        G.weight = o->lagrange_multiplier_weight != 0.0 ? o->lagrange_multiplier_weight : 1.0;
        c->goals.push_back(G);
        for (int j = 0; j < NKC; ++j) { c->gidx.push_back(j); c->gcol.push_back(0); c->gw.push_back(1.0); }
    }
    c->NKC = NKC;
    c->enforce = !o->ignore_constraint_derivatives;
    c->NM = NKC;
    c->NK = c->presc ? 0 : (c->enforce ? 3 * NKC : NKC);
    c->NSL = !c->presc && c->enforce && o->transcription == MH_HERMITE_SIMPSON ? NKC : 0;
    c->OKC = c->NQ + c->NZ + c->NAR;
    c->OQC = c->OKC + c->NK;
    c->NO = c->OQC + (c->NSL ? c->NQ : 0);
    if (!std::isnan(p->multiplier_bounds.lower) || !std::isnan(p->multiplier_bounds.upper)) {
        c->mult_lo = p->multiplier_bounds.lower; c->mult_hi = p->multiplier_bounds.upper;
    }
    if (!std::isnan(p->kinematic_constraint_bounds.lower) || !std::isnan(p->kinematic_constraint_bounds.upper)) {
        c->kc_lo = p->kinematic_constraint_bounds.lower; c->kc_hi = p->kinematic_constraint_bounds.upper;
    }
    if (o->velocity_correction_bounds[0] != 0.0 || o->velocity_correction_bounds[1] != 0.0) {
        c->vc_lo = o->velocity_correction_bounds[0]; c->vc_hi = o->velocity_correction_bounds[1];
    }
    c->NI = c->NS + c->NC + c->NDV + c->NM + c->NSL;
    if (p->npath < 0 || (p->npath > 0 && !p->path)) return set_err(MH_ERR_INVALID, "bad path constraints");
    c->npc = p->npath;
    c->pc.assign(p->path, p->path + p->npath);
    for (int e = 0; e < c->npc; ++e) {
        const mh_path_equation& E = c->pc[e];
        if (E.kind != MH_PATH_CONTROL_BOUND)
            return set_err(MH_ERR_UNSUPPORTED, "path equation %d: kind %d", e, E.kind);
        if (E.index < 0 || E.index >= c->NC || E.table < -1 || E.table >= M.ntables ||
                (E.table >= 0 && (E.column < 0 || E.column >= M.tables[E.table].ncol)))
            return set_err(MH_ERR_INVALID, "path equation %d: bad control/table", e);
    }
    if (p->nendpoint < 0 || (p->nendpoint > 0 && !p->endpoint))
        return set_err(MH_ERR_INVALID, "bad endpoint constraints");
    c->nep = p->nendpoint;
    c->ep.assign(p->endpoint, p->endpoint + p->nendpoint);
    for (int e = 0; e < c->nep; ++e) {
        const mh_endpoint_equation& E = c->ep[e];
        if (E.kind != MH_ENDPOINT_INITIAL_ACTIVATION)
            return set_err(MH_ERR_UNSUPPORTED, "endpoint equation %d: kind %d", e, E.kind);
        if (E.index_a < 0 || E.index_a >= c->NC || E.index_b < 0 || E.index_b >= c->NS)
            return set_err(MH_ERR_INVALID, "endpoint equation %d: bad control/state", e);
    }
    for (int ia = 0; ia < M.nactuators; ++ia) {
        const mh_actuator& a = M.actuators[ia];
        if (a.kind == MH_ACT_MUSCLE) {
            if (a.target < 0 || a.target >= M.nmuscles) return set_err(MH_ERR_INVALID, "actuator %d: bad muscle", ia);
            mus_control[a.target] = ia;
        } else if (a.kind == MH_ACT_COORDINATE) {
            if (a.target < 0 || a.target >= M.nq) return set_err(MH_ERR_INVALID, "actuator %d: bad coordinate", ia);
        } else {
            return set_err(MH_ERR_INVALID, "actuator %d: bad kind", ia);
        }
    }
    for (int im = 0; im < M.nmuscles; ++im)
        if (mus_control[im] < 0) return set_err(MH_ERR_INVALID, "muscle %d has no actuator", im);
    coord_body.assign(M.nq, -1);
    for (int b = 0; b < M.nbodies; ++b) {
        const mh_body& B = M.bodies[b];
        if (B.parent >= b || B.parent < -1) return set_err(MH_ERR_INVALID, "body %d not topologically ordered", b);
        if (B.axis_begin < 0 || B.axis_begin + B.axis_count > M.naxes) return set_err(MH_ERR_INVALID, "body %d: bad axes", b);
        for (int a = B.axis_begin; a < B.axis_begin + B.axis_count; ++a) {
            const int f = M.axes[a].func;
            if (f < 0 || f >= M.nfunctions) return set_err(MH_ERR_INVALID, "axis %d: bad function", a);
            const mh_function& F = M.functions[f];
            if (F.kind == MH_FN_CONSTANT) continue;
            if (F.coord < 0 || F.coord >= M.nq) return set_err(MH_ERR_INVALID, "axis %d: bad coordinate", a);
            if (coord_body[F.coord] >= 0 && coord_body[F.coord] != b)
                return set_err(MH_ERR_UNSUPPORTED, "coordinate %d drives axes of two bodies", F.coord);
            coord_body[F.coord] = b;
        }
    }
    for (int j = 0; j < M.nq; ++j)
        if (coord_body[j] < 0) return set_err(MH_ERR_INVALID, "coordinate %d drives no axis", j);
    for (int f = 0; f < M.nfunctions; ++f) {
        const mh_function& F = M.functions[f];
        if (F.kind == MH_FN_SIMMSPLINE &&
                (F.knot_count < 1 || F.knot_begin < 0 || F.knot_begin + F.knot_count > M.nknots))
            return set_err(MH_ERR_INVALID, "function %d: bad knots", f);
        if (F.kind != MH_FN_CONSTANT && (F.coord < 0 || F.coord >= M.nq))
            return set_err(MH_ERR_INVALID, "function %d: bad coordinate", f);
    }
    for (int i = 0; i < M.npoints; ++i) {
        const mh_path_point& pt = M.points[i];
        if (pt.body < -1 || pt.body >= M.nbodies) return set_err(MH_ERR_INVALID, "path point %d: bad body", i);
        if (pt.kind == MH_PP_CONDITIONAL && (pt.coord < 0 || pt.coord >= M.nq))
            return set_err(MH_ERR_INVALID, "path point %d: bad coordinate", i);
    }
    // wrap surfaces and PathWraps (grouped by muscle, at most 8 per muscle)
    if (M.nwraps < 0 || M.npathwraps < 0 || (M.nwraps > 0 && !M.wraps) || (M.npathwraps > 0 && !M.pathwraps))
        return set_err(MH_ERR_INVALID, "bad wrap objects");
    for (int i = 0; i < M.nwraps; ++i) {
        const mh_wrap_object& W = M.wraps[i];
        if (W.kind != MH_WRAP_CYLINDER || W.body < -1 || W.body >= M.nbodies || !(W.radius > 0.0) ||
                W.wrap_axis < 0 || W.wrap_axis > 1 || W.wrap_sign < -1 || W.wrap_sign > 1)
            return set_err(MH_ERR_INVALID, "wrap object %d: bad kind/body/radius/quadrant", i);
    }
    c->mus_pw_begin.assign(M.nmuscles, 0);
    c->mus_pw_count.assign(M.nmuscles, 0);
    for (int k = 0; k < M.npathwraps; ++k) {
        const mh_path_wrap& W = M.pathwraps[k];
        if (W.muscle < 0 || W.muscle >= M.nmuscles || W.wrap < 0 || W.wrap >= M.nwraps ||
                (k > 0 && W.muscle < M.pathwraps[k - 1].muscle))
            return set_err(MH_ERR_INVALID, "path wrap %d: bad muscle/wrap or not grouped by muscle", k);
        if (c->mus_pw_count[W.muscle]++ == 0) c->mus_pw_begin[W.muscle] = k;
        if (c->mus_pw_count[W.muscle] > 8)
            return set_err(MH_ERR_UNSUPPORTED, "muscle %d: more than 8 PathWraps", W.muscle);
    }
    // goals: kind, term range, and every term index within its kind's range
    // (a bad index would be an out-of-bounds device read)
    for (int g = 0; g < p->ngoals; ++g) {
        const mh_goal& G = p->goals[g];
        if (G.kind < MH_GOAL_CONTROL || G.kind > MH_GOAL_MARKER_FINAL)
            return set_err(MH_ERR_INVALID, "goal %d: unknown kind %d", g, G.kind);
        if (G.term_begin < 0 || G.term_count < 0 || G.term_begin + G.term_count > p->nterms ||
                (G.kind == MH_GOAL_MARKER_FINAL && G.term_count != 6))
            return set_err(MH_ERR_INVALID, "goal %d: bad terms", g);
        if (G.kind == MH_GOAL_STATE_TRACKING && (G.table < 0 || G.table >= M.ntables))
            return set_err(MH_ERR_INVALID, "goal %d: bad table", g);
        if (G.kind == MH_GOAL_MARKER_FINAL && (c->presc || M.nq > MH_MARKER_MAX_Q))
            return set_err(MH_ERR_UNSUPPORTED, "goal %d: marker goal needs coordinate states (<= %d)", g,
                    MH_MARKER_MAX_Q);
        for (int k = G.term_begin; k < G.term_begin + G.term_count; ++k) {
            const int idx = p->goal_index[k];
            int hi;
            switch (G.kind) {
            case MH_GOAL_CONTROL: hi = c->NC; break;
            case MH_GOAL_STATE_TRACKING: case MH_GOAL_SUM_SQUARED_STATE: hi = c->NS; break;
            case MH_GOAL_AUX_DERIVATIVES: hi = c->NAR; break;
            case MH_GOAL_MARKER_FINAL: hi = M.nbodies; break;
            default: hi = INT32_MAX; break;   // final time: no terms read
            }
            if (idx < (G.kind == MH_GOAL_MARKER_FINAL ? -1 : 0) || idx >= hi)
                return set_err(MH_ERR_INVALID, "goal %d: term %d index %d out of range", g, k, idx);
            if (G.kind == MH_GOAL_STATE_TRACKING &&
                    (p->goal_column[k] < 0 || p->goal_column[k] >= M.tables[G.table].ncol))
                return set_err(MH_ERR_INVALID, "goal %d: term %d column out of range", g, k);
        }
    }
    for (int e = 0; e < M.nexternal; ++e) {
        const mh_external_force& E = M.external[e];
        if (E.body < 0 || E.body >= M.nbodies || E.table < 0 || E.table >= M.ntables)
            return set_err(MH_ERR_INVALID, "external force %d: bad body/table", e);
    }
    // SpringGeneralizedForce elements (ABI v8)
    if (M.nsprings < 0 || (M.nsprings > 0 && !M.springs)) return set_err(MH_ERR_INVALID, "bad springs");
    for (int i = 0; i < M.nsprings; ++i)
        if (M.springs[i].coord < 0 || M.springs[i].coord >= M.nq)
            return set_err(MH_ERR_INVALID, "spring %d: bad coordinate", i);
    c->nsprings = M.nsprings;
    // MocoParameters (ABI v8): bounds per parameter, the properties each writes
    if (p->nparameters < 0 || p->nparameter_targets < 0 || (p->nparameters > 0 && !p->parameter_bounds) ||
            (p->nparameter_targets > 0 && !p->parameter_targets))
        return set_err(MH_ERR_INVALID, "bad parameters");
    c->NPAR = p->nparameters;
    c->par_bounds.assign(p->parameter_bounds, p->parameter_bounds + c->NPAR);
    c->par_targets.assign(p->parameter_targets, p->parameter_targets + p->nparameter_targets);
    std::vector<int> written(c->NPAR, 0);
    for (int t = 0; t < p->nparameter_targets; ++t) {
        const mh_parameter_target& T = c->par_targets[t];
        if (T.parameter < 0 || T.parameter >= c->NPAR)
            return set_err(MH_ERR_INVALID, "parameter target %d: bad parameter %d", t, T.parameter);
        int count = 0, elems = 1;
        switch (T.kind) {
        case MH_PARAM_BODY_MASS: count = M.nbodies; break;
        case MH_PARAM_BODY_MASS_CENTER: count = M.nbodies; elems = 3; break;
        case MH_PARAM_BODY_INERTIA: count = M.nbodies; elems = 6; break;
        case MH_PARAM_SPRING_STIFFNESS: case MH_PARAM_SPRING_REST_LENGTH: case MH_PARAM_SPRING_VISCOSITY:
            count = M.nsprings; break;
        case MH_PARAM_ACTUATOR_OPTIMAL_FORCE: count = M.nactuators; break;
        case MH_PARAM_MUSCLE_MAX_ISOMETRIC_FORCE: count = M.nmuscles; break;
        default: return set_err(MH_ERR_UNSUPPORTED, "parameter target %d: kind %d", t, T.kind);
        }
        if (T.index < 0 || T.index >= count || T.element < 0 || T.element >= elems)
            return set_err(MH_ERR_INVALID, "parameter target %d: bad index / element", t);
        if (T.kind == MH_PARAM_ACTUATOR_OPTIMAL_FORCE && M.actuators[T.index].kind != MH_ACT_COORDINATE)
            return set_err(MH_ERR_INVALID, "parameter target %d: optimal_force of a non-coordinate actuator", t);
        written[T.parameter] = 1;
    }
    for (int q = 0; q < c->NPAR; ++q)
        if (!written[q]) return set_err(MH_ERR_INVALID, "parameter %d writes no model property", q);
    // transcription
    c->scheme = o->transcription;
    c->N = o->num_mesh_intervals;
    c->interp = (o->interpolate_control_midpoints && c->NC > 0) ? 1 : 0;
    c->G = c->scheme == MH_HERMITE_SIMPSON ? 2 * c->N + 1 : c->N + 1;
    c->grid.assign(c->G, 0.0);
    c->quad.assign(c->G, 0.0);
    std::vector<double> mesh(c->N + 1);
    for (int i = 0; i <= c->N; ++i) mesh[i] = i / (double)c->N;   // CasOCSolver.h:38-42
    if (c->scheme == MH_HERMITE_SIMPSON) {
        for (int k = 0; k < c->G; ++k)
            c->grid[k] = (k % 2 == 0) ? mesh[k / 2] : .5 * (mesh[k / 2] + mesh[k / 2 + 1]);
        for (int i = 0; i < c->N; ++i) {  // CasOCHermiteSimpson.cpp:36-43
            const double dm = mesh[i + 1] - mesh[i];
            c->quad[2 * i] += (1.0 / 6.0) * dm;
            c->quad[2 * i + 1] += (2.0 / 3.0) * dm;
            c->quad[2 * i + 2] += (1.0 / 6.0) * dm;
        }
    } else {
        for (int k = 0; k < c->G; ++k) c->grid[k] = mesh[k];
        for (int i = 0; i < c->N; ++i) {  // CasOCTrapezoidal.cpp:26-37
            const double dm = mesh[i + 1] - mesh[i];
            c->quad[i] += 0.5 * dm;
            c->quad[i + 1] += 0.5 * dm;
        }
    }
    c->n = 2 + (int64_t)(c->NS + c->NC + c->NDV + c->NM) * c->G + (int64_t)c->NSL * c->N;
    c->XP = c->n;   // the parameters: the last block of x (CasOCIterate.h:27-44)
    c->n += c->NPAR;
    build_template(c);
    // (kinematic rows precede the path rows: such contexts never run
    // k_interval, whose path loop needs the path entries first)
    if (!c->NK && !path_entries_lead(c)) return set_err(MH_ERR_INVALID, "internal: path-constraint template layout");
    // endpoint rows first, then the intervals, then the tail (the final mesh
    // point's path rows and residuals)
    c->m = c->nep + (int64_t)c->rpi * c->N + c->ntail;
    c->nnz = c->nnz_ep + (int64_t)c->nnz_int * c->N + c->nnz_tail;
    c->ib = std::max(0, o->interval_begin);
    c->ie = o->interval_end > 0 ? std::min(o->interval_end, c->N) : c->N;
    shard_quadrature(c);
    if (c->ib >= c->ie) return set_err(MH_ERR_INVALID, "empty interval shard [%d, %d)", c->ib, c->ie);
    c->k0 = c->scheme == MH_HERMITE_SIMPSON ? 2 * c->ib : c->ib;
    const int klast = c->scheme == MH_HERMITE_SIMPSON ? 2 * c->ie : c->ie;
    c->nk = klast - c->k0 + 1;
    c->fd = o->finite_difference_scheme;
    c->h = o->fd_step > 0 ? o->fd_step : 1e-8;
    c->sinfo.assign(p->state_infos, p->state_infos + c->NS);
    c->cinfo.assign(p->control_infos, p->control_infos + c->NC);
    c->t_init = p->time_initial;
    c->t_final = p->time_final;
    c->ngoals = (int)c->goals.size();
    // size class
    int maxpts = 0;   // current-path capacity: points + 2 tangent points per PathWrap
    for (int im = 0; im < M.nmuscles; ++im)
        maxpts = std::max(maxpts, M.muscles[im].point_count + 2 * c->mus_pw_count[im]);
    auto fits = [&](int MB, int MQ, int MP, int MI, int MO) {
        return M.nbodies <= MB && M.nq <= MQ && maxpts <= MP && c->NI <= MI && c->NO <= MO;
    };
    if (fits(SzSmall::MB, SzSmall::MQ, SzSmall::MP, SzSmall::MI, SzSmall::MO)) c->size_class = 0;
    else if (fits(SzMedium::MB, SzMedium::MQ, SzMedium::MP, SzMedium::MI, SzMedium::MO)) c->size_class = 1;
    else if (fits(SzBody::MB, SzBody::MQ, SzBody::MP, SzBody::MI, SzBody::MO)) c->size_class = 3;
    else if (fits(SzLarge::MB, SzLarge::MQ, SzLarge::MP, SzLarge::MI, SzLarge::MO)) c->size_class = 2;
    else return set_err(MH_ERR_UNSUPPORTED, "model exceeds the largest size class");
    return MH_OK;
}

// FNV-1a 64 over everything the per-point DAE depends on (table *values* are
// excluded: they are read from HBM at run time; so are tables the DAE never
// reads, e.g. tracking references and path-constraint bounds).  Selects
// generated back ends.
static uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ULL; }
    return h;
}
static uint64_t model_hash(const mh_model* M) {
    uint64_t h = 1469598103934665603ULL;
    const int32_t counts[] = {M->nq, M->nbodies, M->naxes, M->nfunctions, M->nknots, M->nmuscles,
            M->npoints, M->nactuators, M->nexternal};
    h = fnv1a(h, counts, sizeof counts);
    h = fnv1a(h, M->gravity, sizeof M->gravity);
    h = fnv1a(h, M->bodies, sizeof(mh_body) * (size_t)M->nbodies);
    h = fnv1a(h, M->axes, sizeof(mh_axis) * (size_t)M->naxes);
    h = fnv1a(h, M->functions, sizeof(mh_function) * (size_t)M->nfunctions);
    h = fnv1a(h, M->knot_x, sizeof(double) * (size_t)M->nknots);
    h = fnv1a(h, M->knot_y, sizeof(double) * (size_t)M->nknots);
    h = fnv1a(h, M->muscles, sizeof(mh_muscle) * (size_t)M->nmuscles);
    h = fnv1a(h, M->points, sizeof(mh_path_point) * (size_t)M->npoints);
    h = fnv1a(h, M->actuators, sizeof(mh_actuator) * (size_t)M->nactuators);
    h = fnv1a(h, M->external, sizeof(mh_external_force) * (size_t)M->nexternal);
    for (int e = 0; e < M->nexternal; ++e) {
        const int t = M->external[e].table;
        if (t < 0 || t >= M->ntables) continue;
        const int32_t shape[2] = {M->tables[t].degree, M->tables[t].ncol};
        h = fnv1a(h, shape, sizeof shape);
    }
    // wrapping (ABI v5) salts the hash only when present, so that models
    // without wraps keep their generated back ends
    if (M->nwraps > 0 || M->npathwraps > 0) {
        const int32_t wc[2] = {M->nwraps, M->npathwraps};
        h = fnv1a(h, wc, sizeof wc);
        if (M->wraps) h = fnv1a(h, M->wraps, sizeof(mh_wrap_object) * (size_t)M->nwraps);
        if (M->pathwraps) h = fnv1a(h, M->pathwraps, sizeof(mh_path_wrap) * (size_t)M->npathwraps);
    }
    return h;
}

extern "C" int mh_model_hash(const mh_model* M, uint64_t* hash) {
    if (!M || !hash) return set_err(MH_ERR_INVALID, "null argument");
    *hash = model_hash(M);
    return MH_OK;
}

static const Backend* select_backend(mh_ctx* c, const mh_problem* p);
static int detect_sparsity(mh_ctx* c, const mh_options* o);
static int build_seeds(mh_ctx* c);
static const TaskInfo* backend_tasks(const Backend* b);
static bool interval_fits(const mh_ctx* c, int mode);

extern "C" int mh_create(const mh_problem* p, const mh_options* o, mh_ctx** out) {
    if (!p || !o || !out) return set_err(MH_ERR_INVALID, "null argument");
    *out = nullptr;
    std::unique_ptr<mh_ctx> c(new mh_ctx());
    std::vector<int> coord_body, act_state, ftn_state, mus_control;
    double tau_act, tau_deact;
    int rc = validate_and_layout(c.get(), p, o, coord_body, act_state, ftn_state, mus_control,
            tau_act, tau_deact);
    if (rc) return rc;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return set_err(MH_ERR_HIP, "no HIP device available (the hot path has no CPU fallback)");
    if (o->device < 0 || o->device >= ndev) return set_err(MH_ERR_HIP, "device %d out of range", o->device);
    c->device = o->device;
    if (c->NPAR > 0 && o->sparsity_detection != MH_SPARSITY_NONE)
        return set_err(MH_ERR_UNSUPPORTED, "MocoParameters with sparsity detection");
    c->be = select_backend(c.get(), p);
    HIPCHK(hipSetDevice(c->device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, c->device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(MH_ERR_HIP, "device %d is %s; this build targets gfx950 only", c->device,
                prop.gcnArchName);
    c->nsimd = 4 * prop.multiProcessorCount;

    const mh_model& M = p->model;
    // host-derived tables
    std::vector<double> kb(M.nknots + 1, 0.0), kc(M.nknots + 1, 0.0), kd(M.nknots + 1, 0.0);
    for (int f = 0; f < M.nfunctions; ++f) {
        const mh_function& F = M.functions[f];
        if (F.kind == MH_FN_SIMMSPLINE)
            simm_coefficients(F.knot_count, M.knot_x + F.knot_begin, M.knot_y + F.knot_begin,
                    kb.data() + F.knot_begin, kc.data() + F.knot_begin, kd.data() + F.knot_begin);
    }
    std::vector<double> mder((size_t)MUS_DERIVED * std::max(1, M.nmuscles), 0.0);
    for (int im = 0; im < M.nmuscles; ++im) {
        const mh_muscle& mu = M.muscles[im];
        double* d = &mder[(size_t)im * MUS_DERIVED];
        d[0] = mu.optimal_fiber_length * std::sin(mu.pennation_angle_at_optimal);
        d[1] = d[0] * d[0];
        d[2] = mu.max_contraction_velocity * mu.optimal_fiber_length;
        d[3] = std::log((1.0 + 0.2) / 0.2) / (1.0 + mu.tendon_strain_at_one_norm_force - 1.0);
        const double e0 = mu.passive_fiber_strain_at_one_norm_force;
        d[4] = std::exp(4.0 * (0.2 - 1.0) / e0);
        d[5] = std::exp(4.0) - d[4];
    }

    Arena A;
    const size_t o_bodies = A.put(M.bodies, M.nbodies), o_axes = A.put(M.axes, M.naxes),
                 o_funcs = A.put(M.functions, M.nfunctions), o_kx = A.put(M.knot_x, M.nknots),
                 o_ky = A.put(M.knot_y, M.nknots), o_kb = A.put(kb.data(), kb.size()),
                 o_kc = A.put(kc.data(), kc.size()), o_kd = A.put(kd.data(), kd.size()),
                 o_mus = A.put(M.muscles, M.nmuscles), o_pts = A.put(M.points, M.npoints),
                 o_acts = A.put(M.actuators, M.nactuators), o_tabs = A.put(M.tables, M.ntables),
                 o_brk = A.put(M.table_breaks, M.nbreaks), o_coef = A.put(M.table_coefs, M.ncoefs),
                 o_ext = A.put(M.external, M.nexternal),
                 o_cb = A.put(coord_body.data(), coord_body.size()),
                 o_as = A.put(act_state.data(), act_state.size()),
                 o_fs = A.put(ftn_state.data(), ftn_state.size()),
                 o_mc = A.put(mus_control.data(), mus_control.size()),
                 o_mi = A.put(c->mus_ider.data(), c->mus_ider.size()),
                 o_kcol = A.put(c->kin_col.data(), c->kin_col.size()),
                 o_md = A.put(mder.data(), mder.size()),
                 o_wr = A.put(M.wraps, M.nwraps), o_pw = A.put(M.pathwraps, M.npathwraps),
                 o_pwb = A.put(c->mus_pw_begin.data(), c->mus_pw_begin.size()),
                 o_pwc = A.put(c->mus_pw_count.data(), c->mus_pw_count.size()),
                 o_goals = A.put(c->goals.data(), c->goals.size()), o_gidx = A.put(c->gidx.data(), c->gidx.size()),
                 o_gcol = A.put(c->gcol.data(), c->gcol.size()), o_gw = A.put(c->gw.data(), c->gw.size()),
                 o_grid = A.put(c->grid.data(), c->grid.size()),
                 o_quad = A.put(c->quad.data(), c->quad.size()),
                 o_quadp = A.put(c->quadp.data(), c->quadp.size()),
                 o_ldss = A.put(&kZeroInt, 1),
                 o_tpl = A.put(c->tpl.data(), c->tpl.size()),
                 o_pc = A.put(c->pc.data(), c->pc.size()),
                 o_ep = A.put(c->ep.data(), c->ep.size()),
                 o_eptpl = A.put(c->eptpl.data(), c->eptpl.size()),
                 o_kcs = A.put(c->kcs.data(), c->kcs.size()),
                 o_sp = A.put(M.springs, M.nsprings);
    // MocoParameters: NCOPY copies of the parameterized arrays (ParamCopies)
    c->NCOPY = c->NPAR > 0 ? 1 + c->NPAR * (o->finite_difference_scheme == MH_FD_CENTRAL ? 2 : 1) : 1;
    size_t o_cb2 = 0, o_ca2 = 0, o_cm2 = 0, o_cs2 = 0, o_ptg = 0;
    if (c->NPAR > 0) {
        o_cb2 = A.reserve(sizeof(mh_body) * (size_t)c->NCOPY * std::max(1, M.nbodies));
        o_ca2 = A.reserve(sizeof(mh_actuator) * (size_t)c->NCOPY * std::max(1, M.nactuators));
        o_cm2 = A.reserve(sizeof(mh_muscle) * (size_t)c->NCOPY * std::max(1, M.nmuscles));
        o_cs2 = A.reserve(sizeof(mh_spring) * (size_t)c->NCOPY * std::max(1, M.nsprings));
        o_ptg = A.put(c->par_targets.data(), c->par_targets.size());
    }
    // a generated back end's constant pool for this model
    std::vector<double> pool;
    if (c->gen) {
        pool.assign((size_t)c->gen->npool, 0.0);
        c->gen->fill(M, pool.data());
    }
    const size_t o_pool = A.put(pool.data(), pool.size());
    // compiled template of the Jacobian lanes (k_interval), capacity of the
    // block-dense template (sparsity detection only removes entries)
    if (!compile_template(c.get())) return set_err(MH_ERR_UNSUPPORTED, "Jacobian template does not compile");
    const size_t o_ctpl = A.put(c->ctpl.data(), c->ctpl.size());
    const size_t o_ctgen = A.put(c->ctgen.data(), c->ctgen.size());
    const size_t o_rl_e = A.put(c->rl_e.data(), c->rl_e.size());
    const size_t o_rl_w = A.put(c->rl_w.data(), c->rl_w.size());

    const int nint = c->ie - c->ib;
    const int ND = c->NI + 2 + c->NPAR;   // t0, tf, the point inputs, the parameters
    const size_t o_x = A.reserve(sizeof(double) * c->n);
    const size_t o_times = A.reserve(sizeof(double) * c->nk);
    const int stride = c->fd == MH_FD_CENTRAL ? 2 * ND + 1 : ND + 1;
    c->lanes_jac = Lanes{c->fd, ND, stride, stride - 1, c->h};
    c->lanes_g = Lanes{c->fd, ND, 1, 0, c->h};
    // excitation lanes (k_exc_lanes): a direction that perturbs the control
    // of exactly one muscle with activation dynamics, read by nothing else
    // in the DAE (coordinate actuators read their own controls only)
    std::vector<int> exc_lane(stride, -1), exc_mus(stride, -1);
    if (!(std::getenv("MOCOHIP_EXC_LANES") && std::strcmp(std::getenv("MOCOHIP_EXC_LANES"), "0") == 0)) {
        for (int dir = 2; dir < ND; ++dir) {
            const int ci = dir - 2 - c->NS;
            if (ci < 0 || ci >= c->NC || ci >= M.nactuators || M.actuators[ci].kind != MH_ACT_MUSCLE) continue;
            int mus = -1, users = 0;
            for (int im = 0; im < M.nmuscles; ++im)
                if (mus_control[im] == ci) { mus = im; ++users; }
            if (users != 1 || act_state[mus] < 0) continue;
            exc_mus[dir] = mus;
            if (c->fd == MH_FD_CENTRAL) exc_mus[dir + ND] = mus;
        }
        if (!backend_tasks(c->be) && std::strncmp(c->be->name, "generic", 7) == 0) {
            exc_lane = exc_mus;
            for (int v : exc_lane) c->n_exc_lanes += v >= 0;
        }
    }
    std::vector<int> lane_map;
    for (int r = 0; r < stride; ++r)
        if (exc_lane[r] < 0) lane_map.push_back(r);
    const size_t o_exc = c->n_exc_lanes ? A.put(exc_lane.data(), exc_lane.size()) : 0;
    const size_t o_lmap = c->n_exc_lanes ? A.put(lane_map.data(), lane_map.size()) : 0;
    // parameter lanes: the lane of model copy cp (1 + p: +h, or -h for
    // backward differences; central: 1 + NPAR + p at -h), evaluated by a
    // launch of their own over that copy; the other lanes by the main launch
    size_t o_lmain = 0, o_plan = 0;
    if (c->NPAR > 0) {
        const int pd = 2 + c->NI;
        std::vector<int> plan, lmain;
        for (int cp = 1; cp < c->NCOPY; ++cp)
            plan.push_back(cp <= c->NPAR ? pd + (cp - 1) : ND + pd + (cp - 1 - c->NPAR));
        for (int r = 0; r < stride; ++r)
            if (exc_lane[r] < 0 && std::find(plan.begin(), plan.end(), r) == plan.end()) lmain.push_back(r);
        c->n_lane_main = (int)lmain.size();
        o_lmain = A.put(lmain.data(), lmain.size());
        o_plan = A.put(plan.data(), plan.size());
    }
    const size_t o_Y = A.reserve(sizeof(double) * (size_t)c->nk * std::max(1, c->NO) * stride);
    const size_t o_Yg = A.reserve(sizeof(double) * (size_t)c->nk * std::max(1, c->NO));
    const size_t o_g = A.reserve(sizeof(double) * ((size_t)c->nep + (size_t)nint * c->rpi + c->ntail));
    const size_t o_vals = A.reserve(sizeof(double) * ((size_t)c->nnz_ep + (size_t)nint * c->nnz_int + c->nnz_tail));
    const size_t o_C = A.reserve(sizeof(double) * (size_t)c->G * std::max(1, c->ngoals));
    const size_t o_grad = A.reserve(sizeof(double) * c->n);
    const size_t o_tpart = A.reserve(sizeof(double) * 2 * (size_t)c->G);
    const size_t o_f = A.reserve(sizeof(double) * 4);
    const size_t o_epc = A.reserve(sizeof(double) * (size_t)std::max(1, c->ngoals));   // endpoint costs
    const int npts_iv = c->scheme == MH_HERMITE_SIMPSON ? 3 : 2;
    const size_t o_xch = A.reserve(sizeof(double) * (size_t)std::max(nint, 1) * npts_iv * std::max(1, c->NO) * XCH_W);
    // tropter global seeds: the coloring and per-seed lists, perturbed
    // iterates and constraint vectors
    c->jac_seeds = o->jacobian_mode == MH_JACOBIAN_GLOBAL_SEEDS;
    if (o->jacobian_mode != MH_JACOBIAN_CALLBACK_FD && !c->jac_seeds)
        return set_err(MH_ERR_INVALID, "unknown jacobian_mode %d", o->jacobian_mode);
    if (c->jac_seeds && (c->ib != 0 || c->ie != c->N || o->sparsity_detection != MH_SPARSITY_NONE))
        return set_err(MH_ERR_UNSUPPORTED, "MH_JACOBIAN_GLOBAL_SEEDS needs an unsharded context and "
                       "the block-dense structure");
    if (o->coloring_order != MH_COLORING_SMALLEST_LAST && o->coloring_order != MH_COLORING_NATURAL)
        return set_err(MH_ERR_INVALID, "unknown coloring_order %d", o->coloring_order);
    c->coloring_order = o->coloring_order;
    size_t o_scol = 0, o_sent = 0, o_srow = 0, o_xp = 0, o_xm = 0, o_gp = 0, o_gm = 0;
    if (c->jac_seeds) {
        int rc2 = build_seeds(c.get());
        if (rc2) return rc2;
        o_scol = A.put(c->seed_cols.data(), c->seed_cols.size());
        o_sent = A.put(c->seed_ents.data(), c->seed_ents.size());
        o_srow = A.put(c->seed_rows.data(), c->seed_rows.size());
        o_xp = A.reserve(sizeof(double) * c->n);
        o_xm = A.reserve(sizeof(double) * c->n);
        o_gp = A.reserve(sizeof(double) * std::max<int64_t>(1, c->m));
        o_gm = A.reserve(sizeof(double) * std::max<int64_t>(1, c->m));
    }

    TaskOffsets to_jac{}, to_g{};
    size_t o_T = 0, o_H = 0, o_Tg = 0, o_Hg = 0, o_xsl = 0, o_cmap = 0;
    const TaskInfo* ti = backend_tasks(c->be);
    if (ti) {
        // the blocks of both task sets in k_interval's XCD order (groups_xcd)
        // (MOCOHIP_IV_XCD=0, the plain interval order, keeps the plain block order too)
        const char* eiv = std::getenv("MOCOHIP_IV_XCD");
        const bool ivx = !(eiv && std::strcmp(eiv, "0") == 0);
        const int nint = ivx ? c->ie - c->ib : 0, ppi = c->scheme == MH_HERMITE_SIMPSON ? 2 : 1;
        build_taskset(*ti, c->lanes_jac, c->nk, c->nsimd, c->ts_jac, nint, ppi);
        build_taskset(*ti, c->lanes_g, c->nk, c->nsimd, c->ts_g, nint, ppi);
        to_jac = put_taskset(A, c->ts_jac);
        to_g = put_taskset(A, c->ts_g);
        // eval_g's task records as kernel arguments (core.hpp k_groups_kr):
        // stride-1 lanes, one task per grid point and group, <= KR_MAX blocks;
        // opt-in (MOCOHIP_GROUPS_KR=1): measured no faster than the table
        // (eval_g's k_groups 7.12 vs 7.05 us, profiles/r05_n)
        {
            const char* ekr = std::getenv("MOCOHIP_GROUPS_KR");
            bool ok = MOCOHIP_AB_VARIANTS && ekr && std::strcmp(ekr, "1") == 0 && c->lanes_g.stride == 1 &&
                      c->ts_g.nblocks > 0 && c->ts_g.nblocks <= KR_MAX &&
                      c->ts_g.blk.size() >= 4 * (size_t)c->ts_g.nblocks;
            const float one = 1.0f;
            int one_bits;
            std::memcpy(&one_bits, &one, sizeof one_bits);
            for (int b = 0; ok && b < c->ts_g.nblocks; ++b) {
                const int* r = &c->ts_g.blk[4 * (size_t)b];
                if (r[2] != 1 || r[3] != one_bits) ok = false;
                else c->krec_g.r[b] = make_int2(r[0], r[1]);
            }
            c->krec_ok = ok;
        }
        // excitation lanes of the generated back end (k_exc_fill): the lane
        // re-evaluates exactly one group besides none of the mass factor's,
        // of one field (the activation derivative)
        if (!c->presc) {
            const int ng = ti->ng;
            std::vector<int> xs, cmap;   // xs: [lane][role, slot, output]
            for (int r = 0; r < stride; ++r) {
                bool fill = false;
                if (exc_mus[r] >= 0 && c->ts_jac.jd[(size_t)r * ng] == 0) {
                    int gx = -1, nre = 0;
                    for (int gg = 1; gg < ng; ++gg)
                        if (c->ts_jac.jd[(size_t)r * ng + gg] != c->ts_jac.off[gg]) { gx = gg; ++nre; }
                    if (nre == 1 && ti->group_nf[gx] == 1) {
                        xs.push_back(r);
                        xs.push_back(c->ts_jac.jd[(size_t)r * ng + gx]);
                        xs.push_back(c->NQ + act_state[exc_mus[r]] - 2 * M.nq);
                        ++c->n_exc_gen;
                        fill = true;
                    }
                }
                if (!fill) cmap.push_back(r);
            }
            if (c->n_exc_gen) {
                o_xsl = A.put(xs.data(), xs.size());
                o_cmap = A.put(cmap.data(), cmap.size());
                c->exc_xs = xs;   // redirect_exc_words, once the quotient modes are known
            }
        }
        o_T = A.reserve(sizeof(double) * std::max(c->ts_jac.t_doubles, c->ts_g.t_doubles));
        o_H = A.reserve(sizeof(double) * std::max(c->ts_jac.h_doubles, c->ts_g.h_doubles));
        o_Tg = A.reserve(sizeof(double) * c->ts_g.t_doubles);
        o_Hg = A.reserve(sizeof(double) * c->ts_g.h_doubles);
    }
    A.size = A.used;
    HIPCHK(hipMalloc(&c->dmem, A.size));
    for (auto& up : A.uploads)
        HIPCHK(hipMemcpy(c->dmem + up.first, up.second.data(), up.second.size(), hipMemcpyHostToDevice));
    char* b = c->dmem;
    DevModel& D = c->M;
    D.nq = M.nq; D.nb = M.nbodies; D.nmus = M.nmuscles; D.nact = M.nactuators; D.next = M.nexternal;
    D.ns = c->NS; D.nz = c->NZ; D.nc = c->NC; D.no = c->NO; D.np = c->NI;
    D.implicit = c->NACC > 0 ? 1 : 0;
    D.nacc = c->NACC;
    D.mus_ider = (const int*)(b + o_mi);
    D.nkc = c->NKC;
    D.kcs = (const mh_constraint*)(b + o_kcs);
    D.okc = c->NK ? c->OKC : -1;
    D.oqc = c->NSL ? c->OQC : -1;
    D.enforce = c->enforce;
    D.mult = c->NC + c->NDV;   // multipliers after the controls and derivatives
    D.presc = c->presc;
    D.kin_table = c->kin_table;
    D.kin_col = (const int*)(b + o_kcol);
    for (int i = 0; i < 3; ++i) D.gravity[i] = M.gravity[i];
    D.tau_act = tau_act; D.tau_deact = tau_deact;
    D.bodies = (const mh_body*)(b + o_bodies); D.axes = (const mh_axis*)(b + o_axes);
    D.funcs = (const mh_function*)(b + o_funcs);
    D.kx = (const double*)(b + o_kx); D.ky = (const double*)(b + o_ky);
    D.kb = (const double*)(b + o_kb); D.kc = (const double*)(b + o_kc); D.kd = (const double*)(b + o_kd);
    D.mus = (const mh_muscle*)(b + o_mus); D.pts = (const mh_path_point*)(b + o_pts);
    D.acts = (const mh_actuator*)(b + o_acts); D.tabs = (const mh_table*)(b + o_tabs);
    D.brk = (const double*)(b + o_brk); D.coef = (const double*)(b + o_coef);
    D.ext = (const mh_external_force*)(b + o_ext);
    D.coord_body = (const int*)(b + o_cb); D.mus_act_state = (const int*)(b + o_as);
    D.mus_ftn_state = (const int*)(b + o_fs); D.mus_control = (const int*)(b + o_mc);
    D.mus_derived = (const double*)(b + o_md);
    D.wr = (const mh_wrap_object*)(b + o_wr);
    D.pw = (const mh_path_wrap*)(b + o_pw);
    D.mus_pw_begin = (const int*)(b + o_pwb);
    D.mus_pw_count = (const int*)(b + o_pwc);
    D.pool = c->gen ? (const double*)(b + o_pool) : nullptr;
    D.nsp = M.nsprings;
    D.sp = (const mh_spring*)(b + o_sp);
    c->M0 = D;   // the pristine model (mh_eval_dae)
    if (c->NPAR > 0) {
        // the copies: every DevModel reads its own parameterized arrays;
        // copy 0 (the iterate's values) is the context's model
        c->Mp.assign(c->NCOPY, D);
        for (int cp = 0; cp < c->NCOPY; ++cp) {
            DevModel& Q = c->Mp[cp];
            Q.bodies = (const mh_body*)(b + o_cb2) + (size_t)cp * M.nbodies;
            Q.acts = (const mh_actuator*)(b + o_ca2) + (size_t)cp * M.nactuators;
            Q.mus = (const mh_muscle*)(b + o_cm2) + (size_t)cp * M.nmuscles;
            Q.sp = (const mh_spring*)(b + o_cs2) + (size_t)cp * M.nsprings;
        }
        D = c->Mp[0];
        c->d_par_targets = (mh_parameter_target*)(b + o_ptg);
        c->d_lane_main = (int*)(b + o_lmain);
        c->d_par_lanes = (int*)(b + o_plan);
        // every copy starts as the pristine model (no targets written): a
        // copy is a valid model before the first iterate's values arrive
        const DevModel& B0 = c->M0;
        const DevModel& Q0 = c->Mp[0];
        ParamCopies P{B0.bodies, B0.acts, B0.mus, B0.sp, (mh_body*)Q0.bodies, (mh_actuator*)Q0.acts,
                      (mh_muscle*)Q0.mus, (mh_spring*)Q0.sp, B0.nb, B0.nact, B0.nmus, B0.nsp, c->NCOPY, c->NPAR};
        hipLaunchKernelGGL(k_apply_params, dim3(1), dim3(256), 0, 0, P, c->d_par_targets, 0,
                (const double*)(b + o_x), c->h, c->fd);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(0));
    }
    c->GS.ngoals = c->ngoals;
    c->GS.ndv = c->NDV;
    c->GS.nc = c->NC;
    c->GS.nacc = c->NACC;
    c->GS.goals = (const mh_goal*)(b + o_goals);
    c->GS.gidx = (const int*)(b + o_gidx);
    c->GS.gcol = (const int*)(b + o_gcol);
    c->GS.gw = (const double*)(b + o_gw);
    if (c->n_exc_lanes) { c->d_exc = (int*)(b + o_exc); c->d_lane_map = (int*)(b + o_lmap); }
    if (c->n_exc_gen) { c->d_exc_slot = (int*)(b + o_xsl); c->d_cmb_map = (int*)(b + o_cmap); }
    if (const char* eb = std::getenv("MOCOHIP_G_BLOCK")) c->g_block = std::min(64, std::max(1, std::atoi(eb)));
    if (const char* el = std::getenv("MOCOHIP_G_LDS")) c->g_lds = std::atoi(el) != 0;
    if (const char* eg = std::getenv("MOCOHIP_G_LDS_GUARD")) c->g_lds_guard = std::min(64, std::max(0, std::atoi(eg)));
    if (const char* es = std::getenv("MOCOHIP_GROUPS_SPLIT")) c->groups_split = std::atoi(es) != 0 ? 1 : 0;
    if (const char* ec = std::getenv("MOCOHIP_COMBINE"))
        c->combine_mode = std::strcmp(ec, "global") == 0 ? 1 : std::strcmp(ec, "lds") == 0 ? 0 : -1;
    c->d_grid = (double*)(b + o_grid); c->d_quad = (double*)(b + o_quad);
    c->d_quadp = (double*)(b + o_quadp);
    c->d_lds_status = (int*)(b + o_ldss);
    c->d_tpl = (TplEntry*)(b + o_tpl);
    c->d_ctpl = (uint32_t*)(b + o_ctpl);
    c->d_ctgen = (int*)(b + o_ctgen);
    c->d_rl_e = (int*)(b + o_rl_e);
    c->d_rl_w = (uint32_t*)(b + o_rl_w);
    c->P = PathEqs{c->npc, (const mh_path_equation*)(b + o_pc), D.tabs, D.brk, D.coef, c->d_grid};
    c->E = EndpointEqs{c->nep, c->nnz_ep, 1 + c->NI, (const mh_endpoint_equation*)(b + o_ep),
                       (const TplEntry*)(b + o_eptpl)};

    c->d_x = (double*)(b + o_x); c->d_times = (double*)(b + o_times); c->d_Y = (double*)(b + o_Y);
    c->d_Yg = (double*)(b + o_Yg); c->d_g = (double*)(b + o_g); c->d_vals = (double*)(b + o_vals);
    c->d_C = (double*)(b + o_C); c->d_grad = (double*)(b + o_grad); c->d_tpart = (double*)(b + o_tpart);
    c->d_f = (double*)(b + o_f);
    c->d_ep = (double*)(b + o_epc);
    c->has_marker = false;
    for (int g = 0; g < p->ngoals; ++g) c->has_marker |= p->goals[g].kind == MH_GOAL_MARKER_FINAL;
    c->d_xch = (double*)(b + o_xch);
    if (c->jac_seeds) {
        c->d_seed_cols = (int32_t*)(b + o_scol);
        c->d_seed_ents = (int32_t*)(b + o_sent);
        c->d_seed_rows = (int32_t*)(b + o_srow);
        c->d_xp = (double*)(b + o_xp); c->d_xm = (double*)(b + o_xm);
        c->d_gp = (double*)(b + o_gp); c->d_gm = (double*)(b + o_gm);
    }
    if (ti) {
        bind_taskset(b, to_jac, c->ts_jac);
        bind_taskset(b, to_g, c->ts_g);
        c->d_T = (double*)(b + o_T);
        c->d_H = (double*)(b + o_H);
        c->d_Tg = (double*)(b + o_Tg);
        c->d_Hg = (double*)(b + o_Hg);
    }
    HIPCHK(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;
    {
        // diagnostic (profiling the phases of k_interval; results are
        // incomplete): MOCOHIP_IV_DEBUG_STOP=1 returns after staging, 2 after
        // the combine
        const char* ed = std::getenv("MOCOHIP_IV_DEBUG_STOP");
        c->iv_dbg_stop = ed ? std::atoi(ed) : 0;
        const char* ef = std::getenv("MOCOHIP_IV_PF");
        c->iv_pf = ef && std::strcmp(ef, "0") == 0 ? 0 : 1;
        // XCD-contiguous interval order in k_interval / kb_interval
        // (xcd_interval, core.hpp; gait N=200: k_interval's HBM reads 10.4 ->
        // 7.5 MB per launch, profiles/r04_xcd); MOCOHIP_IV_XCD=0: plain order
        const char* ex = std::getenv("MOCOHIP_IV_XCD");
        c->iv_xcd = ex && std::strcmp(ex, "0") == 0 ? 0 : 1;
        // the combine of a large model's lanes (k_combine_global's case) with
        // its independent sums spread over a workgroup's waves, then the
        // factorization and solves per lane role (k_combine_split: D::
        // combine_sum / combine_finish): opt-in, MOCOHIP_CSPLIT=1 -- measured
        // slower (configs[3]: DAE stage 0.39 -> 0.47 ms, 1,585 -> 1,380
        // calls/s, profiles/r05_c; so was the same split inside k_interval,
        // profiles/r05_b): the combine is not bound by its sums' chains
        const char* ecs = std::getenv("MOCOHIP_CSPLIT");
        c->csplit = MOCOHIP_AB_VARIANTS && ecs && std::strcmp(ecs, "1") == 0 ? 1 : 0;   // AB build only
        // eval_g's k_interval with the group results at compile-time base
        // slots (core.hpp TaskLoadBase; MOCOHIP_IVG_BASE=0: the slot table)
        const char* eb = std::getenv("MOCOHIP_IVG_BASE");
        c->ivg_base = eb && std::strcmp(eb, "0") == 0 ? 0 : 1;
        const char* esl = std::getenv("MOCOHIP_IV_SLOTS_LDS");
        c->iv_slots_lds = MOCOHIP_AB_VARIANTS && esl && std::strcmp(esl, "1") == 0 ? 1 : 0;   // AB build only
        const char* egm = std::getenv("MOCOHIP_IVG_GM");
        c->ivg_gm = !egm ? -1 : std::strcmp(egm, "0") == 0 ? 0 : 1;
        const TaskInfo* tib = backend_tasks(c->be);
        if (c->ivg_base && (c->lanes_g.stride != 1 || !tib || c->ts_g.jd.size() < (size_t)tib->ng ||
                            !base_slots_match(*tib, c->ts_g)))
            c->ivg_base = 0;
        // hipGraph replay of the stages: measured slower than direct launches
        // on ROCm 7.2 for this sequence (opt-in, MOCOHIP_GRAPHS=1)
        const char* eg = std::getenv("MOCOHIP_GRAPHS");
        c->use_graphs = eg && std::strcmp(eg, "1") == 0;
        // poll for completion instead of a blocking wait (opt-in,
        // MOCOHIP_SPIN=1; no measurable gain on the bench workload)
        const char* es = std::getenv("MOCOHIP_SPIN");
        c->spin_wait = es && std::strcmp(es, "1") == 0;
        // fused combine + transcription per mesh interval unless the LDS
        // budget is exceeded (MOCOHIP_INTERVAL=0 forces the split path)
        const char* ei = std::getenv("MOCOHIP_INTERVAL");
        const bool allow = !(ei && std::strcmp(ei, "0") == 0);
        const char* ec = std::getenv("MOCOHIP_CTPL");
        c->use_ctpl = !(ec && std::strcmp(ec, "0") == 0);
        setup_assembly_variants(c.get());
        const char* er = std::getenv("MOCOHIP_ROLES");
        c->use_roles = er && std::strcmp(er, "1") == 0 && c->NM == 0;   // measured slower
        const char* et = std::getenv("MOCOHIP_ROLE_THREADS");
        if (et) c->role_threads = std::min(512, std::max(64, std::atoi(et) / 64 * 64));
        const char* eqf = std::getenv("MOCOHIP_IV_QFUSE");
        c->iv_qfuse = !(eqf && std::strcmp(eqf, "0") == 0);   // default: measured faster
        const char* eth = std::getenv("MOCOHIP_IV_THREADS");
        if (eth) c->iv_threads = std::min(1024, std::max(256, std::atoi(eth) / 64 * 64));
        const char* egt = std::getenv("MOCOHIP_IVG_THREADS");
        if (egt) c->ivg_threads = std::min(1024, std::max(64, std::atoi(egt) / 64 * 64));
        const char* eo = std::getenv("MOCOHIP_ROLE_COUPLE");
        c->role_couple = !(eo && std::strcmp(eo, "0") == 0);
        const char* ea = std::getenv("MOCOHIP_ASM");
        c->asm_grid_stride = ea && std::strcmp(ea, "gs") == 0;
        const char* eac = std::getenv("MOCOHIP_ASM_CTPL");
        c->asm_ctpl = !(eac && std::strcmp(eac, "0") == 0);
        if (const char* ech = std::getenv("MOCOHIP_ASM_CHUNK"))
            c->asm_chunk_ct = std::min(1 << 20, std::max(256, std::atoi(ech)));
        const char* ee = std::getenv("MOCOHIP_EVENTS");
        c->timing = ee && std::strcmp(ee, "1") == 0;
        const char* egl = std::getenv("MOCOHIP_G_LANE");
        c->g_lane = egl && std::strcmp(egl, "1") == 0;
        const char* eq = std::getenv("MOCOHIP_QUOT");
        c->quot = eq && std::strcmp(eq, "1") == 0;   // opt-in: measured slower
        // the words read the base lane for an excitation lane's copies
        if (redirect_exc_words(c.get()) > 0) {
            setup_assembly_variants(c.get());
            HIPCHK(hipMemcpy(c->d_ctpl, c->ctpl.data(), sizeof(uint32_t) * c->ctpl.size(),
                    hipMemcpyHostToDevice));
        }
        if (o->sparsity_detection != MH_SPARSITY_NONE) {
            // detect on the device, then rebuild the (smaller) template in
            // place of the block-dense one
            const size_t cap = c->tpl.size(), cap_ep = c->eptpl.size();
            int rc2 = detect_sparsity(c.get(), o);
            if (rc2) return rc2;
            c->tpl.clear();
            c->tpl_col_pt.clear();
            build_template(c.get());
            if (!path_entries_lead(c.get()) || c->tpl.size() > cap || c->eptpl.size() > cap_ep)
                return set_err(MH_ERR_INVALID, "internal: detected template layout");
            if (!c->eptpl.empty())
                HIPCHK(hipMemcpy((void*)c->E.tpl, c->eptpl.data(), sizeof(TplEntry) * c->eptpl.size(),
                        hipMemcpyHostToDevice));
            c->E.nnz = c->nnz_ep;
            c->nnz = c->nnz_ep + (int64_t)c->nnz_int * c->N + c->nnz_tail;
            if (!compile_template(c.get())) return set_err(MH_ERR_UNSUPPORTED, "Jacobian template does not compile");
            (void)redirect_exc_words(c.get());
            setup_assembly_variants(c.get());
            HIPCHK(hipMemcpy(c->d_tpl, c->tpl.data(), sizeof(TplEntry) * c->tpl.size(), hipMemcpyHostToDevice));
            HIPCHK(hipMemcpy(c->d_ctpl, c->ctpl.data(), sizeof(uint32_t) * c->ctpl.size(),
                    hipMemcpyHostToDevice));
            if (!c->ctgen.empty())
                HIPCHK(hipMemcpy(c->d_ctgen, c->ctgen.data(), sizeof(int) * c->ctgen.size(),
                        hipMemcpyHostToDevice));
            if (!c->rl_e.empty()) {
                HIPCHK(hipMemcpy(c->d_rl_e, c->rl_e.data(), sizeof(int) * c->rl_e.size(), hipMemcpyHostToDevice));
                HIPCHK(hipMemcpy(c->d_rl_w, c->rl_w.data(), sizeof(uint32_t) * c->rl_w.size(),
                        hipMemcpyHostToDevice));
            }
            c->P.npc = c->npc;
        }
        for (int mode = 0; mode < 2; ++mode)
            c->use_interval[mode] = allow && interval_fits(c.get(), mode);
    }
    for (auto& e : c->ev) HIPCHK(hipEventCreate(&e));
    if (const char* ek = std::getenv("MOCOHIP_D2H_CHUNKS"))
        c->d2h_chunks = std::min(mh_ctx::kMaxD2hChunks, std::max(1, std::atoi(ek)));
    HIPCHK(hipStreamCreateWithFlags(&c->aux_stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&c->ev_x, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_aux, hipEventDisableTiming));
    if (const char* eov = std::getenv("MOCOHIP_OVERLAP")) c->overlap = std::strcmp(eov, "1") == 0;
    HIPCHK(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
    for (auto& e : c->ev_chunk) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&c->ev_copied, hipEventDisableTiming));
    *out = c.release();
    return MH_OK;
}

extern "C" void mh_destroy(mh_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : c->ev_chunk)
        if (e) (void)hipEventDestroy(e);
    if (c->ev_copied) (void)hipEventDestroy(c->ev_copied);
    if (c->aux_stream) {
        (void)hipStreamSynchronize(c->aux_stream);
        (void)hipStreamDestroy(c->aux_stream);
    }
    if (c->ev_x) (void)hipEventDestroy(c->ev_x);
    if (c->ev_aux) (void)hipEventDestroy(c->ev_aux);
    if (c->copy_stream) {
        (void)hipStreamSynchronize(c->copy_stream);
        (void)hipStreamDestroy(c->copy_stream);
    }
    if (c->own_stream) {
        (void)hipStreamSynchronize(c->own_stream);
        (void)hipStreamDestroy(c->own_stream);
    }
    if (c->dmem) (void)hipFree(c->dmem);
    if (c->probe_mem) (void)hipFree(c->probe_mem);
    for (auto& e : c->graphs) (void)hipGraphExecDestroy(e.exec);
    delete c;
}

extern "C" int mh_get_nlp_info(const mh_ctx* c, mh_nlp_info* info) {
    if (!c || !info) return set_err(MH_ERR_INVALID, "null argument");
    std::memset(info, 0, sizeof *info);
    info->n = c->n;
    info->m = c->m;
    info->nnz_jac_g = c->nnz;
    info->nnz_h_lag = 0;
    info->num_grid_points = c->G;
    info->num_states = c->NS;
    info->num_controls = c->NC;
    // the head (endpoint rows) belongs to the shard owning interval 0
    info->row_begin = c->ib == 0 ? 0 : c->nep + (int64_t)c->ib * c->rpi;
    info->row_end = c->nep + (int64_t)c->ie * c->rpi + (c->ie == c->N ? c->ntail : 0);
    info->nnz_begin = c->ib == 0 ? 0 : c->nnz_ep + (int64_t)c->ib * c->nnz_int;
    info->nnz_end = c->nnz_ep + (int64_t)c->ie * c->nnz_int + (c->ie == c->N ? c->nnz_tail : 0);
    return MH_OK;
}

// CasOC::Problem::clipEndpointBounds (CasOCProblem.h:603-606).
static mh_bounds clip(mh_bounds b, mh_bounds e) {
    mh_bounds r;
    r.lower = std::max(b.lower, e.lower);
    r.upper = std::min(b.upper, e.upper);
    return r;
}
static void put_bounds(mh_bounds b, double& lo, double& up) {
    if (!std::isnan(b.lower) && !std::isnan(b.upper)) { lo = b.lower; up = b.upper; }
    else { lo = -INFINITY; up = INFINITY; }
}

extern "C" int mh_get_bounds(const mh_ctx* c, double* xl, double* xu, double* gl, double* gu) {
    if (!c || !xl || !xu) return set_err(MH_ERR_INVALID, "null argument");
    put_bounds(c->t_init, xl[0], xu[0]);
    put_bounds(c->t_final, xl[1], xu[1]);
    auto fill = [&](const mh_variable_info& vi, auto col) {
        const mh_bounds ib = clip(vi.bounds, vi.initial), fb = clip(vi.bounds, vi.final);
        for (int k = 1; k < c->G - 1; ++k) put_bounds(vi.bounds, xl[col(k)], xu[col(k)]);
        put_bounds(ib, xl[col(0)], xu[col(0)]);
        put_bounds(fb, xl[col(c->G - 1)], xu[col(c->G - 1)]);
    };
    for (int s = 0; s < c->NS; ++s) fill(c->sinfo[s], [&](int k) { return col_state(c, k, s); });
    for (int j = 0; j < c->NC; ++j) fill(c->cinfo[j], [&](int k) { return col_control(c, k, j); });
    // implicit: acceleration bounds at every grid point (CasOCTranscription.cpp:222-226)
    // implicit auxiliary derivatives after them (CasOCTranscription.cpp:228-232)
    for (int j = 0; j < c->NDV; ++j) {
        const bool aux = j >= c->NACC;
        for (int k = 0; k < c->G; ++k) {
            xl[col_deriv(c, k, j)] = aux ? c->aux_lo : c->acc_lo;
            xu[col_deriv(c, k, j)] = aux ? c->aux_hi : c->acc_hi;
        }
    }
    // multipliers: multiplier_bounds everywhere (CasOCTranscription.cpp:
    // 209-219); slacks: velocity_correction_bounds (:235-241)
    for (int j = 0; j < c->NM; ++j)
        for (int k = 0; k < c->G; ++k) { xl[col_mult(c, k, j)] = c->mult_lo; xu[col_mult(c, k, j)] = c->mult_hi; }
    for (int l = 0; l < c->NSL; ++l)
        for (int i = 0; i < c->N; ++i) { xl[col_slack(c, i, l)] = c->vc_lo; xu[col_slack(c, i, l)] = c->vc_hi; }
    // parameters: the MocoParameter's bounds (CasOCTranscription.cpp:243-248)
    for (int q = 0; q < c->NPAR; ++q) put_bounds(c->par_bounds[q], xl[c->XP + q], xu[c->XP + q]);
    if (gl && gu) {
        for (int64_t r = 0; r < c->m; ++r) { gl[r] = 0.0; gu[r] = 0.0; }
        // kinematic rows: kinematic_constraint_bounds (CasOCTranscription.cpp:303-309)
        for (int i = 0; i <= c->N; ++i)
            for (int r = 0; r < c->NK; ++r) {
                gl[c->nep + (int64_t)i * c->rpi + r] = c->kc_lo;
                gu[c->nep + (int64_t)i * c->rpi + r] = c->kc_hi;
            }
        // endpoint rows: the constraint info's bounds (CasOCTranscription.cpp:582-583)
        for (int e = 0; e < c->nep; ++e) { gl[e] = c->ep[e].g.lower; gu[e] = c->ep[e].g.upper; }
        // path rows: the equation's bounds at every mesh point
        // (CasOCTranscription.cpp:429-432); mesh point N opens the tail
        for (int i = 0; i <= c->N; ++i)
            for (int e = 0; e < c->npc; ++e) {
                gl[c->nep + (int64_t)i * c->rpi + c->NK + e] = c->pc[e].g.lower;
                gu[c->nep + (int64_t)i * c->rpi + c->NK + e] = c->pc[e].g.upper;
            }
    }
    return MH_OK;
}

extern "C" int mh_get_initial_guess_from_bounds(const mh_ctx* c, double* x) {
    if (!c || !x) return set_err(MH_ERR_INVALID, "null argument");
    std::vector<double> lo(c->n), up(c->n);
    mh_get_bounds(c, lo.data(), up.data(), nullptr, nullptr);
    for (int64_t i = 0; i < c->n; ++i) {  // CasOCTranscription.cpp:1124-1139
        const double l = lo[i], u = up[i];
        if (!std::isinf(l) && !std::isinf(u)) x[i] = 0.5 * (u + l);
        else if (!std::isinf(l)) x[i] = l;
        else if (!std::isinf(u)) x[i] = u;
        else x[i] = 0;
    }
    return MH_OK;
}

extern "C" int mh_get_random_iterate(const mh_ctx* c, const double* rnd, double* x) {
    if (!c || !rnd || !x) return set_err(MH_ERR_INVALID, "null argument");
    std::vector<double> lo(c->n), up(c->n);
    mh_get_bounds(c, lo.data(), up.data(), nullptr, nullptr);
    for (int64_t i = 0; i < c->n; ++i) {  // CasOCTranscription.cpp:1156-1166
        const double l = lo[i], u = up[i], r = rnd[i];
        double v = 0.5 * (r + 1.0) * (u - l) + l;
        if (std::isnan(v)) v = r < l ? l : (r > u ? u : r);
        x[i] = v;
    }
    return MH_OK;
}

extern "C" int mh_get_jac_structure(const mh_ctx* c, int32_t* iRow, int32_t* jCol) {
    if (!c || !iRow || !jCol) return set_err(MH_ERR_INVALID, "null argument");
    const int step = c->scheme == MH_HERMITE_SIMPSON ? 2 : 1;
    int64_t e = 0;
    for (const TplEntry& T : c->eptpl) {   // the head: endpoint rows
        iRow[e] = T.row;
        jCol[e] = (int32_t)ep_col(c, T.dir);
        ++e;
    }
    for (int i = 0; i < c->N; ++i) {
        // the last interval also carries the tail (final-point residual rows)
        const size_t ne = (size_t)c->nnz_int + (i == c->N - 1 ? (size_t)c->nnz_tail : 0);
        for (size_t t = 0; t < ne; ++t) {
            const TplEntry& T = c->tpl[t];
            iRow[e] = (int32_t)(c->nep + (int64_t)i * c->rpi + T.row);
            int64_t col;
            if (T.dir < 2) col = T.dir;
            else if (T.dir >= 2 + c->NI) col = c->XP + (T.dir - 2 - c->NI);   // parameter
            else col = col_input(c, (int64_t)i * step + T.pt, T.dir - 2);
            jCol[e] = (int32_t)col;
            ++e;
        }
    }
    return MH_OK;
}

// ------------------------------------------------------------------------
// Back ends and launchers.
// ------------------------------------------------------------------------


static const TaskInfo* backend_tasks(const Backend* b) { return b->tasks; }
static bool interval_fits(const mh_ctx* c, int mode) {
    return c->be->interval && c->be->interval_bytes(c, mode) <= kMaxLds;
}

// Model-specialized back ends (tools/gen_models.py): generated/gen_*.hip
// define the entries, generated/models_table.inc lists them.
#define MH_GEN_MODEL(SYM) const GenEntry& SYM();
#include "generated/models_table.inc"
#undef MH_GEN_MODEL
#define MH_GEN_MODEL(SYM) &SYM,
static const GenEntry& (*const kGeneratedModels[])() = {
#include "generated/models_table.inc"
};
#undef MH_GEN_MODEL

// One evaluation = two stages on the context stream: the DAE stage (eval
// kernels) and the transcription stage (defects and/or Jacobian assembly),
// with timing events recorded between them.  kind 0: g, 1: Jacobian, 2: both
// from one DAE pass (the base lane of every grid point feeds the defects;
// IPOPT's eval_g(new_x=true) -> eval_jac_g(new_x=false) sequence).
static int launch_stage(mh_ctx* c, int stage, int kind, const double* x, double* a, double* b) {
    // eval_g alone through the model's one-lane-per-DAE kernel (one lane per
    // grid point) and the split transcription (MOCOHIP_G_LANE=1)
    const bool glane = kind == 0 && c->g_lane && c->be_lane;
    if (stage == 0) {
        apply_params(c, x);   // MocoParameters: the model copies for this iterate
        (glane ? c->be_lane : c->be)->eval(c, x, kind == 0 ? 0 : 1, kind == 0 ? c->d_Yg : c->d_Y);
        HIPCHK(hipGetLastError());
        return MH_OK;
    }
    Layout L = make_layout(c, c->k0, c->nk);
    const Lanes& ln = kind == 0 ? c->lanes_g : c->lanes_jac;
    const double* Y = kind == 0 ? c->d_Yg : c->d_Y;
    // the compiled-template assembly's workgroups take asm_chunk_ct nonzeros
    // each (a few per thread and pass); jac_entry's ASM_CHUNK
    const bool ctw = c->use_ctpl && c->asm_ctpl;
    const int chunk = ctw ? c->asm_chunk_ct : ASM_CHUNK;
    const int nchunks = kind == 0 ? 0 : (c->nnz_int + (c->ie == c->N ? c->nnz_tail : 0) + chunk - 1) / chunk;
    double* g = kind == 1 ? nullptr : a;
    double* v = kind == 0 ? nullptr : (kind == 1 ? a : b);
    if (c->use_interval[kind == 0 ? 0 : 1] && !glane) {
        c->be->interval(c, x, kind == 0 ? 0 : 1, g, v, 0, -1);
        HIPCHK(hipGetLastError());
        return MH_OK;
    }
    const Interval I = make_interval(c, g, v);
    const int nint = c->ie - c->ib;
    if (c->asm_grid_stride) {
        const long work = (long)nint * ((v ? c->nnz_int : 0) + (g ? c->rpi : 0));
        const unsigned blocks = (unsigned)std::max(1L, std::min((long)c->nsimd, (work + 255) / 256));
        hipLaunchKernelGGL(k_transcribe_gs, dim3(blocks), dim3(256), 0, c->stream, L, I, ln, c->d_tpl, x,
                c->d_grid, c->d_times, Y, g, v, nint, c->yq[kind == 0 ? 0 : 1]);
    } else {
        hipLaunchKernelGGL(k_transcribe, dim3((unsigned)(nchunks + (g ? 1 : 0)), (unsigned)nint), dim3(256), 0,
                c->stream, L, I, ln, c->d_tpl, ctw ? c->d_ctpl : nullptr, c->d_ctgen, (int)c->ctgen.size(), x,
                c->d_grid, c->d_times, Y, g,
                v, nchunks, c->yq[kind == 0 ? 0 : 1], chunk);
    }
    HIPCHK(hipGetLastError());
    return MH_OK;
}

// A stage as one hipGraph launch, captured on first use for a given set of
// device pointers (IPOPT and the device entry points reuse the same buffers
// every call).  Opt-in: MOCOHIP_GRAPHS=1.
static int run_stage(mh_ctx* c, int stage, int kind, const double* x, double* a, double* b) {
    if (!c->use_graphs) return launch_stage(c, stage, kind, x, a, b);
    const int key = stage * 4 + kind;
    for (const auto& e : c->graphs)
        if (e.kind == key && e.x == x && e.a == a && e.b == b) {
            HIPCHK(hipGraphLaunch(e.exec, c->stream));
            return MH_OK;
        }
    hipGraph_t graph = nullptr;
    HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    const int rc = launch_stage(c, stage, kind, x, a, b);
    const hipError_t ec = hipStreamEndCapture(c->stream, &graph);
    if (rc) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
    }
    HIPCHK(ec);
    hipGraphExec_t exec = nullptr;
    const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    HIPCHK(ei);
    if (c->graphs.size() >= 16) {
        (void)hipGraphExecDestroy(c->graphs.front().exec);
        c->graphs.erase(c->graphs.begin());
    }
    c->graphs.push_back({key, x, a, b, exec});
    HIPCHK(hipGraphLaunch(exec, c->stream));
    return MH_OK;
}

// Stage timing (mh_set_timing / MOCOHIP_EVENTS=1): events recorded
// between the stages on the context stream.  Off by default: each event
// packet costs several microseconds on a call that is itself tens of
// microseconds.
// ------------------------------------------------------------------------
// MH_JACOBIAN_GLOBAL_SEEDS: tropter's Jacobian (ProblemDecorator_double.cpp:
// 261-291).  For every seed of the column coloring, g at x + eps d and
// x - eps d (d = the seed's columns), central quotient, recovered into the
// nonzeros of the seed's columns (each row meets at most one of them, so
// the quotient is that column's derivative).
// ------------------------------------------------------------------------
// Greedy column partial distance-2 coloring over CSR rows / CSC columns,
// the columns visited in natural order (order = MH_COLORING_NATURAL) or in
// the smallest-last order of the column intersection graph
// (MH_COLORING_SMALLEST_LAST, ColPack's ordering in tropter,
// GraphColoring.cpp:91-94; Matula & Beck 1983).  Smallest-last as restated
// here (oracle/oracle.c restates it independently; both follow this text):
// two columns are adjacent iff they share a row; deg(v) = the number of
// distinct adjacent columns.  Columns sit in buckets by current degree,
// inserted in natural order.  n times: take the LAST column of the lowest
// non-empty bucket, place it at the end of the order still free (the first
// removed is colored last), and for each of its distinct adjacent columns
// not yet removed -- visited row by row in ascending row order, each row's
// columns ascending -- remove it from its bucket (the bucket's last column
// takes its place) and append it to the bucket one degree lower.
static void smallest_last_order(int64_t ncols, const std::vector<int64_t>& roff,
        const std::vector<int64_t>& coff, const std::vector<int32_t>& rcol, const std::vector<int32_t>& crow,
        std::vector<int32_t>& order) {
    std::vector<int64_t> deg(ncols, 0), stamp(ncols, -1);
    for (int64_t v = 0; v < ncols; ++v) {
        stamp[v] = v;
        for (int64_t q = coff[v]; q < coff[v + 1]; ++q)
            for (int64_t t = roff[crow[q]]; t < roff[crow[q] + 1]; ++t)
                if (stamp[rcol[t]] != v) { stamp[rcol[t]] = v; ++deg[v]; }
    }
    int64_t maxdeg = 0;
    for (int64_t v = 0; v < ncols; ++v) maxdeg = std::max(maxdeg, deg[v]);
    std::vector<std::vector<int32_t>> bucket((size_t)maxdeg + 1);
    std::vector<int64_t> pos(ncols);
    for (int64_t v = 0; v < ncols; ++v) {
        pos[v] = (int64_t)bucket[deg[v]].size();
        bucket[deg[v]].push_back((int32_t)v);
    }
    std::vector<char> removed(ncols, 0);
    std::fill(stamp.begin(), stamp.end(), -1);
    order.assign(ncols, -1);
    int64_t lo = 0;
    for (int64_t i = 0; i < ncols; ++i) {
        while (bucket[lo].empty()) ++lo;
        const int32_t u = bucket[lo].back();
        bucket[lo].pop_back();
        removed[u] = 1;
        order[ncols - 1 - i] = u;
        stamp[u] = u;
        for (int64_t q = coff[u]; q < coff[u + 1]; ++q)
            for (int64_t t = roff[crow[q]]; t < roff[crow[q] + 1]; ++t) {
                const int32_t x = rcol[t];
                if (stamp[x] == u || removed[x]) continue;
                stamp[x] = u;
                std::vector<int32_t>& b = bucket[deg[x]];
                const int32_t last = b.back();
                b[pos[x]] = last;
                pos[last] = pos[x];
                b.pop_back();
                --deg[x];
                pos[x] = (int64_t)bucket[deg[x]].size();
                bucket[deg[x]].push_back(x);
            }
        if (lo > 0) --lo;   // a neighbour may now sit one bucket lower
    }
}

static int color_columns(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow,
        const int32_t* jCol, int32_t* color, int order_kind = MH_COLORING_NATURAL) {
    std::vector<int64_t> roff(nrows + 1, 0), coff(ncols + 1, 0);
    for (int64_t e = 0; e < nnz; ++e) {
        if (iRow[e] < 0 || iRow[e] >= nrows || jCol[e] < 0 || jCol[e] >= ncols) return -1;
        ++roff[iRow[e] + 1];
        ++coff[jCol[e] + 1];
    }
    for (int64_t r = 0; r < nrows; ++r) roff[r + 1] += roff[r];
    for (int64_t j = 0; j < ncols; ++j) coff[j + 1] += coff[j];
    std::vector<int32_t> rcol(nnz), crow(nnz);
    {
        std::vector<int64_t> rp(roff.begin(), roff.end() - 1), cp(coff.begin(), coff.end() - 1);
        for (int64_t e = 0; e < nnz; ++e) {
            rcol[rp[iRow[e]]++] = jCol[e];
            crow[cp[jCol[e]]++] = iRow[e];
        }
    }
    std::vector<int32_t> order;
    if (order_kind == MH_COLORING_SMALLEST_LAST) smallest_last_order(ncols, roff, coff, rcol, crow, order);
    std::vector<int64_t> stamp;   // stamp[color] == column: color forbidden for it
    int32_t ncolors = 0;
    for (int64_t j = 0; j < ncols; ++j) color[j] = -1;
    for (int64_t jj = 0; jj < ncols; ++jj) {
        const int64_t j = order.empty() ? jj : order[jj];
        for (int64_t q = coff[j]; q < coff[j + 1]; ++q) {
            const int32_t r = crow[q];
            for (int64_t t = roff[r]; t < roff[r + 1]; ++t) {
                const int32_t k = color[rcol[t]];
                if (k >= 0) stamp[k] = j;
            }
        }
        int32_t k = 0;
        while (k < ncolors && stamp[k] == j) ++k;
        if (k == ncolors) { ++ncolors; stamp.push_back(-1); }
        color[j] = k;
    }
    return ncolors;
}

extern "C" int mh_color_jacobian(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow,
        const int32_t* jCol, int32_t* color, int32_t* ncolors) {
    if (nrows < 0 || ncols < 0 || nnz < 0 || (nnz && (!iRow || !jCol)) || (ncols && !color) || !ncolors)
        return set_err(MH_ERR_INVALID, "bad argument");
    const int k = color_columns(nrows, ncols, nnz, iRow, jCol, color);
    if (k < 0) return set_err(MH_ERR_INVALID, "index out of range");
    *ncolors = k;
    return MH_OK;
}

extern "C" int mh_color_jacobian_ordered(int64_t nrows, int64_t ncols, int64_t nnz, const int32_t* iRow,
        const int32_t* jCol, int32_t order, int32_t* color, int32_t* ncolors) {
    if (nrows < 0 || ncols < 0 || nnz < 0 || (nnz && (!iRow || !jCol)) || (ncols && !color) || !ncolors)
        return set_err(MH_ERR_INVALID, "bad argument");
    if (order != MH_COLORING_SMALLEST_LAST && order != MH_COLORING_NATURAL)
        return set_err(MH_ERR_INVALID, "unknown coloring order %d", order);
    const int k = color_columns(nrows, ncols, nnz, iRow, jCol, color, order);
    if (k < 0) return set_err(MH_ERR_INVALID, "index out of range");
    *ncolors = k;
    return MH_OK;
}

extern "C" int mh_get_jacobian_seeds(const mh_ctx* c, int32_t* color, int32_t* nseeds) {
    if (!c || !color || !nseeds) return set_err(MH_ERR_INVALID, "null argument");
    if (!c->jac_seeds) return set_err(MH_ERR_INVALID, "context not in MH_JACOBIAN_GLOBAL_SEEDS mode");
    std::memcpy(color, c->seed_color.data(), sizeof(int32_t) * c->n);
    *nseeds = c->nseeds;
    return MH_OK;
}

// The coloring of the Jacobian structure and its per-seed lists (mh_create).
static int build_seeds(mh_ctx* c) {
    std::vector<int32_t> ir(c->nnz), jc(c->nnz);
    int rc = mh_get_jac_structure(c, ir.data(), jc.data());
    if (rc) return rc;
    c->seed_color.assign(c->n, -1);
    c->nseeds = color_columns(c->m, c->n, c->nnz, ir.data(), jc.data(), c->seed_color.data(), c->coloring_order);
    if (c->nseeds < 0) return set_err(MH_ERR_INVALID, "internal: Jacobian structure out of range");
    const int S = c->nseeds;
    c->seed_col_off.assign(S + 1, 0);
    c->seed_ent_off.assign(S + 1, 0);
    for (int64_t j = 0; j < c->n; ++j) ++c->seed_col_off[c->seed_color[j] + 1];
    for (int64_t e = 0; e < c->nnz; ++e) ++c->seed_ent_off[c->seed_color[jc[e]] + 1];
    for (int k = 0; k < S; ++k) {
        c->seed_col_off[k + 1] += c->seed_col_off[k];
        c->seed_ent_off[k + 1] += c->seed_ent_off[k];
    }
    c->seed_cols.resize(c->n);
    c->seed_ents.resize(c->nnz);
    c->seed_rows.resize(c->nnz);
    std::vector<int32_t> cp(c->seed_col_off.begin(), c->seed_col_off.end() - 1),
            ep(c->seed_ent_off.begin(), c->seed_ent_off.end() - 1);
    for (int64_t j = 0; j < c->n; ++j) c->seed_cols[cp[c->seed_color[j]]++] = (int32_t)j;
    for (int64_t e = 0; e < c->nnz; ++e) {
        const int k = c->seed_color[jc[e]];
        c->seed_ents[ep[k]] = (int32_t)e;
        c->seed_rows[ep[k]] = ir[e];
        ++ep[k];
    }
    return MH_OK;
}

// xp / xm: columns [b, e) of the seed list at x +- eps (set = 1) or back at
// x (set = 0); tropter: x0 + eps * direction with direction entries 1.
__global__ void __launch_bounds__(256) k_seed_set(const double* __restrict__ x, double* __restrict__ xp,
        double* __restrict__ xm, const int32_t* __restrict__ cols, int b, int e, double eps, int set) {
    const int i = b + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= e) return;
    const int j = cols[i];
    xp[j] = set ? x[j] + eps : x[j];
    xm[j] = set ? x[j] - eps : x[j];
}
// values of the seed's nonzeros: (g+ - g-) / (2 eps) of their rows.
__global__ void __launch_bounds__(256) k_seed_recover(const double* __restrict__ gp,
        const double* __restrict__ gm, const int32_t* __restrict__ ents, const int32_t* __restrict__ rows,
        int b, int e, double two_eps, double* __restrict__ values) {
    const int i = b + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= e) return;
    const int r = rows[i];
    values[ents[i]] = (gp[r] - gm[r]) / two_eps;
}

static int run_seeds(mh_ctx* c, const double* x, double* values) {
    const double eps = std::sqrt(std::numeric_limits<double>::epsilon());
    const double two_eps = 2 * eps;
    HIPCHK(hipMemcpyAsync(c->d_xp, x, sizeof(double) * c->n, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_xm, x, sizeof(double) * c->n, hipMemcpyDeviceToDevice, c->stream));
    for (int k = 0; k < c->nseeds; ++k) {
        const int cb = c->seed_col_off[k], ce = c->seed_col_off[k + 1];
        const int eb = c->seed_ent_off[k], ee = c->seed_ent_off[k + 1];
        const unsigned gc = (unsigned)std::max(1, (ce - cb + 255) / 256), ge = (unsigned)std::max(1, (ee - eb + 255) / 256);
        hipLaunchKernelGGL(k_seed_set, dim3(gc), dim3(256), 0, c->stream, x, c->d_xp, c->d_xm, c->d_seed_cols,
                cb, ce, eps, 1);
        for (int side = 0; side < 2; ++side) {
            const double* xs = side ? c->d_xm : c->d_xp;
            double* gs = side ? c->d_gm : c->d_gp;
            int rc = launch_stage(c, 0, 0, xs, gs, nullptr);
            if (rc) return rc;
            rc = launch_stage(c, 1, 0, xs, gs, nullptr);
            if (rc) return rc;
        }
        hipLaunchKernelGGL(k_seed_recover, dim3(ge), dim3(256), 0, c->stream, c->d_gp, c->d_gm, c->d_seed_ents,
                c->d_seed_rows, eb, ee, two_eps, values);
        hipLaunchKernelGGL(k_seed_set, dim3(gc), dim3(256), 0, c->stream, x, c->d_xp, c->d_xm, c->d_seed_cols,
                cb, ce, eps, 0);
    }
    HIPCHK(hipGetLastError());
    return MH_OK;
}

static int run_cached(mh_ctx* c, int kind, const double* x, double* a, double* b) {
    if (kind != 0) c->x_last = nullptr;   // the Jacobian slabs are in use from here on
    if (c->jac_seeds && kind != 0) {   // tropter's global-seed Jacobian
        if (kind == 2) {
            int rc = run_stage(c, 0, 0, x, a, nullptr);
            if (rc) return rc;
            rc = run_stage(c, 1, 0, x, a, nullptr);
            if (rc) return rc;
        }
        c->groups_timed = false;
        if (c->timing) HIPCHK(hipEventRecord(c->ev[0], c->stream));
        int rc = run_seeds(c, x, kind == 1 ? a : b);
        if (c->timing) {
            HIPCHK(hipEventRecord(c->ev[1], c->stream));
            HIPCHK(hipEventRecord(c->ev[2], c->stream));
        }
        return rc;
    }
    // ev[4] (after k_groups) is recorded only by the split task path
    c->groups_timed = c->timing && c->be->tasks && !c->use_interval[kind == 0 ? 0 : 1];
    if (c->timing) HIPCHK(hipEventRecord(c->ev[0], c->stream));
    int rc = run_stage(c, 0, kind, x, a, b);
    if (rc) return rc;
    if (c->timing) HIPCHK(hipEventRecord(c->ev[1], c->stream));
    rc = run_stage(c, 1, kind, x, a, b);
    if (rc) return rc;
    if (c->timing) HIPCHK(hipEventRecord(c->ev[2], c->stream));
    return MH_OK;
}

// async: the device entries return once their work is enqueued
static int finish(mh_ctx* c, bool device_entry = false) {
    if (device_entry && c->async && !c->timing) return MH_OK;
    if (!c->timing) {
        HIPCHK(hipStreamSynchronize(c->stream));
        return MH_OK;
    }
    HIPCHK(hipEventRecord(c->ev[3], c->stream));
    if (c->spin_wait) {
        // poll instead of a blocking wait: the call is latency-bound and the
        // wake-up of a blocking synchronize costs several microseconds
        hipError_t q;
        while ((q = hipEventQuery(c->ev[3])) == hipErrorNotReady) {}
        HIPCHK(q);
    } else {
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    float a = 0, b = 0, d = 0, e = 0;
    (void)hipEventElapsedTime(&a, c->ev[0], c->ev[3]);
    (void)hipEventElapsedTime(&b, c->ev[0], c->ev[1]);
    (void)hipEventElapsedTime(&d, c->ev[1], c->ev[2]);
    if (c->groups_timed) (void)hipEventElapsedTime(&e, c->ev[0], c->ev[4]);
    c->timings[0] = a; c->timings[1] = b; c->timings[2] = d; c->timings[3] = c->groups_timed ? e : b;
    return MH_OK;
}

// rows / nonzeros of this context's shard (the last shard includes the
// final grid point's residual rows in implicit mode)
static size_t shard_rows(const mh_ctx* c) {
    return (c->ib == 0 ? (size_t)c->nep : 0) + (size_t)(c->ie - c->ib) * c->rpi + (c->ie == c->N ? c->ntail : 0);
}
static size_t shard_nnz(const mh_ctx* c) {
    return (c->ib == 0 ? (size_t)c->nnz_ep : 0) + (size_t)(c->ie - c->ib) * c->nnz_int +
           (c->ie == c->N ? c->nnz_tail : 0);
}

extern "C" int mh_eval_g(mh_ctx* c, const double* x, int, double* g) {
    if (!c || !x || !g) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    int rc = run_cached(c, 0, c->d_x, c->d_g, nullptr);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(g, c->d_g, sizeof(double) * shard_rows(c),
            hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

// The host entries' Jacobian: eval_jac_g's k_interval launched in interval
// chunks, each chunk's values (a contiguous slice: the head with the first,
// the tail with the last) copied to the host on copy_stream as soon as that
// chunk's launch completes, while the next chunk assembles -- the PCIe
// transfer, which bounds a host-buffer call (15.4 MB at N = 200), overlaps the
// assembly instead of following it.  Same kernels, same values.  Paths
// without a per-interval task launch copy the whole block after the call.
static int jac_to_host(mh_ctx* c, int kind, double* g_host, double* v_host) {
    c->x_last = nullptr;   // every Jacobian evaluation invalidates the overlap point (run_cached's rule)
    const int nint = c->ie - c->ib;
    const int nch = std::min(c->d2h_chunks, nint);
    const size_t nnz = shard_nnz(c), rows = shard_rows(c);
    double* gd = kind == 2 ? c->d_g : nullptr;
    if (nch <= 1 || c->use_graphs || c->jac_seeds || c->timing || !c->be->tasks || !c->be->interval ||
            !c->use_interval[1] || c->use_roles || c->iv_dbg_stop) {
        int rc = run_cached(c, kind, c->d_x, kind == 2 ? c->d_g : c->d_vals, kind == 2 ? c->d_vals : nullptr);
        if (rc) return rc;
        if (kind == 2)
            HIPCHK(hipMemcpyAsync(g_host, c->d_g, sizeof(double) * rows, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(v_host, c->d_vals, sizeof(double) * nnz, hipMemcpyDeviceToHost, c->stream));
        return MH_OK;
    }
    int rc = run_stage(c, 0, kind, c->d_x, kind == 2 ? c->d_g : c->d_vals, kind == 2 ? c->d_vals : nullptr);
    if (rc) return rc;
    const size_t head = c->ib == 0 ? (size_t)c->nnz_ep : 0;
    // every chunk's launch first (a copy into pageable memory can block the
    // host until it completes; the kernels are queued by then), then the copies
    for (int k = 0; k < nch; ++k) {
        const int i0 = (int)((long)nint * k / nch), i1 = (int)((long)nint * (k + 1) / nch);
        c->be->interval(c, c->d_x, 1, gd, c->d_vals, i0, i1);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(c->ev_chunk[k], c->stream));
    }
    for (int k = 0; k < nch; ++k) {
        const int i0 = (int)((long)nint * k / nch), i1 = (int)((long)nint * (k + 1) / nch);
        HIPCHK(hipStreamWaitEvent(c->copy_stream, c->ev_chunk[k], 0));
        const size_t from = k == 0 ? 0 : head + (size_t)i0 * c->nnz_int;
        const size_t to = k == nch - 1 ? nnz : head + (size_t)i1 * c->nnz_int;
        HIPCHK(hipMemcpyAsync(v_host + from, c->d_vals + from, sizeof(double) * (to - from),
                hipMemcpyDeviceToHost, c->copy_stream));
    }
    if (kind == 2)
        HIPCHK(hipMemcpyAsync(g_host, c->d_g, sizeof(double) * rows, hipMemcpyDeviceToHost, c->copy_stream));
    HIPCHK(hipEventRecord(c->ev_copied, c->copy_stream));
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_copied, 0));
    return MH_OK;
}

extern "C" int mh_eval_jac_g(mh_ctx* c, const double* x, int, double* values) {
    if (!c || !x || !values) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    const int rc = jac_to_host(c, 1, nullptr, values);
    if (rc) return rc;
    return finish(c);
}

extern "C" int mh_eval_g_device(mh_ctx* c, const double* x_dev, double* g_dev) {
    if (!c || !x_dev || !g_dev) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    int rc = run_cached(c, 0, x_dev, g_dev, nullptr);
    if (rc) return rc;
    return finish(c, true);
}

extern "C" int mh_eval_jac_g_device(mh_ctx* c, const double* x_dev, double* v_dev) {
    if (!c || !x_dev || !v_dev) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    int rc = run_cached(c, 1, x_dev, v_dev, nullptr);
    if (rc) return rc;
    return finish(c, true);
}

// mh_tnlp_eval_*_device: an eval_jac_g with new_x = 0 at the iterate of the
// last mh_tnlp_eval_g_device runs on aux_stream from that eval_g's start
// (ev_x), concurrently with the eval_g kernels the caller's stream holds.
// Only the default task path qualifies (k_groups + k_interval, reading x and
// the Jacobian lanes' own slabs d_T / d_H; eval_g uses d_Tg / d_Hg); any
// other evaluation in between invalidates the point (run_cached clears
// x_last for every Jacobian evaluation), so the Jacobian never runs beside
// work that shares its buffers.
static bool can_overlap(const mh_ctx* c) {
    return c->overlap && !c->timing && !c->use_graphs && !c->jac_seeds && c->be->tasks && c->be->interval &&
           c->use_interval[1] && !c->use_roles && !c->iv_dbg_stop && c->aux_stream;
}

extern "C" int mh_tnlp_eval_g_device(mh_ctx* c, const double* x_dev, int new_x, double* g_dev) {
    (void)new_x;   // x's state at this call is what the eval_g kernels read either way
    if (!c || !x_dev || !g_dev) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    c->x_last = nullptr;
    if (can_overlap(c)) {
        HIPCHK(hipEventRecord(c->ev_x, c->stream));
        c->x_last = x_dev;
    }
    int rc = run_cached(c, 0, x_dev, g_dev, nullptr);
    if (rc) return rc;
    return finish(c, true);
}

extern "C" int mh_tnlp_eval_jac_g_device(mh_ctx* c, const double* x_dev, int new_x, double* v_dev) {
    if (!c || !x_dev || !v_dev) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    if (new_x || x_dev != c->x_last || !can_overlap(c)) {
        int rc = run_cached(c, 1, x_dev, v_dev, nullptr);
        if (rc) return rc;
        return finish(c, true);
    }
    hipStream_t caller = c->stream;
    HIPCHK(hipStreamWaitEvent(c->aux_stream, c->ev_x, 0));
    c->stream = c->aux_stream;
    const int rc = run_cached(c, 1, x_dev, v_dev, nullptr);
    c->stream = caller;
    if (rc) return rc;
    HIPCHK(hipEventRecord(c->ev_aux, c->aux_stream));
    HIPCHK(hipStreamWaitEvent(caller, c->ev_aux, 0));
    return finish(c, true);
}

extern "C" int mh_eval_g_jac_g_device(mh_ctx* c, const double* x_dev, double* g_dev, double* v_dev) {
    if (!c || !x_dev || !g_dev || !v_dev) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    int rc = run_cached(c, 2, x_dev, g_dev, v_dev);
    if (rc) return rc;
    return finish(c, true);
}

// ---- the context interface of the device KKT module (csrc/kkt.hip) -------
int mh_internal_error(int code, const char* msg) { return set_err(code, "%s", msg); }
hipStream_t mh_internal_stream(const mh_ctx* c) { return c->stream; }
int mh_internal_device(const mh_ctx* c) { return c->device; }
int mh_internal_shape(const mh_ctx* c, int64_t* n, int64_t* m, int64_t* nnz, int* unsharded) {
    if (!c) return set_err(MH_ERR_INVALID, "null context");
    *n = c->n;
    *m = (int64_t)shard_rows(c);
    *nnz = (int64_t)shard_nnz(c);
    *unsharded = c->ib == 0 && c->ie == c->N;
    return MH_OK;
}
// The whole NLP's m and nnz and this shard's nonzero range (mh_nlp_info).
int mh_internal_shard(const mh_ctx* c, int64_t* m_full, int64_t* nnz_full, int64_t* nnz_begin, int64_t* nnz_end) {
    if (!c) return set_err(MH_ERR_INVALID, "null context");
    mh_nlp_info info;
    const int rc = mh_get_nlp_info(c, &info);
    if (rc) return rc;
    *m_full = info.m;
    *nnz_full = info.nnz_jac_g;
    *nnz_begin = info.nnz_begin;
    *nnz_end = info.nnz_end;
    return MH_OK;
}
// eval_jac_g at a device iterate into a device buffer, enqueued on the
// context stream (no synchronization: the KKT module's kernels follow)
int mh_internal_jac_device(mh_ctx* c, const double* x_dev, double* v_dev) {
    HIPCHK(hipSetDevice(c->device));
    (void)hipGetLastError();
    return run_cached(c, 1, x_dev, v_dev, nullptr);
}

// ---- batches (include/mocohip.h mh_batch_*) -------------------------------
extern "C" int mh_batch_create(mh_ctx* const* ctxs, int32_t count, mh_batch** out) {
    if (!ctxs || !out || count < 1) return set_err(MH_ERR_INVALID, "null argument or empty batch");
    if (count > MH_BATCH_MAX) return set_err(MH_ERR_INVALID, "at most %d contexts per batch", MH_BATCH_MAX);
    *out = nullptr;
    const mh_ctx* a = ctxs[0];
    for (int b = 0; b < count; ++b) {
        const mh_ctx* c = ctxs[b];
        if (!c) return set_err(MH_ERR_INVALID, "null context %d", b);
        if (!c->be->batch || !c->use_interval[0] || !c->use_interval[1] || c->jac_seeds || c->use_roles)
            return set_err(MH_ERR_UNSUPPORTED, "context %d: batches need the task back end with the fused "
                           "interval kernel (no global seeds, no k_role)", b);
        // the same problem shape: back end, layout, lanes, tasks, template
        const bool same = c->be == a->be && c->device == a->device && c->N == a->N && c->G == a->G &&
                c->ib == a->ib && c->ie == a->ie && c->k0 == a->k0 && c->nk == a->nk &&
                c->scheme == a->scheme && c->n == a->n && c->m == a->m && c->nnz == a->nnz &&
                c->nnz_int == a->nnz_int && c->rpi == a->rpi && c->nep == a->nep && c->nnz_ep == a->nnz_ep &&
                c->fd == a->fd && c->h == a->h && c->NS == a->NS && c->NC == a->NC && c->NDV == a->NDV &&
                c->NM == a->NM && c->NSL == a->NSL && c->lanes_jac.stride == a->lanes_jac.stride &&
                c->lanes_g.stride == a->lanes_g.stride && c->ts_jac.nblocks == a->ts_jac.nblocks &&
                c->ts_g.nblocks == a->ts_g.nblocks && c->ts_jac.t_doubles == a->ts_jac.t_doubles &&
                c->ts_jac.h_doubles == a->ts_jac.h_doubles && c->iv_threads == a->iv_threads &&
                c->use_ctpl == a->use_ctpl && c->tpl.size() == a->tpl.size() &&
                std::memcmp(c->tpl.data(), a->tpl.data(), sizeof(TplEntry) * a->tpl.size()) == 0 &&
                c->ctgen == a->ctgen;
        if (!same) return set_err(MH_ERR_INVALID, "context %d: problem shape differs from context 0", b);
    }
    auto* bt = new mh_batch();
    bt->ctx.assign(ctxs, ctxs + count);
    bt->B = count;
    const char* eg = std::getenv("MOCOHIP_BATCH_GM");
    if (eg) bt->gm = std::atoi(eg) != 0;
    // defaults measured on MI355X (8 gait NLPs, fused steps, tools/batch_threads_ab.sh):
    // 512-thread interval blocks reading group results from global memory
    // 54.4 k calls/s vs 47.3 k at 1024 threads with LDS staging; kb_groups
    // at >= 3 waves / SIMD +1-2 %
    const char* ew = std::getenv("MOCOHIP_BATCH_WAVES");
    if (ew) bt->waves = std::atoi(ew) == 3 ? 3 : 0;
    const char* et = std::getenv("MOCOHIP_BATCH_THREADS");
    if (et) bt->threads = std::min(1024, std::max(256, std::atoi(et) / 64 * 64));
    std::vector<BatchItem> items(count);
    for (int b = 0; b < count; ++b) {
        const mh_ctx* c = ctxs[b];
        items[b] = BatchItem{c->M, c->d_T, c->d_H, c->P, c->E, c->d_grid};
    }
    if (hipSetDevice(a->device) != hipSuccess ||
            hipMalloc(&bt->d_items, sizeof(BatchItem) * count) != hipSuccess ||
            hipMemcpy(bt->d_items, items.data(), sizeof(BatchItem) * count, hipMemcpyHostToDevice) != hipSuccess) {
        if (bt->d_items) (void)hipFree(bt->d_items);
        delete bt;
        return set_err(MH_ERR_HIP, "batch allocation failed");
    }
    *out = bt;
    return MH_OK;
}
extern "C" void mh_batch_destroy(mh_batch* bt) {
    if (!bt) return;
    if (bt->d_items) {
        (void)hipSetDevice(bt->ctx[0]->device);
        (void)hipFree(bt->d_items);
    }
    delete bt;
}
extern "C" int mh_batch_set_group_results_global(mh_batch* bt, int on) {
    if (!bt) return set_err(MH_ERR_INVALID, "null batch");
    bt->gm = on != 0;
    return MH_OK;
}
static int batch_run(mh_batch* bt, int kind, const double* const* x, double* const* g, double* const* v) {
    if (!bt || !x || (kind != 1 && !g) || (kind != 0 && !v)) return set_err(MH_ERR_INVALID, "null argument");
    BatchPtrs P{};
    for (int b = 0; b < bt->B; ++b) bt->ctx[b]->x_last = nullptr;   // writes every slab (d_T)
    for (int b = 0; b < bt->B; ++b) {
        if (!x[b] || (kind != 1 && !g[b]) || (kind != 0 && !v[b]))
            return set_err(MH_ERR_INVALID, "null pointer for batch item %d", b);
        P.x[b] = x[b];
        P.g[b] = kind != 1 ? g[b] : nullptr;
        P.v[b] = kind != 0 ? v[b] : nullptr;
    }
    mh_ctx* c = bt->ctx[0];
    HIPCHK(hipSetDevice(c->device));
    c->be->batch(bt, kind == 0 ? 0 : 1, P, kind != 1, kind != 0);
    HIPCHK(hipGetLastError());
    if (c->async) return MH_OK;
    HIPCHK(hipStreamSynchronize(c->stream));
    return MH_OK;
}
extern "C" int mh_batch_eval_g_device(mh_batch* bt, const double* const* x, double* const* g) {
    return batch_run(bt, 0, x, g, nullptr);
}
extern "C" int mh_batch_eval_jac_g_device(mh_batch* bt, const double* const* x, double* const* v) {
    return batch_run(bt, 1, x, nullptr, v);
}
extern "C" int mh_batch_eval_g_jac_g_device(mh_batch* bt, const double* const* x, double* const* g,
        double* const* v) {
    return batch_run(bt, 2, x, g, v);
}

extern "C" int mh_eval_g_jac_g(mh_ctx* c, const double* x, double* g, double* values) {
    if (!c || !x || !g || !values) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    const int rc = jac_to_host(c, 2, g, values);
    if (rc) return rc;
    return finish(c);
}

// The objective (partial = false) or this shard's partial of it (partial =
// true: the integrals over the shard's own mesh intervals, d_quadp, and the
// endpoint goals -- final time, final marker -- on the shard that owns the
// final grid point only).  Swapping d_quad lets the back ends' integrand /
// gradient launches read the shard's weights unchanged.
static int eval_f_impl(mh_ctx* c, const double* x, double* f, bool partial) {
    if (!c || !x || !f) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    (void)hipGetLastError();   // report only this call's launch errors
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    if (c->timing) HIPCHK(hipEventRecord(c->ev[0], c->stream));
    const bool endpoint = !partial || c->ie == c->N;
    apply_params(c, c->d_x);   // the goals read the context's model, copy 0
    double* quad = c->d_quad;
    if (partial) c->d_quad = c->d_quadp;
    Layout L = make_layout(c, 0, c->G);
    if (c->ngoals > 0) c->be->integrand(c, c->d_x);
    c->d_quad = quad;
    HIPCHK(hipGetLastError());
    if (c->has_marker && endpoint)
        hipLaunchKernelGGL(k_marker_final, dim3((unsigned)c->ngoals), dim3(128), 0, c->stream, c->M, L, c->GS,
                c->fd, c->h, 0, c->d_x, c->d_ep, c->d_grad);
    if (c->timing) HIPCHK(hipEventRecord(c->ev[1], c->stream));
    hipLaunchKernelGGL(k_reduce_obj, dim3(1), dim3(256), 0, c->stream, L, c->GS, 0, endpoint ? 1 : 0, c->d_x,
            c->d_C, c->d_tpart, c->d_ep, c->d_f);
    HIPCHK(hipGetLastError());
    if (c->timing) HIPCHK(hipEventRecord(c->ev[2], c->stream));
    HIPCHK(hipMemcpyAsync(f, c->d_f, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

static int eval_grad_f_impl(mh_ctx* c, const double* x, double* grad, bool partial) {
    if (!c || !x || !grad) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    (void)hipGetLastError();   // report only this call's launch errors
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    if (c->timing) HIPCHK(hipEventRecord(c->ev[0], c->stream));
    const bool endpoint = !partial || c->ie == c->N;
    apply_params(c, c->d_x);   // the goals read the context's model, copy 0
    Layout L = make_layout(c, 0, c->G);
    HIPCHK(hipMemsetAsync(c->d_grad, 0, sizeof(double) * c->n, c->stream));
    HIPCHK(hipMemsetAsync(c->d_tpart, 0, sizeof(double) * 2 * c->G, c->stream));
    HIPCHK(hipMemsetAsync(c->d_C, 0, sizeof(double) * c->G * std::max(1, c->ngoals), c->stream));
    double* quad = c->d_quad;
    if (partial) c->d_quad = c->d_quadp;
    if (c->ngoals > 0) {
        c->be->integrand(c, c->d_x);
        c->be->grad(c, c->d_x);
    }
    c->d_quad = quad;
    HIPCHK(hipGetLastError());
    if (c->has_marker && endpoint)   // after k_grad: adds to the final coordinates' entries
        hipLaunchKernelGGL(k_marker_final, dim3((unsigned)c->ngoals), dim3(128), 0, c->stream, c->M, L, c->GS,
                c->fd, c->h, 1, c->d_x, c->d_ep, c->d_grad);
    if (c->timing) HIPCHK(hipEventRecord(c->ev[1], c->stream));
    hipLaunchKernelGGL(k_reduce_obj, dim3(1), dim3(256), 0, c->stream, L, c->GS, 1, endpoint ? 1 : 0, c->d_x,
            c->d_C, c->d_tpart, c->d_ep, c->d_f);
    HIPCHK(hipGetLastError());
    if (c->timing) HIPCHK(hipEventRecord(c->ev[2], c->stream));
    HIPCHK(hipMemcpyAsync(c->d_grad, c->d_f, sizeof(double) * 2, hipMemcpyDeviceToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(grad, c->d_grad, sizeof(double) * c->n, hipMemcpyDeviceToHost, c->stream));
    return finish(c);
}

extern "C" int mh_eval_f(mh_ctx* c, const double* x, int, double* f) { return eval_f_impl(c, x, f, false); }

// The objective's terms, one per goal (the solution's objective breakdown,
// MocoCasADiSolver.cpp:395-402; CasOCTranscription.cpp:699-702 evaluates the
// objective terms at the solution): eval_f's arithmetic, each goal's weighted
// value kept apart instead of summed.
extern "C" int mh_eval_objective_terms(mh_ctx* c, const double* x, double* terms, int32_t* nterms) {
    if (!c || !x || !terms || !nterms) return set_err(MH_ERR_INVALID, "null argument");
    if (*nterms < c->ngoals) {
        const int have = *nterms;
        *nterms = c->ngoals;
        return set_err(MH_ERR_INVALID, "terms holds %d doubles, the problem has %d goals", have, c->ngoals);
    }
    *nterms = c->ngoals;
    if (c->ngoals == 0) return MH_OK;
    HIPCHK(hipSetDevice(c->device));
    (void)hipGetLastError();
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    apply_params(c, c->d_x);   // the goals read the context's model, copy 0
    Layout L = make_layout(c, 0, c->G);
    c->be->integrand(c, c->d_x);
    HIPCHK(hipGetLastError());
    if (c->has_marker)
        hipLaunchKernelGGL(k_marker_final, dim3((unsigned)c->ngoals), dim3(128), 0, c->stream, c->M, L, c->GS,
                c->fd, c->h, 0, c->d_x, c->d_ep, c->d_grad);
    // the per-goal terms into the gradient's buffer (n >= goals; scratch here)
    hipLaunchKernelGGL(k_reduce_obj, dim3(1), dim3(256), 0, c->stream, L, c->GS, 2, 1, c->d_x, c->d_C, c->d_tpart,
            c->d_ep, c->d_grad);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(terms, c->d_grad, sizeof(double) * c->ngoals, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MH_OK;
}
extern "C" int mh_eval_grad_f(mh_ctx* c, const double* x, int, double* grad) {
    return eval_grad_f_impl(c, x, grad, false);
}
extern "C" int mh_eval_f_partial(mh_ctx* c, const double* x, double* f) { return eval_f_impl(c, x, f, true); }
extern "C" int mh_eval_grad_f_partial(mh_ctx* c, const double* x, double* grad) {
    return eval_grad_f_impl(c, x, grad, true);
}

extern "C" int mh_eval_dae(mh_ctx* c, int32_t np, const double* inputs, double* outputs) {
    if (!c || !inputs || !outputs || np < 0) return set_err(MH_ERR_INVALID, "bad argument");
    if (np == 0) return MH_OK;
    HIPCHK(hipSetDevice(c->device));
    double *din = nullptr, *dout = nullptr;
    const size_t nin = (size_t)np * (1 + c->NI), nout = (size_t)np * c->NO;
    HIPCHK(hipMalloc(&din, sizeof(double) * nin));
    HIPCHK(hipMalloc(&dout, sizeof(double) * std::max<size_t>(nout, 1)));
    HIPCHK(hipMemcpyAsync(din, inputs, sizeof(double) * nin, hipMemcpyHostToDevice, c->stream));
    (void)hipGetLastError();
    c->be->probe(c, np, din, dout);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(outputs, dout, sizeof(double) * nout, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    (void)hipFree(din);
    (void)hipFree(dout);
    return MH_OK;
}


// Path-constraint values of np probe rows [t, states, controls, ...]
// (sparsity detection of the path-constraint callbacks).
__global__ void __launch_bounds__(256) k_path_probe(PathEqs P, int np, int NS, int W,
        const double* __restrict__ in, double* __restrict__ out) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= np * P.npc) return;
    const int q = w / P.npc, e = w - q * P.npc;
    const double* r = in + (long)q * W;
    out[w] = path_value(P, e, r[0], r[1 + NS + P.eq[e].index]);
}

// Endpoint-equation values of np probe rows [initial_time, initial inputs,
// final_time, final inputs] (sparsity detection of the Endpoint callbacks).
__global__ void __launch_bounds__(256) k_endpoint_probe(EndpointEqs E, int np, int NS,
        const double* __restrict__ in, double* __restrict__ out) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= np * E.nep) return;
    const int q = w / E.nep, e = w - q * E.nep;
    const double* r = in + (long)q * 2 * E.W;
    out[w] = ep_eval(E.eq[e], NS, [&](int si) { return r[si]; });
}

// splitmix64 uniform(-1, 1) stream (include/mocohip.h
// mh_options.sparsity_detection; stands in for SimTK::Random::Uniform).
static double splitmix_uniform(uint64_t& st) {
    uint64_t z = (st += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return (double)(z >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

// calcJacobianSparsityWithPerturbation (CasOCFunction.cpp:25-71) of the DAE
// callback and of each path equation, evaluated on the device at
// getSubsetPoint of each detection iterate (CasOCFunction.h:72-86: time =
// initial_time, the first grid point's variables; iterates per
// CasOCSolver.cpp:70-92): input j perturbed by +1e-5, a change (or NaN)
// marks the dependency; OR over the iterates.
// The coupling test of a detection probe (include/mocohip.h
// mh_sparsity_rule): d = perturbed - base output, scale = the callback's
// magnitude at the detection point (sparsity_scale).
static inline bool sparsity_coupled(int rule, double d, double scale) {
    if (std::isnan(d)) return true;
    if (rule == MH_SPARSITY_RULE_ANY_CHANGE) return d != 0;
    return std::fabs(d) > MH_SPARSITY_ROBUST_TOL * scale;
}
static inline double sparsity_scale(const double* y0, int n) {
    double s = 1.0;
    for (int k = 0; k < n; ++k)
        if (std::isfinite(y0[k])) s = std::max(s, std::fabs(y0[k]));
    return s;
}

static int detect_sparsity(mh_ctx* c, const mh_options* o) {
    const int W = 1 + c->NI, NO = c->NO, NPC = c->npc;
    const int rule = o->sparsity_rule;
    if (rule != MH_SPARSITY_RULE_ROBUST && rule != MH_SPARSITY_RULE_ANY_CHANGE)
        return set_err(MH_ERR_INVALID, "unknown sparsity rule %d", rule);
    std::vector<double> pts;
    int npts = 1;
    if (o->sparsity_detection == MH_SPARSITY_RANDOM) {
        npts = o->sparsity_random_count > 0 ? o->sparsity_random_count : 3;
        pts.resize((size_t)c->n * npts);
        std::vector<double> r(c->n);
        uint64_t st = 0;
        for (int q = 0; q < npts; ++q) {
            for (auto& v : r) v = splitmix_uniform(st);
            mh_get_random_iterate(c, r.data(), pts.data() + (size_t)q * c->n);
        }
    } else if (o->sparsity_detection == MH_SPARSITY_INITIAL_GUESS) {
        // no guess given: the default "bounds" guess (midpoints,
        // CasOCTranscription.cpp:1123-1149)
        if (o->sparsity_guess) pts.assign(o->sparsity_guess, o->sparsity_guess + c->n);
        else {
            pts.resize(c->n);
            mh_get_initial_guess_from_bounds(c, pts.data());
        }
    } else if (o->sparsity_detection == MH_SPARSITY_GIVEN) {
        if (!o->sparsity_pattern) return set_err(MH_ERR_INVALID, "GIVEN sparsity needs sparsity_pattern");
        c->sp.assign(o->sparsity_pattern, o->sparsity_pattern + (size_t)NO * W);
        c->sp_pc.assign(o->sparsity_pattern + (size_t)NO * W, o->sparsity_pattern + (size_t)(NO + NPC) * W);
        c->sp_ep.assign(o->sparsity_pattern + (size_t)(NO + NPC) * W,
                        o->sparsity_pattern + (size_t)(NO + NPC + 2 * c->nep) * W);
        return MH_OK;
    } else {
        return set_err(MH_ERR_INVALID, "unknown sparsity detection %d", o->sparsity_detection);
    }
    const int rows = npts * (1 + W);
    std::vector<double> in((size_t)rows * W);
    for (int q = 0; q < npts; ++q) {
        const double* x = pts.data() + (size_t)q * c->n;
        double* base = in.data() + (size_t)q * (1 + W) * W;
        base[0] = x[0];
        for (int s = 0; s < c->NS; ++s) base[1 + s] = x[col_state(c, 0, s)];
        for (int j = 0; j < c->NC; ++j) base[1 + c->NS + j] = x[col_control(c, 0, j)];
        for (int j = 0; j < c->NDV; ++j) base[1 + c->NS + c->NC + j] = x[col_deriv(c, 0, j)];
        for (int j = 0; j < W; ++j) {
            double* r = base + (size_t)(1 + j) * W;
            std::memcpy(r, base, sizeof(double) * W);
            r[j] = base[j] + 1e-5;
        }
    }
    std::vector<double> out((size_t)rows * std::max(NO, 1)), pout((size_t)rows * std::max(NPC, 1));
    if (NO > 0) {
        const int rc = mh_eval_dae(c, rows, in.data(), out.data());
        if (rc) return rc;
    }
    if (NPC > 0) {
        double *din = nullptr, *dout = nullptr;
        HIPCHK(hipMalloc(&din, sizeof(double) * in.size()));
        HIPCHK(hipMalloc(&dout, sizeof(double) * pout.size()));
        HIPCHK(hipMemcpyAsync(din, in.data(), sizeof(double) * in.size(), hipMemcpyHostToDevice, c->stream));
        const int nthr = rows * NPC;
        k_path_probe<<<(nthr + 255) / 256, 256, 0, c->stream>>>(c->P, rows, c->NS, W, din, dout);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(pout.data(), dout, sizeof(double) * pout.size(), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        (void)hipFree(din);
        (void)hipFree(dout);
    }
    // the endpoint functions at their subset point (Endpoint::getSubsetPoint,
    // CasOCFunction.h:214-237: the integral input is 0 there and, being no NLP
    // variable, adds no column): every input perturbed by +1e-5
    const int WE = 2 * W, NEP = c->nep;
    const int erows = npts * (1 + WE);
    std::vector<double> ein((size_t)erows * WE), eout((size_t)erows * std::max(NEP, 1));
    if (NEP > 0) {
        for (int q = 0; q < npts; ++q) {
            const double* x = pts.data() + (size_t)q * c->n;
            double* base = ein.data() + (size_t)q * (1 + WE) * WE;
            for (int si = 0; si < WE; ++si) base[si] = x[ep_col(c, si)];
            for (int j = 0; j < WE; ++j) {
                double* r = base + (size_t)(1 + j) * WE;
                std::memcpy(r, base, sizeof(double) * WE);
                r[j] = base[j] + 1e-5;
            }
        }
        double *din = nullptr, *dout = nullptr;
        HIPCHK(hipMalloc(&din, sizeof(double) * ein.size()));
        HIPCHK(hipMalloc(&dout, sizeof(double) * eout.size()));
        HIPCHK(hipMemcpyAsync(din, ein.data(), sizeof(double) * ein.size(), hipMemcpyHostToDevice, c->stream));
        const int nthr = erows * NEP;
        k_endpoint_probe<<<(nthr + 255) / 256, 256, 0, c->stream>>>(c->E, erows, c->NS, din, dout);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(eout.data(), dout, sizeof(double) * eout.size(), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        (void)hipFree(din);
        (void)hipFree(dout);
    }
    c->sp_ep.assign((size_t)NEP * WE, 0);
    for (int q = 0; q < npts; ++q) {
        const size_t r0 = (size_t)q * (1 + WE);
        const double se = sparsity_scale(eout.data() + r0 * NEP, NEP);
        for (int j = 0; j < WE; ++j)
            for (int e = 0; e < NEP; ++e) {
                const double d = eout[(r0 + 1 + j) * NEP + e] - eout[r0 * NEP + e];
                if (sparsity_coupled(rule, d, se)) c->sp_ep[(size_t)e * WE + j] = 1;
            }
    }
    c->sp.assign((size_t)NO * W, 0);
    c->sp_pc.assign((size_t)NPC * W, 0);
    for (int q = 0; q < npts; ++q) {
        const size_t r0 = (size_t)q * (1 + W);
        const double sd = sparsity_scale(out.data() + r0 * NO, NO);
        const double sp = sparsity_scale(pout.data() + r0 * NPC, NPC);
        for (int j = 0; j < W; ++j) {
            for (int k = 0; k < NO; ++k) {
                const double d = out[(r0 + 1 + j) * NO + k] - out[r0 * NO + k];
                if (sparsity_coupled(rule, d, sd)) c->sp[(size_t)k * W + j] = 1;
            }
            for (int e = 0; e < NPC; ++e) {
                const double d = pout[(r0 + 1 + j) * NPC + e] - pout[r0 * NPC + e];
                if (sparsity_coupled(rule, d, sp)) c->sp_pc[(size_t)e * W + j] = 1;
            }
        }
    }
    return MH_OK;
}


extern "C" int mh_debug_jacobian_lanes(mh_ctx* c, const double* x, double* times, double* Y) {
    if (!c || !x || !times || !Y) return set_err(MH_ERR_INVALID, "null argument");
    if (c->ib != 0 || c->ie != c->N) return set_err(MH_ERR_INVALID, "mh_debug_jacobian_lanes: unsharded contexts only");
    HIPCHK(hipSetDevice(c->device));
    (void)hipGetLastError();
    HIPCHK(hipMemcpyAsync(c->d_x, x, sizeof(double) * c->n, hipMemcpyHostToDevice, c->stream));
    apply_params(c, c->d_x);
    c->exc_full = true;   // every lane complete (the eval path fills the read outputs only)
    c->be->lanes(c, c->d_x, c->d_Y);
    c->exc_full = false;
    HIPCHK(hipGetLastError());
    const size_t ny = (size_t)c->nk * c->NO * c->lanes_jac.stride;
    HIPCHK(hipMemcpyAsync(times, c->d_times, sizeof(double) * c->nk, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(Y, c->d_Y, sizeof(double) * ny, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MH_OK;
}

extern "C" int mh_set_stream(mh_ctx* c, void* stream) {
    if (!c) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->own_stream;
    if (s != c->stream) {
        // work already enqueued on the previous stream completes first
        HIPCHK(hipStreamSynchronize(c->stream));
        for (auto& e : c->graphs) (void)hipGraphExecDestroy(e.exec);
        c->graphs.clear();
        c->stream = s;
    }
    return MH_OK;
}

extern "C" int mh_set_async(mh_ctx* c, int on) {
    if (!c) return set_err(MH_ERR_INVALID, "null argument");
    c->async = on != 0;
    return MH_OK;
}

extern "C" int mh_synchronize(mh_ctx* c) {
    if (!c) return set_err(MH_ERR_INVALID, "null argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return MH_OK;
}

extern "C" int mh_debug_time_stages(mh_ctx* c, const double* x, int kind, int reps, double* ms2) {
    if (!c || !x || !ms2 || reps < 1 || kind < 0 || kind > 1) return set_err(MH_ERR_INVALID, "bad argument");
    HIPCHK(hipSetDevice(c->device));
    (void)hipGetLastError();
    double* a = kind == 0 ? c->d_g : c->d_vals;
    int rc = launch_stage(c, 0, kind, x, a, nullptr);   // warm: the transcription reads its results
    if (!rc) rc = launch_stage(c, 1, kind, x, a, nullptr);
    if (rc) return rc;
    // the two stages in their real order (the DAE stage, then the
    // transcription reading what it just wrote), an event after each: every
    // launch is timed in the sequence a call runs, as a kernel trace sees it
    // (back-to-back launches of one stage alone read up to ~10 % faster)
    // The event packets themselves take time on the queue: the same pairs
    // are also timed with events at the two ends only, and each stage's
    // figure loses its share of the difference (one event per stage), so
    // that the two stages add up to the measured pair time.
    reps = std::min(reps, 500);
    HIPCHK(hipEventRecord(c->ev[0], c->stream));
    for (int r = 0; r < reps && !rc; ++r) {
        rc = launch_stage(c, 0, kind, x, a, nullptr);
        if (!rc) rc = launch_stage(c, 1, kind, x, a, nullptr);
    }
    HIPCHK(hipEventRecord(c->ev[1], c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (rc) return rc;
    float tpair = 0;
    HIPCHK(hipEventElapsedTime(&tpair, c->ev[0], c->ev[1]));
    std::vector<hipEvent_t> ev((size_t)2 * reps + 1, nullptr);
    for (auto& e : ev) HIPCHK(hipEventCreate(&e));
    HIPCHK(hipEventRecord(ev[0], c->stream));
    for (int r = 0; r < reps && !rc; ++r) {
        rc = launch_stage(c, 0, kind, x, a, nullptr);
        if (!rc) (void)hipEventRecord(ev[2 * r + 1], c->stream);
        if (!rc) rc = launch_stage(c, 1, kind, x, a, nullptr);
        if (!rc) (void)hipEventRecord(ev[2 * r + 2], c->stream);
    }
    const hipError_t es = hipStreamSynchronize(c->stream);
    double t0 = 0.0, t1 = 0.0;
    for (int r = 0; r < reps && !rc && es == hipSuccess; ++r) {
        float a0 = 0, a1 = 0;
        (void)hipEventElapsedTime(&a0, ev[2 * r], ev[2 * r + 1]);
        (void)hipEventElapsedTime(&a1, ev[2 * r + 1], ev[2 * r + 2]);
        t0 += a0;
        t1 += a1;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    HIPCHK(es);
    if (rc) return rc;
    const double per_event = std::max(0.0, (t0 + t1 - (double)tpair) / (2.0 * reps));
    ms2[0] = t0 / reps - per_event;
    ms2[1] = t1 / reps - per_event;
    return MH_OK;
}

extern "C" int mh_set_timing(mh_ctx* c, int on) {
    if (!c) return set_err(MH_ERR_INVALID, "null argument");
    c->timing = on != 0;
    return MH_OK;
}

extern "C" int mh_last_timings(const mh_ctx* c, double* ms4) {
    if (!c || !ms4) return set_err(MH_ERR_INVALID, "null argument");
    for (int i = 0; i < 4; ++i) ms4[i] = c->timings[i];
    return MH_OK;
}

extern "C" int mh_get_backend(const mh_ctx* c, char* name, int32_t name_len, double* flops_per_eval,
        uint64_t* model_hash) {
    if (!c) return set_err(MH_ERR_INVALID, "null argument");
    if (name && name_len > 0) {
        std::strncpy(name, c->be->name, (size_t)name_len - 1);
        name[name_len - 1] = 0;
    }
    if (flops_per_eval) *flops_per_eval = c->be->flops_per_eval;
    if (model_hash) *model_hash = c->model_hash;
    return MH_OK;
}

extern "C" int mh_get_nlp_info_for(const mh_problem* p, const mh_options* o, mh_nlp_info* info) {
    if (!p || !o || !info) return set_err(MH_ERR_INVALID, "null argument");
    std::unique_ptr<mh_ctx> c(new mh_ctx());
    std::vector<int> coord_body, act_state, ftn_state, mus_control;
    double tau_act, tau_deact;
    int rc = validate_and_layout(c.get(), p, o, coord_body, act_state, ftn_state, mus_control, tau_act,
            tau_deact);
    if (rc) return rc;
    return mh_get_nlp_info(c.get(), info);
}

extern "C" int mh_backend_for(const mh_problem* p, const mh_options* o, char* name, int32_t name_len) {
    if (!p || !o || !name || name_len <= 0) return set_err(MH_ERR_INVALID, "bad argument");
    std::unique_ptr<mh_ctx> c(new mh_ctx());
    std::vector<int> coord_body, act_state, ftn_state, mus_control;
    double tau_act, tau_deact;
    int rc = validate_and_layout(c.get(), p, o, coord_body, act_state, ftn_state, mus_control, tau_act,
            tau_deact);
    if (rc) return rc;
    const Backend* be = select_backend(c.get(), p);
    std::strncpy(name, be->name, (size_t)name_len - 1);
    name[name_len - 1] = 0;
    return MH_OK;
}

extern "C" int mh_get_callback_sparsity(const mh_ctx* c, uint8_t* pattern, int64_t len) {
    if (!c || !pattern) return set_err(MH_ERR_INVALID, "null argument");
    const size_t W = 1 + (size_t)c->NI, nd = (size_t)c->NO * W, np = nd + (size_t)c->npc * W;
    const size_t need = np + (size_t)c->nep * 2 * W;
    if (len < (int64_t)need) return set_err(MH_ERR_INVALID, "pattern needs %zu bytes", need);
    for (size_t i = 0; i < need; ++i)
        pattern[i] = i < nd ? (c->sp.empty() ? 1 : c->sp[i])
                   : i < np ? (c->sp_pc.empty() ? 1 : c->sp_pc[i - nd])
                            : (c->sp_ep.empty() ? 1 : c->sp_ep[i - np]);
    return MH_OK;
}

extern "C" int mh_get_backend_flags(const mh_ctx* c, char* flags, int32_t len) {
    if (!c || !flags || len <= 0) return set_err(MH_ERR_INVALID, "bad argument");
    std::string f = c->be->tasks ? "tasks" : (std::strncmp(c->be->name, "generic", 7) == 0 ? "generic" : "lane");
    f += c->use_interval[1] ? " interval" : " split";
    if (c->use_interval[0]) f += c->ivg_base ? " interval-g base-slots" : " interval-g";
    if (c->krec_ok) f += " groups-kernarg";
    if (!c->use_ctpl) f += " no-ctpl";
    if (c->iv_dbase) f += " dbase";
    if (c->iv_qdiv) f += " qdiv";
    if (c->use_roles && c->use_interval[1]) f += " roles";
    if (c->quot) f += " quot";
    if (c->asm_grid_stride) f += " asm-gs";
    if (c->d_exc) f += " exc-lanes";
    if (c->d_exc_slot)
        f += c->exc_redirected && c->use_ctpl && c->asm_ctpl && !c->asm_grid_stride ? " exc-fill adot-only"
                                                                                     : " exc-fill";
    if (c->g_lds && !c->be->tasks && std::strncmp(c->be->name, "generic", 7) == 0) {
        f += " g-lds";
        if (c->g_lds_guard) {
            // the guard bands' verdict over every k_eval_lds launch so far
            // ordered after every k_eval_lds launch still in flight on the
            // context's (non-blocking) stream
            int st = 0;
            if (hipMemcpyAsync(&st, c->d_lds_status, sizeof(int), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
                    hipStreamSynchronize(c->stream) != hipSuccess)
                return set_err(MH_ERR_HIP, "reading the LDS guard status failed");
            f += st ? " g-lds-guard-violated" : " g-lds-guard-intact";
        }
    }
    std::strncpy(flags, f.c_str(), (size_t)len - 1);
    flags[len - 1] = 0;
    return MH_OK;
}

extern "C" int mh_get_work(const mh_ctx* c, double* work4) {
    if (!c || !work4) return set_err(MH_ERR_INVALID, "null argument");
    const double lanes_jac = (double)c->nk * c->lanes_jac.stride, lanes_g = (double)c->nk;
    if (c->be->tasks) {
        work4[0] = c->ts_jac.flops;
        work4[1] = c->ts_g.flops;
        work4[2] = c->ts_jac.ntasks;
    } else {
        work4[0] = lanes_jac * c->be->flops_per_eval;
        work4[1] = lanes_g * c->be->flops_per_eval;
        work4[2] = 0.0;
    }
    work4[3] = lanes_jac;
    return MH_OK;
}

static const Backend* select_backend(mh_ctx* c, const mh_problem* p) {
    c->model_hash = model_hash(&p->model);
    const char* force = std::getenv("MOCOHIP_BACKEND");
    const bool generic = force && std::strcmp(force, "generic") == 0;
    const bool lane = force && std::strcmp(force, "lane") == 0;
    // a generated back end runs any model of the structure it was generated
    // for (match: topology, joint / path / wrap / constraint wiring, zero
    // pattern); its numbers come from the model's constant pool (fill, in
    // mh_create)
    // MocoParameters write model properties a generated back end folds into
    // its constant pool, and SpringGeneralizedForce is not in the generated
    // code: both run on the generic interpreter
    if (!generic && c->NPAR == 0 && c->nsprings == 0) {
        for (auto entry : kGeneratedModels) {
            const GenEntry& e = entry();
            if (e.implicit != (c->NMB > 0) || e.prescribed != (c->presc != 0)) continue;
            if (c->NKC && !c->presc && (e.kc_enforce != (c->enforce != 0) || e.kc_slacks != (c->NSL > 0)))
                continue;
            if (!e.match(p->model)) continue;
            c->gen = &e;
            c->be_lane = &e.lane;
            return lane ? &e.lane : &e.tasks;
        }
    }
    return &generic_backends()[c->size_class];
}
