// A/B microbenchmark: the mass-matrix
// task's spatial-inertia contractions, M_ij = S_j . (Ic_i S_i) for the NQ
// = 10 coordinates of gait10dof18musc (composite inertia Ic_i of the body
// carrying coordinate i, ground-frame motion subspace S_i; lower triangle,
// 55 entries), for T independent (grid point, lane role) tasks:
//   V64  -- the k_groups layout: one task per lane, 64 tasks per wave, FP64 VALU;
//   W1V  -- one task per wave: lanes compute F = [Ic_i S_i] (60 entries) and
//           then the 55 dot products, FP64 VALU;
//   W1M  -- one task per wave: F on the VALU, M = S^T F on the matrix core
//           (v_mfma_f64_16x16x4f64, K = 6 padded to 8: two MFMAs).
// Each kernel runs alone between HIP events (rocprofv3 sees the same
// launches); results are checked against V64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

constexpr int NQ = 10, NM = NQ * (NQ + 1) / 2;
// per task: Ic as 6x6 row-major (36) per coordinate, S 6 per coordinate
constexpr int IC = 36 * NQ, SS = 6 * NQ;

__global__ void __launch_bounds__(64) k_v64(const double* __restrict__ Ic, const double* __restrict__ S,
        double* __restrict__ M, int T) {
    // lane-interleaved (structure-of-arrays) operands: element e of task t
    // at e * T + t, so that every load of a wave is one coalesced run
    const int t = blockIdx.x * 64 + threadIdx.x;
    if (t >= T) return;
    double F[NQ][6];
#pragma unroll
    for (int i = 0; i < NQ; ++i)
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            double a = 0.0;
#pragma unroll
            for (int c = 0; c < 6; ++c) a += Ic[(long)(i * 36 + r * 6 + c) * T + t] * S[(long)(i * 6 + c) * T + t];
            F[i][r] = a;
        }
    int q = 0;
#pragma unroll
    for (int i = 0; i < NQ; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) {
            double a = 0.0;
#pragma unroll
            for (int r = 0; r < 6; ++r) a += S[(long)(j * 6 + r) * T + t] * F[i][r];
            M[(long)q * T + t] = a;
            ++q;
        }
}

__global__ void __launch_bounds__(64) k_w1v(const double* __restrict__ Ic, const double* __restrict__ S,
        double* __restrict__ M, int T) {
    __shared__ double sF[NQ * 6], sS[NQ * 6];
    const int t = blockIdx.x, l = threadIdx.x;
    const double* I = Ic + (long)t * IC;
    const double* s = S + (long)t * SS;
    if (l < SS) sS[l] = s[l];
    if (l < SS) {   // F[i][r], l = i * 6 + r
        const int i = l / 6, r = l % 6;
        double a = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) a += I[i * 36 + r * 6 + c] * s[i * 6 + c];
        sF[l] = a;
    }
    __syncthreads();
    if (l < NM) {   // (i, j) of lower-triangle entry l
        int i = 0;
        while ((i + 1) * (i + 2) / 2 <= l) ++i;
        const int j = l - i * (i + 1) / 2;
        double a = 0.0;
#pragma unroll
        for (int r = 0; r < 6; ++r) a += sS[j * 6 + r] * sF[i * 6 + r];
        M[(long)t * NM + l] = a;
    }
}

typedef double v4d __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(64) k_w1m(const double* __restrict__ Ic, const double* __restrict__ S,
        double* __restrict__ M, int T) {
    __shared__ double sF[NQ * 6], sS[NQ * 6];
    const int t = blockIdx.x, l = threadIdx.x;
    const double* I = Ic + (long)t * IC;
    const double* s = S + (long)t * SS;
    if (l < SS) sS[l] = s[l];
    if (l < SS) {
        const int i = l / 6, r = l % 6;
        double a = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) a += I[i * 36 + r * 6 + c] * s[i * 6 + c];
        sF[l] = a;
    }
    __syncthreads();
    // D[row j][col i] = sum_k A[j][k] B[k][i], A = S^T (A[j][k] = S_j[k]),
    // B[k][i] = F_i[k]; 16x16x4 f64: lane supplies A[l & 15][l >> 4] and
    // B[l >> 4][l & 15] of the K-slice; D: col = l & 15, row = (l >> 4) + 4 r
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    const int row = l & 15, kk = l >> 4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
        const int k = kk + 4 * ks;
        const double a = (row < NQ && k < 6) ? sS[row * 6 + k] : 0.0;
        const double b = (row < NQ && k < 6) ? sF[row * 6 + k] : 0.0;   // B[k][col = l & 15]
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int j = (l >> 4) + 4 * r, i = l & 15;   // D[j][i] = S_j . F_i
        if (i < NQ && j <= i) M[(long)t * NM + i * (i + 1) / 2 + j] = acc[r];
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s\n", hipGetErrorString(e_)); return 1; } } while (0)

int main(int argc, char** argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 4411;   // 401 grid points x 11 mass-matrix roles
    const int reps = 200;
    std::vector<double> hI((size_t)T * IC), hS((size_t)T * SS);
    srand(1);
    for (auto& v : hI) v = rand() / (double)RAND_MAX - 0.5;
    for (auto& v : hS) v = rand() / (double)RAND_MAX - 0.5;
    // V64 reads the same operands lane-interleaved
    std::vector<double> tI(hI.size()), tS(hS.size());
    for (int t = 0; t < T; ++t) {
        for (int e = 0; e < IC; ++e) tI[(size_t)e * T + t] = hI[(size_t)t * IC + e];
        for (int e = 0; e < SS; ++e) tS[(size_t)e * T + t] = hS[(size_t)t * SS + e];
    }
    double *dI, *dS, *dIt, *dSt, *dM[3];
    CK(hipMalloc(&dI, hI.size() * 8));
    CK(hipMalloc(&dS, hS.size() * 8));
    CK(hipMalloc(&dIt, hI.size() * 8));
    CK(hipMalloc(&dSt, hS.size() * 8));
    CK(hipMemcpy(dIt, tI.data(), tI.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dSt, tS.data(), tS.size() * 8, hipMemcpyHostToDevice));
    for (auto& p : dM) CK(hipMalloc(&p, (size_t)T * NM * 8));
    CK(hipMemcpy(dI, hI.data(), hI.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dS, hS.data(), hS.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* names[3] = {"V64 (64 tasks/wave, VALU)", "W1V (1 task/wave, VALU)", "W1M (1 task/wave, MFMA f64)"};
    float ms[3];
    for (int v = 0; v < 3; ++v) {
        auto launch = [&]() {
            if (v == 0) hipLaunchKernelGGL(k_v64, dim3((T + 63) / 64), dim3(64), 0, 0, dIt, dSt, dM[0], T);
            else if (v == 1) hipLaunchKernelGGL(k_w1v, dim3(T), dim3(64), 0, 0, dI, dS, dM[1], T);
            else hipLaunchKernelGGL(k_w1m, dim3(T), dim3(64), 0, 0, dI, dS, dM[2], T);
        };
        for (int w = 0; w < 20; ++w) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms[v], e0, e1));
    }
    std::vector<double> m0((size_t)T * NM), m1(m0.size()), m2(m0.size()), mt(m0.size());
    CK(hipMemcpy(mt.data(), dM[0], mt.size() * 8, hipMemcpyDeviceToHost));
    for (int t = 0; t < T; ++t)
        for (int q = 0; q < NM; ++q) m0[(size_t)t * NM + q] = mt[(size_t)q * T + t];
    CK(hipMemcpy(m1.data(), dM[1], m1.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m2.data(), dM[2], m2.size() * 8, hipMemcpyDeviceToHost));
    double d1 = 0, d2 = 0, sc = 0;
    for (size_t i = 0; i < m0.size(); ++i) {
        d1 = std::fmax(d1, std::fabs(m1[i] - m0[i]));
        d2 = std::fmax(d2, std::fabs(m2[i] - m0[i]));
        sc = std::fmax(sc, std::fabs(m0[i]));
    }
    std::printf("{\"tasks\": %d, \"reps\": %d", T, reps);
    for (int v = 0; v < 3; ++v) std::printf(", \"%s_us\": %.3f", names[v], 1e3 * ms[v] / reps);
    std::printf(", \"max_diff_W1V\": %.3e, \"max_diff_W1M\": %.3e, \"scale\": %.3e}\n", d1, d2, sc);
    return 0;
}
