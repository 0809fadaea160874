// Post-fit alignment of estimated state trajectories with true ones on gfx950
// (SURVEY §8f row f4).  Reference: src/utils/alignment.py
//   procrustes_alignment   :31-100   R = U Vt of svd(X_true^T X_est), det fix
//   align_signs (rows)     :137-145  flip row i when -x_i is closer to y_i
//   align_latent_positions :202-221  Procrustes on U and on V, then row signs
//   align_temporal_states  :265-321  per time step, or one rotation of the
//                                     time-averaged (U,V) block
//   compute_alignment_error:359-385  mean squared error after alignment
//
// Layout: X (n, T, d) fp32, row-major, d = 2 + 2r (what get_variational_means
// returns).  Two kernels around a batched r x r SVD the host does on the device:
//   ame_align_cross : C = A_true^T A_est per block, fp64 sums over the n nodes,
//                     rows staged through LDS in chunks of 32 nodes;
//   ame_align_apply : x_out = signs(x_est R) per (node, t) row, plus per-block
//                     fp64 partial sums of |x_out - x_true|^2.
// Both are HBM-bound streaming passes (each reads X_est and X_true once).
#include <stdio.h>

#include "ame_common.h"

namespace {

constexpr int kAT = 256;    // threads per workgroup
constexpr int kACH = 32;    // nodes per LDS chunk (cross products)
constexpr int kAMAXW = 64;  // widest block: 2r for r = 32

// Cross products of one block (blockIdx.x = time step, blockIdx.y = U / V, or
// one block over the time-averaged rows in the global mode).  src rows are
// fp32 (n, T, d) rows or, global mode, fp64 (n, w) time averages.
template <typename TIn>
__global__ void __launch_bounds__(kAT)
ame_align_cross_kernel(const TIn* est, const TIn* tru, int n, long long rstride,
                       long long tstride, int col0, int colstep, int w, double* C) {
    __shared__ double se[kACH][kAMAXW + 1];
    __shared__ double st[kACH][kAMAXW + 1];
    const int tid = threadIdx.x;
    const long long base = (long long)blockIdx.x * tstride + col0 + (long long)blockIdx.y * colstep;
    const int ne = w * w;
    double acc[(kAMAXW * kAMAXW + kAT - 1) / kAT];
    constexpr int NQ = (kAMAXW * kAMAXW + kAT - 1) / kAT;
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
    for (int i0 = 0; i0 < n; i0 += kACH) {
        const int cnt = min(kACH, n - i0);
        __syncthreads();
        for (int e = tid; e < cnt * w; e += kAT) {
            const int ii = e / w, c = e - ii * w;
            const long long o = base + (long long)(i0 + ii) * rstride + c;
            se[ii][c] = (double)est[o];
            st[ii][c] = (double)tru[o];
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int e = tid + kAT * q;
            if (e < ne) {
                const int p = e / w, c = e - p * w;   // C[p][c] = sum_i tru[i][p] est[i][c]
                double a = acc[q];
                for (int ii = 0; ii < cnt; ++ii) a = fma(st[ii][p], se[ii][c], a);
                acc[q] = a;
            }
        }
    }
    double* out = C + ((size_t)blockIdx.x * gridDim.y + blockIdx.y) * ne;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        const int e = tid + kAT * q;
        if (e < ne) out[e] = acc[q];
    }
}

// Time averages of the (U,V) block: mean[i][c] = (1/T) sum_t X[i,t,2+c] (fp64).
__global__ void __launch_bounds__(kAT)
ame_align_means_kernel(const float* est, const float* tru, int n, int T, int d,
                       double* mest, double* mtru) {
    const int w = d - 2;
    const long long e = (long long)blockIdx.x * kAT + threadIdx.x;
    if (e >= (long long)n * w) return;
    const int i = (int)(e / w), c = (int)(e - (long long)i * w);
    double se = 0.0, st = 0.0;
    for (int t = 0; t < T; ++t) {
        const long long o = ((long long)i * T + t) * d + 2 + c;
        se += (double)est[o];
        st += (double)tru[o];
    }
    mest[e] = se / T;
    mtru[e] = st / T;
}

// row sign rule of align_signs: flip when ||-x - y|| < ||x - y|| (fp32 norms)
template <int W>
__device__ __forceinline__ bool flip_row(const float* x, const float* y) {
    float dp = 0.f, dn = 0.f;
#pragma unroll
    for (int c = 0; c < W; ++c) {
        const float a = x[c] - y[c], b = -x[c] - y[c];
        dp = fmaf(a, a, dp);
        dn = fmaf(b, b, dn);
    }
    return sqrtf(dn) < sqrtf(dp);
}

// One thread per (node, t) row; blockIdx.y = t, R of that t staged in LDS.
// rot: each mode [T][2][r][r] (U then V), global mode [2r][2r].
template <int R>
__global__ void __launch_bounds__(kAT)
ame_align_apply_kernel(const float* est, const float* tru, int n, int T, int global_mode,
                       const double* rot, float* out, double* partials) {
    constexpr int D = 2 + 2 * R, W = 2 * R;
    __shared__ double rs[W * W];
    __shared__ double red[kAT / 64];
    const int t = blockIdx.y, tid = threadIdx.x;
    if (global_mode) {
        for (int e = tid; e < W * W; e += kAT) rs[e] = rot[e];
    } else {
        for (int e = tid; e < 2 * R * R; e += kAT) rs[e] = rot[(size_t)t * 2 * R * R + e];
    }
    __syncthreads();
    const int i = blockIdx.x * kAT + tid;
    double sq = 0.0;
    if (i < n) {
        const size_t o = ((size_t)i * T + t) * D;
        float x[D], y[D], z[D];
#pragma unroll
        for (int c = 0; c < D; ++c) {
            x[c] = est[o + c];
            y[c] = tru[o + c];
        }
        // additive effects: signs only (alignment.py:275-278 / 306-313)
        const bool fa = flip_row<2>(x, y);
        z[0] = fa ? -x[0] : x[0];
        z[1] = fa ? -x[1] : x[1];
        if (global_mode) {   // (U,V) row times the one 2r x 2r rotation (:316-318)
#pragma unroll
            for (int q = 0; q < W; ++q) {
                double a = 0.0;
#pragma unroll
                for (int p = 0; p < W; ++p) a = fma((double)x[2 + p], rs[p * W + q], a);
                z[2 + q] = (float)a;
            }
            const bool fm = flip_row<W>(z + 2, y + 2);
#pragma unroll
            for (int q = 0; q < W; ++q) z[2 + q] = fm ? -z[2 + q] : z[2 + q];
        } else {             // U and V each times its own r x r rotation (:210-216)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const double* Rb = rs + b * R * R;
                float* zb = z + 2 + b * R;
                const float* xb = x + 2 + b * R;
#pragma unroll
                for (int q = 0; q < R; ++q) {
                    double a = 0.0;
#pragma unroll
                    for (int p = 0; p < R; ++p) a = fma((double)xb[p], Rb[p * R + q], a);
                    zb[q] = (float)a;
                }
                const bool fb = flip_row<R>(zb, y + 2 + b * R);
#pragma unroll
                for (int q = 0; q < R; ++q) zb[q] = fb ? -zb[q] : zb[q];
            }
        }
#pragma unroll
        for (int c = 0; c < D; ++c) {
            out[o + c] = z[c];
            const double e = (double)z[c] - (double)y[c];
            sq = fma(e, e, sq);
        }
    }
    // deterministic block sum -> partials[t][blockIdx.x]
    sq = wave_sum(sq);
    if ((tid & 63) == 0) red[tid >> 6] = sq;
    __syncthreads();
    if (tid == 0) {
        double s = 0.0;
        for (int w = 0; w < kAT / 64; ++w) s += red[w];
        partials[(size_t)t * gridDim.x + blockIdx.x] = s;
    }
}

}  // namespace

int ame_align_cross_dispatch(const float* est, const float* tru, int n, int T, int r,
                             int global_mode, double* cross, double* work, hipStream_t st) {
    const int d = 2 + 2 * r;
    if (global_mode) {
        const int w = 2 * r;
        double* mest = work;
        double* mtru = work + (size_t)n * w;
        const long long tot = (long long)n * w;
        hipLaunchKernelGGL(ame_align_means_kernel, dim3((unsigned)((tot + kAT - 1) / kAT)), dim3(kAT),
                           0, st, est, tru, n, T, d, mest, mtru);
        hipLaunchKernelGGL(ame_align_cross_kernel<double>, dim3(1, 1), dim3(kAT), 0, st,
                           (const double*)mest, (const double*)mtru, n, (long long)w, 0LL, 0, 0, w,
                           cross);
    } else {
        hipLaunchKernelGGL(ame_align_cross_kernel<float>, dim3(T, 2), dim3(kAT), 0, st, est, tru, n,
                           (long long)T * d, (long long)d, 2, r, r, cross);
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ame_align_apply_dispatch(const float* est, const float* tru, int n, int T, int r,
                             int global_mode, const double* rot, float* out, double* partials,
                             hipStream_t st) {
    const dim3 grid((n + kAT - 1) / kAT, T);
    switch (r) {
#define X(RR)                                                                                    \
    case RR:                                                                                     \
        hipLaunchKernelGGL(ame_align_apply_kernel<RR>, grid, dim3(kAT), 0, st, est, tru, n, T,   \
                           global_mode, rot, out, partials);                                     \
        break;
        AME_FOR_EACH_R(X)
#undef X
        default:
            return -1;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

long long ame_align_partials_count(int n, int T) { return (long long)((n + kAT - 1) / kAT) * T; }
