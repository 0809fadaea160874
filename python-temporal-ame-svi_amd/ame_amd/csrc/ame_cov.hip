// K1b: per-(node,time) covariance terms of the ELBO.
//
// Reference: entropy logdet (structured_mf.py:202-209), the trace correction of
// the expected log-likelihood (:142-144), tr(S0^-1 S_i0) (:166) and
// tr(Q^-1 S_it) (:193).  The covariances themselves are written by the sweep
// (ame_sweep.hip); this kernel reads each stored fp32 covariance once.
//
// One wave per (node, slice), column-per-lane fp64 registers (lane m holds
// column m).  log|S| is the sum of log pivots of a forward elimination
// (LDL^T), torch.logdet semantics for indefinite input.  Pivot steps are
// template-recursive so every register index is a compile-time constant.
#include "ame_common.h"

// Bound the scheduler's load hoisting inside fully-unrolled D-loops: without it
// hipcc issues every global/LDS load of the loop up front (>400 registers).
#define AME_CHUNK(k) \
    if (((k) & 3) == 3) asm volatile("" ::: "memory")

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Forward elimination of pivot P (and all later ones): accumulates log|piv|.
template <int D, int P>
__device__ __forceinline__ void elim_from(double (&col)[D], double* row, int lane, double& ld,
                                          int& neg, bool& zero) {
    if constexpr (P < D) {
        row[lane] = col[P];
        wave_sync();
        const double piv = row[P];
        zero |= (piv == 0.0);
        neg ^= (piv < 0.0) ? 1 : 0;
        ld += log(fabs(piv));
        const double f = (lane > P) ? col[P] / piv : 0.0;
#pragma unroll
        for (int k0 = P + 1; k0 < D; k0 += 4) {
#pragma unroll
            for (int k = k0; k < k0 + 4 && k < D; ++k) col[k] = fma(-row[k], f, col[k]);
            asm volatile("" ::: "memory");
        }
        wave_sync();
        elim_from<D, P + 1>(col, row, lane, ld, neg, zero);
    }
}


template <int R>
__global__ void __launch_bounds__(AME_NT)
ame_cov_kernel(ame_dims dm, ame_cov_args a) {
    constexpr int D = 2 + 2 * R;
    const int n = dm.n;
    const int per = (n + 3) / 4;
    const int tl = blockIdx.x / per;
    const int i = (blockIdx.x - tl * per) * 4 + (threadIdx.x >> 6);
    const int tg = dm.t_begin + tl;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    __shared__ double rows[AME_NT / 64][64];
    if (i >= n) return;   // whole wave exits; no workgroup barrier below
    const size_t DD = (size_t)D * D;
    const bool mlane = lane < D;
    const float* cv = a.cov + (((size_t)tl * n + i) * D) * D;
    const double* consts = a.consts;
    int m = mlane ? lane : 0;
    asm volatile("" : "+s"(consts));
    asm volatile("" : "+v"(m), "+v"(cv));
    double col[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        col[k] = mlane ? (double)cv[(size_t)k * D + m] : 0.0;
        AME_CHUNK(k);
    }
    double tr = 0.0, trq = 0.0, trs = 0.0;
    if (mlane) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if (k == m) tr = col[k];
            trq = fma(consts[DD + (size_t)k * D + m], col[k], trq);
            if (tg == 0) trs = fma(consts[(size_t)k * D + m], col[k], trs);
            AME_CHUNK(k);
        }
    }
    double ld = 0.0;
    int neg = 0;
    bool zero = false;
    elim_from<D, 0>(col, rows[w], lane, ld, neg, zero);
    if (zero) ld = -INFINITY;
    else if (neg) ld = NAN;
    tr = wave_sum(tr);
    trq = wave_sum(trq);
    trs = wave_sum(trs);
    if (lane == 0) {
        double* o = a.cov_terms + ((size_t)tl * n + i) * 4;
        o[0] = ld;
        o[1] = tr;
        o[2] = (tg >= 1) ? trq : 0.0;
        o[3] = (tg == 0) ? trs : 0.0;
    }
}

template <int R>
static int launch_cov(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    const int per = (dm->n + 3) / 4;
    hipLaunchKernelGGL(ame_cov_kernel<R>, dim3(dm->T_local * per), dim3(AME_NT), 0, st, *dm, *a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ame_cov_dispatch(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    switch (dm->r) {
#define X(RR) \
    case RR: return launch_cov<RR>(dm, a, st);
        AME_FOR_EACH_R(X)
#undef X
        default: return -1;
    }
}
