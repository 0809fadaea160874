// K1b: covariance update + per-(node,time) covariance terms of the ELBO.
//
// Reference: the covariance half of _update_node_i (structured_mf.py:266-287:
// C = inv(P); bad: zero off-diagonal blocks; C = (C+C^T)/2 + 1e-6 I; damped
// into X_cov), naive_mf.py:270-282 (C = diag(1/(diag P + 1e-8))), and the
// covariance-only ELBO pieces: entropy logdet (structured_mf.py:202-209),
// trace correction (:142-144), tr(S0^-1 S) (:166), tr(Q^-1 S) (:193).
//
// Covariances never feed back into the means, so this work is
// off the sweep's critical path and runs fully parallel: one wave per
// (node, slice).  Each wave rebuilds the precision the sweep used for its
// step from the sweep's statistic snapshot + replay of the intervening nodes'
// (old -> new) statistic deltas, with the same explicitly-rounded operations
// (ame_common.h), so P is bit-identical to the sweep's.
//
// Linear algebra on a column-per-lane register layout: lane m holds column m.
// The symmetric sweep operator (Goodnight 1979) inverts in place; written so
// that products are formed symmetrically, the result is EXACTLY symmetric,
// which makes the reference's symmetrisation (C + C^T)/2 an identity.
#include "ame_common.h"

// Per-wave LDS: replayed statistics, a row buffer and the nodes' (U,V).
template <int R>
struct CovWaveLds {
    static constexpr int NS = AmeCfg<R>::NS, D = AmeCfg<R>::D, M2 = AmeCfg<R>::M2;
    double S[NS];
    double row[64];
    float uv_old[M2];
    float uv_new[M2];
};

// In-place symmetric sweep of every pivot: col (lane m's column of A) -> -A^-1.
template <int D>
__device__ __forceinline__ void sweep_all(double (&col)[D], double* row, int lane) {
#pragma unroll
    for (int pv = 0; pv < D; ++pv) {
        row[lane] = col[pv];   // A[pv][lane] (symmetric: = A[lane][pv])
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double piv = row[pv];
        const double rinv = 1.0 / piv;
        const double apm = col[pv];
        const bool isp = (lane == pv);
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if (k == pv) continue;
            const double rk = row[k];
            col[k] = isp ? col[k] * rinv : col[k] - (rk * apm) * rinv;
        }
        col[pv] = isp ? -rinv : apm * rinv;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// log|det| by forward elimination (pivots of the LDL^T factorisation), torch
// semantics: nan for a negative determinant, -inf for a zero one.
template <int D>
__device__ __forceinline__ double logdet_sym(double (&col)[D], double* row, int lane) {
    double ld = 0.0;
    int neg = 0;
    bool zero = false;
#pragma unroll
    for (int pv = 0; pv < D; ++pv) {
        row[lane] = col[pv];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const double piv = row[pv];
        if (piv == 0.0) zero = true;
        if (piv < 0.0) neg ^= 1;
        ld += log(fabs(piv));
        const double rinv = 1.0 / piv;
        const double apm = col[pv];
        if (lane > pv) {
#pragma unroll
            for (int k = pv + 1; k < D; ++k) col[k] = col[k] - (row[k] * apm) * rinv;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (zero) return -INFINITY;
    if (neg) return NAN;
    return ld;
}

template <int R>
__global__ void __launch_bounds__(AME_NT)
ame_cov_kernel(ame_dims dm, ame_cov_args a) {
    using C = AmeCfg<R>;
    constexpr int D = C::D, M2 = C::M2, NS = C::NS;
    const int n = dm.n, Tt = dm.T_total;
    const int nblk = (n + AME_SNAP_NB - 1) / AME_SNAP_NB;
    const int tl = blockIdx.x / nblk, b = blockIdx.x - tl * nblk;
    const int tg = dm.t_begin + tl;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int variant = dm.variant;
    const int i0 = b * AME_SNAP_NB;
    const int i1 = min(n, i0 + AME_SNAP_NB);

    __shared__ CovWaveLds<R> lds[AME_NT / 64];
    CovWaveLds<R>& L = lds[w];

    const double p = a.rinv[0], s = a.rinv[3];
    const double q = 0.5 * (a.rinv[1] + a.rinv[2]);
    const double nm1 = (double)(n - 1);
    const size_t DD = (size_t)D * D;
    const float* xo = a.x_old + (size_t)tl * n * D;
    const float* xn = a.x_new + (size_t)tl * n * D;

    // this wave's replay state: S before node `cur`
    int cur = i0;
    if (a.update) {
        const double* src = a.snap + ((size_t)tl * nblk + b) * NS;
        for (int e = lane; e < NS; e += 64) L.S[e] = src[e];
    }
    const bool mlane = lane < D;
    const int m = mlane ? lane : 0;

    for (int i = i0 + w; i < i1; i += AME_NT / 64) {
        float* cv = a.cov + (((size_t)tl * n + i) * D) * D;
        double sig[D];   // new covariance, column m
        if (a.update) {
            // replay statistics up to node i
            while (cur < i) {
                if (lane < M2) {
                    L.uv_old[lane] = xo[(size_t)cur * D + 2 + lane];
                    L.uv_new[lane] = xn[(size_t)cur * D + 2 + lane];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int e = lane; e < NS; e += 64)
                    L.S[e] = stat_apply<R>(L.S[e], e, L.uv_new, L.uv_new + R, L.uv_old,
                                           L.uv_old + R);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                ++cur;
            }
            if (lane < M2) L.uv_old[lane] = xo[(size_t)i * D + 2 + lane];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const float* Uo = L.uv_old;
            const float* Vo = L.uv_old + R;

            // column m of the precision (bit-identical to the sweep's)
            double col[D];
#pragma unroll
            for (int k = 0; k < D; ++k)
                col[k] = __dadd_rn(pobs_entry<R>(k, m, L.S, Uo, Vo, p, q, s, nm1),
                                   pconst_entry(a.consts, D, k, m, tg, Tt));
            const float lr = a.lr, om = a.one_minus_lr;
            if (variant == AME_NAIVE) {
                // C = diag(1 / (diag(P) + 1e-8))  (naive_mf.py:271-274)
                float cm = 0.f;
#pragma unroll
                for (int k = 0; k < D; ++k)
                    if (k == m) cm = 1.0f / ((float)col[k] + 1e-8f);
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    const float c32 = (k == m) ? cm : 0.f;
                    const float old = mlane ? cv[(size_t)k * D + m] : 0.f;
                    sig[k] = (double)__fadd_rn(__fmul_rn(lr, c32), __fmul_rn(om, old));
                }
            } else {
                sweep_all<D>(col, L.row, lane);   // col = -P^-1 column m
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    float c32 = (float)(-col[k]);
                    if (variant == AME_BAD && ((k < 2) != (m < 2))) c32 = 0.f;
                    if (k == m) c32 = c32 + 1e-6f;
                    const float old = mlane ? cv[(size_t)k * D + m] : 0.f;
                    sig[k] = (double)__fadd_rn(__fmul_rn(lr, c32), __fmul_rn(om, old));
                }
            }
            if (mlane) {
#pragma unroll
                for (int k = 0; k < D; ++k) cv[(size_t)k * D + m] = (float)sig[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) sig[k] = mlane ? (double)cv[(size_t)k * D + m] : 0.0;
        }
        // ---- covariance terms of the ELBO ----
        double tr = 0.0, trq = 0.0, trs = 0.0;
        if (mlane) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                if (k == m) tr = sig[k];
                trq = fma(a.consts[DD + (size_t)k * D + m], sig[k], trq);
                if (tg == 0) trs = fma(a.consts[(size_t)k * D + m], sig[k], trs);
            }
        }
        // logdet of the stored (fp32) covariance; lanes >= D carry identity columns
        if (!mlane) {
#pragma unroll
            for (int k = 0; k < D; ++k) sig[k] = 0.0;
        }
        const double ld = logdet_sym<D>(sig, L.row, lane);
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
    (void)Tt;
}

template <int R>
static int launch_cov(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    const int nblk = (dm->n + AME_SNAP_NB - 1) / AME_SNAP_NB;
    hipLaunchKernelGGL(ame_cov_kernel<R>, dim3(dm->T_local * nblk), dim3(AME_NT), 0, st, *dm, *a);
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
