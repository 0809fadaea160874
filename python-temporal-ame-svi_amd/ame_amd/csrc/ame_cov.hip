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
// Linear algebra on a column-per-lane register layout: lane m holds column m
// (fp64).  Pivot steps are template-recursive so every register index is a
// compile-time constant (no scratch).  The symmetric sweep operator
// (Goodnight 1979) inverts in place; products are formed symmetrically, so
// the result is EXACTLY symmetric and the reference's symmetrisation
// (C + C^T)/2 is an identity.
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

// Symmetric sweep of pivot P (and all later ones): col -> -A^-1 column.
template <int D, int P>
__device__ __forceinline__ void sweep_from(double (&col)[D], double* row, int lane) {
    if constexpr (P < D) {
        row[lane] = col[P];   // A[P][lane] (= A[lane][P])
        wave_sync();
        const double rinv = 1.0 / row[P];
        const double apm = col[P];
        const bool isp = (lane == P);
#pragma unroll
        for (int k0 = 0; k0 < D; k0 += 4) {
#pragma unroll
            for (int k = k0; k < k0 + 4 && k < D; ++k) {
                if (k == P) continue;
                const double rk = row[k];
                col[k] = isp ? col[k] * rinv : col[k] - (rk * apm) * rinv;
            }
            asm volatile("" ::: "memory");   // consume the broadcast row in chunks
        }
        col[P] = isp ? -rinv : apm * rinv;
        wave_sync();
        sweep_from<D, P + 1>(col, row, lane);
    }
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
struct CovWaveLds {
    static constexpr int NS = AmeCfg<R>::NS, M2 = AmeCfg<R>::M2;
    double S[NS];
    double row[64];
    float uv_old[M2];
    float uv_new[M2];
};

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
    const bool mlane = lane < D;
    const int m0 = mlane ? lane : 0;
    const float lr = a.lr, om = a.one_minus_lr;

    int cur = i0;
    if (a.update) {
        const double* src = a.snap + ((size_t)tl * nblk + b) * NS;
        for (int e = lane; e < NS; e += 64) L.S[e] = src[e];
    }

    for (int i = i0 + w; i < i1; i += AME_NT / 64) {
        float* cv = a.cov + (((size_t)tl * n + i) * D) * D;
        // opaque per-iteration copies: stop LICM from hoisting D per-k addresses
        // and compare masks out of the node loop (they spill otherwise)
        const double* consts = a.consts;
        int m = m0;
        asm volatile("" : "+s"(consts));
        asm volatile("" : "+v"(m), "+v"(cv));
        double col[D];
        if (a.update) {
            while (cur < i) {   // replay the statistics up to node i
                if (lane < M2) {
                    L.uv_old[lane] = xo[(size_t)cur * D + 2 + lane];
                    L.uv_new[lane] = xn[(size_t)cur * D + 2 + lane];
                }
                wave_sync();
                for (int e = lane; e < NS; e += 64)
                    L.S[e] = stat_apply<R>(L.S[e], e, L.uv_new, L.uv_new + R, L.uv_old,
                                           L.uv_old + R);
                wave_sync();
                ++cur;
            }
            if (lane < M2) L.uv_old[lane] = xo[(size_t)i * D + 2 + lane];
            wave_sync();
            // column m of the precision, bit-identical to the sweep's
#pragma unroll
            for (int k = 0; k < D; ++k) {
                col[k] = __dadd_rn(pobs_entry<R>(k, m, L.S, L.uv_old, L.uv_old + R, p, q, s, nm1),
                                   pconst_entry(consts, D, k, m, tg, Tt));
                AME_CHUNK(k);
            }
            if (variant == AME_NAIVE) {
                // C = diag(1 / (diag(P) + 1e-8))  (naive_mf.py:271-274)
                double pmm = 0.0;
#pragma unroll
                for (int k = 0; k < D; ++k)
                    if (k == m) pmm = col[k];
                const float cm = 1.0f / ((float)pmm + 1e-8f);
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    const float c32 = (k == m) ? cm : 0.f;
                    const float old = mlane ? cv[(size_t)k * D + m] : 0.f;
                    const float nw = __fadd_rn(__fmul_rn(lr, c32), __fmul_rn(om, old));
                    if (mlane) cv[(size_t)k * D + m] = nw;
                    col[k] = (double)nw;
                    AME_CHUNK(k);
                }
            } else {
                sweep_from<D, 0>(col, L.row, lane);   // col = -(P^-1) column m
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    float c32 = (float)(-col[k]);
                    if (variant == AME_BAD && ((k < 2) != (m < 2))) c32 = 0.f;
                    if (k == m) c32 = c32 + 1e-6f;
                    const float old = mlane ? cv[(size_t)k * D + m] : 0.f;
                    const float nw = __fadd_rn(__fmul_rn(lr, c32), __fmul_rn(om, old));
                    if (mlane) cv[(size_t)k * D + m] = nw;
                    col[k] = (double)nw;
                    AME_CHUNK(k);
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                col[k] = mlane ? (double)cv[(size_t)k * D + m] : 0.0;
                AME_CHUNK(k);
            }
        }
        // ---- covariance terms of the ELBO (of the stored fp32 covariance) ----
        double tr = 0.0, trq = 0.0, trs = 0.0;
        if (mlane) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                if (k == m) tr = col[k];
                trq = fma(consts[DD + (size_t)k * D + m], col[k], trq);
                if (tg == 0) trs = fma(consts[(size_t)k * D + m], col[k], trs);
                AME_CHUNK(k);
            }
        } else {
#pragma unroll
            for (int k = 0; k < D; ++k) col[k] = 0.0;
        }
        double ld = 0.0;
        int neg = 0;
        bool zero = false;
        elim_from<D, 0>(col, L.row, lane, ld, neg, zero);
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
