// Shared device helpers for the temporal-AME VI kernels (gfx950 / CDNA4).
//
// The sweep kernel (ame_sweep.hip) and the covariance kernel (ame_cov.hip) must
// build BIT-IDENTICAL precision matrices for step (i,t): the covariance kernel
// replays the sweep's running statistics from snapshots.  Every operation on
// that path therefore goes through the explicitly-rounded helpers below
// (__dadd_rn / __dsub_rn / __dmul_rn), so no FMA contraction can make the two
// kernels diverge.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/ame_amd.h"

#define AME_NT 256          // threads per workgroup
#define AME_SNAP_NB 16      // sweep statistic snapshot stride (nodes)
// Spin bounds in s_memrealtime ticks (constant 100 MHz clock): a hand-off that
// does not arrive within this time sets a status bit and the sweep finishes.
#define AME_SPIN_TICKS_LOCAL (200ull * 1000 * 1000)   // 2 s, lane -> lane on one GPU
#define AME_SPIN_TICKS_HALO (1000ull * 1000 * 1000)   // 10 s, rank -> rank

template <int R>
struct AmeCfg {
    static constexpr int D = 2 + 2 * R;            // state dim
    static constexpr int M2 = 2 * R;               // (U, V) width
    static constexpr int NS = 2 * R + 3 * R * R;   // running statistics
    // GEMV vector width: a chunk never straddles the U/V halves.
    static constexpr int VEC = (R % 4 == 0) ? 4 : ((R % 2 == 0) ? 2 : 1);
    static constexpr int CW = M2 / VEC;            // column chunks
    static constexpr int G = AME_NT / CW;          // node groups
    static constexpr int PW = M2 + 2;              // partial row width (+ sum z0, sum z1)
    static constexpr int W = D + 2;                // augmented matrix row stride
    static constexpr int QN = (D * D + AME_NT - 1) / AME_NT;   // P entries per thread
    static constexpr int MC = (D + 3) / 4;         // AR matvec columns per thread
};

// ---------------------------------------------------------------------------
// Running statistics of node means at one time slice.  Entry e:
//   [0,R)            sum U_k
//   [R,2R)           sum V_k
//   [2R,2R+R^2)      sum U_k U_l     (k*R + l)
//   [.., +R^2)       sum V_k V_l
//   [.., +R^2)       sum V_k U_l
// These are the sufficient statistics of P_obs: the reference
// accumulates J^T R^-1 J over j != i (structured_mf.py:303-324).
// ---------------------------------------------------------------------------
template <int R>
__device__ __forceinline__ double stat_val(int e, const float* U, const float* V) {
    constexpr int R2 = R * R;
    if (e < R) return (double)U[e];
    if (e < 2 * R) return (double)V[e - R];
    int f = e - 2 * R;
    if (f < R2) { int k = f / R, l = f - k * R; return __dmul_rn((double)U[k], (double)U[l]); }
    f -= R2;
    if (f < R2) { int k = f / R, l = f - k * R; return __dmul_rn((double)V[k], (double)V[l]); }
    f -= R2;
    { int k = f / R, l = f - k * R; return __dmul_rn((double)V[k], (double)U[l]); }
}

// S[e] += stat(new) - stat(old): the only way the statistics ever change.
template <int R>
__device__ __forceinline__ double stat_apply(double s, int e, const float* Un, const float* Vn,
                                             const float* Uo, const float* Vo) {
    return __dadd_rn(s, __dsub_rn(stat_val<R>(e, Un, Vn), stat_val<R>(e, Uo, Vo)));
}

// P_obs[k][m] for node i from S (all nodes, current) minus node i's own (old)
// contribution.  J_j = [[1,0,V_j,0],[0,1,0,U_j]] (structured_mf.py:309-320);
// q = symmetrised off-diagonal of R_inv.
template <int R>
__device__ __forceinline__ double pobs_entry(int k, int m, const double* S, const float* Uo,
                                             const float* Vo, double p, double q, double s,
                                             double nm1) {
    constexpr int R2 = R * R;
    if (k < 2 && m < 2) {
        const double c = (k == 0 && m == 0) ? p : ((k == 1 && m == 1) ? s : q);
        return __dmul_rn(c, nm1);
    }
    if (k < 2 || m < 2) {
        const int ab = (k < 2) ? k : m;
        const int c = ((k < 2) ? m : k) - 2;
        if (c < R) {   // U_c column: a -> p*sum V_c, b -> q*sum V_c
            const double sv = __dsub_rn(S[R + c], (double)Vo[c]);
            return __dmul_rn(ab == 0 ? p : q, sv);
        }
        const double su = __dsub_rn(S[c - R], (double)Uo[c - R]);   // V column
        return __dmul_rn(ab == 0 ? q : s, su);
    }
    const int ck = k - 2, cm = m - 2;
    if (ck < R && cm < R) {   // U,U block: p * sum V_ck V_cm
        const int e = 2 * R + R2 + ck * R + cm;
        return __dmul_rn(p, __dsub_rn(S[e], __dmul_rn((double)Vo[ck], (double)Vo[cm])));
    }
    if (ck >= R && cm >= R) {   // V,V block: s * sum U U
        const int e = 2 * R + (ck - R) * R + (cm - R);
        return __dmul_rn(s, __dsub_rn(S[e], __dmul_rn((double)Uo[ck - R], (double)Uo[cm - R])));
    }
    if (ck < R) {   // row U_ck, col V_(cm-R): q * sum V_ck U_(cm-R)
        const int e = 2 * R + 2 * R2 + ck * R + (cm - R);
        return __dmul_rn(q, __dsub_rn(S[e], __dmul_rn((double)Vo[ck], (double)Uo[cm - R])));
    }
    {   // row V_(ck-R), col U_cm: q * sum V_cm U_(ck-R)
        const int e = 2 * R + 2 * R2 + cm * R + (ck - R);
        return __dmul_rn(q, __dsub_rn(S[e], __dmul_rn((double)Vo[cm], (double)Uo[ck - R])));
    }
}

// Constant part of the precision at global time tg (structured_mf.py:251-264):
//   [t==0] Sigma0^-1 + [t>0] Q^-1 + [t<T-1] Phi^T Q^-1 Phi.
__device__ __forceinline__ double pconst_entry(const double* consts, int D, int k, int m, int tg,
                                               int T) {
    const size_t DD = (size_t)D * D;
    const size_t o = (size_t)k * D + m;
    double v = (tg == 0) ? consts[o] : consts[DD + o];
    if (tg < T - 1) v = __dadd_rn(v, consts[2 * DD + o]);
    return v;
}

// Granule hand-off (cdna_hip_programming.md G16 R2): one 8-byte {epoch, value}
// word written by ONE sc1 store; the consumer re-reads until every tag matches.
__device__ __forceinline__ uint64_t gran_load_agent(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t gran_load_system(const uint64_t* p) {
    return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void gran_store_agent(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gran_store_system(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Deterministic workgroup sum of NV doubles per thread (fixed tree order).
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* scratch /* 4*NV */) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NV; ++q) v[q] = wave_sum(v[q]);
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < NV; ++q) scratch[w * NV + q] = v[q];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            double s = 0.0;
            for (int ww = 0; ww < (int)(blockDim.x >> 6); ++ww) s += scratch[ww * NV + q];
            v[q] = s;
        }
    }
}

// Dynamic LDS carve-up of the sweep kernel (host and device agree).
struct SweepLds {
    long long oS, oA, oVh, oVar, oF, oPart, oZ, oM, total;
};
__host__ __device__ inline long long ame_align16(long long x) { return (x + 15) & ~15LL; }
__host__ __device__ inline SweepLds sweep_lds_layout(int n, int R) {
    const int D = 2 + 2 * R, M2 = 2 * R, NS = 2 * R + 3 * R * R, W = D + 2;
    const int VEC = (R % 4 == 0) ? 4 : ((R % 2 == 0) ? 2 : 1);
    const int G = AME_NT / (M2 / VEC);
    SweepLds L;
    long long o = 0;
    L.oS = o;    o = ame_align16(o + 8LL * NS);
    L.oA = o;    o = ame_align16(o + 8LL * D * W);
    L.oVh = o;   o = ame_align16(o + 8LL * D);
    L.oVar = o;  o = ame_align16(o + 8LL * D);
    L.oF = o;    o = ame_align16(o + 4LL * 4 * D);          // mu_prev, mu_next, mu_old, mu_new
    L.oPart = o; o = ame_align16(o + 4LL * G * (M2 + 2));
    L.oZ = o;    o = ame_align16(o + 8LL * n);
    L.oM = o;    o = ame_align16(o + 4LL * n * M2);
    L.total = o;
    return L;
}

#ifdef AME_ONLY_R   // diagnostic builds: one latent dim only
#define AME_FOR_EACH_R(X) X(AME_ONLY_R)
#else
#define AME_FOR_EACH_R(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(12) X(16) X(24)
#endif
