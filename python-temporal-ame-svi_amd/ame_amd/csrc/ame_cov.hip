// K2: per-(node,time) covariance terms of the ELBO.
//
// Reference: entropy logdet (structured_mf.py:202-209), the trace correction of
// the expected log-likelihood (:142-144), tr(S0^-1 S_i0) (:166) and
// tr(Q^-1 S_it) (:193).  The covariances are written by the sweep; this kernel
// reads each stored fp32 covariance once (4 d^2 bytes).
//
// Work split (x = [a, b, U(r), V(r)], d = 2 + 2r):
//  * the (a,b) 2x2 block is eliminated first with its closed-form inverse,
//    leaving the 2r x 2r Schur complement S = A_xx - A_xa A_aa^-1 A_ax;
//  * S is factorised LDL^T with column c of S in lane c, so 64 / 2r
//    covariances share a wave (2 at r = 16) and no lane idles; the pivot row
//    goes through LDS (one store per lane, broadcast reads back).
// The input is taken as symmetric: the sweep writes symmetric covariances and
// the reference's initialisation symmetrises (structured_mf.py:94-96).
// log|A| = log|A_aa| + sum log pivots, accumulated as one product with
// periodic exponent extraction (one log per covariance); torch.logdet
// semantics: -inf for a zero pivot, nan for a negative determinant.
#include "ame_common.h"

template <int B>
struct CovLanes {   // lanes per covariance: next power of two >= 2r
    static constexpr int v = B <= 2 ? 2 : B <= 4 ? 4 : B <= 8 ? 8 : B <= 16 ? 16 : B <= 32 ? 32 : 64;
};

// Waves per SIMD the register budget must allow (the unrolled elimination
// otherwise takes 364 VGPRs: one wave per SIMD, latency-bound).
#ifndef AME_COV_WAVES
#define AME_COV_WAVES 1
#endif
template <int R>
__global__ void __launch_bounds__(AME_NT, AME_COV_WAVES)
ame_cov_kernel(ame_dims dm, ame_cov_args a) {
    constexpr int D = 2 + 2 * R, B = 2 * R, DD = D * D;
    constexpr int LPM = CovLanes<B>::v, MPW = 64 / LPM, WPB = AME_NT / 64;
    __shared__ double qs[2 * DD];                                   // S0inv, Qinv
    __shared__ __attribute__((aligned(16))) double rows[WPB][64];   // pivot rows
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int e = tid; e < 2 * DD; e += AME_NT) qs[e] = a.consts[e];
    __syncthreads();
    const long long total = (long long)dm.T_local * dm.n;
    const long long first = ((long long)blockIdx.x * WPB + w) * MPW;
    if (first >= total) return;   // whole wave; no barrier follows
    const int sub = lane / LPM, l = lane - sub * LPM;
    const bool mv = first + sub < total;
    const long long mc = mv ? first + sub : total - 1;
    const int tl = (int)(mc / dm.n);
    const int tg = dm.t_begin + tl;
    const bool lv = l < B;
    const int c = 2 + (lv ? l : 0);
    const float* A = a.cov + mc * DD;
    const double* S0 = qs;
    const double* Qi = qs + DD;

    // the (a,b) block and this lane's column c in rows 0, 1
    const double a00 = A[0], a01 = A[1], a10 = A[D], a11 = A[D + 1];
    const double u0 = A[c], u1 = A[D + c];
    const double det2 = a00 * a11 - a01 * a10;
    const double id2 = 1.0 / det2;
    const double w0 = (a11 * u0 - a01 * u1) * id2;   // A_aa^-1 (A_0c, A_1c)
    const double w1 = (a00 * u1 - a10 * u0) * id2;
    // traces: column c (rows 0, 1 here, rows >= 2 in the loop) and columns 0, 1
    // (every lane computes them, lane l == 0 keeps them)
    double tq = Qi[c] * u0 + Qi[D + c] * u1;
    double tq0 = Qi[0] * a00 + Qi[1] * a10 + Qi[D] * a01 + Qi[D + 1] * a11;
    double tr = 0.0;
    double col[B];
#pragma unroll
    for (int k = 0; k < B; ++k) {
        const float* rk = A + (2 + k) * D;
        const double x = rk[c], c0 = rk[0], c1 = rk[1];
        tq = fma(Qi[(2 + k) * D + c], x, tq);
        tr = (k == l) ? x : tr;
        tq0 = fma(Qi[2 + k], c0, fma(Qi[D + 2 + k], c1, tq0));
        col[k] = x - (c0 * w0 + c1 * w1);
        if ((k & 7) == 7) asm volatile("" ::: "memory");
    }
    double ts = 0.0;
    if (__any(tg == 0)) {   // tr(S0inv A): first time slice only (wave-uniform branch)
        ts = S0[c] * u0 + S0[D + c] * u1;
        double ts0 = S0[0] * a00 + S0[1] * a10 + S0[D] * a01 + S0[D + 1] * a11;
        for (int k = 0; k < B; ++k) {
            const float* rk = A + (2 + k) * D;
            ts = fma(S0[(2 + k) * D + c], (double)rk[c], ts);
            ts0 = fma(S0[2 + k], (double)rk[0], fma(S0[D + 2 + k], (double)rk[1], ts0));
        }
        if (l == 0) ts += ts0;
    }

    // LDL^T of the complement: lane c holds column c; pivot row through LDS
    double* rb = rows[w] + sub * LPM;
    double prod = det2;
    int e2 = 0, neg = det2 < 0.0 ? 1 : 0;
    bool zero = det2 == 0.0;
#pragma unroll
    for (int P = 0; P < B; ++P) {
        rb[l] = col[P];
        asm volatile("" ::: "memory");   // one wave: its LDS ops complete in issue order
        const double piv = rb[P];
        zero |= piv == 0.0;
        neg ^= piv < 0.0 ? 1 : 0;
        prod *= piv;
        if ((P & 7) == 7 || P == B - 1) {
            int ex;
            prod = frexp(prod, &ex);
            e2 += ex;
        }
        double ri = __builtin_amdgcn_rcp(piv);
        ri = fma(fma(-piv, ri, 1.0), ri, ri);
        ri = fma(fma(-piv, ri, 1.0), ri, ri);
        const double f = col[P] * ri;
#pragma unroll
        for (int k = P + 1; k < B; ++k) col[k] = fma(-rb[k], f, col[k]);
        asm volatile("" ::: "memory");
    }
    double ld = log(fabs(prod)) + (double)e2 * 0.69314718055994530942;
    if (zero) ld = -INFINITY;
    else if (neg) ld = NAN;

    double s_tr = lv ? tr : 0.0, s_tq = lv ? tq : 0.0, s_ts = lv ? ts : 0.0;
    if (l == 0) {
        s_tr += a00 + a11;
        s_tq += tq0;
    }
#pragma unroll
    for (int o = 1; o < LPM; o <<= 1) {
        s_tr += __shfl_xor(s_tr, o);
        s_tq += __shfl_xor(s_tq, o);
        s_ts += __shfl_xor(s_ts, o);
    }
    if (l == 0 && mv) {
        double* o = a.cov_terms + mc * 4;
        o[0] = ld;
        o[1] = s_tr;
        o[2] = (tg >= 1) ? s_tq : 0.0;
        o[3] = (tg == 0) ? s_ts : 0.0;
    }
}

template <int R>
static int launch_cov(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    constexpr int per_block = (AME_NT / 64) * (64 / CovLanes<2 * R>::v);
    const long long total = (long long)dm->T_local * dm->n;
    const long long blocks = (total + per_block - 1) / per_block;
    hipLaunchKernelGGL(ame_cov_kernel<R>, dim3((unsigned)blocks), dim3(AME_NT), 0, st, *dm, *a);
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
