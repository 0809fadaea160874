// K2: per-(node,time) covariance terms of the ELBO.
//
// Reference: entropy logdet (structured_mf.py:202-209), the trace correction of
// the expected log-likelihood (:142-144), tr(S0^-1 S_i0) (:166) and
// tr(Q^-1 S_it) (:193).  The covariances are written by the sweep; this kernel
// reads each stored fp32 covariance once (4 d^2 bytes).
//
// Work split (x = [a, b, U(r), V(r)], d = 2 + 2r, B = 2r):
//  * lane l of a covariance's lane group holds column 2 + l of A (rows 0..d-1,
//    one coalesced row-slice per row) -- at 16 <= B <= 32 columns 2 + l and
//    2 + l + LPM (CPL = 2), so one LDS read of each pivot row serves two
//    columns; 64 / LPM covariances per wave, LPM the power of two >= B / CPL;
//  * traces need no elimination: tr A from the diagonal, tr(M A) (M = Q^-1 for
//    t >= 1, Sigma0^-1 at t = 0) as sum_k M[k][2+l] A[k][2+l] per lane (columns
//    0, 1 from rows 0, 1 of the lanes' columns: A is symmetric);
//  * the (a,b) block is eliminated in closed form (the lanes swap their rows
//    0, 1 through LDS), leaving the B x B Schur complement S, factorised LDL^T
//    with column l of S in lane l; the pivot row goes through LDS (one store per
//    lane, broadcast 16-byte reads back).  log|A| = log|A_aa| + sum log pivots,
//    one product with periodic exponent extraction, one log per covariance;
//    torch.logdet semantics: -inf for a zero pivot, nan for a negative
//    determinant.  fp64 throughout;
//  * persistent waves: each wave walks covariance groups with a grid stride and
//    loads the next group's columns while it factorises the current one, and
//    the register footprint allows 2 (r = 32) to 4 (r <= 16) waves per SIMD, so
//    the per-pivot dependent chain (LDS round trip, reciprocal) of one wave
//    overlaps other waves' work.  (Round 2's kernel held one group per wave
//    with no prefetch and spilled at r = 32: 0.61 ms at config 3, 9.9 ms at
//    config 5's rank shape; one column per lane with prefetch: 0.31 ms at
//    config 3; two columns: 0.21 ms, profiles/r03_cov_ab.txt.)
// The input is taken as symmetric: the sweep writes symmetric covariances and
// the reference's initialisation symmetrises (structured_mf.py:94-96).
#include "ame_common.h"

template <int R>
struct CovCfg {
    static constexpr int B = 2 * R, D = B + 2, DD = D * D;
    // columns of the complement per lane: 2 at 16 <= B <= 32, so one LDS read of
    // the pivot row serves two columns (the pivot-row reads, not the FMAs, set
    // the time at one column per lane)
    static constexpr int CPL = (B >= 16 && B <= 32) ? 2 : 1;
    static constexpr int NC = (B + CPL - 1) / CPL;   // lanes one covariance needs
    static constexpr int LPM = NC <= 2 ? 2 : NC <= 4 ? 4 : NC <= 8 ? 8 : NC <= 16 ? 16 : NC <= 32 ? 32 : 64;
    static constexpr int MPW = 64 / LPM;   // covariances per wave-task
    static constexpr int WPB = 4;          // waves per block
    static constexpr int XB = 3 * MPW * B; // LDS doubles per wave: pivot rows | (u0, u1) pairs
    // waves per SIMD the registers allow, and whether the next group's columns
    // are loaded during the elimination (B > 32: the column stays in registers
    // only until the complement is formed; 2 waves per SIMD hide the load instead)
    static constexpr int WAVES = (B > 32 || CPL == 2) ? 2 : 3;
    static constexpr bool PREFETCH = B <= 32;
};

template <int R>
__global__ void __launch_bounds__(256, CovCfg<R>::WAVES)
ame_cov_kernel(ame_dims dm, ame_cov_args a) {
    using C = CovCfg<R>;
    constexpr int B = C::B, D = C::D, DD = C::DD, LPM = C::LPM, MPW = C::MPW, WPB = C::WPB, CPL = C::CPL;
    __shared__ __attribute__((aligned(16))) double qs[2 * DD];          // S0inv, Qinv
    __shared__ __attribute__((aligned(16))) double xb[WPB][C::XB];      // per wave
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int e = tid; e < 2 * DD; e += 256) qs[e] = a.consts[e];
    __syncthreads();
    const long long total = (long long)dm.T_local * dm.n;
    const long long ntask = (total + MPW - 1) / MPW;
    const long long stride = (long long)gridDim.x * WPB;
    const int sub = lane / LPM, l = lane - sub * LPM;
    // column slot c of this lane: complement column l + c * LPM (A column 2 + that);
    // idle slots shadow the last column (same values, so their LDS writes agree)
    int lc[CPL];
    bool lv[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
        const int cl = l + c * LPM;
        lv[c] = cl < B;
        lc[c] = lv[c] ? cl : B - 1;
    }
    double* rb = xb[w] + sub * B;                 // pivot row of this covariance
    double* ub = xb[w] + MPW * B + 2 * sub * B;   // (u0, u1) pairs of its columns

    // loads of one covariance group: this lane's columns (rows 0..D-1) and the (a,b) block
    float v[CPL][D], aa[4];
    auto load = [&](long long task) {
        const long long mc0 = task * MPW + sub;
        const long long mc = mc0 < total ? mc0 : total - 1;
        const float* A = a.cov + mc * DD;
#pragma unroll
        for (int c = 0; c < CPL; ++c)
#pragma unroll
            for (int k = 0; k < D; ++k) v[c][k] = A[k * D + 2 + lc[c]];
        aa[0] = A[0];
        aa[1] = A[1];
        aa[2] = A[D];
        aa[3] = A[D + 1];
    };
    long long task = (long long)blockIdx.x * WPB + w;
    if (task >= ntask) return;   // whole wave; no barrier follows
    if constexpr (C::PREFETCH) load(task);
    for (; task < ntask; task += stride) {
        if constexpr (!C::PREFETCH) load(task);
        const long long mc0 = task * MPW + sub;
        const bool mv = mc0 < total;
        const long long mc = mv ? mc0 : total - 1;
        const int tg = dm.t_begin + (int)(mc / dm.n);
        const double a00 = aa[0], a01 = aa[1], a10 = aa[2], a11 = aa[3];
        // traces: tr A, tr(M A) with M = Sigma0^-1 (t = 0) or Q^-1 (t >= 1)
        const double* M = qs + ((tg == 0) ? 0 : DD);
        const double det2 = a00 * a11 - a01 * a10;
        const double id2 = 1.0 / det2;
        double tm = 0.0, tr = 0.0, w0[CPL], w1[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const int q = lc[c];
            const double u0 = v[c][0], u1 = v[c][1];
            double tmc = M[2 + q] * u0 + M[D + 2 + q] * u1     // rows 0, 1 of column 2 + q
                       + M[(2 + q) * D] * u0 + M[(2 + q) * D + 1] * u1;   // A[2+q][0..1]
            double trc = 0.0;
#pragma unroll
            for (int k = 0; k < B; ++k) {
                const double x = v[c][2 + k];
                tmc = fma(M[(2 + k) * D + 2 + q], x, tmc);
                trc = (k == q) ? x : trc;
            }
            if (lv[c]) {
                tm += tmc;
                tr += trc;
            }
            // Schur complement column: S[k][q] = A[2+k][2+q] - u_k^T A_aa^-1 u_q
            w0[c] = (a11 * u0 - a01 * u1) * id2;
            w1[c] = (a00 * u1 - a10 * u0) * id2;
            ub[2 * q] = u0;
            ub[2 * q + 1] = u1;
        }
        if (l == 0) {
            tr += a00 + a11;
            tm += M[0] * a00 + M[1] * a10 + M[D] * a01 + M[D + 1] * a11;
        }
        asm volatile("" ::: "memory");   // one wave: its LDS ops complete in issue order
        double col[CPL][B];
#pragma unroll
        for (int k = 0; k < B; ++k) {
            const double2 uk = *(const double2*)(ub + 2 * k);
#pragma unroll
            for (int c = 0; c < CPL; ++c) col[c][k] = (double)v[c][2 + k] - (uk.x * w0[c] + uk.y * w1[c]);
        }
        asm volatile("" ::: "memory");
        // LDL^T of S: lane l holds columns l (+ LPM); pivot row through LDS
        double prod = det2;
        int e2 = 0, neg = det2 < 0.0 ? 1 : 0;
        bool zero = det2 == 0.0;
#pragma unroll
        for (int P = 0; P < B; ++P) {
            // slot c is still needed while one of its columns lies past the pivot
#pragma unroll
            for (int c = 0; c < CPL; ++c)
                if ((c + 1) * LPM - 1 >= P) rb[lc[c]] = col[c][P];
            asm volatile("" ::: "memory");
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
            double f[CPL];
#pragma unroll
            for (int c = 0; c < CPL; ++c) f[c] = col[c][P] * ri;
            int k = P + 1;
            if (k & 1) {   // to an even index, then 16-byte reads of two entries
                const double r1 = rb[k];
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    if ((c + 1) * LPM - 1 > P) col[c][k] = fma(-r1, f[c], col[c][k]);
                ++k;
            }
#pragma unroll
            for (; k + 1 < B; k += 2) {
                const double2 r2 = *(const double2*)(rb + k);
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    if ((c + 1) * LPM - 1 > P) {
                        col[c][k] = fma(-r2.x, f[c], col[c][k]);
                        col[c][k + 1] = fma(-r2.y, f[c], col[c][k + 1]);
                    }
                }
            }
            if (k < B) {
                const double r1 = rb[k];
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    if ((c + 1) * LPM - 1 > P) col[c][k] = fma(-r1, f[c], col[c][k]);
            }
            asm volatile("" ::: "memory");
            // the next group's loads fly during the second half of the
            // elimination (half of the columns are dead by then: no spills)
            if constexpr (C::PREFETCH) {   // (clamped: the last round reloads a valid group)
                if (P == B / 2) load(task + stride < ntask ? task + stride : task);
            }
        }
        double ld = log(fabs(prod)) + (double)e2 * 0.69314718055994530942;
        if (zero) ld = -INFINITY;
        else if (neg) ld = NAN;
#pragma unroll
        for (int o = 1; o < LPM; o <<= 1) {
            tr += __shfl_xor(tr, o);
            tm += __shfl_xor(tm, o);
        }
        if (l == 0 && mv) {
            double* o = a.cov_terms + mc * 4;
            o[0] = ld;
            o[1] = tr;
            o[2] = (tg >= 1) ? tm : 0.0;
            o[3] = (tg == 0) ? tm : 0.0;
        }
    }
}

template <int R>
static int launch_cov(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    using C = CovCfg<R>;
    const long long total = (long long)dm->T_local * dm->n;
    const long long waves = (total + C::MPW - 1) / C::MPW;
    long long blocks = (waves + C::WPB - 1) / C::WPB;
    // persistent grid: as many blocks as are co-resident (each wave then walks
    // several covariance groups, prefetching the next)
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ame_cov_kernel<R>, 256, 0) == hipSuccess &&
        cus > 0 && per_cu > 0) {
        const long long cap = (long long)cus * per_cu;
        if (blocks > cap) blocks = cap;
    }
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(ame_cov_kernel<R>, dim3((unsigned)blocks), dim3(256), 0, st, *dm, *a);
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
