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
// Two forms: the column-per-lane LDL^T below (r < AME_COV_MFMA_MIN_R) and, for
// wide states, a blocked LDL^T on fp64 MFMA (ame_cov_mfma_kernel, further down;
// DESIGN.md §4 K2, profiles/r05_cov_ab.txt).
#include "ame_common.h"
#include "ame_wave.h"
#include <type_traits>

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

// ---------------------------------------------------------------------------
// MFMA form (r >= AME_COV_MFMA_MIN_R).  Why: the column-per-lane form above
// delivers the pivot row to every lane through LDS -- one 8-byte LDS return
// per FMA, ~1 MB of LDS data per 64 x 64 complement -- and at r = 32 that is
// its bound (1.9 ms at config 5's rank shape, 0.15 of HBM).  Here one wave
// owns one covariance and keeps the 2r x 2r complement as the lower 16 x 16
// tiles of v_mfma_f64_16x16x4_f64's accumulator layout (lane l, register v:
// row (l >> 4) + 4 v, column l & 15), padded to a multiple of 16 with the
// identity (pivots 1: no change to log|S|).  Right-looking blocked LDL^T in
// panels of 4 columns:
//  a) the panel's 4 columns (rows >= 16 J_p) leave the tiles through LDS into
//     row-per-lane form (lane r: row r; rows above the panel zeroed);
//  b) its 4 pivots eliminate inside the panel, the pivot row by v_readlane;
//  c) every trailing tile takes the panel's rank-4 update as ONE MFMA (K = 4):
//     S_IJ -= (W_I diag(1/piv)) W_J^T, operands read back column-major (lane
//     (i, k) holds W[16 I + i][k]).
// Tile entries left of / above the trailing block are updated as well and
// never read again (each panel leaves the tiles before its update).  The
// (a,b) block's Schur correction S = A22 - U A_aa^-1 U^T is one MFMA per tile
// too (K = 2 of 4, the other operand lanes zero).  Traces come from the
// loaded entries with per-lane weights (tiles below the diagonal count their
// mirror: M symmetric), Q^-1's from LDS, S0^-1's (slice 0 only) from global.
// LDS carries ~60 KB per 64 x 64 covariance instead of ~1 MB.
// ---------------------------------------------------------------------------
#ifndef AME_COV_MFMA_MIN_R
#define AME_COV_MFMA_MIN_R 20
#endif
typedef double ame_d4 __attribute__((ext_vector_type(4)));

#ifdef AME_COV_STAMPS
// Diagnostic build only (tools/build_variant.py --defs=AME_COV_STAMPS): wave 0
// of block 0 records s_memtime at the phase boundaries of its first 16
// covariances (tools/cov_stamps.py).
__device__ unsigned long long g_cov_st[16 * 8];
#define CST(slot)                                                                              \
    do {                                                                                       \
        if (blockIdx.x == 0 && w == 0 && lane == 0 && it < 16) {                               \
            unsigned long long t_;                                                             \
            __builtin_amdgcn_sched_barrier(0);                                                 \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
            __builtin_amdgcn_sched_barrier(0);                                                 \
            g_cov_st[it * 8 + (slot)] = t_;                                                    \
        }                                                                                      \
    } while (0)
extern "C" int ame_debug_read_cov_stamps(unsigned long long* st) {
    return hipMemcpyFromSymbol(st, HIP_SYMBOL(g_cov_st), sizeof(g_cov_st), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define CST(slot) do { } while (0)
#endif

template <int R>
struct CovM {
    static constexpr int B = 2 * R, D = B + 2, DD = D * D;
    static constexpr int NT = (B + 15) / 16;          // tiles per dimension
    static constexpr int BP = 16 * NT;                // padded complement
    static constexpr int NTL = NT * (NT + 1) / 2;     // lower tiles, I >= J
    static constexpr int NWT = 4 * NTL + 2 * NT;      // trace weights per lane
    static constexpr int WPB = 4;                     // waves per block
};
__host__ __device__ constexpr int cov_ti(int I, int J) { return I * (I + 1) / 2 + J; }

// weight of this lane's loaded entry `pos` in tr(M A), M symmetric: entries
// 0 .. 4 NTL-1 are tile registers (below-diagonal tiles stand for their mirror
// as well), then the (a,b)-column pairs of rows 16 I + (lane & 15) (counted on
// lanes 0..15, for A[k][0..1] and A[0..1][k])
template <int R>
__device__ __forceinline__ double cov_mweight(const double* M, int pos, int lane) {
    using C = CovM<R>;
    if (pos < 4 * C::NTL) {
        const int t = pos >> 2, v = pos & 3;
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int J = t - I * (I + 1) / 2;
        const int row = 16 * I + (lane >> 4) + 4 * v, col = 16 * J + (lane & 15);
        if (row >= C::B || col >= C::B) return 0.0;
        const double m = M[(2 + row) * C::D + 2 + col];
        return I > J ? 2.0 * m : m;
    }
    const int q = pos - 4 * C::NTL, I = q >> 1, kk = q & 1;
    const int row = 16 * I + (lane & 15);
    if ((lane >> 4) != 0 || row >= C::B) return 0.0;
    return 2.0 * M[kk * C::D + 2 + row];
}

template <int R, class WF>
__device__ __forceinline__ double cov_mtrace(const ame_d4 (&tile)[CovM<R>::NTL], const float2 (&u)[CovM<R>::NT],
                                             WF wf) {
    using C = CovM<R>;
    double tm = 0.0;
#pragma unroll
    for (int t = 0; t < C::NTL; ++t) {
#pragma unroll
        for (int v = 0; v < 4; ++v) tm = fma(wf(4 * t + v), tile[t][v], tm);
    }
#pragma unroll
    for (int I = 0; I < C::NT; ++I) {
        tm = fma(wf(4 * C::NTL + 2 * I), (double)u[I].x, tm);
        tm = fma(wf(4 * C::NTL + 2 * I + 1), (double)u[I].y, tm);
    }
    return tm;
}

// Covariances [mc0, mc1) of the local block, all with the same trace matrix:
// msel 0 = S0^-1 (slice 0), 1 = Q^-1 (the host splits the launch at slice 1)
#ifndef AME_COV_MFMA_WAVES
#define AME_COV_MFMA_WAVES 3
#endif
template <int R>
__global__ void __launch_bounds__(256, AME_COV_MFMA_WAVES)
ame_cov_mfma_kernel(ame_dims dm, ame_cov_args a, long long mc0, long long mc1, int msel) {
    using C = CovM<R>;
    constexpr int B = C::B, D = C::D, DD = C::DD, NT = C::NT, BP = C::BP, NTL = C::NTL, NWT = C::NWT,
                  WPB = C::WPB;
    __shared__ double wq[NWT * 64];                                  // trace weights [pos][lane]
    __shared__ __attribute__((aligned(16))) double pbuf[WPB][64 * 4];   // per wave: the panel
    // w uniform (readfirstlane): the covariance's base address stays in SGPRs and
    // the tile loads take 32-bit lane offsets
    const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const double* M = a.consts + (msel ? DD : 0);
    for (int e = tid; e < NWT * 64; e += 256) wq[e] = cov_mweight<R>(M, e >> 6, e & 63);
    __syncthreads();
    const double m00 = M[0], m01 = M[1], m10 = M[D], m11 = M[D + 1];
    const long long stride = (long long)gridDim.x * WPB;
    const int g = lane >> 4, c = lane & 15;
    double* pb = pbuf[w];
    int it = 0;   // (stamps only)
    for (long long mc = mc0 + (long long)blockIdx.x * WPB + w; mc < mc1; mc += stride, ++it) {
        CST(0);
        const float* A = a.cov + mc * DD;
        const double a00 = A[0], a01 = A[1], a10 = A[D], a11 = A[D + 1];
        float2 u[NT];   // A[2 + row][0..1], row = 16 I + c
        float ft[NTL][4];   // tile entries as loaded (padding: the identity)
#pragma unroll
        for (int I = 0; I < NT; ++I) {
            const int row = 16 * I + c;
            u[I] = row < B ? *(const float2*)(A + (2 + row) * D) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int row = 16 * I + g + 4 * v, col = 16 * J + c;
                    ft[cov_ti(I, J)][v] = (row < B && col < B) ? A[(2 + row) * D + 2 + col]
                                                               : (row == col ? 1.f : 0.f);
                }
        // ---- traces, from the entries as loaded; the weights stream through
        // (scheduling regions of two tiles: hoisted all at once, the 48 fp64
        // weights held 96 VGPRs beside the tiles) ----
        double tr = (lane == 0) ? a00 + a11 : 0.0;
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int row = 16 * I + g + 4 * v;
                if (row < B && g + 4 * v == c) tr += (double)ft[cov_ti(I, I)][v];
            }
        double tm = (lane == 0) ? m00 * a00 + m01 * a10 + m10 * a01 + m11 * a11 : 0.0;
#pragma unroll
        for (int I = 0; I < NT; ++I) {
            tm = fma(wq[(4 * NTL + 2 * I) * 64 + lane], (double)u[I].x, tm);
            tm = fma(wq[(4 * NTL + 2 * I + 1) * 64 + lane], (double)u[I].y, tm);
        }
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
#pragma unroll
            for (int v = 0; v < 4; ++v) tm = fma(wq[(4 * t + v) * 64 + lane], (double)ft[t][v], tm);
            if (t & 1) asm volatile("" : "+v"(tm)::"memory");
        }
        CST(1);
        // ---- Schur complement of the (a,b) block: S = A22 - U (A_aa^-1 U^T) ----
        const double det2 = a00 * a11 - a01 * a10;
        const double id2 = 1.0 / det2;
        ame_d4 tile[NTL];
        {
            double ua[NT], wb[NT];
#pragma unroll
            for (int I = 0; I < NT; ++I) {
                const double u0 = u[I].x, u1 = u[I].y;
                const double w0 = (a11 * u0 - a01 * u1) * id2, w1 = (a00 * u1 - a10 * u0) * id2;
                ua[I] = g == 0 ? -u0 : (g == 1 ? -u1 : 0.0);
                wb[I] = g == 0 ? w0 : (g == 1 ? w1 : 0.0);
            }
#pragma unroll
            for (int I = 0; I < NT; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J) {
                    const int t = cov_ti(I, J);
                    const ame_d4 a4 = {(double)ft[t][0], (double)ft[t][1], (double)ft[t][2], (double)ft[t][3]};
                    tile[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ua[I], wb[J], a4, 0, 0, 0);
                }
        }
        // ---- blocked LDL^T, panels of 4 columns ----
        double prod = det2;   // its sign is the determinant's (frexp keeps it)
        int e2 = 0;
        bool zero = det2 == 0.0;
        // one tile column at a time (compile-time tile indices), its 4 panels in
        // a loop (a full unroll let the compiler hoist across panels: 376 VGPRs)
        auto tile_column = [&](auto JPc) {
            constexpr int Jp = decltype(JPc)::value;
#pragma unroll 1
            for (int sub = 0; sub < 4; ++sub) {
                const int p = 4 * Jp + sub, cb = 4 * sub;
                // a) the panel's columns, rows >= 16 Jp, into LDS rows [r][k]
                asm volatile("" ::: "memory");
                if (c >= cb && c < cb + 4) {
#pragma unroll
                    for (int I = Jp; I < NT; ++I)
#pragma unroll
                        for (int v = 0; v < 4; ++v)
                            pb[(16 * I + g + 4 * v) * 4 + (c - cb)] = tile[cov_ti(I, Jp)][v];
                }
                asm volatile("" ::: "memory");
                const double2 x01 = *(const double2*)(pb + lane * 4);
                const double2 x23 = *(const double2*)(pb + lane * 4 + 2);
                const bool live = lane >= 4 * p && lane < BP;   // rows above the panel: zero
                double x[4] = {live ? x01.x : 0.0, live ? x01.y : 0.0, live ? x23.x : 0.0, live ? x23.y : 0.0};
                // b) the 4 pivots inside the panel
                double rp[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) {
                    const int P = 4 * p + kk;
                    const double piv = ame::lane_bcast(x[kk], P);
                    zero |= piv == 0.0;
                    prod *= piv;
                    if (kk == 3 && (sub & 1)) {   // every 8 pivots
                        int ex;
                        prod = frexp(prod, &ex);
                        e2 += ex;
                    }
                    double ri = __builtin_amdgcn_rcp(piv);
                    ri = fma(fma(-piv, ri, 1.0), ri, ri);
                    ri = fma(fma(-piv, ri, 1.0), ri, ri);
                    rp[kk] = ri;
                    const double f = x[kk] * ri;
#pragma unroll
                    for (int kq = kk + 1; kq < 4; ++kq) x[kq] = fma(-ame::lane_bcast(x[kq], P), f, x[kq]);
                }
                // c) rank-4 update of the trailing tiles (J >= Jp, and J > Jp after
                // the column's last panel), one MFMA each
                if (Jp + 1 < NT || sub < 3) {
                    asm volatile("" ::: "memory");
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) pb[kk * 64 + lane] = x[kk];   // column-major [k][r]
                    asm volatile("" ::: "memory");
                    const double rk = g == 0 ? rp[0] : (g == 1 ? rp[1] : (g == 2 ? rp[2] : rp[3]));
                    double xa[NT], xb[NT];
#pragma unroll
                    for (int I = Jp; I < NT; ++I) {
                        xb[I] = pb[g * 64 + 16 * I + c];
                        xa[I] = -xb[I] * rk;
                    }
                    // the next panel's tile column first: its extraction waits
                    // only for those MFMAs
                    if (sub < 3) {
#pragma unroll
                        for (int I = Jp; I < NT; ++I)
                            tile[cov_ti(I, Jp)] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[I], xb[Jp], tile[cov_ti(I, Jp)], 0, 0, 0);
                    }
#pragma unroll
                    for (int J = Jp + 1; J < NT; ++J)
#pragma unroll
                        for (int I = J; I < NT; ++I)
                            tile[cov_ti(I, J)] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[I], xb[J], tile[cov_ti(I, J)], 0, 0, 0);
                }
            }
        };
        static_assert(NT >= 1 && NT <= 4, "r <= 32");
        CST(2);
        tile_column(std::integral_constant<int, 0>{});
        CST(3);
        if constexpr (NT > 1) tile_column(std::integral_constant<int, 1>{});
        CST(4);
        if constexpr (NT > 2) tile_column(std::integral_constant<int, 2>{});
        CST(5);
        if constexpr (NT > 3) tile_column(std::integral_constant<int, 3>{});
        CST(6);
        double ld = log(fabs(prod)) + (double)e2 * 0.69314718055994530942;
        if (zero) ld = -INFINITY;
        else if (prod < 0.0) ld = NAN;
        tr = wave_sum(tr);
        tm = wave_sum(tm);
        if (lane == 0) {
            double* o = a.cov_terms + mc * 4;
            o[0] = ld;
            o[1] = tr;
            o[2] = msel ? tm : 0.0;
            o[3] = msel ? 0.0 : tm;
        }
        CST(7);
    }
}

template <int R>
static int launch_cov_mfma(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    using C = CovM<R>;
    const long long total = (long long)dm->T_local * dm->n;
    int dev = 0, cus = 0, per_cu = 0;
    long long cap = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ame_cov_mfma_kernel<R>, 256, 0) == hipSuccess &&
        cus > 0 && per_cu > 0)
        cap = (long long)cus * per_cu;
    // slice 0 (S0^-1) and the rest (Q^-1) as two launches
    const long long split = (dm->t_begin == 0) ? (total < dm->n ? total : (long long)dm->n) : 0;
    const long long lo[2] = {0, split}, hi[2] = {split, total};
    for (int q = 0; q < 2; ++q) {
        if (hi[q] <= lo[q]) continue;
        long long blocks = (hi[q] - lo[q] + C::WPB - 1) / C::WPB;   // persistent grid
        if (cap > 0 && blocks > cap) blocks = cap;
        hipLaunchKernelGGL(ame_cov_mfma_kernel<R>, dim3((unsigned)blocks), dim3(256), 0, st, *dm, *a, lo[q],
                           hi[q], q);
        if (hipGetLastError() != hipSuccess) return -3;
    }
    return 0;
}

template <int R>
static int launch_cov(const ame_dims* dm, const ame_cov_args* a, hipStream_t st) {
    if constexpr (R >= AME_COV_MFMA_MIN_R) return launch_cov_mfma<R>(dm, a, st);
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
