// K1 (v3): latency-optimised Gauss-Seidel sweep of TemporalAMEStructuredMFVI /
// TemporalAMENaiveMFVI on gfx950 -- new means AND new covariances of every
// (node, time) step.
//
// Reference semantics (Alfieriek/Python-Temporal-AME-SVI):
//   _update_step                structured_mf.py:211-218  (for i in range(n))
//   _update_node_i              structured_mf.py:220-287  (for t in range(T))
//   _compute_observation_terms  structured_mf.py:289-326
//   naive variant               naive_mf.py:207-282
// Step (i,t) reads the NEW means of nodes j<i at t and of node i at t-1 and the
// OLD means of nodes j>i at t and of node i at t+1 (2-D wavefront).
//
// Design (the algebra is restated and checked on CPU in
// tests/test_sweep_algebra.py):
//  * one 512-thread workgroup per time slice ("lane" t), all co-resident;
//    lane t-1 hands mu_{i,t-1}^new to lane t through {epoch,value} granules;
//  * wave 0 = SOLVER.  The only work between node i-1's new mean and node i's
//    is one d x 2r matvec with the fp64 base inverse B_i (rows in registers),
//    one 40-value cross-lane reduction (24 sums that involve mu_{i-1} and the 16
//    that do not, formed from the lane's own registers) and 2x2 algebra:
//       K_i  = B_i - L_{i-1} W_{i-1}^T + G_{i-1} X_{i-1}^T   (applied lazily)
//       W_i  = K_i J_{i-1}^T ,  M_i = R + J_{i-1} W_i ,  L_i = W_i M_i^-1
//       mu_i = u_i + W_i M_i^-1 (y_{i,i-1} - J_{i-1} u_i) ,  u_i = K_i g_i
//       X_i  = P_i^-1 J_{i+1}^T , S_i = R - J_{i+1} X_i , G_i = X_i S_i^-1
//  * waves 1-7 = HELPERS (448 lanes), one step behind / ahead of the solver:
//       HB  next base K_i = B_i + rank-4, fused with node i-1's covariance
//           P_{i-1}^-1 = B_i - L_{i-1} W_{i-1}^T, damped and stored (hw 0-5);
//       HE  h_obs GEMV of node i+2 over the slice's (U,V): register-resident
//           (node j -> helper lane j % 448, slot j / 448), overflow in LDS;
//       HF1 AR(1) terms + natural parameter g_{i+1} and node i+2's (U, V) for
//           the solver's v = K_i g_{i+1}, yv = K_i J_{i+2}^T (hw 0-2);
//       LOADER (hw 6): LDS-DMA (global_load_lds) rings, 3 steps ahead, for Y
//           rows, old covariances and old means, so no wave holds prefetch
//           registers; hw 5 reads the hand-off granules one step ahead.
//  * one workgroup barrier per step; intra-step hand-offs through LDS
//    counters;
//  * the slice's base inverse P_0^-1 is formed in the prologue (fp64 sums over
//    the slice's old means + symmetric sweep operator), so a slice can start
//    as soon as its own inputs exist: with wait_epoch set, the workgroup of
//    slice t first waits until the previous sweep has finished slices t and
//    t+1 (per-slice done flags, agent-scope release / acquire).  The next sweep
//    is then queued while this one runs, and consecutive sweeps overlap instead
//    of each paying the wavefront fill.
#include "ame_common.h"
#include "ame_wave.h"
#include "ame_sweep_dev.h"

using namespace ame;

namespace {
// 2x2 inverse with the reciprocal of the determinant from v_rcp_f64 plus two
// Newton steps (instead of the IEEE division sequence): full fp64 accuracy for
// the well-scaled determinants here, a shorter dependent chain
__device__ __forceinline__ Mat2 inv2s_fast(Mat2 m) {
    const double det = m.a * m.d - m.b * m.c;
    double r = __builtin_amdgcn_rcp(det);
    r = fma(r, fma(-det, r, 1.0), r);
    r = fma(r, fma(-det, r, 1.0), r);
    const double o = 0.5 * (-m.b * r - m.c * r);
    return {m.d * r, o, o, m.a * r};
}
}  // namespace

#ifdef AME_STAMPS
// Diagnostic build only (cdna_hip_programming.md §7, in-kernel stamps): the
// middle lane records s_memtime at marked points of steps [S3_I0, S3_I0+16) for
// every wave (0 = solver, w = helper wave w-1); every lane records
// s_memrealtime when it reaches steps 0, n/4, n/2, 3n/4 and n.
#define S3_I0 256
__device__ unsigned long long g_s3_stamps[8 * 16 * 16];
__device__ unsigned long long g_s3_prog[256 * 5];
__device__ unsigned int g_s3_hwid[8];
#define S3W(w) (w)
#define STAMP3(slot)                                                                           \
    do {                                                                                       \
        if (tl == TL / 2 && lane == 0 && i >= S3_I0 && i < S3_I0 + 16 && S3W(wave) >= 0) {     \
            unsigned long long t_;                                                             \
            __builtin_amdgcn_sched_barrier(0);                                                 \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
            __builtin_amdgcn_sched_barrier(0);                                                 \
            g_s3_stamps[(S3W(wave) * 16 + (i - S3_I0)) * 16 + (slot)] = t_;                    \
        }                                                                                      \
    } while (0)
#define PROG3()                                                                                \
    do {                                                                                       \
        if (tid == 0 && (i == 0 || i == n / 4 || i == n / 2 || i == 3 * n / 4 || i == n)) {    \
            const int q_ = (i == 0) ? 0 : (i == n / 4) ? 1 : (i == n / 2) ? 2 : (i == 3 * n / 4) ? 3 : 4; \
            g_s3_prog[tl * 5 + q_] = __builtin_amdgcn_s_memrealtime();                         \
        }                                                                                      \
    } while (0)
extern "C" int ame_debug_read_hwid3(unsigned int* h) {
    return hipMemcpyFromSymbol(h, HIP_SYMBOL(g_s3_hwid), sizeof(g_s3_hwid), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int ame_debug_read_stamps3(unsigned long long* st, unsigned long long* prog) {
    if (hipMemcpyFromSymbol(st, HIP_SYMBOL(g_s3_stamps), sizeof(g_s3_stamps), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(prog, HIP_SYMBOL(g_s3_prog), sizeof(g_s3_prog), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define STAMP3(slot) do { } while (0)
#define PROG3() do { } while (0)
#endif

namespace {

#ifndef AME_S3_MOLD_EARLY
#define AME_S3_MOLD_EARLY 1
#endif
constexpr int kNT = 512;    // threads per workgroup
constexpr int kNH = 448;    // helper lanes
// Node j of the slice's GEMV belongs to helper lane (j + kGOFF) % 448, slot
// j / 448.  With n > 896 the third slot is partial and, at offset 0, falls on
// hw 0-1, whose HB + HF1 + GEMV chain is the longest of the step.  Measured at
// config 3 (profiles/r02_goff.txt): offset 192 (hw 3-4) and 320 (hw 5-6) are
// no faster (2.75 / 2.77 vs 2.74 ms per iteration), so 0 stays.
constexpr int kGOFF = 0;
constexpr int kMREG = 96;   // VGPR budget for the register-resident part of the node slice
constexpr int kLDSMAX = 160 * 1024;

template <int R>
struct Cfg {
    static constexpr int D = 2 + 2 * R, M2 = 2 * R, DD = D * D;
    // node j -> helper lane j % 448, slot j / 448; slots < NSREG in registers,
    // further slots in LDS ([slot][c/2][lane] float2: conflict-free reads)
    static constexpr int NSREG = (kMREG / M2) < 1 ? 1 : ((kMREG / M2) > 16 ? 16 : (kMREG / M2));
    static constexpr int MP = (M2 + 1) / 2;
    static constexpr int NLT = D * (D + 1) / 2;
    static constexpr int NHB = 384;                           // HB lanes (hw 0-5)
    static constexpr int LTQ = (NLT + NHB - 1) / NHB;
    static constexpr int NP = (4 * D <= 192) ? 4 : 2;       // AR row parts (HF1)
    static constexpr int MC = (D + NP - 1) / NP;
    static constexpr int NC = (DD * 4 + 1023) / 1024;       // DMA KiB per covariance
};

// LDS carve-up (bytes); host and device agree.  Everything but the Y ring and
// the overflow node slots has a compile-time offset (folds into ds_* immediate
// offsets instead of occupying SGPRs).  Ring slots are whole KiB multiples: one
// LDS-DMA instruction writes 64 lanes x 16 B = 1 KiB.
__host__ __device__ constexpr int al16(int x) { return (x + 15) & ~15; }
template <int R>
struct Lay {
    static constexpr int D = 2 + 2 * R, DD = D * D;
    static constexpr int cs = ((DD * 4 + 1023) / 1024) * 256;     // covariance ring slot (floats)
    static constexpr int oK = 0;                                   // base inverse, double buffer
    static constexpr int NPA = (4 * D <= 192) ? 4 : 2;
    static constexpr int MCP = ((D + NPA - 1) / NPA) * NPA;       // AR row stride (zero padded)
    static constexpr int KS = D + 1;                               // base inverse row stride (odd: no bank conflicts)
    static constexpr int KSZ = D * KS;
    static constexpr int oAR = al16(oK + 8 * 2 * KSZ);             // Qinv Phi, Phi^T Qinv (fp64) [D][MCP]
    static constexpr int RS = 10;                                  // rec row stride (doubles)
    static constexpr int oRec = al16(oAR + 8 * 2 * D * MCP);       // [par][k][RS]: L0 L1 W0 W1 G0 G1 X0 X1
    static constexpr int oMu64 = al16(oRec + 8 * 2 * D * RS);      // [par][k] new mean (fp64)
    static constexpr int oMu32 = al16(oMu64 + 8 * 2 * D);          // [par][k] new mean (fp32)
    static constexpr int oG = al16(oMu32 + 4 * 2 * D);             // [node&1][k] g of node
    static constexpr int oJn = al16(oG + 8 * 2 * D);               // [node&1][c] (U, V) of node i+2 (old, fp64)
    static constexpr int oV = al16(oJn + 8 * 4 * D);               // [node&1][k]{v, yv0, yv1, vA}
    static constexpr int oRed = al16(oV + 8 * 2 * D * 4);          // solver reduction gather (40 sums)
    static constexpr int oGP = al16(oRed + 8 * 64);                // [node&1][wave][k] GEMV partials
    static constexpr int oYst = al16(oGP + 4 * 2 * 7 * D);         // [node&3]{y(m,m-1), y(m,m-2)} raw
    static constexpr int oMuL = al16(oYst + 4 * 4 * 4);            // [wave][64] mu_{m,t-1}, zero padded
    static constexpr int oPd = al16(oMuL + 4 * 3 * 64);            // [par][k] naive diag(P)
    static constexpr int oPc = al16(oPd + 8 * 2 * D);              // [k] diag of Pconst(t) (naive)
    static constexpr int oSq = al16(oPc + 8 * D);                  // [k] naive running column sums of squares
    static constexpr int oFlag = al16(oSq + 8 * D);                // kcnt, (unused), gcnt, (unused)
    static constexpr int oCr = al16(oFlag + 16);                   // [node&3] old covariances, DMA
    static constexpr int oXr = al16(oCr + 4 * 4 * cs);             // [node&7] old means slice t, DMA
    static constexpr int oRr = al16(oXr + 8 * 256);                // [node&3] old means slice t+1, DMA
    static constexpr int oPr = al16(oRr + 4 * 256);                // [node&3] hand-off granules, DMA
    static constexpr int oCs = al16(oPr + 4 * 1024);               // [node&1] new covariance, staged
    static constexpr int oYr = al16(oCs + 4 * 2 * cs);             // [node&3] Y rows (raw), DMA
    __host__ __device__ static int ys(int n) { return ((n * 8 + 1023) / 1024) * 128; }   // float2
    __host__ __device__ static int oML(int n) { return al16(oYr + 4 * 8 * ys(n)); }
    __host__ __device__ static int total(int n, int nsreg) {
        const int nsl = (n + 447) / 448 - nsreg;
        return al16(oML(n) + 8 * (nsl > 0 ? nsl : 0) * ((2 * R + 1) / 2) * 448);
    }
};

}  // namespace

// VAR: the factorization (enum ame_variant) as a template parameter, so each
// variant's kernel carries only its own code (good: 238 instead of 252 VGPRs
// at r = 16, fewer SGPR spills); the launch picks it from dims.variant
template <int R, int VAR>
__global__ void __launch_bounds__(kNT)
ame_sweep3_kernel(ame_dims dm, ame_sweep_args a) {
    using C = Cfg<R>;
    constexpr int D = C::D, M2 = C::M2, DD = C::DD, NSREG = C::NSREG, MP = C::MP;
    constexpr int NLT = C::NLT, LTQ = C::LTQ, NP = C::NP, MC = C::MC;
    constexpr int NC = C::NC;
    const int n = dm.n, TL = dm.T_local, Tt = dm.T_total;
    const int b = blockIdx.x;
    // XCD-aware lane order: consecutive time slices share an XCD (speed only)
    const int tl = (TL % 8 == 0) ? ((b & 7) * (TL >> 3) + (b >> 3)) : b;
    const int tg = dm.t_begin + tl;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hl = tid - 64, hw = wave - 1;   // helper lane / helper wave (valid for wave >= 1)
    const int hj = (hl + kNH - kGOFF) % kNH;    // first node of helper lane hl (slot 0)
    constexpr bool is_naive = VAR == AME_NAIVE, is_bad = VAR == AME_BAD;
    const int ns = (n + kNH - 1) / kNH;
    const int NY = (n * 8 + 1023) / 1024;     // DMA KiB per Y row
    const int KDMA = NY + NC + 2;             // DMA instructions per step (loader wave)

    extern __shared__ __attribute__((aligned(16))) char smem[];
    using LY = Lay<R>;
    const int YS = LY::ys(n);
    double* Kbuf = (double*)(smem + LY::oK);          // [par][k][KS]
    constexpr int KS = LY::KS, KSZ = LY::KSZ;
    constexpr int MCP = LY::MCP;
    double* arQ = (double*)(smem + LY::oAR);          // Qinv Phi   [D][MCP]
    double* arP = arQ + D * MCP;                       // Phi^T Qinv [D][MCP]
    double* rec = (double*)(smem + LY::oRec);
    double* mu64 = (double*)(smem + LY::oMu64);
    float* mu32 = (float*)(smem + LY::oMu32);
    double* g64 = (double*)(smem + LY::oG);
    double* jn64 = (double*)(smem + LY::oJn);
    double* vbuf = (double*)(smem + LY::oV);          // prologue pivot scratch
    double* red = (double*)(smem + LY::oRed);
    float* gp = (float*)(smem + LY::oGP);
    float* yst = (float*)(smem + LY::oYst);
    float* muL = (float*)(smem + LY::oMuL);
    double* pdl = (double*)(smem + LY::oPd);
    double* pcdl = (double*)(smem + LY::oPc);
    double* ssq = (double*)(smem + LY::oSq);
    uint32_t* flags = (uint32_t*)(smem + LY::oFlag);
    uint32_t* kcnt = flags;
    uint32_t* gcnt = flags + 2;
    float2* yring = (float2*)(smem + LY::oYr);
    float* cring = (float*)(smem + LY::oCr);
    float* xring = (float*)(smem + LY::oXr);
    float* rring = (float*)(smem + LY::oRr);
    uint64_t* pring = (uint64_t*)(smem + LY::oPr);
    float* cst = (float*)(smem + LY::oCs);
    float2* mlds = (float2*)(smem + LY::oML(n));

    const double r00 = a.rinv[0], r01 = a.rinv[1], r10 = a.rinv[2], r11 = a.rinv[3];
    const float r00f = (float)r00, r01f = (float)r01, r10f = (float)r10, r11f = (float)r11;
    const Mat2 Rm = inv2s(m2(r00, r01, r10, r11));   // R = R_inv^-1, symmetrised
    const float lr = a.lr, om = a.one_minus_lr;
    const float* xo = a.x_old + (size_t)tl * n * D;
    float* xn = a.x_new + (size_t)tl * n * D;
    float* cvs = a.cov + (size_t)tl * n * DD;
    float* cvw = (a.cov_new != nullptr ? a.cov_new : a.cov) + (size_t)tl * n * DD;   // damped output
    const int nys = ame_ystride(n);
    const float* ysl = a.Yt + (size_t)tl * n * nys * 2;
    // old means of slice t+1: the next local slice, or for the last local slice the
    // right rank's first slice -- next_old (gathered before the sweep), or in a
    // pipelined launch the back channel that rank fills when its slice finishes
    const bool back_rd = (a.wait_epoch != 0u) && (tl == TL - 1) && (a.back_in != nullptr);
    const float* xr = (tg < Tt - 1) ? ((tl < TL - 1) ? a.x_old + (size_t)(tl + 1) * n * D
                                                     : (back_rd ? a.back_in : a.next_old))
                                    : nullptr;
    const double* QiPhi = a.consts + 3 * (size_t)DD;
    bool dead = false;

    // ---- hand-off of mu_{node, t-1} ----
    auto gran_src = [&](int node) -> const uint64_t* {
        return (tl == 0) ? a.halo_in + (size_t)node * D : a.hand + ((size_t)(tl - 1) * n + node) * D;
    };
    // v = granule of this lane (k = lane < D) as read earlier; spin until its tag
    // is current.  A failed wait (AmeSpin rules, include/ame_amd.h) marks this
    // wave dead and passes AME_LDS_DEAD to the solver through gcnt, so the slice
    // stops publishing current-epoch granules and its done flag.
    auto gran_finish = [&](int node, uint64_t v, float* dst) {
        if (tg == 0) {
            if (lane < D) dst[lane] = 0.f;
            return;
        }
        bool ok = (lane >= D) || (uint32_t)(v >> 32) == a.epoch;
        if (!__all(ok) && !dead) {
            // the left rank, or (AME_SWEEP_FLAG_PREV_GROUP) the previous slice group
            // on this GPU: a local wait then
            const bool cross = tl == 0 && !(a.flags & AME_SWEEP_FLAG_PREV_GROUP);
            AmeSpin w(a.status, cross, lane == 0, hw == 0 ? AME_ST_HALO_US : 0);   // hw 0-2 wait alike
            const uint64_t* src = gran_src(node);
            while (true) {
                // a tag above this sweep's epoch cannot come from slice t-1 of
                // this sweep or an earlier one (the next sweep's slice t-1 waits
                // for this slice's done flag): stale memory, reported, not consumed
                bool stale = false;
                if (lane < D) {
                    v = cross ? gran_load_system(src + lane) : gran_load_agent(src + lane);
                    ok = (uint32_t)(v >> 32) == a.epoch;
                    stale = (uint32_t)(v >> 32) > a.epoch;
                }
                const bool st_hit = __any(stale);
                if (__all(ok) && !st_hit) break;
                const int r = st_hit ? 3 : w.poll();
                if (r != 0) {
                    // the record names the first lane whose tag is not current
                    const uint64_t bad = __ballot(!ok);
                    const int fl = bad ? (int)__builtin_ctzll(bad) : 0;
                    const uint32_t obs = (uint32_t)(__shfl(v, fl) >> 32);
                    if (lane == 0 && r >= 2)
                        ame_fail(a.status, (r == 3) ? AME_STATUS_STALE_EPOCH
                                                    : (cross ? AME_STATUS_HALO_TIMEOUT : AME_STATUS_SPIN_TIMEOUT),
                                 cross ? AME_WAIT_GRAN_HALO : AME_WAIT_GRAN_LOCAL, tg, (uint32_t)node, obs,
                                 a.epoch, w.waited(), a.epoch);
                    if (lane == 0)
                        __hip_atomic_fetch_or(gcnt, AME_LDS_DEAD, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    dead = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
            w.end();
        }
        if (lane < D) dst[lane] = __uint_as_float((uint32_t)v);
    };

    // ---- loader DMA pieces (whole-wave; every call issues a fixed instruction count) ----
    auto dma_y = [&](int row) {   // Y row (raw float2) -> slot row & 3 : NY instructions
        const int rw = (row < n) ? row : 0;
        const char* base = (const char*)(ysl + (size_t)rw * nys * 2);
        const uint32_t dst = lds_off(yring + (size_t)(row & 3) * YS);
        for (int q = 0; q < NY; ++q) {
            int off = (q * 64 + lane) * 16;
            if (off >= n * 8) off = 0;
            dma16(base + off, dst + q * 1024);
        }
    };
    auto dma_cov = [&](int node) {   // old covariance -> slot node & 3 : NC instructions
        const int cn = (node >= 0 && node < n) ? node : 0;
        const char* base = (const char*)(cvs + (size_t)cn * DD);
        const uint32_t dst = lds_off(cring + (size_t)(node & 3) * LY::cs);
#pragma unroll
        for (int q = 0; q < NC; ++q) {
            int off = (q * 64 + lane) * 16;
            if (off >= DD * 4) off = 0;
            dma16(base + off, dst + q * 1024);
        }
    };
    auto dma_x = [&](int node) {   // old mean, slice t -> slot node & 7 : 1 instruction
        const int xnn = (node < n) ? node : 0;
        dma4(xo + (size_t)xnn * D + (lane < D ? lane : 0), lds_off(xring + (node & 7) * 64));
    };
    auto dma_r = [&](int node) {   // old mean, slice t+1 -> slot node & 3 : 1 instruction
        const float* src = (xr != nullptr && node < n) ? xr + (size_t)node * D : xo;
        if (back_rd) dma4_sys(src + (lane < D ? lane : 0), lds_off(rring + (node & 3) * 64));
        else dma4(src + (lane < D ? lane : 0), lds_off(rring + (node & 3) * 64));
    };

    // staged new covariance of `node` -> cvw, 16 B per lane, whole rows (DD % 4 == 0)
    auto flush_cov = [&](int node) {
        const float4* src = (const float4*)(cst + (size_t)((node + 1) & 1) * LY::cs);
        float4* dst = (float4*)(cvw + (size_t)node * DD);
#pragma unroll
        for (int q = 0; q < NC; ++q) {
            const int e = q * 64 + lane;
            if (e * 4 < DD) dst[e] = src[e];
        }
    };

#ifdef AME_STAMPS
    if (tl == TL / 2 && lane == 0) {
        unsigned int hwid;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
        g_s3_hwid[wave] = hwid;
    }
#endif
    // ============================ prologue ============================
    // pipelined launch: the previous sweep must have finished slices t and t+1
    // (their means and covariances are this sweep's inputs; slice t+1 also reads
    // this slice's hand-off granules, which this sweep overwrites)
    if (a.wait_epoch != 0u) {
        // Epoch window: while this sweep (wait_epoch + 1) waits, neither flag can
        // exceed wait_epoch -- sweep wait_epoch + 1 writes done[t] only when it
        // finishes slice t, the sweeps queued behind it wait for that, and slice
        // t+1 cannot finish before slice t.  A larger value is stale memory (a
        // recycled buffer, a host write not yet ordered before this launch): it
        // sets AME_STATUS_STALE_EPOCH instead of being taken as done.  (done[TL]:
        // the next slice group's first slice, when one follows.)  The back
        // channel (the right rank's first slice of the previous sweep) has the
        // same window: that slice of THIS sweep needs this slice's granules.
        // tid 0 waits; a failure marks it dead, which the solver wave (tid 0 is
        // its lane 0) takes over, so the slice publishes nothing current.
        if (tid == 0) ame_wait_prev_done(a, tl, TL, tg, back_rd, n * D, dead);
        __syncthreads();
    }
    // P_0 = Pconst + sum_{j>=1} F_j(old), F_j = J_j^T R^-1 J_j (fp64), and its
    // inverse -> Kbuf[0] by the in-place symmetric sweep operator; naive variant:
    // column sums of squares of (U, V) over all nodes -> ssq[2 + c]
    {
        double* piv = vbuf;
        double* K = Kbuf;
        const double pp = r00, ss = r11, qq = 0.5 * (r01 + r10);
        // G = sum_{j>=1} x_j x_j^T (fp64 MFMA, ame_sweep_dev.h) straight into K's
        // (U, V) block, column sums into vbuf (free until the pivot loop)
        double* colsum = vbuf;
        float* x0 = (float*)(vbuf + M2);
        p0_gram_mfma<R, kNT / 64>(xo, n, D, K, KS, colsum, x0);
        if (tid < M2) {   // node 0 joins the sums of squares
            const int kq = 2 + (tid >= R ? tid - R : tid + R);   // the row that holds column tid
            const double v = (double)x0[tid];
            ssq[2 + tid] = fma(v, v, K[kq * KS + kq]);
        }
        __syncthreads();
        for (int e = tid; e < NLT; e += kNT) {
            int k, m;
            tri_decode3(e, k, m);
            double v;
            if (k < 2) {
                v = ((k == 0 && m == 0) ? pp : (k == 1 && m == 1) ? ss : qq) * (double)(n - 1);
            } else {
                const bool ku = (k - 2) < R;
                if (m < 2) {
                    const int ck = k - 2, kc = (ck < R) ? R + ck : ck - R;
                    v = (ku ? (m == 0 ? pp : qq) : (m == 0 ? qq : ss)) * colsum[kc];
                } else {
                    const bool mu_ = (m - 2) < R;
                    v = ((ku && mu_) ? pp : ((!ku && !mu_) ? ss : qq)) * K[k * KS + m];
                }
            }
            v += pconst_entry(a.consts, D, k, m, tg, Tt);
            K[k * KS + m] = v;
            K[m * KS + k] = v;
        }
        __syncthreads();
        for (int pv = 0; pv < D; ++pv) {   // K -> -P_0^-1
            if (tid < D) piv[tid] = K[pv * KS + tid];
            __syncthreads();
            const double rinv = 1.0 / piv[pv];
            for (int e = tid; e < NLT; e += kNT) {
                int k, m;
                tri_decode3(e, k, m);
                double v;
                if (k == pv && m == pv) v = -rinv;
                else if (k == pv) v = piv[m] * rinv;
                else if (m == pv) v = piv[k] * rinv;
                else v = K[k * KS + m] - (piv[k] * piv[m]) * rinv;
                K[k * KS + m] = v;
                K[m * KS + k] = v;
            }
            __syncthreads();
        }
        for (int e = tid; e < KSZ; e += kNT) K[e] = -K[e];
        __syncthreads();
    }
    for (int e = tid; e < 2 * D * MCP; e += kNT) {   // QiPhi, PhiTQi (adjacent in consts), padded
        const int mat = e / (D * MCP), rc = e - mat * D * MCP, rr = rc / MCP, cc = rc - rr * MCP;
        arQ[e] = (cc < D) ? QiPhi[(size_t)mat * DD + rr * D + cc] : 0.0;
    }
    for (int e = tid; e < 3 * 64; e += kNT) muL[e] = 0.f;
    if (tid < D) pcdl[tid] = pconst_entry(a.consts, D, tid, tid, tg, Tt);
    constexpr int RS = LY::RS;
    for (int e = tid; e < 2 * D * RS; e += kNT) rec[e] = 0.0;
    for (int e = tid; e < 2 * D; e += kNT) {
        mu64[e] = 0.0;
        mu32[e] = 0.f;
    }
    if (tid < 16) yst[tid] = 0.f;
    if (tid < 4) flags[tid] = 0u;
    float mreg[NSREG][M2];      // (U, V) of nodes hl + 448 s, s < NSREG
    if (wave >= 1) {
#pragma unroll
        for (int s = 0; s < NSREG; ++s) {
            const int j = hj + kNH * s;
            const bool ok = s < ns && j < n;
#pragma unroll
            for (int c = 0; c < M2; ++c) mreg[s][c] = ok ? xo[(size_t)j * D + 2 + c] : 0.f;
        }
        for (int s = NSREG; s < ns; ++s) {
            const int j = hj + kNH * s;
            const bool ok = j < n;
            for (int c2 = 0; c2 < MP; ++c2) {
                float2 v = make_float2(0.f, 0.f);
                if (ok) {
                    v.x = xo[(size_t)j * D + 2 + 2 * c2];
                    if (2 * c2 + 1 < M2) v.y = xo[(size_t)j * D + 3 + 2 * c2];
                }
                mlds[((s - NSREG) * MP + c2) * kNH + hl] = v;
            }
        }
        // Y rows 0 and 1 into ring slots 0 and 1 (plain loads)
        for (int e = hl; e < 2 * n; e += kNH) {
            const int rw = e / n, j = e - rw * n;
            yring[(size_t)rw * YS + j] = (rw < n) ? *(const float2*)(ysl + ((size_t)rw * nys + j) * 2)
                                                    : make_float2(0.f, 0.f);
        }
    }
    if (wave == 7) {   // rings read by steps 0..2 and the prologue
        for (int q = 0; q < 5; ++q) dma_x(q);
        for (int q = 0; q < 4; ++q) dma_r(q);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();

    // GEMV of node m over nodes j (excluding j in {m-2, m-1, m}) from raw Y values
    // ysrc[j]; stashes y_{m,m-1}, y_{m,m-2}; partials -> gp[m&1][hw][.]
    auto gemv = [&](int m, const float2* ysrc, int i) {   // i: the step (stamps only)
        float acc[D];
#pragma unroll
        for (int c = 0; c < D; ++c) acc[c] = 0.f;
        float2 yv[NSREG];
#pragma unroll
        for (int s = 0; s < NSREG; ++s) {   // ring slots are >= n long: loads need no guard
            const int j = hj + kNH * s;
            const float2 y = ysrc[j];
            yv[s] = (j < n) ? y : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int s = 0; s < NSREG; ++s) {
            if (s < ns) {
                const int j = hj + kNH * s;
                const bool ex = (j >= m - 2) && (j <= m);
                const float z0 = ex ? 0.f : r00f * yv[s].x + r01f * yv[s].y;
                const float z1 = ex ? 0.f : r10f * yv[s].x + r11f * yv[s].y;
                acc[0] += z0;
                acc[1] += z1;
#pragma unroll
                for (int c = 0; c < R; ++c) {
                    acc[2 + c] = fmaf(z0, mreg[s][R + c], acc[2 + c]);       // h_U += z0 V
                    acc[2 + R + c] = fmaf(z1, mreg[s][c], acc[2 + R + c]);   // h_V += z1 U
                }
            }
        }
        for (int s = NSREG; s < ns; ++s) {
            const int j = hj + kNH * s;
            float2 y = ysrc[j];
            if (j >= n) y = make_float2(0.f, 0.f);
            const bool ex = (j >= m - 2) && (j <= m);
            const float z0 = ex ? 0.f : r00f * y.x + r01f * y.y;
            const float z1 = ex ? 0.f : r10f * y.x + r11f * y.y;
            acc[0] += z0;
            acc[1] += z1;
            const float2* ml = mlds + (size_t)(s - NSREG) * MP * kNH + hl;
#pragma unroll
            for (int c2 = 0; c2 < MP; ++c2) {   // column c: U_c -> h_V (z1), V_c -> h_U (z0)
                const float2 t = ml[c2 * kNH];
                const int c = 2 * c2;
                if (c < R) acc[2 + R + c] = fmaf(z1, t.x, acc[2 + R + c]);
                else acc[2 + (c - R)] = fmaf(z0, t.x, acc[2 + (c - R)]);
                if (c + 1 < M2) {
                    if (c + 1 < R) acc[2 + R + c + 1] = fmaf(z1, t.y, acc[2 + R + c + 1]);
                    else acc[2 + (c + 1 - R)] = fmaf(z0, t.y, acc[2 + (c + 1 - R)]);
                }
            }
        }
        STAMP3(7);
        int idx;
        const float v = wave_reduce_scatter<D>(acc, lane, idx);
        STAMP3(8);
        if (idx < D) gp[((m & 1) * 7 + hw) * D + idx] = v;
        // raw y_{m,m-1}, y_{m,m-2} for the solver / HF1 (owner lanes only)
        const int jm1 = m - 1, jm2 = m - 2;
        if (jm1 >= 0 && ((jm1 + kGOFF) % kNH) == hl) {
            const float2 y = ysrc[jm1];
            yst[(m & 3) * 4 + 0] = y.x;
            yst[(m & 3) * 4 + 1] = y.y;
        }
        if (jm2 >= 0 && ((jm2 + kGOFF) % kNH) == hl) {
            const float2 y = ysrc[jm2];
            yst[(m & 3) * 4 + 2] = y.x;
            yst[(m & 3) * 4 + 3] = y.y;
        }
    };
    // HF1 (hw 0..2): AR terms + natural parameter g of node m.
    // mu_{m,t-1} in muL[hw], mu_{m,t+1}^old in rring[m&3].
    auto hf1 = [&](int m) {
        const int q = hl;   // 0..191
        const int k = q / NP, p = q - k * NP;
        const int kc = (k < D) ? k : 0;
        const float* ml = muL + hw * 64;          // zero beyond D; zero when tg == 0
        const float* mr = rring + (m & 3) * 64;   // finite beyond D (padded coefficients are 0)
        const double* aq = arQ + kc * MCP + p * MC;
        const double* ap = arP + kc * MCP + p * MC;
        // every LDS read first (one round trip), then the arithmetic
        double av[MC], bv[MC];
        float lv[MC], rv[MC], gv[7];
#pragma unroll
        for (int mm = 0; mm < MC; ++mm) {
            av[mm] = aq[mm];
            bv[mm] = ap[mm];
            lv[mm] = ml[p * MC + mm];
            rv[mm] = mr[p * MC + mm];
        }
#pragma unroll
        for (int w = 0; w < 7; ++w) gv[w] = gp[((m & 1) * 7 + w) * D + kc];
        const float mv2 = jcol_load<R>(mu32 + ((m - 2) & 1) * D, kc);
        const float ys0 = yst[(m & 3) * 4 + 2], ys1 = yst[(m & 3) * 4 + 3];
        __builtin_amdgcn_sched_barrier(0);
        double accL = 0.0, accR = 0.0;
#pragma unroll
        for (int mm = 0; mm < MC; ++mm) {
            accL = fma(av[mm], (double)lv[mm], accL);
            accR = fma(bv[mm], (double)rv[mm], accR);
        }
        double acc = accL + ((tg < Tt - 1) ? accR : 0.0);
        acc = dpp_add_xor1(acc);
        if constexpr (NP == 4) acc = dpp_add_mirror4(acc);
        // lane (k, 0) assembles g_k = GEMV partials + AR + node m-2's term
        double g = 0.0;
#pragma unroll
        for (int w = 0; w < 7; ++w) g += (double)gv[w];
        g += acc;
        if (m >= 2) {   // node m-2 was excluded from the GEMV; its new mean is known now
            double j0, j1;
            jcol_sel<R>(mv2, true, kc, j0, j1);
            const double y0 = (double)ys0, y1 = (double)ys1;
            const double z0 = r00 * y0 + r01 * y1, z1 = r10 * y0 + r11 * y1;
            g = fma(j0, z0, fma(j1, z1, g));
        }
        if (k < D && p == 0) g64[(m & 1) * D + k] = g;
    };
    // (U, V) of `node` (old, fp64) -> jn64 slot node & 1 (lanes < 2r of the calling
    // wave): the only non-constant entries of its J rows J0 = [1, 0, V, 0],
    // J1 = [0, 1, 0, U].  Double-buffered: hw 0 fills node i+2 during step i while
    // the solver may still be reading node i+1's (its prologue prep of step 0
    // overlaps step 0)
    auto jn_fill = [&](int node) {
        if (lane < M2) {
            const float* xm = xring + (node & 7) * 64;
            jn64[(node & 1) * 2 * D + lane] = (node < n) ? (double)xm[2 + lane] : 0.0;
        }
    };

    // ---- prologue work: g_0, GEMV partials of node 1, v_0 / yv_0; rings for steps 0..2 ----
    if (wave >= 1) {
        gemv(0, yring, -1);
        gemv(1, yring + YS, -1);
        if (hw <= 2) {
            uint64_t g0 = 0;
            if (tg > 0 && lane < D)
                g0 = (tl == 0) ? gran_load_system(gran_src(0) + lane) : gran_load_agent(gran_src(0) + lane);
            gran_finish(0, g0, muL + hw * 64);
        }
        if (hw == 3) jn_fill(1);
    }
    __syncthreads();
    if (wave >= 1 && hw <= 2) hf1(0);
    __syncthreads();
    if (wave == 7) {   // Y rows 2..4 (slots 2,3,0), covariances of nodes 0,1
        for (int q = 2; q <= 4; ++q) dma_y(q);
        for (int q = 0; q <= 1; ++q) dma_cov(q);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (wave == 6 && lane < D) {   // granules of node 1 (8-byte atomic loads, see below)
        uint64_t g1 = 0;
        if (tg > 0 && n > 1)
            g1 = (tl == 0) ? gran_load_system(gran_src(1) + lane) : gran_load_agent(gran_src(1) + lane);
        pring[(size_t)1 * 128 + lane] = g1;
    }
    __syncthreads();

    if (wave == 0) {
        // ============================ SOLVER ============================
        __builtin_amdgcn_s_setprio(3);
        // the prologue's wait ran on lane 0; node 0's hand-off wait (hw 0-2) leaves
        // AME_LDS_DEAD in gcnt
        dead = __any(dead) || (*(volatile uint32_t*)gcnt & AME_LDS_DEAD) != 0u;
        const int k = lane;
        const bool kl = k < D;
        const int kc = kl ? k : 0;
        double brow[D];   // row k of the base inverse B_i
#pragma unroll
        for (int c = 0; c < D; ++c) brow[c] = kl ? Kbuf[(size_t)k * KS + c] : 0.0;
        // v = B g, yv = B Jn^T (Jn: J rows of node i+1, old) and this lane's Jn
        // entries, for the coming step; B = brow, g and node i+1's (U, V) from
        // HF1 / jn_fill.  J0 = [1, 0, V, 0], J1 = [0, 1, 0, U]: yv needs 2r
        // products, not 2d.  Runs at the end of the previous step, after the
        // solver's own work.
        double v = 0, yv0 = 0, yv1 = 0, vA = 0, nq0 = 0, nq1 = 0;
        auto prep = [&](int node) {
            const double* jx = jn64 + ((node + 1) & 1) * 2 * D;   // (U, V) of node + 1
            if (!kl) return;
            const double* gg = g64 + (node & 1) * D;
            const bool ex1 = node + 1 < n;                          // J of a missing node is 0
            double s0 = 0, t0 = 0, s1 = ex1 ? brow[0] : 0.0, t1 = 0, s2 = ex1 ? brow[1] : 0.0, t2 = 0;
#pragma unroll
            for (int c = 0; c < D; c += 2) {
                s0 = fma(brow[c], gg[c], s0);
                t0 = fma(brow[c + 1], gg[c + 1], t0);
            }
#pragma unroll
            for (int c = 0; c < R; c += 2) {
                s1 = fma(brow[2 + c], jx[R + c], s1);       // J0: V at columns 2 .. 2+R
                s2 = fma(brow[2 + R + c], jx[c], s2);       // J1: U at columns 2+R .. D
                if (c + 1 < R) {
                    t1 = fma(brow[3 + c], jx[R + c + 1], t1);
                    t2 = fma(brow[3 + R + c], jx[c + 1], t2);
                }
            }
            v = s0 + t0;
            yv0 = s1 + t1;
            yv1 = s2 + t2;
            vA = brow[0] * gg[0] + brow[1] * gg[1];
            const double xj = jx[(k >= 2 && k < 2 + R) ? k - 2 + R : ((k >= 2 + R && k < D) ? k - 2 - R : 0)];
            nq0 = (k == 0) ? (ex1 ? 1.0 : 0.0) : ((k >= 2 && k < 2 + R) ? xj : 0.0);
            nq1 = (k == 1) ? (ex1 ? 1.0 : 0.0) : ((k >= 2 + R && k < D) ? xj : 0.0);
        };
        prep(0);
        double Wp0 = 0, Wp1 = 0, Xp0 = 0, Xp1 = 0, Lp0 = 0, Lp1 = 0, Gp0 = 0, Gp1 = 0;
        Mat2 Mip = m2(0, 0, 0, 0), Sip = m2(0, 0, 0, 0);
        for (int i = 0; i < n; ++i) {
            PROG3();
            STAMP3(0);
            const int par = i & 1, ppar = (i + 1) & 1;
            const bool has_prev = i > 0;
            const float* mup = mu32 + ppar * D;       // mu_{i-1} (fp32)
            const double* mupd = mu64 + ppar * D;     // mu_{i-1} (fp64)
            const double msk = kl ? 1.0 : 0.0;
            const double g = msk * g64[par * D + kc];
#if AME_S3_MOLD_EARLY
            // node i's old mean for the publish's damping, read with this step's
            // first LDS reads (its ring slot was loaded three steps ahead) instead
            // of a dependent LDS round trip in the publish
            const float mold_pf = xring[(i & 7) * 64 + kc];
#endif
            double J0, J1;
            jcol<R>(mup, has_prev && kl, kc, J0, J1);
            // kj = B J^T (the one critical matvec)
            double kj0 = 0, kj1 = 0;
            if (has_prev) {
                double s0a = brow[0], s0b = 0, s1a = brow[1], s1b = 0;
#pragma unroll
                for (int c = 0; c < R; c += 2) {
                    s0a = fma(brow[2 + c], mupd[2 + R + c], s0a);
                    s1a = fma(brow[2 + R + c], mupd[2 + c], s1a);
                    if (c + 1 < R) {
                        s0b = fma(brow[3 + c], mupd[3 + R + c], s0b);
                        s1b = fma(brow[3 + R + c], mupd[3 + c], s1b);
                    }
                }
                kj0 = s0a + s0b;
                kj1 = s1a + s1b;
            }
            STAMP3(1);
            // one reduction per step: a1(4) a2(4) c(4) e(2) jy(4) ny(4), and the
            // dots that do not involve mu_{i-1}: b1(2) b2(2) f1(4) f2(4); the bad
            // variant adds eA(2) b1A(2) b2A(2) at the end (40 values, 41 pair steps
            // of the tree; good 34, 37 pair steps).  c = J B J^T and ny = Jn B Jn^T
            // are symmetric and only bad reads them other than through sym(): the
            // naive instance reduces their upper triangles (the off-diagonal as the
            // lanes' mean of both products), 32 values, 32 pair steps.  The same
            // packing measured 0.8 % slower for good, 5.7 % faster for naive
            // (profiles/r06_ab_sym_pack.txt), so only naive packs
            // (W, X of the previous step, g_i and node i+1's J entries are this
            // lane's own registers; until round 3 a helper wave formed them, "HX",
            // and the solver waited for it: profiles/r03_v3_ab_hx_in_solver.txt)
            constexpr bool pack = is_naive;
            constexpr int NV = is_bad ? 40 : (pack ? 32 : 34);
            constexpr int IE = pack ? 11 : 12, IJY = IE + 2, INY = IJY + 4;
            constexpr int IB = INY + (pack ? 3 : 4), IF1 = IB + 4, IF2 = IF1 + 4;
            double pr[NV];
            pr[0] = Wp0 * J0; pr[1] = Wp0 * J1; pr[2] = Wp1 * J0; pr[3] = Wp1 * J1;       // a1[p][q]
            pr[4] = Xp0 * J0; pr[5] = Xp0 * J1; pr[6] = Xp1 * J0; pr[7] = Xp1 * J1;       // a2[p][q]
            if constexpr (!pack) {
                pr[8] = J0 * kj0; pr[9] = J0 * kj1; pr[10] = J1 * kj0; pr[11] = J1 * kj1;     // c[q][p]
            } else {
                pr[8] = J0 * kj0; pr[9] = 0.5 * (J0 * kj1 + J1 * kj0); pr[10] = J1 * kj1;     // c, sym
            }
            pr[IE] = J0 * v; pr[IE + 1] = J1 * v;                                                 // e[q]
            pr[IJY] = J0 * yv0; pr[IJY + 1] = J0 * yv1; pr[IJY + 2] = J1 * yv0; pr[IJY + 3] = J1 * yv1;   // jy[q][p]
            if constexpr (!pack) {
                pr[INY] = nq0 * yv0; pr[INY + 1] = nq0 * yv1; pr[INY + 2] = nq1 * yv0; pr[INY + 3] = nq1 * yv1;   // ny[q][p]
            } else {
                pr[INY] = nq0 * yv0; pr[INY + 1] = 0.5 * (nq0 * yv1 + nq1 * yv0); pr[INY + 2] = nq1 * yv1;   // ny, sym
            }
            pr[IB] = Wp0 * g; pr[IB + 1] = Wp1 * g; pr[IB + 2] = Xp0 * g; pr[IB + 3] = Xp1 * g;           // b1, b2
            pr[IF1] = Wp0 * nq0; pr[IF1 + 1] = Wp0 * nq1; pr[IF1 + 2] = Wp1 * nq0; pr[IF1 + 3] = Wp1 * nq1;   // f1[p][q]
            pr[IF2] = Xp0 * nq0; pr[IF2 + 1] = Xp0 * nq1; pr[IF2 + 2] = Xp1 * nq0; pr[IF2 + 3] = Xp1 * nq1;   // f2[p][q]
            if constexpr (is_bad) {
                const double gA = (k < 2) ? g : 0.0;
                pr[34] = J0 * vA; pr[35] = J1 * vA;                                           // eA[q]
                pr[36] = Wp0 * gA; pr[37] = Wp1 * gA; pr[38] = Xp0 * gA; pr[39] = Xp1 * gA;   // b1A, b2A
            }
            {
                int idx;
                const double sv = wave_reduce_scatter<NV>(pr, lane, idx);
                if (idx < NV) red[idx] = sv;
            }
            wave_lds_sync3();
            double o[NV];
#pragma unroll
            for (int q = 0; q < NV; ++q) o[q] = red[q];
            const Mat2 a1 = m2(o[0], o[1], o[2], o[3]);
            const Mat2 a2 = m2(o[4], o[5], o[6], o[7]);
            const Mat2 cc = !pack ? m2(o[8], o[9], o[10], o[11]) : m2(o[8], o[9], o[9], o[10]);
            const V2 e = {o[IE], o[IE + 1]};
            const Mat2 jy = m2(o[IJY], o[IJY + 1], o[IJY + 2], o[IJY + 3]);
            const Mat2 ny = !pack ? m2(o[INY], o[INY + 1], o[INY + 2], o[INY + 3])
                                   : m2(o[INY], o[INY + 1], o[INY + 1], o[INY + 2]);
            STAMP3(2);
            STAMP3(3);
            const V2 b1 = {o[IB], o[IB + 1]}, b2 = {o[IB + 2], o[IB + 3]};
            const Mat2 f1 = m2(o[IF1], o[IF1 + 1], o[IF1 + 2], o[IF1 + 3]);
            const Mat2 f2 = m2(o[IF2], o[IF2 + 1], o[IF2 + 2], o[IF2 + 3]);
            // raw y_{i,i-1}
            double y0 = 0, y1 = 0;
            if (has_prev) { y0 = (double)yst[(i & 3) * 4 + 0]; y1 = (double)yst[(i & 3) * 4 + 1]; }
            const double zp0 = r00 * y0 + r01 * y1, zp1 = r10 * y0 + r11 * y1;
            // ---- 2x2 algebra ----
            const Mat2 JW = add(sub(cc, quad(a1, Mip, a1)), quad(a2, Sip, a2));
            const Mat2 Mm = add(Rm, sym(JW));
            const Mat2 Mi = has_prev ? inv2s_fast(Mm) : m2(0, 0, 0, 0);
            const V2 t1 = mtv(a1, mv(Mip, b1)), t2 = mtv(a2, mv(Sip, b2));
            const V2 Ju = {e.x - t1.x + t2.x, e.y - t1.y + t2.y};
            const V2 cvec = mv(Mi, V2{y0 - Ju.x, y1 - Ju.y});
            const Mat2 wn = add(sub(jy, quad(a1, Mip, f1)), quad(a2, Sip, f2));
            const Mat2 JnK = add(sub(ny, quad(f1, Mip, f1)), quad(f2, Sip, f2));
            const Mat2 JnX = sub(JnK, quad(wn, Mi, wn));
            const Mat2 Si = inv2s_fast(sub(Rm, sym(JnX)));
            // ---- lane-local assembly ----
            const double W0 = kj0 - (Lp0 * a1.a + Lp1 * a1.c) + (Gp0 * a2.a + Gp1 * a2.c);
            const double W1 = kj1 - (Lp0 * a1.b + Lp1 * a1.d) + (Gp0 * a2.b + Gp1 * a2.d);
            const double u = v - (Lp0 * b1.x + Lp1 * b1.y) + (Gp0 * b2.x + Gp1 * b2.y);
            const double kn0 = yv0 - (Lp0 * f1.a + Lp1 * f1.c) + (Gp0 * f2.a + Gp1 * f2.c);
            const double kn1 = yv1 - (Lp0 * f1.b + Lp1 * f1.d) + (Gp0 * f2.b + Gp1 * f2.d);
            double mus;
            if constexpr (!is_bad) {
                mus = u + W0 * cvec.x + W1 * cvec.y;
            } else {
                const V2 eA = {o[34], o[35]};
                const V2 b1A = {o[36], o[37]}, b2A = {o[38], o[39]};
                const double uA = vA - (Lp0 * b1A.x + Lp1 * b1A.y) + (Gp0 * b2A.x + Gp1 * b2A.y);
                const V2 s1 = mtv(a1, mv(Mip, b1A)), s2 = mtv(a2, mv(Sip, b2A));
                const V2 JuA = {eA.x - s1.x + s2.x, eA.y - s1.y + s2.y};
                // K_i[:, 0:2] (row k) and W_i rows 0, 1 (uniform)
                const double* rq = rec + (size_t)ppar * D * RS;   // [k][field]
                const double KE0 = brow[0] - (Lp0 * rq[2] + Lp1 * rq[3]) + (Gp0 * rq[6] + Gp1 * rq[7]);
                const double KE1 = brow[1] - (Lp0 * rq[RS + 2] + Lp1 * rq[RS + 3]) +
                                   (Gp0 * rq[RS + 6] + Gp1 * rq[RS + 7]);
                const double WE00 = lane_bcast(W0, 0), WE01 = lane_bcast(W1, 0);   // W row 0
                const double WE10 = lane_bcast(W0, 1), WE11 = lane_bcast(W1, 1);   // W row 1
                const double wz0 = WE00 * zp0 + WE10 * zp1, wz1 = WE01 * zp0 + WE11 * zp1;
                const double tA = uA + KE0 * zp0 + KE1 * zp1;
                const V2 jA = {JuA.x + wz0, JuA.y + wz1};
                const double tX = (u - uA) + (W0 * zp0 + W1 * zp1) - (KE0 * zp0 + KE1 * zp1);
                const V2 jX = {(Ju.x - JuA.x) + (JW.a * zp0 + JW.b * zp1) - wz0,
                               (Ju.y - JuA.y) + (JW.c * zp0 + JW.d * zp1) - wz1};
                const V2 cA = mv(Mi, jA), cX = mv(Mi, jX);
                mus = (k < 2) ? (tA - (W0 * cA.x + W1 * cA.y)) : (tX - (W0 * cX.x + W1 * cX.y));
            }
            if (!is_naive) mus += 1e-6 * (g + J0 * zp0 + J1 * zp1);
            const double Ln0 = W0 * Mi.a + W1 * Mi.c, Ln1 = W0 * Mi.b + W1 * Mi.d;
            const double Xn0 = kn0 - (Ln0 * wn.a + Ln1 * wn.c);
            const double Xn1 = kn1 - (Ln0 * wn.b + Ln1 * wn.d);
            const double Gn0 = Xn0 * Si.a + Xn1 * Si.c, Gn1 = Xn0 * Si.b + Xn1 * Si.d;
            STAMP3(4);
            // ---- publish ----
            float mold = 0.f, nw = 0.f;
            if (kl) {
#if AME_S3_MOLD_EARLY
                mold = mold_pf;
#else
                const float* xold = xring + (i & 7) * 64;
                mold = xold[k];
#endif
                nw = mul_add_rn(lr, (float)mus, om, mold);
                xn[(size_t)i * D + k] = nw;
                // a dead slice tags its granules 0: no sweep waits for that epoch
                const uint64_t gr = ((uint64_t)(dead ? 0u : a.epoch) << 32) | (uint64_t)__float_as_uint(nw);
                gran_store_agent(a.hand + ((size_t)tl * n + i) * D + k, gr);
                if (tl == TL - 1 && a.halo_out != nullptr)
                    gran_store_system(a.halo_out + (size_t)i * D + k, gr);
                mu32[par * D + k] = nw;
                mu64[par * D + k] = (double)nw;
                double* rc = rec + ((size_t)par * D + k) * RS;   // [k][field]
                rc[0] = Ln0; rc[1] = Ln1; rc[2] = W0; rc[3] = W1;
                rc[4] = Gn0; rc[5] = Gn1; rc[6] = Xn0; rc[7] = Xn1;
            }
            // naive: diag(P_i) from running sums of squares (own old value removed),
            // for node i's covariance (HB, next step); after the mean is published,
            // so its cross-lane read is off the mean's path
            if (is_naive) {
                const int src = (k >= 2 && k < 2 + R) ? k + R : ((k >= 2 + R && k < D) ? k - R : k);
                if (kl) {
                    const float* xold = xring + (i & 7) * 64;
                    const double p = r00, s = r11;
                    // lane k reads its partner column's sum before any lane
                    // updates its own: the read is issued first and the compiler
                    // may not move it past the barrier below (the two addresses
                    // differ per lane, so without it the store could be hoisted
                    // above another lane's read of the same word)
                    const double sq_src = ssq[src];
                    asm volatile("" ::: "memory");
                    double pd;
                    if (k == 0) pd = p * (double)(n - 1);
                    else if (k == 1) pd = s * (double)(n - 1);
                    else {
                        const double oo = (k < 2 + R) ? (double)xold[k + R] : (double)xold[k - R];
                        pd = ((k < 2 + R) ? p : s) * (sq_src - oo * oo);
                    }
                    pdl[par * D + k] = pd + pcdl[k];
                    const double mo = (double)mold, mn = (double)nw;
                    // LDS, not a register: a loop-carried naive-only value spills
                    // (256-VGPR cap) and its reload waits on the publish stores
                    if (k >= 2) ssq[k] = ssq[k] - mo * mo + mn * mn;
                }
            }
            Wp0 = W0; Wp1 = W1; Xp0 = Xn0; Xp1 = Xn1; Lp0 = Ln0; Lp1 = Ln1; Gp0 = Gn0; Gp1 = Gn1;
            Mip = Mi;
            Sip = Si;
            STAMP3(5);
            // next base rows, once every helper wave has written K_i
            lds_wait_ge(kcnt, 7u * (uint32_t)(i + 1), a.status, dead, tg, (uint32_t)i, a.epoch);
            STAMP3(6);
            const double* Kn = Kbuf + (size_t)ppar * KSZ;
            if (kl) {
#pragma unroll
                for (int c = 0; c < D; ++c) brow[c] = Kn[(size_t)k * KS + c];
            }
            STAMP3(7);
            if (i + 1 < n) {   // g_{i+1} and Jn of node i+2 from HF1 (hw 0..2)
                lds_wait_ge(gcnt, 3u * (uint32_t)(i + 1), a.status, dead, tg, (uint32_t)i, a.epoch);
                STAMP3(8);
                prep(i + 1);
                STAMP3(9);
            }
            lds_barrier3();
        }
        {
            const int i = n;
            PROG3();
        }
        lds_barrier3();   // epilogue step n
    } else {
        // ============================ HELPERS ============================
        int lk[LTQ], lm[LTQ];
#pragma unroll
        for (int q = 0; q < LTQ; ++q) {
            const int e = hl + C::NHB * q;
            int k = -1, m = -1;
            if (hl < C::NHB && e < NLT) tri_decode3(e, k, m);
            lk[q] = k;
            lm[q] = m;
        }
        for (int i = 0; i <= n; ++i) {
            STAMP3(0);
            const int par = i & 1, ppar = (i + 1) & 1;
            const double* Bi = Kbuf + (size_t)par * KSZ;     // B_i
            double* Kn = Kbuf + (size_t)ppar * KSZ;          // K_i = B_{i+1}
            // new covariance of node i-2 (staged by HB last step): coalesced stores
            // (hw 4: no loads of its own to wait for)
            if (hw == 4 && i >= 2) flush_cov(i - 2);
            // hand-off granules of mu_{i+2,t-1} for HF1 at step i+1: one step ahead
            // only, so they are current when read (slice t trails t-1 by ~2 steps).
            // Loaded with 8-byte atomic loads, not LDS-DMA: a 16-byte DMA that
            // races the producer's store may see a granule half-written (new epoch,
            // old value), which the epoch check cannot tell apart.
            // (set and consumed only inside hw 5's branches, so the compiler's wait
            // on this register's previous load stays out of the other waves' path --
            // a vmcnt(0) there would also drain the loader's LDS-DMA and hw 4's
            // covariance stores at every step start)
            uint64_t pgr;
            if (hw == 5) {
                if (i + 2 < n && tg > 0 && lane < D)
                    pgr = (tl == 0) ? gran_load_system(gran_src(i + 2) + lane)
                                    : gran_load_agent(gran_src(i + 2) + lane);
                else
                    pgr = 0;
            }
            // HB (hw 0..5): K_i = B_i - L W^T + G X^T, fused covariance of node i-1
            if (hw <= 5) {
                const double* rp = rec + (size_t)ppar * D * RS;   // [k][field]
                const double* pdp = pdl + (size_t)ppar * D;
                const float* co = cring + (size_t)((i + 3) & 3) * LY::cs;   // node i-1
                float* cv = cst + (size_t)(i & 1) * LY::cs;                  // node i-1, staged
#pragma unroll
                for (int q = 0; q < LTQ; ++q) {
                    const bool ok = lk[q] >= 0;
                    const int k = ok ? lk[q] : 0, m = ok ? lm[q] : 0;
                    const double* rk = rp + k * RS;
                    const double* rm = rp + m * RS;
                    const double bkm = Bi[k * KS + m];
                    const float ckm = co[k * D + m], cmk = co[m * D + k];
                    const double c = bkm - (rk[0] * rm[2] + rk[1] * rm[3]);
                    const double kn = c + (rk[4] * rm[6] + rk[5] * rm[7]);
                    float c32;
                    if (is_naive) {
                        c32 = (k == m) ? 1.0f / ((float)pdp[k] + 1e-8f) : 0.f;
                    } else {
                        c32 = (float)c;
                        if (is_bad && ((k < 2) != (m < 2))) c32 = 0.f;
                        if (k == m) c32 = c32 + 1e-6f;
                    }
                    const float n_km = mul_add_rn(lr, c32, om, ckm);
                    const float n_mk = mul_add_rn(lr, c32, om, cmk);
                    if (ok && i < n) {
                        Kn[k * KS + m] = kn;
                        Kn[m * KS + k] = kn;
                    }
                    if (ok && i >= 1) {
                        cv[k * D + m] = n_km;
                        if (k != m) cv[m * D + k] = n_mk;
                    }
                }
            }
            STAMP3(4);
            if (lane == 0) lds_signal_add(kcnt, 1u);
            // HF1 (hw 0..2): hand-off of mu_{i+1,t-1} (DMA'd 3 steps ago), AR terms, g_{i+1}
            if (hw <= 2 && i + 1 < n) {
                uint64_t gv = 0;
                if (lane < D) gv = pring[(size_t)((i + 1) & 3) * 128 + lane];
#ifdef AME_STAMPS
                STAMP3(1);
                if (!__all((lane >= D) || (uint32_t)(gv >> 32) == a.epoch)) STAMP3(6);
#endif
                gran_finish(i + 1, gv, muL + hw * 64);
                STAMP3(2);
                wave_lds_sync3();
                hf1(i + 1);
                STAMP3(3);
                if (hw == 0) jn_fill(i + 2);   // J rows of node i+2 for the solver
                if (lane == 0) lds_signal_add(gcnt, 1u);
            }
            if (i < n) {
                // M update with mu_{i-1} (owner lane)
                if (i >= 1) {
                    const int j = i - 1, so = j / kNH, ho = (j - so * kNH + kGOFF) % kNH;
                    if (hl == ho) {
                        const float* mup = mu32 + ppar * D;
                        if (so < NSREG) {
#pragma unroll
                            for (int s = 0; s < NSREG; ++s)
                                if (s == so) {
#pragma unroll
                                    for (int c = 0; c < M2; ++c) mreg[s][c] = mup[2 + c];
                                }
                        } else {
                            for (int c2 = 0; c2 < MP; ++c2) {
                                float2 v = make_float2(mup[2 + 2 * c2], 0.f);
                                if (2 * c2 + 1 < M2) v.y = mup[3 + 2 * c2];
                                mlds[((so - NSREG) * MP + c2) * kNH + hl] = v;
                            }
                        }
                    }
                }
                // HE: GEMV of node i+2 (its Y row landed in the ring by step i-1)
                if (i + 2 < n) gemv(i + 2, yring + (size_t)((i + 2) & 3) * YS, i);
                STAMP3(5);
                // loader: this step's batch -- Y row i+5, covariance of node i+2, old
                // means of node i+5 (slice t) and i+4 (slice t+1)
                if (hw == 6) {
                    dma_y(i + 5);
                    dma_cov(i + 2);
                    dma_x(i + 5);
                    dma_r(i + 4);
                    STAMP3(6);
                }
            }
            // the batch issued 2 steps ago must have landed before the next step reads it
            if (hw == 6) vm_wait_le(2 * KDMA);
            // granules of node i+2, read by HF1 next step (slot (i+2) & 3: not read
            // this step)
            if (hw == 5 && i < n && lane < D) pring[(size_t)((i + 2) & 3) * 128 + lane] = pgr;
            STAMP3(9);
            lds_barrier3();
        }
    }
    // the last node's new covariance (staged by HB in the epilogue step n)
    if (wave == 5 && n >= 1) flush_cov(n - 1);
    // ---- slice done: release its means, covariances and granules, then flag it
    // for the next sweep (every wave drains its own stores first).  A slice with
    // a failed or abandoned wait flags nothing: what waits on it gives up
    // quietly (the status block already holds the cause) ----
    bool any_dead = false;
    if (a.done != nullptr || (tl == 0 && a.back_out != nullptr)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // (an LDS word, not __syncthreads_or: that one adds 256 bytes of static
        // LDS to the launch)
        if (dead) flags[1] = 1u;
        __syncthreads();
        any_dead = flags[1] != 0u;
    }
    if (a.done != nullptr && !any_dead) {
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.done + tl, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // ---- first slice of a rank with a left neighbour: its new means are that
    // rank's next_old in the next (pipelined) sweep; system-scope release ----
    if (tl == 0 && a.back_out != nullptr && !any_dead) {
        for (int e = tid; e < n * D; e += kNT)
            a.back_out[e] = __uint_as_float(__hip_atomic_load(
                const_cast<uint32_t*>((const uint32_t*)(xn + e)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store((uint32_t*)(a.back_out + AME_BACK_DONE_OFFSET(n * D)), a.epoch,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}


// v3 keeps one state row per solver lane: D = 2 + 2r <= 64.
constexpr int kV3MaxR = 31;

template <int R>
static int l3_total(int n) { return Lay<R>::total(n, Cfg<R>::NSREG); }

template <int R>
static int sweep3_occupancy(int n) {
    const int lds = l3_total<R>(n);
    auto kern = ame_sweep3_kernel<R, AME_GOOD>;   // the variants share the launch shape
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
        return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kNT, (size_t)lds) != hipSuccess)
        return 0;
    return per_cu;
}

int AME_PFN(ame_sweep3_blocks_per_cu)(int n, int r) {
    switch (r) {
#define X(RR) \
    case RR: if constexpr (RR <= kV3MaxR) return sweep3_occupancy<RR>(n); else return 0;
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}

// v3 needs: the slice's LDS (rings + overflow node slots) within one CU, at
// most 2 x 31 loader DMA instructions in flight (vmcnt range) and D <= 64.
template <int R>
static int sweep3_fits(int n) {
    using C = Cfg<R>;
    if (n < 2 || C::D > 64) return 0;
    const int ny = (n * 8 + 1023) / 1024;
    if (2 * (ny + C::NC + 3) > 63) return 0;
    return l3_total<R>(n) <= kLDSMAX;
}

int AME_PFN(ame_sweep3_supported)(int n, int r) {
    switch (r) {
#define X(RR) \
    case RR: if constexpr (RR <= kV3MaxR) return sweep3_fits<RR>(n); else return 0;
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}

int AME_PFN(ame_sweep3_lds)(int n, int r) {
    switch (r) {
#define X(RR) \
    case RR: if constexpr (RR <= kV3MaxR) return l3_total<RR>(n); else return 0;
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}

template <int R>
static int launch_sweep3(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    const int lds = l3_total<R>(dm->n);
    auto kern = dm->variant == AME_NAIVE ? ame_sweep3_kernel<R, AME_NAIVE>
              : dm->variant == AME_BAD   ? ame_sweep3_kernel<R, AME_BAD>
                                         : ame_sweep3_kernel<R, AME_GOOD>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) !=
        hipSuccess)
        return -2;
    hipLaunchKernelGGL(kern, dim3(dm->T_local), dim3(kNT), (size_t)lds, st, *dm, *a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int AME_PFN(ame_sweep3_dispatch)(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    switch (dm->r) {
#define X(RR) \
    case RR: if constexpr (RR <= kV3MaxR) return launch_sweep3<RR>(dm, a, st); else return -1;
        AME_FOR_EACH_R(X)
#undef X
        default: return -1;
    }
}

#if AME_PART0
long long ame_sweep3_work_doubles(const ame_dims* dm) {
    (void)dm;   // the base inverse lives in LDS (formed in the sweep prologue)
    return 0;
}
#endif
