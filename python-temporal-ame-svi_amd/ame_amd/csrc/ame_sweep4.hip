// K1 (v4): Gauss-Seidel sweep of TemporalAMEStructuredMFVI / TemporalAMENaiveMFVI
// on gfx950 with the observation natural parameter formed by MFMA block GEMMs.
//
// Reference semantics (Alfieriek/Python-Temporal-AME-SVI):
//   _update_step                structured_mf.py:211-218  (for i in range(n))
//   _update_node_i              structured_mf.py:220-287  (for t in range(T))
//   _compute_observation_terms  structured_mf.py:289-326
//   naive variant               naive_mf.py:207-282
//
// Same solver / helper-wave structure and Woodbury algebra as v3
// (ame_sweep3.hip, restated in tests/test_sweep_algebra.py).  What changes is
// h_obs(m) = sum_{j != m} J_j^T z_mj (z = R^-1 y; new means for j < m, old for
// j > m).  v3 formed it per step as a 1024-long GEMV on seven helper waves,
// each ending in a 34-value cross-lane reduce-scatter: ~60 % of the step's VALU
// work.  v4 splits it (schedule checked on the CPU by
// tests/test_sweep4_schedule.py):
//   * block GEMM: for the 16 nodes of block b, every column j outside the
//     window W(b) = [16b - 22, 16b + 16), on v_mfma_f32_16x16x4_f32
//     (A = z of the block's Y rows, B = the slice's (U, V) from a transposed
//     HBM copy Mt), spread over the 16 helper steps [16b - 18, 16b - 2) on
//     four helper waves (4 K-steps each per step), partials reduced in fp64;
//   * window GEMV: at step m - 2, the <= 34 columns of W(b) other than
//     m-3 .. m, from a 64-slot LDS ring of (U, V) rows (old rows DMA'd 22
//     steps ahead, new rows written as nodes finish), two half-waves;
//   * HF1 (step m - 1) adds nodes m - 3 and m - 2; the solver adds m - 1.
// Columns outside the window read new means only for j < 16b - 22, which
// every copy has by the time the GEMM loads them (Mt store of node j at step
// j + 1, drained at the start of step j + 2, loaded from step j + 3), and old means for
// j >= 16b + 16, which nothing has touched yet.
//
// Accuracy: each GEMM output is 4 fp32 MFMA chains of <= n/64 K-steps per
// wave, summed in fp32 pairs then in fp64 over the 4 waves; the window is
// <= 16 sequential fp32 terms per half; HF1 adds everything in fp64.
#include "ame_common.h"
#include "ame_wave.h"
#include "ame_sweep_dev.h"

using namespace ame;

#ifdef AME_STAMPS
#define S4_I0 256
__device__ unsigned long long g_s4_stamps[5 * 16 * 16];
__device__ unsigned long long g_s4_prog[256 * 5];
#define S4W(w) ((w) == 0 ? 0 : (w) == 1 ? 1 : (w) == 4 ? 2 : (w) == 5 ? 3 : (w) == 7 ? 4 : -1)
#define STAMP4(slot)                                                                           \
    do {                                                                                       \
        if (tl == TL / 2 && lane == 0 && i >= S4_I0 && i < S4_I0 + 16 && S4W(wave) >= 0) {     \
            unsigned long long t_;                                                             \
            __builtin_amdgcn_sched_barrier(0);                                                 \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
            __builtin_amdgcn_sched_barrier(0);                                                 \
            g_s4_stamps[(S4W(wave) * 16 + (i - S4_I0)) * 16 + (slot)] = t_;                    \
        }                                                                                      \
    } while (0)
#define PROG4()                                                                                \
    do {                                                                                       \
        if (tid == 0 && (i == 0 || i == n / 4 || i == n / 2 || i == 3 * n / 4 || i == n)) {    \
            const int q_ = (i == 0) ? 0 : (i == n / 4) ? 1 : (i == n / 2) ? 2 : (i == 3 * n / 4) ? 3 : 4; \
            g_s4_prog[tl * 5 + q_] = __builtin_amdgcn_s_memrealtime();                         \
        }                                                                                      \
    } while (0)
extern "C" int ame_debug_read_stamps4(unsigned long long* st, unsigned long long* prog) {
    if (hipMemcpyFromSymbol(st, HIP_SYMBOL(g_s4_stamps), sizeof(g_s4_stamps), 0, hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(prog, HIP_SYMBOL(g_s4_prog), sizeof(g_s4_prog), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define STAMP4(slot) do { } while (0)
#define PROG4() do { } while (0)
#endif

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kNT = 512;     // threads per workgroup: solver wave + 7 helper waves
constexpr int kBS = 16;      // GEMM block: 16 nodes (MFMA rows)
constexpr int kGL = 22;      // window lead: W(b) = [16b - kGL, 16b + kBS)
constexpr int kGS = 18;      // GEMM of block b runs at helper steps [16b - kGS, 16b - 2)
constexpr int kVM = 2;       // 16-column groups per GEMM wave per step (n <= 2048)
constexpr int kMR = 64;      // (U, V) ring slots
constexpr int kYW = 8;       // Y window ring slots (1 KiB = 128 columns each)
constexpr int kLAG = 6;      // slice t starts once slice t-1 has finished this node (see prologue)
constexpr int kLDSMAX = 160 * 1024;

__host__ __device__ constexpr int al16(int x) { return (x + 15) & ~15; }

template <int R>
struct Cfg4 {
    static constexpr int D = 2 + 2 * R, M2 = 2 * R, DD = D * D;
    static constexpr int NLT = D * (D + 1) / 2;
    static constexpr int NHB = 384;                           // HB lanes (hw 0-5)
    static constexpr int LTQ = (NLT + NHB - 1) / NHB;
    static constexpr int NP = (4 * D <= 192) ? 4 : 2;       // AR row parts (HF1)
    static constexpr int MC = (D + NP - 1) / NP;
    static constexpr int NHALF = (6 * D <= 256) ? 2 : 1;    // HF2 row halves
    static constexpr int HD = D / NHALF;
    static constexpr int NC = (DD * 4 + 1023) / 1024;       // DMA KiB per covariance
};

// LDS carve-up (bytes), all compile-time: nothing scales with n.
template <int R>
struct Lay4 {
    static constexpr int D = 2 + 2 * R, DD = D * D;
    static constexpr int cs = ((DD * 4 + 1023) / 1024) * 256;     // covariance ring slot (floats)
    static constexpr int oK = 0;                                   // base inverse, double buffer
    static constexpr int NPA = (4 * D <= 192) ? 4 : 2;
    static constexpr int MCP = ((D + NPA - 1) / NPA) * NPA;
    static constexpr int oAR = al16(oK + 8 * 2 * DD);              // Qinv Phi, Phi^T Qinv [D][MCP]
    static constexpr int oRec = al16(oAR + 8 * 2 * D * MCP);       // [par][k]{L0 L1 W0 W1 G0 G1 X0 X1}
    static constexpr int oMu64 = al16(oRec + 8 * 2 * D * 8);
    static constexpr int oMu32 = al16(oMu64 + 8 * 2 * D);
    static constexpr int oG = al16(oMu32 + 4 * 2 * D);
    static constexpr int oJn = al16(oG + 8 * 2 * D);
    static constexpr int oV = al16(oJn + 8 * 2 * D);
    static constexpr int oDots = al16(oV + 8 * 2 * D * 4);
    static constexpr int oRed = al16(oDots + 8 * 32);
    static constexpr int oWP = al16(oRed + 8 * 64);                // [m&1][half][k] window partials (f32)
    static constexpr int oHB = al16(oWP + 4 * 2 * 2 * D);          // [b&1][row][k] block h (f64)
    static constexpr int oGP = al16(oHB + 8 * 2 * kBS * D);        // [wave][row][k] GEMM partials (f32)
    static constexpr int oGS = al16(oGP + 4 * 4 * kBS * D);        // [wave][kq][row][2] z row sums (f32)
    static constexpr int oMuL = al16(oGS + 4 * 4 * 4 * kBS * 2);   // [wave][64] mu_{m,t-1}
    static constexpr int oPd = al16(oMuL + 4 * 3 * 64);
    static constexpr int oPc = al16(oPd + 8 * 2 * D);
    static constexpr int oFlag = al16(oPc + 8 * D);
    static constexpr int oCr = al16(oFlag + 16);                   // [node&3] old covariances, DMA
    static constexpr int oXr = al16(oCr + 4 * 4 * cs);             // [node&7] old means slice t, DMA
    static constexpr int oRr = al16(oXr + 8 * 256);                // [node&3] old means slice t+1, DMA
    static constexpr int oPr = al16(oRr + 4 * 256);                // [node&3] hand-off granules, DMA
    static constexpr int oYw = al16(oPr + 4 * 1024);               // [row&7] Y window rows, DMA
    static constexpr int oMR = al16(oYw + kYW * 1024);             // [node&63][64] (U,V) ring
    static constexpr int total = al16(oMR + kMR * 256);
};

// J entries for state index k from a ring row [U(R), V(R)]:
// J0 = [1, 0, V, 0], J1 = [0, 1, 0, U].
template <int R>
__device__ __forceinline__ void jcol_uv(const float* uv, int k, double& j0, double& j1) {
    constexpr int D = 2 + 2 * R;
    const bool ku = (k >= 2 && k < 2 + R), kv = (k >= 2 + R && k < D);
    const double v = (double)uv[ku ? (k + R - 2) : (kv ? (k - 2 - R) : 0)];
    j0 = (k == 0) ? 1.0 : (ku ? v : 0.0);
    j1 = (k == 1) ? 1.0 : (kv ? v : 0.0);
}

__device__ __forceinline__ int win_lo(int b) { return max(0, kBS * b - kGL); }

}  // namespace

template <int R>
__global__ void __launch_bounds__(kNT)
ame_sweep4_kernel(ame_dims dm, ame_sweep_args a) {
    using C = Cfg4<R>;
    constexpr int D = C::D, M2 = C::M2, DD = C::DD;
    constexpr int NLT = C::NLT, LTQ = C::LTQ, NP = C::NP, MC = C::MC, NHALF = C::NHALF, HD = C::HD;
    constexpr int NC = C::NC;
    const int n = dm.n, TL = dm.T_local, Tt = dm.T_total;
    const int ns = (n + 15) & ~15;            // Mt row stride (floats)
    const int NG = ns >> 4;                   // 16-column groups
    const int b = blockIdx.x;
    const int tl = (TL % 8 == 0) ? ((b & 7) * (TL >> 3) + (b >> 3)) : b;   // XCD-aware (speed only)
    const int tg = dm.t_begin + tl;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int hl = tid - 64, hw = wave - 1;
    const bool is_naive = dm.variant == AME_NAIVE, is_bad = dm.variant == AME_BAD;
    constexpr int KDMA = NC + 5;              // DMA instructions per step (loader wave)

    extern __shared__ __attribute__((aligned(16))) char smem[];
    using LY = Lay4<R>;
    double* Kbuf = (double*)(smem + LY::oK);
    constexpr int MCP = LY::MCP;
    double* arQ = (double*)(smem + LY::oAR);
    double* arP = arQ + D * MCP;
    double* rec = (double*)(smem + LY::oRec);
    double* mu64 = (double*)(smem + LY::oMu64);
    float* mu32 = (float*)(smem + LY::oMu32);
    double* g64 = (double*)(smem + LY::oG);
    double* jn64 = (double*)(smem + LY::oJn);
    double* vbuf = (double*)(smem + LY::oV);
    double* dots = (double*)(smem + LY::oDots);
    double* red = (double*)(smem + LY::oRed);
    float* wpart = (float*)(smem + LY::oWP);
    double* hblk = (double*)(smem + LY::oHB);
    float* gpart = (float*)(smem + LY::oGP);
    float* gsum = (float*)(smem + LY::oGS);
    float* muL = (float*)(smem + LY::oMuL);
    double* pdl = (double*)(smem + LY::oPd);
    double* pcdl = (double*)(smem + LY::oPc);
    uint32_t* flags = (uint32_t*)(smem + LY::oFlag);
    uint32_t* kcnt = flags;
    uint32_t* ddone = flags + 1;
    uint32_t* gcnt = flags + 2;
    float* cring = (float*)(smem + LY::oCr);
    float* xring = (float*)(smem + LY::oXr);
    float* rring = (float*)(smem + LY::oRr);
    uint64_t* pring = (uint64_t*)(smem + LY::oPr);
    float2* ywin = (float2*)(smem + LY::oYw);
    float* mring = (float*)(smem + LY::oMR);

    const double r00 = a.rinv[0], r01 = a.rinv[1], r10 = a.rinv[2], r11 = a.rinv[3];
    const float r00f = (float)r00, r01f = (float)r01, r10f = (float)r10, r11f = (float)r11;
    const Mat2 Rm = inv2s(m2(r00, r01, r10, r11));
    const float lr = a.lr, om = a.one_minus_lr;
    const float* xo = a.x_old + (size_t)tl * n * D;
    float* xn = a.x_new + (size_t)tl * n * D;
    float* cvs = a.cov + (size_t)tl * n * DD;
    float* cvw = (a.cov_new != nullptr ? a.cov_new : a.cov) + (size_t)tl * n * DD;
    const float* ysl = a.Yt + (size_t)tl * n * n * 2;
    float* Mt = (float*)a.work + (size_t)tl * M2 * ns;      // [2r][ns] current (U, V), transposed
    const bool back_rd = (a.wait_epoch != 0u) && (tl == TL - 1) && (a.back_in != nullptr);
    const float* xr = (tg < Tt - 1) ? ((tl < TL - 1) ? a.x_old + (size_t)(tl + 1) * n * D
                                                     : (back_rd ? a.back_in : a.next_old))
                                    : nullptr;
    const double* QiPhi = a.consts + 3 * (size_t)DD;
    bool dead = false;

    // ---- hand-off of mu_{node, t-1} (as v3) ----
    auto gran_src = [&](int node) -> const uint64_t* {
        return (tl == 0) ? a.halo_in + (size_t)node * D : a.hand + ((size_t)(tl - 1) * n + node) * D;
    };
    auto gran_finish = [&](int node, uint64_t v, float* dst) {
        if (tg == 0) {
            if (lane < D) dst[lane] = 0.f;
            return;
        }
        bool ok = (lane >= D) || (uint32_t)(v >> 32) == a.epoch;
        if (!__all(ok) && !dead) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            const uint64_t budget = (tl == 0) ? AME_SPIN_TICKS_HALO : AME_SPIN_TICKS_LOCAL;
            const uint64_t* src = gran_src(node);
            while (true) {
                if (lane < D) {
                    v = (tl == 0) ? gran_load_system(src + lane) : gran_load_agent(src + lane);
                    ok = (uint32_t)(v >> 32) == a.epoch;
                }
                if (__all(ok)) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > budget) {
                    if (lane == 0)
                        atomicOr(a.status, (tl == 0) ? AME_STATUS_HALO_TIMEOUT : AME_STATUS_SPIN_TIMEOUT);
                    dead = true;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        if (lane < D) dst[lane] = __uint_as_float((uint32_t)v);
    };

    // ---- loader DMA pieces (whole-wave; fixed instruction count per call) ----
    auto dma_yw = [&](int row) {   // Y row `row`, columns [win_lo, +128) -> slot row & 7 : 1 instruction
        const int rw = (row < n) ? row : 0;
        const int c0 = win_lo(rw >> 4);
        const char* base = (const char*)(ysl + ((size_t)rw * n + c0) * 2);
        int off = lane * 16;
        if (c0 * 8 + off >= n * 8) off = 0;
        dma16(base + off, lds_off(ywin + (size_t)(row & (kYW - 1)) * 128));
    };
    auto dma_cov = [&](int node) {
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
    auto dma_x = [&](int node) {
        const int xnn = (node < n) ? node : 0;
        dma4(xo + (size_t)xnn * D + (lane < D ? lane : 0), lds_off(xring + (node & 7) * 64));
    };
    auto dma_r = [&](int node) {
        const float* src = (xr != nullptr && node < n) ? xr + (size_t)node * D : xo;
        if (back_rd) dma4_sys(src + (lane < D ? lane : 0), lds_off(rring + (node & 3) * 64));
        else dma4(src + (lane < D ? lane : 0), lds_off(rring + (node & 3) * 64));
    };
    // NOTE: a 16-byte LDS-DMA of granules can tear one {epoch, value} pair if it
    // races the producer's store (v3 therefore reads them with 8-byte atomic
    // loads, ame_sweep3.hip).  Here the DMA runs 3 steps ahead, where the
    // granule is either long written or still stale (epoch mismatch -> poll);
    // v4 is an opt-in experiment.
    auto dma_p = [&](int node) {
        const uint32_t dst = lds_off(pring + (size_t)(node & 3) * 128);
        const int g2 = (lane * 2 < D) ? lane * 2 : 0;
        if (tg == 0 || node >= n) dma16(xo, dst);
        else if (tl == 0) dma16_sys(gran_src(node) + g2, dst);
        else dma16_sc1(gran_src(node) + g2, dst);
    };
    auto dma_m = [&](int node) {   // old (U, V) of `node` -> ring slot node & 63 : 1 instruction
        const int mn = (node < n) ? node : 0;
        dma4(xo + (size_t)mn * D + 2 + (lane < M2 ? lane : 0), lds_off(mring + (node & (kMR - 1)) * 64));
    };

    // ============================ prologue ============================
    if (a.wait_epoch != 0u) {
        if (tid == 0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            for (int q = 0; q < 2 && tl + q < TL; ++q) {
                while (__hip_atomic_load(a.done + tl + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                       a.wait_epoch) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 > AME_SPIN_TICKS_LOCAL) {
                        atomicOr(a.status, AME_STATUS_SPIN_TIMEOUT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
            }
            if (back_rd) {
                const uint32_t* bd = (const uint32_t*)(a.back_in + AME_BACK_DONE_OFFSET(n * D));
                while (__hip_atomic_load(const_cast<uint32_t*>(bd), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_SYSTEM) < a.wait_epoch) {
                    if (__builtin_amdgcn_s_memrealtime() - t0 > AME_SPIN_TICKS_HALO) {
                        atomicOr(a.status, AME_STATUS_HALO_TIMEOUT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(8);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    // P_0 = Pconst + sum_{j>=1} F_j(old) (fp64) and its inverse -> Kbuf[0]; naive:
    // column sums of squares of (U, V) over all nodes -> red[]   (as v3)
    {
        constexpr int EQ = (NLT + kNT - 1) / kNT;
        float* st = mring;   // staging: CH nodes x 2r (the ring is not live yet)
        double* piv = vbuf;
        double* K = Kbuf;
        constexpr int CH = (kMR * 64) / M2 < 64 ? (kMR * 64) / M2 : 64;
        const double pp = r00, ss = r11, qq = 0.5 * (r01 + r10);
        double acc[EQ];
        int ek[EQ], em[EQ];
#pragma unroll
        for (int u = 0; u < EQ; ++u) {
            acc[u] = 0.0;
            const int e = tid + kNT * u;
            int k = -1, m = -1;
            if (e < NLT) tri_decode3(e, k, m);
            ek[u] = k;
            em[u] = m;
        }
        double sq = 0.0;
        for (int j0 = 1; j0 < n; j0 += CH) {
            const int cnt = min(CH, n - j0);
            __syncthreads();
            for (int e = tid; e < cnt * M2; e += kNT) {
                const int jj = e / M2, c = e - jj * M2;
                st[e] = xo[(size_t)(j0 + jj) * D + 2 + c];
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < EQ; ++u) {
                const int k = ek[u], m = em[u];
                if (k < 2) continue;
                const int ck = k - 2;
                const int kc = (ck < R) ? R + ck : ck - R;
                double a0 = 0.0;
                if (m < 2) {
                    for (int jj = 0; jj < cnt; ++jj) a0 += (double)st[jj * M2 + kc];
                } else {
                    const int cm = m - 2;
                    const int mc = (cm < R) ? R + cm : cm - R;
                    for (int jj = 0; jj < cnt; ++jj)
                        a0 = fma((double)st[jj * M2 + kc], (double)st[jj * M2 + mc], a0);
                }
                acc[u] += a0;
            }
            if (tid < M2)
                for (int jj = 0; jj < cnt; ++jj) {
                    const double v = (double)st[jj * M2 + tid];
                    sq = fma(v, v, sq);
                }
        }
        if (tid < M2) {
            const double v = (double)xo[2 + tid];
            red[tid] = fma(v, v, sq);
        }
#pragma unroll
        for (int u = 0; u < EQ; ++u) {
            const int k = ek[u], m = em[u];
            if (k < 0) continue;
            double v;
            if (k < 2) {
                v = ((k == 0 && m == 0) ? pp : (k == 1 && m == 1) ? ss : qq) * (double)(n - 1);
            } else {
                const bool ku = (k - 2) < R;
                if (m < 2) {
                    v = (ku ? (m == 0 ? pp : qq) : (m == 0 ? qq : ss)) * acc[u];
                } else {
                    const bool mu_ = (m - 2) < R;
                    v = ((ku && mu_) ? pp : ((!ku && !mu_) ? ss : qq)) * acc[u];
                }
            }
            v += pconst_entry(a.consts, D, k, m, tg, Tt);
            K[k * D + m] = v;
            K[m * D + k] = v;
        }
        __syncthreads();
        for (int pv = 0; pv < D; ++pv) {
            if (tid < D) piv[tid] = K[pv * D + tid];
            __syncthreads();
            const double rinv = 1.0 / piv[pv];
            for (int e = tid; e < NLT; e += kNT) {
                int k, m;
                tri_decode3(e, k, m);
                double v;
                if (k == pv && m == pv) v = -rinv;
                else if (k == pv) v = piv[m] * rinv;
                else if (m == pv) v = piv[k] * rinv;
                else v = K[k * D + m] - (piv[k] * piv[m]) * rinv;
                K[k * D + m] = v;
                K[m * D + k] = v;
            }
            __syncthreads();
        }
        for (int e = tid; e < DD; e += kNT) K[e] = -K[e];
        __syncthreads();
    }
    for (int e = tid; e < 2 * D * MCP; e += kNT) {
        const int mat = e / (D * MCP), rc = e - mat * D * MCP, rr = rc / MCP, cc = rc - rr * MCP;
        arQ[e] = (cc < D) ? QiPhi[(size_t)mat * DD + rr * D + cc] : 0.0;
    }
    for (int e = tid; e < 3 * 64; e += kNT) muL[e] = 0.f;
    if (tid < D) pcdl[tid] = pconst_entry(a.consts, D, tid, tid, tg, Tt);
    for (int e = tid; e < 2 * D * 8; e += kNT) rec[e] = 0.0;
    for (int e = tid; e < 2 * D; e += kNT) {
        mu64[e] = 0.0;
        mu32[e] = 0.f;
    }
    if (tid < 4) flags[tid] = 0u;
    // transposed (U, V) copy of the slice's old means (padding columns zero)
    for (int e = tid; e < M2 * ns; e += kNT) {
        const int c = e / ns, j = e - c * ns;
        Mt[e] = (j < n) ? xo[(size_t)j * D + 2 + c] : 0.f;
    }
    __syncthreads();   // the P_0 staging in the ring region is no longer read
    // (U, V) ring rows of nodes 0..19; Y windows of rows 0..4
    for (int e = tid; e < kGL * 64; e += kNT) {
        const int j = e >> 6, c = e & 63;
        mring[e] = (j < n && c < M2) ? xo[(size_t)j * D + 2 + c] : 0.f;
    }
    for (int e = tid; e < 5 * 128; e += kNT) {
        const int row = e >> 7, c = e & 127;
        const int c0 = win_lo(row >> 4);
        ywin[e] = (row < n && c0 + c < n) ? *(const float2*)(ysl + ((size_t)row * n + c0 + c) * 2)
                                           : make_float2(0.f, 0.f);
    }
    double ssq_l = 0.0;
    if (tid < D && is_naive && tid >= 2) ssq_l = red[tid - 2];
    if (wave == 7) {
        for (int q = 0; q < 5; ++q) dma_x(q);
        for (int q = 0; q < 4; ++q) dma_r(q);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // Mt stores and the DMAs
    __syncthreads();

    // ---------------- block GEMM (helper waves hw 0..3) ----------------
    f32x4 accV[4], accU[4];
    float rs0 = 0.f, rs1 = 0.f;
    f32x4 pa0[kVM], pa1[kVM], pv[kVM], pu[kVM];
    const int gw = hw;              // GEMM wave index (valid for hw 0..3)
    const int grow = lane & 15, gkq = lane >> 4;
    auto gemm_load = [&](int bb, int q) {
        if (bb < 0 || kBS * bb >= n) return;
        int m = kBS * bb + grow;
        if (m >= n) m = n - 1;
        const int cu = (grow < R) ? grow : 0;
#pragma unroll
        for (int v = 0; v < kVM; ++v) {
            const int u = 4 * q + gw + 64 * v;
            if (u < NG) {
                int j0 = 16 * u + 4 * gkq;
                const int jy = (j0 < n) ? j0 : 0;   // n % 4 == 0: a chunk is all in or all out
                const float4* ya = (const float4*)(ysl + ((size_t)m * n + jy) * 2);
                const float4 y0 = ya[0], y1 = ya[1];
                pa0[v] = f32x4{y0.x, y0.y, y0.z, y0.w};
                pa1[v] = f32x4{y1.x, y1.y, y1.z, y1.w};
                const float4 bv = *(const float4*)(Mt + (size_t)(R + cu) * ns + j0);
                const float4 bu = *(const float4*)(Mt + (size_t)cu * ns + j0);
                pv[v] = f32x4{bv.x, bv.y, bv.z, bv.w};
                pu[v] = f32x4{bu.x, bu.y, bu.z, bu.w};
            }
        }
    };
    auto gemm_compute = [&](int bb, int q) {
        if (bb < 0 || kBS * bb >= n) return;
        if (q == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                accV[e] = f32x4{0.f, 0.f, 0.f, 0.f};
                accU[e] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            rs0 = rs1 = 0.f;
        }
        const int wlo = win_lo(bb), whi = min(n, kBS * bb + kBS);
        const bool colok = grow < R;
#pragma unroll
        for (int v = 0; v < kVM; ++v) {
            const int u = 4 * q + gw + 64 * v;
            if (u < NG) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int j = 16 * u + 4 * gkq + e;
                    const float yx = (e < 2) ? pa0[v][2 * e] : pa1[v][2 * e - 4];
                    const float yy = (e < 2) ? pa0[v][2 * e + 1] : pa1[v][2 * e - 3];
                    const bool ok = (j < n) && (j < wlo || j >= whi);
                    const float z0 = ok ? r00f * yx + r01f * yy : 0.f;
                    const float z1 = ok ? r10f * yx + r11f * yy : 0.f;
                    rs0 += z0;
                    rs1 += z1;
                    const float bvv = colok ? pv[v][e] : 0.f;
                    const float buu = colok ? pu[v][e] : 0.f;
                    accV[e] = __builtin_amdgcn_mfma_f32_16x16x4f32(z0, bvv, accV[e], 0, 0, 0);
                    accU[e] = __builtin_amdgcn_mfma_f32_16x16x4f32(z1, buu, accU[e], 0, 0, 0);
                }
            }
        }
        if (q == 15) {   // block done: this wave's partial -> LDS
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const int row = 4 * gkq + v, col = grow;
                const float sV = (accV[0][v] + accV[1][v]) + (accV[2][v] + accV[3][v]);
                const float sU = (accU[0][v] + accU[1][v]) + (accU[2][v] + accU[3][v]);
                if (col < R) {
                    gpart[(gw * kBS + row) * D + 2 + col] = sV;       // h_U = sum z0 V
                    gpart[(gw * kBS + row) * D + 2 + R + col] = sU;   // h_V = sum z1 U
                }
            }
            gsum[((gw * 4 + gkq) * kBS + grow) * 2 + 0] = rs0;
            gsum[((gw * 4 + gkq) * kBS + grow) * 2 + 1] = rs1;
        }
    };
    // block b's partials -> hblk[b & 1] (fp64, fixed order); one wave
    auto gemm_reduce = [&](int bb) {
        double* hb = hblk + (size_t)(bb & 1) * kBS * D;
        for (int e = lane; e < kBS * D; e += 64) {
            const int row = e / D, k = e - row * D;
            double s = 0.0;
            if (k < 2) {
#pragma unroll
                for (int w = 0; w < 4; ++w)
#pragma unroll
                    for (int kq = 0; kq < 4; ++kq) s += (double)gsum[((w * 4 + kq) * kBS + row) * 2 + k];
            } else {
#pragma unroll
                for (int w = 0; w < 4; ++w) s += (double)gpart[(w * kBS + row) * D + k];
            }
            hb[e] = s;
        }
    };
    // window GEMV of node m, half h: columns of W(m >> 4) with the same parity as
    // win_lo + h, other than m-3 .. m  -> wpart[m & 1][h][.]
    auto wgemv = [&](int m, int h) {
        const int bb = m >> 4, c0 = win_lo(bb), c1 = min(n, kBS * bb + kBS);
        const int k = lane;
        const bool ku = (k >= 2 && k < 2 + R), kv = (k >= 2 + R && k < D);
        const int src = ku ? (k + R - 2) : (kv ? (k - 2 - R) : 0);
        const bool use_z1 = (k == 1) || kv;
        const bool unit = k < 2;
        const float2* yr = ywin + (size_t)(m & (kYW - 1)) * 128;
        // fixed trip count (the window is at most kGL + kBS columns), predicated,
        // so the compiler issues every LDS read of the half up front
        constexpr int NWJ = (kGL + kBS + 1) / 2;
        float yx[NWJ], yy[NWJ], mvv[NWJ];
        bool okj[NWJ];
#pragma unroll
        for (int q = 0; q < NWJ; ++q) {
            const int j = c0 + h + 2 * q;
            okj[q] = j < c1 && (j < m - 3 || j > m);
            const int jj = okj[q] ? j : c0;
            const float2 y = yr[jj - c0];
            yx[q] = y.x;
            yy[q] = y.y;
            mvv[q] = mring[(jj & (kMR - 1)) * 64 + src];
        }
        float acc = 0.f;
#pragma unroll
        for (int q = 0; q < NWJ; ++q) {
            const float z0 = r00f * yx[q] + r01f * yy[q], z1 = r10f * yx[q] + r11f * yy[q];
            const float f = okj[q] ? (unit ? 1.f : mvv[q]) : 0.f;
            acc = fmaf(use_z1 ? z1 : z0, f, acc);
        }
        if (k < D) wpart[((m & 1) * 2 + h) * D + k] = acc;
    };
    // HF1 (hw 0..2): AR terms + natural parameter g of node m.
    auto hf1 = [&](int m) {
        const int q = hl;
        const int k = q / NP, p = q - k * NP;
        const int kc = (k < D) ? k : 0;
        const float* ml = muL + hw * 64;
        const float* mr = rring + (m & 3) * 64;
        const double* aq = arQ + kc * MCP + p * MC;
        const double* ap = arP + kc * MCP + p * MC;
        double accL = 0.0, accR = 0.0;
#pragma unroll
        for (int mm = 0; mm < MC; ++mm) {
            const int c = p * MC + mm;
            accL = fma(aq[mm], (double)ml[c], accL);
            accR = fma(ap[mm], (double)mr[c], accR);
        }
        double acc = accL + ((tg < Tt - 1) ? accR : 0.0);
        acc = dpp_add_xor1(acc);
        if constexpr (NP == 4) acc = dpp_add_mirror4(acc);
        const int bb = m >> 4, c0 = win_lo(bb);
        double g = hblk[((bb & 1) * kBS + (m & 15)) * D + kc];
        g += (double)wpart[((m & 1) * 2 + 0) * D + kc] + (double)wpart[((m & 1) * 2 + 1) * D + kc];
        g += acc;
        const float2* yr = ywin + (size_t)(m & (kYW - 1)) * 128;
        if (m >= 3) {   // node m-3: new mean from the ring (written at step m-2)
            double j0, j1;
            jcol_uv<R>(mring + ((m - 3) & (kMR - 1)) * 64, kc, j0, j1);
            const float2 y = yr[m - 3 - c0];
            const double z0 = r00 * (double)y.x + r01 * (double)y.y, z1 = r10 * (double)y.x + r11 * (double)y.y;
            g = fma(j0, z0, fma(j1, z1, g));
        }
        if (m >= 2) {   // node m-2: the solver's LDS copy
            double j0, j1;
            jcol<R>(mu32 + ((m - 2) & 1) * D, true, kc, j0, j1);
            const float2 y = yr[m - 2 - c0];
            const double z0 = r00 * (double)y.x + r01 * (double)y.y, z1 = r10 * (double)y.x + r11 * (double)y.y;
            g = fma(j0, z0, fma(j1, z1, g));
        }
        if (k < D && p == 0) g64[(m & 1) * D + k] = g;
    };
    auto hf2 = [&](int m, const double* Kb) {
        const int q = tid - 256;
        const int k = q / (3 * NHALF), rem = q - k * (3 * NHALF);
        const int vsel = rem / NHALF, half = rem - vsel * NHALF;
        const int kc = (k < D) ? k : 0;
        const double* vec = (vsel == 0) ? g64 + (m & 1) * D : jn64 + (vsel - 1) * D;
        const double* kr = Kb + (size_t)kc * D;
        const int c0 = half * HD;
        double acc = 0.0;
#pragma unroll
        for (int c = 0; c < HD; ++c) acc = fma(kr[c0 + c], vec[c0 + c], acc);
        const double accA = kr[0] * vec[0] + kr[1] * vec[1];
        if constexpr (NHALF == 2) acc = dpp_add_xor1(acc);
        if (k < D && half == 0) {
            double* vo = vbuf + ((m & 1) * D + k) * 4;
            vo[vsel] = acc;
            if (vsel == 0) vo[3] = accA;
        }
    };
    auto jn_fill = [&](int node) {
        if (lane < D) {
            double j0, j1;
            jcol<R>(xring + (node & 7) * 64, node < n, lane, j0, j1);
            jn64[lane] = j0;
            jn64[D + lane] = j1;
        }
    };

    // ---- prologue work: block h of blocks 0 and 1, window h of nodes 0 and 1,
    // g_0, v_0 / yv_0; DMA rings for steps 0..2 ----
    for (int bb = 0; bb < 2; ++bb) {
        if (wave >= 1 && hw <= 3) {
            for (int q = 0; q < 16; ++q) {
                gemm_load(bb, q);
                gemm_compute(bb, q);
            }
        }
        __syncthreads();
        if (wave == 7 && kBS * bb < n) gemm_reduce(bb);
        __syncthreads();
    }
    if (wave == 5 || wave == 6) {
        wgemv(0, wave - 5);
        if (n > 1) wgemv(1, wave - 5);
    }
    if (wave >= 1 && hw <= 2) {
        uint64_t g0 = 0;
        if (tg > 0 && lane < D)
            g0 = (tl == 0) ? gran_load_system(gran_src(0) + lane) : gran_load_agent(gran_src(0) + lane);
        gran_finish(0, g0, muL + hw * 64);
        // Keep slice t at least kLAG + 1 steps behind slice t-1: then the hand-off
        // granule the loader DMAs 3 steps ahead of its use is already current, and
        // HF1 does not wait on the left slice's L2 round trip every step.  Costs a
        // wavefront fill of (kLAG + 1) steps per slice once per pipelined fit().
        if (hw == 0 && tg > 0 && n > 1) {
            const int lagn = min(n - 1, kLAG);
            uint64_t gl = 0;
            if (lane < D)
                gl = (tl == 0) ? gran_load_system(gran_src(lagn) + lane) : gran_load_agent(gran_src(lagn) + lane);
            gran_finish(lagn, gl, (float*)red + 64);
        }
    }
    if (wave == 4) jn_fill(1);
    __syncthreads();
    if (wave >= 1 && hw <= 2) hf1(0);
    __syncthreads();
    if (wave >= 4) hf2(0, Kbuf);
    if (wave == 7) {
        for (int q = 0; q <= 1; ++q) dma_cov(q);
        for (int q = 1; q <= 3; ++q) dma_p(q);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();

    if (wave == 0) {
        // ============================ SOLVER (as v3) ============================
        __builtin_amdgcn_s_setprio(3);
        const int k = lane;
        const bool kl = k < D;
        const int kc = kl ? k : 0;
        double brow[D];
#pragma unroll
        for (int c = 0; c < D; ++c) brow[c] = kl ? Kbuf[(size_t)k * D + c] : 0.0;
        double Wp0 = 0, Wp1 = 0, Xp0 = 0, Xp1 = 0, Lp0 = 0, Lp1 = 0, Gp0 = 0, Gp1 = 0;
        Mat2 Mip = m2(0, 0, 0, 0), Sip = m2(0, 0, 0, 0);
        for (int i = 0; i < n; ++i) {
            PROG4();
            STAMP4(0);
            const int par = i & 1, ppar = (i + 1) & 1;
            const bool has_prev = i > 0;
            const float* mup = mu32 + ppar * D;
            const double* mupd = mu64 + ppar * D;
            const double msk = kl ? 1.0 : 0.0;
            const double* vi = vbuf + (par * D + kc) * 4;
            const double v = msk * vi[0], yv0 = msk * vi[1], yv1 = msk * vi[2], vA = msk * vi[3];
            const double g = msk * g64[par * D + kc];
            double J0, J1;
            jcol<R>(mup, has_prev && kl, kc, J0, J1);
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
            STAMP4(1);
            constexpr int NV = 20;
            double pr[NV];
            pr[0] = Wp0 * J0; pr[1] = Wp0 * J1; pr[2] = Wp1 * J0; pr[3] = Wp1 * J1;
            pr[4] = Xp0 * J0; pr[5] = Xp0 * J1; pr[6] = Xp1 * J0; pr[7] = Xp1 * J1;
            pr[8] = J0 * kj0; pr[9] = J0 * kj1; pr[10] = J1 * kj0; pr[11] = J1 * kj1;
            pr[12] = J0 * v; pr[13] = J1 * v;
            pr[14] = J0 * yv0; pr[15] = J0 * yv1; pr[16] = J1 * yv0; pr[17] = J1 * yv1;
            pr[18] = J0 * vA; pr[19] = J1 * vA;
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
            const Mat2 cc = m2(o[8], o[9], o[10], o[11]);
            const V2 e = {o[12], o[13]};
            const Mat2 jy = m2(o[14], o[15], o[16], o[17]);
            const V2 eA = {o[18], o[19]};
            STAMP4(2);
            lds_wait_ge(ddone, (uint32_t)(i + 1), a.status, dead);
            STAMP4(3);
            const V2 b1 = {dots[0], dots[1]}, b2 = {dots[2], dots[3]};
            const Mat2 f1 = m2(dots[4], dots[5], dots[6], dots[7]);
            const Mat2 f2 = m2(dots[8], dots[9], dots[10], dots[11]);
            const Mat2 ny = m2(dots[12], dots[13], dots[14], dots[15]);
            const V2 b1A = {dots[16], dots[17]}, b2A = {dots[18], dots[19]};
            // raw y_{i,i-1} from row i's Y window
            double y0 = 0, y1 = 0;
            if (has_prev) {
                const float2 yy = ywin[(size_t)(i & (kYW - 1)) * 128 + (i - 1 - win_lo(i >> 4))];
                y0 = (double)yy.x;
                y1 = (double)yy.y;
            }
            const double zp0 = r00 * y0 + r01 * y1, zp1 = r10 * y0 + r11 * y1;
            const Mat2 JW = add(sub(cc, quad(a1, Mip, a1)), quad(a2, Sip, a2));
            const Mat2 Mm = add(Rm, sym(JW));
            const Mat2 Mi = has_prev ? inv2s(Mm) : m2(0, 0, 0, 0);
            const V2 t1 = mtv(a1, mv(Mip, b1)), t2 = mtv(a2, mv(Sip, b2));
            const V2 Ju = {e.x - t1.x + t2.x, e.y - t1.y + t2.y};
            const V2 cvec = mv(Mi, V2{y0 - Ju.x, y1 - Ju.y});
            const Mat2 wn = add(sub(jy, quad(a1, Mip, f1)), quad(a2, Sip, f2));
            const Mat2 JnK = add(sub(ny, quad(f1, Mip, f1)), quad(f2, Sip, f2));
            const Mat2 JnX = sub(JnK, quad(wn, Mi, wn));
            const Mat2 Si = inv2s(sub(Rm, sym(JnX)));
            const double W0 = kj0 - (Lp0 * a1.a + Lp1 * a1.c) + (Gp0 * a2.a + Gp1 * a2.c);
            const double W1 = kj1 - (Lp0 * a1.b + Lp1 * a1.d) + (Gp0 * a2.b + Gp1 * a2.d);
            const double u = v - (Lp0 * b1.x + Lp1 * b1.y) + (Gp0 * b2.x + Gp1 * b2.y);
            const double kn0 = yv0 - (Lp0 * f1.a + Lp1 * f1.c) + (Gp0 * f2.a + Gp1 * f2.c);
            const double kn1 = yv1 - (Lp0 * f1.b + Lp1 * f1.d) + (Gp0 * f2.b + Gp1 * f2.d);
            double mus;
            if (!is_bad) {
                mus = u + W0 * cvec.x + W1 * cvec.y;
            } else {
                const double uA = vA - (Lp0 * b1A.x + Lp1 * b1A.y) + (Gp0 * b2A.x + Gp1 * b2A.y);
                const V2 s1 = mtv(a1, mv(Mip, b1A)), s2 = mtv(a2, mv(Sip, b2A));
                const V2 JuA = {eA.x - s1.x + s2.x, eA.y - s1.y + s2.y};
                const double* r0 = rec + (ppar * D + 0) * 8;
                const double* r1 = rec + (ppar * D + 1) * 8;
                const double KE0 = brow[0] - (Lp0 * r0[2] + Lp1 * r0[3]) + (Gp0 * r0[6] + Gp1 * r0[7]);
                const double KE1 = brow[1] - (Lp0 * r1[2] + Lp1 * r1[3]) + (Gp0 * r1[6] + Gp1 * r1[7]);
                const double WE00 = __shfl(W0, 0), WE01 = __shfl(W1, 0);
                const double WE10 = __shfl(W0, 1), WE11 = __shfl(W1, 1);
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
            STAMP4(4);
            double sq_other = 0.0;
            if (is_naive) {
                const int src = (k >= 2 && k < 2 + R) ? k + R : ((k >= 2 + R && k < D) ? k - R : k);
                sq_other = __shfl(ssq_l, src);
            }
            if (kl) {
                const float* xold = xring + (i & 7) * 64;
                const float mold = xold[k];
                const float nw = __fadd_rn(__fmul_rn(lr, (float)mus), __fmul_rn(om, mold));
                // LDS copies first: the helpers of the next step read them
                mu32[par * D + k] = nw;
                mu64[par * D + k] = (double)nw;
                double* rc = rec + (par * D + k) * 8;
                rc[0] = Ln0; rc[1] = Ln1; rc[2] = W0; rc[3] = W1;
                rc[4] = Gn0; rc[5] = Gn1; rc[6] = Xn0; rc[7] = Xn1;
                xn[(size_t)i * D + k] = nw;
                const uint64_t gr = ((uint64_t)a.epoch << 32) | (uint64_t)__float_as_uint(nw);
                gran_store_agent(a.hand + ((size_t)tl * n + i) * D + k, gr);
                if (tl == TL - 1 && a.halo_out != nullptr)
                    gran_store_system(a.halo_out + (size_t)i * D + k, gr);
                if (is_naive) {
                    const double p = r00, s = r11;
                    double pd;
                    if (k == 0) pd = p * (double)(n - 1);
                    else if (k == 1) pd = s * (double)(n - 1);
                    else {
                        const double oo = (k < 2 + R) ? (double)xold[k + R] : (double)xold[k - R];
                        pd = ((k < 2 + R) ? p : s) * (sq_other - oo * oo);
                    }
                    pdl[par * D + k] = pd + pcdl[k];
                    const double mo = (double)mold, mn = (double)nw;
                    if (k >= 2) ssq_l = ssq_l - mo * mo + mn * mn;
                }
            }
            Wp0 = W0; Wp1 = W1; Xp0 = Xn0; Xp1 = Xn1; Lp0 = Ln0; Lp1 = Ln1; Gp0 = Gn0; Gp1 = Gn1;
            Mip = Mi;
            Sip = Si;
            STAMP4(5);
            lds_wait_ge(kcnt, 7u * (uint32_t)(i + 1), a.status, dead);
            STAMP4(6);
            const double* Kn = Kbuf + (size_t)ppar * DD;
            if (kl) {
#pragma unroll
                for (int c = 0; c < D; ++c) brow[c] = Kn[(size_t)k * D + c];
            }
            STAMP4(7);
            lds_barrier3();
        }
        {
            const int i = n;
            PROG4();
        }
        lds_barrier3();
    } else {
        // ============================ HELPERS ============================
        // HBK lanes (hw 0..5): entries of the K rebuild; HBC lanes (hw 3..5): entries of
        // the covariance output, stored after the wave's GEMM loads are issued (vmcnt
        // retires in order: stores ahead of those loads would delay the next GEMM part).
        constexpr int NHC = 192, LTQC = (NLT + NHC - 1) / NHC;
        int lk[LTQ], lm[LTQ], ck[LTQC], cm[LTQC];
#pragma unroll
        for (int q = 0; q < LTQ; ++q) {
            const int e = hl + C::NHB * q;
            int k = -1, m = -1;
            if (hl < C::NHB && e < NLT) tri_decode3(e, k, m);
            lk[q] = k;
            lm[q] = m;
        }
#pragma unroll
        for (int q = 0; q < LTQC; ++q) {
            const int e = (tid - 256) + NHC * q;
            int k = -1, m = -1;
            if (hw >= 3 && hw <= 5 && e < NLT) tri_decode3(e, k, m);
            ck[q] = k;
            cm[q] = m;
        }
        // static priority: HF1 (hw 0..2) and HX (hw 6) feed the solver's next step
        if (hw <= 2 || hw == 6) __builtin_amdgcn_s_setprio(2);
        for (int i = 0; i <= n; ++i) {
            STAMP4(0);
            const int par = i & 1, ppar = (i + 1) & 1;
            const double* Bi = Kbuf + (size_t)par * DD;
            double* Kn = Kbuf + (size_t)ppar * DD;
            const double* rp = rec + (size_t)ppar * D * 8;
            // HX (hw 6): dots that do not involve mu_{i-1} (the solver waits for them)
            if (hw == 6 && i < n) {
                const int k = lane;
                const int kc = (k < D) ? k : 0;
                const double msk = (k < D) ? 1.0 : 0.0;
                const double* rc = rec + (ppar * D + kc) * 8;
                const double W0 = msk * rc[2], W1 = msk * rc[3], X0 = msk * rc[6], X1 = msk * rc[7];
                const double g = g64[par * D + kc];
                const double yv0 = vbuf[(par * D + kc) * 4 + 1], yv1 = vbuf[(par * D + kc) * 4 + 2];
                double n0, n1;
                jcol<R>(xring + ((i + 1) & 7) * 64, i + 1 < n, kc, n0, n1);
                const double gA = (k < 2) ? g : 0.0;
                double pr[20];
                pr[0] = W0 * g; pr[1] = W1 * g; pr[2] = X0 * g; pr[3] = X1 * g;
                pr[4] = W0 * n0; pr[5] = W0 * n1; pr[6] = W1 * n0; pr[7] = W1 * n1;
                pr[8] = X0 * n0; pr[9] = X0 * n1; pr[10] = X1 * n0; pr[11] = X1 * n1;
                pr[12] = msk * n0 * yv0; pr[13] = msk * n0 * yv1;
                pr[14] = msk * n1 * yv0; pr[15] = msk * n1 * yv1;
                pr[16] = W0 * gA; pr[17] = W1 * gA; pr[18] = X0 * gA; pr[19] = X1 * gA;
                int idx;
                const double sv = wave_reduce_scatter<20>(pr, lane, idx);
                if (idx < 20) dots[idx] = sv;
                if (lane == 0) lds_signal_set(ddone, (uint32_t)(i + 1));
                STAMP4(1);
            }
            // ring + transposed copy of node i-1's new (U, V)  (hw 4).  The wave's
            // stores of the previous step are drained first (a step old: free), so
            // that Mt store is visible to loads issued after this step's barrier.
            if (hw == 4) {
#ifndef AME_S4_EAGER_DRAIN
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
                if (i >= 1 && lane < M2) {
                    const float vnew = mu32[ppar * D + 2 + lane];
                    mring[((i - 1) & (kMR - 1)) * 64 + lane] = vnew;
                    Mt[(size_t)lane * ns + (i - 1)] = vnew;
                }
            }
            // HBK (hw 0..5): K_i = B_i - L W^T + G X^T  (LDS only)
            if (hw <= 5 && i < n) {
#pragma unroll
                for (int q = 0; q < LTQ; ++q) {
                    if (lk[q] < 0) continue;
                    const int k = lk[q], m = lm[q];
                    const double* rk = rp + k * 8;
                    const double* rm = rp + m * 8;
                    const double c = Bi[k * D + m] - (rk[0] * rm[2] + rk[1] * rm[3]);
                    const double kn = c + (rk[4] * rm[6] + rk[5] * rm[7]);
                    Kn[k * D + m] = kn;
                    Kn[m * D + k] = kn;
                }
            }
            STAMP4(4);
            if (lane == 0) lds_signal_add(kcnt, 1u);
            // HF1 (hw 0..2): hand-off of mu_{i+1,t-1}, AR terms, g_{i+1}
            if (hw <= 2 && i + 1 < n) {
                uint64_t gv = 0;
                if (lane < D) gv = pring[(size_t)((i + 1) & 3) * 128 + lane];
                gran_finish(i + 1, gv, muL + hw * 64);
                STAMP4(2);
                wave_lds_sync3();
                hf1(i + 1);
                STAMP4(3);
                if (hw == 0) jn_fill(i + 2);
                if (lane == 0) lds_signal_add(gcnt, 1u);
            }
            if (i < n) {
                // block GEMM (hw 0..3): this step's part, then the loads of the next
#ifndef AME_S4_ABL_GEMM
                if (hw <= 3) {
#else
                if (false) {
#endif
                    const int bq = i + kGS;
                    if ((bq >> 4) >= 2) gemm_compute(bq >> 4, bq & 15);
                    const int bq1 = bq + 1;
                    if ((bq1 >> 4) >= 2 && i + 1 < n) gemm_load(bq1 >> 4, bq1 & 15);
                }
                // window GEMV of node i+2 (hw 4, 5: one half each)
#ifndef AME_S4_ABL_WIN
                if ((hw == 4 || hw == 5) && i + 2 < n) wgemv(i + 2, hw - 4);
#endif
                STAMP4(5);
                if (hw == 6) {
                    // loader: Y window row i+5, covariance of node i+2, old means of
                    // node i+5 (slice t) and i+4 (slice t+1), granules of node i+4,
                    // old (U, V) of node i+22
                    dma_yw(i + 5);
                    dma_cov(i + 2);
                    dma_x(i + 5);
                    dma_r(i + 4);
                    dma_p(i + 4);
                    dma_m(i + kGL);
                    // block reduction: block (i+2)/16 finished its GEMM last step
                    if (((i + kGS) & 15) == 0) {
                        const int bb = (i + 2) >> 4;
                        if (bb >= 2 && kBS * bb < n) gemm_reduce(bb);
                    }
                    STAMP4(6);
                }
            }
            // HBC (hw 3..5): damped covariance of node i-1,
            // P_{i-1}^-1 = B_i - L_{i-1} W_{i-1}^T  (+ bad mask, jitter; naive: diag)
#ifndef AME_S4_ABL_HBC
            if (hw >= 3 && hw <= 5 && i >= 1) {
#else
            if (false) {
#endif
                const double* pdp = pdl + (size_t)ppar * D;
                const float* co = cring + (size_t)((i + 3) & 3) * LY::cs;   // node i-1
                float* cv = cvw + (size_t)(i - 1) * DD;
#pragma unroll
                for (int q = 0; q < LTQC; ++q) {
                    if (ck[q] < 0) continue;
                    const int k = ck[q], m = cm[q];
                    const double* rk = rp + k * 8;
                    const double* rm = rp + m * 8;
                    const double c = Bi[k * D + m] - (rk[0] * rm[2] + rk[1] * rm[3]);
                    float c32;
                    if (is_naive) {
                        c32 = (k == m) ? 1.0f / ((float)pdp[k] + 1e-8f) : 0.f;
                    } else {
                        c32 = (float)c;
                        if (is_bad && ((k < 2) != (m < 2))) c32 = 0.f;
                        if (k == m) c32 = c32 + 1e-6f;
                    }
                    cv[k * D + m] = __fadd_rn(__fmul_rn(lr, c32), __fmul_rn(om, co[k * D + m]));
                    if (k != m) cv[m * D + k] = __fadd_rn(__fmul_rn(lr, c32), __fmul_rn(om, co[m * D + k]));
                }
            }
            if (i < n && hw >= 3 && i + 1 < n) {
                lds_wait_ge(kcnt, 7u * (uint32_t)(i + 1), a.status, dead);
                lds_wait_ge(gcnt, 3u * (uint32_t)(i + 1), a.status, dead);
                STAMP4(7);
                hf2(i + 1, Kn);
                STAMP4(8);
            }
            if (hw == 6) vm_wait_le(2 * KDMA);
#ifdef AME_S4_EAGER_DRAIN
            if (hw == 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            STAMP4(9);
            lds_barrier3();
        }
    }
    // ---- slice done: release, flag (as v3) ----
    if (a.done != nullptr) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(a.done + tl, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (tl == 0 && a.back_out != nullptr) {
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

// v4 covers r <= 16 (one 16-column MFMA tile per GEMM), n % 4 == 0, 8 <= n <= 2048.
template <int R>
static int sweep4_fits(int n) {
    if (R > 16 || n < 8 || (n & 3) != 0 || n > 64 * 16 * kVM) return 0;
    using C = Cfg4<R>;
    if (2 * (C::NC + 5) > 63) return 0;
    return Lay4<R>::total <= kLDSMAX;
}

template <int R>
static int sweep4_occupancy() {
    const int lds = Lay4<R>::total;
    auto kern = ame_sweep4_kernel<R>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kNT, (size_t)lds) != hipSuccess) return 0;
    return per_cu;
}

int ame_sweep4_supported(int n, int r) {
    switch (r) {
#define X(RR) \
    case RR: if constexpr (RR <= 16) return sweep4_fits<RR>(n); else return 0;
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}

int ame_sweep4_blocks_per_cu(int n, int r) {
    (void)n;
    switch (r) {
#define X(RR) \
    case RR: if constexpr (RR <= 16) return sweep4_occupancy<RR>(); else return 0;
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}

template <int R>
static int launch_sweep4(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    const int lds = Lay4<R>::total;
    auto kern = ame_sweep4_kernel<R>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
        return -2;
    hipLaunchKernelGGL(kern, dim3(dm->T_local), dim3(kNT), (size_t)lds, st, *dm, *a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int ame_sweep4_dispatch(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    switch (dm->r) {
#define X(RR) \
    case RR: if constexpr (RR <= 16) return launch_sweep4<RR>(dm, a, st); else return -1;
        AME_FOR_EACH_R(X)
#undef X
        default: return -1;
    }
}

// the transposed (U, V) copy: [T_local][2r][roundup(n, 16)] fp32, in doubles
long long ame_sweep4_work_doubles(const ame_dims* dm) {
    const long long ns = (dm->n + 15) & ~15;
    return ((long long)dm->T_local * 2 * dm->r * ns + 1) / 2;
}
