// K1: the Gauss-Seidel sweep of TemporalAMEStructuredMFVI / TemporalAMENaiveMFVI
// on gfx950: new means AND new covariances of every (node, time) step.
//
// Reference semantics (Alfieriek/Python-Temporal-AME-SVI):
//   _update_step                structured_mf.py:211-218  (for i in range(n))
//   _update_node_i              structured_mf.py:220-287  (for t in range(T))
//   _compute_observation_terms  structured_mf.py:289-326
//   naive variant               naive_mf.py:207-282 (mu = solve(P,h), C = diag(1/diag P))
// Step (i,t) reads the NEW means of nodes j<i at t and of node i at t-1 and the
// OLD means of nodes j>i at t and of node i at t+1: a 2-D wavefront.
//
// Design:
//  * one workgroup per time slice ("lane" t), all lanes co-resident; lane t-1
//    hands mu_{i,t-1}^new to lane t through {epoch,value} granules;
//  * the lane keeps its slice's (U,V) in LDS for the GEMV h_obs = Z_i . [V|U];
//  * no factorisation per step.  With F_j = J_j^T R^-1 J_j (J_j = [[1,0,V_j,0],
//    [0,1,0,U_j]]) the precision of node i is
//        P_i = P_const(t) + sum_{j != i} F_j(current),
//    so consecutive precisions differ by rank 4.  The lane keeps
//        K_i = (P_i - F_{i-1}(new))^-1                      (fp64, LDS)
//    and per step (Woodbury):
//        W = K J_{i-1}^T, M = R + J_{i-1} W, u = K g   (g = h minus node i-1's part)
//        mu_i = u + W M^-1 (y_{i,i-1} - J_{i-1} u)      (= P_i^-1 h_i)
//        P_i^-1 = K - W M^-1 W^T                         (-> X_cov output)
//        K_{i+1} = P_i^-1 downdated by F_{i+1}(old)      (second rank-2 Woodbury)
//    K_0 = P_0^-1 comes from one in-place sweep-operator inversion per sweep.
//    Lower triangles are computed and mirrored, so K and every covariance are
//    exactly symmetric (the reference's (C+C^T)/2 is an identity).
//  * phases per step (3 workgroup barriers):
//      1 all   : K-matvecs (W, Y' = K J_{i+1}^T, u) ; stage z row of node i+1
//      2 wave 0: reductions, 2x2 solves, mu_i, publish ;
//        waves 1-3: GEMV for node i+1, poll mu_{i+1,t-1}, load mu_{i+1,t+1}
//      3 all   : K rank-4 update + covariance write ; AR terms of node i+1
//  * GEMV workers (MODE 2): when the chip has room, the h_obs
//    GEMV leaves the slice's workgroup.  AME_GW workgroups per slice (other
//    CUs) each own a node range of the slice's (U,V) block in registers and
//    publish, per node m, the partial sum over their range with the nodes
//    m-3..m left out, as {tag, value} granules in a ring.  They use node j's
//    new mean once the slice's own hand-off granules show it (j <= m-4).  The
//    slice's workgroup adds the partials in a fixed order plus nodes m-3, m-2
//    (new means, LDS ring); node m-1 stays the Woodbury observation.
#include "ame_common.h"
#include "ame_sweep_dev.h"

#ifdef AME_STAMPS
// Diagnostic build only (cdna_hip_programming.md §7, in-kernel stamps): lane
// T_local/2 records s_memtime after each phase for nodes
// [AME_STAMP_I0, AME_STAMP_I0 + 16).  Never compiled into the product library.
#define AME_STAMP_I0 256
#define AME_STAMP_NPH 32
__device__ unsigned long long g_ame_stamps[16 * AME_STAMP_NPH];
// s_memrealtime (constant 100 MHz, one clock for the whole device) beside each
// s_memtime stamp: the slice workgroup and its workers run on different CUs,
// often different XCDs, whose s_memtime counters are not comparable
__device__ unsigned long long g_ame_rt[16 * AME_STAMP_NPH];
__device__ unsigned long long g_ame_wrt[16 * 8];
#define STAMP(ph) STAMPW(ph, 0)
#define STAMPW(ph, who)                                                                    \
    do {                                                                                   \
        if (stamp_on && tid == (who)) {                                                    \
            unsigned long long t_, r_;                                                     \
            __builtin_amdgcn_sched_barrier(0);                                             \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory"); \
            __builtin_amdgcn_sched_barrier(0);                                             \
            g_ame_stamps[(i - AME_STAMP_I0) * AME_STAMP_NPH + (ph)] = t_;                  \
            g_ame_rt[(i - AME_STAMP_I0) * AME_STAMP_NPH + (ph)] = r_;                      \
        }                                                                                  \
    } while (0)
// GEMV worker 0 of the middle slice: per node m in [I0+4, I0+20): loop top,
// node m-4 seen, z staged, GEMV done, partial stored
__device__ unsigned long long g_ame_wstamps[16 * 8];
#define WSTAMP(ph)                                                                         \
    do {                                                                                   \
        if (t == TL / 2 && g == 0 && tid == 0 && m >= AME_STAMP_I0 + 4 && m < AME_STAMP_I0 + 20) { \
            unsigned long long t_, r_;                                                     \
            __builtin_amdgcn_sched_barrier(0);                                             \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory"); \
            __builtin_amdgcn_sched_barrier(0);                                             \
            g_ame_wstamps[(m - AME_STAMP_I0 - 4) * 8 + (ph)] = t_;                         \
            g_ame_wrt[(m - AME_STAMP_I0 - 4) * 8 + (ph)] = r_;                             \
        }                                                                                  \
    } while (0)
// phase-2 detail of the middle slice's waves 1-3 (WK): slot = 2 * wave-1 + {0: signalled, 1: reduce+AR done}
__device__ unsigned long long g_ame_p2stamps[16 * 16];
#define P2STAMP(sl)                                                                        \
    do {                                                                                   \
        if (stamp_on && lane == 0) {                                                       \
            unsigned long long t_;                                                         \
            __builtin_amdgcn_sched_barrier(0);                                             \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
            __builtin_amdgcn_sched_barrier(0);                                             \
            g_ame_p2stamps[(i - AME_STAMP_I0) * 16 + (sl)] = t_;                            \
        }                                                                                  \
    } while (0)
extern "C" int ame_debug_read_p2stamps(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ame_p2stamps), sizeof(g_ame_p2stamps), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int ame_debug_read_rt(unsigned long long* main_rt, unsigned long long* worker_rt) {
    if (hipMemcpyFromSymbol(main_rt, HIP_SYMBOL(g_ame_rt), sizeof(g_ame_rt), 0, hipMemcpyDeviceToHost) !=
        hipSuccess)
        return -1;
    return hipMemcpyFromSymbol(worker_rt, HIP_SYMBOL(g_ame_wrt), sizeof(g_ame_wrt), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int ame_debug_read_wstamps(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ame_wstamps), sizeof(g_ame_wstamps), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
// wavefront lag: s_memrealtime at the start of steps AME_STAMP_I0,
// AME_STAMP_I0 + 64 and 0 on thread 0 of every slice (local slice < 64); slots
// 3-5: prologue marks (LAGMARK)
__device__ unsigned long long g_ame_lag[64 * 8];
extern "C" int ame_debug_read_lag(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ame_lag), sizeof(g_ame_lag), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#define LAGMARK(tl_, slot)                                                                 \
    do {                                                                                   \
        if ((tl_) < 64) {                                                                  \
            unsigned long long r_;                                                         \
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory"); \
            g_ame_lag[(tl_) * 8 + (slot)] = r_;                                            \
        }                                                                                  \
    } while (0)
// s_memrealtime at kernel entry of every workgroup (blockIdx < 512), and its
// hardware placement (HW_ID: CU / SE / XCC bits)
__device__ unsigned long long g_ame_entry[512 * 2];
extern "C" int ame_debug_read_entry(unsigned long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ame_entry), sizeof(g_ame_entry), 0,
                               hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int ame_debug_read_stamps(unsigned long long* host, int count) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ame_stamps), sizeof(unsigned long long) * count,
                               0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define LAGMARK(tl_, slot) do { } while (0)
#define WSTAMP(ph) do { } while (0)
#define P2STAMP(sl) do { } while (0)
#define STAMP(ph) \
    do {          \
    } while (0)
#define STAMPW(ph, who) \
    do {                \
    } while (0)
#endif

#define AME_YPF 8   // Y-row prefetch registers per thread (n <= 2048 fully prefetched)
// AME_GW, AME_GW_RING, AME_GW_MAXPW, ame_gw_tag: ame_common.h
#ifndef AME_MG_UNROLL
#define AME_MG_UNROLL 8   // GEMV rows in flight per thread when the slice is read from HBM
#endif

// Workgroup barrier that orders LDS only.  __syncthreads() lowers to a release
// fence that waits vmcnt(0), exposing every in-flight prefetch load and every
// covariance store at each barrier; here global traffic stays in flight across
// phases (loads are waited for by the compiler at their first use; no other
// wave of this workgroup reads what this kernel stores to global memory).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-0 multi-dot: lane L holds p[h][v] of state rows k = L + 64h < D (KH
// rows per lane; KH = 2 only for D > 64); every lane gets all NV sums.  The
// lane's rows are added, then one 64-lane reduce-scatter (permlane swaps +
// DPP, fixed tree: deterministic) leaves sum v on one lane, which writes it
// to LDS for the others.  Only the first NR <= NV sums are formed (the rest of
// out is left alone).  NV <= 64.
template <int NV, int D, int KH, int NR = NV>
__device__ __forceinline__ void wave_multidot(const double (&pv)[KH][NV], double (&out)[NV],
                                              double* red /* unused */, double* sums, int lane) {
    static_assert(NR <= NV, "wave_multidot: NR > NV");
    (void)red;
    double v[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) {
        v[q] = pv[0][q];
#pragma unroll
        for (int h = 1; h < KH; ++h) v[q] += pv[h][q];
    }
    int idx;
    const double s = ame::wave_reduce_scatter<NR>(v, lane, idx);
    if (idx < NR) sums[idx] = s;
    wave_lds_sync();
#pragma unroll
    for (int qq = 0; qq < NR; ++qq) out[qq] = sums[qq];
    wave_lds_sync();
}

struct M22 {
    double a, b, c, d;   // [[a b][c d]]
};
__device__ __forceinline__ M22 inv22(M22 m) {
    const double id = 1.0 / (m.a * m.d - m.b * m.c);
    return {m.d * id, -m.b * id, -m.c * id, m.a * id};
}
// Per-step 2x2 inverses of wave 0's Woodbury chain: the determinant's
// reciprocal from v_rcp_f64 plus two Newton steps (as the v3 solver) -- a
// shorter dependent chain than the IEEE division sequence, full fp64 accuracy
// for these well-scaled determinants
__device__ __forceinline__ M22 inv22_fast(M22 m) {
    const double det = m.a * m.d - m.b * m.c;
    double r = __builtin_amdgcn_rcp(det);
    r = fma(r, fma(-det, r, 1.0), r);
    r = fma(r, fma(-det, r, 1.0), r);
    return {m.d * r, -m.b * r, -m.c * r, m.a * r};
}

// lower-triangle index e -> (k, m), m <= k
__device__ __forceinline__ void tri_decode(int e, int& k, int& m) {
    k = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
    if ((k + 1) * (k + 2) / 2 <= e) ++k;
    if (k * (k + 1) / 2 > e) --k;
    m = e - k * (k + 1) / 2;
}

// AR-term partition of the natural parameter (the sweep's AR threads): thread
// `at` < NPA * D owns row k = at / NPA, part pp = at % NPA, columns
// [pp * MC, pp * MC + MC).  WK runs the AR terms on 192 threads, the others on
// the whole workgroup.
template <int R, bool WK>
struct ArPart {
    static constexpr int D = 2 + 2 * R;
    static constexpr int ART = WK ? 192 : AME_NT;
    static constexpr int NPA = (4 * D <= ART) ? 4 : 2;
    static constexpr int MC = (D + NPA - 1) / NPA;
};

// mreg[sn] = val for a wave-uniform runtime slot index sn: a binary search of
// uniform branches down to a compile-time index (log2(N) scalar compares and
// one write) instead of a select on every slot -- the registers may live in
// AGPRs, where each select costs a read, a cndmask and a write
template <int LO, int HI, int N>
__device__ __forceinline__ void set_slot(float (&mreg)[N], int sn, float val, bool col) {
    if constexpr (HI - LO == 1) {
        if (col) mreg[LO] = val;
        // opaque per leaf: otherwise the leaves' stores merge into one store at a
        // runtime index, which demotes mreg to scratch memory
        asm volatile("" : "+v"(mreg[LO]));
    } else {
        constexpr int MID = (LO + HI) / 2;
        if (sn < MID) set_slot<LO, MID, N>(mreg, sn, val, col);
        else set_slot<MID, HI, N>(mreg, sn, val, col);
    }
}

// Pipelined launch (MODE 3, wait_epoch != 0): every workgroup of slice t -- the
// slice's own and its GEMV workers -- reads the previous sweep's outputs for
// slices t and t+1 (old means, covariances; slice t+1 also reads the hand-off
// granules this sweep overwrites), so it starts only once that sweep flagged
// both done: done[t], done[t+1] (done[T_local] when the next slice group
// follows, AME_SWEEP_FLAG_NEXT_GROUP), or for the rank's last slice the right
// rank's back-channel done word.  Same epoch window as ame_sweep3.hip: a flag
// above wait_epoch cannot be current and sets AME_STATUS_STALE_EPOCH.
// Thread 0 waits (ame_wait_prev_done: the wait rules of include/ame_amd.h);
// `dead` is set on thread 0 when it failed or gave up.
__device__ __forceinline__ void ame_v2_wait_prev(const ame_sweep_args& a, int t, int TL, int tg, bool back_rd,
                                                 int nd /* n * d: the back channel's done word */,
                                                 bool& dead, bool account) {
    if (a.wait_epoch == 0u) return;
    if (threadIdx.x == 0) ame::ame_wait_prev_done(a, t, TL, tg, back_rd, nd, dead, account);
    __syncthreads();
}

// GEMV worker (MODE 2): workgroup TL + t*AME_GW + g owns nodes
// [g*NW, (g+1)*NW) of slice t, NW = ceil(n / AME_GW); wave q holds nodes
// base + q + 4s (s < AME_GW_MAXPW), lane c column c of (U,V), in registers.
// Per node m it publishes (ring slot m % 8, tag = ame_gw_tag(epoch, m))
//   part[c'] = sum_{j in range, j not in [m-3, m]} z_mj . [V | U]_j   (c' < 2r)
//   part[2r + p] = sum z_mj[p]
// with node j's new mean for j <= m-4 (read from the slice's hand-off
// granules, which the slice's workgroup stores when it publishes node j).
template <int R, int MODE>
__device__ __forceinline__ void gemv_worker(const ame_dims& dm, const ame_sweep_args& a, char* smem,
                                            const int t, const int g) {
    constexpr int D = 2 + 2 * R, M2 = 2 * R, PW = M2 + 2;
    // MODE 2: seven workers per slice (kind 22); MODE 3: four (kind 23, pipelined)
    constexpr int NG = ame_v2_nworkers(MODE);
    constexpr int MAXPW = ame_v2_maxpw(MODE);
    const int n = dm.n, TL = dm.T_local;
    const int NW = (n + NG - 1) / NG, base = g * NW;
    const int cnt = max(0, min(n, base + NW) - base);
    const int tid = threadIdx.x, lane = tid & 63, q = tid >> 6;
    const int npw = (cnt > q) ? (cnt - q + 3) / 4 : 0;
    // z of the range; entries past it stay zero, so the GEMV reads every
    // register slot's z unconditionally (loads can be batched)
    constexpr int ZN = 4 * MAXPW;
    float2* zb = (float2*)smem;                                   // [max(NW, ZN)]
    float* red = (float*)(smem + ame_align16(8LL * (NW > ZN ? NW : ZN)));   // [4][PW]
    const float* xo = a.x_old + (size_t)t * n * D;
    const uint64_t* hand = a.hand + (size_t)t * n * D;
    uint64_t* hp = (uint64_t*)a.work + (size_t)(t * NG + g) * AME_GW_RING * PW;
    const int nys = ame_ystride(n);
    const float* ysl = a.Yt + (size_t)t * n * nys * 2;
    const float r00f = (float)a.rinv[0], r01f = (float)a.rinv[1], r10f = (float)a.rinv[2], r11f = (float)a.rinv[3];
    const bool col = lane < M2;
    bool dead = false;
    // set by a wave whose wait failed or gave up: the worker then tags its
    // partials 0, which no slice waits for (include/ame_amd.h wait rules)
    uint32_t* wdead = (uint32_t*)(smem + ame_v2_worker_dead_off(n, R, MODE));
    if (tid == 0) *wdead = 0u;
    __syncthreads();
    // MODE 3, pipelined launch: this worker's inputs (old means of slices t and
    // t+1) are the previous sweep's outputs -- wait for its done flags as the
    // slice's workgroup does (ame_v2_wait_prev)
    const bool back_rd = (MODE == 3) && (a.wait_epoch != 0u) && (t == TL - 1) && (a.back_in != nullptr);
    if constexpr (MODE == 3) {
        ame_v2_wait_prev(a, t, TL, dm.t_begin + t, back_rd, n * D, dead, false);   // the slice accounts
        if (tid == 0 && dead) *wdead = 1u;
    }
    // Right-neighbour AR terms PhiTQi mu_{j,t+1}^old of this worker's nodes, for
    // the slice workgroup's phase 2 (same products, order and zero padding as
    // its in-sweep form): formed here, before partial 0, and released with it --
    // the slice reads them only after it has seen every worker's partial 0 and
    // fenced (see the prologue).  Inputs are old means, fixed for the sweep.
    {
        using P = ArPart<R, true>;
        constexpr int NPA = P::NPA, MC = P::MC, NB = 16;   // NB nodes' means per LDS stage (zb scratch)
        const int Tt = dm.T_total, tg = dm.t_begin + t;
        const bool act = tid < NPA * D;
        const int k = act ? tid / NPA : 0, pp = tid % NPA;
        const size_t DD = (size_t)D * D;
        double c[MC];
#pragma unroll
        for (int mm = 0; mm < MC; ++mm) {
            const int m = pp * MC + mm;
            c[mm] = (m < D) ? a.consts[4 * DD + (size_t)k * D + m] : 0.0;
        }
        float* ms = (float*)zb;
        double* outp = a.work + ame_v2_ring_doubles(&dm, MODE) + ((size_t)t * n + base) * (NPA * D);
        // old means of slice t+1: the next local slice; for the last local slice
        // next_old, or in a pipelined launch the right rank's back channel
        const float* src = (tg >= Tt - 1) ? nullptr
                         : (t < TL - 1) ? a.x_old + ((size_t)(t + 1) * n + base) * D
                         : back_rd      ? a.back_in + (size_t)base * D
                                        : a.next_old + (size_t)base * D;
        for (int j0 = 0; j0 < cnt; j0 += NB) {
            const int nb = min(NB, cnt - j0);
            for (int e = tid; e < nb * D; e += AME_NT) ms[e] = src ? src[(size_t)j0 * D + e] : 0.f;
            __syncthreads();
            if (act) {
                for (int qn = 0; qn < nb; ++qn) {
                    const float* mr = ms + qn * D;
                    double pR[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int mm = 0; mm < MC; ++mm) {
                        const int m = pp * MC + mm;
                        const float x = (m < D) ? mr[m] : 0.f;
                        pR[mm & 3] = fma(c[mm], (double)x, pR[mm & 3]);
                    }
                    outp[(size_t)(j0 + qn) * (NPA * D) + tid] = (pR[0] + pR[1]) + (pR[2] + pR[3]);
                }
            }
            __syncthreads();
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // before any partial store
    }
    // MODE 3 may hold more slots per wave than registers allow: the first NREG in
    // registers, the rest
    // in this workgroup's LDS past zb / red ([wave][slot][lane], conflict-free)
    constexpr int NREG = ame_v2_nreg(MODE), NLD = MAXPW - NREG;
    float* mld = (float*)(smem + ame_align16(8LL * (NW > ZN ? NW : ZN)) + ame_align16(4LL * 4 * PW));
    float mreg[NREG];
#pragma unroll
    for (int s2 = 0; s2 < NREG; ++s2) {
        const int j = base + q + 4 * s2;
        mreg[s2] = (s2 < npw && col) ? xo[(size_t)j * D + 2 + lane] : 0.f;
    }
    for (int sl = 0; sl < NLD; ++sl) {
        const int s2 = NREG + sl, j = base + q + 4 * s2;
        mld[(q * NLD + sl) * 64 + lane] = (s2 < npw && col) ? xo[(size_t)j * D + 2 + lane] : 0.f;
    }
    for (int e = cnt + tid; e < ZN; e += AME_NT) zb[e] = make_float2(0.f, 0.f);
    // Y row of the next node, prefetched into registers one node ahead
    constexpr int YQ = (4 * MAXPW + AME_NT - 1) / AME_NT;
    float2 ypf[YQ];
    auto y_prefetch = [&](int m) {
        const float2* yrow = (const float2*)(ysl + (size_t)(m < n ? m : 0) * nys * 2) + base;
#pragma unroll
        for (int u = 0; u < YQ; ++u) {
            const int e = tid + AME_NT * u;
            ypf[u] = (e < cnt) ? yrow[e] : make_float2(0.f, 0.f);
        }
    };
    y_prefetch(0);
    if (g == 0 && tid == 0) LAGMARK(t, 6);
    for (int m = 0; m < n; ++m) {
        WSTAMP(0);
        // node m-4's new mean replaces its old one (owner wave); every worker
        // waits for it (wave 0 of a non-owner polls one granule), which also
        // keeps it at most 4 nodes ahead of the slice: ring slot m % 8 is free
        const int jn = m - 4;
        const bool own = jn >= base && jn < base + cnt;
        if (jn >= 0 && ((own && ((jn - base) & 3) == q) || (!own && q == 0))) {
            const int sn = own ? (jn - base) >> 2 : -1;
            const bool need = own ? col : lane == 0;
            uint64_t v = 0;
            bool ok = true;
            if (need) {
                v = gran_load_agent(hand + (size_t)jn * D + 2 + lane);
                ok = (uint32_t)(v >> 32) == a.epoch;
            }
            if (!__all(ok) && !dead) {
                AmeSpin w(a.status, false, lane == 0);
                while (true) {
                    __builtin_amdgcn_s_sleep(2);
                    bool stale = false;
                    if (need) {
                        v = gran_load_agent(hand + (size_t)jn * D + 2 + lane);
                        ok = (uint32_t)(v >> 32) == a.epoch;
                        stale = (uint32_t)(v >> 32) > a.epoch;   // no later sweep can have written it yet
                    }
                    const bool st_hit = __any(stale);
                    if (__all(ok) && !st_hit) break;
                    const int r = st_hit ? 3 : w.poll();
                    if (r != 0) {
                        const uint64_t bad = __ballot(!ok);
                        const int fl = bad ? (int)__builtin_ctzll(bad) : 0;
                        const uint32_t obs = (uint32_t)(__shfl(v, fl) >> 32);
                        if (lane == 0 && r >= 2)
                            ame_fail(a.status, r == 3 ? AME_STATUS_STALE_EPOCH : AME_STATUS_SPIN_TIMEOUT,
                                     AME_WAIT_WORKER_GRAN, dm.t_begin + t, (uint32_t)jn, obs, a.epoch, w.waited(),
                                     a.epoch);
#ifdef AME_WDEBUG
                        if (lane == 0)
                            printf("worker t=%d g=%d m=%d jn=%d q=%d: granule epoch %u want %u\n", t, g, m, jn,
                                   q, obs, a.epoch);
#endif
                        if (lane == 0) *wdead = 1u;
                        dead = true;
                        break;
                    }
                }
                w.end();
            }
            const float val = __uint_as_float((uint32_t)v);
            const int snu = __builtin_amdgcn_readfirstlane(sn);   // wave-uniform (owner wave)
            if (snu >= 0 && snu < NREG) set_slot<0, NREG, NREG>(mreg, snu, val, col);
            if (NLD > 0 && snu >= NREG && col) mld[(q * NLD + (snu - NREG)) * 64 + lane] = val;
        }
        WSTAMP(1);
        // z row of node m over the range (nodes m-3..m left out)
#pragma unroll
        for (int u = 0; u < YQ; ++u) {
            const int e = tid + AME_NT * u;
            if (e < cnt) {
                const float2 y = ypf[u];
                const int j = base + e;
                const bool ex = (j >= m - 3) && (j <= m);
                zb[e] = ex ? make_float2(0.f, 0.f)
                           : make_float2(r00f * y.x + r01f * y.y, r10f * y.x + r11f * y.y);
            }
        }
        if (m + 1 < n) y_prefetch(m + 1);
        // LDS-only barriers in this loop: __syncthreads() would also wait for the
        // Y prefetch just issued and for the last partial's store (vmcnt(0)),
        // a full memory round trip per node
        lds_barrier();
        WSTAMP(2);
        // U_c -> h_V (z1), V -> h_U (z0); four independent chains
        float a4[4] = {0.f, 0.f, 0.f, 0.f};
        // register slots as kind 22; MODE 3's LDS-held slots after them, same
        // summation order (a4[slot & 3])
#pragma unroll
        for (int s2 = 0; s2 < NREG; ++s2) {
            const float2 z = zb[q + 4 * s2];
            a4[s2 & 3] = fmaf(lane < R ? z.y : z.x, mreg[s2], a4[s2 & 3]);
        }
        if constexpr (NLD > 0) {
            // only the LDS slots that hold nodes (none below n = 4 * 4 * NREG)
            const int nlv = min(NLD, max(0, npw - NREG));
#pragma unroll 8
            for (int sl = 0; sl < nlv; ++sl) {
                const int s2 = NREG + sl;
                const float2 z = zb[q + 4 * s2];
                a4[s2 & 3] = fmaf(lane < R ? z.y : z.x, mld[(q * NLD + sl) * 64 + lane], a4[s2 & 3]);
            }
        }
        const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        // sum of z over the wave's nodes: lane l takes slots l, l+64, l+128, then a
        // fixed xor tree over the wave
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int u = 0; u < (MAXPW + 63) / 64; ++u) {
            const int s2 = lane + 64 * u;
            if (s2 < MAXPW) {
                const float2 z = zb[q + 4 * s2];
                s0 += z.x;
                s1 += z.y;
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            s0 += __shfl_xor(s0, o);
            s1 += __shfl_xor(s1, o);
        }
        WSTAMP(3);
        if (col) red[q * PW + (lane < R ? R + lane : lane - R)] = acc;
        if (lane == 0) {
            red[q * PW + M2] = s0;
            red[q * PW + M2 + 1] = s1;
        }
        lds_barrier();
        if (tid < PW) {
            const float v = ((red[tid] + red[PW + tid]) + red[2 * PW + tid]) + red[3 * PW + tid];
            const uint32_t tag = (*wdead != 0u) ? 0u : ame_gw_tag(a.epoch, m);
            gran_store_agent(hp + (size_t)(m % AME_GW_RING) * PW + tid,
                             ((uint64_t)tag << 32) | (uint64_t)__float_as_uint(v));
        }
        if (m == 0 && g == 0 && tid == 0) LAGMARK(t, 5);
        WSTAMP(4);
    }
}

// MG = false: the slice's (U,V) block lives in LDS (M).  MG = true: it lives in
// a compact HBM copy (a.work, [T_local][n][2R] fp32, 16-byte aligned rows)
// that wave 0 updates when it publishes a new mean; wave 0 drains its stores
// (vmcnt(0)) before the barrier that precedes the next GEMV, the
// workgroup-scope release of the AMDGPU memory model (one CU, shared vL1D).
// Old values the step itself needs (node i-1 in phase 1, node i in phase 3)
// come from x_old in that mode.
// MODE 0: (U,V) in LDS; MODE 1: in HBM (MG); MODE 2: GEMV workers (no slice
// block in this workgroup at all; old rows of single nodes come from x_old).
// Block -> (slice, role) of a worker launch: role 0 is the slice's own
// workgroup, role 1 + g its GEMV worker g.  MODE 2: the slices' workgroups
// first, then the workers slice by slice.  MODE 3 with T_local % 8 == 0:
// XCD-aware (workgroup b runs on XCD b % 8): each XCD holds T_local / 8
// consecutive slices with all their workers, so hand-off granules and worker
// partials stay in that XCD's L2.
template <int MODE>
__device__ __forceinline__ void v2_block_role(int TL, int& slice, int& role) {
    constexpr int NG = ame_v2_nworkers(MODE);
    const int b = blockIdx.x;
    if (MODE == 3 && (TL & 7) == 0) {
        const int per = TL >> 3, w = b >> 3;
        slice = (b & 7) * per + (w % per);
        role = w / per;
    } else if (b < TL) {
        slice = b;
        role = 0;
    } else {
        const int w = b - TL;
        slice = w / NG;
        role = 1 + (w - slice * NG);
    }
}

// Phase-3 block tiling (AME_PH3_BLOCK): edge PB = ceil(D / 22), so the lower
// triangle of blocks (<= 22 * 23 / 2 = 253) fits the workgroup's 256 threads
#ifndef AME_PH3_BLOCK
#define AME_PH3_BLOCK 1
#endif
template <int D>
struct Ph3 {
    static constexpr int PB = (D + 21) / 22, NBK = (D + PB - 1) / PB, NBT = NBK * (NBK + 1) / 2;
    static_assert(NBT <= AME_NT, "phase-3 blocks exceed the workgroup");
};

// VAR: the factorization (enum ame_variant) as a template parameter for the
// GEMV-worker sweep of config 5 (MODE 2), so each variant's kernel carries only
// its own code (as the v3 sweep, ame_sweep3.hip); -1 = read from dims.variant
template <int R, int MODE, int VAR = -1>
__global__ void __launch_bounds__(AME_NT)
ame_sweep_kernel(ame_dims dm, ame_sweep_args a) {
    // MODE 2: seven GEMV workers per slice (kind 22); MODE 3: four, pipelined (kind 23)
    constexpr bool MG = MODE == 1, WK = MODE >= 2, PIPE = MODE == 3;
    constexpr int NGW = ame_v2_nworkers(MODE);
    constexpr int D = 2 + 2 * R, M2 = 2 * R, KS = D + 1, US = (M2 + 15) / 16;
    constexpr int KH = (D + 63) / 64;   // state rows per solver lane
    constexpr int VEC = (R % 4 == 0) ? 4 : ((R % 2 == 0) ? 2 : 1);
    constexpr int CW = M2 / VEC, GW = 192 / CW, PW = M2 + 2;
    // AR row parts; WK: the AR terms run on waves 1-3 (192 threads) in phase 2
    constexpr int ART = ArPart<R, WK>::ART;
    constexpr int NPA = ArPart<R, WK>::NPA;
    constexpr int MC = ArPart<R, WK>::MC;
    static_assert(D <= 128 && 128 + D <= AME_NT && NPA * D <= ART, "sweep v2: D too large");
    constexpr int NLT = D * (D + 1) / 2, LTQ = (NLT + AME_NT - 1) / AME_NT;
    const int n = dm.n, TL = dm.T_local, Tt = dm.T_total;
    extern __shared__ __attribute__((aligned(16))) char smem[];
#ifdef AME_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 512) {
        unsigned long long r_;
        unsigned int hw_, xcc_;
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory");
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));
        g_ame_entry[blockIdx.x * 2] = r_;
        g_ame_entry[blockIdx.x * 2 + 1] = ((unsigned long long)xcc_ << 32) | hw_;
    }
#endif
    int slice = blockIdx.x, role = 0;
    if constexpr (WK) {
        v2_block_role<MODE>(TL, slice, role);
        if (role > 0) {
            gemv_worker<R, MODE>(dm, a, smem, slice, role - 1);
            return;
        }
    }
    const int tl = slice, tg = dm.t_begin + tl;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const bool is_naive = (VAR >= 0) ? (VAR == AME_NAIVE) : (dm.variant == AME_NAIVE);
    const bool is_bad = (VAR >= 0) ? (VAR == AME_BAD) : (dm.variant == AME_BAD);

    const SweepLds L = sweep_lds_layout(n, R, MODE != 0 ? 1 : 0, WK ? 1 : 0);
    double* K = (double*)(smem + L.oK);          // D x KS
    double* vec = (double*)(smem + L.oVec);      // (5+US) x D  K-matvec results
    double* upd = (double*)(smem + L.oUpd);      // 8 x D       rank-4 update vectors
    double* red = (double*)(smem + L.oRed);      // 16 x D      wave-0 reduction scratch
    double* scal = (double*)(smem + L.oScal);    // 64          sums / y_{i+1,i}
    double* gobs_b = (double*)(smem + L.oG);     // [node&1] {D g_obs, D AR terms}
    auto gob = [&](int node) { return gobs_b + (node & 1) * 2 * D; };
    // WK phase-2 signals: [0] the worker partials of node i+1 are in LDS (waves
    // 2-3), [1] mu_{i+1,t-1} is in LDS (wave 1)
    uint32_t* wsync = (uint32_t*)(scal + 60);
    double* ssq = (double*)(smem + L.oSsq);      // 2R          sum U^2, sum V^2 (naive diag)
    double* pcd = ssq + 2 * R;                   // D           diag of P_const
    float* ndiag = (float*)(pcd + D);            // D           naive: diag of the new covariance
    float* mu_prev = (float*)(smem + L.oF);      // mu_{i-1,t}^new (becomes mu_i in phase 2)
    float* mu_left = mu_prev + D;                // mu_{i+1,t-1}^new
    float* mu_right = mu_prev + 2 * D;           // mu_{i+1,t+1}^old
    float* mu_old = mu_prev + 3 * D;             // mu_{i,t}^old
    float* mu_old_n = mu_prev + 4 * D;           // mu_{i+1,t}^old
    // old means of nodes i-1 .. i+2 (slot j & 3), loaded two steps ahead: the
    // step's single-node reads of old rows never wait on HBM
    float* oring = mu_prev + 5 * D;
    auto orow = [&](int j) -> const float* { return oring + (j & 3) * D + 2; };
    // WK: fp64 copies of mu_{i-1,t}^new and of the old-row ring (phase 1's row dots
    // read doubles: no conversions on the waves that run them)
    double* mu_prev64 = WK ? (double*)(smem + L.oV64) : nullptr;
    double* oring64 = WK ? mu_prev64 + D : nullptr;
    double* mu_left64 = WK ? mu_prev64 + 5 * D : nullptr;   // wave 1's poll, fp64
    double* qlds = WK ? mu_prev64 + 6 * D : nullptr;         // QiPhi [k][part][MCP]
    float* part = (float*)(smem + L.oPart);      // GW x PW   GEMV partials
    float* cst = (float*)(smem + L.oCst);        // D x D     new covariance of node i (phase 3)
    float* cob = (float*)(smem + L.oCob);        // D x D     old covariance of node i (phase 1)
    float2* z = (float2*)(smem + L.oZ);          // n         z row of the next node
    float* mring = (float*)(smem + L.oZ);        // 4 x D     (WK) new means of nodes i & 3
    float* M = (float*)(smem + L.oM);            // n x 2R    (U,V) of the slice (!MG)

    const double p = a.rinv[0], s = a.rinv[3], q = 0.5 * (a.rinv[1] + a.rinv[2]);
    const double r00 = a.rinv[0], r01 = a.rinv[1], r10 = a.rinv[2], r11 = a.rinv[3];
    const float r00f = (float)r00, r01f = (float)r01, r10f = (float)r10, r11f = (float)r11;
    M22 Rm;   // R = R_inv^-1, symmetrised
    {
        Rm = inv22(M22{r00, r01, r10, r11});
        Rm.b = Rm.c = 0.5 * (Rm.b + Rm.c);
    }
    const size_t DD = (size_t)D * D;
    const float* xo = a.x_old + (size_t)tl * n * D;
    float* xn = a.x_new + (size_t)tl * n * D;
    float* cvs = a.cov + (size_t)tl * n * DD;
    float* cvw = (a.cov_new != nullptr ? a.cov_new : a.cov) + (size_t)tl * n * DD;   // damped output
    const int nys = ame_ystride(n);
    const float* ysl = a.Yt + (size_t)tl * n * nys * 2;
    const float lr = a.lr, om = a.one_minus_lr;
    bool dead = false;
    float* Mg = MG ? (float*)a.work + (size_t)tl * n * M2 : nullptr;
    // (U,V) row of node j as the GEMV sees it (new for nodes already published)
    auto mrow = [&](int j) -> const float* {
        if constexpr (MG) return Mg + (size_t)j * M2;
        else if constexpr (WK) return xo + (size_t)j * D + 2;   // only asked for old rows
        else return M + j * M2;
    };
    // OLD (U,V) row of node j
    auto mold = [&](int j) -> const float* {
        if constexpr (MG || WK) return xo + (size_t)j * D + 2;
        else return M + j * M2;
    };

    // set by a wave whose wait failed or gave up; wave 0 then tags its hand-off
    // granules 0 and the slice flags nothing (include/ame_amd.h wait rules)
    uint32_t* wdead = (uint32_t*)(scal + 62);
    // pipelined launch (MODE 3): the previous sweep's slices t, t+1 first
    if constexpr (PIPE)
        ame_v2_wait_prev(a, tl, TL, tg, (a.wait_epoch != 0u) && (tl == TL - 1) && (a.back_in != nullptr), n * D,
                         dead, true);

    // ------------------------------------------------------------------
    // init: slice state, P_0 = P_const + sum_{j != 0} F_j, K_0 = P_0^-1
    // ------------------------------------------------------------------
    if constexpr (!WK) {
        for (int idx = tid; idx < n * M2; idx += AME_NT) {
            const int j = idx / M2, c = idx - j * M2;
            if constexpr (MG) Mg[idx] = xo[(size_t)j * D + 2 + c];
            else M[idx] = xo[(size_t)j * D + 2 + c];
        }
    }
    if (tid < D) pcd[tid] = pconst_entry(a.consts, D, tid, tid, tg, Tt);
    if (tid == 0) {
        wsync[0] = wsync[1] = 0u;
        *wdead = dead ? 1u : 0u;   // thread 0 ran the pipelined wait
    }
    __syncthreads();
    // entry (k, m) of P_0 from its node sum (k >= 2: sum of U/V entries, or of
    // products of two); k < 2 rows are constants times n - 1
    auto p0_entry = [&](int k, int m, double acc) -> double {
        double v;
        if (k < 2) {
            v = ((k == 0 && m == 0) ? p : (k == 1 && m == 1) ? s : q) * (double)(n - 1);
        } else {
            const bool ku = k - 2 < R;
            if (m < 2) {
                v = (ku ? (m == 0 ? p : q) : (m == 0 ? q : s)) * acc;
            } else {
                const bool mu_ = m - 2 < R;
                v = ((ku && mu_) ? p : ((!ku && !mu_) ? s : q)) * acc;
            }
        }
        return v + pconst_entry(a.consts, D, k, m, tg, Tt);
    };
    // the U/V column of row k (k >= 2) that J carries: row U_c has entry V_c, row V_c entry U_c
    auto jcol = [&](int k) { const int ck = k - 2; return ck < R ? R + ck : ck - R; };
    if constexpr (MG || WK) {
        // The old (U,V) rows live in HBM here.  Their Gram matrix, column sums
        // and sums of squares on fp64 MFMA (p0_gram_mfma, ame_sweep_dev.h): the
        // node-by-node loop before it made one dependent round trip per node,
        // ~290 node steps of prologue per launch at config 5's rank shape
        // (profiles/r05_c5_prologue_stamps.txt; 2 200 before round 5's staging).
        // G lands in K's (U, V) block; red is free until the pivot loop.
        double* colsum = red;
        float* x0 = (float*)(red + M2);
        ame::p0_gram_mfma<R, AME_NT / 64>(xo, n, D, K, KS, colsum, x0);
        if (tid < M2) {   // node 0 joins the sums of squares
            const int kq = 2 + (tid >= R ? tid - R : tid + R);   // the row that holds column tid
            const double v = (double)x0[tid];
            ssq[tid] = fma(v, v, K[kq * KS + kq]);
        }
        __syncthreads();
        for (int e = tid; e < NLT; e += AME_NT) {
            int k, m;
            tri_decode(e, k, m);
            const double acc = (k < 2) ? 0.0 : (m < 2) ? colsum[jcol(k)] : K[k * KS + m];
            const double v = p0_entry(k, m, acc);
            K[k * KS + m] = v;
            K[m * KS + k] = v;
        }
    } else {
        if (tid < M2) {   // sum of squares over all nodes: ssq[c<R] = sum U_c^2, ssq[R+c] = sum V_c^2
            double acc = 0.0;
            for (int j = 0; j < n; ++j) {
                const double v = (double)mold(j)[tid];
                acc = fma(v, v, acc);
            }
            ssq[tid] = acc;
        }
        for (int e = tid; e < NLT; e += AME_NT) {
            int k, m;
            tri_decode(e, k, m);
            double acc = 0.0;
            if (k >= 2) {
                const int kc = jcol(k);
                if (m < 2) {
                    for (int j = 1; j < n; ++j) acc += (double)mold(j)[kc];
                } else {
                    const int mc = jcol(m);
                    for (int j = 1; j < n; ++j)
                        acc = fma((double)mold(j)[kc], (double)mold(j)[mc], acc);
                }
            }
            const double v = p0_entry(k, m, acc);
            K[k * KS + m] = v;
            K[m * KS + k] = v;
        }
    }
    if (tid == 0 && tg == 0) LAGMARK(tl, 3);   // slice 0 has no left poll (slot 3)
    __syncthreads();
    for (int pv = 0; pv < D; ++pv) {   // in-place symmetric sweep: K -> -P_0^-1
        if (tid < D) red[tid] = K[pv * KS + tid];
        __syncthreads();
        const double rinv = 1.0 / red[pv];
        for (int e = tid; e < NLT; e += AME_NT) {
            int k, m;
            tri_decode(e, k, m);
            double v;
            if (k == pv && m == pv) v = -rinv;
            else if (k == pv) v = red[m] * rinv;
            else if (m == pv) v = red[k] * rinv;
            else v = K[k * KS + m] - (red[k] * red[m]) * rinv;
            K[k * KS + m] = v;
            K[m * KS + k] = v;
        }
        __syncthreads();
    }
    for (int e = tid; e < D * D; e += AME_NT) {
        const int k = e / D, m = e - k * D;
        K[k * KS + m] = -K[k * KS + m];
    }
    if (tid == 0) LAGMARK(tl, 7);

    const int at = WK ? tid - 64 : tid;   // AR thread index
    // AR rows: thread (k = at / NPA, part = at % NPA); WK reads the PhiTQi half
    // precomputed by the GEMV workers before the sweep loop
    // WK keeps QiPhi in LDS by row part (MCP: MC padded to even, 16-B rows)
    constexpr int MCP = (MC + 1) & ~1;
    double qiphi[WK ? 1 : MC], phitqi[WK ? 1 : MC];
    if constexpr (WK) {
        for (int e = tid; e < D * NPA * MCP; e += AME_NT) {
            const int k = e / (NPA * MCP), r2 = e - k * (NPA * MCP), pp = r2 / MCP, mm = r2 - pp * MCP;
            const int m = pp * MC + mm;
            qlds[e] = (mm < MC && m < D) ? a.consts[3 * DD + (size_t)k * D + m] : 0.0;
        }
        for (int e = tid; e < D; e += AME_NT) mu_left64[e] = 0.0;
    } else {
        const int k = at / NPA, pp = at % NPA;
#pragma unroll
        for (int mm = 0; mm < MC; ++mm) {
            const int m = pp * MC + mm;
            const bool ok = (at >= 0) && (at < NPA * D) && (m < D);
            qiphi[mm] = ok ? a.consts[3 * DD + (size_t)k * D + m] : 0.0;
            phitqi[mm] = ok ? a.consts[4 * DD + (size_t)k * D + m] : 0.0;
        }
    }
    int lk[LTQ], lm[LTQ];   // lower-triangle entries owned for the update / cov write
#pragma unroll
    for (int qq = 0; qq < LTQ; ++qq) {
        const int e = tid + AME_NT * qq;
        int k = -1, m = -1;
        if (e < NLT) tri_decode(e, k, m);
        lk[qq] = k;
        lm[qq] = m;
    }
    // per-entry flags as bits of one register (bit qq): diagonal entry, and an
    // entry off the block diagonal of the bad factorization.  As lane masks the
    // compiler kept them in SGPR pairs, which spill (v_readlane per use)
    uint32_t dflag = 0u, oflag = 0u;
#pragma unroll
    for (int qq = 0; qq < LTQ; ++qq) {
        if (lk[qq] >= 0 && lk[qq] == lm[qq]) dflag |= 1u << qq;
        if (lk[qq] >= 0 && ((lk[qq] < 2) != (lm[qq] < 2))) oflag |= 1u << qq;
    }
    // phase 3 in PB x PB blocks of the lower triangle, one block per thread:
    // a block reads its PB rows of L and PB rows of R once (instead of one L
    // row and one R row per entry: 64 of the 84 bytes an entry read from LDS)
    // (kinds 23 and 24 keep the per-entry form: with the block form their
    // LDS-slot worker code path spilled)
    constexpr bool PH3B = AME_PH3_BLOCK && MODE != 3 && MODE != 4;
    int pkb = -1, pmb = -1;
    if (PH3B && tid < Ph3<D>::NBT) tri_decode(tid, pkb, pmb);

    // ---- helpers ----
    float2 ypf[AME_YPF];
    auto prefetch_y = [&](int node) {   // Y row of `node` -> registers
        const float2* yrow = (const float2*)(ysl + (size_t)node * nys * 2);
#pragma unroll
        for (int r = 0; r < AME_YPF; ++r) {
            const int j = tid + AME_NT * r;
            ypf[r] = (j < n) ? yrow[j] : make_float2(0.f, 0.f);
        }
    };
    auto stage_z = [&](int node, int excl) {   // z row of `node` from ypf (+ tail loads)
        auto put = [&](int j, float2 y) {
            float z0 = r00f * y.x + r01f * y.y;
            float z1 = r10f * y.x + r11f * y.y;
            if (j == excl) {   // y_{node,node-1}: Woodbury observation of the next step
                scal[40] = (double)y.x;
                scal[41] = (double)y.y;
            }
            if (j == node || j == excl) { z0 = 0.f; z1 = 0.f; }
            z[j] = make_float2(z0, z1);
        };
#pragma unroll
        for (int r = 0; r < AME_YPF; ++r) {
            const int j = tid + AME_NT * r;
            if (j < n) put(j, ypf[r]);
        }
        const float2* yrow = (const float2*)(ysl + (size_t)node * nys * 2);
        for (int j = tid + AME_NT * AME_YPF; j < n; j += AME_NT) put(j, yrow[j]);
    };
    auto gemv = [&](int tw) {   // partial h_obs over node group (waves 1-3: tw < 192)
        const int g = tw / CW, cq = tw - g * CW;
        if (g < GW) {
            const int c0 = cq * VEC;
            const bool upart = c0 < R;
            const int mo = upart ? (R + c0) : (c0 - R);
            float acc[VEC];
#pragma unroll
            for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
            float s0 = 0.f, s1 = 0.f;
            // HBM rows (MG): more loads in flight per thread
            constexpr int kUnroll = MG ? AME_MG_UNROLL : 4;
#pragma unroll kUnroll
            for (int j = g; j < n; j += GW) {
                const float2 zz = z[j];
                const float zc = upart ? zz.x : zz.y;
                const float* mr = mrow(j) + mo;
                if constexpr (VEC == 4) {
                    const float4 mv = *(const float4*)mr;
                    acc[0] = fmaf(zc, mv.x, acc[0]);
                    acc[1] = fmaf(zc, mv.y, acc[1]);
                    acc[2] = fmaf(zc, mv.z, acc[2]);
                    acc[3] = fmaf(zc, mv.w, acc[3]);
                } else if constexpr (VEC == 2) {
                    const float2 mv = *(const float2*)mr;
                    acc[0] = fmaf(zc, mv.x, acc[0]);
                    acc[1] = fmaf(zc, mv.y, acc[1]);
                } else {
                    acc[0] = fmaf(zc, mr[0], acc[0]);
                }
                s0 += zz.x;
                s1 += zz.y;
            }
#pragma unroll
            for (int v = 0; v < VEC; ++v) part[g * PW + c0 + v] = acc[v];
            if (cq == 0) {
                part[g * PW + M2] = s0;
                part[g * PW + M2 + 1] = s1;
            }
        }
    };
    auto gemv_reduce = [&](int node) {   // threads < PW -> g_obs of node
        // WK: wave 3 (few AR items, gathers early) takes rt < 64, wave 1's first
        // lanes the rest (rt 64, 65 at d = 66); wave 2 gathers and runs 64 AR items
        const int rt = WK ? (tid >= 192 ? tid - 192 : ((tid >= 64 && tid < 64 + PW - 64) ? tid : -1)) : tid;
        if (rt >= 0 && rt < PW) {
            float acc = 0.f;
            for (int g = 0; g < (WK ? NGW + 1 : GW); ++g) acc += part[g * PW + rt];
            gob(node)[(rt < M2) ? 2 + rt : rt - M2] = (double)acc;
        }
    };
    // WK, waves 2-3 (wave 1 polls the left slice meanwhile; a load queued
    // behind that poll would wait for it): h_obs partials of `node` from the
    // workers (fixed order),
    // plus row AME_GW = nodes node-3, node-2 (new means, LDS ring), and the raw
    // y_{node,node-1} for the Woodbury observation of the next step
    // every load issued before any is checked: each is a cross-CU round trip.
    // gather_issue(node) runs a phase ahead of gather(node) (phase 1 of the same
    // step; the prologue for node 0): the workers publish partial m as soon as
    // node m-4 is known, so the partials of node i+1 are normally in L2 by then
    // and phase 2 mostly checks tags.  Every gather(node) must follow a
    // gather_issue(node): the entries past the partials are pre-tagged there.
    constexpr int GNE = NGW * PW, GGE = (GNE + 127) / 128;
    uint64_t gv[GGE];
    // raw y_{node,node-3}, y_{node,node-2} (threads ht < PW) and y_{node,node-1}
    // (ht == 0), loaded with the partials: in phase 2 they were HBM round trips
    // on the waves that signal the partials
    float2 gy[3];
    // per-thread ring offsets of the partial entries this thread gathers (fixed
    // for the sweep); entries past the GNE real ones load entry 0 and are
    // pre-tagged after the load (no branch, no per-step division)
    int goff[GGE];
    uint32_t gvalid = 0u;
#pragma unroll
    for (int u = 0; u < GGE; ++u) {
        const int e = max(tid - 128, 0) + 128 * u, g = e / PW, c = e - g * PW;
        goff[u] = (e < GNE) ? g * AME_GW_RING * PW + c : 0;
        if (e < GNE) gvalid |= 1u << u;
    }
    auto gather_issue = [&](int node) {
        const int ht = tid - 128;
        if (ht < 0) return;
        if (ht < PW) {
            // y_{node, node-3+q}, column clamped to >= 0 (gather ignores j < 0).
            // Raw loads only: a select on a loaded value here would wait for it
            const float2* yr = (const float2*)(ysl + (size_t)node * nys * 2);
#pragma unroll
            for (int q = 0; q < 3; ++q) gy[q] = yr[max(node - 3 + q, 0)];
        }
        const uint64_t* hs = (const uint64_t*)a.work + ((size_t)tl * NGW * AME_GW_RING + (node % AME_GW_RING)) * PW;
#pragma unroll
        for (int u = 0; u < GGE; ++u) gv[u] = gran_load_agent(hs + goff[u]);
    };
    auto gather = [&](int node) {
        const int ht = tid - 128;
        if (ht < 0) return;
        const uint32_t want = ame_gw_tag(a.epoch, node);
        const uint64_t* hp = (const uint64_t*)a.work + (size_t)tl * NGW * AME_GW_RING * PW;
        constexpr int NE = GNE, GE = GGE;
        const uint64_t* hs = hp + (size_t)(node % AME_GW_RING) * PW;
        uint64_t (&v)[GE] = gv;   // issued by gather_issue(node)
        bool ok = true;
#pragma unroll
        for (int u = 0; u < GE; ++u) ok = ok && (!((gvalid >> u) & 1u) || (uint32_t)(v[u] >> 32) == want);
        if (!ok && !dead) {
            // per thread (each holds its own partial words); every thread that
            // gives up reports (ame_fail keeps the first record)
            AmeSpin w(a.status, false, true);
            while (true) {
                __builtin_amdgcn_s_sleep(1);
                ok = true;
                uint32_t obs = want;
#pragma unroll
                for (int u = 0; u < GE; ++u) {
                    if (((gvalid >> u) & 1u) && (uint32_t)(v[u] >> 32) != want) {
                        v[u] = gran_load_agent(hs + goff[u]);
                        ok = ok && (uint32_t)(v[u] >> 32) == want;
                        if ((uint32_t)(v[u] >> 32) != want) obs = (uint32_t)(v[u] >> 32);
                    }
                }
                if (ok) break;
                const int r = w.poll();
                if (r != 0) {
                    if (r == 2)
                        ame_fail(a.status, AME_STATUS_SPIN_TIMEOUT, AME_WAIT_PARTIAL, tg, (uint32_t)node, obs, want,
                                 w.waited(), a.epoch);
#ifdef AME_WDEBUG
                    printf("main tl=%d node=%d: partial tags stale (want %x)\n", tl, node, want);
#endif
                    *wdead = 1u;
                    dead = true;
                    break;
                }
            }
            w.end();
        }
#pragma unroll
        for (int u = 0; u < GE; ++u) {
            const int e = ht + 128 * u;
            if (e < NE) part[e] = __uint_as_float((uint32_t)v[u]);   // part[g][c], stride PW
        }
        if (ht < PW) {
            float acc = 0.f;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int j = node - 3 + q;
                if (j < 0) continue;
                const float2 y = gy[q];
                // products rounded, then added: the compiler's contraction choice
                // for a*b + c*d otherwise moves with the surrounding code
                const float z0 = mul_add_rn(r00f, y.x, r01f, y.y);
                const float z1 = mul_add_rn(r10f, y.x, r11f, y.y);
                const float* mj = mring + (j & 3) * D;
                if (ht < R) acc = fmaf(z0, mj[2 + R + ht], acc);          // h_U += z0 V
                else if (ht < M2) acc = fmaf(z1, mj[2 + ht - R], acc);    // h_V += z1 U
                else acc += (ht == M2) ? z0 : z1;
            }
            part[NGW * PW + ht] = acc;
        }
        if (ht == 0 && node >= 1) {   // j = node - 1 >= 0
            scal[40] = (double)gy[2].x;
            scal[41] = (double)gy[2].y;
        }
    };
    // WK: the PhiTQi mu_right half of node `node`, precomputed before the sweep
    // (by the GEMV workers; the work buffer past the partial ring); the QiPhi
    // mu_left half once wave 1 has polled mu_left
    const double* arr = WK ? a.work + ame_v2_ring_doubles(&dm, MODE) + (size_t)tl * n * (NPA * D) : nullptr;
    auto ar_right_load = [&](int node) -> double {
        return (at >= 0 && at < NPA * D && node < n) ? arr[(size_t)node * (NPA * D) + at] : 0.0;
    };
    auto ar_left_finish = [&](int node, double aR) {
        if (at >= 0 && at < NPA * D) {
            const int k = at / NPA, pp = at % NPA;
            // WK: coefficients and mu_left from LDS (fp64), every read first
            const double* qr = qlds + (size_t)at * MCP;
            double cq[MC], ml[MC];
#pragma unroll
            for (int mm = 0; mm < MC; ++mm) {
                const int m = pp * MC + mm;
                cq[mm] = qr[mm];
                ml[mm] = mu_left64[m < D ? m : D - 1];
            }
            __builtin_amdgcn_sched_barrier(0);
            double pL[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int mm = 0; mm < MC; ++mm) {
                const int m = pp * MC + mm;
                pL[mm & 3] = fma(cq[mm], (m < D) ? ml[mm] : 0.0, pL[mm & 3]);
            }
            const double aL = (pL[0] + pL[1]) + (pL[2] + pL[3]);
            double acc = ((tg > 0) ? aL : 0.0) + ((tg < Tt - 1) ? aR : 0.0);
            acc = ame::group_sum<NPA>(acc);
            if (pp == 0) gob(node)[D + k] = acc;
        }
    };
    auto ar_terms = [&](int node) {   // AR threads < NPA*D: QiPhi mu_left + PhiTQi mu_right
        if constexpr (WK) return;
        else if (at >= 0 && at < NPA * D) {
            const int k = at / NPA, pp = at % NPA;
            // all LDS reads first, then two independent FMA chains
            float ml[MC], mr[MC];
#pragma unroll
            for (int mm = 0; mm < MC; ++mm) {
                const int m = pp * MC + mm;
                ml[mm] = (m < D) ? mu_left[m] : 0.f;
                mr[mm] = (m < D) ? mu_right[m] : 0.f;
            }
            double pL[4] = {0.0, 0.0, 0.0, 0.0}, pR[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int mm = 0; mm < MC; ++mm) {
                pL[mm & 3] = fma(qiphi[mm], (double)ml[mm], pL[mm & 3]);
                pR[mm & 3] = fma(phitqi[mm], (double)mr[mm], pR[mm & 3]);
            }
            const double aL = (pL[0] + pL[1]) + (pL[2] + pL[3]);
            const double aR = (pR[0] + pR[1]) + (pR[2] + pR[3]);
            double acc = ((tg > 0) ? aL : 0.0) + ((tg < Tt - 1) ? aR : 0.0);
            acc = ame::group_sum<NPA>(acc);
            if (pp == 0) gob(node)[D + k] = acc;
        }
    };
    // wave 1: wait for the granules of mu_{node,t-1}^new (returns when done or timed out);
    // lane L owns state rows L + 64h
    auto poll_left = [&](int node, const uint64_t (&first)[KH]) {
        // halo_in: the left rank's peer buffer, or (AME_SWEEP_FLAG_PREV_GROUP) the
        // previous slice group's granules on this GPU -- then a local wait
        const bool from_halo = (tl == 0) && !(a.flags & AME_SWEEP_FLAG_PREV_GROUP);
        const uint64_t* src = (tl == 0) ? a.halo_in + (size_t)node * D
                                        : a.hand + ((size_t)(tl - 1) * n + node) * D;
        uint64_t v[KH];
        bool ok = true;
#pragma unroll
        for (int h = 0; h < KH; ++h) {
            v[h] = first[h];
            if (lane + 64 * h < D) ok = ok && (uint32_t)(v[h] >> 32) == a.epoch;
        }
        if (!__all(ok) && !dead) {
            AmeSpin w(a.status, from_halo, lane == 0, AME_ST_HALO_US);
            while (true) {
                __builtin_amdgcn_s_sleep(2);
                ok = true;
                bool stale = false;
                uint32_t obs = a.epoch;
#pragma unroll
                for (int h = 0; h < KH; ++h) {
                    const int k = lane + 64 * h;
                    if (k < D) {
                        v[h] = from_halo ? gran_load_system(src + k) : gran_load_agent(src + k);
                        ok = ok && (uint32_t)(v[h] >> 32) == a.epoch;
                        stale = stale || (uint32_t)(v[h] >> 32) > a.epoch;   // see ame_sweep3.hip gran_finish
                        if ((uint32_t)(v[h] >> 32) != a.epoch) obs = (uint32_t)(v[h] >> 32);
                    }
                }
                const bool st_hit = __any(stale);
                if (__all(ok) && !st_hit) break;
                const int r = st_hit ? 3 : w.poll();
                if (r != 0) {
                    const uint64_t bad = __ballot(!ok);
                    const uint32_t o1 = __shfl(obs, bad ? (int)__builtin_ctzll(bad) : 0);
                    if (lane == 0 && r >= 2)
                        ame_fail(a.status,
                                 r == 3 ? AME_STATUS_STALE_EPOCH
                                        : (from_halo ? AME_STATUS_HALO_TIMEOUT : AME_STATUS_SPIN_TIMEOUT),
                                 from_halo ? AME_WAIT_GRAN_HALO : AME_WAIT_GRAN_LOCAL, tg, (uint32_t)node, o1,
                                 a.epoch, w.waited(), a.epoch);
                    if (lane == 0) *wdead = 1u;
                    dead = true;
                    break;
                }
            }
            w.end();
        }
#pragma unroll
        for (int h = 0; h < KH; ++h)
            if (lane + 64 * h < D) {
                mu_left[lane + 64 * h] = __uint_as_float((uint32_t)v[h]);
                if constexpr (WK) mu_left64[lane + 64 * h] = (double)__uint_as_float((uint32_t)v[h]);
            }
    };
    auto first_poll = [&](int node, uint64_t (&g)[KH]) {   // wave 1: issue the first granule loads
        const bool from_halo = (tl == 0) && !(a.flags & AME_SWEEP_FLAG_PREV_GROUP);
        const uint64_t* src = (tl == 0) ? a.halo_in + (size_t)node * D
                                        : a.hand + ((size_t)(tl - 1) * n + node) * D;
#pragma unroll
        for (int h = 0; h < KH; ++h) {
            const int k = lane + 64 * h;
            g[h] = 0;
            if (tg > 0 && k < D) g[h] = from_halo ? gran_load_system(src + k) : gran_load_agent(src + k);
        }
    };
    auto zero_left = [&]() {   // wave 1, global slice 0: no left neighbour
#pragma unroll
        for (int h = 0; h < KH; ++h)
            if (lane + 64 * h < D) {
                mu_left[lane + 64 * h] = 0.f;
                if constexpr (WK) mu_left64[lane + 64 * h] = 0.0;
            }
    };
    auto right_regs = [&](int node, float& nx, float& ol) {   // threads 128..128+D
        const int k = tid - 128;
        nx = 0.f;
        // WK: the right AR terms come precomputed from the workers (mu_right is
        // not read; next_old may be absent in a pipelined launch)
        if (tg < Tt - 1 && !WK)
            nx = (tl < TL - 1) ? a.x_old[((size_t)(tl + 1) * n + node) * D + k]
                               : a.next_old[(size_t)node * D + k];
        ol = xo[(size_t)node * D + k];
    };

    // Covariances move as whole 16-B rows: the old one of node i+1 is loaded
    // into registers during step i and parked in LDS at step i+1; the new one of
    // node i is staged in LDS by phase 3 and stored during step i+1.
    constexpr int NC4 = D * D / 4;                          // D is even
    constexpr int CQ = (NC4 + AME_NT - 1) / AME_NT;
    float4 cpf[CQ];
    // rounds u < CF cover every thread (tid < AME_NT): only the last is masked.
    // The flush reads every row from LDS before its first store (one round trip).
    constexpr int CF = NC4 / AME_NT;
    auto cov_prefetch = [&](int node) {
        const float4* src = (const float4*)(cvs + (size_t)(node < n ? node : 0) * DD);
#pragma unroll
        for (int u = 0; u < CQ; ++u) {
            const int e = tid + AME_NT * u;
            cpf[u] = (u < CF || e < NC4) ? src[e] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto cov_park = [&]() {
#pragma unroll
        for (int u = 0; u < CQ; ++u) {
            const int e = tid + AME_NT * u;
            if (u < CF || e < NC4) ((float4*)cob)[e] = cpf[u];
        }
    };
    auto cov_flush = [&](int node) {
        float4* dst = (float4*)(cvw + (size_t)node * DD);
        float4 rows[CQ];
#pragma unroll
        for (int u = 0; u < CQ; ++u) {
            const int e = min(tid + AME_NT * u, NC4 - 1);
            rows[u] = ((const float4*)cst)[e];
        }
#pragma unroll
        for (int u = 0; u < CQ; ++u) {
            const int e = tid + AME_NT * u;
            if (u < CF || e < NC4) dst[e] = rows[u];
        }
    };
    cov_prefetch(0);

    // ---- prologue: vectors, g_obs and AR of node 0 ----
    if constexpr (!WK) prefetch_y(0);
    {
        float nx = 0.f, ol = 0.f;
        if (tid >= 128 && tid < 128 + D) right_regs(0, nx, ol);
        if constexpr (!WK) stage_z(0, -1);
        if (wave == 1) {
            if (tg > 0) {
                uint64_t g0[KH];
                first_poll(0, g0);
                poll_left(0, g0);
                if (lane == 0) LAGMARK(tl, 3);
            } else {
                zero_left();
            }
        }
        if (tid >= 128 && tid < 128 + D) {
            mu_right[tid - 128] = nx;
            mu_old[tid - 128] = ol;
        }
        for (int e = tid; e < 2 * D; e += AME_NT) {
            const int j = e / D, k = e - j * D;
            oring[j * D + k] = (j < n) ? xo[(size_t)j * D + k] : 0.f;
            if constexpr (WK) oring64[j * D + k] = (double)oring[j * D + k];
        }
    }
    if (!WK && n > 1) prefetch_y(1);
    __syncthreads();
    if (wave >= 1) {
        if constexpr (WK) {   // waves 2-3
            gather_issue(0);
            gather(0);
        }
        else gemv(tid - 64);
    }
    __syncthreads();
    // WK: every worker stored its nodes' right AR terms before its partial 0,
    // which the gather above has seen: acquire them for the whole workgroup
    if constexpr (WK) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    gemv_reduce(0);
    if (tid == 0) LAGMARK(tl, 4);
    if constexpr (WK) ar_left_finish(0, ar_right_load(0));
    else ar_terms(0);
    __syncthreads();
    // WK: the natural parameter's two parts (h_obs, AR terms) summed once into
    // gob(node)[k] (the K-matvec items of phase 1 read one value instead of two)
    if (WK && tid < D) gob(0)[tid] += gob(0)[D + tid];
    if constexpr (WK) __syncthreads();

    float y_prev0 = 0.f, y_prev1 = 0.f;   // y_{i,i-1} (raw)
    for (int i = 0; i < n; ++i) {
#ifdef AME_STAMPS
        const bool stamp_on = (tl == TL / 2) && i >= AME_STAMP_I0 && i < AME_STAMP_I0 + 16;
        if (tid == 0 && tl < 64 && (i == AME_STAMP_I0 || i == AME_STAMP_I0 + 64 || i == 0)) {
            unsigned long long r_;
            asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(r_)::"memory");
            g_ame_lag[tl * 8 + (i == 0 ? 2 : (i != AME_STAMP_I0))] = r_;
        }
#endif
        STAMP(0);
        const bool has_prev = i > 0, has_next = i + 1 < n;
        // park first: waiting for last step's prefetch must not also wait for
        // this step's flush stores (vmcnt counts both, in order)
        cov_park();                      // old covariance of node i -> cob
        STAMPW(16, 0);
        if (i >= 1) cov_flush(i - 1);   // staged by phase 3 of step i-1
        if (i + 1 < n) cov_prefetch(i + 1);
        STAMPW(17, 0);
        // ---------------- phase 1 ----------------
        // WK: node i+1's partials, Y entries and precomputed right AR term (read
        // in phase 2) and node i+2's old row (parked in the old-row ring at the
        // end of phase 3) load now; node i's old mean is read from that ring
        float o21 = 0.f;
        double aR1 = 0.0;
        if constexpr (WK) {
            if (has_next) gather_issue(i + 1);
            if (has_next) aR1 = ar_right_load(i + 1);
            if (has_next && tid >= 128 && tid < 128 + D && i + 2 < n) o21 = xo[(size_t)(i + 2) * D + (tid - 128)];
        }
        STAMPW(20, 128);
        if (has_prev && tid < M2) {   // node i-1: statistics and slice (U,V) <- new
            const double vo = (double)orow(i - 1)[tid], vn = (double)mu_prev[2 + tid];
            ssq[tid] = ssq[tid] - vo * vo + vn * vn;
            if constexpr (MODE == 0) M[(i - 1) * M2 + tid] = mu_prev[2 + tid];
        }
        {
            // one item per (row k, vector); independent partial sums so a
            // wave's dependent FMA chain is short (one wave per SIMD here)
            // items: W/Y (one per (row k, vector), R FMAs), u chunks (16 FMAs),
            // u a-part (2 FMAs).  Independent partial sums keep a wave's
            // dependent FMA chain short (one wave per SIMD here).
            auto wy_item = [&](int it) -> double {
                const int k = it >> 2, qv = it & 3;
                const bool prevv = qv < 2;
                if (!(prevv ? has_prev : has_next)) return 0.0;
                const bool row0 = (qv & 1) == 0;   // e0 = [1,0,V,0] ; e1 = [0,1,0,U]
                const float* src = prevv ? (mu_prev + 2) : orow(i + 1);
                const int cb = row0 ? 2 : 2 + R;
                const float* vv = row0 ? (src + R) : src;
                const double* kr = K + k * KS + cb;
                double p4[4] = {K[k * KS + (row0 ? 0 : 1)], 0.0, 0.0, 0.0};
                if constexpr (R % 2 == 0) {
                    // the node vector as 8-byte pairs (it starts 8-byte aligned when
                    // r is even): half the LDS read instructions, same sums.  Every
                    // read is issued before the arithmetic: left to the scheduler,
                    // each pair of reads waited for a full LDS round trip (one wave
                    // per SIMD here, so nothing else hides it)
                    const float2* v2 = (const float2*)vv;
                    float2 t[R / 2];
                    double kv[R];
#pragma unroll
                    for (int c2 = 0; c2 < R / 2; ++c2) t[c2] = v2[c2];
#pragma unroll
                    for (int c = 0; c < R; ++c) kv[c] = kr[c];
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int c2 = 0; c2 < R / 2; ++c2) {
                        p4[(2 * c2) & 3] = fma(kv[2 * c2], (double)t[c2].x, p4[(2 * c2) & 3]);
                        p4[(2 * c2 + 1) & 3] = fma(kv[2 * c2 + 1], (double)t[c2].y, p4[(2 * c2 + 1) & 3]);
                    }
                } else {
#pragma unroll
                    for (int c = 0; c < R; ++c) p4[c & 3] = fma(kr[c], (double)vv[c], p4[c & 3]);
                }
                return (p4[0] + p4[1]) + (p4[2] + p4[3]);
            };
            auto chunk = [&](int r2) -> double {   // u, (U,V)-part chunk r2 = ch * D + k
                const int ch = r2 / D, k = r2 - ch * D;
                const int m0 = 2 + ch * 16;
                const double* gi = gob(i);
                double p2[2] = {0.0, 0.0};
                double kv[16], gv2[16];   // reads first (see wy_item)
#pragma unroll
                for (int mm = 0; mm < 16; ++mm) {
                    const int m = min(m0 + mm, D - 1);
                    kv[mm] = K[k * KS + m];
                    gv2[mm] = WK ? gi[m] : gi[m] + gi[D + m];
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int mm = 0; mm < 16; ++mm) {
                    const int m = m0 + mm;
                    if (m < D) p2[mm & 1] = fma(kv[mm], gv2[mm], p2[mm & 1]);
                }
                return p2[0] + p2[1];
            };
            auto apart = [&](int k) -> double {   // u, a-part
                const double* gi = gob(i);
                if constexpr (WK) return K[k * KS + 0] * gi[0] + K[k * KS + 1] * gi[1];
                return K[k * KS + 0] * (gi[0] + gi[D]) + K[k * KS + 1] * (gi[1] + gi[D + 1]);
            };
            if constexpr (WK) {
                // One pass over K per step (round 4): the W/Y items and u chunks
                // read rows of K once per vector; here thread (k, h) takes row
                // k >= 2, columns 2 + hR .. 2 + hR + R (the V half for h = 0, the
                // U half for h = 1) and forms all three dots over them -- J0 / J1
                // of node i-1 (W), of node i+1 (Y) and g (u) -- from fp64 copies
                // of the vectors; rows 0 and 1 take one column per lane on waves
                // 2 and 3 with a wave reduce-scatter.  Every read before the
                // arithmetic.
                const double* gi = gob(i);
                const double* on64 = oring64 + ((i + 1) & 3) * D;   // node i+1, old (slot valid for any i)
                // waves 0-1: lane l of wave w takes row 2 + 32 w + (l & 31), half
                // h = l >> 5.  The halves of a row sit 2R dwords apart, on the same
                // LDS banks, so they go to different 32-lane groups; within a group
                // the 32 rows (stride KS = D + 1 doubles) cover all 64 banks
                const int kk = 32 * wave + (lane & 31);
                if (wave < 2 && kk < M2) {
                    const int k = 2 + kk, h = lane >> 5;
                    const double* kr = K + k * KS + 2 + h * R;
                    const double* pj = mu_prev64 + 2 + (h ? 0 : R);   // J0: V (at 2+R), J1: U (at 2)
                    const double* nj = on64 + 2 + (h ? 0 : R);
                    const double* gg = gi + 2 + h * R;
                    // the row part first (R reads), then the vectors in blocks of 8
                    // columns, each block's reads before its arithmetic (register
                    // budget: all four R-vectors at once would spill)
                    double kv[R];
#pragma unroll
                    for (int c = 0; c < R; ++c) kv[c] = kr[c];
                    const double kb = K[k * KS + h], k0 = K[k * KS], k1 = K[k * KS + 1];
                    double w[4] = {0.0, 0.0, 0.0, 0.0}, y[4] = {0.0, 0.0, 0.0, 0.0}, u[4] = {0.0, 0.0, 0.0, 0.0};
                    constexpr int CB = 8;
#pragma unroll
                    for (int c0 = 0; c0 < R; c0 += CB) {
                        double pv[CB], nv[CB], gv[CB];
#pragma unroll
                        for (int b = 0; b < CB; ++b) {
                            const int c = c0 + b < R ? c0 + b : R - 1;
                            pv[b] = pj[c];
                            nv[b] = nj[c];
                            gv[b] = gg[c];
                        }
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int b = 0; b < CB; ++b) {
                            const int c = c0 + b;
                            if (c < R) {
                                w[c & 3] = fma(kv[c], pv[b], w[c & 3]);
                                y[c & 3] = fma(kv[c], nv[b], y[c & 3]);
                                u[c & 3] = fma(kv[c], gv[b], u[c & 3]);
                            }
                        }
                    }
                    const double W = kb + ((w[0] + w[1]) + (w[2] + w[3]));
                    const double Y = kb + ((y[0] + y[1]) + (y[2] + y[3]));
                    const double uh = (u[0] + u[1]) + (u[2] + u[3]);
                    const double U = ame::pair_step<0>(uh, uh, false);   // + the other half (lane l ^ 32)
                    vec[h * D + k] = has_prev ? W : 0.0;
                    vec[(2 + h) * D + k] = has_next ? Y : 0.0;
                    if (h == 0) {
                        vec[4 * D + k] = k0 * gi[0] + k1 * gi[1];
                        vec[5 * D + k] = U;
                    }
                } else if (wave >= 2) {
                    // rows 0 (wave 2) and 1 (wave 3): lane c takes column 2 + c
                    const int r = (tid >= 192) ? 1 : 0, c = lane;
                    const bool in = c < M2, hv = c >= R;   // hv: U half (J1)
                    const int cm = in ? c : 0;
                    const int src = 2 + (hv ? cm - R : cm + R);
                    const double kv = in ? K[r * KS + 2 + cm] : 0.0;
                    const double pv = in ? mu_prev64[src] : 0.0;
                    const double nv = in ? on64[src] : 0.0;
                    const double gv = in ? gi[2 + cm] : 0.0;
                    double v5[5] = {hv ? 0.0 : kv * pv, hv ? kv * pv : 0.0, hv ? 0.0 : kv * nv, hv ? kv * nv : 0.0,
                                    kv * gv};
                    int idx;
                    const double sv = ame::wave_reduce_scatter<5>(v5, lane, idx);
                    if (idx < 5) {
                        const double kb0 = K[r * KS], kb1 = K[r * KS + 1];
                        if (idx == 0) vec[r] = has_prev ? kb0 + sv : 0.0;
                        else if (idx == 1) vec[D + r] = has_prev ? kb1 + sv : 0.0;
                        else if (idx == 2) vec[2 * D + r] = has_next ? kb0 + sv : 0.0;
                        else if (idx == 3) vec[3 * D + r] = has_next ? kb1 + sv : 0.0;
                        else {
                            vec[5 * D + r] = sv;
                            vec[4 * D + r] = kb0 * gi[0] + kb1 * gi[1];
                        }
                    }
                }
            } else if constexpr (R == 32 && AME_NT == 256) {
                // d = 66: 264 W/Y items, 264 chunks, 66 a-parts.  Every round is
                // one item type per wave (divergent item types in one wave run
                // back to back): W/Y 0..255, chunks 0..255, then wave 0 splits
                // the 8 W/Y items of rows 64, 65 into 8 column parts each, wave 1
                // takes chunks 256..263, waves 2-3 the a-parts.
                vec[(tid & 3) * D + (tid >> 2)] = wy_item(tid);
                STAMPW(18, 0);
                STAMPW(21, 128);
                {
                    const int ch = tid / D;
                    vec[(5 + ch) * D + (tid - ch * D)] = chunk(tid);
                }
                STAMPW(19, 0);
                STAMPW(22, 128);
                if (wave == 0) {
                    const int it = 256 + (lane >> 3), pp = lane & 7;
                    double v = 0.0;
                    {   // columns [4 pp, 4 pp + 4) of W/Y item `it`
                        const int k = it >> 2, qv = it & 3;
                        const bool prevv = qv < 2, row0 = (qv & 1) == 0;
                        if (prevv ? has_prev : has_next) {
                            const float* src = prevv ? (mu_prev + 2) : orow(i + 1);
                            const float* vv = (row0 ? (src + R) : src) + 4 * pp;
                            const double* kr = K + k * KS + (row0 ? 2 : 2 + R) + 4 * pp;
                            double p2[2] = {pp == 0 ? K[k * KS + (row0 ? 0 : 1)] : 0.0, 0.0};
#pragma unroll
                            for (int c = 0; c < 4; ++c) p2[c & 1] = fma(kr[c], (double)vv[c], p2[c & 1]);
                            v = p2[0] + p2[1];
                        }
                    }
                    v = ame::group_sum<8>(v);
                    if (pp == 0) vec[(it & 3) * D + (it >> 2)] = v;
                } else if (wave == 1) {
                    // chunks 256..263 split 8 ways like wave 0's W/Y items (one
                    // 16-FMA chunk on 8 lanes made this wave finish phase 1 ~2k
                    // cycles after the others, profiles/r02_c5_workers_stamps.txt)
                    const int r2 = 256 + (lane >> 3), pp = lane & 7;
                    const int ch = r2 / D, k = r2 - ch * D;
                    const int m0 = 2 + ch * 16 + 2 * pp;
                    const double* gi = gob(i);
                    double v = 0.0;
#pragma unroll
                    for (int mm = 0; mm < 2; ++mm) {
                        const int m = m0 + mm;
                        if (m < D) v = fma(K[k * KS + m], WK ? gi[m] : gi[m] + gi[D + m], v);
                    }
                    v = ame::group_sum<8>(v);
                    if (pp == 0) vec[(5 + ch) * D + k] = v;
                } else {
                    const int k = tid - 128;
                    if (k < D) vec[4 * D + k] = apart(k);
                }
            } else {
                constexpr int NIT = 4 * D + (1 + US) * D;
                for (int it = tid; it < NIT; it += AME_NT) {
                    if (it < 4 * D) vec[(it & 3) * D + (it >> 2)] = wy_item(it);
                    else if (it < 5 * D) vec[4 * D + (it - 4 * D)] = apart(it - 4 * D);
                    else {
                        const int r2 = it - 5 * D, ch = r2 / D;
                        vec[(5 + ch) * D + (r2 - ch * D)] = chunk(r2);
                    }
                }
            }
            STAMPW(4, 0);
            STAMPW(5, 128);
            STAMPW(6, 192);
            if (wave == 1) P2STAMP(7);
            if (!WK && has_next) stage_z(i + 1, i);
            STAMPW(7, 0);
        }
        // MG: node i-1's (U,V) row (stored by wave 0 in the previous step) is
        // read by this step's GEMV in waves 1-3: drain it before the barrier
        if constexpr (MG) {
            if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        STAMPW(23, 128);
        lds_barrier();   // B1
        STAMP(1);
        // ---------------- phase 2 ----------------
        if (wave == 0) {
            // any wave of the slice dead (its word was written before B1 or an
            // earlier barrier): read with the step's first LDS reads
            const bool wd = dead || *wdead != 0u;
            // lane owns state rows k = lane + 64h (h < KH)
            double W0[KH], W1[KH], Y0[KH], Y1[KH], ua[KH], uM[KH], gk[KH], K0[KH], K1[KH];
            double jp0[KH], jp1[KH], jn0[KH], jn1[KH];
            const float* mnext = has_next ? orow(i + 1) : nullptr;
#pragma unroll
            for (int h = 0; h < KH; ++h) {
                const int k = lane + 64 * h;
                W0[h] = W1[h] = Y0[h] = Y1[h] = ua[h] = uM[h] = gk[h] = K0[h] = K1[h] = 0;
                jp0[h] = jp1[h] = jn0[h] = jn1[h] = 0;
                if (k < D) {
                    W0[h] = vec[k]; W1[h] = vec[D + k]; Y0[h] = vec[2 * D + k]; Y1[h] = vec[3 * D + k];
                    ua[h] = vec[4 * D + k];
                    if constexpr (WK) {
                        uM[h] = vec[5 * D + k];   // one (U,V) sum per row (phase 1)
                    } else {
#pragma unroll
                        for (int ch = 0; ch < US; ++ch) uM[h] += vec[(5 + ch) * D + k];
                    }
                    gk[h] = WK ? gob(i)[k] : gob(i)[k] + gob(i)[D + k];
                    K0[h] = K[k * KS + 0];
                    K1[h] = K[k * KS + 1];
                    if (k == 0) { jp0[h] = 1.0; jn0[h] = 1.0; }
                    if (k == 1) { jp1[h] = 1.0; jn1[h] = 1.0; }
                    if (k >= 2 && k < 2 + R) {
                        jp0[h] = (double)mu_prev[2 + R + (k - 2)];
                        if (has_next) jn0[h] = (double)mnext[R + (k - 2)];
                    }
                    if (k >= 2 + R) {
                        jp1[h] = (double)mu_prev[2 + (k - 2 - R)];
                        if (has_next) jn1[h] = (double)mnext[k - 2 - R];
                    }
                }
            }
            const double z0 = r00 * (double)y_prev0 + r01 * (double)y_prev1;
            const double z1 = r10 * (double)y_prev0 + r11 * (double)y_prev1;
            double u[KH], hk[KH], mus[KH];
            double Lp0[KH], Lp1[KH], Rp0[KH], Rp1[KH];   // P_i^-1 = K - Lp Rp^T
            double Xp0[KH], Xp1[KH];                     // X' = P_i^-1 J_{i+1}^T
#pragma unroll
            for (int h = 0; h < KH; ++h) {
                u[h] = ua[h] + uM[h];
                hk[h] = has_prev ? gk[h] + jp0[h] * z0 + jp1[h] * z1 : gk[h];   // natural parameter
                Lp0[h] = Lp1[h] = Rp0[h] = Rp1[h] = 0;
                Xp0[h] = Y0[h];
                Xp1[h] = Y1[h];
            }
            if (has_prev) {
                double pr[KH][14], o[14];
#pragma unroll
                for (int h = 0; h < KH; ++h) {
                    pr[h][0] = jp0[h] * W0[h]; pr[h][1] = jp0[h] * W1[h];
                    pr[h][2] = jp1[h] * W0[h]; pr[h][3] = jp1[h] * W1[h];
                    pr[h][4] = jp0[h] * u[h];  pr[h][5] = jp1[h] * u[h];
                    pr[h][6] = jp0[h] * Y0[h]; pr[h][7] = jp0[h] * Y1[h];
                    pr[h][8] = jp1[h] * Y0[h]; pr[h][9] = jp1[h] * Y1[h];
                    pr[h][10] = jp0[h] * ua[h]; pr[h][11] = jp1[h] * ua[h];
                    pr[h][12] = jp0[h] * uM[h]; pr[h][13] = jp1[h] * uM[h];
                }
                // sums 10-13 serve the bad variant only: a kernel instantiated for
                // good / naive reduces 10 (13 pair steps of the tree instead of 16)
                constexpr int NR = (VAR == AME_GOOD || VAR == AME_NAIVE) ? 10 : 14;
                wave_multidot<14, D, KH, NR>(pr, o, red, scal, lane);
                STAMPW(8, 0);
                M22 Mm = {Rm.a + o[0], Rm.b + 0.5 * (o[1] + o[2]), 0.0, Rm.d + o[3]};
                Mm.c = Mm.b;
                M22 Mi = inv22_fast(Mm);
                Mi.b = Mi.c = 0.5 * (Mi.b + Mi.c);
                // rows 0, 1 of W (J K[:,b] = (W0[b], W1[b])) live in lanes 0, 1 of h = 0
                const double Wa00 = ame::lane_bcast(W0[0], 0), Wa01 = ame::lane_bcast(W0[0], 1);
                const double Wa10 = ame::lane_bcast(W1[0], 0), Wa11 = ame::lane_bcast(W1[0], 1);
#pragma unroll
                for (int h = 0; h < KH; ++h) {
                    const int k = lane + 64 * h;
                    const double wm0 = W0[h] * Mi.a + W1[h] * Mi.c, wm1 = W0[h] * Mi.b + W1[h] * Mi.d;
                    Lp0[h] = wm0; Lp1[h] = wm1; Rp0[h] = W0[h]; Rp1[h] = W1[h];
                    if (!is_bad) {
                        mus[h] = u[h] + wm0 * ((double)y_prev0 - o[4]) + wm1 * ((double)y_prev1 - o[5]);
                    } else {
                        // P^-1 h^(x) = K h^(x) - W M^-1 (J K h^(x))
                        const double ta = ua[h] + z0 * K0[h] + z1 * K1[h];
                        const double tM = uM[h] + z0 * (W0[h] - K0[h]) + z1 * (W1[h] - K1[h]);
                        if (k < 2) {
                            const double j0 = o[10] + z0 * Wa00 + z1 * Wa01;
                            const double j1 = o[11] + z0 * Wa10 + z1 * Wa11;
                            mus[h] = ta - (wm0 * j0 + wm1 * j1);
                        } else {
                            const double j0 = o[12] + z0 * (o[0] - Wa00) + z1 * (o[1] - Wa01);
                            const double j1 = o[13] + z0 * (o[2] - Wa10) + z1 * (o[3] - Wa11);
                            mus[h] = tM - (wm0 * j0 + wm1 * j1);
                        }
                    }
                    Xp0[h] = Y0[h] - (wm0 * o[6] + wm1 * o[8]);
                    Xp1[h] = Y1[h] - (wm0 * o[7] + wm1 * o[9]);
                }
            } else {
#pragma unroll
                for (int h = 0; h < KH; ++h)
                    mus[h] = is_bad ? ((lane + 64 * h < 2) ? ua[h] : uM[h]) : u[h];
            }
#pragma unroll
            for (int h = 0; h < KH; ++h) {
                const int k = lane + 64 * h;
                if (!is_naive) mus[h] += 1e-6 * hk[h];
                if (k < D) {   // damped new mean; publish (mu_prev: readers above are done, wave-ordered)
                    const float mo = WK ? oring[(i & 3) * D + k] : mu_old[k];   // node i, old
                    const float nw = mul_add_rn(lr, (float)mus[h], om, mo);
                    xn[(size_t)i * D + k] = nw;
                    if constexpr (MG) {
                        if (k >= 2) Mg[(size_t)i * M2 + (k - 2)] = nw;
                    }
                    mu_prev[k] = nw;
                    if constexpr (WK) mu_prev64[k] = (double)nw;
                    if constexpr (WK) mring[(i & 3) * D + k] = nw;
                    // a dead slice tags its granules 0: no sweep waits for that epoch
                    const uint64_t g = ((uint64_t)(wd ? 0u : a.epoch) << 32) | (uint64_t)__float_as_uint(nw);
                    gran_store_agent(a.hand + ((size_t)tl * n + i) * D + k, g);
                    if (tl == TL - 1 && a.halo_out != nullptr)
                        gran_store_system(a.halo_out + (size_t)i * D + k, g);
                }
            }
            STAMPW(9, 0);
            double Lm0[KH], Lm1[KH], Rm0[KH], Rm1[KH];   // downdate: + X' S'^-1 X'^T
#pragma unroll
            for (int h = 0; h < KH; ++h) Lm0[h] = Lm1[h] = Rm0[h] = Rm1[h] = 0;
            if (has_next) {
                double pr2[KH][4], o2[4];
#pragma unroll
                for (int h = 0; h < KH; ++h) {
                    pr2[h][0] = jn0[h] * Xp0[h]; pr2[h][1] = jn0[h] * Xp1[h];
                    pr2[h][2] = jn1[h] * Xp0[h]; pr2[h][3] = jn1[h] * Xp1[h];
                }
                wave_multidot<4, D, KH>(pr2, o2, red, scal + 16, lane);
                M22 Sm = {Rm.a - o2[0], Rm.b - 0.5 * (o2[1] + o2[2]), 0.0, Rm.d - o2[3]};
                Sm.c = Sm.b;
                M22 Si = inv22_fast(Sm);
                Si.b = Si.c = 0.5 * (Si.b + Si.c);
#pragma unroll
                for (int h = 0; h < KH; ++h) {
                    Lm0[h] = Xp0[h] * Si.a + Xp1[h] * Si.c;
                    Lm1[h] = Xp0[h] * Si.b + Xp1[h] * Si.d;
                    Rm0[h] = Xp0[h];
                    Rm1[h] = Xp1[h];
                }
            }
            STAMPW(10, 0);
#pragma unroll
            for (int h = 0; h < KH; ++h) {
                const int k = lane + 64 * h;
                if (k < D) {
                    // row-interleaved: the k-side four of an entry, then its m-side
                    // four, each one 32-byte run (two 16-byte LDS reads in phase 3)
                    double* ur = upd + 8 * k;
                    ur[0] = Lp0[h]; ur[1] = Lp1[h]; ur[2] = Lm0[h]; ur[3] = Lm1[h];
                    ur[4] = Rp0[h]; ur[5] = Rp1[h]; ur[6] = Rm0[h]; ur[7] = Rm1[h];
                }
            }
            if (is_naive) {
                // C = diag(1 / (diag(P_i) + 1e-8)) (naive_mf.py:271-274), formed here
                // where wave 0 waits for waves 1-3 (in phase 3 each wave met the
                // diagonal entries in most of its rounds, a divergent branch with
                // a load and a division each time: +3.8k cycles per step at r = 32)
#pragma unroll
                for (int h = 0; h < KH; ++h) {
                    const int k = lane + 64 * h;
                    if (k < D) {
                        double pd;
                        if (k == 0) pd = p * (double)(n - 1);
                        else if (k == 1) pd = s * (double)(n - 1);
                        else if (k < 2 + R) {
                            const double vo = (double)orow(i)[R + (k - 2)];
                            pd = p * (ssq[R + (k - 2)] - vo * vo);
                        } else {
                            const double uo = (double)orow(i)[k - 2 - R];
                            pd = s * (ssq[k - 2 - R] - uo * uo);
                        }
                        ndiag[k] = 1.0f / ((float)(pd + pcd[k]) + 1e-8f);
                    }
                }
            }
        } else if (has_next) {
            // waves 1-3: next-node loads first (latency hidden by the GEMV), GEMV, then hand-offs
            float nx = 0.f, ol = 0.f;
            float o2 = 0.f;
            if (!WK && tid >= 128 && tid < 128 + D) {
                right_regs(i + 1, nx, ol);
                if (i + 2 < n) o2 = xo[(size_t)(i + 2) * D + (tid - 128)];
            }
            uint64_t g0[KH];
            if (wave == 1) first_poll(i + 1, g0);
            double aR = 0.0;
            if constexpr (WK) {
                gather(i + 1);
                STAMPW(24, 128);
                aR = aR1;   // loaded in phase 1
                STAMPW(25, 128);
            } else {
                if (i + 2 < n) prefetch_y(i + 2);
                gemv(tid - 64);
            }
            STAMPW(11, 64);
            STAMPW(13, 128);
            if (wave == 1) {
                if (tg > 0) poll_left(i + 1, g0);
                else zero_left();
                STAMPW(12, 64);
            }
            if (!WK && tid >= 128 && tid < 128 + D) {
                mu_right[tid - 128] = nx;
                mu_old_n[tid - 128] = ol;
                oring[((i + 2) & 3) * D + (tid - 128)] = o2;   // node i-2's slot: not read this step
            }
            if constexpr (WK) {
                // g_obs and the AR terms of node i+1, off phase 3.  The AR terms
                // need only mu_{i+1,t-1} (wave 1's poll), the g_obs sum only the
                // partials (waves 2-3's gather): two signals, so each starts as
                // soon as its input is in LDS
                P2STAMP(2 * (wave - 1));
                if (lane == 0) ame::lds_signal_add(wave == 1 ? wsync + 1 : wsync, 1u);
                ame::lds_wait_ge(wsync + 1, (uint32_t)(i + 1), a.status, dead, tg, (uint32_t)i, a.epoch);
                P2STAMP(8 + 2 * (wave - 1));
                ar_left_finish(i + 1, aR);
                P2STAMP(9 + 2 * (wave - 1));
                P2STAMP(6);
                ame::lds_wait_ge(wsync, 2u * (uint32_t)(i + 1), a.status, dead, tg, (uint32_t)i, a.epoch);
                if (dead && lane == 0) *wdead = 1u;
                gemv_reduce(i + 1);
                STAMPW(26, 64);
                STAMPW(27, 128);
                P2STAMP(2 * (wave - 1) + 1);
            }
        }
        if (!WK && wave == 0 && i + 2 < n && has_next) prefetch_y(i + 2);
        lds_barrier();   // B2
        STAMP(2);
        // ---------------- phase 3 ----------------
        // WK: node i+1's natural parameter in one piece (its parts were written
        // in phase 2, before B2; read from phase 1 of the next step on)
        if (WK && has_next && tid < D) gob(i + 1)[tid] += gob(i + 1)[D + tid];
        STAMPW(28, 0);
        {
            // the LDS reads of QB rounds first, then their stores: a round's K / cst
            // stores otherwise keep the next round's reads behind them (the compiler
            // cannot tell the addresses apart), serialising the rounds.  Each
            // thread owns its (k, m) entries, and only k >= m is read.
            // Branch-free: every round but the last has an entry on every
            // thread (LTF full rounds); flags select the variant's value; a
            // diagonal entry stores its (equal) mirror value twice.
            if constexpr (PH3B) {
            if (pkb >= 0) {
                constexpr int PB = Ph3<D>::PB;
                const int k0 = PB * pkb, m0 = PB * pmb;
                // every LDS read of the block first, then the arithmetic and stores
                double ul[PB][4], ur[PB][4], kr[PB][PB];
                float ckm[PB][PB], cmk[PB][PB], nd[PB];
#pragma unroll
                for (int q = 0; q < PB; ++q) {
                    const int k = min(k0 + q, D - 1), m = min(m0 + q, D - 1);
                    const double2 l01 = *(const double2*)(upd + 8 * k), l23 = *(const double2*)(upd + 8 * k + 2);
                    const double2 r01 = *(const double2*)(upd + 8 * m + 4), r23 = *(const double2*)(upd + 8 * m + 6);
                    ul[q][0] = l01.x; ul[q][1] = l01.y; ul[q][2] = l23.x; ul[q][3] = l23.y;
                    ur[q][0] = r01.x; ur[q][1] = r01.y; ur[q][2] = r23.x; ur[q][3] = r23.y;
                    nd[q] = ndiag[k];   // naive only
                }
#pragma unroll
                for (int x = 0; x < PB; ++x)
#pragma unroll
                    for (int y = 0; y < PB; ++y) {
                        const int k = min(k0 + x, D - 1), m = min(m0 + y, D - 1);
                        kr[x][y] = K[k * KS + m];
                        ckm[x][y] = cob[k * D + m];
                        cmk[x][y] = cob[m * D + k];
                    }
#pragma unroll
                for (int x = 0; x < PB; ++x)
#pragma unroll
                    for (int y = 0; y < PB; ++y) {
                        const int k = k0 + x, m = m0 + y;
                        if (k >= D || m >= D || (pkb == pmb && y > x)) continue;
                        const double c = kr[x][y] - (ul[x][0] * ur[y][0] + ul[x][1] * ur[y][1]);
                        const double kn = c + (ul[x][2] * ur[y][2] + ul[x][3] * ur[y][3]);
                        const bool dg = k == m, ob = (k < 2) != (m < 2);
                        float c32 = (float)c;
                        c32 = (is_bad && ob) ? 0.f : c32;
                        c32 = dg ? c32 + 1e-6f : c32;
                        c32 = is_naive ? (dg ? nd[x] : 0.f) : c32;
                        const float vkm = mul_add_rn(lr, c32, om, ckm[x][y]);
                        const float vmk = mul_add_rn(lr, c32, om, cmk[x][y]);
                        K[k * KS + m] = kn;
                        K[m * KS + k] = kn;
                        cst[k * D + m] = vkm;
                        cst[m * D + k] = vmk;
                    }
            }
            } else {
            constexpr int QB = 5;   // 9 entries per thread at d = 66: rounds of 5 and 4
            constexpr int LTF = NLT / AME_NT;
            // opaque per step: hoisted out of the loop, each flag test became a
            // lane mask in an SGPR pair, spilled and reloaded per entry
            uint32_t df = dflag, of = oflag;
            asm volatile("" : "+v"(df), "+v"(of));
#pragma unroll
            for (int q0 = 0; q0 < LTQ; q0 += QB) {
            double kr[QB], u0[QB], u1[QB], u2[QB], u3[QB], u4[QB], u5[QB], u6[QB], u7[QB];
            float ckm[QB], cmk[QB], nd[QB];
#pragma unroll
            for (int b = 0; b < QB; ++b) {
                const int qq = q0 + b < LTQ ? q0 + b : LTQ - 1;
                const int k = max(lk[qq], 0), m = max(lm[qq], 0);
                kr[b] = K[k * KS + m];
                const double* uk = upd + 8 * k;       // Lp0 Lp1 Lm0 Lm1 of row k
                const double* um = upd + 8 * m + 4;   // Rp0 Rp1 Rm0 Rm1 of row m
                u0[b] = uk[0]; u2[b] = uk[1]; u4[b] = uk[2]; u6[b] = uk[3];
                u1[b] = um[0]; u3[b] = um[1]; u5[b] = um[2]; u7[b] = um[3];
                ckm[b] = cob[k * D + m];
                cmk[b] = cob[m * D + k];
                nd[b] = ndiag[k];   // naive only (C = diag(1 / (diag(P_i) + 1e-8)), formed in phase 2)
            }
#pragma unroll
            for (int b = 0; b < QB; ++b) {
                const int qq = q0 + b;
                if (qq >= LTQ) continue;
                const int k = max(lk[qq], 0), m = max(lm[qq], 0);
                const double c = kr[b] - (u0[b] * u1[b] + u2[b] * u3[b]);
                const double kn = c + (u4[b] * u5[b] + u6[b] * u7[b]);
                const bool dg = (df >> qq) & 1u, ob = (of >> qq) & 1u;
                float c32 = (float)c;
                c32 = (is_bad && ob) ? 0.f : c32;
                c32 = dg ? c32 + 1e-6f : c32;
                c32 = is_naive ? (dg ? nd[b] : 0.f) : c32;
                const float vkm = mul_add_rn(lr, c32, om, ckm[b]);
                const float vmk = mul_add_rn(lr, c32, om, cmk[b]);
                if (qq < LTF || lk[qq] >= 0) {
                    K[k * KS + m] = kn;
                    K[m * KS + k] = kn;
                    cst[k * D + m] = vkm;
                    cst[m * D + k] = vmk;
                }
            }
            }
            }
            STAMPW(14, 0);
            if (!WK && has_next) {
                gemv_reduce(i + 1);
                ar_terms(i + 1);
            }
            STAMPW(15, 0);
            if constexpr (WK) {
                // node i+2's old row into node i-2's ring slot (not read this step)
                if (has_next && tid >= 128 && tid < 128 + D) {
                    oring[((i + 2) & 3) * D + (tid - 128)] = o21;
                    oring64[((i + 2) & 3) * D + (tid - 128)] = (double)o21;
                }
            } else {
                if (tid >= 128 && tid < 128 + D) mu_old[tid - 128] = mu_old_n[tid - 128];
            }
            y_prev0 = (float)scal[40];
            y_prev1 = (float)scal[41];
        }
        lds_barrier();   // B3
        STAMP(3);
    }
    cov_flush(n - 1);
    // ---- slice done: release its means, covariances and granules, then flag it
    // for the next sweep (ame_sweep3.hip's epilogue; every wave drains its own
    // stores first).  A dead slice flags nothing ----
    bool any_dead = false;
    if (a.done != nullptr || (tl == 0 && a.back_out != nullptr)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // (the LDS word, not __syncthreads_or: that one adds 256 bytes of
        // static LDS to the launch)
        if (dead) *wdead = 1u;
        __syncthreads();
        any_dead = *wdead != 0u;
    }
    if (a.done != nullptr && tid == 0 && !any_dead) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.done + tl, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // ---- first slice of a rank with a left neighbour: its new means are that
    // rank's next_old in the next (pipelined) sweep; system-scope release ----
    if (tl == 0 && a.back_out != nullptr && !any_dead) {
        for (int e = tid; e < n * D; e += AME_NT)
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

template <int R, int MODE>
static int launch_sweep_t(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    const long long lds = ame_v2_mode_lds(dm->n, R, MODE);
    void (*kern)(ame_dims, ame_sweep_args);
    if constexpr (MODE == 2)   // per-variant kernels (config 5's sweep)
        kern = dm->variant == AME_NAIVE ? ame_sweep_kernel<R, MODE, AME_NAIVE>
             : dm->variant == AME_BAD   ? ame_sweep_kernel<R, MODE, AME_BAD>
                                        : ame_sweep_kernel<R, MODE, AME_GOOD>;
    else
        kern = ame_sweep_kernel<R, MODE>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
        return -2;
    int blocks = dm->T_local;
    if constexpr (MODE >= 2) {
        blocks = dm->T_local * (1 + ame_v2_nworkers(MODE));
        // partial ring: zero never matches a tag (ame_gw_tag sets bit 31)
        const size_t bytes = (size_t)ame_v2_ring_doubles(dm, MODE) * 8;
        if (hipMemsetAsync(a->work, 0, bytes, st) != hipSuccess) return -3;
        static_assert(ArPart<R, true>::NPA == ((4 * (2 + 2 * R) <= 192) ? 4 : 2),
                      "ame_v2_arr_doubles sizes the AR parts");
    }
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(AME_NT), (size_t)lds, st, *dm, *a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int R, int MODE>
static int sweep_occupancy_t(int n) {
    const long long lds = ame_v2_mode_lds(n, R, MODE);
    if (lds > AME_LDS_MAX) return 0;
    // the variants of MODE 2 share the launch shape; the good one stands for them
    auto kern = ame_sweep_kernel<R, MODE, MODE == 2 ? AME_GOOD : -1>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
        hipSuccess)
        return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, AME_NT, (size_t)lds) != hipSuccess)
        return 0;
    return per_cu;
}

// MODE 2 / 3 can run when its T_local * (1 + workers) workgroups are co-resident
// and a worker wave's node share fits its registers
template <int R, int MODE>
static bool workers_fit(int n, int T_local) {
    const int nw = ame_v2_nworkers(MODE);
    const int NW = (n + nw - 1) / nw;
    if ((NW + 3) / 4 > ame_v2_maxpw(MODE) || n > 65535) return false;
    if (ame_v2_mode_lds(n, R, MODE) > AME_LDS_MAX) return false;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
    return (long long)T_local * (1 + nw) <= (long long)sweep_occupancy_t<R, MODE>(n) * cus;
}

// a->kind is concrete here (ame_capi.hip resolved and checked it)
template <int R>
static int launch_sweep(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    switch (a->kind) {
        case AME_SWEEP_V2_WORKERS: return launch_sweep_t<R, 2>(dm, a, st);
        case AME_SWEEP_V2_PIPE: return launch_sweep_t<R, 3>(dm, a, st);
        case AME_SWEEP_V2_W6: return launch_sweep_t<R, 4>(dm, a, st);
        case AME_SWEEP_V2_HBM: return launch_sweep_t<R, 1>(dm, a, st);
        case AME_SWEEP_V2_LDS: return launch_sweep_t<R, 0>(dm, a, st);
        default: return -1;
    }
}

template <int R>
static int sweep_occupancy(int n, int mode) {
    switch (mode) {
        case 0: return sweep_occupancy_t<R, 0>(n);
        case 1: return sweep_occupancy_t<R, 1>(n);
        case 2: return sweep_occupancy_t<R, 2>(n);
        case 3: return sweep_occupancy_t<R, 3>(n);
        case 4: return sweep_occupancy_t<R, 4>(n);
        default: return 0;
    }
}

int AME_PFN(ame_sweep_dispatch)(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    switch (dm->r) {
#define X(RR) \
    case RR: return launch_sweep<RR>(dm, a, st);
        AME_FOR_EACH_R(X)
#undef X
        default: return -1;
    }
}

// workgroups of one v2 launch per CU for a mode (0: block in LDS, 1: HBM, 2: workers)
int AME_PFN(ame_sweep_blocks_per_cu)(int n, int r, int mode) {
    switch (r) {
#define X(RR) \
    case RR: return sweep_occupancy<RR>(n, mode);
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}

// 1 when the v2 sweep with GEMV workers can run these dims
int AME_PFN(ame_sweep_workers_fit)(const ame_dims* dm, int mode) {
    switch (dm->r) {
#define X(RR) \
    case RR: return (mode == 3   ? workers_fit<RR, 3>(dm->n, dm->T_local) \
                     : mode == 4 ? workers_fit<RR, 4>(dm->n, dm->T_local) \
                                 : workers_fit<RR, 2>(dm->n, dm->T_local)) ? 1 : 0;
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}
