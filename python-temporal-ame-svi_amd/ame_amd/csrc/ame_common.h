// Shared device helpers for the temporal-AME VI kernels (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../../include/ame_amd.h"

#define AME_NT 256          // threads per workgroup
// Spin bounds in s_memrealtime ticks (constant 100 MHz clock): a hand-off that
// does not arrive within this time sets a status bit and the sweep finishes.
#define AME_SPIN_TICKS_LOCAL (200ull * 1000 * 1000)   // 2 s, lane -> lane on one GPU
#define AME_SPIN_TICKS_HALO (1000ull * 1000 * 1000)   // 10 s, rank -> rank

// ---- bounded waits and the status block (include/ame_amd.h) ----
#define AME_ST_CLAIM 1
#define AME_ST_CROSS 9    // workgroups inside a cross-rank wait right now
#define AME_ST_QUIET 10   // waits that gave up quietly after the first failure
#define AME_ST_HALO_US 11 // microseconds first slices spun on the left rank's granules
#define AME_ST_BACK_US 12 // microseconds last slices spun on the right rank's back channel
// node index of a wait before the node loop (prologue)
#define AME_NODE_NONE 0xFFFFFFFFu

__device__ __forceinline__ uint32_t ame_st_load(uint32_t* st, int w) {
    return __hip_atomic_load(st + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One lane.  A failure sets its bit unless an earlier one already set a bit
// (then it only counts a quiet give-up: the first failure is the cause, the
// rest are its consequences); the first to claim the record fills it.
__device__ __forceinline__ void ame_fail(uint32_t* st, uint32_t bit, int site, int slice, uint32_t node,
                                         uint32_t observed, uint32_t expected, uint64_t ticks,
                                         uint32_t epoch) {
    if (ame_st_load(st, 0) != 0u) {
        atomicAdd(st + AME_ST_QUIET, 1u);
        return;
    }
    atomicOr(st, bit);
    if (atomicCAS(st + AME_ST_CLAIM, 0u, 1u) == 0u) {
        const uint64_t us = ticks / 100u;
        st[2] = (uint32_t)site;
        st[3] = (uint32_t)slice;
        st[4] = node;
        st[5] = observed;
        st[6] = expected;
        st[7] = (uint32_t)(us > 0xFFFFFFFFull ? 0xFFFFFFFFull : us);
        st[8] = epoch;
        __threadfence();
    }
}

// The slow path of one bounded wait, run by the waiting wave (or thread):
//   AmeSpin w(st, cross, leader);  while (!arrived) { switch (w.poll()) ... }  w.end();
// poll(): 0 keep waiting, 1 give up quietly (the status block already holds a
// failure), 2 budget spent (the caller reports through ame_fail).  A wait on
// this GPU restarts its budget while any workgroup sharing the status block is
// inside a cross-rank wait: its producer may stand behind that rank (no
// progress is expected until it arrives, and that wait has its own budget).
// The status words are read at most once per AME_SPIN_TICKS_CHECK: a poll
// before that costs one clock read, as the plain bounded spin did (two global
// loads per poll delayed every wake-up: +0.7 % at config 3,
// profiles/r06_ab_prologue.txt).
// acct (a cross-rank wait's leader only): status word that end() adds the
// microseconds spent to -- AME_ST_HALO_US / AME_ST_BACK_US, the per-rank halo
// wait time the bench reports; 0 = none.
#define AME_SPIN_TICKS_CHECK (100ull * 1000)   // 1 ms
struct AmeSpin {
    uint32_t* st;
    uint64_t t_first, t0, t_chk;
    bool cross, leader;
    int acct;
    __device__ __forceinline__ AmeSpin(uint32_t* s, bool cr, bool ld, int ac = 0)
        : st(s), cross(cr), leader(ld), acct(ac) {
        t_first = t0 = t_chk = __builtin_amdgcn_s_memrealtime();
        if (cross && leader) atomicAdd(st + AME_ST_CROSS, 1u);
    }
    __device__ __forceinline__ int poll() {
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (now - t_chk < AME_SPIN_TICKS_CHECK) return 0;
        t_chk = now;
        if (ame_st_load(st, 0) != 0u) {
            if (leader) atomicAdd(st + AME_ST_QUIET, 1u);
            return 1;
        }
        if (!cross && ame_st_load(st, AME_ST_CROSS) != 0u) {
            t0 = now;
            return 0;
        }
        return (now - t0 > (cross ? AME_SPIN_TICKS_HALO : AME_SPIN_TICKS_LOCAL)) ? 2 : 0;
    }
    __device__ __forceinline__ uint64_t waited() const { return __builtin_amdgcn_s_memrealtime() - t_first; }
    __device__ __forceinline__ void end() {
        if (cross && leader) {
            atomicSub(st + AME_ST_CROSS, 1u);
            if (acct > 0) atomicAdd(st + acct, (uint32_t)(waited() / 100u));
        }
    }
};

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

// Row stride (in (y0, y1) pairs) of the packed observed network Yt: n rounded up
// to even, so every row starts 16-byte aligned (16-byte / LDS-DMA loads of any
// row; the pad pair is zero and never used as a node).
__host__ __device__ inline int ame_ystride(int n) { return n + (n & 1); }

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

// a*b + c*d with both products and the sum rounded, never contracted into an
// FMA: the reference's fp32 elementwise forms (damping lr * new + (1 - lr) * old,
// z = R^-1 y).  __fadd_rn / __fmul_rn are plain + and * in this HIP, which
// -ffp-contract=fast may fuse -- differently for a covariance entry and its
// mirror, so the damped covariance was not exactly symmetric.
__device__ __forceinline__ float mul_add_rn(float a, float b, float c, float d) {
#pragma clang fp contract(off)
    return a * b + c * d;
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

// Dynamic LDS carve-up of the sweep kernel (host and device agree).  The
// slice's (U,V) block (n x 2R floats) lives in LDS when everything fits one
// CU's 160 KiB; otherwise (m_global = 1, e.g. n = 4096 or r = 32) the GEMV
// reads it from the slice's mean buffers in HBM/L2 (new means for nodes already
// updated this sweep, old ones after), and it takes no LDS.
#define AME_LDS_MAX 163840LL
struct SweepLds {
    long long oK, oVec, oUpd, oRed, oScal, oG, oSsq, oF, oPart, oCst, oCob, oZ, oV64, oM, total;
    int m_global;
};
__host__ __device__ inline long long ame_align16(long long x) { return (x + 15) & ~15LL; }
__host__ __device__ inline SweepLds sweep_lds_layout(int n, int R, int force_global = 0, int wk = 0) {
    const int D = 2 + 2 * R, M2 = 2 * R, KS = D + 1, US = (M2 + 15) / 16;
    const int VEC = (R % 4 == 0) ? 4 : ((R % 2 == 0) ? 2 : 1);
    const int GW = 192 / (M2 / VEC);
    SweepLds L;
    long long o = 0;
    L.oK = o;    o = ame_align16(o + 8LL * D * KS);
    L.oVec = o;  o = ame_align16(o + 8LL * (5 + US) * D);
    L.oUpd = o;  o = ame_align16(o + 8LL * 8 * D);
    L.oRed = o;  o = ame_align16(o + 8LL * 16 * D);
    L.oScal = o; o = ame_align16(o + 8LL * 64);
    L.oG = o;    o = ame_align16(o + 8LL * 4 * D);   // [node & 1] {g_obs, AR}
    L.oSsq = o;  o = ame_align16(o + 8LL * (2 * R + D) + 4LL * D);   // ssq, diag P_const, naive diag C
    L.oF = o;    o = ame_align16(o + 4LL * 9 * D);   // 5 mean rows + 4-slot old-row ring
    L.oPart = o; o = ame_align16(o + 4LL * GW * (M2 + 2));
    L.oCst = o;  o = ame_align16(o + 4LL * D * D);   // new covariance of the step, staged
    L.oCob = o;  o = ame_align16(o + 4LL * D * D);   // old covariance of the step
    // z row; with workers only the 4-slot new-mean ring lives there
    L.oZ = o;    o = ame_align16(o + (wk ? 16LL * D : 8LL * (n > 2 * D ? n : 2 * D)));
    // (workers) fp64: mu_{i-1} and the old-row ring (phase 1's row dots), mu_{i+1,t-1}
    // and QiPhi by AR row part (the AR-left sum of phase 2: LDS reads instead of
    // coefficient registers)
    L.oV64 = o;
    if (wk) {
        const int npa = (4 * D <= 192) ? 4 : 2, mcp = ((D + npa - 1) / npa + 1) & ~1;
        o = ame_align16(o + 8LL * 6 * D + 8LL * D * npa * mcp);
    }
    L.oM = o;
    const long long withM = ame_align16(o + 4LL * n * M2);
    L.m_global = (force_global || withM > AME_LDS_MAX) ? 1 : 0;
    L.total = L.m_global ? o : withM;
    return L;
}

// v2 sweep with GEMV workers (kind AME_SWEEP_V2_WORKERS, ame_sweep.hip)
#define AME_GW 7          // GEMV worker workgroups per slice
#define AME_GW_RING 8     // partial ring slots per worker
#define AME_GW_MAXPW 152  // nodes per worker wave held in registers: n <= 7 * 4 * 152
// pipelined v2 sweep (kind AME_SWEEP_V2_PIPE, MODE 3): four workers per slice,
// so a slice is 5 workgroups and two consecutive launches of up to 25 slices
// (one workgroup per CU) are co-resident.  A worker wave holds up to 256 nodes
// (n <= 4 * 4 * 256): 152 in registers -- kind 22's count, whose owner update
// compiles to one select per slot; 256 register slots compiled to a
// pathological owner update (10x slower node period in the stamped build), and
// three workers (344 slots) spill ~1 000 VGPRs at every split tried -- and the
// other 104 in the worker's LDS ([wave][slot][lane], 104 KB)
#define AME_GW_P 4
#ifndef AME_GW_P_MAXPW       // (variant builds for A/B runs may override both)
#define AME_GW_P_MAXPW 256
#endif
#ifndef AME_GW_P_NREG
#define AME_GW_P_NREG 152
#endif
// six-worker v2 sweep (kind AME_SWEEP_V2_W6, MODE 4): 7 workgroups per slice, so
// config 5's 32 slices hold 224 CUs and leave 32 to the ELBO kernels on a
// CU-masked stream (engine option elbo_cus); a worker wave holds up to 176
// nodes (n <= 6 * 4 * 176): kind 22's 152 in registers, 24 in LDS
#define AME_GW_6 6
#define AME_GW_6_MAXPW 176
#define AME_GW_6_NREG 152
__host__ __device__ constexpr int ame_v2_nworkers(int mode) {
    return mode == 3 ? AME_GW_P : (mode == 4 ? AME_GW_6 : AME_GW);
}
__host__ __device__ constexpr int ame_v2_maxpw(int mode) {
    return mode == 3 ? AME_GW_P_MAXPW : (mode == 4 ? AME_GW_6_MAXPW : AME_GW_MAXPW);
}
__host__ __device__ constexpr int ame_v2_nreg(int mode) {
    return mode == 3 ? AME_GW_P_NREG : (mode == 4 ? AME_GW_6_NREG : AME_GW_MAXPW);
}

// Tag of worker partial m of sweep `epoch` in the partial ring.  Bit 31 is
// always set, so a slot the launch zeroed can never match (an all-zero word
// would otherwise equal node 0's tag whenever epoch % 2^15 == 0); 15 epoch
// bits, 16 node bits (n <= 65535 when workers run).
__host__ __device__ inline uint32_t ame_gw_tag(uint32_t epoch, int m) {
    return 0x80000000u | ((epoch & 0x7FFFu) << 16) | ((uint32_t)m & 0xFFFFu);
}

// LDS of one v2 slice workgroup per mode (0: (U,V) in LDS, 1: in HBM, 2 / 3:
// workers) and of a GEMV worker workgroup; a worker launch sizes for the larger
__host__ __device__ inline long long ame_v2_worker_lds(int n, int R, int mode = 2) {
    const int nw = ame_v2_nworkers(mode);
    const int NW = (n + nw - 1) / nw, ZN = 4 * ame_v2_maxpw(mode);
    // zb, red, (MODES 3, 4) the LDS-held node slots [4 waves][MAXPW - NREG][64],
    // and 16 bytes for the worker's dead word (ame_v2_worker_dead_off)
    const long long mld = 4LL * 4 * (ame_v2_maxpw(mode) - ame_v2_nreg(mode)) * 64;
    return ame_align16(8LL * (NW > ZN ? NW : ZN)) + ame_align16(4LL * 4 * (2 * R + 2)) + mld + 16;
}
__host__ __device__ inline long long ame_v2_worker_dead_off(int n, int R, int mode) {
    return ame_v2_worker_lds(n, R, mode) - 16;
}
__host__ __device__ inline long long ame_v2_mode_lds(int n, int R, int mode) {
    const long long m = sweep_lds_layout(n, R, mode != 0 ? 1 : 0, mode >= 2 ? 1 : 0).total;
    if (mode < 2) return m;
    const long long w = ame_v2_worker_lds(n, R, mode);
    return m > w ? m : w;
}
__host__ __device__ inline long long ame_v2_ring_doubles(const ame_dims* d, int mode = 2) {
    return (long long)d->T_local * ame_v2_nworkers(mode) * AME_GW_RING * (2 * d->r + 2);
}
__host__ __device__ inline long long ame_v2_arr_doubles(const ame_dims* d) {
    const int D = 2 + 2 * d->r, npa = (4 * D <= 192) ? 4 : 2;
    return (long long)d->T_local * d->n * npa * D;
}


// Latent dims compiled into the library.  r = 32 (d = 66, BASELINE config 5)
// runs on the v2 sweep only (two state rows per lane in the solver wave).
#ifdef AME_ONLY_R   // diagnostic builds: one latent dim only
#define AME_FOR_EACH_R(X) X(AME_ONLY_R)
#elif defined(AME_R_PART)
// Split build (build.py): the heaviest sources are compiled once per part,
// part p of AME_R_NPART holding the r with r % AME_R_NPART == p; their
// r-dependent entry points carry a _p<part> suffix (AME_PFN) and
// ame_parts.hip routes each call to its part.
#if AME_R_NPART == 2 && AME_R_PART == 0
#define AME_FOR_EACH_R(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(22) X(24) X(26) X(28) X(30) X(32)
#elif AME_R_NPART == 2 && AME_R_PART == 1
#define AME_FOR_EACH_R(X) X(1) X(3) X(5) X(7) X(9) X(11) X(13) X(15) X(17) X(19) X(21) X(23) X(25) X(27) X(29) X(31)
#elif AME_R_NPART == 3 && AME_R_PART == 0
#define AME_FOR_EACH_R(X) X(3) X(6) X(9) X(12) X(15) X(18) X(21) X(24) X(27) X(30)
#elif AME_R_NPART == 3 && AME_R_PART == 1
#define AME_FOR_EACH_R(X) X(1) X(4) X(7) X(10) X(13) X(16) X(19) X(22) X(25) X(28) X(31)
#elif AME_R_NPART == 3 && AME_R_PART == 2
#define AME_FOR_EACH_R(X) X(2) X(5) X(8) X(11) X(14) X(17) X(20) X(23) X(26) X(29) X(32)
#else
#error "AME_R_PART / AME_R_NPART: unsupported split"
#endif
#else
// every latent dim 1..32 (reference: any r, temporal_ame.py:114-120)
#define AME_FOR_EACH_R(X) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) \
    X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)
#endif
#define AME_MAX_R 32

// entry-point names of a split part, and code that only part 0 carries
#define AME_PFN_CAT2(a, b) a##_p##b
#define AME_PFN_CAT(a, b) AME_PFN_CAT2(a, b)
#ifdef AME_R_PART
#define AME_PFN(name) AME_PFN_CAT(name, AME_R_PART)
#define AME_PART0 (AME_R_PART == 0)
#else
#define AME_PFN(name) name
#define AME_PART0 1
#endif
