// Device helpers of the LDS-DMA kernels (ame_sweep3.hip, ame_sweep.hip,
// ame_elbo.hip): workgroup-local hand-off counters in LDS, LDS-DMA
// (global_load_lds) issue wrappers with manual vmcnt accounting, the packed
// triangle index decode, the J entries of a node and two DPP pair-adds.
#pragma once
#include "ame_common.h"
#include "ame_wave.h"

namespace ame {

__device__ __forceinline__ void lds_barrier3() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wave_lds_sync3() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}
// LDS counters (workgroup-coherent); writers drain their LDS stores first.
__device__ __forceinline__ void lds_signal_add(uint32_t* f, uint32_t v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_signal_set(uint32_t* f, uint32_t v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// A wave whose global wait failed adds this bit to the LDS counter it signals
// next, so the wave waiting on that counter (the one that publishes the slice's
// hand-off granules) learns it without an extra LDS read (AME_STATUS_WORDS).
#define AME_LDS_DEAD 0x40000000u
// The spin of lds_wait_ge (AmeSpin rules), out of line.  Measured at config 3
// (same box, 5 rounds, profiles/r06_ab_lds_wait.txt): out of line 2.424 ms per
// iteration; the plain inline spin of rounds 1-5 2.542; the inline spin with
// this call only after 1 ms 2.546; the rules inline (no call, 2 VGPR spills)
// 2.441 -- the solver's loop schedules better without a spin loop inside it;
// s_sleep 1 / 3 / 8 in this loop: 2.423 / 2.427 / 2.425 (r06_ab_sleep.txt).
// (The helpers' granule wait out of line instead: 3.10 -- a call per wait on
// hw 0-2, whose waits are frequent.)
// Returns the counter's value, with AME_LDS_DEAD set when the wait failed or
// gave up (one wave).
static __device__ __attribute__((noinline)) uint32_t lds_wait_slow(uint32_t* f, uint32_t target, uint32_t* status,
                                                                   int slice, uint32_t node, uint32_t epoch) {
    const bool ld = (threadIdx.x & 63) == 0;
    AmeSpin w(status, false, ld);
    uint32_t v;
    while ((v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < target) {
        __builtin_amdgcn_s_sleep(8);
        const int r = w.poll();
        if (r == 0) continue;
        if (r == 2 && ld)
            ame_fail(status, AME_STATUS_LDS_TIMEOUT, AME_WAIT_LDS, slice, node, v, target, w.waited(), epoch);
        v |= AME_LDS_DEAD;
        break;
    }
    w.end();
    return v;
}
// Bounded: a wait that outlives its budget sets AME_STATUS_LDS_TIMEOUT and gives
// up (the launch then finishes with wrong values and a raised status, never
// hangs).  A counter carrying AME_LDS_DEAD marks the waiting wave dead as well.
__device__ __forceinline__ void lds_wait_ge(uint32_t* f, uint32_t target, uint32_t* status, bool& dead,
                                            int slice = 0, uint32_t node = AME_NODE_NONE,
                                            uint32_t epoch = 0) {
    uint32_t v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (!dead && v < target) v = lds_wait_slow(f, target, status, slice, node, epoch);
    dead = dead || (v & AME_LDS_DEAD) != 0u;
    asm volatile("" ::: "memory");
}

// Pipelined launch (wait_epoch != 0), ONE thread: wait until the previous sweep
// (epoch wait_epoch) flagged local slices t and t+1 done (done[t + 1] is the next
// slice group's first slice under AME_SWEEP_FLAG_NEXT_GROUP) and, for a rank's
// last slice, the right rank's back-channel done word.  A word above
// wait_epoch is outside the protocol's window (AME_STATUS_STALE_EPOCH); the
// back channel is a cross-rank wait (10 s budget, counted in the status
// block), the done flags local ones (AmeSpin rules).  Any failure, or a quiet
// give-up after another one, sets `dead` and skips the remaining waits.
__device__ __forceinline__ void ame_wait_prev_done(const ame_sweep_args& a, int t, int TL, int tg,
                                                   bool back_rd, int nd, bool& dead, bool account = true) {
    const int qn = (t + 1 < TL || (a.flags & AME_SWEEP_FLAG_NEXT_GROUP)) ? 2 : 1;
    for (int q = 0; q <= qn && !dead; ++q) {
        const bool back = q == qn;
        if (back && !back_rd) break;
        const uint32_t* w = back ? (const uint32_t*)(a.back_in + AME_BACK_DONE_OFFSET(nd)) : a.done + t + q;
        const int site = back ? AME_WAIT_BACK : (q == 0 ? AME_WAIT_DONE_SELF : AME_WAIT_DONE_RIGHT);
        auto load = [&]() -> uint32_t {
            return back ? __hip_atomic_load(const_cast<uint32_t*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                        : __hip_atomic_load(const_cast<uint32_t*>(w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        };
        uint32_t dv = load();
        if (dv == a.wait_epoch) continue;
        AmeSpin sp(a.status, back, true, (back && account) ? AME_ST_BACK_US : 0);
        while (true) {
            if (dv > a.wait_epoch) {
                ame_fail(a.status, AME_STATUS_STALE_EPOCH, site, tg, AME_NODE_NONE, dv, a.wait_epoch,
                         sp.waited(), a.epoch);
                dead = true;
                break;
            }
            if (dv == a.wait_epoch) break;
            const int r = sp.poll();
            if (r != 0) {
                if (r == 2)
                    ame_fail(a.status, back ? AME_STATUS_HALO_TIMEOUT : AME_STATUS_SPIN_TIMEOUT, site, tg,
                             AME_NODE_NONE, dv, a.wait_epoch, sp.waited(), a.epoch);
                dead = true;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
            dv = load();
        }
        sp.end();
    }
    if (back_rd) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- P_0's node sums on fp64 MFMA (sweep prologues, v3 and v2) ----
// The base precision P_0 of a slice (structured_mf.py:251-264 summed over the
// other nodes) needs, over the slice's old (U, V) rows x_j
// (M2 = 2R floats, node 0 excluded): the Gram matrix G = sum_{j>=1} x_j x_j^T,
// the column sums sum_{j>=1} x_j, and (naive) sum_{j>=0} x_j^2.  G is a
// K = n - 1 GEMM: v_mfma_f64_16x16x4f64 over chunks of 4 nodes (lane l holds
// x[4c + (l >> 4)][16 I + (l & 15)], the A operand of tile row I and the B
// operand of tile column I alike; the accumulator of tile (I, J) holds row
// 16 I + (l >> 4) + 4 v, column 16 J + (l & 15), as in ame_cov.hip), chunks
// dealt round-robin to the NW waves, the waves' partial tiles added in wave
// order (deterministic).  fp32 inputs, fp64 products (exact) and sums: the
// node-by-node fp64 loop it replaces summed in another order, so results move
// by fp64 rounding only (~1e-16 relative).  The loop made one dependent LDS /
// HBM round trip per node: ~60 us of every v3 slice prologue at config 3 and
// ~1.4 ms of every kind-22 launch at config 5's rank shape.
//
// Output: gram[kk(a) * ks + kk(b)] = G[a][b] for a, b < M2, both triangles,
// where kk(a) = the state row whose J entry is column a (row U_c carries V_c:
// kk(R + c) = 2 + c, kk(c) = 2 + R + c); colsum[a] = sum_{j>=1} x_ja;
// x0[a] = node 0's entry.  All threads of the workgroup call it (barriers).
typedef double ame_p0d4 __attribute__((ext_vector_type(4)));
template <int R, int NW>
__device__ __forceinline__ void p0_gram_mfma(const float* xo, int n, int D, double* gram, int ks,
                                             double* colsum, float* x0) {
    constexpr int M2 = 2 * R, NT = (M2 + 15) / 16, NTL = NT * (NT + 1) / 2;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int ci = lane & 15, ck = lane >> 4;
    ame_p0d4 acc[NTL];
#pragma unroll
    for (int t = 0; t < NTL; ++t) acc[t] = ame_p0d4{0.0, 0.0, 0.0, 0.0};
    double cs[NT];
#pragma unroll
    for (int I = 0; I < NT; ++I) cs[I] = 0.0;
    const int nch = (n + 3) / 4;
    constexpr int U = 4;   // chunks whose loads are issued together
    for (int c0 = w; c0 < nch; c0 += NW * U) {
        float xv[U][NT];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = 4 * (c0 + NW * u) + ck;
#pragma unroll
            for (int I = 0; I < NT; ++I) {
                const int col = 16 * I + ci;
                const bool ok = j >= 1 && j < n && col < M2;
                xv[u][I] = ok ? xo[(size_t)j * D + 2 + col] : 0.f;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            double xd[NT];
#pragma unroll
            for (int I = 0; I < NT; ++I) {
                xd[I] = (double)xv[u][I];
                cs[I] += xd[I];
            }
#pragma unroll
            for (int I = 0; I < NT; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J) {
                    const int t = I * (I + 1) / 2 + J;
                    acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(xd[I], xd[J], acc[t], 0, 0, 0);
                }
        }
    }
    // column sums: the 4 node lanes of a column, fixed tree
#pragma unroll
    for (int I = 0; I < NT; ++I) {
        const double s1 = cs[I] + __shfl_xor(cs[I], 16);
        cs[I] = s1 + __shfl_xor(s1, 32);
    }
    auto kk = [](int a) { return 2 + (a >= R ? a - R : a + R); };
    for (int ww = 0; ww < NW; ++ww) {
        if (w == ww) {
#pragma unroll
            for (int I = 0; I < NT; ++I)
#pragma unroll
                for (int J = 0; J <= I; ++J) {
                    const int t = I * (I + 1) / 2 + J;
#pragma unroll
                    for (int v = 0; v < 4; ++v) {
                        const int a = 16 * I + ck + 4 * v, b = 16 * J + ci;
                        if (a >= M2 || b >= M2) continue;
                        double* p = gram + kk(a) * ks + kk(b);
                        double* q = gram + kk(b) * ks + kk(a);
                        const double g = acc[t][v];
                        *p = (ww == 0) ? g : *p + g;
                        if (I != J) *q = *p;
                    }
                }
            if (ck == 0) {
#pragma unroll
                for (int I = 0; I < NT; ++I) {
                    const int a = 16 * I + ci;
                    if (a < M2) colsum[a] = (ww == 0) ? cs[I] : colsum[a] + cs[I];
                }
            }
        }
        __syncthreads();
    }
    if (tid < M2) x0[tid] = xo[2 + tid];
    __syncthreads();
}

// LDS-DMA: each lane's 16 (4) bytes from gsrc land at LDS byte lds + lane*16 (*4).
// Issued as inline asm so hipcc's waitcnt pass does not serialise LDS reads
// behind it; the loader wave counts completion itself (vmcnt).
__device__ __forceinline__ uint32_t lds_off(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ void dma16(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma16_sc1(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma16_sys(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc0 sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4_sys(const void* gsrc, uint32_t lds) {   // system-coherent (peer) source
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off sc0 sc1\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
// s_waitcnt vmcnt(<= n): waits for at most 3 more operations than asked.
__device__ __forceinline__ void vm_wait_le(int n) {
    if (n >= 60) asm volatile("s_waitcnt vmcnt(60)" ::: "memory");
    else if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
    else if (n >= 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
    else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else if (n >= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
    else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void tri_decode3(int e, int& k, int& m) {
    k = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
    if ((k + 1) * (k + 2) / 2 <= e) ++k;
    if (k * (k + 1) / 2 > e) --k;
    m = e - k * (k + 1) / 2;
}

// jcol in two halves, so the LDS read can be issued ahead of its use:
// jcol_load reads the one mean entry row k needs, jcol_sel forms J's entries.
template <int R>
__device__ __forceinline__ float jcol_load(const float* mu, int k) {
    constexpr int D = 2 + 2 * R;
    const int src = (k < 2 + R) ? (k + R) : (k - R);
    return mu[(k >= 2 && k < D) ? src : 0];
}
template <int R>
__device__ __forceinline__ void jcol_sel(float mv, bool exists, int k, double& j0, double& j1) {
    constexpr int D = 2 + 2 * R;
    const double v = (double)mv;
    j0 = !exists ? 0.0 : (k == 0) ? 1.0 : (k >= 2 && k < 2 + R) ? v : 0.0;
    j1 = !exists ? 0.0 : (k == 1) ? 1.0 : (k >= 2 + R && k < D) ? v : 0.0;
}

// J entries of a node for state index k, from its (fp32) mean in LDS:
// J = [[1, 0, V, 0], [0, 1, 0, U]]; zero when the node does not exist.
template <int R>
__device__ __forceinline__ void jcol(const float* mu, bool exists, int k, double& j0, double& j1) {
    constexpr int D = 2 + 2 * R;
    // branch-free: one unconditional LDS read, then selects
    const int src = (k < 2 + R) ? (k + R) : (k - R);
    const double v = (double)mu[(k >= 2 && k < D) ? src : 0];
    j0 = !exists ? 0.0 : (k == 0) ? 1.0 : (k >= 2 && k < 2 + R) ? v : 0.0;
    j1 = !exists ? 0.0 : (k == 1) ? 1.0 : (k >= 2 + R && k < D) ? v : 0.0;
}

__device__ __forceinline__ double dpp_add_xor1(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = dpp_partner<5>((uint32_t)b), hi = dpp_partner<5>((uint32_t)(b >> 32));
    return v + __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double dpp_add_mirror4(double v) {   // lane 0<->3, 1<->2
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = dpp_partner<4>((uint32_t)b), hi = dpp_partner<4>((uint32_t)(b >> 32));
    return v + __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}


}  // namespace ame
