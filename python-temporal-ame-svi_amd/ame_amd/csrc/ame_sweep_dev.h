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
// The slow path of lds_wait_ge (AmeSpin rules), out of line: inlined, its
// record stores cost the v3 solver loop VGPR spills.  Returns the counter's
// value, with AME_LDS_DEAD set when the wait failed or gave up (one wave).
static __device__ __attribute__((noinline)) uint32_t lds_wait_slow(uint32_t* f, uint32_t target, uint32_t* status,
                                                                   int slice, uint32_t node, uint32_t epoch) {
    const bool ld = (threadIdx.x & 63) == 0;
    AmeSpin w(status, false, ld);
    uint32_t v;
    while ((v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < target) {
        __builtin_amdgcn_s_sleep(1);
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
#ifdef AME_R6_LDS_SIMPLE
    if (!dead && v < target) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while ((v = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > AME_SPIN_TICKS_LOCAL) {
                if ((threadIdx.x & 63) == 0) atomicOr(status, AME_STATUS_LDS_TIMEOUT);
                dead = true;
                break;
            }
        }
    }
#else
    if (!dead && v < target) v = lds_wait_slow(f, target, status, slice, node, epoch);
#endif
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
