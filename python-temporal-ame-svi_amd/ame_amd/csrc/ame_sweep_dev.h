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
// Bounded: a wait that outlives AME_SPIN_TICKS_LOCAL sets AME_STATUS_LDS_TIMEOUT
// and gives up (the launch then finishes with wrong values, never hangs).
__device__ __forceinline__ void lds_wait_ge(uint32_t* f, uint32_t target, uint32_t* status, bool& dead) {
    if (!dead && __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > AME_SPIN_TICKS_LOCAL) {
                if ((threadIdx.x & 63) == 0) atomicOr(status, AME_STATUS_LDS_TIMEOUT);
                dead = true;
                break;
            }
        }
    }
    asm volatile("" ::: "memory");
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
