// Device self-test of the wave/LDS primitives the sweep kernel is built on
// (ame_wave.h reduce-scatter, LDS-DMA placement).  Exported for the GPU test
// suite only (tests/test_gpu_primitives.py); not part of include/ame_amd.h.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ame_wave.h"

using namespace ame;

namespace {

__device__ __forceinline__ void dma16t(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void dma4t(const void* gsrc, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}

// out layout: [0..63] float idx, [64..127] float value, [128..191] double idx,
// [192..255] double value (as float), [256..] DMA readback
__global__ void selftest_kernel(const float* src, float* out) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    float vf[34];
#pragma unroll
    for (int q = 0; q < 34; ++q) vf[q] = (float)(lane * 3 + q);
    int idx;
    const float rf = wave_reduce_scatter<34>(vf, lane, idx);
    out[lane] = (float)idx;
    out[64 + lane] = rf;
    double vd[20];
#pragma unroll
    for (int q = 0; q < 20; ++q) vd[q] = (double)(lane * 5 + q) + 0.25;
    const double rd = wave_reduce_scatter<20>(vd, lane, idx);
    out[128 + lane] = (float)idx;
    out[192 + lane] = (float)rd;
    // DMA: 2 KiB with dwordx4 at LDS offset 1024, 256 B with dword at offset 4096
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
    dma16t(src + lane * 4, base + 1024);
    dma16t(src + 256 + lane * 4, base + 2048);
    dma4t(src + 600 + lane, base + 4096);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const float* l = (const float*)(smem + 1024);
    for (int e = lane; e < 512; e += 64) out[256 + e] = l[e];
    const float* l2 = (const float*)(smem + 4096);
    out[768 + lane] = l2[lane];
}

// CU hog (tests/test_gpu_coresidency.py): each workgroup holds `lds` bytes of
// LDS, so no sweep workgroup fits beside it on its CU, and sleeps until
// `ticks` of the 100 MHz clock have passed since it started; then it exits.
// Every wave reaches the exit on its own clock: the grid always drains.
__global__ void occupy_kernel(unsigned long long ticks, int* touched) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) smem[0] = 1;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(64);
    if (threadIdx.x == 0 && blockIdx.x == 0) *touched = (int)smem[0];
}

}  // namespace

// Diagnostic: `workgroups` one-wave workgroups of `lds_bytes` LDS each that stay
// resident for `microseconds` (at most 5 s), on `stream`.  Not part of
// include/ame_amd.h.
extern "C" int ame_debug_occupy(int workgroups, int lds_bytes, unsigned int microseconds, int* touched,
                                void* stream) {
    if (workgroups < 1 || workgroups > 4096 || lds_bytes < 0 || lds_bytes > 160 * 1024 ||
        microseconds > 5000000u || touched == nullptr)
        return -1;
    if (hipFuncSetAttribute((const void*)occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) !=
        hipSuccess)
        return -2;
    hipLaunchKernelGGL(occupy_kernel, dim3(workgroups), dim3(64), (size_t)lds_bytes, (hipStream_t)stream,
                       100ull * microseconds, touched);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

extern "C" int ame_debug_selftest(const float* src_dev, float* out_dev) {
    hipLaunchKernelGGL(selftest_kernel, dim3(1), dim3(64), 8192, 0, src_dev, out_dev);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -2;
}
