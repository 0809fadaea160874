// Microbenchmark: gfx950 fp64 issue rates the covariance kernel (K2) depends on.
//   hipcc --offload-arch=gfx950 -O3 -o tools/_lib/probe_f64_rates tools/probe_f64_rates.hip
//   tools/_lib/probe_f64_rates
// (a) v_mfma_f64_16x16x4_f64, 4 independent accumulators per wave (throughput);
// (b) the same, one dependent chain (latency);
// (c) v_fma_f64, 8 independent chains per lane;
// (d) v_readlane_b32 pairs feeding v_fma_f64 (the pivot-row broadcast).
// Each kernel runs WAVES waves per SIMD on every CU; prints cycles per
// instruction per SIMD (from hipEvent time and the device clock).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

__global__ void __launch_bounds__(256) k_mfma_tp(double* out, double a, double b) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double x = a + threadIdx.x, y = b - threadIdx.x;
    for (int i = 0; i < ITERS; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, c3, 0, 0, 0);
    }
    d4 s = c0 + c1 + c2 + c3;
    if (s[0] == 12345.0) out[threadIdx.x] = s[1] + s[2] + s[3];
}

__global__ void __launch_bounds__(256) k_mfma_lat(double* out, double a, double b) {
    d4 c0 = {0, 0, 0, 0};
    double x = a + threadIdx.x, y = b - threadIdx.x;
    for (int i = 0; i < ITERS; ++i) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
    if (c0[0] == 12345.0) out[threadIdx.x] = c0[1] + c0[2] + c0[3];
}

__global__ void __launch_bounds__(256) k_fma(double* out, double a, double b) {
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = a + k + threadIdx.x;
    for (int i = 0; i < ITERS; ++i)
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = fma(v[k], b, a);
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
    if (s == 12345.0) out[threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_readlane(double* out, double a, double b) {
    double v = a + threadIdx.x, acc = 0;
    for (int i = 0; i < ITERS; ++i) {
        const unsigned long long u = (unsigned long long)__double_as_longlong(v);
        const int l = i & 63;
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
        const double s = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        acc = fma(s, b, acc);
        v = fma(v, b, a);
    }
    if (acc == 12345.0) out[threadIdx.x] = acc;
}

template <class K>
static void run(const char* name, K kern, int waves, int per_wave_instr, double* out) {
    int dev = 0, cus = 0, clk = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);   // kHz
    const int blocks = cus * waves;   // 4 waves per block = one per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0, 0.999);
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, 1.0, 0.999);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double cycles = ms * 1e-3 * clk * 1e3;
    const double per = cycles / ((double)waves * ITERS * per_wave_instr);
    printf("%-34s waves/SIMD %d: %.3f ms, %.1f cycles per instruction per SIMD (clock %d MHz)\n", name, waves, ms,
           per, clk / 1000);
}

int main() {
    double* out;
    if (hipMalloc(&out, 4096 * sizeof(double)) != hipSuccess) return 1;
    for (int w = 1; w <= 4; w *= 2) {
        run("mfma_f64_16x16x4, 4 chains", k_mfma_tp, w, 4, out);
        run("mfma_f64_16x16x4, 1 chain", k_mfma_lat, w, 1, out);
        run("v_fma_f64, 8 chains", k_fma, w, 8, out);
        run("readlane x2 + 2 fma", k_readlane, w, 1, out);
    }
    hipFree(out);
    return 0;
}
