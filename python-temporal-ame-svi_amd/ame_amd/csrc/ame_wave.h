// Wave-level building blocks for the gfx950 sweep kernel (ame_sweep3.hip):
// cross-lane reduce-scatter on 64-lane waves and 2x2 symmetric algebra.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ame {

// ---- 32-bit lane exchanges ----------------------------------------------
// Stage s of a 6-stage reduce-scatter pairs lanes that differ in bit (5 - s):
//   s=0 bit 5: v_permlane32_swap   s=1 bit 4: v_permlane16_swap
//   s=2 bit 3: DPP row_mirror      s=3 bit 2: DPP row_half_mirror
//   s=4 bit 1: DPP quad_perm 3210  s=5 bit 0: DPP quad_perm 1032
// Every DPP pattern used is an involution inside its row, and partners always
// differ in the stage's bit, so "keep A if bit==0 else B" pairs up exactly.
template <int S>
__device__ __forceinline__ uint32_t dpp_partner(uint32_t x) {
    if constexpr (S == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);
    else if constexpr (S == 3) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x141, 0xF, 0xF, false);
    else if constexpr (S == 4) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x1B, 0xF, 0xF, false);
    else return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);
}

// Lane l's value on every lane (v_readlane into SGPRs: no LDS round trip,
// unlike __shfl's ds_bpermute); l is a compile-time or wave-uniform index.
__device__ __forceinline__ double lane_bcast(double v, int l) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Sum over aligned groups of G = 2, 4 or 8 lanes, left on every lane of the
// group (DPP, no LDS round trip).  quad_perm 1032 pairs lanes differing in bit
// 0; quad_perm 3210 then adds the other pair's sum, row_half_mirror the other
// quad's: each step adds a partner holding the same partial sums an xor
// exchange (__shfl_xor 1, 2, 4) would deliver, and + commutes exactly, so lane
// results are bit-identical to the xor tree.
template <int S>
__device__ __forceinline__ double dpp_partner_d(double x) {
    const uint64_t u = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = dpp_partner<S>((uint32_t)u), hi = dpp_partner<S>((uint32_t)(u >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int G>
__device__ __forceinline__ double group_sum(double v) {
    static_assert(G == 2 || G == 4 || G == 8, "group_sum: G in {2, 4, 8}");
    v += dpp_partner_d<5>(v);
    if constexpr (G >= 4) v += dpp_partner_d<4>(v);
    if constexpr (G >= 8) v += dpp_partner_d<3>(v);
    return v;
}

// One pair step: lanes with bit==0 return A_own + A_partner, bit==1 lanes
// return B_own + B_partner.
template <int S>
__device__ __forceinline__ float pair_step(float A, float B, bool hi) {
    if constexpr (S == 0) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(A), __float_as_uint(B), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else if constexpr (S == 1) {
        auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(A), __float_as_uint(B), false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    } else {
        const float send = hi ? A : B, keep = hi ? B : A;
        return keep + __uint_as_float(dpp_partner<S>(__float_as_uint(send)));
    }
}

template <int S>
__device__ __forceinline__ double pair_step(double A, double B, bool hi) {
    const uint64_t a = (uint64_t)__double_as_longlong(A), b = (uint64_t)__double_as_longlong(B);
    const uint32_t alo = (uint32_t)a, ahi = (uint32_t)(a >> 32);
    const uint32_t blo = (uint32_t)b, bhi = (uint32_t)(b >> 32);
    if constexpr (S <= 1) {
        uint32_t x0, x1, y0, y1;
        if constexpr (S == 0) {
            auto l = __builtin_amdgcn_permlane32_swap(alo, blo, false, false);
            auto h = __builtin_amdgcn_permlane32_swap(ahi, bhi, false, false);
            x0 = l[0]; y0 = l[1]; x1 = h[0]; y1 = h[1];
        } else {
            auto l = __builtin_amdgcn_permlane16_swap(alo, blo, false, false);
            auto h = __builtin_amdgcn_permlane16_swap(ahi, bhi, false, false);
            x0 = l[0]; y0 = l[1]; x1 = h[0]; y1 = h[1];
        }
        const double X = __longlong_as_double((long long)(((uint64_t)x1 << 32) | x0));
        const double Y = __longlong_as_double((long long)(((uint64_t)y1 << 32) | y0));
        return X + Y;
    } else {
        const uint32_t slo = hi ? alo : blo, shi = hi ? ahi : bhi;
        const uint32_t rlo = dpp_partner<S>(slo), rhi = dpp_partner<S>(shi);
        const double recv = __longlong_as_double((long long)(((uint64_t)rhi << 32) | rlo));
        return (hi ? B : A) + recv;
    }
}

// `cnt` = how many of this lane's current values are real (the rest pad): the
// upper half of an odd-length array is one short, so its last slot is padding
// whose computed index would collide with a real index further up the tree.
template <int S, int C, typename T>
__device__ __forceinline__ void rs_stages(T* v, int lane, int& idx, int& cnt) {
    if constexpr (S < 6) {
        constexpr int H = (C + 1) / 2;
        const bool hi = (lane >> (5 - S)) & 1;
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const T A = v[j];
            const T B = (j + H < C) ? v[j + H] : T(0);
            v[j] = pair_step<S>(A, B, hi);
        }
        if (hi) {
            idx += H;
            cnt = cnt > H ? cnt - H : 0;
        } else {
            cnt = cnt < H ? cnt : H;
        }
        rs_stages<S + 1, H, T>(v, lane, idx, cnt);
    }
}

// Reduce-scatter NV values over the 64 lanes of a wave (fixed tree, so the
// result is deterministic).  Returns the value this lane ends up owning and
// its index via idx; idx == NV means the lane owns padding.  Each index in
// [0, NV) is owned by exactly one lane.  Every lane of the wave must execute
// it (EXEC full).
template <int NV, typename T>
__device__ __forceinline__ T wave_reduce_scatter(T (&v)[NV], int lane, int& idx) {
    idx = 0;
    int cnt = NV;
    rs_stages<0, NV, T>(v, lane, idx, cnt);
    if (cnt < 1) idx = NV;
    return v[0];
}

// ---- 2x2 algebra (fp64) ---------------------------------------------------
struct Mat2 {
    double a, b, c, d;   // [[a b][c d]]
};
__device__ __forceinline__ Mat2 m2(double a, double b, double c, double d) { return Mat2{a, b, c, d}; }
__device__ __forceinline__ Mat2 add(Mat2 x, Mat2 y) { return {x.a + y.a, x.b + y.b, x.c + y.c, x.d + y.d}; }
__device__ __forceinline__ Mat2 sub(Mat2 x, Mat2 y) { return {x.a - y.a, x.b - y.b, x.c - y.c, x.d - y.d}; }
__device__ __forceinline__ Mat2 tr(Mat2 x) { return {x.a, x.c, x.b, x.d}; }
__device__ __forceinline__ Mat2 mul(Mat2 x, Mat2 y) {
    return {x.a * y.a + x.b * y.c, x.a * y.b + x.b * y.d, x.c * y.a + x.d * y.c, x.c * y.b + x.d * y.d};
}
// X^T S Y
__device__ __forceinline__ Mat2 quad(Mat2 x, Mat2 s, Mat2 y) { return mul(tr(x), mul(s, y)); }
__device__ __forceinline__ Mat2 sym(Mat2 x) {
    const double o = 0.5 * (x.b + x.c);
    return {x.a, o, o, x.d};
}
// inverse with the off-diagonal symmetrised afterwards
__device__ __forceinline__ Mat2 inv2s(Mat2 m) {
    const double id = 1.0 / (m.a * m.d - m.b * m.c);
    const double o = 0.5 * (-m.b * id - m.c * id);
    return {m.d * id, o, o, m.a * id};
}
struct V2 {
    double x, y;
};
__device__ __forceinline__ V2 mv(Mat2 m, V2 v) { return {m.a * v.x + m.b * v.y, m.c * v.x + m.d * v.y}; }
// X^T v
__device__ __forceinline__ V2 mtv(Mat2 m, V2 v) { return {m.a * v.x + m.c * v.y, m.b * v.x + m.d * v.y}; }

}  // namespace ame
