// K0 (Y relayout) and K2/K3 (ELBO + reconstruction sufficient sums).
//
// Reference:
//   _compute_expected_log_likelihood  structured_mf.py:124-150 (naive_mf.py:114-132)
//   StaticAMEModel.compute_mean        static_ame.py:189-238
//   _compute_log_prior_initial         structured_mf.py:152-173
//   _compute_log_prior_transitions     structured_mf.py:175-200
//   compute_temporal_reconstruction_error  temporal_ame.py:255-291
//
// K2 walks 64x64 (i-block, j-block) tiles of one time slice.  The plug-in mean
// m_ij = [a_i + b_j + U_i.V_j, a_j + b_i + U_j.V_i] needs G1 = U_I V_J^T and
// G2^T = V_I U_J^T on the same (i,j) -> one f32 MFMA (v_mfma_f32_16x16x4_f32,
// exact f32) chain each per 16x16 sub-tile, so both land in the same lane and
// register.  The residual quadratic form and squared error are fused into the
// epilogue while the tile's Y bytes stream in once.  When Y is swap-consistent
// (Y_ji = swap(Y_ij), checked by K0) only the upper-triangle tiles are read and
// the mirror half of the reconstruction error is counted twice.
#include "ame_common.h"
#include "ame_sweep_dev.h"
#include <type_traits>
using namespace ame;

// ---------------------------------------------------------------------------
// K0: Y [n][n][T_total][2] -> Yt [T_local][n][ny][2] (ny = ame_ystride(n), the
// pad pair zero); count swap mismatches.
// ---------------------------------------------------------------------------
#if AME_PART0
__global__ void __launch_bounds__(AME_NT)
ame_pack_kernel(const float* __restrict__ Y, float* __restrict__ Yt, ame_dims dm,
                unsigned long long* mismatch) {
    const int n = dm.n, TL = dm.T_local, Tt = dm.T_total, ny = ame_ystride(n);
    const size_t total = (size_t)TL * n * ny;
    unsigned long long bad = 0;
    for (size_t idx = (size_t)blockIdx.x * AME_NT + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * AME_NT) {
        const int j = (int)(idx % ny);
        const size_t r = idx / ny;
        const int i = (int)(r % n);
        const int tl = (int)(r / n);
        const int tg = dm.t_begin + tl;
        if (j >= n) {   // pad pair
            *(float2*)(Yt + idx * 2) = make_float2(0.f, 0.f);
            continue;
        }
        const float2 y = *(const float2*)(Y + (((size_t)i * n + j) * Tt + tg) * 2);
        *(float2*)(Yt + idx * 2) = y;
        if (i < j && mismatch != nullptr) {
            const float2 yt = *(const float2*)(Y + (((size_t)j * n + i) * Tt + tg) * 2);
            if (__float_as_uint(yt.x) != __float_as_uint(y.y) ||
                __float_as_uint(yt.y) != __float_as_uint(y.x))
                ++bad;
        }
    }
    if (mismatch != nullptr && bad) atomicAdd(mismatch, bad);
}

int ame_pack_dispatch(const float* Y, float* Yt, const ame_dims* dm, unsigned long long* mm,
                      hipStream_t st) {
    const size_t total = (size_t)dm->T_local * dm->n * ame_ystride(dm->n);
    size_t blocks = (total + AME_NT - 1) / AME_NT;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(ame_pack_kernel, dim3((unsigned)blocks), dim3(AME_NT), 0, st, Y, Yt, *dm,
                       mm);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

#endif

// ---------------------------------------------------------------------------
// K2: pair terms.  work layout: [nwg][2] = {sum quad (i<j), sum sq-err}
//
// One workgroup walks whole 64-row strips of one slice: when Y is
// swap-consistent, strip s and strip nb-1-s (the upper-triangle tiles J >= I
// of both: nb + 1 tiles, so every workgroup gets the same work); otherwise one
// strip over all nb tiles.  Wave w owns rows I0 + 16w .. +15 of the strip and
// keeps U_I, V_I (its MFMA B operands) and a_I, b_I in registers for the whole
// strip; the column tile's U_J, V_J, a_J, b_J are staged in LDS (double
// buffered, one barrier per tile).  The products are formed transposed,
//   G1^T = V_J U_I^T,  G2^T = U_J V_I^T   (v_mfma_f32_16x16x4_f32, exact f32),
// with the A operand rows permuted so that a lane's 4 accumulator values are
// columns {2lq, 2lq+1, 8+2lq, 9+2lq} of one row i: its Y values are two 16-byte
// loads and the 4 lanes of a row cover 64 contiguous bytes.  Y streams in half
// tiles (two 16x16 sub-tiles) through two rotating register buffers, so the
// next half is in flight while the current one is consumed.
// ---------------------------------------------------------------------------
#define AME_TILE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int R>
__global__ void __launch_bounds__(AME_NT, (R <= 16) ? 4 : 2)   // r <= 16: 4 waves / SIMD, all strips resident
ame_pairs_kernel(ame_dims dm, const float* __restrict__ Yt, const float* __restrict__ x,
                 double r00, double r01, double r10, double r11, int swap_mode,
                 double* __restrict__ partial) {
    constexpr int D = 2 + 2 * R;
    constexpr int RP = (R + 3) & ~3;   // MFMA K padded to 4
    constexpr int LD = RP + 1;         // LDS row stride (bank spread)
    const int n = dm.n;
    const int nb = (n + AME_TILE - 1) / AME_TILE;
    const int nws = swap_mode ? (nb + 1) / 2 : nb;     // workgroups per slice
    // XCD-aware: workgroup b runs on XCD b % 8; all workgroups of one slice
    // share an XCD, so its U, V are fetched into one L2 instead of eight
    const int b = blockIdx.x;
    int tl, s;
    if ((dm.T_local & 7) == 0) {
        const int k = b >> 3, q = k / nws;
        tl = (b & 7) * (dm.T_local >> 3) + q;
        s = k - q * nws;
    } else {
        tl = b / nws;
        s = b - tl * nws;
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int li = lane & 15, lq = lane >> 4;

    __shared__ float UJ[2][AME_TILE * LD], VJ[2][AME_TILE * LD];
    __shared__ float aJ[2][AME_TILE], bJ[2][AME_TILE];
    __shared__ double red[8];

    const int ny = ame_ystride(n);
    const float* xs = x + (size_t)tl * n * D;
    const float* ys = Yt + (size_t)tl * n * ny * 2;
    const float p = (float)r00, q01 = (float)r01, q10 = (float)r10, sr = (float)r11;

    // staging of a column tile's U, V, a, b: global loads into registers first
    // (issued a tile ahead), LDS stores after the current tile's compute
    constexpr int SQ = (AME_TILE * RP + AME_NT - 1) / AME_NT;
    float su[SQ], sv[SQ], sa = 0.f, sb = 0.f;
    auto stage_load = [&](int J) {
        const int J0 = J * AME_TILE;
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
            const int idx = threadIdx.x + AME_NT * q;
            const int row = idx / RP, k = idx - row * RP;
            const int jj = J0 + row;
            const bool ok = idx < AME_TILE * RP && k < R && jj < n;
            su[q] = ok ? xs[(size_t)jj * D + 2 + k] : 0.f;
            sv[q] = ok ? xs[(size_t)jj * D + 2 + R + k] : 0.f;
        }
        if (threadIdx.x < AME_TILE) {
            const int jj = J0 + threadIdx.x;
            sa = jj < n ? xs[(size_t)jj * D + 0] : 0.f;
            sb = jj < n ? xs[(size_t)jj * D + 1] : 0.f;
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < SQ; ++q) {
            const int idx = threadIdx.x + AME_NT * q;
            if (idx < AME_TILE * RP) {
                const int row = idx / RP, k = idx - row * RP;
                UJ[buf][row * LD + k] = su[q];
                VJ[buf][row * LD + k] = sv[q];
            }
        }
        if (threadIdx.x < AME_TILE) {
            aJ[buf][threadIdx.x] = sa;
            bJ[buf][threadIdx.x] = sb;
        }
    };
    auto stage = [&](int J, int buf) {
        stage_load(J);
        stage_store(buf);
    };

    double quad = 0.0, sq = 0.0;
    const int nstrip = (swap_mode && nb - 1 - s != s) ? 2 : 1;
    for (int st = 0; st < nstrip; ++st) {
        const int I = (st == 0) ? s : nb - 1 - s;
        const int I0 = I * AME_TILE;
        const int i = I0 + 16 * w + li;          // this lane's row (C column)
        const bool irow = i < n;
        // B operands: U_I / V_I [row i][k0 + lq]; lane's own a_i, b_i
        float bu[RP / 4], bv[RP / 4];
#pragma unroll
        for (int kk = 0; kk < RP / 4; ++kk) {
            const int k = 4 * kk + lq;
            bu[kk] = (irow && k < R) ? xs[(size_t)i * D + 2 + k] : 0.f;
            bv[kk] = (irow && k < R) ? xs[(size_t)i * D + 2 + R + k] : 0.f;
        }
        const float ai = irow ? xs[(size_t)i * D + 0] : 0.f;
        const float bi = irow ? xs[(size_t)i * D + 1] : 0.f;
        const int Jb = swap_mode ? I : 0;
        __syncthreads();   // the previous strip's last tile is done with both buffers
        stage(Jb, 0);
        __syncthreads();
        // Y of half a tile (sub-tiles 2 hf, 2 hf + 1) of tile J: row i, columns
        // J0 + 16 sub + {2 lq, 2 lq + 1} and {8 + 2 lq, 9 + 2 lq}; each 16-byte load of
        // a wave covers 64 contiguous bytes of 16 rows (the A operand rows are
        // permuted to match, below).  Half tiles rotate through two register
        // buffers: the next half is always in flight behind the one being used.
        auto load_half = [&](int J, int hf, float4 (&y)[2][2]) {
            const int J0 = J * AME_TILE;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int j0 = J0 + 16 * (2 * hf + s2) + 8 * h + 2 * lq;
                    if (irow && j0 + 2 <= n) {
                        // default cache policy: non-temporal loads measured slower here
                        // (166 vs 155 us at config 3)
                        y[s2][h] = *(const float4*)(ys + ((size_t)i * ny + j0) * 2);
                    } else {                                  // row end / odd n: per element
                        float t[4];
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const bool ok = irow && j0 + e < n;
                            const float2 v = ok ? *(const float2*)(ys + ((size_t)i * ny + j0 + e) * 2)
                                                : make_float2(0.f, 0.f);
                            t[2 * e] = v.x;
                            t[2 * e + 1] = v.y;
                        }
                        y[s2][h] = make_float4(t[0], t[1], t[2], t[3]);
                    }
                }
            }
        };
        float tq = 0.f, ts = 0.f;
        auto half = [&](int J, int hf, int buf, const float4 (&y)[2][2]) {
            const int J0 = J * AME_TILE;
#pragma unroll
            for (int s2 = 0; s2 < 2; ++s2) {
                const int sub = 2 * hf + s2;
                f32x4 g1 = {0.f, 0.f, 0.f, 0.f}, g2 = {0.f, 0.f, 0.f, 0.f};
                // A operand row r = li holds column perm(r) = 2(r>>2) + (r&1) + 8((r>>1)&1),
                // so accumulator v of lane (li, lq) is column 2 lq + (v&1) + 8 (v>>1)
                const int jr = 16 * sub + 2 * (li >> 2) + (li & 1) + 8 * ((li >> 1) & 1);
#pragma unroll
                for (int kk = 0; kk < RP / 4; ++kk) {
                    const float av = VJ[buf][jr * LD + 4 * kk + lq];
                    const float au = UJ[buf][jr * LD + 4 * kk + lq];
                    g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bu[kk], g1, 0, 0, 0);
                    g2 = __builtin_amdgcn_mfma_f32_16x16x4f32(au, bv[kk], g2, 0, 0, 0);
                }
                const float yv[8] = {y[s2][0].x, y[s2][0].y, y[s2][0].z, y[s2][0].w,
                                     y[s2][1].x, y[s2][1].y, y[s2][1].z, y[s2][1].w};
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int jl = 16 * sub + 2 * lq + (v & 1) + 8 * (v >> 1);
                    const int j = J0 + jl;
                    if (!irow || j >= n || i == j) continue;
                    if (swap_mode && i > j) continue;
                    const float mu0 = (ai + bJ[buf][jl]) + g1[v];
                    const float mu1 = (aJ[buf][jl] + bi) + g2[v];
                    const float e0 = yv[2 * v] - mu0, e1 = yv[2 * v + 1] - mu1;
                    const float se = e0 * e0 + e1 * e1;
                    if (i < j) {
                        tq += e0 * (p * e0 + q01 * e1) + e1 * (q10 * e0 + sr * e1);
                        ts += swap_mode ? 2.f * se : se;
                    } else {
                        ts += se;
                    }
                }
            }
        };
        float4 y0[2][2], y1[2][2];
        load_half(Jb, 0, y0);
        for (int J = Jb; J < nb; ++J) {
            const int buf = (J - Jb) & 1;
            if (J + 1 < nb) stage_load(J + 1);
            load_half(J, 1, y1);
            half(J, 0, buf, y0);
            if (J + 1 < nb) load_half(J + 1, 0, y0);
            half(J, 1, buf, y1);
            quad += (double)tq;      // this tile's sums (<= 16 terms per lane)
            sq += (double)ts;
            tq = ts = 0.f;
            if (J + 1 < nb) stage_store(buf ^ 1);
            __syncthreads();
        }
    }
    double v2[2] = {quad, sq};
    block_sum<2>(v2, red);
    if (threadIdx.x == 0) {
        partial[(size_t)blockIdx.x * 2 + 0] = v2[0];
        partial[(size_t)blockIdx.x * 2 + 1] = v2[1];
    }
}

// ---------------------------------------------------------------------------
// K2 v2 (n even): the same tiles, products and sums as ame_pairs_kernel, but
// every byte arrives by LDS-DMA (global_load_lds), so no VGPR holds a load in
// flight and the count of outstanding loads is known exactly:
//  * Y: each wave streams its own 16 rows in half tiles (16 rows x 32 columns =
//    4 KiB = 4 DMA instructions, each 4 rows x 256 contiguous bytes) through a
//    private LDS ring (AME_P2_NSLOT slots), NSLOT - 1 half tiles ahead of the
//    one it computes.
//    Within a row the 16-byte chunks are stored XOR-swizzled by the row
//    (position p holds chunk p ^ row), so the accumulator-order ds_read_b128 of
//    16 rows hits 16 distinct bank groups; a wave waits only for its own DMA.
//  * U_J, V_J, a_J, b_J of the next column tile: 4-byte DMA into the other of
//    two staging buffers, [U rows (stride LD) | V rows | a | b] = 2 (RP + 2)
//    instructions, spread over the 4 waves, landed by the end-of-tile barrier.
// The DMA issue order is the same for every wave and every tile (missing tiles
// are issued as dummy loads into slots nobody reads), so one fixed vmcnt per
// wait is exact.
// ---------------------------------------------------------------------------
template <int R>
struct Pairs2 {
    static constexpr int RP = (R + 3) & ~3, LD = RP + 1;
    static constexpr int SF = 2 * AME_TILE * LD + 2 * AME_TILE;   // staging floats per buffer
    static constexpr int NUV = SF / 64;                             // 4-byte DMA instructions per buffer
    static constexpr int NUW = NUV / 4;                             // ... per wave
// 2 slots (one half tile in flight while one is computed) keep the LDS at
// 50 KB, so 3 workgroups share a CU: 109 us at config 3 vs 117 us with 3 slots
// and 2 workgroups per CU (profiles/r02_pairs_nslot.txt)
#ifndef AME_P2_NSLOT
#define AME_P2_NSLOT 2
#endif
    static constexpr int NSLOT = AME_P2_NSLOT, SLOTB = 4096;   // half-tile slots per wave
    static constexpr int AHEAD = NSLOT - 1;                      // half tiles in flight
    static_assert(SF % 256 == 0, "staging must split evenly over 4 waves");
    static_assert(4 * AHEAD + NUW <= 63, "vmcnt range");
};

template <int R>
__global__ void __launch_bounds__(AME_NT, (AME_P2_NSLOT <= 2 && R <= 16) ? 3 : 2)
ame_pairs2_kernel(ame_dims dm, const float* __restrict__ Yt, const float* __restrict__ x,
                  double r00, double r01, double r10, double r11, int swap_mode,
                  double* __restrict__ partial) {
    using P2 = Pairs2<R>;
    constexpr int D = 2 + 2 * R;
    constexpr int RP = P2::RP, LD = P2::LD, SF = P2::SF, NUW = P2::NUW, NSLOT = P2::NSLOT, AHEAD = P2::AHEAD;
    const int n = dm.n;
    const int nb = (n + AME_TILE - 1) / AME_TILE;
    const int nws = swap_mode ? (nb + 1) / 2 : nb;
    const int b = blockIdx.x;
    int tl, s;
    if ((dm.T_local & 7) == 0) {   // XCD-aware, as ame_pairs_kernel
        const int k = b >> 3, q = k / nws;
        tl = (b & 7) * (dm.T_local >> 3) + q;
        s = k - q * nws;
    } else {
        tl = b / nws;
        s = b - tl * nws;
    }
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int li = lane & 15, lq = lane >> 4;

    __shared__ __attribute__((aligned(16))) float stg[2][SF];
    __shared__ __attribute__((aligned(16))) char yl[4][NSLOT][P2::SLOTB];
    __shared__ double red[8];

    const int ny = ame_ystride(n);   // even: every row 16-byte aligned
    const float* xs = x + (size_t)tl * n * D;
    const float* ys = Yt + (size_t)tl * n * ny * 2;

    // tile sequence of this workgroup: swap mode walks strip s (J >= s) then
    // strip nb-1-s (J >= nb-1-s); otherwise strip s over all J
    const int sB = nb - 1 - s;
    const int nA = swap_mode ? nb - s : nb;
    const int NT = swap_mode ? (sB != s ? nA + (s + 1) : nA) : nb;
    auto tile = [&](int tt, int& I, int& J) {
        if (tt < nA) { I = s; J = (swap_mode ? s : 0) + tt; }
        else { I = sB; J = sB + (tt - nA); }
    };

    // ---- DMA issue (each call: a fixed instruction count per wave) ----
    // lane-constant parts of the DMA addresses, formed once
    int yoff[4], yrr[4], ygc[4];   // Y: row / chunk of this lane in instruction u, offset in floats
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        yrr[u] = 4 * u + (lane >> 4);
        ygc[u] = (lane & 15) ^ yrr[u];
        yoff[u] = (yrr[u] * ny + 2 * ygc[u]) * 2;
    }
    int uoff[NUW], urow[NUW];      // staging: offset from row J0 (floats), row (>= 2^20: pad)
#pragma unroll
    for (int c = 0; c < NUW; ++c) {
        const int f = (w * NUW + c) * 64 + lane;
        if (f < 2 * AME_TILE * LD) {
            const int mat = f / (AME_TILE * LD), g = f - mat * (AME_TILE * LD);
            const int row = g / LD, k = g - row * LD;
            const bool ok = k < R;
            uoff[c] = ok ? row * D + 2 + mat * R + k : 0;
            urow[c] = ok ? row : (1 << 20);
        } else {
            const int g = f - 2 * AME_TILE * LD, ab = g / AME_TILE, row = g - ab * AME_TILE;
            uoff[c] = row * D + ab;
            urow[c] = row;
        }
    }

    // ---- DMA issue (each call: a fixed instruction count per wave) ----
    auto issue_y = [&](int q) {   // half tile q -> this wave's slot q % NSLOT : 4 instructions
        const int tt = q >> 1, hf = q & 1;
        int I = 0, J = 0;
        const bool real = tt < NT;
        if (real) tile(tt, I, J);
        const int c0 = J * AME_TILE + 32 * hf, r0 = I * AME_TILE + 16 * w;
        const float* base = ys + ((size_t)r0 * ny + c0) * 2;
        const uint32_t dst = lds_off(&yl[w][q % NSLOT][0]);
        const bool diag = swap_mode && I == J;
        if (real && !diag && r0 + 16 <= n && c0 + 32 <= n) {
#pragma unroll
            for (int u = 0; u < 4; ++u) dma16(base + yoff[u], dst + u * 1024);
        } else {
            // edge or diagonal tile: chunks outside the slice, and on a diagonal
            // tile of the upper-triangle walk the chunks no pair i < j needs
            // (j + 1 <= i), read the slice's first (cached) bytes instead
            const int lr = real ? n - r0 : 0, lc = real ? n - c0 : 0;
            const int dd = diag ? r0 - c0 : -(1 << 20);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const bool ok = yrr[u] < lr && 2 * ygc[u] < lc && 2 * ygc[u] + 1 > dd + yrr[u];
                dma16(ok ? base + yoff[u] : ys, dst + u * 1024);
            }
        }
    };
    auto issue_uv = [&](int tt) {   // column tile of tile tt -> stg[tt & 1] : NUW instructions
        int I = 0, J = 0;
        if (tt < NT) tile(tt, I, J);
        const int J0 = J * AME_TILE;
        const float* base = xs + (size_t)J0 * D;
        const int lr = (tt < NT) ? n - J0 : 0;
        const uint32_t dst = lds_off(&stg[tt & 1][w * NUW * 64]);   // wave-uniform (readfirstlane)
#pragma unroll
        for (int c = 0; c < NUW; ++c) dma4(urow[c] < lr ? base + uoff[c] : xs, dst + (uint32_t)(c * 256));
    };

    // B operands of both strips: K chunks of U_I / V_I (rows i, k = 4 kk + lq),
    // then one extra chunk that folds the additive terms into the products:
    //   ch 0: [U_i, a_i, 1, 0] . [V_j, 1, b_j, 0] = a_i + b_j + U_i.V_j
    //   ch 1: [V_i, 1, b_i, 0] . [U_j, a_j, 1, 0] = a_j + b_i + U_j.V_i
    constexpr int KC = RP / 4 + 1;
    float bu[2][KC], bv[2][KC];
    bool irow2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int I = (h == 0) ? s : sB;
        const int i = I * AME_TILE + 16 * w + li;
        const bool irow = i < n && I < nb;
        irow2[h] = irow;
#pragma unroll
        for (int kk = 0; kk < RP / 4; ++kk) {
            const int k = 4 * kk + lq;
            bu[h][kk] = (irow && k < R) ? xs[(size_t)i * D + 2 + k] : 0.f;
            bv[h][kk] = (irow && k < R) ? xs[(size_t)i * D + 2 + R + k] : 0.f;
        }
        const float ai = irow ? xs[(size_t)i * D + 0] : 0.f;
        const float bi = irow ? xs[(size_t)i * D + 1] : 0.f;
        bu[h][KC - 1] = (lq == 0) ? ai : (lq == 1) ? 1.f : 0.f;
        bv[h][KC - 1] = (lq == 0) ? 1.f : (lq == 1) ? bi : 0.f;
    }

    issue_uv(0);
#pragma unroll
    for (int q = 0; q < AHEAD; ++q) issue_y(q);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * AHEAD) : "memory");   // staging of tile 0
    lds_barrier3();   // LDS-only barrier: the Y prefetch stays in flight

    // residual sufficient statistics, packed over two columns (v_pk_fma_f32):
    // pairs with i < j -> A00 = sum e0^2, A01 = sum e0 e1, A11 = sum e1^2;
    // i > j (only when Y is not swap-consistent) -> S = sum e0^2 + e1^2
    const double p = r00, qs = r01 + r10, sr = r11;
    double quad = 0.0, sq = 0.0;
    for (int tt = 0; tt < NT; ++tt) {
        int I, J;
        tile(tt, I, J);
        const int h = (tt < nA) ? 0 : 1;
        const int i = I * AME_TILE + 16 * w + li;
        const bool irow = irow2[h];
        const int J0 = J * AME_TILE;
        const float* UJ = &stg[tt & 1][0];
        const float* VJ = UJ + AME_TILE * LD;
        const float* aJ = VJ + AME_TILE * LD;
        const float* bJ = aJ + AME_TILE;
        // uniform tile class: every pair valid with i < j (interior, above the
        // diagonal), every pair valid with i > j (non-swap, below), or mixed
        const bool upper = J > I && J0 + AME_TILE <= n;
        const bool lower = !swap_mode && J < I && (I + 1) * AME_TILE <= n;
        issue_uv(tt + 1);   // its buffer was last read by tile tt - 1 (barrier since)
        f32x2 A00 = {0.f, 0.f}, A01 = {0.f, 0.f}, A11 = {0.f, 0.f}, S = {0.f, 0.f};
        // one copy of the tile body per class (MODE 0 upper, 1 lower, 2 mixed),
        // so the class test is one branch per tile
        auto tile_body = [&](auto mode) {
            constexpr int MODE = decltype(mode)::value;
#pragma unroll
            for (int hf = 0; hf < 2; ++hf) {
                const int q = 2 * tt + hf;
                issue_y(q + AHEAD);
                // outstanding after half q: halves q+1 .. q+AHEAD (4 each) and, at
                // hf 0, the staging of tile tt+1 (NUW); at hf 1 that has landed too
                if (hf == 0) {
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * AHEAD + NUW) : "memory");
                } else {
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * AHEAD) : "memory");
                }
                const float* ysl = (const float*)&yl[w][q % NSLOT][0] + li * 64;
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) {
                    const int sub = 2 * hf + s2;
                    f32x4 g1 = {0.f, 0.f, 0.f, 0.f}, g2 = {0.f, 0.f, 0.f, 0.f};
                    const int jr = 16 * sub + 2 * (li >> 2) + (li & 1) + 8 * ((li >> 1) & 1);
#pragma unroll
                    for (int kk = 0; kk < RP / 4; ++kk) {
                        const float av = VJ[jr * LD + 4 * kk + lq];
                        const float au = UJ[jr * LD + 4 * kk + lq];
                        g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bu[h][kk], g1, 0, 0, 0);
                        g2 = __builtin_amdgcn_mfma_f32_16x16x4f32(au, bv[h][kk], g2, 0, 0, 0);
                    }
                    {   // fold chunk: A rows [1, b_j, 0, 0] (ch 0) and [a_j, 1, 0, 0] (ch 1)
                        const float ab = (lq == 1) ? bJ[jr] : aJ[jr];
                        const float av = (lq == 0) ? 1.f : (lq == 1) ? ab : 0.f;
                        const float au = (lq == 0) ? ab : (lq == 1) ? 1.f : 0.f;
                        g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bu[h][KC - 1], g1, 0, 0, 0);
                        g2 = __builtin_amdgcn_mfma_f32_16x16x4f32(au, bv[h][KC - 1], g2, 0, 0, 0);
                    }
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                        // columns 16 sub + 8 hh + 2 lq, +1: chunk 8 s2 + 4 hh + lq of the
                        // half (16 B = {ch0, ch1} of two columns), stored at position ^ li
                        const float* yc = ysl + ((((8 * s2 + 4 * hh + lq) ^ li)) << 2);
                        const f32x2 y0 = {yc[0], yc[2]}, y1 = {yc[1], yc[3]};   // ds_read2_b32 x 2
                        const f32x2 m0 = {g1[2 * hh], g1[2 * hh + 1]}, m1 = {g2[2 * hh], g2[2 * hh + 1]};
                        const f32x2 e0 = y0 - m0, e1 = y1 - m1;
                        if constexpr (MODE == 0) {
                            A00 += e0 * e0;
                            A01 += e0 * e1;
                            A11 += e1 * e1;
                        } else if constexpr (MODE == 1) {
                            S += e0 * e0;
                            S += e1 * e1;
                        } else {
                            const int j = J0 + 16 * sub + 8 * hh + 2 * lq;
                            const bool v0 = irow && j < n && i != j, v1 = irow && j + 1 < n && i != j + 1;
                            const bool q0 = v0 && i < j, q1 = v1 && i < j + 1;
                            const f32x2 e0q = {q0 ? e0.x : 0.f, q1 ? e0.y : 0.f};
                            const f32x2 e1q = {q0 ? e1.x : 0.f, q1 ? e1.y : 0.f};
                            A00 += e0q * e0q;
                            A01 += e0q * e1q;
                            A11 += e1q * e1q;
                            if (!swap_mode) {
                                const bool t0 = v0 && i > j, t1 = v1 && i > j + 1;
                                const f32x2 e0s = {t0 ? e0.x : 0.f, t1 ? e0.y : 0.f};
                                const f32x2 e1s = {t0 ? e1.x : 0.f, t1 ? e1.y : 0.f};
                                S += e0s * e0s;
                                S += e1s * e1s;
                            }
                        }
                    }
                }
            }
        };
        if (upper) tile_body(std::integral_constant<int, 0>{});
        else if (lower) tile_body(std::integral_constant<int, 1>{});
        else tile_body(std::integral_constant<int, 2>{});
        // this tile's sums (<= 16 terms per lane and statistic) into fp64
        const double a00 = (double)A00.x + (double)A00.y, a01 = (double)A01.x + (double)A01.y;
        const double a11 = (double)A11.x + (double)A11.y;
        quad += p * a00 + qs * a01 + sr * a11;
        sq += (swap_mode ? 2.0 : 1.0) * (a00 + a11) + ((double)S.x + (double)S.y);
        lds_barrier3();       // staging of tile tt+1 visible; stg[tt & 1] free
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // dummy DMAs drained before exit
    double v2[2] = {quad, sq};
    block_sum<2>(v2, red);
    if (threadIdx.x == 0) {
        partial[(size_t)blockIdx.x * 2 + 0] = v2[0];
        partial[(size_t)blockIdx.x * 2 + 1] = v2[1];
    }
}

// ---------------------------------------------------------------------------
// K3: per-(node, slice) terms.  partial3 layout [nwg3][6]:
//   {mu0' S0i mu0, tr(S0i S_0), e' Qi e (t>=1), tr(Qi S) (t>=1), logdet S, tr S}
// ---------------------------------------------------------------------------
template <int R>
__global__ void __launch_bounds__(AME_NT)
ame_nodes_kernel(ame_dims dm, const float* __restrict__ x, const float* __restrict__ prev_final,
                 const double* __restrict__ cov_terms, const double* __restrict__ consts,
                 const double* __restrict__ phi, double* __restrict__ partial) {
    // One thread per (node, slice); the three d x d matrices it contracts with
    // (Sigma0^-1, Q^-1, Phi) are staged in LDS once per workgroup, so every
    // thread's matvecs read broadcast LDS words instead of global memory.
    constexpr int D = 2 + 2 * R;
    constexpr int DD = D * D;
    const int n = dm.n;
    __shared__ __attribute__((aligned(16))) double cS0[DD], cQ[DD], cPhi[DD];   // D even: rows 16-B aligned
    __shared__ double red[4 * 6];
    for (int e = threadIdx.x; e < DD; e += AME_NT) {
        cS0[e] = consts[e];
        cQ[e] = consts[DD + e];
        cPhi[e] = phi[e];
    }
    __syncthreads();
    const int idx = blockIdx.x * AME_NT + threadIdx.x;
    double v[6] = {0, 0, 0, 0, 0, 0};
    if (idx < dm.T_local * n) {
        const int tl = idx / n, i = idx - tl * n;
        const int tg = dm.t_begin + tl;
        const float* mu = x + ((size_t)tl * n + i) * D;
        const double* ct = cov_terms + ((size_t)tl * n + i) * 4;
        v[4] = ct[0];
        v[5] = ct[1];
        double e[D];
        const double* M;
        if (tg == 0) {
#pragma unroll
            for (int k = 0; k < D; ++k) e[k] = (double)mu[k];
            M = cS0;
            v[1] = ct[3];
        } else {
            const float* pr = (tl > 0) ? x + ((size_t)(tl - 1) * n + i) * D : prev_final + (size_t)i * D;
            double pm[D];
#pragma unroll
            for (int m = 0; m < D; ++m) pm[m] = (double)pr[m];
#pragma unroll
            for (int k = 0; k < D; ++k) {   // two FMA chains, one ds_read_b128 per pair
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int m = 0; m < D; m += 2) {
                    const double2 c = *(const double2*)&cPhi[k * D + m];
                    a0 = fma(c.x, pm[m], a0);
                    a1 = fma(c.y, pm[m + 1], a1);
                }
                e[k] = (double)mu[k] - (a0 + a1);
            }
            M = cQ;
            v[3] = ct[2];
        }
        double qsum = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            double r0 = 0.0, r1 = 0.0;
#pragma unroll
            for (int m = 0; m < D; m += 2) {
                const double2 c = *(const double2*)&M[k * D + m];
                r0 = fma(c.x, e[m], r0);
                r1 = fma(c.y, e[m + 1], r1);
            }
            qsum = fma(e[k], r0 + r1, qsum);
        }
        v[(tg == 0) ? 0 : 2] = qsum;
    }
    block_sum<6>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < 6; ++q) partial[(size_t)blockIdx.x * 6 + q] = v[q];
}

// Final deterministic reduction -> out[8] (internal linkage: one copy per split part)
static __global__ void __launch_bounds__(AME_NT)
ame_final_kernel(const double* __restrict__ p2, int n2, const double* __restrict__ p3, int n3,
                 double* __restrict__ out) {
    __shared__ double red[4 * 8];
    double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = threadIdx.x; b < n2; b += AME_NT) {
        v[0] += p2[(size_t)b * 2 + 0];
        v[7] += p2[(size_t)b * 2 + 1];
    }
    for (int b = threadIdx.x; b < n3; b += AME_NT) {
        const double* r = p3 + (size_t)b * 6;
        v[2] += r[0];
        v[3] += r[1];
        v[4] += r[2];
        v[5] += r[3];
        v[6] += r[4];
        v[1] += r[5];
    }
    block_sum<8>(v, red);
    if (threadIdx.x == 0)
        for (int q = 0; q < 8; ++q) out[q] = v[q];
}

static inline long long pairs_blocks(const ame_dims* dm, int swap_mode) {
    const long long nb = (dm->n + AME_TILE - 1) / AME_TILE;
    return (long long)dm->T_local * (swap_mode ? (nb + 1) / 2 : nb);
}
static inline long long nodes_blocks(const ame_dims* dm) {
    return ((long long)dm->T_local * dm->n + AME_NT - 1) / AME_NT;
}

#if AME_PART0
long long ame_elbo_work_doubles(const ame_dims* dm) {
    return 2 * pairs_blocks(dm, 0) + 6 * nodes_blocks(dm) + 16;
}
#endif

template <int R>
static int launch_elbo(const ame_dims* dm, const ame_elbo_args* a, hipStream_t st, bool pairs_only) {
    const long long b2 = pairs_blocks(dm, a->swap_consistent);
    const long long b3 = nodes_blocks(dm);
    double* p2 = a->work;
    double* p3 = a->work + 2 * b2;
    if (b2 > 0) {
        // LDS-DMA pair kernel (every Yt row starts 16-byte aligned, odd n
        // included: ame_ystride); args.pairs_kernel = AME_PAIRS_V1 keeps the
        // register-streaming kernel
        const bool v1 = a->pairs_kernel == AME_PAIRS_V1;
        if (v1)
            hipLaunchKernelGGL(ame_pairs_kernel<R>, dim3((unsigned)b2), dim3(AME_NT), 0, st, *dm, a->Yt,
                               a->x, a->rinv[0], a->rinv[1], a->rinv[2], a->rinv[3],
                               a->swap_consistent, p2);
        else
            hipLaunchKernelGGL(ame_pairs2_kernel<R>, dim3((unsigned)b2), dim3(AME_NT), 0, st, *dm, a->Yt,
                               a->x, a->rinv[0], a->rinv[1], a->rinv[2], a->rinv[3],
                               a->swap_consistent, p2);
    }
    if (pairs_only)   // ame_elbo_pairs_diag: timing of the pair kernel alone
        return hipGetLastError() == hipSuccess ? 0 : -3;
    if (b3 > 0)
        hipLaunchKernelGGL(ame_nodes_kernel<R>, dim3((unsigned)b3), dim3(AME_NT), 0, st, *dm, a->x,
                           a->prev_final, a->cov_terms, a->consts, a->phi, p3);
    hipLaunchKernelGGL(ame_final_kernel, dim3(1), dim3(AME_NT), 0, st, p2, (int)b2, p3, (int)b3,
                       a->out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int AME_PFN(ame_elbo_dispatch)(const ame_dims* dm, const ame_elbo_args* a, hipStream_t st, int pairs_only) {
    switch (dm->r) {
#define X(RR) \
    case RR: return launch_elbo<RR>(dm, a, st, pairs_only != 0);
        AME_FOR_EACH_R(X)
#undef X
        default: return -1;
    }
}
