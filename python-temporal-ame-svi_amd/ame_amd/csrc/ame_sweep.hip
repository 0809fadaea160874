// K1: the Gauss-Seidel sweep (means only) of TemporalAMEStructuredMFVI /
// TemporalAMENaiveMFVI for gfx950.
//
// Reference semantics (Alfieriek/Python-Temporal-AME-SVI):
//   _update_step            structured_mf.py:211-218  (for i in range(n))
//   _update_node_i          structured_mf.py:220-287  (for t in range(T))
//   _compute_observation_terms  structured_mf.py:289-326
//   naive variant           naive_mf.py:207-282 (mu = solve(P, h))
// Step (i,t) reads the NEW means of nodes j<i at t and of node i at t-1 and the
// OLD means of nodes j>i at t and of node i at t+1, so one sweep is a 2-D
// wavefront.  Design:
//   * one workgroup per time slice ("lane" t), all lanes co-resident;
//   * the lane keeps its slice's (U,V) means in LDS and fp64 running
//     statistics S_t = sum_j stat(U_j, V_j) (SURVEY App. A closed form), so
//     P_obs(i,t) = F(S_t - stat(node i)) costs O(r^2) instead of O(n r^2);
//   * h_obs(i,t) is a GEMV of the Y row (n x 2, streamed from HBM) with the
//     slice's (U,V) matrix in LDS;
//   * lane t-1 hands mu_{i,t-1}^new to lane t through {epoch,value} granules
//     (no fence on the critical path);
//   * the d x d system is solved by Gauss-Jordan in fp64 in LDS;
//   * every AME_SNAP_NB nodes the statistics are snapshotted so the
//     covariance kernel can rebuild bit-identical precisions in parallel.
#include "ame_common.h"

#ifdef AME_STAMPS
// Diagnostic build only (cdna_hip_programming.md §7, in-kernel stamps): lane
// AME_STAMP_LANE records s_memtime after each phase for nodes
// [AME_STAMP_I0, AME_STAMP_I0 + 16).  Never compiled into the product library.
#define AME_STAMP_I0 256
#define AME_STAMP_NPH 8
__device__ unsigned long long g_ame_stamps[16 * AME_STAMP_NPH];
#define STAMP(ph)                                                                          \
    do {                                                                                   \
        if (stamp_on && tid == 0) {                                                        \
            unsigned long long t_;                                                         \
            __builtin_amdgcn_sched_barrier(0);                                             \
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");     \
            __builtin_amdgcn_sched_barrier(0);                                             \
            g_ame_stamps[(i - AME_STAMP_I0) * AME_STAMP_NPH + (ph)] = t_;                  \
        }                                                                                  \
    } while (0)
extern "C" int ame_debug_read_stamps(unsigned long long* host, int count) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ame_stamps), sizeof(unsigned long long) * count,
                               0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#else
#define STAMP(ph) \
    do {          \
    } while (0)
#endif

template <int R>
__global__ void __launch_bounds__(AME_NT)
ame_sweep_kernel(ame_dims dm, ame_sweep_args a) {
    using C = AmeCfg<R>;
    constexpr int D = C::D, M2 = C::M2, NS = C::NS, VEC = C::VEC, CW = C::CW, G = C::G,
                  PW = C::PW, W = C::W, QN = C::QN, MC = C::MC;
    const int n = dm.n, TL = dm.T_local, Tt = dm.T_total;
    const int tl = blockIdx.x, tg = dm.t_begin + tl;
    const int tid = threadIdx.x;
    const int variant = dm.variant;
    const int nblk = (n + AME_SNAP_NB - 1) / AME_SNAP_NB;

    extern __shared__ __attribute__((aligned(16))) char smem[];
    const SweepLds L = sweep_lds_layout(n, R);
    double* S = (double*)(smem + L.oS);
    double* A = (double*)(smem + L.oA);
    double* vh = (double*)(smem + L.oVh);
    double* var = (double*)(smem + L.oVar);
    float* mu_prev = (float*)(smem + L.oF);
    float* mu_next = mu_prev + D;
    float* mu_old = mu_next + D;
    float* mu_new = mu_old + D;
    float* part = (float*)(smem + L.oPart);
    float2* z = (float2*)(smem + L.oZ);
    float* M = (float*)(smem + L.oM);

    const double p = a.rinv[0], s = a.rinv[3];
    const double q = 0.5 * (a.rinv[1] + a.rinv[2]);
    const float r00 = (float)a.rinv[0], r01 = (float)a.rinv[1], r10 = (float)a.rinv[2],
                r11 = (float)a.rinv[3];
    const double nm1 = (double)(n - 1);

    // ---- slice state: (U,V) of all nodes, then fp64 statistics ----
    const float* xo = a.x_old + (size_t)tl * n * D;
    for (int idx = tid; idx < n * M2; idx += AME_NT) {
        const int j = idx / M2, c = idx - j * M2;
        M[idx] = xo[(size_t)j * D + 2 + c];
    }
    // constant precision entries owned by this thread (fixed for the slice)
    double pc[QN];
    int pk[QN], pm[QN];
#pragma unroll
    for (int qq = 0; qq < QN; ++qq) {
        const int e = tid + AME_NT * qq;
        pk[qq] = (e < D * D) ? e / D : 0;
        pm[qq] = (e < D * D) ? e - (e / D) * D : 0;
        pc[qq] = (e < D * D) ? pconst_entry(a.consts, D, pk[qq], pm[qq], tg, Tt) : 0.0;
    }
    // AR rows: thread (k = tid>>2, part = tid&3) owns columns [part*MC, part*MC+MC)
    double qiphi[MC], phitqi[MC];
    {
        const int k = tid >> 2, pp = tid & 3;
        const size_t DD = (size_t)D * D;
#pragma unroll
        for (int mm = 0; mm < MC; ++mm) {
            const int m = pp * MC + mm;
            const bool ok = (tid < 4 * D) && (m < D);
            qiphi[mm] = ok ? a.consts[3 * DD + (size_t)k * D + m] : 0.0;
            phitqi[mm] = ok ? a.consts[4 * DD + (size_t)k * D + m] : 0.0;
        }
    }
    __syncthreads();
    for (int e = tid; e < NS; e += AME_NT) {
        double acc = 0.0;
        for (int j = 0; j < n; ++j) acc = __dadd_rn(acc, stat_val<R>(e, M + j * M2, M + j * M2 + R));
        S[e] = acc;
    }
    // Gauss-Jordan work split (compile-time stride W)
    constexpr int GJ_PER = (D * W + AME_NT - 1) / AME_NT;
    int gk[GJ_PER], gm[GJ_PER];
#pragma unroll
    for (int qq = 0; qq < GJ_PER; ++qq) {
        const int e = tid + AME_NT * qq;
        gk[qq] = (e < D * W) ? e / W : -1;
        gm[qq] = (e < D * W) ? e - (e / W) * W : -1;
    }
    const int ncol = D + ((variant == AME_BAD) ? 2 : 1);
    bool dead = false;   // a spin timed out: stop waiting, finish the sweep
    __syncthreads();

    const float* yslice = a.Yt + (size_t)tl * n * n * 2;
    float* xn = a.x_new + (size_t)tl * n * D;

    for (int i = 0; i < n; ++i) {
#ifdef AME_STAMPS
        const bool stamp_on = (tl == TL / 2) && i >= AME_STAMP_I0 && i < AME_STAMP_I0 + 16;
#endif
        STAMP(0);
        // (a) statistic snapshot for the covariance kernel
        if ((i % AME_SNAP_NB) == 0) {
            double* dst = a.snap + ((size_t)tl * nblk + i / AME_SNAP_NB) * NS;
            for (int e = tid; e < NS; e += AME_NT) dst[e] = S[e];
        }
        // (b) z_ij = R^-1 y_ij for the Y row of node i (j == i masked)
        {
            const float2* yrow = (const float2*)(yslice + (size_t)i * n * 2);
            for (int j = tid; j < n; j += AME_NT) {
                const float2 y = yrow[j];
                float z0 = r00 * y.x + r01 * y.y;
                float z1 = r10 * y.x + r11 * y.y;
                if (j == i) { z0 = 0.f; z1 = 0.f; }
                z[j] = make_float2(z0, z1);
            }
        }
        // (c) node vectors: old mean, right neighbour (old), left neighbour (new)
        if (tid < D) {
            mu_old[tid] = xo[(size_t)i * D + tid];
            float nx = 0.f;
            if (tg < Tt - 1)
                nx = (tl < TL - 1) ? a.x_old[((size_t)(tl + 1) * n + i) * D + tid]
                                   : a.next_old[(size_t)i * D + tid];
            mu_next[tid] = nx;
        }
        if (tg > 0) {
            if (tid >= 64 && tid < 128) {   // wave 1 polls the hand-off granules
                const int k = tid - 64;
                const bool from_halo = (tl == 0);
                const uint64_t* src = from_halo ? a.halo_in + (size_t)i * D
                                                : a.hand + ((size_t)(tl - 1) * n + i) * D;
                uint64_t v = 0;
                const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
                const uint64_t budget = from_halo ? AME_SPIN_TICKS_HALO : AME_SPIN_TICKS_LOCAL;
                while (true) {
                    bool ok = true;
                    if (k < D) {
                        v = from_halo ? gran_load_system(src + k) : gran_load_agent(src + k);
                        ok = (uint32_t)(v >> 32) == a.epoch;
                    }
                    if (__all(ok) || dead) break;
                    if (__builtin_amdgcn_s_memrealtime() - t_start > budget) {
                        if (k == 0)
                            atomicOr(a.status, from_halo ? AME_STATUS_HALO_TIMEOUT
                                                         : AME_STATUS_SPIN_TIMEOUT);
                        dead = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                if (k < D) mu_prev[k] = __uint_as_float((uint32_t)v);
            }
        } else if (tid < D) {
            mu_prev[tid] = 0.f;
        }
        __syncthreads();   // B1
        STAMP(1);

        // (d) GEMV partials: h_U = sum_j z0_j V_j, h_V = sum_j z1_j U_j (+ sums of z)
        {
            const int g = tid / CW, cq = tid - g * CW;
            if (g < G) {
                const int c0 = cq * VEC;
                const bool upart = c0 < R;
                const int mo = upart ? (R + c0) : (c0 - R);
                float acc[VEC];
#pragma unroll
                for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
                float s0 = 0.f, s1 = 0.f;
                for (int j = g; j < n; j += G) {
                    const float2 zz = z[j];
                    const float zc = upart ? zz.x : zz.y;
                    const float* mr = M + j * M2 + mo;
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
            // AR terms: Qinv Phi mu_{i,t-1}^new + Phi^T Qinv mu_{i,t+1}^old
            if (tid < 4 * D) {
                const int k = tid >> 2, pp = tid & 3;
                double acc = 0.0;
#pragma unroll
                for (int mm = 0; mm < MC; ++mm) {
                    const int m = pp * MC + mm;
                    if (m < D) {
                        if (tg > 0) acc = fma(qiphi[mm], (double)mu_prev[m], acc);
                        if (tg < Tt - 1) acc = fma(phitqi[mm], (double)mu_next[m], acc);
                    }
                }
                acc += __shfl_xor(acc, 1);
                acc += __shfl_xor(acc, 2);
                if (pp == 0) var[k] = acc;
            }
        }
        __syncthreads();   // B2
        STAMP(2);

        // (e) natural parameter (reduce partials) and augmented precision [P | rhs]
        if (tid < PW) {
            float acc = 0.f;
            for (int g = 0; g < G; ++g) acc += part[g * PW + tid];
            const int kk = (tid < M2) ? 2 + tid : tid - M2;
            const double h = (double)acc + var[kk];
            vh[kk] = h;
            if (variant == AME_BAD) {
                A[kk * W + D] = (kk < 2) ? h : 0.0;
                A[kk * W + D + 1] = (kk < 2) ? 0.0 : h;
            } else {
                A[kk * W + D] = h;
            }
        }
        {
            const float* Uo = M + i * M2;
            const float* Vo = Uo + R;
#pragma unroll
            for (int qq = 0; qq < QN; ++qq) {
                const int e = tid + AME_NT * qq;
                if (e < D * D) {
                    const double po = pobs_entry<R>(pk[qq], pm[qq], S, Uo, Vo, p, q, s, nm1);
                    A[pk[qq] * W + pm[qq]] = __dadd_rn(po, pc[qq]);
                }
            }
        }
        __syncthreads();   // B3
        STAMP(3);

        // (f) Gauss-Jordan elimination (SPD: no pivoting), fp64
        for (int pv = 0; pv < D; ++pv) {
            const double pinv = 1.0 / A[pv * W + pv];
#pragma unroll
            for (int qq = 0; qq < GJ_PER; ++qq) {
                const int k = gk[qq], m = gm[qq];
                if (k >= 0 && k != pv && m > pv && m < ncol) {
                    const double f = A[k * W + pv] * pinv;
                    A[k * W + m] = fma(-f, A[pv * W + m], A[k * W + m]);
                }
            }
            __syncthreads();
        }

        STAMP(4);
        // (g) new mean: mu* = C h with C = sym(P^-1) (+1e-6 I), damped
        if (tid < D) {
            const int k = tid;
            const int col = (variant == AME_BAD && k >= 2) ? D + 1 : D;
            double x = A[k * W + col] / A[k * W + k];
            if (variant != AME_NAIVE) x += 1e-6 * vh[k];
            const float mu = (float)x;
            const float nw = __fadd_rn(__fmul_rn(a.lr, mu), __fmul_rn(a.one_minus_lr, mu_old[k]));
            mu_new[k] = nw;
            xn[(size_t)i * D + k] = nw;
            const uint64_t gv = ((uint64_t)a.epoch << 32) | (uint64_t)__float_as_uint(nw);
            gran_store_agent(a.hand + ((size_t)tl * n + i) * D + k, gv);
            if (tl == TL - 1 && a.halo_out != nullptr)
                gran_store_system(a.halo_out + (size_t)i * D + k, gv);
        }
        __syncthreads();   // B4
        STAMP(5);

        // (h) statistics: S += stat(new) - stat(old)
        {
            const float* Uo = M + i * M2;
            for (int e = tid; e < NS; e += AME_NT)
                S[e] = stat_apply<R>(S[e], e, mu_new + 2, mu_new + 2 + R, Uo, Uo + R);
        }
        __syncthreads();   // B5
        STAMP(6);
        if (tid < M2) M[i * M2 + tid] = mu_new[2 + tid];
    }
}

template <int R>
static int launch_sweep(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    const SweepLds L = sweep_lds_layout(dm->n, R);
    auto kern = ame_sweep_kernel<R>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)L.total) != hipSuccess)
        return -2;
    hipLaunchKernelGGL(kern, dim3(dm->T_local), dim3(AME_NT), (size_t)L.total, st, *dm, *a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int R>
static int sweep_occupancy(int n) {
    const SweepLds L = sweep_lds_layout(n, R);
    auto kern = ame_sweep_kernel<R>;
    if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)L.total) != hipSuccess)
        return 0;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, AME_NT, (size_t)L.total) !=
        hipSuccess)
        return 0;
    return per_cu;
}

int ame_sweep_dispatch(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    switch (dm->r) {
#define X(RR) \
    case RR: return launch_sweep<RR>(dm, a, st);
        AME_FOR_EACH_R(X)
#undef X
        default: return -1;
    }
}

int ame_sweep_blocks_per_cu(int n, int r) {
    switch (r) {
#define X(RR) \
    case RR: return sweep_occupancy<RR>(n);
        AME_FOR_EACH_R(X)
#undef X
        default: return 0;
    }
}
