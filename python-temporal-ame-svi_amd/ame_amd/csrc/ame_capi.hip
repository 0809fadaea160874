// extern "C" boundary of libame_amd.so (declared in include/ame_amd.h).
// Argument validation lives here so a bad call fails loudly with a message
// instead of faulting on the GPU.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ame_common.h"

int ame_sweep_dispatch(const ame_dims*, const ame_sweep_args*, hipStream_t);
int ame_sweep_blocks_per_cu(int n, int r);
long long ame_sweep_v2w_doubles(const ame_dims* dm);
int ame_sweep3_dispatch(const ame_dims*, const ame_sweep_args*, hipStream_t);
int ame_sweep3_supported(int n, int r);
int ame_sweep3_blocks_per_cu(int n, int r);
long long ame_sweep3_work_doubles(const ame_dims*);
int ame_sweep4_dispatch(const ame_dims*, const ame_sweep_args*, hipStream_t);
int ame_sweep4_supported(int n, int r);
int ame_sweep4_blocks_per_cu(int n, int r);
long long ame_sweep4_work_doubles(const ame_dims*);
int ame_cov_dispatch(const ame_dims*, const ame_cov_args*, hipStream_t);
int ame_elbo_dispatch(const ame_dims*, const ame_elbo_args*, hipStream_t);
long long ame_elbo_work_doubles(const ame_dims*);
int ame_align_cross_dispatch(const float*, const float*, int, int, int, int, double*, double*,
                             hipStream_t);
int ame_align_apply_dispatch(const float*, const float*, int, int, int, int, const double*, float*,
                             double*, hipStream_t);
long long ame_align_partials_count(int n, int T);
int ame_pack_dispatch(const float*, float*, const ame_dims*, unsigned long long*, hipStream_t);

static thread_local char g_err[512] = "";

static int fail(const char* fmt, int a = 0, int b = 0) {
    snprintf(g_err, sizeof(g_err), fmt, a, b);
    return -1;
}

static bool r_supported(int r) {
    switch (r) {
#define X(RR) \
    case RR: return true;
        AME_FOR_EACH_R(X)
#undef X
        default: return false;
    }
}

static bool env_on(const char* name) {
    const char* e = getenv(name);
    return e && e[0] && e[0] != '0';
}
// v3 (solver + helper waves, register-resident slice GEMV) when the slice fits
// its register budget, else v2.  v4 (the observation term on MFMA block GEMMs
// plus a window GEMV, r <= 16, n % 4 == 0, n <= 2048) is opt-in with
// AME_SWEEP_V4=1: it is exact (tests/test_gpu_sweep4.py) but its step period
// measured longer than v3's (profiles/r02_v4_*).  AME_SWEEP_V2=1
// forces the v2 kernel (A/B runs, tests).
static bool use_v4(int n, int r) {
    if (env_on("AME_SWEEP_V2") || !env_on("AME_SWEEP_V4")) return false;
    return ame_sweep4_supported(n, r) != 0;
}
static bool use_v3(int n, int r) {
    if (env_on("AME_SWEEP_V2")) return false;
    return use_v4(n, r) || ame_sweep3_supported(n, r) != 0;
}

static int check_dims(const ame_dims* d) {
    if (d == nullptr) return fail("ame: dims is NULL");
    if (d->n < 2) return fail("ame: n must be >= 2 (got %d)", d->n);
    if (!r_supported(d->r)) return fail("ame: latent_dim r=%d not compiled into this library", d->r);
    if (d->T_local < 1 || d->T_total < 1) return fail("ame: bad T_local=%d T_total=%d", d->T_local, d->T_total);
    if (d->t_begin < 0 || d->t_begin + d->T_local > d->T_total)
        return fail("ame: slice range [%d, +T_local) outside T_total", d->t_begin);
    if (d->variant < AME_GOOD || d->variant > AME_NAIVE) return fail("ame: bad variant %d", d->variant);
    return 0;
}

static int launched(int rc, const char* what) {
    if (rc == 0) return 0;
    hipError_t e = hipGetLastError();
    snprintf(g_err, sizeof(g_err), "ame: %s launch failed (rc=%d, hip=%s)", what, rc,
             hipGetErrorString(e));
    return -1;
}

extern "C" {

const char* ame_last_error(void) { return g_err; }

const char* ame_version(void) { return "ame_amd 0.1 gfx950"; }

int ame_supported_r(int* out, int cap) {
    int c = 0;
#define X(RR)                       \
    if (c < cap && out) out[c] = RR; \
    ++c;
    AME_FOR_EACH_R(X)
#undef X
    return c;
}

int ame_host_register(void* host, unsigned long long bytes, void** dev) {
    if (!host || !dev || bytes == 0) return fail("ame_host_register: bad arguments");
    hipError_t e = hipHostRegister(host, (size_t)bytes, hipHostRegisterMapped | hipHostRegisterPortable);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_host_register: hipHostRegister: %s", hipGetErrorString(e));
        return -1;
    }
    e = hipHostGetDevicePointer(dev, host, 0);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_host_register: hipHostGetDevicePointer: %s",
                 hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int ame_host_unregister(void* host) {
    if (!host) return fail("ame_host_unregister: NULL");
    return hipHostUnregister(host) == hipSuccess ? 0 : fail("ame_host_unregister failed");
}

int ame_peer_alloc(unsigned long long bytes, void** dev, void* handle) {
    if (!dev || !handle || bytes == 0) return fail("ame_peer_alloc: bad arguments");
    hipError_t e = hipExtMallocWithFlags(dev, (size_t)bytes, hipDeviceMallocFinegrained);
    if (e == hipSuccess) e = hipMemset(*dev, 0, (size_t)bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipIpcGetMemHandle((hipIpcMemHandle_t*)handle, *dev);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_peer_alloc: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int ame_peer_free(void* dev) {
    if (!dev) return fail("ame_peer_free: NULL");
    return hipFree(dev) == hipSuccess ? 0 : fail("ame_peer_free failed");
}

int ame_peer_open(const void* handle, void** dev) {
    if (!handle || !dev) return fail("ame_peer_open: bad arguments");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    hipError_t e = hipIpcOpenMemHandle(dev, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_peer_open: hipIpcOpenMemHandle: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int ame_peer_close(void* dev) {
    if (!dev) return fail("ame_peer_close: NULL");
    return hipIpcCloseMemHandle(dev) == hipSuccess ? 0 : fail("ame_peer_close failed");
}

long long ame_sweep_lds_bytes(int n, int r) {
    if (!r_supported(r) || n < 1) return 0;
    return sweep_lds_layout(n, r, ame_sweep_force_global()).total;
}

int ame_sweep_max_slices(int n, int r) {
    if (!r_supported(r)) return 0;
    const bool v3 = use_v3(n, r);
    if (!v3 && sweep_lds_layout(n, r, ame_sweep_force_global()).total > AME_LDS_MAX) return 0;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    const int per_cu = use_v4(n, r) ? ame_sweep4_blocks_per_cu(n, r)
                       : v3 ? ame_sweep3_blocks_per_cu(n, r) : ame_sweep_blocks_per_cu(n, r);
    return per_cu * cus;
}

int ame_sweep_orders_slices(int n, int r) { return r_supported(r) && use_v3(n, r) ? 1 : 0; }

// v2 with GEMV workers: their partial ring; else v2 with the slice's (U,V)
// block in HBM: [T_local][n][2r] fp32 in the work buffer
static long long v2_global_doubles(const ame_dims* d) {
    if (use_v3(d->n, d->r)) return 0;
    if (const long long w = ame_sweep_v2w_doubles(d)) return w;
    if (!sweep_lds_layout(d->n, d->r, ame_sweep_force_global()).m_global) return 0;
    return ((long long)d->T_local * d->n * 2 * d->r + 1) / 2;
}

int ame_sweep_kind(const ame_dims* dims) {
    if (check_dims(dims)) return -1;
    if (use_v4(dims->n, dims->r)) return 4;
    if (use_v3(dims->n, dims->r)) return 3;
    if (ame_sweep_v2w_doubles(dims) > 0) return 22;
    return sweep_lds_layout(dims->n, dims->r, ame_sweep_force_global()).m_global ? 21 : 20;
}

long long ame_sweep_work_size(const ame_dims* dims) {
    if (check_dims(dims)) return -1;
    if (use_v4(dims->n, dims->r)) return ame_sweep4_work_doubles(dims);
    const long long a = ame_sweep3_work_doubles(dims), b = v2_global_doubles(dims);
    return a > b ? a : b;
}

int ame_pack_y(const float* Y, float* Yt, const ame_dims* dims, unsigned long long* mismatch,
               void* stream) {
    if (int e = check_dims(dims)) return e;
    if (!Y || !Yt) return fail("ame_pack_y: NULL buffer");
    return launched(ame_pack_dispatch(Y, Yt, dims, mismatch, (hipStream_t)stream), "pack");
}

int ame_sweep(const ame_dims* dims, const ame_sweep_args* a, void* stream) {
    if (int e = check_dims(dims)) return e;
    if (!a || !a->Yt || !a->x_old || !a->x_new || !a->cov || !a->hand || !a->consts || !a->status)
        return fail("ame_sweep: NULL buffer");
    if (a->epoch == 0) return fail("ame_sweep: epoch must be >= 1");
    if (dims->t_begin > 0 && !a->halo_in)
        return fail("ame_sweep: t_begin=%d > 0 needs halo_in", dims->t_begin);
    if (dims->t_begin + dims->T_local < dims->T_total && !a->next_old && !(a->wait_epoch && a->back_in))
        return fail("ame_sweep: rank does not hold T-1 and next_old is NULL");
    const bool v3 = use_v3(dims->n, dims->r);
    if (!v3 && sweep_lds_layout(dims->n, dims->r, ame_sweep_force_global()).total > AME_LDS_MAX)
        return fail("ame_sweep: slice state (n=%d, r=%d) exceeds one workgroup's LDS", dims->n, dims->r);
    if ((v2_global_doubles(dims) > 0 || use_v4(dims->n, dims->r)) && !a->work)
        return fail("ame_sweep: n=%d, r=%d keeps the slice in HBM and needs the work buffer", dims->n, dims->r);
    if (a->wait_epoch != 0 && (!v3 || !a->done))
        return fail("ame_sweep: wait_epoch needs the v3 sweep and a done array");
    const int maxs = ame_sweep_max_slices(dims->n, dims->r);
    if (dims->T_local > maxs)
        return fail("ame_sweep: T_local=%d exceeds co-resident workgroups (%d)", dims->T_local, maxs);
    if (use_v4(dims->n, dims->r)) return launched(ame_sweep4_dispatch(dims, a, (hipStream_t)stream), "sweep4");
    if (v3) return launched(ame_sweep3_dispatch(dims, a, (hipStream_t)stream), "sweep3");
    return launched(ame_sweep_dispatch(dims, a, (hipStream_t)stream), "sweep");
}

int ame_cov(const ame_dims* dims, const ame_cov_args* a, void* stream) {
    if (int e = check_dims(dims)) return e;
    if (!a || !a->cov || !a->consts || !a->cov_terms) return fail("ame_cov: NULL buffer");
    return launched(ame_cov_dispatch(dims, a, (hipStream_t)stream), "cov");
}

long long ame_elbo_work_size(const ame_dims* dims) {
    if (check_dims(dims)) return -1;
    return ame_elbo_work_doubles(dims);
}

int ame_elbo(const ame_dims* dims, const ame_elbo_args* a, void* stream) {
    if (int e = check_dims(dims)) return e;
    if (!a || !a->Yt || !a->x || !a->cov_terms || !a->consts || !a->phi || !a->work || !a->out)
        return fail("ame_elbo: NULL buffer");
    if (dims->t_begin > 0 && !a->prev_final)
        return fail("ame_elbo: t_begin=%d > 0 needs prev_final", dims->t_begin);
    return launched(ame_elbo_dispatch(dims, a, (hipStream_t)stream), "elbo");
}

static int check_align(int n, int T, int r) {
    if (n < 1 || T < 1) return fail("ame_align: bad n=%d T=%d", n, T);
    if (!r_supported(r)) return fail("ame_align: latent_dim r=%d not compiled into this library", r);
    return 0;
}

long long ame_align_work_size(int n, int T, int r) {
    if (check_align(n, T, r)) return -1;
    return 2LL * n * 2 * r;
}

long long ame_align_cross_size(int n, int T, int r, int global_mode) {
    if (check_align(n, T, r)) return -1;
    return global_mode ? 4LL * r * r : 2LL * T * r * r;
}

long long ame_align_partials_size(int n, int T) {
    if (n < 1 || T < 1) return fail("ame_align: bad n=%d T=%d", n, T);
    return ame_align_partials_count(n, T);
}

int ame_align_cross(const float* x_est, const float* x_true, int n, int T, int r, int global_mode,
                    double* cross, double* work, void* stream) {
    if (int e = check_align(n, T, r)) return e;
    if (!x_est || !x_true || !cross || (global_mode && !work)) return fail("ame_align_cross: NULL buffer");
    return launched(ame_align_cross_dispatch(x_est, x_true, n, T, r, global_mode, cross, work,
                                             (hipStream_t)stream), "align_cross");
}

int ame_align_apply(const float* x_est, const float* x_true, int n, int T, int r, int global_mode,
                    const double* rot, float* x_out, double* partials, void* stream) {
    if (int e = check_align(n, T, r)) return e;
    if (!x_est || !x_true || !rot || !x_out || !partials) return fail("ame_align_apply: NULL buffer");
    return launched(ame_align_apply_dispatch(x_est, x_true, n, T, r, global_mode, rot, x_out,
                                             partials, (hipStream_t)stream), "align_apply");
}

}  // extern "C"
