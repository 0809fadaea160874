// extern "C" boundary of libame_amd.so (declared in include/ame_amd.h).
// Argument validation lives here so a bad call fails loudly with a message
// instead of faulting on the GPU.
#include <stdio.h>
#include <string.h>

#include "ame_common.h"

int ame_sweep_dispatch(const ame_dims*, const ame_sweep_args*, hipStream_t);
int ame_sweep_blocks_per_cu(int n, int r, int mode);
int ame_sweep_workers_fit(const ame_dims* dm, int mode);   // mode 2: kind 22, 3: kind 23, 4: kind 24
int ame_sweep3_dispatch(const ame_dims*, const ame_sweep_args*, hipStream_t);
int ame_sweep3_supported(int n, int r);
int ame_sweep3_blocks_per_cu(int n, int r);
long long ame_sweep3_work_doubles(const ame_dims*);
int ame_sweep3_lds(int n, int r);
int ame_cov_dispatch(const ame_dims*, const ame_cov_args*, hipStream_t);
int ame_elbo_dispatch(const ame_dims*, const ame_elbo_args*, hipStream_t, int pairs_only);
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

// AME_SRC_HASH: SHA-256 prefix of every source, header and build flag that
// went into this library (ame_amd/build.py source_hash()); build() compares it
// with the tree and rebuilds on a mismatch, and tests / bench report it
#ifndef AME_SRC_HASH
#define AME_SRC_HASH "unknown"
#endif
const char* ame_version(void) { return "ame_amd 0.4 gfx950 src=" AME_SRC_HASH; }

// test hook (not in the header): the GEMV-worker partial tag (ame_common.h)
unsigned int ame_debug_gw_tag(unsigned int epoch, int m) { return ame_gw_tag(epoch, m); }

int ame_supported_r(int* out, int cap) {
    int c = 0;
#define X(RR)                       \
    if (c < cap && out) out[c] = RR; \
    ++c;
    AME_FOR_EACH_R(X)
#undef X
    return c;
}

#define AME_MAX_CUS 1024
static int device_cus();
int ame_stream_create_cu_range(int first_cu, int num_cus, void** stream) {
    if (!stream) return fail("ame_stream_create_cu_range: NULL");
    const int cus = device_cus();
    if (first_cu < 0 || num_cus < 1 || first_cu + num_cus > cus)
        return fail("ame_stream_create_cu_range: CUs [%d, %d) outside the device", first_cu,
                    first_cu + num_cus);
    uint32_t mask[(AME_MAX_CUS + 31) / 32] = {0};
    if (cus > AME_MAX_CUS) return fail("ame_stream_create_cu_range: %d CUs", cus);
    for (int c = first_cu; c < first_cu + num_cus; ++c) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)((cus + 31) / 32), mask);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_stream_create_cu_range: %s", hipGetErrorString(e));
        return -1;
    }
    *stream = (void*)s;
    return 0;
}

int ame_stream_destroy(void* stream) {
    if (!stream) return fail("ame_stream_destroy: NULL");
    return hipStreamDestroy((hipStream_t)stream) == hipSuccess ? 0 : fail("ame_stream_destroy failed");
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

__global__ void ame_peer_probe_kernel(unsigned long long* dst, unsigned long long v) {
    if (threadIdx.x == 0) {
        __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
}

int ame_peer_probe(void* peer_dev, unsigned long long value) {
    if (!peer_dev) return fail("ame_peer_probe: NULL");
    hipLaunchKernelGGL(ame_peer_probe_kernel, dim3(1), dim3(64), 0, 0,
                       (unsigned long long*)peer_dev, value);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_peer_probe: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int ame_peer_read_u64(const void* own_dev, unsigned long long* out) {
    if (!own_dev || !out) return fail("ame_peer_read_u64: NULL");
    hipError_t e = hipMemcpy(out, own_dev, sizeof(*out), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_peer_read_u64: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

int ame_peer_clear(void* own_dev, unsigned long long bytes) {
    if (!own_dev || bytes == 0) return fail("ame_peer_clear: bad arguments");
    hipError_t e = hipMemset(own_dev, 0, (size_t)bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "ame_peer_clear: %s", hipGetErrorString(e));
        return -1;
    }
    return 0;
}

static int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return cus;
}

static bool v2_block_in_lds(int n, int r) { return !sweep_lds_layout(n, r, 0).m_global; }
static bool v2_single_fits(int n, int r) { return sweep_lds_layout(n, r, 1).total <= AME_LDS_MAX; }
static bool is_concrete(int k) {
    return k == AME_SWEEP_V3 || k == AME_SWEEP_V2_LDS || k == AME_SWEEP_V2_HBM || k == AME_SWEEP_V2_WORKERS ||
           k == AME_SWEEP_V2_PIPE || k == AME_SWEEP_V2_W6;
}

// Request -> concrete kernel for these dims (-1 + message when it cannot run).
// The choice depends only on the request and the shape: nothing reads the
// environment, so a caller that sized its buffers for a kind gets that kind.
static int resolve_kind(const ame_dims* d, int request) {
    const int n = d->n, r = d->r;
    switch (request) {
        case AME_SWEEP_AUTO:
            if (ame_sweep3_supported(n, r)) return AME_SWEEP_V3;
            // fall through
        case AME_SWEEP_V2_AUTO:
            if (ame_sweep_workers_fit(d, 2)) return AME_SWEEP_V2_WORKERS;
            // fall through
        case AME_SWEEP_V2_SINGLE:
            if (v2_block_in_lds(n, r)) return AME_SWEEP_V2_LDS;
            if (v2_single_fits(n, r)) return AME_SWEEP_V2_HBM;
            return fail("ame_sweep: no sweep kernel fits n=%d, r=%d", n, r);
        case AME_SWEEP_V3:
            if (ame_sweep3_supported(n, r)) return AME_SWEEP_V3;
            return fail("ame_sweep: the v3 sweep does not fit n=%d, r=%d", n, r);
        case AME_SWEEP_V2_LDS:
            if (v2_block_in_lds(n, r)) return AME_SWEEP_V2_LDS;
            return fail("ame_sweep: the (U,V) block of n=%d, r=%d does not fit in LDS", n, r);
        case AME_SWEEP_V2_HBM:
            if (v2_single_fits(n, r)) return AME_SWEEP_V2_HBM;
            return fail("ame_sweep: the v2 sweep does not fit n=%d, r=%d", n, r);
        case AME_SWEEP_V2_WORKERS:
            if (ame_sweep_workers_fit(d, 2)) return AME_SWEEP_V2_WORKERS;
            return fail("ame_sweep: GEMV workers do not fit n=%d, T_local=%d", n, d->T_local);
        case AME_SWEEP_V2_PIPE:
            if (ame_sweep_workers_fit(d, 3)) return AME_SWEEP_V2_PIPE;
            return fail("ame_sweep: the pipelined GEMV-worker sweep does not fit n=%d, T_local=%d",
                        n, d->T_local);
        case AME_SWEEP_V2_W6:
            if (ame_sweep_workers_fit(d, 4)) return AME_SWEEP_V2_W6;
            return fail("ame_sweep: the six-worker sweep does not fit n=%d, T_local=%d", n, d->T_local);
        default:
            return fail("ame_sweep: unknown sweep kind request %d", request);
    }
}

long long ame_sweep_lds_bytes(int n, int r, int kind) {
    if (!r_supported(r) || n < 1) return 0;
    switch (kind) {
        case AME_SWEEP_V3: return ame_sweep3_supported(n, r) ? ame_sweep3_lds(n, r) : 0;
        case AME_SWEEP_V2_LDS: return ame_v2_mode_lds(n, r, 0);
        case AME_SWEEP_V2_HBM: return ame_v2_mode_lds(n, r, 1);
        case AME_SWEEP_V2_WORKERS: return ame_v2_mode_lds(n, r, 2);
        case AME_SWEEP_V2_PIPE: return ame_v2_mode_lds(n, r, 3);
        case AME_SWEEP_V2_W6: return ame_v2_mode_lds(n, r, 4);
        default: return 0;
    }
}

int ame_sweep_max_slices(int n, int r, int request) {
    if (!r_supported(r) || n < 2) return 0;
    const int cus = device_cus();
    switch (request) {
        case AME_SWEEP_AUTO:
            if (ame_sweep3_supported(n, r)) return ame_sweep3_blocks_per_cu(n, r) * cus;
            // fall through
        case AME_SWEEP_V2_AUTO:
        case AME_SWEEP_V2_SINGLE:
            if (v2_block_in_lds(n, r)) return ame_sweep_blocks_per_cu(n, r, 0) * cus;
            return v2_single_fits(n, r) ? ame_sweep_blocks_per_cu(n, r, 1) * cus : 0;
        case AME_SWEEP_V3:
            return ame_sweep3_supported(n, r) ? ame_sweep3_blocks_per_cu(n, r) * cus : 0;
        case AME_SWEEP_V2_LDS:
            return v2_block_in_lds(n, r) ? ame_sweep_blocks_per_cu(n, r, 0) * cus : 0;
        case AME_SWEEP_V2_HBM:
            return v2_single_fits(n, r) ? ame_sweep_blocks_per_cu(n, r, 1) * cus : 0;
        case AME_SWEEP_V2_WORKERS:
            return ame_sweep_blocks_per_cu(n, r, 2) * cus / (1 + AME_GW);
        case AME_SWEEP_V2_PIPE: {
            ame_dims one = {n, r, 1, 0, 1, 0};
            if (!ame_sweep_workers_fit(&one, 3)) return 0;
            return ame_sweep_blocks_per_cu(n, r, 3) * cus / (1 + AME_GW_P);
        }
        case AME_SWEEP_V2_W6: {
            ame_dims one = {n, r, 1, 0, 1, 0};
            if (!ame_sweep_workers_fit(&one, 4)) return 0;
            return ame_sweep_blocks_per_cu(n, r, 4) * cus / (1 + AME_GW_6);
        }
        default:
            return 0;
    }
}

int ame_sweep_slice_workgroups(int kind) {
    switch (kind) {
        case AME_SWEEP_V3:
        case AME_SWEEP_V2_LDS:
        case AME_SWEEP_V2_HBM: return 1;
        case AME_SWEEP_V2_WORKERS: return 1 + ame_v2_nworkers(2);
        case AME_SWEEP_V2_PIPE: return 1 + ame_v2_nworkers(3);
        case AME_SWEEP_V2_W6: return 1 + ame_v2_nworkers(4);
        default: return fail("ame_sweep_slice_workgroups: %d is not a concrete sweep kind", kind);
    }
}

int ame_sweep_orders_slices(int n, int r, int kind) {
    if (!r_supported(r) || n < 2) return 0;
    if (kind == AME_SWEEP_V3) return ame_sweep3_supported(n, r) ? 1 : 0;
    if (kind == AME_SWEEP_V2_PIPE) {
        ame_dims one = {n, r, 1, 0, 1, 0};
        return ame_sweep_workers_fit(&one, 3) ? 1 : 0;
    }
    return 0;
}

int ame_sweep_kind(const ame_dims* dims, int request) {
    if (check_dims(dims)) return -1;
    return resolve_kind(dims, request);
}

long long ame_sweep_work_size(const ame_dims* dims, int kind) {
    if (check_dims(dims)) return -1;
    switch (kind) {
        case AME_SWEEP_V3: return ame_sweep3_work_doubles(dims);
        case AME_SWEEP_V2_LDS: return 0;
        // [T_local][n][2r] fp32 (U,V) copy
        case AME_SWEEP_V2_HBM: return ((long long)dims->T_local * dims->n * 2 * dims->r + 1) / 2;
        // partial ring, then the precomputed right AR terms
        case AME_SWEEP_V2_WORKERS: return ame_v2_ring_doubles(dims, 2) + ame_v2_arr_doubles(dims);
        case AME_SWEEP_V2_PIPE: return ame_v2_ring_doubles(dims, 3) + ame_v2_arr_doubles(dims);
        case AME_SWEEP_V2_W6: return ame_v2_ring_doubles(dims, 4) + ame_v2_arr_doubles(dims);
        default: return fail("ame_sweep_work_size: %d is not a concrete sweep kind", kind);
    }
}

long long ame_pack_y_size(const ame_dims* dims) {
    if (check_dims(dims)) return -1;
    return (long long)dims->T_local * dims->n * ame_ystride(dims->n) * 2;
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
    const int kind = resolve_kind(dims, a->kind);
    if (kind < 0) return -1;
    if (is_concrete(a->kind) && kind != a->kind)
        return fail("ame_sweep: requested kind %d resolves to %d", a->kind, kind);
    const long long need = ame_sweep_work_size(dims, kind);
    if (need > 0 && (!a->work || a->work_doubles < (unsigned long long)need))
        return fail("ame_sweep: the work buffer holds %d doubles, kind %d needs more", (int)a->work_doubles, kind);
    if (a->wait_epoch != 0 && (!ame_sweep_orders_slices(dims->n, dims->r, kind) || !a->done))
        return fail("ame_sweep: wait_epoch needs a kernel that orders slices (kind %d) and a done array", kind);
    const int maxs = (kind == AME_SWEEP_V2_WORKERS || kind == AME_SWEEP_V2_PIPE || kind == AME_SWEEP_V2_W6)
                          ? dims->T_local   // resolve_kind checked that the launch co-resides
                          : ame_sweep_max_slices(dims->n, dims->r, kind);
    if (dims->T_local > maxs)
        return fail("ame_sweep: T_local=%d exceeds co-resident workgroups (%d)", dims->T_local, maxs);
    ame_sweep_args c = *a;
    c.kind = kind;
    if (kind == AME_SWEEP_V3) return launched(ame_sweep3_dispatch(dims, &c, (hipStream_t)stream), "sweep3");
    return launched(ame_sweep_dispatch(dims, &c, (hipStream_t)stream), "sweep");
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
    if (a->pairs_kernel < AME_PAIRS_AUTO || a->pairs_kernel > AME_PAIRS_V2)
        return fail("ame_elbo: bad pairs_kernel %d", a->pairs_kernel);
    return launched(ame_elbo_dispatch(dims, a, (hipStream_t)stream, 0), "elbo");
}

int ame_elbo_pairs_diag(const ame_dims* dims, const ame_elbo_args* a, void* stream) {
    if (int e = check_dims(dims)) return e;
    if (!a || !a->Yt || !a->x || !a->work) return fail("ame_elbo_pairs_diag: NULL buffer");
    if (a->pairs_kernel < AME_PAIRS_AUTO || a->pairs_kernel > AME_PAIRS_V2)
        return fail("ame_elbo_pairs_diag: bad pairs_kernel %d", a->pairs_kernel);
    return launched(ame_elbo_dispatch(dims, a, (hipStream_t)stream, 1), "elbo_pairs");
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
