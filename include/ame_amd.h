/*
 * ame_amd.h — C ABI of the MI355X (gfx950) implementation of the temporal-AME
 * structured / naive mean-field VI hot path.
 *
 * Drop-in boundary.  The reference (Alfieriek/Python-Temporal-AME-SVI) is pure
 * Python: its "interface" for this path is the template-method hooks of
 * BaseVariationalInference (src/inference/base.py:84-125) that fit()
 * (base.py:127-208) calls once per iteration.  Each entry point below replaces
 * one of those hooks (or the loop nest inside it); the Python host classes in
 * ame_amd/inference mirror the reference classes on top of this ABI.
 *
 *   ame_pack_y        replaces nothing in the reference: relayout of the
 *                     observed network Y (n,n,T,2) (temporal_ame.py:174) into
 *                     the time-major (T,n,n,2) layout the kernels stream.
 *   ame_sweep         replaces _update_step -> _update_node_i ->
 *                     _compute_observation_terms (structured_mf.py:211-326,
 *                     naive_mf.py:193-376): the sequential Gauss-Seidel sweep,
 *                     new means AND new (damped) covariances.
 *   ame_cov           the per-(node,time) covariance terms of the ELBO
 *                     (_compute_entropy :202-209, trace terms :142-144, :166,
 *                     :193) of the stored covariances.
 *   ame_elbo          replaces _compute_elbo (structured_mf.py:115-209,
 *                     naive_mf.py:89-191) and
 *                     compute_temporal_reconstruction_error
 *                     (temporal_ame.py:255-291): returns the sufficient sums
 *                     from which the host assembles ELBO and MSE.
 *
 * Conventions: all pointers are DEVICE pointers (hipMalloc / torch CUDA
 * tensors) unless the field says otherwise; `stream` is a hipStream_t (NULL =
 * default stream); no entry point allocates, frees or synchronises.  Return
 * value 0 = launched; negative = argument error (see ame_last_error()).
 * Device-side failures (spin timeout, non-finite pivot) are reported through
 * the `status` word, which the host reads after the iteration.
 *
 * Layouts (row-major, fp32 unless stated):
 *   Yt      [T_local][n][ny][2]   Yt[t][i][j] = Y[i][j][t0+t] of the reference for j < n;
 *                                 ny = n rounded up to even (rows 16-byte aligned), the
 *                                 pad pair j = n (odd n) is zero; ame_pack_y_size()
 *   X mean  [T_local][n][d]       d = 2 + 2r, x = [a, b, U(r), V(r)]
 *   X cov   [T_local][n][d][d]
 *   consts  fp64 [5][d][d]: S0inv, Qinv, PhiT*Qinv*Phi, Qinv*Phi, PhiT*Qinv
 */
#ifndef AME_AMD_H
#define AME_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum ame_variant { AME_GOOD = 0, AME_BAD = 1, AME_NAIVE = 2 };

/* status word bits (device-written) */
#define AME_STATUS_SPIN_TIMEOUT 1u
#define AME_STATUS_HALO_TIMEOUT 2u
#define AME_STATUS_LDS_TIMEOUT 4u   /* intra-workgroup hand-off timed out (internal error) */
/* a hand-off word (done flag, back-channel done word, {epoch, value} granule)
 * carried an epoch the protocol cannot have produced yet: a stale buffer or an
 * unordered host write; the word is not consumed as if it were current */
#define AME_STATUS_STALE_EPOCH 8u

/* The status block: AME_STATUS_WORDS uint32 words (the caller zeroes it once
 * and again after reading a failure).
 *   [0]  AME_STATUS_* bits
 *   [1]  1 once the FIRST failing wait has written its record into [2..8]
 *   [2]  wait site (enum ame_wait_site)     [3] global time slice of the waiter
 *   [4]  node index (0xFFFFFFFF: before the node loop)
 *   [5]  word observed (epoch tag, done value, LDS count)   [6] value expected
 *   [7]  microseconds waited                [8] the sweep's epoch
 *   [9]  device bookkeeping: workgroups inside a cross-rank wait right now
 *   [10] waits that gave up quietly because [0] was already non-zero
 *   [11] microseconds the rank's first slice spun on the left rank's granules
 *   [12] microseconds its last slice spun on the right rank's back channel
 *        ([11], [12] accumulate over sweeps; the caller reads differences)
 * Wait rules (every kernel that spins): a wait gives up quietly -- no bit of its
 * own -- once [0] is non-zero (one failure does not manufacture more); a wait
 * on this GPU (slice -> slice, done flags, LDS counters) restarts its 2 s
 * budget while [9] > 0, since its producer may then sit behind a neighbouring
 * rank, whose own wait has the 10 s budget; a workgroup that failed or gave up
 * stores no done flag, back channel or current-epoch hand-off granule. */
#define AME_STATUS_WORDS 16
enum ame_wait_site {
    AME_WAIT_DONE_SELF = 1,     /* pipelined prologue: done[t] of the previous sweep */
    AME_WAIT_DONE_RIGHT = 2,    /* pipelined prologue: done[t+1] (or the next group's first slice) */
    AME_WAIT_BACK = 3,          /* pipelined prologue: the right rank's back-channel done word */
    AME_WAIT_GRAN_LOCAL = 4,    /* hand-off granule of slice t-1 on this GPU */
    AME_WAIT_GRAN_HALO = 5,     /* hand-off granule of the left rank's last slice */
    AME_WAIT_LDS = 6,           /* intra-workgroup LDS counter */
    AME_WAIT_WORKER_GRAN = 7,   /* GEMV worker: new-mean granule of its slice */
    AME_WAIT_PARTIAL = 8        /* slice workgroup: a GEMV worker's partial */
};

/* float offset of the done word in a back channel of n*d floats */
#define AME_BACK_DONE_OFFSET(nd) ((((nd) + 63) / 64) * 64)

/* Sweep kernels.  Concrete kinds (what ame_sweep launches):
 *   AME_SWEEP_V3          one 512-thread workgroup per slice (solver wave + 7
 *                         helper waves, slice (U,V) in registers/LDS); d <= 64
 *   AME_SWEEP_V2_LDS      one 256-thread workgroup per slice, (U,V) block in LDS
 *   AME_SWEEP_V2_HBM      same, (U,V) block in HBM (args.work)
 *   AME_SWEEP_V2_WORKERS  v2 plus seven GEMV worker workgroups per slice holding
 *                         the (U,V) block in registers (partial ring in args.work)
 *   AME_SWEEP_V2_PIPE     v2 plus four GEMV worker workgroups per slice (5 per
 *                         slice): two launches of up to half the co-resident
 *                         slices fit at once and the kernel orders itself slice
 *                         by slice (done flags, wait_epoch), so sweeps and slice
 *                         groups pipeline like AME_SWEEP_V3; d > 64, n <= 4096
 *   AME_SWEEP_V2_W6       v2 plus six GEMV worker workgroups per slice (7 per
 *                         slice), not pipelined: BASELINE config 5's 32 slices
 *                         hold 224 CUs, so the ELBO kernels can run beside the
 *                         next sweep on the other 32 (CU-masked streams,
 *                         ame_stream_create_cu_range); n <= 4224
 * Requests (resolved by ame_sweep_kind for given dims):
 *   AME_SWEEP_AUTO        V3 when the shape fits it, else AME_SWEEP_V2_AUTO
 *   AME_SWEEP_V2_AUTO     V2_WORKERS when their workgroups are co-resident, else
 *                         AME_SWEEP_V2_SINGLE
 *   AME_SWEEP_V2_SINGLE   V2_LDS when the block fits one CU's LDS, else V2_HBM
 * A concrete kind is also a valid request (resolved to itself or rejected). */
enum ame_sweep_kind_code {
    AME_SWEEP_AUTO = 0,
    AME_SWEEP_V2_SINGLE = 1,
    AME_SWEEP_V2_AUTO = 2,
    AME_SWEEP_V3 = 3,
    AME_SWEEP_V2_LDS = 20,
    AME_SWEEP_V2_HBM = 21,
    AME_SWEEP_V2_WORKERS = 22,
    AME_SWEEP_V2_PIPE = 23,
    AME_SWEEP_V2_W6 = 24
};

/* ame_sweep_args.flags */
#define AME_SWEEP_FLAG_NEXT_GROUP 1u   /* done[T_local] is the next slice group's first slice
                                          (same rank): with wait_epoch, the last slice also
                                          waits for it, as for any other right neighbour */
#define AME_SWEEP_FLAG_PREV_GROUP 2u   /* halo_in is the previous slice group's hand-off
                                          buffer on this GPU, not a neighbouring rank's: the
                                          first slice's wait on it is a local wait (2 s
                                          budget, not counted in status words 9 / 11) */

/* ELBO pair kernels (ame_elbo_args.pairs_kernel): AUTO = V2 (LDS-DMA rows). */
enum ame_pairs_kernel_code { AME_PAIRS_AUTO = 0, AME_PAIRS_V1 = 1, AME_PAIRS_V2 = 2 };

typedef struct ame_dims {
    int32_t n;        /* nodes */
    int32_t r;        /* latent_dim; d = 2 + 2r */
    int32_t T_local;  /* time slices held by this rank */
    int32_t t_begin;  /* global index of local slice 0 */
    int32_t T_total;  /* global number of time steps */
    int32_t variant;  /* enum ame_variant */
} ame_dims;

typedef struct ame_sweep_args {
    const float* Yt;             /* [T_local][n][ny][2] */
    const float* x_old;          /* [T_local][n][d] means before the sweep */
    float* x_new;                /* [T_local][n][d] means after the sweep */
    const float* next_old;       /* [n][d] old means at global slice t_begin+T_local
                                    (right halo), NULL if this rank holds T-1 */
    uint64_t* hand;              /* [T_local][n][d] {epoch,value} granules, lane hand-off */
    const uint64_t* halo_in;     /* [n][d] granules of slice t_begin-1 (left rank), or NULL */
    uint64_t* halo_out;          /* [n][d] granules of slice t_begin+T_local-1 for the right
                                    rank (its peer buffer, ame_peer_open), or NULL */
    float* cov;                  /* [T_local][n][d][d] covariances before the sweep (damped in
                                    place when cov_new is NULL) */
    const double* consts;        /* fp64 [5][d][d] */
    double rinv[4];              /* R_inv row-major (host values) */
    float lr;                    /* learning_rate (damping) */
    float one_minus_lr;          /* (float)(1 - lr) computed in double on the host */
    uint32_t epoch;              /* sweep counter, >= 1, identical on every rank */
    uint32_t* status;            /* [AME_STATUS_WORDS] status block (bits + first-failure record) */
    double* work;                /* scratch, >= ame_sweep_work_size() doubles: 0 for the v3
                                    sweep; the GEMV workers' partial ring (zeroed by the call
                                    itself) and the right-neighbour AR terms (filled by the call)
                                    for v2 with workers (kinds 22 / 23: n = 4096, r = 32, ...);
                                    [T_local][n][2r] fp32 (U,V) copy when v2 keeps the slice in
                                    HBM without workers (kind 21); may be NULL
                                    when the size is 0 */
    float* cov_new;              /* [T_local][n][d][d] damped covariances after the sweep, or NULL
                                    (in place).  A separate buffer lets ame_cov / ame_elbo read
                                    `cov` while the next sweep already runs (engine speculation) */
    uint32_t* done;              /* [T_local] per-slice "finished sweep <epoch>" words (zeroed once by
                                    the caller), or NULL */
    uint32_t wait_epoch;         /* 0, or: slice t starts only once done[t] and done[t+1] reach this
                                    epoch, so the next sweep can be queued while the previous one
                                    (epoch wait_epoch) still runs.  Needs ame_sweep_orders_slices()
                                    and room for both sweeps' workgroups (2 T_local <= max_slices) */
    float* back_out;             /* time-sharded, rank with a left neighbour: that rank's peer
                                    buffer [n*d floats | done word at AME_BACK_DONE_OFFSET] the first
                                    slice fills with its new means when it finishes, or NULL */
    const float* back_in;        /* the right neighbour's back_out: in a pipelined launch
                                    (wait_epoch != 0) it replaces next_old */
    int32_t kind;                /* enum ame_sweep_kind_code: the kernel the caller sized the
                                    buffers for (normally the concrete kind ame_sweep_kind
                                    returned); a request it does not resolve to is rejected */
    uint32_t flags;              /* AME_SWEEP_FLAG_* (0 for one launch over all local slices) */
    uint64_t work_doubles;       /* size of `work` in doubles, checked against
                                    ame_sweep_work_size(dims, kind) */
} ame_sweep_args;

typedef struct ame_cov_args {
    const float* cov;            /* [T_local][n][d][d] */
    const double* consts;        /* fp64 [5][d][d] */
    double* cov_terms;           /* [T_local][n][4] fp64: logdet, trace, tr(Qinv S), tr(S0inv S) */
} ame_cov_args;

typedef struct ame_elbo_args {
    const float* Yt;             /* [T_local][n][ny][2] */
    const float* x;              /* [T_local][n][d] means */
    const float* prev_final;     /* [n][d] means at global slice t_begin-1 (left halo) or NULL */
    const double* cov_terms;     /* [T_local][n][4] from ame_cov */
    const double* consts;        /* fp64 [5][d][d] */
    const double* phi;           /* fp64 [d][d] Phi */
    double rinv[4];
    int32_t swap_consistent;     /* 1: Y[j][i] == swap(Y[i][j]) for all pairs (checked at pack) */
    double* work;                /* scratch, >= ame_elbo_work_size() doubles */
    double* out;                 /* [8] sufficient sums (see ame_elbo doc) */
    int32_t pairs_kernel;        /* enum ame_pairs_kernel_code (0 = default) */
} ame_elbo_args;

/* Relayout Y [n][n][T_total][2] -> Yt [T_local][n][ny][2] for slices
 * [t_begin, t_begin+T_local), and count pairs with Y[j][i] != swap(Y[i][j])
 * into *mismatch (device uint64, caller zeroes it). */
int ame_pack_y(const float* Y, float* Yt, const ame_dims* dims,
               unsigned long long* mismatch, void* stream);

/* Floats of Yt for these dims (T_local * n * ny * 2), -1 on bad dims. */
long long ame_pack_y_size(const ame_dims* dims);

/* One Gauss-Seidel sweep over all n nodes for the local slices: new means and
 * new (damped) covariances.  One workgroup per local slice; all T_local
 * workgroups must be co-resident (see ame_sweep_max_slices).  Reproduces the
 * reference node order exactly: step (i,t) sees new means of nodes j<i at t
 * and of node i at t-1, and old means of nodes j>i at t and of node i at t+1. */
int ame_sweep(const ame_dims* dims, const ame_sweep_args* args, void* stream);

/* 1 when the sweep kernel `kind` (concrete) honours done / wait_epoch, else 0. */
int ame_sweep_orders_slices(int n, int r, int kind);

/* The concrete kernel (enum ame_sweep_kind_code) a request resolves to for
 * these dims, or -1 (unsupported dims, or the requested kernel cannot run
 * them; see ame_last_error).  Nothing in the library reads the environment:
 * the kind is chosen here, by the caller's request, once. */
int ame_sweep_kind(const ame_dims* dims, int request);

/* Scratch doubles ame_sweep needs in args->work for a concrete kind (see the
 * field); -1 on bad dims / kind. */
long long ame_sweep_work_size(const ame_dims* dims, int kind);

/* Largest T_local one ame_sweep launch can hold for (n, r) and a request on
 * this device (all its workgroups co-resident), 0 if the per-slice state does
 * not fit.  For AME_SWEEP_AUTO / V2_AUTO with v2 this counts the slice
 * workgroups alone (workers are then used when they fit, ame_sweep_kind). */
int ame_sweep_max_slices(int n, int r, int request);

/* Workgroups one slice occupies in a launch of a concrete kind (the slice's
 * own plus its GEMV workers; each is one CU's worth of LDS), -1 for a request
 * or an unknown kind.  A caller that confines the sweep to a CU range
 * (ame_stream_create_cu_range) sizes the launch with it. */
int ame_sweep_slice_workgroups(int kind);

/* Dynamic LDS bytes per slice workgroup of a concrete kind (0 = unsupported). */
long long ame_sweep_lds_bytes(int n, int r, int kind);

/* Per-(node, local slice) covariance terms of the ELBO (log|S|, tr S,
 * tr(Qinv S), tr(S0inv S)), fully parallel: 64/(2r) covariances per wave. */
int ame_cov(const ame_dims* dims, const ame_cov_args* args, void* stream);

/* ELBO / reconstruction sufficient sums over the local slices:
 *  out[0] sum_{t, i<j} r^T Rinv r          out[1] sum_{i,t} tr(S_it)
 *  out[2] sum_i mu_i0^T S0inv mu_i0        out[3] sum_i tr(S0inv S_i0)
 *  out[4] sum_{i,t>=1} e^T Qinv e          out[5] sum_{i,t>=1} tr(Qinv S_it)
 *  out[6] sum_{i,t} logdet S_it            out[7] sum_{t, i!=j} |Y_ij - m_ij|^2
 * (slice-0 / t>=1 terms use global time; the host adds the constants). */
int ame_elbo(const ame_dims* dims, const ame_elbo_args* args, void* stream);

/* Scratch doubles ame_elbo needs. */
long long ame_elbo_work_size(const ame_dims* dims);

/* Diagnostic (timing) entry point: launches ONLY the pair kernel of ame_elbo
 * (its per-workgroup partials land in args->work; args->out is NOT written).
 * Not part of an iteration; bench.py times the pair kernel alone with it. */
int ame_elbo_pairs_diag(const ame_dims* dims, const ame_elbo_args* args, void* stream);

/* A HIP stream whose kernels run only on compute units [first_cu, first_cu +
 * num_cus) of the current device (hipExtStreamCreateWithCUMask); *stream
 * receives the hipStream_t.  With AME_SWEEP_V2_W6 the engine puts the sweep on
 * one CU range and the ELBO kernels on the rest, so they run side by side
 * instead of queueing behind the sweep's workgroups.  Replaces nothing in the
 * reference (CPU).  ame_stream_destroy releases it. */
int ame_stream_create_cu_range(int first_cu, int num_cus, void** stream);
int ame_stream_destroy(void* stream);

/* Pin + map host memory for device access; *dev receives the device address
 * (utility; the multi-GPU path uses the peer buffers below). */
int ame_host_register(void* host, unsigned long long bytes, void** dev);
int ame_host_unregister(void* host);

/* Peer hand-off buffers of the time-sharded multi-GPU path (one process per
 * GPU, all on one node, xGMI).  ame_peer_alloc: zeroed fine-grained device
 * memory on the current device plus its IPC handle (AME_PEER_HANDLE_BYTES
 * bytes written to *handle); a neighbour process maps it with ame_peer_open and
 * writes boundary means into it with system-scope stores while the owner's
 * sweep polls it locally.  No host memory is involved.  Replaces nothing in the
 * reference (single process, structured_mf.py:240 loops over all T). */
#define AME_PEER_HANDLE_BYTES 64
int ame_peer_alloc(unsigned long long bytes, void** dev, void* handle);
int ame_peer_free(void* dev);
int ame_peer_open(const void* handle, void** dev);
int ame_peer_close(void* dev);
/* Setup-time pre-flight of one peer link (no sweep involved): ame_peer_probe
 * stores `value` into the first 8 bytes of a MAPPED neighbour buffer from a
 * one-lane kernel on the caller's device (system-scope store + release, the
 * store the sweep's hand-off uses) and waits for it; ame_peer_read_u64 copies
 * the first 8 bytes of an OWNED buffer to the host; ame_peer_clear zeroes an
 * owned buffer again (sentinels must never look like a sweep epoch).  A rank
 * pair whose probe value does not arrive is named before the first sweep
 * instead of the sweep spinning into AME_STATUS_HALO_TIMEOUT. */
int ame_peer_probe(void* peer_dev, unsigned long long value);
int ame_peer_read_u64(const void* own_dev, unsigned long long* out);
int ame_peer_clear(void* own_dev, unsigned long long bytes);

/* ---- post-fit alignment -------------------------------
 * Replaces the per-time-step loops of src/utils/alignment.py:
 * align_temporal_states (:224-321) and compute_alignment_error (:324-385).
 * x_est, x_true: (n, T, d) fp32 device arrays, d = 2 + 2r.
 * ame_align_cross: global_mode = 0 -> cross[T][2][r][r] = U_true^T U_est and
 *   V_true^T V_est per time step (alignment.py:76, called from :211-212);
 *   global_mode = 1 -> cross[2r][2r] = Mbar_true^T Mbar_est of the time-averaged
 *   (U,V) blocks (:293-303), using work (ame_align_work_size doubles).
 * The caller turns each cross block into R = U Vt (svd, det(R) < 0 -> last
 * row of Vt negated, :79-87) and passes the rotations to
 * ame_align_apply: x_out = sign-aligned x_est (additive pair by row sign,
 *   (U,V) rotated then sign-aligned per row, :275-289 / :306-319) and
 *   partials[ame_align_partials_size] = fp64 partial sums of |x_out - x_true|^2. */
long long ame_align_work_size(int n, int T, int r);
long long ame_align_cross_size(int n, int T, int r, int global_mode);
long long ame_align_partials_size(int n, int T);
int ame_align_cross(const float* x_est, const float* x_true, int n, int T, int r, int global_mode,
                    double* cross, double* work, void* stream);
int ame_align_apply(const float* x_est, const float* x_true, int n, int T, int r, int global_mode,
                    const double* rot, float* x_out, double* partials, void* stream);

/* Latent dims compiled into this library (fills up to cap entries, returns count). */
int ame_supported_r(int* out, int cap);

/* Human-readable message for the last argument error on this thread. */
const char* ame_last_error(void);

/* Build/version string (includes the offload arch). */
const char* ame_version(void);

#ifdef __cplusplus
}
#endif
#endif /* AME_AMD_H */
