// Routes the r-dependent entry points of the split build (build.py compiles
// ame_sweep.hip in 3 parts, ame_sweep3.hip and ame_elbo.hip in 2; part p holds
// the latent dims r with r % parts == p, ame_common.h) to the part that holds r.
#include "ame_common.h"

#define AME_DECL_SWEEP(P)                                                                 \
    int ame_sweep_dispatch_p##P(const ame_dims*, const ame_sweep_args*, hipStream_t);     \
    int ame_sweep_blocks_per_cu_p##P(int, int, int);                                      \
    int ame_sweep_workers_fit_p##P(const ame_dims*, int);
AME_DECL_SWEEP(0)
AME_DECL_SWEEP(1)
AME_DECL_SWEEP(2)
#define AME_DECL_2(P)                                                                     \
    int ame_sweep3_dispatch_p##P(const ame_dims*, const ame_sweep_args*, hipStream_t);    \
    int ame_sweep3_supported_p##P(int, int);                                              \
    int ame_sweep3_blocks_per_cu_p##P(int, int);                                          \
    int ame_sweep3_lds_p##P(int, int);                                                    \
    int ame_elbo_dispatch_p##P(const ame_dims*, const ame_elbo_args*, hipStream_t, int);
AME_DECL_2(0)
AME_DECL_2(1)

int ame_sweep_dispatch(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    switch (dm->r % 3) {
        case 0: return ame_sweep_dispatch_p0(dm, a, st);
        case 1: return ame_sweep_dispatch_p1(dm, a, st);
        default: return ame_sweep_dispatch_p2(dm, a, st);
    }
}
int ame_sweep_blocks_per_cu(int n, int r, int mode) {
    switch (r % 3) {
        case 0: return ame_sweep_blocks_per_cu_p0(n, r, mode);
        case 1: return ame_sweep_blocks_per_cu_p1(n, r, mode);
        default: return ame_sweep_blocks_per_cu_p2(n, r, mode);
    }
}
int ame_sweep_workers_fit(const ame_dims* dm, int mode) {
    switch (dm->r % 3) {
        case 0: return ame_sweep_workers_fit_p0(dm, mode);
        case 1: return ame_sweep_workers_fit_p1(dm, mode);
        default: return ame_sweep_workers_fit_p2(dm, mode);
    }
}
int ame_sweep3_dispatch(const ame_dims* dm, const ame_sweep_args* a, hipStream_t st) {
    return (dm->r & 1) ? ame_sweep3_dispatch_p1(dm, a, st) : ame_sweep3_dispatch_p0(dm, a, st);
}
int ame_sweep3_supported(int n, int r) {
    return (r & 1) ? ame_sweep3_supported_p1(n, r) : ame_sweep3_supported_p0(n, r);
}
int ame_sweep3_blocks_per_cu(int n, int r) {
    return (r & 1) ? ame_sweep3_blocks_per_cu_p1(n, r) : ame_sweep3_blocks_per_cu_p0(n, r);
}
int ame_sweep3_lds(int n, int r) {
    return (r & 1) ? ame_sweep3_lds_p1(n, r) : ame_sweep3_lds_p0(n, r);
}
int ame_elbo_dispatch(const ame_dims* dm, const ame_elbo_args* a, hipStream_t st, int pairs_only) {
    return (dm->r & 1) ? ame_elbo_dispatch_p1(dm, a, st, pairs_only)
                       : ame_elbo_dispatch_p0(dm, a, st, pairs_only);
}
