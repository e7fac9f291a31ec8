// HBM-staged kernels (wst_staged.h) of one big level size WST_BIG_N, set by the Makefile; the
// object built with WST_BIG_N=0 carries the size-independent k_big_mean / k_big_final.
#if defined(WST_BIG_N) && WST_BIG_N == 0
#define WST_BIG_COMMON_KERNELS
#endif
#include "wst_launch.h"

#ifndef WST_BIG_N
#error "WST_BIG_N must be defined (one object per big level size, 0 = common kernels)"
#endif

namespace wstlaunch {

#if WST_BIG_N > 0
namespace {

constexpr int N = WST_BIG_N;

hipError_t set_attrs() {
    hipError_t e;
    const void* ks[4] = {reinterpret_cast<const void*>(wstbig::k_big_rows<N, false>),
                         reinterpret_cast<const void*>(wstbig::k_big_rows<N, true>),
                         reinterpret_cast<const void*>(wstbig::k_big_cols<N, false>),
                         reinterpret_cast<const void*>(wstbig::k_big_cols<N, true>)};
    for (const void* k : ks)
        if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     wstdev::kMaxLds)) != hipSuccess)
            return e;
    return hipSuccess;
}

void rows(bool inverse, const Launch& q, const DevParams& dp, const wstbig::BigArgs& a) {
    if (inverse)
        hipLaunchKernelGGL((wstbig::k_big_rows<N, true>), q.grid, q.block, q.lds, q.st, dp, a);
    else
        hipLaunchKernelGGL((wstbig::k_big_rows<N, false>), q.grid, q.block, q.lds, q.st, dp, a);
}

void cols(bool inverse, const Launch& q, const DevParams& dp, const wstbig::BigArgs& a) {
    if (inverse)
        hipLaunchKernelGGL((wstbig::k_big_cols<N, true>), q.grid, q.block, q.lds, q.st, dp, a);
    else
        hipLaunchKernelGGL((wstbig::k_big_cols<N, false>), q.grid, q.block, q.lds, q.st, dp, a);
}

}  // namespace

#define WST_BIG_NAME(N_) WST_BIG_GETTER(N_)
#define WST_BIG_EXPAND(N_) WST_BIG_NAME(N_)
const BigOps& WST_BIG_EXPAND(WST_BIG_N)() {
    static const BigOps ops{N, set_attrs, rows, cols};
    return ops;
}

#else
namespace {

hipError_t common_attrs() { return hipSuccess; }

void mean(const Launch& q, const DevParams& dp, const float* in, float* m) {
    hipLaunchKernelGGL(wstbig::k_big_mean, q.grid, q.block, q.lds, q.st, dp, in, m);
}

void final_(const Launch& q, const DevParams& dp, int fmode, int kind, int n, int oms,
            const float* part, const float* G, const float* csum, float* mean_out, int L, int j1,
            int l1, int j2, int npath, long long img0, float* out, int pooled) {
    hipLaunchKernelGGL(wstbig::k_big_final, q.grid, q.block, q.lds, q.st, dp, fmode, kind, n, oms,
                       part, G, csum, mean_out, L, j1, l1, j2, npath, img0, out, pooled);
}

}  // namespace

const BigCommonOps& wst_big_common_ops() {
    static const BigCommonOps ops{common_attrs, mean, final_};
    return ops;
}
#endif

}  // namespace wstlaunch
