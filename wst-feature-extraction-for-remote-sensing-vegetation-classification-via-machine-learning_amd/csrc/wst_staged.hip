// HBM-staged kernels (wst_staged.h) of one line length WST_BIG_N, set by the Makefile (0 = the
// runtime-length instantiation); the object built with WST_BIG_COMMON carries the size-independent
// k_big_mean / k_big_final.
#ifdef WST_BIG_COMMON
#define WST_BIG_COMMON_KERNELS
#endif
#include "wst_launch.h"

#if !defined(WST_BIG_N) && !defined(WST_BIG_COMMON)
#error "WST_BIG_N (one object per line length, 0 = runtime length) or WST_BIG_COMMON must be defined"
#endif

namespace wstlaunch {

#ifndef WST_BIG_COMMON
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

// k_big_final holds the oM x oN map of an array in dynamic LDS (wide maps exceed the 64 KiB default)
hipError_t common_attrs() {
    // (less its static reduction scratch: the attribute bounds dynamic + static <= 160 KiB)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(wstbig::k_big_final),
                               hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds - 256);
}

void mean(const Launch& q, const DevParams& dp, const float* in, float* m) {
    hipLaunchKernelGGL(wstbig::k_big_mean, q.grid, q.block, q.lds, q.st, dp, in, m);
}

void final_(const Launch& q, const DevParams& dp, int fmode, int kind, int n, int n_other, int oms,
            const float* part, const float* G, const float* csum, float* mean_out, int L, int j1,
            int l1, int j2, int npath, long long img0, float* out, int pooled) {
    hipLaunchKernelGGL(wstbig::k_big_final, q.grid, q.block, q.lds, q.st, dp, fmode, kind, n, n_other, oms,
                       part, G, csum, mean_out, L, j1, l1, j2, npath, img0, out, pooled);
}

}  // namespace

const BigCommonOps& wst_big_common_ops() {
    static const BigCommonOps ops{common_attrs, mean, final_};
    return ops;
}
#endif

}  // namespace wstlaunch
