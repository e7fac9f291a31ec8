// Kernel instantiations of one FFT size-family pair (WST_FAM_M, WST_FAM_N), set by the Makefile:
// k_prep, and k_o1 / k_o2 per size class (caps 12/24/48/136), generic and -- for square families
// -- the bounded, fused-low-pass variant and the global-spectrum k_o2 after a big level
// (wst_device.h).
#include "wst_launch.h"

#ifndef WST_FAM_M
#error "WST_FAM_M / WST_FAM_N must be defined (one object per family pair)"
#endif

namespace wstlaunch {
namespace {

constexpr int FM = WST_FAM_M, FN = WST_FAM_N;
constexpr bool kSquareFamily = (FM == FN) && FM > 0;

template <int C, int SQ>
hipError_t attrs_cap() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o1<FM, FN, C, SQ>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds);
    if (e != hipSuccess) return e;
    return hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o2<FM, FN, C, SQ, 0>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds);
}

template <int SQ>
hipError_t attrs_all() {
    hipError_t e;
    if ((e = attrs_cap<12, SQ>()) != hipSuccess) return e;
    if ((e = attrs_cap<24, SQ>()) != hipSuccess) return e;
    if ((e = attrs_cap<48, SQ>()) != hipSuccess) return e;
    return attrs_cap<136, SQ>();
}

hipError_t set_attrs() {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_prep<FM, FN>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds);
    if (e != hipSuccess) return e;
    if ((e = attrs_all<0>()) != hipSuccess) return e;
    if constexpr (kSquareFamily) {
        if ((e = attrs_all<1>()) != hipSuccess) return e;
        if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o2<FM, FN, 136, 0, 1>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds)) != hipSuccess)
            return e;
        return hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o2<FM, FN, 136, 1, 1>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds);
    }
    return hipSuccess;
}

void prep(const Launch& q, const DevParams& dp, const LdsLayout& lay, const float* in,
          long long img0, float2* xhat, float* out, int pooled) {
    hipLaunchKernelGGL((wstdev::k_prep<FM, FN>), q.grid, q.block, q.lds, q.st, dp, lay, in, img0,
                       xhat, out, pooled);
}

template <int SQ>
void o1_sq(int cap, const Launch& q, const DevParams& dp, const LdsLayout& lay, int j1, int nimg,
           long long img0, const float2* xhat, float2* hexp, float* out, int pooled) {
#define WST_O1_CAP(C)                                                                            \
    if (cap == C) {                                                                              \
        hipLaunchKernelGGL((wstdev::k_o1<FM, FN, C, SQ>), q.grid, q.block, q.lds, q.st, dp, lay, \
                           j1, nimg, img0, xhat, hexp, out, pooled);                             \
        return;                                                                                  \
    }
    WST_O1_CAP(12) WST_O1_CAP(24) WST_O1_CAP(48) WST_O1_CAP(136)
#undef WST_O1_CAP
}

template <int SQ, int HG>
void o2_sq(int cap, const Launch& q, const DevParams& dp, const LdsLayout& lay, int j1, int nimg,
           long long img0, const float2* hexp, float* out, int pooled, int j2first) {
#define WST_O2_CAP(C)                                                                              \
    if (cap == C) {                                                                                \
        hipLaunchKernelGGL((wstdev::k_o2<FM, FN, C, SQ, HG>), q.grid, q.block, q.lds, q.st, dp,   \
                           lay, j1, nimg, img0, hexp, out, pooled, j2first);                       \
        return;                                                                                    \
    }
    if constexpr (HG) {
        WST_O2_CAP(136)
    } else {
        WST_O2_CAP(12) WST_O2_CAP(24) WST_O2_CAP(48) WST_O2_CAP(136)
    }
#undef WST_O2_CAP
}

void o1(int cap, int sq, const Launch& q, const DevParams& dp, const LdsLayout& lay, int j1,
        int nimg, long long img0, const float2* xhat, float2* hexp, float* out, int pooled) {
    if constexpr (kSquareFamily)
        if (sq) return o1_sq<1>(cap, q, dp, lay, j1, nimg, img0, xhat, hexp, out, pooled);
    o1_sq<0>(cap, q, dp, lay, j1, nimg, img0, xhat, hexp, out, pooled);
}

void o2(int cap, int sq, int hg, const Launch& q, const DevParams& dp, const LdsLayout& lay, int j1,
        int nimg, long long img0, const float2* hexp, float* out, int pooled, int j2first) {
    if constexpr (kSquareFamily) {
        // hg: the spectrum in HBM -- after a staged big level (square fused kernels) or exported
        // fully transformed by k_o1 for a wide-output level (plan o2_export)
        if (hg) return sq ? o2_sq<1, 1>(cap, q, dp, lay, j1, nimg, img0, hexp, out, pooled, j2first)
                          : o2_sq<0, 1>(cap, q, dp, lay, j1, nimg, img0, hexp, out, pooled, j2first);
        if (sq) return o2_sq<1, 0>(cap, q, dp, lay, j1, nimg, img0, hexp, out, pooled, j2first);
    }
    o2_sq<0, 0>(cap, q, dp, lay, j1, nimg, img0, hexp, out, pooled, j2first);
}

}  // namespace

#define WST_GETTER_NAME(A, B) WST_FAMILY_GETTER(A, B)
#define WST_GETTER_EXPAND(A, B) WST_GETTER_NAME(A, B)
const FamilyOps& WST_GETTER_EXPAND(WST_FAM_M, WST_FAM_N)() {
    static const FamilyOps ops{FM, FN, set_attrs, prep, o1, o2};
    return ops;
}

}  // namespace wstlaunch
