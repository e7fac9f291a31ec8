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
// k_o2r level sizes 96 and 48 (wst_wave.h) belong to family 3
constexpr bool kO2r = kSquareFamily && FM == 3;

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
        if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o2<FM, FN, 136, 1, 1>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds)) != hipSuccess)
            return e;
        {
            const void* ks[3] = {reinterpret_cast<const void*>(wstdev::k_o12<FM, FN, 24, 1>),
                                 reinterpret_cast<const void*>(wstdev::k_o12<FM, FN, 48, 1>),
                                 reinterpret_cast<const void*>(wstdev::k_o12<FM, FN, 136, 1>)};
            for (const void* k : ks)
                if ((e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds)) !=
                    hipSuccess)
                    return e;
        }
        if constexpr (kO2r) {
            if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o2r<FM, 96>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds)) != hipSuccess)
                return e;
            if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(wstdev::k_o2r<FM, 48>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, wstdev::kMaxLds)) != hipSuccess)
                return e;
        }
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

bool o2r(int n1c, const Launch& q, const DevParams& dp, const LdsLayout& lay2, int nwl, int j1, int nimg,
         long long img0, const float2* hexp, float* out, int pooled) {
    if constexpr (kO2r) {
        if (n1c == 96) {
            hipLaunchKernelGGL((wstdev::k_o2r<FM, 96>), q.grid, q.block, q.lds, q.st, dp, lay2, nwl, j1, nimg, img0, hexp,
                               out, pooled);
            return true;
        }
        if (n1c == 48) {
            hipLaunchKernelGGL((wstdev::k_o2r<FM, 48>), q.grid, q.block, q.lds, q.st, dp, lay2, nwl, j1, nimg, img0, hexp,
                               out, pooled);
            return true;
        }
    }
    (void)n1c; (void)q; (void)dp; (void)lay2; (void)nwl; (void)j1; (void)nimg; (void)img0; (void)hexp; (void)out;
    (void)pooled;
    return false;
}

bool o12(int cap, const Launch& q, const DevParams& dp, const LdsLayout& lay1, const LdsLayout& lay2, int j1,
         int nimg, long long img0, const float2* xhat, float* out, int pooled) {
    if constexpr (kSquareFamily) {
#define WST_O12_CAP(C)                                                                                \
    if (cap == C) {                                                                                   \
        hipLaunchKernelGGL((wstdev::k_o12<FM, FN, C, 1>), q.grid, q.block, q.lds, q.st, dp, lay1, lay2, j1, \
                           nimg, img0, xhat, out, pooled);                                            \
        return true;                                                                                  \
    }
        WST_O12_CAP(24) WST_O12_CAP(48) WST_O12_CAP(136)
#undef WST_O12_CAP
    }
    (void)cap; (void)q; (void)dp; (void)lay1; (void)lay2; (void)j1; (void)nimg; (void)img0; (void)xhat;
    (void)out; (void)pooled;
    return false;
}

}  // namespace

#define WST_GETTER_NAME(A, B) WST_FAMILY_GETTER(A, B)
#define WST_GETTER_EXPAND(A, B) WST_GETTER_NAME(A, B)
const FamilyOps& WST_GETTER_EXPAND(WST_FAM_M, WST_FAM_N)() {
    static const FamilyOps ops{FM, FN, set_attrs, prep, o1, o2, o2r, o12};
    return ops;
}

}  // namespace wstlaunch

#ifdef WST_STAMPS
// diagnostic read-back of this family's k_o2 phase stamps (WST_STAMPS builds only)
#define WST_STAMP_FN(A, B) wst_dbg_stamps_##A##_##B
#define WST_STAMP_FN2(A, B) WST_STAMP_FN(A, B)
extern "C" int WST_STAMP_FN2(WST_FAM_M, WST_FAM_N)(unsigned long long* host, int n) {
    const int cap = kStampBlocks * kStampSlots;
    return static_cast<int>(hipMemcpyFromSymbol(host, HIP_SYMBOL(wst_stamps),
                                                sizeof(unsigned long long) * (n < cap ? n : cap)));
}
#define WST_CLEAR_FN(A, B) wst_dbg_clear_##A##_##B
#define WST_CLEAR_FN2(A, B) WST_CLEAR_FN(A, B)
extern "C" int WST_CLEAR_FN2(WST_FAM_M, WST_FAM_N)(void) {
    static unsigned long long z[kStampBlocks * kStampSlots];
    return static_cast<int>(hipMemcpyToSymbol(HIP_SYMBOL(wst_stamps), z, sizeof(z)));
}
#endif
