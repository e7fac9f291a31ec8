// Launch table between the host plan code (wst_hip.hip) and the kernel instantiations, which are
// compiled per FFT size-family pair in separate translation units (wst_kernels.hip built once per
// pair by the Makefile) so the build runs in parallel and each object carries one family's code.
#pragma once

#include <hip/hip_runtime.h>

#include "wst_device.h"
#include "wst_staged.h"

namespace wstlaunch {

struct Launch {
    dim3 grid, block;
    size_t lds;
    hipStream_t st;
};

using wstdev::DevParams;
using wstdev::LdsLayout;

struct FamilyOps {
    int fm, fn;
    // raise every kernel's dynamic-LDS limit to the full 160 KiB
    hipError_t (*set_attrs)();
    void (*prep)(const Launch&, const DevParams&, const LdsLayout&, const float* in, long long img0,
                 float2* xhat, float* out, int pooled);
    // cap: size class (12/24/48/136); sq: square fused variant (only for fm == fn > 0).
    // false: the selected instantiation is not compiled (wst_compiled.h), nothing was launched
    bool (*o1)(int cap, int sq, const Launch&, const DevParams&, const LdsLayout&, int j1, int nimg,
               long long img0, const float2* xhat, float2* hexp, float* out, int pooled);
    // hg: spectrum of a big level read from HBM (square families, cap 136), paths from j2first
    bool (*o2)(int cap, int sq, int hg, const Launch&, const DevParams&, const LdsLayout&, int j1,
               int nimg, long long img0, const float2* hexp, float* out, int pooled, int j2first);
};

// HBM-staged passes of one line length N (wst_staged.h), compiled per N (wst_staged.hip); n = 0:
// the runtime-length instantiation.
struct BigOps {
    int n;
    hipError_t (*set_attrs)();
    void (*rows)(bool inverse, const Launch&, const DevParams&, const wstbig::BigArgs&);
    void (*cols)(bool inverse, const Launch&, const DevParams&, const wstbig::BigArgs&);
};
// Compiled line lengths; every other length runs the N = 0 instantiation (generic DFT, n at run
// time).  Keep in step with the Makefile's BIGNS.
#define WST_BIG_SIZES(X) X(96) X(144) X(160) X(192) X(256) X(272) X(288) X(320) X(384) X(512)
#define WST_BIG_GETTER(N) wst_big_ops_##N
#define WST_DECLARE_BIG(N) const BigOps& WST_BIG_GETTER(N)();
WST_BIG_SIZES(WST_DECLARE_BIG)
WST_DECLARE_BIG(0)
#undef WST_DECLARE_BIG

// size-independent staged kernels (k_big_mean, k_big_final), in the N = 0 object
struct BigCommonOps {
    hipError_t (*set_attrs)();
    void (*mean)(const Launch&, const DevParams&, const float* in, float* mean);
    void (*final_)(const Launch&, const DevParams&, int fmode, int kind, int n, int n_other, int oms,
                   const float* part, const float* G, const float* csum, float* mean_out, int L,
                   int j1, int l1, int j2, int npath, long long img0, float* out, int pooled);
};
const BigCommonOps& wst_big_common_ops();

// The compiled family pairs (rows, columns); family 0 = generic O(n) DFT.
#define WST_FAMILY_PAIRS(X) \
    X(0, 0) X(1, 1) X(3, 3) X(5, 5) X(7, 7) X(9, 9) X(11, 11) X(13, 13) X(15, 15) X(17, 17) X(27, 27) \
    X(3, 1) X(1, 3)
#define WST_FAMILY_GETTER(A, B) wst_family_ops_##A##_##B
#define WST_DECLARE_GETTER(A, B) const FamilyOps& WST_FAMILY_GETTER(A, B)();
WST_FAMILY_PAIRS(WST_DECLARE_GETTER)
#undef WST_DECLARE_GETTER

}  // namespace wstlaunch
