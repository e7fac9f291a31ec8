// Device side of the MI355X wavelet scattering transform: LDS helpers and the three kernels.
//
// Replaces kymatio 0.3.0's scattering2d cascade as reached from the
// reference at src/training/train_and_save_model.py:359-376 and src/inference/inference.py:242-257.
//
// Per chunk of planes (plane = one channel of one patch):
//   k_prep  (1 WG / plane)            reflect-pad gather -> S0 (separable spatial low-pass) ->
//                                     mean-centred forward 2-D FFT -> Xhat (workspace)
//   k_o1    (1 WG / (plane, theta1))  fold(Xhat * psi0) -> inverse FFT, |.| fused -> S1 low-pass
//                                     -> mean-centred real-input row FFT (two rows per complex
//                                     row) -> Hermitian half-spectrum rows -> workspace
//   k_o2    (1 WG / (plane, theta1))  half-spectrum column FFTs -> for every (j2 > j1, theta2):
//                                     Hermitian fold(U1hat * psi) -> inverse FFT, |.| fused ->
//                                     S2 low-pass
// Each kernel stays under ~80 KiB of LDS at the headline geometry (96^2 planes), so two
// workgroups share a CU and one's barriers overlap the other's work.
//
// Exact rewrites (identities of the kymatio algorithm, not approximations):
//   * sub(Y, k) then ifft at n/k  ==  ifft at n then spatial decimation by k;
//   * phi low-pass + subsample + ifft + unpad == a separable spatial filter evaluated only at the
//     kept output points (phi_hat levels are outer products of 1-D masked crops);
//   * constants are removed before the psi paths (psi_hat(0) ~ 1e-16, reflect padding preserves
//     constants), which conditions the fp32 band-pass content;
//   * U1 is real, so U1hat(-k) = conj(U1hat(k)): only columns 0..n/2 are formed and stored.
#pragma once

#include <hip/hip_runtime.h>

#include "fft_lds.h"

// Phase-skipping ablation mask (DevParams::dbg_skip): compiled in only for diagnostic builds
// (-DWST_DIAG); production kernels see a constant 0 and carry no skip branches.
#ifdef WST_DIAG
#define WST_DBG_MASK(p) ((p).flags & 0x3fffffff)
#else
#define WST_DBG_MASK(p) 0
#endif

namespace wstdev {

// s = 2 order-2 fold / order-1 product fused with the rows' stage A from these row lengths on
// (compile-time square levels); elements whose fold loads one fused unit keeps in flight
constexpr int kFuseMin = 48;
constexpr int kFuse1Min = 48;
#ifndef WST_FUSE_GROUP   // A/B builds (tools/variant.sh -DWST_FUSE_GROUP=n)
#define WST_FUSE_GROUP 4
#endif
constexpr int kFuseGroup = WST_FUSE_GROUP;
// SQ k_o2 of size classes up to this cap: B holds all L paths of the first order-2 level too (host:
// bcap), so that level runs as one batch instead of L / 2 filter-pair batches (c2 k_o2 j1 = 2
// 0.160 -> 0.122 ms per step; at the 48 class, j1 = 1, 0.509 -> 0.604: the larger B cuts the
// workgroups per CU from 7 to 3)
constexpr int kWholeFirstCap = 24;
// Row split of the order-2 paths whose s = 2 fold is fused with the rows' stage A (0: split_n2):
// 48 = 6 x 8 gives the fused phase 384 units of 6 elements per filter pair instead of 288 of 8 on
// 512 threads.  The columns keep split_n2 (grouped column partials); the S2 pass reads each
// logical column's partial from its position in the rows' order (cols_modlp RS).
constexpr int fused_row_n2(int n) { return n == 48 ? 8 : 0; }
// Column split of the fused column pass + |.| + S2 (cols_modlp; 0: split_n2).  The tap matrices GM
// are built for split_n2's digit-reversed row order; another split reads each physical row's taps
// from that row's position in split_n2's order (cols_modlp, needs split_n2's N1 divisible by its N1).
#ifndef WST_COL48_N2   // A/B builds (tools/variant.sh -DWST_COL48_N2=n)
#define WST_COL48_N2 12
#endif
constexpr int fused_col_n2(int n) { return n == 48 ? WST_COL48_N2 : 0; }
constexpr int kPrepBatch = 8;   // k_prep gather loads per thread in flight
#ifndef WST_O1_PACK_HALF   // A/B builds (tools/variant.sh -DWST_O1_PACK_HALF=0: k_o1 packs rows 2r, 2r + 1)
#define WST_O1_PACK_HALF 1
#endif


constexpr int kMaxLds = 160 * 1024;
constexpr int kMaxO = 8;  // outputs per thread per generic-DFT chunk

// Kernel-side description of a plan (POD, passed by value).
struct DevParams {
    int M, N, PM, PN, J, L, max_order, pre_pad, K;
    int mM, mN, oM, oN, padTop, padLeft;
    int flags;                    // bits 0-29: timing-ablation mask (env WST_DEBUG_SKIP, WST_DIAG
                                  // builds only); kFlagTrace: variant trace on (wst_plan_trace)
    const float* psi;             // concatenated psi Fourier levels (fp32)
    const long long* psi_off;     // [(j*L + l)*J + r]
    const float* lp;              // spatial low-pass taps per level, each stored twice
    const int* lp_off;            // [2r] -> hM[r], [2r+1] -> hN[r]  (r < J); [2J] = total
    const float2* tw;             // twiddle tables exp(-2 pi i k / n)
    const int* tw_off;            // [2r] -> n = PM>>r, [2r+1] -> n = PN>>r (r <= J); [2J+2] = total
    const int* perm;              // digit-reversal maps: physical position -> logical index
    const int* perm_off;          // [2r], [2r+1] (r <= J); [2J+2] = total
    const int* o2_base;           // first order-2 coefficient of each n1 = j1*L + l1
    const float2* psi2;           // order-2 filters, 2 consecutive l2 interleaved per bin
    const long long* psi2_off;    // [(j2*J + r)*ceil(L/2) + q] -> level r of l2 in {2q, 2q+1}
    const int* box;               // order-2 alias boxes: per pair, nM2 row then nN2 column
                                  // entries (first alias | count << 8); pairs of one (j2, r)
                                  // contiguous, stride box_stride[j2]
    const int* box_off;           // [j2*J + r] -> first pair's entries
    const int* box1_off;          // order-1 boxes (same pool, s >= 4): [j*L + l] -> nM1 + nN1
                                  // entries of psi_{j,l} at level 0, -1 = dense
    int box1_min_s;               // smallest order-1 alias count using the box-sparse fold
    const float* lpt;             // low-pass tap matrices in physical (digit-reversed) order:
    const int* lpt_off;           // [2r] GM_r (PM>>r rows x kLpOM), [2r+1] GN_r (PN>>r x oN)
    // wide tap matrices for the MFMA low-pass (max(oM, oN) > kLpOM): GMw_r (PM>>r rows x oMp)
    // and GNw_r (PN>>r rows x oNp), columns zero-padded to multiples of 16; [2r + d] in physical
    // order (r < J), [2J + d] level 0 in natural order (k_prep)
    const float* lpw;
    const int* lpw_off;
    int oMp, oNp;
    // order-2 tile tap lists of square levels at s = 4 / 8 (fold2_tile_list): per (j2, r) the
    // headers of pair 0's tiles at taph + taph_off[j2*J + r] (int4 {first tap, direct groups of 4,
    // mirrored groups of 4, 0} per (pair, tile of 64 bins)); taps: (LDS byte offset, filter byte
    // offset) pairs relative to a lane's bases
    const int4* taph;
    const int* taph_off;
    const int2* taps;
};
// DevParams::flags bit: the variant trace is on; its words follow the o2_base table (J L ints).
// (No separate pointer: one more kernel argument made the headline k_o2 spill SGPRs, +3 %.)
constexpr int kFlagTrace = 1 << 30;

// Per-launch LDS layout (byte offsets) and the table slices copied into LDS.
struct LdsLayout {
    int off_b;              // second data region (k_o2: B batches)
    int off_tw, tw0, ntw;   // twiddles: M block [tw0, tw0+ntw) then N block [twn0, twn0+ntwn)
    int twn0, ntwn;         //   (ntwn == 0: square kernel, N tables == M tables)
    int off_lp, lp0, nlp;   // low-pass taps
    int off_pm, pm0, npm;   // permutations
    int off_lt, lt0, nlt;   // low-pass tap matrices (lpt pool): GM block, then GN block
    int ltn0, nltn;         //   (nltn == 0: square kernel, GN == GM)
    int oms;                // row stride of the tap matrices (4 or kLpOM)
    int off_s, off_red;     // S (coefficients) and reduction scratch
    int bcap;               // complex capacity of B (k_o2)
    int xs;                 // bit 0 (k_o1): export the fully transformed half spectra (natural order)
                            // for a k_o2 that folds from HBM (HG = 1) instead of the row-transformed
                            // ones; bits 1..: the launch's variant-trace site (kFlagTrace).  One
                            // field: a separate site field made the headline k_o2 1.3 % slower
                            // (its kernel arguments grew; measured, round 5)
    int nsplit;             // k_o2 HG: workgroups per (plane, theta1), batch b run by workgroup
                            // b % nsplit; one item's workgroups share an XCD (its L2 holds H)
    int hgroup;             // k_o2 HG split: items per dispatch group of an XCD; within a group
                            // the slots run batch-major (one batch of hgroup items, then the next)
    int hext;               // resident levels: an item's half spectrum in the workspace holds
                            // nM1 + 1 rows (row nM1 = row 0 for the tile folds' mirrored taps;
                            // written by an exporting k_o1, formed in LDS by k_o2 otherwise)
};
__host__ __device__ inline int export_full(const LdsLayout& l) { return l.xs & 1; }
__host__ __device__ inline void set_export_full(LdsLayout& l) { l.xs |= 1; }
__host__ __device__ inline int get_tslot(const LdsLayout& l) { return l.xs >> 1; }
__host__ __device__ inline void set_tslot(LdsLayout& l, int s) { l.xs = (l.xs & 1) | (s << 1); }

// ------------------------------------------------------------------------------------------
// Variant trace (tests: wst_plan_trace / wst_describe_variants, include/wst_hip.h).  With
// kFlagTrace set in DevParams::flags, workgroup 0 of every traced launch writes kTraceW words at its site
// (LdsLayout::tslot / BigArgs::tslot): word 0 the kernel instantiation, word 1 the body it
// dispatched to at run time, words 2.. (k_o2) the branch of each order-2 level it ran (index
// j2 - j1 - 1).  The host mirror in wst_hip.hip (describe_chunk) predicts the same words from the
// plan alone; tests/test_variants*.py check the two agree on the GPU and that the GPU oracle tests'
// geometries reach every variant a geometry can select.  Plain vector stores by one lane.
// ------------------------------------------------------------------------------------------
constexpr int kTraceW = 12;
constexpr int kTraceSites = 512;
enum TraceKind : int { kTkPrep = 1, kTkO1 = 2, kTkO2 = 3, kTkBigRows = 4, kTkBigCols = 5 };
// low-pass forms: tap matrices (SQ), MFMA with compile-time K, MFMA, 1-D taps
enum TraceLp : int { kLpTap = 0, kLpMfmaRc = 1, kLpMfma = 2, kLpPlain = 3 };
// order-2 fold forms
enum TraceFold : int { kFdFused = 1, kFdTileS2 = 2, kFdTileList = 3, kFdDenseS2 = 4, kFdBox = 5 };
constexpr int tr_log2(int v) {
    int l = 0;
    while (v > 1) {
        v >>= 1;
        ++l;
    }
    return l;
}
// word 0: kind | family M | family N | size class (or staged line length) | SQ | HG (INV)
constexpr int tr_kernel(int kind, int fm, int fn, int cap, int sq, int hg) {
    return (kind << 28) | (fm << 22) | (fn << 16) | (cap << 4) | (sq << 1) | hg;
}
// k_prep body: compile-time size | low-pass form
constexpr int tr_prep(int pc, int lp) { return pc | (lp << 8); }
// k_o1 body: OC | compile-time level size | fused s = 1 fold + row stage A | S1 low-pass form |
// order 2 follows | exports the full spectrum | order-1 fold form (0 fused, 1 s=1, 2 s=2, 3 box,
// 4 s=4, 5 runtime s)
constexpr int tr_o1(int oc, int n1c, int fused1, int lp, int do2, int exp, int fold) {
    return oc | (n1c << 4) | (fused1 << 12) | (lp << 13) | (do2 << 15) | (exp << 16) | (fold << 17);
}
// k_o2 body: OC | LC | compile-time level size | spectrum load (0 HBM fold, 1 first column stage
// from the workspace, 2 copy) | level-dispatch branch (1 N1C, 2-4 HG compile-time / exported /
// runtime after a big level, 5-6 exported-spectrum compile-time / runtime, 7 runtime)
constexpr int tr_o2(int oc, int lc, int n1c, int spec, int branch) {
    return oc | (lc << 4) | (n1c << 9) | (spec << 17) | (branch << 19);
}
// order-2 level: valid | log2 s | low-pass form | fold form | compile-time path size | log2 SC
// (0: runtime) | PB | j2
constexpr int tr_level(int j2, int pb, int sc, int nc, int fold, int lp, int s2) {
    return 1 | (tr_log2(s2) << 1) | (lp << 5) | (fold << 7) | (nc << 10) | ((sc ? tr_log2(sc) : 0) << 18) |
           (pb << 21) | (j2 << 26);
}
// staged passes: mode (3 bits) | fold_all | order-1 fold form (1 s = 1, 2 s > 1) | box fold | wide
// maps | tap matrix in LDS | U stored
constexpr int tr_big(int mode, int fold_all, int fold1, int box, int wide, int glds, int ustore) {
    return mode | (fold_all << 3) | (fold1 << 4) | (box << 6) | (wide << 7) | (glds << 8) | (ustore << 9);
}
// The writer of a site: lane 0 of workgroup 0, only while tracing.  Callers wrap the whole
// word computation in `if (tracing(p, tslot))` so a production launch (kFlagTrace clear) skips
// it with one uniform branch.  Compiled in only with -DWST_TRACE (libwst_hip_trace.so, the tests'
// build): any trace code in the product kernels cost 1-2.5 % (measured, round 5).
__device__ __forceinline__ bool tracing(const DevParams& p, int tslot) {
#ifndef WST_TRACE   // product library: no trace code at all (any form of it measured 1-2.5 % on the
                    // headline kernels); libwst_hip_trace.so is the same sources with -DWST_TRACE
    (void)p;
    (void)tslot;
    return false;
#endif
    return (p.flags & kFlagTrace) && tslot >= 0 && tslot < kTraceSites && threadIdx.x == 0 &&
           blockIdx.x == 0 && blockIdx.y == 0;
}
__device__ __forceinline__ void trace_word(const DevParams& p, int tslot, int k, int v) {
    const_cast<int*>(p.o2_base)[p.J * p.L + tslot * kTraceW + k] = v;
}

// ------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------
// wave index within the workgroup as a provably uniform (scalar) value
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ int reflect_index(int i, int n) {
    // numpy.pad(mode='reflect') for any pad width: even periodic extension, period 2(n-1)
    if (n == 1) return 0;
    const int period = 2 * (n - 1);
    int t = i % period;
    if (t < 0) t += period;
    return t < n ? t : period - t;
}

// Sum over aligned groups of G lanes (G a power of two <= 64), every lane of a group receiving the
// group's sum.  Within a row of 16 lanes the steps are DPP-modified moves (quad_perm [1,0,3,2],
// [2,3,0,1], row_half_mirror, row_mirror): VALU work instead of ds_bpermute round trips through the
// LDS crossbar.  A whole group must be active (the callers' loop bounds are multiples of G).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                                 0xF, 0xF, false));
}
template <int G>
__device__ __forceinline__ float group_sum(float v) {
    static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "group size");
    if constexpr (G >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
    if constexpr (G >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
    if constexpr (G >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
    if constexpr (G >= 16) v += dpp_mov<0x140>(v); // row_mirror
    if constexpr (G >= 32) v += __shfl_xor(v, 16, 64);
    if constexpr (G >= 64) v += __shfl_xor(v, 32, 64);
    return v;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float s = 0.f;
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) s += red[w];
    return s;
}

// |z| * scale stored as a real value (.y = 0); accumulates the per-thread sum (for means)
struct EpiModulus {
    float scale;
    float sum;
    __device__ float2 operator()(float2 z) {
        const float m = __builtin_amdgcn_sqrtf(fmaf(z.x, z.x, z.y * z.y)) * scale;   // v_sqrt_f32
        sum += m;
        return make_float2(m, 0.f);
    }
};

// Row-major iteration of an (rows x cols) grid with stride blockDim.x, division-free.
struct GridIter {
    int u, v, du, dv, cols;
    __device__ __forceinline__ GridIter(int cols_) : cols(cols_) {
        u = threadIdx.x / cols;
        v = threadIdx.x - u * cols;
        du = blockDim.x / cols;
        dv = blockDim.x - du * cols;
    }
    __device__ __forceinline__ void next() {
        u += du;
        v += dv;
        if (v >= cols) {
            v -= cols;
            ++u;
        }
    }
};

// Generic O(n) DFT along lines (fallback family 0).  Lines are processed in chunks of whole lines
// that fit the register tile: read phase -> barrier -> write phase.  Ends with a barrier.
template <class Epi>
__device__ __forceinline__ void lds_dft_lines_generic(float2* base, const wstfft::Lines g, int n,
                                                      const float2* tw, bool inverse, Epi& epi) {
    const int T = blockDim.x;
    const int lines_total = g.nlines();
    int lpc = (T * kMaxO) / n;
    if (lpc < 1) lpc = 1;
    const float sgn = inverse ? -1.f : 1.f;
    for (int l0 = 0; l0 < lines_total; l0 += lpc) {
        const int nlc = min(lpc, lines_total - l0);
        const int nout = nlc * n;
        float2 acc[kMaxO];
        int addr[kMaxO];
#pragma unroll
        for (int i = 0; i < kMaxO; ++i) {
            const int o = threadIdx.x + i * T;
            addr[i] = -1;
            acc[i] = make_float2(0.f, 0.f);
            if (o < nout) {
                const int lc = o / n;
                const int k = o - lc * n;
                const int off = g.offset(l0 + lc);
                const float2* src = base + off;
                float sr = 0.f, si = 0.f;
                int idx = 0;
                for (int e = 0; e < n; ++e) {
                    const float2 x = src[e * g.es];
                    const float2 w = tw[idx];
                    const float wy = sgn * w.y;
                    sr = fmaf(x.x, w.x, fmaf(-x.y, wy, sr));
                    si = fmaf(x.x, wy, fmaf(x.y, w.x, si));
                    idx += k;
                    if (idx >= n) idx -= n;
                }
                acc[i] = make_float2(sr, si);
                addr[i] = off + k * g.es;
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kMaxO; ++i)
            if (addr[i] >= 0) base[addr[i]] = epi(acc[i]);
    }
    __syncthreads();
}

// Line-transform orders: natural -> natural (transposing store rounds), natural -> digit-reversed
// (in place, F_DR) and digit-reversed -> natural (in place, G).
enum { kNat = 0, kDR = 1, kRD = 2 };

template <int FAM, int K, int LO, int HI, int KIND, bool INV, class Epi>
__device__ __forceinline__ void family_fft(float2* base, const wstfft::Lines& g, int n,
                                           const float2* tw, Epi& epi) {
    constexpr int NN = FAM << K;
    if constexpr (NN <= HI && NN <= wstfft::kMaxFamilyN) {
        if constexpr (NN >= 2 && NN > LO) {
            if (n == NN) {
                if constexpr (KIND == kNat) wstfft::fft_lines<NN, INV>(base, g, tw, epi);
                else if constexpr (KIND == kDR) wstfft::fft_lines_dr<NN, INV>(base, g, tw, epi);
                else wstfft::fft_lines_rd<NN, INV>(base, g, tw, epi);
                return;
            }
        }
        family_fft<FAM, K + 1, LO, HI, KIND, INV>(base, g, n, tw, epi);
    }
}

// n-point transforms along lines.  FAM > 0: the compiled FFTs n = FAM * 2^k in (LO, HI] (a plan's
// level sizes always belong to its family; the bounds keep a kernel's code to the sizes its
// launches can meet); FAM == 0: generic DFT (natural order for every KIND; the plan's
// permutation maps are then identity).
template <int FAM, int LO, int HI, int KIND, bool INV, class Epi>
__device__ __forceinline__ void lds_fft_lines(float2* base, const wstfft::Lines g, int n,
                                              const float2* tw, Epi& epi) {
    if constexpr (FAM > 0)
        family_fft<FAM, 0, LO, HI, KIND, INV>(base, g, n, tw, epi);
    else
        lds_dft_lines_generic(base, g, n, tw, INV, epi);
}

// 2-D transform of nb (rows x cols) arrays with row stride ld (odd), spaced bs apart; `epi` is
// applied to the final (column-pass) stores.
template <int FM, int FN, int LO, int HI, int KIND, bool INV, class Epi>
__device__ __forceinline__ void lds_fft2(float2* buf, int nb, int bs, int rows, int cols, int ld,
                                         const float2* twR, const float2* twC, Epi& epi) {
    wstfft::EpiIdentity id;
    lds_fft_lines<FN, LO, HI, KIND, INV>(buf, wstfft::Lines{nb, bs, rows, ld, 1}, cols, twC, id);
    lds_fft_lines<FM, LO, HI, KIND, INV>(buf, wstfft::Lines{nb, bs, cols, 1, ld}, rows, twR, epi);
}

// Separable phi low-pass at the kept output points (unpad folded in):
//   S[b][a][c] = sum_p hM[s(a+1) - p] * sum_q hN[s(c+1) - q] * U[b][p][q]   (indices mod n)
// hM2 / hN2: taps stored twice so s(c+1) + n - q never wraps.  U real in .x, row stride ld;
// permM / permN (nullable): logical index of each physical row / column.  The row partial sums
// T[b][p][c] are parked in the .y slots of row p (the .y of a real array is free), so no scratch.
// Step 1: QC lanes split a row and shuffle-reduce OW columns; step 2: PC lanes split the rows.
template <int OW, int QC, int PC>
__device__ __forceinline__ void lds_lowpass_t(float2* U, int nb, int bs, int rows, int cols, int ld,
                                              const float* hM2, const float* hN2,
                                              const int* permM, const int* permN, int s, int oM,
                                              int oN, float* S) {
    const int T = blockDim.x;
    const int nch = (oN + OW - 1) / OW;
    const int tot1 = nb * rows * nch * QC;
    for (int w = threadIdx.x; w < tot1; w += T) {
        const int qc = w & (QC - 1);
        const int r = w / QC;
        const int ch = r % nch;
        const int bp = r / nch;
        const int b = bp / rows;
        const int p = bp - b * rows;
        const int c0 = ch * OW;
        float2* row = U + b * bs + p * ld;
        const float* h0 = hN2 + cols + s * (c0 + 1);
        float acc[OW];
#pragma unroll
        for (int c = 0; c < OW; ++c) acc[c] = 0.f;
#pragma unroll 2
        for (int q = qc; q < cols; q += QC) {
            const float x = row[q].x;
            const float* hq = h0 - (permN ? permN[q] : q);
#pragma unroll
            for (int c = 0; c < OW; ++c) acc[c] = fmaf(x, hq[s * c], acc[c]);
        }
#pragma unroll
        for (int c = 0; c < OW; ++c) acc[c] = group_sum<QC>(acc[c]);
        if (qc == 0) {
#pragma unroll
            for (int c = 0; c < OW; ++c)
                if (c0 + c < oN) row[c0 + c].y = acc[c];
        }
    }
    __syncthreads();
    const int tot2 = nb * oM * oN * PC;
    for (int w = threadIdx.x; w < tot2; w += T) {
        const int pc = w & (PC - 1);
        const int o = w / PC;
        const int c = o % oN;
        const int a = (o / oN) % oM;
        const int b = o / (oN * oM);
        const float2* t = U + b * bs + c;
        const float* h = hM2 + rows + s * (a + 1);
        float acc = 0.f;
#pragma unroll 2
        for (int p = pc; p < rows; p += PC) acc = fmaf(h[-(permM ? permM[p] : p)], t[p * ld].y, acc);
        acc = group_sum<PC>(acc);
        if (pc == 0) S[o] = acc;
    }
    __syncthreads();
}

// Register-tiled form for large outputs (oN > 8, e.g. 32 x 32 maps of 128^2 planes at J = 2): a
// step-1 thread owns RP rows x OW output columns (each tap read once for RP rows), a step-2 thread
// owns AP x CW outputs (taps and row partials read once per p for the whole tile); QC / PC lanes
// split the reduction index.  Out-of-range tile rows / columns re-read the last valid one and are
// not stored (the tap index stays inside the doubled tables: s * oN <= cols).
template <int RP, int OW, int QC, int AP, int CW, int PC>
__device__ __forceinline__ void lds_lowpass_tiled(float2* U, int nb, int bs, int rows, int cols,
                                                  int ld, const float* hM2, const float* hN2,
                                                  const int* permM, const int* permN, int s, int oM,
                                                  int oN, float* S) {
    const int T = blockDim.x;
    const int npb = (rows + RP - 1) / RP, ncb = (oN + OW - 1) / OW;
    const wstfft::FastDiv dcb(ncb), dpb(npb);
    for (int w = threadIdx.x; w < nb * npb * ncb * QC; w += T) {
        const int qc = w & (QC - 1);
        int t = w / QC;
        const int t1 = dcb.div(t);
        const int cb = t - t1 * ncb;
        const int b = dpb.div(t1);
        const int p0 = (t1 - b * npb) * RP, c0 = cb * OW;
        float2* base = U + b * bs;
        float acc[RP][OW];
#pragma unroll
        for (int r = 0; r < RP; ++r)
#pragma unroll
            for (int c = 0; c < OW; ++c) acc[r][c] = 0.f;
        for (int q = qc; q < cols; q += QC) {
            const float* hq = hN2 + cols + s * (c0 + 1) - (permN ? permN[q] : q);
            float tap[OW];
#pragma unroll
            for (int c = 0; c < OW; ++c) tap[c] = hq[s * min(c, oN - 1 - c0)];
#pragma unroll
            for (int r = 0; r < RP; ++r) {
                const float x = base[min(p0 + r, rows - 1) * ld + q].x;
#pragma unroll
                for (int c = 0; c < OW; ++c) acc[r][c] = fmaf(x, tap[c], acc[r][c]);
            }
        }
#pragma unroll
        for (int r = 0; r < RP; ++r)
#pragma unroll
            for (int c = 0; c < OW; ++c)
                acc[r][c] = group_sum<QC>(acc[r][c]);
        if (qc == 0) {
#pragma unroll
            for (int r = 0; r < RP; ++r)
#pragma unroll
                for (int c = 0; c < OW; ++c)
                    if (p0 + r < rows && c0 + c < oN) base[(p0 + r) * ld + c0 + c].y = acc[r][c];
        }
    }
    __syncthreads();
    const int nab = (oM + AP - 1) / AP, ncw = (oN + CW - 1) / CW;
    const wstfft::FastDiv dcw(ncw), dab(nab);
    for (int w = threadIdx.x; w < nb * nab * ncw * PC; w += T) {
        const int pc = w & (PC - 1);
        int t = w / PC;
        const int t1 = dcw.div(t);
        const int cw = t - t1 * ncw;
        const int b = dab.div(t1);
        const int a0 = (t1 - b * nab) * AP, c0 = cw * CW;
        const float2* base = U + b * bs;
        float acc[AP][CW];
#pragma unroll
        for (int a = 0; a < AP; ++a)
#pragma unroll
            for (int c = 0; c < CW; ++c) acc[a][c] = 0.f;
        for (int p = pc; p < rows; p += PC) {
            const float* hp = hM2 + rows + s * (a0 + 1) - (permM ? permM[p] : p);
            float tap[AP], tv[CW];
#pragma unroll
            for (int a = 0; a < AP; ++a) tap[a] = hp[s * min(a, oM - 1 - a0)];
#pragma unroll
            for (int c = 0; c < CW; ++c) tv[c] = base[p * ld + min(c0 + c, oN - 1)].y;
#pragma unroll
            for (int a = 0; a < AP; ++a)
#pragma unroll
                for (int c = 0; c < CW; ++c) acc[a][c] = fmaf(tap[a], tv[c], acc[a][c]);
        }
#pragma unroll
        for (int a = 0; a < AP; ++a)
#pragma unroll
            for (int c = 0; c < CW; ++c)
                acc[a][c] = group_sum<PC>(acc[a][c]);
        if (pc == 0) {
#pragma unroll
            for (int a = 0; a < AP; ++a)
#pragma unroll
                for (int c = 0; c < CW; ++c)
                    if (a0 + a < oM && c0 + c < oN) S[(b * oM + a0 + a) * oN + c0 + c] = acc[a][c];
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void lds_lowpass(float2* U, int nb, int bs, int rows, int cols, int ld,
                                            const float* hM2, const float* hN2, const int* permM,
                                            const int* permN, int s, int oM, int oN, float* S) {
    if (oN <= 4)
        lds_lowpass_t<4, 8, 16>(U, nb, bs, rows, cols, ld, hM2, hN2, permM, permN, s, oM, oN, S);
    else if (oN <= 8)
        lds_lowpass_t<8, 8, 16>(U, nb, bs, rows, cols, ld, hM2, hN2, permM, permN, s, oM, oN, S);
    else
        lds_lowpass_tiled<4, 8, 8, 4, 4, 8>(U, nb, bs, rows, cols, ld, hM2, hN2, permM, permN, s,
                                             oM, oN, S);
}

// Block-size bound of the exported-spectrum k_o2 (HG, non-SQ: f3 / c1 geometries).  A 512 bound
// lets the compiler use 160 VGPRs instead of the 128 of a 1024 bound (f3: 11 VGPRs spilled), but
// measured: f3 k_o2 1.53 -> 1.94-2.83 ms (256-512 threads), c1 1.50 -> 1.46; kept at 1024.
constexpr int kLpOM = 8;  // row stride of the GM tap matrices = largest oM of the fused path

// Separable phi low-pass on the matrix cores (v_mfma_f32_16x16x4_f32: exact fp32, the fmaf chain
// of the VALU form at the same rate, on the separate matrix pipe), for wide outputs
// (max(oM, oN) > kLpOM: the reference's 128^2 J=2 geometry maps to 32 x 32, 64^2 J=2 to 16 x 16).
// The low-pass at the kept output points is two small GEMMs per array b:
//   1. T[p][c] = sum_q U[p][q] GN[q][c]      (rows x cols) . (cols x oNp), parked in the free .y
//      slots of row p of U (c < oN);
//   2. S[a][c] = sum_p GM[p][a] T[p][c]      (oMp x rows) . (rows x oNp)  -> S (nb x oM x oN).
// U real in .x (row stride ld, array stride bs), in the physical order the tap matrices were
// built for.  GM / GN: global (L2-resident) tap matrices, columns zero-padded to oMp / oNp (x16),
// in MFMA operand order (wst_hip.hip: 16-row blocks of 64 lanes x 4 K steps, then the tail rows
// row-major).
// One wave per 16 x 16 output tile, K in steps of 4 x KU (loads of a step issued together, two
// accumulators alternate so consecutive MFMAs do not wait on each other).  Lane map of the
// 16x16x4 form: A[m = lane & 15][k = lane >> 4], B[k = lane >> 4][n = lane & 15],
// D[row = 4 (lane >> 4) + i][col = lane & 15].  Ends with a barrier.
typedef float f32x4_t __attribute__((ext_vector_type(4)));
// The .x / .y half of an LDS float2 read as one ds_read_b64: the bank argument of the MFMA
// low-pass's operand reads holds for 8-byte reads (the compiler would narrow a plain .x to
// ds_read_b32, which maps a 32-lane half onto 16 even banks: 2-way conflicts at best).
__device__ __forceinline__ float lds_half64(const float2* q, int hi) {
    unsigned long long w = *reinterpret_cast<const unsigned long long*>(q);
    asm volatile("" : "+v"(w));
    return __uint_as_float(static_cast<unsigned>(hi ? (w >> 32) : w));
}
// S addressing: map b, value i = a * oN + c at S[b * s_bs + i * s_es] (default: contiguous maps;
// k_o2 passes the .x slots of the arrays U themselves, free once step 1 has read them).
__device__ __forceinline__ void lds_lowpass_mfma(float2* U, int nb, int bs, int rows, int cols, int ld,
                                                 const float* __restrict__ GM,
                                                 const float* __restrict__ GN, int oMp, int oNp,
                                                 int oM, int oN, float* S, int s_bs = -1, int s_es = 1) {
    if (s_bs < 0) s_bs = oM * oN;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int nmt = (rows + 15) >> 4, nnt = oNp >> 4, nat = oMp >> 4;
    // K parts (host: wst_hip.hip lpw): 64-row blocks (step u reads row 64 b + u + 16 lk: the
    // U operand reads are conflict-free ds_read_b64), 16-row blocks (row 16 b + 4 u + lk), single
    // 4-row steps; no MFMA is issued on an all-padding step (68 rows = 64 + 4 x 1: 17 steps)
    // 1. T = U GN
    const int ntask1 = nb * nmt * nnt;
    for (int t = wave; t < ntask1; t += nw) {
        const int b = t / (nmt * nnt);
        const int r = t - b * nmt * nnt;
        const int mt = r / nnt, nt = r - mt * nnt;
        float2* Ub = U + b * bs;
        const int p = mt * 16 + li;
        const bool pok = p < rows;
        const float2* urow = Ub + (pok ? p : rows - 1) * ld;
        const int n64 = cols >> 6, n16 = (cols - 64 * n64) >> 4;
        const float4* g64 = reinterpret_cast<const float4*>(GN) + (nt * 64 + lane) * 4;
        const float4* g16 = reinterpret_cast<const float4*>(GN) + n64 * nnt * 256 + nt * 64 + lane;
        const float* gcol = GN + (n64 * 4 + n16) * nnt * 256 - (64 * n64 + 16 * n16) * oNp + nt * 16 + li;
        f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        int q0 = 0;
        for (int blk = 0; blk < n64; ++blk, q0 += 64) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {   // two halves of 8 steps (registers)
                const float4 b4a = g64[blk * nnt * 256 + 2 * h];
                const float4 b4b = g64[blk * nnt * 256 + 2 * h + 1];
                const float bv[8] = {b4a.x, b4a.y, b4a.z, b4a.w, b4b.x, b4b.y, b4b.z, b4b.w};
                float a[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float v = lds_half64(urow + q0 + 8 * h + u + 16 * lk, 0);
                    a[u] = pok ? v : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 8; u += 2) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], bv[u], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u + 1], bv[u + 1], acc1, 0, 0, 0);
                }
            }
        }
        for (int blk = 0; blk < n16; ++blk, q0 += 16) {
            const float4 b4 = g16[blk * nnt * 64];
            float a[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] = pok ? urow[q0 + 4 * u + lk].x : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b4.x, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b4.y, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b4.z, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b4.w, acc1, 0, 0, 0);
        }
        for (; q0 < cols; q0 += 4) {
            const int q = q0 + lk;
            const bool ok = q < cols;
            const int qc = ok ? q : 0;
            const float a = (ok && pok) ? urow[qc].x : 0.f;
            const float bv = ok ? gcol[qc * oNp] : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc0, 0, 0, 0);
        }
        const int c = nt * 16 + li;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int pp = mt * 16 + lk * 4 + i;
            if (pp < rows && c < oN) Ub[pp * ld + c].y = acc0[i] + acc1[i];
        }
    }
    __syncthreads();
    // 2. S = GM^T T
    const int ntask2 = nb * nat * nnt;
    for (int t = wave; t < ntask2; t += nw) {
        const int b = t / (nat * nnt);
        const int r = t - b * nat * nnt;
        const int at = r / nnt, ct = r - at * nnt;
        const float2* Ub = U + b * bs;
        const int c = ct * 16 + li;
        const bool cok = c < oN;
        const int n64 = rows >> 6, n16 = (rows - 64 * n64) >> 4;
        const float4* g64 = reinterpret_cast<const float4*>(GM) + (at * 64 + lane) * 4;
        const float4* g16 = reinterpret_cast<const float4*>(GM) + n64 * nat * 256 + at * 64 + lane;
        const float* gcol = GM + (n64 * 4 + n16) * nat * 256 - (64 * n64 + 16 * n16) * oMp + at * 16 + li;
        f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        int p0 = 0;
        for (int blk = 0; blk < n64; ++blk, p0 += 64) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float4 a4a = g64[blk * nat * 256 + 2 * h];
                const float4 a4b = g64[blk * nat * 256 + 2 * h + 1];
                const float av[8] = {a4a.x, a4a.y, a4a.z, a4a.w, a4b.x, a4b.y, a4b.z, a4b.w};
                float bv[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const float v = lds_half64(Ub + (p0 + 8 * h + u + 16 * lk) * ld + (cok ? c : 0), 1);
                    bv[u] = cok ? v : 0.f;
                }
#pragma unroll
                for (int u = 0; u < 8; u += 2) {
                    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u + 1], bv[u + 1], acc1, 0, 0, 0);
                }
            }
        }
        for (int blk = 0; blk < n16; ++blk, p0 += 16) {
            const float4 a4 = g16[blk * nat * 64];
            float bv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) bv[u] = cok ? Ub[(p0 + 4 * u + lk) * ld + c].y : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, bv[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, bv[1], acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, bv[2], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, bv[3], acc1, 0, 0, 0);
        }
        for (; p0 < rows; p0 += 4) {
            const int pp = p0 + lk;
            const bool ok = pp < rows;
            const int pc = ok ? pp : 0;
            const float a = ok ? gcol[pc * oMp] : 0.f;
            const float bv = (ok && cok) ? Ub[pc * ld + c].y : 0.f;
            acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int a_ = at * 16 + lk * 4 + i;
            if (a_ < oM && cok) S[b * s_bs + (a_ * oN + c) * s_es] = acc0[i] + acc1[i];
        }
    }
    __syncthreads();
}

// Register-cached MFMA low-pass of square K x K arrays (K compile-time): the tap operands of a
// whole tile (every K step: KS floats per lane) are loaded once per wave and call -- step 1 fixes a
// wave's column tile (nt = wave % nnt) for all of its (b, row-tile) tasks, step 2's operands are
// issued at entry, behind step 1 -- instead of once per 8 K steps of every task (the L2 latency of
// the tap loads, not the matrix pipe, bounded the phase).  Same operand order, K parts and results
// as lds_lowpass_mfma.  Needs nw >= nnt (step 1; checked at plan creation).  Ends with a barrier.
constexpr int mfma_k_steps(int k) {
    return 16 * (k / 64) + 4 * ((k % 64) / 16) + ((k % 16) + 3) / 4;
}
template <int K>
__device__ __forceinline__ void lds_lowpass_mfma_rc(float2* U, int nb, int bs, int ld,
                                                    const float* __restrict__ GM,
                                                    const float* __restrict__ GN, int oMp, int oNp,
                                                    int oM, int oN, float* S, int s_bs = -1, int s_es = 1) {
    constexpr int N64 = K / 64, N16 = (K % 64) / 16, NTL = ((K % 16) + 3) / 4;
    constexpr int KS = mfma_k_steps(K), NMT = (K + 15) / 16, Q16 = 64 * N64, QT = 64 * N64 + 16 * N16;
    if (s_bs < 0) s_bs = oM * oN;
    const int lane = threadIdx.x & 63, wave = wave_id(), nw = blockDim.x >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const int nnt = oNp >> 4, nat = oMp >> 4;
    // lane's operand of every K step of tile t of a tap matrix with ntile column tiles
    auto load_ops = [&](const float* G, int ntile, int t, float (&g)[KS]) __attribute__((always_inline)) {
        const float4* g64 = reinterpret_cast<const float4*>(G) + (t * 64 + lane) * 4;
        wstfft::static_for<0, N64>([&](auto bc) {
            constexpr int blk = decltype(bc)::value;
            wstfft::static_for<0, 4>([&](auto jc) {
                constexpr int j = decltype(jc)::value;
                const float4 v = g64[blk * ntile * 256 + j];
                g[16 * blk + 4 * j] = v.x;
                g[16 * blk + 4 * j + 1] = v.y;
                g[16 * blk + 4 * j + 2] = v.z;
                g[16 * blk + 4 * j + 3] = v.w;
            });
        });
        const float4* g16 = reinterpret_cast<const float4*>(G) + N64 * ntile * 256 + t * 64 + lane;
        wstfft::static_for<0, N16>([&](auto bc) {
            constexpr int blk = decltype(bc)::value;
            const float4 v = g16[blk * ntile * 64];
            g[16 * N64 + 4 * blk] = v.x;
            g[16 * N64 + 4 * blk + 1] = v.y;
            g[16 * N64 + 4 * blk + 2] = v.z;
            g[16 * N64 + 4 * blk + 3] = v.w;
        });
        const float* gcol = G + (N64 * 4 + N16) * ntile * 256 - QT * (ntile * 16) + t * 16 + li;
        wstfft::static_for<0, NTL>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const int q = QT + 4 * s + lk;
            g[16 * N64 + 4 * N16 + s] = q < K ? gcol[q * (ntile * 16)] : 0.f;
        });
    };
    // row / column index of K step s for this lane
    auto kidx = [&](auto sc) __attribute__((always_inline)) {
        constexpr int s = decltype(sc)::value;
        if constexpr (s < 16 * N64) return 64 * (s / 16) + (s % 16) + 16 * lk;
        else if constexpr (s < 16 * N64 + 4 * N16) return Q16 + 16 * ((s - 16 * N64) / 4) + 4 * ((s - 16 * N64) % 4) + lk;
        else return QT + 4 * (s - 16 * N64 - 4 * N16) + lk;
    };
    float g2[KS];
    const int t2_0 = wave;   // first step-2 task of this wave
    int at2 = -1;
    if (t2_0 < nb * nat * nnt) {
        at2 = (t2_0 % (nat * nnt)) / nnt;
        load_ops(GM, nat, at2, g2);
    }
    // 1. T = U GN: every wave keeps one column tile (waves w and w + nnt share it, splitting its
    //    row tiles).  Needs nw >= nnt: the plan checks it for every launch that takes this form
    //    (wst_hip.hip, rc_waves_ok).  (A
    //    nested loop serving nw < nnt here cost the f3 k_o2 1.8 %, measured round 5.)  Should a
    //    launch break it anyway, the stride stays >= 1 (wrong maps, never a hang); waves beyond the
    //    last whole group of nnt would only repeat other waves' tiles and skip step 1.
    const int tstep = nw >= nnt ? nw / nnt : 1;
    if (wave < nnt * tstep || nw < nnt) {
        float g[KS];
        const int nt = wave % nnt;
        load_ops(GN, nnt, nt, g);
        for (int tk = wave / nnt; tk < nb * NMT; tk += tstep) {
            const int b = tk / NMT, mt = tk - b * NMT;
            float2* Ub = U + b * bs;
            const int p = mt * 16 + li;
            const bool pok = p < K;
            const float2* urow = Ub + (pok ? p : K - 1) * ld;
            f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
            wstfft::static_for<0, KS>([&](auto sc) {
                constexpr int s = decltype(sc)::value;
                const int q = kidx(sc);
                float a = lds_half64(urow + (s >= 16 * N64 + 4 * N16 ? (q < K ? q : 0) : q), 0);
                if constexpr (s >= 16 * N64 + 4 * N16) a = q < K ? a : 0.f;
                a = pok ? a : 0.f;
                if constexpr (s % 2 == 0) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, g[s], acc0, 0, 0, 0);
                else acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, g[s], acc1, 0, 0, 0);
            });
            const int c = nt * 16 + li;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pp = mt * 16 + lk * 4 + i;
                if (pp < K && c < oN) Ub[pp * ld + c].y = acc0[i] + acc1[i];
            }
        }
    }
    __syncthreads();
    // 2. S = GM^T T
    for (int t = wave; t < nb * nat * nnt; t += nw) {
        const int b = t / (nat * nnt);
        const int r = t - b * nat * nnt;
        const int at = r / nnt, ct = r - at * nnt;
        if (at != at2) {
            at2 = at;
            load_ops(GM, nat, at, g2);
        }
        const float2* Ub = U + b * bs;
        const int c = ct * 16 + li;
        const bool cok = c < oN;
        f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        wstfft::static_for<0, KS>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const int p = kidx(sc);
            const int pc = (s >= 16 * N64 + 4 * N16 && p >= K) ? 0 : p;
            float bv = lds_half64(Ub + pc * ld + (cok ? c : 0), 1);
            if constexpr (s >= 16 * N64 + 4 * N16) bv = p < K ? bv : 0.f;
            bv = cok ? bv : 0.f;
            if constexpr (s % 2 == 0) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(g2[s], bv, acc0, 0, 0, 0);
            else acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(g2[s], bv, acc1, 0, 0, 0);
        });
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int a_ = at * 16 + lk * 4 + i;
            if (a_ < oM && cok) S[b * s_bs + (a_ * oN + c) * s_es] = acc0[i] + acc1[i];
        }
    }
    __syncthreads();
}

// register-cached form for compile-time square sizes with at most 18 K steps (72^2, 68^2, 36^2 ...)
template <int K>
constexpr bool mfma_rc_ok() { return K > 0 && mfma_k_steps(K) <= 18; }

__device__ __forceinline__ bool wide_lowpass(const DevParams& p) { return p.oM > kLpOM || p.oN > kLpOM; }
__device__ __forceinline__ const float* lpw_M(const DevParams& p, int slot) { return p.lpw + p.lpw_off[2 * slot]; }
__device__ __forceinline__ const float* lpw_N(const DevParams& p, int slot) { return p.lpw + p.lpw_off[2 * slot + 1]; }

// Separable phi low-pass of one (rows x cols) real array (U[p][q].x, row stride ld) at the kept
// output points through the level's tap matrices (physical order, unpad and decimation folded in;
// host: lpt):  S[a][c] = sum_p GM[p][a] sum_q GN[q][c] U[p][q], oM, oN <= oms (4 or 8).  The
// row partials T[p][c] are parked in the free .y slots of row p.  One float4 load brings four
// taps (lds_lowpass: a table load and a permutation lookup per tap).  Ends with a barrier.
template <int QC, int PC>
__device__ __forceinline__ void lds_lowpass_taps(float2* U, int rows, int cols, int ld,
                                                 const float* GM, const float* GN, int oms, int oM,
                                                 int oN, float* S) {
    const int T = blockDim.x;
    const bool w8 = oms > 4;
    // 1. T[p][c] = sum_q GN[q][c] U[p][q]: QC lanes per row
    for (int w = threadIdx.x; w < rows * QC; w += T) {
        const int qc = w & (QC - 1);
        const int p = w / QC;
        float2* row = U + p * ld;
        float acc[kLpOM];
#pragma unroll
        for (int c = 0; c < kLpOM; ++c) acc[c] = 0.f;
        for (int q = qc; q < cols; q += QC) {
            const float x = row[q].x;
            const float4 g0 = *reinterpret_cast<const float4*>(GN + q * oms);
            acc[0] = fmaf(g0.x, x, acc[0]);
            acc[1] = fmaf(g0.y, x, acc[1]);
            acc[2] = fmaf(g0.z, x, acc[2]);
            acc[3] = fmaf(g0.w, x, acc[3]);
            if (w8) {
                const float4 g1 = *reinterpret_cast<const float4*>(GN + q * oms + 4);
                acc[4] = fmaf(g1.x, x, acc[4]);
                acc[5] = fmaf(g1.y, x, acc[5]);
                acc[6] = fmaf(g1.z, x, acc[6]);
                acc[7] = fmaf(g1.w, x, acc[7]);
            }
        }
#pragma unroll
        for (int c = 0; c < kLpOM; ++c) {
            if (c >= 4 && !w8) break;
            acc[c] = group_sum<QC>(acc[c]);
        }
        if (qc == 0) {
#pragma unroll
            for (int c = 0; c < kLpOM; ++c)
                if (c < oN) row[c].y = acc[c];
        }
    }
    __syncthreads();
    // 2. S[a][c] = sum_p GM[p][a] T[p][c]: PC lanes per output column c
    for (int w = threadIdx.x; w < oN * PC; w += T) {
        const int pc = w & (PC - 1);
        const int c = w / PC;
        float acc[kLpOM];
#pragma unroll
        for (int a = 0; a < kLpOM; ++a) acc[a] = 0.f;
        for (int p = pc; p < rows; p += PC) {
            const float t = U[p * ld + c].y;
            const float4 g0 = *reinterpret_cast<const float4*>(GM + p * oms);
            acc[0] = fmaf(g0.x, t, acc[0]);
            acc[1] = fmaf(g0.y, t, acc[1]);
            acc[2] = fmaf(g0.z, t, acc[2]);
            acc[3] = fmaf(g0.w, t, acc[3]);
            if (w8) {
                const float4 g1 = *reinterpret_cast<const float4*>(GM + p * oms + 4);
                acc[4] = fmaf(g1.x, t, acc[4]);
                acc[5] = fmaf(g1.y, t, acc[5]);
                acc[6] = fmaf(g1.z, t, acc[6]);
                acc[7] = fmaf(g1.w, t, acc[7]);
            }
        }
#pragma unroll
        for (int a = 0; a < kLpOM; ++a) {
            if (a >= 4 && !w8) break;
            acc[a] = group_sum<PC>(acc[a]);
        }
        if (pc == 0) {
#pragma unroll
            for (int a = 0; a < kLpOM; ++a)
                if (a < oM) S[a * oN + c] = acc[a];
        }
    }
    __syncthreads();
}

// Inverse column pass (in place, natural -> digit-reversed rows) of nb (NN x cols) arrays U_b,
// fused with |.| * scale and the phi low-pass (unpad and decimation folded
// into the tap matrices GM (physical row p -> kept output row a) and GN (column q -> output c)):
//   1. after the last butterfly the unit holding physical rows [RU k, RU k + RU) of column q
//      stores V_k[a] = sum_p GM[p][a] |z_p| scale (a < oM; GM rows oms = 4 or 8 floats) in its own
//      first slots: row RU k + a/2,
//      component a & 1 (the modulus itself is never stored);
//   2. W[a][q] = sum_k V_k[a][q], written over V_0;
//   3. S[b][a][c] = sum_q GN[q][c] W[a][q]  (QC lanes per output, shuffle-reduced).
// Requires oM <= min(kLpOM, 2 RU) (host: fused_lowpass_ok).  Ends with a barrier.
// RS > 0: the rows were transformed with the split N = (NN / RS) x RS (fused_row_n2), so physical
// column q holds another logical column than GN's rows (split_n2 order) assume: the S pass walks
// GN's order and reads each column's partial from its position in the rows' order.
// Address-space-typed pointers (global / LDS) for stores the compiler must not merge into flat ones
typedef __attribute__((address_space(1))) float* gfloat_p;
typedef __attribute__((address_space(3))) float* lfloat_p;
typedef const __attribute__((address_space(1))) float* gcfloat_p;
typedef const __attribute__((address_space(3))) float* lcfloat_p;

template <int NN, int RS = 0>
__device__ __forceinline__ void cols_modlp(float2* U, int nb, int bs, int cols, int ld,
                                           const float2* tw, const float* GM, const float* GN,
                                           int oms, int oM, int oN, float scale, float* S,
                                           float* outd) {
    using F = wstfft::LineFFT<NN, true, fused_col_n2(NN)>;
    using FS = wstfft::LineFFT<NN, true>;    // the split GM's rows are ordered for
    constexpr bool single = (F::N2 == 1);
    constexpr int RU = single ? NN : F::N2;  // rows per unit
    constexpr int NU = single ? 1 : F::N1;   // units per column
    // remap: physical row RU k + e holds logical row k + NU e, whose taps sit in GM row
    // FS::N2 (k + NU t) + m (e = RR m + t, RR = FS::N1 / NU): a per-unit base plus a per-e constant
    constexpr bool remap = !single && F::N2 != FS::N2;
    static_assert(!remap || (FS::N2 > 1 && FS::N1 % F::N1 == 0), "column split must refine split_n2's N1");
    constexpr int RR = remap ? FS::N1 / F::N1 : 1;
    constexpr int GU = remap ? FS::N2 : RU;  // GM rows per unit step k
    // grouped: the NU units of a column sit in NU adjacent lanes and their partials are summed
    // there (DPP), so the S pass reads one partial per column instead of NU
    constexpr bool grouped = !single && (NU & (NU - 1)) == 0 && NU <= 16;
    constexpr int NUS = grouped ? 1 : NU;    // partials per column left for the S pass
    const wstfft::Lines g(nb, bs, cols, 1, ld);
    const int T = blockDim.x;
    const int nlines = nb * cols;
    if constexpr (!single) {
        for (int u = threadIdx.x; u < nlines * F::N2; u += T) F::stageA_unit(U, g, tw, u);
        __syncthreads();
    }
    for (int u = threadIdx.x; u < nlines * NU; u += T) {
        int k = 0;
        int line;
        if constexpr (single) line = u;
        else if constexpr (grouped) { line = u / NU; k = u & (NU - 1); }
        else line = g.split(u, k);
        float2* p = U + g.offset(line) + (RU * k) * ld;
        float2 v[RU];
        wstfft::static_for<0, RU>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = p[e * ld];
        });
        wstfft::rfft<RU, true>(v);
        const float* gm = GM + (GU * k) * oms;
        if constexpr (single) {
            // whole column in one unit: the tap loads of a rolled loop over output-row pairs keep
            // the register footprint to the RU moduli (unrolled, the RU x oms GM loads hoist)
            float m[RU];
            wstfft::static_for<0, RU>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                m[e] = __builtin_amdgcn_sqrtf(fmaf(v[e].x, v[e].x, v[e].y * v[e].y)) * scale;
            });
#pragma unroll 1
            for (int t = 0; 2 * t < oM; ++t) {
                float V0 = 0.f, V1 = 0.f;
                wstfft::static_for<0, RU>([&](auto ec) {
                    constexpr int e = decltype(ec)::value;
                    const float2 g = *reinterpret_cast<const float2*>(gm + e * oms + 2 * t);
                    V0 = fmaf(g.x, m[e], V0);
                    V1 = fmaf(g.y, m[e], V1);
                });
                p[t * ld] = make_float2(V0, V1);
            }
            continue;
        }
        float V[kLpOM];
#pragma unroll
        for (int a = 0; a < kLpOM; ++a) V[a] = 0.f;
        wstfft::static_for<0, RU>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            const float m = __builtin_amdgcn_sqrtf(fmaf(v[e].x, v[e].x, v[e].y * v[e].y)) * scale;
            constexpr int ge = remap ? FS::N2 * NU * (e % RR) + e / RR : e;
            const float4 g0 = *reinterpret_cast<const float4*>(gm + ge * oms);
            V[0] = fmaf(g0.x, m, V[0]);
            V[1] = fmaf(g0.y, m, V[1]);
            V[2] = fmaf(g0.z, m, V[2]);
            V[3] = fmaf(g0.w, m, V[3]);
            if (oM > 4) {
                const float4 g1 = *reinterpret_cast<const float4*>(gm + ge * oms + 4);
                V[4] = fmaf(g1.x, m, V[4]);
                V[5] = fmaf(g1.y, m, V[5]);
                V[6] = fmaf(g1.z, m, V[6]);
                V[7] = fmaf(g1.w, m, V[7]);
            }
        });
        if constexpr (grouped) {
#pragma unroll
            for (int a = 0; a < kLpOM; ++a)
                if (a < oM) V[a] = group_sum<NU>(V[a]);
            if (k != 0) continue;
        }
#pragma unroll
        for (int t = 0; t < kLpOM / 2; ++t)
            if (2 * t < oM) p[t * ld] = make_float2(V[2 * t], V[2 * t + 1]);
    }
    __syncthreads();
    // 2+3. S = (sum_k V_k) GN in one pass: QC lanes split the columns q of output (b, a, c), each
    //      sums the NU unit partials of its columns, shuffle reduction.  outd (nullable): write
    //      S straight to the coefficient maps instead of S (non-pooled output).
    constexpr int QC = NN >= 48 ? 16 : NN >= 24 ? 8 : NN >= 12 ? 4 : 2;   // ~3 columns per lane
    const int nout = nb * oM * oN;
    const wstfft::FastDiv dc(oN), dab(oM * oN);
    for (int w = threadIdx.x; w < nout * QC; w += T) {
        const int qc = w & (QC - 1);
        const int o = w / QC;
        const int b = dab.div(o);
        const int ac = o - b * oM * oN;
        const int a = dc.div(ac);
        const int c = ac - a * oN;
        const float* f = reinterpret_cast<const float*>(U + b * bs + (a >> 1) * ld) + (a & 1);
        auto column = [&](int q, float acc) __attribute__((always_inline)) {
            int qr = q;   // position of GN row q's logical column in the rows' order
            if constexpr (RS > 0) {
                constexpr int N2d = wstfft::split_n2(NN), N1d = NN / N2d, N1r = NN / RS;
                const int lg = q / N2d + N1d * (q % N2d);
                qr = RS * (lg % N1r) + lg / N1r;
            }
            float wq = 0.f;
            wstfft::static_for<0, NUS>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                wq += f[2 * (qr + RU * k * ld)];
            });
            return fmaf(GN[q * oms + c], wq, acc);
        };
        // the NN / QC columns of a lane unrolled (their LDS reads issue together: a rolled loop
        // waited out the LDS latency once per column); same order of accumulation
        constexpr int CQ = (NN + QC - 1) / QC;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < CQ; ++i)
            if (qc + i * QC < cols) acc = column(qc + i * QC, acc);
        for (int q = qc + CQ * QC; q < cols; q += QC) acc = column(q, acc);
        acc = group_sum<QC>(acc);
        if (qc == 0) {
            // typed global / LDS pointers: as one generic pointer the compiler merges the two stores
            // into a flat store, which the next LDS wait (and barrier) must see complete in HBM
            if (outd) __builtin_nontemporal_store(acc, (gfloat_p)outd + o);
            else ((lfloat_p)S)[o] = acc;
        }
    }
    __syncthreads();
}

template <int FAM, int K, int HI, int RS = 0>
__device__ __forceinline__ void family_cols_modlp(float2* U, int nb, int bs, int rows, int cols,
                                                  int ld, const float2* tw, const float* GM,
                                                  const float* GN, int oms, int oM, int oN,
                                                  float scale, float* S, float* outd) {
    constexpr int NN = FAM << K;
    if constexpr (FAM > 0 && NN <= HI && NN <= wstfft::kMaxFamilyN) {
        // RS > 0 belongs to the fused 48-point rows only: no other size is compiled for it
        if constexpr (NN >= 2 && (RS == 0 || fused_row_n2(NN) == RS)) {
            if (rows == NN) {
                cols_modlp<NN, RS>(U, nb, bs, cols, ld, tw, GM, GN, oms, oM, oN, scale, S, outd);
                return;
            }
        }
        family_cols_modlp<FAM, K + 1, HI, RS>(U, nb, bs, rows, cols, ld, tw, GM, GN, oms, oM, oN, scale, S, outd);
    }
}

// Write nb coefficient maps (S: nb x oM x oN) of plane `img`, coefficient k0 + b.
// pooled: out[img][k] = mean, out[img][K + k] = population std -- one thread per map for small
// maps, else one wave per map with lanes strided over its values and shuffle sums (a map of the
// reference's 128^2 J=2 geometry holds 1024 values: 11.4 -> 3.2 ms per 256 RGB patches).
// Called by every thread of the block (whole waves).
// S addressing as lds_lowpass_mfma (s_bs < 0: contiguous maps).
__device__ __forceinline__ void emit(const float* S, int nb, int k0, long long img, int K, int oM,
                                     int oN, float* out, int pooled, int s_bs = -1, int s_es = 1) {
    const int npix = oM * oN;
    if (s_bs < 0) s_bs = npix;
    if (!pooled) {
        const int tot = nb * npix;
        const wstfft::FastDiv dpix(npix);
        for (int o = threadIdx.x; o < tot; o += blockDim.x) {
            const int b = dpix.div(o);
            const int i = o - b * npix;
            out[(img * K + k0 + b) * npix + i] = S[b * s_bs + i * s_es];
        }
    } else if (npix <= 32) {   // small maps (the headline's 4 x 4): one thread per map
        for (int b = threadIdx.x; b < nb; b += blockDim.x) {
            const float* v = S + b * s_bs;
            float m = 0.f;
            for (int i = 0; i < npix; ++i) m += v[i * s_es];
            m /= npix;
            float q = 0.f;
            for (int i = 0; i < npix; ++i) {
                const float d = v[i * s_es] - m;
                q = fmaf(d, d, q);
            }
            out[img * 2 * K + k0 + b] = m;
            out[img * 2 * K + K + k0 + b] = sqrtf(q / npix);
        }
    } else {
        const int lane = threadIdx.x & 63, nw = (blockDim.x + 63) >> 6;
        for (int b = threadIdx.x >> 6; b < nb; b += nw) {
            const float* v = S + b * s_bs;
            float m = 0.f;
            for (int i = lane; i < npix; i += 64) m += v[i * s_es];
            m = group_sum<64>(m) / npix;
            float q = 0.f;
            for (int i = lane; i < npix; i += 64) {
                const float d = v[i * s_es] - m;
                q = fmaf(d, d, q);
            }
            q = group_sum<64>(q);
            if (lane == 0) {
                out[img * 2 * K + k0 + b] = m;
                out[img * 2 * K + K + k0 + b] = sqrtf(q / npix);
            }
        }
    }
}

// Table slices of the plan pools copied into LDS; accessors rebase global offsets.
struct Tables {
    float2* tw;
    float* lp;
    int* pm;
    float* lt;
    int tw0, lp0, pm0, lt0, ntw, twn0, ntwn, nlt, ltn0, nltn;
    const DevParams* p;
    __device__ __forceinline__ const float2* twM(int r) const { return tw + (p->tw_off[2 * r] - tw0); }
    __device__ __forceinline__ const float2* twN(int r) const {
        return ntwn ? tw + ntw + (p->tw_off[2 * r + 1] - twn0) : twM(r);
    }
    __device__ __forceinline__ const float* lpM(int r) const { return lp + (p->lp_off[2 * r] - lp0); }
    __device__ __forceinline__ const float* lpN(int r) const { return lp + (p->lp_off[2 * r + 1] - lp0); }
    __device__ __forceinline__ const int* pmM(int r) const { return pm + (p->perm_off[2 * r] - pm0); }
    __device__ __forceinline__ const int* pmN(int r) const { return pm + (p->perm_off[2 * r + 1] - pm0); }
    __device__ __forceinline__ const float* gM(int r) const { return lt + (p->lpt_off[2 * r] - lt0); }
    __device__ __forceinline__ const float* gN(int r) const {
        return nltn ? lt + nlt + (p->lpt_off[2 * r + 1] - ltn0) : gM(r);
    }
};

__device__ __forceinline__ Tables load_tables(const DevParams& p, const LdsLayout& lay,
                                              unsigned char* smem) {
    Tables t;
    t.tw = reinterpret_cast<float2*>(smem + lay.off_tw);
    t.lp = reinterpret_cast<float*>(smem + lay.off_lp);
    t.pm = reinterpret_cast<int*>(smem + lay.off_pm);
    t.lt = reinterpret_cast<float*>(smem + lay.off_lt);
    t.tw0 = lay.tw0;
    t.lp0 = lay.lp0;
    t.pm0 = lay.pm0;
    t.lt0 = lay.lt0;
    t.ntw = lay.ntw;
    t.twn0 = lay.twn0;
    t.ntwn = lay.ntwn;
    t.nlt = lay.nlt;
    t.ltn0 = lay.ltn0;
    t.nltn = lay.nltn;
    t.p = &p;
    for (int i = threadIdx.x; i < lay.ntw; i += blockDim.x) t.tw[i] = p.tw[lay.tw0 + i];
    for (int i = threadIdx.x; i < lay.ntwn; i += blockDim.x) t.tw[lay.ntw + i] = p.tw[lay.twn0 + i];
    for (int i = threadIdx.x; i < lay.nlp; i += blockDim.x) t.lp[i] = p.lp[lay.lp0 + i];
    for (int i = threadIdx.x; i < lay.npm; i += blockDim.x) t.pm[i] = p.perm[lay.pm0 + i];
    for (int i = threadIdx.x; i < lay.nlt; i += blockDim.x) t.lt[i] = p.lpt[lay.lt0 + i];
    for (int i = threadIdx.x; i < lay.nltn; i += blockDim.x) t.lt[lay.nlt + i] = p.lpt[lay.ltn0 + i];
    return t;
}

__host__ __device__ inline int odd_ld(int n) { return n | 1; }
// Half spectra of one (plane, theta1) in the workspace: nM1 rows of hld columns, plus row nM1 =
// row 0 when hext (resident levels), padded to a whole 16 bytes so every item's rows start
// 16-byte aligned (k_o2 copies them with 16-byte loads; an odd float2 count left every other item
// on the 8-byte path)
__host__ __device__ inline long long hspec_stride(int nM1, int hld, int hext) {
    const long long n = static_cast<long long>(nM1 + hext) * hld;
    return hext ? (n + 1) & ~1LL : n;
}

// Streaming (non-temporal) 8-byte load / store: the half-spectrum hand-off k_o1 -> k_o2 is
// written and read once (~0.9 GB per 2048-plane chunk at the 96^2 level), kept from displacing
// the filters the folds re-read from L2 (c2: -2.5 %, measured).
__device__ __forceinline__ float2 ldnt(const float2* p) {
    return __builtin_bit_cast(float2,
                              __builtin_nontemporal_load(reinterpret_cast<const unsigned long long*>(p)));
}
__device__ __forceinline__ void stnt(float2* p, float2 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
}

// dst[i] = src[i] for i < n (global -> LDS): eight loads per thread in flight before the stores
// (a plain loop waits out the HBM latency once per element).
__device__ __forceinline__ void copy_to_lds(float2* dst, const float2* __restrict__ src, int n) {
    constexpr int K = 8;
    const int T = blockDim.x;
    if ((n & 1) == 0 && ((reinterpret_cast<unsigned long long>(src) | reinterpret_cast<unsigned long long>(dst)) & 15) == 0) {
        // 16-byte non-temporal loads (8-byte ones stream at 0.54-0.70x the rate, MI355X_MICROARCH.md)
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v* s4 = reinterpret_cast<const f4v*>(src);
        f4v* d4 = reinterpret_cast<f4v*>(dst);
        const int n4 = n >> 1;
        for (int i0 = threadIdx.x; i0 < n4; i0 += K * T) {
            f4v t[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                t[k] = __builtin_nontemporal_load(s4 + min(i0 + k * T, n4 - 1));
            }
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (i0 + k * T < n4) d4[i0 + k * T] = t[k];
        }
        return;
    }
    for (int i0 = threadIdx.x; i0 < n; i0 += K * T) {
        float2 t[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float2* q = src + min(i0 + k * T, n - 1);
            t[k] = ldnt(q);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (i0 + k * T < n) dst[i0 + k * T] = t[k];
    }
}

// Order-1 fold from HBM/L2: A[u][v] = sum_{i,j < s} X[u + i nM1][v + j nN1] * psi0[...]
// S > 0: compile-time alias count; S == 0: runtime s.  U items per thread keep loads in flight.
template <int S>
__device__ __forceinline__ void fold1(const float2* __restrict__ X, const float* __restrict__ psi0,
                                      int PN, float2* A, int ld1, int nM1, int nN1, int s_rt) {
    if constexpr (S == 1) {
        if ((nN1 & 1) == 0) {
            // s = 1: element pairs (v, v + 1) per lane, Xhat as 16-byte loads (offsets even), the
            // filter as 8-byte ones; U pairs per thread in flight (f3 k_o1 j1 = 0 0.790 -> 0.736 ms,
            // c1 0.632 -> 0.596; profiles/r06_ab.txt r06y)
            constexpr int U = 4;
            const int T = blockDim.x;
            const int nh = nN1 >> 1, items = nM1 * nh;
            const wstfft::FastDiv dn(nh);
            for (int it0 = threadIdx.x; it0 < items; it0 += U * T) {
                float4 xv[U];
                float2 f[U];
                int dst[U];
#pragma unroll
                for (int k = 0; k < U; ++k) {
                    const int it = it0 + k * T;
                    const int ic = min(it, items - 1);
                    const int u = dn.div(ic), v = 2 * (ic - u * nh);
                    const int idx = u * PN + v;
                    xv[k] = *reinterpret_cast<const float4*>(X + idx);
                    f[k] = *reinterpret_cast<const float2*>(psi0 + idx);
                    dst[k] = it < items ? u * ld1 + v : -1;
                }
#pragma unroll
                for (int k = 0; k < U; ++k)
                    if (dst[k] >= 0) {
                        A[dst[k]] = make_float2(xv[k].x * f[k].x, xv[k].y * f[k].x);
                        A[dst[k] + 1] = make_float2(xv[k].z * f[k].y, xv[k].w * f[k].y);
                    }
            }
            return;
        }
    }
    const int s = (S > 0) ? S : s_rt;
    const int items = nM1 * nN1;
    const int T = blockDim.x;
    const wstfft::FastDiv dn(nN1);
    constexpr int U = (S == 1) ? 4 : (S == 2 ? 2 : 1);
    constexpr int UI = S > 0 ? S : 1, UJ = S > 0 ? S : 4;
    for (int it0 = threadIdx.x; it0 < items; it0 += U * T) {
        float2 acc[U];
        int dst[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int it = it0 + k * T;
            acc[k] = make_float2(0.f, 0.f);
            dst[k] = -1;
            if (it < items) {
                const int u = dn.div(it), v = it - u * nN1;
                dst[k] = u * ld1 + v;
#pragma unroll UI
                for (int i = 0; i < s; ++i) {
#pragma unroll UJ
                    for (int j = 0; j < s; ++j) {
                        const int idx = (u + i * nM1) * PN + v + j * nN1;
                        const float f = psi0[idx];
                        const float2 xv = X[idx];
                        acc[k] = make_float2(fmaf(xv.x, f, acc[k].x), fmaf(xv.y, f, acc[k].y));
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (dst[k] >= 0) A[dst[k]] = acc[k];
    }
}

// s = 1 order-1 "fold" (Xhat * psi0, level 0) fused with stage A of the inverse row transform
// (F_DR, two-stage N = NA * NB): unit (u, n2) multiplies the elements v = n2 + NB e of row u
// straight from HBM / L2 into registers, runs the DFT-NA and the twiddles and stores the stage-A
// result (the product is never written to LDS and read back).  Stage B follows after a barrier.
template <int N>
__device__ __forceinline__ void fold1_rowA(const float2* __restrict__ X, const float* __restrict__ psi0,
                                           float2* __restrict__ A, const float2* __restrict__ tw) {
    using F = wstfft::LineFFT<N, true>;
    static_assert(F::N2 > 1, "two-stage row sizes only");
    constexpr int NA = F::N1, NB = F::N2, LD = N | 1;
    int w0 = threadIdx.x;
    asm volatile("" : "+v"(w0));   // no hoisting of the unit's bases / twiddles (see fold2_s2_rowA)
    for (int w = w0; w < N * NB; w += blockDim.x) {
        const int u = w / NB, n2 = w - u * NB;
        const float2* xr = X + u * N + n2;
        const float* pr = psi0 + u * N + n2;
        float2 x[NA];
        wstfft::static_for<0, NA>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            const float2 xv = xr[NB * e];
            const float f = pr[NB * e];
            x[e] = make_float2(xv.x * f, xv.y * f);
        });
        wstfft::rfft<NA, true>(x);
        wstfft::static_for<1, NA>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            x[k] = wstfft::cmul_tw(x[k], tw[n2 * k], true);
        });
        float2* d = A + u * LD + n2;
        wstfft::static_for<0, NA>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            d[NB * e] = x[e];
        });
    }
}

// Box-sparse order-1 fold (s >= 4): aliases i in [i0, i0 + ni) of row u and j in [j0, j0 + nj) of
// column v only (see fold2 / box tables); predicated blocks of 4 keep the loads in flight.
__device__ __forceinline__ void fold1_box(const float2* __restrict__ X, const float* __restrict__ psi0,
                                          int PN, float2* A, int ld1, int nM1, int nN1, int s,
                                          const int* __restrict__ box) {
    const int items = nM1 * nN1;
    const int smask = s - 1;
    const wstfft::FastDiv dn(nN1);
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
        const int u = dn.div(it), v = it - u * nN1;
        const int rb = box[u], cb = box[nM1 + v];
        const int i0 = rb & 255, ni = rb >> 8, j0 = cb & 255, nj = cb >> 8;
        float2 acc = make_float2(0.f, 0.f);
        for (int ib = 0; ib < ni; ib += 4) {
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2) {
                if (ib + i2 >= ni) continue;
                const int rowoff = (u + ((i0 + ib + i2) & smask) * nM1) * PN + v;
                for (int jb = 0; jb < nj; jb += 4) {
#pragma unroll
                    for (int j2 = 0; j2 < 4; ++j2) {
                        if (jb + j2 >= nj) continue;
                        const int idx = rowoff + ((j0 + jb + j2) & smask) * nN1;
                        const float f = psi0[idx];
                        const float2 xv = X[idx];
                        acc = make_float2(fmaf(xv.x, f, acc.x), fmaf(xv.y, f, acc.y));
                    }
                }
            }
        }
        A[u * ld1 + v] = acc;
    }
}

__device__ __forceinline__ void fold1_any(int s1, const float2* X, const float* psi0, int PN,
                                          float2* A, int ld1, int nM1, int nN1, const int* box) {
    if (s1 == 1) fold1<1>(X, psi0, PN, A, ld1, nM1, nN1, 1);
    else if (s1 == 2) fold1<2>(X, psi0, PN, A, ld1, nM1, nN1, 2);
    else if (box) fold1_box(X, psi0, PN, A, ld1, nM1, nN1, s1, box);
    else if (s1 == 4) fold1<4>(X, psi0, PN, A, ld1, nM1, nN1, 4);
    else fold1<0>(X, psi0, PN, A, ld1, nM1, nN1, s1);
}

// 8-byte load through a buffer descriptor: 32-bit lane offset + wave-uniform offset, no 64-bit
// address arithmetic per load.
// Buffer descriptor over [base, base + bytes) from wave-uniform inputs, made provably uniform
// (readfirstlane) so the compiler emits no waterfall loop around the loads.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* base, int bytes) {
    const unsigned long long a = reinterpret_cast<unsigned long long>(base);
    const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(a));
    const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(a >> 32));
    void* b = reinterpret_cast<void*>((static_cast<unsigned long long>(hi) << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(b, static_cast<short>(0),
                                             __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

__device__ __forceinline__ float2 buf_load2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ float4 buf_load4(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Order-2 Hermitian fold of npair filter pairs (2 paths each) into B:
//   B_b[u][v] = sum_{i,j < s} U1hat[u + i nM2][v + j nN2] * psi_b[...]
// U1hat is read from the half spectrum H (nM1 x hld, columns 0..nN1/2):
//   U1hat[kr][kc] = kc <= nN1/2 ? H[kr][kc] : conj(H[(nM1 - kr) % nM1][nN1 - kc]).
// Box-sparse: only the aliases i in [i0, i0 + ni) (mod s) of row u and j in [j0, j0 + nj) of
// column v are summed, where the pair's alias boxes (host: box_bins) cover every bin at which
// either filter exceeds kBoxThreshold * its maximum; the dropped terms are below that bound.
// Column taps go in blocks of four, set up once per block (H column, mirror, sign; taps past the
// box are skipped), then the block walks the box rows: per tap one read of H, one buffer load
// (32-bit offsets) and the products.
template <int S>
__device__ __forceinline__ void fold2(const float2* __restrict__ H, int hld, int nM1, int nN1,
                                      const float2* __restrict__ psi2, long long pstride,
                                      int npair, int npath, float2* __restrict__ B, int pslot,
                                      int ld2, int nM2, int nN2, int s_rt,
                                      const int* __restrict__ box, int bstride) {
    const int s = (S > 0) ? S : s_rt;
    const int smask = s - 1;
    const int half = nN1 >> 1;
    const int items = nM2 * nN2;
    const int total = npair * items;
    const wstfft::FastDiv ditems(items), dn(nN2);
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psi2, static_cast<int>(npair * pstride * 8));
    // the next bin's box header is loaded while this bin's taps are summed (c5 k_o2 j1 = 0
    // 9.84 -> 9.54 ms; profiles/r06_ab.txt r06z)
    int rbn = 0, cbn = 0;
    if (threadIdx.x < total) {
        const int pr = ditems.div(threadIdx.x);
        const int it = threadIdx.x - pr * items;
        const int u = dn.div(it), v = it - u * nN2;
        rbn = box[pr * bstride + u];
        cbn = box[pr * bstride + nM2 + v];
    }
    for (int w = threadIdx.x; w < total; w += blockDim.x) {
        const int pr = ditems.div(w);
        const int it = w - pr * items;
        const int u = dn.div(it), v = it - u * nN2;
        const int rb = rbn, cb = cbn;
        const int wn = w + blockDim.x;
        if (wn < total) {
            const int prn = ditems.div(wn);
            const int itn = wn - prn * items;
            const int un = dn.div(itn), vn = itn - un * nN2;
            rbn = box[prn * bstride + un];
            cbn = box[prn * bstride + nM2 + vn];
        }
        const int i0 = rb & 255, ni = rb >> 8, j0 = cb & 255, nj = cb >> 8;
        const int fpr = static_cast<int>(pr * pstride);
        float2 a0 = make_float2(0.f, 0.f), a1 = make_float2(0.f, 0.f);
        for (int jb = 0; jb < nj; jb += 4) {
            int hc[4], fc[4];
            bool mir[4], ok[4];
            float wy[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                ok[c] = jb + c < nj;
                const int kc = v + ((j0 + jb + c) & smask) * nN2;
                mir[c] = kc > half;
                hc[c] = mir[c] ? nN1 - kc : kc;
                fc[c] = kc * 8;
                wy[c] = mir[c] ? -1.f : 1.f;
            }
            for (int i = 0; i < ni; ++i) {
                const int kr = u + ((i0 + i) & smask) * nM2;
                const int krm = kr == 0 ? 0 : nM1 - kr;
                const float2* hd = H + kr * hld;
                const float2* hm = H + krm * hld;
                const int fo = (fpr + kr * nN1) * 8;
                float2 hv[4], fv[4];
                // taps past the box are not loaded (boxes are 1-3 aliases wide at c5's s >= 4
                // levels: the padded block of 4 had loaded half its taps for nothing)
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    hv[c] = make_float2(0.f, 0.f);
                    fv[c] = make_float2(0.f, 0.f);
                    if (ok[c]) {
                        hv[c] = (mir[c] ? hm : hd)[hc[c]];
                        fv[c] = buf_load2(rs, fo + fc[c], 0);
                    }
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float hx = hv[c].x, hy = hv[c].y * wy[c];
                    a0 = make_float2(fmaf(hx, fv[c].x, a0.x), fmaf(hy, fv[c].x, a0.y));
                    a1 = make_float2(fmaf(hx, fv[c].y, a1.x), fmaf(hy, fv[c].y, a1.y));
                }
            }
        }
        float2* dst = B + 2 * pr * pslot + u * ld2 + v;
        dst[0] = a0;
        if (2 * pr + 1 < npath) dst[pslot] = a1;
    }
}

// s = 2 fold (j2 = j1 + 1, ~93 % of the alias box is significant, so dense): with nN2 = nN1 / 2
// the four taps of (u, v) are rows u, u + nM2 and columns v (direct) and v + nN2 (the Hermitian
// mirror conj(H[krm][nN2 - v]) for v > 0, H[kr][nN2] for v = 0); krm(u) = (nM1 - u) % nM1 and
// krm(u + nM2) = nM2 - u.
// Each lane keeps one column v (its mirror column and sign are fixed) and walks the rows
// (pair, u) of the batch in steps of rpp = T / nN2 (lanes beyond rpp * nN2 idle); the filter
// taps come through a buffer descriptor with the row offsets as wave-uniform soffsets.
// R rows of a lane in flight per iteration (R = 3 when H is read from HBM / L2: HG kernels).
// X: the filters from the pairs' alias-interleaved copy (square planes; host: wst_hip.hip psi2),
// the four aliases of a bin as two 16-byte loads.
template <int R = 1, bool X = false>
__device__ __forceinline__ void fold2_s2(const float2* __restrict__ H, int hld, int nM1, int nN1,
                                         const float2* __restrict__ psi2, long long pstride,
                                         int npair, int npath, float2* __restrict__ B, int pslot,
                                         int ld2, int nM2, int nN2) {
    const int rpp = blockDim.x / nN2;
    const int t0 = threadIdx.x / nN2;
    if (t0 >= rpp) return;
    const int v = threadIdx.x - t0 * nN2;
    const bool v0 = v == 0;
    const int cB = v0 ? nN2 : nN2 - v;  // column of the two mirrored taps
    const float sg = v0 ? 1.f : -1.f;   // their conjugation
    const int hq = nM2 * hld;           // H offset of row u + nM2
    const int fq = nM2 * nN1 * 8;       // filter byte offset of row u + nM2
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psi2, static_cast<int>(npair * pstride * 8));
    const wstfft::FastDiv dm(nM2);
    const int rows = npair * nM2;
    for (int pu0 = t0; pu0 < rows; pu0 += R * rpp) {
        float2 h[R][4], f[R][4];
        int pr[R], dst[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int pu = min(pu0 + r * rpp, rows - 1);
            pr[r] = dm.div(pu);
            const int u = pu - pr[r] * nM2;
            dst[r] = pu0 + r * rpp < rows ? 2 * pr[r] * pslot + u * ld2 + v : -1;
            const int hr = u * hld;
            const int hm0 = v0 ? hr : (u == 0 ? 0 : (nM1 - u) * hld);
            const int hm1 = v0 ? hr + hq : (nM2 - u) * hld;
            h[r][0] = H[hr + v];
            h[r][1] = H[hm0 + cB];
            h[r][2] = H[hr + hq + v];
            h[r][3] = H[hm1 + cB];
            if constexpr (X) {
                // psi2 points at the copy: aliases (u, v), (u + nM2, v), (u, v + nN2), (u + nM2, v + nN2)
                const int xo = (static_cast<int>(pr[r] * pstride) + (u * nN2 + v) * 4) * 8;
                const float4 A = buf_load4(rs, xo, 0), Bq = buf_load4(rs, xo, 16);
                f[r][0] = make_float2(A.x, A.y);
                f[r][2] = make_float2(A.z, A.w);
                f[r][1] = make_float2(Bq.x, Bq.y);
                f[r][3] = make_float2(Bq.z, Bq.w);
            } else {
                const int fo = (static_cast<int>(pr[r] * pstride) + u * nN1 + v) * 8;
                f[r][0] = buf_load2(rs, fo, 0);
                f[r][1] = buf_load2(rs, fo, nN2 * 8);
                f[r][2] = buf_load2(rs, fo, fq);
                f[r][3] = buf_load2(rs, fo, fq + nN2 * 8);
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            h[r][1].y *= sg;
            h[r][3].y *= sg;
            float2 a0, a1;
            a0.x = fmaf(h[r][0].x, f[r][0].x, fmaf(h[r][1].x, f[r][1].x, fmaf(h[r][2].x, f[r][2].x, h[r][3].x * f[r][3].x)));
            a0.y = fmaf(h[r][0].y, f[r][0].x, fmaf(h[r][1].y, f[r][1].x, fmaf(h[r][2].y, f[r][2].x, h[r][3].y * f[r][3].x)));
            a1.x = fmaf(h[r][0].x, f[r][0].y, fmaf(h[r][1].x, f[r][1].y, fmaf(h[r][2].x, f[r][2].y, h[r][3].x * f[r][3].y)));
            a1.y = fmaf(h[r][0].y, f[r][0].y, fmaf(h[r][1].y, f[r][1].y, fmaf(h[r][2].y, f[r][2].y, h[r][3].y * f[r][3].y)));
            if (dst[r] >= 0) {
                float2* d = B + dst[r];
                d[0] = a0;
                if (2 * pr[r] + 1 < npath) d[pslot] = a1;
            }
        }
    }
}

// Two adjacent columns (v, v + 1) per lane (even nN2): the filter taps of both as one 16-byte
// buffer load (offsets (pr pstride + u nN1 + v) even), the spectrum taps 8-byte (the mirror runs
// backwards over odd-length rows); rows walked in steps of T / (nN2 / 2).
template <int R = 1>
__device__ __forceinline__ void fold2_s2_pairs(const float2* __restrict__ H, int hld, int nM1, int nN1,
                                               const float2* __restrict__ psi2, long long pstride,
                                               int npair, int npath, float2* __restrict__ B, int pslot,
                                               int ld2, int nM2, int nN2) {
    const int nh = nN2 >> 1;
    const int rpp = blockDim.x / nh;
    const int t0 = threadIdx.x / nh;
    if (t0 >= rpp) return;
    const int v = 2 * (threadIdx.x - t0 * nh);
    const int hq = nM2 * hld;
    const int fq = nM2 * nN1 * 8;
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psi2, static_cast<int>(npair * pstride * 8));
    const wstfft::FastDiv dm(nM2);
    const int rows = npair * nM2;
    for (int pu0 = t0; pu0 < rows; pu0 += R * rpp) {
        float2 h[R][2][4];
        float4 f[R][4];
        int pr[R], dst[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int pu = min(pu0 + r * rpp, rows - 1);
            pr[r] = dm.div(pu);
            const int u = pu - pr[r] * nM2;
            dst[r] = pu0 + r * rpp < rows ? 2 * pr[r] * pslot + u * ld2 + v : -1;
            const int hr = u * hld;
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int c = v + e;
                const bool c0 = c == 0;
                const int cB = c0 ? nN2 : nN2 - c;
                const int hm0 = c0 ? hr : (u == 0 ? 0 : (nM1 - u) * hld);
                const int hm1 = c0 ? hr + hq : (nM2 - u) * hld;
                h[r][e][0] = H[hr + c];
                h[r][e][1] = H[hm0 + cB];
                h[r][e][2] = H[hr + hq + c];
                h[r][e][3] = H[hm1 + cB];
                const float sg = c0 ? 1.f : -1.f;
                h[r][e][1].y *= sg;
                h[r][e][3].y *= sg;
            }
            const int fo = (static_cast<int>(pr[r] * pstride) + u * nN1 + v) * 8;
            f[r][0] = buf_load4(rs, fo, 0);
            f[r][1] = buf_load4(rs, fo, nN2 * 8);
            f[r][2] = buf_load4(rs, fo, fq);
            f[r][3] = buf_load4(rs, fo, fq + nN2 * 8);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                float fa[4], fb[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    fa[t] = e ? f[r][t].z : f[r][t].x;
                    fb[t] = e ? f[r][t].w : f[r][t].y;
                }
                const float2* hh = h[r][e];
                float2 a0, a1;
                a0.x = fmaf(hh[0].x, fa[0], fmaf(hh[1].x, fa[1], fmaf(hh[2].x, fa[2], hh[3].x * fa[3])));
                a0.y = fmaf(hh[0].y, fa[0], fmaf(hh[1].y, fa[1], fmaf(hh[2].y, fa[2], hh[3].y * fa[3])));
                a1.x = fmaf(hh[0].x, fb[0], fmaf(hh[1].x, fb[1], fmaf(hh[2].x, fb[2], hh[3].x * fb[3])));
                a1.y = fmaf(hh[0].y, fb[0], fmaf(hh[1].y, fb[1], fmaf(hh[2].y, fb[2], hh[3].y * fb[3])));
                if (dst[r] >= 0) {
                    float2* d = B + dst[r] + e;
                    d[0] = a0;
                    if (2 * pr[r] + 1 < npath) d[pslot] = a1;
                }
            }
        }
    }
}

template <int R = 1>
__device__ __forceinline__ void fold2_any(int s2, const float2* H, int hld, int nM1, int nN1,
                                          const float2* psi2, long long pstride, int npair,
                                          int npath, float2* B, int pslot, int ld2, int nM2,
                                          int nN2, const int* box, int bstride,
                                          const float2* psx = nullptr) {
    if (s2 == 2) {
        // column pairs where they keep > 6 % more lanes busy (f3's 68-column paths on 512 lanes:
        // 476 -> 510, k_o2 1.216 -> 1.166 ms; c1's 36 columns on 256 lanes gain no lanes and
        // measured 1.3 % slower, c5's 96 on 1024 +5 % lanes, neutral; profiles/r06_ab.txt r06w),
        // one row pair per lane in flight (two: 0.6 % slower, three: 4 %; r06x); the dense form
        // with the interleaved filters takes R = 3 rows per lane in flight for HG (c1 k_o2 1.18 ->
        // 1.135 ms, c5 HG j1 = 1 2.17 -> 2.08 ms against R = 2; r06g8)
        const int T = blockDim.x;
        if (R >= 2 && (nN2 & 1) == 0 && (T / (nN2 >> 1)) * (nN2 >> 1) * 100 > (T / nN2) * nN2 * 106)
            fold2_s2_pairs<1>(H, hld, nM1, nN1, psi2, pstride, npair, npath, B, pslot, ld2, nM2, nN2);
        else if (psx)   // c1 k_o2 1.192 -> 1.153 ms, c5 HG j1 = 1 2.19 -> 2.12 ms (r06_ab.txt r06g4)
            fold2_s2<R, true>(H, hld, nM1, nN1, psx, pstride, npair, npath, B, pslot, ld2, nM2, nN2);
        else
            fold2_s2<R>(H, hld, nM1, nN1, psi2, pstride, npair, npath, B, pslot, ld2, nM2, nN2);
    }
    else fold2<0>(H, hld, nM1, nN1, psi2, pstride, npair, npath, B, pslot, ld2, nM2, nN2, s2, box, bstride);
}

// ---- tile-mapped folds of a square level with compile-time sizes (SQ geometry kernels) ----
// The npair x N2^2 (pair, bin) outputs of a batch go to whole waves in tiles of 64 consecutive
// bins of one pair (wave-uniform tile loop), so every alias of a tile is one uniform offset from
// two per-lane bases: the direct tap (a, b) of bin (u, v) (b < s/2: column v + N2 b < N1/2) reads
// H[u + N2 a][v + N2 b] = dbase + (N2 a HLD + N2 b), the mirrored one (b >= s/2) reads
// conj(H[(N1 - u - N2 a) % N1][N1 - v - N2 b]) = mbase + (N2 (s-1-a) HLD + N2 (s-1-b)) with
// mbase = (N2 - u) HLD + (N2 - v) (H carries row N1 = row 0 for u = a = 0), and the filter pair
// sits at fbase + (N2 a N1 + N2 b) with fbase = u N1 + v.  The tap offsets are compile-time
// immediates (s = 2, dense) or come from host-built per-tile tap lists (s = 4, 8: only the
// aliases where some bin of the tile meets a significant bin of either filter).
__device__ __forceinline__ float2 lds_at(const char* base, int byte_off) {
    return *reinterpret_cast<const float2*>(base + byte_off);
}
// read-only table in the constant address space: loads at wave-uniform addresses become s_load
typedef const __attribute__((address_space(4))) int* cint_p;
template <typename T>
__device__ __forceinline__ cint_p to_const_as(const T* p) {
    return (cint_p)(reinterpret_cast<unsigned long long>(p));
}

template <int N1>
__device__ __forceinline__ void fold2_tile_s2(const float2* __restrict__ H, const float2* __restrict__ psi2,
                                              int npair, int npath, float2* __restrict__ B,
                                              const float2* __restrict__ psx) {
    constexpr int N2 = N1 / 2, HLD = N1 / 2 + 1, LD2 = N2 | 1, PSLOT = N2 * LD2;
    constexpr int ITEMS = N2 * N2, NT = (ITEMS + 63) / 64, PST = N1 * N1;
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    (void)psi2;   // the filters from the alias-interleaved copy (c2 k_o2 j1 = 1 0.475 -> 0.454 ms; r06g5)
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psx, npair * PST * 8);
    const char* Hb = reinterpret_cast<const char*>(H);
    const int w0 = wave_id();
    for (int k = 0;; ++k) {
        // wave-uniform tile index (readfirstlane: scalar loop control, pair and header offsets)
        const int wi = __builtin_amdgcn_readfirstlane(w0 + k * nw);
        if (wi >= npair * NT) break;
        const int pr = wi / NT;
        const int bin0 = (wi - pr * NT) * 64 + lane;
        const int bin = min(bin0, ITEMS - 1);
        const int u = bin / N2, v = bin - u * N2;
        const int db = (u * HLD + v) * 8, mb = ((N2 - u) * HLD + (N2 - v)) * 8;
        const int po = pr * PST * 8;
        const float2 h0 = lds_at(Hb, db), h1 = lds_at(Hb, db + N2 * HLD * 8);   // (0,0) (1,0)
        const float2 m0 = lds_at(Hb, mb + N2 * HLD * 8), m1 = lds_at(Hb, mb);   // (0,1) (1,1)
        const int xo = (u * N2 + v) * 32;
        const float4 A = buf_load4(rs, xo, po), Bq = buf_load4(rs, xo, po + 16);
        const float2 f0 = make_float2(A.x, A.y), f1 = make_float2(A.z, A.w);
        const float2 g0 = make_float2(Bq.x, Bq.y), g1 = make_float2(Bq.z, Bq.w);
        float2 a0, a1;
        a0.x = fmaf(h0.x, f0.x, fmaf(h1.x, f1.x, fmaf(m0.x, g0.x, m1.x * g1.x)));
        a0.y = fmaf(h0.y, f0.x, fmaf(h1.y, f1.x, fmaf(-m0.y, g0.x, -m1.y * g1.x)));
        a1.x = fmaf(h0.x, f0.y, fmaf(h1.x, f1.y, fmaf(m0.x, g0.y, m1.x * g1.y)));
        a1.y = fmaf(h0.y, f0.y, fmaf(h1.y, f1.y, fmaf(-m0.y, g0.y, -m1.y * g1.y)));
        if (bin0 < ITEMS) {
            float2* d = B + 2 * pr * PSLOT + u * LD2 + v;
            d[0] = a0;
            if (2 * pr + 1 < npath) d[PSLOT] = a1;
        }
    }
}

// s = 2 fold fused with stage A of the inverse row transform (F_DR order, two-stage sizes
// N2 = NA * NB): unit (pair, u, n2) folds the bins v = n2 + NB e (e < NA) of row u for both paths
// of the pair straight into registers, runs the DFT-NA and the twiddles W^(n2 k) and stores the
// stage-A result in place of the batch rows (B is never written by a separate fold pass and read
// back).  Offsets relative to the unit's bases are compile-time immediates: direct
// db + (NB e) (+ N2 HLD for a = 1), mirrored mb + NB (NA-1-e) (+ N2 HLD for a = 0) with mb at the
// unit's largest column, filters xo + 32 NB e (the four aliases as two 16-byte loads of the
// alias-interleaved copy).  Stage B follows after a
// barrier (fft_lines_dr_stageB).
// The filters come from the pairs' alias-interleaved copy psx (host: wst_hip.hip psi2): two
// 16-byte loads per bin instead of four 8-byte ones (c2 k_o2 j1 = 0 -1 %; r06_ab.txt r06g3).
template <int N1>
__device__ __forceinline__ void fold2_s2_rowA(const float2* __restrict__ H, const float2* __restrict__ psi2,
                                              int npair, int npath, float2* __restrict__ B,
                                              const float2* __restrict__ tw,
                                              const float2* __restrict__ psx) {
    constexpr int N2 = N1 / 2, HLD = N1 / 2 + 1, LD2 = N2 | 1, PSLOT = N2 * LD2, PST = N1 * N1;
    using F = wstfft::LineFFT<N2, true, fused_row_n2(N2)>;
    static_assert(F::N2 > 1, "two-stage row sizes only");
    constexpr int NA = F::N1, NB = F::N2, UNITS = N2 * NB;
    (void)psi2;
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psx, npair * PST * 8);
    const char* Hb = reinterpret_cast<const char*>(H);
    // opaque start index: keeps the compiler from hoisting the unit's bases and twiddles out of
    // the caller's batch loop (live across the whole level, they pushed k_o2 into spills)
    int w0 = threadIdx.x;
    asm volatile("" : "+v"(w0));
    for (int w = w0; w < npair * UNITS; w += blockDim.x) {
        const int pr = w / UNITS;
        const int r = w - pr * UNITS;
        const int g = r / NB, n2 = r - g * NB;
        // row of lane group g (NB lanes of one row): with NB = 8 a half-wave holds 4 groups; taking
        // rows h, h + 8, h + 16, h + 24 for them puts their stride-HLD / stride-LD2 LDS rows (odd,
        // = 17 mod 32 float2) on disjoint banks (the first 32 rows; the rest keep their order)
        int u = g;
        if constexpr (NB == 8 && N2 >= 32 && (UNITS % 32) == 0)
            if (g < 32) u = 8 * (g & 3) + (g >> 2);
        const int db = (u * HLD + n2) * 8;
        const int mb = ((N2 - u) * HLD + (NB - n2)) * 8;
        const int xo = ((u * N2 + n2) * 4 + pr * PST) * 8;   // lanes of a wave may straddle pairs
        float2 x0[NA], x1[NA];
        wstfft::static_for<0, NA>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            constexpr int dv = NB * e, dm = NB * (NA - 1 - e);
            const float2 h0 = lds_at(Hb, db + dv * 8), h1 = lds_at(Hb, db + (N2 * HLD + dv) * 8);
            const float2 m0 = lds_at(Hb, mb + (N2 * HLD + dm) * 8), m1 = lds_at(Hb, mb + dm * 8);
            const float4 A = buf_load4(rs, xo, dv * 32), Bq = buf_load4(rs, xo, dv * 32 + 16);
            const float2 f0 = make_float2(A.x, A.y), f1 = make_float2(A.z, A.w);
            const float2 g0 = make_float2(Bq.x, Bq.y), g1 = make_float2(Bq.z, Bq.w);
            x0[e].x = fmaf(h0.x, f0.x, fmaf(h1.x, f1.x, fmaf(m0.x, g0.x, m1.x * g1.x)));
            x0[e].y = fmaf(h0.y, f0.x, fmaf(h1.y, f1.x, fmaf(-m0.y, g0.x, -m1.y * g1.x)));
            x1[e].x = fmaf(h0.x, f0.y, fmaf(h1.x, f1.y, fmaf(m0.x, g0.y, m1.x * g1.y)));
            x1[e].y = fmaf(h0.y, f0.y, fmaf(h1.y, f1.y, fmaf(-m0.y, g0.y, -m1.y * g1.y)));
            // pin both paths' sums here: sunk to their DFTs, the other path's filter values stayed
            // live (spilled) across the first path's transform
            asm volatile("" : "+v"(x0[e].x), "+v"(x0[e].y), "+v"(x1[e].x), "+v"(x1[e].y));
            // at most kFuseGroup elements' loads in flight (register budget of 4 waves per SIMD)
            if constexpr ((e + 1) % kFuseGroup == 0) __builtin_amdgcn_sched_barrier(0);
        });
        wstfft::rfft<NA, true>(x0);
        wstfft::rfft<NA, true>(x1);
        wstfft::static_for<1, NA>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const float2 t = tw[n2 * k];
            x0[k] = wstfft::cmul_tw(x0[k], t, true);
            x1[k] = wstfft::cmul_tw(x1[k], t, true);
        });
        float2* d = B + 2 * pr * PSLOT + u * LD2 + n2;
        wstfft::static_for<0, NA>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            d[NB * e] = x0[e];
        });
        if (2 * pr + 1 < npath)
            wstfft::static_for<0, NA>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                d[PSLOT + NB * e] = x1[e];
            });
    }
}

// s = 4 / 8: per (pair, tile) header {first tap, direct groups, mirrored groups} and tap lists
// padded to groups of four with dummy taps (LDS offset 0, filter offset into the zero block past
// the filters), so four taps are in flight per group with no per-tap test.
template <int N1, int S>
__device__ __forceinline__ void fold2_tile_list(const float2* __restrict__ H, const float2* __restrict__ psi2,
                                                int npair, int npath, float2* __restrict__ B,
                                                const int4* __restrict__ hdr, const int2* __restrict__ taps) {
    constexpr int N2 = N1 / S, HLD = N1 / 2 + 1, LD2 = N2 | 1, PSLOT = N2 * LD2;
    constexpr int ITEMS = N2 * N2, NT = (ITEMS + 63) / 64, PST = N1 * N1;
    const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psi2, 0x7ffffff0);
    const char* Hb = reinterpret_cast<const char*>(H);
    const int w0 = wave_id();
    for (int k = 0;; ++k) {
        // wave-uniform tile index (readfirstlane: scalar loop control, pair and header offsets)
        const int wi = __builtin_amdgcn_readfirstlane(w0 + k * nw);
        if (wi >= npair * NT) break;
        const int pr = wi / NT;
        const int bin0 = (wi - pr * NT) * 64 + lane;
        const int bin = min(bin0, ITEMS - 1);
        const int u = bin / N2, v = bin - u * N2;
        const int db = (u * HLD + v) * 8, mb = ((N2 - u) * HLD + (N2 - v)) * 8;
        const int fo = (u * N1 + v) * 8, po = pr * PST * 8;
        // header and tap lists through the constant address space: scalar loads into SGPRs
        const cint_p hp = to_const_as(hdr) + 4 * wi;
        const int ng_dir = hp[1], ng_mir = hp[2];
        cint_p tl = to_const_as(taps) + 2 * hp[0];
        float2 a0 = make_float2(0.f, 0.f), a1 = make_float2(0.f, 0.f);
        for (int g = 0; g < ng_dir; ++g, tl += 8) {
            float2 hv[4], fv[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                hv[c] = lds_at(Hb, db + tl[2 * c]);
                fv[c] = buf_load2(rs, fo, tl[2 * c + 1] + po);
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                a0 = make_float2(fmaf(hv[c].x, fv[c].x, a0.x), fmaf(hv[c].y, fv[c].x, a0.y));
                a1 = make_float2(fmaf(hv[c].x, fv[c].y, a1.x), fmaf(hv[c].y, fv[c].y, a1.y));
            }
        }
        for (int g = 0; g < ng_mir; ++g, tl += 8) {
            float2 hv[4], fv[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                hv[c] = lds_at(Hb, mb + tl[2 * c]);
                fv[c] = buf_load2(rs, fo, tl[2 * c + 1] + po);
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                a0 = make_float2(fmaf(hv[c].x, fv[c].x, a0.x), fmaf(-hv[c].y, fv[c].x, a0.y));
                a1 = make_float2(fmaf(hv[c].x, fv[c].y, a1.x), fmaf(-hv[c].y, fv[c].y, a1.y));
            }
        }
        if (bin0 < ITEMS) {
            float2* d = B + 2 * pr * PSLOT + u * LD2 + v;
            d[0] = a0;
            if (2 * pr + 1 < npath) d[PSLOT] = a1;
        }
    }
}

// XCD-aware decode of (plane, theta1) items: blocks b and b+8 share an XCD; give each XCD a
// contiguous range so the L workgroups of a plane read its Xhat from one L2.
__device__ __forceinline__ int xcd_item(int total) {
    int item = blockIdx.x;
    if ((total & 7) == 0) item = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    return item;
}

// ------------------------------------------------------------------------------------------
// k_prep: one workgroup per plane
// ------------------------------------------------------------------------------------------
constexpr int prev_cap(int c) { return c <= 12 ? 0 : c <= 24 ? 12 : c <= 48 ? 24 : 48; }
// The level size of an SQ launch when its size class holds exactly one size of the family
// (family 3: 96 / 48 / 24, family 5: 80 / 40 / 20, family 9: 72 / 36 / 18), else 0 (runtime).
// With it every level size of the kernel is a compile-time constant: loop bounds, strides and
// index decodes fold, the FFT-size dispatch disappears (geometry-specialised kernels).
constexpr int unique_level(int fam, int cap) {
    if (fam <= 0) return 0;
    int found = 0, count = 0;
    for (int n = fam; n <= cap; n *= 2)
        if (n > prev_cap(cap)) {
            found = n;
            ++count;
        }
    return count == 1 ? found : 0;
}

template <int FM, int FN, int PC>
__device__ __forceinline__ void prep_body(unsigned char* smem, const DevParams& p, const LdsLayout& lay,
                                          const float* __restrict__ in, long long img0,
                                          float2* __restrict__ xhat, float* __restrict__ out,
                                          int pooled) {
    const int PM = PC ? PC : p.PM, PN = PC ? PC : p.PN, n = PM * PN, ld = odd_ld(PN);
    float2* A = reinterpret_cast<float2*>(smem);
    float* S = reinterpret_cast<float*>(smem + lay.off_s);
    float* red = reinterpret_cast<float*>(smem + lay.off_red);
    const Tables tb = load_tables(p, lay, smem);

    const long long local = blockIdx.x;
    const long long img = img0 + local;
    const int inM = p.pre_pad ? PM : p.M, inN = p.pre_pad ? PN : p.N;
    const float* x = in + local * inM * inN;
    float part = 0.f;
    {
        // kPrepBatch gather loads per thread in flight before their LDS stores (a load-store loop
        // waited out the HBM latency once per element: c2 k_prep 0.173 -> 0.158 ms per step)
        constexpr int KB = kPrepBatch;
        const int T = blockDim.x;
        const wstfft::FastDiv dpn(PN);
        for (int i0 = threadIdx.x; i0 < n; i0 += KB * T) {
            float xv[KB];
            int dst[KB];
#pragma unroll
            for (int k = 0; k < KB; ++k) {
                const int i = i0 + k * T;
                const int ii = min(i, n - 1);
                const int u = PC ? ii / PC : dpn.div(ii), v = ii - u * PN;
                const int su = p.pre_pad ? u : reflect_index(u - p.padTop, p.M);
                const int sv = p.pre_pad ? v : reflect_index(v - p.padLeft, p.N);
                xv[k] = x[su * inN + sv];
                dst[k] = i < n ? u * ld + v : -1;
            }
#pragma unroll
            for (int k = 0; k < KB; ++k)
                if (dst[k] >= 0) {
                    A[dst[k]] = make_float2(xv[k], 0.f);
                    part += xv[k];
                }
        }
    }
    const float mean = block_sum(part, red) / n;  // contains the barrier after the gather

    // S0: low-pass at level 0, decimation 2^J
    if (wide_lowpass(p))   // natural-order level-0 tap matrices (slot J)
    {
        if constexpr (mfma_rc_ok<PC>())
            lds_lowpass_mfma_rc<PC>(A, 1, 0, ld, lpw_M(p, p.J), lpw_N(p, p.J), p.oMp, p.oNp, p.oM, p.oN, S);
        else
            lds_lowpass_mfma(A, 1, 0, PM, PN, ld, lpw_M(p, p.J), lpw_N(p, p.J), p.oMp, p.oNp, p.oM, p.oN, S);
    }
    else
        lds_lowpass(A, 1, 0, PM, PN, ld, tb.lpM(0), tb.lpN(0), nullptr, nullptr, 1 << p.J, p.oM, p.oN, S);
    emit(S, 1, 0, img, p.K, p.oM, p.oN, out, pooled);

    // mean-centred forward DFT for the band-pass paths (.y reset: the low-pass parked sums there)
    for (GridIter it(PN); it.u < PM; it.next()) {
        float2& a = A[it.u * ld + it.v];
        a = make_float2(a.x - mean, 0.f);
    }
    __syncthreads();
    wstfft::EpiIdentity id;
    lds_fft2<FM, FN, 0, wstfft::kMaxFamilyN, kNat, false>(A, 1, 0, PM, PN, ld, tb.twM(0), tb.twN(0), id);
    float2* dst = xhat + local * n;
    for (GridIter it(PN); it.u < PM; it.next()) dst[it.u * PN + it.v] = A[it.u * ld + it.v];
#ifdef WST_TRACE
    if (tracing(p, get_tslot(lay))) {   // (after the work: the body is laid out as without it)
        trace_word(p, get_tslot(lay), 0, tr_kernel(kTkPrep, FM, FN, 0, 0, 0));
        trace_word(p, get_tslot(lay), 1, tr_prep(PC, wide_lowpass(p) ? (mfma_rc_ok<PC>() ? kLpMfmaRc : kLpMfma) : kLpPlain));
    }
#endif
}

// One workgroup per plane.  Square planes of the family's sizes in (48, 136] run with compile-time
// sizes.
template <int FM, int FN>
__global__ void __launch_bounds__(1024) k_prep(DevParams p, LdsLayout lay,
                                               const float* __restrict__ in, long long img0,
                                               float2* __restrict__ xhat, float* __restrict__ out,
                                               int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if constexpr (FM == FN && FM > 0) {
        // square planes of the family's sizes in (48, 136]: compile-time size
        bool done = false;
        wstfft::static_for<0, 8>([&](auto mc) {
            constexpr int PC = FM << decltype(mc)::value;
            if constexpr (PC > 48 && PC <= 136) {
                if (!done && p.PM == PC && p.PN == PC) {
                    done = true;
                    prep_body<FM, FN, PC>(smem, p, lay, in, img0, xhat, out, pooled);
                }
            }
        });
        if (done) return;
    }
    prep_body<FM, FN, 0>(smem, p, lay, in, img0, xhat, out, pooled);
}

// Size classes of the k_o1 / k_o2 instantiations: CAP = largest level size of a launch
// (max(PM, PN) >> j1).  SQ = 1: square plane whose order-2 low-pass fuses (fused_lowpass_ok), so
// every level-j1 size is in (prev_cap(CAP), CAP] and the order-2 paths are <= CAP / 2: the
// kernel carries only those FFTs (code size stays well inside the instruction cache).
// Minimum waves per SIMD for k_o1 per size class: the 96^2-class level runs 768-thread
// workgroups, two per CU (LDS-bound), so it needs <= 80 VGPRs (6 waves per SIMD).
// (families 3, 5, 9 square: the others' FFT sizes spill at that budget and keep 512 threads;
// host side: o1_wide in wst_hip.hip)
constexpr int o1_min_waves(int cap, int fm, int fn) {
    return (cap == 136 && fm == fn && (fm == 3 || fm == 5 || fm == 9)) ? 6 : 1;
}

// ------------------------------------------------------------------------------------------
// k_o1: one workgroup per (plane, theta1) at fixed j1 -- order 1 + half-spectrum export
// ------------------------------------------------------------------------------------------
// k_o1 body; OC > 0: the output maps are OC x OC (compile-time; the common 4 x 4 of the headline);
// N1T > 0: the (square) level size at compile time
template <int FM, int FN, int MAXN, int SQ, int OC, int N1T = 0>
__device__ __forceinline__ void k_o1_body(unsigned char* smem, const DevParams& p,
                                          const LdsLayout& lay, int j1, int nimg, long long img0,
                                          const float2* __restrict__ xhat, float2* __restrict__ hexp,
                                          float* __restrict__ out, int pooled) {
    const int oM = OC ? OC : p.oM, oN = OC ? OC : p.oN;
    const int oms = OC ? 4 : lay.oms;
    const int J = p.J, L = p.L;
    const int item = xcd_item(nimg * L);
    const int local = item / L;
    const int l1 = item - local * L;
    const long long img = img0 + local;
    const int PM = p.PM, PN = p.PN;
    constexpr int N1C = N1T ? N1T : SQ ? unique_level(FM, MAXN) : 0;
    const int nM1 = N1C ? N1C : PM >> j1, nN1 = N1C ? N1C : PN >> j1;
    const int n1 = nM1 * nN1, ld1 = odd_ld(nN1);
    const bool do2 = (p.max_order >= 2) && (j1 < J - 1);
    float2* A = reinterpret_cast<float2*>(smem);
    float* S = reinterpret_cast<float*>(smem + lay.off_s);
    float* red = reinterpret_cast<float*>(smem + lay.off_red);
    const Tables tb = load_tables(p, lay, smem);
    const int dbg = WST_DBG_MASK(p);

    // 1. fold_{2^j1}(Xhat * psi0_{j1,l1}) straight from HBM/L2
    const float* psi0 = p.psi + p.psi_off[(j1 * L + l1) * J + 0];
    const float2* X = xhat + static_cast<long long>(local) * PM * PN;
    const int b1 = p.box1_off[j1 * L + l1];
    const bool use_box1 = b1 >= 0 && (1 << j1) >= p.box1_min_s;
    // square level-0 plane of a compile-time two-stage size: the product fused with the rows'
    // stage A (fold1_rowA)
    // (SQ geometry kernels: c2 k_o1 j1 = 0 0.778 -> 0.726 ms; the non-SQ 136^2 level of f3 measured
    // 0.78 -> 0.79, so the exported-spectrum kernels keep the separate fold)
    constexpr bool FUSE1 = SQ && N1C >= kFuse1Min && wstfft::LineFFT<(N1C > 0 ? N1C : 2), true>::N2 > 1;
    const bool fused1 = FUSE1 && j1 == 0;
    EpiModulus mod1{1.f / (static_cast<float>(PM) * static_cast<float>(PN)), 0.f};
    if (fused1) {
        if constexpr (FUSE1) {
            fold1_rowA<N1C>(X, psi0, A, tb.twN(j1));
            __syncthreads();
            wstfft::EpiIdentity id1;
            wstfft::fft_lines_dr_stageB<N1C, true>(A, wstfft::Lines{1, 0, nM1, ld1, 1}, id1);
            lds_fft_lines<FM, SQ ? prev_cap(MAXN) : 0, MAXN, kDR, true>(A, wstfft::Lines{1, 0, nN1, 1, ld1}, nM1,
                                                                       tb.twM(j1), mod1);
        }
    } else {
        if (!(dbg & 128)) fold1_any(1 << j1, X, psi0, PN, A, ld1, nM1, nN1, use_box1 ? p.box + b1 : nullptr);
        __syncthreads();

        // 2. U1 = |ifft(.)|, modulus fused into the last pass; fold-mean + ifft scale = 1/(PM PN).
        //    In place (digit-reversed rows and columns); the low-pass maps the permutation.
        if (!(dbg & 1))
            lds_fft2<FM, FN, SQ ? prev_cap(MAXN) : 0, MAXN, kDR, true>(A, 1, 0, nM1, nN1, ld1, tb.twM(j1),
                                                                      tb.twN(j1), mod1);
    }
    const float mean1 = block_sum(mod1.sum, red) / n1;

    // 3. S1 at level j1, decimation 2^(J-j1)
    const int n1idx = j1 * L + l1;
    if (!(dbg & 2)) {
        if constexpr (SQ)
            lds_lowpass_taps<8, 16>(A, nM1, nN1, ld1, tb.gM(j1), tb.gN(j1), oms, oM, oN, S);
        else if (wide_lowpass(p))
        {
            if constexpr (mfma_rc_ok<N1C>())
                lds_lowpass_mfma_rc<N1C>(A, 1, 0, ld1, lpw_M(p, j1), lpw_N(p, j1), p.oMp, p.oNp, oM, oN, S);
            else
                lds_lowpass_mfma(A, 1, 0, nM1, nN1, ld1, lpw_M(p, j1), lpw_N(p, j1), p.oMp, p.oNp, oM,
                                 oN, S);
        }
        else
            lds_lowpass(A, 1, 0, nM1, nN1, ld1, tb.lpM(j1), tb.lpN(j1), tb.pmM(j1), tb.pmN(j1),
                        1 << (J - j1), oM, oN, S);
        emit(S, 1, 1 + n1idx, img, p.K, oM, oN, out, pooled);
    }
    if (!do2) return;

    // 4. real-input row FFT of (U1 - mean): physical rows r, r + nh packed as re/im of row r
    //    (packing inside the transform's first stage measured neutral: c2 k_o1 0.728 -> 0.727 ms).
    //    Rows r and r + nh rather than 2r and 2r + 1: the packed lines keep the odd row stride, so
    //    the transform's lane groups do not meet 2-way bank conflicts (stride 2 ld1: 4 banks apart)
    const int nh = nM1 >> 1;
    constexpr int PK = WST_O1_PACK_HALF;   // 1: rows (r, r + nh); 0: rows (2r, 2r + 1) (A/B builds)
    const int prow = PK ? 1 : 2;           // packed line r sits at row prow * r
    const int pmate = PK ? nh : 1;         // its imaginary part's row, relative to it
    for (GridIter it(nN1); it.u < nh; it.next()) {
        float2* a = A + (prow * it.u) * ld1 + it.v;
        *a = make_float2(a->x - mean1, a[pmate * ld1].x - mean1);
    }
    __syncthreads();
    wstfft::EpiIdentity id;
    if (!(dbg & 4))
        lds_fft_lines<FN, SQ ? prev_cap(MAXN) : 0, MAXN, kRD, false>(A, wstfft::Lines{1, 0, nh, prow * ld1, 1}, nN1,
                                            tb.twN(j1), id);

    // 5. split into the two rows' half spectra (columns 0..nN1/2) and export them
    const int hld = (nN1 >> 1) + 1;
    float2* H = hexp + item * hspec_stride(nM1, hld, lay.hext);
    if (export_full(lay)) {
        // in place: packed row t -> half-spectrum rows t and t + nh (rows nh.. of A are free),
        // then the column FFTs (rows digit-reversed -> natural); k_o2 folds the fully transformed
        // spectrum from HBM/L2 and keeps only its path batches in LDS (host: nh * hld <= KS * T)
        constexpr int KS = 8;
        const int T = blockDim.x, nitems = nh * hld;
        const wstfft::FastDiv dh(hld);
        float2 e0[KS], e1[KS];
        int dst[KS];
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            const int w = threadIdx.x + k * T;
            dst[k] = -1;
            if (w < nitems) {
                const int t = dh.div(w), v = w - t * hld;
                const float2* row = A + (prow * t) * ld1;
                const float2 z = row[v];
                const float2 zm = row[v == 0 ? 0 : nN1 - v];
                e0[k] = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
                e1[k] = make_float2(0.5f * (z.y + zm.y), -0.5f * (z.x - zm.x));
                dst[k] = (prow * t) * ld1 + v;
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < KS; ++k)
            if (dst[k] >= 0) {
                A[dst[k]] = e0[k];
                A[dst[k] + pmate * ld1] = e1[k];
            }
        __syncthreads();
        lds_fft_lines<FM, SQ ? prev_cap(MAXN) : 0, MAXN, kRD, false>(A, wstfft::Lines{1, 0, hld, 1, ld1}, nM1,
                                                                     tb.twM(j1), id);
        for (GridIter it(hld); it.u < nM1; it.next()) stnt(H + it.u * hld + it.v, A[it.u * ld1 + it.v]);
        if (lay.hext)
            for (int i = threadIdx.x; i < hld; i += blockDim.x) stnt(H + nM1 * hld + i, A[i]);
        return;
    }
    for (GridIter it(hld); it.u < nh; it.next()) {
        const float2* row = A + (prow * it.u) * ld1;
        const float2 z = row[it.v];
        const float2 zm = row[it.v == 0 ? 0 : nN1 - it.v];
        const float2 h0 = make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
        const float2 h1 = make_float2(0.5f * (z.y + zm.y), -0.5f * (z.x - zm.x));
        float2* d = H + (prow * it.u) * hld + it.v;
        stnt(d, h0);
        stnt(d + pmate * hld, h1);
    }
}

// Variant trace of a k_o1 body, written after it ran (so the body's code is laid out as without
// it): the same compile-time constants and run-time tests the body's dispatch used.
template <int FM, int FN, int MAXN, int SQ, int OC, int N1T = 0>
__device__ __forceinline__ void trace_o1(const DevParams& p, const LdsLayout& lay, int j1) {
#ifndef WST_TRACE
    (void)p;
    (void)lay;
    (void)j1;
    return;
#endif
    if (!tracing(p, get_tslot(lay))) return;
    constexpr int N1C = N1T ? N1T : SQ ? unique_level(FM, MAXN) : 0;
    constexpr bool FUSE1 = SQ && N1C >= kFuse1Min && wstfft::LineFFT<(N1C > 0 ? N1C : 2), true>::N2 > 1;
    const bool fused1 = FUSE1 && j1 == 0;
    const bool do2 = (p.max_order >= 2) && (j1 < p.J - 1);
    const int b1 = p.box1_off[j1 * p.L + 0];   // workgroup 0 writes: item 0, theta1 = 0
    const bool use_box1 = b1 >= 0 && (1 << j1) >= p.box1_min_s;
    const int s1 = 1 << j1;
    const int f1 = fused1 ? 0 : s1 == 1 ? 1 : s1 == 2 ? 2 : use_box1 ? 3 : s1 == 4 ? 4 : 5;
    const int lp1 = SQ ? kLpTap : wide_lowpass(p) ? (mfma_rc_ok<N1C>() ? kLpMfmaRc : kLpMfma) : kLpPlain;
    trace_word(p, get_tslot(lay), 0, tr_kernel(kTkO1, FM, FN, MAXN, SQ, 0));
    trace_word(p, get_tslot(lay), 1, tr_o1(OC, N1C, fused1 ? 1 : 0, lp1, do2 ? 1 : 0, export_full(lay), f1));
}

template <int FM, int FN, int MAXN, int SQ>
__global__ void __launch_bounds__(1024, o1_min_waves(MAXN, FM, FN)) k_o1(DevParams p, LdsLayout lay, int j1, int nimg,
                                             long long img0, const float2* __restrict__ xhat,
                                             float2* __restrict__ hexp, float* __restrict__ out,
                                             int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    // (the 4 x 4 variant measured neutral for the smaller classes: only the 96^2 class carries it)
    if constexpr (SQ && MAXN == 136) {
        if (p.oM == 4 && p.oN == 4 && lay.oms == 4) {
            k_o1_body<FM, FN, MAXN, SQ, 4>(smem, p, lay, j1, nimg, img0, xhat, hexp, out, pooled);
            trace_o1<FM, FN, MAXN, SQ, 4>(p, lay, j1);
            return;
        }
    }
    if constexpr (!SQ && FM == FN && FM > 0) {
        // square levels of the family's sizes in this class: compile-time level size (f3 / c1)
        if (p.PM == p.PN) {
            bool done = false;
            wstfft::static_for<0, 8>([&](auto mc) {
                constexpr int N1X = FM << decltype(mc)::value;
                if constexpr (N1X <= MAXN && N1X > prev_cap(MAXN)) {
                    if (!done && (p.PM >> j1) == N1X) {
                        done = true;
                        k_o1_body<FM, FN, MAXN, SQ, 0, N1X>(smem, p, lay, j1, nimg, img0, xhat, hexp, out, pooled);
                        trace_o1<FM, FN, MAXN, SQ, 0, N1X>(p, lay, j1);
                    }
                }
            });
            if (done) return;
        }
    }
    k_o1_body<FM, FN, MAXN, SQ, 0>(smem, p, lay, j1, nimg, img0, xhat, hexp, out, pooled);
    trace_o1<FM, FN, MAXN, SQ, 0>(p, lay, j1);
}

// ------------------------------------------------------------------------------------------
// k_o2: one workgroup per (plane, theta1) at fixed j1 -- all order-2 paths from U1hat
// ------------------------------------------------------------------------------------------
// Minimum waves per SIMD requested for k_o2 per size class (the VGPR budget follows): the small
// levels run many workgroups per CU and gain from 5-6 waves (cap 48: 1.09 -> 0.98 ms at c2); the
// 96^2 level is held at 2 workgroups per CU by LDS and spills below ~112 VGPRs (measured).
constexpr int o2_min_waves(int cap) { return cap == 48 ? 6 : cap == 24 ? 5 : 1; }
// HG = 1: the level-j1 spectrum is a big (HBM-staged, wst_staged.h) level: `hexp` holds the
// fully transformed half spectra in natural order, the fold reads them from HBM (no LDS copy,
// no column FFT) and the paths start at j2first (the first LDS-resident level).
// k_o2 body; OC > 0: the output maps are OC x OC (compile-time; the common 4 x 4 of the headline).
// LC > 0 (even): L = LC at compile time; the first order-2 level (j2 = j1 + 1) runs in batches of
// two paths (one filter pair; a smaller batch than the layout allows is always valid) and every
// deeper level in one batch of all LC paths (the layout's B holds LC paths of level j1 + 2, so of
// every level below it), so each batch shape -- paths, pairs, lines, loop bounds and divisors --
// folds at compile time.
template <int FM, int FN, int MAXN, int SQ, int HG, int OC, int LC = 0>
__device__ __forceinline__ void k_o2_body(unsigned char* smem, const DevParams& p,
                                          const LdsLayout& lay, int j1, int nimg, long long img0,
                                          const float2* __restrict__ hexp, float* __restrict__ out,
                                          int pooled, int j2first) {
    const int oM = OC ? OC : p.oM, oN = OC ? OC : p.oN;
    const int oms = OC ? 4 : lay.oms;
    const int J = p.J, L = LC ? LC : p.L;
    const int nsplit = HG ? max(1, lay.nsplit) : 1;
    int item, ksplit = 0;
    if (nsplit > 1) {
        // blocks x and x + 8 share an XCD: the nsplit workgroups of an item take consecutive
        // dispatch slots of one XCD, so they run together and read H through the same L2
        const int total = nimg * L;
        const int x = blockIdx.x;
        if ((total & 7) == 0) {
            // hgroup items per group, batch-major inside it: concurrent workgroups of the XCD fold
            // the same batch (its filter pairs stay in L2) for neighbouring items
            const int slot = x >> 3;
            const int nper = total >> 3;
            const int G = max(1, lay.hgroup);
            const int grp = slot / (nsplit * G);
            const int rem = slot - grp * nsplit * G;
            const int gc = min(G, nper - grp * G);
            ksplit = rem / gc;
            item = (x & 7) * nper + grp * G + (rem - ksplit * gc);
        } else {
            item = x / nsplit;
            ksplit = x - item * nsplit;
        }
    } else {
        item = xcd_item(nimg * L);
    }
    const int PM = p.PM, PN = p.PN;
    constexpr int N1C = (SQ && !HG) ? unique_level(FM, MAXN) : 0;
    const int nM1 = N1C ? N1C : PM >> j1, nN1 = N1C ? N1C : PN >> j1;
    const int n1 = nM1 * nN1;
    const int hld = (nN1 >> 1) + 1;
    float2* B = reinterpret_cast<float2*>(smem + lay.off_b);
    float* S = reinterpret_cast<float*>(smem + lay.off_s);
    const Tables tb = load_tables(p, lay, smem);
    const int dbg = WST_DBG_MASK(p);
    wstfft::EpiIdentity id;
    // order-2 path sizes: <= MAXN / 2 below an LDS-resident level of class MAXN, <= MAXN after a
    // big level
    constexpr int PHI = (SQ && !HG) ? MAXN / 2 : MAXN;
    const int local = item / L;
    const int l1 = item - local * L;
    const long long img = img0 + local;
    const float2* Hg = hexp + item * hspec_stride(nM1, hld, lay.hext);
    const float2* H = HG ? Hg : reinterpret_cast<const float2*>(smem);

    if constexpr (!HG) {
        // 1. half spectrum rows -> LDS, then the column FFTs (rows digit-reversed -> natural)
        float2* Hl = reinterpret_cast<float2*>(smem);
        if constexpr (N1C > 0 && wstfft::LineFFT<(N1C > 0 ? N1C : 2), false>::N2 > 1) {
            // compile-time two-stage size: the column transform's first stage reads the rows from
            // the workspace itself (no separate copy pass and barrier; tables ready after one)
            __syncthreads();
            wstfft::fft_lines_rd_from<N1C, false>(Hl, Hg, wstfft::Lines{1, 0, hld, 1, hld}, tb.twM(j1), id);
        } else {
            if (!(dbg & 1024)) copy_to_lds(Hl, Hg, nM1 * hld);
            __syncthreads();
            if (!(dbg & 4))
                lds_fft_lines<FM, SQ ? prev_cap(MAXN) : 0, MAXN, kRD, false>(
                    Hl, wstfft::Lines{1, 0, hld, 1, hld}, nM1, tb.twM(j1), id);
        }
        if constexpr (N1C > 0) {
            // row N1 = row 0: the tile folds' mirrored taps of bin row u = 0 at alias a = 0
            for (int i = threadIdx.x; i < hld; i += blockDim.x) Hl[nM1 * hld + i] = Hl[i];
            __syncthreads();
        }
    }

    // 2. order-2 paths in batches: Hermitian fold -> |ifft| -> S2 low-pass
    const int kbase = p.o2_base[j1 * L + l1];
    const int nq = (L + 1) >> 1;
    int bctr = 0;   // batch counter (split HG launches)
    // every batch of paths of level j2 (sizes nM2 x nN2); PB > 0: compile-time paths per batch
    // SC > 0: the alias count s is a compile-time constant (square level N1C: tile-mapped folds)
    // NC > 0: the (square) path size is a compile-time constant
    auto level = [&](int j2, int nM2, int nN2, auto pbc, auto scc, auto ncc) __attribute__((always_inline)) {
        constexpr int PB = decltype(pbc)::value;
        constexpr int SC = decltype(scc)::value;
        constexpr int NC = decltype(ncc)::value;
        // s = 2 fold fused with the rows' stage A (two-stage row sizes >= kFuseMin)
        // N1F > 0: the spectrum's (square) size at compile time -- tile-mapped folds, reading H from
        // LDS or, in the exported-spectrum SQ kernel (HG), from HBM / L2 with the same offsets
        constexpr int N1F = (SQ && NC > 0 && SC > 0) ? NC * SC : 0;
        constexpr bool FUSE = N1F > 0 && SC == 2 && N1F / 2 >= kFuseMin &&
                              wstfft::LineFFT<(N1F > 0 ? N1F / 2 : 2), true>::N2 > 1;
        const int ld2 = odd_ld(nN2);
        const int pslot = nM2 * ld2;
        const int s2 = 1 << (j2 - j1);
        int pb = lay.bcap / pslot;                 // paths per batch (multiple of 2)
        pb = PB ? PB : max(2, min(pb & ~1, 2 * nq));
#pragma unroll 1
        for (int l2a = 0; l2a < L; l2a += pb) {
            if (nsplit > 1) {
                const int bi = bctr++;
                if (bi % nsplit != ksplit) continue;
            }
            const int npath = (PB > 0 && LC % (PB > 0 ? PB : 1) == 0) ? PB : min(pb, L - l2a);
            const int npair = (npath + 1) >> 1;
            const float2* ps = p.psi2 + p.psi2_off[(j2 * J + j1) * nq + (l2a >> 1)];
            const long long pstride = static_cast<long long>(n1);
            const int* bx = p.box + p.box_off[j2 * J + j1] + (l2a >> 1) * (nM2 + nN2);
            if (!(dbg & 8) && !(dbg & (s2 == 2 ? 256 : 512))) {
                if constexpr (FUSE) {
                    fold2_s2_rowA<N1F>(H, ps, npair, npath, B, tb.twN(j2), ps + nq * pstride);
                } else if constexpr (N1F > 0 && SC == 2) {
                    fold2_tile_s2<N1F>(H, ps, npair, npath, B, ps + nq * pstride);
                } else if constexpr (N1F > 0 && (SC == 4 || SC == 8)) {
                    constexpr int NT = ((N1F / SC) * (N1F / SC) + 63) / 64;
                    fold2_tile_list<N1F, SC>(H, ps, npair, npath, B,
                                             p.taph + p.taph_off[j2 * J + j1] + (l2a >> 1) * NT, p.taps);
                } else {
                    // the alias-interleaved copy exists for every s = 2 level of a square plane
                    fold2_any<HG ? 3 : 1>(s2, H, hld, nM1, nN1, ps, pstride, npair, npath, B, pslot, ld2, nM2,
                                          nN2, bx, nM2 + nN2, p.PM == p.PN ? ps + nq * pstride : nullptr);
                }
            }
            __syncthreads();
            const float scale2 = 1.f / static_cast<float>(n1);
            if constexpr (SQ) {
                // rows, then the column pass fused with |.| and the S2 low-pass
                if (!(dbg & 16)) {
                    if constexpr (FUSE)
                        wstfft::fft_lines_dr_stageB<(N1F > 0 ? N1F / 2 : 2), true,
                                                    fused_row_n2(N1F > 0 ? N1F / 2 : 2)>(
                            B, wstfft::Lines{npath, pslot, nM2, ld2, 1}, id);
                    else
                        lds_fft_lines<FN, 0, PHI, kDR, true>(
                            B, wstfft::Lines{npath, pslot, nM2, ld2, 1}, nN2, tb.twN(j2), id);
                }
                const int k0 = kbase + (j2 - j1 - 1) * L + l2a;
                float* outd = pooled ? nullptr : out + (img * p.K + k0) * (oM * oN);
                if (!(dbg & 64))
                    family_cols_modlp<FM, 0, PHI, FUSE ? fused_row_n2(N1F > 0 ? N1F / 2 : 2) : 0>(
                                                       B, npath, pslot, nM2, nN2, ld2, tb.twM(j2),
                                                       tb.gM(j2), tb.gN(j2), oms, oM, oN,
                                                       scale2, S, outd);
                if (!outd) emit(S, npath, k0, img, p.K, oM, oN, out, pooled);
            } else {
                EpiModulus mod2{scale2, 0.f};
                if (!(dbg & 16))
                    lds_fft2<FM, FN, 0, MAXN, kDR, true>(B, npath, pslot, nM2, nN2, ld2, tb.twM(j2),
                                                         tb.twN(j2), mod2);
                if (!(dbg & 64)) {
                    const int k0 = kbase + (j2 - j1 - 1) * L + l2a;
                    if (wide_lowpass(p)) {
                        // the maps go to the .x slots of the arrays (no S region: the exported-
                        // spectrum k_o2 fits two workgroups per CU); the next fold rewrites B
                        float* SB = reinterpret_cast<float*>(B);
                        if constexpr (mfma_rc_ok<NC>())
                            lds_lowpass_mfma_rc<NC>(B, npath, pslot, ld2, lpw_M(p, j2), lpw_N(p, j2), p.oMp,
                                                    p.oNp, oM, oN, SB, 2 * pslot, 2);
                        else
                            lds_lowpass_mfma(B, npath, pslot, nM2, nN2, ld2, lpw_M(p, j2), lpw_N(p, j2),
                                             p.oMp, p.oNp, oM, oN, SB, 2 * pslot, 2);
                        if (!(dbg & 2048)) emit(SB, npath, k0, img, p.K, oM, oN, out, pooled, 2 * pslot, 2);
                        __syncthreads();
                    } else {
                        lds_lowpass(B, npath, pslot, nM2, nN2, ld2, tb.lpM(j2), tb.lpN(j2), tb.pmM(j2),
                                    tb.pmN(j2), 1 << (J - j2), oM, oN, S);
                        emit(S, npath, k0, img, p.K, oM, oN, out, pooled);
                    }
                }
            }
            // no barrier here: the next batch's fold writes B only, and S is rewritten only after
            // that batch's transform barriers (emit above reads S alone)
        }
    };
    // The order-2 levels of this launch and their compile-time shapes, in one place: FN_ is
    // called once per level as FN_(j2, nM2, nN2, PB, SC, NC).  The trace pass (below) and the
    // work expand the same dispatch, so the trace records the path the work takes.  (A macro,
    // not a lambda taking the functor: the lambda form cost the f3 k_o2 1 % -- 1570 more
    // instructions, SGPR spills from the kernel entry on; measured round 5.)
    // Branches: N1C > 0 -- compile-time level sizes N1C / 2^k (an SQ launch's paths start at
    // j2 = j1 + 1); SQ HG -- after a big level the paths start at the first LDS-resident level,
    // the family's single size of this class (> 136 / 2): compile-time sizes from there on (from
    // the exported spectrum with tile-mapped folds when k_o1 finished that level's column FFTs;
    // runtime sizes when a plan stages that level too and starts further down); !SQ HG (f3 / c1)
    // -- a square level of one of the family's sizes runs with compile-time path sizes (and, with
    // LC, compile-time batch shapes); otherwise runtime sizes.
#define WST_O2_DISPATCH(FN_)                                                                                                                      \
    if constexpr (N1C > 0) {                                                                                                                      \
        wstfft::static_for<1, 8>([&](auto kc) {                                                                                                   \
            constexpr int k = decltype(kc)::value;                                                                                                \
            constexpr int NN2 = N1C >> k;                                                                                                         \
            if constexpr ((NN2 << k) == N1C && NN2 >= 1)                                                                                          \
                if (j1 + k < J && j1 + k >= j2first)                                                                                              \
                    FN_(j1 + k, NN2, NN2,                                                                                                         \
                          std::integral_constant<int, LC == 0 ? 0 : (k == 1 && MAXN > kWholeFirstCap) ? 2 : LC>{},                                \
                          std::integral_constant<int, (1 << k)>{}, std::integral_constant<int, NN2>{});                                           \
        });                                                                                                                                       \
    } else if constexpr (SQ && HG == 1 && unique_level(FM, MAXN) > 0) {                                                                           \
        constexpr int N2C = unique_level(FM, MAXN);                                                                                               \
        if (j2first == j1 + 1 && (PM >> j1) == N2C && PM == PN) {                                                                                 \
            wstfft::static_for<1, 8>([&](auto kc) {                                                                                               \
                constexpr int k = decltype(kc)::value;                                                                                            \
                constexpr int NN2 = N2C >> k;                                                                                                     \
                if constexpr ((NN2 << k) == N2C && NN2 >= 1)                                                                                      \
                    if (j1 + k < J)                                                                                                               \
                        FN_(j1 + k, NN2, NN2, std::integral_constant<int, LC == 0 ? 0 : k == 1 ? 2 : LC>{},                                       \
                              std::integral_constant<int, (1 << k)>{}, std::integral_constant<int, NN2>{});                                       \
            });                                                                                                                                   \
        } else if ((PM >> j2first) == N2C) {                                                                                                      \
            wstfft::static_for<0, 8>([&](auto kc) {                                                                                               \
                constexpr int k = decltype(kc)::value;                                                                                            \
                constexpr int NN2 = N2C >> k;                                                                                                     \
                if constexpr ((NN2 << k) == N2C && NN2 >= 1)                                                                                      \
                    if (j2first + k < J) FN_(j2first + k, NN2, NN2, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},           \
                  std::integral_constant<int, 0>{});                                                                                              \
            });                                                                                                                                   \
        } else {                                                                                                                                  \
            for (int j2 = j2first; j2 < J; ++j2) FN_(j2, PM >> j2, PN >> j2, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},  \
                  std::integral_constant<int, 0>{});                                                                                              \
        }                                                                                                                                         \
    } else if constexpr (!SQ && HG == 1 && FM == FN && FM > 0) {                                                                                  \
        bool done = false;                                                                                                                        \
        if (PM == PN && j2first == j1 + 1) {                                                                                                      \
            wstfft::static_for<0, 8>([&](auto mc) {                                                                                               \
                constexpr int N1X = FM << decltype(mc)::value;                                                                                    \
                if constexpr (N1X <= MAXN && N1X > prev_cap(MAXN)) {                                                                              \
                    if (!done && (PM >> j1) == N1X) {                                                                                             \
                        done = true;                                                                                                              \
                        wstfft::static_for<1, 8>([&](auto kc) {                                                                                   \
                            constexpr int k = decltype(kc)::value;                                                                                \
                            constexpr int NN2 = N1X >> k;                                                                                         \
                            if constexpr ((NN2 << k) == N1X && NN2 >= 1)                                                                          \
                                if (j1 + k < J)                                                                                                   \
                                    FN_(j1 + k, NN2, NN2,                                                                                         \
                                          std::integral_constant<int, LC == 0 ? 0 : k == 1 ? 2 : LC>{},                                           \
                                          std::integral_constant<int, 0>{}, std::integral_constant<int, NN2>{});                                  \
                        });                                                                                                                       \
                    }                                                                                                                             \
                }                                                                                                                                 \
            });                                                                                                                                   \
        }                                                                                                                                         \
        if (!done)                                                                                                                                \
            for (int j2 = j2first; j2 < J; ++j2) FN_(j2, PM >> j2, PN >> j2, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},  \
                  std::integral_constant<int, 0>{});                                                                                              \
    } else {                                                                                                                                      \
        for (int j2 = j2first; j2 < J; ++j2) FN_(j2, PM >> j2, PN >> j2, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},      \
                  std::integral_constant<int, 0>{});                                                                                              \
    }
    WST_O2_DISPATCH(level)
#ifdef WST_TRACE   // (the trace build only: not even dead code in the product)
    if (tracing(p, get_tslot(lay))) {
        // trace pass, after the work (the hot code's layout and registers stay as without it):
        // the same dispatch with a functor that only records each level's path
        constexpr int spec = HG ? 0 : (N1C > 0 && wstfft::LineFFT<(N1C > 0 ? N1C : 2), false>::N2 > 1) ? 1 : 2;
        // the branch the dispatch takes (same tests, in the same order)
        int br = 7;
        if constexpr (N1C > 0) {
            br = 1;
        } else if constexpr (SQ && HG == 1 && unique_level(FM, MAXN) > 0) {
            constexpr int N2C = unique_level(FM, MAXN);
            br = (j2first == j1 + 1 && (PM >> j1) == N2C && PM == PN) ? 2 : (PM >> j2first) == N2C ? 3 : 4;
        } else if constexpr (!SQ && HG == 1 && FM == FN && FM > 0) {
            br = 6;
            if (PM == PN && j2first == j1 + 1)
                wstfft::static_for<0, 8>([&](auto mc) {
                    constexpr int N1X = FM << decltype(mc)::value;
                    if constexpr (N1X <= MAXN && N1X > prev_cap(MAXN))
                        if ((PM >> j1) == N1X) br = 5;
                });
        }
        const int lpw = wide_lowpass(p) ? 1 : 0;
        auto record = [&](int j2, int, int, auto pbc, auto scc, auto ncc) __attribute__((always_inline)) {
            constexpr int PB = decltype(pbc)::value, SC = decltype(scc)::value, NC = decltype(ncc)::value;
            constexpr int N1F = (SQ && NC > 0 && SC > 0) ? NC * SC : 0;
            constexpr bool FUSE = N1F > 0 && SC == 2 && N1F / 2 >= kFuseMin &&
                                  wstfft::LineFFT<(N1F > 0 ? N1F / 2 : 2), true>::N2 > 1;
            constexpr int fk = FUSE ? kFdFused : (N1F > 0 && SC == 2) ? kFdTileS2
                             : (N1F > 0 && (SC == 4 || SC == 8)) ? kFdTileList : 0;
            const int s2 = 1 << (j2 - j1);
            const int lpk = SQ ? kLpTap : lpw ? (mfma_rc_ok<NC>() ? kLpMfmaRc : kLpMfma) : kLpPlain;
            if (2 + (j2 - j1 - 1) < kTraceW)
                trace_word(p, get_tslot(lay), 2 + (j2 - j1 - 1),
                           tr_level(j2, PB, SC, NC, fk ? fk : (s2 == 2 ? kFdDenseS2 : kFdBox), lpk, s2));
        };
        WST_O2_DISPATCH(record)
        trace_word(p, get_tslot(lay), 0, tr_kernel(kTkO2, FM, FN, MAXN, SQ, HG));
        trace_word(p, get_tslot(lay), 1, tr_o2(OC, LC, N1C, spec, br));
    }
#endif
#undef WST_O2_DISPATCH
}


template <int FM, int FN, int MAXN, int SQ, int HG = 0>
__global__ void __launch_bounds__(1024, o2_min_waves(MAXN)) k_o2(DevParams p, LdsLayout lay, int j1, int nimg,
                                             long long img0, const float2* __restrict__ hexp,
                                             float* __restrict__ out, int pooled, int j2first) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    if constexpr (SQ) {
        if (p.oM == 4 && p.oN == 4 && lay.oms == 4) {
            if constexpr (unique_level(FM, MAXN) > 0) {
                if (p.L == 8) {
                    k_o2_body<FM, FN, MAXN, SQ, HG, 4, 8>(smem, p, lay, j1, nimg, img0, hexp, out, pooled, j2first);
                    return;
                }
            }
            k_o2_body<FM, FN, MAXN, SQ, HG, 4>(smem, p, lay, j1, nimg, img0, hexp, out, pooled, j2first);
            return;
        }
    }
    if constexpr (!SQ && HG && FM == FN && FM > 0) {
        if (p.L == 8) {
            k_o2_body<FM, FN, MAXN, SQ, HG, 0, 8>(smem, p, lay, j1, nimg, img0, hexp, out, pooled, j2first);
            return;
        }
    }
    k_o2_body<FM, FN, MAXN, SQ, HG, 0>(smem, p, lay, j1, nimg, img0, hexp, out, pooled, j2first);
}

}  // namespace wstdev
