// HBM-staged passes for the levels whose planes do not fit the LDS-resident kernels (n > 136,
// e.g. BASELINE config c5: 256x256 bands, J=6 -> 384^2 and 192^2 levels).
//
// A big n x n level is transformed as a row pass then a column pass through HBM; each pass stages
// a block of whole lines in LDS and runs the same LDS FFT engine (fft_lds.h, natural order).  The
// kymatio steps around each transform are fused into the passes:
//   k_big_rows (forward):  kRowPad   reflect-pad gather of the input plane, S0 row partials,
//                                    mean removal (conditioning only, as k_prep)
//                          kRowHalf  rows 0..m/2 of the column-transformed U1 (kColModLpFwd), the
//                                    global mean removed at row 0, forward row FFT, written with
//                                    their Hermitian mirrors as the natural-order half spectra
//   k_big_rows (inverse):  kRowFold1 fold_{2^j1}(Xhat * psi0) (order-1 subsample_fourier)
//                          kRowFold2 Hermitian fold_{2^(j2-j1)}(U1hat * psi2 pair), 2 paths
//   k_big_cols:            kColStore plain column transform
//                          kColModLp |.| * scale, optional U store, phi low-pass column partials
//                                    V[q][a] = sum_p GMnat[p][a] |z[p][q]| and column sums
//                          kColModLpFwd  kColModLp, then the forward column FFT of U (two columns
//                                    minus their own means per complex line) and its Hermitian
//                                    split: rows 0..m/2 of each column's spectrum (order 2 follows;
//                                    round 5: replaces a U store, a packed real-row pass and a
//                                    column pass per staged j1)
//   k_big_final:           S[a][c] from the partials (+ U1 mean), emitted like the LDS kernels
// SURVEY.md Appendix A.4; reference call sites train_and_save_model.py:359-376.
#pragma once

#include "wst_device.h"

namespace wstbig {

using wstdev::DevParams;

constexpr int kBigMinN = wstfft::kMaxFamilyN;   // levels with n > kBigMinN are staged
constexpr int kBigThreads = 256;   // row passes, plane means (512: c5 +5 %, measured round 5)
// Column-pass workgroup by line length: the 384- and 512-point tiles (58-70 KB, two workgroups per
// CU) keep more loads in flight with 512 threads (c5's 384^2 order-1 column pass 5.54 -> 5.10 ms
// per step), the shorter ones hold more workgroups per CU and lose with it (192: +0.2 / +1.1 ms;
// 1024 threads: worse everywhere).  0 = runtime length.
constexpr int big_col_threads(int n) { return n >= 384 ? 512 : 256; }
constexpr int kColTile = 16;         // columns per column-pass workgroup (128 B rows)
constexpr int kMeanParts = 16;                  // k_big_mean partial sums per plane
constexpr int kLoadBatch = 8;                   // global loads per thread in flight (tile loads)
// Loads per thread in flight in the staged passes (measured at c5, profiles/r06_ab.txt r06n-r06q):
// a compiled length's whole column-tile share in one batch (12 at 192 and 384 points: -2 %), the
// 384-point s = 1 order-1 row fold 24 per batch, the reflect-pad gather / column-spectrum rows /
// s = 2 order-1 row fold kInBatch per batch (each was one load per loop iteration: -5 %)
constexpr int kTileBatchMax = 16;
constexpr int kRowBatch = 8;
constexpr int kRowBatch384 = 24;
constexpr int kInBatch = 4;
// Column-tile loads per thread in flight: a compiled length's whole tile share (N x kColTile /
// threads) in one batch, up to kTileBatchMax; runtime lengths kLoadBatch
constexpr int col_tile_batch(int N) {
    return N > 0 ? ((N * kColTile + big_col_threads(N) - 1) / big_col_threads(N) < kTileBatchMax
                        ? (N * kColTile + big_col_threads(N) - 1) / big_col_threads(N)
                        : kTileBatchMax)
                 : kLoadBatch;
}
// 16-byte streaming I/O: compiled (even) lengths move element pairs per lane -- column-tile loads,
// row-pass and column-spectrum stores, the column-spectrum rows' loads, Xhat in the order-1 row
// folds (8-byte accesses stream at a fraction of the 16-byte rate; c5 -4 %, r06p / r06q)
typedef float wst_f4 __attribute__((ext_vector_type(4)));
// two consecutive complex elements as one 16-byte streaming load / store (16-byte aligned)
__device__ __forceinline__ wst_f4 ldnt2(const float2* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const wst_f4*>(p));
}
__device__ __forceinline__ void stnt2(float2* p, float2 a, float2 b) {
    wst_f4 v = {a.x, a.y, b.x, b.y};
    __builtin_nontemporal_store(v, reinterpret_cast<wst_f4*>(p));
}
constexpr int kBigOGroup = 16;                  // outputs per accumulation round of wide low-passes

enum RowMode { kRowPad = 0, kRowFold1 = 2, kRowFold2 = 3, kRowHalf = 4 };   // (1: retired)
enum ColMode { kColStore = 0, kColModLp = 1, kColModLpFwd = 2 };
enum FinalMode { kFinalRows = 0, kFinalCols = 1 };

// Arguments of one staged launch (POD, by value).  A level's arrays are nrows x ncols (PM >> r by
// PN >> r, or PN >> r / 2 + 1 columns for half spectra); a row pass transforms lines of n = ncols
// points, a column pass lines of n = nrows points.  Kernels instantiated with N = 0 take n at run
// time (generic DFT: sizes without a compiled FFT).
struct BigArgs {
    int mode;
    int n;                       // line length of this pass
    int lvl;                     // level r (twiddles, tap matrices)
    int rows;                    // rows per workgroup (row pass)
    int nrows;                   // row pass: rows of the array
    int ncols;                   // column pass: columns of the array (its row stride)
    int L;
    long long img0;              // first plane of the chunk (output row)
    // kRowPad
    const float* in;
    const float* mean;           // kRowPad: plane sum partials (kMeanParts per plane);
                                 // kRowHalf: (plane, l1) U1 means
    float* tpart;                // kRowPad: S0 row partials (nrows x oms per plane)
    // kRowFold1
    const float2* xhat;
    int j1;                      // kRowFold1: psi level-0 filters of scale j1; s = 2^j1
    // kRowFold2
    const float2* hsrc;          // half spectra at level j1 ((nrows s) x (n1/2+1) per (plane, l1))
    int n1, l1, j2;              // n1: row length at level j1 (= n s)
    const float2* psi2;          // pair 0 of (j2, j1) in the psi2 pool
    long long pstride;           // (nrows s) n1 (pool stride between pairs)
    const int* box;              // alias boxes of the pairs (s >= 4), stride nrows + n
    int npair, npath;            // pairs / paths per (plane, l1); one launch per l1, one
                                 // workgroup per (plane, row block) loops over the pairs
    int fold_all;                // kRowFold2, s = 2: every path of the block folded from one
                                 // read of the spectrum taps, one FFT pass over npath * rows lines
    // outputs
    float2* dst;
    float2* colt;                // kColModLpFwd: column spectra rows 0..m/2 ((m/2+1) x ncols per
                                 // array); kRowHalf: their source (nrows = m/2 + 1 valid rows)
    float* vpart;                // kColModLp: V[q][a] (ncols x oms per array)
    float* csum;                 // kColModLp: column sums (ncols per array)
    float scale;                 // kColModLp
    const float* gnat;           // natural-order tap matrix: GN_0 (kRowPad) / GM_lvl (kColModLp)
    int g_lds;                   // kColModLp: tap matrix staged in LDS (0: read from L2)
    int oms;                     // row stride of the tap matrices and of tpart / vpart
    int tslot;                   // variant-trace site (wstdev::trace_word)
};

// twiddles exp(-2 pi i k / n) of level r: side 0 = M (column lines), 1 = N (row lines)
__device__ __forceinline__ const float2* level_tw(const DevParams& p, int r, int side) {
    return p.tw + p.tw_off[2 * r + side];
}

// n-point transforms along LDS lines: the compiled FFT for N > 0, the generic DFT for N = 0
template <int N, bool INV, class Epi>
__device__ __forceinline__ void big_fft(float2* A, const wstfft::Lines& g, int n, const float2* tw,
                                        Epi& epi) {
    if constexpr (N > 0)
        wstfft::fft_lines<N, INV>(A, g, tw, epi);
    else
        wstdev::lds_dft_lines_generic(A, g, n, tw, INV, epi);
}

// --------------------------------------------------------------------------------------------
// row pass
// --------------------------------------------------------------------------------------------
// LDS: twiddles (n) | lines (nlines x ld, ld = n | 1) | scratch.
template <int N, bool INV>
__global__ void __launch_bounds__(kBigThreads) k_big_rows(DevParams p, BigArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int n = N > 0 ? N : a.n;
    const int ld = n | 1;
    const int m = a.nrows;
    float2* tw = reinterpret_cast<float2*>(smem);
    float2* A = tw + n;
    const int T = blockDim.x;
    const int arr = blockIdx.y;
    const int r0 = blockIdx.x * a.rows;
    const float2* gtw = level_tw(p, a.lvl, 1);
    for (int i = threadIdx.x; i < n; i += T) tw[i] = gtw[i];
    int nlines = a.rows;
    if (wstdev::tracing(p, a.tslot)) {
        wstdev::trace_word(p, a.tslot, 0, wstdev::tr_kernel(wstdev::kTkBigRows, 0, 0, N, 0, INV ? 1 : 0));
        wstdev::trace_word(p, a.tslot, 1,
                           wstdev::tr_big(a.mode, a.fold_all, a.mode == kRowFold1 ? (a.j1 == 0 ? 1 : 2) : 0,
                                          (a.mode == kRowFold2 && !a.fold_all && a.box && a.n1 / n >= 4) ? 1 : 0,
                                          0, 0, 0));
    }

    if (a.mode == kRowPad) {
        // arr = chunk-local plane; raw values first (S0 partials), then mean-centred
        const int inM = p.pre_pad ? p.PM : p.M, inN = p.pre_pad ? p.PN : p.N;
        const float* x = a.in + static_cast<long long>(arr) * inM * inN;
        constexpr int IB = kInBatch;   // gather loads per thread in flight
        for (int i0 = threadIdx.x; i0 < a.rows * n; i0 += IB * T) {
            float xv[IB];
#pragma unroll
            for (int k = 0; k < IB; ++k) {
                const int i = min(i0 + k * T, a.rows * n - 1);
                const int rr = i / n, q = i - (i / n) * n;
                const int u = r0 + rr;
                const int su = p.pre_pad ? u : wstdev::reflect_index(u - p.padTop, p.M);
                const int sv = p.pre_pad ? q : wstdev::reflect_index(q - p.padLeft, p.N);
                xv[k] = x[su * inN + sv];
            }
#pragma unroll
            for (int k = 0; k < IB; ++k) {
                const int i = i0 + k * T;
                const int rr = i / n, q = i - (i / n) * n;
                if (i < a.rows * n) A[rr * ld + q] = make_float2(xv[k], 0.f);
            }
        }
        __syncthreads();
        // S0 row partials T[p][c] = sum_q GN0[q][c] x[p][q] (natural order), 8 lanes per output
        for (int w = threadIdx.x; w < a.rows * p.oN * 8; w += T) {
            const int qc = w & 7;
            const int o = w >> 3;
            const int rr = o / p.oN, c = o - (o / p.oN) * p.oN;
            float acc = 0.f;
            for (int q = qc; q < n; q += 8) acc = fmaf(a.gnat[q * a.oms + c], A[rr * ld + q].x, acc);
            acc = wstdev::group_sum<8>(acc);
            if (qc == 0) a.tpart[(static_cast<long long>(arr) * m + r0 + rr) * a.oms + c] = acc;
        }
        float msum = 0.f;   // plane mean from k_big_mean's partials, fixed order (deterministic)
        for (int k = 0; k < kMeanParts; ++k) msum += a.mean[arr * kMeanParts + k];
        const float mu = msum / (static_cast<float>(p.PM) * static_cast<float>(p.PN));
        __syncthreads();
        for (int i = threadIdx.x; i < a.rows * n; i += T) {
            const int rr = i / n, q = i - (i / n) * n;
            A[rr * ld + q].x -= mu;
        }
    } else if (a.mode == kRowHalf) {
        // arr = plane * L + l1; rows r0.. of the m/2 + 1 column-spectrum rows (a.nrows of them).
        // Row 0 holds sum_p (U[p][q] - mu_q) (each column minus its own mean, kColModLpFwd); the
        // global-mean-removed row is that + m (mu_q - mu) = + csum[q] - m mu.
        nlines = min(a.rows, a.nrows - r0);
        const float2* Cs = a.colt + static_cast<long long>(arr) * a.nrows * n;
        const int mm = 2 * (a.nrows - 1);
        const float mu = a.mean[arr];
        constexpr int IB = kInBatch;   // loads per thread in flight
        if constexpr (N > 0 && N % 2 == 0) {
            // element pairs per lane: 16-byte streaming loads
            constexpr int H2 = N / 2;
            for (int i0 = threadIdx.x; i0 < nlines * H2; i0 += IB * T) {
                wst_f4 v[IB];
#pragma unroll
                for (int k = 0; k < IB; ++k) {
                    const int i = min(i0 + k * T, nlines * H2 - 1);
                    const int t = i / H2, q = 2 * (i - (i / H2) * H2);
                    v[k] = ldnt2(Cs + static_cast<long long>(r0 + t) * n + q);
                }
#pragma unroll
                for (int k = 0; k < IB; ++k) {
                    const int i = i0 + k * T;
                    const int t = i / H2, q = 2 * (i - (i / H2) * H2);
                    if (i < nlines * H2) {
                        float2 e0 = make_float2(v[k].x, v[k].y), e1 = make_float2(v[k].z, v[k].w);
                        if (r0 + t == 0) {
                            e0.x += a.csum[static_cast<long long>(arr) * n + q] - static_cast<float>(mm) * mu;
                            e1.x += a.csum[static_cast<long long>(arr) * n + q + 1] - static_cast<float>(mm) * mu;
                        }
                        A[t * ld + q] = e0;
                        A[t * ld + q + 1] = e1;
                    }
                }
            }
        } else
        for (int i0 = threadIdx.x; i0 < nlines * n; i0 += IB * T) {
            float2 v[IB];
#pragma unroll
            for (int k = 0; k < IB; ++k) {
                const int i = min(i0 + k * T, nlines * n - 1);
                const int t = i / n, q = i - (i / n) * n;
                v[k] = wstdev::ldnt(Cs + static_cast<long long>(r0 + t) * n + q);
            }
#pragma unroll
            for (int k = 0; k < IB; ++k) {
                const int i = i0 + k * T;
                const int t = i / n, q = i - (i / n) * n;
                if (i < nlines * n) {
                    if (r0 + t == 0) v[k].x += a.csum[static_cast<long long>(arr) * n + q] - static_cast<float>(mm) * mu;
                    A[t * ld + q] = v[k];
                }
            }
        }
    } else if (a.mode == kRowFold1) {
        // arr = plane * L + l1: rows of fold_s(Xhat * psi0_{j1, l1}), Xhat is (m s) x (n s)
        const int plane = arr / a.L, l1 = arr - (arr / a.L) * a.L;
        const int s = 1 << a.j1;
        const int PN = n * s;
        const float2* X = a.xhat + static_cast<long long>(plane) * (m * s) * PN;
        const float* psi0 = p.psi + p.psi_off[(a.j1 * a.L + l1) * p.J + 0];
        if (N > 0 && N % 2 == 0 && s == 1) {
            // element pairs per lane: Xhat as 16-byte loads (cacheable: every theta1 re-reads it),
            // the real filter as 8-byte ones
            constexpr int RB2 = ((N >= 384 && INV) ? kRowBatch384 : kRowBatch) / 2;
            constexpr int H2 = N > 0 ? N / 2 : 1;
            for (int i0 = threadIdx.x; i0 < a.rows * H2; i0 += RB2 * T) {
                wst_f4 xv[RB2];
                float2 f[RB2];
#pragma unroll
                for (int k = 0; k < RB2; ++k) {
                    const int i = min(i0 + k * T, a.rows * H2 - 1);
                    const int rr = i / H2, q = 2 * (i - (i / H2) * H2);
                    const long long idx = static_cast<long long>(r0 + rr) * PN + q;
                    f[k] = *reinterpret_cast<const float2*>(psi0 + idx);
                    xv[k] = *reinterpret_cast<const wst_f4*>(X + idx);
                }
#pragma unroll
                for (int k = 0; k < RB2; ++k) {
                    const int i = i0 + k * T;
                    const int rr = i / H2, q = 2 * (i - (i / H2) * H2);
                    if (i < a.rows * H2) {
                        A[rr * ld + q] = make_float2(xv[k].x * f[k].x, xv[k].y * f[k].x);
                        A[rr * ld + q + 1] = make_float2(xv[k].z * f[k].y, xv[k].w * f[k].y);
                    }
                }
            }
        } else if (s == 1) {
            constexpr int RB = (N >= 384 && INV) ? kRowBatch384 : kRowBatch;
            for (int i0 = threadIdx.x; i0 < a.rows * n; i0 += RB * T) {
                float2 xv[RB];
                float f[RB];
#pragma unroll
                for (int k = 0; k < RB; ++k) {
                    const int i = min(i0 + k * T, a.rows * n - 1);
                    const int rr = i / n, q = i - (i / n) * n;
                    const long long idx = static_cast<long long>(r0 + rr) * PN + q;
                    f[k] = psi0[idx];
                    xv[k] = X[idx];
                }
#pragma unroll
                for (int k = 0; k < RB; ++k) {
                    const int i = i0 + k * T;
                    const int rr = i / n, q = i - (i / n) * n;
                    if (i < a.rows * n) A[rr * ld + q] = make_float2(xv[k].x * f[k], xv[k].y * f[k]);
                }
            }
        } else if (N > 0 && N % 2 == 0 && s == 2) {
            // the four aliases of element pairs: 16-byte Xhat loads, 8-byte filter loads
            constexpr int IB2 = kInBatch > 1 ? kInBatch / 2 : 1;
            constexpr int H2 = N > 0 ? N / 2 : 1;
            for (int i0 = threadIdx.x; i0 < a.rows * H2; i0 += IB2 * T) {
                wst_f4 xv[IB2][4];
                float2 f[IB2][4];
#pragma unroll
                for (int k = 0; k < IB2; ++k) {
                    const int i = min(i0 + k * T, a.rows * H2 - 1);
                    const int rr = i / H2, q = 2 * (i - (i / H2) * H2);
                    const int u = r0 + rr;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const long long idx = static_cast<long long>(u + (t >> 1) * m) * PN + q + (t & 1) * n;
                        f[k][t] = *reinterpret_cast<const float2*>(psi0 + idx);
                        xv[k][t] = *reinterpret_cast<const wst_f4*>(X + idx);
                    }
                }
#pragma unroll
                for (int k = 0; k < IB2; ++k) {
                    const int i = i0 + k * T;
                    const int rr = i / H2, q = 2 * (i - (i / H2) * H2);
                    float2 acc0 = make_float2(0.f, 0.f), acc1 = make_float2(0.f, 0.f);
#pragma unroll
                    for (int t = 0; t < 4; ++t) {   // same order as the generic loop (ii, jj)
                        acc0 = make_float2(fmaf(xv[k][t].x, f[k][t].x, acc0.x), fmaf(xv[k][t].y, f[k][t].x, acc0.y));
                        acc1 = make_float2(fmaf(xv[k][t].z, f[k][t].y, acc1.x), fmaf(xv[k][t].w, f[k][t].y, acc1.y));
                    }
                    if (i < a.rows * H2) {
                        A[rr * ld + q] = acc0;
                        A[rr * ld + q + 1] = acc1;
                    }
                }
            }
        } else if (kInBatch > 1 && s == 2) {
            // the four aliases of IB elements in flight (8 IB independent loads before the sums)
            constexpr int IB = kInBatch;
            for (int i0 = threadIdx.x; i0 < a.rows * n; i0 += IB * T) {
                float2 xv[IB][4];
                float f[IB][4];
#pragma unroll
                for (int k = 0; k < IB; ++k) {
                    const int i = min(i0 + k * T, a.rows * n - 1);
                    const int rr = i / n, q = i - (i / n) * n;
                    const int u = r0 + rr;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const long long idx = static_cast<long long>(u + (t >> 1) * m) * PN + q + (t & 1) * n;
                        f[k][t] = psi0[idx];
                        xv[k][t] = X[idx];
                    }
                }
#pragma unroll
                for (int k = 0; k < IB; ++k) {
                    const int i = i0 + k * T;
                    const int rr = i / n, q = i - (i / n) * n;
                    float2 acc = make_float2(0.f, 0.f);
#pragma unroll
                    for (int t = 0; t < 4; ++t)   // same order as the generic loop (ii, jj)
                        acc = make_float2(fmaf(xv[k][t].x, f[k][t], acc.x), fmaf(xv[k][t].y, f[k][t], acc.y));
                    if (i < a.rows * n) A[rr * ld + q] = acc;
                }
            }
        } else
        for (int i = threadIdx.x; i < a.rows * n; i += T) {
            const int rr = i / n, q = i - (i / n) * n;
            const int u = r0 + rr;
            float2 acc = make_float2(0.f, 0.f);
            for (int ii = 0; ii < s; ++ii)
                for (int jj = 0; jj < s; ++jj) {
                    const long long idx = static_cast<long long>(u + ii * m) * PN + q + jj * n;
                    const float f = psi0[idx];
                    const float2 xv = X[idx];
                    acc = make_float2(fmaf(xv.x, f, acc.x), fmaf(xv.y, f, acc.y));
                }
            A[rr * ld + q] = acc;
        }
    } else {  // kRowFold2: arr = plane (one l1 per launch); every pair in turn, 2 paths each
        // level j1 is (m s) x n1, its real U1 held as half spectra of n1 / 2 + 1 columns
        const int n1 = a.n1, hld = n1 / 2 + 1, half = n1 / 2;
        const int s = n1 / n, smask = s - 1;
        const int m1 = m * s;
        const float2* H = a.hsrc + (static_cast<long long>(arr) * a.L + a.l1) * m1 * hld;
        wstfft::EpiIdentity id;
        if (a.fold_all) {
            // s = 2 (dense): the four spectrum taps of an output bin are read once and serve every
            // pair's filters (the per-pair passes re-read the spectrum from HBM: 8.5x the compulsory
            // bytes at c5); path p of row rr lands on line p * rows + rr
            // KI bins per thread in flight: their 4 KI spectrum taps, then per pair 4 KI filter taps
            constexpr int KI = 2;
            if constexpr (N > 0 && N % 2 == 0) {
                // a lane takes two adjacent bins (v, v + 1) of a row: every filter tap pair is one
                // 16-byte load (offsets kr n1 + kc even), the spectrum taps stay 8-byte loads (the
                // Hermitian mirror runs backwards and the half-spectrum rows are odd-length); c5
                // 18.60 -> 18.15 ms per step (r06u)
                constexpr int H2 = N / 2;
                for (int i = threadIdx.x; i < a.rows * H2; i += T) {
                    const int rr = i / H2, v = 2 * (i - (i / H2) * H2);
                    const int u = r0 + rr;
                    float2 h[2][4];
                    int fo[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int kr = u + (t >> 1) * m;
                        const int krm = kr == 0 ? 0 : m1 - kr;
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            const int kc = v + e + (t & 1) * n;
                            const bool mir = kc > half;
                            h[e][t] = H[mir ? krm * hld + (n1 - kc) : kr * hld + kc];
                            h[e][t].y = mir ? -h[e][t].y : h[e][t].y;
                        }
                        fo[t] = kr * n1 + v + (t & 1) * n;
                    }
                    for (int pr = 0; pr < a.npair; ++pr) {
                        const float2* ps = a.psi2 + pr * a.pstride;
                        wst_f4 f[4];
#pragma unroll
                        for (int t = 0; t < 4; ++t) f[t] = *reinterpret_cast<const wst_f4*>(ps + fo[t]);
#pragma unroll
                        for (int e = 0; e < 2; ++e) {
                            float2 a0 = make_float2(0.f, 0.f), a1 = make_float2(0.f, 0.f);
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                const float fa = e ? f[t].z : f[t].x, fb = e ? f[t].w : f[t].y;
                                a0 = make_float2(fmaf(h[e][t].x, fa, a0.x), fmaf(h[e][t].y, fa, a0.y));
                                a1 = make_float2(fmaf(h[e][t].x, fb, a1.x), fmaf(h[e][t].y, fb, a1.y));
                            }
                            A[(2 * pr * a.rows + rr) * ld + v + e] = a0;
                            if (2 * pr + 1 < a.npath) A[((2 * pr + 1) * a.rows + rr) * ld + v + e] = a1;
                        }
                    }
                }
            } else
            for (int i0 = threadIdx.x; i0 < a.rows * n; i0 += KI * T) {
                float2 h[KI][4];
                int fo[KI][4];
#pragma unroll
                for (int k = 0; k < KI; ++k) {
                    const int i = min(i0 + k * T, a.rows * n - 1);
                    const int rr = i / n, v = i - (i / n) * n;
                    const int u = r0 + rr;
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int kr = u + (t >> 1) * m, kc = v + (t & 1) * n;
                        const int krm = kr == 0 ? 0 : m1 - kr;
                        const bool mir = kc > half;
                        h[k][t] = H[mir ? krm * hld + (n1 - kc) : kr * hld + kc];
                        h[k][t].y = mir ? -h[k][t].y : h[k][t].y;
                        fo[k][t] = kr * n1 + kc;
                    }
                }
                for (int pr = 0; pr < a.npair; ++pr) {
                    const float2* ps = a.psi2 + pr * a.pstride;
                    float2 f[KI][4];
#pragma unroll
                    for (int k = 0; k < KI; ++k)
#pragma unroll
                        for (int t = 0; t < 4; ++t) f[k][t] = ps[fo[k][t]];
#pragma unroll
                    for (int k = 0; k < KI; ++k) {
                        const int i = i0 + k * T;
                        if (i >= a.rows * n) break;
                        const int rr = i / n, v = i - (i / n) * n;
                        float2 a0 = make_float2(0.f, 0.f), a1 = make_float2(0.f, 0.f);
#pragma unroll
                        for (int t = 0; t < 4; ++t) {
                            a0 = make_float2(fmaf(h[k][t].x, f[k][t].x, a0.x), fmaf(h[k][t].y, f[k][t].x, a0.y));
                            a1 = make_float2(fmaf(h[k][t].x, f[k][t].y, a1.x), fmaf(h[k][t].y, f[k][t].y, a1.y));
                        }
                        A[(2 * pr * a.rows + rr) * ld + v] = a0;
                        if (2 * pr + 1 < a.npath) A[((2 * pr + 1) * a.rows + rr) * ld + v] = a1;
                    }
                }
            }
            __syncthreads();
            big_fft<N, INV>(A, wstfft::Lines(1, 0, a.npath * a.rows, ld, 1), n, tw, id);
            if constexpr (N > 0 && N % 2 == 0) {
                // element pairs (q, q + 1) per lane: 16-byte streaming stores
                constexpr int H2 = N / 2;
                for (int i = threadIdx.x; i < a.npath * a.rows * H2; i += T) {
                    const int line = i / H2, q = 2 * (i - (i / H2) * H2);
                    const int path = line / a.rows, rr = line - path * a.rows;
                    float2* D = a.dst + (static_cast<long long>(arr) * a.npath + path) * m * n;
                    stnt2(D + (r0 + rr) * n + q, A[line * ld + q], A[line * ld + q + 1]);
                }
                return;
            }
            for (int i = threadIdx.x; i < a.npath * a.rows * n; i += T) {
                const int line = i / n, q = i - (i / n) * n;
                const int path = line / a.rows, rr = line - path * a.rows;
                float2* D = a.dst + (static_cast<long long>(arr) * a.npath + path) * m * n;
                wstdev::stnt(D + (r0 + rr) * n + q, A[line * ld + q]);
            }
            return;
        }
        for (int pr = 0; pr < a.npair; ++pr) {
            const float2* ps = a.psi2 + pr * a.pstride;
            const int* bx = a.box + pr * (m + n);
            for (int i = threadIdx.x; i < a.rows * n; i += T) {
                const int rr = i / n, v = i - (i / n) * n;
                const int u = r0 + rr;
                int i0 = 0, ni = s, j0 = 0, nj = s;
                if (bx && s >= 4) {
                    const int rb = bx[u], cb = bx[m + v];
                    i0 = rb & 255; ni = rb >> 8; j0 = cb & 255; nj = cb >> 8;
                }
                float2 a0 = make_float2(0.f, 0.f), a1 = make_float2(0.f, 0.f);
                for (int ii = 0; ii < ni; ++ii) {
                    const int kr = u + ((i0 + ii) & smask) * m;
                    const int krm = kr == 0 ? 0 : m1 - kr;
                    for (int jj = 0; jj < nj; ++jj) {
                        const int kc = v + ((j0 + jj) & smask) * n;
                        const bool mir = kc > half;
                        float2 h = H[mir ? krm * hld + (n1 - kc) : kr * hld + kc];
                        h.y = mir ? -h.y : h.y;
                        const float2 f = ps[static_cast<long long>(kr) * n1 + kc];
                        a0 = make_float2(fmaf(h.x, f.x, a0.x), fmaf(h.y, f.x, a0.y));
                        a1 = make_float2(fmaf(h.x, f.y, a1.x), fmaf(h.y, f.y, a1.y));
                    }
                }
                A[rr * ld + v] = a0;
                A[(a.rows + rr) * ld + v] = a1;
            }
            __syncthreads();
            big_fft<N, INV>(A, wstfft::Lines(1, 0, 2 * a.rows, ld, 1), n, tw, id);
            for (int b = 0; b < 2; ++b) {
                const int path = 2 * pr + b;
                if (path >= a.npath) break;
                float2* D = a.dst + (static_cast<long long>(arr) * a.npath + path) * m * n;
                for (int i = threadIdx.x; i < a.rows * n; i += T) {
                    const int rr = i / n, q = i - (i / n) * n;
                    wstdev::stnt(D + (r0 + rr) * n + q, A[(b * a.rows + rr) * ld + q]);
                }
            }
            __syncthreads();
        }
        return;
    }
    __syncthreads();
    wstfft::EpiIdentity id;
    big_fft<N, INV>(A, wstfft::Lines(1, 0, nlines, ld, 1), n, tw, id);

    if (a.mode == kRowHalf) {
        // U1hat rows k1 = r0 + t (0 <= k1 <= m/2) as the natural-order half spectra (hld = n/2 + 1
        // columns, m rows): row k1 directly, row m - k1 (0 < k1 < m/2) from the conjugate mirror
        const int hld = n / 2 + 1, mm = 2 * (a.nrows - 1);
        float2* D = a.dst + static_cast<long long>(arr) * mm * hld;
        for (int i = threadIdx.x; i < nlines * hld; i += T) {
            const int t = i / hld, c = i - (i / hld) * hld;
            const int k1 = r0 + t;
            wstdev::stnt(D + static_cast<long long>(k1) * hld + c, A[t * ld + c]);
            if (k1 > 0 && 2 * k1 < mm) {
                const float2 z = A[t * ld + (c == 0 ? 0 : n - c)];
                wstdev::stnt(D + static_cast<long long>(mm - k1) * hld + c, make_float2(z.x, -z.y));
            }
        }
        return;
    }
    if (a.mode == kRowPad || a.mode == kRowFold1) {
        float2* D = a.dst + static_cast<long long>(arr) * m * n;
        if constexpr (N > 0 && N % 2 == 0) {
            constexpr int H2 = N / 2;   // element pairs per lane: 16-byte streaming stores
            for (int i = threadIdx.x; i < a.rows * H2; i += T) {
                const int rr = i / H2, q = 2 * (i - (i / H2) * H2);
                stnt2(D + (r0 + rr) * n + q, A[rr * ld + q], A[rr * ld + q + 1]);
            }
            return;
        }
        for (int i = threadIdx.x; i < a.rows * n; i += T) {
            const int rr = i / n, q = i - (i / n) * n;
            wstdev::stnt(D + (r0 + rr) * n + q, A[rr * ld + q]);
        }
    }
}

// kColModLpFwd tail: the tile's U columns (.x, |.| * scale) minus their own means, two per complex
// line (column 2c' real, 2c' + 1 imaginary, in column 2c''s slots), forward n-point FFT, Hermitian
// split into the two columns' spectra, rows 0..n/2 stored to colt ((n/2 + 1) x ncols per array).
// Subtracting each column's own mean leaves row 0 ~ 0; kRowHalf restores the global-mean-removed
// row 0 from the column sums (the conditioning of U - mu, which the packed real-row pass applied).
template <int N>
__device__ __forceinline__ void col_spectra(float2* A, const float2* tw, const BigArgs& a, int arr, int c0,
                                            int nc, int n, const float* csum_t) {
    const int ld = n | 1, T = blockDim.x, npair = (nc + 1) / 2;
    const float inv_n = 1.f / static_cast<float>(n);
    __syncthreads();   // column sums in csum_t; every lane done reading .x of the tile
    for (int i = threadIdx.x; i < npair * n; i += T) {
        const int cp = i / n, u = i - (i / n) * n;
        const int ca = 2 * cp, cb = 2 * cp + 1;
        const float re = A[ca * ld + u].x - csum_t[ca] * inv_n;
        const float im = cb < nc ? A[cb * ld + u].x - csum_t[cb] * inv_n : 0.f;
        A[ca * ld + u] = make_float2(re, im);
    }
    __syncthreads();
    wstfft::EpiIdentity id;
    big_fft<N, false>(A, wstfft::Lines(1, 0, npair, 2 * ld, 1), n, tw, id);
    const int hrows = n / 2 + 1;
    float2* D = a.colt + static_cast<long long>(arr) * hrows * a.ncols;
    if constexpr (N > 0) if ((nc & 1) == 0 && (a.ncols & 1) == 0) {
        // both columns of a packed pair from one lane: one 16-byte streaming store
        for (int i = threadIdx.x; i < hrows * (kColTile / 2); i += T) {
            const int k1 = i / (kColTile / 2), cp = i - (i / (kColTile / 2)) * (kColTile / 2);
            if (2 * cp >= nc) continue;
            const float2 z = A[2 * cp * ld + k1];
            const float2 zm = A[2 * cp * ld + (k1 == 0 ? 0 : n - k1)];
            stnt2(D + static_cast<long long>(k1) * a.ncols + c0 + 2 * cp,
                  make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y)),
                  make_float2(0.5f * (z.y + zm.y), -0.5f * (z.x - zm.x)));
        }
        return;
    }
    for (int i = threadIdx.x; i < hrows * kColTile; i += T) {
        const int k1 = i / kColTile, c = i - (i / kColTile) * kColTile;
        if (c >= nc) continue;
        const int cp = c >> 1;
        const float2 z = A[2 * cp * ld + k1];
        const float2 zm = A[2 * cp * ld + (k1 == 0 ? 0 : n - k1)];
        const float2 h = (c & 1) ? make_float2(0.5f * (z.y + zm.y), -0.5f * (z.x - zm.x))
                                 : make_float2(0.5f * (z.x + zm.x), 0.5f * (z.y - zm.y));
        wstdev::stnt(D + static_cast<long long>(k1) * a.ncols + c0 + c, h);
    }
}

// --------------------------------------------------------------------------------------------
// column pass: kColTile columns of one array per workgroup, each column contiguous in LDS
// --------------------------------------------------------------------------------------------
template <int N, bool INV>
__global__ void __launch_bounds__(big_col_threads(N)) k_big_cols(DevParams p, BigArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int n = N > 0 ? N : a.n;
    const int ld = n | 1;
    constexpr int C = kColTile;
    float2* tw = reinterpret_cast<float2*>(smem);
    float2* A = tw + n;
    const int T = blockDim.x;
    const int arr = blockIdx.y;
    const int c0 = blockIdx.x * C;
    const int nc = min(C, a.ncols - c0);
    const float2* gtw = level_tw(p, a.lvl, 0);
    for (int i = threadIdx.x; i < n; i += T) tw[i] = gtw[i];
    if (wstdev::tracing(p, a.tslot)) {
        wstdev::trace_word(p, a.tslot, 0, wstdev::tr_kernel(wstdev::kTkBigCols, 0, 0, N, 0, INV ? 1 : 0));
        wstdev::trace_word(p, a.tslot, 1,
                           wstdev::tr_big(a.mode, 0, 0, 0, a.mode != kColStore && p.oM > 8 ? 1 : 0,
                                          a.mode != kColStore ? a.g_lds : 0, 0));
    }
    float2* src = a.dst + static_cast<long long>(arr) * n * a.ncols;
    // kLoadBatch loads per thread in flight before their LDS stores (a load-store loop waits out
    // the HBM latency once per element: ~2.2 TB/s at c5)
    constexpr int TB = col_tile_batch(N);
    bool wide_done = false;
    if constexpr (N > 0) if ((nc & 1) == 0 && (a.ncols & 1) == 0) {
        // column pairs (2c, 2c + 1) of a row per lane: 16-byte streaming loads, 8 lanes per 128 B
        wide_done = true;
        constexpr int C2 = C / 2;
        constexpr int TB2 = (N * C2 + big_col_threads(N) - 1) / big_col_threads(N);
        const int nc2 = nc / 2;
        for (int i0 = threadIdx.x; i0 < n * C2; i0 += TB2 * T) {
            wst_f4 t[TB2];
#pragma unroll
            for (int k = 0; k < TB2; ++k) {
                const int i = min(i0 + k * T, n * C2 - 1);
                const int u = i / C2, c = min(i - (i / C2) * C2, nc2 - 1);
                t[k] = ldnt2(src + static_cast<long long>(u) * a.ncols + c0 + 2 * c);
            }
#pragma unroll
            for (int k = 0; k < TB2; ++k) {
                const int i = i0 + k * T;
                const int u = i / C2, c = i - (i / C2) * C2;
                if (i < n * C2 && c < nc2) {
                    A[(2 * c) * ld + u] = make_float2(t[k].x, t[k].y);
                    A[(2 * c + 1) * ld + u] = make_float2(t[k].z, t[k].w);
                }
            }
        }
    }
    if (!wide_done)
    for (int i0 = threadIdx.x; i0 < n * C; i0 += TB * T) {
        float2 t[TB];
#pragma unroll
        for (int k = 0; k < TB; ++k) {
            const int i = min(i0 + k * T, n * C - 1);
            const int u = i / C, c = min(i - (i / C) * C, nc - 1);
            t[k] = wstdev::ldnt(src + static_cast<long long>(u) * a.ncols + c0 + c);
        }
#pragma unroll
        for (int k = 0; k < TB; ++k) {
            const int i = i0 + k * T;
            const int u = i / C, c = i - (i / C) * C;
            if (i < n * C && c < nc) A[c * ld + u] = t[k];
        }
    }
    __syncthreads();
    if (a.mode == kColStore) {
        wstfft::EpiIdentity id;
        big_fft<N, INV>(A, wstfft::Lines(1, 0, nc, ld, 1), n, tw, id);
        if (wide_done) {   // column pairs per lane: 16-byte streaming stores
            for (int i = threadIdx.x; i < n * (C / 2); i += T) {
                const int u = i / (C / 2), c = 2 * (i - (i / (C / 2)) * (C / 2));
                if (c < nc) stnt2(src + static_cast<long long>(u) * a.ncols + c0 + c, A[c * ld + u], A[(c + 1) * ld + u]);
            }
            return;
        }
        for (int i = threadIdx.x; i < n * C; i += T) {
            const int u = i / C, c = i - (i / C) * C;
            if (c < nc) wstdev::stnt(src + static_cast<long long>(u) * a.ncols + c0 + c, A[c * ld + u]);
        }
        return;
    }
    // kColModLp / kColModLpFwd: |.| * scale in place (.x), then partials over the rows of each
    // column (and, Fwd, the column spectra of U)
    // kColModLpFwd: this tile's column sums, in the dynamic LDS after the tile and its taps (a
    // static array would leave less than the 160 KiB the launch may request)
    float* csum_t = reinterpret_cast<float*>(A + C * ld) + (a.g_lds ? n * a.oms : 0);
    wstdev::EpiModulus mod{a.scale, 0.f};
    big_fft<N, INV>(A, wstfft::Lines(1, 0, nc, ld, 1), n, tw, mod);
    const int oms = a.oms;
    float* Gl = reinterpret_cast<float*>(A + C * ld);   // n x oms taps after the column tile
    if (a.g_lds)
        for (int i = threadIdx.x; i < n * oms; i += T) Gl[i] = a.gnat[i];
    __syncthreads();
    // the tap reads typed by where the taps are (LDS / global): through one generic pointer they
    // are flat loads, and every wait on them waits for both the LDS and the memory counter
    auto partials = [&](auto G) __attribute__((always_inline)) {
        constexpr int PC = 16;
        if (p.oM <= 8) {
            for (int w = threadIdx.x; w < nc * PC; w += T) {
                const int pc = w & (PC - 1);
                const int c = w / PC;
                const float2* col = A + c * ld;
                float acc[9];
#pragma unroll
                for (int k = 0; k < 9; ++k) acc[k] = 0.f;
                for (int u = pc; u < n; u += PC) {
                    const float mv = col[u].x;
                    const auto g = G + u * oms;
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (k < p.oM) acc[k] = fmaf(g[k], mv, acc[k]);
                    acc[8] += mv;
                }
#pragma unroll
                for (int k = 0; k < 9; ++k) acc[k] = wstdev::group_sum<PC>(acc[k]);
                if (pc == 0) {
                    for (int k = 0; k < p.oM; ++k) a.vpart[(static_cast<long long>(arr) * a.ncols + c0 + c) * oms + k] = acc[k];
                    a.csum[static_cast<long long>(arr) * a.ncols + c0 + c] = acc[8];
                    csum_t[c] = acc[8];
                }
            }
            return;
        }
        // wide output maps: kBigOGroup outputs per round over the column tile held in LDS
        for (int a0 = 0; a0 < p.oM; a0 += kBigOGroup) {
            for (int w = threadIdx.x; w < nc * PC; w += T) {
                const int pc = w & (PC - 1);
                const int c = w / PC;
                const float2* col = A + c * ld;
                float acc[kBigOGroup + 1];
#pragma unroll
                for (int k = 0; k <= kBigOGroup; ++k) acc[k] = 0.f;
                for (int u = pc; u < n; u += PC) {
                    const float mv = col[u].x;
                    const auto g = G + u * oms + a0;
#pragma unroll
                    for (int k = 0; k < kBigOGroup; ++k)
                        if (a0 + k < p.oM) acc[k] = fmaf(g[k], mv, acc[k]);
                    acc[kBigOGroup] += mv;
                }
#pragma unroll
                for (int k = 0; k <= kBigOGroup; ++k) acc[k] = wstdev::group_sum<PC>(acc[k]);
                if (pc == 0) {
                    for (int k = 0; k < kBigOGroup && a0 + k < p.oM; ++k)
                        a.vpart[(static_cast<long long>(arr) * a.ncols + c0 + c) * oms + a0 + k] = acc[k];
                    if (a0 == 0) {
                        a.csum[static_cast<long long>(arr) * a.ncols + c0 + c] = acc[kBigOGroup];
                        csum_t[c] = acc[kBigOGroup];
                    }
                }
            }
        }
    };
    // V[q][a] = sum_p GMnat[p][a] m[p][q] (a < oM) and the column sum: the taps are staged in LDS
    // after the column tile (when they fit), one thread per (column, 16-row chunk) accumulates
    // every output of its rows, then the 16 chunks of a column are shuffle-reduced
    if (a.g_lds)
        partials((wstdev::lcfloat_p)Gl);
    else
        partials((wstdev::gcfloat_p)a.gnat);
    if (a.mode == kColModLpFwd) col_spectra<N>(A, tw, a, arr, c0, nc, n, csum_t);
}

// Size-independent kernels: defined in one object only (wst_staged.hip with WST_BIG_N = 0).
#ifdef WST_BIG_COMMON_KERNELS
// --------------------------------------------------------------------------------------------
// plane sums of the reflect-padded input, kMeanParts partials per plane (the conditioning mean of
// k_prep's FFT input; kRowPad adds the partials in a fixed order)
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBigThreads) k_big_mean(DevParams p, const float* __restrict__ in,
                                                          float* __restrict__ part) {
    __shared__ float red[16];
    const int PM = p.PM, PN = p.PN;
    const int inM = p.pre_pad ? PM : p.M, inN = p.pre_pad ? PN : p.N;
    const float* x = in + static_cast<long long>(blockIdx.x) * inM * inN;
    const int u0 = blockIdx.y * PM / kMeanParts, u1 = (blockIdx.y + 1) * PM / kMeanParts;
    float s = 0.f;
    for (int u = u0; u < u1; ++u) {
        const int su = p.pre_pad ? u : wstdev::reflect_index(u - p.padTop, p.M);
#pragma unroll 4
        for (int v = threadIdx.x; v < PN; v += blockDim.x) {
            const int sv = p.pre_pad ? v : wstdev::reflect_index(v - p.padLeft, p.N);
            s += x[su * inN + sv];
        }
    }
    s = wstdev::block_sum(s, red);
    if (threadIdx.x == 0) part[blockIdx.x * kMeanParts + blockIdx.y] = s;
}

// --------------------------------------------------------------------------------------------
// final low-pass contraction + emit, one workgroup per array
//   kFinalRows: S[a][c] = sum_p G[p][a] T[p][c]   (T = S0 row partials, G = GMnat level 0; n rows)
//   kFinalCols: S[a][c] = sum_q G[q][c] V[q][a]   (V = column partials, G = GNnat level lvl; n columns)
// Coefficient of array `arr`: kind 0 -> k = 0 (plane = arr); 1 -> S1 (arr = plane*L + l1,
// k = 1 + j1 L + l1); 2 -> S2 (arr = plane*npath + l2 for one l1, k = o2_base + (j2-j1-1) L + l2).
// With `mean_out`, the U1 mean (sum of the column sums / (n n_other)) of the array is stored too.
// --------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) k_big_final(DevParams p, int fmode, int kind, int n, int n_other,
                                                  int oms, const float* __restrict__ part,
                                                  const float* __restrict__ G,
                                                  const float* __restrict__ csum,
                                                  float* __restrict__ mean_out, int L, int j1,
                                                  int l1, int j2, int npath, long long img0,
                                                  float* __restrict__ out, int pooled) {
    extern __shared__ float S[];   // oM x oN (dynamic)
    __shared__ float red[16];
    const int arr = blockIdx.x;
    if (l1 < 0) {
        // every theta1 of a staged order-2 level in one launch: l1 = blockIdx.y, whose partials
        // follow the previous theta1's (gridDim.x arrays each)
        l1 = blockIdx.y;
        part += static_cast<long long>(blockIdx.y) * gridDim.x * n * oms;
    }
    const float* P = part + static_cast<long long>(arr) * n * oms;
    const int nout = p.oM * p.oN;
    // KS lanes per output split the contraction (shuffle sum): 16 outputs (4 x 4) use every lane
    const int KS = nout <= 16 ? 4 : nout <= 32 ? 2 : 1;
    for (int w = threadIdx.x; w < nout * KS; w += blockDim.x) {
        const int o = w / KS, ks = w - o * KS;
        const int ra = o / p.oN, c = o - (o / p.oN) * p.oN;
        float acc = 0.f;
        // unrolled so the loads of eight steps issue before the first use (a rolled loop waited out
        // the memory latency once per step: ~27 us per launch at c5); same order of accumulation
        if (fmode == kFinalRows) {
#pragma unroll 8
            for (int k = ks; k < n; k += KS) acc = fmaf(G[k * oms + ra], P[k * oms + c], acc);
        } else {
#pragma unroll 8
            for (int k = ks; k < n; k += KS) acc = fmaf(G[k * oms + c], P[k * oms + ra], acc);
        }
        if (KS == 4) acc = wstdev::group_sum<4>(acc);
        else if (KS == 2) acc = wstdev::group_sum<2>(acc);
        if (ks == 0) S[o] = acc;
    }
    if (mean_out) {
        float s = 0.f;
        for (int q = threadIdx.x; q < n; q += blockDim.x) s += csum[static_cast<long long>(arr) * n + q];
        s = wstdev::block_sum(s, red);
        if (threadIdx.x == 0) mean_out[arr] = s / (static_cast<float>(n) * static_cast<float>(n_other));
    }
    __syncthreads();
    long long plane;
    int k;
    if (kind == 0) {
        plane = arr;
        k = 0;
    } else if (kind == 1) {
        plane = arr / L;
        k = 1 + j1 * L + (arr - (arr / L) * L);
    } else {
        plane = arr / npath;
        k = p.o2_base[j1 * L + l1] + (j2 - j1 - 1) * L + (arr - (arr / npath) * npath);
    }
    wstdev::emit(S, 1, k, img0 + plane, p.K, p.oM, p.oN, out, pooled);
}

#endif  // WST_BIG_COMMON_KERNELS

}  // namespace wstbig
