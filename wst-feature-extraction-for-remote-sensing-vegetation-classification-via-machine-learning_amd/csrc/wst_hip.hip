// MI355X (gfx950) wavelet scattering transform: kernels + C ABI (include/wst_hip.h).
//
// Replaces kymatio 0.3.0's scattering2d cascade as reached from the
// reference at src/training/train_and_save_model.py:359-376 and src/inference/inference.py:242-257.
//
// Pipeline per chunk of planes (one plane = one channel of one patch):
//   k_prep     (1 workgroup / plane):  reflect-pad gather -> S0 (separable spatial low-pass) ->
//                                       mean-centred forward 2-D DFT -> Xhat (HBM workspace)
//   k_order12  (1 workgroup / (plane, theta1), one launch per j1):
//                                       fold(Xhat * psi0) -> inverse DFT -> |.| -> S1 low-pass;
//                                       forward DFT of U1 kept in LDS -> for every (j2 > j1, theta2)
//                                       fold(U1hat * psi) -> inverse DFT -> |.| -> S2 low-pass.
// All per-path intermediates stay in LDS; HBM sees the input plane, Xhat (written once, re-read
// by the L workgroups of the plane on the same XCD) and the K output coefficients.
//
// Exact rewrites used (identities of the kymatio algorithm, not approximations):
//   * sub(Y, k) then ifft at n/k   ==  ifft at n then spatial decimation by k;
//   * the phi low-pass + subsample + ifft + unpad == a separable spatial filter evaluated only at
//     the (Mo x No) kept points (phi_hat levels are outer products of 1-D masked crops);
//   * constants are removed before the psi paths (psi_hat(0) ~ 1e-16, reflect padding preserves
//     constants), which conditions the fp32 band-pass content.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "fft_lds.h"
#include "filter_bank.h"
#include "wst_hip.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define WST_HIP_CHECK(expr)                                                                   \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(WST_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(e_)); \
    } while (0)

constexpr int kMaxLds = 160 * 1024;
constexpr int kMaxO = 8;  // outputs per thread per DFT chunk (register tile)

// Kernel-side description of a plan (POD, passed by value).
struct DevParams {
    int M, N, PM, PN, J, L, max_order, pre_pad, K;
    int mM, mN, oM, oN, padTop, padLeft;
    int tw_total, lp_total;       // element counts of the twiddle / low-pass pools
    int dbg_skip;                 // timing-ablation mask (env WST_DEBUG_SKIP; 0 in production)
    const float* psi;             // concatenated psi Fourier levels (fp32)
    const long long* psi_off;     // [(j*L + l)*J + r]
    const float* lp;              // concatenated spatial low-pass taps hM[r], hN[r]
    const int* lp_off;            // [2r] -> hM[r], [2r+1] -> hN[r]
    const float2* tw;             // concatenated twiddle tables exp(-2 pi i k / n)
    const int* tw_off;            // [2r] -> n = PM>>r, [2r+1] -> n = PN>>r, r in [0, J]
    const int* o2_base;           // first order-2 coefficient of each n1 = j1*L + l1
    const int* perm;              // digit-reversal maps: physical position -> logical index
    const int* perm_off;          // [2r] -> size PM>>r, [2r+1] -> size PN>>r, r in [0, J]
    int perm_total;
    const float4* psi4;           // order-2 filters, 4 consecutive l2 interleaved per bin
    const long long* psi4_off;    // [(j2*J + r)*ceil(L/4) + q] -> level r of l2 in [4q, 4q+4)
};

// ------------------------------------------------------------------------------------------
// device helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int reflect_index(int i, int n) {
    // numpy.pad(mode='reflect') for any pad width: even periodic extension, period 2(n-1)
    if (n == 1) return 0;
    const int period = 2 * (n - 1);
    int t = i % period;
    if (t < 0) t += period;
    return t < n ? t : period - t;
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

// |z| * scale stored as a real value; optionally accumulates the per-thread sum (for means)
struct EpiModulus {
    float scale;
    float sum;
    __device__ float2 operator()(float2 z) {
        const float m = __builtin_amdgcn_sqrtf(fmaf(z.x, z.x, z.y * z.y)) * scale;   // v_sqrt_f32
        sum += m;
        return make_float2(m, 0.f);
    }
};

// Generic O(n) DFT along lines (fallback for sizes without a compiled FFT).  Lines are processed
// in chunks of whole lines that fit the register tile: read phase -> barrier -> write phase.
template <class Epi>
__device__ __forceinline__ void lds_dft_lines_generic(float2* base, const wstfft::Lines g, int n, const float2* tw,
                                      bool inverse, Epi& epi) {
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

// n-point transforms along lines.  FAM > 0: compiled FFTs for n = FAM * 2^k <= kMaxFamilyN;
// FAM == 0 or any other n: generic DFT.
// n-point transforms along lines.  FAM > 0: the compiled FFTs n = FAM * 2^k <= MAXN (a plan's
// level sizes always belong to its family, so no fallback is compiled into these kernels);
// FAM == 0: generic DFT for any n.
// Line-transform orders: natural -> natural (transposing store rounds), natural -> digit-reversed
// (in place, F_DR) and digit-reversed -> natural (in place, G).
enum { kNat = 0, kDR = 1, kRD = 2 };

template <int FAM, int K, int MAXN, int KIND, bool INV, class Epi>
__device__ __forceinline__ void family_fft(float2* base, const wstfft::Lines& g, int n,
                                           const float2* tw, Epi& epi) {
    constexpr int NN = FAM << K;
    if constexpr (NN <= MAXN && NN <= wstfft::kMaxFamilyN) {
        if constexpr (NN >= 2) {
            if (n == NN) {
                if constexpr (KIND == kNat) wstfft::fft_lines<NN, INV>(base, g, tw, epi);
                else if constexpr (KIND == kDR) wstfft::fft_lines_dr<NN, INV>(base, g, tw, epi);
                else wstfft::fft_lines_rd<NN, INV>(base, g, tw, epi);
                return;
            }
        }
        family_fft<FAM, K + 1, MAXN, KIND, INV>(base, g, n, tw, epi);
    }
}

// n-point transforms along lines.  FAM > 0: the compiled FFTs n = FAM * 2^k <= MAXN (a plan's
// level sizes always belong to its family, so no fallback is compiled into these kernels);
// FAM == 0: generic DFT (natural order for every KIND; the plan's permutation maps are identity).
template <int FAM, int MAXN, int KIND, bool INV, class Epi>
__device__ __forceinline__ void lds_fft_lines(float2* base, const wstfft::Lines g, int n, const float2* tw, Epi& epi) {
    if constexpr (FAM > 0)
        family_fft<FAM, 0, MAXN, KIND, INV>(base, g, n, tw, epi);
    else
        lds_dft_lines_generic(base, g, n, tw, INV, epi);
}

// 2-D transform of nb (rows x cols) arrays with row stride ld (odd), spaced bs apart; `epi` is
// applied to the final (column-pass) stores.  FM / FN: size families of rows / cols; MAXN caps
// the compiled sizes (smaller caps -> fewer registers for the small-level kernels).
template <int FM, int FN, int MAXN, int KIND, bool INV, class Epi>
__device__ __forceinline__ void lds_fft2(float2* buf, int nb, int bs, int rows, int cols, int ld, const float2* twR,
                         const float2* twC, Epi& epi) {
    wstfft::EpiIdentity id;
    lds_fft_lines<FN, MAXN, KIND, INV>(buf, wstfft::Lines{nb, bs, rows, ld, 1}, cols, twC, id);
    lds_fft_lines<FM, MAXN, KIND, INV>(buf, wstfft::Lines{nb, bs, cols, 1, ld}, rows, twR, epi);
}

// Separable phi low-pass evaluated at the kept output points (unpad folded in):
//   S[b][a][c] = sum_p hM[s(a+1) - p] * sum_q hN[s(c+1) - q] * U[b][p][q]   (indices mod n)
// hM2 / hN2 are the taps stored twice (length 2n) so s(c+1) + n - q never wraps.  U real (.x),
// row stride ld; permM / permN (nullable): logical row / column index of each physical one.
// Step 1: QC consecutive lanes split one row's q range and shuffle-reduce OW output columns;
// step 2: PC consecutive lanes split the p range of one output.  tmp: nb*rows*oN floats (logical
// rows), S: nb*oM*oN floats.  Ends with a barrier.
template <int OW, int QC, int PC>
__device__ __forceinline__ void lds_lowpass_t(const float2* U, int nb, int bs, int rows, int cols,
                                              int ld, const float* hM2, const float* hN2,
                                              const int* permM, const int* permN, int s, int oM,
                                              int oN, float* tmp, float* S) {
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
        const float2* row = U + b * bs + p * ld;
        const float* h0 = hN2 + cols + s * (c0 + 1);   // tap index s(c+1) + cols - q
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
        for (int off = QC / 2; off >= 1; off >>= 1)
#pragma unroll
            for (int c = 0; c < OW; ++c) acc[c] += __shfl_xor(acc[c], off, 64);
        if (qc == 0) {
            const int pl = permM ? permM[p] : p;   // store at the logical row
#pragma unroll
            for (int c = 0; c < OW; ++c)
                if (c0 + c < oN) tmp[(b * rows + pl) * oN + c0 + c] = acc[c];
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
        const float* t = tmp + b * rows * oN + c;
        const float* h = hM2 + rows + s * (a + 1);
        float acc = 0.f;
#pragma unroll 2
        for (int p = pc; p < rows; p += PC) acc = fmaf(h[-p], t[p * oN], acc);
#pragma unroll
        for (int off = PC / 2; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (pc == 0) S[o] = acc;
    }
    __syncthreads();
}

__device__ __forceinline__ void lds_lowpass(const float2* U, int nb, int bs, int rows, int cols,
                                            int ld, const float* hM2, const float* hN2,
                                            const int* permM, const int* permN, int s, int oM,
                                            int oN, float* tmp, float* S) {
    if (oN <= 4)
        lds_lowpass_t<4, 8, 16>(U, nb, bs, rows, cols, ld, hM2, hN2, permM, permN, s, oM, oN, tmp, S);
    else
        lds_lowpass_t<8, 8, 16>(U, nb, bs, rows, cols, ld, hM2, hN2, permM, permN, s, oM, oN, tmp, S);
}

// Write nb coefficient maps (S: nb x oM x oN) of plane `img`, coefficient k0 + b*kstride.
// pooled: out[img][k] = mean, out[img][K + k] = population std.
__device__ __forceinline__ void emit(const float* S, int nb, int k0, int kstride, long long img, int K, int oM,
                     int oN, float* out, int pooled) {
    const int npix = oM * oN;
    if (!pooled) {
        const int tot = nb * npix;
        for (int o = threadIdx.x; o < tot; o += blockDim.x) {
            const int b = o / npix;
            const int k = k0 + b * kstride;
            out[(img * K + k) * npix + (o - b * npix)] = S[o];
        }
    } else {
        for (int b = threadIdx.x; b < nb; b += blockDim.x) {
            const float* v = S + b * npix;
            float m = 0.f;
            for (int i = 0; i < npix; ++i) m += v[i];
            m /= npix;
            float q = 0.f;
            for (int i = 0; i < npix; ++i) {
                const float d = v[i] - m;
                q = fmaf(d, d, q);
            }
            const int k = k0 + b * kstride;
            out[img * 2 * K + k] = m;
            out[img * 2 * K + K + k] = sqrtf(q / npix);
        }
    }
}

// Copy the twiddle and low-pass pools into LDS.
__device__ __forceinline__ void load_tables(const DevParams& p, float2* tw_l, float* lp_l) {
    for (int i = threadIdx.x; i < p.tw_total; i += blockDim.x) tw_l[i] = p.tw[i];
    for (int i = threadIdx.x; i < p.lp_total; i += blockDim.x) lp_l[i] = p.lp[i];
}

// Row stride of LDS arrays: odd (conflict-free row-wise b64 access); WST_LD_EVEN for A/B tests.
#ifdef WST_LD_EVEN
__host__ __device__ inline int odd_ld(int n) { return n; }
#else
__host__ __device__ inline int odd_ld(int n) { return n | 1; }
#endif

// Order-2 fold of one group of (up to) 4 paths:
//   B_b[u][v] = sum_{i,j < s} A[u + i nM2][v + j nN2] * psi_b[u + i nM2][v + j nN2]
// A: U1hat (stride ld1), psi4: the 4 paths' filters interleaved per bin (float4, dense nN1 rows).
// S > 0: compile-time alias count (fully unrolled); S == 0: runtime s (large s = tiny outputs).
template <int S>
__device__ __forceinline__ void fold4(const float2* A, int ld1, int nN1,
                                      const float4* __restrict__ psi4, float2* B, int slot, int ld2,
                                      int nM2, int nN2, int g, int s_rt) {
    const int s = (S > 0) ? S : s_rt;
    const int items = nM2 * nN2;
    for (int it = threadIdx.x; it < items; it += blockDim.x) {
        const int u = it / nN2, v = it - (it / nN2) * nN2;
        float2 acc[4];
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[b] = make_float2(0.f, 0.f);
#pragma unroll(S == 2 ? 2 : 1)
        for (int i = 0; i < s; ++i) {
            const int su = u + i * nM2;
            const float2* arow = A + su * ld1 + v;
            const float4* frow = psi4 + su * nN1 + v;
#pragma unroll(S > 0 ? S : 2)
            for (int j = 0; j < s; ++j) {
                const float2 a = arow[j * nN2];
                const float4 f = frow[j * nN2];
                acc[0] = make_float2(fmaf(a.x, f.x, acc[0].x), fmaf(a.y, f.x, acc[0].y));
                acc[1] = make_float2(fmaf(a.x, f.y, acc[1].x), fmaf(a.y, f.y, acc[1].y));
                acc[2] = make_float2(fmaf(a.x, f.z, acc[2].x), fmaf(a.y, f.z, acc[2].y));
                acc[3] = make_float2(fmaf(a.x, f.w, acc[3].x), fmaf(a.y, f.w, acc[3].y));
            }
        }
        float2* dst = B + u * ld2 + v;
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (b < g) dst[b * slot] = acc[b];
    }
}

__device__ __forceinline__ void fold4_any(int s2, const float2* A, int ld1, int nN1,
                                          const float4* psi4, float2* B, int slot, int ld2,
                                          int nM2, int nN2, int g) {
    if (s2 == 2) fold4<2>(A, ld1, nN1, psi4, B, slot, ld2, nM2, nN2, g, 2);
    else if (s2 == 4) fold4<4>(A, ld1, nN1, psi4, B, slot, ld2, nM2, nN2, g, 4);
    else fold4<0>(A, ld1, nN1, psi4, B, slot, ld2, nM2, nN2, g, s2);
}

// Order-1 fold from HBM/L2: A[u][v] = sum_{i,j < s} X[u + i nM1][v + j nN1] * psi0[...]
// S > 0: compile-time alias count; S == 0: runtime s.  U items per thread keep loads in flight.
template <int S>
__device__ __forceinline__ void fold1(const float2* __restrict__ X, const float* __restrict__ psi0,
                                      int PN, float2* A, int ld1, int nM1, int nN1, int s_rt) {
    const int s = (S > 0) ? S : s_rt;
    const int items = nM1 * nN1;
    const int T = blockDim.x;
    constexpr int U = (S == 1) ? 4 : (S == 2 ? 2 : 1);
    for (int it0 = threadIdx.x; it0 < items; it0 += U * T) {
        float2 acc[U];
        int dst[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int it = it0 + k * T;
            acc[k] = make_float2(0.f, 0.f);
            dst[k] = -1;
            if (it < items) {
                const int u = it / nN1, v = it - (it / nN1) * nN1;
                dst[k] = u * ld1 + v;
#pragma unroll(S > 0 ? S : 1)
                for (int i = 0; i < s; ++i) {
#pragma unroll(S > 0 ? S : 4)
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

__device__ __forceinline__ void fold1_any(int s1, const float2* X, const float* psi0, int PN,
                                          float2* A, int ld1, int nM1, int nN1) {
    if (s1 == 1) fold1<1>(X, psi0, PN, A, ld1, nM1, nN1, 1);
    else if (s1 == 2) fold1<2>(X, psi0, PN, A, ld1, nM1, nN1, 2);
    else if (s1 == 4) fold1<4>(X, psi0, PN, A, ld1, nM1, nN1, 4);
    else fold1<0>(X, psi0, PN, A, ld1, nM1, nN1, s1);
}

// ------------------------------------------------------------------------------------------
// k_prep: one workgroup per plane
// ------------------------------------------------------------------------------------------
template <int FM, int FN>
__global__ void __launch_bounds__(512) k_prep(DevParams p, const float* __restrict__ in,
                                              long long img0, float2* __restrict__ xhat,
                                              float* __restrict__ out, int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int PM = p.PM, PN = p.PN, n = PM * PN, ld = odd_ld(PN);
    float2* A = reinterpret_cast<float2*>(smem);
    float2* tw_l = A + PM * ld;
    float* lp_l = reinterpret_cast<float*>(tw_l + p.tw_total);
    float* tmp = lp_l + p.lp_total;                 // PM * oN
    float* S = tmp + PM * p.oN;                     // oM * oN
    float* red = S + p.oM * p.oN;                   // 16

    const long long local = blockIdx.x;
    const long long img = img0 + local;
    load_tables(p, tw_l, lp_l);
    const int inM = p.pre_pad ? PM : p.M, inN = p.pre_pad ? PN : p.N;
    const float* x = in + local * inM * inN;
    float part = 0.f;
    for (int o = threadIdx.x; o < n; o += blockDim.x) {
        const int u = o / PN, v = o - (o / PN) * PN;
        int su, sv;
        if (p.pre_pad) {
            su = u;
            sv = v;
        } else {
            su = reflect_index(u - p.padTop, p.M);
            sv = reflect_index(v - p.padLeft, p.N);
        }
        const float val = x[su * inN + sv];
        A[u * ld + v] = make_float2(val, 0.f);
        part += val;
    }
    const float mean = block_sum(part, red) / n;  // contains the barrier after the gather

    // S0: low-pass at level 0, decimation 2^J
    lds_lowpass(A, 1, 0, PM, PN, ld, lp_l + p.lp_off[0], lp_l + p.lp_off[1], nullptr, nullptr,
                1 << p.J, p.oM, p.oN, tmp, S);
    emit(S, 1, 0, 1, img, p.K, p.oM, p.oN, out, pooled);

    // mean-centred forward DFT for the band-pass paths
    for (int o = threadIdx.x; o < n; o += blockDim.x) {
        const int u = o / PN, v = o - (o / PN) * PN;
        A[u * ld + v].x -= mean;
    }
    __syncthreads();
    wstfft::EpiIdentity id;
    lds_fft2<FM, FN, wstfft::kMaxFamilyN, kNat, false>(A, 1, 0, PM, PN, ld, tw_l + p.tw_off[0],
                                                       tw_l + p.tw_off[1], id);
    float2* dst = xhat + local * n;
    for (int o = threadIdx.x; o < n; o += blockDim.x) {
        const int u = o / PN, v = o - (o / PN) * PN;
        dst[o] = A[u * ld + v];
    }
}

// ------------------------------------------------------------------------------------------
// k_order12: one workgroup per (plane, theta1) at fixed j1
// ------------------------------------------------------------------------------------------
template <int FM, int FN, int MAXN>
__global__ void __launch_bounds__(1024) k_order12(DevParams p, int j1, int G, int tmpN, int nimg,
                                                 long long img0, const float2* __restrict__ xhat,
                                                 float* __restrict__ out, int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int J = p.J, L = p.L;
    // XCD-aware decode: blocks b and b+8 share an XCD; give each XCD a contiguous range of
    // (plane, theta1) items so a plane's L workgroups re-read its Xhat from one L2.
    const int total = nimg * L;
    int item = blockIdx.x;
    if ((total & 7) == 0) item = (blockIdx.x & 7) * (total >> 3) + (blockIdx.x >> 3);
    const int local = item / L;
    const int l1 = item - local * L;
    const long long img = img0 + local;

    const int PM = p.PM, PN = p.PN;
    const int nM1 = PM >> j1, nN1 = PN >> j1, n1 = nM1 * nN1, ld1 = odd_ld(nN1);
    const bool do2 = (p.max_order >= 2) && (j1 < J - 1);
    const int slot = do2 ? (nM1 >> 1) * odd_ld(nN1 >> 1) : 0;

    float2* A = reinterpret_cast<float2*>(smem);
    float2* B = A + nM1 * ld1;
    float2* tw_l = B + G * slot;
    float* lp_l = reinterpret_cast<float*>(tw_l + p.tw_total);
    int* perm_l = reinterpret_cast<int*>(lp_l + p.lp_total);
    float* tmp = reinterpret_cast<float*>(perm_l + p.perm_total);   // tmpN floats (low-pass scratch)
    float* S = tmp + tmpN;                            // <= max(G, L) * oM * oN
    float* red = S + max(G, L) * p.oM * p.oN;         // 16

    load_tables(p, tw_l, lp_l);
    for (int i = threadIdx.x; i < p.perm_total; i += blockDim.x) perm_l[i] = p.perm[i];
    const int dbg = p.dbg_skip;

    // 1. fold_{2^j1}(Xhat * psi0_{j1,l1}) straight from HBM/L2
    const float* psi0 = p.psi + p.psi_off[(j1 * L + l1) * J + 0];
    const float2* X = xhat + static_cast<long long>(local) * PM * PN;
    if (!(dbg & 128)) fold1_any(1 << j1, X, psi0, PN, A, ld1, nM1, nN1);
    __syncthreads();

    // 2. U1 = |ifft(.)| fused into the last FFT pass; normalisation of fold-mean + ifft = 1/(PM PN)
    EpiModulus mod1{1.f / (static_cast<float>(PM) * static_cast<float>(PN)), 0.f};
    if (!(dbg & 1))
        lds_fft2<FM, FN, MAXN, kDR, true>(A, 1, 0, nM1, nN1, ld1, tw_l + p.tw_off[2 * j1],
                                          tw_l + p.tw_off[2 * j1 + 1], mod1);
    const float mean1 = block_sum(mod1.sum, red) / n1;

    // 3. S1 at level j1, decimation 2^(J-j1)
    const int n1idx = j1 * L + l1;
    if (!(dbg & 2)) {
        lds_lowpass(A, 1, 0, nM1, nN1, ld1, lp_l + p.lp_off[2 * j1], lp_l + p.lp_off[2 * j1 + 1],
                    perm_l + p.perm_off[2 * j1], perm_l + p.perm_off[2 * j1 + 1], 1 << (J - j1),
                    p.oM, p.oN, tmp, S);
        emit(S, 1, 1 + n1idx, 1, img, p.K, p.oM, p.oN, out, pooled);
    }
    if (!do2) return;

    // 4. U1hat = fft(U1 - mean) kept in LDS
    for (int u = threadIdx.x / nN1, v = threadIdx.x % nN1, du = blockDim.x / nN1,
             dv = blockDim.x % nN1; u < nM1;) {
        A[u * ld1 + v].x -= mean1;
        u += du;
        v += dv;
        if (v >= nN1) { v -= nN1; ++u; }
    }
    __syncthreads();
    wstfft::EpiIdentity id;
    if (!(dbg & 4))
        lds_fft2<FM, FN, MAXN, kRD, false>(A, 1, 0, nM1, nN1, ld1, tw_l + p.tw_off[2 * j1],
                                           tw_l + p.tw_off[2 * j1 + 1], id);

    const int kbase = p.o2_base[n1idx];
    const int nq = (L + 3) >> 2;
    const int bcap = G * slot;   // complex capacity of the B region
    for (int j2 = j1 + 1; j2 < J; ++j2) {
        const int nM2 = PM >> j2, nN2 = PN >> j2, ld2 = odd_ld(nN2);
        const int pslot = nM2 * ld2;                   // one path's array at this level
        const int s2 = 1 << (j2 - j1);
        int qpb = bcap / (4 * pslot);                  // 4-groups per batch
        qpb = max(1, min(qpb, nq));
        for (int q0 = 0; q0 < nq; q0 += qpb) {
            const int nqb = min(qpb, nq - q0);
            const int npath = min(4 * nqb, L - 4 * q0);
            // 5. fold_{2^(j2-j1)}(U1hat * psi^{j1}_{j2, l2}) for every path of the batch
            if (!(dbg & 8))
                for (int qq = 0; qq < nqb; ++qq) {
                    const int q = q0 + qq;
                    const float4* ps4 = p.psi4 + p.psi4_off[(j2 * J + j1) * nq + q];
                    fold4_any(s2, A, ld1, nN1, ps4, B + qq * 4 * pslot, pslot, ld2, nM2, nN2,
                              min(4, L - 4 * q));
                }
            __syncthreads();
            // 6. U2 = |ifft(.)| (modulus fused), scale 1/(nM1 nN1)
            EpiModulus mod2{1.f / static_cast<float>(n1), 0.f};
            if (!(dbg & 16))
                lds_fft2<FM, FN, MAXN, kDR, true>(B, npath, pslot, nM2, nN2, ld2,
                                                  tw_l + p.tw_off[2 * j2], tw_l + p.tw_off[2 * j2 + 1],
                                                  mod2);
            // 7. S2 at level j2, decimation 2^(J-j2)
            if (!(dbg & 64)) {
                lds_lowpass(B, npath, pslot, nM2, nN2, ld2, lp_l + p.lp_off[2 * j2],
                            lp_l + p.lp_off[2 * j2 + 1], perm_l + p.perm_off[2 * j2],
                            perm_l + p.perm_off[2 * j2 + 1], 1 << (J - j2), p.oM, p.oN, tmp, S);
                emit(S, npath, kbase + (j2 - j1 - 1) * L + 4 * q0, 1, img, p.K, p.oM, p.oN, out,
                     pooled);
            }
            __syncthreads();
        }
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// size-family instantiations
// ------------------------------------------------------------------------------------------
#define WST_FAMILY_PAIRS(X) X(0, 0) X(1, 1) X(3, 3) X(5, 5) X(9, 9) X(17, 17) X(3, 1) X(1, 3)

namespace {

int odd_part(int n) {
    while (n > 0 && (n % 2) == 0) n /= 2;
    return n;
}
int family_of(int P) {
    const int o = odd_part(P);
    const bool compiled = (o == 1 || o == 3 || o == 5 || o == 9 || o == 17);
    return (compiled && P <= wstfft::kMaxFamilyN) ? o : 0;
}
bool pair_compiled(int fm, int fn) {
#define WST_PAIR_EQ(A, B) if (fm == A && fn == B) return true;
    WST_FAMILY_PAIRS(WST_PAIR_EQ)
#undef WST_PAIR_EQ
    return false;
}
// size caps of the k_order12 instantiations (largest FFT a launch may need = PM>>j1, PN>>j1)
#define WST_CAPS(Y, A, B) Y(A, B, 12) Y(A, B, 24) Y(A, B, 48) Y(A, B, 136)
int cap_for(int n) { return n <= 12 ? 12 : n <= 24 ? 24 : n <= 48 ? 48 : 136; }

int set_lds_attributes() {
#define WST_O12_ATTR(A, B, C)                                                                    \
    WST_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_order12<A, B, C>),        \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds));
#define WST_PAIR_ATTR(A, B)                                                                      \
    WST_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_prep<A, B>),              \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLds));    \
    WST_CAPS(WST_O12_ATTR, A, B)
    WST_FAMILY_PAIRS(WST_PAIR_ATTR)
#undef WST_PAIR_ATTR
#undef WST_O12_ATTR
    return WST_OK;
}
void launch_prep(int fm, int fn, dim3 grid, dim3 block, size_t lds, hipStream_t st,
                 const DevParams& dp, const float* in, long long img0, float2* xhat, float* out,
                 int pooled) {
#define WST_PAIR_PREP(A, B)                                                                      \
    if (fm == A && fn == B) {                                                                    \
        hipLaunchKernelGGL((k_prep<A, B>), grid, block, lds, st, dp, in, img0, xhat, out, pooled); \
        return;                                                                                  \
    }
    WST_FAMILY_PAIRS(WST_PAIR_PREP)
#undef WST_PAIR_PREP
}
void launch_order12(int fm, int fn, int cap, dim3 grid, dim3 block, size_t lds, hipStream_t st,
                    const DevParams& dp, int j1, int G, int tmpN, int nimg, long long img0,
                    const float2* xhat, float* out, int pooled) {
#define WST_O12_LAUNCH(A, B, C)                                                                  \
    if (fm == A && fn == B && cap == C) {                                                        \
        hipLaunchKernelGGL((k_order12<A, B, C>), grid, block, lds, st, dp, j1, G, tmpN, nimg,     \
                           img0, xhat, out, pooled);                                             \
        return;                                                                                  \
    }
#define WST_PAIR_O12(A, B) WST_CAPS(WST_O12_LAUNCH, A, B)
    WST_FAMILY_PAIRS(WST_PAIR_O12)
#undef WST_PAIR_O12
#undef WST_O12_LAUNCH
}

}  // namespace

// ------------------------------------------------------------------------------------------
// plan
// ------------------------------------------------------------------------------------------
struct wst_plan {
    wst::Geometry g;
    int device = 0;
    DevParams dp{};
    // device allocations
    float* d_psi = nullptr;
    long long* d_psi_off = nullptr;
    float* d_lp = nullptr;
    float4* d_psi4 = nullptr;
    long long* d_psi4_off = nullptr;
    int* d_lp_off = nullptr;
    float2* d_tw = nullptr;
    int* d_tw_off = nullptr;
    int* d_o2 = nullptr;
    int* d_perm = nullptr;
    int* d_perm_off = nullptr;
    // launch geometry
    int fam_m = 0, fam_n = 0;   // FFT size families (odd part of PM / PN), 0 = generic DFT
    int prep_threads = 256;
    size_t prep_lds = 0;
    std::vector<int> k1_threads, k1_G, k1_tmpN, k1_cap;
    std::vector<size_t> k1_lds;
    // internal workspace (used when the caller passes none)
    mutable std::mutex ws_mu;
    mutable void* ws = nullptr;
    mutable size_t ws_bytes = 0;
    std::vector<int> lp_off_h, tw_off_h;
};

namespace {

void free_plan(wst_plan* p) {
    if (!p) return;
    (void)hipFree(p->d_psi);
    (void)hipFree(p->d_psi_off);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_lp_off);
    (void)hipFree(p->d_tw);
    (void)hipFree(p->d_tw_off);
    (void)hipFree(p->d_o2);
    (void)hipFree(p->d_perm);
    (void)hipFree(p->d_perm_off);
    (void)hipFree(p->d_psi4);
    (void)hipFree(p->d_psi4_off);
    if (p->ws) (void)hipFree(p->ws);
    delete p;
}

template <typename T>
int upload(T** dst, const std::vector<T>& src) {
    const size_t bytes = std::max<size_t>(1, src.size()) * sizeof(T);
    WST_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dst), bytes));
    if (!src.empty()) WST_HIP_CHECK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return WST_OK;
}

size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

}  // namespace

extern "C" {

int wst_abi_version(void) { return WST_ABI_VERSION; }

const char* wst_last_error(void) { return g_last_error.c_str(); }

int wst_plan_create(int M, int N, int J, int L, int max_order, int pre_pad, wst_plan** out) {
    if (!out) return fail(WST_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (J < 1) return fail(WST_ERR_INVALID, "J must be >= 1 (kymatio needs phi level 0)");
    wst::Geometry g;
    std::string err;
    if (!wst::make_geometry(M, N, J, L, max_order, g, err)) return fail(WST_ERR_INVALID, err);
    wst::FilterBank fb;
    try {
        fb = wst::build_filter_bank(g);
    } catch (const std::exception& e) {
        return fail(WST_ERR_UNSUPPORTED, e.what());
    }

    std::unique_ptr<wst_plan, void (*)(wst_plan*)> plan(new (std::nothrow) wst_plan(), free_plan);
    if (!plan) return fail(WST_ERR_NOMEM, "host allocation failed");
    plan->g = g;
    WST_HIP_CHECK(hipGetDevice(&plan->device));

    plan->fam_m = family_of(g.PM);
    plan->fam_n = family_of(g.PN);
    if (!pair_compiled(plan->fam_m, plan->fam_n)) plan->fam_m = plan->fam_n = 0;
    // digit-reversal maps of k_order12's in-place transforms (identity for the generic DFT)
    std::vector<int> perm;
    std::vector<int> perm_off(2 * static_cast<size_t>(J + 1));
    for (int r = 0; r <= J; ++r)
        for (int d = 0; d < 2; ++d) {
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            const bool compiled = (d == 0 ? plan->fam_m : plan->fam_n) > 0;
            perm_off[2 * r + d] = static_cast<int>(perm.size());
            for (int pos = 0; pos < n; ++pos)
                perm.push_back(compiled ? wstfft::dr_logical_host(n, pos) : pos);
        }

    // --- flatten filters ---
    std::vector<float> psi;
    std::vector<long long> psi_off(static_cast<size_t>(J) * L * J, -1);
    for (int j = 0; j < J; ++j)
        for (int l = 0; l < L; ++l) {
            const auto& lev = fb.psi[static_cast<size_t>(j) * L + l];
            for (int r = 0; r < static_cast<int>(lev.size()); ++r) {
                psi_off[(static_cast<size_t>(j) * L + l) * J + r] = static_cast<long long>(psi.size());
                for (double v : lev[r]) psi.push_back(static_cast<float>(v));
            }
        }
    std::vector<float> lp;
    std::vector<int> lp_off(2 * static_cast<size_t>(J));
    for (int r = 0; r < J; ++r) {  // taps stored twice so kernels index s(c+1) + n - q unwrapped
        lp_off[2 * r] = static_cast<int>(lp.size());
        for (int rep = 0; rep < 2; ++rep)
            for (double v : fb.hM[r]) lp.push_back(static_cast<float>(v));
        lp_off[2 * r + 1] = static_cast<int>(lp.size());
        for (int rep = 0; rep < 2; ++rep)
            for (double v : fb.hN[r]) lp.push_back(static_cast<float>(v));
    }
    // order-2 filters psi_{j2, l2} at level r < j2, four consecutive l2 interleaved per bin
    const int nq = (L + 3) / 4;
    std::vector<float4> psi4;
    std::vector<long long> psi4_off(static_cast<size_t>(J) * J * nq, -1);
    if (max_order >= 2) {
        for (int j2 = 1; j2 < J; ++j2)
            for (int r = 0; r < j2 && r < wst::psi_levels(j2, J); ++r)
                for (int q = 0; q < nq; ++q) {
                    psi4_off[(static_cast<size_t>(j2) * J + r) * nq + q] = static_cast<long long>(psi4.size());
                    const size_t nb = static_cast<size_t>(g.PM >> r) * (g.PN >> r);
                    for (size_t i = 0; i < nb; ++i) {
                        float v[4] = {0.f, 0.f, 0.f, 0.f};
                        for (int t = 0; t < 4; ++t) {
                            const int l2 = 4 * q + t;
                            if (l2 < L) v[t] = static_cast<float>(fb.psi[static_cast<size_t>(j2) * L + l2][r][i]);
                        }
                        psi4.push_back(make_float4(v[0], v[1], v[2], v[3]));
                    }
                }
    }
    std::vector<float2> tw;
    std::vector<int> tw_off(2 * static_cast<size_t>(J + 1));
    for (int r = 0; r <= J; ++r)
        for (int d = 0; d < 2; ++d) {
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            tw_off[2 * r + d] = static_cast<int>(tw.size());
            for (int k = 0; k < n; ++k) {
                const double a = 2.0 * 3.14159265358979323846 * k / n;
                tw.push_back(make_float2(static_cast<float>(std::cos(a)), static_cast<float>(-std::sin(a))));
            }
        }
    std::vector<int> o2(static_cast<size_t>(J) * L, 0);
    {
        int k = 1 + J * L;
        for (int j1 = 0; j1 < J; ++j1)
            for (int l1 = 0; l1 < L; ++l1) {
                o2[static_cast<size_t>(j1) * L + l1] = k;
                if (max_order >= 2) k += L * (J - 1 - j1);
            }
    }

    int rc;
    if ((rc = upload(&plan->d_psi, psi)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_psi_off, psi_off)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_lp, lp)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_lp_off, lp_off)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_tw, tw)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_tw_off, tw_off)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_o2, o2)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_psi4, psi4)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_psi4_off, psi4_off)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_perm, perm)) != WST_OK) return rc;
    if ((rc = upload(&plan->d_perm_off, perm_off)) != WST_OK) return rc;
    plan->lp_off_h = lp_off;
    plan->tw_off_h = tw_off;

    DevParams& dp = plan->dp;
    dp.M = g.M; dp.N = g.N; dp.PM = g.PM; dp.PN = g.PN; dp.J = J; dp.L = L;
    dp.max_order = max_order; dp.pre_pad = pre_pad ? 1 : 0; dp.K = g.K;
    dp.mM = g.mM; dp.mN = g.mN; dp.oM = g.oM; dp.oN = g.oN;
    dp.padTop = g.padTop; dp.padLeft = g.padLeft;
    dp.tw_total = static_cast<int>(tw.size());
    {
        const char* dbg = std::getenv("WST_DEBUG_SKIP");
        dp.dbg_skip = dbg ? std::atoi(dbg) : 0;
        const char* dfft = std::getenv("WST_DEBUG_FFT");
        const int v = dfft ? std::atoi(dfft) : 0;
        WST_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(wstfft::g_dbg_fft), &v, sizeof(int)));
    }
    dp.lp_total = static_cast<int>(lp.size());
    dp.psi = plan->d_psi; dp.psi_off = plan->d_psi_off;
    dp.lp = plan->d_lp; dp.lp_off = plan->d_lp_off;
    dp.tw = plan->d_tw; dp.tw_off = plan->d_tw_off;
    dp.o2_base = plan->d_o2;
    dp.psi4 = plan->d_psi4;
    dp.psi4_off = plan->d_psi4_off;
    dp.perm = plan->d_perm;
    dp.perm_off = plan->d_perm_off;
    dp.perm_total = static_cast<int>(perm.size());

    // --- LDS budgets ---
    const size_t tables = align16(tw.size() * sizeof(float2)) + align16(lp.size() * sizeof(float));
    const size_t P2 = static_cast<size_t>(g.PM) * g.PN;
    plan->prep_lds = align16(static_cast<size_t>(g.PM) * odd_ld(g.PN) * sizeof(float2)) + tables +
                     align16((static_cast<size_t>(g.PM) * g.oN + g.oM * g.oN + 16) * sizeof(float));
    if (plan->prep_lds > static_cast<size_t>(kMaxLds))
        return fail(WST_ERR_UNSUPPORTED,
                    "padded plane " + std::to_string(g.PM) + "x" + std::to_string(g.PN) +
                        " exceeds the LDS-resident path (160 KiB per CU)");
    plan->prep_threads = P2 >= 4096 ? 512 : 256;
    plan->k1_threads.resize(J);
    plan->k1_G.resize(J);
    plan->k1_lds.resize(J);
    plan->k1_tmpN.resize(J);
    plan->k1_cap.resize(J);
    for (int j1 = 0; j1 < J; ++j1) {
        const size_t n1 = static_cast<size_t>(g.PM >> j1) * (g.PN >> j1);
        const size_t n1p = static_cast<size_t>(g.PM >> j1) * odd_ld(g.PN >> j1);
        const bool do2 = max_order >= 2 && j1 < J - 1;
        const size_t slot = do2 ? static_cast<size_t>(g.PM >> (j1 + 1)) * odd_ld(g.PN >> (j1 + 1)) : 0;
        const int G = do2 ? 4 : 1;   // B region = 4 arrays of level j1+1 (float4 filter groups)
        // low-pass scratch: rows of the largest batch the order-2 loop forms (mirrors the kernel)
        const int nM1 = g.PM >> j1;
        size_t tmp_rows = static_cast<size_t>(nM1);
        int maxnp = std::max(G, L);
        if (do2) {
            const int nqq = (L + 3) / 4;
            const size_t bcap = static_cast<size_t>(G) * slot;
            for (int j2 = j1 + 1; j2 < J; ++j2) {
                const int nM2 = g.PM >> j2;
                const size_t pslot = static_cast<size_t>(nM2) * odd_ld(g.PN >> j2);
                int qpb = static_cast<int>(bcap / (4 * pslot));
                qpb = std::max(1, std::min(qpb, nqq));
                const int npath = std::min(4 * qpb, L);
                tmp_rows = std::max(tmp_rows, static_cast<size_t>(npath) * nM2);
            }
        }
        const size_t tmpN = tmp_rows * g.oN;
        const size_t lds = align16(n1p * sizeof(float2)) + align16(G * slot * sizeof(float2)) +
                           tables + align16(perm.size() * sizeof(int)) +
                           align16((tmpN + static_cast<size_t>(maxnp) * g.oM * g.oN + 16) * sizeof(float));
        if (lds > static_cast<size_t>(kMaxLds))
            return fail(WST_ERR_UNSUPPORTED, "order-1 plane at j1=" + std::to_string(j1) +
                                                 " exceeds the LDS-resident path (160 KiB per CU)");
        plan->k1_G[j1] = G;
        plan->k1_lds[j1] = lds;
        plan->k1_tmpN[j1] = static_cast<int>(tmpN);
        plan->k1_cap[j1] = cap_for(std::max(g.PM >> j1, g.PN >> j1));
        // measured on MI355X (c2): 96^2 -> 1024, 48^2 -> 256, 24^2 -> 128, 12^2 -> 64 threads
        plan->k1_threads[j1] = n1 >= 8192 ? 1024 : n1 >= 2048 ? 256 : n1 >= 512 ? 128 : 64;
    }
    if (const char* thr = std::getenv("WST_K1_THREADS")) {   // tuning override "t0,t1,..."
        int j = 0;
        for (const char* c = thr; *c && j < J; ++j) {
            const int t = std::atoi(c);
            if (t >= 64 && t <= 1024 && t % 64 == 0) plan->k1_threads[j] = t;
            while (*c && *c != ',') ++c;
            if (*c == ',') ++c;
        }
    }
    if ((rc = set_lds_attributes()) != WST_OK) return rc;

    *out = plan.release();
    g_last_error.clear();
    return WST_OK;
}

int wst_plan_destroy(wst_plan* plan) {
    free_plan(plan);
    return WST_OK;
}

int wst_output_shape(const wst_plan* plan, int* K, int* Mo, int* No) {
    if (!plan) return fail(WST_ERR_INVALID, "plan is NULL");
    if (K) *K = plan->g.K;
    if (Mo) *Mo = plan->g.oM;
    if (No) *No = plan->g.oN;
    return WST_OK;
}

int wst_padded_shape(const wst_plan* plan, int* PM, int* PN) {
    if (!plan) return fail(WST_ERR_INVALID, "plan is NULL");
    if (PM) *PM = plan->g.PM;
    if (PN) *PN = plan->g.PN;
    return WST_OK;
}

int wst_workspace_bytes(const wst_plan* plan, int64_t nbatch, size_t* bytes) {
    if (!plan || !bytes) return fail(WST_ERR_INVALID, "plan/bytes is NULL");
    if (nbatch < 0) return fail(WST_ERR_INVALID, "nbatch < 0");
    *bytes = static_cast<size_t>(nbatch) * plan->g.PM * plan->g.PN * sizeof(float2);
    return WST_OK;
}

}  // extern "C"

namespace {

// Launch-time timer: when `kms` is non-null, every launch is bracketed by events on `stream`
// and its duration is added to kms[slot].
struct LaunchTimer {
    float* kms = nullptr;
    int nkms = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    ~LaunchTimer() {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }
    int init(float* k, int n) {
        kms = k;
        nkms = n;
        if (!kms) return WST_OK;
        for (int i = 0; i < n; ++i) kms[i] = 0.f;
        WST_HIP_CHECK(hipEventCreate(&e0));
        WST_HIP_CHECK(hipEventCreate(&e1));
        return WST_OK;
    }
    int begin(hipStream_t s) {
        if (kms) WST_HIP_CHECK(hipEventRecord(e0, s));
        return WST_OK;
    }
    int end(hipStream_t s, int slot) {
        if (!kms) return WST_OK;
        WST_HIP_CHECK(hipEventRecord(e1, s));
        WST_HIP_CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        WST_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (slot < nkms) kms[slot] += ms;
        return WST_OK;
    }
};

int forward_impl(const wst_plan* plan, const float* d_in, int64_t nbatch, float* d_out, int pooled,
                 void* d_workspace, size_t workspace_bytes, void* stream_, float* kms, int nkms) {
    if (!plan) return fail(WST_ERR_INVALID, "plan is NULL");
    if (nbatch < 0) return fail(WST_ERR_INVALID, "nbatch < 0");
    if (nbatch == 0) return WST_OK;
    if (!d_in || !d_out) return fail(WST_ERR_INVALID, "input/output pointer is NULL");
    int dev = -1;
    WST_HIP_CHECK(hipGetDevice(&dev));
    if (dev != plan->device)
        return fail(WST_ERR_HIP, "plan was created on device " + std::to_string(plan->device) +
                                     " but device " + std::to_string(dev) + " is current");
    hipStream_t stream = reinterpret_cast<hipStream_t>(stream_);
    const wst::Geometry& g = plan->g;
    const size_t plane_ws = static_cast<size_t>(g.PM) * g.PN * sizeof(float2);
    void* ws = d_workspace;
    size_t wsb = workspace_bytes;
    if (!ws) {
        // internal workspace: up to 2048 planes per chunk (Xhat chunk stays MALL-resident)
        const int64_t want = std::min<int64_t>(nbatch, 2048);
        std::lock_guard<std::mutex> lk(plan->ws_mu);
        if (plan->ws_bytes < want * plane_ws) {
            if (plan->ws) {
                WST_HIP_CHECK(hipStreamSynchronize(stream));
                (void)hipFree(plan->ws);
                plan->ws = nullptr;
                plan->ws_bytes = 0;
            }
            WST_HIP_CHECK(hipMalloc(&plan->ws, want * plane_ws));
            plan->ws_bytes = want * plane_ws;
        }
        ws = plan->ws;
        wsb = plan->ws_bytes;
    }
    const int64_t chunk = static_cast<int64_t>(wsb / plane_ws);
    if (chunk < 1) return fail(WST_ERR_INVALID, "workspace smaller than one padded plane");
    const int inM = plan->dp.pre_pad ? g.PM : g.M, inN = plan->dp.pre_pad ? g.PN : g.N;
    float2* xhat = reinterpret_cast<float2*>(ws);
    LaunchTimer timer;
    int rc;
    if ((rc = timer.init(kms, nkms)) != WST_OK) return rc;
    for (int64_t c0 = 0; c0 < nbatch; c0 += chunk) {
        const int nimg = static_cast<int>(std::min<int64_t>(chunk, nbatch - c0));
        if ((rc = timer.begin(stream)) != WST_OK) return rc;
        launch_prep(plan->fam_m, plan->fam_n, dim3(nimg), dim3(plan->prep_threads), plan->prep_lds,
                    stream, plan->dp, d_in + c0 * inM * inN, static_cast<long long>(c0), xhat, d_out,
                    pooled);
        WST_HIP_CHECK(hipGetLastError());
        if ((rc = timer.end(stream, 0)) != WST_OK) return rc;
        for (int j1 = 0; j1 < g.J; ++j1) {
            if ((rc = timer.begin(stream)) != WST_OK) return rc;
            launch_order12(plan->fam_m, plan->fam_n, plan->k1_cap[j1], dim3(nimg * g.L),
                           dim3(plan->k1_threads[j1]), plan->k1_lds[j1], stream, plan->dp, j1,
                           plan->k1_G[j1], plan->k1_tmpN[j1], nimg, static_cast<long long>(c0), xhat,
                           d_out, pooled);
            WST_HIP_CHECK(hipGetLastError());
            if ((rc = timer.end(stream, 1 + j1)) != WST_OK) return rc;
        }
    }
    return WST_OK;
}

}  // namespace

extern "C" {

int wst_forward(const wst_plan* plan, const float* d_in, int64_t nbatch, float* d_out, int pooled,
                void* d_workspace, size_t workspace_bytes, void* stream) {
    return forward_impl(plan, d_in, nbatch, d_out, pooled, d_workspace, workspace_bytes, stream,
                        nullptr, 0);
}

int wst_forward_profiled(const wst_plan* plan, const float* d_in, int64_t nbatch, float* d_out,
                         int pooled, void* d_workspace, size_t workspace_bytes, void* stream,
                         float* kernel_ms, int n_kernel_ms) {
    if (!kernel_ms || n_kernel_ms < 1) return fail(WST_ERR_INVALID, "kernel_ms is NULL/empty");
    return forward_impl(plan, d_in, nbatch, d_out, pooled, d_workspace, workspace_bytes, stream,
                        kernel_ms, n_kernel_ms);
}

int wst_host_filter(int M, int N, int J, int L, int kind, int j, int l, int r, double* out,
                    int64_t len) {
    if (!out) return fail(WST_ERR_INVALID, "out is NULL");
    if (J < 1) return fail(WST_ERR_INVALID, "J must be >= 1");
    wst::Geometry g;
    std::string err;
    if (!wst::make_geometry(M, N, J, L, 2, g, err)) return fail(WST_ERR_INVALID, err);
    try {
        // cache the last bank: the test-suite inspects every filter of one geometry in turn
        static thread_local std::unique_ptr<wst::FilterBank> cached;
        if (!cached || cached->g.M != M || cached->g.N != N || cached->g.J != J || cached->g.L != L)
            cached.reset(new wst::FilterBank(wst::build_filter_bank(g)));
        const wst::FilterBank& fb = *cached;
        std::vector<double> v;
        if (kind == 0) {
            if (j < 0 || j >= J || l < 0 || l >= L) return fail(WST_ERR_INVALID, "bad (j, l)");
            const auto& lev = fb.psi[static_cast<size_t>(j) * L + l];
            if (r < 0 || r >= static_cast<int>(lev.size())) return fail(WST_ERR_INVALID, "bad level");
            v = lev[r];
        } else if (kind >= 1 && kind <= 3) {
            if (r < 0 || r >= J) return fail(WST_ERR_INVALID, "bad level");
            if (kind == 1) {
                const auto& a = fb.aM[r];
                const auto& b = fb.aN[r];
                v.resize(a.size() * b.size());
                for (size_t i = 0; i < a.size(); ++i)
                    for (size_t k = 0; k < b.size(); ++k) v[i * b.size() + k] = a[i] * b[k];
            } else {
                v = (kind == 2) ? fb.hM[r] : fb.hN[r];
            }
        } else {
            return fail(WST_ERR_INVALID, "bad kind");
        }
        if (static_cast<int64_t>(v.size()) > len) return fail(WST_ERR_INVALID, "output buffer too small");
        std::memcpy(out, v.data(), v.size() * sizeof(double));
    } catch (const std::exception& e) {
        return fail(WST_ERR_UNSUPPORTED, e.what());
    }
    return WST_OK;
}

int wst_host_fft_lines(int n, int inverse, int mode, float* data, int nb, int bs, int nl, int ls,
                       int es, int threads, int* perm) {
    if (!data || n < 1 || nb < 1 || nl < 1 || threads < 1 || mode < 0 || mode > 2)
        return fail(WST_ERR_INVALID, "bad arguments");
    std::vector<float2> tw(static_cast<size_t>(n));
    for (int k = 0; k < n; ++k) {
        const double a = 2.0 * 3.14159265358979323846 * k / n;
        tw[k] = make_float2(static_cast<float>(std::cos(a)), static_cast<float>(-std::sin(a)));
    }
    float2* base = reinterpret_cast<float2*>(data);
    const wstfft::Lines g{nb, bs, nl, ls, es};
    bool compiled = false;
    switch (n) {
#define WST_HOST_CASE(NN)                                                                  \
    case NN:                                                                               \
        compiled = true;                                                                   \
        if (mode == 0) {                                                                   \
            if (inverse) wstfft::fft_lines_host<NN, true>(base, g, tw.data(), threads);    \
            else wstfft::fft_lines_host<NN, false>(base, g, tw.data(), threads);           \
        } else {                                                                           \
            if (inverse) wstfft::fft_lines_inplace_host<NN, true>(base, g, tw.data(), mode); \
            else wstfft::fft_lines_inplace_host<NN, false>(base, g, tw.data(), mode);      \
        }                                                                                  \
        break;
        WST_FFT_SIZES(WST_HOST_CASE)
#undef WST_HOST_CASE
        default:
            break;
    }
    if (perm)
        for (int pos = 0; pos < n; ++pos) perm[pos] = compiled ? wstfft::dr_logical_host(n, pos) : pos;
    if (compiled) return WST_OK;
    if (mode != 0) return fail(WST_ERR_UNSUPPORTED, "in-place modes need a compiled FFT size");
    // generic DFT, same arithmetic as lds_dft_lines_generic
    const float sgn = inverse ? -1.f : 1.f;
    std::vector<float2> line(static_cast<size_t>(n));
    for (int L0 = 0; L0 < g.nlines(); ++L0) {
        const int off = g.offset(L0);
        for (int e = 0; e < n; ++e) line[e] = base[off + e * es];
        for (int k = 0; k < n; ++k) {
            float sr = 0.f, si = 0.f;
            int idx = 0;
            for (int e = 0; e < n; ++e) {
                const float2 x = line[e];
                const float2 w = tw[idx];
                const float wy = sgn * w.y;
                sr = std::fma(x.x, w.x, std::fma(-x.y, wy, sr));
                si = std::fma(x.x, wy, std::fma(x.y, w.x, si));
                idx += k;
                if (idx >= n) idx -= n;
            }
            base[off + k * es] = make_float2(sr, si);
        }
    }
    return WST_OK;
}

}  // extern "C"
