// k_o2w: the first order-2 level of square LDS-resident levels with 4 x 4 output maps, one path per
// wave with every line of the 2-D transform in registers (the headline geometry: 64^2 patches,
// J = 4, P = 96: the 8 x 48^2 paths of each (plane, theta1) at j1 = 0).
//
// Same cascade as k_o2 (kymatio 0.3.0 scattering2d, SURVEY.md Appendix A.4: U1hat * psi_{j2,l2}
// -> periodize by 2 -> ifft -> |.| -> phi low-pass + subsample + unpad), organised for CDNA4
// registers instead of LDS batches.  One workgroup per (plane, theta1) at level j1, eight waves:
//   1. the block loads the U1 half spectrum (rows transformed by k_o1) into LDS and runs its column
//      FFTs;
//   2. wave w folds path l2 = w (Hermitian, s = 2, dense) straight into registers: lane v holds
//      column v, every LDS and filter address is a compile-time offset from the lane base, the
//      filter taps of the next rows are in flight;
//   3. barrier: the spectrum is dead, its LDS becomes eight per-wave transposition buffers;
//   4. each wave alone (no further barrier): column iFFT in registers (compile-time twiddles,
//      wstfft::rfft), transposition real part then imaginary part through its n2 x (n2|1) float
//      buffer, row iFFT, modulus and the row half of the low-pass in registers, the column half
//      as a halving exchange across the lanes, then the 4 x 4 map (or its mean / std).
// The smaller order-2 levels of the same j1 stay in k_o2 (launched with j2first = j1 + 2).
//
// The low-pass uses the natural-order tap matrices of the level (GM_nat[p][a] =
// h[(2^(J-j2) (a + 1) - p) mod n2], host lpn pool): S[a][c] = sum_p sum_q G[p][a] G[q][c] |z[p][q]|.
#pragma once

#include "wst_device.h"

namespace wstdev {

constexpr int kO2wWaves = 8;     // waves per k_o2w workgroup (one order-2 path each, L <= 8)
#ifndef WST_O2W_AHEAD
#define WST_O2W_AHEAD 4
#endif
#ifndef WST_O2W_WPE
#define WST_O2W_WPE 4            // waves per SIMD the register budget is sized for (2 WGs x 8 waves / CU)
#endif
constexpr int kFoldAhead = WST_O2W_AHEAD;   // fold rows whose filter taps are in flight

// The first order-2 level (n2 = n1c / 2 lines) goes through k_o2w when one lane can own a line.
constexpr bool o2w_reg(int n1c, int n2) { return n2 * 2 == n1c && n2 > 32 && n2 <= 64; }
// floats of one wave's transposition buffer (n2 x (n2 | 1), 16-byte multiple)
constexpr int o2w_wave_floats(int n1c) { return ((n1c / 2) * ((n1c / 2) | 1) + 3) & ~3; }
// level sizes of family fam that k_o2w is compiled for
constexpr bool o2w_supported(int fam, int n1c) {
    if (fam <= 0 || !o2w_reg(n1c, n1c / 2)) return false;
    int n = fam;
    while (n < n1c) n *= 2;
    return n == n1c;
}

// Orders this wave's LDS accesses: LDS executes a wave's instructions in order, so another lane's
// earlier store is visible to a later load once the compiler keeps them in program order.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// v from the lane whose index differs in bit D (D < 64).  Within a row of 16 lanes the partner is
// reached by DPP (D = 1, 2 exact xor; D = 4, 8 the row half-mirror / mirror, which also pairs
// lanes across bit D); D = 16, 32 through ds_bpermute.
template <int D>
__device__ __forceinline__ float lane_swap(float v) {
    if constexpr (D == 1) return dpp_mov<0xB1>(v);
    else if constexpr (D == 2) return dpp_mov<0x4E>(v);
    else if constexpr (D == 4) return dpp_mov<0x141>(v);
    else if constexpr (D == 8) return dpp_mov<0x140>(v);
    else return __shfl_xor(v, D, 64);
}

// Sums 16 per-lane values over aligned groups of G lanes.  Halving exchange: at distances
// D = G/2, G/4, ... a lane keeps the half of its values selected by its lane bit D and adds the
// partner's copy of that half; once one value is left the remaining distances just add it.
// Afterwards a lane holds NV = max(1, 16 / G) group sums P[0..NV) of values idx0 .. idx0 + NV - 1
// (returned); lanes with (lane & sum_mask) != 0 hold copies.
template <int G>
struct Reduce16 {
    static constexpr int steps_halving() {
        int s = 0, cur = 16;
        for (int d = G / 2; d >= 1 && cur > 1; d /= 2) ++s, cur /= 2;
        return s;
    }
    static constexpr int NV = 16 >> steps_halving();
    static constexpr int sum_mask() {
        int m = 0, cur = 16;
        for (int d = G / 2; d >= 1; d /= 2) {
            if (cur > 1) cur /= 2;
            else m |= d;
        }
        return m;
    }
    template <int D, int CUR>
    static __device__ __forceinline__ void step(float (&P)[16], int lane, int& idx0) {
        if constexpr (D >= 1) {
            if constexpr (CUR > 1) {
                constexpr int H = CUR / 2;
                const bool hi = (lane & D) != 0;
                wstfft::static_for<0, H>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    const float snd = hi ? P[i] : P[i + H];
                    const float kp = hi ? P[i + H] : P[i];
                    P[i] = kp + lane_swap<D>(snd);
                });
                if (hi) idx0 += H;
                step<D / 2, H>(P, lane, idx0);
            } else {
                P[0] += lane_swap<D>(P[0]);
                step<D / 2, 1>(P, lane, idx0);
            }
        }
    }
    static __device__ __forceinline__ int run(float (&P)[16], int lane) {
        int idx0 = 0;
        step<G / 2, 16>(P, lane, idx0);
        return idx0;
    }
};

__device__ __forceinline__ float buf_load1(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// Emits the G-lane-reduced 4 x 4 map of path k (coefficient index k0) from Reduce16 output.
template <int G>
__device__ __forceinline__ void o2w_emit(const float (&P)[16], int idx0, int lane, bool path_ok,
                                         long long img, int K, int k0, float* __restrict__ out,
                                         int pooled) {
    using R = Reduce16<G>;
    constexpr int NV = R::NV;
    constexpr int SM = R::sum_mask();
    if (!pooled) {
        if (path_ok && (lane & SM) == 0) {
            float* o = out + (img * K + k0) * 16 + idx0;
            wstfft::static_for<0, NV>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                __builtin_nontemporal_store(P[i], o + i);
            });
        }
        return;
    }
    // pooled: mean and population std of the 16 values (spread over the lanes of the group)
    float s = 0.f;
    wstfft::static_for<0, NV>([&](auto ic) { s += P[decltype(ic)::value]; });
    // sum over the halving bits (every lane of a sum_mask class holds the same values)
    wstfft::static_for<0, 6>([&](auto bc) {
        constexpr int D = 1 << decltype(bc)::value;
        if constexpr (D < G && !(SM & D)) s += lane_swap<D>(s);
    });
    const float mean = s * (1.f / 16.f);
    float q = 0.f;
    wstfft::static_for<0, NV>([&](auto ic) {
        const float d = P[decltype(ic)::value] - mean;
        q = fmaf(d, d, q);
    });
    wstfft::static_for<0, 6>([&](auto bc) {
        constexpr int D = 1 << decltype(bc)::value;
        if constexpr (D < G && !(SM & D)) q += lane_swap<D>(q);
    });
    if (path_ok && (lane & (G - 1)) == 0) {
        out[img * 2 * K + k0] = mean;
        out[img * 2 * K + K + k0] = sqrtf(q * (1.f / 16.f));
    }
}

// First order-2 level, path l2 in one wave: dense Hermitian s = 2 fold into registers (lane v
// holds column v; every LDS and filter address a compile-time offset from the lane base).
template <int N1C>
__device__ __forceinline__ void o2w_fold_reg(const float2* __restrict__ H, const DevParams& p, int j1,
                                             int l2, int lane, float2 (&col)[N1C / 2]) {
    constexpr int N2 = N1C / 2, HLD = N1C / 2 + 1;
    const int v = lane < N2 ? lane : N2 - 1;
    const float* psi = p.psi2s + p.psi2s_off[j1 * p.L + l2];
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(psi, N1C * N1C * 4);
    const float2* hv = H + v;             // direct taps: column v
    const float2* hm = H + (N2 - v);      // mirrored taps: column N2 - v (conjugated)
    const int fo = v * 4;
    // the filter taps of rows u .. u + kFoldAhead - 1 are in flight while row u is summed (L2
    // latency; one load wait per row otherwise serialises the fold)
    constexpr int AH = kFoldAhead;
    float f[AH][4];
    auto load_row = [&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u < N2) {
            constexpr int kr0 = u, kr1 = u + N2;
            f[u % AH][0] = buf_load1(rs, fo, kr0 * N1C * 4);
            f[u % AH][1] = buf_load1(rs, fo, (kr0 * N1C + N2) * 4);
            f[u % AH][2] = buf_load1(rs, fo, kr1 * N1C * 4);
            f[u % AH][3] = buf_load1(rs, fo, (kr1 * N1C + N2) * 4);
        }
    };
    // the four spectrum taps of rows u .. u + HA - 1 likewise (LDS latency)
    constexpr int HA = 2;
    float2 hb[HA][4];
    auto load_h = [&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        if constexpr (u < N2) {
            constexpr int kr0 = u, kr1 = u + N2, krm0 = u ? N1C - u : 0, krm1 = N2 - u;
            hb[u % HA][0] = hv[kr0 * HLD];
            hb[u % HA][1] = hm[krm0 * HLD];
            hb[u % HA][2] = hv[kr1 * HLD];
            hb[u % HA][3] = hm[krm1 * HLD];
        }
    };
    wstfft::static_for<0, AH>(load_row);
    wstfft::static_for<0, HA>(load_h);
    wstfft::static_for<0, N2>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const float2 h0 = hb[u % HA][0], h1 = hb[u % HA][1], h2 = hb[u % HA][2], h3 = hb[u % HA][3];
        const float f0 = f[u % AH][0], f1 = f[u % AH][1], f2 = f[u % AH][2], f3 = f[u % AH][3];
        col[u].x = fmaf(h0.x, f0, fmaf(h1.x, f1, fmaf(h2.x, f2, h3.x * f3)));
        col[u].y = fmaf(h0.y, f0, fmaf(-h1.y, f1, fmaf(h2.y, f2, -h3.y * f3)));
        load_row(std::integral_constant<int, u + AH>{});
        load_h(std::integral_constant<int, u + HA>{});
    });
}

// The folded path (lane v: column v) -> column iFFT -> transposition (re, then im) through the
// wave's buffer -> row iFFT -> |.| -> S2 low-pass -> emit.
template <int N1C>
__device__ __forceinline__ void o2w_path_reg(float2 (&col)[N1C / 2], float* __restrict__ wb,
                                             const float* __restrict__ G2, const DevParams& p,
                                             int lane, long long img, int k0, float* __restrict__ out,
                                             int pooled, int& sctr, bool stamp_on) {
    constexpr int N2 = N1C / 2, TL = N2 | 1;
    const int v = lane < N2 ? lane : N2 - 1;
    WST_STAMP(sctr);
    wstfft::rfft<N2, true>(col);
    WST_STAMP(sctr);
    // transposition through the wave buffer: lane v writes column v, lane k reads row k
    const int kr = lane < N2 ? lane : N2 - 1;
    float2 row[N2];
    if (lane < N2)
        wstfft::static_for<0, N2>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            wb[k * TL + v] = col[k].x;
        });
    wave_lds_sync();
    wstfft::static_for<0, N2>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        row[q].x = wb[kr * TL + q];
    });
    wave_lds_sync();
    if (lane < N2)
        wstfft::static_for<0, N2>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            wb[k * TL + v] = col[k].y;
        });
    wave_lds_sync();
    wstfft::static_for<0, N2>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        row[q].y = wb[kr * TL + q];
    });
    wave_lds_sync();
    WST_STAMP(sctr);
    wstfft::rfft<N2, true>(row);
    WST_STAMP(sctr);
    // |z| and the low-pass: T[c] = sum_q G[q][c] |z[kr][q]|, P[a][c] = G[kr][a] T[c] (G2: the
    // level's natural tap matrix in LDS, uniform rows read by broadcast)
    const float scale2 = 1.f / static_cast<float>(N1C * N1C);
    float T[4] = {0.f, 0.f, 0.f, 0.f};
    wstfft::static_for<0, N2>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const float m = __builtin_amdgcn_sqrtf(fmaf(row[q].x, row[q].x, row[q].y * row[q].y));
        T[0] = fmaf(G2[q * 4 + 0], m, T[0]);
        T[1] = fmaf(G2[q * 4 + 1], m, T[1]);
        T[2] = fmaf(G2[q * 4 + 2], m, T[2]);
        T[3] = fmaf(G2[q * 4 + 3], m, T[3]);
    });
    const float4 gk = *reinterpret_cast<const float4*>(G2 + kr * 4);
    const bool ok = lane < N2;
    const float ga[4] = {ok ? gk.x * scale2 : 0.f, ok ? gk.y * scale2 : 0.f, ok ? gk.z * scale2 : 0.f,
                         ok ? gk.w * scale2 : 0.f};
    float P[16];
    wstfft::static_for<0, 16>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        P[i] = ga[i / 4] * T[i % 4];
    });
    WST_STAMP(sctr);
    const int idx0 = Reduce16<64>::run(P, lane);
    o2w_emit<64>(P, idx0, lane, true, img, p.K, k0, out, pooled);
    WST_STAMP(sctr);
}

template <int FAM, int N1C>
__global__ void __launch_bounds__(64 * kO2wWaves) __attribute__((amdgpu_waves_per_eu(WST_O2W_WPE, WST_O2W_WPE)))
    k_o2w(DevParams p, LdsLayout lay, int j1, int nimg, long long img0,
          const float2* __restrict__ hexp, float* __restrict__ out, int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int HLD = N1C / 2 + 1, N2 = N1C / 2;
    static_assert(o2w_reg(N1C, N2), "k_o2w: first order-2 level of 33..64 lines");
    [[maybe_unused]] constexpr int CAP = N1C <= 12 ? 12 : N1C <= 24 ? 24 : N1C <= 48 ? 48 : 136;
    const int L = p.L;
    const int item = xcd_item(nimg * L);
    const int local = item / L;
    const int l1 = item - local * L;
    const long long img = img0 + local;
    float2* H = reinterpret_cast<float2*>(smem);
    [[maybe_unused]] int sctr = 0;
    [[maybe_unused]] const bool stamp_on = (j1 == 0);
    WST_STAMP(sctr);
    const Tables tb = load_tables(p, lay, smem);
    // 1. half spectrum -> LDS, column FFTs (rows digit-reversed -> natural): block-wide
    copy_to_lds(H, hexp + static_cast<long long>(item) * N1C * HLD, N1C * HLD);
    // natural tap matrix of level j1 + 1 (lpn pool)
    float* G2 = reinterpret_cast<float*>(smem + lay.off_s);
    const float* g2src = p.lpn + p.lpn_off[2 * (j1 + 1)];
    for (int i = threadIdx.x; i < N2 * 4; i += blockDim.x) G2[i] = g2src[i];
    __syncthreads();
    WST_STAMP(sctr);
    wstfft::EpiIdentity id;
#ifndef WST_O2W_NOCOLFFT
    lds_fft_lines<FAM, prev_cap(CAP), CAP, kRD, false>(H, wstfft::Lines{1, 0, HLD, 1, HLD}, N1C,
                                                       tb.twM(j1), id);
#else
    (void)tb;
    (void)id;
#endif
    WST_STAMP(sctr);
    // 2. wave w: path l2 = w of level j1 + 1 -- fold into registers; then the spectrum is dead and
    //    its LDS becomes the per-wave transposition buffers
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const bool active = wave < L;
    float2 col[N2];
    if (active) o2w_fold_reg<N1C>(H, p, j1, wave, lane, col);
    __syncthreads();
    WST_STAMP(sctr);
    if (!active) return;
    float* wb = reinterpret_cast<float*>(smem) + wave * o2w_wave_floats(N1C);
    const int k0 = p.o2_base[j1 * L + l1] + wave;
    o2w_path_reg<N1C>(col, wb, G2, p, lane, img, k0, out, pooled, sctr, stamp_on);
}

}  // namespace wstdev
