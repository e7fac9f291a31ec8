// k_o2r: the first order-2 level of an LDS-resident level j1 (paths j2 = j1 + 1, s = 2) with every
// path held in the registers of ONE wave -- no LDS batches and no workgroup barrier after the
// spectrum is in place.  The headline geometry (64^2 patches, J = 4, P = 96): the 8 paths of
// 48 x 48 per (plane, theta1) at j1 = 0, and the 24 x 24 paths at j1 = 1.
//
// Same cascade as k_o2 (kymatio 0.3.0 scattering2d, SURVEY.md Appendix A.4: U1hat * psi_{j2,l2}
// -> periodize by 2 -> ifft2 -> |.| -> phi low-pass + subsample + unpad), replacing the reference
// calls reached from src/training/train_and_save_model.py:364-368.
//
// Layout of one n x n path (n = N1C / 2 = 8 R) in a wave: lane (h, g) of an 8 x 8 lane grid holds
// the R x R elements (i, k) -> B[8 i + rev(h)][8 k + rev(g)] (rev = 3-bit reversal).  A line
// transform of length n = R x 8 is an in-lane DFT-R, the twiddle w_n^(n1 rev(g)) and a DFT-8 across
// the 8 lanes of the line (radix-2 DIT, bit-reversed lane input, natural lane output), so the
// output element (i, n1) of lane g is column n1 + R g.  Cross-lane partners:
//   row pass (g bits): xor 1, xor 2 (DPP quad_perm), xor 7 (DPP row_half_mirror) -- with
//     b0 = g0 ^ g2, b1 = g1 ^ g2, b2 = g2 every logical bit flip is one DPP pairing;
//   column pass (h bits = b3, b4, b5): DPP row_ror:8, v_permlane16_swap, v_permlane32_swap.
// A butterfly stage is y = r_own + beta * r_partner on premultiplied values r (beta = -1 on the
// lanes of the odd half, which then hold the negated output -- a per-lane sign that the next
// stage's premultiplier absorbs and the modulus removes), so the DPP forms fold into v_fmac_f32_dpp.
//
// Per path: the s = 2 Hermitian fold reads its 4 spectrum taps per element from LDS at
// compile-time offsets and its 4 filter taps as one 16-byte load from a lane-ordered table (host:
// psil); the modulus and the separable low-pass (natural tap matrices) run on the final lane
// layout (rows m1 + R h, columns n1 + R g), then a halving reduction over the 64 lanes.
#pragma once

#include "wst_device.h"

namespace wstdev {

// ---------------------------------------------------------------------------------------------
// lane roles (shared with the host table builder)
// ---------------------------------------------------------------------------------------------
__host__ __device__ constexpr int rev3(int x) { return ((x & 1) << 2) | (x & 2) | ((x >> 2) & 1); }
// logical row-pass index g and column-pass index h of hardware lane `lane`
__host__ __device__ inline int o2r_g(int lane) {
    const int b0 = lane & 1, b1 = (lane >> 1) & 1, b2 = (lane >> 2) & 1;
    return (b0 ^ b2) | ((b1 ^ b2) << 1) | (b2 << 2);
}
__host__ __device__ inline int o2r_h(int lane) { return (lane >> 3) & 7; }
// level sizes k_o2r is compiled for: N1C = 16 R with an in-lane DFT-R
__host__ __device__ constexpr bool o2r_size(int n1c) { return n1c == 96 || n1c == 48; }
// LDS row stride (complex) of the spectrum: >= N1C / 2 + 1 and = 4 mod 16, so the 32 lanes of a
// ds_read_b64 half (4 row groups x 8 column groups) hit 32 distinct bank pairs
__host__ __device__ constexpr int o2r_stride(int n1c) {
    int s = n1c / 2 + 1;
    while (s % 16 != 4) ++s;
    return s;
}
// LDS bytes of k_o2r: spectrum (N1C + 1 rows; row N1C repeats row 0), twiddles of levels j1 and
// j1 + 1, natural tap matrices GM, GN of level j1 + 1 (4 floats per row)
__host__ __device__ constexpr int o2r_lds(int n1c) {
    return (n1c + 1) * o2r_stride(n1c) * 8 + n1c * 8 + (n1c / 2) * 8 + 2 * (n1c / 2) * 16;
}
constexpr int kO2rWaves = 8;   // waves per workgroup: one path each
#ifndef WST_O2R_AHEAD
#define WST_O2R_AHEAD 2
#endif
constexpr int kO2rFoldAhead = WST_O2R_AHEAD;   // fold elements whose spectrum taps are in flight
#ifndef WST_O2R_FAHEAD
#define WST_O2R_FAHEAD 4
#endif
constexpr int kO2rFiltAhead = WST_O2R_FAHEAD;  // fold elements whose filter taps are in flight
#ifndef WST_O2R_CHAIN
#define WST_O2R_CHAIN 2
#endif
constexpr int kO2rChain = WST_O2R_CHAIN;   // cross-lane butterfly chains scheduled together

// ---------------------------------------------------------------------------------------------
// cross-lane exchange
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    // bound_ctrl: every source lane is valid here; lets the compiler drop the "old" operand
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                                 0xF, 0xF, true));
}
// y = own + beta * partner, partner through DPP (OP 0: xor 1, 1: xor 2, 2: xor 7, 3: xor 8)
template <int OP>
__device__ __forceinline__ float bfly_dpp(float own, float beta) {
    constexpr int ctrl = OP == 0 ? 0xB1 : OP == 1 ? 0x4E : OP == 2 ? 0x141 : 0x128;
    return fmaf(dpp_f<ctrl>(own), beta, own);
}
// y = own + beta * partner for the partner across bit 4 (OP 4) or bit 5 (OP 5): the swap hands
// every lane the values of both members (lo: bit clear, hi: bit set); y = hi + beta * lo
template <int OP>
__device__ __forceinline__ float bfly_swap(float own, float beta) {
    const unsigned u = __builtin_bit_cast(unsigned, own);
    unsigned lo, hi;
    if constexpr (OP == 4) {
        const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
        lo = r[0];
        hi = r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
        lo = r[0];
        hi = r[1];
    }
    return fmaf(__builtin_bit_cast(float, lo), beta, __builtin_bit_cast(float, hi));
}
template <int OP>
__device__ __forceinline__ float2 bfly(float2 v, float beta) {
    if constexpr (OP <= 3) return make_float2(bfly_dpp<OP>(v.x, beta), bfly_dpp<OP>(v.y, beta));
    else return make_float2(bfly_swap<OP>(v.x, beta), bfly_swap<OP>(v.y, beta));
}
// Materialise v here: keeps the compiler from sinking the last butterfly of a value to its far
// use and holding the operands of every value live meanwhile.
__device__ __forceinline__ void pin(float2& v) { asm volatile("" : "+v"(v.x), "+v"(v.y)); }
__device__ __forceinline__ float2 cmulf(float2 a, float2 w) {
    return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}

// Per-lane constants of one pass (inverse transform of length n = 8 R over lane index q, q = g or
// h): stage premultipliers c1, c2 and the stage signs.
struct PassConst {
    float2 c1, c2;
    float beta0, beta1, beta2;
};
// tw2: forward twiddles exp(-2 pi i k / n) of the path level in LDS (inverse = conjugate)
template <int R>
__device__ __forceinline__ PassConst pass_const(const float2* tw2, int q) {
    constexpr int n = 8 * R;
    PassConst c;
    const int q0 = q & 1, q1 = (q >> 1) & 1, q2 = (q >> 2) & 1;
    c.beta0 = q0 ? -1.f : 1.f;
    c.beta1 = q1 ? -1.f : 1.f;
    c.beta2 = q2 ? -1.f : 1.f;
    // stage 1: lanes with q1 premultiply by w_4^(q0); all by the stage-0 sign
    const float2 w4 = tw2[q0 * (n / 4)];
    c.c1 = q1 ? make_float2(c.beta0 * w4.x, -c.beta0 * w4.y) : make_float2(c.beta0, 0.f);
    const float2 w8 = tw2[(q0 + 2 * q1) * (n / 8)];
    c.c2 = q2 ? make_float2(c.beta1 * w8.x, -c.beta1 * w8.y) : make_float2(c.beta1, 0.f);
    return c;
}
// in-lane twiddle w_n^(n1 c0) of output n1 (inverse: conjugate of the forward table)
__device__ __forceinline__ float2 pass_tw(const float2* tw2, int n1, int c0) {
    const float2 t = tw2[n1 * c0];
    return make_float2(t.x, -t.y);
}

// Inverse DFT-8 across the lanes of the line (stage ops S0, S1, S2) on one value.
template <int S0, int S1, int S2>
__device__ __forceinline__ float2 xlane8(float2 v, const PassConst& c) {
    v = bfly<S0>(v, c.beta0);
    v = bfly<S1>(cmulf(v, c.c1), c.beta1);
    v = bfly<S2>(cmulf(v, c.c2), c.beta2);
    return v;
}

// ---------------------------------------------------------------------------------------------
// halving reduction of 16 per-lane values over the wave and the map emit (4 x 4 maps)
// ---------------------------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ float lane_swap(float v) {
    if constexpr (D == 1) return dpp_f<0xB1>(v);
    else if constexpr (D == 2) return dpp_f<0x4E>(v);
    else if constexpr (D == 4) return dpp_f<0x141>(v);   // row_half_mirror: pairs across bit 2
    else if constexpr (D == 8) return dpp_f<0x128>(v);   // row_ror:8 = xor 8
    else return __shfl_xor(v, D, 64);
}
// After run(): lane holds the 64-lane sums P[0 .. NV) of values idx0 .. idx0 + NV (NV = 1: each
// lane one of the 16 sums, lanes differing only in bits 0, 1 hold copies... see sum_mask).
struct Reduce16 {
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
    // D = 32, 16, 8, 4 halve (16 -> 1 value), D = 2, 1 add: every lane ends with one of the 16
    // sums; lanes that differ only in bits 0 and 1 hold the same one
    static __device__ __forceinline__ int run(float (&P)[16], int lane) {
        int idx0 = 0;
        step<32, 16>(P, lane, idx0);
        return idx0;
    }
};

// One 4 x 4 map (coefficient k0 of plane img) from the reduced values: value idx0 in P[0].
__device__ __forceinline__ void o2r_emit(float v, int idx0, int lane, long long img, int K, int k0,
                                         float* __restrict__ out, int pooled) {
    if (!pooled) {
        if ((lane & 3) == 0) __builtin_nontemporal_store(v, out + (img * K + k0) * 16 + idx0);
        return;
    }
    // mean and population std of the 16 values: lanes 0, 4, ..., 60 hold the 16 distinct values
    float s = v;
    s += lane_swap<4>(s);
    s += lane_swap<8>(s);
    s += lane_swap<16>(s);
    s += lane_swap<32>(s);
    const float mean = s * (1.f / 16.f);
    const float d = v - mean;
    float q = d * d;
    q += lane_swap<4>(q);
    q += lane_swap<8>(q);
    q += lane_swap<16>(q);
    q += lane_swap<32>(q);
    if (lane == 0) {
        out[img * 2 * K + k0] = mean;
        out[img * 2 * K + K + k0] = sqrtf(q * (1.f / 16.f));
    }
}

// ---------------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------------
// One workgroup of 8 waves per (plane, theta1) at level j1 (N1C x N1C, square family FAM); 4 x 4
// output maps.  hexp: k_o1's half spectra (rows transformed, digit-reversed row order).
template <int FAM, int N1C>
__global__ void __launch_bounds__(64 * kO2rWaves, 4) k_o2r(DevParams p, int j1, int nimg, long long img0,
                                                          const float2* __restrict__ hexp,
                                                          float* __restrict__ out, int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int N2 = N1C / 2, R = N2 / 8, HLD = N2 + 1, S = o2r_stride(N1C);
    constexpr int CAP = N1C <= 12 ? 12 : N1C <= 24 ? 24 : N1C <= 48 ? 48 : 136;
    static_assert(o2r_size(N1C), "k_o2r level size");
    float2* H = reinterpret_cast<float2*>(smem);
    float2* tw1 = H + (N1C + 1) * S;
    float2* tw2 = tw1 + N1C;
    float* GM = reinterpret_cast<float*>(tw2 + N2);
    float* GN = GM + N2 * 4;
    const int L = p.L;
    const int item = xcd_item(nimg * L);
    const int local = item / L;
    const int l1 = item - local * L;
    const long long img = img0 + local;
    const int j2 = j1 + 1;

    // 1. tables, then the half spectrum into LDS (row stride S) and its column FFTs
    for (int i = threadIdx.x; i < N1C; i += blockDim.x) tw1[i] = p.tw[p.tw_off[2 * j1] + i];
    for (int i = threadIdx.x; i < N2; i += blockDim.x) tw2[i] = p.tw[p.tw_off[2 * j2] + i];
    for (int i = threadIdx.x; i < N2 * 4; i += blockDim.x) {
        GM[i] = p.lpn[p.lpn_off[2 * j2] + i];
        GN[i] = p.lpn[p.lpn_off[2 * j2 + 1] + i];
    }
    {
        const float2* src = hexp + static_cast<long long>(item) * N1C * HLD;
        constexpr int K = 8, NI = N1C * HLD;
        for (int i0 = threadIdx.x; i0 < NI; i0 += K * blockDim.x) {
            float2 t[K];
#pragma unroll
            for (int k = 0; k < K; ++k) t[k] = ldnt(src + min(i0 + k * static_cast<int>(blockDim.x), NI - 1));
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = i0 + k * blockDim.x;
                if (i < NI) {
                    const int r = i / HLD;
                    H[r * S + (i - r * HLD)] = t[k];
                }
            }
        }
    }
    __syncthreads();
    {
        wstfft::EpiIdentity id;
        lds_fft_lines<FAM, prev_cap(CAP), CAP, kRD, false>(H, wstfft::Lines{1, 0, HLD, 1, S}, N1C, tw1, id);
    }
    for (int c = threadIdx.x; c < HLD; c += blockDim.x) H[N1C * S + c] = H[c];   // row N1C = row 0
    __syncthreads();

    // 2. each wave: its paths l2 = wave, wave + 8, ... (no further barrier)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int g = o2r_g(lane), h = o2r_h(lane);
    const int c0 = rev3(g), r0 = rev3(h);
    const int kbase = p.o2_base[j1 * L + l1];
    const float scale2 = 1.f / static_cast<float>(N1C * N1C);
    // fold taps: t0 H[u][v], t1 conj H[N1C - u][N2 - v], t2 H[u + N2][v], t3 conj H[N2 - u][N2 - v]
    // with u = 8 i + r0, v = 8 k + c0; t1 / t3 based at their smallest address (offsets >= 0)
    const float2* hp0 = H + r0 * S + c0;
    const float2* hp2 = H + (r0 + N2) * S + c0;
    const float2* hp1 = H + (N1C - r0 - 8 * (R - 1)) * S + (N2 - c0 - 8 * (R - 1));
    const float2* hp3 = H + (N2 - r0 - 8 * (R - 1)) * S + (N2 - c0 - 8 * (R - 1));
#ifndef WST_O2R_SKIP
#define WST_O2R_SKIP 0   // timing ablation (variant builds): 1 no paths, 2 no FFT passes, 4 no fold
#endif
    for (int l2 = (WST_O2R_SKIP & 1) ? L : wave; l2 < L; l2 += kO2rWaves) {
        // the tap bases re-materialised per path: without this the compiler hoists every one of
        // the 4 R^2 tap addresses out of the path loop and keeps them live (hundreds of VGPRs)
        int ob0 = static_cast<int>(hp0 - H), ob1 = static_cast<int>(hp1 - H);
        int ob2 = static_cast<int>(hp2 - H), ob3 = static_cast<int>(hp3 - H);
        asm volatile("" : "+v"(ob0), "+v"(ob1), "+v"(ob2), "+v"(ob3));
        const float2* q0 = H + ob0;
        const float2* q1 = H + ob1;
        const float2* q2 = H + ob2;
        const float2* q3 = H + ob3;
        const float* fl = p.psil + p.psil_off[j1 * L + l2];
        const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(fl, R * R * 64 * 16);
        float2 v[R][R];
        if constexpr (WST_O2R_SKIP & 4) {
            wstfft::static_for<0, R * R>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                v[e / R][e % R] = q0[e * 8];
            });
        } else
        // fold, software-pipelined: the taps of element e + kFoldAhead are loaded while element e
        // is summed (scheduling barriers keep the compiler from hoisting every load of the path,
        // which would need ~12 registers per element in flight)
        {
            constexpr int NE = R * R, AH = kO2rFoldAhead, W = AH + 1, AF = kO2rFiltAhead, WF = AF + 1;
            float4 fb[WF];
            float2 hb[W][4];
            auto load_f = [&](auto ec) __attribute__((always_inline)) {
                constexpr int e = decltype(ec)::value;
                if constexpr (e < NE)
                    fb[e % WF] = __builtin_bit_cast(
                        float4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, e * 1024, 0));
            };
            auto load = [&](auto ec) __attribute__((always_inline)) {
                constexpr int e = decltype(ec)::value;
                if constexpr (e < NE) {
                    constexpr int i = e / R, k = e % R;
                    hb[e % W][0] = q0[i * 8 * S + k * 8];
                    hb[e % W][1] = q1[(R - 1 - i) * 8 * S + (R - 1 - k) * 8];
                    hb[e % W][2] = q2[i * 8 * S + k * 8];
                    hb[e % W][3] = q3[(R - 1 - i) * 8 * S + (R - 1 - k) * 8];
                }
            };
            wstfft::static_for<0, AF>(load_f);
            wstfft::static_for<0, AH>(load);
            wstfft::static_for<0, NE>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                constexpr int i = e / R, k = e % R;
                load_f(std::integral_constant<int, e + AF>{});
                load(std::integral_constant<int, e + AH>{});
                const float4 f = fb[e % WF];
                const float2 h0 = hb[e % W][0], h1 = hb[e % W][1], h2 = hb[e % W][2], h3 = hb[e % W][3];
                v[i][k].x = fmaf(h0.x, f.x, fmaf(h1.x, f.y, fmaf(h2.x, f.z, h3.x * f.w)));
                v[i][k].y = fmaf(h0.y, f.x, fmaf(-h1.y, f.y, fmaf(h2.y, f.z, -h3.y * f.w)));
                // materialise the element here (the compiler otherwise sinks the products to the
                // row pass and keeps every tap of the path live)
                pin(v[i][k]);
                __builtin_amdgcn_sched_barrier(0);
            });
        }
        if constexpr (!(WST_O2R_SKIP & 2)) {
        // row pass: DFT-R in lane along k, then per output n1 the twiddle w_n^(n1 rev(g)) and the
        // DFT-8 across the g lanes (one twiddle live at a time)
        {
            const PassConst pc = pass_const<R>(tw2, g);
            wstfft::static_for<0, R>([&](auto ic) { wstfft::rfft<R, true>(v[decltype(ic)::value]); });
            wstfft::static_for<0, R>([&](auto nc) {
                constexpr int n1 = decltype(nc)::value;
                const float2 tw = pass_tw(tw2, n1, c0);
                wstfft::static_for<0, R>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    float2 t = v[i][n1];
                    if constexpr (n1 > 0) t = cmulf(t, tw);
                    v[i][n1] = xlane8<0, 1, 2>(t, pc);
                    pin(v[i][n1]);
                    if constexpr (i % kO2rChain == kO2rChain - 1) __builtin_amdgcn_sched_barrier(0);
                });
            });
        }
        // column pass: DFT-R in lane along i, twiddle, DFT-8 across the h lanes
        {
            const PassConst pc = pass_const<R>(tw2, h);
            wstfft::static_for<0, R>([&](auto nc) {
                constexpr int n1 = decltype(nc)::value;
                float2 col[R];
                wstfft::static_for<0, R>([&](auto ic) { col[decltype(ic)::value] = v[decltype(ic)::value][n1]; });
                wstfft::rfft<R, true>(col);
                wstfft::static_for<0, R>([&](auto ic) { v[decltype(ic)::value][n1] = col[decltype(ic)::value]; });
            });
            wstfft::static_for<0, R>([&](auto mc) {
                constexpr int m1 = decltype(mc)::value;
                const float2 tw = pass_tw(tw2, m1, r0);
                wstfft::static_for<0, R>([&](auto nc) {
                    constexpr int n1 = decltype(nc)::value;
                    float2 t = v[m1][n1];
                    if constexpr (m1 > 0) t = cmulf(t, tw);
                    v[m1][n1] = xlane8<3, 4, 5>(t, pc);
                    pin(v[m1][n1]);
                    if constexpr (n1 % kO2rChain == kO2rChain - 1) __builtin_amdgcn_sched_barrier(0);
                });
            });
        }
        }
        // |.| and the low-pass at the kept points: lane holds rows m1 + R h, columns n1 + R g
        float P[16];
        {
            float T[R][4];
            wstfft::static_for<0, R>([&](auto mc) {
                constexpr int m1 = decltype(mc)::value;
                T[m1][0] = T[m1][1] = T[m1][2] = T[m1][3] = 0.f;
                wstfft::static_for<0, R>([&](auto nc) {
                    constexpr int n1 = decltype(nc)::value;
                    const float2 z = v[m1][n1];
                    const float m = __builtin_amdgcn_sqrtf(fmaf(z.x, z.x, z.y * z.y));
                    const float4 gn = *reinterpret_cast<const float4*>(GN + (n1 + R * g) * 4);
                    T[m1][0] = fmaf(gn.x, m, T[m1][0]);
                    T[m1][1] = fmaf(gn.y, m, T[m1][1]);
                    T[m1][2] = fmaf(gn.z, m, T[m1][2]);
                    T[m1][3] = fmaf(gn.w, m, T[m1][3]);
                });
            });
            wstfft::static_for<0, 16>([&](auto ic) { P[decltype(ic)::value] = 0.f; });
            wstfft::static_for<0, R>([&](auto mc) {
                constexpr int m1 = decltype(mc)::value;
                const float4 gm = *reinterpret_cast<const float4*>(GM + (m1 + R * h) * 4);
                const float ga[4] = {gm.x * scale2, gm.y * scale2, gm.z * scale2, gm.w * scale2};
                wstfft::static_for<0, 16>([&](auto ic) {
                    constexpr int o = decltype(ic)::value;
                    P[o] = fmaf(ga[o / 4], T[m1][o % 4], P[o]);
                });
            });
        }
        const int idx0 = Reduce16::run(P, lane);
        o2r_emit(P[0], idx0, lane, img, p.K, kbase + l2, out, pooled);
    }
}

}  // namespace wstdev
