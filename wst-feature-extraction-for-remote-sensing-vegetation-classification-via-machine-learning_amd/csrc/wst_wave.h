// k_o2r: every order-2 path of an LDS-resident level j1 held in the registers of ONE wave -- no
// LDS batches and no workgroup barrier once the U1 spectrum is in place.  The headline geometry
// (64^2 patches, J = 4, P = 96): per (plane, theta1) at j1 = 0 the 8 paths of 48 x 48, 8 of 24 x 24
// and 8 of 12 x 12; at j1 = 1 the 8 of 24 x 24 and 8 of 12 x 12.  Wave w runs theta2 = w of every
// level.
//
// Same cascade as k_o2 (kymatio 0.3.0 scattering2d, SURVEY.md Appendix A.4: U1hat * psi_{j2,l2}
// -> periodize by s = 2^(j2 - j1) -> ifft2 -> |.| -> phi low-pass + subsample + unpad), replacing
// the reference calls reached from src/training/train_and_save_model.py:364-368.
//
// Layout of one n x n path (n = G R) on a G x G lane grid (G = 8: the 64 lanes; G = 4: 16 lanes,
// with the 4 lane groups of the wave splitting the fold's alias rows): lane (h, g) holds the R x R
// elements (i, k) -> B[G i + rev(h)][G k + rev(g)] (rev = bit reversal over log2 G bits).  A line
// transform of length n = R G is an in-lane DFT-R, the twiddle w_n^(n1 rev(g)) and a DFT-G across
// the G lanes of the line (radix-2 DIT, bit-reversed lane input, natural lane output), so output
// element (i, n1) of lane g is column n1 + R g.  Cross-lane partners, one instruction each:
//   G = 8: row pass over g: xor 1, xor 2 (DPP quad_perm), xor 7 (DPP row_half_mirror) with
//          b0 = g0 ^ g2, b1 = g1 ^ g2, b2 = g2; column pass over h = (b3, b4, b5): DPP row_ror:8,
//          v_permlane16_swap, v_permlane32_swap;
//   G = 4: row pass over g: xor 1, xor 2; column pass over h: xor 7, xor 8 (g0 = b0 ^ b2,
//          g1 = b1 ^ b2, h0 = b2, h1 = b3).
// A butterfly stage is y = r_own + beta * r_partner on premultiplied values r (beta = -1 on the
// lanes of the odd half, which then hold the negated output -- a per-lane sign that the next
// stage's premultiplier absorbs and the modulus removes).
//
// The fold (dense over the s x s aliases) reads its spectrum taps from the Hermitian half spectrum
// in LDS at compile-time offsets from two per-lane bases (direct columns for alias b < s / 2, the
// conjugate mirror for b >= s / 2) and its filter taps, four per 16-byte load, from a lane-ordered
// table (host: psil).  The modulus and the separable low-pass (natural tap matrices) run on the
// final layout (rows m1 + R h, columns n1 + R g), then a halving reduction over the grid's lanes.
#pragma once

#include "wst_device.h"

namespace wstdev {

// ---------------------------------------------------------------------------------------------
// lane roles (shared with the host table builder)
// ---------------------------------------------------------------------------------------------
__host__ __device__ constexpr int rev3(int x) { return ((x & 1) << 2) | (x & 2) | ((x >> 2) & 1); }
__host__ __device__ constexpr int rev2(int x) { return ((x & 1) << 1) | ((x >> 1) & 1); }
// logical row-pass index g and column-pass index h of hardware lane `lane` on a G x G grid
__host__ __device__ inline int o2r_g(int lane, int G) {
    const int b0 = lane & 1, b1 = (lane >> 1) & 1, b2 = (lane >> 2) & 1;
    return G == 8 ? (b0 ^ b2) | ((b1 ^ b2) << 1) | (b2 << 2) : (b0 ^ b2) | ((b1 ^ b2) << 1);
}
__host__ __device__ inline int o2r_h(int lane, int G) { return G == 8 ? (lane >> 3) & 7 : (lane >> 2) & 3; }
__host__ __device__ inline int o2r_rev(int x, int G) { return G == 8 ? rev3(x) : rev2(x); }
// lane grid of a path level n2: G = 8 for n2 = 8 R (R = 3, 6), G = 4 for n2 = 12 (R = 3)
__host__ __device__ constexpr int o2r_grid(int n2) { return n2 == 12 ? 4 : 8; }
// level sizes k_o2r is compiled for (the first order-2 level n1 / 2 and its halvings down to 12)
__host__ __device__ constexpr bool o2r_size(int n1c) { return n1c == 96 || n1c == 48; }
// the paths of level j1 + d (d >= 1) that k_o2r runs for N1C: n2 = N1C >> d >= 12
__host__ __device__ constexpr int o2r_depth(int n1c) { return n1c == 96 ? 3 : n1c == 48 ? 2 : 0; }
// LDS row stride (complex) of the spectrum: >= N1C / 2 + 1 and = 4 mod 16, so the 32 lanes of a
// ds_read_b64 half (4 row groups x 8 column groups) hit 32 distinct bank pairs
__host__ __device__ constexpr int o2r_stride(int n1c) {
    int s = n1c / 2 + 1;
    while (s % 16 != 4) ++s;
    return s;
}
// per path level d = 1 .. depth: twiddles (n2 complex), GM and GN (n2 rows of 4 floats)
__host__ __device__ constexpr int o2r_level_bytes(int n1c, int depth) {
    int b = 0;
    for (int d = 1; d <= depth; ++d) b += (n1c >> d) * (8 + 32);
    return b;
}
// LDS bytes of k_o2r: spectrum (N1C + 1 rows; row N1C repeats row 0), twiddles of level j1, the
// per-level tables
__host__ __device__ constexpr int o2r_lds(int n1c) {
    return (n1c + 1) * o2r_stride(n1c) * 8 + n1c * 8 + o2r_level_bytes(n1c, o2r_depth(n1c));
}
// filter taps per element and lane of a path level: s^2 / (alias groups)
__host__ __device__ constexpr int o2r_taps(int n1c, int n2) {
    return o2r_grid(n2) == 4 ? 4 : (n1c / n2) * (n1c / n2);   // 4 x 4 grids: the windowed fold
}
constexpr int kO2rWaves = 8;   // waves per workgroup: one theta2 each
#ifndef WST_O2R_AHEAD
#define WST_O2R_AHEAD 2
#endif
constexpr int kO2rFoldAhead = WST_O2R_AHEAD;   // fold steps whose spectrum taps are in flight
#ifndef WST_O2R_FAHEAD
#define WST_O2R_FAHEAD 2
#endif
constexpr int kO2rFiltAhead = WST_O2R_FAHEAD;  // fold steps whose filter taps are in flight
#ifndef WST_O2R_AHEAD_S
#define WST_O2R_AHEAD_S 4
#endif
#ifndef WST_O2R_FAHEAD_S
#define WST_O2R_FAHEAD_S 6
#endif
constexpr int kO2rFoldAheadSmall = WST_O2R_AHEAD_S;   // the same for the R = 3 levels
constexpr int kO2rFiltAheadSmall = WST_O2R_FAHEAD_S;
#ifndef WST_O2R_CHAIN
#define WST_O2R_CHAIN 2
#endif
constexpr int kO2rChain = WST_O2R_CHAIN;   // cross-lane butterfly chains scheduled together
#ifndef WST_O2R_LEVELS
#define WST_O2R_LEVELS 7   // timing ablation (variant builds): path levels d = 1, 2, 3 as bits
#endif
#ifndef WST_O2R_SKIP
#define WST_O2R_SKIP 0   // timing ablation (variant builds): 1 no paths, 2 no FFT passes, 4 no fold
#endif

// ---------------------------------------------------------------------------------------------
// cross-lane exchange
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    // bound_ctrl: every source lane is valid here; lets the compiler drop the "old" operand
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                                 0xF, 0xF, true));
}
// partner exchange ops: 0 xor 1, 1 xor 2, 2 xor 7 (row_half_mirror), 3 xor 8 (row_ror:8),
// 4 xor 16 (permlane16 swap), 5 xor 32 (permlane32 swap)
template <int OP>
__device__ __forceinline__ float bfly1(float own, float beta) {
    if constexpr (OP <= 3) {
        constexpr int ctrl = OP == 0 ? 0xB1 : OP == 1 ? 0x4E : OP == 2 ? 0x141 : 0x128;
        return fmaf(dpp_f<ctrl>(own), beta, own);   // own + beta * partner
    } else {
        // the swap hands every lane the values of both members (lo: bit clear, hi: bit set);
        // own + beta * partner = hi + beta * lo
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
}
template <int OP>
__device__ __forceinline__ float2 bfly(float2 v, float beta) {
    return make_float2(bfly1<OP>(v.x, beta), bfly1<OP>(v.y, beta));
}
// Materialise v here: keeps the compiler from sinking a value's last operations to its far use
// and holding their operands live meanwhile.
__device__ __forceinline__ void pin(float2& v) { asm volatile("" : "+v"(v.x), "+v"(v.y)); }
__device__ __forceinline__ float2 cmulf(float2 a, float2 w) {
    return make_float2(fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x));
}

// Per-lane constants of one pass (inverse transform of length n = G R over the lane index q):
// stage premultipliers c1, c2 and the stage signs.
struct PassConst {
    float2 c1, c2;
    float beta0, beta1, beta2;
};
// tw2: forward twiddles exp(-2 pi i k / n) of the path level in LDS (inverse = conjugate)
template <int N>
__device__ __forceinline__ PassConst pass_const(const float2* tw2, int q) {
    PassConst c;
    const int q0 = q & 1, q1 = (q >> 1) & 1, q2 = (q >> 2) & 1;
    c.beta0 = q0 ? -1.f : 1.f;
    c.beta1 = q1 ? -1.f : 1.f;
    c.beta2 = q2 ? -1.f : 1.f;
    // stage 1: lanes with q1 premultiply by w_4^(q0); all by the stage-0 sign
    const float2 w4 = tw2[q0 * (N / 4)];
    c.c1 = q1 ? make_float2(c.beta0 * w4.x, -c.beta0 * w4.y) : make_float2(c.beta0, 0.f);
    // stage 2 (G = 8): lanes with q2 premultiply by w_8^(q0 + 2 q1); all by the stage-1 sign
    const float2 w8 = tw2[((q0 + 2 * q1) * (N / 8)) % N];
    c.c2 = q2 ? make_float2(c.beta1 * w8.x, -c.beta1 * w8.y) : make_float2(c.beta1, 0.f);
    return c;
}
// in-lane twiddle w_n^(n1 c0) of output n1 (inverse: conjugate of the forward table)
__device__ __forceinline__ float2 pass_tw(const float2* tw2, int n1, int c0) {
    const float2 t = tw2[n1 * c0];
    return make_float2(t.x, -t.y);
}
// Inverse DFT-G across the lanes of the line on one value: stage ops S0, S1 (, S2 for G = 8).
template <int G, int S0, int S1, int S2>
__device__ __forceinline__ float2 xlane(float2 v, const PassConst& c) {
    v = bfly<S0>(v, c.beta0);
    v = bfly<S1>(cmulf(v, c.c1), c.beta1);
    if constexpr (G == 8) v = bfly<S2>(cmulf(v, c.c2), c.beta2);
    return v;
}

// ---------------------------------------------------------------------------------------------
// halving reduction of 16 per-lane values over a grid's lanes and the map emit (4 x 4 maps)
// ---------------------------------------------------------------------------------------------
template <int D>
__device__ __forceinline__ float lane_swap(float v) {
    if constexpr (D == 1) return dpp_f<0xB1>(v);
    else if constexpr (D == 2) return dpp_f<0x4E>(v);
    else if constexpr (D == 4) return dpp_f<0x141>(v);   // row_half_mirror: pairs across bit 2
    else if constexpr (D == 8) return dpp_f<0x128>(v);   // row_ror:8 = xor 8
    else return __shfl_xor(v, D, 64);
}
// Halving from distance D0 down: a lane keeps the half of its values selected by its lane bit D
// and adds the partner's copy of that half; once one value is left, the remaining distances add.
// G = 8 (D0 = 32): every lane ends with one of the 16 sums over the 64 lanes, lanes that differ
// only in bits 0, 1 holding the same one.  G = 4 (D0 = 8): one distinct sum over the 16 lanes of
// the lane group per lane.
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
    template <int G>
    static __device__ __forceinline__ int run(float (&P)[16], int lane) {
        int idx0 = 0;
        step<G == 8 ? 32 : 8, 16>(P, lane, idx0);
        return idx0;
    }
};

// One 4 x 4 map (coefficient k0 of plane img) from the reduced values: value idx0 in v.
template <int G>
__device__ __forceinline__ void o2r_emit(float v, int idx0, int lane, long long img, int K, int k0,
                                         float* __restrict__ out, int pooled) {
    // G = 8: lanes 0, 4, ..., 60 hold the 16 distinct values; G = 4: lanes 0 .. 15 do
    constexpr int MASK = G == 8 ? 3 : 48;
    if (!pooled) {
        if ((lane & MASK) == 0) __builtin_nontemporal_store(v, out + (img * K + k0) * 16 + idx0);
        return;
    }
    float s = v;
    if constexpr (G == 4) {
        s += lane_swap<1>(s);
        s += lane_swap<2>(s);
    }
    s += lane_swap<4>(s);
    s += lane_swap<8>(s);
    if constexpr (G == 8) {
        s += lane_swap<16>(s);
        s += lane_swap<32>(s);
    }
    const float mean = s * (1.f / 16.f);
    const float d = v - mean;
    float q = d * d;
    if constexpr (G == 4) {
        q += lane_swap<1>(q);
        q += lane_swap<2>(q);
    }
    q += lane_swap<4>(q);
    q += lane_swap<8>(q);
    if constexpr (G == 8) {
        q += lane_swap<16>(q);
        q += lane_swap<32>(q);
    }
    if (lane == 0) {
        out[img * 2 * K + k0] = mean;
        out[img * 2 * K + K + k0] = sqrtf(q * (1.f / 16.f));
    }
}

// ---------------------------------------------------------------------------------------------
// one path of level n2 in a wave
// ---------------------------------------------------------------------------------------------
// N1C: level j1 size; N2: path level size.  Hs: the half spectrum in LDS (row stride S, row N1C =
// row 0); fl: the path's lane-ordered filter taps; tw2 / GM / GN: the path level's tables in LDS.
template <int N1C, int N2>
__device__ __forceinline__ void o2r_path(const float2* Hs, const float* __restrict__ fl, int win,
                                         const float2* tw2, const float* GM, const float* GN, int lane,
                                         long long img, int K, int k0, float* __restrict__ out, int pooled) {
    constexpr int G = o2r_grid(N2), R = N2 / G, S = o2r_stride(N1C), SS = N1C / N2;
    constexpr int NG = G == 4 ? 4 : 1;          // alias groups (lane bits 4, 5 when G = 4)
    constexpr int SA = SS / NG;                 // alias rows per group (dense fold)
    constexpr int T = G == 4 ? 4 : SA * SS, T4 = T / 4;   // filter taps per element, float4 loads
    static_assert(T % 4 == 0 && R * G == N2, "k_o2r level");
    const int g = o2r_g(lane, G), h = o2r_h(lane, G);
    const int c0 = o2r_rev(g, G), r0 = o2r_rev(h, G);
    const int ag = NG > 1 ? lane >> 4 : 0;       // alias group: rows a = ag SA + a'
    // tap bases (complex units), re-materialised per path: without this the compiler hoists every
    // tap address out of the path loop and keeps them live
    //   direct (alias b < SS / 2): H[u + N2 a][v + N2 b], u = G i + r0, v = G k + c0
    //   mirror (b >= SS / 2): conj H[N1C - u - N2 a][N1C - v - N2 b], based at its smallest
    //   address (i = R - 1, a' = SA - 1, k = R - 1, b = SS - 1) so every offset is >= 0
    int od = (r0 + N2 * SA * ag) * S + c0;
    int om = (N1C - r0 - N2 * SA * ag - G * (R - 1) - N2 * (SA - 1)) * S + (N1C - c0 - G * (R - 1) - N2 * (SS - 1));
    asm volatile("" : "+v"(od), "+v"(om));
    const float2* qd = Hs + od;
    const float2* qm = Hs + om;
    const __amdgpu_buffer_rsrc_t rs = uniform_rsrc(fl, R * R * T4 * 1024);
    float2 v[R][R];
    if constexpr (WST_O2R_SKIP & 4) {
        wstfft::static_for<0, R * R>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e / R][e % R] = qd[e * 8];
        });
    } else if constexpr (G == 4) {
        // windowed fold (the 12 x 12 paths: s = 4 or 8, filters compact): the filter's significant
        // bins lie in a window of 4 x 4 alias tiles starting at tile (alpha, beta) (host: psil_win;
        // a band of width n2 in each direction at most 3 tiles long, plus the offset within a tile).
        // Lane group ag takes alias row rho = alpha + ag, every lane the 4 alias columns
        // kappa_j = beta + j (mod s); whether column kappa_j is read direct or as the conjugate
        // mirror is wave-uniform.
        const int alpha = win & 255, beta = win >> 8;
        const int rho = (alpha + ag) & (SS - 1);
        int wd = (r0 + N2 * rho) * S + c0;
        int wm = (N1C - r0 - N2 * rho - G * (R - 1)) * S + (N1C - c0 - G * (R - 1));
        float4 f[R * R];
        wstfft::static_for<0, R * R>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            f[e] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, e * 1024, 0));
        });
        wstfft::static_for<0, R * R>([&](auto ec) { v[decltype(ec)::value / R][decltype(ec)::value % R] = make_float2(0.f, 0.f); });
        wstfft::static_for<0, 4>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            const int kappa = (beta + j) & (SS - 1);
            float2 hv[R * R];
            float sg;
            if (2 * kappa < SS) {
                const float2* q = Hs + (wd + N2 * kappa);
                wstfft::static_for<0, R * R>([&](auto ec) {
                    constexpr int e = decltype(ec)::value;
                    hv[e] = q[G * (e / R) * S + G * (e % R)];
                });
                sg = 1.f;
            } else {
                const float2* q = Hs + (wm - N2 * kappa);
                wstfft::static_for<0, R * R>([&](auto ec) {
                    constexpr int e = decltype(ec)::value;
                    hv[e] = q[G * (R - 1 - e / R) * S + G * (R - 1 - e % R)];
                });
                sg = -1.f;
            }
            wstfft::static_for<0, R * R>([&](auto ec) {
                constexpr int e = decltype(ec)::value;
                const float fj = j == 0 ? f[e].x : j == 1 ? f[e].y : j == 2 ? f[e].z : f[e].w;
                float2& a = v[e / R][e % R];
                a.x = fmaf(hv[e].x, fj, a.x);
                a.y = fmaf(sg * hv[e].y, fj, a.y);
            });
        });
    } else {
        // fold, software-pipelined over the steps (element e, tap quad t4): the taps of step
        // q + ahead are loaded while step q is summed (scheduling barriers keep the compiler from
        // hoisting every load of the path)
        // (the small levels hold 9 elements, so their registers allow deeper pipelines)
        constexpr int NQ = R * R * T4, AH = R > 3 ? kO2rFoldAhead : kO2rFoldAheadSmall, W = AH + 1;
        constexpr int AF = R > 3 ? kO2rFiltAhead : kO2rFiltAheadSmall, WF = AF + 1;
        float4 fb[WF];
        float2 hb[W][4];
        auto load_f = [&](auto qc) __attribute__((always_inline)) {
            constexpr int q = decltype(qc)::value;
            if constexpr (q < NQ)
                fb[q % WF] = __builtin_bit_cast(
                    float4, __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16, q * 1024, 0));
        };
        auto load_h = [&](auto qc) __attribute__((always_inline)) {
            constexpr int q = decltype(qc)::value;
            if constexpr (q < NQ) {
                constexpr int e = q / T4, t4 = q % T4, i = e / R, k = e % R;
                wstfft::static_for<0, 4>([&](auto tc) {
                    constexpr int t = 4 * t4 + decltype(tc)::value;
                    constexpr int a = t / SS, b = t % SS;   // a: alias row within the group
                    if constexpr (2 * b < SS)
                        hb[q % W][t % 4] = qd[(G * i + N2 * a) * S + G * k + N2 * b];
                    else
                        hb[q % W][t % 4] = qm[(G * (R - 1 - i) + N2 * (SA - 1 - a)) * S +
                                              G * (R - 1 - k) + N2 * (SS - 1 - b)];
                });
            }
        };
        wstfft::static_for<0, AF>(load_f);
        wstfft::static_for<0, AH>(load_h);
        wstfft::static_for<0, NQ>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            constexpr int e = q / T4, t4 = q % T4, i = e / R, k = e % R;
            load_f(std::integral_constant<int, q + AF>{});
            load_h(std::integral_constant<int, q + AH>{});
            const float4 f4 = fb[q % WF];
            const float f[4] = {f4.x, f4.y, f4.z, f4.w};
            float2 acc = t4 == 0 ? make_float2(0.f, 0.f) : v[i][k];
            wstfft::static_for<0, 4>([&](auto tc) {
                constexpr int t = 4 * t4 + decltype(tc)::value;
                constexpr int b = t % SS;
                const float2 hv = hb[q % W][t % 4];
                acc.x = fmaf(hv.x, f[t % 4], acc.x);
                acc.y = fmaf(2 * b < SS ? hv.y : -hv.y, f[t % 4], acc.y);   // mirror taps: conj
            });
            v[i][k] = acc;
            // materialise the element here (the compiler otherwise sinks the products to the
            // row pass and keeps every tap of the path live)
            pin(v[i][k]);
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    if constexpr (NG > 1) {
        // the alias groups' partial folds: sum over lane bits 4 and 5 (every group ends with it)
        wstfft::static_for<0, R * R>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e / R][e % R] = bfly<5>(bfly<4>(v[e / R][e % R], 1.f), 1.f);
        });
    }
    if constexpr (!(WST_O2R_SKIP & 2)) {
        // row pass: DFT-R in lane along k, then per output n1 the twiddle w_n^(n1 rev(g)) and the
        // DFT-G across the g lanes (one twiddle live at a time)
        constexpr int RS0 = 0, RS1 = 1, RS2 = 2;            // xor 1, xor 2, xor 7
        constexpr int CS0 = G == 8 ? 3 : 2, CS1 = G == 8 ? 4 : 3, CS2 = 5;
        {
            const PassConst pc = pass_const<N2>(tw2, g);
            wstfft::static_for<0, R>([&](auto ic) { wstfft::rfft<R, true>(v[decltype(ic)::value]); });
            wstfft::static_for<0, R>([&](auto nc) {
                constexpr int n1 = decltype(nc)::value;
                const float2 tw = pass_tw(tw2, n1, c0);
                wstfft::static_for<0, R>([&](auto ic) {
                    constexpr int i = decltype(ic)::value;
                    float2 t = v[i][n1];
                    if constexpr (n1 > 0) t = cmulf(t, tw);
                    v[i][n1] = xlane<G, RS0, RS1, RS2>(t, pc);
                    pin(v[i][n1]);
                    if constexpr (i % kO2rChain == kO2rChain - 1) __builtin_amdgcn_sched_barrier(0);
                });
            });
        }
        // column pass: DFT-R in lane along i, twiddle, DFT-G across the h lanes
        {
            const PassConst pc = pass_const<N2>(tw2, h);
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
                    v[m1][n1] = xlane<G, CS0, CS1, CS2>(t, pc);
                    pin(v[m1][n1]);
                    if constexpr (n1 % kO2rChain == kO2rChain - 1) __builtin_amdgcn_sched_barrier(0);
                });
            });
        }
    }
    // |.| and the low-pass at the kept points: lane holds rows m1 + R h, columns n1 + R g
    float P[16];
    {
        constexpr float scale2 = 1.f / static_cast<float>(N1C * N1C);
        float T4v[R][4];
        wstfft::static_for<0, R>([&](auto mc) {
            constexpr int m1 = decltype(mc)::value;
            T4v[m1][0] = T4v[m1][1] = T4v[m1][2] = T4v[m1][3] = 0.f;
            wstfft::static_for<0, R>([&](auto nc) {
                constexpr int n1 = decltype(nc)::value;
                const float2 z = v[m1][n1];
                const float m = __builtin_amdgcn_sqrtf(fmaf(z.x, z.x, z.y * z.y));
                const float4 gn = *reinterpret_cast<const float4*>(GN + (n1 + R * g) * 4);
                T4v[m1][0] = fmaf(gn.x, m, T4v[m1][0]);
                T4v[m1][1] = fmaf(gn.y, m, T4v[m1][1]);
                T4v[m1][2] = fmaf(gn.z, m, T4v[m1][2]);
                T4v[m1][3] = fmaf(gn.w, m, T4v[m1][3]);
            });
        });
        wstfft::static_for<0, 16>([&](auto ic) { P[decltype(ic)::value] = 0.f; });
        wstfft::static_for<0, R>([&](auto mc) {
            constexpr int m1 = decltype(mc)::value;
            const float4 gm = *reinterpret_cast<const float4*>(GM + (m1 + R * h) * 4);
            const float ga[4] = {gm.x * scale2, gm.y * scale2, gm.z * scale2, gm.w * scale2};
            wstfft::static_for<0, 16>([&](auto ic) {
                constexpr int o = decltype(ic)::value;
                P[o] = fmaf(ga[o / 4], T4v[m1][o % 4], P[o]);
            });
        });
    }
    const int idx0 = Reduce16::run<G>(P, lane);
    o2r_emit<G>(P[0], idx0, lane, img, K, k0, out, pooled);
}

// ---------------------------------------------------------------------------------------------
// the kernel
// ---------------------------------------------------------------------------------------------
// One workgroup of 8 waves per (plane, theta1) at level j1 (N1C x N1C, square family FAM); 4 x 4
// output maps.  hexp: k_o1's half spectra (rows transformed, digit-reversed row order).
// nwl: path levels j1 + 1 .. j1 + nwl run wave-resident; when nwl < DEPTH the workgroup then
// runs the remaining levels j1 + nwl + 1 .. J - 1 through k_o2_body's LDS batches (layout lay2:
// the same spectrum at row stride S, a B region of its own) after one barrier -- the hybrid
// measured fastest at c2 (the wave form's dense s = 4 / 8 folds read 4x the filter bytes of
// the box-sparse batch folds).
template <int FAM, int N1C>
__global__ void __launch_bounds__(64 * kO2rWaves, 4) k_o2r(DevParams p, LdsLayout lay2, int nwl, int j1, int nimg,
                                                          long long img0, const float2* __restrict__ hexp,
                                                          float* __restrict__ out, int pooled) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int HLD = N1C / 2 + 1, S = o2r_stride(N1C), DEPTH = o2r_depth(N1C);
    constexpr int CAP = N1C <= 12 ? 12 : N1C <= 24 ? 24 : N1C <= 48 ? 48 : 136;
    static_assert(o2r_size(N1C), "k_o2r level size");
    float2* H = reinterpret_cast<float2*>(smem);
    float2* tw1 = H + (N1C + 1) * S;
    unsigned char* lvl = reinterpret_cast<unsigned char*>(tw1 + N1C);   // per path level tables
    const int L = p.L, J = p.J;
    const int item = xcd_item(nimg * L);
    const int local = item / L;
    const int l1 = item - local * L;
    const long long img = img0 + local;

    // 1. tables, then the half spectrum into LDS (row stride S) and its column FFTs
    for (int i = threadIdx.x; i < N1C; i += blockDim.x) tw1[i] = p.tw[p.tw_off[2 * j1] + i];
    {
        unsigned char* t = lvl;
        for (int d = 1; d <= DEPTH; ++d) {
            const int n2 = N1C >> d, j2 = j1 + d;
            float2* tw2 = reinterpret_cast<float2*>(t);
            float* GM = reinterpret_cast<float*>(tw2 + n2);
            float* GN = GM + n2 * 4;
            if (j2 < J) {
                for (int i = threadIdx.x; i < n2; i += blockDim.x) tw2[i] = p.tw[p.tw_off[2 * j2] + i];
                for (int i = threadIdx.x; i < n2 * 4; i += blockDim.x) {
                    GM[i] = p.lpn[p.lpn_off[2 * j2] + i];
                    GN[i] = p.lpn[p.lpn_off[2 * j2 + 1] + i];
                }
            }
            t += n2 * (8 + 32);
        }
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

    // 2. each wave: theta2 = wave, wave + 8, ... of every path level (no further barrier)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int kbase = p.o2_base[j1 * L + l1];
    // waves 4..7 take the levels in a rotated order (2, 3, 1): the two halves of the workgroup
    // are then in different phases (L2-bound folds beside VALU-bound transforms) instead of
    // reaching the same phase together
#ifndef WST_O2R_ROT
#define WST_O2R_ROT 1
#endif
    const int rot = WST_O2R_ROT && (wave >= kO2rWaves / 2) && nwl > 1 ? 1 : 0;
    for (int l2 = (WST_O2R_SKIP & 1) ? L : wave; l2 < L; l2 += kO2rWaves) {
#pragma unroll 1
        for (int step = 0; step < nwl; ++step) {
            const int d = (step + rot) % nwl + 1;
            wstfft::static_for<1, DEPTH + 1>([&](auto dc) {
                constexpr int dd = decltype(dc)::value;
                constexpr int n2 = N1C >> dd;
                const int j2 = j1 + dd;
                const float2* tw2 = reinterpret_cast<const float2*>(lvl + o2r_level_bytes(N1C, dd - 1));
                const float* GM = reinterpret_cast<const float*>(tw2 + n2);
                const float* GN = GM + n2 * 4;
                const int pi = (j1 * J + j2) * L + l2;
                if (d == dd && j2 < J && ((WST_O2R_LEVELS >> (dd - 1)) & 1))
                    o2r_path<N1C, n2>(H, p.psil + p.psil_off[pi], p.psil_win[pi], tw2, GM, GN, lane, img,
                                      p.K, kbase + (dd - 1) * L + l2, out, pooled);
            });
        }
    }
    if (nwl < DEPTH && j1 + nwl + 1 < J) {
        __syncthreads();   // every wave done with this kernel's tables (B reuses their LDS)
        k_o2_body<FAM, FAM, CAP, 1, 0, 4, true>(smem, p, lay2, j1, nimg, img0, nullptr, out, pooled, j1 + nwl + 1, S);
    }
}

}  // namespace wstdev
