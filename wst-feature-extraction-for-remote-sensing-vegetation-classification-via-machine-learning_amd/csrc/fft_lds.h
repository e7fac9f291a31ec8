// LDS-resident batched 1-D / 2-D FFTs for gfx950 (wave64).
//
// * rfft<R, INV>(x): length-R DFT of a register array, fully unrolled at compile time.  Composite
//   R: decimation-in-time Cooley-Tukey R = P*Q with compile-time twiddles (constexpr double sin/cos
//   rounded once to fp32); R in {2, 4}: hand butterflies; odd primes: symmetric direct DFT.
// * LineFFT<N, INV>: N-point transforms along lines of LDS arrays.  N <= 16 (or prime): one unit
//   per line, in place.  Otherwise the four-step split N = N1*N2:
//     stage A  unit (line, n2): DFT-N1 over elements n2 + N2*n1, times W_N^(n2*k1), in place;
//     stage B  unit (line, k1): DFT-N2 over the contiguous block N2*k1 + n2 -> stored to the
//              natural position k1 + N1*k2 (all loads of a round of lines precede its stores).
//   Lanes walk consecutive LINES: along rows the row stride is odd (conflict-free b64 access on
//   32-lane halves), along columns consecutive lines are contiguous.
//   Natural order in, natural order out; INV = unnormalised inverse.
// The per-unit bodies are __host__ __device__ so the CPU test-suite can run the exact index math
// through a sequential emulation (fft_lines_host) against numpy.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#define WST_HD __host__ __device__ __forceinline__

// Every level size of a plan is odd * 2^k (P = (M/2^J + 2) * 2^J), so kernels are instantiated
// per "size family" (the odd part of P) and compile only that family's FFTs (kMaxFamilyN bounds
// the LDS-resident sizes).  Families with compiled FFTs: 1, 3, 5, 7, 9, 11, 13, 15, 17, 27 (the
// odd parts of P for the common patch sizes: 48 -> 56 = 7 x 8 at J = 2, 96 -> 104 = 13 x 8,
// 112 -> 120 = 15 x 8, 100 -> 108 = 27 x 4 ...; others: generic DFT).
#define WST_FFT_SIZES(X) \
    X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18)  \
    X(20) X(22) X(24) X(26) X(27) X(28) X(30) X(32) X(34) X(36) X(40) X(44) X(48) X(52) X(54)      \
    X(56) X(60) X(64) X(68) X(72) X(80) X(88) X(96) X(104) X(108) X(112) X(120) X(128) X(136)

namespace wstfft {

constexpr int kMaxFamilyN = 136;

// ---------------------------------------------------------------------------------------------
// compile-time trigonometry (double), exact quarter-turn reduction from integers
// ---------------------------------------------------------------------------------------------
constexpr double kHalfPi = 1.5707963267948966192313216916397514;

constexpr double taylor_sin(double x) {
    double x2 = x * x, term = x, sum = x;
    for (int i = 1; i < 14; ++i) {
        term *= -x2 / ((2.0 * i) * (2.0 * i + 1.0));
        sum += term;
    }
    return sum;
}
constexpr double taylor_cos(double x) {
    double x2 = x * x, term = 1.0, sum = 1.0;
    for (int i = 1; i < 14; ++i) {
        term *= -x2 / ((2.0 * i - 1.0) * (2.0 * i));
        sum += term;
    }
    return sum;
}
// cos / sin of 2 pi m / n
constexpr double cos2pi(long long m, long long n) {
    const long long mm = ((m % n) + n) % n;
    const long long q = (4 * mm + n / 2) / n;  // nearest quarter turn
    const double d = kHalfPi * static_cast<double>(4 * mm - q * n) / static_cast<double>(n);
    switch (q & 3) {
        case 0: return taylor_cos(d);
        case 1: return -taylor_sin(d);
        case 2: return -taylor_cos(d);
        default: return taylor_sin(d);
    }
}
constexpr double sin2pi(long long m, long long n) {
    const long long mm = ((m % n) + n) % n;
    const long long q = (4 * mm + n / 2) / n;
    const double d = kHalfPi * static_cast<double>(4 * mm - q * n) / static_cast<double>(n);
    switch (q & 3) {
        case 0: return taylor_sin(d);
        case 1: return taylor_cos(d);
        case 2: return -taylor_sin(d);
        default: return -taylor_cos(d);
    }
}

template <int B, int E, typename F>
WST_HD void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

constexpr bool is_prime(int n) {
    if (n < 2) return false;
    for (int p = 2; p * p <= n; ++p)
        if (n % p == 0) return false;
    return true;
}
constexpr int pick_radix(int n) {  // outer radix of the register Cooley-Tukey split
    if (n % 4 == 0 && n != 4) return 4;
    for (int p = 2; p <= n; ++p)
        if (n % p == 0) return p;
    return n;
}

WST_HD float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
WST_HD float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// x * W_R^M (forward W = exp(-2 pi i / R); INV conjugates), trivial twiddles short-cut.
template <int R, int M, bool INV>
WST_HD float2 twiddle(float2 x) {
    constexpr int m = ((M % R) + R) % R;
    if constexpr (m == 0) {
        return x;
    } else if constexpr (2 * m == R) {
        return make_float2(-x.x, -x.y);
    } else if constexpr (4 * m == R) {  // forward: -i, inverse: +i
        return INV ? make_float2(-x.y, x.x) : make_float2(x.y, -x.x);
    } else if constexpr (4 * m == 3 * R) {  // forward: +i, inverse: -i
        return INV ? make_float2(x.y, -x.x) : make_float2(-x.y, x.x);
    } else {
        constexpr float c = static_cast<float>(cos2pi(m, R));
        constexpr float s = static_cast<float>(INV ? sin2pi(m, R) : -sin2pi(m, R));
        return make_float2(fmaf(x.x, c, -x.y * s), fmaf(x.x, s, x.y * c));
    }
}

template <int R, bool INV>
WST_HD void rfft(float2 (&x)[R]) {
    if constexpr (R == 1) {
        return;
    } else if constexpr (R == 2) {
        const float2 t = x[0];
        x[0] = cadd(t, x[1]);
        x[1] = csub(t, x[1]);
    } else if constexpr (R == 4) {
        const float2 a0 = cadd(x[0], x[2]), a1 = csub(x[0], x[2]);
        const float2 b0 = cadd(x[1], x[3]), b1 = csub(x[1], x[3]);
        const float2 rb1 = INV ? make_float2(-b1.y, b1.x) : make_float2(b1.y, -b1.x);
        x[0] = cadd(a0, b0);
        x[2] = csub(a0, b0);
        x[1] = cadd(a1, rb1);
        x[3] = csub(a1, rb1);
    } else if constexpr (is_prime(R)) {
        // symmetric direct DFT: a_n = x_n + x_{R-n}, b_n = x_n - x_{R-n}
        constexpr int H = (R - 1) / 2;
        float2 a[H + 1], b[H + 1];
        const float2 x0 = x[0];
        float2 sum = x0;
        static_for<1, H + 1>([&](auto nc) {
            constexpr int n = decltype(nc)::value;
            a[n] = cadd(x[n], x[R - n]);
            b[n] = csub(x[n], x[R - n]);
            sum = cadd(sum, a[n]);
        });
        static_for<1, H + 1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            float tr = x0.x, ti = x0.y, ur = 0.f, ui = 0.f;
            static_for<1, H + 1>([&](auto nc) {
                constexpr int n = decltype(nc)::value;
                constexpr float c = static_cast<float>(cos2pi(static_cast<long long>(n) * k, R));
                constexpr float s = static_cast<float>(sin2pi(static_cast<long long>(n) * k, R));
                tr = fmaf(a[n].x, c, tr);
                ti = fmaf(a[n].y, c, ti);
                ur = fmaf(b[n].x, s, ur);
                ui = fmaf(b[n].y, s, ui);
            });
            // forward: X[k] = t - i u, X[R-k] = t + i u ; inverse swaps the signs
            if constexpr (!INV) {
                x[k] = make_float2(tr + ui, ti - ur);
                x[R - k] = make_float2(tr - ui, ti + ur);
            } else {
                x[k] = make_float2(tr - ui, ti + ur);
                x[R - k] = make_float2(tr + ui, ti - ur);
            }
        });
        x[0] = sum;
    } else {
        constexpr int P = pick_radix(R);
        constexpr int Q = R / P;
        float2 y[P][Q];
        static_for<0, P>([&](auto pc) {
            constexpr int p = decltype(pc)::value;
            static_for<0, Q>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                y[p][q] = x[p + P * q];
            });
            rfft<Q, INV>(y[p]);
        });
        static_for<0, Q>([&](auto k1c) {
            constexpr int k1 = decltype(k1c)::value;
            float2 z[P];
            static_for<0, P>([&](auto pc) {
                constexpr int p = decltype(pc)::value;
                z[p] = twiddle<R, p * k1, INV>(y[p][k1]);
            });
            rfft<P, INV>(z);
            static_for<0, P>([&](auto k2c) {
                constexpr int k2 = decltype(k2c)::value;
                x[k1 + Q * k2] = z[k2];
            });
        });
    }
}

// ---------------------------------------------------------------------------------------------
// four-step line transforms
// ---------------------------------------------------------------------------------------------
constexpr int split_n2(int n) {  // N2 = largest divisor <= sqrt(n); 1 means a single stage
    if (n <= 16 || is_prime(n)) return 1;
    int best = 1;
    for (int d = 2; d * d <= n; ++d)
        if (n % d == 0) best = d;
    return best;
}

WST_HD float2 cmul_tw(float2 a, float2 w, bool conj) {
    const float wy = conj ? -w.y : w.y;
    return make_float2(fmaf(a.x, w.x, -a.y * wy), fmaf(a.x, wy, a.y * w.x));
}

// Exact division by a runtime divisor d (1 <= d < 2^20) for 0 <= x < 2^31 as one mul-hi, one add
// and one shift (round-up magic number, as in PyTorch's IntDivider); replaces the ~20-instruction
// integer division the compiler emits for a runtime divisor in the per-unit index decode.
// m = floor(2^32 (2^sh - d) / d) + 1 with 2^sh >= d; 2^32 (2^sh - d) < 2^52, exact in uint64.
constexpr unsigned fastdiv_magic(int d, int sh) {
    return static_cast<unsigned>(((1ull << 32) * ((1ull << sh) - static_cast<unsigned long long>(d))) /
                                 static_cast<unsigned long long>(d)) + 1u;
}
constexpr int fastdiv_shift(int d) {
    int sh = 0;
    while ((1 << sh) < d) ++sh;
    return sh;
}
// Device-side magics of every divisor up to kFastDivTab, built at compile time: a FastDiv built
// in a kernel is then a clz plus one (uniform, scalar) table load instead of a double-precision
// division (which the kernels' per-batch Lines / decode set-ups executed dozens of times per
// workgroup).
constexpr int kFastDivTab = 16384;
struct FastDivTable {
    unsigned m[kFastDivTab + 1];
};
constexpr FastDivTable make_fastdiv_table() {
    FastDivTable t{};
    for (int d = 1; d <= kFastDivTab; ++d) t.m[d] = fastdiv_magic(d, fastdiv_shift(d));
    return t;
}
#if defined(__HIP_DEVICE_COMPILE__)
__device__ static const FastDivTable kFastDivMagic = make_fastdiv_table();
#endif

struct FastDiv {
    unsigned m = 1;
    int sh = 0;
    WST_HD FastDiv() {}
    WST_HD explicit FastDiv(int d) {
#if defined(__HIP_DEVICE_COMPILE__)
        sh = d > 1 ? 32 - __clz(d - 1) : 0;
        // beyond the table (not met by the LDS-resident kernels): the double quotient is exact
        // to the floor for d < 2^20
        m = d <= kFastDivTab ? kFastDivMagic.m[d]
                             : static_cast<unsigned>(4294967296.0 * static_cast<double>((1 << sh) - d) /
                                                     static_cast<double>(d)) + 1u;
#else
        sh = fastdiv_shift(d);
        m = fastdiv_magic(d, sh);
#endif
    }
    WST_HD int div(int x) const {
#if defined(__HIP_DEVICE_COMPILE__)
        const unsigned t = __umulhi(static_cast<unsigned>(x), m);
#else
        const unsigned t = static_cast<unsigned>((static_cast<unsigned long long>(x) * m) >> 32);
#endif
        return static_cast<int>((t + static_cast<unsigned>(x)) >> sh);
    }
};

// Geometry of a batch of lines: line (b, l) element e at base[b*bs + l*ls + e*es].
struct Lines {
    int nb, bs, nl, ls, es;
    FastDiv dnl, dlines;  // / nl and / (nb * nl)
    WST_HD Lines(int nb_, int bs_, int nl_, int ls_, int es_)
        : nb(nb_), bs(bs_), nl(nl_), ls(ls_), es(es_), dnl(nl_), dlines(nb_ * nl_) {}
    WST_HD int nlines() const { return nb * nl; }
    WST_HD int offset(int line) const {
        const int b = dnl.div(line);
        return b * bs + (line - b * nl) * ls;
    }
    // unit u of a per-line stage -> (line = u % nlines, k = u / nlines)
    WST_HD int split(int u, int& k) const {
        k = dlines.div(u);
        return u - k * nb * nl;
    }
};

// Epilogue applied to every value of a line transform's final store (e.g. |.| * scale).
struct EpiIdentity {
    WST_HD float2 operator()(float2 v) const { return v; }
};

// N2O > 0: use the split N = (N / N2O) x N2O instead of split_n2(N) (a transform whose digit-reversed
// order only its own consumers see, e.g. the fused order-2 rows)
template <int N, bool INV, int N2O = 0>
struct LineFFT {
    static constexpr int N2 = N2O > 0 ? N2O : split_n2(N);
    static constexpr int N1 = N / N2;
    static constexpr int UPT = (N2 <= 4) ? 4 : (N2 <= 8 ? 2 : 1);  // stage-B units per thread

    // single stage: unit = whole line
    template <class Epi>
    static WST_HD void single_unit(float2* base, const Lines& g, int u, Epi& epi) {
        float2* p = base + g.offset(u);
        float2 v[N];
        static_for<0, N>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = p[e * g.es];
        });
        rfft<N, INV>(v);
        static_for<0, N>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            p[e * g.es] = epi(v[e]);
        });
    }
    // stage A: unit u -> (line = u % nlines, n2 = u / nlines)
    static WST_HD void stageA_unit(float2* base, const Lines& g, const float2* tw, int u) {
        int n2;
        const int line = g.split(u, n2);
        float2* p = base + g.offset(line) + n2 * g.es;
        float2 v[N1];
        static_for<0, N1>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = p[e * N2 * g.es];
        });
        rfft<N1, INV>(v);
        static_for<1, N1>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            v[k] = cmul_tw(v[k], tw[n2 * k], INV);
        });
        static_for<0, N1>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            p[e * N2 * g.es] = v[e];
        });
    }
    // stage B load+compute: round lines [L0, L0+nlr), unit w -> (line = L0 + w % nlr, k1 = w / nlr)
    static WST_HD int stageB_load(const float2* base, const Lines& g, int L0, int nlr, int w,
                                  float2 (&v)[N2]) {
        const int k1 = w / nlr;
        const int line = L0 + (w - k1 * nlr);
        const int lb = g.offset(line);
        const float2* p = base + lb + (N2 * k1) * g.es;
        static_for<0, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = p[e * g.es];
        });
        rfft<N2, INV>(v);
        return lb + k1 * g.es;
    }
    template <class Epi>
    static WST_HD void stageB_store(float2* base, const Lines& g, int addr, const float2 (&v)[N2],
                                    Epi& epi) {
        float2* q = base + addr;
        static_for<0, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            q[e * N1 * g.es] = epi(v[e]);
        });
    }
    // ---- in-place digit-reversed variants (no transposing store) ----
    // F_DR = stageA_unit then stageB_inplace: natural in -> position k2 + N2*k1 holds k1 + N1*k2.
    template <class Epi>
    static WST_HD void stageB_inplace(float2* base, const Lines& g, int u, Epi& epi) {
        int k1;
        const int line = g.split(u, k1);
        float2* p = base + g.offset(line) + (N2 * k1) * g.es;
        float2 v[N2];
        static_for<0, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = p[e * g.es];
        });
        rfft<N2, INV>(v);
        static_for<0, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            p[e * g.es] = epi(v[e]);
        });
    }
    // G = stageBp_unit then stageAp_unit: digit-reversed in -> natural out.  GL: the stage reads its
    // inputs from `gsrc` (global memory laid out like base) instead of base.
    template <bool GL = false>
    static WST_HD void stageBp_unit(float2* base, const Lines& g, const float2* tw, int u,
                                    const float2* gsrc = nullptr) {
        int k1;
        const int line = g.split(u, k1);
        const int off = g.offset(line) + (N2 * k1) * g.es;
        float2* p = base + off;
        float2 v[N2];
        static_for<0, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            if constexpr (GL) {
#if defined(__HIP_DEVICE_COMPILE__)
                v[e] = __builtin_bit_cast(float2, __builtin_nontemporal_load(
                                                      reinterpret_cast<const unsigned long long*>(gsrc + off + e * g.es)));
#else
                v[e] = gsrc[off + e * g.es];
#endif
            } else {
                v[e] = p[e * g.es];
            }
        });
        rfft<N2, INV>(v);
        static_for<1, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = cmul_tw(v[e], tw[e * k1], INV);
        });
        static_for<0, N2>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            p[e * g.es] = v[e];
        });
    }
    template <class Epi>
    static WST_HD void stageAp_unit(float2* base, const Lines& g, int u, Epi& epi) {
        int n2;
        const int line = g.split(u, n2);
        float2* p = base + g.offset(line) + n2 * g.es;
        float2 v[N1];
        static_for<0, N1>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            v[e] = p[e * N2 * g.es];
        });
        rfft<N1, INV>(v);
        static_for<0, N1>([&](auto ec) {
            constexpr int e = decltype(ec)::value;
            p[e * N2 * g.es] = epi(v[e]);
        });
    }
    // logical index held at physical position `pos` after F_DR (identity for single-stage sizes)
    static constexpr WST_HD int dr_logical(int pos) {
        return (N2 == 1) ? pos : (pos / N2) + N1 * (pos % N2);
    }

    static WST_HD int lines_per_round(int T) {
        const int l = (T * UPT) / N1;
        return l < 1 ? 1 : l;
    }
};

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// Device driver.  Ends with a barrier.
template <int N, bool INV, class Epi = EpiIdentity>
__device__ __forceinline__ void fft_lines(float2* base, const Lines g, const float2* tw, Epi& epi) {
    using F = LineFFT<N, INV>;
    const int T = blockDim.x;
    const int nlines = g.nlines();
    if constexpr (F::N2 == 1) {
        for (int u = threadIdx.x; u < nlines; u += T) F::single_unit(base, g, u, epi);
        __syncthreads();
    } else {
        const int unitsA = nlines * F::N2;
        for (int u = threadIdx.x; u < unitsA; u += T) F::stageA_unit(base, g, tw, u);
        __syncthreads();
        const int lpr = F::lines_per_round(T);
        for (int L0 = 0; L0 < nlines; L0 += lpr) {
            const int nlr = min(lpr, nlines - L0);
            const int units = nlr * F::N1;
            float2 v[F::UPT][F::N2];
            int addr[F::UPT];
            static_for<0, F::UPT>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                const int w = threadIdx.x + i * T;
                addr[i] = (w < units) ? F::stageB_load(base, g, L0, nlr, w, v[i]) : -1;
            });
            __syncthreads();
            static_for<0, F::UPT>([&](auto ic) {
                constexpr int i = decltype(ic)::value;
                if (addr[i] >= 0) F::stageB_store(base, g, addr[i], v[i], epi);
            });
        }
        __syncthreads();
    }
}
#endif

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// In-place natural -> digit-reversed transform (F_DR).  Ends with a barrier.
template <int N, bool INV, class Epi>
__device__ __forceinline__ void fft_lines_dr(float2* base, const Lines g, const float2* tw, Epi& epi) {
    using F = LineFFT<N, INV>;
    const int T = blockDim.x;
    const int nlines = g.nlines();
    if constexpr (F::N2 == 1) {
        for (int u = threadIdx.x; u < nlines; u += T) F::single_unit(base, g, u, epi);
    } else {
        for (int u = threadIdx.x; u < nlines * F::N2; u += T) F::stageA_unit(base, g, tw, u);
        __syncthreads();
        for (int u = threadIdx.x; u < nlines * F::N1; u += T) F::stageB_inplace(base, g, u, epi);
    }
    __syncthreads();
}
// Stage B alone of F_DR (stage A done by the caller, e.g. fused with a fold).  Ends with a barrier.
template <int N, bool INV, int N2O = 0, class Epi = EpiIdentity>
__device__ __forceinline__ void fft_lines_dr_stageB(float2* base, const Lines g, Epi& epi) {
    using F = LineFFT<N, INV, N2O>;
    static_assert(F::N2 > 1, "two-stage sizes only");
    for (int u = threadIdx.x; u < g.nlines() * F::N1; u += blockDim.x) F::stageB_inplace(base, g, u, epi);
    __syncthreads();
}
// In-place digit-reversed -> natural transform (G).  Ends with a barrier.
template <int N, bool INV, class Epi>
__device__ __forceinline__ void fft_lines_rd(float2* base, const Lines g, const float2* tw, Epi& epi) {
    using F = LineFFT<N, INV>;
    const int T = blockDim.x;
    const int nlines = g.nlines();
    if constexpr (F::N2 == 1) {
        for (int u = threadIdx.x; u < nlines; u += T) F::single_unit(base, g, u, epi);
    } else {
        for (int u = threadIdx.x; u < nlines * F::N1; u += T) F::stageBp_unit(base, g, tw, u);
        __syncthreads();
        for (int u = threadIdx.x; u < nlines * F::N2; u += T) F::stageAp_unit(base, g, u, epi);
    }
    __syncthreads();
}
// G whose first stage reads its lines from global memory `src` (same layout as base) and leaves the
// result in base (LDS): the copy into LDS and its barrier fold into the transform.  Two-stage sizes
// only.  Ends with a barrier.
template <int N, bool INV, class Epi>
__device__ __forceinline__ void fft_lines_rd_from(float2* base, const float2* __restrict__ src, const Lines g,
                                                  const float2* tw, Epi& epi) {
    using F = LineFFT<N, INV>;
    static_assert(F::N2 > 1, "two-stage sizes only");
    const int T = blockDim.x;
    const int nlines = g.nlines();
    for (int u = threadIdx.x; u < nlines * F::N1; u += T)
        F::template stageBp_unit<true>(base, g, tw, u, src);
    __syncthreads();
    for (int u = threadIdx.x; u < nlines * F::N2; u += T) F::stageAp_unit(base, g, u, epi);
    __syncthreads();
}

#endif

// Host emulation of the in-place variants: mode 1 = F_DR, mode 2 = G.
template <int N, bool INV>
inline void fft_lines_inplace_host(float2* base, const Lines g, const float2* tw, int mode) {
    using F = LineFFT<N, INV>;
    EpiIdentity epi;
    const int nlines = g.nlines();
    if constexpr (F::N2 == 1) {
        for (int u = 0; u < nlines; ++u) F::single_unit(base, g, u, epi);
    } else if (mode == 1) {
        for (int u = 0; u < nlines * F::N2; ++u) F::stageA_unit(base, g, tw, u);
        for (int u = 0; u < nlines * F::N1; ++u) F::stageB_inplace(base, g, u, epi);
    } else {
        for (int u = 0; u < nlines * F::N1; ++u) F::stageBp_unit(base, g, tw, u);
        for (int u = 0; u < nlines * F::N2; ++u) F::stageAp_unit(base, g, u, epi);
    }
}

// Host emulation of fft_lines_rd_from (G with the first stage reading `src`, two-stage sizes).
template <int N, bool INV>
inline void fft_lines_rd_from_host(float2* base, const float2* src, const Lines g, const float2* tw) {
    using F = LineFFT<N, INV>;
    EpiIdentity epi;
    const int nlines = g.nlines();
    if constexpr (F::N2 > 1) {
        for (int u = 0; u < nlines * F::N1; ++u) F::template stageBp_unit<true>(base, g, tw, u, src);
        for (int u = 0; u < nlines * F::N2; ++u) F::stageAp_unit(base, g, u, epi);
    }
}

// Host-side digit-reversal map (same split as the device code): logical index at `pos`.
inline int dr_logical_host(int n, int pos) {
    const int n2 = split_n2(n);
    if (n2 == 1) return pos;
    const int n1 = n / n2;
    return pos / n2 + n1 * (pos % n2);
}

// Host emulation with the same unit bodies (sequential "threads", barriers implicit).
template <int N, bool INV>
inline void fft_lines_host(float2* base, const Lines g, const float2* tw, int T) {
    using F = LineFFT<N, INV>;
    EpiIdentity epi;
    const int nlines = g.nlines();
    if constexpr (F::N2 == 1) {
        for (int u = 0; u < nlines; ++u) F::single_unit(base, g, u, epi);
    } else {
        for (int u = 0; u < nlines * F::N2; ++u) F::stageA_unit(base, g, tw, u);
        const int lpr = F::lines_per_round(T);
        for (int L0 = 0; L0 < nlines; L0 += lpr) {
            const int nlr = (lpr < nlines - L0) ? lpr : nlines - L0;
            const int units = nlr * F::N1;
            float2* v = new float2[static_cast<size_t>(units) * F::N2];
            int* addr = new int[units];
            for (int w = 0; w < units; ++w) {
                float2 tmp[F::N2];
                addr[w] = F::stageB_load(base, g, L0, nlr, w, tmp);
                for (int e = 0; e < F::N2; ++e) v[static_cast<size_t>(w) * F::N2 + e] = tmp[e];
            }
            for (int w = 0; w < units; ++w) {
                float2 tmp[F::N2];
                for (int e = 0; e < F::N2; ++e) tmp[e] = v[static_cast<size_t>(w) * F::N2 + e];
                F::stageB_store(base, g, addr[w], tmp, epi);
            }
            delete[] v;
            delete[] addr;
        }
    }
}

}  // namespace wstfft
