// Operators either side of the WST path:
//   F2  noise injection of the c4 robustness sweep -- src/preprocessing/add_noise.py:14-72
//       k_noise_formula : the reference formulas on caller-supplied draws (bit-exact parity)
//       k_noise_philox  : the same formulas on on-device Philox4x32-10 draws (production)
//       k_salt / k_pepper: salt-and-pepper scatter (salt first, then pepper, every channel)
//   F4  advanced_stats -- src/training/train_and_save_model.py:58-112, one workgroup per plane:
//       moments, exact float32 numpy percentiles (bitonic sort in LDS), scipy sobel / laplace
//       with their exact float32 rounding order, edge density.
//   c3  synthetic patches keyed by (seed, global patch index): k_patch_generate
//   F3  batched uint8 HWC -> float32 CHW / 255 ingest: k_u8_to_chw
//   probes for bench.py's measured rooflines: k_probe_copy (HBM), k_probe_fma (FP32 VALU)
// Inputs are the reference's formats: uint8 HWC images (PIL arrays) in, uint8 HWC (what
// add_noise.py saves) or float32 CHW / 255 (load_rgb_image, train_and_save_model.py:51-56) out.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "wst_hip.h"

namespace {

enum NoiseType { kGaussian = 0, kSaltPepper = 1, kSpeckle = 2, kPoisson = 3, kUniform = 4 };

// clip(v, 0, 255).astype(uint8): float64 clip, then truncation toward zero
__device__ __forceinline__ uint8_t clip_u8(double v) {
    v = v < 0.0 ? 0.0 : (v > 255.0 ? 255.0 : v);
    return static_cast<uint8_t>(static_cast<int>(v));
}

// The add_noise.py formulas in float64, same operation order (no contraction).
__device__ __forceinline__ uint8_t noise_formula(int type, double intensity, uint8_t px, double d) {
    const double x = static_cast<double>(px);
    switch (type) {
        case kGaussian:   // image + gauss
        case kUniform:    // image + noise
            return clip_u8(__dadd_rn(x, d));
        case kSpeckle: {  // image + image * gauss * (I / 100)
            const double nf = intensity / 100.0;
            return clip_u8(__dadd_rn(x, __dmul_rn(__dmul_rn(x, d), nf)));
        }
        case kPoisson: {  // poisson(.) * 255.0 / sf
            const double sf = __dadd_rn(10.0, __dmul_rn(intensity / 100.0, 90.0));
            return clip_u8(__dmul_rn(d, 255.0) / sf);
        }
        default:
            return px;
    }
}

// out_kind 0: uint8 HWC; 1: float32 CHW = uint8 / 255.0f (load_rgb_image)
__device__ __forceinline__ void store_px(void* out, int out_kind, long long img, int H, int W, int C,
                                         int r, int c, int ch, uint8_t v) {
    if (out_kind == 0) {
        static_cast<uint8_t*>(out)[((img * H + r) * W + c) * C + ch] = v;
    } else {
        static_cast<float*>(out)[((img * C + ch) * H + r) * W + c] =
            static_cast<float>(v) / 255.0f;
    }
}

__global__ void k_noise_formula(int type, double intensity, const uint8_t* __restrict__ in,
                                long long total, int H, int W, int C,
                                const double* __restrict__ draws, int out_kind, void* out) {
    for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
         i += static_cast<long long>(gridDim.x) * blockDim.x) {
        const int ch = static_cast<int>(i % C);
        const long long p = i / C;
        const int c = static_cast<int>(p % W);
        const long long q = p / W;
        const int r = static_cast<int>(q % H);
        const long long img = q / H;
        const uint8_t v = (type == kSaltPepper) ? in[i] : noise_formula(type, intensity, in[i], draws[i]);
        store_px(out, out_kind, img, H, W, C, r, c, ch, v);
    }
}

// ---- Philox4x32-10 (Salmon et al., SC'11) ----
struct U4 {
    uint32_t x, y, z, w;
};
__device__ __forceinline__ U4 philox(U4 ctr, uint32_t k0, uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, ctr.x), lo0 = 0xD2511F53u * ctr.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, ctr.z), lo1 = 0xCD9E8D57u * ctr.z;
        ctr = U4{hi1 ^ ctr.y ^ k0, lo1, hi0 ^ ctr.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return ctr;
}
// uniform double in (0, 1) from two words (53 bits, never 0)
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    const uint64_t m = (static_cast<uint64_t>(a >> 5) << 26) | (b >> 6);
    return (static_cast<double>(m) + 0.5) * (1.0 / 9007199254740992.0);
}

__device__ double draw_for(int type, double intensity, uint8_t px, uint64_t seed, long long i,
                           long long img) {
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32) ^ 0x85EBCA6Bu;
    U4 ctr{static_cast<uint32_t>(i), static_cast<uint32_t>(i >> 32), static_cast<uint32_t>(img), 0u};
    U4 r = philox(ctr, k0, k1);
    if (type == kUniform) {
        const double rng = intensity * 255.0 / 100.0;
        return -rng / 2 + (rng / 2 - (-rng / 2)) * u53(r.x, r.y);
    }
    if (type == kGaussian || type == kSpeckle) {
        const double u1 = u53(r.x, r.y), u2 = u53(r.z, r.w);
        const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        return type == kGaussian ? z * (intensity * 255.0 / 100.0) : z;
    }
    // Poisson(lambda), lambda = px * sf / 255 <= 100: sequential inversion from 0
    const double sf = 10.0 + (intensity / 100.0) * 90.0;
    const double lam = static_cast<double>(px) * sf / 255.0;
    if (lam <= 0.0) return 0.0;
    double u = u53(r.x, r.y);
    double pk = exp(-lam), cdf = pk;
    int k = 0;
    const int kmax = static_cast<int>(lam + 12.0 * sqrt(lam) + 40.0);
    while (u > cdf && k < kmax) {
        ++k;
        pk *= lam / k;
        cdf += pk;
        if (pk < 1e-300 && k > lam) break;
    }
    return static_cast<double>(k);
}

__global__ void k_noise_philox(int type, double intensity, const uint8_t* __restrict__ in,
                               long long total, int H, int W, int C, unsigned long long seed,
                               int out_kind, void* out) {
    for (long long i = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; i < total;
         i += static_cast<long long>(gridDim.x) * blockDim.x) {
        const int ch = static_cast<int>(i % C);
        const long long p = i / C;
        const int c = static_cast<int>(p % W);
        const long long q = p / W;
        const int r = static_cast<int>(q % H);
        const long long img = q / H;
        uint8_t v = in[i];
        if (type != kSaltPepper)
            v = noise_formula(type, intensity, v, draw_for(type, intensity, v, seed, i, img));
        store_px(out, out_kind, img, H, W, C, r, c, ch, v);
    }
}

// Salt-and-pepper scatter: coordinate k of image img is (rc[img][0][k], rc[img][1][k]) from the
// caller, or Philox draws of randint(0, H - 1) / randint(0, W - 1) (the last row / column is
// never hit, as in add_noise.py:31-39); every channel is set to `val`.
__global__ void k_sp_scatter(const int32_t* __restrict__ rc, long long nimg, long long count,
                             int H, int W, int C, unsigned long long seed, int phase, int val,
                             int out_kind, void* out) {
    const long long total = nimg * count;
    for (long long t = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; t < total;
         t += static_cast<long long>(gridDim.x) * blockDim.x) {
        const long long img = t / count, k = t - (t / count) * count;
        int r, c;
        if (rc) {
            r = rc[(img * 2 + 0) * count + k];
            c = rc[(img * 2 + 1) * count + k];
        } else {
            U4 ctr{static_cast<uint32_t>(k), static_cast<uint32_t>(k >> 32),
                   static_cast<uint32_t>(img), static_cast<uint32_t>(phase + 1)};
            U4 w = philox(ctr, static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32) ^ 0x5851F42Du);
            r = H > 1 ? static_cast<int>(u53(w.x, w.y) * (H - 1)) : 0;
            c = W > 1 ? static_cast<int>(u53(w.z, w.w) * (W - 1)) : 0;
        }
        for (int ch = 0; ch < C; ++ch) store_px(out, out_kind, img, H, W, C, r, c, ch, static_cast<uint8_t>(val));
    }
}

// ------------------------------------------------------------------------------------------
// advanced_stats
// ------------------------------------------------------------------------------------------
constexpr int kStatThreads = 1024;
constexpr int kStatMaxN = 16384;     // pixels per plane held in LDS (two float arrays, 128 KiB)

__device__ __forceinline__ int refl(int i, int n) {   // scipy.ndimage mode='reflect' (d c b a|a b c d)
    return i < 0 ? -i - 1 : (i >= n ? 2 * n - 1 - i : i);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// block-wide sum of doubles; all threads get the result
__device__ double block_sum_d(double v, double* red) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < static_cast<int>((blockDim.x + 63) >> 6); ++w) s += red[w];
    return s;
}

__device__ float block_minmax(float v, bool is_max, float* red) {
    for (int o = 32; o > 0; o >>= 1) {
        const float u = __shfl_xor(v, o, 64);
        v = is_max ? fmaxf(v, u) : fminf(v, u);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wid] = v;
    __syncthreads();
    float s = red[0];
    for (int w = 1; w < static_cast<int>((blockDim.x + 63) >> 6); ++w) s = is_max ? fmaxf(s, red[w]) : fminf(s, red[w]);
    return s;
}

__device__ void bitonic_sort(float* s, int np2) {
    for (int k = 2; k <= np2; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < np2; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const float a = s[i], b = s[ixj];
                    const bool up = (i & k) == 0;
                    if ((a > b) == up) {
                        s[i] = b;
                        s[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
}

// numpy.percentile(a, q) (method 'linear') of the n sorted float32 values s, in float32 exactly
// as numpy 2.x computes it: index (n - 1) * float32(q / 100) rounded to float32, then
// _lerp(a, b, g) = a + (b - a) g  (g < 0.5)  or  b - (b - a)(1 - g).
__device__ float np_percentile(const float* s, int n, float q100) {
    const float vi = __fmul_rn(static_cast<float>(n - 1), q100);
    const float fl = floorf(vi);
    const int lo = static_cast<int>(fl);
    const int hi = min(lo + 1, n - 1);
    const float g = __fsub_rn(vi, fl);
    const float a = s[lo], b = s[hi];
    const float d = __fsub_rn(b, a);
    return g >= 0.5f ? __fsub_rn(b, __fmul_rn(d, __fsub_rn(1.0f, g))) : __fadd_rn(a, __fmul_rn(d, g));
}

__global__ void __launch_bounds__(kStatThreads) k_advanced_stats(const float* __restrict__ in, int H,
                                                                 int W, double* __restrict__ out) {
    __shared__ float xs[kStatMaxN];
    __shared__ float es[kStatMaxN];
    __shared__ double redd[16];
    __shared__ float redf[16];
    const int n = H * W;
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    const long long plane = blockIdx.x;
    const float* x = in + plane * n;
    double* f = out + plane * 18;
    const float INF = __int_as_float(0x7f800000);

    // finite values (ch_clean), sum, min, max
    double sum = 0.0, cnt = 0.0;
    float mn = INF, mx = -INF;
    for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        float v = INF;
        if (i < n) {
            v = x[i];
            if (isfinite(v)) {
                sum += v;
                cnt += 1.0;
                mn = fminf(mn, v);
                mx = fmaxf(mx, v);
            } else {
                v = INF;
            }
        }
        xs[i] = v;
    }
    sum = block_sum_d(sum, redd);
    cnt = block_sum_d(cnt, redd);
    mn = block_minmax(mn, false, redf);
    mx = block_minmax(mx, true, redf);
    const int nf = static_cast<int>(cnt);
    const double mean = nf > 0 ? sum / cnt : 0.0;

    // central moments and MAD (population)
    double m2 = 0.0, m3 = 0.0, m4 = 0.0, mad = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float v = x[i];
        if (!isfinite(v)) continue;
        const double d = static_cast<double>(v) - mean;
        const double d2 = d * d;
        m2 += d2;
        m3 += d2 * d;
        m4 += d2 * d2;
        mad += fabs(d);
    }
    m2 = block_sum_d(m2, redd) / cnt;
    m3 = block_sum_d(m3, redd) / cnt;
    m4 = block_sum_d(m4, redd) / cnt;
    mad = block_sum_d(mad, redd) / cnt;

    // sobel (axis 0 and 1) and laplace, scipy's float32 rounding order, reflect boundary
    double gsum = 0.0;
    for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        float e = INF;
        if (i < n) {
            const int r = i / W, c = i - (i / W) * W;
            auto X = [&](int rr, int cc) { return static_cast<double>(x[refl(rr, H) * W + refl(cc, W)]); };
            // derivative along axis a at (rr, cc): f32(x[+1] - x[-1]) (antisymmetric [-1, 0, 1])
            auto D0 = [&](int rr, int cc) {
                rr = refl(rr, H);
                cc = refl(cc, W);
                return static_cast<float>(__dadd_rn(0.0, __dsub_rn(X(rr + 1, cc), X(rr - 1, cc))));
            };
            auto D1 = [&](int rr, int cc) {
                rr = refl(rr, H);
                cc = refl(cc, W);
                return static_cast<float>(__dadd_rn(0.0, __dsub_rn(X(rr, cc + 1), X(rr, cc - 1))));
            };
            // smoothing [1, 2, 1] (symmetric: y0 * 2 + (y-1 + y+1) * 1)
            const float gx = static_cast<float>(__dadd_rn(
                __dmul_rn(static_cast<double>(D0(r, c)), 2.0),
                __dadd_rn(static_cast<double>(D0(r, c - 1)), static_cast<double>(D0(r, c + 1)))));
            const float gy = static_cast<float>(__dadd_rn(
                __dmul_rn(static_cast<double>(D1(r, c)), 2.0),
                __dadd_rn(static_cast<double>(D1(r - 1, c)), static_cast<double>(D1(r + 1, c)))));
            const float gm = __fsqrt_rn(__fadd_rn(__fmul_rn(gx, gx), __fmul_rn(gy, gy)));
            gsum += gm;
            // laplace: f32(d2 axis 0) + f32(d2 axis 1), d2 = x0 * (-2) + (x-1 + x+1)
            const double x0 = X(r, c);
            const float l0 = static_cast<float>(__dadd_rn(__dmul_rn(x0, -2.0), __dadd_rn(X(r - 1, c), X(r + 1, c))));
            const float l1 = static_cast<float>(__dadd_rn(__dmul_rn(x0, -2.0), __dadd_rn(X(r, c - 1), X(r, c + 1))));
            e = fabsf(__fadd_rn(l0, l1));
            if (isnan(e)) e = INF;   // NaN edges: percentile -> NaN in numpy; handled below
        }
        es[i] = e;
    }
    gsum = block_sum_d(gsum, redd);
    __syncthreads();

    bitonic_sort(xs, np2);
    bitonic_sort(es, np2);

    if (threadIdx.x == 0) {
        for (int k = 0; k < 18; ++k) f[k] = 0.0;
    }
    if (nf == 0) return;   // reference: `continue` -> the channel's 18 features stay 0
    const float thr = np_percentile(es, n, 0.9f);
    double above = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) above += (es[i] > thr && es[i] != INF) ? 1.0 : 0.0;
    above = block_sum_d(above, redd);
    if (threadIdx.x == 0) {
        const double sd = sqrt(m2);
        // scipy.stats.skew / kurtosis (bias=True, fisher=True): NaN where m2 <= (eps * mean)^2
        const double eps32 = 1.1920928955078125e-07;
        const bool zero = m2 <= (eps32 * mean) * (eps32 * mean);
        const double nan = __longlong_as_double(0x7ff8000000000000ll);
        f[0] = mean;
        f[1] = sd;
        f[2] = m2;
        f[3] = mn;
        f[4] = mx;
        f[5] = __fsub_rn(mx, mn);   // np.ptp of the float32 channel: a float32 subtraction
        f[6] = zero ? nan : m3 / pow(m2, 1.5);
        f[7] = zero ? nan : m4 / (m2 * m2) - 3.0;
        f[8] = sd / fmax(mean, 1e-8);
        const float p10 = np_percentile(xs, nf, 0.1f), p25 = np_percentile(xs, nf, 0.25f);
        const float p50 = np_percentile(xs, nf, 0.5f), p75 = np_percentile(xs, nf, 0.75f);
        const float p90 = np_percentile(xs, nf, 0.9f);
        f[9] = p10;
        f[10] = p25;
        f[11] = p50;
        f[12] = p75;
        f[13] = p90;
        f[14] = static_cast<double>(p75) - static_cast<double>(p25);
        f[15] = mad;
        f[16] = gsum / n;
        f[17] = above / n;
    }
}

// ---- synthetic patches keyed by (seed, global patch index) ----
// Element e of patch p (CHW order, e < C*H*W) is byte (e & 15) of the 16-byte Philox4x32-10
// block counter (e >> 4, 0, p, p >> 32) under key (seed, seed >> 32 ^ 0x3C6EF372): a patch's
// values never depend on how the patches are split across ranks or chunks.  out_kind 0: uint8
// CHW; 1: float32 CHW / 255 (the load_rgb_image distribution, train_and_save_model.py:51-56).
// One thread per 16-byte block.
__global__ void k_patch_generate(unsigned long long seed, long long first, long long npatch,
                                 long long per, int out_kind, void* out) {
    const long long nblk = (per + 15) >> 4;
    const uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32) ^ 0x3C6EF372u;
    for (long long t = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; t < npatch * nblk;
         t += static_cast<long long>(gridDim.x) * blockDim.x) {
        const long long lp = t / nblk, q = t - lp * nblk;
        const unsigned long long p = static_cast<unsigned long long>(first + lp);
        const U4 r = philox(U4{static_cast<uint32_t>(q), static_cast<uint32_t>(q >> 32),
                               static_cast<uint32_t>(p), static_cast<uint32_t>(p >> 32)}, k0, k1);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
        const long long e0 = q << 4;
        const long long n = per - e0 < 16 ? per - e0 : 16;
        if (out_kind == 0) {
            uint8_t* o = static_cast<uint8_t*>(out) + lp * per + e0;
            for (int k = 0; k < n; ++k) o[k] = static_cast<uint8_t>(w[k >> 2] >> (8 * (k & 3)));
        } else {
            float* o = static_cast<float*>(out) + lp * per + e0;
            for (int k = 0; k < n; ++k)
                o[k] = static_cast<float>(static_cast<uint8_t>(w[k >> 2] >> (8 * (k & 3)))) / 255.0f;
        }
    }
}

// ---- uint8 HWC -> float32 CHW / 255 (load_rgb_image's ingest, train_and_save_model.py:51-56) ----
// One thread per 4 consecutive pixels of a row-major image: 4*C bytes in, four floats to each
// of the C planes (float4 stores when the row of 4 is aligned and complete).
__global__ void k_u8_to_chw(const uint8_t* __restrict__ in, long long nimg, int HW, int C,
                            float* __restrict__ out) {
    const long long q4 = (HW + 3) >> 2;
    for (long long t = blockIdx.x * static_cast<long long>(blockDim.x) + threadIdx.x; t < nimg * q4;
         t += static_cast<long long>(gridDim.x) * blockDim.x) {
        const long long img = t / q4;
        const int p0 = static_cast<int>(t - img * q4) << 2;
        const int np_ = HW - p0 < 4 ? HW - p0 : 4;
        const uint8_t* src = in + (img * HW + p0) * C;
        float* dst = out + img * C * static_cast<long long>(HW) + p0;
        for (int ch = 0; ch < C; ++ch) {
            float v[4];
            for (int k = 0; k < 4; ++k) v[k] = k < np_ ? static_cast<float>(src[k * C + ch]) / 255.0f : 0.f;
            float* d = dst + static_cast<long long>(ch) * HW;
            if (np_ == 4 && (reinterpret_cast<uintptr_t>(d) & 15) == 0) {
                *reinterpret_cast<float4*>(d) = make_float4(v[0], v[1], v[2], v[3]);
            } else {
                for (int k = 0; k < np_; ++k) d[k] = v[k];
            }
        }
    }
}

// ---- measurement probes (bench.py: BW_meas, FP32_meas of SURVEY.md §8(d)) ----
// Streaming copy: every workgroup copies one contiguous 8 KiB tile, 16 B per lane, two
// non-temporal loads in flight per lane before their stores.  Measured on MI355X (2 GiB -> 2 GiB,
// read + written bytes; tools/micro/copy_probe.hip): grid-stride forms 4.4-4.7 TB/s, contiguous
// 64 / 32 / 16 / 8 KiB tiles with nt loads 5.66 / 5.84 / 5.74 / 6.00 TB/s; hipMemcpy D2D 4.8 TB/s.
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr long long kProbeTile = 512;    // float4 per workgroup tile (8 KiB)
__global__ void __launch_bounds__(256) k_probe_copy(const v4f* __restrict__ src, v4f* __restrict__ dst,
                                                    long long n) {
    constexpr int U = 4;
    const long long b0 = blockIdx.x * kProbeTile;
    const long long e = b0 + kProbeTile < n ? b0 + kProbeTile : n;
    for (long long i = b0 + threadIdx.x; i < e; i += U * 256) {
        v4f t[U];
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (i + k * 256 < e) t[k] = __builtin_nontemporal_load(src + i + k * 256);
#pragma unroll
        for (int k = 0; k < U; ++k)
            if (i + k * 256 < e) __builtin_nontemporal_store(t[k], dst + i + k * 256);
    }
}
// 32 independent FMA chains per lane, the step loop unrolled by 4 (loop overhead < 2 % of the
// VALU issue); a, b are runtime values so nothing folds.
__global__ void __launch_bounds__(256) k_probe_fma(float* out, int iters, float a, float b) {
    float acc[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) acc[k] = static_cast<float>(threadIdx.x + k);
#pragma unroll 4
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int k = 0; k < 32; ++k) acc[k] = fmaf(acc[k], a, b);
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) s += acc[k];
    if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;   // never true: keeps the work
}

thread_local std::string g_aux_error;

int aux_fail(int code, const char* msg) {
    g_aux_error = msg;
    return code;
}

dim3 grid_for(long long total, int threads) {
    long long g = (total + threads - 1) / threads;
    if (g > 65536) g = 65536;
    if (g < 1) g = 1;
    return dim3(static_cast<unsigned>(g));
}

}  // namespace

extern "C" {

const char* wst_aux_last_error(void) { return g_aux_error.c_str(); }

int wst_salt_pepper_counts(int H, int W, int C, double intensity, int64_t* n_salt, int64_t* n_pepper) {
    if (!n_salt || !n_pepper || H < 1 || W < 1 || C < 1) return aux_fail(WST_ERR_INVALID, "bad arguments");
    const double size = static_cast<double>(H) * W * C;
    const double amount = intensity / 100.0;
    *n_salt = static_cast<int64_t>(std::ceil(amount * size * 0.5));
    *n_pepper = static_cast<int64_t>(std::ceil(amount * size * (1.0 - 0.5)));
    return WST_OK;
}

int wst_noise_apply(int noise_type, double intensity, const uint8_t* d_in, int64_t nimg, int H, int W,
                    int C, const double* d_draws, const int32_t* d_salt_rc, const int32_t* d_pepper_rc,
                    int out_kind, void* d_out, void* stream) {
    if (nimg < 0 || H < 1 || W < 1 || C < 1 || out_kind < 0 || out_kind > 1 || noise_type < 0 ||
        noise_type > 4)
        return aux_fail(WST_ERR_INVALID, "bad arguments");
    if (nimg == 0) return WST_OK;
    if (!d_in || !d_out) return aux_fail(WST_ERR_INVALID, "input/output pointer is NULL");
    if (noise_type != kSaltPepper && !d_draws) return aux_fail(WST_ERR_INVALID, "draws pointer is NULL");
    if (noise_type == kSaltPepper && (!d_salt_rc || !d_pepper_rc))
        return aux_fail(WST_ERR_INVALID, "salt/pepper coordinates are NULL");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const long long total = static_cast<long long>(nimg) * H * W * C;
    hipLaunchKernelGGL(k_noise_formula, grid_for(total, 256), dim3(256), 0, st, noise_type, intensity,
                       d_in, total, H, W, C, d_draws, out_kind, d_out);
    if (noise_type == kSaltPepper) {
        int64_t ns = 0, np_ = 0;
        wst_salt_pepper_counts(H, W, C, intensity, &ns, &np_);
        if (ns > 0)
            hipLaunchKernelGGL(k_sp_scatter, grid_for(nimg * ns, 256), dim3(256), 0, st, d_salt_rc,
                               static_cast<long long>(nimg), static_cast<long long>(ns), H, W, C, 0ull, 0, 255,
                               out_kind, d_out);
        if (np_ > 0)
            hipLaunchKernelGGL(k_sp_scatter, grid_for(nimg * np_, 256), dim3(256), 0, st, d_pepper_rc,
                               static_cast<long long>(nimg), static_cast<long long>(np_), H, W, C, 0ull, 1, 0,
                               out_kind, d_out);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

int wst_noise_generate(int noise_type, double intensity, const uint8_t* d_in, int64_t nimg, int H,
                       int W, int C, uint64_t seed, int out_kind, void* d_out, void* stream) {
    if (nimg < 0 || H < 1 || W < 1 || C < 1 || out_kind < 0 || out_kind > 1 || noise_type < 0 ||
        noise_type > 4)
        return aux_fail(WST_ERR_INVALID, "bad arguments");
    if (nimg == 0) return WST_OK;
    if (!d_in || !d_out) return aux_fail(WST_ERR_INVALID, "input/output pointer is NULL");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const long long total = static_cast<long long>(nimg) * H * W * C;
    hipLaunchKernelGGL(k_noise_philox, grid_for(total, 256), dim3(256), 0, st, noise_type, intensity,
                       d_in, total, H, W, C, static_cast<unsigned long long>(seed), out_kind, d_out);
    if (noise_type == kSaltPepper) {
        int64_t ns = 0, np_ = 0;
        wst_salt_pepper_counts(H, W, C, intensity, &ns, &np_);
        if (ns > 0)
            hipLaunchKernelGGL(k_sp_scatter, grid_for(nimg * ns, 256), dim3(256), 0, st,
                               static_cast<const int32_t*>(nullptr), static_cast<long long>(nimg),
                               static_cast<long long>(ns), H, W, C, static_cast<unsigned long long>(seed), 0,
                               255, out_kind, d_out);
        if (np_ > 0)
            hipLaunchKernelGGL(k_sp_scatter, grid_for(nimg * np_, 256), dim3(256), 0, st,
                               static_cast<const int32_t*>(nullptr), static_cast<long long>(nimg),
                               static_cast<long long>(np_), H, W, C, static_cast<unsigned long long>(seed), 1,
                               0, out_kind, d_out);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

int wst_patch_generate(uint64_t seed, int64_t first_patch, int64_t npatch, int C, int H, int W,
                       int out_kind, void* d_out, void* stream) {
    if (first_patch < 0 || npatch < 0 || C < 1 || H < 1 || W < 1 || out_kind < 0 || out_kind > 1)
        return aux_fail(WST_ERR_INVALID, "bad arguments");
    if (npatch == 0) return WST_OK;
    if (!d_out) return aux_fail(WST_ERR_INVALID, "output pointer is NULL");
    const long long per = static_cast<long long>(C) * H * W;
    hipLaunchKernelGGL(k_patch_generate, grid_for(npatch * ((per + 15) >> 4), 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), static_cast<unsigned long long>(seed),
                       static_cast<long long>(first_patch), static_cast<long long>(npatch), per, out_kind,
                       d_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

int wst_u8_to_chw(const uint8_t* d_in, int64_t nimg, int H, int W, int C, float* d_out, void* stream) {
    if (nimg < 0 || H < 1 || W < 1 || C < 1) return aux_fail(WST_ERR_INVALID, "bad arguments");
    if (nimg == 0) return WST_OK;
    if (!d_in || !d_out) return aux_fail(WST_ERR_INVALID, "input/output pointer is NULL");
    const int HW = H * W;
    hipLaunchKernelGGL(k_u8_to_chw, grid_for(nimg * ((HW + 3) / 4), 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), d_in, static_cast<long long>(nimg), HW, C,
                       d_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

int wst_probe_copy(const void* d_src, void* d_dst, size_t bytes, void* stream) {
    if (!d_src || !d_dst || (bytes & 15) || (reinterpret_cast<uintptr_t>(d_src) & 15) ||
        (reinterpret_cast<uintptr_t>(d_dst) & 15))
        return aux_fail(WST_ERR_INVALID, "copy probe needs 16-byte aligned buffers and size");
    const long long n = static_cast<long long>(bytes / 16);
    hipLaunchKernelGGL(k_probe_copy, dim3(static_cast<unsigned>((n + kProbeTile - 1) / kProbeTile)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       static_cast<const v4f*>(d_src), static_cast<v4f*>(d_dst), n);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

int wst_probe_fma(float* d_scratch, int64_t nthreads, int iters, void* stream) {
    if (!d_scratch || nthreads < 256 || (nthreads % 256) || iters < 1)
        return aux_fail(WST_ERR_INVALID, "fma probe: nthreads a positive multiple of 256, iters >= 1");
    hipLaunchKernelGGL(k_probe_fma, dim3(static_cast<unsigned>(nthreads / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), d_scratch, iters, 0.999f, 1e-3f);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

int wst_advanced_stats(const float* d_in, int64_t nplanes, int H, int W, double* d_out, void* stream) {
    if (nplanes < 0 || H < 1 || W < 1) return aux_fail(WST_ERR_INVALID, "bad arguments");
    if (static_cast<long long>(H) * W > kStatMaxN)
        return aux_fail(WST_ERR_UNSUPPORTED, "advanced_stats holds a plane in LDS: H * W <= 16384");
    if (nplanes == 0) return WST_OK;
    if (!d_in || !d_out) return aux_fail(WST_ERR_INVALID, "input/output pointer is NULL");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_advanced_stats, dim3(static_cast<unsigned>(nplanes)), dim3(kStatThreads), 0,
                       st, d_in, H, W, d_out);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return aux_fail(WST_ERR_HIP, hipGetErrorString(e));
    return WST_OK;
}

}  // extern "C"
