// Host-side float64 filter bank (see filter_bank.h for provenance).
#include "filter_bank.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>

namespace wst {

namespace {
constexpr double kPi = 3.14159265358979323846;

int smallest_factor(int n) {
    for (int p = 2; p * p <= n; ++p)
        if (n % p == 0) return p;
    return n;
}
}  // namespace

bool make_geometry(int M, int N, int J, int L, int max_order, Geometry& g, std::string& err) {
    if (M < 1 || N < 1) { err = "shape must be positive"; return false; }
    if (J < 0 || J > 12) { err = "J out of range [0, 12]"; return false; }
    if (L < 1 || L > 64) { err = "L out of range [1, 64]"; return false; }
    if (max_order != 1 && max_order != 2) { err = "max_order must be 1 or 2"; return false; }
    if ((1 << J) > M || (1 << J) > N) {
        err = "The smallest dimension should be larger than 2^J.";
        return false;
    }
    g.M = M; g.N = N; g.J = J; g.L = L; g.max_order = max_order;
    const int s = 1 << J;
    // [kymatio 0.3.0] utils.compute_padding
    g.PM = ((M + s) / s + 1) * s;
    g.PN = ((N + s) / s + 1) * s;
    // [kymatio 0.3.0] base_frontend.build: top/left = (P-M)//2, bottom/right = (P-M+1)//2
    g.padTop = (g.PM - M) / 2;
    g.padLeft = (g.PN - N) / 2;
    g.mM = g.PM >> J;
    g.mN = g.PN >> J;
    g.oM = g.mM - 2;
    g.oN = g.mN - 2;
    g.K = 1 + J * L + (max_order >= 2 ? L * L * J * (J - 1) / 2 : 0);
    return true;
}

// Exact-index twiddles of one (length, sign): w[idx] = e^{sign 2 pi i idx / n}, computed with
// the same expression the direct evaluation used (tables are a cache, not an approximation).
// One cache per thread (the filter bank builds its filters on several threads).
static const cdouble* twiddles(int n, int sign) {
    thread_local std::map<std::pair<int, int>, std::vector<cdouble>> cache;
    auto& t = cache[{n, sign}];
    if (t.empty()) {
        t.resize(static_cast<size_t>(n));
        for (int idx = 0; idx < n; ++idx) {
            const double ang = sign * 2.0 * kPi * static_cast<double>(idx) / n;
            t[idx] = cdouble(std::cos(ang), std::sin(ang));
        }
    }
    return t.data();
}

// Recursive decimation-in-time mixed-radix DFT (float64, any length).
static void dft_rec(const cdouble* in, int n, int stride, int sign, cdouble* out) {
    if (n == 1) { out[0] = in[0]; return; }
    const int p = smallest_factor(n);
    const int m = n / p;
    const cdouble* w = twiddles(n, sign);
    if (p == n) {  // prime length: direct O(n^2) with exact-index twiddles
        for (int k = 0; k < n; ++k) {
            cdouble acc(0.0, 0.0);
            for (int t = 0; t < n; ++t)
                acc += in[static_cast<long long>(t) * stride] * w[(static_cast<long long>(t) * k) % n];
            out[k] = acc;
        }
        return;
    }
    std::vector<cdouble> sub(static_cast<size_t>(n));
    for (int r = 0; r < p; ++r)  // subsequence r: in[r + p*t]
        dft_rec(in + static_cast<long long>(r) * stride, m, stride * p, sign, sub.data() + r * m);
    for (int k = 0; k < m; ++k) {
        for (int q = 0; q < p; ++q) {
            const int kk = k + m * q;
            cdouble acc(0.0, 0.0);
            for (int r = 0; r < p; ++r) acc += sub[r * m + k] * w[(static_cast<long long>(r) * kk) % n];
            out[kk] = acc;
        }
    }
}

void dft_inplace(cdouble* x, int n, int stride, int sign) {
    std::vector<cdouble> tmp(static_cast<size_t>(n)), res(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) tmp[i] = x[static_cast<long long>(i) * stride];
    dft_rec(tmp.data(), n, 1, sign, res.data());
    for (int i = 0; i < n; ++i) x[static_cast<long long>(i) * stride] = res[i];
}

void fft2(std::vector<cdouble>& a, int rows, int cols, int sign) {
    for (int r = 0; r < rows; ++r) dft_inplace(a.data() + static_cast<long long>(r) * cols, cols, 1, sign);
    for (int c = 0; c < cols; ++c) dft_inplace(a.data() + c, rows, cols, sign);
}

// [kymatio 0.3.0] filter_bank.gabor_2d.  `env` (nullable) accumulates the same filter at xi = 0
// (its envelope alone) in the same pass: morlet_2d needs both.  Rows whose every term underflows
// (exp(re) == 0 for re < -746: far periodisation copies of a narrow envelope) are skipped; they
// add exact zeros.
static void gabor_acc(int M, int N, double sigma, double theta, double xi, double slant,
                      const FilterConvention& conv, std::vector<cdouble>& gab, std::vector<cdouble>* env) {
    gab.assign(static_cast<size_t>(M) * N, cdouble(0.0, 0.0));
    if (env) env->assign(static_cast<size_t>(M) * N, cdouble(0.0, 0.0));
    double c = std::cos(theta), s = std::sin(theta);
    const double cx = c * xi, sy = s * xi;   // the modulation uses cos / sin of theta unrounded
    if (conv.rot_f32) {                      // R, R_inv stored as float32 (convention flag)
        c = static_cast<double>(static_cast<float>(c));
        s = static_cast<double>(static_cast<float>(s));
    }
    // curv = R diag(1, slant^2) R^-1 / (2 sigma^2),  R = [[c, -s], [s, c]]
    const double d1 = 1.0, d2 = slant * slant;
    const double inv = 1.0 / (2.0 * sigma * sigma);
    const double c00 = (c * c * d1 + s * s * d2) * inv;
    const double c01 = (c * s * d1 - s * c * d2) * inv;
    const double c10 = (s * c * d1 - c * s * d2) * inv;
    const double c11 = (s * s * d1 + c * c * d2) * inv;
    const int h = conv.periodize_half;
    // max over yy of the exponent of row xx: -(c00 - b^2 / (4 c11)) xx^2 (c11 > 0)
    const double b = c01 + c10;
    const double rowq = c11 > 0.0 ? c00 - b * b / (4.0 * c11) : 0.0;
    for (int ex = -h; ex <= h; ++ex) {
        for (int ey = -h; ey <= h; ++ey) {
            for (int i = 0; i < M; ++i) {
                const double xx = static_cast<double>(ex) * M + i;
                if (-rowq * xx * xx < -746.0) continue;
                cdouble* g = gab.data() + static_cast<size_t>(i) * N;
                cdouble* e = env ? env->data() + static_cast<size_t>(i) * N : nullptr;
                for (int jj = 0; jj < N; ++jj) {
                    const double yy = static_cast<double>(ey) * N + jj;
                    const double re = -(c00 * xx * xx + (c01 + c10) * xx * yy + c11 * yy * yy);
                    const double im = xx * cx + yy * sy;
                    const double ev = std::exp(re);
                    g[jj] += ev * cdouble(std::cos(im), std::sin(im));
                    // xi = 0: the modulation is cos(0) + i sin(0) = 1 exactly
                    if (e) e[jj] += ev * cdouble(1.0, 0.0);
                }
            }
        }
    }
    const double norm = 2.0 * conv.norm_pi * sigma * sigma / slant;  // literal 3.1415 upstream
    for (auto& v : gab) v /= norm;
    if (env)
        for (auto& v : *env) v /= norm;
}

std::vector<cdouble> gabor_2d(int M, int N, double sigma, double theta, double xi, double slant,
                              const FilterConvention& conv) {
    std::vector<cdouble> gab;
    gabor_acc(M, N, sigma, theta, xi, slant, conv, gab, nullptr);
    return gab;
}

// [kymatio 0.3.0] filter_bank.morlet_2d
std::vector<cdouble> morlet_2d(int M, int N, double sigma, double theta, double xi, double slant,
                               const FilterConvention& conv) {
    std::vector<cdouble> wv, wm;
    gabor_acc(M, N, sigma, theta, xi, slant, conv, wv, &wm);
    cdouble sw(0.0, 0.0), sm(0.0, 0.0);
    for (size_t i = 0; i < wv.size(); ++i) { sw += wv[i]; sm += wm[i]; }
    const cdouble K = sw / sm;
    for (size_t i = 0; i < wv.size(); ++i) wv[i] -= K * wm[i];
    return wv;
}

// [kymatio 0.3.0] filter_bank.periodize_filter_fft (masked crop)
std::vector<double> periodize_filter_fft(const std::vector<double>& x, int M, int N, int res) {
    const int s = 1 << res;
    const int Ms = M / s, Ns = N / s;
    const int len_x = static_cast<int>(M * (1.0 - std::ldexp(1.0, -res)));
    const int start_x = static_cast<int>(M * std::ldexp(1.0, -res - 1));
    const int len_y = static_cast<int>(N * (1.0 - std::ldexp(1.0, -res)));
    const int start_y = static_cast<int>(N * std::ldexp(1.0, -res - 1));
    std::vector<double> crop(static_cast<size_t>(Ms) * Ns, 0.0);
    for (int k = 0; k < Ms; ++k)
        for (int l = 0; l < Ns; ++l) {
            double acc = 0.0;
            for (int i = 0; i < s; ++i) {
                const int r = k + i * Ms;
                if (r >= start_x && r < start_x + len_x) continue;
                for (int j = 0; j < s; ++j) {
                    const int c = l + j * Ns;
                    if (c >= start_y && c < start_y + len_y) continue;
                    acc += x[static_cast<size_t>(r) * N + c];
                }
            }
            crop[static_cast<size_t>(k) * Ns + l] = acc;
        }
    return crop;
}

std::vector<double> periodize_1d(const std::vector<double>& x, int n, int res) {
    const int s = 1 << res;
    const int ns = n / s;
    const int len = static_cast<int>(n * (1.0 - std::ldexp(1.0, -res)));
    const int start = static_cast<int>(n * std::ldexp(1.0, -res - 1));
    std::vector<double> crop(static_cast<size_t>(ns), 0.0);
    for (int k = 0; k < ns; ++k)
        for (int i = 0; i < s; ++i) {
            const int r = k + i * ns;
            if (r >= start && r < start + len) continue;
            crop[k] += x[r];
        }
    return crop;
}

// 1-D periodised Gaussian g(x) = sum_{e=-h..h} exp(-(x + e n)^2 / (2 sigma^2)) on [0, n): the
// separable factor of gabor_2d(sigma, theta=0, xi=0, slant=1) (phi).
static std::vector<double> gauss_1d(int n, double sigma, int h) {
    std::vector<double> g(static_cast<size_t>(n), 0.0);
    for (int e = -h; e <= h; ++e)
        for (int i = 0; i < n; ++i) {
            const double x = static_cast<double>(e) * n + i;
            g[i] += std::exp(-x * x / (2.0 * sigma * sigma));
        }
    return g;
}

FilterBank build_filter_bank(const Geometry& g, const FilterConvention& conv) {
    FilterBank fb;
    fb.g = g;
    fb.conv = conv;
    const int PM = g.PM, PN = g.PN, J = g.J, L = g.L;
    // [kymatio 0.3.0] filter_bank: psi_{j, theta}
    fb.psi.resize(static_cast<size_t>(J) * L);
    // every (j, theta) filter is independent: built on up to min(cores, OMP_NUM_THREADS, J L)
    // host threads (a 480^2 J=5 L=12 bank: one thread ~40 s)
    auto build_one = [&](int idx) {
        const int j = idx / L, t = idx % L;
        const double sigma = 0.8 * std::ldexp(1.0, j);
        const double theta = (static_cast<int>(L - L / 2.0 - 1) - t) * kPi / L;
        const double xi = 3.0 / 4.0 * kPi / std::ldexp(1.0, j);
        const double slant = 4.0 / L;
        std::vector<cdouble> sig = morlet_2d(PM, PN, sigma, theta, xi, slant, conv);
        fft2(sig, PM, PN, -1);
        std::vector<double> re(sig.size());
        for (size_t i = 0; i < sig.size(); ++i) re[i] = sig[i].real();
        auto& levels = fb.psi[static_cast<size_t>(idx)];
        for (int r = 0; r < psi_levels(j, J); ++r) levels.push_back(periodize_filter_fft(re, PM, PN, r));
    };
    const int ntask = J * L;
    int nthr = static_cast<int>(std::max(1u, std::thread::hardware_concurrency()));
    if (const char* omp = std::getenv("OMP_NUM_THREADS"))
        if (std::atoi(omp) > 0) nthr = std::min(nthr, std::atoi(omp));
    nthr = std::min({nthr, ntask, 16});
    if (nthr <= 1 || static_cast<long long>(PM) * PN * ntask < (1 << 18)) {
        for (int idx = 0; idx < ntask; ++idx) build_one(idx);
    } else {
        std::vector<std::thread> pool;
        std::vector<std::string> errs(static_cast<size_t>(nthr));
        for (int w = 0; w < nthr; ++w)
            pool.emplace_back([&, w]() {
                try {
                    for (int idx = w; idx < ntask; idx += nthr) build_one(idx);
                } catch (const std::exception& e) {
                    errs[static_cast<size_t>(w)] = e.what();
                }
            });
        for (auto& th : pool) th.join();
        for (const auto& e : errs)
            if (!e.empty()) throw std::runtime_error(e);
    }
    // phi = gabor_2d(sigma=0.8*2^(J-1), theta=0, xi=0, slant=1) = gM(x) gN(y) / (2*norm_pi*sigma^2)
    // phi_hat = Re(fft2(phi)) = Re(GM) Re(GN) / norm - Im(GM) Im(GN) / norm; the second term is
    // checked to be negligible (gM symmetric), so every masked-crop level is the outer product
    // of two 1-D crops.  J == 0 has no phi level used by the cascade except level 0 semantics
    // of S0 (kymatio builds range(J) levels; S0 then uses level 0 -> we need J >= 1 levels).
    const double sigma_phi = 0.8 * std::ldexp(1.0, J - 1);
    const double norm = 2.0 * conv.norm_pi * sigma_phi * sigma_phi;
    auto spectrum_1d = [&](int n, std::vector<double>& re_out) {
        std::vector<double> gs = gauss_1d(n, sigma_phi, conv.periodize_half);
        std::vector<cdouble> G(gs.begin(), gs.end());
        dft_inplace(G.data(), n, 1, -1);
        double mre = 0.0, mim = 0.0;
        re_out.resize(static_cast<size_t>(n));
        for (int i = 0; i < n; ++i) {
            re_out[i] = G[i].real() / std::sqrt(norm);
            mre = std::max(mre, std::fabs(G[i].real()));
            mim = std::max(mim, std::fabs(G[i].imag()));
        }
        if (mim > 1e-9 * mre)
            throw std::runtime_error("phi spectrum not separable (periodised Gaussian asymmetric)");
    };
    std::vector<double> GM, GN;
    spectrum_1d(PM, GM);
    spectrum_1d(PN, GN);
    const int nlev = J > 0 ? J : 1;
    fb.aM.resize(nlev); fb.aN.resize(nlev); fb.hM.resize(nlev); fb.hN.resize(nlev);
    for (int r = 0; r < nlev; ++r) {
        fb.aM[r] = periodize_1d(GM, PM, r);
        fb.aN[r] = periodize_1d(GN, PN, r);
        auto spatial = [](const std::vector<double>& a) {
            const int n = static_cast<int>(a.size());
            std::vector<cdouble> h(a.begin(), a.end());
            dft_inplace(h.data(), n, 1, +1);
            std::vector<double> out(static_cast<size_t>(n));
            for (int i = 0; i < n; ++i) out[i] = h[i].real() / n;
            return out;
        };
        fb.hM[r] = spatial(fb.aM[r]);
        fb.hN[r] = spatial(fb.aN[r]);
    }
    return fb;
}

FilterBank shape_filter_bank(const Geometry& g) {
    FilterBank fb;
    fb.g = g;
    fb.conv = kKymatio030;
    const int J = g.J, L = g.L;
    fb.psi.resize(static_cast<size_t>(J) * L);   // no band-pass values: a host-only plan reads none
    (void)L;
    const int nlev = J > 0 ? J : 1;
    fb.aM.resize(nlev); fb.aN.resize(nlev); fb.hM.resize(nlev); fb.hN.resize(nlev);
    for (int r = 0; r < nlev; ++r) {
        fb.aM[r].assign(static_cast<size_t>(g.PM >> r), 0.0);
        fb.aN[r].assign(static_cast<size_t>(g.PN >> r), 0.0);
        fb.hM[r].assign(static_cast<size_t>(g.PM >> r), 0.0);
        fb.hN[r].assign(static_cast<size_t>(g.PN >> r), 0.0);
    }
    return fb;
}

}  // namespace wst
