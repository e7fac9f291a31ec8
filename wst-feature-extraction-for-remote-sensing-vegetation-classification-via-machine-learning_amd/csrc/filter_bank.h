// Host-side (float64) construction of the Scattering2D filter bank.
//
// Restates kymatio 0.3.0 scattering2d/filter_bank.py (gabor_2d, morlet_2d, periodize_filter_fft,
// filter_bank) and utils.py (compute_padding) -- the third-party code the reference reaches at
// src/training/train_and_save_model.py:359 and src/inference/inference.py:242.  See SURVEY.md
// Appendix A.2-A.3 for the exact semantics (asymmetric periodisation grid, literal 3.1415,
// masked-crop levels).
#pragma once

#include <complex>
#include <vector>

namespace wst {

using cdouble = std::complex<double>;

// Version-dependent constants of kymatio's gabor_2d, recalled from upstream 0.3.0 (kymatio is
// not in the container: SURVEY.md §8(c)).  One struct, mirrored by the oracle's
// FilterConvention (oracle/kymatio_ref.py) and exposed as the plan parameter
// wst_filter_convention (include/wst_hip.h), so the oracle and the product switch together.
struct FilterConvention {
    double norm_pi = 3.1415;   // "pi" of gabor_2d's normaliser 2*pi*sigma^2/slant (literal 3.1415)
    int periodize_half = 2;    // periodisation copies ex, ey in [-h, h] (5x5 grid)
    bool rot_f32 = false;      // rotation matrices R, R_inv of the envelope rounded to float32
};
constexpr FilterConvention kKymatio030{3.1415, 2, false};

struct Geometry {
    int M = 0, N = 0;     // input plane
    int J = 0, L = 0;
    int max_order = 2;
    int PM = 0, PN = 0;   // padded plane (compute_padding)
    int padTop = 0, padLeft = 0;
    int mM = 0, mN = 0;   // PM >> J, PN >> J   (pre-unpad output)
    int oM = 0, oN = 0;   // mM - 2, mN - 2     (output, == M / 2^J)
    int K = 0;            // coefficients
};

// Returns false (and fills `err`) when 2^J > min(M, N) or the config is invalid.
bool make_geometry(int M, int N, int J, int L, int max_order, Geometry& g, std::string& err);

// In-place complex DFT of length n with stride (any n: mixed radix, direct DFT for primes).
// sign = -1 forward, +1 inverse (unnormalised).
void dft_inplace(cdouble* x, int n, int stride, int sign);
// 2-D forward DFT of a row-major rows x cols array.
void fft2(std::vector<cdouble>& a, int rows, int cols, int sign);

// gabor_2d / morlet_2d on an (M, N) grid, row-major.
std::vector<cdouble> gabor_2d(int M, int N, double sigma, double theta, double xi, double slant,
                              const FilterConvention& conv = kKymatio030);
std::vector<cdouble> morlet_2d(int M, int N, double sigma, double theta, double xi, double slant,
                               const FilterConvention& conv = kKymatio030);

// Masked crop of a real (M, N) spectrum to level `res` -> (M>>res, N>>res).
std::vector<double> periodize_filter_fft(const std::vector<double>& x, int M, int N, int res);
// 1-D form of the same crop (the 2-D mask and alias sum are separable).
std::vector<double> periodize_1d(const std::vector<double>& x, int n, int res);

// Number of Fourier levels kymatio keeps for psi_j: min(j+1, max(J-1, 1)).
inline int psi_levels(int j, int J) {
    int a = j + 1, b = (J - 1 > 1 ? J - 1 : 1);
    return a < b ? a : b;
}

struct FilterBank {
    Geometry g;
    FilterConvention conv;
    // psi[(j*L + l)][r] : (PM>>r) x (PN>>r) real Fourier filter, row-major
    std::vector<std::vector<std::vector<double>>> psi;
    // 1-D factors of phi's Fourier levels: phi_hat^r(k, l) = aM[r][k] * aN[r][l]
    std::vector<std::vector<double>> aM, aN;
    // spatial low-pass taps at level r: hM[r] = Re ifft(aM[r]) (length PM>>r), same for N
    std::vector<std::vector<double>> hM, hN;
};

// Build the full bank (float64).  Throws std::runtime_error on internal inconsistency (e.g. a
// phi spectrum that is not separable to 1e-12, which would invalidate the separable low-pass).
FilterBank build_filter_bank(const Geometry& g, const FilterConvention& conv = kKymatio030);
// Host-only plans (wst_describe_variants): the low-pass factors with their shapes (zero-valued)
// and no band-pass filters -- every structural decision of a plan, no float64 construction.
FilterBank shape_filter_bank(const Geometry& g);

}  // namespace wst
