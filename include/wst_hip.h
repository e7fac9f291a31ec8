/*
 * wst_hip.h -- C ABI of the MI355X-native 2-D wavelet scattering transform (WST).
 *
 * Drop-in boundary for the reference's WST feature path.  The reference reaches kymatio 0.3.0's
 * Scattering2D from these call sites (all file:line into the reference repository):
 *   - src/training/train_and_save_model.py:46   `from kymatio.numpy import Scattering2D`
 *   - src/training/train_and_save_model.py:359  `Scattering2D(J=J, L=L, shape=(H, W))`
 *   - src/training/train_and_save_model.py:368  `scattering(channel)`            (H,W)->(K,H',W')
 *   - src/training/train_and_save_model.py:371-375 per-coefficient spatial mean/std pooling
 *   - src/inference/inference.py:39,242,254     torch frontend `S(channel_tensor)` (1,1,H,W)
 *   - src/visualization/compare_wst_coefficients.py:37 `Scattering2D(..., frontend='numpy')`
 * kymatio is pure Python, so the "FFI" this library replaces is the Python-level operator API;
 * the Python frontends in wst_amd/ bind these symbols with ctypes.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Device pointers are HIP device allocations (e.g. torch
 *     tensors' data_ptr()).  `stream` is a hipStream_t passed as void* (0 = null stream).
 *   - Every entry point returns an int status (WST_OK = 0).  No C++ exception crosses the ABI.
 *     wst_last_error() returns a thread-local, NUL-terminated description of the last failure.
 *   - A plan is immutable after creation and bound to the device that was current at creation.
 *     wst_forward is asynchronous on `stream` and re-entrant across streams when each call gets
 *     its own workspace.
 */
#ifndef WST_HIP_H
#define WST_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WST_ABI_VERSION 2

enum wst_status {
    WST_OK = 0,
    WST_ERR_INVALID = 1,     /* bad argument (maps to RuntimeError/TypeError in the frontends) */
    WST_ERR_UNSUPPORTED = 2, /* size/config the kernels do not implement                        */
    WST_ERR_HIP = 3,         /* HIP runtime error (launch, copy, device mismatch)               */
    WST_ERR_NOMEM = 4        /* host or device allocation failed                                */
};

typedef struct wst_plan wst_plan;

/* ABI version of the loaded library (== WST_ABI_VERSION of the header it was built with). */
int wst_abi_version(void);

/* Thread-local description of the last error ("" if none). */
const char* wst_last_error(void);

/*
 * Build a plan for Scattering2D(J, shape=(M, N), L, max_order, pre_pad).
 * Replaces kymatio 0.3.0 ScatteringBase2D.build()/create_filters() (reached from
 * train_and_save_model.py:359 and inference.py:242): padding (compute_padding), the Morlet/Gabor
 * filter bank built on the host in float64 (filter_bank, masked-crop levels), uploaded once as
 * fp32, plus twiddle tables.  Errors: 2^J > min(M, N) -> WST_ERR_INVALID (kymatio raises
 * RuntimeError); max_order not in {1, 2} -> WST_ERR_INVALID.
 */
int wst_plan_create(int M, int N, int J, int L, int max_order, int pre_pad, wst_plan** out);

/*
 * Version-dependent constants of kymatio's gabor_2d (recalled from upstream 0.3.0, which is not
 * in the container): one named plan parameter shared with the oracle's FilterConvention
 * (oracle/kymatio_ref.py).  wst_plan_create uses wst_default_convention's values:
 *   norm_pi        = 3.1415  "pi" of the normaliser 2*pi*sigma^2/slant (upstream's literal)
 *   periodize_half = 2       periodisation copies ex, ey in [-2, 2] (5x5 grid)
 * tests/test_convention.py measures how far each alternative moves the coefficients relative
 * to the 1e-5 parity bar.
 */
typedef struct wst_filter_convention {
    double norm_pi;
    int periodize_half;   /* 0..8 */
    int flags;            /* bit 0: gabor_2d's rotation matrices R, R_inv in float32 (default 0:
                             float64); other bits 0 */
} wst_filter_convention;

int wst_default_convention(wst_filter_convention* out);

/* wst_plan_create with an explicit filter convention (NULL = the default). */
int wst_plan_create_ex(int M, int N, int J, int L, int max_order, int pre_pad,
                       const wst_filter_convention* conv, wst_plan** out);

/* Release the plan and its device memory. NULL is accepted. */
int wst_plan_destroy(wst_plan* plan);

/* Output geometry: K coefficients of (Mo, No) = (M / 2^J, N / 2^J); padded grid (PM, PN). */
int wst_output_shape(const wst_plan* plan, int* K, int* Mo, int* No);
int wst_padded_shape(const wst_plan* plan, int* PM, int* PN);

/* Bytes of device workspace wst_forward needs to process `nbatch` planes in one pass.
 * Any smaller (non-zero) workspace is accepted: the batch is then processed in chunks. */
int wst_workspace_bytes(const wst_plan* plan, int64_t nbatch, size_t* bytes);

/* Internal workspaces (wst_forward with d_workspace == NULL) the plan holds: one per stream,
 * at most 4 streams (a new stream evicts a buffer whose last work has completed, else the least
 * recently used one once its work completes).  Lets callers and tests bound the plan's device
 * memory. */
int wst_internal_workspaces(const wst_plan* plan, int* count, size_t* bytes);

/* Planes per workspace chunk the plan is tuned for (2048 for LDS-resident geometries; fewer for
 * geometries with HBM-staged levels, whose workspace is tens of MB per plane).  wst_forward
 * never processes more planes than this per chunk; size the workspace for
 * min(nbatch, preferred) planes.  (No kymatio counterpart: sizing helper of the batched ABI.) */
int wst_preferred_batch(const wst_plan* plan, int64_t* planes);

/* How the plan runs its levels (no kymatio counterpart; profiling / launch-sequence helper):
 * rb = leading levels run HBM-staged (wst_staged.h), nst = levels with staged order-2 passes
 * (rb, or J when no order-2 level folds from the global spectrum), sq = the square fused
 * LDS-resident kernels are used. */
int wst_plan_staging(const wst_plan* plan, int* rb, int* nst, int* sq);

/*
 * Scattering of `nbatch` float32 planes.
 *   d_in  : device, nbatch x M x N (or PM x PN if pre_pad), contiguous.
 *   d_out : device, pooled == 0 -> nbatch x K x Mo x No   (kymatio `S(x)` layout, stack order
 *                                   [S0; S1 (j1,l1); S2 (j1,l1,j2>j1,l2)])
 *                   pooled == 1 -> nbatch x 2K: per plane [mean_k (K) | std_k (K)], population
 *                                   std over (Mo, No) -- train_and_save_model.py:371-375 order.
 *   d_workspace / workspace_bytes : caller-owned scratch (see wst_workspace_bytes); NULL/0 lets
 *                   the plan use an internal buffer kept per stream (allocated on first use and
 *                   grown after synchronising that stream; freed with the plan; not
 *                   graph-capturable).  Calls on different streams never share it; calls that
 *                   pass their own workspace are re-entrant across streams as long as no two
 *                   in-flight calls share one workspace.
 *   stream : hipStream_t as void*.
 * Replaces: kymatio scattering2d() over the flattened batch (one call on (B,C,H,W) replaces the
 * reference's B*C serial calls at train_and_save_model.py:364-368 / inference.py:248-254).
 */
int wst_forward(const wst_plan* plan, const float* d_in, int64_t nbatch, float* d_out, int pooled,
                void* d_workspace, size_t workspace_bytes, void* stream);

/*
 * wst_forward + per-kernel timing with HIP events recorded on `stream` around every launch
 * (the launches stay back to back: the events are read once the last one has completed;
 * synchronises before returning).  kernel_ms[0] = sum of k_prep launches,
 * kernel_ms[1 + j1] = sum of the k_o1 launches at scale j1 (0 <= j1 < J), kernel_ms[1 + J + j1]
 * = sum of the k_o2 launches at scale j1 (0 <= j1 < J - 1; slot 2J stays 0); n_kernel_ms is the
 * capacity of kernel_ms (slots beyond it are not reported).  Used by bench.py for the
 * roofline's per-kernel durations; not meant for production calls.
 */
int wst_forward_profiled(const wst_plan* plan, const float* d_in, int64_t nbatch, float* d_out,
                         int pooled, void* d_workspace, size_t workspace_bytes, void* stream,
                         float* kernel_ms, int n_kernel_ms);

/*
 * Kernel-variant introspection (test hooks; no kymatio counterpart).  Every launch of a forward
 * is a "site" of 12 int32 words: word 0 the kernel instantiation (family pair, size class / line
 * length, SQ, HG), word 1 the body it dispatches to at run time (compile-time sizes, output-map
 * and L specialisations, fold and low-pass forms), words 2.. the branch of each order-2 level
 * (k_o2).  Encoding: wst_device.h tr_* (decoded by wst_amd/variants.py).
 *   wst_plan_variants     : the sites one chunk of `plan` launches, from the host mirror of the
 *                           kernels' dispatch (no GPU work).
 *   wst_describe_variants : the same for a geometry, without a GPU (a host-only plan: no
 *                           device allocation, zero-valued filters of the right shapes).
 *   wst_plan_trace        : enable (1) / disable (0) the device trace: every later forward's
 *                           launches record the words they actually ran.  Only in the trace build
 *                           (libwst_hip_trace.so = the same sources with -DWST_TRACE); the product
 *                           library has no trace code and returns WST_ERR_UNSUPPORTED for enable.
 *                           Needs a quiescent plan: call it with no forward of this plan in flight
 *                           or being issued on another thread (it drains the device and takes the
 *                           plan's workspace lock, but forwards with caller workspaces do not take
 *                           that lock).  WST_ERR_UNSUPPORTED for plans with more launch sites per
 *                           chunk than the trace area holds (512).
 *   wst_plan_read_trace   : copy the device trace (synchronises the device); *nwords = the
 *                           plan's site count x 12 (never truncated: WST_ERR_UNSUPPORTED above 512
 *                           sites).
 * out may be NULL for a size query in the first two (then only *nwords is set).
 */
int wst_plan_variants(const wst_plan* plan, int32_t* out, int64_t max_words, int64_t* nwords);
int wst_describe_variants(int M, int N, int J, int L, int max_order, int32_t* out, int64_t max_words,
                          int64_t* nwords);
int wst_plan_trace(wst_plan* plan, int enable);
int wst_plan_read_trace(const wst_plan* plan, int32_t* out, int64_t max_words, int64_t* nwords);

/*
 * Host-only filter inspection (no GPU needed; used by the CPU test-suite to pin the library's
 * float64 filter construction against the oracle).  kind:
 *   0 = psi_{j,l} Fourier level r        -> (PM>>r) x (PN>>r) doubles
 *   1 = phi Fourier level r (2-D)        -> (PM>>r) x (PN>>r) doubles (separable product)
 *   2 = phi spatial low-pass, rows (M)   -> (PM>>r) doubles
 *   3 = phi spatial low-pass, cols (N)   -> (PN>>r) doubles
 * `len` is the capacity of `out` in doubles.
 */
int wst_host_filter(int M, int N, int J, int L, int kind, int j, int l, int r, double* out,
                    int64_t len);
/* wst_host_filter under an explicit filter convention (NULL = the default). */
int wst_host_filter_ex(int M, int N, int J, int L, int kind, int j, int l, int r,
                       const wst_filter_convention* conv, double* out, int64_t len);

/*
 * Host emulation of the device line-FFT engine (test hook, no GPU): runs the exact per-unit code
 * of the LDS FFTs (csrc/fft_lds.h) sequentially on `data` (complex64 interleaved), in place.
 * Line (b, l) element e lives at complex index b*bs + l*ls + e*es; n is the line length,
 * `threads` the workgroup size whose round structure is emulated; inverse is unnormalised.
 * mode 0: natural -> natural; 1: natural -> digit-reversed (in place); 2: digit-reversed ->
 * natural (in place); 3: mode 2 with the first stage reading a copy of the input (k_o2's
 * fft_lines_rd_from); 4: mode 1 with the fused order-2 rows' split (N = (N / N2O) x N2O,
 * wst_device.h fused_row_n2; n = 48 only).  `perm` (nullable, n ints) receives the
 * digit-reversal map (physical position -> logical index) of the transform that ran.  Sizes
 * without a compiled FFT run the generic DFT (mode 0 only).
 */
int wst_host_fft_lines(int n, int inverse, int mode, float* data, int nb, int bs, int nl, int ls,
                       int es, int threads, int* perm);

/* ------------------------------------------------------------------------------------------
 * Operators either side of the path (csrc/wst_aux.hip).
 * ------------------------------------------------------------------------------------------ */

/* Noise types of src/preprocessing/add_noise.py:14-72 (process_image's noise_type strings). */
enum wst_noise_type {
    WST_NOISE_GAUSSIAN = 0,        /* add_gaussian_noise        (:14-21)  */
    WST_NOISE_SALT_AND_PEPPER = 1, /* add_salt_and_pepper_noise (:23-42)  */
    WST_NOISE_SPECKLE = 2,         /* add_speckle_noise         (:44-53)  */
    WST_NOISE_POISSON = 3,         /* add_poisson_noise         (:55-63)  */
    WST_NOISE_UNIFORM = 4          /* add_uniform_noise         (:65-71)  */
};

/* Salt / pepper coordinate counts of add_noise.py:30,36: ceil(I/100 * H*W*C * 0.5) each. */
int wst_salt_pepper_counts(int H, int W, int C, double intensity, int64_t* n_salt, int64_t* n_pepper);

/*
 * The add_noise.py formulas on caller-supplied draws (float64, same operation order, clip to
 * [0, 255] then truncation to uint8) -- bit-exact with the reference given the same draws.
 *   d_in    : device uint8, nimg x H x W x C (PIL HWC arrays).
 *   d_draws : device float64, same shape: the N(0, I*255/100) gauss (gaussian), randn (speckle),
 *             poisson draws (poisson), U(-r/2, r/2) noise (uniform); unused for salt & pepper.
 *   d_salt_rc / d_pepper_rc : device int32, nimg x 2 x count (rows, then columns), counts from
 *             wst_salt_pepper_counts; salt is applied first, then pepper, to every channel.
 *   out_kind: 0 -> uint8 HWC (what add_noise.py saves); 1 -> float32 CHW / 255 (load_rgb_image,
 *             train_and_save_model.py:51-56: the WST input).
 */
int wst_noise_apply(int noise_type, double intensity, const uint8_t* d_in, int64_t nimg, int H, int W,
                    int C, const double* d_draws, const int32_t* d_salt_rc, const int32_t* d_pepper_rc,
                    int out_kind, void* d_out, void* stream);

/* Same formulas on on-device Philox4x32-10 draws keyed by (seed, image, element): the
 * production path of the c4 noise sweep (numpy's MT19937 stream is not reproduced). */
int wst_noise_generate(int noise_type, double intensity, const uint8_t* d_in, int64_t nimg, int H,
                       int W, int C, uint64_t seed, int out_kind, void* d_out, void* stream);

/*
 * advanced_stats of src/training/train_and_save_model.py:58-112 per float32 plane (H*W <= 16384):
 * d_out[plane][0..17] = mean, std, var, min, max, range, skew, kurt, cv, p10, p25, p50, p75, p90,
 * iqr, mad, grad_mean, edge_density (float64).  Percentiles, sobel / laplace and the edge density
 * reproduce numpy / scipy's float32 arithmetic exactly; moments are computed in float64.
 */
int wst_advanced_stats(const float* d_in, int64_t nplanes, int H, int W, double* d_out, void* stream);

/*
 * Synthetic patches keyed by (seed, global patch index) -- the c3 data path of SURVEY.md §8(d)
 * (1M patches generated on the device, each rank its own shard; a patch's bytes never depend on
 * the rank / chunk split).  Patch p (first_patch <= p < first_patch + npatch), CHW element e:
 * byte (e & 15) of Philox4x32-10(counter = (e >> 4, 0, p, p >> 32), key = (seed, (seed >> 32) ^
 * 0x3C6EF372)), little-endian within each 32-bit word.  out_kind 0: uint8 CHW; 1: float32 CHW / 255
 * (the load_rgb_image distribution of train_and_save_model.py:51-56).
 */
int wst_patch_generate(uint64_t seed, int64_t first_patch, int64_t npatch, int C, int H, int W,
                       int out_kind, void* d_out, void* stream);

/* Batched uint8 HWC (PIL arrays) -> float32 CHW / 255: load_rgb_image's conversion
 * (train_and_save_model.py:51-56, inference.py:163-168) for nimg images of H x W x C. */
int wst_u8_to_chw(const uint8_t* d_in, int64_t nimg, int H, int W, int C, float* d_out, void* stream);

/* Measurement probes for bench.py's measured rooflines (SURVEY.md §8(d) BW_meas / FP32_meas;
 * no kymatio counterpart): a 16-B-per-lane streaming copy of `bytes` (16-byte aligned), and
 * nthreads (multiple of 256) lanes each running 32 independent FMA chains for `iters` steps
 * (2 * 32 * iters FLOP per lane). */
int wst_probe_copy(const void* d_src, void* d_dst, size_t bytes, void* stream);
int wst_probe_fma(float* d_scratch, int64_t nthreads, int iters, void* stream);

/* Thread-local message of the last failed wst_noise_* / wst_advanced_stats call. */
const char* wst_aux_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* WST_HIP_H */
