// MI355X (gfx950) wavelet scattering transform: plans, launches and the C ABI (include/wst_hip.h).
//
// Replaces kymatio 0.3.0's Scattering2D forward as reached from the
// reference at src/training/train_and_save_model.py:359-376 and src/inference/inference.py:242-257.
// Device code lives in wst_device.h (k_prep, k_o1, k_o2); this file builds the fp32 tables from
// the float64 filter bank (filter_bank.cpp), sizes the per-kernel LDS layouts and drives the
// chunked launch sequence:  k_prep, then for j1 = 0..J-1: k_o1[j1], k_o2[j1] (j1 < J-1).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "filter_bank.h"
#include "wst_hip.h"
#include "wst_compiled.h"
#include "wst_launch.h"

using wstdev::DevParams;
using wstdev::LdsLayout;
using wstdev::kMaxLds;
using wstdev::odd_ld;
using wstlaunch::FamilyOps;
using wstlaunch::Launch;

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

// ------------------------------------------------------------------------------------------
// size families (kernels are compiled per pair of families: wst_kernels.hip, wst_launch.h)
// ------------------------------------------------------------------------------------------
int odd_part(int n) {
    while (n > 0 && (n % 2) == 0) n /= 2;
    return n;
}
int family_of(int P) {
    const int o = odd_part(P);
    const bool compiled = (o == 1 || o == 3 || o == 5 || o == 7 || o == 9 || o == 11 || o == 13 ||
                           o == 15 || o == 17 || o == 27);
    return compiled ? o : 0;
}
// staged passes over lines of n points: the compiled FFT of that length, else the runtime-length
// instantiation (generic DFT)
const wstlaunch::BigOps* big_ops(int n) {
#define WST_BIG_OPS(N) \
    if (n == N) return &wstlaunch::WST_BIG_GETTER(N)();
    WST_BIG_SIZES(WST_BIG_OPS)
#undef WST_BIG_OPS
    return &wstlaunch::WST_BIG_GETTER(0)();
}
const FamilyOps* family_ops(int fm, int fn) {
#define WST_PAIR_OPS(A, B) \
    if (fm == A && fn == B) return &wstlaunch::WST_FAMILY_GETTER(A, B)();
    WST_FAMILY_PAIRS(WST_PAIR_OPS)
#undef WST_PAIR_OPS
    return nullptr;
}
int cap_for(int n) { return n <= 12 ? 12 : n <= 24 ? 24 : n <= 48 ? 48 : 136; }
constexpr int kBigRows = 8;   // rows per row-pass workgroup of the staged levels (kRowFold2: 2 paths)
// Rows per row-pass workgroup by mode: the LDS holds 2 kBigRows lines, so the single-path modes
// take 2 kBigRows rows when the row count allows (at n = 384 the 8-line FFT stages left half the
// 256 threads idle); otherwise the largest power of two dividing it (the grid has nrows / rows
// blocks).  kRowHalf sets its own (m/2 + 1 rows, ragged last block).
int big_rows(int mode, int nrows) {
    int r = mode == wstbig::kRowFold2 ? kBigRows : 2 * kBigRows;
    while (r > 1 && nrows % r != 0) r /= 2;
    return r;
}

size_t align16(size_t b) { return (b + 15) & ~size_t(15); }

// threads per workgroup by level size (measured on MI355X at the c2 geometry: two 512-thread
// workgroups per CU at 96^2, smaller groups for the decimated levels)
int default_threads(size_t n) { return n >= 8192 ? 512 : n >= 2048 ? 256 : n >= 512 ? 128 : 64; }

// Workgroup size so that the workgroups LDS lets share a CU carry at least 1024 threads (16 waves):
// a kernel held to one or a few workgroups per CU by its LDS otherwise runs at 2-3 waves per SIMD
// (P = 136 planes: 512 -> 1024 threads, -24 % in k_o2; P = 72: 256 -> 512, -10 % overall).
// k_o2 is content with 768 (P = 72: 3 x 256-thread workgroups, 1.92 -> 1.80 ms against 3 x 512).
int fill_cu(int threads, size_t lds, int target = 1024) {
    const size_t wgs = std::max<size_t>(1, static_cast<size_t>(160 * 1024) / std::max<size_t>(lds, 1));
    while (threads < 1024 && wgs * static_cast<size_t>(threads) < static_cast<size_t>(target)) threads *= 2;
    return threads;
}

// Tuning / ablation knobs read from the environment exist only in diagnostic builds
// (make EXTRA=-DWST_DIAG): a production library never changes its algorithm, launch shape or
// results because of an inherited variable.
const char* diag_env(const char* name) {
#ifdef WST_DIAG
    return std::getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

// "t0,t1,..." tuning override of per-j1 thread counts (diagnostic builds)
void threads_override(const char* env, std::vector<int>& v) {
    const char* s = diag_env(env);
    if (!s) return;
    int j = 0;
    for (const char* c = s; *c && j < static_cast<int>(v.size()); ++j) {
        const int t = std::atoi(c);
        if (t >= 64 && t <= 1024 && t % 64 == 0) v[j] = t;
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
    }
}

}  // namespace

// ------------------------------------------------------------------------------------------
// plan
// ------------------------------------------------------------------------------------------
struct wst_plan {
    wst::Geometry g;
    int device = 0;
    bool host_only = false;     // wst_describe_variants: structure only, no device allocations
    std::vector<int> box1_l0;   // per scale j: box1_off of (j, l = 0) (host mirror of k_o1)
    DevParams dp{};
    // device allocations
    float* d_psi = nullptr;
    long long* d_psi_off = nullptr;
    float* d_lp = nullptr;
    int* d_lp_off = nullptr;
    float2* d_tw = nullptr;
    int* d_tw_off = nullptr;
    int* d_o2 = nullptr;
    int* d_perm = nullptr;
    int* d_perm_off = nullptr;
    float2* d_psi2 = nullptr;
    long long* d_psi2_off = nullptr;
    int* d_box = nullptr;
    int* d_box_off = nullptr;
    int* d_box1_off = nullptr;
    int* d_taph = nullptr;
    int* d_taph_off = nullptr;
    int* d_taps = nullptr;
    std::vector<long long> psi2_off_host;
    std::vector<int> box_off_host;
    float* d_lpt = nullptr;
    int* d_lpt_off = nullptr;
    // launch geometry
    int fam_m = 0, fam_n = 0;   // FFT size families (odd part of PM / PN), 0 = generic DFT
    const FamilyOps* ops = nullptr;
    int sq = 0;                 // square plane with the fused order-2 low-pass (k_o1/k_o2 SQ=1)
    int prep_threads = 256;
    size_t prep_lds = 0;
    LdsLayout prep_lay{};
    std::vector<int> o1_threads, o2_threads, cap;
    std::vector<size_t> o1_lds, o2_lds;
    std::vector<LdsLayout> o1_lay, o2_lay;
    // HBM-staged leading levels (n > kBigMinN): wst_staged.h
    int rb = 0;
    int nst = 0;                                  // levels with staged passes: rb, or J when the
                                                  // staged j1's order-2 levels all run staged
    int oms = 4;                                  // tap-matrix row stride (LDS-resident kernels)
    int noms = 4;                                 // row stride of the natural tap matrices (staged)
    std::vector<const wstlaunch::BigOps*> big_r;  // per staged level: row lines (PN >> r points)
    std::vector<const wstlaunch::BigOps*> big_c;  //   column lines (PM >> r points)
    std::vector<int> lpn_off;                     // natural tap matrices: [2r] GM_r, [2r+1] GN_r
    float* d_lpn = nullptr;
    float* d_lpw = nullptr;                       // wide tap matrices (MFMA low-pass)
    int* d_lpw_off = nullptr;
    std::vector<int> o2_export;                   // per resident j1: k_o1 exports the full spectrum,
    std::vector<LdsLayout> o2x_lay;               //   k_o2 folds it from HBM (HG = 1, no spectrum in
    std::vector<size_t> o2x_lds;                  //   LDS): two workgroups per CU where the spectrum
    std::vector<int> o2x_threads;                 //   held them to one
    std::vector<LdsLayout> hg_lay;                // k_o2 (global spectrum) after a staged j1
    std::vector<size_t> hg_lds;
    std::vector<int> hg_threads, hg_j2first;
    std::vector<size_t> big_rows_lds, big_cols_lds;   // per staged level (2 R lines / 16 columns)
    std::vector<int> big_g_lds;                   // per staged level: kColModLp taps in LDS
    std::vector<int> fold_all_rows;               // per staged level: rows of the all-paths s = 2
    std::vector<size_t> fold_all_lds;             //   order-2 row pass (0: per-pair passes)
    std::vector<size_t> ws_hbig;                  // U1hat half spectra of staged j1 (per plane)
    size_t ws_tmp = 0, ws_colt = 0, ws_part = 0, ws_csum = 0, ws_mean = 0;
    int64_t max_chunk = 2048;                     // planes per workspace chunk
    // workspace per plane: Xhat, then the half spectra of every j1 < J-1
    size_t ws_xhat = 0;
    std::vector<size_t> ws_h_off;   // byte offset of level j1's half spectra (per plane units)
    size_t ws_plane = 0;
    // internal workspaces (used when the caller passes none), one per stream: calls on one
    // stream are ordered by the stream, calls on different streams never share scratch.  ws_mu
    // is held while a call enqueues on its buffer, so a buffer is only grown (stream-synchronised,
    // then freed) when no other host thread is between fetching it and launching on it.
    struct StreamWs {
        void* ptr = nullptr;
        size_t bytes = 0;
        hipEvent_t done = nullptr;     // recorded after the last call's work on this buffer
        unsigned long long tick = 0;   // last use (LRU eviction)
    };
    mutable unsigned long long ws_tick = 0;
    mutable std::mutex ws_mu;
    mutable std::map<hipStream_t, StreamWs> ws_by_stream;
};

namespace {

void free_plan(wst_plan* p) {
    if (!p) return;
    if (p->host_only) {
        delete p;
        return;
    }
    (void)hipFree(p->d_psi);
    (void)hipFree(p->d_psi_off);
    (void)hipFree(p->d_lp);
    (void)hipFree(p->d_lp_off);
    (void)hipFree(p->d_tw);
    (void)hipFree(p->d_tw_off);
    (void)hipFree(p->d_o2);
    (void)hipFree(p->d_perm);
    (void)hipFree(p->d_perm_off);
    (void)hipFree(p->d_psi2);
    (void)hipFree(p->d_psi2_off);
    (void)hipFree(p->d_box);
    (void)hipFree(p->d_box_off);
    (void)hipFree(p->d_box1_off);
    (void)hipFree(p->d_taph);
    (void)hipFree(p->d_taph_off);
    (void)hipFree(p->d_taps);
    (void)hipFree(p->d_lpt);
    (void)hipFree(p->d_lpt_off);
    (void)hipFree(p->d_lpn);
    (void)hipFree(p->d_lpw);
    (void)hipFree(p->d_lpw_off);
    for (auto& kv : p->ws_by_stream) {
        if (kv.second.done) (void)hipEventSynchronize(kv.second.done);
        if (kv.second.ptr) (void)hipFree(kv.second.ptr);
        if (kv.second.done) (void)hipEventDestroy(kv.second.done);
    }
    delete p;
}

template <typename T>
int upload(T** dst, const std::vector<T>& src) {
    const size_t bytes = std::max<size_t>(1, src.size()) * sizeof(T);
    WST_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(dst), bytes));
    if (!src.empty()) WST_HIP_CHECK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return WST_OK;
}

// Lays out one kernel's LDS: data regions first (16-byte aligned), then the table slices of
// levels [r_tw0, r_tw1] (twiddles), [r_lp0, r_lp1] (low-pass taps, permutations), S and the
// reduction scratch.  An empty range has r0 > r1.
struct TableOffsets {
    std::vector<int> tw_off, lp_off, perm_off, lpt_off;   // each with a trailing total
    std::vector<int> tw_len, lpt_len;                      // table lengths ([2r + d])
};

// Table blocks per kernel: levels [r0, r1] of the twiddle and tap-matrix pools, whose M-side
// and N-side tables are stored as two blocks (all M levels, then all N levels); a square kernel
// (n_side = false) loads only the M block and reads it for both dimensions.
struct Blocks {
    int r0 = 1, r1 = 0;
    bool n_side = true;
};

size_t layout(LdsLayout& lay, size_t data_a, size_t data_b, const TableOffsets& t, Blocks tw,
              int r_lp0, int r_lp1, size_t s_floats, Blocks lt = Blocks{}, int oms = 4) {
    size_t o = align16(data_a);
    lay.off_b = static_cast<int>(o);
    o += align16(data_b);
    lay.bcap = static_cast<int>(data_b / sizeof(float2));
    lay.oms = oms;
    auto slice = [](const std::vector<int>& off, int r0, int r1, int& base, int& n) {
        if (r0 > r1) {
            base = 0;
            n = 0;
            return;
        }
        base = off[2 * r0];
        n = off[2 * r1 + 2] - base;
    };
    // one side's levels [r0, r1]: tables of that side are contiguous in level order
    auto side = [](const std::vector<int>& off, const std::vector<int>& len, Blocks b, int d,
                   int& base, int& n) {
        if (b.r0 > b.r1 || (d == 1 && !b.n_side)) {
            base = 0;
            n = 0;
            return;
        }
        base = off[2 * b.r0 + d];
        n = off[2 * b.r1 + d] + len[2 * b.r1 + d] - base;
    };
    side(t.tw_off, t.tw_len, tw, 0, lay.tw0, lay.ntw);
    side(t.tw_off, t.tw_len, tw, 1, lay.twn0, lay.ntwn);
    slice(t.lp_off, r_lp0, r_lp1, lay.lp0, lay.nlp);
    slice(t.perm_off, r_lp0, r_lp1, lay.pm0, lay.npm);
    side(t.lpt_off, t.lpt_len, lt, 0, lay.lt0, lay.nlt);
    side(t.lpt_off, t.lpt_len, lt, 1, lay.ltn0, lay.nltn);
    lay.off_tw = static_cast<int>(o);
    o += align16(static_cast<size_t>(lay.ntw + lay.ntwn) * sizeof(float2));
    lay.off_lp = static_cast<int>(o);
    o += align16(static_cast<size_t>(lay.nlp) * sizeof(float));
    lay.off_pm = static_cast<int>(o);
    o += align16(static_cast<size_t>(lay.npm) * sizeof(int));
    lay.off_lt = static_cast<int>(o);
    o += align16(static_cast<size_t>(lay.nlt + lay.nltn) * sizeof(float));
    lay.off_s = static_cast<int>(o);
    o += align16(s_floats * sizeof(float));
    lay.off_red = static_cast<int>(o);
    o += 16 * sizeof(float);
    return o;
}

constexpr size_t kMaxStreamWs = 4;   // streams that keep an internal workspace per plan

// paths per order-2 batch at level j2 (mirrors k_o2)
constexpr int kHgSplit = 1;   // k_o2 HG workgroups per (plane, theta1) (4 until round 5)
#ifndef WST_STAGED_WS_GB   // A/B builds only (tools/variant.sh HOST_ONLY=1 -DWST_STAGED_WS_GB=...)
#define WST_STAGED_WS_GB 8
#endif
// Staged plans: chunk workspace cap.  c5 holds 31.5 MB per plane: 8 GB (of 288 GB HBM) runs BASELINE
// config 5's 256 planes as one chunk, every staged launch over all of them (22.19 -> 20.85-20.91 ms
// per step against 2 GB = 4 chunks of 64; 4 GB: 21.25; profiles/r06_ab.txt r06e)
constexpr size_t kStagedWsBytes = size_t(WST_STAGED_WS_GB) << 30;
constexpr int kHgGroup = 16;  // k_o2 HG items per batch-major dispatch group of an XCD

int paths_per_batch(size_t bcap, size_t pslot, int L) {
    const int nq = (L + 1) / 2;
    int pb = static_cast<int>(bcap / pslot);
    return std::max(2, std::min(pb & ~1, 2 * nq));
}

// Rows per unit of the last (column) stage of an in-place transform of size n.
int rows_per_unit(int n) {
    const int n2 = wstfft::split_n2(n);
    return n2 == 1 ? n : n2;
}

// Bins of a filter (pair) below this fraction of the filter's maximum are skipped by the box-sparse
// folds.  Zeroing every psi bin below it moves the float64 oracle's coefficients by at most
// 1.7e-8 (64^2 J=4), 5.3e-9 (128^2 J=2), 2.5e-8 (256^2 J=6 L=12) of each coefficient's maximum on
// random planes, and at c5's geometry on the structured patterns by at most 3.4e-7 (edge; 2.5e-8
// impulse / checkerboard / gradients) per coefficient and 3.1e-5 elementwise on the significant
// entries (edge, whose fp32 noise floor is 2.2e-3) -- 30x below the 1e-5 parity bar
// (tests/golden/box_threshold.py, profiles/r06_box_threshold_patterns.txt; GPU:
// tests/test_gpu_patterns.py::test_structured_patterns_c5_geometry).  1e-10, the round-1..4
// value, kept 11 % more bins at c5.
#ifndef WST_BOX_THR   // A/B builds only (tools/variant.sh HOST_ONLY=1 -DWST_BOX_THR=...)
#define WST_BOX_THR 1e-8
#endif
constexpr double kBoxThreshold = WST_BOX_THR;

// Minimal cyclic window [i0, i0 + n) of Z_s covering the set bits of `hit` -> i0 | n << 8.
int cyclic_window(const std::vector<char>& hit) {
    const int s = static_cast<int>(hit.size());
    std::vector<int> on;
    for (int i = 0; i < s; ++i)
        if (hit[i]) on.push_back(i);
    if (on.empty()) return 0;
    if (static_cast<int>(on.size()) == s) return s << 8;
    // the window starts after the largest cyclic gap between consecutive set positions
    int best_gap = -1, start = on[0];
    for (size_t k = 0; k < on.size(); ++k) {
        const int a = on[k], b = on[(k + 1) % on.size()];
        const int gap = ((b - a) % s + s) % s;
        const int g = (on.size() == 1) ? s : gap;
        if (g > best_gap) {
            best_gap = g;
            start = b;
        }
    }
    const int len = s - best_gap + 1;
    return start | (len << 8);
}

int create_plan(int M, int N, int J, int L, int max_order, int pre_pad,
                const wst_filter_convention* conv_in, bool device, wst_plan** out);
std::vector<int> describe_chunk(const wst_plan* pl);
bool rc_waves_ok(const wst_plan* pl, std::string& why);

// C-ABI convention -> host struct (NULL = kymatio 0.3.0 as recalled); false on a bad value.
bool to_convention(const wst_filter_convention* c, wst::FilterConvention& out) {
    out = wst::kKymatio030;
    if (!c) return true;
    if (!(c->norm_pi > 0.0) || c->periodize_half < 0 || c->periodize_half > 8 || (c->flags & ~1) != 0) {
        fail(WST_ERR_INVALID, "bad wst_filter_convention (norm_pi > 0, 0 <= periodize_half <= 8, "
                              "flags in {0, 1})");
        return false;
    }
    out.norm_pi = c->norm_pi;
    out.periodize_half = c->periodize_half;
    out.rot_f32 = (c->flags & 1) != 0;
    return true;
}

}  // namespace

extern "C" {

int wst_abi_version(void) { return WST_ABI_VERSION; }

const char* wst_last_error(void) { return g_last_error.c_str(); }

int wst_default_convention(wst_filter_convention* out) {
    if (!out) return fail(WST_ERR_INVALID, "out is NULL");
    out->norm_pi = wst::kKymatio030.norm_pi;
    out->periodize_half = wst::kKymatio030.periodize_half;
    out->flags = wst::kKymatio030.rot_f32 ? 1 : 0;
    return WST_OK;
}

int wst_plan_create(int M, int N, int J, int L, int max_order, int pre_pad, wst_plan** out) {
    return wst_plan_create_ex(M, N, J, L, max_order, pre_pad, nullptr, out);
}

int wst_plan_create_ex(int M, int N, int J, int L, int max_order, int pre_pad,
                       const wst_filter_convention* conv_in, wst_plan** out) {
    return create_plan(M, N, J, L, max_order, pre_pad, conv_in, true, out);
}

}  // extern "C"

namespace {

// device = false: a host-only plan (wst_describe_variants): every structural decision of
// wst_plan_create_ex (families, SQ, staging, layouts, export, launch shapes) on a zero-valued
// filter bank of the right shapes, no HIP call; only the host mirror of the launch sequence may
// read it.
int create_plan(int M, int N, int J, int L, int max_order, int pre_pad,
                const wst_filter_convention* conv_in, bool device, wst_plan** out) {
    if (!out) return fail(WST_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (J < 1) return fail(WST_ERR_INVALID, "J must be >= 1 (kymatio needs phi level 0)");
    wst::FilterConvention conv;
    if (!to_convention(conv_in, conv)) return WST_ERR_INVALID;
    wst::Geometry g;
    std::string err;
    if (!wst::make_geometry(M, N, J, L, max_order, g, err)) return fail(WST_ERR_INVALID, err);
    // staged levels hold 2 kBigRows row lines / kColTile column lines of their level in LDS (the
    // column pass also its tap matrix when the maps are at most kLpOM wide): checked before the
    // (size-proportional) filter bank is built, with the same formula as the plan's big_*_lds
    {
        const int omax = std::max(g.oM, g.oN);
        const size_t tapw = omax <= wstdev::kLpOM ? static_cast<size_t>(std::max(omax <= 4 ? 4 : wstdev::kLpOM,
                                                                                  (omax + 3) & ~3))
                                                  : 0;
        const auto fits = [&](size_t nl) {
            const size_t lines = std::max<size_t>(2 * kBigRows, wstbig::kColTile);
            return (nl + lines * (nl | 1)) * sizeof(float2) + nl * tapw * sizeof(float) +
                       wstbig::kColTile * sizeof(float) <= static_cast<size_t>(kMaxLds);
        };
        for (int r = 0; r < J && std::max(g.PM, g.PN) >> r > wstbig::kBigMinN; ++r) {
            const size_t nl = static_cast<size_t>(std::max(g.PM, g.PN) >> r);
            if (!fits(nl)) {
                size_t lim = nl;
                while (lim > 0 && !fits(lim)) --lim;
                return fail(WST_ERR_UNSUPPORTED, "padded plane " + std::to_string(g.PM) + "x" +
                                                     std::to_string(g.PN) + ": staged level " + std::to_string(r) +
                                                     " lines of " + std::to_string(nl) +
                                                     " points exceed the LDS line tiles (160 KiB per CU; at most " +
                                                     std::to_string(lim) + " points)");
            }
        }
        // k_big_final holds one whole oM x oN output map in dynamic LDS
        if (std::max(g.PM, g.PN) > wstbig::kBigMinN &&
            static_cast<size_t>(g.oM) * g.oN * sizeof(float) > static_cast<size_t>(kMaxLds - 256))
            return fail(WST_ERR_UNSUPPORTED, "padded plane " + std::to_string(g.PM) + "x" + std::to_string(g.PN) +
                                                 ": its " + std::to_string(g.oM) + "x" + std::to_string(g.oN) +
                                                 " output maps exceed the staged final pass's LDS map (at most " +
                                                 std::to_string((kMaxLds - 256) / 4) + " values)");
    }
    wst::FilterBank fb;
    try {
        fb = device ? wst::build_filter_bank(g, conv) : wst::shape_filter_bank(g);
    } catch (const std::exception& e) {
        return fail(WST_ERR_UNSUPPORTED, e.what());
    }

    std::unique_ptr<wst_plan, void (*)(wst_plan*)> plan(new (std::nothrow) wst_plan(), free_plan);
    if (!plan) return fail(WST_ERR_NOMEM, "host allocation failed");
    plan->g = g;
    plan->host_only = !device;
    if (device) WST_HIP_CHECK(hipGetDevice(&plan->device));

    plan->fam_m = family_of(g.PM);
    plan->fam_n = family_of(g.PN);
    plan->ops = family_ops(plan->fam_m, plan->fam_n);
    if (!plan->ops) {
        plan->fam_m = plan->fam_n = 0;
        plan->ops = family_ops(0, 0);
    }

    TableOffsets t;
    // digit-reversal maps of the in-place transforms (identity for the generic DFT)
    std::vector<int> perm;
    t.perm_off.resize(2 * static_cast<size_t>(J + 1) + 1);
    for (int r = 0; r <= J; ++r)
        for (int d = 0; d < 2; ++d) {
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            const bool compiled = (d == 0 ? plan->fam_m : plan->fam_n) > 0;
            t.perm_off[2 * r + d] = static_cast<int>(perm.size());
            for (int pos = 0; pos < n; ++pos)
                perm.push_back(compiled ? wstfft::dr_logical_host(n, pos) : pos);
        }
    t.perm_off.back() = static_cast<int>(perm.size());

    // --- flatten filters ---
    // order-1 filters psi_{j,l} (fp32 real), every kymatio level
    std::vector<float> psi;
    std::vector<long long> psi_off(static_cast<size_t>(J) * L * J, -1);
    // (host-only plans skip the value-only tables below: filters, boxes, tap lists)
    for (int j = 0; j < J && device; ++j)
        for (int l = 0; l < L; ++l) {
            const auto& lev = fb.psi[static_cast<size_t>(j) * L + l];
            for (int r = 0; r < static_cast<int>(lev.size()); ++r) {
                psi_off[(static_cast<size_t>(j) * L + l) * J + r] = static_cast<long long>(psi.size());
                for (double v : lev[r]) psi.push_back(static_cast<float>(v));
            }
        }
    // spatial low-pass taps, each level stored twice so kernels index s(c+1) + n - q unwrapped
    std::vector<float> lp;
    t.lp_off.resize(2 * static_cast<size_t>(J) + 1);
    for (int r = 0; r < J; ++r) {
        t.lp_off[2 * r] = static_cast<int>(lp.size());
        for (int rep = 0; rep < 2; ++rep)
            for (double v : fb.hM[r]) lp.push_back(static_cast<float>(v));
        t.lp_off[2 * r + 1] = static_cast<int>(lp.size());
        for (int rep = 0; rep < 2; ++rep)
            for (double v : fb.hN[r]) lp.push_back(static_cast<float>(v));
    }
    t.lp_off.back() = static_cast<int>(lp.size());
    // order-2 filters psi_{j2, l2} at level r < j2, two consecutive l2 interleaved per bin;
    // the pairs of one (j2, r) are contiguous (k_o2 strides between them by (PM>>r)(PN>>r))
    const int nq = (L + 1) / 2;
    std::vector<float2> psi2;
    std::vector<long long> psi2_off(static_cast<size_t>(J) * J * nq, -1);
    if (max_order >= 2 && device) {
        for (int j2 = 1; j2 < J; ++j2)
            for (int r = 0; r < j2 && r < wst::psi_levels(j2, J); ++r) {
                for (int q = 0; q < nq; ++q) {
                    psi2_off[(static_cast<size_t>(j2) * J + r) * nq + q] = static_cast<long long>(psi2.size());
                    const size_t nb = static_cast<size_t>(g.PM >> r) * (g.PN >> r);
                    for (size_t i = 0; i < nb; ++i) {
                        float v[2] = {0.f, 0.f};
                        for (int u = 0; u < 2; ++u) {
                            const int l2 = 2 * q + u;
                            if (l2 < L) v[u] = static_cast<float>(fb.psi[static_cast<size_t>(j2) * L + l2][r][i]);
                        }
                        psi2.push_back(make_float2(v[0], v[1]));
                    }
                }
                // s = 2 level (r = j2 - 1) of a square plane: an alias-interleaved copy of every pair
                // after the (j2, r) block (pair q at psi2_off[(j2, r, 0)] + (nq + q) n^2): per folded
                // bin (u, v) the aliases (u, v), (u + n/2, v), (u, v + n/2), (u + n/2, v + n/2) -- two
                // 16-byte loads in fold2_s2_rowA (the other folds read the plain blocks)
                const int n = g.PM >> r;
                if (r == j2 - 1 && g.PM == g.PN && n % 2 == 0) {
                    const int h = n / 2;
                    const size_t base = static_cast<size_t>(psi2_off[(static_cast<size_t>(j2) * J + r) * nq]);
                    for (int q = 0; q < nq; ++q) {
                        const size_t b = base + static_cast<size_t>(q) * n * n;
                        for (int u = 0; u < h; ++u)
                            for (int v = 0; v < h; ++v) {
                                const size_t i0 = b + static_cast<size_t>(u) * n + v, i1 = i0 + static_cast<size_t>(h) * n;
                                const float2 a0 = psi2[i0], a1 = psi2[i1], a2 = psi2[i0 + h], a3 = psi2[i1 + h];
                                psi2.push_back(a0);
                                psi2.push_back(a1);
                                psi2.push_back(a2);
                                psi2.push_back(a3);
                            }
                    }
                }
            }
    }
    // alias boxes of the order-2 pairs (see fold2): per (j2, r) all pairs, stride nM2 + nN2
    std::vector<int> box;
    std::vector<int> box_off(static_cast<size_t>(J) * J, 0);
    if (max_order >= 2 && device) {
        for (int j2 = 1; j2 < J; ++j2)
            for (int r = 0; r < j2 && r < wst::psi_levels(j2, J); ++r) {
                box_off[static_cast<size_t>(j2) * J + r] = static_cast<int>(box.size());
                const int nM1 = g.PM >> r, nN1 = g.PN >> r, nM2 = g.PM >> j2, nN2 = g.PN >> j2;
                const int sa = 1 << (j2 - r);
                for (int q = 0; q < nq; ++q) {
                    std::vector<char> rsig(nM1, 0), csig(nN1, 0);
                    for (int u = 0; u < 2; ++u) {
                        const int l2 = 2 * q + u;
                        if (l2 >= L) continue;
                        const auto& f = fb.psi[static_cast<size_t>(j2) * L + l2][r];
                        double mx = 0.0;
                        for (double v : f) mx = std::max(mx, std::fabs(v));
                        for (int kr = 0; kr < nM1; ++kr)
                            for (int kc = 0; kc < nN1; ++kc)
                                if (std::fabs(f[static_cast<size_t>(kr) * nN1 + kc]) > kBoxThreshold * mx) {
                                    rsig[kr] = 1;
                                    csig[kc] = 1;
                                }
                    }
                    if (const char* e = diag_env("WST_BOX"))   // 0: dense fold (A/B timing)
                        if (std::atoi(e) == 0) std::fill(rsig.begin(), rsig.end(), 1), std::fill(csig.begin(), csig.end(), 1);
                    std::vector<char> hit(sa);
                    for (int u = 0; u < nM2; ++u) {
                        for (int i = 0; i < sa; ++i) hit[i] = rsig[u + i * nM2];
                        box.push_back(cyclic_window(hit));
                    }
                    for (int v = 0; v < nN2; ++v) {
                        for (int i = 0; i < sa; ++i) hit[i] = csig[v + i * nN2];
                        box.push_back(cyclic_window(hit));
                    }
                }
            }
    }
    // tile tap lists of the square order-2 folds at s = 4 / 8 (wst_device.h fold2_tile_list): per
    // (j2, r) and pair q the N2^2 bins in tiles of 64; a tile's list holds every alias (a, b) at
    // which some bin of the tile meets a bin where either filter of the pair exceeds kBoxThreshold
    // of its maximum (every tap the box fold keeps at that bin), direct (b < s/2) then mirrored,
    // each padded to groups of four with dummy taps that read the zero block appended to psi2.
    // square variant (bounded FFT sizes + fused order-2 low-pass): square plane of a compiled
    // family, oM <= kLpOM and every order-2 level's column units hold ceil(oM / 2) slots
    plan->sq = (plan->fam_m > 0 && plan->fam_m == plan->fam_n && g.PM == g.PN &&
                g.oM <= wstdev::kLpOM) ? 1 : 0;
    for (int j2 = 1; j2 < J; ++j2)
        if (rows_per_unit(g.PM >> j2) < (g.oM + 1) / 2) plan->sq = 0;
    if (const char* e = diag_env("WST_SQ")) plan->sq = plan->sq && std::atoi(e) != 0;

    // Only the levels that run them get lists: LDS-resident levels of SQ plans whose size class
    // holds one size of the family (the kernels' compile-time level N1C, k_o2 branch N1C).
    std::vector<int> taph, taps;
    std::vector<int> taph_off(static_cast<size_t>(J) * J, 0);
    size_t psi2_zero = 0;   // float2 index of the zero block (dummy taps)
    const auto tile_level = [&](int j2, int r) {
        const int S = 1 << (j2 - r), N1 = g.PM >> r;
        return S >= 4 && S <= 8 && plan->sq && N1 <= wstbig::kBigMinN &&
               wstdev::unique_level(plan->fam_m, cap_for(N1)) == N1;
    };
    bool any_tiles = false;
    for (int j2 = 1; j2 < J; ++j2)
        for (int r = 0; r < j2 && r < wst::psi_levels(j2, J); ++r) any_tiles = any_tiles || tile_level(j2, r);
    if (max_order >= 2 && g.PM == g.PN && device && any_tiles) {
        psi2_zero = psi2.size();
        psi2.resize(psi2.size() + static_cast<size_t>(g.PM) * g.PM / 2 + 64, make_float2(0.f, 0.f));
        for (int j2 = 1; j2 < J; ++j2)
            for (int r = 0; r < j2 && r < wst::psi_levels(j2, J); ++r) {
                const int S = 1 << (j2 - r), N1 = g.PM >> r, N2 = g.PM >> j2, HLD = N1 / 2 + 1;
                if (!tile_level(j2, r)) continue;
                const int items = N2 * N2, nt = (items + 63) / 64;
                taph_off[static_cast<size_t>(j2) * J + r] = static_cast<int>(taph.size() / 4);
                for (int q = 0; q < nq; ++q) {
                    const long long fbase = psi2_off[(static_cast<size_t>(j2) * J + r) * nq + q];
                    std::vector<char> sig(static_cast<size_t>(N1) * N1, 0);
                    for (int u = 0; u < 2; ++u) {
                        const int l2 = 2 * q + u;
                        if (l2 >= L) continue;
                        const auto& f = fb.psi[static_cast<size_t>(j2) * L + l2][r];
                        double mx = 0.0;
                        for (double v : f) mx = std::max(mx, std::fabs(v));
                        for (size_t i = 0; i < f.size(); ++i)
                            if (std::fabs(f[i]) > kBoxThreshold * mx) sig[i] = 1;
                    }
                    for (int t = 0; t < nt; ++t) {
                        std::vector<int> dir, mir;
                        for (int a = 0; a < S; ++a)
                            for (int b = 0; b < S; ++b) {
                                bool hit = false;
                                for (int bin = 64 * t; bin < std::min(items, 64 * t + 64) && !hit; ++bin) {
                                    const int u = bin / N2, v = bin % N2;
                                    hit = sig[static_cast<size_t>(u + N2 * a) * N1 + v + N2 * b] != 0;
                                }
                                if (!hit) continue;
                                const int fo = (N2 * a * N1 + N2 * b) * 8;
                                if (b < S / 2) {
                                    dir.push_back((N2 * a * HLD + N2 * b) * 8);
                                    dir.push_back(fo);
                                } else {
                                    mir.push_back((N2 * (S - 1 - a) * HLD + N2 * (S - 1 - b)) * 8);
                                    mir.push_back(fo);
                                }
                            }
                        const int dummy = static_cast<int>((static_cast<long long>(psi2_zero) - fbase) * 8);
                        for (auto* lst : {&dir, &mir})
                            while (lst->size() % 8) {
                                lst->push_back(0);
                                lst->push_back(dummy);
                            }
                        taph.push_back(static_cast<int>(taps.size() / 2));
                        taph.push_back(static_cast<int>(dir.size() / 8));
                        taph.push_back(static_cast<int>(mir.size() / 8));
                        taph.push_back(0);
                        taps.insert(taps.end(), dir.begin(), dir.end());
                        taps.insert(taps.end(), mir.begin(), mir.end());
                    }
                }
            }
    }
    // order-1 alias boxes (psi_{j,l} at level 0 folded by s = 2^j; s >= 4 only)
    std::vector<int> box1_off(static_cast<size_t>(J) * L, -1);
    for (int j = 2; j < J; ++j)
        for (int l = 0; l < L; ++l) {
            if (!device) {   // host-only plan: whether a box exists is all the mirror reads
                const char* e = diag_env("WST_BOX");
                if (!(e && std::atoi(e) == 0)) box1_off[static_cast<size_t>(j) * L + l] = 0;
                continue;
            }
            const int sa = 1 << j, nM1 = g.PM >> j, nN1 = g.PN >> j;
            const auto& f = fb.psi[static_cast<size_t>(j) * L + l][0];
            double mx = 0.0;
            for (double v : f) mx = std::max(mx, std::fabs(v));
            std::vector<char> rsig(g.PM, 0), csig(g.PN, 0);
            for (int kr = 0; kr < g.PM; ++kr)
                for (int kc = 0; kc < g.PN; ++kc)
                    if (std::fabs(f[static_cast<size_t>(kr) * g.PN + kc]) > kBoxThreshold * mx) {
                        rsig[kr] = 1;
                        csig[kc] = 1;
                    }
            if (const char* e = diag_env("WST_BOX"))
                if (std::atoi(e) == 0) continue;
            box1_off[static_cast<size_t>(j) * L + l] = static_cast<int>(box.size());
            std::vector<char> hit(sa);
            for (int u = 0; u < nM1; ++u) {
                for (int i = 0; i < sa; ++i) hit[i] = rsig[u + i * nM1];
                box.push_back(cyclic_window(hit));
            }
            for (int v = 0; v < nN1; ++v) {
                for (int i = 0; i < sa; ++i) hit[i] = csig[v + i * nN1];
                box.push_back(cyclic_window(hit));
            }
        }
    // low-pass tap matrices in physical (digit-reversed) order, unpad + decimation folded in:
    //   GM_r[p][a] = hM_r[(s (a + 1) - perm_r(p)) mod n], s = 2^(J - r); rows padded to oms floats.
    //   Pool order: GM_0 .. GM_{J-1}, then GN_0 .. GN_{J-1} (see Blocks).
    const int oms = std::max(g.oM, g.oN) <= 4 ? 4 : wstdev::kLpOM;
    std::vector<float> lpt;
    t.lpt_off.assign(2 * static_cast<size_t>(J) + 1, 0);
    t.lpt_len.assign(2 * static_cast<size_t>(J), 0);
    for (int d = 0; d < 2; ++d)
        for (int r = 0; r < J; ++r) {
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            const int no = d == 0 ? g.oM : g.oN;
            const int sdec = 1 << (J - r);
            const auto& h = d == 0 ? fb.hM[r] : fb.hN[r];
            const int* pm = perm.data() + t.perm_off[2 * r + d];
            t.lpt_off[2 * r + d] = static_cast<int>(lpt.size());
            for (int p = 0; p < n; ++p)
                for (int a = 0; a < oms; ++a)
                    lpt.push_back(a < no ? static_cast<float>(h[((sdec * (a + 1) - pm[p]) % n + n) % n]) : 0.f);
            t.lpt_len[2 * r + d] = n * oms;
        }
    t.lpt_off.back() = static_cast<int>(lpt.size());
    // the same tap matrices in natural order (HBM-staged levels use natural-order transforms); row
    // stride noms >= max(oM, oN)
    const int noms = std::max(oms, (std::max(g.oM, g.oN) + 3) & ~3);
    std::vector<float> lpn;
    plan->lpn_off.assign(2 * static_cast<size_t>(J), 0);
    for (int r = 0; r < J; ++r)
        for (int d = 0; d < 2; ++d) {
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            const int no = d == 0 ? g.oM : g.oN;
            const int sdec = 1 << (J - r);
            const auto& h = d == 0 ? fb.hM[r] : fb.hN[r];
            plan->lpn_off[2 * r + d] = static_cast<int>(lpn.size());
            for (int p = 0; p < n; ++p)
                for (int a = 0; a < noms; ++a)
                    lpn.push_back(a < no ? static_cast<float>(h[((sdec * (a + 1) - p) % n + n) % n]) : 0.f);
        }
    plan->oms = oms;
    plan->noms = noms;
    // wide tap matrices for the MFMA low-pass (lds_lowpass_mfma), columns padded to x16:
    //   [2r + d] level r in physical order (r < J), [2J + d] level 0 in natural order (k_prep)
    const int oMp = (g.oM + 15) & ~15, oNp = (g.oN + 15) & ~15;
    // Stored in the MFMA operand order, K (the rows q) in three parts:
    //  * 64-row blocks: per 16-column tile 64 lanes x 16 K steps, step u of lane (lk = lane >> 4)
    //    taking row 64 b + u + 16 lk (the lanes of one 32-lane half read U rows 16 apart: for any
    //    odd row stride ld those 32 rows fall on distinct bank pairs, so the kernel's ds_read_b64
    //    operand reads are conflict-free; with rows 4 u + lk they were 2-way);
    //  * then 16-row blocks: 64 lanes x 4 K steps, row 16 b + 4 u + lk;
    //  * the rows past the last whole block row-major.
    // A lane's values of a block are contiguous (16-byte loads, each feeding 4 MFMAs).
    std::vector<float> lpw;
    std::vector<int> lpw_off(2 * static_cast<size_t>(J + 1), 0);
    for (int slot = 0; slot <= J; ++slot)
        for (int d = 0; d < 2; ++d) {
            const int r = slot < J ? slot : 0;
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            const int no = d == 0 ? g.oM : g.oN, np_ = d == 0 ? oMp : oNp;
            const int sdec = 1 << (J - r);
            const auto& h = d == 0 ? fb.hM[r] : fb.hN[r];
            const int* pm = perm.data() + t.perm_off[2 * r + d];
            const auto tap = [&](int q, int a) {
                const int phys = slot < J ? pm[q] : q;
                return a < no ? static_cast<float>(h[((sdec * (a + 1) - phys) % n + n) % n]) : 0.f;
            };
            while (lpw.size() % 4) lpw.push_back(0.f);
            lpw_off[2 * slot + d] = static_cast<int>(lpw.size());
            const int n64 = n / 64, n16 = (n - 64 * n64) / 16, ntile = np_ / 16;
            for (int b = 0; b < n64; ++b)
                for (int tl = 0; tl < ntile; ++tl)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int u = 0; u < 16; ++u)
                            lpw.push_back(tap(64 * b + u + 16 * (lane >> 4), 16 * tl + (lane & 15)));
            for (int b = 0; b < n16; ++b)
                for (int tl = 0; tl < ntile; ++tl)
                    for (int lane = 0; lane < 64; ++lane)
                        for (int u = 0; u < 4; ++u)
                            lpw.push_back(tap(64 * n64 + 16 * b + 4 * u + (lane >> 4), 16 * tl + (lane & 15)));
            for (int q = 64 * n64 + 16 * n16; q < n; ++q)
                for (int a = 0; a < np_; ++a) lpw.push_back(tap(q, a));
        }
    // twiddles exp(-2 pi i k / n) per level and side; pool order: M levels 0..J, then N levels
    std::vector<float2> tw;
    t.tw_off.assign(2 * static_cast<size_t>(J + 1) + 1, 0);
    t.tw_len.assign(2 * static_cast<size_t>(J + 1), 0);
    for (int d = 0; d < 2; ++d)
        for (int r = 0; r <= J; ++r) {
            const int n = (d == 0 ? g.PM : g.PN) >> r;
            t.tw_off[2 * r + d] = static_cast<int>(tw.size());
            t.tw_len[2 * r + d] = n;
            for (int k = 0; k < n; ++k) {
                const double a = 2.0 * 3.14159265358979323846 * k / n;
                tw.push_back(make_float2(static_cast<float>(std::cos(a)), static_cast<float>(-std::sin(a))));
            }
        }
    t.tw_off.back() = static_cast<int>(tw.size());
    // (the variant-trace words of wst_plan_trace live after the J L coefficient bases)
    std::vector<int> o2(static_cast<size_t>(J) * L + static_cast<size_t>(wstdev::kTraceSites) * wstdev::kTraceW, 0);
    {
        int k = 1 + J * L;
        for (int j1 = 0; j1 < J; ++j1)
            for (int l1 = 0; l1 < L; ++l1) {
                o2[static_cast<size_t>(j1) * L + l1] = k;
                if (max_order >= 2) k += L * (J - 1 - j1);
            }
    }

    int rc;
    const auto up = [&](auto** dst, const auto& src) { return device ? upload(dst, src) : WST_OK; };
    if ((rc = up(&plan->d_psi, psi)) != WST_OK) return rc;
    if ((rc = up(&plan->d_psi_off, psi_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_lp, lp)) != WST_OK) return rc;
    if ((rc = up(&plan->d_lp_off, t.lp_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_tw, tw)) != WST_OK) return rc;
    if ((rc = up(&plan->d_tw_off, t.tw_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_o2, o2)) != WST_OK) return rc;
    if ((rc = up(&plan->d_psi2, psi2)) != WST_OK) return rc;
    if ((rc = up(&plan->d_psi2_off, psi2_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_perm, perm)) != WST_OK) return rc;
    if ((rc = up(&plan->d_perm_off, t.perm_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_box, box)) != WST_OK) return rc;
    if ((rc = up(&plan->d_box_off, box_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_box1_off, box1_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_taph, taph)) != WST_OK) return rc;
    if ((rc = up(&plan->d_taph_off, taph_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_taps, taps)) != WST_OK) return rc;
    plan->psi2_off_host = psi2_off;
    plan->box_off_host = box_off;
    if ((rc = up(&plan->d_lpt, lpt)) != WST_OK) return rc;
    if ((rc = up(&plan->d_lpt_off, t.lpt_off)) != WST_OK) return rc;
    if ((rc = up(&plan->d_lpn, lpn)) != WST_OK) return rc;
    if ((rc = up(&plan->d_lpw, lpw)) != WST_OK) return rc;
    if ((rc = up(&plan->d_lpw_off, lpw_off)) != WST_OK) return rc;

    DevParams& dp = plan->dp;
    dp.M = g.M; dp.N = g.N; dp.PM = g.PM; dp.PN = g.PN; dp.J = J; dp.L = L;
    dp.max_order = max_order; dp.pre_pad = pre_pad ? 1 : 0; dp.K = g.K;
    dp.mM = g.mM; dp.mN = g.mN; dp.oM = g.oM; dp.oN = g.oN;
    dp.padTop = g.padTop; dp.padLeft = g.padLeft;
    {
        // phase-skipping timing ablation: diagnostic builds only (the results are wrong by design)
        const char* dbg = diag_env("WST_DEBUG_SKIP");
        dp.flags = dbg ? (std::atoi(dbg) & 0x3fffffff) : 0;
    }
    dp.psi = plan->d_psi; dp.psi_off = plan->d_psi_off;
    dp.lp = plan->d_lp; dp.lp_off = plan->d_lp_off;
    dp.tw = plan->d_tw; dp.tw_off = plan->d_tw_off;
    dp.perm = plan->d_perm; dp.perm_off = plan->d_perm_off;
    dp.o2_base = plan->d_o2;
    dp.psi2 = plan->d_psi2; dp.psi2_off = plan->d_psi2_off;
    dp.box = plan->d_box; dp.box_off = plan->d_box_off; dp.box1_off = plan->d_box1_off;
    dp.taph = reinterpret_cast<const int4*>(plan->d_taph);
    dp.taph_off = plan->d_taph_off;
    dp.taps = reinterpret_cast<const int2*>(plan->d_taps);
    // the order-1 box-sparse fold pays off from s = 8 on (measured on MI355X at c2); order 2
    // uses it for every s >= 4
    dp.box1_min_s = 8;
    if (const char* e = diag_env("WST_BOX1_MIN_S")) dp.box1_min_s = std::atoi(e);
    dp.lpt = plan->d_lpt; dp.lpt_off = plan->d_lpt_off;
    dp.lpw = plan->d_lpw; dp.lpw_off = plan->d_lpw_off; dp.oMp = oMp; dp.oNp = oNp;
    // --- LDS layouts ---
    const size_t omn = static_cast<size_t>(g.oM) * g.oN;
    const auto too_big = [&](const char* what, int j) {
        return fail(WST_ERR_UNSUPPORTED,
                    std::string(what) + " of the " + std::to_string(g.PM) + "x" +
                        std::to_string(g.PN) + " padded plane at level " + std::to_string(j) +
                        " exceeds the LDS-resident path (160 KiB per CU)");
    };
    // leading levels too large for the LDS-resident kernels run HBM-staged (wst_staged.h)
    while (plan->rb < J && std::max(g.PM, g.PN) >> plan->rb > wstbig::kBigMinN) ++plan->rb;
    if (plan->rb > 0) {
        // square compiled-family planes (sq) fold the order-2 levels from rb on out of the global
        // spectrum (k_o2 HG); any other plane runs every order-2 level of a staged j1 staged
        plan->nst = plan->sq ? plan->rb : J;
        if (const char* e = diag_env("WST_NST"))   // staged order-2 levels below rb (A/B timing)
            if (plan->sq) plan->nst = std::max(plan->rb, std::min(J, std::atoi(e)));
        const int nst = plan->nst;
        plan->big_r.assign(nst, nullptr);
        plan->big_c.assign(nst, nullptr);
        plan->big_rows_lds.assign(nst, 0);
        plan->big_cols_lds.assign(nst, 0);
        plan->big_g_lds.assign(nst, 1);
        for (int r = 0; r < nst; ++r) {
            const size_t nm = static_cast<size_t>(g.PM >> r), nn = static_cast<size_t>(g.PN >> r);
            plan->big_r[r] = big_ops(g.PN >> r);
            plan->big_c[r] = big_ops(g.PM >> r);
            plan->big_rows_lds[r] = (nn + 2 * kBigRows * (nn | 1)) * sizeof(float2);
            // + tap matrix + the tile's column sums (kColModLpFwd)
            plan->big_cols_lds[r] = (nm + wstbig::kColTile * (nm | 1)) * sizeof(float2) +
                                    nm * static_cast<size_t>(noms) * sizeof(float) + wstbig::kColTile * sizeof(float);
            if (plan->big_cols_lds[r] > static_cast<size_t>(kMaxLds) && g.oM > 8) {
                // wide output maps: the tap matrix stays in L2
                plan->big_g_lds[r] = 0;
                plan->big_cols_lds[r] = (nm + wstbig::kColTile * (nm | 1)) * sizeof(float2) +
                                        wstbig::kColTile * sizeof(float);
            }
            if (std::max(plan->big_rows_lds[r], plan->big_cols_lds[r]) > static_cast<size_t>(kMaxLds))
                return fail(WST_ERR_UNSUPPORTED, "level " + std::to_string(r) + " (" + std::to_string(nm) + "x" +
                                                     std::to_string(nn) + ") exceeds the staged passes' " +
                                                     "LDS line tiles (160 KiB per CU)");
        }
        // the all-paths s = 2 order-2 row pass: rows x L paths of lines, four workgroups per CU (c5:
        // 2 rows, 28.96 -> 27.92 ms against 4 rows at two workgroups per CU; 1 row: 28.39)
        plan->fold_all_rows.assign(nst, 0);
        plan->fold_all_lds.assign(nst, 0);
        for (int r = 1; r < nst; ++r) {
            const size_t nm = static_cast<size_t>(g.PM >> r), nn = static_cast<size_t>(g.PN >> r);
            for (int rows = 4; rows >= 1; rows /= 2) {
                const size_t lds = (nn + static_cast<size_t>(L) * rows * (nn | 1)) * sizeof(float2);
                if (nm % rows == 0 && lds <= static_cast<size_t>(kMaxLds) / 4) {
                    plan->fold_all_rows[r] = rows;
                    plan->fold_all_lds[r] = lds;
                    break;
                }
            }
        }
    } else {
        plan->prep_lds = layout(plan->prep_lay, static_cast<size_t>(g.PM) * odd_ld(g.PN) * sizeof(float2),
                                0, t, Blocks{0, 0, true}, 0, 0, omn);
        plan->prep_lay.npm = 0;   // k_prep works in natural order
        if (plan->prep_lds > static_cast<size_t>(kMaxLds)) return too_big("k_prep", 0);
        plan->prep_threads = static_cast<size_t>(g.PM) * g.PN >= 4096 ? 512 : 256;
    }

    plan->o1_threads.assign(J, 64);
    plan->o2_threads.assign(J, 64);
    plan->cap.assign(J, 12);
    plan->o1_lds.assign(J, 0);
    plan->o2_lds.assign(J, 0);
    plan->o1_lay.assign(J, LdsLayout{});
    plan->o2_lay.assign(J, LdsLayout{});
    plan->ws_h_off.assign(J, 0);
    plan->ws_xhat = static_cast<size_t>(g.PM) * g.PN * sizeof(float2);
    size_t wsp = plan->ws_xhat;
    auto pslot = [&](int j) { return static_cast<size_t>(g.PM >> j) * odd_ld(g.PN >> j); };
    plan->ws_hbig.assign(J, 0);
    plan->hg_lay.assign(J, LdsLayout{});
    plan->hg_lds.assign(J, 0);
    plan->hg_threads.assign(J, 64);
    plan->hg_j2first.assign(J, J);
    size_t tmp_c = 0, part_n = static_cast<size_t>(g.PM);
    for (int j1 = 0; j1 < plan->rb; ++j1) {
        // staged order 1 (+ U1hat for order 2); order-2 paths staged while j2 < nst, then k_o2 HG
        const size_t m1 = static_cast<size_t>(g.PM >> j1), n1 = static_cast<size_t>(g.PN >> j1);
        const bool do2 = max_order >= 2 && j1 < J - 1;
        tmp_c = std::max(tmp_c, static_cast<size_t>(L) * m1 * n1);
        part_n = std::max(part_n, static_cast<size_t>(L) * n1);
        if (!do2) continue;
        // kRowHalf derives the spectrum height from its half-row count (m = 2 (rows - 1)) and
        // writes row m - k as the mirror of row k: both hold only for an even m (padding to
        // multiples of 2^J makes every staged level with order 2 even; checked, not assumed)
        if (m1 % 2 != 0 || n1 % 2 != 0)
            return fail(WST_ERR_UNSUPPORTED, "staged order-2 level " + std::to_string(j1) + " (" +
                                                 std::to_string(m1) + "x" + std::to_string(n1) + ") must be even");
        plan->ws_hbig[j1] = wsp;
        wsp += align16(static_cast<size_t>(L) * m1 * (n1 / 2 + 1) * sizeof(float2));
        // column spectra of U1, rows 0..m1/2 (kColModLpFwd -> kRowHalf)
        plan->ws_colt = std::max(plan->ws_colt, static_cast<size_t>(L) * (m1 / 2 + 1) * n1 * sizeof(float2));
        for (int j2 = j1 + 1; j2 < plan->nst; ++j2) {
            const size_t m2 = static_cast<size_t>(g.PM >> j2), n2 = static_cast<size_t>(g.PN >> j2);
            tmp_c = std::max(tmp_c, static_cast<size_t>(L) * m2 * n2);
            part_n = std::max(part_n, static_cast<size_t>(L) * L * n2);   // every theta1's partials
        }
        const int j2f = std::max(j1 + 1, plan->nst);
        plan->hg_j2first[j1] = j2f;
        if (j2f >= J) continue;
        // two paths of the first resident level (the smaller levels batch as many as fit)
        const size_t bcap = 2 * pslot(j2f);
        size_t smax = 0;
        for (int j2 = j2f; j2 < J; ++j2)
            smax = std::max(smax, static_cast<size_t>(paths_per_batch(bcap, pslot(j2), L)) * omn);
        plan->hg_lds[j1] = layout(plan->hg_lay[j1], 0, bcap * sizeof(float2), t, Blocks{j2f, J - 1, false},
                                  1, 0, smax, Blocks{j2f, J - 1, false}, oms);
        // (one workgroup per CU at c5's 96^2 batches: 1024 threads, k_o2 j1=0/1 17.9/3.19 -> 16.7/2.84 ms)
        plan->hg_threads[j1] = default_threads(static_cast<size_t>(g.PM >> j2f) * (g.PN >> j2f));
        if (plan->hg_lds[j1] > static_cast<size_t>(kMaxLds)) return too_big("k_o2 (global spectrum)", j1);
        plan->hg_threads[j1] = fill_cu(plan->hg_threads[j1], plan->hg_lds[j1]);
        // the batches of an item split over kHgSplit workgroups on one XCD: they fold from the same
        // H, which that XCD's L2 then serves (one workgroup per item re-reads it from HBM once per
        // batch; one workgroup per batch repeats the table set-up 10x at c5: measured 1 / 3 / 6 /
        // 10 workgroups per item, c5 29.66 / 29.08 / 29.35 / 30.09 ms).  Dispatch slots run
        // batch-major over groups of kHgGroup items, so the workgroups an XCD runs together fold the
        // same filter pairs (c5 split x group, ms/step: 3 x 1 26.29, 5 x 16 26.10, 4 x 16 25.89,
        // 6 x 8 26.16; HG fetch per chunk at j1 = 0 / 1: 4.04 / 0.54 GB -> 2.46 / 0.27 GB at 4 x 16).
        // Round 5: with the box fold loading only in-box taps the split no longer pays (c5 split
        // 4 / 3 / 2 / 1: 23.49 / 23.39 / 23.11 / 23.06 ms per step, profiles/r05_ab.txt r05r): one
        // workgroup per item; the split stays a diagnostic knob (WST_HG_SPLIT / WST_HG_GROUP)
        int nbatch = 0;
        for (int j2 = j2f; j2 < J; ++j2) {
            const int pb = paths_per_batch(bcap, pslot(j2), L);
            nbatch += (L + pb - 1) / pb;
        }
        plan->hg_lay[j1].nsplit = std::min(nbatch, kHgSplit);
        plan->hg_lay[j1].hgroup = kHgGroup;
        if (const char* e = diag_env("WST_HG_GROUP")) plan->hg_lay[j1].hgroup = std::max(1, std::atoi(e));
        if (const char* e = diag_env("WST_HG_SPLIT")) {   // "n0,n1,...": per j1 (last one repeats)
            const char* q = e;
            for (int k = 0; k < j1 && std::strchr(q, ','); ++k) q = std::strchr(q, ',') + 1;
            plan->hg_lay[j1].nsplit = std::max(1, std::atoi(q));
        }
    }
    if (plan->rb > 0) {
        plan->ws_tmp = wsp;
        wsp += align16(tmp_c * sizeof(float2));
        const size_t colt_bytes = plan->ws_colt;
        plan->ws_colt = wsp;
        wsp += align16(colt_bytes);
        plan->ws_part = wsp;
        wsp += align16(part_n * noms * sizeof(float));
        plan->ws_csum = wsp;
        wsp += align16(part_n * sizeof(float));
        plan->ws_mean = wsp;
        wsp += align16((wstbig::kMeanParts + static_cast<size_t>(L)) * sizeof(float));
    }
    for (int j1 = plan->rb; j1 < J; ++j1) {
        const int nM1 = g.PM >> j1, nN1 = g.PN >> j1;
        const size_t n1 = static_cast<size_t>(nM1) * nN1;
        const bool do2 = max_order >= 2 && j1 < J - 1;
        plan->cap[j1] = cap_for(std::max(nM1, nN1));
        plan->o1_threads[j1] = default_threads(n1);
        // k_o1 of the 96^2 class in families 3/5/9 is built for 6 waves per SIMD
        // (wst_device.h o1_min_waves): 768-thread workgroups, two per CU
        if (plan->cap[j1] == 136 && plan->o1_threads[j1] == 512 && plan->fam_m == plan->fam_n &&
            (plan->fam_m == 3 || plan->fam_m == 5 || plan->fam_m == 9))
            plan->o1_threads[j1] = 768;
        plan->o2_threads[j1] = default_threads(n1);
        // SQ kernels: the S1 low-pass runs on the level's tap matrices (lds_lowpass_taps) instead
        // of the 1-D taps and permutations
        if (plan->sq)
            plan->o1_lds[j1] = layout(plan->o1_lay[j1], static_cast<size_t>(nM1) * odd_ld(nN1) * sizeof(float2),
                                      0, t, Blocks{j1, j1, false}, 1, 0, omn, Blocks{j1, j1, false}, oms);
        else
            plan->o1_lds[j1] = layout(plan->o1_lay[j1], static_cast<size_t>(nM1) * odd_ld(nN1) * sizeof(float2),
                                      0, t, Blocks{j1, j1, true}, j1, j1, omn);
        if (plan->o1_lds[j1] > static_cast<size_t>(kMaxLds)) return too_big("k_o1", j1);
        if (!do2) continue;
        if (nM1 % 2 != 0 || nN1 % 2 != 0)
            return fail(WST_ERR_UNSUPPORTED, "order-2 level sizes must be even");
        const int hld = nN1 / 2 + 1;
        plan->ws_h_off[j1] = wsp;
        // nM1 + 1 rows per item (LdsLayout::hext: row nM1 = row 0 for the tile folds)
        wsp += static_cast<size_t>(L) * wstdev::hspec_stride(nM1, hld, 1) * sizeof(float2);
        // B holds two paths of level j1+1 or all L paths of level j1+2, whichever is larger; the
        // small SQ classes hold all L paths of level j1+1 (one batch: wstdev::kWholeFirstCap)
        size_t bcap = 2 * pslot(j1 + 1);
        if (j1 + 2 < J) bcap = std::max(bcap, static_cast<size_t>(L) * pslot(j1 + 2));
        if (plan->sq && plan->cap[j1] <= wstdev::kWholeFirstCap)
            bcap = std::max(bcap, static_cast<size_t>(L) * pslot(j1 + 1));
        size_t smax = 0;
        for (int j2 = j1 + 1; j2 < J; ++j2)
            smax = std::max(smax, static_cast<size_t>(paths_per_batch(bcap, pslot(j2), L)) * omn);
        if (plan->sq)   // tap matrices replace the 1-D taps and permutations; M-side tables only;
                        // H holds row nM1 = row 0 (the tile folds' mirrored taps)
            plan->o2_lds[j1] = layout(plan->o2_lay[j1], static_cast<size_t>(nM1 + 1) * hld * sizeof(float2),
                                      bcap * sizeof(float2), t, Blocks{j1, J - 1, false}, 1, 0, smax,
                                      Blocks{j1 + 1, J - 1, false}, oms);
        else
            plan->o2_lds[j1] = layout(plan->o2_lay[j1], static_cast<size_t>(nM1) * hld * sizeof(float2),
                                      bcap * sizeof(float2), t, Blocks{j1, J - 1, true}, j1 + 1, J - 1,
                                      smax);
        if (plan->o2_lds[j1] > static_cast<size_t>(kMaxLds)) return too_big("k_o2", j1);
        plan->o1_lay[j1].hext = plan->o2_lay[j1].hext = 1;
    }
    plan->ws_plane = align16(wsp);
    if (plan->rb > 0)   // staged plans hold ~tens of MB per plane: bound the chunk's workspace
        plan->max_chunk = std::max<int64_t>(1, std::min<int64_t>(2048, kStagedWsBytes / plan->ws_plane));
    if (std::getenv("WST_VERBOSE")) {
        std::fprintf(stderr, "[wst] plan %dx%d J=%d L=%d P=%dx%d fam=(%d,%d) sq=%d prep_lds=%zu\n", M, N, J, L,
                     g.PM, g.PN, plan->fam_m, plan->fam_n, plan->sq, plan->prep_lds);
        for (int j1 = 0; j1 < J; ++j1)
            std::fprintf(stderr, "[wst]   j1=%d cap=%d o1: %d thr %zu B   o2: %d thr %zu B\n", j1,
                         plan->cap[j1], plan->o1_threads[j1], plan->o1_lds[j1], plan->o2_threads[j1],
                         plan->o2_lds[j1]);
    }
    // Wide-output square levels whose k_o2 holds one workgroup per CU because of the level-j1
    // spectrum in LDS (the reference's 128^2 J=2 geometry: 75 KB spectrum + 75 KB path batch): k_o1
    // exports the fully transformed spectrum and k_o2 folds it from HBM / L2, two workgroups per CU.
    plan->o2_export.assign(J, 0);
    plan->o2x_lay.assign(J, LdsLayout{});
    plan->o2x_lds.assign(J, 0);
    plan->o2x_threads.assign(J, 64);
    bool export_on = true;
    if (const char* e = diag_env("WST_O2_EXPORT")) export_on = std::atoi(e) != 0;
    if (const char* e = diag_env("WST_FOLD_ALL")) {   // 0: per-pair passes; r > 0: r rows per workgroup
        const int r = std::atoi(e);
        for (int k = 0; k < plan->nst; ++k) {
            if (plan->fold_all_rows[k] == 0) continue;
            const size_t n = static_cast<size_t>(g.PN >> k);
            plan->fold_all_rows[k] = r;
            plan->fold_all_lds[k] = (n + static_cast<size_t>(L) * std::max(r, 1) * (n | 1)) * sizeof(float2);
        }
    }
    for (int j1 = plan->rb; j1 + 1 < J && max_order >= 2; ++j1) {
        const int nM1 = g.PM >> j1, nN1 = g.PN >> j1, hld = nN1 / 2 + 1;
        // the SQ geometry kernels with the exported spectrum too (diagnostic builds: A/B timing)
        const char* sqx_env = diag_env("WST_SQ_EXPORT");
        const bool sq_export = sqx_env && std::atoi(sqx_env) != 0;
        if (!export_on || (plan->sq && !sq_export) || g.PM != g.PN || plan->fam_m == 0 ||
            plan->fam_m != plan->fam_n || plan->cap[j1] != 136)
            continue;
        size_t bcap = 2 * pslot(j1 + 1);
        if (j1 + 2 < J) bcap = std::max(bcap, static_cast<size_t>(L) * pslot(j1 + 2));
        size_t smax = 0;
        for (int j2 = j1 + 1; j2 < J; ++j2)
            smax = std::max(smax, static_cast<size_t>(paths_per_batch(bcap, pslot(j2), L)) * omn);
        // wide maps are written into the path arrays themselves (no S region); square: M-side
        // twiddle tables serve both dimensions
        const size_t lds =
            plan->sq ? layout(plan->o2x_lay[j1], 0, bcap * sizeof(float2), t, Blocks{j1 + 1, J - 1, false}, 1, 0, smax,
                              Blocks{j1 + 1, J - 1, false}, oms)
                     : layout(plan->o2x_lay[j1], 0, bcap * sizeof(float2), t, Blocks{j1, J - 1, false}, j1 + 1,
                              J - 1, (g.oM > wstdev::kLpOM || g.oN > wstdev::kLpOM) ? 0 : smax);
        // worth it when the freed spectrum lets more workgroups share a CU
        if (kMaxLds / lds <= kMaxLds / plan->o2_lds[j1]) continue;
        const int o1t = fill_cu(plan->o1_threads[j1], plan->o1_lds[j1]);
        if ((nM1 / 2) * hld > 8 * o1t) continue;   // k_o1's in-place split holds 8 items per thread
        plan->o2_export[j1] = 1;
        plan->o2x_lds[j1] = lds;
        plan->o2x_threads[j1] = std::min(fill_cu(default_threads(static_cast<size_t>(nM1) * nN1), lds, 768),
                                         1024);
        plan->o2x_lay[j1].hext = 1;
        set_export_full(plan->o1_lay[j1]);
        // one workgroup per item: splitting its batches over 2 / 4 workgroups of one XCD (as the
        // HG launches after staged levels do) measured slower here (f3 k_o2 1.57 -> 1.67 / 1.66 ms,
        // c1 1.50 -> 1.62): H is 21-75 KB, not the 0.15-0.6 MB of a staged level
        plan->o2x_lay[j1].nsplit = 1;
        if (const char* e = diag_env("WST_O2X_SPLIT")) plan->o2x_lay[j1].nsplit = std::max(1, std::atoi(e));
        plan->o2x_lay[j1].hgroup = 1;
        if (const char* e = diag_env("WST_O2X_GROUP")) plan->o2x_lay[j1].hgroup = std::max(1, std::atoi(e));
    }
    for (int j1 = plan->rb; j1 < J; ++j1) {
        plan->o1_threads[j1] = fill_cu(plan->o1_threads[j1], plan->o1_lds[j1]);
        if (plan->o2_lds[j1] > 0) plan->o2_threads[j1] = fill_cu(plan->o2_threads[j1], plan->o2_lds[j1], 768);
    }
    if (plan->rb == 0) plan->prep_threads = fill_cu(static_cast<int>(plan->prep_threads), plan->prep_lds);
    threads_override("WST_O1_THREADS", plan->o1_threads);
    threads_override("WST_O2_THREADS", plan->o2_threads);
    threads_override("WST_O2X_THREADS", plan->o2x_threads);
    threads_override("WST_HG_THREADS", plan->hg_threads);
    // k_o1's in-place Hermitian split of an exported spectrum holds 8 items per thread: a thread
    // count lowered by an override would silently drop items, so the plan fails instead
    for (int j1 = plan->rb; j1 + 1 < J; ++j1)
        if (export_full(plan->o1_lay[j1]) &&
            static_cast<size_t>((g.PM >> j1) / 2) * ((g.PN >> j1) / 2 + 1) > 8 * static_cast<size_t>(plan->o1_threads[j1]))
            return fail(WST_ERR_INVALID, "k_o1 at level " + std::to_string(j1) + ": " +
                                             std::to_string(plan->o1_threads[j1]) +
                                             " threads cannot hold the exported half spectrum (8 items each)");
    plan->box1_l0.assign(J, -1);
    for (int j = 0; j < J; ++j) plan->box1_l0[j] = box1_off[static_cast<size_t>(j) * L];
    if (device) {
        // every k_o1 / k_o2 the plan launches must be one of the compiled instantiations
        std::string why;
        if (!rc_waves_ok(plan.get(), why)) return fail(WST_ERR_INVALID, why);
        const std::vector<int> w = describe_chunk(plan.get());
        for (size_t i = 0; i < w.size(); i += wstdev::kTraceW) {
            const int kind = w[i] >> 28, fm = (w[i] >> 22) & 63, fn = (w[i] >> 16) & 63, cap = (w[i] >> 4) & 4095;
            const int sq = (w[i] >> 1) & 1, hg = w[i] & 1;
            if ((kind == wstdev::kTkO1 && !wstlaunch::compiled_o1(fm, fn, cap, sq)) ||
                (kind == wstdev::kTkO2 && !wstlaunch::compiled_o2(fm, fn, cap, sq, hg)))
                return fail(WST_ERR_UNSUPPORTED, std::string(kind == wstdev::kTkO1 ? "k_o1" : "k_o2") + "<" +
                                                     std::to_string(fm) + ", " + std::to_string(fn) + ", " +
                                                     std::to_string(cap) + ", " + std::to_string(sq) +
                                                     (kind == wstdev::kTkO2 ? ", " + std::to_string(hg) : "") +
                                                     "> is not compiled (wst_compiled.h; tools/variant_cover.py)");
        }
        WST_HIP_CHECK(plan->ops->set_attrs());
        if (plan->rb > 0) {
            WST_HIP_CHECK(wstlaunch::wst_big_common_ops().set_attrs());
            for (int r = 0; r < plan->nst; ++r) {
                WST_HIP_CHECK(plan->big_r[r]->set_attrs());
                WST_HIP_CHECK(plan->big_c[r]->set_attrs());
            }
        }
    }

    *out = plan.release();
    g_last_error.clear();
    return WST_OK;
}

}  // namespace

extern "C" {

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
    *bytes = static_cast<size_t>(nbatch) * plan->ws_plane;
    return WST_OK;
}

int wst_internal_workspaces(const wst_plan* plan, int* count, size_t* bytes) {
    if (!plan || !count || !bytes) return fail(WST_ERR_INVALID, "plan/count/bytes is NULL");
    std::lock_guard<std::mutex> lk(plan->ws_mu);
    *count = static_cast<int>(plan->ws_by_stream.size());
    size_t b = 0;
    for (const auto& kv : plan->ws_by_stream) b += kv.second.bytes;
    *bytes = b;
    return WST_OK;
}

int wst_plan_staging(const wst_plan* plan, int* rb, int* nst, int* sq) {
    if (!plan || !rb || !nst || !sq) return fail(WST_ERR_INVALID, "plan/rb/nst/sq is NULL");
    *rb = plan->rb;
    *nst = plan->rb > 0 ? plan->nst : 0;
    *sq = plan->sq;
    return WST_OK;
}

int wst_preferred_batch(const wst_plan* plan, int64_t* planes) {
    if (!plan || !planes) return fail(WST_ERR_INVALID, "plan/planes is NULL");
    *planes = plan->max_chunk;
    return WST_OK;
}

}  // extern "C"

namespace {

// Launch-time timer: when `kms` is non-null, every launch (group) is bracketed by events on
// `stream` and its duration is added to kms[slot].  The launches stay back to back: events are
// only recorded while the forward is enqueued, and read after the last one has completed
// (finish), so each kernel runs in the same steady state as in wst_forward (a host wait after
// every kernel let the next one start on an idle, cooler chip: 6 % faster than rocprofv3's
// kernel-trace average of the same launches, round 4).  A segment's begin event is the previous
// segment's end event when nothing was enqueued between them.
struct LaunchTimer {
    float* kms = nullptr;
    int nkms = 0;
    struct Seg {
        int b, e, slot;   // begin / end event indices
    };
    std::vector<hipEvent_t> ev;   // recorded in stream order
    std::vector<Seg> seg;
    int open = -1;                // begin event of the open segment
    ~LaunchTimer() {
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    }
    int init(float* k, int n) {
        kms = k;
        nkms = n;
        if (!kms) return WST_OK;
        for (int i = 0; i < n; ++i) kms[i] = 0.f;
        return WST_OK;
    }
    int record(hipStream_t s) {
        hipEvent_t e = nullptr;
        WST_HIP_CHECK(hipEventCreate(&e));
        ev.push_back(e);
        WST_HIP_CHECK(hipEventRecord(e, s));
        return WST_OK;
    }
    // every enqueue of forward_impl sits inside a segment, so the previous segment's end event
    // (when there is one) also begins the next segment: one marker per kernel boundary
    int begin(hipStream_t s) {
        if (!kms) return WST_OK;
        if (!seg.empty() && seg.back().e == static_cast<int>(ev.size()) - 1) {
            open = seg.back().e;
            return WST_OK;
        }
        const int rc = record(s);
        open = static_cast<int>(ev.size()) - 1;
        return rc;
    }
    int end(hipStream_t s, int slot) {
        if (!kms) return WST_OK;
        const int rc = record(s);
        if (rc != WST_OK) return rc;
        seg.push_back(Seg{open, static_cast<int>(ev.size()) - 1, slot});
        return WST_OK;
    }
    int finish() {
        if (!kms || ev.empty()) return WST_OK;
        WST_HIP_CHECK(hipEventSynchronize(ev.back()));
        for (const Seg& sg : seg) {
            float ms = 0.f;
            WST_HIP_CHECK(hipEventElapsedTime(&ms, ev[sg.b], ev[sg.e]));
            if (sg.slot < nkms) kms[sg.slot] += ms;
        }
        return WST_OK;
    }
};

// One LDS-resident level j1: k_o1 (S1 + U1 half-spectrum export), then k_o2 (every S2 of j1).
int resident_level(const wst_plan* plan, int j1, int nimg, long long img0, unsigned char* base,
                   int64_t chunk, const float2* xhat, float* d_out, int pooled, hipStream_t stream,
                   LaunchTimer& timer, int& site) {
    const wst::Geometry& g = plan->g;
    const bool do2 = g.max_order >= 2 && j1 < g.J - 1;
    float2* hexp = do2 ? reinterpret_cast<float2*>(base + plan->ws_h_off[j1] * chunk) : nullptr;
    int rc;
    if ((rc = timer.begin(stream)) != WST_OK) return rc;
    LdsLayout lay1 = plan->o1_lay[j1];
    set_tslot(lay1, site++);
    if (!plan->ops->o1(plan->cap[j1], plan->sq,
                       Launch{dim3(nimg * g.L), dim3(plan->o1_threads[j1]), plan->o1_lds[j1], stream},
                       plan->dp, lay1, j1, nimg, img0, xhat, hexp, d_out, pooled))
        return fail(WST_ERR_UNSUPPORTED, "k_o1 variant not compiled (wst_compiled.h)");
    WST_HIP_CHECK(hipGetLastError());
    if ((rc = timer.end(stream, 1 + j1)) != WST_OK) return rc;
    if (!do2) return WST_OK;
    if ((rc = timer.begin(stream)) != WST_OK) return rc;
    if (plan->o2_export[j1]) {   // spectrum exported fully transformed: fold from HBM
        LdsLayout lx = plan->o2x_lay[j1];
        set_tslot(lx, site++);
        if (!plan->ops->o2(136, plan->sq, 1, Launch{dim3(nimg * g.L * std::max(1, plan->o2x_lay[j1].nsplit)),
                                             dim3(plan->o2x_threads[j1]), plan->o2x_lds[j1], stream},
                           plan->dp, lx, j1, nimg, img0, hexp, d_out, pooled, j1 + 1))
            return fail(WST_ERR_UNSUPPORTED, "k_o2 variant not compiled (wst_compiled.h)");
        WST_HIP_CHECK(hipGetLastError());
        return timer.end(stream, 1 + g.J + j1);
    }
    LdsLayout lay2 = plan->o2_lay[j1];
    set_tslot(lay2, site++);
    if (!plan->ops->o2(plan->cap[j1], plan->sq, 0,
                       Launch{dim3(nimg * g.L), dim3(plan->o2_threads[j1]), plan->o2_lds[j1], stream},
                       plan->dp, lay2, j1, nimg, img0, hexp, d_out, pooled, j1 + 1))
        return fail(WST_ERR_UNSUPPORTED, "k_o2 variant not compiled (wst_compiled.h)");
    WST_HIP_CHECK(hipGetLastError());
    return timer.end(stream, 1 + g.J + j1);
}

// The HBM-staged levels r < rb of one chunk (wst_staged.h): S0 + Xhat, then per staged j1 the
// order-1 path (S1, U1hat) and its order-2 paths (staged while j2 < nst, then k_o2 on the global
// spectrum).  Level r is m x n = (PM >> r) x (PN >> r): row passes run lines of n points (big_r),
// column passes lines of m points (big_c).  Timing slots as the resident kernels: prep, o1 at j1,
// o2 at j1.
int staged_levels(const wst_plan* plan, const float* in, int nimg, long long img0,
                  unsigned char* base, int64_t chunk, float* d_out, int pooled, hipStream_t stream,
                  LaunchTimer& timer, int& site) {
    using namespace wstbig;
    const wst::Geometry& g = plan->g;
    const DevParams& dp = plan->dp;
    const int J = g.J, L = g.L, PM = g.PM, PN = g.PN, nq = (L + 1) / 2;
    const int noms = plan->noms;
    const auto& cm = wstlaunch::wst_big_common_ops();
    float2* xhat = reinterpret_cast<float2*>(base);
    float2* tmp = reinterpret_cast<float2*>(base + plan->ws_tmp * chunk);
    float2* colt = reinterpret_cast<float2*>(base + plan->ws_colt * chunk);
    float* part = reinterpret_cast<float*>(base + plan->ws_part * chunk);
    float* csum = reinterpret_cast<float*>(base + plan->ws_csum * chunk);
    // [plane][kMeanParts] partial sums, then [plane * L + l1] U1 means
    float* mean = reinterpret_cast<float*>(base + plan->ws_mean * chunk);
    float* umean = mean + static_cast<size_t>(nimg) * kMeanParts;
    const dim3 tb(kBigThreads);
    auto gnat = [&](int r, int d) { return plan->d_lpn + plan->lpn_off[2 * r + d]; };
    // row pass over level r: lines of PN >> r points, PM >> r rows
    auto rargs = [&](int mode, int r) {
        BigArgs a{};
        a.mode = mode;
        a.n = PN >> r;
        a.nrows = PM >> r;
        a.lvl = r;
        a.rows = big_rows(mode, PM >> r);
        a.L = L;
        a.img0 = img0;
        a.oms = noms;
        a.tslot = site++;
        return a;
    };
    // column pass over level r: lines of PM >> r points, `ncols` columns
    auto cargs = [&](int mode, int r, int ncols) {
        BigArgs a{};
        a.mode = mode;
        a.n = PM >> r;
        a.ncols = ncols;
        a.lvl = r;
        a.L = L;
        a.img0 = img0;
        a.oms = noms;
        a.g_lds = plan->big_g_lds[r];
        a.tslot = site++;
        return a;
    };
    auto col_grid = [&](int ncols, int arrays) { return dim3((ncols + kColTile - 1) / kColTile, arrays); };
    const size_t sbytes = static_cast<size_t>(g.oM) * g.oN * sizeof(float);   // k_big_final's S
    int rc;
    // ---- S0 and Xhat (level 0) ----
    if ((rc = timer.begin(stream)) != WST_OK) return rc;
    cm.mean(Launch{dim3(nimg, kMeanParts), tb, 0, stream}, dp, in, mean);
    {
        BigArgs a = rargs(kRowPad, 0);
        a.in = in;
        a.mean = mean;
        a.tpart = part;
        a.gnat = gnat(0, 1);
        a.dst = xhat;
        plan->big_r[0]->rows(false, Launch{dim3(PM / a.rows, nimg), tb, plan->big_rows_lds[0], stream}, dp, a);
        BigArgs c = cargs(kColStore, 0, PN);
        c.dst = xhat;
        plan->big_c[0]->cols(false, Launch{col_grid(PN, nimg), dim3(wstbig::big_col_threads(plan->big_c[0]->n)), plan->big_cols_lds[0], stream}, dp, c);
        cm.final_(Launch{dim3(nimg), dim3(64), sbytes, stream}, dp, kFinalRows, 0, PM, PN, noms, part,
                  gnat(0, 0), nullptr, nullptr, L, 0, 0, 0, 1, img0, d_out, pooled);
    }
    WST_HIP_CHECK(hipGetLastError());
    if ((rc = timer.end(stream, 0)) != WST_OK) return rc;

    for (int j1 = 0; j1 < plan->rb; ++j1) {
        const int m1 = PM >> j1, n1 = PN >> j1;
        const bool do2 = g.max_order >= 2 && j1 < J - 1;
        float2* hbig = do2 ? reinterpret_cast<float2*>(base + plan->ws_hbig[j1] * chunk) : nullptr;
        // ---- order 1: fold + inverse rows, inverse columns + |.| + low-pass partials, S1 ----
        if ((rc = timer.begin(stream)) != WST_OK) return rc;
        BigArgs a = rargs(kRowFold1, j1);
        a.xhat = xhat;
        a.j1 = j1;
        a.dst = tmp;
        plan->big_r[j1]->rows(true, Launch{dim3(m1 / a.rows, nimg * L), tb, plan->big_rows_lds[j1], stream}, dp, a);
        // (order 2 follows: the column pass also forms the column spectra of U1, kColModLpFwd)
        BigArgs c = cargs(do2 ? kColModLpFwd : kColModLp, j1, n1);
        c.dst = tmp;
        c.colt = do2 ? colt : nullptr;
        c.vpart = part;
        c.csum = csum;
        c.scale = 1.f / (static_cast<float>(g.PM) * static_cast<float>(g.PN));
        c.gnat = gnat(j1, 0);
        plan->big_c[j1]->cols(true, Launch{col_grid(n1, nimg * L), dim3(wstbig::big_col_threads(plan->big_c[j1]->n)), plan->big_cols_lds[j1], stream}, dp, c);
        cm.final_(Launch{dim3(nimg * L), dim3(64), sbytes, stream}, dp, kFinalCols, 1, n1, m1, noms, part,
                  gnat(j1, 1), csum, do2 ? umean : nullptr, L, j1, 0, 0, 1, img0, d_out, pooled);
        if (do2) {
            // U1hat = fft2(U1 - mean) as half spectra (natural order) for the order-2 folds: the
            // row transforms of the column spectra's rows 0..m1/2, written with their mirrors
            BigArgs r2 = rargs(kRowHalf, j1);
            r2.nrows = m1 / 2 + 1;
            r2.rows = 2 * kBigRows;
            r2.colt = colt;
            r2.csum = csum;
            r2.mean = umean;
            r2.dst = hbig;
            plan->big_r[j1]->rows(false, Launch{dim3((r2.nrows + r2.rows - 1) / r2.rows, nimg * L), tb,
                                                plan->big_rows_lds[j1], stream}, dp, r2);
        }
        WST_HIP_CHECK(hipGetLastError());
        if ((rc = timer.end(stream, 1 + j1)) != WST_OK) return rc;
        if (!do2) continue;
        // ---- order 2 from the staged U1hat ----
        if ((rc = timer.begin(stream)) != WST_OK) return rc;
        for (int j2 = j1 + 1; j2 < plan->nst; ++j2) {
            const int m2 = PM >> j2, n2 = PN >> j2;
            for (int l1 = 0; l1 < L; ++l1) {
                BigArgs f = rargs(kRowFold2, j2);
                f.hsrc = hbig;
                f.n1 = n1;
                f.l1 = l1;
                f.j2 = j2;
                f.psi2 = dp.psi2 + plan->psi2_off_host[(static_cast<size_t>(j2) * J + j1) * nq];
                f.pstride = static_cast<long long>(m1) * n1;
                f.box = plan->d_box + plan->box_off_host[static_cast<size_t>(j2) * J + j1];
                f.npair = nq;
                f.npath = L;
                f.dst = tmp;
                size_t flds = plan->big_rows_lds[j2];
                if (m1 == 2 * m2 && plan->fold_all_rows[j2] > 0) {
                    f.fold_all = 1;
                    f.rows = plan->fold_all_rows[j2];
                    flds = plan->fold_all_lds[j2];
                }
                plan->big_r[j2]->rows(true, Launch{dim3(m2 / f.rows, nimg), tb, flds, stream}, dp, f);
                BigArgs mc = cargs(kColModLp, j2, n2);
                mc.dst = tmp;
                mc.vpart = part + static_cast<size_t>(l1) * nimg * L * n2 * noms;
                mc.csum = csum + static_cast<size_t>(l1) * nimg * L * n2;
                mc.scale = 1.f / (static_cast<float>(m1) * static_cast<float>(n1));
                mc.gnat = gnat(j2, 0);
                plan->big_c[j2]->cols(true, Launch{col_grid(n2, nimg * L), dim3(wstbig::big_col_threads(plan->big_c[j2]->n)), plan->big_cols_lds[j2], stream}, dp, mc);
            }
            // S2 of every theta1 in one launch (l1 = -1: blockIdx.y)
            cm.final_(Launch{dim3(nimg * L, L), dim3(64), sbytes, stream}, dp, kFinalCols, 2, n2, m2, noms,
                      part, gnat(j2, 1), nullptr, nullptr, L, j1, -1, j2, L, img0, d_out, pooled);
        }
        const int j2f = plan->hg_j2first[j1];
        if (j2f < J) {
            LdsLayout lh = plan->hg_lay[j1];
            set_tslot(lh, site++);
            if (!plan->ops->o2(136, 1, 1, Launch{dim3(nimg * L * std::max(1, plan->hg_lay[j1].nsplit)),
                                                 dim3(plan->hg_threads[j1]), plan->hg_lds[j1], stream},
                               dp, lh, j1, nimg, img0, hbig, d_out, pooled, j2f))
                return fail(WST_ERR_UNSUPPORTED, "k_o2 variant not compiled (wst_compiled.h)");
        }
        WST_HIP_CHECK(hipGetLastError());
        if ((rc = timer.end(stream, 1 + J + j1)) != WST_OK) return rc;
    }
    return WST_OK;
}

// Timing slots of wst_forward_profiled: [0] k_prep, [1 + j1] k_o1 at j1, [1 + J + j1] k_o2 at j1.
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
    const size_t plane_ws = plan->ws_plane;
    void* ws = d_workspace;
    size_t wsb = workspace_bytes;
    std::unique_lock<std::mutex> ws_lock;   // held through the enqueue on an internal buffer
    wst_plan::StreamWs* used = nullptr;
    if (!ws) {
        // internal workspace of this stream: up to max_chunk planes per chunk.  At most
        // kMaxStreamWs streams keep one: a new stream evicts the least recently used buffer once
        // that buffer's last work has completed (its event; valid even if its stream is gone)
        const int64_t want = std::min<int64_t>(nbatch, plan->max_chunk);
        ws_lock = std::unique_lock<std::mutex>(plan->ws_mu);
        // a while, not an if: the lock is dropped while a busy victim drains, and other streams
        // may insert meanwhile, so the bound is checked again after every eviction
        while (plan->ws_by_stream.find(stream) == plan->ws_by_stream.end() &&
               plan->ws_by_stream.size() >= kMaxStreamWs) {
            // prefer an entry whose last work has already completed (least recently used among
            // those); otherwise take the LRU entry out of the map and wait for it with the lock
            // dropped, so other streams' calls on this plan do not block behind it
            auto lru = plan->ws_by_stream.end(), idle = plan->ws_by_stream.end();
            for (auto it = plan->ws_by_stream.begin(); it != plan->ws_by_stream.end(); ++it) {
                if (lru == plan->ws_by_stream.end() || it->second.tick < lru->second.tick) lru = it;
                const bool done = !it->second.done || hipEventQuery(it->second.done) == hipSuccess;
                if (done && (idle == plan->ws_by_stream.end() || it->second.tick < idle->second.tick)) idle = it;
            }
            const bool have_idle = idle != plan->ws_by_stream.end();
            const auto victim = have_idle ? idle : lru;
            const wst_plan::StreamWs ev = victim->second;
            plan->ws_by_stream.erase(victim);
            if (!have_idle && ev.done) {
                ws_lock.unlock();
                const hipError_t se = hipEventSynchronize(ev.done);
                ws_lock.lock();
                if (se != hipSuccess) {
                    if (ev.ptr) (void)hipFree(ev.ptr);
                    (void)hipEventDestroy(ev.done);
                    WST_HIP_CHECK(se);
                }
            }
            if (ev.ptr) (void)hipFree(ev.ptr);
            if (ev.done) (void)hipEventDestroy(ev.done);
        }
        wst_plan::StreamWs& sw = plan->ws_by_stream[stream];
        sw.tick = ++plan->ws_tick;
        used = &sw;
        if (sw.bytes < static_cast<size_t>(want) * plane_ws) {
            if (sw.ptr) {
                // only this stream's calls use the buffer: once it drains, the buffer is idle
                WST_HIP_CHECK(hipStreamSynchronize(stream));
                (void)hipFree(sw.ptr);
                sw.ptr = nullptr;
                sw.bytes = 0;
            }
            WST_HIP_CHECK(hipMalloc(&sw.ptr, static_cast<size_t>(want) * plane_ws));
            sw.bytes = static_cast<size_t>(want) * plane_ws;
        }
        ws = sw.ptr;
        wsb = sw.bytes;
        if (!sw.done) WST_HIP_CHECK(hipEventCreateWithFlags(&sw.done, hipEventDisableTiming));
    }
    const int64_t cap = std::min<int64_t>(static_cast<int64_t>(wsb / plane_ws), plan->max_chunk);
    if (cap < 1) return fail(WST_ERR_INVALID, "workspace smaller than one plane's share");
    // balanced chunks: the fewest launches the workspace allows, all of (nearly) equal size (c2's
    // 3072 planes as 2 x 1536 rather than 2048 + 1024: equal per-plane cost, measured 0.4 % faster)
    const int64_t nchunks = (nbatch + cap - 1) / cap;
    const int64_t chunk = (nbatch + nchunks - 1) / nchunks;
    const int inM = plan->dp.pre_pad ? g.PM : g.M, inN = plan->dp.pre_pad ? g.PN : g.N;
    // workspace regions (chunk-sized): Xhat, then each level's half spectra
    unsigned char* base = reinterpret_cast<unsigned char*>(ws);
    float2* xhat = reinterpret_cast<float2*>(base);
    LaunchTimer timer;
    int rc;
    if ((rc = timer.init(kms, nkms)) != WST_OK) return rc;
    for (int64_t c0 = 0; c0 < nbatch; c0 += chunk) {
        const int nimg = static_cast<int>(std::min<int64_t>(chunk, nbatch - c0));
        const long long img0 = static_cast<long long>(c0);
        int site = 0;   // variant-trace sites, in launch order (describe_chunk)
        if (plan->rb > 0) {
            if ((rc = staged_levels(plan, d_in + c0 * inM * inN, nimg, img0, base, chunk, d_out, pooled,
                                    stream, timer, site)) != WST_OK)
                return rc;
            for (int j1 = plan->rb; j1 < g.J; ++j1)
                if ((rc = resident_level(plan, j1, nimg, img0, base, chunk, xhat, d_out, pooled, stream,
                                         timer, site)) != WST_OK)
                    return rc;
            continue;
        }
        if ((rc = timer.begin(stream)) != WST_OK) return rc;
        LdsLayout lp = plan->prep_lay;
        set_tslot(lp, site++);
        plan->ops->prep(Launch{dim3(nimg), dim3(plan->prep_threads), plan->prep_lds, stream},
                        plan->dp, lp, d_in + c0 * inM * inN, img0, xhat, d_out, pooled);
        WST_HIP_CHECK(hipGetLastError());
        if ((rc = timer.end(stream, 0)) != WST_OK) return rc;
        for (int j1 = 0; j1 < g.J; ++j1)
            if ((rc = resident_level(plan, j1, nimg, img0, base, chunk, xhat, d_out, pooled, stream,
                                     timer, site)) != WST_OK)
                return rc;
    }
    if (used) WST_HIP_CHECK(hipEventRecord(used->done, stream));   // the buffer is busy until here
    if (ws_lock.owns_lock()) ws_lock.unlock();                       // no host wait under the lock
    return timer.finish();
}

// ------------------------------------------------------------------------------------------
// Host mirror of the kernels' run-time dispatch: the trace words (wst_device.h kTraceW) every
// launch site of one chunk writes, predicted from the plan alone.  Mirrors k_prep / k_o1 / k_o2
// (wst_device.h) and the staged passes (wst_staged.h); tests check it against the device trace.
// ------------------------------------------------------------------------------------------
using namespace wstdev;

bool rc_ok(int k) { return k > 0 && mfma_k_steps(k) <= 18; }
int lp_form(bool sq, bool wide, int k) { return sq ? kLpTap : wide ? (rc_ok(k) ? kLpMfmaRc : kLpMfma) : kLpPlain; }

struct Describe {
    const wst_plan* plan;
    std::vector<int> w;
    std::vector<int> thr;   // workgroup size of each site
    int* site(int threads) {
        thr.push_back(threads);
        w.resize(w.size() + kTraceW, 0);
        return w.data() + w.size() - kTraceW;
    }
};

void describe_prep(Describe& d) {
    const wst_plan* pl = d.plan;
    const wst::Geometry& g = pl->g;
    const int FM = pl->fam_m, FN = pl->fam_n;
    int pc = 0;
    if (FM == FN && FM > 0)
        for (int mc = 0; mc < 8 && !pc; ++mc) {
            const int PC = FM << mc;
            if (PC > 48 && PC <= 136 && g.PM == PC && g.PN == PC) pc = PC;
        }
    const bool wide = g.oM > kLpOM || g.oN > kLpOM;
    int* t = d.site(pl->prep_threads);
    t[0] = tr_kernel(kTkPrep, FM, FN, 0, 0, 0);
    t[1] = tr_prep(pc, wide ? (rc_ok(pc) ? kLpMfmaRc : kLpMfma) : kLpPlain);
}

void describe_o1(Describe& d, int j1) {
    const wst_plan* pl = d.plan;
    const wst::Geometry& g = pl->g;
    const int FM = pl->fam_m, FN = pl->fam_n, MAXN = pl->cap[j1];
    const int SQ = (FM == FN && FM > 0 && pl->sq) ? 1 : 0;
    const LdsLayout& lay = pl->o1_lay[j1];
    int oc = 0, n1t = 0;
    if (SQ && MAXN == 136 && g.oM == 4 && g.oN == 4 && lay.oms == 4) {
        oc = 4;
    } else if (!SQ && FM == FN && FM > 0 && g.PM == g.PN) {
        for (int mc = 0; mc < 8 && !n1t; ++mc) {
            const int n1x = FM << mc;
            if (n1x <= MAXN && n1x > prev_cap(MAXN) && (g.PM >> j1) == n1x) n1t = n1x;
        }
    }
    const int n1c = n1t ? n1t : SQ ? unique_level(FM, MAXN) : 0;
    const bool fuse1 = SQ && n1c >= kFuse1Min && wstfft::split_n2(n1c) > 1;
    const bool fused1 = fuse1 && j1 == 0;
    const bool do2 = g.max_order >= 2 && j1 < g.J - 1;
    const int s1 = 1 << j1;
    const bool box1 = pl->box1_l0[j1] >= 0 && s1 >= pl->dp.box1_min_s;
    const int f1 = fused1 ? 0 : s1 == 1 ? 1 : s1 == 2 ? 2 : box1 ? 3 : s1 == 4 ? 4 : 5;
    const bool wide = g.oM > kLpOM || g.oN > kLpOM;
    int* t = d.site(pl->o1_threads[j1]);
    t[0] = tr_kernel(kTkO1, FM, FN, MAXN, SQ, 0);
    t[1] = tr_o1(oc, n1c, fused1 ? 1 : 0, lp_form(SQ, wide, n1c), do2 ? 1 : 0, export_full(lay), f1);
}

void describe_o2(Describe& d, int j1, const LdsLayout& lay, int MAXN, int sq, int HG, int j2first,
                 int threads) {
    const wst_plan* pl = d.plan;
    const wst::Geometry& g = pl->g;
    const int FM = pl->fam_m, FN = pl->fam_n, J = g.J, L = g.L, PM = g.PM, PN = g.PN;
    const bool square_fam = FM == FN && FM > 0;
    const int SQ = (square_fam && sq) ? 1 : 0;
    if (!square_fam) HG = 0;   // FamilyOps::o2 of a non-square pair has no HG kernels
    int oc = 0, lc = 0;
    if (SQ && g.oM == 4 && g.oN == 4 && lay.oms == 4) {
        oc = 4;
        lc = (unique_level(FM, MAXN) > 0 && L == 8) ? 8 : 0;
    } else if (!SQ && HG && square_fam && L == 8) {
        lc = 8;
    }
    const int n1c = (SQ && !HG) ? unique_level(FM, MAXN) : 0;
    const int spec = HG ? 0 : (n1c > 0 && wstfft::split_n2(n1c) > 1) ? 1 : 2;
    const bool wide = g.oM > kLpOM || g.oN > kLpOM;
    int* t = d.site(threads);
    auto level = [&](int j2, int pb, int sc, int nc) {
        const int n1f = (SQ && nc > 0 && sc > 0) ? nc * sc : 0;
        const bool fuse = n1f > 0 && sc == 2 && n1f / 2 >= kFuseMin && wstfft::split_n2(n1f / 2) > 1;
        const int s2 = 1 << (j2 - j1);
        const int fk = fuse ? kFdFused : (n1f > 0 && sc == 2) ? kFdTileS2
                     : (n1f > 0 && (sc == 4 || sc == 8)) ? kFdTileList : s2 == 2 ? kFdDenseS2 : kFdBox;
        if (2 + (j2 - j1 - 1) < kTraceW) t[2 + (j2 - j1 - 1)] = tr_level(j2, pb, sc, nc, fk, lp_form(SQ, wide, nc), s2);
    };
    int branch = 7;
    if (n1c > 0) {
        branch = 1;
        for (int k = 1; k < 8; ++k) {
            const int nn2 = n1c >> k;
            if ((nn2 << k) == n1c && nn2 >= 1 && j1 + k < J && j1 + k >= j2first)
                level(j1 + k, lc == 0 ? 0 : (k == 1 && MAXN > kWholeFirstCap) ? 2 : lc, 1 << k, nn2);
        }
    } else if (SQ && HG && unique_level(FM, MAXN) > 0) {
        const int n2c = unique_level(FM, MAXN);
        if (j2first == j1 + 1 && (PM >> j1) == n2c && PM == PN) {
            branch = 2;
            for (int k = 1; k < 8; ++k) {
                const int nn2 = n2c >> k;
                if ((nn2 << k) == n2c && nn2 >= 1 && j1 + k < J)
                    level(j1 + k, lc == 0 ? 0 : k == 1 ? 2 : lc, 1 << k, nn2);
            }
        } else if ((PM >> j2first) == n2c) {
            branch = 3;
            for (int k = 0; k < 8; ++k) {
                const int nn2 = n2c >> k;
                if ((nn2 << k) == n2c && nn2 >= 1 && j2first + k < J) level(j2first + k, 0, 0, 0);
            }
        } else {
            branch = 4;
            for (int j2 = j2first; j2 < J; ++j2) level(j2, 0, 0, 0);
        }
    } else if (!SQ && HG && square_fam) {
        int n1x = 0;
        if (PM == PN && j2first == j1 + 1)
            for (int mc = 0; mc < 8 && !n1x; ++mc) {
                const int c = FM << mc;
                if (c <= MAXN && c > prev_cap(MAXN) && (PM >> j1) == c) n1x = c;
            }
        if (n1x) {
            branch = 5;
            for (int k = 1; k < 8; ++k) {
                const int nn2 = n1x >> k;
                if ((nn2 << k) == n1x && nn2 >= 1 && j1 + k < J) level(j1 + k, lc == 0 ? 0 : k == 1 ? 2 : lc, 0, nn2);
            }
        } else {
            branch = 6;
            for (int j2 = j2first; j2 < J; ++j2) level(j2, 0, 0, 0);
        }
    } else {
        for (int j2 = j2first; j2 < J; ++j2) level(j2, 0, 0, 0);
    }
    (void)PN;
    t[0] = tr_kernel(kTkO2, FM, FN, MAXN, SQ, HG);
    t[1] = tr_o2(oc, lc, n1c, spec, branch);
}

void describe_big(Describe& d, bool rows, int n, bool inv, int body) {
    int* t = d.site(rows ? wstbig::kBigThreads : wstbig::big_col_threads(n));
    t[0] = tr_kernel(rows ? kTkBigRows : kTkBigCols, 0, 0, n, 0, inv ? 1 : 0);
    t[1] = body;
}

// One chunk's launch sites in forward_impl's order (staged_levels / resident_level).
Describe describe_sites(const wst_plan* pl) {
    Describe d{pl, {}, {}};
    const wst::Geometry& g = pl->g;
    const int J = g.J, L = g.L;
    const int wide_maps = g.oM > 8 ? 1 : 0;
    auto resident = [&](int j1) {
        describe_o1(d, j1);
        if (!(g.max_order >= 2 && j1 < J - 1)) return;
        if (pl->o2_export[j1]) describe_o2(d, j1, pl->o2x_lay[j1], 136, pl->sq, 1, j1 + 1, pl->o2x_threads[j1]);
        else describe_o2(d, j1, pl->o2_lay[j1], pl->cap[j1], pl->sq, 0, j1 + 1, pl->o2_threads[j1]);
    };
    if (pl->rb > 0) {
        using namespace wstbig;
        describe_big(d, true, pl->big_r[0]->n, false, tr_big(kRowPad, 0, 0, 0, 0, 0, 0));
        describe_big(d, false, pl->big_c[0]->n, false, tr_big(kColStore, 0, 0, 0, 0, 0, 0));
        for (int j1 = 0; j1 < pl->rb; ++j1) {
            const bool do2 = g.max_order >= 2 && j1 < J - 1;
            describe_big(d, true, pl->big_r[j1]->n, true, tr_big(kRowFold1, 0, j1 == 0 ? 1 : 2, 0, 0, 0, 0));
            describe_big(d, false, pl->big_c[j1]->n, true,
                         tr_big(do2 ? kColModLpFwd : kColModLp, 0, 0, 0, wide_maps, pl->big_g_lds[j1], 0));
            if (!do2) continue;
            describe_big(d, true, pl->big_r[j1]->n, false, tr_big(kRowHalf, 0, 0, 0, 0, 0, 0));
            for (int j2 = j1 + 1; j2 < pl->nst; ++j2) {
                const int m1 = g.PM >> j1, m2 = g.PM >> j2;
                const bool fold_all = m1 == 2 * m2 && pl->fold_all_rows[j2] > 0;
                const bool box = !fold_all && (1 << (j2 - j1)) >= 4;
                for (int l1 = 0; l1 < L; ++l1) {
                    describe_big(d, true, pl->big_r[j2]->n, true, tr_big(kRowFold2, fold_all ? 1 : 0, 0, box ? 1 : 0, 0, 0, 0));
                    describe_big(d, false, pl->big_c[j2]->n, true,
                                 tr_big(kColModLp, 0, 0, 0, wide_maps, pl->big_g_lds[j2], 0));
                }
            }
            const int j2f = pl->hg_j2first[j1];
            if (j2f < J) describe_o2(d, j1, pl->hg_lay[j1], 136, 1, 1, j2f, pl->hg_threads[j1]);
        }
        for (int j1 = pl->rb; j1 < J; ++j1) resident(j1);
    } else {
        describe_prep(d);
        for (int j1 = 0; j1 < J; ++j1) resident(j1);
    }
    return d;
}
std::vector<int> describe_chunk(const wst_plan* pl) { return describe_sites(pl).w; }

// lds_lowpass_mfma_rc keeps one column tile per wave: every launch that takes it needs at least
// oNp / 16 waves (true of every plan's default launch shapes; a thread override could break it)
bool rc_waves_ok(const wst_plan* pl, std::string& why) {
    const Describe d = describe_sites(pl);
    const int nnt = ((pl->g.oN + 15) & ~15) >> 4;
    for (size_t s = 0; s < d.thr.size(); ++s) {
        const int* t = d.w.data() + s * kTraceW;
        const int kind = t[0] >> 28;
        bool rc = (kind == kTkPrep && ((t[1] >> 8) & 3) == kLpMfmaRc) ||
                  (kind == kTkO1 && ((t[1] >> 13) & 3) == kLpMfmaRc);
        if (kind == kTkO2)
            for (int k = 2; k < kTraceW; ++k) rc = rc || ((t[k] & 1) && ((t[k] >> 5) & 3) == kLpMfmaRc);
        if (rc && d.thr[s] / 64 < nnt) {
            why = "launch " + std::to_string(s) + " has " + std::to_string(d.thr[s] / 64) + " waves for " +
                  std::to_string(nnt) + " MFMA low-pass column tiles";
            return false;
        }
    }
    return true;
}

int copy_words(const std::vector<int>& w, int32_t* out, int64_t max_words, int64_t* nwords) {
    if (!nwords) return fail(WST_ERR_INVALID, "nwords is NULL");
    *nwords = static_cast<int64_t>(w.size());
    if (out) {
        if (max_words < static_cast<int64_t>(w.size())) return fail(WST_ERR_INVALID, "output buffer too small");
        for (size_t i = 0; i < w.size(); ++i) out[i] = w[i];
    }
    return WST_OK;
}

}  // namespace

extern "C" {

int wst_plan_variants(const wst_plan* plan, int32_t* out, int64_t max_words, int64_t* nwords) {
    if (!plan) return fail(WST_ERR_INVALID, "plan is NULL");
    return copy_words(describe_chunk(plan), out, max_words, nwords);
}

int wst_describe_variants(int M, int N, int J, int L, int max_order, int32_t* out, int64_t max_words,
                          int64_t* nwords) {
    wst_plan* p = nullptr;
    const int rc = create_plan(M, N, J, L, max_order, 0, nullptr, false, &p);
    if (rc != WST_OK) return rc;
    std::string why;   // the device plan's launch-shape check, here too (the CPU sweep runs it)
    if (!rc_waves_ok(p, why)) {
        free_plan(p);
        return fail(WST_ERR_INVALID, why);
    }
    const std::vector<int> w = describe_chunk(p);
    free_plan(p);
    return copy_words(w, out, max_words, nwords);
}

int wst_plan_trace(wst_plan* plan, int enable) {
    if (!plan) return fail(WST_ERR_INVALID, "plan is NULL");
    if (plan->host_only) return fail(WST_ERR_INVALID, "host-only plan");
#ifndef WST_TRACE
    if (enable)
        return fail(WST_ERR_UNSUPPORTED, "this library has no trace code: the variant trace is in "
                                         "libwst_hip_trace.so (same sources, -DWST_TRACE)");
#endif
    // The trace switch changes the kernel parameters every later launch copies and clears the
    // trace area: it needs a quiescent plan.  Calls that overlap forwards on other host threads are
    // serialised against their launches (ws_mu), and the device is drained first, so no launch in
    // flight writes the area being cleared (header: wst_plan_trace).
    std::lock_guard<std::mutex> lk(plan->ws_mu);
    WST_HIP_CHECK(hipDeviceSynchronize());
    if (!enable) {
        plan->dp.flags &= ~kFlagTrace;
        return WST_OK;
    }
    if (describe_chunk(plan).size() > static_cast<size_t>(kTraceSites) * kTraceW)
        return fail(WST_ERR_UNSUPPORTED, "plan has more launch sites per chunk than the trace holds (" +
                                             std::to_string(kTraceSites) + ")");
    const size_t bytes = static_cast<size_t>(kTraceSites) * kTraceW * sizeof(int);
    WST_HIP_CHECK(hipMemset(plan->d_o2 + static_cast<size_t>(plan->g.J) * plan->g.L, 0, bytes));
    plan->dp.flags |= kFlagTrace;
    return WST_OK;
}

int wst_plan_read_trace(const wst_plan* plan, int32_t* out, int64_t max_words, int64_t* nwords) {
    if (!plan || !out || !nwords) return fail(WST_ERR_INVALID, "plan/out/nwords is NULL");
    if (!(plan->dp.flags & kFlagTrace)) return fail(WST_ERR_INVALID, "tracing is off (wst_plan_trace)");
    const int64_t n = static_cast<int64_t>(describe_chunk(plan).size());
    if (n > static_cast<int64_t>(kTraceSites) * kTraceW)   // never truncated to a shape unlike the mirror's
        return fail(WST_ERR_UNSUPPORTED, "plan has more launch sites per chunk than the trace holds");
    if (max_words < n) return fail(WST_ERR_INVALID, "output buffer too small");
    WST_HIP_CHECK(hipDeviceSynchronize());
    WST_HIP_CHECK(hipMemcpy(out, plan->d_o2 + static_cast<size_t>(plan->g.J) * plan->g.L,
                            static_cast<size_t>(n) * sizeof(int), hipMemcpyDeviceToHost));
    *nwords = n;
    return WST_OK;
}

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
    return wst_host_filter_ex(M, N, J, L, kind, j, l, r, nullptr, out, len);
}

int wst_host_filter_ex(int M, int N, int J, int L, int kind, int j, int l, int r,
                       const wst_filter_convention* conv_in, double* out, int64_t len) {
    if (!out) return fail(WST_ERR_INVALID, "out is NULL");
    wst::FilterConvention conv;
    if (!to_convention(conv_in, conv)) return WST_ERR_INVALID;
    if (J < 1) return fail(WST_ERR_INVALID, "J must be >= 1");
    wst::Geometry g;
    std::string err;
    if (!wst::make_geometry(M, N, J, L, 2, g, err)) return fail(WST_ERR_INVALID, err);
    try {
        // cache the last bank: the test-suite inspects every filter of one geometry in turn
        static thread_local std::unique_ptr<wst::FilterBank> cached;
        if (!cached || cached->g.M != M || cached->g.N != N || cached->g.J != J || cached->g.L != L ||
            cached->conv.norm_pi != conv.norm_pi || cached->conv.periodize_half != conv.periodize_half ||
            cached->conv.rot_f32 != conv.rot_f32)
            cached.reset(new wst::FilterBank(wst::build_filter_bank(g, conv)));
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
    if (!data || n < 1 || nb < 1 || nl < 1 || threads < 1 || mode < 0 || mode > 4)
        return fail(WST_ERR_INVALID, "bad arguments");
    bool perm_done = false;
    std::vector<float2> tw(static_cast<size_t>(n));
    for (int k = 0; k < n; ++k) {
        const double a = 2.0 * 3.14159265358979323846 * k / n;
        tw[k] = make_float2(static_cast<float>(std::cos(a)), static_cast<float>(-std::sin(a)));
    }
    float2* base = reinterpret_cast<float2*>(data);
    const wstfft::Lines g{nb, bs, nl, ls, es};
    // elements the geometry spans (mode 3 copies them as the global source)
    const size_t extent = static_cast<size_t>(nb - 1) * bs + static_cast<size_t>(nl - 1) * ls +
                          static_cast<size_t>(n - 1) * es + 1;
    bool compiled = false;
    switch (n) {
#define WST_HOST_CASE(NN)                                                                  \
    case NN:                                                                               \
        compiled = true;                                                                   \
        if (mode == 0) {                                                                   \
            if (inverse) wstfft::fft_lines_host<NN, true>(base, g, tw.data(), threads);    \
            else wstfft::fft_lines_host<NN, false>(base, g, tw.data(), threads);           \
        } else if (mode == 4) {                                                            \
            /* F_DR with the fused order-2 rows' split (wstdev::fused_row_n2) */              \
            constexpr int N2O = wstdev::fused_row_n2(NN);                                      \
            if constexpr (N2O > 0) {                                                           \
                using FO = wstfft::LineFFT<NN, true, N2O>;                                     \
                using FF = wstfft::LineFFT<NN, false, N2O>;                                    \
                wstfft::EpiIdentity id4;                                                       \
                for (int u = 0; u < g.nlines() * FO::N2; ++u)                                  \
                    inverse ? FO::stageA_unit(base, g, tw.data(), u) : FF::stageA_unit(base, g, tw.data(), u); \
                for (int u = 0; u < g.nlines() * FO::N1; ++u)                                  \
                    inverse ? FO::stageB_inplace(base, g, u, id4) : FF::stageB_inplace(base, g, u, id4); \
                if (perm)                                                                      \
                    for (int pos = 0; pos < NN; ++pos) perm[pos] = FO::dr_logical(pos);        \
                perm_done = true;                                                              \
            } else {                                                                           \
                return fail(WST_ERR_UNSUPPORTED, "mode 4 needs a fused-row size (48)");        \
            }                                                                                  \
        } else if (mode == 3) {                                                            \
            if (wstfft::LineFFT<NN, false>::N2 == 1)                                       \
                return fail(WST_ERR_UNSUPPORTED, "mode 3 needs a two-stage size");         \
            const std::vector<float2> src(base, base + extent);                            \
            for (size_t i = 0; i < extent; ++i) base[i] = make_float2(NAN, NAN);           \
            if (inverse) wstfft::fft_lines_rd_from_host<NN, true>(base, src.data(), g, tw.data());  \
            else wstfft::fft_lines_rd_from_host<NN, false>(base, src.data(), g, tw.data()); \
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
    if (perm && !perm_done)
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
