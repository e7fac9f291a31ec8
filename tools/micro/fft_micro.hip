// Standalone microbenchmark of the LDS FFT variants (dev tool): one 2-D transform of a
// (rows x rows, stride LD) complex array per workgroup, many workgroups, timed with events.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I<csrc> fft_micro.hip -o fft_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "fft_lds.h"

struct EpiMod {
    float sum = 0.f;
    __device__ float2 operator()(float2 z) {
        const float m = sqrtf(fmaf(z.x, z.x, z.y * z.y));
        sum += m;
        return make_float2(m, 0.f);
    }
};

template <int N, int KIND, bool INV, bool MOD, int LDP, int OFFKB = 0, int TWKB = -1>
__global__ void __launch_bounds__(1024) kfft(const float2* __restrict__ in, float2* __restrict__ out,
                                            const float2* __restrict__ twg, int reps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int LD = N + LDP;
    float2* A = reinterpret_cast<float2*>(smem + OFFKB * 1024);
    float2* tw = (TWKB < 0) ? A + N * LD : reinterpret_cast<float2*>(smem + TWKB * 1024);
    for (int i = threadIdx.x; i < N; i += blockDim.x) tw[i] = twg[i];
    const float2* src = in + (size_t)blockIdx.x * N * N;
    for (int o = threadIdx.x; o < N * N; o += blockDim.x) A[(o / N) * LD + o % N] = src[o];
    __syncthreads();
    wstfft::EpiIdentity id;
    EpiMod em;
    for (int r = 0; r < reps; ++r) {
        const wstfft::Lines rows{1, 0, N, LD, 1}, cols{1, 0, N, 1, LD};
        if constexpr (KIND == 1) {
            wstfft::fft_lines_dr<N, INV>(A, rows, tw, id);
            if constexpr (MOD) wstfft::fft_lines_dr<N, INV>(A, cols, tw, em);
            else wstfft::fft_lines_dr<N, INV>(A, cols, tw, id);
        } else if constexpr (KIND == 2) {
            wstfft::fft_lines_rd<N, INV>(A, rows, tw, id);
            wstfft::fft_lines_rd<N, INV>(A, cols, tw, id);
        } else {
            wstfft::fft_lines<N, INV>(A, rows, tw, id);
            wstfft::fft_lines<N, INV>(A, cols, tw, id);
        }
    }
    float2* dst = out + (size_t)blockIdx.x * N * N;
    for (int o = threadIdx.x; o < N * N; o += blockDim.x) dst[o] = A[(o / N) * LD + o % N];
    if (em.sum == -1.f) dst[0].x = 0.f;
}

template <int N, int KIND, bool INV, bool MOD, int LDP, int OFFKB = 0, int TWKB = -1>
void run(const char* name, int nblk, int threads, int reps, float2* din, float2* dout, float2* dtw) {
    auto k = kfft<N, KIND, INV, MOD, LDP, OFFKB, TWKB>;
    size_t lds = (size_t)OFFKB * 1024 + (size_t)N * (N + LDP) * 8 + N * 8;
    if (TWKB >= 0 && (size_t)TWKB * 1024 + N * 8 > lds) lds = (size_t)TWKB * 1024 + N * 8;
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k, dim3(nblk), dim3(threads), lds, 0, din, dout, dtw, reps);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(nblk), dim3(threads), lds, 0, din, dout, dtw, reps);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double per = ms / 5 / (double)nblk / reps * 1e3;   // us per transform per WG-slot
    printf("%-28s N=%d LD=%d thr=%d: %.3f ms/launch, %.3f us per 2-D transform x WG\n", name, N, N + LDP, threads, ms / 5, per * 256);
}

int main(int argc, char** argv) {
    const int nblk = 2048, reps = 8;
    const int maxn = 128;
    std::vector<float2> h((size_t)nblk * maxn * maxn), tw(maxn);
    for (auto& v : h) v = make_float2(rand() / (float)RAND_MAX, rand() / (float)RAND_MAX);
    float2 *din, *dout, *dtw;
    hipMalloc(&din, h.size() * 8); hipMalloc(&dout, h.size() * 8); hipMalloc(&dtw, 4096 * 8);
    hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    auto settw = [&](int n) {
        for (int k = 0; k < n; ++k) tw[k] = make_float2(cos(2 * M_PI * k / n), -sin(2 * M_PI * k / n));
        hipMemcpy(dtw, tw.data(), n * 8, hipMemcpyHostToDevice);
    };
    settw(96);
    run<96, 1, true, true, 1>("DR+mod 512thr 2WG/CU", nblk, 512, reps, din, dout, dtw);
    run<96, 1, true, true, 1, 80>("DR+mod 512thr 1WG/CU", nblk, 512, reps, din, dout, dtw);
    run<96, 1, true, true, 1, 80>("DR+mod 1024thr 1WG/CU", nblk, 1024, reps, din, dout, dtw);
    run<96, 1, true, true, 1>("DR+mod 1024thr 2WG/CU", nblk, 1024, reps, din, dout, dtw);
    run<96, 1, true, true, 1>("DR+mod 256thr 2WG/CU", nblk, 256, reps, din, dout, dtw);
    settw(48);
    run<48, 1, true, true, 1>("48 DR+mod 256thr ~8WG/CU", nblk, 256, reps, din, dout, dtw);
    run<48, 1, true, true, 1, 130>("48 DR+mod 1024thr 1WG/CU", nblk, 1024, reps, din, dout, dtw);
    run<48, 1, true, true, 1, 60>("48 DR+mod 512thr 2WG/CU", nblk, 512, reps, din, dout, dtw);
    hipDeviceSynchronize();
    return 0;
}
