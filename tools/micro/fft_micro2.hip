// Microbenchmark through the production dispatch templates (dev tool): includes wst_hip.hip.
#include "wst_hip.hip"
#include <cstdio>

namespace {
template <int KIND, int MODE>
__global__ void __launch_bounds__(512) kdisp(const float2* __restrict__ in, float2* __restrict__ out,
                                             const float2* __restrict__ twg, int n, int reps, int ldp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ld = n + ldp;
    float2* A = reinterpret_cast<float2*>(smem);
    float2* tw = A + n * ld;
    for (int i = threadIdx.x; i < n; i += blockDim.x) tw[i] = twg[i];
    const float2* src = in + (size_t)blockIdx.x * n * n;
    for (int o = threadIdx.x; o < n * n; o += blockDim.x) A[(o / n) * ld + o % n] = src[o];
    __syncthreads();
    EpiModulus mod{1.f, 0.f};
    wstfft::EpiIdentity id;
    for (int r = 0; r < reps; ++r) {
        if constexpr (MODE == 0) lds_fft2<3, 3, 136, KIND, true>(A, 1, 0, n, n, ld, tw, tw, mod);
        else lds_fft_lines<3, 136, KIND, true>(A, wstfft::Lines{1, 0, n, ld, 1}, n, tw, id);
    }
    float2* dst = out + (size_t)blockIdx.x * n * n;
    for (int o = threadIdx.x; o < n * n; o += blockDim.x) dst[o] = A[(o / n) * ld + o % n];
    if (mod.sum == -1.f) dst[0].x = 0.f;
}

template <int KIND, int MODE>
void go(const char* name, int n, int ldp, float2* din, float2* dout, float2* dtw) {
    auto k = kdisp<KIND, MODE>;
    const size_t lds = (size_t)n * (n + ldp) * 8 + n * 8;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipLaunchKernelGGL(k, dim3(2048), dim3(512), lds, 0, din, dout, dtw, n, 8, ldp);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(2048), dim3(512), lds, 0, din, dout, dtw, n, 8, ldp);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-26s n=%d ld=%d: %.3f ms/launch\n", name, n, n + ldp, ms / 5);
}
}  // namespace

int main() {
    const size_t sz = (size_t)2048 * 96 * 96;
    float2 *din, *dout, *dtw;
    (void)hipMalloc(&din, sz * 8); (void)hipMalloc(&dout, sz * 8); (void)hipMalloc(&dtw, 4096 * 8);
    (void)hipMemset(din, 0, sz * 8);
    std::vector<float2> tw(96);
    for (int k = 0; k < 96; ++k) tw[k] = make_float2(cos(2 * M_PI * k / 96), -sin(2 * M_PI * k / 96));
    (void)hipMemcpy(dtw, tw.data(), 96 * 8, hipMemcpyHostToDevice);
    go<kDR, 0>("disp fft2 DR inv+mod", 96, 1, din, dout, dtw);
    go<kRD, 0>("disp fft2 RD inv+mod", 96, 1, din, dout, dtw);
    go<kDR, 1>("disp rows DR inv", 96, 1, din, dout, dtw);
    go<kRD, 1>("disp rows RD inv", 96, 1, din, dout, dtw);
    go<kNat, 1>("disp rows NAT inv", 96, 1, din, dout, dtw);
    (void)hipDeviceSynchronize();
    return 0;
}
