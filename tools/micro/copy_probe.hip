// Copy-kernel variants for the HBM probe (dev tool): GB/s (read + written bytes) per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_gs(const v4f* __restrict__ s, v4f* __restrict__ d, long long n) {
    const long long stride = (long long)gridDim.x * blockDim.x;
    long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        v4f t[U];
#pragma unroll
        for (int k = 0; k < U; ++k) t[k] = NT ? __builtin_nontemporal_load(s + i + k * stride) : s[i + k * stride];
#pragma unroll
        for (int k = 0; k < U; ++k) { if (NT) __builtin_nontemporal_store(t[k], d + i + k * stride); else d[i + k * stride] = t[k]; }
    }
    for (; i < n; i += stride) d[i] = s[i];
}
// block-contiguous tiles: block b copies [b*T, (b+1)*T) in U-deep rounds of 256 lanes
template <int U, bool NT>
__global__ void __launch_bounds__(256) k_tile(const v4f* __restrict__ s, v4f* __restrict__ d, long long n, long long per) {
    const long long b0 = blockIdx.x * per, e = b0 + per < n ? b0 + per : n;
    for (long long i = b0 + threadIdx.x; i < e; i += U * 256) {
        v4f t[U];
#pragma unroll
        for (int k = 0; k < U; ++k) { long long j = i + k * 256; if (j < e) t[k] = NT ? __builtin_nontemporal_load(s + j) : s[j]; }
#pragma unroll
        for (int k = 0; k < U; ++k) { long long j = i + k * 256; if (j < e) { if (NT) __builtin_nontemporal_store(t[k], d + j); else d[j] = t[k]; } }
    }
}
int main() {
    const size_t bytes = size_t(1) << 31; const long long n = bytes / 16;
    v4f *s, *d; hipMalloc(&s, bytes); hipMalloc(&d, bytes); hipMemset(s, 0, bytes); hipMemset(d, 0, bytes);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto run = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; ++w) launch();
        hipEventRecord(e0); for (int r = 0; r < 10; ++r) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        printf("%-28s %7.0f GB/s\n", name, 2.0 * bytes * 10 / (ms * 1e-3) / 1e9);
    };
    for (int g : {32768, 65536, 131072, 262144}) {
        char nm[64]; long long per = (n + g - 1) / g;
        snprintf(nm, 64, "tile U4 nt grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_tile<4, true>), dim3(g), dim3(256), 0, 0, s, d, n, per); });
        snprintf(nm, 64, "tile U4 plain grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_tile<4, false>), dim3(g), dim3(256), 0, 0, s, d, n, per); });
        snprintf(nm, 64, "tile U8 plain grid %d", g); run(nm, [&] { hipLaunchKernelGGL((k_tile<8, false>), dim3(g), dim3(256), 0, 0, s, d, n, per); });
    }
    hipMemcpy(d, s, bytes, hipMemcpyDeviceToDevice);
    run("hipMemcpy D2D", [&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); });
    return 0;
}
