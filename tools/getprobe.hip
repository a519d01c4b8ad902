// getprobe.hip — the ceiling of M GetInt's memory shape with no decoding:
// 1M blobs of 256 B, each lane reads its blob's first 32 B (two 16-B loads,
// one 128-B line) and writes 8 B + 1 B; also 1 and 2 lanes' worth of work
// per thread.  Compare with bench.py --config M --op get kernel_ms.
//   hipcc --offload-arch=gfx950 -O3 -o tools/getprobe tools/getprobe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 cgv4;

template <int PER>
__global__ __launch_bounds__(256) void k_probe(const unsigned char* __restrict__ a, unsigned long long* __restrict__ v,
                                               unsigned char* __restrict__ st, size_t n) {
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const size_t i = ((size_t)blockIdx.x * PER + k) * 256 + threadIdx.x;
        if (i >= n) return;
        const u32x4 w0 = *(cgv4*)(a + 256 * i), w1 = *(cgv4*)(a + 256 * i + 16);
        v[i] = (unsigned long long)w1.z | ((unsigned long long)w1.w << 32) ^ w0.x;
        st[i] = (unsigned char)(w0.y & 1);
    }
}

int main() {
    const size_t n = 1 << 20, S = 3;   // 3 rotated sets: cold as bench.py
    unsigned char* a[S];
    unsigned long long* v;
    unsigned char* st;
    for (size_t s = 0; s < S; s++) {
        hipMalloc(&a[s], n * 256);
        hipMemset(a[s], (int)s + 1, n * 256);
    }
    hipMalloc(&v, n * 8);
    hipMalloc(&st, n);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto kern, int per) {
        const unsigned grid = (unsigned)((n + 256 * per - 1) / (256 * per));
        for (int w = 0; w < 6; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a[w % S], v, st, n);
        hipEventRecord(e0);
        const int reps = 30;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a[r % S], v, st, n);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double gran = (double)n * (128 + 9);
        printf("{\"kernel\": \"%s\", \"ms\": %.5f, \"granular_GBs\": %.1f}\n", name, ms / reps, gran / (ms / reps * 1e-3) / 1e9);
    };
    run("per1", k_probe<1>, 1);
    run("per2", k_probe<2>, 2);
    run("per4", k_probe<4>, 4);
    return 0;
}
