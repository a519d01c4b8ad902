// unaligned.hip — do byte-misaligned 16-B global loads stream at full rate?
// copy N bytes src+off -> dst (16-B aligned dst), one chunk per lane, one
// launch = one pass; off = 0 (aligned) vs 1..15.  Checks the bytes first.
//   hipcc --offload-arch=gfx950 -O3 -o tools/unaligned tools/unaligned.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_copy(const unsigned char* __restrict__ src, u32x4* __restrict__ dst,
                                              size_t n16, unsigned off) {
    const size_t base = (size_t)blockIdx.x * 256 * 4;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t i = base + u * 256 + threadIdx.x;
        if (i < n16) v[u] = *(const u32x4*)(src + off + 16 * i);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t i = base + u * 256 + threadIdx.x;
        if (i < n16) __builtin_nontemporal_store(v[u], dst + i);
    }
}

int main() {
    const size_t N = (size_t)1 << 30, n16 = N / 16;
    unsigned char* src;
    u32x4* dst;
    hipMalloc(&src, N + 64);
    hipMalloc(&dst, N);
    std::vector<unsigned char> h(4096 + 64);
    for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned char)(i * 37 + 11);
    hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice);
    // correctness on the first 4 KB for every offset
    for (unsigned off = 0; off < 16; off++) {
        hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, 0, src, dst, (size_t)256, off);
        std::vector<unsigned char> g(4096);
        hipMemcpy(g.data(), dst, 4096, hipMemcpyDeviceToHost);
        if (memcmp(g.data(), h.data() + off, 4096) != 0) { printf("{\"off\": %u, \"correct\": false}\n", off); return 1; }
    }
    printf("{\"correct\": true}\n");
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const unsigned grid = (unsigned)((n16 + 1023) / 1024);
    for (unsigned off : {0u, 1u, 3u, 4u, 8u, 13u}) {
        for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, src, dst, n16, off);
        hipEventRecord(a);
        const int reps = 10;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, src, dst, n16, off);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("{\"off\": %u, \"ms\": %.4f, \"copy_GBs\": %.1f}\n", off, ms / reps, 2.0 * N / (ms / reps * 1e-3) / 1e9);
    }
    return 0;
}
