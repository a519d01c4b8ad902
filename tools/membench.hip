// membench.hip — streaming ceilings on this MI355X (reference numbers for the
// roofline discussion in DESIGN.md).  hipcc --offload-arch=gfx950 -O3 -o membench membench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void k_copy_nt(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}
__global__ void k_read(const u32x4* __restrict__ a, unsigned* out, size_t n) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        u32x4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void k_write(u32x4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = u32x4{(unsigned)i, 1, 2, 3};
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    f();
    hipDeviceSynchronize();
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e0);
        f();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const size_t bytes = 256ull << 20;
    const size_t n = bytes / 16;
    u32x4 *a, *b;
    unsigned* o;
    hipMalloc(&a, bytes);
    hipMalloc(&b, bytes);
    hipMalloc(&o, 64);
    hipMemset(a, 1, bytes);
    for (int grid : {1024, 2048, 4096, 8192, 16384}) {
        float c = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n); }, 30);
        float cn = timeit([&] { hipLaunchKernelGGL(k_copy_nt, dim3(grid), dim3(256), 0, 0, a, b, n); }, 30);
        float r = timeit([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, o, n); }, 30);
        float w = timeit([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, b, n); }, 30);
        printf("{\"grid\": %d, \"copy_GBs\": %.1f, \"copy_nt_GBs\": %.1f, \"read_GBs\": %.1f, \"write_GBs\": %.1f}\n", grid,
               2 * bytes / c / 1e6, 2 * bytes / cn / 1e6, bytes / r / 1e6, bytes / w / 1e6);
    }
    return 0;
}
