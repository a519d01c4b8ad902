// fetch_calib.hip — what does rocprofv3 FETCH_SIZE count for the decode /
// GetAccess read shapes?  Each case reads a known set of bytes; the host
// prints the exact number of distinct 64-B sectors and 128-B lines touched,
// so FETCH_SIZE (run under `rocprofv3 --pmc FETCH_SIZE`) can be divided by a
// known byte count per access shape (MI355X_MICROARCH.md: calibrate
// non-streaming shapes on a known count before trusting an absolute).
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
//   case 0  streaming: 16 B/lane, consecutive lanes consecutive (the ×2 case)
//   case 1  C5-decode shape: thread i reads [i*970 + (i*37 % 16), +23) as
//           two 16-B loads from the 16-B aligned base below it
//   case 2  M-GetInt shape: thread i reads [i*256, +32) as two 16-B loads
//   case 3  one 16-B load per 4 KiB page at offset 48 (one line each)
//   case 4  C3 tile shape: 16 B/lane LDS-DMA-like streaming of a 21 KB range
//           per 256 threads (same as 0 but per-block ranges) — reads all
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <set>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int CASE>
__global__ __launch_bounds__(256) void k_calib(const uint8_t* __restrict__ src, uint32_t* __restrict__ sink, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint32_t acc = 0;
    if (CASE == 0 || CASE == 4) {
        const u32x4 v = *(const u32x4*)(src + 16 * i);
        acc = v.x ^ v.y ^ v.z ^ v.w;
    } else if (CASE == 1) {
        const size_t a = i * 970 + (i * 37 % 16);
        const size_t b = a & ~(size_t)15;
        const u32x4 v0 = *(const u32x4*)(src + b);
        u32x4 v1 = {0, 0, 0, 0};
        if (a + 23 > b + 16) v1 = *(const u32x4*)(src + b + 16);
        acc = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
    } else if (CASE == 2) {
        const u32x4 v0 = *(const u32x4*)(src + i * 256);
        const u32x4 v1 = *(const u32x4*)(src + i * 256 + 16);
        acc = v0.x ^ v0.y ^ v0.z ^ v0.w ^ v1.x ^ v1.y ^ v1.z ^ v1.w;
    } else if (CASE == 3) {
        const u32x4 v = *(const u32x4*)(src + i * 4096 + 48);
        acc = v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;   // never true for the fill below; keeps the loads
}

static void count(const char* name, size_t n, size_t (*lo)(size_t), size_t (*hi)(size_t), float ms) {
    uint64_t s64 = 0, l128 = 0, last64 = ~0ull, last128 = ~0ull, bytes = 0;
    for (size_t i = 0; i < n; i++) {
        const size_t a = lo(i), b = hi(i);
        bytes += b - a;
        for (size_t x = a / 64; x <= (b - 1) / 64; x++) if (x != last64) { s64++; last64 = x; }
        for (size_t x = a / 128; x <= (b - 1) / 128; x++) if (x != last128) { l128++; last128 = x; }
    }
    printf("{\"case\": \"%s\", \"threads\": %zu, \"bytes_loaded\": %llu, \"sectors64\": %llu, \"lines128\": %llu, "
           "\"bytes64\": %llu, \"bytes128\": %llu, \"ms\": %.4f, \"GBs_lines128\": %.1f}\n",
           name, n, (unsigned long long)bytes, (unsigned long long)s64, (unsigned long long)l128,
           (unsigned long long)(s64 * 64), (unsigned long long)(l128 * 128), ms,
           l128 * 128.0 / (ms * 1e-3) / 1e9);
}

template <int CASE>
static float run(const uint8_t* src, uint32_t* sink, size_t n) {
    const unsigned grid = (unsigned)((n + 255) / 256);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL(k_calib<CASE>, dim3(grid), dim3(256), 0, 0, src, sink, n);
    hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_calib<CASE>, dim3(grid), dim3(256), 0, 0, src, sink, n);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main() {
    const size_t N = (size_t)8 << 30;
    uint8_t* src;
    uint32_t* sink;
    if (hipMalloc(&src, N + 4096) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(src, 0x5A, N + 4096);
    hipDeviceSynchronize();
    const size_t n0 = N / 16 / 4, n1 = (N - 64) / 970, n2 = N / 256, n3 = N / 4096;
    float ms;
    ms = run<0>(src, sink, n0);
    count("stream16", n0, [](size_t i) { return 16 * i; }, [](size_t i) { return 16 * i + 16; }, ms);
    ms = run<1>(src, sink, n1);
    count("c5_decode_23B", n1, [](size_t i) { return (i * 970 + (i * 37 % 16)) & ~(size_t)15; },
          [](size_t i) { const size_t a = i * 970 + (i * 37 % 16), b = a & ~(size_t)15; return a + 23 > b + 16 ? b + 32 : b + 16; }, ms);
    ms = run<2>(src, sink, n2);
    count("m_get_32B", n2, [](size_t i) { return 256 * i; }, [](size_t i) { return 256 * i + 32; }, ms);
    ms = run<3>(src, sink, n3);
    count("page_16B", n3, [](size_t i) { return 4096 * i + 48; }, [](size_t i) { return 4096 * i + 64; }, ms);
    return 0;
}
