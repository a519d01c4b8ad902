// looppipe.hip — does a tile's chunk LOOP (many steps per workgroup, as
// k_encode_tiles' chunk pass over a 124 KB C5 tile) lose to one-step
// workgroups, and does issuing step k+1's loads before step k's stores (so a
// load never waits on the VM counter behind older stores) win it back?
// Byte-misaligned 16-B loads, aligned 16-B stores, tile = TB bytes per WG.
//   hipcc --offload-arch=gfx950 -O3 -o tools/looppipe tools/looppipe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gv4;
typedef __attribute__((address_space(1))) const u32x4 cgv4;

// A: per step, U loads then U stores
template <int U>
__global__ __launch_bounds__(256) void k_loop(const unsigned char* __restrict__ src, u32x4* __restrict__ dst,
                                              size_t n16, unsigned off, unsigned tile16) {
    const size_t t0 = (size_t)blockIdx.x * tile16, t1 = min(t0 + tile16, n16);
    for (size_t cb = t0 + threadIdx.x; cb < t1; cb += (size_t)U * 256) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = min(cb + (size_t)u * 256, t1 - 1);
            v[u] = *(cgv4*)(src + off + 16 * i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = cb + (size_t)u * 256;
            if (i < t1) *(gv4*)(dst + i) = v[u];
        }
    }
}

// B: software-pipelined: step k+1's loads issue before step k's stores
template <int U>
__global__ __launch_bounds__(256) void k_pipe(const unsigned char* __restrict__ src, u32x4* __restrict__ dst,
                                              size_t n16, unsigned off, unsigned tile16) {
    const size_t t0 = (size_t)blockIdx.x * tile16, t1 = min(t0 + tile16, n16);
    size_t cb = t0 + threadIdx.x;
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = min(cb + (size_t)u * 256, t1 - 1);   // clamped: no branch around the load
        a[u] = *(cgv4*)(src + off + 16 * i);
    }
    for (; cb < t1; cb += (size_t)U * 256) {
        const size_t nb = cb + (size_t)U * 256;
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = min(nb + (size_t)u * 256, t1 - 1);
            b[u] = *(cgv4*)(src + off + 16 * i);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = cb + (size_t)u * 256;
            if (i < t1) *(gv4*)(dst + i) = a[u];
        }
#pragma unroll
        for (int u = 0; u < U; u++) a[u] = b[u];
    }
}


// C: C5-shaped: the output alternates pieces of PL bytes taken from two source
// regions (str / bytes columns), so a wave's 64 chunks read two streams; a
// prologue of PRO (0/1) does one 2-KB LDS-DMA-free staging load + barrier per tile
template <int U, int PRO>
__global__ __launch_bounds__(256) void k_two(const unsigned char* __restrict__ s0, const unsigned char* __restrict__ s1,
                                             u32x4* __restrict__ dst, size_t n16, unsigned PL, unsigned tile16) {
    __shared__ unsigned pro[512];
    const size_t t0 = (size_t)blockIdx.x * tile16, t1 = min(t0 + tile16, n16);
    if (PRO) {
        pro[threadIdx.x] = ((const unsigned*)s0)[t0 / 4 + threadIdx.x];
        pro[threadIdx.x + 256] = ((const unsigned*)s1)[t0 / 4 + threadIdx.x];
        __syncthreads();
    }
    for (size_t cb = t0 + threadIdx.x; cb < t1; cb += (size_t)U * 256) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = min(cb + (size_t)u * 256, t1 - 1), B = 16 * i;
            const size_t piece = B / PL, k = B % PL;     // piece p: region p & 1, its (p >> 1)-th piece
            const unsigned char* s = (piece & 1) ? s1 : s0;
            v[u] = *(cgv4*)(s + (piece >> 1) * PL + k + 3);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = cb + (size_t)u * 256;
            if (i < t1) *(gv4*)(dst + i) = PRO ? v[u] ^ pro[threadIdx.x & 511] : v[u];
        }
    }
}

int main() {
    const size_t N = (size_t)2 << 30, n16 = N / 16;
    unsigned char* src;
    u32x4* dst;
    hipMalloc(&src, N + 64);
    hipMalloc(&dst, N);
    std::vector<unsigned char> h(1 << 20);
    for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned char)(i * 37 + 11);
    hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, auto kern, unsigned tile16) {
        const unsigned grid = (unsigned)((n16 + tile16 - 1) / tile16);
        // correctness on the first 1 MB
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, dst, n16, 5u, tile16);
        std::vector<unsigned char> g((1 << 20) - 64);
        hipMemcpy(g.data(), dst, g.size(), hipMemcpyDeviceToHost);
        const bool ok = memcmp(g.data(), h.data() + 5, g.size()) == 0;
        for (int w = 0; w < 2; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, dst, n16, 5u, tile16);
        hipEventRecord(a);
        const int reps = 10;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, dst, n16, 5u, tile16);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("{\"kernel\": \"%s\", \"tile_bytes\": %u, \"ok\": %s, \"ms\": %.4f, \"copy_GBs\": %.1f}\n", name,
               16 * tile16, ok ? "true" : "false", ms / reps, 2.0 * N / (ms / reps * 1e-3) / 1e9);
    };
    {
        const unsigned PL = 480, t16 = 126976 / 16;
        auto run2 = [&](const char* name, auto kern) {
            const unsigned grid = (unsigned)((n16 + t16 - 1) / t16);
            const unsigned char* s1 = src + N / 2 + 4096;
            for (int w = 0; w < 2; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, s1, dst, n16 / 2 - 4096, PL, t16);
            hipEventRecord(a);
            const int reps = 10;
            for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, s1, dst, n16 / 2 - 4096, PL, t16);
            hipEventRecord(b);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            const double bytes = 2.0 * 16.0 * (double)(n16 / 2 - 4096);
            printf("{\"kernel\": \"%s\", \"tile_bytes\": 126976, \"ms\": %.4f, \"copy_GBs\": %.1f}\n", name, ms / reps,
                   bytes / (ms / reps * 1e-3) / 1e9);
        };
        run2("two_U4", k_two<4, 0>);
        run2("two_U4_pro", k_two<4, 1>);
        run2("two_U2_pro", k_two<2, 1>);
    }
    for (unsigned tb : {16384u, 126976u}) {
        const unsigned t16 = tb / 16;
        run("loop_U2", k_loop<2>, t16);
        run("loop_U4", k_loop<4>, t16);
        run("loop_U8", k_loop<8>, t16);
        run("pipe_U2", k_pipe<2>, t16);
        run("pipe_U4", k_pipe<4>, t16);
    }
    return 0;
}
