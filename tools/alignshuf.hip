// alignshuf.hip — can a byte-misaligned 16-B-per-lane copy (k_encode_flat's
// var windows) stream faster as ALIGNED 16-B loads + the next lane's block
// through a DPP wave shift + a per-lane funnel shift?  Copy of 2 GB at source
// byte offset 5, aligned 16-B stores, tile = TB bytes per workgroup.
//   hipcc --offload-arch=gfx950 -O3 -o tools/alignshuf tools/alignshuf.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 gv4;
typedef __attribute__((address_space(1))) const u32x4 cgv4;

// baseline: one misaligned 16-B load per lane
template <int U>
__global__ __launch_bounds__(256) void k_mis(const unsigned char* __restrict__ src, u32x4* __restrict__ dst,
                                             size_t n16, unsigned off, unsigned tile16) {
    const size_t t0 = (size_t)blockIdx.x * tile16, t1 = min(t0 + tile16, n16);
    for (size_t cb = t0 + threadIdx.x; cb < t1; cb += (size_t)U * 256) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = *(cgv4*)(src + off + 16 * min(cb + (size_t)u * 256, t1 - 1));
#pragma unroll
        for (int u = 0; u < U; u++)
            if (cb + (size_t)u * 256 < t1) *(gv4*)(dst + cb + (size_t)u * 256) = v[u];
    }
}

__device__ __forceinline__ unsigned shl1(unsigned x) {   // lane l <- lane l + 1 (wave_shl:1)
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xF, 0xF, false);
}

// bytes [m, m + 16) of the 32 bytes a | b, per-lane m in 0..15
__device__ __forceinline__ u32x4 funnel(const u32x4& a, const u32x4& b, unsigned m) {
    unsigned d0 = a.x, d1 = a.y, d2 = a.z, d3 = a.w, d4 = b.x, d5 = b.y, d6 = b.z, d7 = b.w;
    if (m & 8) { d0 = d2; d1 = d3; d2 = d4; d3 = d5; d4 = d6; d5 = d7; }   // selects, not branches
    if (m & 4) { d0 = d1; d1 = d2; d2 = d3; d3 = d4; d4 = d5; }
    const unsigned s = m & 3u;
    return u32x4{__builtin_amdgcn_alignbyte(d1, d0, s), __builtin_amdgcn_alignbyte(d2, d1, s),
                 __builtin_amdgcn_alignbyte(d3, d2, s), __builtin_amdgcn_alignbyte(d4, d3, s)};
}

// aligned 16-B loads; the second block from the next lane when it holds
// exactly the next 16 bytes, else (lane 63, a discontinuity) a second load
template <int U, bool UNIF>
__global__ __launch_bounds__(256) void k_shuf(const unsigned char* __restrict__ src, u32x4* __restrict__ dst,
                                              size_t n16, unsigned off, unsigned tile16) {
    const size_t t0 = (size_t)blockIdx.x * tile16, t1 = min(t0 + tile16, n16);
    for (size_t cb = t0 + threadIdx.x; cb < t1; cb += (size_t)U * 256) {
        u32x4 a[U], b[U];
        unsigned m[U];
        bool own[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t w = (size_t)(src + off) + 16 * min(cb + (size_t)u * 256, t1 - 1);
            const size_t al = w & ~(size_t)15;
            m[u] = (unsigned)(w & 15);
            a[u] = *(cgv4*)al;
            const unsigned nlo = shl1((unsigned)al);   // the next lane's block address (low bits)
            own[u] = m[u] && (nlo != (unsigned)al + 16u || (threadIdx.x & 63) == 63);
            if (own[u]) b[u] = *(cgv4*)(al + 16);
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            u32x4 nb = u32x4{shl1(a[u].x), shl1(a[u].y), shl1(a[u].z), shl1(a[u].w)};
            if (own[u]) nb = b[u];
            u32x4 v;
            if (UNIF) {
                // wave-uniform shift (one value's interior): scalar switch
                const unsigned mu = __builtin_amdgcn_readfirstlane(m[u]);
                const unsigned s = mu & 3u;
#define AB(h, l) __builtin_amdgcn_alignbyte(h, l, s)
                const u32x4 x0 = a[u], x1 = nb;
                switch (mu >> 2) {
                    case 0: v = u32x4{AB(x0.y, x0.x), AB(x0.z, x0.y), AB(x0.w, x0.z), AB(x1.x, x0.w)}; break;
                    case 1: v = u32x4{AB(x0.z, x0.y), AB(x0.w, x0.z), AB(x1.x, x0.w), AB(x1.y, x1.x)}; break;
                    case 2: v = u32x4{AB(x0.w, x0.z), AB(x1.x, x0.w), AB(x1.y, x1.x), AB(x1.z, x1.y)}; break;
                    default: v = u32x4{AB(x1.x, x0.w), AB(x1.y, x1.x), AB(x1.z, x1.y), AB(x1.w, x1.z)}; break;
                }
#undef AB
            } else {
                v = funnel(a[u], nb, m[u]);
            }
            if (cb + (size_t)u * 256 < t1) *(gv4*)(dst + cb + (size_t)u * 256) = v;
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
    for (size_t i = 0; i < h.size(); i++) h[i] = (unsigned char)(i * 37 + 11 + (i >> 8));
    hipMemcpy(src, h.data(), h.size(), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, auto kern, unsigned tile16, unsigned off) {
        const unsigned grid = (unsigned)((n16 - 8 + tile16 - 1) / tile16);
        const size_t n = n16 - 8;
        hipMemset(dst, 0, 1 << 20);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, dst, n, off, tile16);
        std::vector<unsigned char> g((1 << 20) - 64);
        hipMemcpy(g.data(), dst, g.size(), hipMemcpyDeviceToHost);
        const bool ok = memcmp(g.data(), h.data() + off, g.size()) == 0;
        for (int w = 0; w < 2; w++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, dst, n, off, tile16);
        hipEventRecord(a);
        const int reps = 10;
        for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, src, dst, n, off, tile16);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        printf("{\"kernel\": \"%s\", \"tile_bytes\": %u, \"off\": %u, \"ok\": %s, \"ms\": %.4f, \"copy_GBs\": %.1f}\n",
               name, 16 * tile16, off, ok ? "true" : "false", ms / reps, 2.0 * 16 * n / (ms / reps * 1e-3) / 1e9);
    };
    for (unsigned tb : {16384u, 126976u}) {
        const unsigned t16 = tb / 16;
        run("aligned_U2", k_mis<2>, t16, 0);
        run("mis_U2", k_mis<2>, t16, 5);
        run("shuf_U2", k_shuf<2, false>, t16, 5);
        run("shuf_unif_U2", k_shuf<2, true>, t16, 5);
        run("shuf_U2_off13", k_shuf<2, false>, t16, 13);
        run("mis_U4", k_mis<4>, t16, 5);
        run("shuf_U4", k_shuf<4, false>, t16, 5);
    }
    return 0;
}
