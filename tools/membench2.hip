// membench2.hip — streaming ceilings in the shape of metric M (read 238 MiB,
// write 256 MiB per launch), timed two ways: each launch bracketed alone
// (sync between) and back to back (events only, the bench.py regime, where
// the previous launch's dirty lines are written back during the next).
// Store/load cache policies compared: plain, nt, sc1, sc0 sc1, sc0 sc1 nt.
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench2 tools/membench2.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <numeric>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g4;

template <int SP>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
    g4* gp = (g4*)p;
    if constexpr (SP == 0) *gp = v;
    else if constexpr (SP == 1) __builtin_nontemporal_store(v, gp);
    else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(gp), "v"(v) : "memory");
    else if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(gp), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(gp), "v"(v) : "memory");
}
template <int LP>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
    const g4* gp = (const g4*)p;
    if constexpr (LP == 0) return *gp;
    else return __builtin_nontemporal_load(gp);
}

// tile-per-block copy: block b reads tile b of `in` (tin bytes) and writes
// tile b of `out` (tout bytes): the encode kernel's traffic shape.
template <int LP, int SP>
__global__ __launch_bounds__(256) void k_tile(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t tin16,
                                              size_t tout16, size_t ntiles) {
    const size_t b = blockIdx.x;
    const u32x4* src = in + b * tin16;
    u32x4* dst = out + b * tout16;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t k = u * 256 + threadIdx.x;
        v[u] = k < tin16 ? ld16<LP>(src + k) : u32x4{0, 0, 0, 0};
    }
    unsigned x = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t k = u * 256 + threadIdx.x;
        if (k < tout16) st16<SP>(dst + k, u32x4{x, (unsigned)k, v[u].z, v[u].w});
    }
}

__global__ __launch_bounds__(256) void k_tilep(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t tin16,
                                               size_t tout16, size_t ntiles) {
    for (size_t b = blockIdx.x; b < ntiles; b += gridDim.x) {
        const u32x4* src = in + b * tin16;
        u32x4* dst = out + b * tout16;
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const size_t k = u * 256 + threadIdx.x;
            v[u] = k < tin16 ? ld16<0>(src + k) : u32x4{0, 0, 0, 0};
        }
        unsigned x = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const size_t k = u * 256 + threadIdx.x;
            if (k < tout16) st16<1>(dst + k, u32x4{x, (unsigned)k, v[u].z, v[u].w});
        }
    }
}

// same traffic, stores as dwords: wave instruction = 256 contiguous bytes
// (the k_encode_fixed_dw store pattern); LDS round trip + barrier in between
template <bool NT, bool VIA_LDS>
__global__ __launch_bounds__(256) void k_tile_dw(const u32x4* __restrict__ in, unsigned* __restrict__ out, size_t tin16,
                                                 size_t tout16) {
    __shared__ u32x4 sh[1024];
    const size_t b = blockIdx.x;
    const u32x4* src = in + b * tin16;
    unsigned* dst = out + b * tout16 * 4;
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t k = u * 256 + threadIdx.x;
        v[u] = k < tin16 ? ld16<0>(src + k) : u32x4{0, 0, 0, 0};
    }
    if (VIA_LDS) {
#pragma unroll
        for (int u = 0; u < 4; u++) sh[u * 256 + threadIdx.x] = v[u];
        __syncthreads();
        const unsigned* s32 = (const unsigned*)sh;
        for (int u = 0; u < 16; u++) {
            const unsigned k = u * 256 + threadIdx.x;
            unsigned x = s32[k] ^ s32[(k + 5) & 4095];
            if (NT) __builtin_nontemporal_store(x, dst + k);
            else dst[k] = x;
        }
    } else {
        for (int u = 0; u < 16; u++) {
            const unsigned k = u * 256 + threadIdx.x;
            unsigned x = v[u & 3].x ^ k;
            if (NT) __builtin_nontemporal_store(x, dst + k);
            else dst[k] = x;
        }
    }
}

// metric-M input shape: 8 SoA columns (widths 2,4,8,8,1,96,64,55); tile t
// reads rows [64t, 64t+64) of every column as 16-B chunks (952 chunks) and
// writes 16 KiB: the encode kernel's exact HBM traffic without its compute.
// PERSIST: grid-stride over tiles (the persistent kernels' order).
__constant__ unsigned c_w[8] = {2, 4, 8, 8, 1, 96, 64, 55};
template <bool PERSIST>
__global__ __launch_bounds__(256) void k_cols(const unsigned char* __restrict__ in, u32x4* __restrict__ out,
                                              size_t ntiles, size_t nrows) {
    for (size_t t = blockIdx.x; t < ntiles; t += PERSIST ? gridDim.x : ntiles) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            unsigned k = u * 256 + threadIdx.x, cb = 0;
            size_t colbase = 0;
            unsigned w = 0, cbk = 0;
            size_t base = 0;
            for (int g = 0; g < 8; g++) {
                unsigned nch = 64 * c_w[g] / 16;
                if (k >= cb) { w = c_w[g]; cbk = cb; base = colbase; }
                cb += nch;
                colbase += nrows * c_w[g];
            }
            v[u] = k < 952 ? *(const u32x4*)(in + base + t * 64 * w + (k - cbk) * 16) : u32x4{0, 0, 0, 0};
        }
        unsigned x = v[0].x ^ v[1].y ^ v[2].z ^ v[3].w;
        u32x4* dst = out + t * 1024;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned k = u * 256 + threadIdx.x;
            __builtin_nontemporal_store(u32x4{x, k, v[u].z, v[u].w}, (g4*)(dst + k));
        }
    }
}

template <int SP>
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ out, size_t tout16) {
    u32x4* dst = out + blockIdx.x * tout16;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t k = u * 256 + threadIdx.x;
        if (k < tout16) st16<SP>(dst + k, u32x4{(unsigned)k, 1, 2, 3});
    }
}

template <int LP>
__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ in, size_t tin16, unsigned* o) {
    const u32x4* src = in + blockIdx.x * tin16;
    unsigned acc = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const size_t k = u * 256 + threadIdx.x;
        if (k < tin16) {
            u32x4 v = ld16<LP>(src + k);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    }
    if (acc == 0x12345678u) o[0] = acc;
}

struct Res { float alone_med, b2b_mean, b2b_med; };

template <typename F>
Res timeit(F f, int reps) {
    hipEvent_t e[2 * 64];
    for (auto& x : e) hipEventCreate(&x);
    std::vector<float> a, b;
    f();
    hipDeviceSynchronize();
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e[0]);
        f();
        hipEventRecord(e[1]);
        hipEventSynchronize(e[1]);
        float ms;
        hipEventElapsedTime(&ms, e[0], e[1]);
        a.push_back(ms);
    }
    for (int r = 0; r < reps; r++) {
        hipEventRecord(e[2 * r]);
        f();
        hipEventRecord(e[2 * r + 1]);
    }
    hipDeviceSynchronize();
    for (int r = 0; r < reps; r++) {
        float ms;
        hipEventElapsedTime(&ms, e[2 * r], e[2 * r + 1]);
        b.push_back(ms);
    }
    for (auto& x : e) hipEventDestroy(x);
    std::sort(a.begin(), a.end());
    float mean = std::accumulate(b.begin(), b.end(), 0.f) / b.size();
    std::sort(b.begin(), b.end());
    return {a[a.size() / 2], mean, b[b.size() / 2]};
}

static void report(const char* name, double bytes, Res r) {
    printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"alone_med_us\": %.2f, \"b2b_mean_us\": %.2f, \"b2b_med_us\": %.2f, "
           "\"alone_GBs\": %.1f, \"b2b_GBs\": %.1f}\n",
           name, bytes, r.alone_med * 1e3, r.b2b_mean * 1e3, r.b2b_med * 1e3, bytes / r.alone_med / 1e6,
           bytes / r.b2b_mean / 1e6);
    fflush(stdout);
}

int main() {
    const size_t ntiles = 16384;                 // M: 64 blobs per tile
    const size_t tin = 64 * 238, tout = 64 * 256;  // bytes per tile
    const size_t tin16 = (tin + 15) / 16, tout16 = tout / 16;
    u32x4 *a, *b;
    unsigned* o;
    hipMalloc(&a, ntiles * tin16 * 16);
    hipMalloc(&b, ntiles * tout16 * 16);
    hipMalloc(&o, 64);
    hipMemset(a, 1, ntiles * tin16 * 16);
    hipMemset(b, 0, ntiles * tout16 * 16);
    const double cb = (double)ntiles * (tin + tout);
    const int R = 40;
#define RUN(LP, SP, nm) \
    report(nm, cb, timeit([&] { hipLaunchKernelGGL((k_tile<LP, SP>), dim3(ntiles), dim3(256), 0, 0, a, b, tin16, tout16, ntiles); }, R))
    RUN(0, 0, "copy ld plain st plain");
    RUN(0, 1, "copy ld plain st nt");
    RUN(0, 2, "copy ld plain st sc1");
    RUN(0, 3, "copy ld plain st sc0sc1");
    RUN(0, 4, "copy ld plain st sc0sc1nt");
    RUN(1, 0, "copy ld nt st plain");
    RUN(1, 1, "copy ld nt st nt");
    RUN(1, 3, "copy ld nt st sc0sc1");
    report("copy dword st nt", cb, timeit([&] { hipLaunchKernelGGL((k_tile_dw<true, false>), dim3(ntiles), dim3(256), 0, 0, a, (unsigned*)b, tin16, tout16); }, R));
    report("copy dword st plain", cb, timeit([&] { hipLaunchKernelGGL((k_tile_dw<false, false>), dim3(ntiles), dim3(256), 0, 0, a, (unsigned*)b, tin16, tout16); }, R));
    report("copy lds dword st nt", cb, timeit([&] { hipLaunchKernelGGL((k_tile_dw<true, true>), dim3(ntiles), dim3(256), 0, 0, a, (unsigned*)b, tin16, tout16); }, R));
    report("cols 8 streams, tile per WG", cb, timeit([&] { hipLaunchKernelGGL((k_cols<false>), dim3(ntiles), dim3(256), 0, 0, (const unsigned char*)a, b, ntiles, ntiles * 64); }, R));
    for (int g : {1024, 1280, 1536, 2048})
        report(g == 1024 ? "cols persistent 1024" : g == 1280 ? "cols persistent 1280" : g == 1536 ? "cols persistent 1536" : "cols persistent 2048", cb,
               timeit([&] { hipLaunchKernelGGL((k_cols<true>), dim3(g), dim3(256), 0, 0, (const unsigned char*)a, b, ntiles, ntiles * 64); }, R));
    report("copy contiguous persistent 1280", cb, timeit([&] { hipLaunchKernelGGL((k_tilep), dim3(1280), dim3(256), 0, 0, a, b, tin16, tout16, ntiles); }, R));
#define RW(SP, nm) \
    report(nm, (double)ntiles * tout, timeit([&] { hipLaunchKernelGGL((k_write<SP>), dim3(ntiles), dim3(256), 0, 0, b, tout16); }, R))
    RW(0, "write plain");
    RW(1, "write nt");
    RW(3, "write sc0sc1");
    report("read plain", (double)ntiles * tin,
           timeit([&] { hipLaunchKernelGGL((k_read<0>), dim3(ntiles), dim3(256), 0, 0, a, tin16, o); }, R));
    report("read nt", (double)ntiles * tin,
           timeit([&] { hipLaunchKernelGGL((k_read<1>), dim3(ntiles), dim3(256), 0, 0, a, tin16, o); }, R));
    return 0;
}
