// lds_unaligned.hip — are byte-misaligned ds_read/ds_write (b32/b64) exact on
// gfx950 (SH_MEM_CONFIG unaligned mode), and what do they cost?
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lu tools/lds_unaligned.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void k_check(unsigned char* out) {
    __shared__ __attribute__((aligned(16))) unsigned char s[1024];
    const int t = threadIdx.x;
    for (int i = t; i < 1024; i += blockDim.x) s[i] = 0xEE;
    __syncthreads();
    if (t == 0) {
        *(unsigned int*)(s + 1) = 0x44332211u;                 // ds_write_b32 at +1
        *(unsigned long long*)(s + 13) = 0x8877665544332211ull; // ds_write_b64 at +13
        *(unsigned int*)(s + 30) = 0xDDCCBBAAu;                // at +30 (dword-straddling)
    }
    __syncthreads();
    if (t == 0) {
        const unsigned int a = *(const unsigned int*)(s + 3);       // read b32 at +3
        const unsigned long long b = *(const unsigned long long*)(s + 14);
        *(unsigned int*)(out + 64) = a;
        *(unsigned long long*)(out + 72) = b;
    }
    __syncthreads();
    for (int i = t; i < 64; i += blockDim.x) out[i] = s[i];
}

// throughput: every lane writes 4 B at lane*5 + off and reads it back
template <int OFF>
__global__ __launch_bounds__(256) void k_rate(unsigned* out, int iters) {
    __shared__ __attribute__((aligned(16))) unsigned char s[8192];
    const int t = threadIdx.x;
    unsigned acc = t;
    for (int i = 0; i < iters; i++) {
        unsigned a = (unsigned)(t * 8 + OFF + (i & 7) * 2048) & 8191u & ~7u;
        a += OFF;
        *(unsigned int*)(s + a) = acc;
        acc += *(const unsigned int*)(s + ((a + 2048) & 8191u));
    }
    out[blockIdx.x * 256 + t] = acc;
}

int main() {
    unsigned char* d;
    hipMalloc(&d, 128);
    hipMemset(d, 0, 128);
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, d);
    unsigned char h[128];
    hipMemcpy(h, d, 128, hipMemcpyDeviceToHost);
    unsigned char e[64];
    memset(e, 0xEE, 64);
    const unsigned int w1 = 0x44332211u; memcpy(e + 1, &w1, 4);
    const unsigned long long w2 = 0x8877665544332211ull; memcpy(e + 13, &w2, 8);
    const unsigned int w3 = 0xDDCCBBAAu; memcpy(e + 30, &w3, 4);
    unsigned int ra, rb0; unsigned long long rb;
    memcpy(&ra, e + 3, 4); memcpy(&rb, e + 14, 8);
    unsigned int ga; unsigned long long gb;
    memcpy(&ga, h + 64, 4); memcpy(&gb, h + 72, 8);
    (void)rb0;
    printf("{\"writes_exact\": %s, \"read_b32\": %s, \"read_b64\": %s}\n", memcmp(h, e, 64) ? "false" : "true",
           ga == ra ? "true" : "false", gb == rb ? "true" : "false");
    unsigned* o;
    hipMalloc(&o, 4096 * 256 * 4);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int off : {0, 1, 2}) {
        auto run = [&]() {
            if (off == 0) hipLaunchKernelGGL(k_rate<0>, dim3(4096), dim3(256), 0, 0, o, 256);
            else if (off == 1) hipLaunchKernelGGL(k_rate<1>, dim3(4096), dim3(256), 0, 0, o, 256);
            else hipLaunchKernelGGL(k_rate<2>, dim3(4096), dim3(256), 0, 0, o, 256);
        };
        run();
        hipEventRecord(a);
        for (int r = 0; r < 5; r++) run();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("{\"off\": %d, \"ms\": %.4f}\n", off, ms / 5);
    }
    return 0;
}
