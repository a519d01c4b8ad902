// kernels.hip — CDNA4 (gfx950) kernels for bulk PackOS encode/decode and the
// C ABI entry points that launch them (include/packos.h).
//
// Hot path (BASELINE.json north_star): encode of millions of same-schema blobs.
//   k_encode_fixed  fixed-size schemas: a workgroup stages a tile of T blobs'
//                   input columns in LDS with 16-B coalesced loads, then every
//                   lane assembles whole 16-B output chunks (constant header /
//                   key bytes + funnel-shifted column bytes) and stores them
//                   with global_store_dwordx4.  Pure byte/integer work, HBM
//                   bound; no MFMA.
//   k_sizes_affine  var-size schemas with data-independent presence: the
//                   scan telescopes, out_offsets[i] = i*C + sum_v(off_v[i] -
//                   off_v[0]) — a pure map (encode_var.inc)
//   k_stream_sizes  other var-size schemas: blob sizes + decoupled look-back
//                   scan -> out_offsets (encode_var.inc)
//   k_encode_tiles  var-size schemas: one LDS-DMA load round, a compact LDS
//                   frame image of every non-hole byte, then 16-B aligned
//                   output chunks merging image bytes and HBM-resident long
//                   values (encode_var.inc)
//   k_encode_var    generic per-blob kernel (schemas past the tile plan's
//                   tables): one wavefront per blob; item sizes -> wavefront
//                   prefix scan -> header words -> payload staged in an LDS
//                   slot -> aligned 16-B stores
//   k_decode_win    schema.DecodeBuffer semantics (SeqGetAccess + precheck),
//                   one thread per blob, exact error/panic reporting
//   k_get_field     GetAccess random-field gather
#include <hip/hip_runtime.h>

#include <algorithm>
#include <numeric>
#include <type_traits>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "schema_impl.h"

using namespace packos;

#define HIP_TRY(x)                                                                  \
    do {                                                                            \
        hipError_t _e = (x);                                                        \
        if (_e != hipSuccess) {                                                     \
            set_error(std::string(#x) + ": " + hipGetErrorString(_e));              \
            return PACKOS_E_HIP;                                                    \
        }                                                                           \
    } while (0)

namespace {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kSlot = 8192 + 64;      // LDS staging bytes per wavefront (k_encode_var)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint16_t enc_header(int64_t off, int tag) {
    return (uint16_t)((((uint64_t)off) << 3) & 0xFFFFu) | (uint16_t)(tag & 7);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint32_t t = __shfl_up(x, d, kWave);
        if (lane >= d) x += t;
    }
    return x;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, kWave);
    return x;
}

// =========================================================================
// fixed-size encode
// =========================================================================
// Stage the tile's fixed input columns into LDS with 16-B coalesced loads.
// A tile holds at most 16 KiB of input (T*B <= 16 KiB and the input bytes of
// a blob never exceed its size), i.e. <= 1024 16-B chunks = 4 per thread.
// Each chunk's column is found by a uniform walk over the (few) columns with
// per-lane selects, reading the column table from an LDS copy (fcols_to_lds):
// had the table come from global memory, every lookup's s_waitcnt vmcnt(0)
// would also wait for the previous slot's in-flight data load and serialise
// them.  A thread's 4 loads are thus in flight together.  (Precomputing this
// plan once per workgroup costs ~20 VGPRs and halves occupancy; recomputing
// it is a handful of VALU ops per tile.)
constexpr int kStageSlots = 4;

// The column base pointers come from LDS, so the compiler no longer knows they
// address global memory and would emit flat loads (which need vmcnt(0) AND
// lgkmcnt(0) waits).  Cast back to the global address space explicitly.
typedef __attribute__((address_space(1))) const u32x4 g_u32x4;
template <bool NT>
__device__ __forceinline__ u32x4 gload16(const uint8_t* p) {
    const g_u32x4* gp = (const g_u32x4*)p;
    return NT ? __builtin_nontemporal_load(gp) : *gp;
}

struct LFix {                 // LDS copy of a FixCol with its column base resolved
    const uint8_t* base;
    uint32_t width, lds_off, chunk_begin, pad;
};
constexpr int kLFixBytes = sizeof(LFix);  // 24

__device__ __forceinline__ void fcols_to_lds(const FixProgram& P, const EncCols& cols, uint8_t* lds) {
    LFix* l = (LFix*)(lds + P.fc_lds);
    for (int g = threadIdx.x; g < P.n_fcols; g += kBlock) {
        const FixCol fc = P.fcols[g];
        l[g] = LFix{cols.data[fc.col], fc.width, fc.lds_off, fc.chunk_begin, 0};
    }
}

template <bool NTL>
__device__ __forceinline__ void stage_tile(const FixProgram& P, const EncCols& cols, uint8_t* lds, uint64_t blob0,
                                           uint32_t rows, uint32_t T) {
    (void)T;
    const int tid = threadIdx.x;
    (void)cols;
    const LFix* lfc = (const LFix*)(lds + P.fc_lds);
    u32x4 v[kStageSlots];
    uint32_t dst[kStageSlots];
    bool ok[kStageSlots];
#pragma unroll
    for (int u = 0; u < kStageSlots; u++) {
        const int k = u * kBlock + tid;
        const uint8_t* base = nullptr;
        uint32_t w = 0, lo = 0, cb = 0;
        for (int g = 0; g < P.n_fcols; g++) {
            const LFix fc = lfc[g];
            const bool in = k >= (int)fc.chunk_begin;
            base = in ? fc.base : base;
            w = in ? fc.width : w;
            lo = in ? fc.lds_off : lo;
            cb = in ? fc.chunk_begin : cb;
        }
        const uint32_t byte = (uint32_t)(k - (int)cb) * 16u;
        const uint32_t lim = k < P.total_chunks ? rows * w : 0u;
        const uint8_t* src = base + blob0 * w + byte;
        dst[u] = lo + byte;
        ok[u] = byte < lim;
        if (byte + 16 <= lim) {
            v[u] = gload16<NTL>(src);
        } else if (ok[u]) {  // last, partial chunk of the final tile
            uint32_t w4[4] = {0, 0, 0, 0};
            for (uint32_t j = 0; j < lim - byte; j++) w4[j >> 2] |= (uint32_t)src[j] << (8 * (j & 3));
            v[u] = u32x4{w4[0], w4[1], w4[2], w4[3]};
        }
    }
#pragma unroll
    for (int u = 0; u < kStageSlots; u++)
        if (ok[u]) *(u32x4*)(lds + dst[u]) = v[u];
}

__device__ __forceinline__ uint32_t lds_dword_at(const uint32_t* l32, uint32_t addr) {
    const uint32_t lo = l32[addr >> 2], hi = l32[(addr >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, addr & 3);
}

// Lane-invariant form (B % 4 == 0): thread t owns output dword q = t % (B/4)
// of blobs s, s+R, s+2R ... of the tile; its byte sources sit in registers.
// Used for partial last tiles and shapes k_encode_fixed_tile does not take.
__global__ __launch_bounds__(kBlock) void k_encode_fixed_dw(FixProgram P, EncCols cols, uint8_t* __restrict__ out,
                                                            uint64_t n, uint32_t* __restrict__ status,
                                                            uint32_t st_val) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int T = P.T;
    const uint32_t Q4 = (uint32_t)P.B >> 2;
    const uint32_t tid = threadIdx.x;
    const uint32_t q = tid % Q4, s = tid / Q4, R = kBlock / Q4;
    const uint64_t blob0 = (uint64_t)blockIdx.x * (uint64_t)T;
    const uint32_t rows = (uint32_t)min((uint64_t)T, n - blob0);
    DwDesc d;
    if (s < R) d = P.dw[q];
    fcols_to_lds(P, cols, lds);
    __syncthreads();
    stage_tile<false>(P, cols, lds, blob0, rows, (uint32_t)T);
    __syncthreads();
    if (s < R) {
        const uint32_t* l32 = (const uint32_t*)lds;
        uint32_t* o32 = (uint32_t*)(out + blob0 * (uint64_t)P.B) + q;
        for (uint32_t j = s; j < rows; j += R) {
            uint32_t v = d.cval;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                if ((uint32_t)g < d.nseg) {
                    uint32_t x = lds_dword_at(l32, (uint32_t)d.seg[g].a + j * d.seg[g].w) & d.seg[g].mask;
                    if (d.seg[g].flags & 1u) x = x ? (d.seg[g].mask & 0x01010101u) : 0u;
                    v |= x;
                }
            }
            __builtin_nontemporal_store(v, o32 + (uint64_t)j * Q4);
        }
    }
    if (status)
        for (uint32_t i = tid; i < rows; i += kBlock) status[blob0 + i] = st_val;
}

// One 16-B-per-lane LDS-DMA load: lane l's 16 bytes land at LDS byte address
// m0 + 16*l (wave-uniform m0).  Written as asm so the compiler neither waits
// for it (it would drain with vmcnt(0) before every LDS read or barrier) nor
// reorders LDS accesses across it: every wait for it is explicit.
__device__ __forceinline__ void dma16(const uint8_t* gsrc, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}
// the same, non-temporal: rows read once by the fixed-layout kernels (round-4
// A/B on the box: M encode 0.0889 -> 0.0878 ms, M decode 0.1015 -> 0.0982 ms,
// C4 encode 0.332 -> 0.328 ms; the var tile encoder loses with it, 0.050 -> 0.053)
__device__ __forceinline__ void dma16nt(const uint8_t* gsrc, uint32_t lds_addr) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_addr)
                 : "memory");
}

// One tile per workgroup, LDS-DMA staging with a wave-uniform column walk.
// Each wave-instruction fetches 64 consecutive 16-B chunks of ONE column
// (column base + tile offset are scalars, so a load costs ~2 VALU; no per-
// lane column search), straight into that column's LDS region.  Then one
// vmcnt(0) + barrier.  Output dwords fed by more than one column run or by a
// bool byte ("X dwords", 3 of 64 for metric M) are assembled once per blob
// into an LDS X region (bools normalised there) + barrier, so in the main
// assembly EVERY dword has exactly one source: one ds_read2_b32 +
// v_alignbyte + v_and_or per output dword, 1-KiB-strided NT dword stores.
// (A branch-free per-lane segment loop padded to the widest dword doubled the
// LDS reads and their bank conflicts.)  No persistent loop: the workgroup
// exits without waiting for its stores, so every resident workgroup spends
// its life with loads or stores in flight (the shape of the fastest plain
// copy of this traffic, tools/membench2.hip).
template <int PER>  // T == PER * R (the compiler's T = 16 * floor(1024 / B))
__global__ __launch_bounds__(kBlock) void k_encode_fixed_tile(FixProgram P, FixStage S, uint8_t* __restrict__ out,
                                                              uint32_t* __restrict__ status, uint32_t st_val) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t T = (uint32_t)P.T;
    const uint32_t B = (uint32_t)P.B;
    const uint32_t Q4 = B >> 2;
    const uint32_t tid = threadIdx.x;
    const uint32_t q = tid % Q4, s = tid / Q4, R = kBlock / Q4;
    const uint32_t lane = tid % kWave, wv = tid / kWave;
    const uint64_t blob0 = blockIdx.x * (uint64_t)T;  // full tiles only (the launcher sends
                                                      // a partial last tile to k_encode_fixed_dw)
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    for (int g = 0; g < S.n; g++) {
        const uint32_t nch = (T * S.c[g].width) >> 4;
        const uint8_t* cbase = S.c[g].base + blob0 * S.c[g].width;
        // in a register: dma16's memory clobber would make the compiler re-read
        // the kernel argument (a scalar load + wait) before every DMA
        const uint32_t lbase = lds0 + S.c[g].lds_off;
        for (uint32_t c0 = wv * kWave; c0 < nch; c0 += kBlock) {
            if (c0 + lane < nch) dma16nt(cbase + (c0 + lane) * 16u, __builtin_amdgcn_readfirstlane(lbase + c0 * 16u));
        }
    }
    // descriptors (their global loads queue behind the DMA)
    const DwDesc* dd = P.tdw + q;
    const uint32_t cval = dd->cval;
    const DwSeg sg = dd->seg[0];
    // a wave stores G = 64 / Q4 consecutive blobs per instruction (256 B) and
    // its PER instructions continue that run: wave w covers blobs
    // [w PER G, (w + 1) PER G) of the tile (M encode 0.0875 -> 0.0867 ms, A/B;
    // PACKOS_FIXT_STRIDED: the round-3 order, blob groups R apart)
    // (when Q4 divides 64: a wave holds whole blobs; else the strided order)
#ifndef PACKOS_FIXT_STRIDED
    const bool contig = Q4 <= (uint32_t)kWave && (uint32_t)kWave % Q4 == 0;
#else
    const bool contig = false;
#endif
    const uint32_t G = contig ? (uint32_t)kWave / Q4 : 1u;
    const uint32_t b0s = contig ? (s / G) * PER * G + s % G : s;   // this thread's first blob
    uint32_t a = (uint32_t)sg.a + b0s * sg.w;   // LDS byte address of this thread's first dword
    const uint32_t xs = (contig ? G : R) * sg.w, xm = sg.mask;
    // X items i = blob * nx + x, taken at a stride SX that is a multiple of nx
    // (the largest <= the block), so a thread keeps ONE descriptor for all its
    // items, loaded here with the DMAs in flight (a stride of the block size
    // reloaded a descriptor from global memory per item: C2 has 768 X items)
    const uint32_t nx = (uint32_t)P.nx, nxi = T * nx, SX = nx ? (kBlock / nx) * nx : 0u;
    DwDesc xd;  // this thread's X descriptor
    if (tid < nxi && tid < SX) xd = P.xdw[tid % nx];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t* l32 = (uint32_t*)lds;
    if (nxi) {
        auto assemble = [&](uint32_t i, const DwDesc& d) {
            const uint32_t j = i / nx;
            uint32_t val = 0;
#pragma unroll
            for (int g = 0; g < 4; g++) {
                if ((uint32_t)g < d.nseg) {
                    uint32_t x = lds_dword_at(l32, (uint32_t)d.seg[g].a + j * d.seg[g].w) & d.seg[g].mask;
                    if (d.seg[g].flags & 1u) x = x ? (d.seg[g].mask & 0x01010101u) : 0u;
                    val |= x;
                }
            }
            l32[((uint32_t)P.x_lds >> 2) + i] = val;
        };
        if (tid < SX)
            for (uint32_t i = tid; i < nxi; i += SX) assemble(i, xd);
        __syncthreads();
    }
    if (s < R) {  // R * Q4 <= 256: the rest of the threads idle here
        uint32_t* o32 = (uint32_t*)(out + blob0 * B) + b0s * Q4 + q;
        const uint32_t ostep = (contig ? G : R) * Q4;
#pragma unroll
        for (int it = 0; it < PER; it++) {
            uint32_t val = cval;
            const uint32_t lo = l32[a >> 2], hi = l32[(a >> 2) + 1];
            val |= __builtin_amdgcn_alignbyte(hi, lo, a) & xm;  // uses a & 3
            a += xs;
            if (it & 1) asm volatile("" : "+v"(a));  // two iterations' reads in flight, no address table
            __builtin_nontemporal_store(val, o32);
            o32 += ostep;
        }
    }
    if (status)
        for (uint32_t i = tid; i < T; i += kBlock) status[blob0 + i] = st_val;
}

// General form (any B <= 1024): 16-B output chunks, per-dword segment lists
// over a 4-blob period held in LDS.
__global__ __launch_bounds__(kBlock) void k_encode_fixed(FixProgram P, EncCols cols,
                                                         uint8_t* __restrict__ out, uint64_t n,
                                                         uint32_t* __restrict__ status,
                                                         uint32_t st_val) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int T = P.T;
    const uint32_t B = (uint32_t)P.B;
    const uint64_t blob0 = (uint64_t)blockIdx.x * (uint64_t)T;
    const uint32_t rows = (uint32_t)min((uint64_t)T, n - blob0);
    const int tid = threadIdx.x;

    // descriptor tables -> LDS (after the tile region)
    uint32_t* s_index = (uint32_t*)(lds + P.lds_bytes);
    FixSeg* s_segs = (FixSeg*)(lds + P.lds_bytes + ((B + 1) * 4 + 15) / 16 * 16);
    const uint32_t nsegs = P.seg_index[B];
    for (uint32_t k = tid; k <= B; k += kBlock) s_index[k] = P.seg_index[k];
    for (uint32_t k = tid; k < nsegs; k += kBlock) s_segs[k] = P.segs[k];
    fcols_to_lds(P, cols, lds);
    __syncthreads();
    stage_tile<false>(P, cols, lds, blob0, rows, (uint32_t)T);
    __syncthreads();

    // ---- assemble 16-B output chunks
    const uint32_t* l32 = (const uint32_t*)lds;
    const uint32_t tile_bytes = rows * B;
    uint8_t* obase = out + blob0 * (uint64_t)B;
    const uint32_t nchunks = (tile_bytes + 15) / 16;
    for (uint32_t c = tid; c < nchunks; c += kBlock) {
        uint32_t w0 = 4 * c;
        uint32_t per = w0 / B;
        uint32_t r = w0 - per * B;
        uint32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t v = 0;
            const uint32_t s1 = s_index[r + 1];
            for (uint32_t s = s_index[r]; s < s1; s++) {
                const FixSeg g = s_segs[s];
                if (g.stride4 == 0) {
                    v |= g.cval;
                } else {
                    uint32_t x = lds_dword_at(l32, (uint32_t)g.a + per * g.stride4) & g.mask;
                    if (g.cval & 1u) x = x ? (g.mask & 0x01010101u) : 0u;
                    v |= x;
                }
            }
            o[i] = v;
            if (++r == B) { r = 0; per++; }
        }
        const uint32_t ob = 16 * c;
        if (ob + 16 <= tile_bytes) {
            *(uint4*)(obase + ob) = make_uint4(o[0], o[1], o[2], o[3]);
        } else {
            for (uint32_t j = 0; ob + j < tile_bytes; j++) obase[ob + j] = (uint8_t)(o[j >> 2] >> (8 * (j & 3)));
        }
    }
    if (status)
        for (uint32_t i = tid; i < rows; i += kBlock) status[blob0 + i] = st_val;
}

__global__ void k_fill_offsets(uint64_t* offs, uint64_t n, uint64_t B) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) offs[i] = i * B;
}
// host pipelines: offs[i] = base + i * B for i <= n; or offs[i] += add for i < n
__global__ void k_fill_offsets_base(uint64_t* offs, uint64_t n, uint64_t base, uint64_t B) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) offs[i] = base + i * B;
}
__global__ void k_add_base(uint64_t* offs, uint64_t n, uint64_t add) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) offs[i] += add;
}

// =========================================================================
// variable-size encode
// =========================================================================
// var offsets of either width (EncCols::off64 marks u64 columns)
__device__ __forceinline__ uint64_t col_off(const EncCols& cols, int c, uint64_t i) {
    return ((cols.off64 >> c) & 1ull) ? ((const uint64_t*)cols.off[c])[i] : (uint64_t)((const uint32_t*)cols.off[c])[i];
}

__device__ __forceinline__ uint64_t present_mask(const EncProgram& P, const EncCols& cols, uint64_t i) {
    uint64_t pm = 0;
    for (int c = 0; c < P.n_conts; c++) {
        const EncCont ct = P.conts[c];
        bool p = ct.parent < 0 ? true : ((pm >> ct.parent) & 1ull);
        if (p && ct.valid_col >= 0) {
            const uint8_t* v = cols.valid[ct.valid_col];
            if (v) p = v[i] != 0;
        }
        if (p) pm |= 1ull << c;
    }
    return pm;
}

__device__ __forceinline__ uint32_t item_size(const EncItem& it, const EncCols& cols, uint64_t i,
                                              uint64_t pm, uint32_t* slack) {
    if (!((pm >> it.cont) & 1ull)) return 0;
    switch (it.type) {
        case IT_HDR: case IT_CONST: return it.size;
        case IT_FIXED:
            if (it.nullable) {
                const uint8_t* v = cols.valid[it.col];
                if (v && !v[i]) { *slack += it.size; return 0; }
            }
            return it.size;
        case IT_VAR:
            return (uint32_t)(col_off(cols, it.col, i + 1) - col_off(cols, it.col, i));
    }
    return 0;
}

// ---- scan support --------------------------------------------------------
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        uint64_t t = __shfl_up(x, d, kWave);
        if (lane >= d) x += t;
    }
    return x;
}

// One blob, one wavefront: item sizes -> wavefront prefix scan -> header
// words -> payload.  `slot` (LDS, kSlot bytes) stages the blob for aligned
// 16-B stores; with slot == nullptr (or a blob too big for it) bytes go
// straight to HBM.  `pos` is a per-wave LDS array of n_items + 1 words.
__device__ void var_blob_wave(const EncProgram& P, const EncCols& cols, uint64_t i, uint64_t o,
                              uint8_t* __restrict__ out, uint64_t cap, uint32_t* __restrict__ status,
                              uint8_t* slot, uint32_t* pos, int lane) {
    const uint64_t pm = present_mask(P, cols, i);
    // item sizes -> wavefront prefix scan -> positions
    uint32_t running = 0, slack = 0;
    for (int b = 0; b < P.n_items; b += kWave) {
        const int k = b + lane;
        uint32_t sz = 0;
        if (k < P.n_items) sz = item_size(P.items[k], cols, i, pm, &slack);
        const uint32_t incl = wave_incl_scan(sz, lane);
        if (k < P.n_items) pos[k] = running + incl - sz;
        running += __shfl(incl, kWave - 1, kWave);
    }
    slack = wave_sum(slack);
    const uint32_t payload_end = running;
    const uint32_t total = running + (P.mode == PACKOS_MODE_PACKABLE ? slack : 0u);
    if (lane == 0) pos[P.n_items] = running;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    if (o + total > cap) {
        if (status && lane == 0) status[i] = (uint32_t)PACKOS_ERR_ENCODE;
        __builtin_amdgcn_wave_barrier();
        return;
    }
    const bool staged = slot && total + 16 <= (uint32_t)kSlot;
    uint8_t* dst = staged ? (slot + (o & 15)) : (out + o);

    // header words (lane per header)
    bool ovf = false;
    for (int b = 0; b < P.n_hdrs; b += kWave) {
        const int k = b + lane;
        if (k < P.n_hdrs) {
            const EncHdr h = P.hdrs[k];
            if ((pm >> h.cont) & 1ull) {
                const uint32_t hpos = pos[h.hdr_item];
                uint16_t v;
                if (h.relative) {
                    const int64_t off = (int64_t)pos[h.target] - (int64_t)(hpos + P.items[h.hdr_item].size);
                    ovf |= off >= 8192;
                    v = enc_header(off, h.tag);
                } else {
                    v = h.value;
                    ovf |= h.ovf != 0;
                }
                dst[hpos + 2 * h.j] = (uint8_t)v;
                dst[hpos + 2 * h.j + 1] = (uint8_t)(v >> 8);
            }
        }
    }
    // payload bytes (wave per item)
    for (int k = 0; k < P.n_items; k++) {
        const EncItem it = P.items[k];
        if (it.type == IT_HDR) continue;
        const uint32_t p0 = pos[k], p1 = pos[k + 1];
        const uint32_t len = p1 - p0;
        if (len == 0) continue;
        const uint8_t* src;
        if (it.type == IT_CONST) src = P.lits + it.lit;
        else if (it.type == IT_FIXED) src = cols.data[it.col] + i * (uint64_t)it.size;
        else src = cols.data[it.col] + col_off(cols, it.col, i);
        if (it.is_bool) {
            if (lane == 0) dst[p0] = src[0] != 0;
        } else {
            for (uint32_t j = lane; j < len; j += kWave) dst[p0 + j] = src[j];
        }
    }
    // packable.Pack slack: zero bytes after the End-marked payload
    for (uint32_t j = lane; j < total - payload_end; j += kWave) dst[payload_end + j] = 0;
    if (staged) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t mis = (uint32_t)(o & 15);
        const uint32_t head = min(total, (16u - mis) & 15u);
        if ((uint32_t)lane < head) out[o + lane] = dst[lane];
        const uint32_t body = (total - head) / 16;
        const uint8_t* sb = dst + head;              // 16-B aligned in LDS
        uint8_t* gb = out + o + head;                // 16-B aligned in HBM
        for (uint32_t c = lane; c < body; c += kWave) *(uint4*)(gb + 16 * c) = *(const uint4*)(sb + 16 * c);
        const uint32_t done = head + body * 16;
        if ((uint32_t)lane < total - done) out[o + done + lane] = dst[done + lane];
        __builtin_amdgcn_wave_barrier();
    }
    const bool any_ovf = __ballot(ovf) != 0ull;
    if (status && lane == 0) status[i] = any_ovf ? PACKOS_STATUS_OVERFLOW13 : 0u;
    // make sure no lane reuses the slot / pos array before every lane has read it
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// pass 2 (general): one wavefront per blob
__global__ __launch_bounds__(kBlock) void k_encode_var(EncProgram P, EncCols cols, const uint64_t* __restrict__ offs,
                                                       uint64_t stride, uint8_t* __restrict__ out, uint64_t cap,
                                                       uint64_t n, uint32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int npos = P.n_items + 1;
    const int wave_bytes = kSlot + ((npos * 4 + 15) / 16) * 16;
    uint8_t* slot = lds + wave * wave_bytes;
    uint32_t* pos = (uint32_t*)(slot + kSlot);
    for (uint64_t i = (uint64_t)blockIdx.x * kWavesPerBlock + wave; i < n;
         i += (uint64_t)gridDim.x * kWavesPerBlock)
        var_blob_wave(P, cols, i, offs ? offs[i] : i * stride, out, cap, status, slot, pos, lane);
}

// EncodeFunc value checks (Range / SDateRange / CheckFunc Prefix-Suffix),
// one thread per blob, after the encode kernel on the same stream.  The first
// failing check in emission order wins (EncodeValue stops there); values
// inside a nil container or nil themselves are not encoded, so not checked.
// Passing blobs are not touched; a failing blob's status becomes ErrEncode at
// position -1 with the leaf's code in bits 24..29.
__global__ __launch_bounds__(kBlock) void k_encode_checks(const EncCheck* __restrict__ chk, int nchk, EncProgram P,
                                                          EncCols cols, uint64_t n, uint32_t* __restrict__ status,
                                                          int need_pm) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t pm = need_pm ? present_mask(P, cols, i) : ~0ull;
    for (int k = 0; k < nchk; k++) {
        const EncCheck c = chk[k];
        if (c.flags & CHK_PANIC) {   // every field written, then the Go index panic (no bytes)
            status[i] = PACKOS_STATUS_PANIC;
            return;
        }
        if (!((pm >> c.cont) & 1ull)) continue;
        bool bad;
        if (c.flags & CHK_FAIL) {
            bad = true;   // the container is present: its Encode fails whatever the value
        } else if (c.flags & CHK_RANGE) {
            const uint8_t* v = cols.valid[c.col];
            if (v && !v[i]) continue;
            const uint8_t* p = cols.data[c.col] + i * (uint64_t)c.width;
            uint64_t u = 0;
            for (uint32_t b = 0; b < c.width; b++) u |= (uint64_t)p[b] << (8 * b);
            const int sh = 64 - 8 * (int)c.width;
            const int64_t x = (int64_t)(u << sh) >> sh;
            bad = ((c.flags & CHK_MIN) && x < c.rmin) || ((c.flags & CHK_MAX) && x > c.rmax);
        } else {
            const uint8_t* p;
            uint64_t len;
            if (c.width) {
                p = cols.data[c.col] + i * (uint64_t)c.width;
                len = c.width;
            } else {
                const uint64_t a = col_off(cols, c.col, i);
                p = cols.data[c.col] + a;
                len = col_off(cols, c.col, i + 1) - a;
            }
            bad = len < c.lit_len;
            const uint64_t at = (c.flags & CHK_PREFIX) ? 0ull : len - c.lit_len;
            for (uint32_t b = 0; !bad && b < c.lit_len; b++) bad = p[at + b] != P.lits[c.lit + b];
        }
        if (bad) {
            // position -1 (bits 8..23 = 0): EncodeValue wraps every leaf error as
            // SchemaError(ErrEncode, ChainName, "", -1, err) (schema/schema.go:919-936)
            status[i] = (status[i] & (PACKOS_STATUS_PANIC | PACKOS_STATUS_OVERFLOW13)) | (uint32_t)PACKOS_ERR_ENCODE |
                        (c.inner << 24);
            return;
        }
    }
}

typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint64_t g_u64;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

#include "encode_var.inc"
#include "encode_flat.inc"
#include "encode_ext.inc"

// =========================================================================
// decode: schema.DecodeBuffer, one thread per blob
// =========================================================================
constexpr int kDecDepth = 8;

struct DSeq {
    int64_t len, base, count, pos, next_off, cur_off;
    uint64_t start;     // absolute arena offset of this (sub)buffer
    int next_type, cur_type;
    int xw;             // 1: an ADR-001 extended container (u32 entries after a 4-byte lead)
};


// Byte readers for the decoder: straight from the arena, or from a per-blob
// LDS window (the blob's first W bytes) with the arena behind it.
struct GReader {
    const uint8_t* a;
    __host__ __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return a[p]; }
    __host__ __device__ __forceinline__ uint32_t u16(uint64_t p) const { return a[p] | (a[p + 1] << 8); }
    __host__ __device__ __forceinline__ uint32_t u32(uint64_t p) const {
        return a[p] | (a[p + 1] << 8) | (a[p + 2] << 16) | ((uint32_t)a[p + 3] << 24);
    }
};
// LDS window over arena[base, base + W): dword k of the window at
// win32[k * stride] (stride 1: one contiguous window; stride kBlock: the
// per-thread windows interleaved by dword, so the lanes of a wave reading the
// same window dword hit distinct banks).  Reads of 2 / 4 bytes inside the
// window are one or two ds_read_b32 + v_alignbyte.
struct WReader {
    const uint8_t* a;
    const uint32_t* win32;
    uint64_t base;
    uint32_t W, stride;
    __device__ __forceinline__ uint32_t dw(uint32_t k) const { return win32[k * stride]; }
    __device__ __forceinline__ uint32_t operator()(uint64_t p) const {
        const uint64_t d = p - base;
        return d < W ? (dw((uint32_t)d >> 2) >> (8 * (d & 3))) & 0xFFu : a[p];
    }
    __device__ __forceinline__ uint32_t u32(uint64_t p) const {
        const uint64_t d = p - base;
        if (d + 4 <= W) {
            const uint32_t k = (uint32_t)d >> 2, q = (uint32_t)d & 3u;
            const uint32_t lo = dw(k);
            return q ? __builtin_amdgcn_alignbyte(dw(k + 1), lo, q) : lo;
        }
        return (*this)(p) | ((*this)(p + 1) << 8) | ((*this)(p + 2) << 16) | ((*this)(p + 3) << 24);
    }
    __device__ __forceinline__ uint32_t u16(uint64_t p) const {
        const uint64_t d = p - base;
        if (d + 2 <= W && (d & 3) != 3) return (dw((uint32_t)d >> 2) >> (8 * (d & 3))) & 0xFFFFu;
        return (*this)(p) | ((*this)(p + 1) << 8);
    }
};
// LDS-window reader without bounds checks or HBM fallback, for reads the
// caller has proven to lie inside the window (dword k at win32[k * stride]).
// Reads of 2 / 4 bytes are two dword reads + v_alignbyte, branch-free.
struct LReader {
    const uint32_t* win32;
    uint64_t base;
    uint32_t stride;
    __device__ __forceinline__ uint32_t dw(uint32_t k) const { return win32[k * stride]; }
    __device__ __forceinline__ uint32_t u32(uint64_t p) const {
        const uint32_t d = (uint32_t)(p - base), k = d >> 2;
        return __builtin_amdgcn_alignbyte(dw(k + 1), dw(k), d & 3u);
    }
    __device__ __forceinline__ uint32_t u16(uint64_t p) const { return u32(p) & 0xFFFFu; }
    __device__ __forceinline__ uint32_t operator()(uint64_t p) const {
        const uint32_t d = (uint32_t)(p - base);
        return (dw(d >> 2) >> (8 * (d & 3u))) & 0xFFu;
    }
};
template <class R>
__host__ __device__ __forceinline__ uint16_t rd16r(const R& r, uint64_t p) { return (uint16_t)r.u16(p); }

// NewSeqGetAccess (seqget.go:22-47).  xkind != 0 (extended mode only): the
// buffer must be an extended container of that kind (program.h, ADR-001):
// the same cursor over u32 entries, count = (base - 4) / 4.
template <class R>
__host__ __device__ __forceinline__ int dseq_init(DSeq& s, const R& a, uint64_t start, int64_t len, int xkind = 0) {
    if (xkind) {
        if (len < 12 || rd16r(a, start) != kExtMarker || (int)rd16r(a, start + 2) != xkind) return 1;
        const uint32_t e0 = a.u32(start + 4);
        const int64_t base = e0 >> 3;
        if (base < 12 || (base & 3) || len < base) return 1;
        const uint32_t e1 = a.u32(start + 8);
        s.len = len; s.base = base; s.count = (base - 4) / 4; s.pos = 0; s.start = start;
        s.cur_off = base; s.cur_type = e0 & 7;
        s.next_off = (int64_t)(e1 >> 3) + base; s.next_type = e1 & 7;
        s.xw = 1;
        return 0;
    }
    s.xw = 0;
    if (len < 4) return 1;
    const uint16_t h0 = rd16r(a, start);
    const int64_t base = h0 >> 3;
    if (len < base) return 1;
    const uint16_t h1 = rd16r(a, start + 2);
    s.len = len; s.base = base; s.count = base / 2; s.pos = 0; s.start = start;
    s.cur_off = base; s.cur_type = h0 & 7;
    s.next_off = (h1 >> 3) + base; s.next_type = h1 & 7;
    return 0;
}
// Advance (seqget.go:85-103): 0 ok, 1 out of bounds, 2 Go panic (unchecked header read)
template <class R>
__host__ __device__ __forceinline__ int dseq_advance(DSeq& s, const R& a) {
    if (s.pos + 2 > s.count) return 1;
    s.pos++;
    s.cur_off = s.next_off;
    s.cur_type = s.next_type;
    if (s.cur_type != 0) {
        if (s.xw) {   // extended: entry pos + 1 after the 4-byte lead; a short buffer is an EOF error
            if (4 + (s.pos + 1) * 4 + 4 > s.len) return 1;
            const uint32_t h = a.u32(s.start + 4 + (s.pos + 1) * 4);
            s.next_off = (int64_t)(h >> 3) + s.base;
            s.next_type = h & 7;
            return 0;
        }
        if ((s.pos + 1) * 2 + 2 > s.len) return 2;
        const uint16_t h = rd16r(a, s.start + (s.pos + 1) * 2);
        s.next_off = (h >> 3) + s.base;
        s.next_type = h & 7;
    }
    return 0;
}
// precheck (schema.go:997-1013): 0 ok else ErrConstraintViolated
__host__ __device__ __forceinline__ int dprecheck(const DSeq& s, int tag, int64_t hint, bool nullable, int64_t& w) {
    if (s.pos >= s.count) return 3;
    if (s.next_off > s.len) return 3;
    if (s.cur_type != tag) return 3;
    w = s.next_off - s.cur_off;
    if (!nullable && hint != 0 && w != hint) return 3;
    return 0;
}

constexpr int kPanic = 0x100;
constexpr int kPos0 = 0x200;   // the error's position is 0, not the field's (schema.go:1756-1758)

// w bytes from reader position p to a column row; dword stores when aligned
template <class R>
__host__ __device__ __forceinline__ void copy_out(uint8_t* dst, const R& r, uint64_t p, uint32_t w) {
    if ((w & 3) == 0 && ((uintptr_t)dst & 3) == 0) {
        for (uint32_t j = 0; j < w; j += 4) *(uint32_t*)(dst + j) = r.u32(p + j);
    } else {
        for (uint32_t j = 0; j < w; j++) dst[j] = (uint8_t)r(p + j);
    }
}

struct Frame {
    DSeq q;
    int node;
    int k;
};

// DecodeBuffer (schema.go:893-910) for blob i = arena[a0, a1): writes its
// leaves into the output columns and returns the packed status word.  Host +
// device: the host runs it once on the canonical blob to qualify a schema for
// the fixed-layout fast path (same code, so the qualification is exact).
// EXT (PACKOS_MODE_EXTENDED): a top-level blob starting 02 00 and every
// tag-2 field are read as extended containers (program.h).
// VAL: ValidateBuffer (schema.go:880-891) instead — the status under the
// Validate methods' rules, no outputs (cols unused): SBool..SFloat64 never
// read their payload (:596-715, no short-payload panic), CheckFunc passes an
// empty string of a nullable receiver (:1085-1087), SchemaMap has no
// odd-count check (:336-359).
template <class R, bool EXT = false, bool VAL = false>
__host__ __device__ uint32_t decode_blob(const DecProgram& P, const DecCols& cols, const R& arena, uint64_t a0,
                                         uint64_t a1, uint64_t i) {
    // the current frame lives in registers; outer frames are spilled to `stk`
    // (scratch) only while a nested tuple/map is being read
    Frame cur;
    Frame stk[kDecDepth];
    int d = 0;
    const int xroot = EXT && a1 - a0 >= 2 && rd16r(arena, a0) == kExtMarker ? PACKOS_TAG_TUPLE : 0;
    if (dseq_init(cur.q, arena, a0, (int64_t)(a1 - a0), xroot))
        return (uint32_t)PACKOS_ERR_INVALID_FORMAT;  // position -1
    cur.node = P.root;
    cur.k = 0;
    int err = 0;
    for (;;) {
        const DecNode fn = P.nodes[cur.node];
        if (cur.k >= fn.nkids) {
            if (d == 0) break;
            // container finished: mark it present, then Advance the parent past it
            if (!VAL && cols.valid[fn.col]) cols.valid[fn.col][i] = 1;
            d--;
            cur = stk[d];
            const int a = dseq_advance(cur.q, arena);
            if (a) { err = a == 2 ? kPanic : 2; break; }
            cur.k++;
            continue;
        }
        const int nid = P.kids[fn.kid0 + cur.k];
        const DecNode nd = P.nodes[nid];
        DSeq& q = cur.q;
        int64_t w = 0;
        if (nd.kind == K_TUPLE || nd.kind == K_MAP) {
            if (nd.kind == K_TUPLE && (nd.variable & DT_NAMES_BAD)) { err = 3 | kPos0; break; }
            const bool xc = EXT && q.cur_type == PACKOS_TAG_EXTENDED;   // an extended container field
            err = dprecheck(q, xc ? PACKOS_TAG_EXTENDED : nd.tag, -1, nd.nullable, w);
            if (err) break;
            if (!VAL && nd.kind == K_MAP && (nd.nkids & 1)) { err = 3; break; }
            if (w != 0) {
                // PeekNestedSeq (seqget.go:105-121)
                if (q.next_off - q.cur_off <= 0 || q.next_off > q.len) { err = 1; break; }
                if (d + 1 >= kDecDepth) { err = 1; break; }
                Frame c;
                if (dseq_init(c.q, arena, q.start + q.cur_off, q.next_off - q.cur_off, xc ? nd.tag : 0)) {
                    err = 1;
                    break;
                }
                // arg count: TupleSchema checks it only when argCount > 0
                // (schema.go:1607), TupleSchemaNamed always (:1773)
                if (nd.kind == K_TUPLE && !(nd.variable & DT_VARIABLE) && (nd.nkids > 0 || (nd.variable & DT_NAMED)) &&
                    (c.q.count - 1) != nd.nkids) {
                    err = 3;
                    break;
                }
                c.node = nid;
                c.k = 0;
                stk[d] = cur;
                cur = c;
                d++;
                continue;
            }
            if (!VAL && cols.valid[nd.col]) cols.valid[nd.col][i] = 0;  // nil container
            const int a = dseq_advance(q, arena);
            if (a) { err = a == 2 ? kPanic : 2; break; }
            cur.k++;
            continue;
        }
        // primitives: validatePrimitiveAndGetPayload (schema.go:1031-1052)
        const int64_t hint = nd.width;
        err = dprecheck(q, nd.tag, hint, nd.nullable, w);
        if (err) break;
        const int64_t ps = w > 0 ? q.cur_off : -1;
        {
            const int a = dseq_advance(q, arena);
            if (a) { err = a == 2 ? kPanic : 2; break; }
        }
        const uint64_t pay = q.start + (ps < 0 ? 0 : ps);
        const uint32_t have = ps < 0 ? 0u : (uint32_t)w;
        // DefaultDecodeValue: an empty payload reads as the literal (schema.go:283-285)
        const bool dflt = have == 0 && (nd.check & CHK_DEFAULT) && nd.dlit_len > 0;
        switch (nd.kind) {
            case K_INT: case K_UINT: case K_FLOAT: case K_BOOL: {
                if (VAL) {
                    // only Range / SDateRange ValidateFuncs read the payload
                    // (schema.go:1177-1188, 2198-2212)
                    if (ps < 0 || !(nd.check & (CHK_RANGE | CHK_DATE))) break;
                    if (w < nd.width) { err = kPanic; break; }
                } else {
                    if (ps < 0) {
                        if (cols.valid[nd.col]) cols.valid[nd.col][i] = 0;
                        break;
                    }
                    if (w < nd.width) { err = kPanic; break; }  // LittleEndian.UintXX on a short slice
                    uint8_t* dstp = cols.data[nd.col] + i * (uint64_t)nd.width;
                    if (nd.kind == K_BOOL) dstp[0] = arena(pay) != 0;
                    else copy_out(dstp, arena, pay, (uint32_t)nd.width);
                    if (cols.valid[nd.col]) cols.valid[nd.col][i] = 1;
                }
                if (nd.check & CHK_RANGE) {   // CheckIntRange after Advance (schema.go:1187-1201, 2213-2224)
                    uint64_t u = 0;
                    for (int b = 0; b < nd.width; b++) u |= (uint64_t)arena(pay + b) << (8 * b);
                    const int sh = 64 - 8 * nd.width;
                    const int64_t v = (int64_t)(u << sh) >> sh;
                    if (((nd.check & CHK_MIN) && v < nd.rmin) || ((nd.check & CHK_MAX) && v > nd.rmax))
                        err = (nd.check & CHK_DATE) ? PACKOS_ERR_DATE_OUT_OF_RANGE : PACKOS_ERR_OUT_OF_RANGE;
                }
                break;
            }
            case K_STRING: case K_BYTES:
                if (VAL) {
                } else if (nd.width > 0) {
                    uint8_t* dstp = cols.data[nd.col] + i * (uint64_t)nd.width;
                    copy_out(dstp, arena, pay, (uint32_t)nd.width);
                } else {
                    cols.start[nd.col][i] = dflt ? PACKOS_VIEW_DEFAULT : ps < 0 ? 0ull : q.start + (uint64_t)ps;
                    cols.length[nd.col][i] = dflt ? nd.dlit_len : have;
                }
                if ((nd.check & CHK_STR) && !(VAL && nd.nullable && (dflt ? nd.dlit_len : have) == 0)) {
                    // CheckFunc DecodeFunc / ValidateFunc: HasPrefix / HasSuffix (schema.go:1072-1108)
                    const uint32_t len = dflt ? nd.dlit_len : have, L = nd.lit_len;
                    bool ok = len >= L;
                    const uint32_t at = (nd.check & CHK_PREFIX) ? 0u : len - L;
                    for (uint32_t j = 0; ok && j < L; j++) {
                        const uint32_t c = dflt ? P.lits[nd.dlit + at + j] : arena(pay + at + j);
                        ok = c == P.lits[nd.lit + j];
                    }
                    if (!ok) err = (nd.check & CHK_PREFIX) ? PACKOS_ERR_STRING_PREFIX : PACKOS_ERR_STRING_SUFFIX;
                }
                break;
            case K_MATCH: {
                const uint32_t len = dflt ? nd.dlit_len : have;
                if (VAL && nd.nullable && len == 0) break;   // ValidateFunc (schema.go:1085-1087)
                bool eq = len == nd.lit_len;
                for (uint32_t j = 0; eq && j < len; j++)
                    eq = (dflt ? P.lits[nd.dlit + j] : arena(pay + j)) == P.lits[nd.lit + j];
                if (!eq) err = PACKOS_ERR_STRING_MATCH;
                break;
            }
        }
        if (err) break;
        cur.k++;
    }
    uint32_t sv = 0;
    if (err) {
        const uint32_t posv = (uint32_t)((d == 0 ? cur.k : stk[0].k) + 1) << 8;
        if (err & kPos0) sv = d == 0 ? (uint32_t)(err & 0xFF) | (1u << 8) : (uint32_t)PACKOS_ERR_INVALID_FORMAT | posv;
        else if (err == kPanic) sv = PACKOS_STATUS_PANIC | posv;
        else sv = (uint32_t)(d == 0 ? err : PACKOS_ERR_INVALID_FORMAT) | posv;
    }
    return sv;
}

// Canonical fast path of DecodeBuffer for a flat chain of F leaves: when the
// blob is exactly F fields + End (h0 = 2(F+1)), every tag matches, offsets
// rise to End = len, fixed leaves have their width (nullable ones may be
// empty = nil), MATCH literals and value checks hold, the SeqGetAccess walk
// (seqget.go:22-103) and every precheck (schema.go:997-1013) succeed and the
// fields are plain slices: gather them straight from the header words (all
// read up front).  Anything else returns kFlatFallback and decode_blob runs.
constexpr uint32_t kFlatFallback = 0xFFFFFFFFu;
template <class R, bool VAL = false>
__device__ __forceinline__ uint32_t decode_flat(const DecProgram& P, const DecCols& cols, const R& r, uint64_t a0,
                                                uint64_t a1, uint64_t i) {
    const int F = P.flat;
    const int64_t len = (int64_t)(a1 - a0);
    if (len < 4) return kFlatFallback;
    // header words come from the reader (the LDS window for the prefix)
    const uint32_t h0 = r.u16(a0), hend = r.u16(a0 + 2 * F);
    const int64_t base = h0 >> 3;
    if (base != 2 * (F + 1) || len < base || (hend & 7u) != 0 || (int64_t)(hend >> 3) + base != len)
        return kFlatFallback;
    const DecNode root = P.nodes[P.root];
    // pass 1: structure + value checks (no output written)
    int64_t prev = base;
    bool bad = false;
    uint32_t hj = h0;
    for (int j = 0; j < F && !bad; j++) {
        {
            const uint32_t hn = r.u16(a0 + 2 * (j + 1));
            const DecNode nd = P.nodes[P.kids[root.kid0 + j]];
            const int64_t o = j == 0 ? base : (int64_t)(hj >> 3) + base;
            const int64_t nx = (int64_t)(hn >> 3) + base;
            bad = (int)(hj & 7u) != nd.tag || o < prev || nx < o;
            hj = hn;
            prev = o;
            const int64_t w = nx - o;
            const uint64_t pay = a0 + (uint64_t)o;
            if (!bad) {
                if (nd.kind == K_INT || nd.kind == K_UINT || nd.kind == K_FLOAT || nd.kind == K_BOOL) {
                    bad = w != nd.width && !(nd.nullable && w == 0);
                    if (!bad && (nd.check & CHK_RANGE) && w) {
                        uint64_t u = 0;
                        for (int x = 0; x < nd.width; x++) u |= (uint64_t)r(pay + x) << (8 * x);
                        const int sh = 64 - 8 * nd.width;
                        const int64_t v = (int64_t)(u << sh) >> sh;
                        bad = ((nd.check & CHK_MIN) && v < nd.rmin) || ((nd.check & CHK_MAX) && v > nd.rmax);
                    }
                } else if (nd.kind == K_STRING || nd.kind == K_BYTES) {
                    bad = nd.width > 0 && w != nd.width;
                    if (!bad && (nd.check & CHK_STR)) {
                        const bool dflt = w == 0 && (nd.check & CHK_DEFAULT) && nd.dlit_len > 0;
                        const uint32_t L = dflt ? nd.dlit_len : (uint32_t)w, K = nd.lit_len;
                        bad = L < K;
                        const uint32_t at = (nd.check & CHK_PREFIX) ? 0u : L - K;
                        for (uint32_t x = 0; !bad && x < K; x++) {
                            const uint32_t c = dflt ? P.lits[nd.dlit + at + x] : r(pay + at + x);
                            bad = c != P.lits[nd.lit + x];
                        }
                    }
                } else if (nd.kind == K_MATCH) {
                    const bool dflt = w == 0 && (nd.check & CHK_DEFAULT) && nd.dlit_len > 0;
                    const uint32_t L = dflt ? nd.dlit_len : (uint32_t)w;
                    bad = L != nd.lit_len;
                    for (uint32_t x = 0; !bad && x < L; x++)
                        bad = (dflt ? P.lits[nd.dlit + x] : r(pay + x)) != P.lits[nd.lit + x];
                } else {
                    bad = true;
                }
            }
        }
    }
    if (bad) return kFlatFallback;
    if (VAL) return 0;   // a blob DecodeBuffer accepts, ValidateBuffer accepts
    // pass 2: the fields
    hj = h0;
    for (int j = 0; j < F; j++) {
        const uint32_t hn = r.u16(a0 + 2 * (j + 1));
        const DecNode nd = P.nodes[P.kids[root.kid0 + j]];
        const int64_t o = j == 0 ? base : (int64_t)(hj >> 3) + base;
        const int64_t w = (int64_t)(hn >> 3) + base - o;
        hj = hn;
        const uint64_t pay = a0 + (uint64_t)o;
        switch (nd.kind) {
            case K_INT: case K_UINT: case K_FLOAT: case K_BOOL: {
                if (w == 0) {
                    if (cols.valid[nd.col]) cols.valid[nd.col][i] = 0;
                    break;
                }
                uint8_t* dstp = cols.data[nd.col] + i * (uint64_t)nd.width;
                if (nd.kind == K_BOOL) dstp[0] = r(pay) != 0;
                else copy_out(dstp, r, pay, (uint32_t)nd.width);
                if (cols.valid[nd.col]) cols.valid[nd.col][i] = 1;
                break;
            }
            case K_STRING: case K_BYTES:
                if (nd.width > 0) {
                    copy_out(cols.data[nd.col] + i * (uint64_t)nd.width, r, pay, (uint32_t)nd.width);
                } else {
                    const bool dflt = w == 0 && (nd.check & CHK_DEFAULT) && nd.dlit_len > 0;
                    cols.start[nd.col][i] = dflt ? PACKOS_VIEW_DEFAULT : w == 0 ? 0ull : pay;
                    cols.length[nd.col][i] = dflt ? nd.dlit_len : (uint32_t)w;
                }
                break;
            default: break;
        }
    }
    return 0;
}

// Flat chains of plain leaves (no value checks / literals / defaults, plain
// modes): the canonical fast path with each field's descriptor packed into
// one word and its output pointers resolved on the host, all passed by value:
// every per-field value is a uniform kernel-argument (scalar) load, so the
// field loop is scalar control around a few vector ops per blob instead of a
// node-table walk.  Pass 1 validates exactly what decode_flat does (tags,
// monotone offsets, fixed widths / nil nullables, End = len); pass 2 re-reads
// the header words (LDS) and writes each field with one store of its width.
// A blob that is not canonical returns kFlatFallback.
constexpr int kFlatMax = 16;
struct FlatArg {
    int32_t F;                 // 0: not eligible (decode_flat / decode_blob decide)
    uint32_t fd[kFlatMax];     // kind | width << 4 | tag << 20 | nullable << 23
    uint64_t p0[kFlatMax];     // fixed: row base (n x width); var: view starts
    uint64_t p1[kFlatMax];     // nullable fixed: validity; var: view lengths
};
__device__ __forceinline__ int fd_kind(uint32_t d) { return (int)(d & 15u); }
__device__ __forceinline__ int fd_width(uint32_t d) { return (int)(int16_t)((d >> 4) & 0xFFFFu); }   // <= 0: var
__device__ __forceinline__ int fd_tag(uint32_t d) { return (int)((d >> 20) & 7u); }
__device__ __forceinline__ bool fd_null(uint32_t d) { return (d >> 23) & 1u; }

// column stores of the flat decode path: non-temporal (write-once output
// columns; C3 decode 0.041 -> 0.036 ms, C5 0.291 -> 0.284 ms, A/B on the box;
// PACKOS_DEC_PLAIN: plain stores)
#ifdef PACKOS_DEC_PLAIN
#define DST(p, ...) (*(p) = (__VA_ARGS__))
#else
#define DST(p, ...) __builtin_nontemporal_store((__VA_ARGS__), (p))
#endif
template <class R, bool VAL = false>
__device__ __forceinline__ uint32_t decode_flat_k(const FlatArg& A, const R& r, uint64_t a0, uint64_t a1, uint64_t i) {
    const int F = A.F;
    const int64_t len = (int64_t)(a1 - a0);
    if (len < 2 * (F + 1)) return kFlatFallback;
    const uint32_t h0 = r.u16(a0);
    const int64_t base = h0 >> 3;
    bool bad = base != 2 * (F + 1);
    int64_t o = base;
    uint32_t hj = h0;
    for (int j = 0; j < F; j++) {
        const uint32_t d = A.fd[j];
        const uint32_t hn = r.u16(a0 + 2 * (j + 1));
        const int64_t nx = (int64_t)(hn >> 3) + base;
        const int64_t w = nx - o;
        const int k = fd_kind(d), fw = fd_width(d);
        bad |= (int)(hj & 7u) != fd_tag(d) || nx < o;
        if (k == K_STRING || k == K_BYTES) bad |= fw > 0 && w != fw;
        else bad |= w != fw && !(fd_null(d) && w == 0);
        o = nx;
        hj = hn;   // after the last field: the End header
    }
    // the End header: tag 0 and End offset == len
    bad |= (hj & 7u) != 0 || o != len;
    if (bad) return kFlatFallback;
    if (VAL) return 0;
    o = base;
    for (int j = 0; j < F; j++) {
        const uint32_t d = A.fd[j];
        const int64_t nx = (int64_t)(r.u16(a0 + 2 * (j + 1)) >> 3) + base;
        const uint64_t pay = a0 + (uint64_t)o;
        const uint32_t w = (uint32_t)(nx - o);
        o = nx;
        const int k = fd_kind(d), fw = fd_width(d);
        // global (not flat) stores: the pointers are device memory
        typedef __attribute__((address_space(1))) uint8_t g8;
        typedef __attribute__((address_space(1))) uint16_t g16;
        typedef __attribute__((address_space(1))) uint32_t g32;
        typedef __attribute__((address_space(1))) uint64_t g64;
        if ((k == K_STRING || k == K_BYTES) && fw <= 0) {
            DST(((g64*)A.p0[j]) + i, w == 0 ? 0ull : pay);
            DST(((g32*)A.p1[j]) + i, w);
            continue;
        }
        if (fd_null(d) && A.p1[j]) DST(((g8*)A.p1[j]) + i, (uint8_t)(w != 0));
        if (w == 0) continue;
        g8* dp = (g8*)A.p0[j] + i * (uint64_t)fw;
        if (fw == 1) *dp = k == K_BOOL ? (uint8_t)(r(pay) != 0) : (uint8_t)r(pay);
        else if (fw == 2) DST((g16*)dp, (uint16_t)r.u16(pay));
        else if (fw == 4) DST((g32*)dp, r.u32(pay));
        else if (fw == 8) DST((g64*)dp, (uint64_t)r.u32(pay) | ((uint64_t)r.u32(pay + 4) << 32));
        else if (fw == 16 && ((uintptr_t)dp & 15) == 0)   // one 16-B store (lanes 16 B apart: whole lines)
            DST((__attribute__((address_space(1))) u32x4*)dp, u32x4{r.u32(pay), r.u32(pay + 4), r.u32(pay + 8), r.u32(pay + 12)});
        else if ((fw & 3) == 0)
            for (int x = 0; x < fw; x += 4) *(g32*)(dp + x) = r.u32(pay + x);
        else
            for (int x = 0; x < fw; x++) dp[x] = (uint8_t)r(pay + x);
    }
    return 0;
}

// Generic decode with a per-blob LDS window: every thread first fetches its
// blob's first kDecWinChunks x 16 bytes (header block, leading fields) with
// 16-B loads, all in flight, then runs decode_blob reading the window and
// falling back to HBM only beyond it.  Replaces ~one dependent global byte
// load per header word / payload byte with one load round.
constexpr int kDecWinChunks = 8;
#ifndef PACKOS_DECWIN_ATTR
// 6 waves per SIMD (<= 80 VGPRs; the 24-KB window's LDS admits 6 workgroups):
// C3 decode 0.0426 -> 0.0412 ms, C5 unchanged (A/B on the box).  The 32-KB
// window instantiations cannot reach it and keep their allocation.
#define PACKOS_DECWIN_ATTR __attribute__((amdgpu_waves_per_eu(6, 8)))
#endif
#ifndef PACKOS_DECFIX_ATTR
#define PACKOS_DECFIX_ATTR
#endif

// WC: window chunks per blob — enough for the schema's static prefix (bytes
// before the first var payload; compile.cpp), at most kDecWinChunks.
// VAL: ValidateBuffer — status only (decode_blob<..., VAL>), P.win = the
// bytes validation reads before the first var payload.
template <int WC, bool EXT, bool VAL = false>
__global__ __launch_bounds__(kBlock) PACKOS_DECWIN_ATTR void k_decode_win(DecProgram P, DecCols cols, FlatArg FA,
                                                       const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ offs, uint64_t stride, uint64_t n,
                                                       uint32_t* __restrict__ status) {
    // sized by WC: the per-blob windows need kBlock * WC chunks, and a tile
    // staged whole must fit the same bytes (LDS per workgroup sets occupancy)
    __shared__ __attribute__((aligned(16))) uint8_t win[kBlock * WC * 16];
    extern __shared__ __attribute__((aligned(16))) uint8_t ptab[];   // decode program copy (nodes | kids | lits)
    const int tid = threadIdx.x;
    // the program is read once per visited field: keep it in LDS
    DecNode* lnodes = (DecNode*)ptab;
    int32_t* lkids = (int32_t*)(ptab + ((P.n_nodes * sizeof(DecNode) + 15) & ~15));
    uint8_t* llits = (uint8_t*)lkids + ((P.n_kids * 4 + 15) & ~15);
    const uint64_t lo = (uint64_t)blockIdx.x * kBlock, i = lo + tid;
    const uint32_t rows = (uint32_t)min((uint64_t)kBlock, n - lo);
    // the tile's byte range (two scalar loads, one round trip)
    typedef __attribute__((address_space(4))) const uint64_t c_u64;
    uint64_t t0 = lo * stride, t1 = (lo + rows) * stride;
    if (offs) {
        t0 = ((c_u64*)(uintptr_t)offs)[lo];
        t1 = ((c_u64*)(uintptr_t)offs)[lo + rows];
    }
    // the program tables and this blob's offsets: one round of loads (a
    // load -> LDS loop per table would wait once per table before the DMA)
    const uint32_t nnw = (uint32_t)P.n_nodes * (uint32_t)(sizeof(DecNode) / 4);
    const uint32_t* gnodes = (const uint32_t*)P.nodes;
    uint32_t pn0 = 0, pn1 = 0, pk = 0;
    uint8_t pl = 0;
    if ((uint32_t)tid < nnw) pn0 = gnodes[tid];
    if ((uint32_t)tid + kBlock < nnw) pn1 = gnodes[tid + kBlock];
    if (tid < P.n_kids) pk = P.kids[tid];
    if (tid < P.n_lits) pl = P.lits[tid];
    uint64_t a0 = i * stride, a1 = (i + 1) * stride;
    if (i >= n) a0 = a1 = 0;
    else if (offs) {   // both in one block: a wait between them otherwise
        a0 = offs[i];
        a1 = offs[i + 1];
    }
    // Small blobs: when the tile's whole byte range fits the window memory,
    // stage it once with coalesced LDS-DMA and let every blob read from there
    // (same reader, one shared window).  Otherwise each blob's first
    // kDecWinChunks * 16 bytes go to its own window (headers + fixed fields sit
    // at the front; var values are returned as views and never read).
    const uint64_t tb = t0 & ~15ull;
    const bool tile_mode = t1 >= t0 && t1 - tb <= (uint64_t)sizeof(win) && ((uintptr_t)arena & 15) == 0;
    uint8_t* w;
    uint64_t b0;
    uint32_t wbytes;
    auto store_program = [&]() {
        uint32_t* lnw = (uint32_t*)lnodes;
        if ((uint32_t)tid < nnw) lnw[tid] = pn0;
        if ((uint32_t)tid + kBlock < nnw) lnw[tid + kBlock] = pn1;
        for (uint32_t x = tid + 2 * kBlock; x < nnw; x += kBlock) lnw[x] = gnodes[x];
        if (tid < P.n_kids) lkids[tid] = pk;
        for (int x = tid + kBlock; x < P.n_kids; x += kBlock) lkids[x] = P.kids[x];
        if (tid < P.n_lits) llits[tid] = pl;
        for (int x = tid + kBlock; x < P.n_lits; x += kBlock) llits[x] = P.lits[x];
    };
    if (tile_mode) {
        const uint32_t nch = (uint32_t)((t1 - tb + 15) >> 4), lane = tid & 63, c00 = tid & ~63u;
        const uint32_t lds0 = (uint32_t)(uintptr_t)win;
        for (uint32_t c0 = c00; c0 < nch; c0 += kBlock)
            if (c0 + lane < nch) dma16(arena + tb + 16u * (c0 + lane), __builtin_amdgcn_readfirstlane(lds0 + 16u * c0));
        store_program();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        w = win;
        b0 = tb;
        wbytes = 16 * nch;
    } else {
        // dword k of thread t's window at win32[k * kBlock + t]
        w = win + 4 * tid;
        b0 = a0 & ~15ull;
        // only the bytes the decoder reads: the static prefix when nothing but
        // var payloads (returned as views) follows it
        const uint64_t end = min(a1, P.win > 0 ? min(a0 + (uint64_t)P.win, b0 + 16ull * WC) : b0 + 16ull * WC);
        const uint32_t nch = (i < n && end > a0) ? (uint32_t)((end - b0 + 15) >> 4) : 0u;
        u32x4 v[WC];
#pragma unroll
        for (int c = 0; c < WC; c++)
            if ((uint32_t)c < nch) v[c] = *(const g_u32x4*)(arena + b0 + 16 * c);
        store_program();
        uint32_t* w32 = (uint32_t*)w;
#pragma unroll
        for (int c = 0; c < WC; c++)
            if ((uint32_t)c < nch) {
                w32[(4 * c + 0) * kBlock] = v[c].x;
                w32[(4 * c + 1) * kBlock] = v[c].y;
                w32[(4 * c + 2) * kBlock] = v[c].z;
                w32[(4 * c + 3) * kBlock] = v[c].w;
            }
        wbytes = 16 * nch;
    }
    __syncthreads();
    if (i >= n) return;
    const WReader R{arena, (const uint32_t*)w, b0, wbytes, tile_mode ? 1u : (uint32_t)kBlock};
    const DecProgram LP{lnodes, lkids, llits, P.root, P.n_nodes, P.n_kids, P.n_lits, P.flat, P.ext, P.win};
    uint32_t sv = kFlatFallback;
    if (FA.F) {
        // the flat path reads only the header block and fixed payloads: inside
        // the window when the tile holds the whole blob, or (per-blob windows)
        // when no fixed payload follows a var one (P.win > 0: the window is the
        // static prefix, which pass 1 confines every fixed payload to)
        // (and only when that prefix, from the blob's offset in its first
        // chunk, fits the WC chunks: a longer prefix was cut at b0 + 16 * WC)
        const bool inside = tile_mode ? (a0 >= b0 && a1 <= b0 + wbytes && a1 >= a0)
                                      : P.win > 0 && (a0 - b0) + (uint64_t)P.win <= 16ull * WC;
        if (inside) sv = decode_flat_k<LReader, VAL>(FA, LReader{(const uint32_t*)w, b0, tile_mode ? 1u : (uint32_t)kBlock}, a0, a1, i);
        else sv = decode_flat_k<WReader, VAL>(FA, R, a0, a1, i);
    } else if (P.flat) {
        sv = decode_flat<WReader, VAL>(LP, cols, R, a0, a1, i);
    }
    if (sv == kFlatFallback) sv = decode_blob<WReader, EXT, VAL>(LP, cols, R, a0, a1, i);
#ifdef PACKOS_DEC_STNT
    __builtin_nontemporal_store(sv, status + i);
#else
    status[i] = sv;
#endif
}

// Fixed-layout decode (the transpose of k_encode_fixed_dw).  A workgroup
// takes a tile of T consecutive blobs, which must lie back to back in the
// arena (size B each, 16-B aligned start; otherwise the whole tile goes to
// decode_blob):
//   1. stage the tile's T*B bytes in LDS with 16-B loads;
//   2. compare every blob dword's constant bytes (header words, literals,
//      map keys) with the canonical layout -> per-blob fail flag;
//   3. write every fixed column's T rows as 16-B output units gathered from
//      the staged blobs (funnel-shifted dword reads; bools normalised);
//   4. mark validity, then run decode_blob for the (rare) blobs that failed
//      the check, overwriting their rows with the exact reference behaviour.
// The fixed columns with their output pointers resolved, built on the host
// per call and passed as a kernel argument: the column walk reads it with a
// uniform index (scalar loads), so no dependent table load sits in front of
// the first barrier.
constexpr int kDecK = 24;
constexpr int64_t kDecTileBytes = 16384, kDecTileBytesLarge = 24576;   // staged blob bytes per decode tile
// Full tiles write their columns as a list of wave steps built on the host
// (the same for every full tile of a call): a step is one 1-KiB block of one
// column's tile bytes; its word packs column | block << 5 | (dwords - 1) << 13
// | kind << 24.  Unit kinds take a block as 64 16-B units, one per lane, and
// one 16-B store: DS_W16 (w % 16 == 0: the unit inside one row at a uniform
// offset mod 16, two ds_read_b128 + a scalar-chosen shift), DS_G4U / DS_GENU
// (other w > 4: four dwords inside a row, or across two), DS_W8 .. DS_BOOLU
// (16 / w rows per unit).  Dword kinds take it as 4 x 64 dwords, lane l taking
// dwords l, l + 64, ... (consecutive lanes read consecutive LDS dwords: no
// bank conflicts), one 256-B wave store each.  Measured (A/B on the box):
// 256-B blobs (M, C4) decode faster with unit steps (M 0.102 -> 0.093 ms, C4
// 0.37 -> 0.33 ms against the per-column loops), 64-B blobs (C2) with dword
// steps (0.0299 -> 0.0282 ms; unit steps 0.0336).
constexpr int kDecSteps = 96;
enum : uint32_t {
    DS_W16 = 0, DS_G4U = 1, DS_GENU = 2, DS_W8 = 3, DS_W4 = 4, DS_W2 = 5, DS_W1 = 6, DS_BOOLU = 7,   // 16-B units
    DS_D4 = 8, DS_D2 = 9, DS_D1 = 10, DS_BOOL = 11, DS_GEN = 12, DS_BYTE = 13                         // dwords
};
struct DecColsK {
    uint8_t* dst[kDecK];
    uint32_t width[kDecK], blob_off[kDecK], flags[kDecK], magic[kDecK];
    int32_t n;
    int32_t nsteps;              // 0: the per-column loops for every tile
    uint32_t step[kDecSteps];
};

__device__ __forceinline__ uint32_t lds_u8(const uint32_t* lds, uint32_t a) { return (lds[a >> 2] >> (8 * (a & 3))) & 0xFFu; }

// 16 bytes at LDS byte q; m = q & 15 wave-uniform: two ds_read_b128 and a
// byte shift chosen by a scalar branch
__device__ __forceinline__ u32x4 lds16u(const uint8_t* lds, uint32_t q, uint32_t m) {
    const uint32_t qa = q - m;
    const u32x4 x0 = *(const u32x4*)(lds + qa);
    if (m == 0) return x0;
    const u32x4 x1 = *(const u32x4*)(lds + qa + 16);
    const uint32_t sh = m & 3u;
#define AB(h, l) __builtin_amdgcn_alignbyte(h, l, sh)
    switch (m >> 2) {
        case 0: return u32x4{AB(x0.y, x0.x), AB(x0.z, x0.y), AB(x0.w, x0.z), AB(x1.x, x0.w)};
        case 1: return u32x4{AB(x0.z, x0.y), AB(x0.w, x0.z), AB(x1.x, x0.w), AB(x1.y, x1.x)};
        case 2: return u32x4{AB(x0.w, x0.z), AB(x1.x, x0.w), AB(x1.y, x1.x), AB(x1.z, x1.y)};
        default: return u32x4{AB(x1.x, x0.w), AB(x1.y, x1.x), AB(x1.z, x1.y), AB(x1.w, x1.z)};
    }
#undef AB
}

// Staged-row reads of the fixed decoder.  SB % 4 == 0 (fixed fast path): every
// row's value sits at the same offset mod 4 (q), uniform per column.
__device__ __forceinline__ uint32_t lds_w4(const uint32_t* lds, uint32_t a, uint32_t q) {
    return q ? __builtin_amdgcn_alignbyte(lds[(a >> 2) + 1], lds[a >> 2], q) : lds[a >> 2];
}
// dword d (tile column bytes 4d .. 4d + 3) of a column; KIND: a compile-time
// kind, or DS_ANY to switch on `kind`
constexpr uint32_t DS_ANY = 255;
template <uint32_t KIND = DS_ANY>
__device__ __forceinline__ uint32_t dfix_dword(const uint32_t* lds, uint32_t kind, uint32_t d, uint32_t w, uint32_t off,
                                               uint32_t magic, uint32_t SB) {
    const uint32_t b = 4 * d, q = off & 3u;
    if (KIND != DS_ANY) kind = KIND;
    switch (kind) {
        case DS_D4: {    // w % 4 == 0: inside one row
            const uint32_t j = __umulhi(b, magic);
            return lds_w4(lds, j * SB + off + (b - j * w), q);
        }
        case DS_D2: {    // rows 2d, 2d + 1
            const uint32_t a = 2 * d * SB + off;
            return (lds_w4(lds, a, q) & 0xFFFFu) | (lds_w4(lds, a + SB, q) << 16);
        }
        case DS_D1: case DS_BOOL: {   // rows 4d .. 4d + 3
            uint32_t v = 0;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const uint32_t a = (4 * d + y) * SB + off;
                uint32_t c = (lds[a >> 2] >> (8 * (a & 3u))) & 0xFFu;
                if (kind == DS_BOOL) c = c != 0;
                v |= c << (8 * y);
            }
            return v;
        }
        case DS_GEN: {   // w > 4: inside one row, or (a few) across two
            const uint32_t j = __umulhi(b, magic), r = b - j * w;
            uint32_t x = lds_bytes4(lds, j * SB + off + r);
            if (r + 4 > w) {
                const uint32_t m = 8 * (w - r);
                x = (x & ((1u << m) - 1u)) | (lds_bytes4(lds, (j + 1) * SB + off) << m);
            }
            return x;
        }
        default: {       // any width, byte by byte
            uint32_t v = 0;
            for (int y = 0; y < 4; y++) {
                const uint32_t bb = b + y, j = w > 1 ? __umulhi(bb, magic) : bb;
                const uint32_t a = j * SB + off + (bb - j * w);
                v |= ((lds[a >> 2] >> (8 * (a & 3u))) & 0xFFu) << (8 * y);
            }
            return v;
        }
    }
}
// unit u (tile column bytes 16u .. 16u + 15) of a unit step (not DS_W16)
__device__ __forceinline__ u32x4 dfix_unit(const uint32_t* lds, uint32_t kind, uint32_t u, uint32_t w, uint32_t off,
                                           uint32_t magic, uint32_t SB) {
    const uint32_t q = off & 3u;
    switch (kind) {
        case DS_G4U:     // four dwords of the column
            return u32x4{dfix_dword<DS_D4>(lds, 0, 4 * u, w, off, magic, SB), dfix_dword<DS_D4>(lds, 0, 4 * u + 1, w, off, magic, SB),
                         dfix_dword<DS_D4>(lds, 0, 4 * u + 2, w, off, magic, SB), dfix_dword<DS_D4>(lds, 0, 4 * u + 3, w, off, magic, SB)};
        case DS_GENU:
            return u32x4{dfix_dword<DS_GEN>(lds, 0, 4 * u, w, off, magic, SB), dfix_dword<DS_GEN>(lds, 0, 4 * u + 1, w, off, magic, SB),
                         dfix_dword<DS_GEN>(lds, 0, 4 * u + 2, w, off, magic, SB), dfix_dword<DS_GEN>(lds, 0, 4 * u + 3, w, off, magic, SB)};
        case DS_W8: {    // rows 2u, 2u + 1
            const uint32_t a0 = 2 * u * SB + off, a1 = a0 + SB;
            return u32x4{lds_w4(lds, a0, q), lds_w4(lds, a0 + 4, q), lds_w4(lds, a1, q), lds_w4(lds, a1 + 4, q)};
        }
        case DS_W4: {    // rows 4u .. 4u + 3
            const uint32_t a0 = 4 * u * SB + off;
            return u32x4{lds_w4(lds, a0, q), lds_w4(lds, a0 + SB, q), lds_w4(lds, a0 + 2 * SB, q),
                         lds_w4(lds, a0 + 3 * SB, q)};
        }
        case DS_W2:      // rows 8u .. 8u + 7
            return u32x4{dfix_dword<DS_D2>(lds, 0, 4 * u, w, off, magic, SB), dfix_dword<DS_D2>(lds, 0, 4 * u + 1, w, off, magic, SB),
                         dfix_dword<DS_D2>(lds, 0, 4 * u + 2, w, off, magic, SB), dfix_dword<DS_D2>(lds, 0, 4 * u + 3, w, off, magic, SB)};
        case DS_BOOLU:   // rows 16u .. 16u + 15
            return u32x4{dfix_dword<DS_BOOL>(lds, 0, 4 * u, w, off, magic, SB), dfix_dword<DS_BOOL>(lds, 0, 4 * u + 1, w, off, magic, SB),
                         dfix_dword<DS_BOOL>(lds, 0, 4 * u + 2, w, off, magic, SB), dfix_dword<DS_BOOL>(lds, 0, 4 * u + 3, w, off, magic, SB)};
        default:         // DS_W1
            return u32x4{dfix_dword<DS_D1>(lds, 0, 4 * u, w, off, magic, SB), dfix_dword<DS_D1>(lds, 0, 4 * u + 1, w, off, magic, SB),
                         dfix_dword<DS_D1>(lds, 0, 4 * u + 2, w, off, magic, SB), dfix_dword<DS_D1>(lds, 0, 4 * u + 3, w, off, magic, SB)};
    }
}

// Steps 3-4 of a staged tile (column stores, validity) by NCT threads, this
// one being thread ct; the tile's rows start at lds_raw.  A full tile (rows
// == T) runs the host-built step list; the ragged last tile walks the
// columns.  Then, after a barrier, dfix_status: every row's constant-byte and
// value checks and its status, failed rows through decode_blob.
template <int NCT>
__device__ __forceinline__ void dfix_tile(const DecFixProgram& F, const DecCols& cols, const DecColsK& K,
                                          const uint8_t* lds_raw, uint64_t blob0, uint32_t rows, uint32_t ct) {
    const uint32_t* lds = (const uint32_t*)lds_raw;
    const uint32_t B = (uint32_t)F.B, SB = B;
    typedef __attribute__((address_space(1))) u32x4 g_v4;
    if (K.nsteps && rows == (uint32_t)F.T) {
        // wave-uniform steps: wave w takes steps w, w + NCT / 64, ...
        const uint32_t wave = __builtin_amdgcn_readfirstlane(ct >> 6), lane = ct & 63u;
        for (uint32_t si = wave; si < (uint32_t)K.nsteps; si += NCT / kWave) {
            const uint32_t sd = K.step[si];
            const uint32_t c = sd & 31u, blk = (sd >> 5) & 0xFFu, nd = ((sd >> 13) & 0x1FFu) + 1u, kind = sd >> 24;
            const uint32_t w = K.width[c], off = K.blob_off[c], magic = K.magic[c];
            uint8_t* dst = K.dst[c] + blob0 * w + 1024u * blk;
            if (kind == DS_W16) {   // w % 16 == 0, SB % 16 == 0: a unit inside one row, offset mod 16 uniform
                if (4 * lane < nd) {
                    const uint32_t bb = 1024u * blk + 16u * lane, j = __umulhi(bb, magic);
                    __builtin_nontemporal_store(lds16u(lds_raw, j * SB + off + (bb - j * w), off & 15u),
                                                (g_v4*)dst + lane);
                }
            } else if (kind < DS_D4) {
                if (4 * lane < nd)
                    __builtin_nontemporal_store(dfix_unit(lds, kind, 64u * blk + lane, w, off, magic, SB),
                                                (g_v4*)dst + lane);
            } else {
                // the step's kind is wave-uniform: one branch per step, then four
                // dwords of a compile-time kind (no switch per dword)
                auto dwords = [&](auto kc) {
                    constexpr uint32_t KC = decltype(kc)::value;
#pragma unroll
                    for (uint32_t k = 0; k < 4; k++) {
                        const uint32_t dl = lane + 64u * k;
                        if (dl < nd)
                            __builtin_nontemporal_store(dfix_dword<KC>(lds, kind, 256u * blk + dl, w, off, magic, SB),
                                                        (uint32_t*)dst + dl);
                    }
                };
                switch (kind) {
                    case DS_D4: dwords(std::integral_constant<uint32_t, DS_D4>{}); break;
                    case DS_D2: dwords(std::integral_constant<uint32_t, DS_D2>{}); break;
                    case DS_D1: dwords(std::integral_constant<uint32_t, DS_D1>{}); break;
                    case DS_BOOL: dwords(std::integral_constant<uint32_t, DS_BOOL>{}); break;
                    case DS_GEN: dwords(std::integral_constant<uint32_t, DS_GEN>{}); break;
                    default: dwords(std::integral_constant<uint32_t, DS_ANY>{}); break;
                }
            }
        }
    } else {
        // 3. columns: uniform walk over the columns; threads stride the column's
        //    output dwords (consecutive lanes -> consecutive dwords: 256-B stores)
        for (int c = 0; c < K.n; c++) {
            struct { uint8_t* dst; uint32_t blob_off, flags, magic; } L = {K.dst[c], K.blob_off[c], K.flags[c], K.magic[c]};
            const uint32_t w = K.width[c], R = rows * w, D = R >> 2;
            uint32_t* dst = (uint32_t*)(L.dst + blob0 * w);   // 4-B aligned: T*w % 4 == 0, base 16-B aligned
            if ((w & 3) == 0) {
                for (uint32_t d = ct; d < D; d += NCT) {
                    const uint32_t b = 4 * d;
                    const uint32_t j = __umulhi(b, L.magic);
                    const uint32_t a = j * SB + L.blob_off + (b - j * w);
                    __builtin_nontemporal_store(lds_bytes4(lds, a), dst + d);
                }
            } else if (w == 2) {   // a dword = rows 2d, 2d+1
                for (uint32_t d = ct; d < D; d += NCT) {
                    const uint32_t a = 2 * d * SB + L.blob_off;
                    const uint32_t x = (lds_bytes4(lds, a) & 0xFFFFu) | (lds_bytes4(lds, a + SB) << 16);
                    __builtin_nontemporal_store(x, dst + d);
                }
            } else if (w > 4 && !(L.flags & 1u)) {   // most dwords sit inside one row
                for (uint32_t d = ct; d < D; d += NCT) {
                    const uint32_t b = 4 * d;
                    const uint32_t j = __umulhi(b, L.magic);
                    const uint32_t r = b - j * w;
                    uint32_t x;
                    if (r + 4 <= w) {
                        x = lds_bytes4(lds, j * SB + L.blob_off + r);
                    } else {
                        const uint32_t k = w - r;   // 1..3 bytes of row j, then row j + 1
                        x = (lds_bytes4(lds, j * SB + L.blob_off + r) & ((1u << (8 * k)) - 1u)) |
                            (lds_bytes4(lds, (j + 1) * SB + L.blob_off) << (8 * k));
                    }
                    __builtin_nontemporal_store(x, dst + d);
                }
            } else {
                for (uint32_t d = ct; d < D; d += NCT) {
                    uint32_t x = 0;
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const uint32_t b = 4 * d + y;
                        const uint32_t j = w > 1 ? __umulhi(b, L.magic) : b;
                        uint32_t v = lds_u8(lds, j * SB + L.blob_off + (b - j * w));
                        if (L.flags & 1u) v = v != 0;
                        x |= v << (8 * y);
                    }
                    __builtin_nontemporal_store(x, dst + d);
                }
            }
            // ragged tail (R % 4 bytes, last tile only)
            for (uint32_t b = 4 * D + ct; b < R; b += NCT) {
                const uint32_t j = w > 1 ? __umulhi(b, L.magic) : b;
                uint32_t v = lds_u8(lds, j * SB + L.blob_off + (b - j * w));
                if (L.flags & 1u) v = v != 0;
                L.dst[blob0 * w + b] = (uint8_t)v;
            }
        }
    }
    // 4. validity (every node is present in the canonical layout)
    for (int c = 0; c < F.n_all_cols; c++)
        if (cols.valid[c])
            for (uint32_t j = ct; j < rows; j += NCT) cols.valid[c][blob0 + j] = 1;
}

// Every row of the tile: its constant-byte check (the blob dwords that hold
// header words / literals: 5 of 64 for metric M; list built at compile) and
// the value checks of its fixed leaves (Range, Prefix / Suffix of fixed
// strings) against the staged row; a row failing either takes the exact
// per-blob path (decode_blob, which reports it), after the column stores.
template <bool EXT, int NCT, bool VAL = false>
__device__ __forceinline__ void dfix_status(const DecFixProgram& F, const DecProgram& P, const DecCols& cols,
                                            const uint8_t* lds_raw, const uint32_t* chk, const uint8_t* arena,
                                            const uint64_t* offs, uint32_t* status, uint64_t blob0, uint32_t rows,
                                            uint32_t ct) {
    const uint32_t* lds = (const uint32_t*)lds_raw;
    const uint32_t B = (uint32_t)F.B, SB = B;
    const uint32_t nq = (uint32_t)F.n_chk;
    for (uint32_t j = ct; j < rows; j += NCT) {
        bool bad = false;
        for (uint32_t e = 0; e < nq; e++) {
            const uint32_t* c = chk + 3 * e;
            const uint32_t a = j * SB + 4 * c[0];   // blob dword q (B % 4 == 0: aligned)
            bad |= (((B & 3) == 0 ? lds[a >> 2] : lds_bytes4(lds, a)) & c[1]) != c[2];
        }
        for (int e = 0; e < F.n_vchk && !bad; e++) {
            const DecChk c = F.vchk[e];
            const uint32_t a = j * SB + c.blob_off;
            if (c.flags & CHK_RANGE) {
                uint64_t u = 0;
                for (uint32_t b = 0; b < c.width; b++) u |= (uint64_t)lds_u8(lds, a + b) << (8 * b);
                const int sh = 64 - 8 * (int)c.width;
                const int64_t v = (int64_t)(u << sh) >> sh;
                bad = ((c.flags & CHK_MIN) && v < c.rmin) || ((c.flags & CHK_MAX) && v > c.rmax);
            } else {
                bad = c.lit_len > c.width;
                const uint32_t at = (c.flags & CHK_PREFIX) ? 0u : c.width - c.lit_len;
                for (uint32_t b = 0; !bad && b < c.lit_len; b++) bad = lds_u8(lds, a + at + b) != P.lits[c.lit + b];
            }
        }
        const uint64_t i = blob0 + j;
        uint32_t sv = 0;
        if (bad)
            sv = decode_blob<GReader, EXT, VAL>(P, cols, GReader{arena}, offs ? offs[i] : i * B,
                                                offs ? offs[i + 1] : (i + 1) * B, i);
        status[i] = sv;
    }
}

// VAL: ValidateBuffer over the staged tile — the row checks and status only
// (a row the canonical checks accept is one DecodeBuffer, hence
// ValidateBuffer, accepts; the others run decode_blob<VAL>)
template <bool EXT, bool VAL = false>
__device__ __forceinline__ void dfix_oneshot(const DecFixProgram& F, const DecProgram& P, const DecCols& cols,
                                             const DecColsK& K, const uint8_t* __restrict__ arena,
                                             const uint64_t* __restrict__ offs, uint64_t n,
                                             uint32_t* __restrict__ status, uint64_t tile0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    uint32_t* lds = (uint32_t*)lds_raw;
    const uint32_t B = (uint32_t)F.B, T = (uint32_t)F.T;
    // staged row stride (rows padded to B + 16 measured slower: M decode 0.0997
    // -> 0.112 ms with 2.6x fewer bank-conflict cycles; round-4 A/B)
    const uint32_t SB = B;
    const uint64_t blob0 = (tile0 + blockIdx.x) * T;
    const uint32_t rows = (uint32_t)min((uint64_t)T, n - blob0);
    const int tid = threadIdx.x;
    uint32_t* chk = lds + (T * SB / 4 + 4);

    // the tile base is one scalar load; whether the tile's blobs really lie
    // back to back at stride B is checked while the staging DMA is in flight
    typedef __attribute__((address_space(4))) const uint64_t c_u64;
    // the tile's start and end offsets: two scalar loads in one round trip,
    // the only memory latency in front of the staging DMA (the check table's
    // copy to LDS queues behind the DMA)
    uint64_t base = blob0 * B, end = base + (uint64_t)rows * B;
    if (offs) {
        base = ((c_u64*)(uintptr_t)offs)[blob0];
        end = ((c_u64*)(uintptr_t)offs)[blob0 + rows];
    }
    const bool aligned_base = (base & 15) == 0;
    bool ok = true;
    // 1. stage: global -> LDS with global_load_lds_dwordx4 (every chunk of the
    //    tile in flight at once; a load -> ds_write loop waits per chunk)
    //    Staged bytes stop at the tile's end offset: a truncated or corrupt
    //    batch must not read past what its offsets cover (the tile then fails
    //    the contiguity check and takes the per-blob path below).
    uint32_t bytes = rows * B;
    if (offs) bytes = end <= base ? 0u : (uint32_t)min((uint64_t)bytes, end - base);
    if (aligned_base) {
        const uint8_t* src = arena + base;
        const uint32_t n16 = bytes >> 4, lane = tid & 63, c00 = tid & ~63u;
        const uint32_t lds0 = (uint32_t)(uintptr_t)lds_raw;
        for (uint32_t c0 = c00; c0 < n16; c0 += kBlock)
            if (c0 + lane < n16) dma16nt(src + 16u * (c0 + lane), __builtin_amdgcn_readfirstlane(lds0 + 16u * c0));
        for (uint32_t k = n16 * 16 + tid; k < bytes; k += kBlock) lds_raw[k] = src[k];
    }
    // the check table and the contiguity check's offsets: one round of loads,
    // queued behind the DMA (a load -> use loop per table would wait twice)
    const uint32_t nchk = 3u * (uint32_t)F.n_chk;
    {
        uint32_t cv = 0;
        uint64_t ov = 0;
        if ((uint32_t)tid < nchk) cv = F.chk[tid];
        if (offs && (uint32_t)tid <= rows) ov = offs[blob0 + tid];
        if ((uint32_t)tid < nchk) chk[tid] = cv;
        if (offs && (uint32_t)tid <= rows) ok &= ov == base + (uint64_t)tid * B;
    }
    for (uint32_t q = tid + kBlock; q < nchk; q += kBlock) chk[q] = F.chk[q];
    if (offs) {
        for (uint32_t j = tid + kBlock; j <= rows; j += kBlock) ok &= offs[blob0 + j] == base + (uint64_t)j * B;
        ok &= aligned_base;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!__syncthreads_and(ok)) {
        for (uint32_t j = tid; j < rows; j += kBlock) {
            const uint64_t i = blob0 + j;
            status[i] = decode_blob<GReader, EXT, VAL>(P, cols, GReader{arena}, offs ? offs[i] : i * B,
                                                       offs ? offs[i + 1] : (i + 1) * B, i);
        }
        return;
    }
    if (!VAL) {
        dfix_tile<kBlock>(F, cols, K, lds_raw, blob0, rows, (uint32_t)tid);
        __syncthreads();
    }
    dfix_status<EXT, kBlock, VAL>(F, P, cols, lds_raw, chk, arena, offs, status, blob0, rows, (uint32_t)tid);
}

template <bool EXT>
__global__ __launch_bounds__(kBlock) PACKOS_DECFIX_ATTR void k_decode_fixed(DecFixProgram F, DecProgram P, DecCols cols,
                                                                            DecColsK K, const uint8_t* __restrict__ arena,
                                                                            const uint64_t* __restrict__ offs, uint64_t n,
                                                                            uint32_t* __restrict__ status, uint64_t tile0) {
    dfix_oneshot<EXT>(F, P, cols, K, arena, offs, n, status, tile0);
}
// the same at 8 waves per SIMD (64 VGPRs), for blobs under 128 B: their
// 16-KB tiles leave LDS for 9 workgroups per CU, and the one-shot tile's
// fixed latency is what small blobs pay for (C2 decode 0.0315 -> 0.0298 ms;
// M and C4, held to 6 workgroups by their 24-KB tiles, do not gain)
template <bool EXT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_decode_fixed8(
    DecFixProgram F, DecProgram P, DecCols cols, DecColsK K, const uint8_t* __restrict__ arena,
    const uint64_t* __restrict__ offs, uint64_t n, uint32_t* __restrict__ status, uint64_t tile0) {
    dfix_oneshot<EXT>(F, P, cols, K, arena, offs, n, status, tile0);
}

// ValidateBuffer of fixed-layout batches whose checks read most of the blob
template <bool EXT>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_validate_fixed(
    DecFixProgram F, DecProgram P, DecCols cols, DecColsK K, const uint8_t* __restrict__ arena,
    const uint64_t* __restrict__ offs, uint64_t n, uint32_t* __restrict__ status, uint64_t tile0) {
    dfix_oneshot<EXT, true>(F, P, cols, K, arena, offs, n, status, tile0);
}

// =========================================================================
// GetAccess gather
// =========================================================================
struct DGet {
    uint64_t start;
    int64_t len, base, argc;
    int xw;   // ADR-001 extended container: u32 entries after a 4-byte lead
};
// Byte reader over one blob: its first kGetWin bytes sit in registers (one
// round of misaligned 16-B loads, whole loads inside the blob only), the rest
// is read from HBM.  The rangeAt walk of a top-level field then costs one
// memory round trip instead of three dependent rounds of byte loads.
constexpr uint32_t kGetWin = 32;
struct GWin {
    const uint8_t* a;
    uint64_t base;
    uint32_t n;
    uint32_t W[kGetWin / 4];
    __device__ __forceinline__ uint32_t byte(uint64_t p) const {
        const uint64_t d = p - base;
        if (d < n) {
            uint32_t w = 0;
#pragma unroll
            for (uint32_t k = 0; k < kGetWin / 4; k++) w = (uint32_t)(d >> 2) == k ? W[k] : w;
            return (w >> (8 * (d & 3))) & 0xFFu;
        }
        return a[p];
    }
    __device__ __forceinline__ uint32_t u16(uint64_t p) const { return byte(p) | (byte(p + 1) << 8); }
    __device__ __forceinline__ uint32_t u32(uint64_t p) const { return u16(p) | (u16(p + 2) << 16); }
};
__device__ __forceinline__ bool dget_init(DGet& g, const GWin& r, uint64_t start, int64_t len) {
    if (len < 2) return false;
    g.base = r.u16(start) >> 3;
    if (len < g.base) return false;
    g.start = start; g.len = len; g.argc = g.base / 2 - 1; g.xw = 0;
    return true;
}
// extended container (PACKOS_GET_EXTENDED): lead 02 00 | kind (top: 4; nested:
// 4 or 7) | u32 entries
__device__ __forceinline__ bool dget_init_ext(DGet& g, const GWin& r, uint64_t start, int64_t len, bool top) {
    if (len < 12 || r.u16(start) != kExtMarker) return false;
    const uint32_t kind = r.u16(start + 2);
    if (kind != PACKOS_TAG_TUPLE && (top || kind != PACKOS_TAG_MAP)) return false;
    g.base = r.u32(start + 4) >> 3;
    if (g.base < 12 || (g.base & 3) || len < g.base) return false;
    g.start = start; g.len = len; g.argc = (g.base - 4) / 4 - 1; g.xw = 1;
    return true;
}
// rangeAt (get.go:38-58)
__device__ __forceinline__ void dget_range(const DGet& g, const GWin& r, int64_t pos, int& tp, int64_t& s,
                                           int64_t& e) {
    if (pos >= g.argc) { tp = 0; s = -2; e = -1; return; }
    const uint32_t h1 = g.xw ? r.u32(g.start + 4 + pos * 4) : r.u16(g.start + pos * 2);
    const uint32_t h2 = g.xw ? r.u32(g.start + 4 + (pos + 1) * 4) : r.u16(g.start + (pos + 1) * 2);
    s = h1 >> 3; tp = h1 & 7;
    e = (h2 >> 3) + g.base;
    if (pos > 0) s += g.base;
    if (e > g.len) e = -1;
}

struct PathArg {
    int32_t p[16];
};

// One thread per blob: walk the nested path (GetNestedGetAccess, get.go:377-
// 401), then apply one Get* family (see packos_get_batch in packos.h) and
// optionally gather the typed value into a dense output row.  Every output
// is written exactly once, at the end (a value of <= 8 bytes as one store).
__device__ __forceinline__ uint64_t gwin_le(const GWin& r, uint64_t at, int64_t w) {
    const uint64_t d = at - r.base;
    if (d + 8 <= r.n) {   // inside the register window: funnel-shift three words
        const uint32_t k = (uint32_t)d >> 2, q = (uint32_t)d & 3u;
        uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
        for (uint32_t x = 0; x < kGetWin / 4; x++) {
            w0 = x == k ? r.W[x] : w0;
            w1 = x == k + 1 ? r.W[x] : w1;
            w2 = x == k + 2 ? r.W[x] : w2;
        }
        const uint32_t lo = q ? __builtin_amdgcn_alignbyte(w1, w0, q) : w0;
        const uint32_t hi = q ? __builtin_amdgcn_alignbyte(w2, w1, q) : w1;
        uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
        return w >= 8 ? v : v & ((1ull << (8 * w)) - 1);
    }
    uint64_t v = 0;
    for (int64_t k = 0; k < w && k < 8; k++) v |= (uint64_t)r.byte(at + k) << (8 * k);
    return v;
}

__global__ __launch_bounds__(kBlock) void k_get_field(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                                                      uint64_t stride, uint64_t n, PathArg path, int depth, int getter,
                                                      int want_tag, int want_width, uint8_t* __restrict__ out_values,
                                                      uint32_t value_width, uint64_t* __restrict__ out_start,
                                                      uint32_t* __restrict__ out_len, uint8_t* __restrict__ out_tag,
                                                      uint8_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // (one block with both loads merges them into a 16-B load per lane:
    // M GetInt 0.0279 -> 0.0283 ms, A/B; kept as two loads)
    const uint64_t a0 = offs ? offs[i] : i * stride;
    const uint64_t a1 = offs ? offs[i + 1] : (i + 1) * stride;
    GWin r;
    r.a = arena;
    r.base = a0;
    const uint64_t bl = a1 > a0 ? a1 - a0 : 0;
    r.n = bl >= 32 ? 32u : bl >= 16 ? 16u : 0u;
    {
        const u32x4 z = u32x4{0u, 0u, 0u, 0u};
#ifdef PACKOS_GET_NT
        const u32x4 w0 = r.n >= 16 ? __builtin_nontemporal_load((const g_u32x4*)(arena + a0)) : z;
        const u32x4 w1 = r.n >= 32 ? __builtin_nontemporal_load((const g_u32x4*)(arena + a0 + 16)) : z;
#else
        const u32x4 w0 = r.n >= 16 ? *(const g_u32x4*)(arena + a0) : z;
        const u32x4 w1 = r.n >= 32 ? *(const g_u32x4*)(arena + a0 + 16) : z;
#endif
        r.W[0] = w0.x; r.W[1] = w0.y; r.W[2] = w0.z; r.W[3] = w0.w;
        r.W[4] = w1.x; r.W[5] = w1.y; r.W[6] = w1.z; r.W[7] = w1.w;
    }
    const bool xmode = (getter & PACKOS_GET_EXTENDED) != 0;
    getter &= ~PACKOS_GET_EXTENDED;
    uint64_t o_start = 0, val = 0;
    uint32_t o_len = 0;
    int o_tag = 0, rc = 0;
    int64_t w = 0, s = 0, e = 0;
    bool big = false;   // a FIXED / NULLABLE value wider than 8 bytes (byte copy below)
    DGet g;
    const bool xtop = xmode && a1 - a0 >= 2 && r.u16(a0) == kExtMarker;
    if (!(xtop ? dget_init_ext(g, r, a0, (int64_t)(a1 - a0), true) : dget_init(g, r, a0, (int64_t)(a1 - a0)))) {
        rc = 3;
    } else {
        int tp;
        for (int d = 0; d < depth - 1 && !rc; d++) {
            dget_range(g, r, path.p[d], tp, s, e);
            const bool x = xmode && tp == PACKOS_TAG_EXTENDED;
            if (e < s || (tp != 7 && tp != 4 && !x)) { rc = 1; break; }
            if (e == s) { rc = 2; break; }
            DGet nx;
            if (x) {
                if (!dget_init_ext(nx, r, g.start + (uint64_t)s, e - s, false)) { rc = 1; break; }
            } else if (!dget_init(nx, r, g.start + (uint64_t)s, e - s)) {
                rc = 3;
                break;
            }
            g = nx;
        }
        if (!rc) {
            dget_range(g, r, path.p[depth - 1], tp, s, e);
            o_tag = tp;
            w = e - s;
            switch (getter) {
                case PACKOS_GET_NULLABLE:
                    if (w == 0) { rc = 4; break; }
                    [[fallthrough]];
                case PACKOS_GET_FIXED: rc = (tp != want_tag || w != want_width); break;
                case PACKOS_GET_SPAN: rc = (tp != want_tag || e < s); break;
                case PACKOS_GET_INT:
                    rc = tp != PACKOS_TAG_INTEGER ? 1 : w == 0 ? 4 : (w != 1 && w != 2 && w != 4 && w != 8);
                    break;
                case PACKOS_GET_FLOAT: rc = tp != PACKOS_TAG_FLOATING ? 1 : w == 0 ? 4 : (w != 4 && w != 8); break;
                case PACKOS_GET_ANY:   // GetTypeAndValue (get.go:504-510); past argCount buf[-2:-1] panics
                    rc = s < 0 ? 3 : e < s ? 1 : 0;
                    break;
                default: rc = 1;
            }
            if (!rc) {
                const uint64_t at = g.start + (uint64_t)s;
                o_start = at;
                o_len = (uint32_t)w;
                if (out_values && getter != PACKOS_GET_SPAN && getter != PACKOS_GET_ANY) {
                    if (getter == PACKOS_GET_INT) {
                        val = gwin_le(r, at, w);
                        if (w < 8 && ((val >> (8 * w - 1)) & 1)) val |= ~0ull << (8 * w);   // sign-extend
                    } else if (tp == PACKOS_TAG_BOOL && w == 1) {
                        val = gwin_le(r, at, 1) != 0;
                    } else if (w <= 8) {
                        val = gwin_le(r, at, w);
                    } else {
                        big = true;
                    }
                }
            }
        }
    }
    // the span / tag outputs are optional: GetInt / GetFloating / Get<T>
    // return only (value, error), so a typed gather may skip them
#ifndef PACKOS_GET_PLAIN   // non-temporal: M GetInt 0.0276 -> 0.0266 ms, C5 0.248 -> 0.244 (A/B on the box)
    if (out_start) __builtin_nontemporal_store(o_start, out_start + i);
    if (out_len) __builtin_nontemporal_store(o_len, out_len + i);
    if (out_tag) __builtin_nontemporal_store((uint8_t)o_tag, out_tag + i);
    __builtin_nontemporal_store((uint8_t)rc, status + i);
#else
    if (out_start) out_start[i] = o_start;
    if (out_len) out_len[i] = o_len;
    if (out_tag) out_tag[i] = (uint8_t)o_tag;
    status[i] = (uint8_t)rc;
#endif
    if (!out_values) return;
    uint8_t* dst = out_values + i * value_width;
    // a value wider than 8 B (big) is copied bytewise whatever value_width is
    if (!big && value_width == 8 && ((uintptr_t)dst & 7) == 0) {
#ifndef PACKOS_GET_PLAIN
        __builtin_nontemporal_store(val, (uint64_t*)dst);
#else
        *(uint64_t*)dst = val;
#endif
    } else if (!big && value_width == 4 && ((uintptr_t)dst & 3) == 0) {
        *(uint32_t*)dst = (uint32_t)val;
    } else if (!big) {
        for (uint32_t k = 0; k < value_width; k++) dst[k] = k < 8 ? (uint8_t)(val >> (8 * k)) : 0;
    } else {
        const uint64_t at = o_start;
        for (uint32_t k = 0; k < value_width; k++) dst[k] = k < (uint64_t)w ? (uint8_t)r.byte(at + k) : 0;
    }
}

// GetMapStr / GetMapAny (get.go:412-490), one thread per blob: walk the path
// like k_get_field, open the map, then validate every key (GetString) and
// value (GetString, or GetAny with nested maps walked depth first on a small
// explicit stack: the reference's GetMapAny -> GetAny recursion, get.go:377-
// 436) in wire order, writing the first max_pairs top-level pairs' spans.
constexpr int kMapDepth = 32;
struct MapFrame {
    DGet g;
    int64_t j;
};
// GetAny of value position pos of map m (get.go:377-410): 0 ok, 1 error,
// 3 panic (nil accessor), 7 = descend into `child` (a non-empty nested map)
__device__ __forceinline__ int map_value(const DGet& m, const GWin& r, int64_t pos, bool any, bool xmode, DGet& child) {
    int tp; int64_t s, e;
    dget_range(m, r, pos, tp, s, e);
    if (!any) return (e < s || tp != PACKOS_TAG_STRING) ? 1 : 0;   // GetString (get.go:359-365)
    if (pos >= m.argc) return 1;   // GetAny reads the End header; every getter then fails
    const int64_t w = e - s;
    switch (tp) {
        case PACKOS_TAG_INTEGER: return (w == 0 || w == 1 || w == 2 || w == 4 || w == 8) ? 0 : 1;
        case PACKOS_TAG_FLOATING: return (w == 0 || w == 4 || w == 8) ? 0 : 1;
        case PACKOS_TAG_STRING: return e < s ? 1 : 0;
        case PACKOS_TAG_MAP: case PACKOS_TAG_EXTENDED: {
            const bool x = tp == PACKOS_TAG_EXTENDED;
            if ((x && !xmode) || e < s) return 1;
            if (e == s) return 0;   // nil map value
            if (x) return dget_init_ext(child, r, m.start + (uint64_t)s, e - s, false) &&
                                  r.u16(m.start + (uint64_t)s + 2) == PACKOS_TAG_MAP ? 7 : 1;
            return dget_init(child, r, m.start + (uint64_t)s, e - s) ? 7 : 3;
        }
        default: return 1;   // "GetAny: unsupported type tag" (End, Tuple, Bool)
    }
}

__global__ __launch_bounds__(kBlock) void k_get_map(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                                                    uint64_t stride, uint64_t n, PathArg path, int depth, int flags,
                                                    uint32_t max_pairs, uint32_t* __restrict__ out_pairs,
                                                    uint64_t* __restrict__ key_start, uint32_t* __restrict__ key_len,
                                                    uint64_t* __restrict__ val_start, uint32_t* __restrict__ val_len,
                                                    uint8_t* __restrict__ val_tag, uint8_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    // (one block with both loads merges them into a 16-B load per lane:
    // M GetInt 0.0279 -> 0.0283 ms, A/B; kept as two loads)
    const uint64_t a0 = offs ? offs[i] : i * stride;
    const uint64_t a1 = offs ? offs[i + 1] : (i + 1) * stride;
    GWin r;
    r.a = arena;
    r.base = a0;
    const uint64_t bl = a1 > a0 ? a1 - a0 : 0;
    r.n = bl >= 32 ? 32u : bl >= 16 ? 16u : 0u;
    {
        const u32x4 z = u32x4{0u, 0u, 0u, 0u};
#ifdef PACKOS_GET_NT
        const u32x4 w0 = r.n >= 16 ? __builtin_nontemporal_load((const g_u32x4*)(arena + a0)) : z;
        const u32x4 w1 = r.n >= 32 ? __builtin_nontemporal_load((const g_u32x4*)(arena + a0 + 16)) : z;
#else
        const u32x4 w0 = r.n >= 16 ? *(const g_u32x4*)(arena + a0) : z;
        const u32x4 w1 = r.n >= 32 ? *(const g_u32x4*)(arena + a0 + 16) : z;
#endif
        r.W[0] = w0.x; r.W[1] = w0.y; r.W[2] = w0.z; r.W[3] = w0.w;
        r.W[4] = w1.x; r.W[5] = w1.y; r.W[6] = w1.z; r.W[7] = w1.w;
    }
    out_pairs[i] = 0;
    for (uint32_t j = 0; j < max_pairs; j++) {
        const uint64_t k = i * max_pairs + j;
        key_start[k] = 0; key_len[k] = 0; val_start[k] = 0; val_len[k] = 0; val_tag[k] = 0;
    }
    const bool xmode = (flags & PACKOS_GET_EXTENDED) != 0;
    const bool any = (flags & ~PACKOS_GET_EXTENDED) == PACKOS_MAP_ANY;
    DGet g;
    const bool xtop = xmode && a1 - a0 >= 2 && r.u16(a0) == kExtMarker;
    if (!(xtop ? dget_init_ext(g, r, a0, (int64_t)(a1 - a0), true) : dget_init(g, r, a0, (int64_t)(a1 - a0)))) {
        status[i] = 3;
        return;
    }
    int tp; int64_t s, e;
    for (int d = 0; d < depth - 1; d++) {
        dget_range(g, r, path.p[d], tp, s, e);
        const bool x = xmode && tp == PACKOS_TAG_EXTENDED;
        if (e < s || (tp != 7 && tp != 4 && !x)) { status[i] = 1; return; }
        if (e == s) { status[i] = 2; return; }
        DGet nx;
        if (x) {
            if (!dget_init_ext(nx, r, g.start + (uint64_t)s, e - s, false)) { status[i] = 1; return; }
        } else if (!dget_init(nx, r, g.start + (uint64_t)s, e - s)) {
            status[i] = 3;
            return;
        }
        g = nx;
    }
    dget_range(g, r, path.p[depth - 1], tp, s, e);
    const bool x = xmode && tp == PACKOS_TAG_EXTENDED;
    if (e < s || (tp != PACKOS_TAG_MAP && !x)) { status[i] = 1; return; }   // get.go:414-416
    if (e == s) { status[i] = 4; return; }                                    // nil map
    MapFrame stk[kMapDepth];
    int sp = 0;
    if (x) {
        if (!dget_init_ext(stk[0].g, r, g.start + (uint64_t)s, e - s, false) ||
            r.u16(g.start + (uint64_t)s + 2) != PACKOS_TAG_MAP) { status[i] = 1; return; }
    } else if (!dget_init(stk[0].g, r, g.start + (uint64_t)s, e - s)) {
        status[i] = 3;
        return;
    }
    stk[0].j = 0;
    sp = 1;
    uint32_t pairs = 0;
    int rc = 0;
    while (sp > 0) {
        MapFrame& f = stk[sp - 1];
        if (f.j >= f.g.argc) { sp--; continue; }
        const int64_t j = f.j;
        f.j += 2;
        int kt; int64_t ks, ke;
        dget_range(f.g, r, j, kt, ks, ke);   // key: GetString
        if (ke < ks || kt != PACKOS_TAG_STRING) { rc = 1; break; }
        DGet child;
        const int v = map_value(f.g, r, j + 1, any, xmode, child);
        if (sp == 1) {
            if (v != 1 && v != 3 && pairs < max_pairs) {
                int vt; int64_t vs, ve;
                dget_range(f.g, r, j + 1, vt, vs, ve);
                const uint64_t k = i * max_pairs + pairs;
                key_start[k] = f.g.start + (uint64_t)ks; key_len[k] = (uint32_t)(ke - ks);
                val_start[k] = f.g.start + (uint64_t)vs; val_len[k] = (uint32_t)(ve - vs); val_tag[k] = (uint8_t)vt;
            }
            pairs++;
        }
        if (v == 1 || v == 3) { rc = v; break; }
        if (v == 7) {
            if (sp >= kMapDepth) { rc = 6; break; }
            stk[sp].g = child;
            stk[sp].j = 0;
            sp++;
        }
    }
    if (rc) {
        status[i] = (uint8_t)rc;
        for (uint32_t j = 0; j < max_pairs && j < pairs; j++) {   // a failing call returns no map
            const uint64_t k = i * max_pairs + j;
            key_start[k] = 0; key_len[k] = 0; val_start[k] = 0; val_len[k] = 0; val_tag[k] = 0;
        }
        return;
    }
    out_pairs[i] = pairs;
    status[i] = pairs > max_pairs ? 5 : 0;
}

// =========================================================================
// host helpers
// =========================================================================
template <typename T>
size_t put_bytes(std::vector<uint8_t>& blob, const std::vector<T>& v) {
    size_t off = (blob.size() + 15) / 16 * 16;
    blob.resize(off + v.size() * sizeof(T) + 16);
    if (!v.empty()) memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

int current_device(int* dev) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        set_error("no GPU visible");
        return PACKOS_E_NODEVICE;
    }
    HIP_TRY(hipGetDevice(dev));
    return PACKOS_OK;
}

// Does the all-present blob of a fixed schema decode cleanly?  Runs the same
// decode_blob the device runs, on the host, over the canonical blob (zero
// payload bytes).  Only then may k_decode_fixed treat "constant bytes match"
// as "decodes like the canonical blob".
}  // namespace

bool packos::canonical_decodes(const packos_schema* s) {
    if (s->has_var || s->canon.empty() || s->fix_T <= 0) return false;
    int maxd = 0;
    for (const Node& nd : s->nodes) maxd = std::max(maxd, nd.depth);
    if (maxd >= kDecDepth) return false;
    const size_t nc = s->col_node.size();
    std::vector<uint8_t> data(nc * 1024 + 16, 0), valid(nc, 0);
    std::vector<uint64_t> start(nc, 0);
    std::vector<uint32_t> length(nc, 0);
    DecCols dc;
    memset(&dc, 0, sizeof(dc));
    for (size_t c = 0; c < nc; c++) {
        dc.data[c] = data.data() + c * 1024;
        dc.valid[c] = &valid[c];
        dc.start[c] = &start[c];
        dc.length[c] = &length[c];
    }
    // structure only: value checks (ranges, prefixes) of the zero payloads are
    // not the question here; k_decode_fixed re-checks every row's values and
    // sends failing rows to decode_blob
    std::vector<DecNode> nodes = s->dnodes;
    for (DecNode& d : nodes) d.check &= ~(uint32_t)(CHK_RANGE | CHK_STR);
    DecProgram P{nodes.data(), s->dkids.data(), s->lits.data(), 0, (int32_t)nodes.size(),
                 (int32_t)s->dkids.size(), (int32_t)s->lits.size()};
    return decode_blob(P, dc, GReader{s->canon.data()}, 0, s->canon.size(), 0) == 0;
}

namespace {

int fill_enc_cols(const packos_schema* s, const packos_column* cols, EncCols& ec, bool* any_nil) {
    memset(&ec, 0, sizeof(ec));
    *any_nil = false;
    for (size_t c = 0; c < s->col_node.size(); c++) {
        const Node& n = s->nodes[s->col_node[c]];
        ec.data[c] = (const uint8_t*)cols[c].data;
        if (cols[c].offsets64) {
            ec.off[c] = cols[c].offsets64;
            ec.off64 |= 1ull << c;
        } else {
            ec.off[c] = cols[c].offsets;
        }
        ec.valid[c] = cols[c].valid;
        bool scalar = n.kind >= K_INT && n.kind <= K_BOOL;
        bool fixed_str = (n.kind == K_STRING || n.kind == K_BYTES) && n.width > 0;
        bool var = (n.kind == K_STRING || n.kind == K_BYTES) && n.width <= 0;
        if ((scalar || fixed_str || var) && !ec.data[c]) {
            set_error("column " + std::to_string(c) + " has no data pointer");
            return PACKOS_E_INVALID;
        }
        if (var && !ec.off[c]) {
            set_error("var-width column " + std::to_string(c) + " has no offsets");
            return PACKOS_E_INVALID;
        }
        if (!(scalar && n.nullable) && !(n.kind == K_TUPLE && n.nullable) && n.kind != K_MAP) ec.valid[c] = nullptr;
        if (ec.valid[c]) *any_nil = true;
    }
    return PACKOS_OK;
}

}  // namespace

// =========================================================================
// per-device program tables
// =========================================================================
int packos::upload_tables(packos_schema* s, int device, DeviceTables** out) {
    std::lock_guard<std::mutex> lk(s->mu);
    for (auto& d : s->dev)
        if (d.device == device) { *out = &d; return PACKOS_OK; }
    std::vector<uint8_t> blob;
    size_t o_items = put_bytes(blob, s->items);
    size_t o_ipk = put_bytes(blob, s->ipk);
    size_t o_ihr = put_bytes(blob, s->ihr);
    size_t o_hdrs = put_bytes(blob, s->hdrs);
    size_t o_conts = put_bytes(blob, s->conts);
    size_t o_lits = put_bytes(blob, s->lits);
    size_t o_fsegs = put_bytes(blob, s->fsegs);
    size_t o_fidx = put_bytes(blob, s->fseg_index);
    size_t o_fcols = put_bytes(blob, s->fcols);
    size_t o_fdw = put_bytes(blob, s->fdw);
    size_t o_ftdw = put_bytes(blob, s->ftdw);
    size_t o_fxdw = put_bytes(blob, s->fxdw);
    size_t o_fxq = put_bytes(blob, s->fxq);
    size_t o_dnodes = put_bytes(blob, s->dnodes);
    size_t o_dkids = put_bytes(blob, s->dkids);
    size_t o_dfix = put_bytes(blob, s->dfix);
    size_t o_dchk = put_bytes(blob, s->dchk);
    size_t o_dvchk = put_bytes(blob, s->dvchk);
    size_t o_echk = put_bytes(blob, s->echk);
    DeviceTables t;
    t.device = device;
    HIP_TRY(hipMalloc(&t.block, blob.size()));
    HIP_TRY(hipMemcpy(t.block, blob.data(), blob.size(), hipMemcpyHostToDevice));
    uint8_t* b = (uint8_t*)t.block;
    t.enc.items = (const EncItem*)(b + o_items);
    t.enc.ipk = (const uint32_t*)(b + o_ipk);
    t.enc.ihr = (const uint32_t*)(b + o_ihr);
    t.enc.hdrs = (const EncHdr*)(b + o_hdrs);
    t.enc.conts = (const EncCont*)(b + o_conts);
    t.enc.lits = b + o_lits;
    t.enc.n_items = (int)s->items.size();
    t.enc.n_hdrs = (int)s->hdrs.size();
    t.enc.n_conts = (int)s->conts.size();
    t.enc.mode = s->mode;
    t.enc.n_lits = (int)s->lits.size();
    t.enc.ext = s->ext ? 1 : 0;
    t.fix.segs = (const FixSeg*)(b + o_fsegs);
    t.fix.seg_index = (const uint32_t*)(b + o_fidx);
    t.fix.fcols = (const FixCol*)(b + o_fcols);
    t.fix.dw = (const DwDesc*)(b + o_fdw);
    t.fix.tdw = (const DwDesc*)(b + o_ftdw);
    t.fix.xdw = (const DwDesc*)(b + o_fxdw);
    t.fix.xq = (const uint32_t*)(b + o_fxq);
    t.fix.nx = (int32_t)s->fxq.size();
    t.fix.x_lds = s->fix_x_lds;
    t.fix.B = (int)s->all_present_size;
    t.fix.T = s->fix_T;
    t.fix.n_fcols = (int)s->fcols.size();
    t.fix.lds_bytes = s->fix_lds;
    t.fix.total_chunks = s->fix_chunks;
    t.fix.overflow = s->all_present_overflow;
    t.dec.nodes = (const DecNode*)(b + o_dnodes);
    t.dec.kids = (const int32_t*)(b + o_dkids);
    t.dec.lits = b + o_lits;
    t.dec.root = 0;
    t.dec.n_nodes = (int32_t)s->dnodes.size();
    t.dec.n_kids = (int32_t)s->dkids.size();
    t.dec.n_lits = (int32_t)s->lits.size();
    t.dec.ext = s->ext ? 1 : 0;
    t.dec.win = s->has_var && !s->dec_tail_fixed && !s->ext ? (int32_t)s->dec_prefix : 0;
    {   // flat chain of <= 15 leaves: the canonical fast path applies
        const Node& root = s->nodes[0];
        bool flat = !root.kids.empty() && root.kids.size() <= 15;
        for (int k : root.kids) flat = flat && s->nodes[k].kind != K_TUPLE && s->nodes[k].kind != K_MAP;
        t.dec.flat = flat ? (int32_t)root.kids.size() : 0;
    }
    t.dfix.cols = (const DecFix*)(b + o_dfix);
    t.dfix.chk = (const uint32_t*)(b + o_dchk);
    t.dfix.vchk = (const DecChk*)(b + o_dvchk);
    t.dfix.n_vchk = (int32_t)s->dvchk.size();
    t.echk = (const EncCheck*)(b + o_echk);
    t.dfix.n_chk = (int32_t)(s->dchk.size() / 3);
    t.dfix.B = (int)s->all_present_size;
    t.dfix.T = s->fix_T;
    t.dfix.n_cols = (int)s->dfix.size();
    {
        const uint64_t q = (uint64_t)std::max<int64_t>(1, s->all_present_size / 4);
        const uint64_t bb = (uint64_t)std::max<int64_t>(2, s->all_present_size);
        t.dfix.q_magic = q > 1 ? (uint32_t)(((1ull << 32) + q - 1) / q) : 0u;
        t.dfix.b_magic = (uint32_t)(((1ull << 32) + bb - 1) / bb);
    }
    t.dfix.n_all_cols = (int)s->col_node.size();
    s->dev.push_back(t);
    *out = &s->dev.back();
    return PACKOS_OK;
}

namespace packos {
int launch_fill_offsets(uint64_t* offs, size_t n, uint64_t base, uint64_t B, hipStream_t st) {
    hipLaunchKernelGGL(k_fill_offsets_base, dim3((unsigned)((n + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, offs,
                       (uint64_t)n, base, B);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}
int launch_add_base(uint64_t* offs, size_t n, uint64_t add, hipStream_t st) {
    if (n == 0 || add == 0) return PACKOS_OK;
    hipLaunchKernelGGL(k_add_base, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, offs, (uint64_t)n,
                       add);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}
}  // namespace packos

namespace {
// DecodeBufferNamed over a SchemaNamedChain whose FieldNames and Schemas differ
// in length (schema.go:948-956): NewSeqGetAccess, then the length check fails
// every blob — ErrInvalidFormat or ErrConstraintViolated, both at position -1.
// Thread per blob; the output columns are not written (DecodeBufferNamed
// returns nil).
template <bool EXT>
__global__ __launch_bounds__(kBlock) void k_decode_chain_names(const uint8_t* __restrict__ arena,
                                                               const uint64_t* __restrict__ offs, uint64_t stride,
                                                               uint64_t n, uint32_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t a0 = offs ? offs[i] : i * stride, a1 = offs ? offs[i + 1] : (i + 1) * stride;
    const GReader R{arena};
    const int xroot = EXT && a1 - a0 >= 2 && rd16r(R, a0) == kExtMarker ? PACKOS_TAG_TUPLE : 0;
    DSeq q;
    status[i] = dseq_init(q, R, a0, (int64_t)(a1 - a0), xroot) ? (uint32_t)PACKOS_ERR_INVALID_FORMAT
                                                                : (uint32_t)PACKOS_ERR_CONSTRAINT_VIOLATED;
}
}  // namespace

extern "C" {

void packos_schema_free(packos_schema* s) {
    if (!s) return;
    packos::destroy_pipelines(s);
    for (auto& d : s->dev) {
        if (d.block) {
            int cur = -1;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(d.device);
            (void)hipFree(d.block);
            if (cur >= 0) (void)hipSetDevice(cur);
        }
    }
    delete s;
}

// workspace: [look-back ticket + one word per k_stream_sizes tile]
static size_t ws_scan_bytes(size_t n) { return (((n + kSzTile - 1) / kSzTile) + 16) * sizeof(uint64_t); }

size_t packos_encode_workspace_size(const packos_schema* s, size_t n_blobs) {
    (void)s;
    return ((ws_scan_bytes(n_blobs) + 255) & ~(size_t)255) + 256;
}

// data-independent presence: out_offsets has a closed form (k_sizes_affine)
static bool affine_layout(const packos_schema* s, const EncCols& ec, AffPlan* A) {
    AffPlan a{};
    if (s->tune.sizes_scan) return false;
    for (const EncCont& c : s->conts)
        if (c.valid_col >= 0 && ec.valid[c.valid_col]) return false;
    for (const EncItem& it : s->items) {
        if (it.type == IT_VAR) {
            if (a.nv == kAffVar) return false;
            if ((ec.off64 >> it.col) & 1ull) a.w8 |= 1u << a.nv;
            a.off[a.nv++] = ec.off[it.col];
        } else {
            if (it.type == IT_FIXED && it.nullable && ec.valid[it.col] && s->mode != PACKOS_MODE_PACKABLE) return false;
            a.C += it.size;
        }
    }
    if (A) *A = a;
    return true;
}

static int size_pass(packos_schema* s, DeviceTables* t, const EncCols& ec, size_t n, uint64_t* offs, void* ws,
                     size_t ws_bytes, hipStream_t st) {
    if (!offs) { set_error("out_offsets required for a variable-size schema"); return PACKOS_E_INVALID; }
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(offs, 0, sizeof(uint64_t), st));
        return PACKOS_OK;
    }
    if (s->ext) {
        // extended mode: per-blob sizes (k_ext_sizes) then an in-place scan
        if (!ws || ws_bytes < packos_encode_workspace_size(s, n)) {
            set_error("workspace too small");
            return PACKOS_E_WORKSPACE;
        }
        const size_t lds = (size_t)kWavesPerBlock * ext_pos_words((int)s->items.size()) * 4;
        if (lds > 64 * 1024) { set_error("schema has too many items for the LDS budget"); return PACKOS_E_UNSUPPORTED; }
        const uint64_t ntiles = (n + kSzTile - 1) / kSzTile;
        HIP_TRY(hipMemsetAsync(ws, 0, (ntiles + 1) * sizeof(uint64_t), st));
        const unsigned grid = (unsigned)std::min<uint64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 16);
        hipLaunchKernelGGL(k_ext_sizes, dim3(grid), dim3(kBlock), lds, st, t->enc, ec, offs, (uint64_t)n);
        hipLaunchKernelGGL(k_scan_inplace, dim3((unsigned)ntiles), dim3(kBlock), 0, st, offs, (uint64_t)n,
                           (uint64_t*)ws);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    AffPlan A;
    if (affine_layout(s, ec, &A)) {
        const uint64_t per = (uint64_t)kBlock * kAffPer;
        hipLaunchKernelGGL(k_sizes_affine, dim3((unsigned)((n + 1 + per - 1) / per)), dim3(kBlock), 0, st, A,
                           offs, (uint64_t)n);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    if (!ws || ws_bytes < packos_encode_workspace_size(s, n)) {
        set_error("workspace too small");
        return PACKOS_E_WORKSPACE;
    }
    // k_stream_sizes: ticket + per-tile look-back words at the start of ws
    const uint64_t ntiles = (n + kSzTile - 1) / kSzTile;
    HIP_TRY(hipMemsetAsync(ws, 0, (ntiles + 1) * sizeof(uint64_t), st));
    hipLaunchKernelGGL(k_stream_sizes, dim3((unsigned)ntiles), dim3(kBlock),
                       sizes_lds_bytes((int)s->items.size(), (int)s->conts.size()), st, t->enc, ec, (uint64_t*)ws,
                       offs, (uint64_t)n);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

int packos_encoded_size_batch(const packos_schema* cs, const packos_column* cols, size_t n, uint64_t* out_offsets,
                              void* ws, size_t ws_bytes, void* stream) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    if (!s || !cols || !out_offsets) return PACKOS_E_INVALID;
    int dev, r;
    if ((r = current_device(&dev))) return r;
    DeviceTables* t;
    if ((r = upload_tables(s, dev, &t))) return r;
    EncCols ec;
    bool any_nil;
    if ((r = fill_enc_cols(s, cols, ec, &any_nil))) return r;
    hipStream_t st = (hipStream_t)stream;
    if (!s->has_var && !any_nil && !(s->ext && s->all_present_size > (int64_t)kExtMaxPayload)) {
        hipLaunchKernelGGL(k_fill_offsets, dim3((unsigned)((n + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           out_offsets, (uint64_t)n, (uint64_t)s->all_present_size);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    return size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st);
}

static thread_local const char* g_last_encoder = "";   // packos_last_encoder

static int encode_batch_impl(packos_schema* s, DeviceTables* t, const EncCols& ec, bool any_nil, size_t n,
                             uint8_t* out, uint64_t cap, uint64_t* out_offsets, uint32_t* status, void* ws,
                             size_t ws_bytes, uint32_t flags, hipStream_t st);

int packos_encode_batch(const packos_schema* cs, const packos_column* cols, size_t n, uint8_t* out, uint64_t cap,
                        uint64_t* out_offsets, uint32_t* status, void* ws, size_t ws_bytes, uint32_t flags,
                        void* stream) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    g_last_encoder = "";
    if (!s || !cols || (!out && n)) { set_error("packos_encode_batch: bad argument"); return PACKOS_E_INVALID; }
    if (n == 0) {
        if (out_offsets) HIP_TRY(hipMemsetAsync(out_offsets, 0, sizeof(uint64_t), (hipStream_t)stream));
        return PACKOS_OK;
    }
    if (!status && !s->echk.empty()) {
        // EncodeValue returns ErrEncode (and no bytes) for a failing value check:
        // without a status array the failure could not be reported
        set_error("packos_encode_batch: the schema has encode-time checks (Range / date / prefix / suffix values, or a "
                  "named tuple whose fieldNames and schema differ / a map with an odd schema count, which fail every "
                  "present value): status required");
        return PACKOS_E_INVALID;
    }
    int dev, r;
    if ((r = current_device(&dev))) return r;
    DeviceTables* t;
    if ((r = upload_tables(s, dev, &t))) return r;
    EncCols ec;
    bool any_nil;
    if ((r = fill_enc_cols(s, cols, ec, &any_nil))) return r;
    hipStream_t st = (hipStream_t)stream;
    if ((r = encode_batch_impl(s, t, ec, any_nil, n, out, cap, out_offsets, status, ws, ws_bytes, flags, st)))
        return r;
    if (!s->echk.empty()) {
        bool pm = false;
        for (const EncCont& c : s->conts) pm = pm || (c.valid_col >= 0 && ec.valid[c.valid_col]);
        hipLaunchKernelGGL(k_encode_checks, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, t->echk,
                           (int)s->echk.size(), t->enc, ec, (uint64_t)n, status, pm ? 1 : 0);
        HIP_TRY(hipGetLastError());
    }
    return PACKOS_OK;
}


static int encode_batch_impl(packos_schema* s, DeviceTables* t, const EncCols& ec, bool any_nil, size_t n,
                             uint8_t* out, uint64_t cap, uint64_t* out_offsets, uint32_t* status, void* ws,
                             size_t ws_bytes, uint32_t flags, hipStream_t st) {
    int r;
    // extended mode: a fixed schema whose blobs exceed 8191 bytes may hold
    // extended containers, so it takes the extended path with offsets
    const bool fixed_size = !s->has_var && !any_nil && !(s->ext && s->all_present_size > (int64_t)kExtMaxPayload);
    if (fixed_size) {
        const uint64_t B = (uint64_t)s->all_present_size;
        if (B * n > cap) { set_error("output arena too small"); return PACKOS_E_CAPACITY; }
        if (out_offsets) {
            hipLaunchKernelGGL(k_fill_offsets, dim3((unsigned)((n + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                               st, out_offsets, (uint64_t)n, B);
        }
        bool aligned = ((uintptr_t)out & 15) == 0;
        for (const FixCol& fc : s->fcols) aligned = aligned && (((uintptr_t)ec.data[fc.col]) & 15) == 0;
        if (s->fix_ok && B >= 4 && aligned) {
            const uint64_t tiles = (n + s->fix_T - 1) / s->fix_T;
            const uint32_t stv = s->all_present_overflow ? PACKOS_STATUS_OVERFLOW13 : 0u;
            // variant: 13 one-tile-per-workgroup LDS-DMA kernel (default where it
            // applies), 2 lane-invariant dword kernel, 8 general 4-blob-period kernel
            int variant = (int)((flags >> 4) & 0xF);
            if (flags & PACKOS_ENC_FORCE_GENERIC) variant = 8;
            const bool dw_ok = !s->fdw.empty() && B <= 1024;
            const bool tile_ok = dw_ok && B >= 16 && (int)s->fcols.size() <= kStageCols &&
                                 (uint32_t)s->fix_T == 16u * (kBlock / (uint32_t)(B / 4)) &&
                                 s->fix_tile_lds <= 64 * 1024;
            if (variant == 0) variant = tile_ok ? 13 : dw_ok ? 2 : 8;
            if (variant == 13 && !tile_ok) variant = dw_ok ? 2 : 8;
            if (variant == 2 && !dw_ok) variant = 8;
            if (variant != 2 && variant != 13) variant = 8;
            const size_t fcb = ((s->fcols.size() * kLFixBytes) + 15) / 16 * 16;
            // each kernel gets the column table copied right after the LDS it uses
            FixProgram pdw = t->fix, pgen = t->fix;
            pdw.fc_lds = s->fix_lds;
            const size_t gen_tables = (size_t)s->fix_lds + ((B + 1) * 4 + 15) / 16 * 16 + s->fsegs.size() * sizeof(FixSeg);
            pgen.fc_lds = (int32_t)gen_tables;
            const size_t lds_dw = (size_t)pdw.fc_lds + fcb;
            if (variant == 2) {
                g_last_encoder = "fixed_dw";
                hipLaunchKernelGGL(k_encode_fixed_dw, dim3((unsigned)tiles), dim3(kBlock), lds_dw, st, pdw, ec, out,
                                   (uint64_t)n, status, stv);
            } else if (variant == 13) {
                g_last_encoder = "fixed_tile";
                FixStage S;
                memset(&S, 0, sizeof(S));
                S.n = (int32_t)s->fcols.size();
                for (int k = 0; k < S.n; k++) {
                    const FixCol& fc = s->fcols[k];
                    S.c[k] = FixStageCol{ec.data[fc.col], fc.width, fc.lds_off, fc.chunk_begin, fc.flags};
                    S.flags |= (int32_t)(fc.flags & 1u);
                }
                const uint64_t full = n / s->fix_T, rem = n - full * s->fix_T;
                if (full)
                    hipLaunchKernelGGL((k_encode_fixed_tile<16>), dim3((unsigned)full), dim3(kBlock),
                                       (size_t)s->fix_tile_lds, st, pdw, S, out, status, stv);
                if (rem) {  // partial last tile: the lane-invariant dword kernel on the remainder
                    const uint64_t b0 = full * s->fix_T;
                    EncCols et = ec;
                    for (const FixCol& fc : s->fcols) et.data[fc.col] = ec.data[fc.col] + b0 * fc.width;
                    hipLaunchKernelGGL(k_encode_fixed_dw, dim3(1), dim3(kBlock), lds_dw, st, pdw, et,
                                       out + b0 * B, rem, status ? status + b0 : nullptr, stv);
                }
            } else {
                g_last_encoder = "fixed";
                hipLaunchKernelGGL(k_encode_fixed, dim3((unsigned)tiles), dim3(kBlock), gen_tables + fcb, st, pgen, ec,
                                   out, (uint64_t)n, status, stv);
            }
            HIP_TRY(hipGetLastError());
            return PACKOS_OK;
        }
        // large or unaligned fixed blobs: general kernel with a stride
        const size_t npos = s->items.size() + 1;
        const size_t lds = (size_t)kWavesPerBlock * (kSlot + ((npos * 4 + 15) / 16) * 16);
        const unsigned grid = (unsigned)std::min<uint64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 16);
        g_last_encoder = "var";
        hipLaunchKernelGGL(k_encode_var, dim3(grid), dim3(kBlock), lds, st, t->enc, ec, (const uint64_t*)nullptr, B,
                           out, cap, (uint64_t)n, status);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    const bool offs_ready = (flags & PACKOS_ENC_OFFSETS_READY) != 0;
    if (!out_offsets) {
        set_error(offs_ready ? "PACKOS_ENC_OFFSETS_READY without out_offsets"
                             : "out_offsets required for a variable-size schema");
        return PACKOS_E_INVALID;
    }
    if (s->ext) {
        // ADR-001 extended containers: size pass (unless given), then one
        // wavefront per blob
        if (!offs_ready && !(flags & PACKOS_ENC_SIZED)) {
            if ((r = size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st))) return r;
        }
        const size_t lds = (size_t)kWavesPerBlock * ext_pos_words((int)s->items.size()) * 4;
        if (lds > 64 * 1024) { set_error("schema has too many items for the LDS budget"); return PACKOS_E_UNSUPPORTED; }
        const unsigned grid = (unsigned)std::min<uint64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 16);
        g_last_encoder = "ext";
        hipLaunchKernelGGL(k_encode_ext, dim3(grid), dim3(kBlock), lds, st, t->enc, ec, (const uint64_t*)out_offsets,
                           (uint64_t)0, out, cap, (uint64_t)n, status);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    // flat closed-form chains of large blobs: k_encode_flat (encode_flat.inc).
    // Small blobs stay on k_encode_tiles, whose frame builds the whole output
    // image in LDS (C3, 85-B blobs: 0.060 ms there vs 0.106 ms here); large
    // blobs stream their values straight from HBM here (C5, 969-B blobs: 3.57
    // ms vs 4.29).  The choice follows the batch's mean blob size (static
    // bytes + var bytes): out_capacity / n when the caller says it is exact
    // (PACKOS_ENC_CAP_EXACT) or when it is below kFlatMinBlob (an upper bound
    // of the mean); otherwise BOTH kernels are launched and decide on the
    // device (pick_skip, encode_var.inc) — nothing is read back, so the call
    // never waits on the host and can be captured in a graph.
    const bool sized = (flags & PACKOS_ENC_SIZED) != 0;
    AffPlan A{};
    const bool affine = !offs_ready && affine_layout(s, ec, &A);
    // PACKOS_ENC_SIZED: out_offsets already hold the size pass's layout — used
    // as given unless the layout is closed form (the encoders rewrite the same
    // offsets themselves, and the closed-form kernels are the fast ones)
    const bool use_given = offs_ready || (sized && !affine);
    VPlan V;
    const bool planned = !(flags & PACKOS_ENC_FORCE_GENERIC) && var_plan(s, ec, !affine, V, (uint32_t)s->tune.var_per);
    FPlan F;
    uint32_t pick = 0;
    if (s->tune.enc_flat != 0 && affine && !(flags & PACKOS_ENC_FORCE_GENERIC) && flat_plan(s, ec, F)) {
        bool flat = s->tune.enc_flat == 1;
        if (!flat && n && cap / n >= kFlatMinBlob) {   // cap / n bounds the mean from above
            if ((flags & PACKOS_ENC_CAP_EXACT) || A.nv == 0) flat = (A.nv == 0 ? (uint64_t)A.C : cap / n) >= kFlatMinBlob;
            else if (planned) pick = 1;                 // decided per batch on the device
            else flat = true;                           // (no tile plan: the flat encoder beats the generic one)
        }
        if (flat || pick) {
            F.pick = pick;
            F.pick_C = A.C;
            const dim3 g((unsigned)((n + kFT - 1) / kFT));
            g_last_encoder = pick ? "flat|tiles" : "flat";
#define PACKOS_FLAT(NV) \
    hipLaunchKernelGGL((k_encode_flat<NV>), g, dim3(kFNT), F.lds_total, st, F, out_offsets, out, cap, (uint64_t)n, status)
            if (F.nvar <= 1) PACKOS_FLAT(1);
            else if (F.nvar <= 2) PACKOS_FLAT(2);
            else PACKOS_FLAT(4);
#undef PACKOS_FLAT
            HIP_TRY(hipGetLastError());
            if (!pick) return PACKOS_OK;
        }
    }
    // default: k_encode_tiles.  Data-independent presence: the kernel computes
    // (and writes) the out offsets itself, no size pass; otherwise the size pass
    // (or the caller's PACKOS_ENC_OFFSETS_READY offsets) first, loaded per tile.
    // six workgroups per CU (k_encode_tiles<true, NV, 6>) when a closed-form plan with <= 2
    // var columns fits kVLds6; a batch whose mean var bytes per blob are known
    // (exact capacity) and <= 28 may shrink its staging pool to 32 B per blob
    bool six = false;
    if (planned && V.aff && V.nvar <= 2) {
        six = V.lds_total <= kVLds6;
        const uint64_t stat = (uint64_t)A.C * n;
        if (!six && (flags & PACKOS_ENC_CAP_EXACT) && n && cap >= stat && (cap - stat) / n <= 28 &&
            s->tune.var_per > 32) {
            VPlan V32;
            if (var_plan(s, ec, !affine, V32, 32u) && V32.aff && V32.lds_total <= kVLds6) {
                V = V32;
                six = true;
            }
        }
    }
    // closed form, exact capacity: when the batch's var bytes per blob (mean m)
    // overflow the default staging pool, a pool of 1.1 m + 4 B per blob (a
    // tile's mean varies around m; 8-B steps, <= kVPoolMax) — unstaged values
    // are holes, which cost twice as much (labels of 8..110 B: 0.136 -> 0.072
    // ms; a larger pool at the same LDS occupancy estimate measured slower at
    // small m: profiles/r06/var_pool_ab.txt)
    if (planned && !six && V.aff && affine && (flags & PACKOS_ENC_CAP_EXACT) && n && !s->tune.var_per_set &&
        cap >= (uint64_t)A.C * n) {
        const uint64_t m = (cap - (uint64_t)A.C * n) / n;
        const uint64_t per = (m * 11 / 10 + 4 + 7) & ~(uint64_t)7;
        VPlan Vb;
        if (per > (uint64_t)s->tune.var_per && per <= kVPoolMax && var_plan(s, ec, !affine, Vb, (uint32_t)per) &&
            Vb.aff)
            V = Vb;
    }
    V.pick = pick ? 2u : 0u;
    V.pick_C = A.C;
    if (planned) {
        if (!affine && !use_given) {
            if ((r = size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st))) return r;
        }
        V.lits = t->enc.lits;
        if (V.oseg >= 0) {
            V.seg[V.oseg].src = (const uint8_t*)out_offsets;
            V.seg[V.oseg].r0 = V.seg[V.oseg].lds + (uint32_t)((uintptr_t)out_offsets & 15);
        }
        const uint64_t ntiles = (n + kVT - 1) / kVT;
        g_last_encoder = pick ? "flat|tiles" : "tiles";
#ifdef PACKOS_PHASE_PROF
        unsigned long long* prof = nullptr;   // debug build only: per-tile phase clocks
        HIP_TRY(hipMalloc(&prof, ntiles * 8 * sizeof(unsigned long long)));
        HIP_TRY(hipMemsetAsync(prof, 0, ntiles * 8 * sizeof(unsigned long long), st));
        V.prof = prof;
#endif
        // instantiated per var-slot bound: the per-blob loops over var slots
        // (positions, lengths, header offsets) stop at the schema's count
#define PACKOS_TILES(AFF, NV)                                                                             \
    hipLaunchKernelGGL((k_encode_tiles<AFF, NV, 1>), dim3((unsigned)ntiles), dim3(kVNT), V.lds_total, st, V, \
                       out_offsets, out, cap, (uint64_t)n, status)
#define PACKOS_TILES6(NV)                                                                                  \
    hipLaunchKernelGGL((k_encode_tiles<true, NV, 6>), dim3((unsigned)ntiles), dim3(kVNT), V.lds_total, st, V, \
                       out_offsets, out, cap, (uint64_t)n, status)
        const int nv = V.nvar <= 1 ? 1 : V.nvar <= 2 ? 2 : V.nvar <= 4 ? 4 : 8;
        if (six) {
            g_last_encoder = pick ? "flat|tiles6" : "tiles6";
            if (nv == 1) PACKOS_TILES6(1);
            else PACKOS_TILES6(2);
        } else if (V.aff) {
            if (nv == 1) PACKOS_TILES(true, 1);
            else if (nv == 2) PACKOS_TILES(true, 2);
            else if (nv == 4) PACKOS_TILES(true, 4);
            else PACKOS_TILES(true, 8);
        } else {
            if (nv == 1) PACKOS_TILES(false, 1);
            else if (nv == 2) PACKOS_TILES(false, 2);
            else if (nv == 4) PACKOS_TILES(false, 4);
            else PACKOS_TILES(false, 8);
        }
#undef PACKOS_TILES
#undef PACKOS_TILES6
        HIP_TRY(hipGetLastError());
#ifdef PACKOS_PHASE_PROF
        std::vector<unsigned long long> hp(ntiles * 8);
        HIP_TRY(hipMemcpyAsync(hp.data(), prof, hp.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        HIP_TRY(hipFree(prof));
        unsigned long long h[8] = {};
        for (uint64_t x = 0; x < ntiles; x++)
            for (int q = 0; q < 8; q++) h[q] += hp[x * 8 + q];
        fprintf(stderr, "k_encode_tiles lds=%u tiles=%llu clocks/tile: load=%.0f [round2=%.0f blobs=%.0f scan=%.0f] "
                "frame=%.0f [chunks1=%.0f chunks2=%.0f] closed-form frame of waves 0..3: %.0f %.0f %.0f %.0f\n",
                V.lds_total, (unsigned long long)ntiles, (double)h[0] / ntiles, (double)h[4] / ntiles,
                (double)h[5] / ntiles, (double)h[1] / ntiles, (double)h[2] / ntiles, (double)h[6] / ntiles,
                (double)h[3] / ntiles, (double)h[4] / ntiles, (double)h[5] / ntiles, (double)h[6] / ntiles,
                (double)h[7] / ntiles);
#endif
        return PACKOS_OK;
    }
    if (!use_given) {
        if ((r = size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st))) return r;
    }
    const size_t npos = s->items.size() + 1;
    const size_t lds = (size_t)kWavesPerBlock * (kSlot + ((npos * 4 + 15) / 16) * 16);
    if (lds > 64 * 1024) { set_error("schema has too many items for the LDS budget"); return PACKOS_E_UNSUPPORTED; }
    const unsigned grid = (unsigned)std::min<uint64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 16);
    g_last_encoder = "var";
    hipLaunchKernelGGL(k_encode_var, dim3(grid), dim3(kBlock), lds, st, t->enc, ec, (const uint64_t*)out_offsets,
                       (uint64_t)0, out, cap, (uint64_t)n, status);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

const char* packos_last_encoder(void) { return g_last_encoder; }


int packos_decode_batch(const packos_schema* cs, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                        size_t n, packos_column* out_cols, uint32_t* status, void* stream) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    if (!s || !out_cols || !status || (!arena && n)) { set_error("packos_decode_batch: bad argument"); return PACKOS_E_INVALID; }
    if (n == 0) return PACKOS_OK;
    if (!offsets && stride == 0) { set_error("offsets or stride required"); return PACKOS_E_INVALID; }
    int dev, r;
    if ((r = current_device(&dev))) return r;
    DeviceTables* t;
    if ((r = upload_tables(s, dev, &t))) return r;
    int maxd = 0;
    for (const Node& nd : s->nodes) maxd = std::max(maxd, nd.depth);
    if (maxd >= kDecDepth) { set_error("schema nesting too deep for the decoder"); return PACKOS_E_UNSUPPORTED; }
    DecCols dc;
    memset(&dc, 0, sizeof(dc));
    for (size_t c = 0; c < s->col_node.size(); c++) {
        const Node& nd = s->nodes[s->col_node[c]];
        dc.data[c] = (uint8_t*)out_cols[c].data;
        dc.valid[c] = out_cols[c].valid;
        dc.start[c] = out_cols[c].start;
        dc.length[c] = out_cols[c].length;
        bool scalar = nd.kind >= K_INT && nd.kind <= K_BOOL;
        bool fixed_str = (nd.kind == K_STRING || nd.kind == K_BYTES) && nd.width > 0;
        bool var = (nd.kind == K_STRING || nd.kind == K_BYTES) && nd.width <= 0;
        if ((scalar || fixed_str) && !dc.data[c]) { set_error("decode column " + std::to_string(c) + " needs data"); return PACKOS_E_INVALID; }
        if (var && (!dc.start[c] || !dc.length[c])) { set_error("decode var column " + std::to_string(c) + " needs start/length"); return PACKOS_E_INVALID; }
        if (scalar && nd.nullable && !dc.valid[c]) { set_error("decode nullable column " + std::to_string(c) + " needs valid"); return PACKOS_E_INVALID; }
        if (!(scalar && nd.nullable) && nd.kind != K_TUPLE && nd.kind != K_MAP) dc.valid[c] = nullptr;
    }
    hipStream_t st = (hipStream_t)stream;
    if (s->chain_names) {
        if (s->ext) hipLaunchKernelGGL(k_decode_chain_names<true>, dim3((unsigned)((n + kBlock - 1) / kBlock)),
                                       dim3(kBlock), 0, st, arena, offsets, stride, (uint64_t)n, status);
        else hipLaunchKernelGGL(k_decode_chain_names<false>, dim3((unsigned)((n + kBlock - 1) / kBlock)),
                                dim3(kBlock), 0, st, arena, offsets, stride, (uint64_t)n, status);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    const int64_t B = s->all_present_size;
    bool fast = s->dec_fast == 1 && ((uintptr_t)arena & 15) == 0 && (offsets || stride == (uint64_t)B) &&
                !s->tune.decode_generic;
    for (const DecFix& f : s->dfix) fast = fast && ((uintptr_t)dc.data[f.col] & 15) == 0;
    fast = fast && s->dfix.size() <= (size_t)kDecK;
    if (fast) {
        // decode tile: dec_tile_bytes of staged blobs (16-blob multiple, <= 1024 blobs)
        DecFixProgram F = t->dfix;
        // measured (PACKOS_DEC_TILE_BYTES sweep 16/24/32/48 KB): 24 KB tiles are
        // best for B >= 128 (M 0.111 -> 0.103 ms, C4 0.431 -> 0.409 ms); for
        // small blobs the larger tile loses more to fewer workgroups (C2 +7 %)
        int64_t tb = B >= 128 ? kDecTileBytesLarge : kDecTileBytes;
        if (s->tune.dec_tile_bytes) tb = s->tune.dec_tile_bytes;
        F.T = (int32_t)std::min<int64_t>(1024, std::max<int64_t>(16, (tb / B) / 16 * 16));
        const uint32_t T = (uint32_t)F.T, QW = (uint32_t)((B + 3) / 4);
        const size_t lds = (size_t)T * B + 16 + 12 * QW;
        DecColsK K;
        memset(&K, 0, sizeof(K));
        K.n = (int32_t)s->dfix.size();
        for (int c = 0; c < K.n; c++) {
            const DecFix& f = s->dfix[c];
            K.dst[c] = dc.data[f.col];
            K.width[c] = f.width;
            K.blob_off[c] = f.blob_off;
            K.flags[c] = f.flags;
            K.magic[c] = f.magic;
        }
        // full tiles: 64-unit wave steps over every column (T % 16 == 0, so a
        // column's tile bytes T * w are whole 16-B units at a 16-B aligned
        // address), costliest read shapes first so the waves' round-robin share
        // of the list is balanced
        {
            struct St { uint32_t word, cost; };
            std::vector<St> st;
            bool ok = (B & 3) == 0 && T % 16 == 0;
            for (int c = 0; ok && c < K.n; c++) {
                const uint32_t w = K.width[c];
                // sort key per dword (the LDS reads and merges a dword takes;
                // the unit weights measured best for 256-B blobs); 16-B units for
                // blobs of >= 128 B, lane-interleaved dwords for smaller ones
                uint32_t kind, cost;
                const bool q0 = (K.blob_off[c] & 3u) == 0, units = B >= 128;
                if (w % 16 == 0 && B % 16 == 0) kind = DS_W16, cost = 2;
                else if (units && w == 8) kind = DS_W8, cost = 4;
                else if (units && w == 4) kind = DS_W4, cost = 4;
                else if (w % 4 == 0) kind = units ? DS_G4U : DS_D4, cost = units ? (q0 ? 4 : 8) : (q0 ? 1 : 2);
                else if (w > 4) kind = units ? DS_GENU : DS_GEN, cost = units ? 10 : 3;
                else if (w == 2) kind = units ? DS_W2 : DS_D2, cost = units ? 8 : (q0 ? 2 : 4);
                else if (w == 1) kind = (K.flags[c] & 1u) ? (units ? DS_BOOLU : DS_BOOL) : (units ? DS_W1 : DS_D1),
                                 cost = units ? 16 : 4;
                else kind = DS_BYTE, cost = units ? 32 : 4;
                const uint32_t bytes = T * w;   // whole 16-B units (T % 16 == 0)
                for (uint32_t blk = 0; 1024u * blk < bytes; blk++) {
                    const uint32_t nd = std::min<uint32_t>(1024u, bytes - 1024u * blk) / 4;
                    if (blk > 0xFFu) ok = false;
                    st.push_back({(uint32_t)c | (blk << 5) | ((nd - 1) << 13) | (kind << 24), cost * nd});
                }
            }
            if (ok && st.size() <= (size_t)kDecSteps) {
                std::stable_sort(st.begin(), st.end(), [](const St& a, const St& b) { return a.cost > b.cost; });
                K.nsteps = (int32_t)st.size();
                for (size_t k = 0; k < st.size(); k++) K.step[k] = st[k].word;
            }
        }
        const uint64_t tile0 = 0;
        const uint64_t rest = (n + T - 1) / T - tile0;
        if (rest) {
            auto k1 = B < 128 ? (s->ext ? k_decode_fixed8<true> : k_decode_fixed8<false>)
                              : (s->ext ? k_decode_fixed<true> : k_decode_fixed<false>);
            hipLaunchKernelGGL(k1, dim3((unsigned)rest), dim3(kBlock), lds, st, F, t->dec, dc, K, arena, offsets,
                               (uint64_t)n, status, tile0);
        }
    } else {
        const size_t ptab = ((s->dnodes.size() * sizeof(DecNode) + 15) & ~(size_t)15) +
                            ((s->dkids.size() * 4 + 15) & ~(size_t)15) + s->lits.size() + 16;
        // per-blob window: the static prefix from a 16-B aligned start (+15 B)
        // (a fixed payload after a var one is read past the prefix: keep >= 24 KB
        // so tiles of such schemas stay staged whole)
        int64_t need = (s->dec_prefix + 15 + 15) / 16;
        if (s->dec_tail_fixed && need < 6) need = 6;
        const dim3 g((unsigned)((n + kBlock - 1) / kBlock));
        // flat chains of plain leaves: field descriptors + output pointers by value
        FlatArg FA;
        memset(&FA, 0, sizeof(FA));
        {
            const Node& root = s->nodes[0];
            bool ok = !s->ext && !s->tune.decode_generic && !root.kids.empty() && root.kids.size() <= (size_t)kFlatMax;
            for (size_t j = 0; ok && j < root.kids.size(); j++) {
                const Node& nd = s->nodes[root.kids[j]];
                const DecNode& dn = s->dnodes[root.kids[j]];
                ok = nd.kind >= K_INT && nd.kind <= K_BYTES && nd.check == 0 && dn.width < 0x8000;
                if (!ok) break;
                const bool scalar = nd.kind >= K_INT && nd.kind <= K_BOOL;
                const bool var = !scalar && dn.width <= 0;
                FA.fd[j] = (uint32_t)nd.kind | ((uint32_t)(dn.width & 0xFFFF) << 4) | ((uint32_t)dn.tag << 20) |
                           ((dn.nullable ? 1u : 0u) << 23);
                FA.p0[j] = (uint64_t)(uintptr_t)(var ? (void*)dc.start[nd.col] : (void*)dc.data[nd.col]);
                FA.p1[j] = (uint64_t)(uintptr_t)(var ? (void*)dc.length[nd.col] : (void*)dc.valid[nd.col]);
                if (scalar && (dn.width != 1 && dn.width != 2 && dn.width != 4 && dn.width != 8)) ok = false;
                // one naturally aligned store per row (a 16-B aligned column base)
                if (!var && (FA.p0[j] & 15)) ok = false;
                if (var && ((FA.p0[j] & 7) || (FA.p1[j] & 3))) ok = false;
            }
            FA.F = ok ? (int32_t)root.kids.size() : 0;
        }
#define PACKOS_DECWIN(WC, X)                                                                                 \
    hipLaunchKernelGGL((k_decode_win<WC, X>), g, dim3(kBlock), ptab, st, t->dec, dc, FA, arena, offsets, stride, \
                       (uint64_t)n, status)
        if (s->ext) {   // extended containers: bigger blobs, no window sizing games
            PACKOS_DECWIN(kDecWinChunks, true);
        } else if (need <= 2) {
            PACKOS_DECWIN(2, false);
        } else if (need <= 4) {
            PACKOS_DECWIN(4, false);
        } else if (need <= 6) {
            PACKOS_DECWIN(6, false);
        } else {
            PACKOS_DECWIN(kDecWinChunks, false);
        }
#undef PACKOS_DECWIN
    }
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

// schema.ValidateBuffer (schema/schema.go:880-891) per blob: the windowed
// SeqGetAccess decoder in its status-only VAL form, the window cut to the bytes
// validation reads (header words, literals, checked payloads: compile.cpp).
int packos_validate_batch(const packos_schema* cs, const uint8_t* arena, const uint64_t* offsets, uint64_t stride,
                          size_t n, uint32_t* status, void* stream) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    if (!s || !status || (!arena && n)) { set_error("packos_validate_batch: bad argument"); return PACKOS_E_INVALID; }
    if (n == 0) return PACKOS_OK;
    if (!offsets && stride == 0) { set_error("offsets or stride required"); return PACKOS_E_INVALID; }
    int dev, r;
    if ((r = current_device(&dev))) return r;
    DeviceTables* t;
    if ((r = upload_tables(s, dev, &t))) return r;
    int maxd = 0;
    for (const Node& nd : s->nodes) maxd = std::max(maxd, nd.depth);
    if (maxd >= kDecDepth) { set_error("schema nesting too deep for the decoder"); return PACKOS_E_UNSUPPORTED; }
    DecCols dc;
    memset(&dc, 0, sizeof(dc));
    hipStream_t st = (hipStream_t)stream;
    // fixed layouts whose checks read most of each blob (or blobs of <= 2
    // lines): the staged-tile path of the fixed decoder, status only
    const int64_t B = s->all_present_size;
    if (s->dec_fast == 1 && ((uintptr_t)arena & 15) == 0 && (offsets || stride == (uint64_t)B) &&
        !s->tune.decode_generic && (s->val_win == 0 || 2 * s->val_win >= B || B <= 128)) {
        DecFixProgram F = t->dfix;
        const int64_t tb = B >= 128 ? kDecTileBytesLarge : kDecTileBytes;
        F.T = (int32_t)std::min<int64_t>(1024, std::max<int64_t>(16, (tb / B) / 16 * 16));
        const uint32_t T = (uint32_t)F.T, QW = (uint32_t)((B + 3) / 4);
        const size_t lds = (size_t)T * B + 16 + 12 * QW;
        DecColsK K;
        memset(&K, 0, sizeof(K));
        hipLaunchKernelGGL(s->ext ? k_validate_fixed<true> : k_validate_fixed<false>,
                           dim3((unsigned)((n + T - 1) / T)), dim3(kBlock), lds, st, F, t->dec, dc, K, arena, offsets,
                           (uint64_t)n, status, (uint64_t)0);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    DecProgram P = t->dec;
    P.win = (int32_t)s->val_win;
    const size_t ptab = ((s->dnodes.size() * sizeof(DecNode) + 15) & ~(size_t)15) +
                        ((s->dkids.size() * 4 + 15) & ~(size_t)15) + s->lits.size() + 16;
    const int64_t need = s->val_win > 0 ? (s->val_win + 15 + 15) / 16 : kDecWinChunks;
    const dim3 g((unsigned)((n + kBlock - 1) / kBlock));
    // flat chains of plain leaves: pass 1 of the descriptor fast path only
    FlatArg FA;
    memset(&FA, 0, sizeof(FA));
    {
        const Node& root = s->nodes[0];
        bool ok = !s->ext && !s->tune.decode_generic && !root.kids.empty() && root.kids.size() <= (size_t)kFlatMax;
        for (size_t j = 0; ok && j < root.kids.size(); j++) {
            const Node& nd = s->nodes[root.kids[j]];
            const DecNode& dn = s->dnodes[root.kids[j]];
            ok = nd.kind >= K_INT && nd.kind <= K_BYTES && nd.check == 0 && dn.width < 0x8000;
            FA.fd[j] = (uint32_t)nd.kind | ((uint32_t)(dn.width & 0xFFFF) << 4) | ((uint32_t)dn.tag << 20) |
                       ((dn.nullable ? 1u : 0u) << 23);
        }
        FA.F = ok ? (int32_t)root.kids.size() : 0;
    }
#define PACKOS_VALWIN(WC, X) \
    hipLaunchKernelGGL((k_decode_win<WC, X, true>), g, dim3(kBlock), ptab, st, P, dc, FA, arena, offsets, stride, \
                       (uint64_t)n, status)
    if (s->ext) PACKOS_VALWIN(kDecWinChunks, true);
    else if (need <= 2) PACKOS_VALWIN(2, false);
    else if (need <= 4) PACKOS_VALWIN(4, false);
    else PACKOS_VALWIN(kDecWinChunks, false);
#undef PACKOS_VALWIN
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

int packos_get_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n, const int32_t* path,
                     int depth, int getter, int want_tag, int want_width, uint8_t* out_values, uint32_t value_width,
                     uint64_t* out_start, uint32_t* out_len, uint8_t* out_tag, uint8_t* status, void* stream) {
    if (!path || depth < 1 || depth > 16 || !status || (!arena && n)) return PACKOS_E_INVALID;
    const int g_base = getter & ~PACKOS_GET_EXTENDED;
    if (g_base < PACKOS_GET_FIXED || g_base > PACKOS_GET_ANY) {
        set_error("unknown getter");
        return PACKOS_E_INVALID;
    }
    // spans may be skipped only where a typed value carries the result
    if ((!out_start || !out_len || !out_tag) && (g_base == PACKOS_GET_SPAN || g_base == PACKOS_GET_ANY || !out_values)) {
        set_error("out_start / out_len / out_tag may be NULL only for a typed gather (out_values set)");
        return PACKOS_E_INVALID;
    }
    if (out_values && value_width == 0) {
        set_error("out_values needs value_width > 0");
        return PACKOS_E_INVALID;
    }
    if (n == 0) return PACKOS_OK;
    if (!offsets && stride == 0) return PACKOS_E_INVALID;
    int dev, r;
    if ((r = current_device(&dev))) return r;
    PathArg pa{};
    for (int d = 0; d < depth; d++) {
        if (path[d] < 0) { set_error("negative field position"); return PACKOS_E_INVALID; }
        pa.p[d] = path[d];
    }
    hipLaunchKernelGGL(k_get_field, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       (hipStream_t)stream, arena, offsets, stride, (uint64_t)n, pa, depth, getter, want_tag,
                       want_width, out_values, value_width, out_start, out_len, out_tag, status);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

int packos_get_map_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n, const int32_t* path,
                         int depth, int flags, uint32_t max_pairs, uint32_t* out_pairs, uint64_t* key_start,
                         uint32_t* key_len, uint64_t* val_start, uint32_t* val_len, uint8_t* val_tag, uint8_t* status,
                         void* stream) {
    if (!path || depth < 1 || depth > 16 || !out_pairs || !status || (!arena && n)) return PACKOS_E_INVALID;
    const int f = flags & ~PACKOS_GET_EXTENDED;
    if (f != PACKOS_MAP_STR && f != PACKOS_MAP_ANY) { set_error("unknown map getter"); return PACKOS_E_INVALID; }
    if (max_pairs && (!key_start || !key_len || !val_start || !val_len || !val_tag)) {
        set_error("max_pairs > 0 needs the key / value span arrays");
        return PACKOS_E_INVALID;
    }
    if (n == 0) return PACKOS_OK;
    if (!offsets && stride == 0) return PACKOS_E_INVALID;
    int dev, r;
    if ((r = current_device(&dev))) return r;
    PathArg pa{};
    for (int d = 0; d < depth; d++) {
        if (path[d] < 0) { set_error("negative field position"); return PACKOS_E_INVALID; }
        pa.p[d] = path[d];
    }
    hipLaunchKernelGGL(k_get_map, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, (hipStream_t)stream,
                       arena, offsets, stride, (uint64_t)n, pa, depth, flags, max_pairs, out_pairs, key_start, key_len,
                       val_start, val_len, val_tag, status);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

// Exact-width (want_width >= 0) or span (want_width < 0) getter without a
// typed gather: the round-1 entry point, kept for callers that bind it.
int packos_get_field_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                           const int32_t* path, int depth, int want_tag, int want_width, uint64_t* out_start,
                           uint32_t* out_len, uint8_t* out_tag, uint8_t* status, void* stream) {
    return packos_get_batch(arena, offsets, stride, n, path, depth, want_width >= 0 ? PACKOS_GET_FIXED : PACKOS_GET_SPAN,
                            want_tag, want_width, nullptr, 0, out_start, out_len, out_tag, status, stream);
}

}  // extern "C"
