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
//                   off_v[0]) — a pure map (encode_stream.inc)
//   k_stream_sizes  other var-size schemas: blob sizes + decoupled look-back
//                   scan -> out_offsets (encode_stream.inc)
//   k_encode_stream var-size schemas: two bulk staging rounds into LDS, two
//                   emitters per blob into an LDS image, 16-B stores
//                   (encode_stream.inc)
//   k_encode_var    per-blob fallback: one wavefront per blob; item sizes ->
//                   wavefront prefix scan -> header words -> payload staged
//                   in an LDS slot -> aligned 16-B stores
//   k_decode        schema.DecodeBuffer semantics (SeqGetAccess + precheck),
//                   one thread per blob, exact error/panic reporting
//   k_get_field     GetAccess random-field gather
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
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

// fixed-layout encode variant used when the caller does not pick one
// (1..4: dword stores, 5..7: LDS re-staged 16-B stores; NT = non-temporal)
constexpr int kDefaultFixedVariant = 2;

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
template <bool NTS>
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
            if (NTS) __builtin_nontemporal_store(v, o32 + (uint64_t)j * Q4);
            else o32[(uint64_t)j * Q4] = v;
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
#ifndef ENC_ABL
#define ENC_ABL 0
#endif
    const uint32_t lds0 = (uint32_t)(uintptr_t)lds;
    for (int g = 0; g < (ENC_ABL == 2 ? 0 : S.n); g++) {
        const uint32_t nch = (T * S.c[g].width) >> 4;
        const uint8_t* cbase = S.c[g].base + blob0 * S.c[g].width;
        for (uint32_t c0 = wv * kWave; c0 < nch; c0 += kBlock) {
            if (c0 + lane < nch)
                dma16(cbase + (c0 + lane) * 16u, __builtin_amdgcn_readfirstlane(lds0 + S.c[g].lds_off + c0 * 16u));
        }
    }
    // descriptors (their global loads queue behind the DMA)
    const DwDesc* dd = P.tdw + q;
    const uint32_t cval = dd->cval;
    const DwSeg sg = dd->seg[0];
    uint32_t a = (uint32_t)sg.a + s * sg.w;  // LDS byte address of this thread's first dword
    const uint32_t xs = R * sg.w, xm = sg.mask;
    const uint32_t nxi = T * (uint32_t)P.nx;
    DwDesc xd;  // this thread's first X item
    if (tid < nxi) xd = P.xdw[tid % (uint32_t)P.nx];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    uint32_t* l32 = (uint32_t*)lds;
    if (nxi && ENC_ABL != 3) {
        auto assemble = [&](uint32_t i, const DwDesc& d) {
            const uint32_t j = i / (uint32_t)P.nx;
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
        if (tid < nxi) assemble(tid, xd);
        for (uint32_t i = tid + kBlock; i < nxi; i += kBlock) assemble(i, P.xdw[i % (uint32_t)P.nx]);
        __syncthreads();
    }
    if (s < R) {  // R * Q4 <= 256: the rest of the threads idle here
        uint32_t* o32 = (uint32_t*)(out + blob0 * B) + s * Q4 + q;
        const uint32_t ostep = R * Q4;
#pragma unroll
        for (int it = 0; it < PER; it++) {
            uint32_t val = cval;
            if (ENC_ABL != 1) {
                const uint32_t lo = l32[a >> 2], hi = l32[(a >> 2) + 1];
                val |= __builtin_amdgcn_alignbyte(hi, lo, a) & xm;  // uses a & 3
            } else {
                val ^= a * 0x9E3779B1u + (uint32_t)blob0;  // ablation: data-dependent, no LDS read
            }
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

// =========================================================================
// variable-size encode
// =========================================================================
struct BlobCtx {
    uint64_t present;   // container presence bits
};

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
        case IT_VAR: {
            const uint32_t* o = cols.off[it.col];
            return o[i + 1] - o[i];
        }
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
        else src = cols.data[it.col] + cols.off[it.col][i];
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

// Tiled var-size encode.  A workgroup takes VT consecutive blobs; their
// outputs are contiguous in the arena (offsets from the size pass), so the
// group assembles runs of blobs in LDS and writes them with 16-B stores.
// Global-memory latency, not bandwidth, is what a per-blob design pays for,
// so the kernel is organised in two rounds of independent loads:
//   round 1  everything that depends only on kernel arguments, issued
//            together: the schema program (items, header words, containers,
//            literals), the tile's blob offsets, var-column offsets,
//            validity bytes and every fixed column's rows (16-B chunks) —
//            one flattened index space, kVBatch loads in flight per thread;
//   round 2  the var columns' byte ranges (now known) are staged while the
//            threads compute presence masks and item positions (LDS only);
//   runs     the tile is split into runs (blobs whose start falls in one
//            2^win_shift-byte window); per run the LDS buffer is zeroed,
//            header words and items are written by (header|item, blob) pairs
//            from LDS, and the run is stored with 16-B non-temporal stores;
//   direct   var values that did not fit the staging budget (long values)
//            are copied HBM->HBM afterwards, flattened over destination
//            dwords so that every thread keeps several loads in flight.
// Tiles outside the plan (offsets that disagree with the program, a blob
// > 64 KiB, capacity overrun) and runs > bud bytes use var_blob_wave.
constexpr int kVBatch = 4;
constexpr int kVPFix = 32;     // plan limits (more -> one wavefront per blob)
constexpr int kVPVar = 16;
constexpr int kVPVal = 16;

struct VarPlan {               // per-call plan, passed by value
    int32_t nfix, nvar, nval, fix_bytes;
    const uint8_t* fix_ptr[kVPFix];   // fixed leaf columns (one region per IT_FIXED item)
    uint32_t fix_w[kVPFix];
    uint32_t fix_lds[kVPFix];  // staging offset of fixed region r (full tile, 16-B aligned)
    const uint32_t* var_off[kVPVar];  // var leaf columns (one per IT_VAR item)
    const uint8_t* var_data[kVPVar];
    int32_t var_item[kVPVar];
    const uint8_t* val_ptr[kVPVal];   // validity columns passed by the caller
    int8_t col_val[kMaxCols];  // column -> validity slot, -1 none
};

struct VVar {                  // var region of the current tile (LDS)
    uint64_t src;              // column bytes of the tile's first blob
    uint32_t lds_off;          // staging offset, UINT32_MAX = not staged
    uint32_t pad;
};

struct VtLayout {
    uint32_t boff, pmk, bst, misc, subs, items, ipk, ihr, hdrs, conts, lits, voff, vld, pos, vvar, fmis, freg, stg, total;
};
__host__ __device__ inline VtLayout vt_layout(int VT, const EncProgram& P, int nvar, int nval, uint32_t bud,
                                               uint32_t in_bud) {
    auto al16 = [](uint32_t x) { return (x + 15u) & ~15u; };
    const uint32_t NI = (uint32_t)P.n_items;
    VtLayout L;
    uint32_t o = al16(bud + 32);
    L.boff = o;  o += 8 * (VT + 1);
    L.pmk = o;   o += 8 * VT;
    L.bst = o;   o += 4 * VT;
    L.misc = o;  o += 4 * 16;
    L.subs = o;  o += al16(4 * (VT + 1));
    L.items = o; o += al16(sizeof(EncItem) * NI);
    L.ipk = o;   o += al16(4 * NI);
    L.ihr = o;   o += al16(4 * NI);
    L.hdrs = o;  o += al16(sizeof(EncHdr) * (uint32_t)P.n_hdrs);
    L.conts = o; o += al16(sizeof(EncCont) * (uint32_t)P.n_conts);
    L.lits = o;  o += al16((uint32_t)P.n_lits + 4);
    L.voff = o;  o += 4 * nvar * (VT + 1);
    L.vld = o;   o += al16(nval * VT);
    L.pos = o;   o += al16(2 * VT * (NI + 1));
    L.vvar = o;  o += al16(sizeof(VVar) * nvar);
    L.fmis = o;  o += al16(4 * kVPFix);
    L.freg = o;  o += 16 * kVPFix;
    L.stg = o;   o += al16(in_bud + 16);
    L.total = o;
    return L;
}


__device__ __forceinline__ uint32_t magic_of(uint32_t d) {
    return d > 1 ? (uint32_t)((0x100000000ull + d - 1) / d) : 0u;
}
__device__ __forceinline__ uint32_t fast_div(uint32_t t, uint32_t d, uint32_t mg) { return d > 1 ? __umulhi(t, mg) : t; }

typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint64_t g_u64;
typedef __attribute__((address_space(1))) const uint8_t g_u8;

template <int VT>
__global__ __launch_bounds__(kBlock) void k_encode_var_tile(EncProgram P, EncCols cols, VarPlan V,
                                                            const uint64_t* __restrict__ offs,
                                                            uint8_t* __restrict__ out, uint64_t cap, uint64_t n,
                                                            uint32_t* __restrict__ status, uint32_t bud,
                                                            uint32_t win_shift, uint32_t in_bud,
                                                            uint32_t* __restrict__ tflags, uint16_t* __restrict__ vpos,
                                                            unsigned long long* __restrict__ prof) {
    static_assert(VT % kWave == 0 && VT <= kBlock, "tile = whole wavefronts, at most one blob per thread");
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int NI = P.n_items, NP = NI + 1, NH = P.n_hdrs;
    const VtLayout L = vt_layout(VT, P, V.nvar, V.nval, bud, in_bud);
    uint8_t* obuf = lds;
    uint64_t* boff = (uint64_t*)(lds + L.boff);
    uint64_t* pmk = (uint64_t*)(lds + L.pmk);
    uint32_t* bst = (uint32_t*)(lds + L.bst);
    uint32_t* misc = (uint32_t*)(lds + L.misc);   // 0 fallback, 1 #runs, 4..7 wave counts, 8.. scratch
    uint32_t* subs = (uint32_t*)(lds + L.subs);
    EncItem* items = (EncItem*)(lds + L.items);
    EncHdr* hdrs = (EncHdr*)(lds + L.hdrs);
    EncCont* conts = (EncCont*)(lds + L.conts);
    uint32_t* voff = (uint32_t*)(lds + L.voff);
    uint8_t* vld = lds + L.vld;
    uint16_t* pos = (uint16_t*)(lds + L.pos);
    VVar* vvar = (VVar*)(lds + L.vvar);
    uint32_t* fmis = (uint32_t*)(lds + L.fmis);
    u32x4* freg = (u32x4*)(lds + L.freg);        // fixed region: {a0 lo, a0 hi, first chunk, LDS offset}
    const uint32_t* ipk = (const uint32_t*)(lds + L.ipk);
    const uint32_t* ihr = (const uint32_t*)(lds + L.ihr);
    uint8_t* stg = lds + L.stg;

    const uint64_t lo = (uint64_t)blockIdx.x * VT;
    const uint32_t rows = (uint32_t)min((uint64_t)VT, n - lo);
    uint64_t t_last = prof ? __builtin_amdgcn_s_memtime() : 0;
    auto mark = [&](int ph) {
        if (prof && tid == 0) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            atomicAdd(prof + ph, (unsigned long long)(t - t_last));
            t_last = t;
        }
    };

    // ---- round 1 -----------------------------------------------------------
    // one flattened index space; the var-offset and validity segments are
    // padded to whole wavefronts so the column behind an element is
    // wave-uniform (scalar pointer loads, no dependent vector loads)
    {
        auto al64 = [](uint32_t x) { return (x + 63u) & ~63u; };
        const uint32_t e_items = (uint32_t)NI * (sizeof(EncItem) / 4);
        const uint32_t e_hdrs = e_items + (uint32_t)NH * (sizeof(EncHdr) / 4);
        const uint32_t e_conts = e_hdrs + (uint32_t)P.n_conts * (sizeof(EncCont) / 4);
        const uint32_t e_ipk = e_conts + (uint32_t)NI;
        const uint32_t e_ihr = e_ipk + (uint32_t)NI;
        const uint32_t e_lits = e_ihr + ((uint32_t)P.n_lits + 3) / 4;
        const uint32_t e_boff = e_lits + rows + 1;
        const uint32_t s_voff = al64(e_boff), S1 = al64(rows + 1);
        const uint32_t e_voff = s_voff + (uint32_t)V.nvar * S1;
        const uint32_t S0 = al64(rows);
        const uint32_t e_vld = e_voff + (uint32_t)V.nval * S0;
        // fixed-region table, once per workgroup (lane r of wave 0; prefix by scan)
        if (wave == 0) {
            uint32_t nch = 0;
            uint64_t src = 0;
            if (lane < V.nfix) {
                src = (uint64_t)(uintptr_t)V.fix_ptr[lane] + lo * V.fix_w[lane];
                nch = (uint32_t)(((src & 15) + (uint64_t)rows * V.fix_w[lane] + 15) >> 4);
            }
            const uint32_t incl = wave_incl_scan(nch, lane);
            if (lane < V.nfix) {
                freg[lane] = u32x4{(uint32_t)(src & ~15ull), (uint32_t)(src >> 32), incl - nch, V.fix_lds[lane]};
                fmis[lane] = V.fix_lds[lane] + (uint32_t)(src & 15);
            }
            if (lane == 63) misc[15] = incl;
        }
        __syncthreads();
        const uint32_t fix_ch = misc[15];
        const uint32_t E = e_vld + fix_ch;
        for (uint32_t e0 = tid; e0 < E; e0 += kVBatch * kBlock) {
            u32x4 v[kVBatch];
            uint32_t dst[kVBatch], kind[kVBatch];  // kind: 1 dword, 2 qword, 3 byte, 4 16-B chunk
#pragma unroll
            for (int m = 0; m < kVBatch; m++) {
                const uint32_t e = e0 + m * kBlock;
                kind[m] = 0;
                dst[m] = 0;
                v[m] = u32x4{0u, 0u, 0u, 0u};
                if (e >= E) continue;
                if (e < e_lits) {
                    const uint32_t* src;
                    uint32_t x;
                    if (e < e_items) { src = (const uint32_t*)P.items; x = e; dst[m] = L.items + 4 * x; }
                    else if (e < e_hdrs) { src = (const uint32_t*)P.hdrs; x = e - e_items; dst[m] = L.hdrs + 4 * x; }
                    else if (e < e_conts) { src = (const uint32_t*)P.conts; x = e - e_hdrs; dst[m] = L.conts + 4 * x; }
                    else if (e < e_ipk) { src = P.ipk; x = e - e_conts; dst[m] = L.ipk + 4 * x; }
                    else if (e < e_ihr) { src = P.ihr; x = e - e_ipk; dst[m] = L.ihr + 4 * x; }
                    else { src = (const uint32_t*)P.lits; x = e - e_ihr; dst[m] = L.lits + 4 * x; }
                    v[m].x = ((g_u32*)src)[x];
                    kind[m] = 1;
                } else if (e < e_boff) {
                    const uint32_t j = e - e_lits;
                    const uint64_t o = ((g_u64*)offs)[lo + j];
                    v[m].x = (uint32_t)o;
                    v[m].y = (uint32_t)(o >> 32);
                    dst[m] = L.boff + 8 * j;
                    kind[m] = 2;
                } else if (e < s_voff) {
                    continue;
                } else if (e < e_voff) {
                    const uint32_t x = e - s_voff;
                    const uint32_t vv = __builtin_amdgcn_readfirstlane(x / S1), j = x - vv * S1;
                    if (j > rows) continue;
                    v[m].x = ((g_u32*)V.var_off[vv])[lo + j];
                    dst[m] = L.voff + 4 * (vv * (VT + 1) + j);
                    kind[m] = 1;
                } else if (e < e_vld) {
                    const uint32_t x = e - e_voff;
                    const uint32_t vv = __builtin_amdgcn_readfirstlane(x / S0), j = x - vv * S0;
                    if (j >= rows) continue;
                    v[m].x = ((g_u8*)V.val_ptr[vv])[lo + j];
                    dst[m] = L.vld + vv * VT + j;
                    kind[m] = 3;
                } else {
                    const uint32_t c = e - e_vld;
                    u32x4 g = freg[0];
                    for (int r = 1; r < V.nfix; r++) {
                        const u32x4 h = freg[r];
                        if (c >= h.z) g = h;
                    }
                    const uint64_t a0 = ((uint64_t)g.y << 32) | g.x;
                    v[m] = *(const g_u32x4*)(uintptr_t)(a0 + 16ull * (c - g.z));
                    dst[m] = L.stg + g.w + 16 * (c - g.z);
                    kind[m] = 4;
                }
            }
#pragma unroll
            for (int m = 0; m < kVBatch; m++) {
                switch (kind[m]) {
                    case 1: *(uint32_t*)(lds + dst[m]) = v[m].x; break;
                    case 2: *(uint64_t*)(lds + dst[m]) = ((uint64_t)v[m].y << 32) | v[m].x; break;
                    case 3: lds[dst[m]] = (uint8_t)v[m].x; break;
                    case 4: *(u32x4*)(lds + dst[m]) = v[m]; break;
                    default: break;
                }
            }
        }
        if (tid < 8) misc[tid] = 0;  // misc[15] (fixed chunk count) stays
    }
    __syncthreads();
    mark(0);
    // ---- round 2: var staging plan + loads, positions while they fly --------
    uint32_t any_direct = 0, vch = 0;
    {
        uint32_t used = (uint32_t)V.fix_bytes;
        for (int vv = 0; vv < V.nvar; vv++) {
            const uint32_t* vo = voff + vv * (VT + 1);
            const uint64_t src = (uint64_t)(uintptr_t)(V.var_data[vv] + vo[0]);
            const uint32_t bytes = vo[rows] - vo[0];
            const uint32_t nch = bytes ? (uint32_t)(((src & 15) + bytes + 15) >> 4) : 0u;
            const bool st = used + 16 * nch <= in_bud;
            if (tid == 0) vvar[vv] = VVar{src, st ? used : UINT32_MAX, 0};
            if (st) { used += 16 * nch; vch += nch; } else any_direct = 1;
        }
    }
    u32x4 vb[kVBatch];
    uint32_t vdst[kVBatch];
    auto var_load = [&](uint32_t c0) {
#pragma unroll
        for (int m = 0; m < kVBatch; m++) {
            const uint32_t c = c0 + m * kBlock;
            uint64_t a0 = 0;
            uint32_t cb = 0, base = 0, sl = 0, u2 = (uint32_t)V.fix_bytes;
            for (int vv = 0; vv < V.nvar; vv++) {
                const uint32_t* vo = voff + vv * (VT + 1);
                const uint64_t src = (uint64_t)(uintptr_t)(V.var_data[vv] + vo[0]);
                const uint32_t bytes = vo[rows] - vo[0];
                const uint32_t nch = bytes ? (uint32_t)(((src & 15) + bytes + 15) >> 4) : 0u;
                if (u2 + 16 * nch > in_bud) continue;  // not staged (same rule as the plan)
                const bool in = c >= base;
                a0 = in ? (src & ~15ull) : a0;
                cb = in ? base : cb;
                sl = in ? u2 : sl;
                base += nch;
                u2 += 16 * nch;
            }
            vdst[m] = sl + 16 * (c - cb);
            if (c < vch) vb[m] = *(const g_u32x4*)(uintptr_t)(a0 + 16ull * (c - cb));
        }
    };
    auto var_store = [&](uint32_t c0) {
#pragma unroll
        for (int m = 0; m < kVBatch; m++)
            if (c0 + m * kBlock < vch) *(u32x4*)(stg + vdst[m]) = vb[m];
    };
    var_load(tid);
    // presence masks and item positions (LDS only)
    if (V.nval == 0) {
        // no validity columns: every container and leaf is present, so an
        // item's size is static or its var value's length
        const uint64_t pm_all = P.n_conts >= 64 ? ~0ull : ((1ull << P.n_conts) - 1ull);
        for (uint32_t j = tid; j < rows; j += kBlock) {
            pmk[j] = pm_all;
            bst[j] = 0;
            uint32_t p = 0;
            uint16_t* pj = pos + j * NP;
            for (int k = 0; k < NI; k++) {
                const uint32_t x = ipk[k], vs = (x >> 16) & 0xFFu;
                uint32_t sz = x & 0xFFFFu;
                if (vs != 0xFFu) {
                    const uint32_t* vo = voff + vs * (VT + 1);
                    sz = vo[j + 1] - vo[j];
                    if (sz > 0xFFFFu) sz = 0x10000u;
                }
                pj[k] = (uint16_t)p;
                p += sz;
            }
            pj[NI] = (uint16_t)p;
            if (p > 0xFFFFu || boff[j + 1] - boff[j] != p || boff[j] + p > cap) atomicOr(&misc[0], 1u);
        }
    } else
    for (uint32_t j = tid; j < rows; j += kBlock) {
        uint64_t pm = 0;
        for (int c = 0; c < P.n_conts; c++) {
            const EncCont ct = conts[c];
            bool p = ct.parent < 0 ? true : ((pm >> ct.parent) & 1ull);
            if (p && ct.valid_col >= 0) {
                const int vs = V.col_val[ct.valid_col];
                if (vs >= 0) p = vld[vs * VT + j] != 0;
            }
            if (p) pm |= 1ull << c;
        }
        pmk[j] = pm;
        bst[j] = 0;
        uint32_t p = 0, slack = 0;
        uint16_t* pj = pos + j * NP;
        for (int k = 0; k < NI; k++) {
            const EncItem it = items[k];
            uint32_t sz = 0;
            if ((pm >> it.cont) & 1ull) {
                if (it.type == IT_VAR) {
                    const uint32_t* vo = voff + it.vslot * (VT + 1);
                    sz = vo[j + 1] - vo[j];
                } else {
                    sz = it.size;
                    if (it.type == IT_FIXED && it.nullable) {
                        const int vs = V.col_val[it.col];
                        if (vs >= 0 && !vld[vs * VT + j]) { sz = 0; slack += it.size; }
                    }
                }
            }
            pj[k] = (uint16_t)p;
            p += sz;
            if (sz > 0xFFFFu) p = 0x10000u;  // forces the fallback below
        }
        pj[NI] = (uint16_t)p;
        const uint32_t tot = p + (P.mode == PACKOS_MODE_PACKABLE ? slack : 0u);
        if (p > 0xFFFFu || boff[j + 1] - boff[j] != tot || boff[j] + tot > cap) atomicOr(&misc[0], 1u);
    }
    var_store(tid);
    for (uint32_t c0 = tid + kVBatch * kBlock; c0 < vch; c0 += kVBatch * kBlock) {
        var_load(c0);
        var_store(c0);
    }
    __syncthreads();
    mark(1);
    if (misc[0]) {  // outside the tile plan: one wavefront per blob, straight to HBM
        if (tid == 0) tflags[blockIdx.x] = 0u;
        uint32_t* wpos = (uint32_t*)obuf + wave * NP;
        for (uint32_t j = wave; j < rows; j += kWavesPerBlock)
            var_blob_wave(P, cols, lo + j, boff[j], out, cap, status, nullptr, wpos, lane);
        return;
    }
    uint32_t* L32 = (uint32_t*)lds;
    if (any_direct) {
        // ---- direct mode (long unstaged values, e.g. C5): no run buffer.  One
        // thread per blob streams the blob's non-value bytes (header words,
        // fixed and literal items, staged values) to HBM: whole dwords with
        // dword stores, dwords shared with a neighbour or a value hole byte by
        // byte.  k_var_copy then fills the holes.
        for (uint32_t j = tid; j < rows; j += kBlock) {
            const uint16_t* pj = pos + j * NP;
            const uint64_t g0 = boff[j];
            uint64_t acc = 0, D = g0 >> 2;
            uint32_t ph = (uint32_t)(g0 & 3), sb = ph, ovf = 0;
            auto flush_part = [&](uint32_t hi) {
                for (uint32_t y = sb; y < hi; y++) out[4 * D + y] = (uint8_t)(acc >> (8 * y));
            };
            auto put = [&](uint32_t v, uint32_t nb) {
                acc |= (uint64_t)v << (8 * ph);
                ph += nb;
                if (ph >= 4) {
                    if (sb == 0) *(uint32_t*)(out + 4 * D) = (uint32_t)acc;
                    else flush_part(4);
                    sb = 0;
                    D++;
                    acc >>= 32;
                    ph -= 4;
                }
            };
            for (int k = 0; k < NI; k++) {
                const uint32_t p0 = pj[k], len = (uint32_t)(pj[k + 1] - p0);
                if (len == 0) continue;
                const EncItem it = items[k];
                if (it.type == IT_HDR) {
                    const uint32_t hr = ihr[k], hb = hr & 0xFFFFu, cnt = hr >> 16;
                    for (uint32_t e = 0; e < cnt; e++) {
                        const EncHdr h = hdrs[hb + e];
                        uint16_t v;
                        if (h.relative) {
                            const int64_t off = (int64_t)pj[h.target] - (int64_t)(p0 + len);
                            ovf |= off >= 8192;
                            v = enc_header(off, h.tag);
                        } else {
                            v = h.value;
                            ovf |= h.ovf != 0;
                        }
                        put(v, 2);
                    }
                    continue;
                }
                uint32_t so;
                if (it.type == IT_CONST) {
                    so = L.lits + it.lit;
                } else if (it.type == IT_FIXED) {
                    so = L.stg + fmis[it.reg] + j * it.size;
                } else {
                    const VVar g = vvar[it.vslot];
                    const uint32_t* vo = voff + it.vslot * (VT + 1);
                    if (g.lds_off == UINT32_MAX) {  // hole for k_var_copy
                        if (ph > sb) flush_part(ph);
                        const uint64_t dn = 4 * D + ph + len;
                        D = dn >> 2;
                        ph = sb = (uint32_t)(dn & 3);
                        acc = 0;
                        continue;
                    }
                    so = L.stg + g.lds_off + (uint32_t)(g.src & 15) + (vo[j] - vo[0]);
                }
                if (it.is_bool) {
                    put(lds[so] != 0 ? 1u : 0u, 1);
                    continue;
                }
                for (uint32_t x = 0; x < len; x += 4) {
                    const uint32_t nb = min(4u, len - x);
                    const uint32_t sa = so + x, wi = sa >> 2;
                    uint32_t v = __builtin_amdgcn_alignbyte(L32[wi + 1], L32[wi], sa & 3);
                    if (nb < 4) v &= (1u << (8 * nb)) - 1u;
                    put(v, nb);
                }
            }
            const uint32_t tot = (uint32_t)(boff[j + 1] - boff[j]);
            for (uint32_t x = pj[NI]; x < tot; x += 4) put(0u, min(4u, tot - x));
            if (ph > sb) flush_part(ph);
            if (ovf) bst[j] |= 1u;
        }
        mark(2);
    } else {
    // ---- runs (everything staged, e.g. C3) --------------------------------------
    {
        const uint32_t j = tid;
        const uint32_t win = j < rows ? (uint32_t)((boff[j] - boff[0]) >> win_shift) : 0u;
        const uint32_t winp = (j > 0 && j < rows) ? (uint32_t)((boff[j - 1] - boff[0]) >> win_shift) : 0u;
        const bool isnew = j < rows && (j == 0 || win != winp);
        const uint64_t bal = __ballot(isnew);
        if (lane == 0) misc[4 + wave] = (uint32_t)__popcll(bal);
        __syncthreads();
        uint32_t base = 0, tot = 0;
        for (int w = 0; w < kWavesPerBlock; w++) {
            base += w < wave ? misc[4 + w] : 0u;
            tot += misc[4 + w];
        }
        if (isnew) subs[base + __popcll(bal & ((1ull << lane) - 1ull))] = j;
        if (tid == 0) {
            misc[1] = tot;
            subs[tot] = rows;
        }
    }
    __syncthreads();
    mark(2);
    const uint32_t nsub = misc[1];
    for (uint32_t q = 0; q < nsub; q++) {
        const uint32_t a = subs[q], b = subs[q + 1];
        const uint64_t s0 = boff[a], s1 = boff[b];
        const uint64_t al = s0 & ~15ull;
        const uint32_t nb = (uint32_t)(s1 - al);
        if (nb + 16 > bud) {
            uint32_t* wpos = (uint32_t*)obuf + wave * NP;
            for (uint32_t j = a + wave; j < b; j += kWavesPerBlock)
                var_blob_wave(P, cols, lo + j, boff[j], out, cap, status, nullptr, wpos, lane);
            for (uint32_t j = a + tid; j < b; j += kBlock) bst[j] = 2u;  // status written, bytes complete
            __syncthreads();
            continue;
        }
        const uint32_t nch = (nb + 15) >> 4;
        for (uint32_t c = tid; c < nch; c += kBlock) ((u32x4*)obuf)[c] = u32x4{0u, 0u, 0u, 0u};
        __syncthreads();
        mark(5);
        const uint32_t nbr = b - a, nb_mag = magic_of(nbr);
        // header words: (header, blob) pairs, OR-ed into the zeroed buffer
        for (uint32_t t = tid; t < nbr * (uint32_t)NH; t += kBlock) {
            const uint32_t hh = fast_div(t, nbr, nb_mag), j = a + (t - hh * nbr);
            const EncHdr h = hdrs[hh];
            if (!((pmk[j] >> h.cont) & 1ull)) continue;
            const uint16_t* pj = pos + j * NP;
            const uint32_t hpos = pj[h.hdr_item];
            uint16_t v;
            bool ovf;
            if (h.relative) {
                const int64_t off = (int64_t)pj[h.target] - (int64_t)(hpos + items[h.hdr_item].size);
                ovf = off >= 8192;
                v = enc_header(off, h.tag);
            } else {
                v = h.value;
                ovf = h.ovf != 0;
            }
            if (ovf) atomicOr(&bst[j], 1u);
            const uint32_t d = (uint32_t)(boff[j] - al) + hpos + 2 * h.j;
            const uint32_t sh = 8 * (d & 3);
            if (sh <= 16) {
                atomicOr(L32 + (d >> 2), (uint32_t)v << sh);
            } else {
                atomicOr(L32 + (d >> 2), ((uint32_t)v & 0xFFu) << 24);
                atomicOr(L32 + (d >> 2) + 1, (uint32_t)v >> 8);
            }
        }
        // items: (item, blob) pairs, item-major; whole destination dwords
        // stored, partial ones OR-ed; sources funnel-shifted from LDS
        for (uint32_t t = tid; t < nbr * (uint32_t)NI; t += kBlock) {
            const uint32_t k = fast_div(t, nbr, nb_mag), j = a + (t - k * nbr);
            const EncItem it = items[k];
            if (it.type == IT_HDR) continue;
            const uint16_t* pj = pos + j * NP;
            const uint32_t p0 = pj[k], len = (uint32_t)(pj[k + 1] - p0);
            if (len == 0) continue;
            const uint32_t d = (uint32_t)(boff[j] - al) + p0;
            uint32_t so;
            if (it.type == IT_CONST) {
                so = L.lits + it.lit;
            } else if (it.type == IT_FIXED) {
                so = L.stg + fmis[it.reg] + j * it.size;
            } else {
                const VVar g = vvar[it.vslot];
                so = L.stg + g.lds_off + (uint32_t)(g.src & 15) + (voff[it.vslot * (VT + 1) + j] - voff[it.vslot * (VT + 1)]);
            }
            if (it.is_bool) {
                atomicOr(L32 + (d >> 2), (uint32_t)(lds[so] != 0) << (8 * (d & 3)));
                continue;
            }
            const uint32_t D0 = d >> 2, D1 = (d + len - 1) >> 2;
            for (uint32_t D = D0; D <= D1; D++) {
                const uint32_t sa = so + 4 * D - d;
                const uint32_t wi = sa >> 2;
                const uint32_t v = __builtin_amdgcn_alignbyte(L32[wi + 1], L32[wi], sa & 3);
                const uint32_t b0 = 4 * D < d ? d - 4 * D : 0u, b1 = min(4u, d + len - 4 * D);
                if (b0 == 0 && b1 == 4) {
                    L32[D] = v;
                } else {
                    const uint32_t m = (b1 == 4 ? ~0u : ((1u << (8 * b1)) - 1u)) & ~((1u << (8 * b0)) - 1u);
                    atomicOr(L32 + D, v & m);
                }
            }
        }
        __syncthreads();
        mark(6);
        // write [s0, s1)
        for (uint32_t c = tid; c < nch; c += kBlock) {
            const uint64_t g0 = al + 16ull * c;
            if (g0 >= s0 && g0 + 16 <= s1) {
                __builtin_nontemporal_store(((const u32x4*)obuf)[c], (u32x4*)(out + g0));
            } else {
                for (int x = 0; x < 16; x++) {
                    const uint64_t gg = g0 + x;
                    if (gg >= s0 && gg < s1) out[gg] = obuf[16 * c + x];
                }
            }
        }
        __syncthreads();
        mark(7);
    }
    }
    mark(3);
    // ---- unstaged var values: hand their positions to k_var_copy -------------
    if (tid == 0) {
        uint32_t fl = 0;
        for (int vv = 0; vv < V.nvar; vv++) fl |= (vvar[vv].lds_off == UINT32_MAX ? 1u : 0u) << vv;
        tflags[blockIdx.x] = fl;
    }
    if (any_direct) {
        for (int vv = 0; vv < V.nvar; vv++) {
            if (vvar[vv].lds_off != UINT32_MAX) continue;
            const int k = V.var_item[vv];
            for (uint32_t j = tid; j < rows; j += kBlock)
                vpos[(uint64_t)vv * n + lo + j] = (bst[j] & 2u) ? (uint16_t)0xFFFFu : pos[j * NP + k];
        }
    }
    mark(4);
    if (status)
        for (uint32_t j = tid; j < rows; j += kBlock)
            if (!(bst[j] & 2u)) status[lo + j] = (bst[j] & 1u) ? PACKOS_STATUS_OVERFLOW13 : 0u;
}

// Long var values the tile kernel did not stage: a flattened memmove per
// tile over 16-B-aligned destination chunks, consecutive lanes on
// consecutive chunks.  A chunk wholly inside one value takes two aligned 16-B
// source loads, a funnel shift and one 16-B store; the (at most two) edge
// chunks of a value go byte by byte.  Runs after k_encode_var_tile, which
// skipped the whole chunks and wrote the edge chunks' other bytes.
constexpr int kCopyBatch = 4;
// (Measured on MI355X, C5: loading a whole chunk's source with one dwordx4
// at a byte-misaligned address is 1.5x slower, at a dword-aligned address
// 1.3x slower, than two 16-B-aligned loads + the funnel below.)

__device__ __forceinline__ uint32_t sel4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return q == 0 ? a : q == 1 ? b : q == 2 ? c : d;
}

template <int VT>
__global__ __launch_bounds__(kBlock) void k_var_copy(VarPlan V, const uint64_t* __restrict__ offs,
                                                     const uint32_t* __restrict__ tflags,
                                                     const uint16_t* __restrict__ vpos, uint8_t* __restrict__ out,
                                                     uint64_t n) {
    __shared__ uint64_t boff[VT + 1];
    __shared__ uint32_t vo[VT + 1], uo[VT + 1];
    __shared__ uint16_t ps[VT];
    __shared__ uint32_t wsum[kWavesPerBlock];
    const uint32_t fl = tflags[blockIdx.x];
    if (!fl) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t lo = (uint64_t)blockIdx.x * VT;
    const uint32_t rows = (uint32_t)min((uint64_t)VT, n - lo);
    for (uint32_t j = tid; j <= rows; j += kBlock) boff[j] = offs[lo + j];
    for (int v = 0; v < V.nvar; v++) {
        if (!((fl >> v) & 1u)) continue;
        const uint32_t* voff_g = V.var_off[v];
        for (uint32_t j = tid; j <= rows; j += kBlock) vo[j] = voff_g[lo + j];
        for (uint32_t j = tid; j < rows; j += kBlock) ps[j] = vpos[(uint64_t)v * n + lo + j];
        __syncthreads();
        {
            const uint32_t j = tid;
            uint32_t cnt = 0;
            if (j < rows && ps[j] != 0xFFFFu) {
                const uint64_t d0 = boff[j] + ps[j];
                const uint32_t len = vo[j + 1] - vo[j];
                cnt = len ? (uint32_t)(((d0 + len + 15) >> 4) - (d0 >> 4)) : 0u;
            }
            const uint32_t incl = wave_incl_scan(cnt, lane);
            if (lane == 63) wsum[wave] = incl;
            __syncthreads();
            uint32_t wb = 0, tot = 0;
            for (int w = 0; w < kWavesPerBlock; w++) {
                wb += w < wave ? wsum[w] : 0u;
                tot += wsum[w];
            }
            if (j < rows) uo[j] = wb + incl - cnt;
            if (tid == 0) uo[rows] = tot;
            __syncthreads();
        }
        const uint32_t U = uo[rows];
        const uint8_t* col = V.var_data[v];
        // each wavefront takes 64 * kCopyBatch consecutive units per step; one
        // (wave-uniform) binary search for the step's first unit, then each
        // lane walks forward to its units' blobs
        for (uint32_t ub = wave * (kWave * kCopyBatch); ub < U; ub += kWavesPerBlock * kWave * kCopyBatch) {
            uint32_t jw;
            {
                uint32_t l = 0, r = rows - 1;  // last blob j with uo[j] <= ub
                while (l < r) {
                    const uint32_t mm = (l + r + 1) >> 1;
                    if (uo[mm] <= ub) l = mm; else r = mm - 1;
                }
                jw = l;
            }
            u32x4 a[kCopyBatch], b[kCopyBatch];
            uint64_t dst[kCopyBatch];
            uint32_t sh[kCopyBatch], k0[kCopyBatch], k1[kCopyBatch];
            uint32_t j = jw;
#pragma unroll
            for (int m = 0; m < kCopyBatch; m++) {
                const uint32_t u = ub + lane + kWave * m;
                k0[m] = k1[m] = 0;
                sh[m] = 0;
                dst[m] = 0;
                a[m] = b[m] = u32x4{0u, 0u, 0u, 0u};
                if (u >= U) continue;
                while (uo[j + 1] <= u) j++;
                const uint64_t d0 = boff[j] + ps[j];
                const uint32_t ln = vo[j + 1] - vo[j];
                const uint64_t C = 16 * ((d0 >> 4) + (u - uo[j]));
                dst[m] = C;
                k0[m] = C >= d0 ? 0u : (uint32_t)(d0 - C);
                k1[m] = (uint32_t)min((uint64_t)16, d0 + ln - C);
                const uintptr_t xa = (uintptr_t)(col + vo[j]) + (uintptr_t)(C - d0);
                // aligned blocks holding needed bytes only (edge chunks may need one)
                const g_u32x4* xw = (const g_u32x4*)(xa & ~(uintptr_t)15);
                sh[m] = (uint32_t)(xa & 15);
                if (k0[m] < 16 - sh[m]) a[m] = xw[0];
                if (sh[m] && k1[m] > 16 - sh[m]) b[m] = xw[1];
            }
#pragma unroll
            for (int m = 0; m < kCopyBatch; m++) {
                if (k1[m] <= k0[m]) continue;
                u32x4 o4;
                if (sh[m] == 0) {
                    o4 = a[m];
                } else {
                    const uint32_t q = sh[m] >> 2, sb = sh[m] & 3;
                    const uint32_t w[8] = {a[m].x, a[m].y, a[m].z, a[m].w, b[m].x, b[m].y, b[m].z, b[m].w};
                    uint32_t t5[5];
#pragma unroll
                    for (int i = 0; i < 5; i++) t5[i] = sel4(q, w[i], w[i + 1], w[i + 2], w[i + 3]);
                    o4.x = __builtin_amdgcn_alignbyte(t5[1], t5[0], sb);
                    o4.y = __builtin_amdgcn_alignbyte(t5[2], t5[1], sb);
                    o4.z = __builtin_amdgcn_alignbyte(t5[3], t5[2], sb);
                    o4.w = __builtin_amdgcn_alignbyte(t5[4], t5[3], sb);
                }
                if (k0[m] == 0 && k1[m] == 16) {
                    __builtin_nontemporal_store(o4, (u32x4*)(out + dst[m]));
                } else {
                    const uint32_t wv[4] = {o4.x, o4.y, o4.z, o4.w};
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const uint32_t lo4 = 4 * i, s4 = max(k0[m], lo4), e4 = min(k1[m], lo4 + 4);
                        if (s4 >= e4) continue;
                        if (s4 == lo4 && e4 == lo4 + 4) {
                            *(uint32_t*)(out + dst[m] + lo4) = wv[i];
                        } else {
                            for (uint32_t y = s4; y < e4; y++) out[dst[m] + y] = (uint8_t)(wv[i] >> (8 * (y - lo4)));
                        }
                    }
                }
            }
        }
        __syncthreads();
    }
}

#include "encode_stream.inc"

// =========================================================================
// decode: schema.DecodeBuffer, one thread per blob
// =========================================================================
constexpr int kDecDepth = 8;

struct DSeq {
    int64_t len, base, count, pos, next_off, cur_off;
    uint64_t start;     // absolute arena offset of this (sub)buffer
    int next_type, cur_type;
};

__host__ __device__ __forceinline__ uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }

// Byte readers for the decoder: straight from the arena, or from a per-blob
// LDS window (the blob's first W bytes) with the arena behind it.
struct GReader {
    const uint8_t* a;
    __host__ __device__ __forceinline__ uint32_t operator()(uint64_t p) const { return a[p]; }
};
struct WReader {
    const uint8_t* a;
    const uint8_t* win;   // LDS copy of arena[base, base + W)
    uint64_t base;
    uint32_t W;
    __device__ __forceinline__ uint32_t operator()(uint64_t p) const {
        const uint64_t d = p - base;
        return d < W ? win[d] : a[p];
    }
};
template <class R>
__host__ __device__ __forceinline__ uint16_t rd16r(const R& r, uint64_t p) { return (uint16_t)(r(p) | (r(p + 1) << 8)); }

// NewSeqGetAccess (seqget.go:22-47)
template <class R>
__host__ __device__ __forceinline__ int dseq_init(DSeq& s, const R& a, uint64_t start, int64_t len) {
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

// w bytes from reader position p to a column row; dword stores when aligned
template <class R>
__host__ __device__ __forceinline__ void copy_out(uint8_t* dst, const R& r, uint64_t p, uint32_t w) {
    if ((w & 3) == 0 && ((uintptr_t)dst & 3) == 0) {
        for (uint32_t j = 0; j < w; j += 4)
            *(uint32_t*)(dst + j) = r(p + j) | (r(p + j + 1) << 8) | (r(p + j + 2) << 16) | (r(p + j + 3) << 24);
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
template <class R>
__host__ __device__ uint32_t decode_blob(const DecProgram& P, const DecCols& cols, const R& arena, uint64_t a0,
                                         uint64_t a1, uint64_t i) {
    // the current frame lives in registers; outer frames are spilled to `stk`
    // (scratch) only while a nested tuple/map is being read
    Frame cur;
    Frame stk[kDecDepth];
    int d = 0;
    if (dseq_init(cur.q, arena, a0, (int64_t)(a1 - a0)))
        return (uint32_t)PACKOS_ERR_INVALID_FORMAT;  // position -1
    cur.node = P.root;
    cur.k = 0;
    int err = 0;
    for (;;) {
        const DecNode fn = P.nodes[cur.node];
        if (cur.k >= fn.nkids) {
            if (d == 0) break;
            // container finished: mark it present, then Advance the parent past it
            if (cols.valid[fn.col]) cols.valid[fn.col][i] = 1;
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
            err = dprecheck(q, nd.tag, -1, nd.nullable, w);
            if (err) break;
            if (nd.kind == K_MAP && (nd.nkids & 1)) { err = 3; break; }
            if (w != 0) {
                // PeekNestedSeq (seqget.go:105-121)
                if (q.next_off - q.cur_off <= 0 || q.next_off > q.len) { err = 1; break; }
                if (d + 1 >= kDecDepth) { err = 1; break; }
                Frame c;
                if (dseq_init(c.q, arena, q.start + q.cur_off, q.next_off - q.cur_off)) { err = 1; break; }
                if (nd.kind == K_TUPLE && nd.nkids > 0 && (c.q.count - 1) != nd.nkids && !nd.variable) {
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
            if (cols.valid[nd.col]) cols.valid[nd.col][i] = 0;  // nil container
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
        switch (nd.kind) {
            case K_INT: case K_UINT: case K_FLOAT: case K_BOOL: {
                if (ps < 0) {
                    if (cols.valid[nd.col]) cols.valid[nd.col][i] = 0;
                    break;
                }
                if (w < nd.width) { err = kPanic; break; }  // LittleEndian.UintXX on a short slice
                uint8_t* dstp = cols.data[nd.col] + i * (uint64_t)nd.width;
                if (nd.kind == K_BOOL) dstp[0] = arena(pay) != 0;
                else copy_out(dstp, arena, pay, (uint32_t)nd.width);
                if (cols.valid[nd.col]) cols.valid[nd.col][i] = 1;
                break;
            }
            case K_STRING: case K_BYTES:
                if (nd.width > 0) {
                    uint8_t* dstp = cols.data[nd.col] + i * (uint64_t)nd.width;
                    copy_out(dstp, arena, pay, (uint32_t)nd.width);
                } else {
                    cols.start[nd.col][i] = ps < 0 ? 0ull : q.start + (uint64_t)ps;
                    cols.length[nd.col][i] = ps < 0 ? 0u : (uint32_t)w;
                }
                break;
            case K_MATCH: {
                const uint32_t have = ps < 0 ? 0u : (uint32_t)w;
                bool eq = have == nd.lit_len;
                for (uint32_t j = 0; eq && j < have; j++) eq = arena(pay + j) == P.lits[nd.lit + j];
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
        if (err == kPanic) sv = PACKOS_STATUS_PANIC | posv;
        else sv = (uint32_t)(d == 0 ? err : PACKOS_ERR_INVALID_FORMAT) | posv;
    }
    return sv;
}

// generic decode: one thread per blob
__global__ __launch_bounds__(kBlock) void k_decode(DecProgram P, DecCols cols, const uint8_t* __restrict__ arena,
                                                   const uint64_t* __restrict__ offs, uint64_t stride, uint64_t n,
                                                   uint32_t* __restrict__ status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a0 = offs ? offs[i] : i * stride;
    const uint64_t a1 = offs ? offs[i + 1] : (i + 1) * stride;
    status[i] = decode_blob(P, cols, GReader{arena}, a0, a1, i);
}

// Generic decode with a per-blob LDS window: every thread first fetches its
// blob's first kDecWinChunks x 16 bytes (header block, leading fields) with
// 16-B loads, all in flight, then runs decode_blob reading the window and
// falling back to HBM only beyond it.  Replaces ~one dependent global byte
// load per header word / payload byte with one load round.
constexpr int kDecWinChunks = 8;

__global__ __launch_bounds__(kBlock) void k_decode_win(DecProgram P, DecCols cols, const uint8_t* __restrict__ arena,
                                                       const uint64_t* __restrict__ offs, uint64_t stride, uint64_t n,
                                                       uint32_t* __restrict__ status) {
    __shared__ __attribute__((aligned(16))) uint8_t win[kBlock * kDecWinChunks * 16];
    extern __shared__ __attribute__((aligned(16))) uint8_t ptab[];   // decode program copy (nodes | kids | lits)
    const int tid = threadIdx.x;
    // the program is read once per visited field: keep it in LDS
    DecNode* lnodes = (DecNode*)ptab;
    int32_t* lkids = (int32_t*)(ptab + ((P.n_nodes * sizeof(DecNode) + 15) & ~15));
    uint8_t* llits = (uint8_t*)lkids + ((P.n_kids * 4 + 15) & ~15);
    for (int x = tid; x < P.n_nodes; x += kBlock) lnodes[x] = P.nodes[x];
    for (int x = tid; x < P.n_kids; x += kBlock) lkids[x] = P.kids[x];
    for (int x = tid; x < P.n_lits; x += kBlock) llits[x] = P.lits[x];
    const uint64_t lo = (uint64_t)blockIdx.x * kBlock, i = lo + tid;
    const uint32_t rows = (uint32_t)min((uint64_t)kBlock, n - lo);
    uint64_t a0 = 0, a1 = 0;
    if (i < n) {
        a0 = offs ? offs[i] : i * stride;
        a1 = offs ? offs[i + 1] : (i + 1) * stride;
    }
    // Small blobs: when the tile's whole byte range fits the window memory,
    // stage it once with coalesced LDS-DMA and let every blob read from there
    // (same reader, one shared window).  Otherwise each blob's first
    // kDecWinChunks * 16 bytes go to its own window (headers + fixed fields sit
    // at the front; var values are returned as views and never read).
    typedef __attribute__((address_space(4))) const uint64_t c_u64;
    const uint64_t t0 = offs ? ((c_u64*)(uintptr_t)offs)[lo] : lo * stride;
    const uint64_t t1 = offs ? ((c_u64*)(uintptr_t)offs)[lo + rows] : (lo + rows) * stride;
    const uint64_t tb = t0 & ~15ull;
    const bool tile_mode = t1 >= t0 && t1 - tb <= (uint64_t)sizeof(win) && ((uintptr_t)arena & 15) == 0;
    uint8_t* w;
    uint64_t b0;
    uint32_t wbytes;
    if (tile_mode) {
        const uint32_t nch = (uint32_t)((t1 - tb + 15) >> 4), lane = tid & 63, c00 = tid & ~63u;
        const uint32_t lds0 = (uint32_t)(uintptr_t)win;
        for (uint32_t c0 = c00; c0 < nch; c0 += kBlock)
            if (c0 + lane < nch) dma16(arena + tb + 16u * (c0 + lane), __builtin_amdgcn_readfirstlane(lds0 + 16u * c0));
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        w = win;
        b0 = tb;
        wbytes = 16 * nch;
    } else {
        w = win + tid * kDecWinChunks * 16;
        b0 = a0 & ~15ull;
        const uint64_t end = min(a1, b0 + 16ull * kDecWinChunks);
        const uint32_t nch = (i < n && end > a0) ? (uint32_t)((end - b0 + 15) >> 4) : 0u;
        u32x4 v[kDecWinChunks];
#pragma unroll
        for (int c = 0; c < kDecWinChunks; c++)
            if ((uint32_t)c < nch) v[c] = *(const g_u32x4*)(arena + b0 + 16 * c);
#pragma unroll
        for (int c = 0; c < kDecWinChunks; c++)
            if ((uint32_t)c < nch) *(u32x4*)(w + 16 * c) = v[c];
        wbytes = 16 * nch;
    }
    __syncthreads();
    if (i >= n) return;
    const WReader R{arena, w, b0, wbytes};
    const DecProgram LP{lnodes, lkids, llits, P.root, P.n_nodes, P.n_kids, P.n_lits};
    status[i] = decode_blob(LP, cols, R, a0, a1, i);
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
struct DecColsK {
    uint8_t* dst[kDecK];
    uint32_t width[kDecK], blob_off[kDecK], flags[kDecK], magic[kDecK];
    int32_t n;
};

__device__ __forceinline__ uint32_t lds_u8(const uint32_t* lds, uint32_t a) { return (lds[a >> 2] >> (8 * (a & 3))) & 0xFFu; }

__global__ __launch_bounds__(kBlock) void k_decode_fixed(DecFixProgram F, DecProgram P, DecCols cols, DecColsK K,
                                                         const uint8_t* __restrict__ arena,
                                                         const uint64_t* __restrict__ offs, uint64_t n,
                                                         uint32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds_raw[];
    uint32_t* lds = (uint32_t*)lds_raw;
    const uint32_t B = (uint32_t)F.B, T = (uint32_t)F.T, QW = (B + 3) >> 2;
    const uint64_t blob0 = (uint64_t)blockIdx.x * T;
    const uint32_t rows = (uint32_t)min((uint64_t)T, n - blob0);
    const int tid = threadIdx.x;
    uint32_t* chk = lds + (T * B / 4 + 4);
    uint32_t* fail = chk + 3 * QW;

    // the tile base is one scalar load; whether the tile's blobs really lie
    // back to back at stride B is checked while the staging DMA is in flight
    typedef __attribute__((address_space(4))) const uint64_t c_u64;
    const uint64_t base = offs ? ((c_u64*)(uintptr_t)offs)[blob0] : blob0 * B;
    const bool aligned_base = (base & 15) == 0;
    bool ok = true;
    for (uint32_t q = tid; q < 3u * (uint32_t)F.n_chk; q += kBlock) chk[q] = F.chk[q];
    for (uint32_t j = tid; j < rows; j += kBlock) fail[j] = 0;
    // 1. stage: global -> LDS with global_load_lds_dwordx4 (every chunk of the
    //    tile in flight at once; a load -> ds_write loop waits per chunk)
    const uint32_t bytes = rows * B;
    if (aligned_base) {
        const uint8_t* src = arena + base;
        const uint32_t n16 = bytes >> 4, lane = tid & 63, c00 = tid & ~63u;
        const uint32_t lds0 = (uint32_t)(uintptr_t)lds_raw;
        for (uint32_t c0 = c00; c0 < n16; c0 += kBlock)
            if (c0 + lane < n16) dma16(src + 16u * (c0 + lane), __builtin_amdgcn_readfirstlane(lds0 + 16u * c0));
        for (uint32_t k = n16 * 16 + tid; k < bytes; k += kBlock) lds_raw[k] = src[k];
    }
    if (offs) {
        for (uint32_t j = tid; j <= rows; j += kBlock) ok &= offs[blob0 + j] == base + (uint64_t)j * B;
        ok &= aligned_base;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!__syncthreads_and(ok)) {
        for (uint32_t j = tid; j < rows; j += kBlock) {
            const uint64_t i = blob0 + j;
            status[i] = decode_blob(P, cols, GReader{arena}, offs ? offs[i] : i * B, offs ? offs[i + 1] : (i + 1) * B, i);
        }
        return;
    }
    // 2. constant-byte check, over the blob dwords that HOLD constant bytes
    //    (header words, literals: 5 of 64 for metric M; list built at compile)
    {
        const uint32_t nq = (uint32_t)F.n_chk;
        const uint32_t nq_magic = nq > 1 ? (uint32_t)((0x100000000ull + nq - 1) / nq) : 0u;
        for (uint32_t e = tid; e < rows * nq; e += kBlock) {
            const uint32_t j = nq > 1 ? __umulhi(e, nq_magic) : e;
            const uint32_t* c = chk + 3 * (e - j * nq);
            const uint32_t a = j * B + 4 * c[0];   // blob dword q (B % 4 == 0: aligned)
            const uint32_t v = (B & 3) == 0 ? lds[a >> 2] : lds_bytes4(lds, a);
            if ((v & c[1]) != c[2]) fail[j] = 1;
        }
    }
    // 3. columns: uniform walk over the columns; threads stride the column's
    //    output dwords (consecutive lanes -> consecutive dwords: 256-B stores)
    for (int c = 0; c < K.n; c++) {
        struct { uint8_t* dst; uint32_t blob_off, flags, magic; } L = {K.dst[c], K.blob_off[c], K.flags[c], K.magic[c]};
        const uint32_t w = K.width[c], R = rows * w, D = R >> 2;
        uint32_t* dst = (uint32_t*)(L.dst + blob0 * w);   // 4-B aligned: T*w % 4 == 0, base 16-B aligned
        if ((w & 3) == 0) {
            for (uint32_t d = tid; d < D; d += kBlock) {
                const uint32_t b = 4 * d;
                const uint32_t j = __umulhi(b, L.magic);
                const uint32_t a = j * B + L.blob_off + (b - j * w);
                __builtin_nontemporal_store(lds_bytes4(lds, a), dst + d);
            }
        } else if (w == 2) {   // a dword = rows 2d, 2d+1
            for (uint32_t d = tid; d < D; d += kBlock) {
                const uint32_t a = 2 * d * B + L.blob_off;
                const uint32_t x = (lds_bytes4(lds, a) & 0xFFFFu) | (lds_bytes4(lds, a + B) << 16);
                __builtin_nontemporal_store(x, dst + d);
            }
        } else if (w > 4 && !(L.flags & 1u)) {   // most dwords sit inside one row
            for (uint32_t d = tid; d < D; d += kBlock) {
                const uint32_t b = 4 * d;
                const uint32_t j = __umulhi(b, L.magic);
                const uint32_t r = b - j * w;
                uint32_t x;
                if (r + 4 <= w) {
                    x = lds_bytes4(lds, j * B + L.blob_off + r);
                } else {
                    const uint32_t k = w - r;   // 1..3 bytes of row j, then row j + 1
                    x = (lds_bytes4(lds, j * B + L.blob_off + r) & ((1u << (8 * k)) - 1u)) |
                        (lds_bytes4(lds, (j + 1) * B + L.blob_off) << (8 * k));
                }
                __builtin_nontemporal_store(x, dst + d);
            }
        } else {
            for (uint32_t d = tid; d < D; d += kBlock) {
                uint32_t x = 0;
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    const uint32_t b = 4 * d + y;
                    const uint32_t j = w > 1 ? __umulhi(b, L.magic) : b;
                    uint32_t v = lds_u8(lds, j * B + L.blob_off + (b - j * w));
                    if (L.flags & 1u) v = v != 0;
                    x |= v << (8 * y);
                }
                __builtin_nontemporal_store(x, dst + d);
            }
        }
        // ragged tail (R % 4 bytes, last tile only)
        for (uint32_t b = 4 * D + tid; b < R; b += kBlock) {
            const uint32_t j = w > 1 ? __umulhi(b, L.magic) : b;
            uint32_t v = lds_u8(lds, j * B + L.blob_off + (b - j * w));
            if (L.flags & 1u) v = v != 0;
            L.dst[blob0 * w + b] = (uint8_t)v;
        }
    }
    // 4. validity (every node is present in the canonical layout)
    for (int c = 0; c < F.n_all_cols; c++)
        if (cols.valid[c])
            for (uint32_t j = tid; j < rows; j += kBlock) cols.valid[c][blob0 + j] = 1;
    __syncthreads();
    for (uint32_t j = tid; j < rows; j += kBlock) {
        const uint64_t i = blob0 + j;
        uint32_t sv = 0;
        if (fail[j]) sv = decode_blob(P, cols, GReader{arena}, offs ? offs[i] : i * B, offs ? offs[i + 1] : (i + 1) * B, i);
        status[i] = sv;
    }
}

// =========================================================================
// GetAccess gather
// =========================================================================
struct DGet {
    uint64_t start;
    int64_t len, base, argc;
};
__device__ __forceinline__ bool dget_init(DGet& g, const uint8_t* a, uint64_t start, int64_t len) {
    if (len < 2) return false;
    g.base = rd16(a + start) >> 3;
    if (len < g.base) return false;
    g.start = start; g.len = len; g.argc = g.base / 2 - 1;
    return true;
}
// rangeAt (get.go:38-58)
__device__ __forceinline__ void dget_range(const DGet& g, const uint8_t* a, int64_t pos, int& tp, int64_t& s,
                                           int64_t& e) {
    if (pos >= g.argc) { tp = 0; s = -2; e = -1; return; }
    const uint16_t h1 = rd16(a + g.start + pos * 2), h2 = rd16(a + g.start + (pos + 1) * 2);
    s = h1 >> 3; tp = h1 & 7;
    e = (h2 >> 3) + g.base;
    if (pos > 0) s += g.base;
    if (e > g.len) e = -1;
}

struct PathArg {
    int32_t p[16];
};

__global__ __launch_bounds__(kBlock) void k_get_field(const uint8_t* __restrict__ arena, const uint64_t* __restrict__ offs,
                                                      uint64_t stride, uint64_t n, PathArg path, int depth, int want_tag, int want_width, uint64_t* out_start,
                                                      uint32_t* out_len, uint8_t* out_tag, uint8_t* status) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t a0 = offs ? offs[i] : i * stride;
    const uint64_t a1 = offs ? offs[i + 1] : (i + 1) * stride;
    out_start[i] = 0; out_len[i] = 0; out_tag[i] = 0;
    DGet g;
    if (!dget_init(g, arena, a0, (int64_t)(a1 - a0))) { status[i] = 3; return; }
    int tp; int64_t s, e;
    for (int d = 0; d < depth - 1; d++) {
        dget_range(g, arena, path.p[d], tp, s, e);
        if (e < s || (tp != 7 && tp != 4)) { status[i] = 1; return; }
        if (e == s) { status[i] = 2; return; }
        DGet nx;
        if (!dget_init(nx, arena, g.start + (uint64_t)s, e - s)) { status[i] = 3; return; }
        g = nx;
    }
    dget_range(g, arena, path.p[depth - 1], tp, s, e);
    out_tag[i] = (uint8_t)tp;
    const bool ok = want_width >= 0 ? (tp == want_tag && e - s == want_width) : (tp == want_tag && e >= s);
    if (!ok) { status[i] = 1; return; }
    out_start[i] = g.start + (uint64_t)s;
    out_len[i] = (uint32_t)(e - s);
    status[i] = 0;
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
    DecProgram P{s->dnodes.data(), s->dkids.data(), s->lits.data(), 0, (int32_t)s->dnodes.size(),
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
        ec.off[c] = cols[c].offsets;
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
    t.dfix.cols = (const DecFix*)(b + o_dfix);
    t.dfix.chk = (const uint32_t*)(b + o_dchk);
    t.dfix.n_chk = (int32_t)(s->dchk.size() / 3);
    t.dfix.B = (int)s->all_present_size;
    t.dfix.T = s->fix_T;
    t.dfix.n_cols = (int)s->dfix.size();
    t.dfix.total_units = s->dfix_units;
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

extern "C" {

void packos_schema_free(packos_schema* s) {
    if (!s) return;
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

// [scan tile sums][tile flags (k_var_copy)][value positions (u16, per var leaf x blob)]
// (the scan tile sums also hold k_encode_stream's ticket + per-256-blob look-back words)
static size_t ws_scan_bytes(size_t n) { return (((n + kS2T - 1) / kS2T) + 16) * sizeof(uint64_t); }
static size_t ws_flag_bytes(size_t n) { return ((n + 63) / 64 + 4) * sizeof(uint32_t); }

size_t packos_encode_workspace_size(const packos_schema* s, size_t n_blobs) {
    size_t nvar = 0;
    if (s)
        for (const EncItem& it : s->items) nvar += it.type == IT_VAR;
    const size_t a = (ws_scan_bytes(n_blobs) + 255) & ~(size_t)255;
    const size_t b = (ws_flag_bytes(n_blobs) + 255) & ~(size_t)255;
    return a + b + nvar * n_blobs * sizeof(uint16_t) + 256;
}

static int size_pass(packos_schema* s, DeviceTables* t, const EncCols& ec, size_t n, uint64_t* offs, void* ws,
                     size_t ws_bytes, hipStream_t st) {
    if (!offs) { set_error("out_offsets required for a variable-size schema"); return PACKOS_E_INVALID; }
    if (!ws || ws_bytes < packos_encode_workspace_size(s, n)) {
        set_error("workspace too small");
        return PACKOS_E_WORKSPACE;
    }
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(offs, 0, sizeof(uint64_t), st));
        return PACKOS_OK;
    }
    // data-independent presence: closed-form sizes (k_sizes_affine), no scan
    {
        AffPlan A{};
        bool affine = getenv("PACKOS_SIZES_SCAN") == nullptr;
        for (const EncCont& c : s->conts) affine &= c.valid_col < 0 || ec.valid[c.valid_col] == nullptr;
        for (const EncItem& it : s->items) {
            if (!affine) break;
            if (it.type == IT_VAR) {
                if (A.nv == kAffVar) affine = false;
                else A.off[A.nv++] = ec.off[it.col];
            } else {
                if (it.type == IT_FIXED && it.nullable && ec.valid[it.col] && s->mode != PACKOS_MODE_PACKABLE)
                    affine = false;
                A.C += it.size;
            }
        }
        if (affine) {
            const uint64_t per = (uint64_t)kBlock * kAffPer;
            hipLaunchKernelGGL(k_sizes_affine, dim3((unsigned)((n + 1 + per - 1) / per)), dim3(kBlock), 0, st, A,
                               offs, (uint64_t)n);
            HIP_TRY(hipGetLastError());
            return PACKOS_OK;
        }
    }
    // k_stream_sizes: ticket + per-tile look-back words at the start of ws
    const uint64_t ntiles = (n + kSzTile - 1) / kSzTile;
    HIP_TRY(hipMemsetAsync(ws, 0, (ntiles + 1) * sizeof(uint64_t), st));
    static unsigned long long* zprof = nullptr;  // debug: PACKOS_STREAM_PROF=1 prints phase clocks
    const bool want_prof = getenv("PACKOS_STREAM_PROF") != nullptr;
    if (want_prof && !zprof) HIP_TRY(hipMalloc(&zprof, 16 * sizeof(unsigned long long)));
    if (want_prof) HIP_TRY(hipMemsetAsync(zprof, 0, 16 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_stream_sizes, dim3((unsigned)ntiles), dim3(kBlock),
                       sizes_lds_bytes((int)s->items.size(), (int)s->conts.size()), st, t->enc, ec, (uint64_t*)ws,
                       offs, (uint64_t)n, want_prof ? zprof : nullptr);
    HIP_TRY(hipGetLastError());
    if (want_prof) {
        unsigned long long h[16];
        HIP_TRY(hipMemcpyAsync(h, zprof, sizeof(h), hipMemcpyDeviceToHost, st));
        HIP_TRY(hipStreamSynchronize(st));
        fprintf(stderr, "sizes tiles=%llu clocks/tile:", (unsigned long long)ntiles);
        for (int i = 0; i < 5; i++) fprintf(stderr, " p%d=%.0f", i, (double)h[8 + i] / ntiles);
        fprintf(stderr, "\n");
    }
    return PACKOS_OK;
}

// k_encode_stream plan for one call (kernel argument).  false: the schema /
// columns exceed the plan's tables or LDS, use the tiled encoder.
static bool stream_plan(const packos_schema* s, const EncCols& ec, S2Plan& S) {
    memset(&S, 0, sizeof(S));
    const uint32_t NI = (uint32_t)s->items.size();
    if (NI > (uint32_t)kS2Items || s->conts.size() > (size_t)kS2Conts) return false;
    // value staging (fix_cap / var_cap) is off by default: measured on the box, the LDS it
    // takes costs more occupancy than the HBM latency it hides (C3 0.162 -> 0.132 ms)
    uint32_t longv = 48, img_cap = 14336, fix_cap = 0, var_cap = 0, var_per = 36;
    if (const char* e = getenv("PACKOS_STREAM_LONG")) longv = (uint32_t)std::max(32, std::min(4096, atoi(e)));
    if (const char* e = getenv("PACKOS_STREAM_IMG")) img_cap = (uint32_t)std::max(2048, std::min(49152, atoi(e)));
    if (const char* e = getenv("PACKOS_STREAM_VAR")) var_cap = (uint32_t)std::max(0, std::min(32768, atoi(e)));
    if (const char* e = getenv("PACKOS_STREAM_FIX")) fix_cap = (uint32_t)std::max(0, std::min(49152, atoi(e)));
    if (const char* e = getenv("PACKOS_STREAM_VPER")) var_per = (uint32_t)std::max(4, std::min(256, atoi(e)));
    auto al16 = [](uint32_t x) { return (x + 15u) & ~15u; };
    uint32_t o = 0, cb = 0;
    std::vector<int> val_seg(kMaxCols, -1), fix_seg(kMaxCols, -1), off_seg(kMaxCols, -1), var_slot(kMaxCols, -1);
    auto add_seg = [&](const uint8_t* src, uint32_t w, bool extra) -> int {
        if (S.nseg >= kS2Seg) return -1;
        const int k = S.nseg++;
        const uint32_t bytes = (uint32_t)(kS2T + (extra ? 1 : 0)) * w;
        const uint32_t maxch = (bytes + 15) / 16 + 1;
        S.seg_src[k] = src;
        S.seg_w[k] = w;
        S.seg_lds[k] = o;
        S.seg_cb[k] = cb;
        if (extra) S.seg_extra |= 1u << k;
        cb += maxch;
        o += maxch * 16 + 16;   // +16: padding for 2-dword unaligned reads
        return k;
    };
    // validity columns, var offsets, fixed columns (up to fix_cap bytes per tile)
    for (size_t c = 0; c < s->col_node.size() && c < (size_t)kMaxCols; c++) {
        if (!ec.valid[c]) continue;
        if ((val_seg[c] = add_seg(ec.valid[c], 1, false)) < 0) return false;
    }
    uint32_t fix_bytes = 0, worst = 0;
    for (const EncItem& it : s->items) {
        if (it.type == IT_VAR) {
            if (off_seg[it.col] < 0 && (off_seg[it.col] = add_seg((const uint8_t*)ec.off[it.col], 4, true)) < 0)
                return false;
            worst += longv;
            continue;
        }
        worst += it.type == IT_HDR ? it.size : std::min(it.size, longv);
        if (it.type != IT_FIXED || fix_seg[it.col] >= 0) continue;
        if (fix_bytes + kS2T * it.size <= fix_cap && S.nseg < kS2Seg) {
            fix_seg[it.col] = add_seg(ec.data[it.col], it.size, false);
            fix_bytes += kS2T * it.size;
        }
    }
    S.seg_cb[S.nseg] = cb;
    // var columns staged in the same load round (their tile range known from
    // two uniform offset loads)
    uint32_t vb = 0;
    for (const EncItem& it : s->items) {
        if (it.type != IT_VAR || var_slot[it.col] >= 0 || S.nvar >= kS2Var) continue;
        const uint32_t bud = std::min<uint32_t>(al16(kS2T * var_per + 32), var_cap > vb ? var_cap - vb : 0);
        if (bud < 512) break;
        const int k = S.nvar++;
        var_slot[it.col] = k;
        S.var_off[k] = ec.off[it.col];
        S.var_data[k] = ec.data[it.col];
        S.var_lds[k] = o;
        S.var_bud[k] = bud;
        S.var_cb[k] = vb / 16;
        vb += bud;
        o += bud + 16;
    }
    S.var_cb[S.nvar] = vb / 16;
    // per-item plan
    uint32_t nlong = 0;
    for (uint32_t k = 0; k < NI; k++) {
        const EncItem& it = s->items[k];
        S2K& x = S.item[k];
        x.type = it.type;
        x.size = (uint16_t)std::min<uint32_t>(it.size, 0xFFFFu);
        x.cont = (uint16_t)it.cont;
        x.col = it.col;
        x.flags = it.is_bool ? SD_BOOL : 0;
        if (it.type == IT_HDR) {
            x.la = (uint16_t)(s->ihr[k] & 0xFFFFu);
            x.lv = (uint16_t)(s->ihr[k] >> 16);
        } else if (it.type == IT_CONST) {
            if (it.lit > 0xFFFFu) return false;
            x.la = (uint16_t)it.lit;
            if (it.size > longv) { x.flags |= SD_LONG; nlong++; }
        } else if (it.type == IT_FIXED) {
            const int sg = fix_seg[it.col];
            if (sg >= 0) {
                x.la = (uint16_t)S.seg_lds[sg];
                x.src15 = (uint8_t)((uintptr_t)ec.data[it.col] & 15);
                x.flags |= SD_STAGED;
                if (it.size == 1 || it.size == 2 || it.size == 4 || it.size == 8) x.flags |= SD_DIRECT;
            }
            else if ((it.size == 1 || it.size == 2 || it.size == 4 || it.size == 8) &&
                     ((uintptr_t)ec.data[it.col] % it.size) == 0)
                x.flags |= SD_GDIRECT;
            if (!(x.flags & (SD_DIRECT | SD_GDIRECT)) && it.size > longv) { x.flags |= SD_LONG; nlong++; }
            if (it.nullable && val_seg[it.col] >= 0) {
                x.flags |= SD_VALID;
                x.lv = (uint16_t)S.seg_lds[val_seg[it.col]];
                x.vsrc15 = (uint8_t)((uintptr_t)ec.valid[it.col] & 15);
            }
        } else {
            const int sg = off_seg[it.col];
            x.la = (uint16_t)S.seg_lds[sg];
            x.src15 = (uint8_t)((uintptr_t)ec.off[it.col] & 15);
            x.flags |= SD_LONG;
            nlong++;
            if (var_slot[it.col] >= 0) { x.flags |= SD_VSLOT; x.lv = (uint16_t)var_slot[it.col]; }
        }
    }
    for (size_t c = 0; c < s->conts.size(); c++) {
        const EncCont& ct = s->conts[c];
        S2KCont& x = S.cont[c];
        x.parent = ct.parent;
        x.lv = 0xFFFFu;
        if (ct.valid_col >= 0 && val_seg[ct.valid_col] >= 0) {
            x.lv = (uint16_t)S.seg_lds[val_seg[ct.valid_col]];
            x.vsrc15 = (uint8_t)((uintptr_t)ec.valid[ct.valid_col] & 15);
        }
    }
    S.pos_lds = o;
    o += al16(2u * kS2T * (NI + 1));
    uint32_t img = (uint32_t)std::min<uint64_t>(img_cap, (uint64_t)kS2T * worst + 32);
    img = std::max<uint32_t>(img, std::max<uint32_t>(2048u, 16u * (NI + 1) * kWavesPerBlock));
    S.img_bytes = al16(img);
    S.img_lds = o;
    o += S.img_bytes + 16;
    S.hole_cap = std::min<uint32_t>(nlong * kS2T, 1024u);
    S.hole_lds = o;
    o += al16(4 * S.hole_cap + 4 * (S.hole_cap + 2) + 8 * S.hole_cap);
    S.blob_lds = o;
    o += al16((uint32_t)sizeof(S2Blob) * kS2T);
    S.desc_lds = o;
    o += (uint32_t)sizeof(S2Desc) * NI;
    S.hdr_lds = o;
    o += al16((uint32_t)sizeof(S2Hdr) * (uint32_t)s->hdrs.size());
    S.hw_lds = o;
    o += al16(2u * kS2T * (uint32_t)s->hdrs.size()) + 16;
    S.grp_lds = o;
    o += S.hole_cap ? 2u * kS2Grp : 0u;
    S.misc_lds = o;
    o += 64;
    S.lds_total = o;
    S.longv = longv;
    // emitter split: the item boundary closest to half the estimated blob bytes
    uint64_t tot = 0;
    for (const EncItem& it : s->items) tot += it.type == IT_VAR ? 32u : it.size;
    uint64_t run = 0, best = ~0ull;
    S.mid = NI;
    for (uint32_t k = 0; k <= NI; k++) {
        const uint64_t d = 2 * run > tot ? 2 * run - tot : tot - 2 * run;
        if (d < best) { best = d; S.mid = k; }
        if (k < NI) run += s->items[k].type == IT_VAR ? 32u : s->items[k].size;
    }
    if (const char* e = getenv("PACKOS_STREAM_MID")) S.mid = (uint32_t)std::max(0, std::min((int)NI, atoi(e)));
    return o <= 64 * 1024;
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
    if (!s->has_var && !any_nil) {
        hipLaunchKernelGGL(k_fill_offsets, dim3((unsigned)((n + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           out_offsets, (uint64_t)n, (uint64_t)s->all_present_size);
        HIP_TRY(hipGetLastError());
        return PACKOS_OK;
    }
    return size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st);
}

int packos_encode_batch(const packos_schema* cs, const packos_column* cols, size_t n, uint8_t* out, uint64_t cap,
                        uint64_t* out_offsets, uint32_t* status, void* ws, size_t ws_bytes, uint32_t flags,
                        void* stream) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    if (!s || !cols || (!out && n)) { set_error("packos_encode_batch: bad argument"); return PACKOS_E_INVALID; }
    if (n == 0) return PACKOS_OK;
    int dev, r;
    if ((r = current_device(&dev))) return r;
    DeviceTables* t;
    if ((r = upload_tables(s, dev, &t))) return r;
    EncCols ec;
    bool any_nil;
    if ((r = fill_enc_cols(s, cols, ec, &any_nil))) return r;
    hipStream_t st = (hipStream_t)stream;
    const bool fixed_size = !s->has_var && !any_nil;
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
            if (variant == 0) variant = tile_ok ? 13 : dw_ok ? kDefaultFixedVariant : 8;
            if (variant == 13 && !tile_ok) variant = dw_ok ? kDefaultFixedVariant : 8;
            if ((variant == 1 || variant == 2) && !dw_ok) variant = 8;
            const size_t fcb = ((s->fcols.size() * kLFixBytes) + 15) / 16 * 16;
            // each kernel gets the column table copied right after the LDS it uses
            FixProgram pdw = t->fix, pgen = t->fix;
            pdw.fc_lds = s->fix_lds;
            const size_t gen_tables = (size_t)s->fix_lds + ((B + 1) * 4 + 15) / 16 * 16 + s->fsegs.size() * sizeof(FixSeg);
            pgen.fc_lds = (int32_t)gen_tables;
            const size_t lds_dw = (size_t)pdw.fc_lds + fcb;
            switch (variant) {
                case 1: hipLaunchKernelGGL((k_encode_fixed_dw<false>), dim3((unsigned)tiles), dim3(kBlock), lds_dw, st, pdw, ec, out, (uint64_t)n, status, stv); break;
                case 2: hipLaunchKernelGGL((k_encode_fixed_dw<true>), dim3((unsigned)tiles), dim3(kBlock), lds_dw, st, pdw, ec, out, (uint64_t)n, status, stv); break;
                case 13: {
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
                        hipLaunchKernelGGL((k_encode_fixed_dw<true>), dim3(1), dim3(kBlock), lds_dw, st, pdw, et,
                                           out + b0 * B, rem, status ? status + b0 : nullptr, stv);
                    }
                    break;
                }
                default: variant = 8; break;
            }
            if (variant == 8) {
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
    // default: size pass (k_sizes_affine or the k_stream_sizes look-back scan;
    // skipped when the caller's offsets are ready) + k_encode_stream.  PACKOS_VAR_KERNEL=tile selects the
    // two-kernel tiled encoder below.
    const char* vk = getenv("PACKOS_VAR_KERNEL");
    const bool want_stream = !(flags & PACKOS_ENC_FORCE_GENERIC) && !(vk && strcmp(vk, "tile") == 0);
    S2Plan SP;
    if (want_stream && s->conts.size() <= 64 && stream_plan(s, ec, SP)) {
        if (!offs_ready) {
            if ((r = size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st))) return r;
        }
        const uint64_t ntiles = (n + kS2T - 1) / kS2T;
        static unsigned long long* sprof = nullptr;  // debug: PACKOS_STREAM_PROF=1 prints phase clocks
        const bool want_prof = getenv("PACKOS_STREAM_PROF") != nullptr;
        if (want_prof && !sprof) HIP_TRY(hipMalloc(&sprof, 16 * sizeof(unsigned long long)));
        if (want_prof) HIP_TRY(hipMemsetAsync(sprof, 0, 16 * sizeof(unsigned long long), st));
        SP.prof = want_prof ? sprof : nullptr;
        hipLaunchKernelGGL(k_encode_stream, dim3((unsigned)ntiles), dim3(kBlock), SP.lds_total, st, t->enc, ec, SP,
                           (const uint64_t*)out_offsets, out, cap, (uint64_t)n, status);
        HIP_TRY(hipGetLastError());
        if (want_prof) {
            unsigned long long h[16];
            HIP_TRY(hipMemcpyAsync(h, sprof, sizeof(h), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            fprintf(stderr, "stream lds=%u img=%u holes=%u segs=%d vars=%d mid=%u tiles=%llu clocks/tile:",
                    SP.lds_total, SP.img_bytes, SP.hole_cap, SP.nseg, SP.nvar, SP.mid, (unsigned long long)ntiles);
            for (int i = 0; i < 8; i++) fprintf(stderr, " p%d=%.0f", i, (double)h[i] / ntiles);
            fprintf(stderr, "\n");
        }
        return PACKOS_OK;
    }
    if (!offs_ready) {
        if ((r = size_pass(s, t, ec, n, out_offsets, ws, ws_bytes, st))) return r;
    }
    const size_t npos = s->items.size() + 1;
    int vt = 128;
    uint32_t bud = 16384, in_bud = 16384;
    if (const char* e = getenv("PACKOS_VAR_TILE")) vt = atoi(e);
    if (const char* e = getenv("PACKOS_VAR_BUD")) bud = (uint32_t)std::max(2048, std::min(32768, atoi(e)));
    if (const char* e = getenv("PACKOS_VAR_IN")) in_bud = (uint32_t)std::max(0, std::min(32768, atoi(e)));
    if (vt != 64 && vt != 256) vt = 128;
    uint32_t win_shift = 0;
    while ((2u << win_shift) <= bud / 2) win_shift++;
    // per-call plan: fixed regions (IT_FIXED items), var leaves, validity columns
    VarPlan vp;
    memset(&vp, 0, sizeof(vp));
    for (int c = 0; c < kMaxCols; c++) vp.col_val[c] = -1;
    bool plan_ok = !(flags & PACKOS_ENC_FORCE_GENERIC) && s->conts.size() <= 64 && s->items.size() < 255;
    for (size_t c = 0; c < s->col_node.size() && plan_ok; c++) {
        if (!ec.valid[c]) continue;
        if (vp.nval >= kVPVal) { plan_ok = false; break; }
        vp.col_val[c] = (int8_t)vp.nval;
        vp.val_ptr[vp.nval++] = ec.valid[c];
    }
    auto plan_for = [&](int tile) {
        vp.nfix = vp.nvar = 0;
        uint32_t fb = 0;
        for (size_t k = 0; k < s->items.size() && plan_ok; k++) {
            const EncItem& it = s->items[k];
            if (it.type == IT_FIXED) {
                if (vp.nfix >= kVPFix) { plan_ok = false; break; }
                vp.fix_ptr[vp.nfix] = ec.data[it.col];
                vp.fix_w[vp.nfix] = it.size;
                vp.fix_lds[vp.nfix] = fb;
                fb += ((uint32_t)tile * it.size + 16 + 15) & ~15u;
                vp.nfix++;
            } else if (it.type == IT_VAR) {
                if (vp.nvar >= kVPVar) { plan_ok = false; break; }
                vp.var_off[vp.nvar] = ec.off[it.col];
                vp.var_data[vp.nvar] = ec.data[it.col];
                vp.var_item[vp.nvar] = (int)k;
                vp.nvar++;
            }
        }
        vp.fix_bytes = (int32_t)fb;
        return fb;
    };
    VtLayout vl{};
    uint32_t fb = 0;
    for (;;) {
        fb = plan_for(vt);
        const uint32_t ib = std::max(in_bud, fb);  // fixed regions are always staged
        vl = vt_layout(vt, t->enc, vp.nvar, vp.nval, bud, ib);
        if ((vl.total <= 64 * 1024 && fb <= 32768) || vt == 64) break;
        vt /= 2;
    }
    in_bud = std::max(in_bud, fb);
    const bool tiled = plan_ok && vl.total <= 64 * 1024 && npos * 4 * kWavesPerBlock <= (size_t)bud &&
                       ws && ws_bytes >= packos_encode_workspace_size(s, n);
    if (tiled) {
        uint8_t* wsb = (uint8_t*)ws + ((ws_scan_bytes(n) + 255) & ~(size_t)255);
        uint32_t* tflags = (uint32_t*)wsb;
        uint16_t* vpos = (uint16_t*)(wsb + ((ws_flag_bytes(n) + 255) & ~(size_t)255));
        const dim3 g((unsigned)((n + vt - 1) / vt)), b(kBlock);
        const size_t l = vl.total;
        const uint64_t* o = out_offsets;
        static unsigned long long* prof = nullptr;  // debug: PACKOS_VAR_PROF=1 prints phase cycles
        const bool want_prof = getenv("PACKOS_VAR_PROF") != nullptr;
        if (want_prof && !prof) HIP_TRY(hipMalloc(&prof, 16 * sizeof(unsigned long long)));
        if (want_prof) HIP_TRY(hipMemsetAsync(prof, 0, 16 * sizeof(unsigned long long), st));
        unsigned long long* pp = want_prof ? prof : nullptr;
        if (vt == 64)
            hipLaunchKernelGGL(k_encode_var_tile<64>, g, b, l, st, t->enc, ec, vp, o, out, cap, (uint64_t)n, status, bud, win_shift, in_bud, tflags, vpos, pp);
        else if (vt == 128)
            hipLaunchKernelGGL(k_encode_var_tile<128>, g, b, l, st, t->enc, ec, vp, o, out, cap, (uint64_t)n, status, bud, win_shift, in_bud, tflags, vpos, pp);
        else
            hipLaunchKernelGGL(k_encode_var_tile<256>, g, b, l, st, t->enc, ec, vp, o, out, cap, (uint64_t)n, status, bud, win_shift, in_bud, tflags, vpos, pp);
        HIP_TRY(hipGetLastError());
        if (vp.nvar > 0) {
            if (vt == 64) hipLaunchKernelGGL(k_var_copy<64>, g, b, 0, st, vp, o, tflags, vpos, out, (uint64_t)n);
            else if (vt == 128) hipLaunchKernelGGL(k_var_copy<128>, g, b, 0, st, vp, o, tflags, vpos, out, (uint64_t)n);
            else hipLaunchKernelGGL(k_var_copy<256>, g, b, 0, st, vp, o, tflags, vpos, out, (uint64_t)n);
            HIP_TRY(hipGetLastError());
        }
        if (want_prof) {
            unsigned long long h[16];
            HIP_TRY(hipMemcpyAsync(h, prof, sizeof(h), hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            fprintf(stderr, "var_tile vt=%d lds=%zu blocks=%u ticks/block:", vt, l, g.x);
            for (int i = 0; i < 8; i++) fprintf(stderr, " p%d=%.0f", i, (double)h[i] / g.x);
            fprintf(stderr, "\n");
        }
        return PACKOS_OK;
    }
    const size_t lds = (size_t)kWavesPerBlock * (kSlot + ((npos * 4 + 15) / 16) * 16);
    if (lds > 64 * 1024) { set_error("schema has too many items for the LDS budget"); return PACKOS_E_UNSUPPORTED; }
    const unsigned grid = (unsigned)std::min<uint64_t>((n + kWavesPerBlock - 1) / kWavesPerBlock, 256 * 16);
    hipLaunchKernelGGL(k_encode_var, dim3(grid), dim3(kBlock), lds, st, t->enc, ec, (const uint64_t*)out_offsets,
                       (uint64_t)0, out, cap, (uint64_t)n, status);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

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
    const int64_t B = s->all_present_size;
    bool fast = s->dec_fast == 1 && ((uintptr_t)arena & 15) == 0 && (offsets || stride == (uint64_t)B) &&
                !getenv("PACKOS_DECODE_GENERIC");
    for (const DecFix& f : s->dfix) fast = fast && ((uintptr_t)dc.data[f.col] & 15) == 0;
    fast = fast && s->dfix.size() <= (size_t)kDecK;
    if (fast) {
        // decode tile: dec_tile_bytes of staged blobs (16-blob multiple, <= 1024 blobs)
        DecFixProgram F = t->dfix;
        // measured (PACKOS_DEC_TILE_BYTES sweep 16/24/32/48 KB): 24 KB tiles are
        // best for B >= 128 (M 0.111 -> 0.103 ms, C4 0.431 -> 0.409 ms); for
        // small blobs the larger tile loses more to fewer workgroups (C2 +7 %)
        int64_t tb = B >= 128 ? kDecTileBytesLarge : kDecTileBytes;
        if (const char* e = getenv("PACKOS_DEC_TILE_BYTES")) tb = std::min<int64_t>(49152, std::max<int64_t>(1024, atoll(e)));
        F.T = (int32_t)std::min<int64_t>(1024, std::max<int64_t>(16, (tb / B) / 16 * 16));
        const uint32_t T = (uint32_t)F.T, QW = (uint32_t)((B + 3) / 4);
        const size_t lds = (size_t)T * B + 16 + 12 * QW + 4 * ((T + 1) & ~1u);
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
        hipLaunchKernelGGL(k_decode_fixed, dim3((unsigned)((n + T - 1) / T)), dim3(kBlock), lds, st, F, t->dec,
                           dc, K, arena, offsets, (uint64_t)n, status);
    } else if (getenv("PACKOS_DECODE_NOWIN")) {
        hipLaunchKernelGGL(k_decode, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, t->dec, dc,
                           arena, offsets, stride, (uint64_t)n, status);
    } else {
        const size_t ptab = ((s->dnodes.size() * sizeof(DecNode) + 15) & ~(size_t)15) +
                            ((s->dkids.size() * 4 + 15) & ~(size_t)15) + s->lits.size() + 16;
        hipLaunchKernelGGL(k_decode_win, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), ptab, st, t->dec,
                           dc, arena, offsets, stride, (uint64_t)n, status);
    }
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

int packos_get_field_batch(const uint8_t* arena, const uint64_t* offsets, uint64_t stride, size_t n,
                           const int32_t* path, int depth, int want_tag, int want_width, uint64_t* out_start,
                           uint32_t* out_len, uint8_t* out_tag, uint8_t* status, void* stream) {
    if (!path || depth < 1 || depth > 16 || !out_start || !out_len || !out_tag || !status || (!arena && n))
        return PACKOS_E_INVALID;
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
                       (hipStream_t)stream, arena, offsets, stride, (uint64_t)n, pa, depth, want_tag, want_width,
                       out_start, out_len, out_tag, status);
    HIP_TRY(hipGetLastError());
    return PACKOS_OK;
}

}  // extern "C"
