// host_pipeline.cpp — packos_encode_host_batch: a batch whose columns live in
// HOST memory (RPC payloads, BadgerDB values: SURVEY §8(f) rank 3) encoded
// into a host arena.  Chunks of blobs move through per-slot device buffers:
// hipMemcpyAsync H2D -> packos_encode_batch (size kernel + encode kernel, or
// the fixed-layout kernel) -> D2H, two slots on two streams so one chunk's
// copies overlap the other's kernels.  The only host waits are for a chunk's
// byte total (needed to place its output) and for a slot's reuse.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "schema_impl.h"

using namespace packos;

namespace {

#define HP_TRY(x)                                                                   \
    do {                                                                            \
        hipError_t _e = (x);                                                        \
        if (_e != hipSuccess) {                                                     \
            set_error(std::string("host pipeline: ") + #x + ": " + hipGetErrorString(_e)); \
            return PACKOS_E_HIP;                                                    \
        }                                                                           \
    } while (0)

struct ColKind {
    bool fixed = false, var = false;
    uint32_t width = 0;
};

struct Slot {
    hipStream_t st = nullptr;
    std::vector<void*> dfix, dvar, doff, dval;   // per column (nullptr when unused)
    uint8_t* dout = nullptr;
    uint64_t* doffs = nullptr;
    uint32_t* dstatus = nullptr;
    void* ws = nullptr;
    size_t wsb = 0;
    std::vector<uint32_t*> hoff;                 // pinned rebased var offsets, per column
    uint64_t* htotal = nullptr;                  // pinned chunk byte total
    hipEvent_t ev = nullptr;
};

struct Pipeline {
    Slot slot[2];
    ~Pipeline() {
        for (Slot& s : slot) {
            if (s.st) (void)hipStreamSynchronize(s.st);
            for (auto* v : {&s.dfix, &s.dvar, &s.doff, &s.dval})
                for (void* p : *v)
                    if (p) (void)hipFree(p);
            if (s.dout) (void)hipFree(s.dout);
            if (s.doffs) (void)hipFree(s.doffs);
            if (s.dstatus) (void)hipFree(s.dstatus);
            if (s.ws) (void)hipFree(s.ws);
            for (uint32_t* p : s.hoff)
                if (p) (void)hipHostFree(p);
            if (s.htotal) (void)hipHostFree(s.htotal);
            if (s.ev) (void)hipEventDestroy(s.ev);
            if (s.st) (void)hipStreamDestroy(s.st);
        }
    }
};

}  // namespace

extern "C" int packos_encode_host_batch(const packos_schema* cs, const packos_column* hc, size_t n,
                                        uint8_t* host_out, uint64_t out_capacity, uint64_t* host_offsets,
                                        uint32_t* host_status, size_t chunk_blobs) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    if (!s || !hc || (!host_out && n)) { set_error("packos_encode_host_batch: bad argument"); return PACKOS_E_INVALID; }
    if (!host_status && !s->echk.empty()) {
        set_error("packos_encode_host_batch: the schema has value checks: host_status required");
        return PACKOS_E_INVALID;
    }
    if (n == 0) {
        if (host_offsets) host_offsets[0] = 0;
        return PACKOS_OK;
    }
    const size_t ncol = s->col_node.size();
    std::vector<ColKind> kind(ncol);
    bool any_valid = false;
    for (size_t c = 0; c < ncol; c++) {
        const Node& nd = s->nodes[s->col_node[c]];
        const bool scalar = nd.kind >= K_INT && nd.kind <= K_BOOL;
        const bool str = nd.kind == K_STRING || nd.kind == K_BYTES;
        kind[c].fixed = scalar || (str && nd.width > 0);
        kind[c].var = str && nd.width <= 0;
        kind[c].width = kind[c].fixed ? (uint32_t)nd.width : 0u;
        if ((kind[c].fixed || kind[c].var) && !hc[c].data) { set_error("host column without data"); return PACKOS_E_INVALID; }
        if (kind[c].var && !hc[c].offsets && !hc[c].offsets64) {
            set_error("host var column without offsets");
            return PACKOS_E_INVALID;
        }
        any_valid |= hc[c].valid != nullptr;
    }
    const bool fixed_size = !s->has_var && !any_valid && s->all_present_size >= 0 &&
                            !(s->ext && s->all_present_size > (int64_t)kExtMaxPayload);
    if (!fixed_size && !host_offsets) { set_error("host_offsets required for a variable-size batch"); return PACKOS_E_INVALID; }
    // per-blob byte bound without var values: every non-var item present
    // (a nil only removes bytes; packable slack re-adds at most what it removed)
    uint64_t stat = 0;
    for (const EncItem& it : s->items)
        if (it.type != IT_VAR) stat += it.size;
    if (s->ext) stat += (uint64_t)ext_overhead(s);   // extended header blocks (ADR-001)

    // host var offsets of either width; every chunk's device offsets are
    // chunk-relative uint32 (a chunk's var bytes must stay below 4 GiB), so
    // 64-bit host offsets lift the 4 GiB limit of the whole batch
    auto hoff = [&](size_t c, size_t i) -> uint64_t {
        return hc[c].offsets64 ? hc[c].offsets64[i] : (uint64_t)hc[c].offsets[i];
    };
    size_t chunk = chunk_blobs ? chunk_blobs : (size_t)1 << 20;
    chunk = std::min(chunk, n);
    const size_t nch = (n + chunk - 1) / chunk;
    // largest var range / output of any chunk
    std::vector<uint64_t> var_max(ncol, 0);
    uint64_t out_max = 0;
    for (size_t k = 0; k < nch; k++) {
        const size_t s0 = k * chunk, m = std::min(chunk, n - s0);
        uint64_t vb = 0;
        for (size_t c = 0; c < ncol; c++)
            if (kind[c].var) {
                const uint64_t b = hoff(c, s0 + m) - hoff(c, s0);
                var_max[c] = std::max(var_max[c], b);
                vb += b;
            }
        out_max = std::max(out_max, (uint64_t)m * stat + vb);
    }
    for (size_t c = 0; c < ncol; c++)
        if (var_max[c] >= (1ull << 32)) {
            set_error("packos_encode_host_batch: a chunk's var bytes exceed 4 GiB (use smaller chunk_blobs)");
            return PACKOS_E_INVALID;
        }

    int dev = 0;
    HP_TRY(hipGetDevice(&dev));
    Pipeline P;
    for (Slot& sl : P.slot) {
        HP_TRY(hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking));
        HP_TRY(hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming));
        sl.dfix.assign(ncol, nullptr);
        sl.dvar.assign(ncol, nullptr);
        sl.doff.assign(ncol, nullptr);
        sl.dval.assign(ncol, nullptr);
        sl.hoff.assign(ncol, nullptr);
        for (size_t c = 0; c < ncol; c++) {
            if (kind[c].fixed) HP_TRY(hipMalloc(&sl.dfix[c], std::max<size_t>(16, chunk * kind[c].width)));
            if (kind[c].var) {
                HP_TRY(hipMalloc(&sl.dvar[c], std::max<uint64_t>(16, var_max[c])));
                HP_TRY(hipMalloc(&sl.doff[c], (chunk + 1) * sizeof(uint32_t)));
                HP_TRY(hipHostMalloc((void**)&sl.hoff[c], (chunk + 1) * sizeof(uint32_t), hipHostMallocDefault));
            }
            if (hc[c].valid) HP_TRY(hipMalloc(&sl.dval[c], std::max<size_t>(16, chunk)));
        }
        HP_TRY(hipMalloc((void**)&sl.dout, std::max<uint64_t>(16, out_max)));
        HP_TRY(hipMalloc((void**)&sl.doffs, (chunk + 1) * sizeof(uint64_t)));
        if (host_status) HP_TRY(hipMalloc((void**)&sl.dstatus, chunk * sizeof(uint32_t)));
        sl.wsb = packos_encode_workspace_size(s, chunk);
        HP_TRY(hipMalloc(&sl.ws, std::max<size_t>(16, sl.wsb)));
        HP_TRY(hipHostMalloc((void**)&sl.htotal, sizeof(uint64_t), hipHostMallocDefault));
    }

    std::vector<uint64_t> base(nch + 1, 0);
    std::vector<packos_column> dc(ncol);
    int rc = PACKOS_OK;
    // place chunk j's output once its byte total is known
    auto finish = [&](size_t j) -> int {
        Slot& sl = P.slot[j & 1];
        const size_t s0 = j * chunk, m = std::min(chunk, n - s0);
        uint64_t total;
        if (fixed_size) {
            total = (uint64_t)m * (uint64_t)s->all_present_size;
        } else {
            HP_TRY(hipEventSynchronize(sl.ev));
            total = *sl.htotal;
        }
        base[j + 1] = base[j] + total;
        if (base[j + 1] > out_capacity) {
            set_error("packos_encode_host_batch: output capacity exceeded");
            return PACKOS_E_CAPACITY;
        }
        HP_TRY(hipMemcpyAsync(host_out + base[j], sl.dout, total, hipMemcpyDeviceToHost, sl.st));
        if (host_offsets && !fixed_size)
            HP_TRY(hipMemcpyAsync(host_offsets + s0, sl.doffs, m * sizeof(uint64_t), hipMemcpyDeviceToHost, sl.st));
        if (host_status)
            HP_TRY(hipMemcpyAsync(host_status + s0, sl.dstatus, m * sizeof(uint32_t), hipMemcpyDeviceToHost, sl.st));
        return PACKOS_OK;
    };
    for (size_t k = 0; k < nch && rc == PACKOS_OK; k++) {
        Slot& sl = P.slot[k & 1];
        if (k >= 2) HP_TRY(hipStreamSynchronize(sl.st));   // slot reuse: chunk k-2 is out
        const size_t s0 = k * chunk, m = std::min(chunk, n - s0);
        for (size_t c = 0; c < ncol; c++) {
            memset(&dc[c], 0, sizeof(dc[c]));
            if (kind[c].fixed) {
                const size_t w = kind[c].width;
                HP_TRY(hipMemcpyAsync(sl.dfix[c], (const uint8_t*)hc[c].data + s0 * w, m * w, hipMemcpyHostToDevice,
                                      sl.st));
                dc[c].data = sl.dfix[c];
            }
            if (kind[c].var) {
                const uint64_t o0 = hoff(c, s0);
                for (size_t x = 0; x <= m; x++) sl.hoff[c][x] = (uint32_t)(hoff(c, s0 + x) - o0);   // chunk-relative
                HP_TRY(hipMemcpyAsync(sl.doff[c], sl.hoff[c], (m + 1) * sizeof(uint32_t), hipMemcpyHostToDevice,
                                      sl.st));
                const uint64_t vb = hoff(c, s0 + m) - o0;
                if (vb)
                    HP_TRY(hipMemcpyAsync(sl.dvar[c], (const uint8_t*)hc[c].data + o0, vb, hipMemcpyHostToDevice,
                                          sl.st));
                dc[c].data = sl.dvar[c];
                dc[c].offsets = (const uint32_t*)sl.doff[c];
            }
            if (hc[c].valid) {
                HP_TRY(hipMemcpyAsync(sl.dval[c], hc[c].valid + s0, m, hipMemcpyHostToDevice, sl.st));
                dc[c].valid = (uint8_t*)sl.dval[c];
            }
        }
        rc = packos_encode_batch(s, dc.data(), m, sl.dout, std::max<uint64_t>(16, out_max),
                                 fixed_size ? nullptr : sl.doffs, sl.dstatus, sl.ws, sl.wsb, 0, sl.st);
        if (rc != PACKOS_OK) break;
        if (!fixed_size) {
            HP_TRY(hipMemcpyAsync(sl.htotal, sl.doffs + m, sizeof(uint64_t), hipMemcpyDeviceToHost, sl.st));
            HP_TRY(hipEventRecord(sl.ev, sl.st));
        }
        if (k >= 1) rc = finish(k - 1);
    }
    if (rc == PACKOS_OK) rc = finish(nch - 1);
    for (Slot& sl : P.slot) HP_TRY(hipStreamSynchronize(sl.st));
    if (rc != PACKOS_OK) return rc;
    if (host_offsets) {
        if (fixed_size) {
            const uint64_t B = (uint64_t)s->all_present_size;
            for (size_t i = 0; i <= n; i++) host_offsets[i] = i * B;
        } else {
            for (size_t j = 0; j < nch; j++) {   // chunk-relative -> batch offsets
                const size_t s0 = j * chunk, m = std::min(chunk, n - s0);
                for (size_t i = 0; i < m; i++) host_offsets[s0 + i] += base[j];
            }
            host_offsets[n] = base[nch];
        }
    }
    return PACKOS_OK;
}

// packos_decode_host_batch: blobs in a HOST arena (BadgerDB values, RPC
// payloads) decoded into HOST columns.  Chunk k: its offsets (absolute, as
// the caller's) and the arena bytes they cover (from a 16-B aligned start)
// go H2D; packos_decode_batch runs on a device arena pointer biased so that
// absolute offsets land in the chunk buffer, so var views come back as
// absolute host-arena offsets with no fix-up; columns + status go D2H.  All
// sizes are known up front, so the host never waits except for slot reuse.
namespace {
struct DSlot {
    hipStream_t st = nullptr;
    uint8_t* darena = nullptr;
    uint64_t* doffs = nullptr;
    uint64_t* hoffs = nullptr;   // pinned staging for stride-mode offsets
    uint32_t* dstatus = nullptr;
    std::vector<void*> ddata, dvalid, dstart, dlen;
    ~DSlot() {
        if (st) (void)hipStreamSynchronize(st);
        for (auto* v : {&ddata, &dvalid, &dstart, &dlen})
            for (void* p : *v)
                if (p) (void)hipFree(p);
        if (darena) (void)hipFree(darena);
        if (doffs) (void)hipFree(doffs);
        if (dstatus) (void)hipFree(dstatus);
        if (hoffs) (void)hipHostFree(hoffs);
        if (st) (void)hipStreamDestroy(st);
    }
};
}  // namespace

extern "C" int packos_decode_host_batch(const packos_schema* cs, const uint8_t* host_arena,
                                        const uint64_t* host_offsets, uint64_t stride, size_t n,
                                        packos_column* host_cols, uint32_t* host_status, size_t chunk_blobs) {
    packos_schema* s = const_cast<packos_schema*>(cs);
    if (!s || !host_cols || !host_status || (!host_arena && n)) {
        set_error("packos_decode_host_batch: bad argument");
        return PACKOS_E_INVALID;
    }
    if (n == 0) return PACKOS_OK;
    if (!host_offsets && stride == 0) { set_error("offsets or stride required"); return PACKOS_E_INVALID; }
    const size_t ncol = s->col_node.size();
    std::vector<ColKind> kind(ncol);
    std::vector<char> has_valid(ncol, 0);   // the decoder writes validity for these
    for (size_t c = 0; c < ncol; c++) {
        const Node& nd = s->nodes[s->col_node[c]];
        const bool scalar = nd.kind >= K_INT && nd.kind <= K_BOOL;
        const bool str = nd.kind == K_STRING || nd.kind == K_BYTES;
        kind[c].fixed = scalar || (str && nd.width > 0);
        kind[c].var = str && nd.width <= 0;
        kind[c].width = kind[c].fixed ? (uint32_t)nd.width : 0u;
        has_valid[c] = host_cols[c].valid && ((scalar && nd.nullable) || nd.kind == K_TUPLE || nd.kind == K_MAP);
        if (kind[c].fixed && !host_cols[c].data) { set_error("host decode column without data"); return PACKOS_E_INVALID; }
        if (kind[c].var && (!host_cols[c].start || !host_cols[c].length)) {
            set_error("host decode var column without start/length");
            return PACKOS_E_INVALID;
        }
        if (scalar && nd.nullable && !host_cols[c].valid) {
            set_error("host decode nullable column without valid");
            return PACKOS_E_INVALID;
        }
    }
    auto off = [&](size_t i) -> uint64_t { return host_offsets ? host_offsets[i] : (uint64_t)i * stride; };
    size_t chunk = chunk_blobs ? chunk_blobs : (size_t)1 << 20;
    chunk = std::min(chunk, n);
    const size_t nch = (n + chunk - 1) / chunk;
    uint64_t span_max = 0;   // aligned arena bytes of the largest chunk
    for (size_t k = 0; k < nch; k++) {
        const size_t s0 = k * chunk, m = std::min(chunk, n - s0);
        const uint64_t a = off(s0) & ~15ull, b = std::max(off(s0 + m), off(s0));
        span_max = std::max(span_max, b - a);
    }
    DSlot slot[2];
    for (DSlot& sl : slot) {
        HP_TRY(hipStreamCreateWithFlags(&sl.st, hipStreamNonBlocking));
        HP_TRY(hipMalloc((void**)&sl.darena, span_max + 64));
        HP_TRY(hipMalloc((void**)&sl.doffs, (chunk + 1) * sizeof(uint64_t)));
        if (!host_offsets) HP_TRY(hipHostMalloc((void**)&sl.hoffs, (chunk + 1) * sizeof(uint64_t), hipHostMallocDefault));
        HP_TRY(hipMalloc((void**)&sl.dstatus, chunk * sizeof(uint32_t)));
        sl.ddata.assign(ncol, nullptr);
        sl.dvalid.assign(ncol, nullptr);
        sl.dstart.assign(ncol, nullptr);
        sl.dlen.assign(ncol, nullptr);
        for (size_t c = 0; c < ncol; c++) {
            if (kind[c].fixed) HP_TRY(hipMalloc(&sl.ddata[c], std::max<size_t>(16, chunk * kind[c].width)));
            if (has_valid[c]) HP_TRY(hipMalloc(&sl.dvalid[c], std::max<size_t>(16, chunk)));
            if (kind[c].var) {
                HP_TRY(hipMalloc(&sl.dstart[c], chunk * sizeof(uint64_t)));
                HP_TRY(hipMalloc(&sl.dlen[c], chunk * sizeof(uint32_t)));
            }
        }
    }
    std::vector<packos_column> dc(ncol);
    for (size_t k = 0; k < nch; k++) {
        DSlot& sl = slot[k & 1];
        if (k >= 2) HP_TRY(hipStreamSynchronize(sl.st));   // slot reuse: chunk k-2 is out
        const size_t s0 = k * chunk, m = std::min(chunk, n - s0);
        const uint64_t a = off(s0) & ~15ull, b = std::max(off(s0 + m), off(s0));
        if (host_offsets) {
            HP_TRY(hipMemcpyAsync(sl.doffs, host_offsets + s0, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, sl.st));
        } else {
            for (size_t x = 0; x <= m; x++) sl.hoffs[x] = (uint64_t)(s0 + x) * stride;
            HP_TRY(hipMemcpyAsync(sl.doffs, sl.hoffs, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, sl.st));
        }
        if (b > a) HP_TRY(hipMemcpyAsync(sl.darena, host_arena + a, b - a, hipMemcpyHostToDevice, sl.st));
        for (size_t c = 0; c < ncol; c++) {
            // rows the decoder never writes (nil values, values inside nil
            // containers) come back as zero data and views, 0xFF validity
            if (kind[c].fixed) HP_TRY(hipMemsetAsync(sl.ddata[c], 0, m * kind[c].width, sl.st));
            if (has_valid[c]) HP_TRY(hipMemsetAsync(sl.dvalid[c], 0xFF, m, sl.st));
            if (kind[c].var) {
                HP_TRY(hipMemsetAsync(sl.dstart[c], 0, m * sizeof(uint64_t), sl.st));
                HP_TRY(hipMemsetAsync(sl.dlen[c], 0, m * sizeof(uint32_t), sl.st));
            }
            memset(&dc[c], 0, sizeof(dc[c]));
            dc[c].data = sl.ddata[c];
            dc[c].valid = (uint8_t*)sl.dvalid[c];
            dc[c].start = (uint64_t*)sl.dstart[c];
            dc[c].length = (uint32_t*)sl.dlen[c];
        }
        // biased arena: device address of host-arena byte x is darena + (x - a)
        // (only offsets inside [a, b) are ever dereferenced)
        const uint8_t* biased = sl.darena - a;
        int rc = packos_decode_batch(s, biased, sl.doffs, 0, m, dc.data(), sl.dstatus, sl.st);
        if (rc != PACKOS_OK) return rc;
        HP_TRY(hipMemcpyAsync(host_status + s0, sl.dstatus, m * sizeof(uint32_t), hipMemcpyDeviceToHost, sl.st));
        for (size_t c = 0; c < ncol; c++) {
            if (kind[c].fixed) {
                const size_t w = kind[c].width;
                HP_TRY(hipMemcpyAsync((uint8_t*)host_cols[c].data + s0 * w, sl.ddata[c], m * w, hipMemcpyDeviceToHost,
                                      sl.st));
            }
            if (has_valid[c])
                HP_TRY(hipMemcpyAsync(host_cols[c].valid + s0, sl.dvalid[c], m, hipMemcpyDeviceToHost, sl.st));
            if (kind[c].var) {
                HP_TRY(hipMemcpyAsync(host_cols[c].start + s0, sl.dstart[c], m * sizeof(uint64_t),
                                      hipMemcpyDeviceToHost, sl.st));
                HP_TRY(hipMemcpyAsync(host_cols[c].length + s0, sl.dlen[c], m * sizeof(uint32_t),
                                      hipMemcpyDeviceToHost, sl.st));
            }
        }
    }
    for (DSlot& sl : slot) HP_TRY(hipStreamSynchronize(sl.st));
    return PACKOS_OK;
}
