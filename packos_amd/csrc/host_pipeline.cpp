// host_pipeline.cpp — host-resident batches (RPC
// payloads and BadgerDB values that start and end in host memory).
//
// A packos_pipeline owns, per in-flight chunk ("slot"), the device buffers of
// one chunk, and three non-blocking streams shared by every slot:
//
//   H2D stream   chunk k's inputs  ->  device      (waits: slot's kernels of k-S done)
//   kernel stream                      encode / decode of chunk k
//                                                  (waits: H2D of k, D2H of k-S done)
//   D2H stream   chunk k's outputs ->  host        (waits: kernels of k)
//
// so PCIe carries chunk k+1's inputs and chunk k-1's outputs at the same
// time (full duplex) while chunk k's kernels run.  Buffers are sized for the
// largest chunk of a call and kept across calls (grow-only), so a serving
// loop pays no hipMalloc / hipHostMalloc per batch.
//
// Encode output placement needs each chunk's byte total: when the sizes are
// data-independent (no validity columns, plain modes) the totals come from the
// host var offsets up front and nothing waits; otherwise the host reads chunk
// k's total (one 8-byte D2H on the kernel stream) before it enqueues chunk
// k's D2H, after chunk k+1's H2D and kernels are already queued.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <mutex>
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
#define HP_RC(x)                  \
    do {                          \
        int _r = (x);             \
        if (_r != PACKOS_OK) return _r; \
    } while (0)

constexpr size_t kDefaultChunk = 131072;
constexpr uint64_t kPad = 64;   // device slack before / after staged host bytes (16-B window reads)

struct ColKind {
    bool fixed = false, var = false, scalar = false;
    uint32_t width = 0;
};

// grow-only device / pinned buffer
struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool pinned = false;
    int ensure(size_t bytes) {
        bytes = std::max<size_t>(bytes, 64);
        if (bytes <= cap) return PACKOS_OK;
        if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        cap = 0;
        const size_t want = bytes + bytes / 8;   // headroom: a slightly larger next batch reuses it
        HP_TRY(pinned ? hipHostMalloc(&p, want, hipHostMallocDefault) : hipMalloc(&p, want));
        cap = want;
        return PACKOS_OK;
    }
    void release() {
        if (p) (void)(pinned ? hipHostFree(p) : hipFree(p));
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return (T*)p; }
};

struct Slot {
    // encode inputs / outputs
    std::vector<DBuf> efix, evar, eoff, eval;
    DBuf eout, eoffs, estatus, ews;
    DBuf htotal{nullptr, 0, true};   // pinned chunk byte total
    // decode inputs / outputs
    DBuf darena, doffs, dstatus;
    std::vector<DBuf> ddata, dvalid, dstart, dlen;
    hipEvent_t ev_in = nullptr, ev_comp = nullptr, ev_out = nullptr;
    void release() {
        for (auto* v : {&efix, &evar, &eoff, &eval, &ddata, &dvalid, &dstart, &dlen})
            for (DBuf& b : *v) b.release();
        for (DBuf* b : {&eout, &eoffs, &estatus, &ews, &htotal, &darena, &doffs, &dstatus}) b->release();
        for (hipEvent_t e : {ev_in, ev_comp, ev_out})
            if (e) (void)hipEventDestroy(e);
        ev_in = ev_comp = ev_out = nullptr;
    }
};

std::vector<ColKind> col_kinds(const packos_schema* s) {
    std::vector<ColKind> kind(s->col_node.size());
    for (size_t c = 0; c < kind.size(); c++) {
        const Node& nd = s->nodes[s->col_node[c]];
        const bool scalar = nd.kind >= K_INT && nd.kind <= K_BOOL;
        const bool str = nd.kind == K_STRING || nd.kind == K_BYTES;
        kind[c].scalar = scalar;
        kind[c].fixed = scalar || (str && nd.width > 0);
        kind[c].var = str && nd.width <= 0;
        kind[c].width = kind[c].fixed ? (uint32_t)nd.width : 0u;
    }
    return kind;
}

// restores the caller's current device on scope exit
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct packos_pipeline {
    packos_schema* s = nullptr;
    int device = 0;
    size_t chunk = kDefaultChunk;
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    std::vector<Slot> slot;
    std::mutex mu;   // one call at a time

    int init(packos_schema* sc, size_t chunk_blobs, int slots) {
        s = sc;
        chunk = chunk_blobs ? chunk_blobs : kDefaultChunk;
        HP_TRY(hipGetDevice(&device));
        HP_TRY(hipStreamCreateWithFlags(&h2d, hipStreamNonBlocking));
        HP_TRY(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
        HP_TRY(hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking));
        slot.resize((size_t)std::max(2, slots ? slots : 3));
        const size_t ncol = s->col_node.size();
        for (Slot& sl : slot) {
            HP_TRY(hipEventCreateWithFlags(&sl.ev_in, hipEventDisableTiming));
            HP_TRY(hipEventCreateWithFlags(&sl.ev_comp, hipEventDisableTiming));
            HP_TRY(hipEventCreateWithFlags(&sl.ev_out, hipEventDisableTiming));
            for (auto* v : {&sl.efix, &sl.evar, &sl.eoff, &sl.eval, &sl.ddata, &sl.dvalid, &sl.dstart, &sl.dlen})
                v->assign(ncol, DBuf{});
        }
        return PACKOS_OK;
    }
    // drain everything (errors included) so buffers can be reused or freed
    void drain() {
        for (hipStream_t st : {h2d, comp, d2h})
            if (st) (void)hipStreamSynchronize(st);
    }
    ~packos_pipeline() {
        DeviceGuard g(device);
        drain();
        for (Slot& sl : slot) sl.release();
        for (hipStream_t st : {h2d, comp, d2h})
            if (st) (void)hipStreamDestroy(st);
    }

    int encode_impl(const packos_column* hc, size_t n, uint8_t* host_out, uint64_t out_capacity,
                    uint64_t* host_offsets, uint32_t* host_status);
    int decode_impl(const uint8_t* host_arena, const uint64_t* host_offsets, uint64_t stride, size_t n,
                    packos_column* host_cols, uint32_t* host_status, bool val);
    // a failed call still drains its queued work before the buffers are reused
    int encode(const packos_column* hc, size_t n, uint8_t* host_out, uint64_t out_capacity, uint64_t* host_offsets,
               uint32_t* host_status) {
        const int r = encode_impl(hc, n, host_out, out_capacity, host_offsets, host_status);
        if (r != PACKOS_OK) drain();
        return r;
    }
    // val: ValidateBuffer (packos_validate_batch), status only, host_cols unused
    int decode(const uint8_t* host_arena, const uint64_t* host_offsets, uint64_t stride, size_t n,
               packos_column* host_cols, uint32_t* host_status, bool val = false) {
        const int r = decode_impl(host_arena, host_offsets, stride, n, host_cols, host_status, val);
        if (r != PACKOS_OK) drain();
        return r;
    }
};

// ------------------------------------------------------------------ encode
int packos_pipeline::encode_impl(const packos_column* hc, size_t n, uint8_t* host_out, uint64_t out_capacity,
                            uint64_t* host_offsets, uint32_t* host_status) {
    if (!hc || (!host_out && n)) { set_error("packos_encode_host_batch: bad argument"); return PACKOS_E_INVALID; }
    if (!host_status && !s->echk.empty()) {
        set_error("packos_encode_host_batch: the schema has value checks: host_status required");
        return PACKOS_E_INVALID;
    }
    if (n == 0) {
        if (host_offsets) host_offsets[0] = 0;
        return PACKOS_OK;
    }
    const size_t ncol = s->col_node.size();
    const std::vector<ColKind> kind = col_kinds(s);
    bool any_valid = false;
    for (size_t c = 0; c < ncol; c++) {
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
    // per-blob bytes of every non-var item (the whole blob when nothing is nil)
    uint64_t stat = 0;
    for (const EncItem& it : s->items)
        if (it.type != IT_VAR) stat += it.size;
    const uint64_t bound_stat = stat + (s->ext ? (uint64_t)ext_overhead(s) : 0);
    // sizes known on the host: no validity columns, no extended containers
    const bool closed = fixed_size || (!any_valid && !s->ext);
    auto hoff = [&](size_t c, size_t i) -> uint64_t {
        return hc[c].offsets64 ? hc[c].offsets64[i] : (uint64_t)hc[c].offsets[i];
    };
    const size_t ch = std::min(chunk, n);
    const size_t nch = (n + ch - 1) / ch;
    // per chunk: output bound (or exact total when closed); per column: the
    // largest var byte range of any chunk
    std::vector<uint64_t> var_max(ncol, 0), total(nch, 0);
    uint64_t out_max = 0;
    for (size_t k = 0; k < nch; k++) {
        const size_t s0 = k * ch, m = std::min(ch, n - s0);
        uint64_t vb = 0;
        for (size_t c = 0; c < ncol; c++)
            if (kind[c].var) {
                const uint64_t a = hoff(c, s0), b = hoff(c, s0 + m);
                if (b < a) { set_error("packos_encode_host_batch: var offsets must be non-decreasing"); return PACKOS_E_INVALID; }
                var_max[c] = std::max(var_max[c], b - a);
                vb += b - a;
            }
        total[k] = fixed_size ? (uint64_t)m * (uint64_t)s->all_present_size : (uint64_t)m * stat + vb;
        out_max = std::max(out_max, closed ? total[k] : (uint64_t)m * bound_stat + vb);
    }
    std::vector<uint64_t> base(nch + 1, 0);
    if (closed) {
        for (size_t k = 0; k < nch; k++) base[k + 1] = base[k] + total[k];
        if (base[nch] > out_capacity) {
            set_error("packos_encode_host_batch: output capacity exceeded");
            return PACKOS_E_CAPACITY;
        }
    }
    // buffers for the largest chunk
    for (Slot& sl : slot) {
        for (size_t c = 0; c < ncol; c++) {
            if (kind[c].fixed) HP_RC(sl.efix[c].ensure(ch * kind[c].width));
            if (kind[c].var) {
                HP_RC(sl.evar[c].ensure(var_max[c] + 2 * kPad));
                HP_RC(sl.eoff[c].ensure((ch + 1) * (hc[c].offsets64 ? 8 : 4)));
            }
            if (hc[c].valid) HP_RC(sl.eval[c].ensure(ch));
        }
        HP_RC(sl.eout.ensure(out_max));
        HP_RC(sl.eoffs.ensure((ch + 1) * sizeof(uint64_t)));
        if (host_status) HP_RC(sl.estatus.ensure(ch * sizeof(uint32_t)));
        HP_RC(sl.ews.ensure(packos_encode_workspace_size(s, ch)));
        HP_RC(sl.htotal.ensure(sizeof(uint64_t)));
    }
    std::vector<packos_column> dc(ncol);
    const size_t S = slot.size();
    // chunk j's outputs -> host (D2H stream), once base[j] is known
    auto d2h_chunk = [&](size_t j) -> int {
        Slot& sl = slot[j % S];
        const size_t s0 = j * ch, m = std::min(ch, n - s0);
        HP_TRY(hipStreamWaitEvent(d2h, sl.ev_comp, 0));
        const uint64_t tot = base[j + 1] - base[j];
        if (tot) HP_TRY(hipMemcpyAsync(host_out + base[j], sl.eout.p, tot, hipMemcpyDeviceToHost, d2h));
        if (!fixed_size) {
            HP_RC(launch_add_base(sl.eoffs.as<uint64_t>(), m, base[j], d2h));   // chunk-relative -> batch offsets
            HP_TRY(hipMemcpyAsync(host_offsets + s0, sl.eoffs.p, m * sizeof(uint64_t), hipMemcpyDeviceToHost, d2h));
        }
        if (host_status)
            HP_TRY(hipMemcpyAsync(host_status + s0, sl.estatus.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, d2h));
        HP_TRY(hipEventRecord(sl.ev_out, d2h));
        return PACKOS_OK;
    };
    for (size_t k = 0; k < nch; k++) {
        Slot& sl = slot[k % S];
        const size_t s0 = k * ch, m = std::min(ch, n - s0);
        // inputs (H2D stream); the slot's input buffers are free once the
        // kernels of chunk k - S are done
        if (k >= S) HP_TRY(hipStreamWaitEvent(h2d, sl.ev_comp, 0));
        for (size_t c = 0; c < ncol; c++) {
            memset(&dc[c], 0, sizeof(dc[c]));
            if (kind[c].fixed) {
                const size_t w = kind[c].width;
                HP_TRY(hipMemcpyAsync(sl.efix[c].p, (const uint8_t*)hc[c].data + s0 * w, m * w, hipMemcpyHostToDevice,
                                      h2d));
                dc[c].data = sl.efix[c].p;
            }
            if (kind[c].var) {
                // the host offsets go over as they are; the device data pointer
                // is biased so that host offset x lands at evar + kPad + (x - o0)
                const uint64_t o0 = hoff(c, s0), vb = hoff(c, s0 + m) - o0;
                const bool w8 = hc[c].offsets64 != nullptr;
                const void* src = w8 ? (const void*)(hc[c].offsets64 + s0) : (const void*)(hc[c].offsets + s0);
                HP_TRY(hipMemcpyAsync(sl.eoff[c].p, src, (m + 1) * (w8 ? 8 : 4), hipMemcpyHostToDevice, h2d));
                if (vb)
                    HP_TRY(hipMemcpyAsync(sl.evar[c].as<uint8_t>() + kPad, (const uint8_t*)hc[c].data + o0, vb,
                                          hipMemcpyHostToDevice, h2d));
                dc[c].data = sl.evar[c].as<uint8_t>() + kPad - o0;
                if (w8) dc[c].offsets64 = sl.eoff[c].as<uint64_t>();
                else dc[c].offsets = sl.eoff[c].as<uint32_t>();
            }
            if (hc[c].valid) {
                HP_TRY(hipMemcpyAsync(sl.eval[c].p, hc[c].valid + s0, m, hipMemcpyHostToDevice, h2d));
                dc[c].valid = sl.eval[c].as<uint8_t>();
            }
        }
        HP_TRY(hipEventRecord(sl.ev_in, h2d));
        // kernels: after the inputs, and after chunk k - S's outputs left the slot
        HP_TRY(hipStreamWaitEvent(comp, sl.ev_in, 0));
        if (k >= S) HP_TRY(hipStreamWaitEvent(comp, sl.ev_out, 0));
        // closed form: the chunk's exact size, so the var encoder is picked by
        // the bytes per blob without reading the offsets back
        HP_RC(packos_encode_batch(s, dc.data(), m, sl.eout.as<uint8_t>(), closed ? total[k] : sl.eout.cap,
                                  fixed_size ? nullptr : sl.eoffs.as<uint64_t>(),
                                  host_status ? sl.estatus.as<uint32_t>() : nullptr, sl.ews.p, sl.ews.cap,
                                  closed ? PACKOS_ENC_CAP_EXACT : 0u, comp));
        if (!closed)
            HP_TRY(hipMemcpyAsync(sl.htotal.p, sl.eoffs.as<uint64_t>() + m, sizeof(uint64_t), hipMemcpyDeviceToHost, comp));
        HP_TRY(hipEventRecord(sl.ev_comp, comp));
        if (closed) {
            HP_RC(d2h_chunk(k));
        } else if (k >= 1) {
            // chunk k - 1's total (its kernels finished long ago, chunk k is queued)
            Slot& pv = slot[(k - 1) % S];
            HP_TRY(hipEventSynchronize(pv.ev_comp));
            base[k] = base[k - 1] + *pv.htotal.as<uint64_t>();
            if (base[k] > out_capacity) {
                set_error("packos_encode_host_batch: output capacity exceeded");
                return PACKOS_E_CAPACITY;
            }
            HP_RC(d2h_chunk(k - 1));
        }
        // fixed layouts: the host offsets are i * B, written while the GPU works
        if (fixed_size && host_offsets) {
            const uint64_t B = (uint64_t)s->all_present_size;
            for (size_t i = s0; i < s0 + m; i++) host_offsets[i] = i * B;
        }
    }
    if (!closed) {
        Slot& pv = slot[(nch - 1) % S];
        HP_TRY(hipEventSynchronize(pv.ev_comp));
        base[nch] = base[nch - 1] + *pv.htotal.as<uint64_t>();
        if (base[nch] > out_capacity) {
            set_error("packos_encode_host_batch: output capacity exceeded");
            return PACKOS_E_CAPACITY;
        }
        HP_RC(d2h_chunk(nch - 1));
    }
    HP_TRY(hipStreamSynchronize(d2h));
    drain();
    if (host_offsets) host_offsets[n] = base[nch];
    return PACKOS_OK;
}

// ------------------------------------------------------------------ decode
int packos_pipeline::decode_impl(const uint8_t* host_arena, const uint64_t* host_offsets, uint64_t stride, size_t n,
                            packos_column* host_cols, uint32_t* host_status, bool val) {
    if ((!host_cols && !val) || !host_status || (!host_arena && n)) {
        set_error(val ? "packos_validate_host_batch: bad argument" : "packos_decode_host_batch: bad argument");
        return PACKOS_E_INVALID;
    }
    if (n == 0) return PACKOS_OK;
    if (!host_offsets && stride == 0) { set_error("offsets or stride required"); return PACKOS_E_INVALID; }
    const size_t ncol = val ? 0 : s->col_node.size();
    const std::vector<ColKind> kind = col_kinds(s);
    std::vector<char> has_valid(ncol, 0);   // the decoder writes validity for these
    for (size_t c = 0; c < ncol; c++) {
        const Node& nd = s->nodes[s->col_node[c]];
        has_valid[c] = host_cols[c].valid && ((kind[c].scalar && nd.nullable) || nd.kind == K_TUPLE || nd.kind == K_MAP);
        if (kind[c].fixed && !host_cols[c].data) { set_error("host decode column without data"); return PACKOS_E_INVALID; }
        if (kind[c].var && (!host_cols[c].start || !host_cols[c].length)) {
            set_error("host decode var column without start/length");
            return PACKOS_E_INVALID;
        }
        if (kind[c].scalar && nd.nullable && !host_cols[c].valid) {
            set_error("host decode nullable column without valid");
            return PACKOS_E_INVALID;
        }
    }
    const size_t ch = std::min(chunk, n);
    const size_t nch = (n + ch - 1) / ch;
    // the arena bytes a chunk's blobs may touch: [min offset, max offset) —
    // offsets need not be monotone; one pass over them, chunk by chunk
    std::vector<uint64_t> lo(nch), hi(nch);
    uint64_t span_max = 0;
    for (size_t k = 0; k < nch; k++) {
        const size_t s0 = k * ch, m = std::min(ch, n - s0);
        uint64_t a, b;
        if (host_offsets) {
            a = b = host_offsets[s0];
            for (size_t i = s0 + 1; i <= s0 + m; i++) {
                a = std::min(a, host_offsets[i]);
                b = std::max(b, host_offsets[i]);
            }
        } else {
            a = (uint64_t)s0 * stride;
            b = (uint64_t)(s0 + m) * stride;
        }
        lo[k] = a & ~15ull;
        hi[k] = b;
        span_max = std::max(span_max, hi[k] - lo[k]);
    }
    for (Slot& sl : slot) {
        HP_RC(sl.darena.ensure(span_max + 2 * kPad));
        HP_RC(sl.doffs.ensure((ch + 1) * sizeof(uint64_t)));
        HP_RC(sl.dstatus.ensure(ch * sizeof(uint32_t)));
        for (size_t c = 0; c < ncol; c++) {
            if (kind[c].fixed) HP_RC(sl.ddata[c].ensure(ch * kind[c].width));
            if (has_valid[c]) HP_RC(sl.dvalid[c].ensure(ch));
            if (kind[c].var) {
                HP_RC(sl.dstart[c].ensure(ch * sizeof(uint64_t)));
                HP_RC(sl.dlen[c].ensure(ch * sizeof(uint32_t)));
            }
        }
    }
    std::vector<packos_column> dc(ncol);
    const size_t S = slot.size();
    for (size_t k = 0; k < nch; k++) {
        Slot& sl = slot[k % S];
        const size_t s0 = k * ch, m = std::min(ch, n - s0);
        const uint64_t a = lo[k], b = hi[k];
        if (k >= S) HP_TRY(hipStreamWaitEvent(h2d, sl.ev_comp, 0));
        if (host_offsets)
            HP_TRY(hipMemcpyAsync(sl.doffs.p, host_offsets + s0, (m + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, h2d));
        else
            HP_RC(launch_fill_offsets(sl.doffs.as<uint64_t>(), m, (uint64_t)s0 * stride, stride, h2d));
        if (b > a) HP_TRY(hipMemcpyAsync(sl.darena.as<uint8_t>() + kPad, host_arena + a, b - a, hipMemcpyHostToDevice, h2d));
        HP_TRY(hipEventRecord(sl.ev_in, h2d));
        HP_TRY(hipStreamWaitEvent(comp, sl.ev_in, 0));
        if (k >= S) HP_TRY(hipStreamWaitEvent(comp, sl.ev_out, 0));
        for (size_t c = 0; c < ncol; c++) {
            // rows the decoder never writes (nil values, values inside nil
            // containers) come back as zero data and views, 0xFF validity
            if (kind[c].fixed) HP_TRY(hipMemsetAsync(sl.ddata[c].p, 0, m * kind[c].width, comp));
            if (has_valid[c]) HP_TRY(hipMemsetAsync(sl.dvalid[c].p, 0xFF, m, comp));
            if (kind[c].var) {
                HP_TRY(hipMemsetAsync(sl.dstart[c].p, 0, m * sizeof(uint64_t), comp));
                HP_TRY(hipMemsetAsync(sl.dlen[c].p, 0, m * sizeof(uint32_t), comp));
            }
            memset(&dc[c], 0, sizeof(dc[c]));
            dc[c].data = sl.ddata[c].p;
            dc[c].valid = has_valid[c] ? sl.dvalid[c].as<uint8_t>() : nullptr;
            dc[c].start = sl.dstart[c].as<uint64_t>();
            dc[c].length = sl.dlen[c].as<uint32_t>();
        }
        // biased arena: host byte x is at darena + kPad + (x - a); only
        // offsets inside [a, b) (plus the decoders' 16-B window rounding) are read
        const uint8_t* biased = sl.darena.as<uint8_t>() + kPad - a;
        if (val) HP_RC(packos_validate_batch(s, biased, sl.doffs.as<uint64_t>(), 0, m, sl.dstatus.as<uint32_t>(), comp));
        else HP_RC(packos_decode_batch(s, biased, sl.doffs.as<uint64_t>(), 0, m, dc.data(), sl.dstatus.as<uint32_t>(), comp));
        HP_TRY(hipEventRecord(sl.ev_comp, comp));
        HP_TRY(hipStreamWaitEvent(d2h, sl.ev_comp, 0));
        HP_TRY(hipMemcpyAsync(host_status + s0, sl.dstatus.p, m * sizeof(uint32_t), hipMemcpyDeviceToHost, d2h));
        for (size_t c = 0; c < ncol; c++) {
            if (kind[c].fixed) {
                const size_t w = kind[c].width;
                HP_TRY(hipMemcpyAsync((uint8_t*)host_cols[c].data + s0 * w, sl.ddata[c].p, m * w, hipMemcpyDeviceToHost,
                                      d2h));
            }
            if (has_valid[c]) HP_TRY(hipMemcpyAsync(host_cols[c].valid + s0, sl.dvalid[c].p, m, hipMemcpyDeviceToHost, d2h));
            if (kind[c].var) {
                HP_TRY(hipMemcpyAsync(host_cols[c].start + s0, sl.dstart[c].p, m * sizeof(uint64_t),
                                      hipMemcpyDeviceToHost, d2h));
                HP_TRY(hipMemcpyAsync(host_cols[c].length + s0, sl.dlen[c].p, m * sizeof(uint32_t),
                                      hipMemcpyDeviceToHost, d2h));
            }
        }
        HP_TRY(hipEventRecord(sl.ev_out, d2h));
    }
    HP_TRY(hipStreamSynchronize(d2h));
    drain();
    return PACKOS_OK;
}

// ------------------------------------------------------------------ C ABI
namespace packos {
void destroy_pipelines(packos_schema* s) {
    for (packos_pipeline* p : s->pipes) delete p;
    s->pipes.clear();
}
}  // namespace packos

namespace {
// the schema's cached pipeline for the current device, locked; a temporary
// one while another thread holds it
struct PipeLease {
    packos_pipeline* p = nullptr;
    std::unique_ptr<packos_pipeline> tmp;
    std::unique_lock<std::mutex> lk;
};
int lease(packos_schema* s, size_t chunk_blobs, PipeLease& L) {
    int dev = 0;
    HP_TRY(hipGetDevice(&dev));
    const size_t want = chunk_blobs ? chunk_blobs : kDefaultChunk;
    {
        std::lock_guard<std::mutex> g(s->mu);
        packos_pipeline* mine = nullptr;
        for (packos_pipeline* p : s->pipes)
            if (p->device == dev) mine = p;
        if (!mine) {
            std::unique_ptr<packos_pipeline> np(new packos_pipeline());
            HP_RC(np->init(s, want, 3));
            s->pipes.push_back(np.get());
            mine = np.release();
        }
        std::unique_lock<std::mutex> lk(mine->mu, std::try_to_lock);
        if (lk.owns_lock()) {
            mine->chunk = want;   // chunking is per call; buffers are reused
            L.p = mine;
            L.lk = std::move(lk);
            return PACKOS_OK;
        }
    }
    L.tmp.reset(new packos_pipeline());
    HP_RC(L.tmp->init(s, want, 3));
    L.p = L.tmp.get();
    return PACKOS_OK;
}
}  // namespace

extern "C" {

int packos_pipeline_create(const packos_schema* cs, size_t chunk_blobs, int slots, packos_pipeline** out) {
    if (!cs || !out || slots < 0) { set_error("packos_pipeline_create: bad argument"); return PACKOS_E_INVALID; }
    std::unique_ptr<packos_pipeline> p(new packos_pipeline());
    HP_RC(p->init(const_cast<packos_schema*>(cs), chunk_blobs, slots));
    *out = p.release();
    return PACKOS_OK;
}

void packos_pipeline_free(packos_pipeline* p) { delete p; }

int packos_pipeline_encode(packos_pipeline* p, const packos_column* host_cols, size_t n, uint8_t* host_out,
                           uint64_t out_capacity, uint64_t* host_offsets, uint32_t* host_status) {
    if (!p) { set_error("packos_pipeline_encode: null pipeline"); return PACKOS_E_INVALID; }
    std::lock_guard<std::mutex> g(p->mu);
    DeviceGuard dg(p->device);
    return p->encode(host_cols, n, host_out, out_capacity, host_offsets, host_status);
}

int packos_pipeline_decode(packos_pipeline* p, const uint8_t* host_arena, const uint64_t* host_offsets, uint64_t stride,
                           size_t n, packos_column* host_cols, uint32_t* host_status) {
    if (!p) { set_error("packos_pipeline_decode: null pipeline"); return PACKOS_E_INVALID; }
    std::lock_guard<std::mutex> g(p->mu);
    DeviceGuard dg(p->device);
    return p->decode(host_arena, host_offsets, stride, n, host_cols, host_status);
}

int packos_pipeline_validate(packos_pipeline* p, const uint8_t* host_arena, const uint64_t* host_offsets,
                             uint64_t stride, size_t n, uint32_t* host_status) {
    if (!p) { set_error("packos_pipeline_validate: null pipeline"); return PACKOS_E_INVALID; }
    std::lock_guard<std::mutex> g(p->mu);
    DeviceGuard dg(p->device);
    return p->decode(host_arena, host_offsets, stride, n, nullptr, host_status, true);
}

int packos_encode_host_batch(const packos_schema* cs, const packos_column* hc, size_t n, uint8_t* host_out,
                             uint64_t out_capacity, uint64_t* host_offsets, uint32_t* host_status, size_t chunk_blobs) {
    if (!cs) { set_error("packos_encode_host_batch: bad argument"); return PACKOS_E_INVALID; }
    PipeLease L;
    HP_RC(lease(const_cast<packos_schema*>(cs), chunk_blobs, L));
    return L.p->encode(hc, n, host_out, out_capacity, host_offsets, host_status);
}

int packos_decode_host_batch(const packos_schema* cs, const uint8_t* host_arena, const uint64_t* host_offsets,
                             uint64_t stride, size_t n, packos_column* host_cols, uint32_t* host_status,
                             size_t chunk_blobs) {
    if (!cs) { set_error("packos_decode_host_batch: bad argument"); return PACKOS_E_INVALID; }
    PipeLease L;
    HP_RC(lease(const_cast<packos_schema*>(cs), chunk_blobs, L));
    return L.p->decode(host_arena, host_offsets, stride, n, host_cols, host_status);
}

int packos_validate_host_batch(const packos_schema* cs, const uint8_t* host_arena, const uint64_t* host_offsets,
                               uint64_t stride, size_t n, uint32_t* host_status, size_t chunk_blobs) {
    if (!cs) { set_error("packos_validate_host_batch: bad argument"); return PACKOS_E_INVALID; }
    PipeLease L;
    HP_RC(lease(const_cast<packos_schema*>(cs), chunk_blobs, L));
    return L.p->decode(host_arena, host_offsets, stride, n, nullptr, host_status, true);
}

}  // extern "C"
