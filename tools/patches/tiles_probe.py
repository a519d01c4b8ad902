# Experiment builds only (refactor investigation): applied to a
# COPY of packos_amd/csrc by tools/abl_build.sh-style scripts, never to the
# product.  Usage: python tiles_probe.py <csrc copy> [planptr] [flatptr] [dbg]
#   planptr: k_encode_tiles reads its plan through an opaque pointer to the
#            kernel-argument segment (same values, different load placement)
#   flatptr: the same for k_encode_flat's plan
#   dbg:     per-tile layout values and per-chunk classification of the
#            non-closed-form chunk passes into device globals, read back by
#            packos_dbg_read() (tools/tiles_diag.py --dbg)
import sys

d = sys.argv[1]
opts = set(sys.argv[2:])
p = d + "/encode_var.inc"
s = open(p).read()


def sub(old, new, count=1):
    global s
    assert s.count(old) >= count, old
    s = s.replace(old, new, count)


if "planptr" in opts:
    sub("""    VPlan V, uint64_t* __restrict__ offs, uint8_t* __restrict__ out, uint64_t cap, uint64_t n,
    uint32_t* __restrict__ status) {
#else""", """    VPlan V_, uint64_t* __restrict__ offs, uint8_t* __restrict__ out, uint64_t cap, uint64_t n,
    uint32_t* __restrict__ status) {
    typedef __attribute__((address_space(4))) const VPlan c_plan;
    c_plan* vp4 = (c_plan*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(vp4));
    const VPlan& V = *(const VPlan*)vp4;
#else""")
if "flatptr" in opts:   # the same perturbation of k_encode_flat (encode_flat.inc)
    q = d + "/encode_flat.inc"
    f = open(q).read()
    old = """void k_encode_flat(FPlan F, uint64_t* __restrict__ offs, uint8_t* __restrict__ out,
                                                      uint64_t cap, uint64_t n, uint32_t* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];"""
    assert old in f, "flat signature"
    f = f.replace(old, """void k_encode_flat(FPlan F_, uint64_t* __restrict__ offs, uint8_t* __restrict__ out,
                                                      uint64_t cap, uint64_t n, uint32_t* __restrict__ status) {
    typedef __attribute__((address_space(4))) const FPlan c_fplan;
    c_fplan* fp4 = (c_fplan*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(fp4));
    const FPlan& F = *(const FPlan*)fp4;
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];""")
    open(q, "w").write(f)
if "dbg" in opts:
    sub("""// k_encode_tiles helpers
""", """// k_encode_tiles helpers
__device__ unsigned long long g_tdbg[4096 * 8];
__device__ unsigned char g_tkind[4096 * 2048];
""")
    if "            if (valid && !in_hole && !in_img) edges[atomicAdd(ne_cnt, 1u)] = c;" in s:   # round-6 form
        sub("""            if (valid && !in_hole && !in_img) edges[atomicAdd(ne_cnt, 1u)] = c;""",
            """            if (valid && !in_hole && !in_img) edges[atomicAdd(ne_cnt, 1u)] = c;
            if (valid && !in_hole && !in_img && blockIdx.x < 4096 && c < 2048) g_tkind[blockIdx.x * 2048 + c] = 3;""")
    else:
        sub("""                    edges[atomicAdd(ne_cnt, 1u)] = c;""",
            """                    edges[atomicAdd(ne_cnt, 1u)] = c;
                    if (blockIdx.x < 4096 && c < 2048) g_tkind[blockIdx.x * 2048 + c] = 3;""")
    sub("""            if (kind[m] == 1) store_chunk(out, ga, 16u * c, org, erel, a0[m]);""",
        """            if (blockIdx.x < 4096 && c < 2048 && kind[m]) g_tkind[blockIdx.x * 2048 + c] = (unsigned char)kind[m];
            if (kind[m] == 1) store_chunk(out, ga, 16u * c, org, erel, a0[m]);""")
    sub("""    const uint32_t ne = *ne_cnt;""", """    const uint32_t ne = *ne_cnt;
    if (tid == 0 && blockIdx.x < 4096) {
        unsigned long long* D = g_tdbg + blockIdx.x * 8;
        D[0] = HT; D[1] = NC; D[2] = ne; D[3] = org; D[4] = erel; D[5] = ga; D[6] = o_end; D[7] = 1;
    }""")
    sub("""            store_chunk(out, ga, R, org, erel, o);""", """            if (blockIdx.x < 4096 && c < 2048) g_tkind[blockIdx.x * 2048 + c] |= 4;
            store_chunk(out, ga, R, org, erel, o);""")
    k = open(d + "/kernels.hip").read()
    k = k.replace("""const char* packos_last_encoder(void) { return g_last_encoder; }""",
                  """const char* packos_last_encoder(void) { return g_last_encoder; }
int packos_dbg_read(void* tdbg, void* tkind, int clear) {
    if (tdbg && hipMemcpyFromSymbol(tdbg, HIP_SYMBOL(g_tdbg), sizeof(g_tdbg)) != hipSuccess) return -1;
    if (tkind && hipMemcpyFromSymbol(tkind, HIP_SYMBOL(g_tkind), sizeof(g_tkind)) != hipSuccess) return -1;
    if (clear) {
        static unsigned long long z8[4096 * 8];
        static unsigned char zk[4096 * 2048];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tdbg), z8, sizeof(z8)) != hipSuccess) return -1;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tkind), zk, sizeof(zk)) != hipSuccess) return -1;
    }
    return 0;
}""")
    open(d + "/kernels.hip", "w").write(k)
open(p, "w").write(s)
