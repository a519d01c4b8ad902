"""Where do two encoders' bytes differ?  For the random-schema encode cases of
tests/test_gpu_parity.py (seeds x modes x offsets paths), run the library
PACKOS_LIB points at and report, per failing case, the kernel that ran, the
tile-relative position of every differing blob and byte, and which encode
item (header block / literal / fixed / var) the first differing bytes belong
to.  Diagnostic only (never a test): compares with the CPU oracle.

    PACKOS_LIB=abl/libpackos_x.so python tools/tiles_diag.py [seeds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import oracle_bridge as ob  # noqa: E402
from packos_amd import _lib  # noqa: E402
from packos_amd.columns import HostColumns  # noqa: E402
from schema_gen import rand_chain, rand_rows  # noqa: E402
from test_gpu_parity import gpu_encode  # noqa: E402


def main():
    import torch
    torch.cuda.init()   # the HIP runtime up before the library's first call
    seeds = range(int(sys.argv[1])) if len(sys.argv) > 1 else range(60)
    L = _lib.lib()
    dbg = hasattr(L, "packos_dbg_read")
    if dbg:
        import ctypes
        L.packos_dbg_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    nfail = 0
    for seed in seeds:
        chain = rand_chain(seed)
        n = 257 + 300 * (seed % 3)
        hc = HostColumns.from_rows(chain, rand_rows(chain, n, seed * 7 + 1))
        for mode in (0, 1):
            for fused in (False, True):
                a0, o0, s0 = ob.encode(chain, hc, mode, nthreads=8)
                if dbg:   # probe build (tools/patches/tiles_probe.py dbg): clear its tables
                    L.packos_dbg_read(None, None, 1)
                a1, o1, s1 = gpu_encode(chain, hc, mode, 0, fused, poison=True)
                enc = L.packos_last_encoder().decode() if hasattr(L, "packos_last_encoder") else "?"
                if np.array_equal(a0, a1) and np.array_equal(o0, o1) and np.array_equal(s0, s1):
                    continue
                nfail += 1
                bad = np.nonzero(a0 != a1)[0]
                blobs = np.unique(np.searchsorted(o0, bad, side="right") - 1)
                valid = [c for c, v in enumerate(hc.valid) if v is not None]
                print(f"FAIL seed {seed} mode {mode} fused {fused} n {n} kernel {enc}: {bad.size} bytes in "
                      f"{blobs.size} blobs; offsets equal {np.array_equal(o0, o1)}, status equal "
                      f"{np.array_equal(s0, s1)}; validity columns {valid}")
                print(f"   schema {chain!r}"[:400])
                tiles = np.unique(blobs // 128)
                print(f"   tiles {tiles[:20].tolist()} blob-in-tile {sorted(set((blobs % 128).tolist()))[:40]}")
                # runs of differing bytes: tile, offset from the tile's 16-B chunk
                # origin, and what was there (cd: never stored, 00: zero stored)
                runs, st_ = [], None
                for x in bad.tolist() + [None]:
                    if st_ is not None and (x is None or x != pv + 1):
                        runs.append((st_, pv + 1))
                        st_ = None
                    if x is not None and st_ is None:
                        st_ = x
                    pv = x
                spans = []   # top-level item spans (GetAccess GET_SPAN): which item a run lies in
                for k in range(len(chain.Schemas)):
                    _, _, _, tg, _ = ob.get_batch(a0, o0, n, [k], 2, values=False)
                    ss, sl, sst = np.zeros(n, np.int64), np.zeros(n, np.int64), np.ones(n, np.uint8)
                    for t_ in np.unique(tg):
                        _, s_, l_, _, st_2 = ob.get_batch(a0, o0, n, [k], 2, int(t_), -1, values=False)
                        m_ = (tg == t_) & (st_2 == 0)
                        ss[m_], sl[m_], sst[m_] = s_[m_], l_[m_], 0
                    spans.append((ss, sl, sst))
                for r0_, r1_ in runs[:8]:
                    bl = int(np.searchsorted(o0, r0_, side="right") - 1)
                    t = bl // 128
                    ga = int(o0[128 * t]) & ~15
                    got = a1[r0_:r1_]
                    kind = "cd" if (got == 0xCD).all() else "00" if (got == 0).all() else "mixed"
                    print(f"   run [{r0_},{r1_}) len {r1_ - r0_} tile {t} rel-ga [{r0_ - ga},{r1_ - ga}) "
                          f"chunks {(r0_ - ga) >> 4}..{(r1_ - 1 - ga) >> 4} got {kind} "
                          f"blob {bl} [{int(o0[bl])},{int(o0[bl + 1])}) items " + ",".join(
                              f"{k}:{chain.Schemas[k].kind}{'v' if chain.Schemas[k].variable else ''}[{int(ss[bl])},{int(ss[bl] + sl[bl])})"
                              for k, (ss, sl, sst) in enumerate(spans)
                              if sst[bl] == 0 and ss[bl] < r1_ and ss[bl] + sl[bl] > r0_))
                # tile 0's never-stored 16-B chunks as (wave, chunk step m, lane):
                # chunk c of a tile belongs to wave (c / 64) % 4, step c / 256, lane c % 64
                t0e = int(o0[min(128, n)])
                miss = sorted({(x >> 4) for x in bad.tolist() if x < t0e and a1[x] == 0xCD})
                print(f"   tile 0: {len(miss)} of {(t0e + 15) >> 4} chunks never stored; by (wave, m): " + "; ".join(
                    f"w{w} m{m}: lanes " + ",".join(str(c % 64) for c in miss if (c // 64) % 4 == w and c // 256 == m)
                    for m in range(4) for w in range(4)
                    if any((c // 64) % 4 == w and c // 256 == m for c in miss)))
                if dbg:
                    D = np.zeros(4096 * 8, np.uint64)
                    K = np.zeros(4096 * 2048, np.uint8)
                    L.packos_dbg_read(D.ctypes.data, K.ctypes.data, 0)
                    print(f"   tile 0 probe: HT {D[0]} NC {D[1]} ne {D[2]} org {D[3]} erel {D[4]} ga {D[5]} "
                          f"o_end {D[6]} written {D[7]}")
                    kc = K[:2048]
                    nc = int(D[1])
                    print("   tile 0 chunk kinds (0 none, 1 hole, 2 image, 3 edge listed, 7 edge stored): all " +
                          str({int(v): int((kc[:nc] == v).sum()) for v in np.unique(kc[:nc])}) +
                          "; never-stored " + str({int(v): sum(1 for c in miss if kc[c] == v) for v in
                                                   np.unique([kc[c] for c in miss])} if miss else {}))
                    print("   never-stored chunk: kind " + " ".join(f"{c}:{kc[c]}" for c in miss[:40]))
                for b in blobs[:2]:
                    lo, hi = int(o0[b]), int(o0[b + 1])
                    d = np.nonzero(a0[lo:hi] != a1[lo:hi])[0]
                    print(f"   blob {b} ({hi - lo} B) differs at {d[:16].tolist()}")
                    print(f"     want {a0[lo:hi][:64].tobytes().hex()}")
                    print(f"     got  {a1[lo:hi][:64].tobytes().hex()}")
                sys.stdout.flush()
    print(f"{nfail} failing cases")


if __name__ == "__main__":
    main()
