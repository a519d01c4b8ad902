# k_encode_flat phase ablation (experiment builds only): ABL_NOCHUNK returns after
# the prologue (loads, per-blob offsets / static image / blob map)
s = open("encode_flat.inc").read()
a = "    const FTile<NV> T = flat_prologue<NV>(F, lds, lo, rows, n, offs, status, true);\n"
assert a in s
s = s.replace(a, a + "#ifdef ABL_NOCHUNK\n    if (T.o_end != ~0ull) return;\n#endif\n")
open("encode_flat.inc", "w").write(s)
