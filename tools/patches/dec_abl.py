# decode phase ablation switches (experiment builds only): ABL_NOCOL skips the
# fixed decoder's column stores, ABL_NOCHK its constant-byte check, ABL_NOST
# its status stores
s = open("kernels.hip").read()
a = "    // 3. columns: uniform walk over the columns; threads stride the column's"
assert a in s
s = ("#ifndef ABL_NOCOL\n#define ABL_NOCOL 0\n#endif\n#ifndef ABL_NOCHK\n#define ABL_NOCHK 0\n#endif\n"
     "#ifndef ABL_NOST\n#define ABL_NOST 0\n#endif\n") + s
s = s.replace("    for (int c = 0; c < K.n; c++) {\n        struct { uint8_t* dst;", "    for (int c = 0; !ABL_NOCOL && c < K.n; c++) {\n        struct { uint8_t* dst;")
b = "        for (uint32_t e = ct; e < rows * nq; e += NCT) {"
assert b in s
s = s.replace(b, "        for (uint32_t e = ct; !ABL_NOCHK && e < rows * nq; e += NCT) {")
c = """#ifdef PACKOS_DEC_STNT
        __builtin_nontemporal_store(sv, status + i);
#else
        status[i] = sv;
#endif
    }
}"""
assert c in s
s = s.replace(c, """        if (!ABL_NOST) status[i] = sv;
    }
}""")
open("kernels.hip", "w").write(s)
