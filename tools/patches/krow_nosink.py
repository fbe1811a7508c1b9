# nw_krow.hip without the dead LDS regions (zfill, sink) and the zero-row stores.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("    uint32_t q, sub, ring, zfill, sink, flags;", "    uint32_t q, sub, ring, flags;")
rep("""    L.zfill = L.ring + (uint32_t)(ns + 1) * kRing * 4u;
    L.sink = L.zfill + 64u;
    L.flags = L.sink + (uint32_t)ns * 1024u;""", """    L.flags = L.ring + (uint32_t)(ns + 1) * kRing * 4u;""")
rep("    if (threadIdx.x < 16) lds_st(L.zfill + 4u * threadIdx.x, 0);\n", "")
