# nw_krow.hip variant: header-column stores through a buffer resource of the strip's tile row,
# every lane storing and the other lane groups' stores dropped by the range check (offset past
# the records): no exec branch, 32-bit offsets.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:80], s.count(a))
    s = s.replace(a, b)
rep("""    gptr<int> hcolP = G(a.hcol) + ((size_t)iT * (size_t)tcols + 1) * (size_t)(tBy + 1) + ea;""",
"""    // the strip's tile row of tileHcolMat as a buffer: tile jT of it at ints jT * (tBy + 1)
    const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.hcol + (size_t)iT * (size_t)tcols * (size_t)(tBy + 1)), 0, tcols * (tBy + 1) * 4, 0x00020000);
    uint32_t hoff = 4u * (uint32_t)((tBy + 1) + ea);  // tile column jb = 1, element ea""")
rep("""            const int gb = (rl + kBlk * nbb) * g;  // un-shift: + (row + bc) g
            if ((lane >> 4) == b - nbb)
            {
#pragma unroll
                for (int k = 0; k < K; ++k) hcolP[k] = v[k] + gb + k * g;
            }""", """            const int gb = (rl + kBlk * nbb) * g;  // un-shift: + (row + bc) g
            // lanes of the other groups store past the buffer's records: dropped
            const uint32_t off = ((lane >> 4) == b - nbb) ? hoff : 0x7ffffff0u;
            if constexpr (K == 4)
                __builtin_amdgcn_raw_buffer_store_b128(int4v {v[0] + gb, v[1] + gb + g, v[2] + gb + 2 * g, v[3] + gb + 3 * g},
                                                       hrs, off, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b64(int2v {v[0] + gb, v[1] + gb + g}, hrs, off, 0, 0);""")
rep("""                hcolP += (size_t)(tBy + 1);""", """                hoff += 4u * (uint32_t)(tBy + 1);""")
