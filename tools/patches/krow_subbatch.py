# nw_krow.hip variant: the loader builds a 128-column profile batch in 4 passes of 8 letters, one
# per loop iteration, so the granule poll is consumed and re-issued between them (the feed delay's
# tail sets strip 0's lag).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("""    int xm = letter(2 * lane - 1), x0 = letter(2 * lane), x1 = letter(2 * lane + 1);""",
    """    int xm = letter(2 * lane - 1), x0 = letter(2 * lane), x1 = letter(2 * lane + 1);
    int nxm = 0, nx0 = 0, nx1 = 0;  // the batch after (loaded in pass 0)
    int qsub = 0;                   // next pass (8 letters each) of the batch at qn""")
rep("""        if (qn <= Cp && qn + 192 > pl + kLW) pl = flag_ld(F + kr_prog(NS));
        if (qn <= Cp && qn + 192 <= pl + kLW)
        {
            int4v vm[8], v0[8], v1[8];
            subrow(xm, vm);
            subrow(x0, v0);
            subrow(x1, v1);
            {
                const int cn = qn + kBatch + 2 * lane;
                xm = letter(cn - 1);
                x0 = letter(cn);
                x1 = letter(cn + 1);
            }
            const uint32_t d = (uint32_t)((qn / 2 + lane) & (kQW - 1));  // dword of columns (cl, cl+1) / (cl-1, cl)
            const bool guard = d < 8;                                     // ring head: also the guard copy at d + kQW
#pragma unroll
            for (int yy = 0; yy < 32; ++yy)
            {
                if (yy < a.substsz)
                {
                    const int s0 = v0[yy >> 2][yy & 3];
                    const int p0 = (s0 & 0xffff) | (v1[yy >> 2][yy & 3] << 16);  // copy 0: (cl, cl+1)
                    const int p1 = (vm[yy >> 2][yy & 3] & 0xffff) | (s0 << 16);  // copy 1: (cl-1, cl)
                    const uint32_t r0a = L.q + 4u * (kQRS * (uint32_t)yy + d);
                    const uint32_t r1a = L.q + 4u * (kr_copy1(LW, a.substsz) + kQRS * (uint32_t)yy + d);
                    lds_st(r0a, p0);
                    lds_st(r1a, p1);
                    if (guard)
                    {
                        lds_st(r0a + 4u * kQW, p0);
                        lds_st(r1a + 4u * kQW, p1);
                    }
                }
            }
            qn += kBatch;
            flag_st(F + kFXo, qn > Cp ? kBig : qn);
            moved = true;
        }""", """        if (qsub == 0 && qn <= Cp && qn + 192 > pl + kLW) pl = flag_ld(F + kr_prog(NS));
        if (qsub > 0 || (qn <= Cp && qn + 192 <= pl + kLW))
        {
            // letters yy = 8 qsub .. 8 qsub + 7: dwords 2 qsub, 2 qsub + 1 of the three subT rows
            int4v vm[2], v0[2], v1[2];
            {
                const uint32_t o = 32u * (uint32_t)qsub;
#pragma unroll
                for (int j = 0; j < 2; ++j)
                {
                    vm[j] = lds_ld4(L.sub + 4u * kSubRow * (uint32_t)xm + o + 16u * j);
                    v0[j] = lds_ld4(L.sub + 4u * kSubRow * (uint32_t)x0 + o + 16u * j);
                    v1[j] = lds_ld4(L.sub + 4u * kSubRow * (uint32_t)x1 + o + 16u * j);
                }
            }
            if (qsub == 0)
            {
                const int cn = qn + kBatch + 2 * lane;
                nxm = letter(cn - 1);
                nx0 = letter(cn);
                nx1 = letter(cn + 1);
            }
            const uint32_t d = (uint32_t)((qn / 2 + lane) & (kQW - 1));  // dword of columns (cl, cl+1) / (cl-1, cl)
            const bool guard = d < 8;                                     // ring head: also the guard copy at d + kQW
#pragma unroll
            for (int i = 0; i < 8; ++i)
            {
                const int yy = 8 * qsub + i;
                if (yy < a.substsz)
                {
                    const int s0 = v0[i >> 2][i & 3];
                    const int p0 = (s0 & 0xffff) | (v1[i >> 2][i & 3] << 16);  // copy 0: (cl, cl+1)
                    const int p1 = (vm[i >> 2][i & 3] & 0xffff) | (s0 << 16);  // copy 1: (cl-1, cl)
                    const uint32_t r0a = L.q + 4u * (kQRS * (uint32_t)yy + d);
                    const uint32_t r1a = L.q + 4u * (kr_copy1(LW, a.substsz) + kQRS * (uint32_t)yy + d);
                    lds_st(r0a, p0);
                    lds_st(r1a, p1);
                    if (guard)
                    {
                        lds_st(r0a + 4u * kQW, p0);
                        lds_st(r1a + 4u * kQW, p1);
                    }
                }
            }
            if (++qsub == 4 || 8 * qsub >= a.substsz)
            {
                qsub = 0;
                xm = nxm;
                x0 = nx0;
                x1 = nx1;
                qn += kBatch;
                flag_st(F + kFXo, qn > Cp ? kBig : qn);
            }
            moved = true;
        }""")
