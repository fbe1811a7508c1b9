# nw_lane.hip variant: the loader writes a 64-column Q pass in two halves of 16 letters, one per
# loop iteration, so the granule poll is consumed and re-issued between them (as nw_krow's loader).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a[:80]
    s = s.replace(a, b)
rep("""    int xl = letter(lane);""", """    int xl = letter(lane);
    int qh = 0;  // next half (16 letters) of the pass at qn""")
rep("""        if (qn <= C && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (qn <= C && qn <= pl + kLW - 128)
        {
            const uint32_t p = (uint32_t)((qn + lane) & (kLW - 1));
            const uint32_t sb = L.sub + 4u * kLSubRow * (uint32_t)xl;
            int4v v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = lds_ld4(sb + 16u * j);
            const uint32_t qa = L.q + 4u * p;
#pragma unroll
            for (int yy = 0; yy < 32; ++yy)
                if (yy < a.substsz) lds_st(qa + 4u * kLQRS * yy, v[yy >> 2][yy & 3]);
            if ((qn & (kLW - 1)) == 0 && lane < kLBlk)
            {
                // guard copy of columns p < kLBlk at p + kLW: a block's reads run past the wrap
#pragma unroll
                for (int yy = 0; yy < 32; ++yy)
                    if (yy < a.substsz) lds_st(qa + 4u * (kLQRS * yy + kLW), v[yy >> 2][yy & 3]);
            }
            qn += 64;
            xl = letter(qn + lane);
            flag_st(F + kFXo, qn > C ? kLBig : qn);
            moved = true;
        }""", """        if (qh == 0 && qn <= C && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (qh > 0 || (qn <= C && qn <= pl + kLW - 128))
        {
            const uint32_t p = (uint32_t)((qn + lane) & (kLW - 1));
            const uint32_t sb = L.sub + 4u * kLSubRow * (uint32_t)xl + 64u * (uint32_t)qh;
            int4v v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = lds_ld4(sb + 16u * j);
            const uint32_t qa = L.q + 4u * p;
#pragma unroll
            for (int i = 0; i < 16; ++i)
            {
                const int yy = 16 * qh + i;
                if (yy < a.substsz) lds_st(qa + 4u * kLQRS * yy, v[i >> 2][i & 3]);
            }
            if ((qn & (kLW - 1)) == 0 && lane < kLBlk)
            {
                // guard copy of columns p < kLBlk at p + kLW: a block's reads run past the wrap
#pragma unroll
                for (int i = 0; i < 16; ++i)
                {
                    const int yy = 16 * qh + i;
                    if (yy < a.substsz) lds_st(qa + 4u * (kLQRS * yy + kLW), v[i >> 2][i & 3]);
                }
            }
            if (++qh == 2 || 16 * qh >= a.substsz)
            {
                qh = 0;
                qn += 64;
                xl = letter(qn + lane);
                flag_st(F + kFXo, qn > C ? kLBig : qn);
            }
            moved = true;
        }""")
