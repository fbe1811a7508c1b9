# nw_krow.hip variant: the loader's profile passes take 4 letters (8 passes per batch).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("""            int4v vm[2], v0[2], v1[2];
            {
                const uint32_t o = 32u * (uint32_t)qsub;
#pragma unroll
                for (int j = 0; j < 2; ++j)""", """            int4v vm[1], v0[1], v1[1];
            {
                const uint32_t o = 16u * (uint32_t)qsub;
#pragma unroll
                for (int j = 0; j < 1; ++j)""")
rep("""            for (int i = 0; i < 8; ++i)
            {
                const int yy = 8 * qsub + i;""", """            for (int i = 0; i < 4; ++i)
            {
                const int yy = 4 * qsub + i;""")
rep("""            if (++qsub == 4 || 8 * qsub >= a.substsz)""", """            if (++qsub == 8 || 4 * qsub >= a.substsz)""")
