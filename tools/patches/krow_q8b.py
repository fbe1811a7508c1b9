# nw_krow.hip variant (krow_q8.py with the loader's ring width fixed): int8 column profile in 4 byte-shifted copies (copy p = lane & 3), so a lane
# reads its 16 columns of a row as 4 dwords (2 ds_read2_b32) instead of 8; |s - 2g| <= 127 only.
def rep(a, b, n=1):
    global s
    assert s.count(a) >= n, (a[:90], s.count(a))
    s = s.replace(a, b, 1)
rep("__host__ __device__ constexpr int kr_qrs(int lw) { return lw / 2 + 32; }",
    "__host__ __device__ constexpr int kr_qrs(int lw) { return lw / 4 + 32; }")
rep("__host__ __device__ constexpr uint32_t kr_copy1(int lw, int substsz) { return (uint32_t)substsz * kr_qrs(lw) + 16u; }",
    "__host__ __device__ constexpr uint32_t kr_copy1(int lw, int substsz) { return (uint32_t)substsz * kr_qrs(lw) + 8u; }\n"
    "// copy p (p = 0..3, 8 banks apart) at dword p * kr_copy1\n")
rep("    L.sub = (kr_copy1(lw, substsz) + (uint32_t)substsz * kr_qrs(lw) + 16u) * 4u;",
    "    L.sub = 4u * kr_copy1(lw, substsz) * 4u;")
rep("""    constexpr int kQW = kLW / 2;  // profile dwords per copy row (ring)""", """    constexpr int kQW = kLW / 4;  // profile dwords per copy row (ring)""")
rep("""        qrow[k] = L.q + 4u * ((lane & 1) * kr_copy1(LW, a.substsz) + (uint32_t)y * kQRS);""",
    """        qrow[k] = L.q + 4u * ((lane & 3) * kr_copy1(LW, a.substsz) + (uint32_t)y * kQRS);""")
rep("""    auto q_off = [&](int b) { return 4u * (uint32_t)((8 * b - (lane >> 1)) & (kQW - 1)); };
    int qA[K][8], qB[K][8];""", """    auto q_off = [&](int b) { return 4u * (uint32_t)((4 * b - (lane >> 2)) & (kQW - 1)); };
    int qA[K][4], qB[K][4];""")
rep("""            for (int j = 0; j < 8; ++j) qA[k][j] = 0;""", """            for (int j = 0; j < 4; ++j) qA[k][j] = 0;""")
rep("""            for (int j = 0; j < 8; ++j) qA[k][j] = lds_ld(qrow[k] + p + 4u * j);""", """            for (int j = 0; j < 4; ++j) qA[k][j] = lds_ld(qrow[k] + p + 4u * j);""")
rep("""    auto block = [&](int b, int (&qc)[K][8], int (&qn)[K][8], auto rampT, bool cap) {""",
    """    auto block = [&](int b, int (&qc)[K][4], int (&qn)[K][4], auto rampT, bool cap) {""")
rep("""                const int q = (u & 1) ? qhi(qc[0][u >> 1]) : qlo(qc[0][u >> 1]);""",
    """                const int q = (int)(signed char)(qc[0][u >> 2] >> (8 * (u & 3)));""")
rep("""                const int q = (u & 1) ? qhi(qc[k][u >> 1]) : qlo(qc[k][u >> 1]);""",
    """                const int q = (int)(signed char)(qc[k][u >> 2] >> (8 * (u & 3)));""")
rep("""            if (u < 8)""", """            if (u < 4)""")
# loader: letters 4d-1-2cp .. 4d+3-2cp, copies 2cp (even) and 2cp+1 (odd)
rep("""    int xm = letter(2 * lane - 1), x0 = letter(2 * lane), x1 = letter(2 * lane + 1);
    int nxm = 0, nx0 = 0, nx1 = 0;  // the batch after (loaded in pass 0)""",
"""    const int cp = lane >> 5;                       // copies 2cp, 2cp+1
    const int lb = 4 * (lane & 31) - 1 - 2 * cp;    // first column of the lane's 5 letters, batch-relative
    int xl[5], nxl[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) xl[i] = letter(lb + i), nxl[i] = 0;""")
rep("""            int4v vm[2], v0[2], v1[2];
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
                x1 = nx1;""", """            int4v vx[5][2];
            {
                const uint32_t o = 32u * (uint32_t)qsub;
#pragma unroll
                for (int i = 0; i < 5; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) vx[i][j] = lds_ld4(L.sub + 4u * kSubRow * (uint32_t)xl[i] + o + 16u * j);
            }
            if (qsub == 0)
            {
#pragma unroll
                for (int i = 0; i < 5; ++i) nxl[i] = letter(qn + kBatch + lb + i);
            }
            // dword d of copy p holds columns 4d-p .. 4d-p+3 (int8); lanes 0-31 copies 0/1, 32-63 copies 2/3
            const uint32_t d = (uint32_t)((qn / 4 + (lane & 31)) & (kQW - 1));
            const bool guard = d < 4;  // ring head: also the guard copy at d + kQW
            const uint32_t ce = L.q + 4u * ((uint32_t)(2 * cp) * kr_copy1(LW, a.substsz) + d);
            const uint32_t co = ce + 4u * kr_copy1(LW, a.substsz);
#pragma unroll
            for (int i = 0; i < 8; ++i)
            {
                const int yy = 8 * qsub + i;
                if (yy < a.substsz)
                {
                    const int w0 = vx[0][i >> 2][i & 3], w1 = vx[1][i >> 2][i & 3], w2 = vx[2][i >> 2][i & 3];
                    const int w3 = vx[3][i >> 2][i & 3], w4 = vx[4][i >> 2][i & 3];
                    const int lo = (w0 & 0xff) | ((w1 & 0xff) << 8) | ((w2 & 0xff) << 16) | (w3 << 24);  // odd copy
                    const int ev = (int)__builtin_amdgcn_alignbyte((unsigned)w4, (unsigned)lo, 1u);   // even copy
                    const uint32_t ra = 4u * kQRS * (uint32_t)yy;
                    lds_st(ce + ra, ev);
                    lds_st(co + ra, lo);
                    if (guard)
                    {
                        lds_st(ce + ra + 4u * kQW, ev);
                        lds_st(co + ra + 4u * kQW, lo);
                    }
                }
            }
            if (++qsub == 4 || 8 * qsub >= a.substsz)
            {
                qsub = 0;
#pragma unroll
                for (int i = 0; i < 5; ++i) xl[i] = nxl[i];""")
rep("""        bad |= v < -32768 || v > 32767;  // the profile holds int16""", """        bad |= v < -128 || v > 127;  // the profile holds int8""")
rep("""    constexpr int kLW = LW, kQRS = kr_qrs(LW), kQW = kLW / 2;""", """    constexpr int kLW = LW, kQRS = kr_qrs(LW), kQW = kLW / 4;""")
