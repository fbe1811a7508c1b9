# nw_lane.hip variant: int16 column profile in 2 copies (as the K-rows kernel's: dword d of copy p =
# columns (2d-p, 2d-p+1), lane l reads copy l & 1), so a strip reads its 16 columns of a block as 8
# dwords (4 ds_read2_b32 instead of 8); the loader builds 128 columns per batch.  |s - g| must fit
# int16 (error bit 2 otherwise).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:100], s.count(a))
    s = s.replace(a, b)
rep("""__host__ __device__ constexpr int lane_qrs(int ns) { return lane_lw(ns) + 32; }  // Q row stride in dwords: == 0 mod 32, 32 guard columns""",
    """__host__ __device__ constexpr int lane_qrs(int ns) { return lane_lw(ns) / 2 + 32; }  // Q row stride in dwords (int16 pairs): == 0 mod 32
// copy 1 of the profile: 16 banks from copy 0 (lanes 2m, 2m+1 read the same dword index)
__host__ __device__ constexpr uint32_t lane_copy1(int ns, int substsz) { return (uint32_t)substsz * lane_qrs(ns) + 16u; }""")
rep("""    L.sub = (uint32_t)substsz * lane_qrs(ns) * 4u;""", """    L.sub = (2u * lane_copy1(ns, substsz)) * 4u;""")
rep("""    const uint32_t qrow = L.q + (uint32_t)y * (kLQRS * 4u);""", """    const uint32_t qrow = L.q + 4u * ((uint32_t)(lane & 1) * lane_copy1(NS, a.substsz) + (uint32_t)y * kLQRS);
    constexpr int kQW = kLW / 2;""")
rep("""    int qA[kLBlk], qB[kLBlk];""", """    int qA[kLBlk / 2], qB[kLBlk / 2];""")
rep("""        const uint32_t qb = qrow + 4u * (uint32_t)((-lane) & (kLW - 1));
#pragma unroll
        for (int u = 0; u < kLBlk; ++u) qA[u] = lds_ld(qb + 4u * u);""", """        const uint32_t qb = qrow + 4u * (uint32_t)((-(lane >> 1)) & (kQW - 1));
#pragma unroll
        for (int u = 0; u < kLBlk / 2; ++u) qA[u] = lds_ld(qb + 4u * u);""")
rep("""    auto block = [&](int b, int (&qc)[kLBlk], int (&qn)[kLBlk], int4v (&hc)[kLH], int4v (&hn)[kLH], auto rampT) {""",
    """    auto block = [&](int b, int (&qc)[kLBlk / 2], int (&qn)[kLBlk / 2], int4v (&hc)[kLH], int4v (&hn)[kLH], auto rampT) {""")
rep("""            const uint32_t qb = qrow + 4u * (uint32_t)((kLBlk * b + kLBlk - lane) & (kLW - 1));
#pragma unroll
            for (int u = 0; u < kLBlk; ++u) qn[u] = lds_ld(qb + 4u * u);""", """            const uint32_t qb = qrow + 4u * (uint32_t)((8 * b + 8 - (lane >> 1)) & (kQW - 1));
#pragma unroll
            for (int u = 0; u < kLBlk / 2; ++u) qn[u] = lds_ld(qb + 4u * u);""")
rep("""            const int t1 = U + qc[u];""", """            const int t1 = U + ((u & 1) ? (qc[u >> 1] >> 16) : (int)(short)qc[u >> 1]);""")
# loader: 128 columns per batch, 2 copies
rep("""    int xl = letter(lane);""", """    int xm = letter(2 * lane - 1), x0 = letter(2 * lane), x1 = letter(2 * lane + 1);
    constexpr int kQW = kLW / 2;""")
rep("""        if (ROLE != 1 && qn <= C && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (ROLE != 1 && qn <= C && qn <= pl + kLW - 128)
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
        }""", """        if (ROLE != 1 && qn <= C && qn + 192 > pl + kLW) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (ROLE != 1 && qn <= C && qn + 192 <= pl + kLW)
        {
            // dword d = qn/2 + lane of copy 0 (columns 2d, 2d+1) and copy 1 (2d-1, 2d), 8 letters a pass
            const uint32_t d = (uint32_t)((qn / 2 + lane) & (kQW - 1));
            const bool guard = d < 8;  // ring head: also the guard copy at d + kQW
            const uint32_t sm = L.sub + 4u * kLSubRow * (uint32_t)xm, s0 = L.sub + 4u * kLSubRow * (uint32_t)x0;
            const uint32_t s1 = L.sub + 4u * kLSubRow * (uint32_t)x1;
            const uint32_t q0 = L.q + 4u * d, q1 = q0 + 4u * lane_copy1(NS, a.substsz);
#pragma unroll
            for (int j = 0; j < 8; ++j)
            {
                const int4v vm = lds_ld4(sm + 16u * j), v0 = lds_ld4(s0 + 16u * j), v1 = lds_ld4(s1 + 16u * j);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                {
                    const int yy = 4 * j + i;
                    if (yy < a.substsz)
                    {
                        const int p0 = (v0[i] & 0xffff) | (v1[i] << 16), p1 = (vm[i] & 0xffff) | (v0[i] << 16);
                        lds_st(q0 + 4u * kLQRS * yy, p0);
                        lds_st(q1 + 4u * kLQRS * yy, p1);
                        if (guard)
                        {
                            lds_st(q0 + 4u * (kLQRS * yy + kQW), p0);
                            lds_st(q1 + 4u * (kLQRS * yy + kQW), p1);
                        }
                    }
                }
            }
            qn += 128;
            xm = letter(qn + 2 * lane - 1);
            x0 = letter(qn + 2 * lane);
            x1 = letter(qn + 2 * lane + 1);
            flag_st(F + kFXo, qn > C ? kLBig : qn);
            moved = true;
        }""")
# int16 range check in the prologue
rep("""        lds_st(L.sub + 4u * k, yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - a.g : 0);
    }""", """        const int v = yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - a.g : 0;
        if (v < -32768 || v > 32767) atomicOr(a.err, 2u);  // the profile holds int16
        lds_st(L.sub + 4u * k, v);
    }""")
