# K-rows variant: the next block's profile reads as asm volatile ds_read2_b32 at steps 0-7 (two per
# step, k = u/2), each pinned between its step and the next: the asm takes the step's D (the up value the next step adds its profile to)
# as an in-out operand ("+v", no instruction), so it issues after the step computed it and before the
# next step's DPP reads it.  The compiler does not count these reads; their results are used only in
# the next block, after the halo asm's lgkmcnt(0).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
rep("""// int16 half of a profile dword""", """template <int P>
__device__ __forceinline__ int2v q_rd2(uint32_t a, int& pin)
{
    int2v r;
    asm volatile("ds_read2_b32 %0, %2 offset0:%3 offset1:%4" : "=&v"(r), "+v"(pin) : "v"(a), "n"(2 * P), "n"(2 * P + 1));
    return r;
}
// int16 half of a profile dword""")
rep("""            if (u < 8)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);
""", "")
rep("""                if constexpr (CAP) va[k][u] = nh[k];
            }
""", """                if constexpr (CAP) va[k][u] = nh[k];
            }
            if (u < 2 * K)
            {
                const int kk = u >> 1;
                const int2v r0 = (u & 1) ? q_rd2<2>(qrow[kk] + pn, D) : q_rd2<0>(qrow[kk] + pn, D);
                const int2v r1 = (u & 1) ? q_rd2<3>(qrow[kk] + pn, D) : q_rd2<1>(qrow[kk] + pn, D);
                qn[kk][4 * (u & 1) + 0] = r0.x;
                qn[kk][4 * (u & 1) + 1] = r0.y;
                qn[kk][4 * (u & 1) + 2] = r1.x;
                qn[kk][4 * (u & 1) + 3] = r1.y;
            }
""")
