# K-rows variant: the next block's profile reads pinned at steps 0-7 (K reads per step, a scheduling
# barrier after each step's reads) instead of clustered by the compiler after step 7, so the wave's
# LDS queue has drained before the step-14 progress read.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
rep("""            if (u < 8)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);""", """            if (u < 8)
            {
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);
                __builtin_amdgcn_sched_barrier(0);
            }""")
