# K-rows variant: the next block's profile reads issued at block start, right after the halo read
# (pinned with a scheduling barrier), instead of interleaved over steps 0-7 (the compiler clusters
# them after step ~7, in front of the step-14 progress read in the wave's in-order LDS queue).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("""        halo_load(b);
        const uint32_t pn = q_off(b + 1);""", """        halo_load(b);
        const uint32_t pn = q_off(b + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int k = 0; k < K; ++k) qn[k][j] = lds_ld(qrow[k] + pn + 4u * j);
        __builtin_amdgcn_sched_barrier(0);""")
rep("""            if (u < 8)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);
""", "")
