# nw_krow.hip variant: one profile buffer: dword j of a row is re-read for the next block right
# after its last use (step 2j+1), ~15 steps before the next block needs it (32 fewer VGPRs).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:80], s.count(a))
    s = s.replace(a, b)
rep("""            if (u < 8)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);""",
"""            if (u & 1)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u >> 1] = lds_ld(qrow[k] + pn + 4u * (u >> 1));""")
rep("""        if (!block(b, qA, qB, T(), false)) return;
        if (!block(b + 1, qB, qA, T(), false)) return;""", """        if (!block(b, qA, qA, T(), false)) return;
        if (!block(b + 1, qA, qA, T(), false)) return;""")
rep("""        if (!block(b, qA, qB, F(), advance(b))) return;""", """        if (!block(b, qA, qA, F(), advance(b))) return;""")
rep("""        if (!block(b + 1, qB, qA, F(), advance(b + 1))) return;""", """        if (!block(b + 1, qA, qA, F(), advance(b + 1))) return;""")
