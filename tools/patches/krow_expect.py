# nw_krow.hip variant: the block's common path falls through (branch weights on the progress
# check and the capture; strip 0's profile word read by every strip, no branch on w).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:80], s.count(a))
    s = s.replace(a, b)
rep("""            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;""",
    """            const int pxo = __builtin_amdgcn_readfirstlane(rpxo);
            if (__builtin_expect(!ok(pin, pco, pxo, b), 0) && !spin(b)) return false;""")
rep("""        if (CAP && cap)""", """        if (CAP && __builtin_expect(cap, 0))""")
