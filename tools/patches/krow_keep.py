# nw_krow.hip variant: the step-14 progress read's 4 words stay live until the next block's check
# (an empty asm takes them all), so the compiler does not reuse the unread words' registers and
# wait for the read at the block end.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)
rep("""    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block""",
    """    int2v rlo = int2v {0, 0}, rhi = int2v {0, 0};  // progress words read in mid-block, checked at the next block""")
rep("""            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;""",
    """            asm volatile("" : "+v"(rlo), "+v"(rhi));
            const int pin = __builtin_amdgcn_readfirstlane(rlo.x), pco = __builtin_amdgcn_readfirstlane(rhi.y);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rlo.y) : 0;""")
rep("""                rpin = lo.x;
                rpxo = lo.y;
                rpco = hi.y;""", """                rlo = lo;
                rhi = hi;""")
