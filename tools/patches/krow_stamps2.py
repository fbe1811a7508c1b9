# Timing build of nw_krow.hip: per-block s_memtime stamps of the first 32 strips (tickets 0..7): block
# entry, check passed, hand-off published, plus which readiness condition failed at the first check
# (bit 0 halo/prog, bit 1 ring room/cons, bit 2 profile/xo).  Read back with gsa_dbg_kst2
# (tools/kr_stamps2.py).  Diagnostics only.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)

rep("extern __shared__ __attribute__((aligned(16))) char krsm[];",
    "extern __shared__ __attribute__((aligned(16))) char krsm[];\n__device__ unsigned long long g_kst[32][6400][4];")
rep("""        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }""",
"""        const unsigned long long st0 = __builtin_amdgcn_s_memtime();
        unsigned long long why = 0;
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            why = (pin >= kBlk * b + 64 + kBlk ? 0 : 1) | (pco >= kBlk * b + kBlk - kRing ? 0 : 2) |
                  ((w != 0 || pxo >= kBlk * b + 2 * kBlk) ? 0 : 4);
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        const unsigned long long st1 = __builtin_amdgcn_s_memtime();""")
rep("""        handoff(b);
        if (CAP && cap)""", """        handoff(b);
        {
            const unsigned long long st2 = __builtin_amdgcn_s_memtime();
            if (tk < 8 && b < 6400 && lane == 0)
            {
                g_kst[tk * NS + w][b][0] = st0;
                g_kst[tk * NS + w][b][1] = st1;
                g_kst[tk * NS + w][b][2] = st2;
                g_kst[tk * NS + w][b][3] = why;
            }
        }
        if (CAP && cap)""")
s += """
extern "C" int gsa_dbg_kst2(void* dst, size_t n)
{
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(gsa::g_kst), n, 0, hipMemcpyDeviceToHost);
}
"""
