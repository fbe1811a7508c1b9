# Timing build of nw_krow.hip: per-block s_memtime stamps of the first 32 strips of a pair (tickets
# 0..7): block entry (before the progress check), block start (check passed), hand-off published.
# Read back with gsa_dbg_kst (tools/kr_stamps.py).  Diagnostics only; perturbs the kernel slightly.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, a
    s = s.replace(a, b)

rep("extern __shared__ __attribute__((aligned(16))) char krsm[];",
    "extern __shared__ __attribute__((aligned(16))) char krsm[];\n__device__ unsigned long long g_kst[32][6400][3];")
rep("""        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);""",
"""        const unsigned long long st0 = __builtin_amdgcn_s_memtime();
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);""")
rep("""        halo_load(b);
        const uint32_t pn = q_off(b + 1);""", """        const unsigned long long st1 = __builtin_amdgcn_s_memtime();
        halo_load(b);
        const uint32_t pn = q_off(b + 1);""")
rep("""        handoff(b);
        if (CAP && cap)""", """        handoff(b);
        {
            const unsigned long long st2 = __builtin_amdgcn_s_memtime();
            if (tk < 8 && b < 6400 && lane == 0)
            {
                g_kst[tk * NS + w][b][0] = st0;
                g_kst[tk * NS + w][b][1] = st1;
                g_kst[tk * NS + w][b][2] = st2;
            }
        }
        if (CAP && cap)""")
s += """
extern "C" int gsa_dbg_kst(void* dst, size_t n)
{
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(gsa::g_kst), n, 0, hipMemcpyDeviceToHost);
}
"""

# loader / drain stamps: time at which the drain has stored, and the loader has fed into ring 0,
# the columns < 16 c (c = 0 .. 6399), tickets 0..7
rep("__device__ unsigned long long g_kst[32][6400][3];",
    "__device__ unsigned long long g_kst[32][6400][3];\n__device__ unsigned long long g_kld[8][6400][2];")
rep("""                hnext += n;""", """                {
                    const unsigned long long tn = __builtin_amdgcn_s_memtime();
                    if (tk < 8 && lane == 0)
                        for (int c = hnext / 16 + 1; c <= (hnext + n) / 16 && c < 6400; ++c) g_kld[tk][c][0] = tn;
                }
                hnext += n;""")
rep("""                dnext = min(dnext + 64, avail);
                flag_st(F + kr_cons(NS), dnext > Cp ? kBig : dnext + 64);
                last = __builtin_amdgcn_s_memrealtime();""", """                {
                    const int dn = min(dnext + 64, avail);
                    const unsigned long long tn = __builtin_amdgcn_s_memtime();
                    if (tk < 8 && lane == 0)
                        for (int c = dnext / 16 + 1; c <= dn / 16 && c < 6400; ++c) g_kld[tk][c][1] = tn;
                }
                dnext = min(dnext + 64, avail);
                flag_st(F + kr_cons(NS), dnext > Cp ? kBig : dnext + 64);
                last = __builtin_amdgcn_s_memrealtime();""")
s += """
extern "C" int gsa_dbg_kld(void* dst, size_t n)
{
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(gsa::g_kld), n, 0, hipMemcpyDeviceToHost);
}
"""
