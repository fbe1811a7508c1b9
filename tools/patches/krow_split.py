# nw_krow.hip variant: the loader's two jobs in two waves: a feeder (granule polls -> ring 0) and a
# profiler (profile passes), so the feed is never behind a pass (workgroup of NS + 3 waves).
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:80], s.count(a))
    s = s.replace(a, b)
rep("""template <int NS, int K, int LW>
__device__ __forceinline__ void kr_loader(const StripArgs& a, const KrLds& L, int tk, int lane)
{""", """template <int NS, int K, int LW, int ROLE>
__device__ __forceinline__ void kr_loader(const StripArgs& a, const KrLds& L, int tk, int lane)
{""")
rep("""    while (qn <= Cp || hnext <= Cp)
    {
        bool moved = false;""", """    while ((ROLE != 1 && qn <= Cp) || (ROLE != 2 && hnext <= Cp))
    {
        bool moved = false;""")
rep("""        if (hnext <= Cp && hnext + 128 > c0 + kRing) c0 = flag_ld(F + kr_cons(0));
        const bool feed = hnext <= Cp && hnext + 128 <= c0 + kRing;""", """        if (ROLE != 2 && hnext <= Cp && hnext + 128 > c0 + kRing) c0 = flag_ld(F + kr_cons(0));
        const bool feed = ROLE != 2 && hnext <= Cp && hnext + 128 <= c0 + kRing;""")
rep("""        if (qsub == 0 && qn <= Cp && qn + 192 > pl + kLW) pl = flag_ld(F + kr_prog(NS));
        if (qsub > 0 || (qn <= Cp && qn + 192 <= pl + kLW))""", """        if (ROLE != 1 && qsub == 0 && qn <= Cp && qn + 192 > pl + kLW) pl = flag_ld(F + kr_prog(NS));
        if (ROLE != 1 && (qsub > 0 || (qn <= Cp && qn + 192 <= pl + kLW)))""")
rep("""            if (tk == 0 || hnext > Cp) __builtin_amdgcn_s_sleep(1);""", """            if (ROLE == 2 || tk == 0 || hnext > Cp) __builtin_amdgcn_s_sleep(1);""")
rep("""__global__ void __launch_bounds__(64 * (NS + 2)) nw_krow_kernel(StripArgs a)""", """__global__ void __launch_bounds__(64 * (NS + 3)) nw_krow_kernel(StripArgs a)""")
rep("""    for (int k = threadIdx.x; k < a.substsz * kSubRow; k += 64 * (NS + 2))""", """    for (int k = threadIdx.x; k < a.substsz * kSubRow; k += 64 * (NS + 3))""")
rep("""            kr_loader<NS, K, LW>(pa, L, tk, lane);""", """            kr_loader<NS, K, LW, 1>(pa, L, tk, lane);
        else if (w == NS + 2)
            kr_loader<NS, K, LW, 2>(pa, L, tk, lane);""")
rep("""        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * (NS + 2), lds);""", """        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * (NS + 3), lds);""")
rep("""    if ((e = record_foot((const void*)kern, lds, 64 * (NS + 2), grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (NS + 2)), lds, stream, a);""", """    if ((e = record_foot((const void*)kern, lds, 64 * (NS + 3), grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (NS + 3)), lds, stream, a);""")
