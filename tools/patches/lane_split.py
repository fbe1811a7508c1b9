# nw_lane.hip variant: the loader's two jobs in two waves (feeder: granule polls -> ring 0;
# profiler: Q passes), as nw_krow's single-pair geometry.
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a[:80], s.count(a))
    s = s.replace(a, b)
rep("""template <int NS>
__device__ __forceinline__ void lane_loader(const StripArgs& a, const LaneLds& L, int tk, int lane)""",
"""template <int NS, int ROLE>
__device__ __forceinline__ void lane_loader(const StripArgs& a, const LaneLds& L, int tk, int lane)""")
rep("""    while (qn <= C || hnext <= C)
    {
        bool moved = false;""", """    while ((ROLE != 1 && qn <= C) || (ROLE != 2 && hnext <= C))
    {
        bool moved = false;""")
rep("""        if (hnext <= C && hnext + 128 > c0 + kLRing) c0 = flag_ld(F + kFCons);  // ring 0 consumed
        const bool feed = hnext <= C && hnext + 128 <= c0 + kLRing;""", """        if (ROLE != 2 && hnext <= C && hnext + 128 > c0 + kLRing) c0 = flag_ld(F + kFCons);  // ring 0 consumed
        const bool feed = ROLE != 2 && hnext <= C && hnext + 128 <= c0 + kLRing;""")
rep("""        if (qn <= C && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (qn <= C && qn <= pl + kLW - 128)""", """        if (ROLE != 1 && qn <= C && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (ROLE != 1 && qn <= C && qn <= pl + kLW - 128)""")
rep("""            if (tk == 0 || hnext > C) __builtin_amdgcn_s_sleep(1);""", """            if (ROLE == 2 || tk == 0 || hnext > C) __builtin_amdgcn_s_sleep(1);""")
rep("""__global__ void __launch_bounds__(64 * (NS + 2)) nw_lane_kernel(StripArgs a)""", """__global__ void __launch_bounds__(64 * (NS + 3)) nw_lane_kernel(StripArgs a)""")
rep("""    for (int k = threadIdx.x; k < a.substsz * kLSubRow; k += 64 * (NS + 2))""", """    for (int k = threadIdx.x; k < a.substsz * kLSubRow; k += 64 * (NS + 3))""")
rep("""            lane_loader<NS>(pa, L, tk, lane);""", """            lane_loader<NS, 1>(pa, L, tk, lane);
        else if (w == NS + 2)
            lane_loader<NS, 2>(pa, L, tk, lane);""")
rep("""        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * (NS + 2), lds);""", """        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * (NS + 3), lds);""")
rep("""    if ((e = record_foot((const void*)kern, lds, 64 * (NS + 2), grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (NS + 2)), lds, stream, a);""", """    if ((e = record_foot((const void*)kern, lds, 64 * (NS + 3), grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (NS + 3)), lds, stream, a);""")
