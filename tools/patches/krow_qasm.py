# K-rows variant: the next block's profile reads as asm volatile ds_read2_b32 at steps 0-7 (two per
# step, k = u/2), each anchored after its step's last row by a register input (DEP), so the compiler
# cannot cluster them in front of the step-14 progress read; VALU still schedules freely around
# them.  Their results are used only in the next block, after the halo asm's lgkmcnt(0).
import os
DEP = os.environ.get("QASM_DEP", "1") == "1"
def rep(a, b, n=1):
    global s
    assert s.count(a) == n, (a, s.count(a))
    s = s.replace(a, b)
rep("""// int16 half of a profile dword""", """template <int P>
__device__ __forceinline__ int2v q_rd2(uint32_t a, int dep)
{
    int2v r;
    asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(r) : "v"(a), "n"(2 * P), "n"(2 * P + 1), "v"(dep));
    return r;
}
// int16 half of a profile dword""")
rep("""            if (u < 8)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);""", """            if (u < 2 * K)
            {
                const int kk = u >> 1;
                const int dep = %s;
                const int2v r0 = (u & 1) ? q_rd2<2>(qrow[kk] + pn, dep) : q_rd2<0>(qrow[kk] + pn, dep);
                const int2v r1 = (u & 1) ? q_rd2<3>(qrow[kk] + pn, dep) : q_rd2<1>(qrow[kk] + pn, dep);
                qn[kk][4 * (u & 1) + 0] = r0.x;
                qn[kk][4 * (u & 1) + 1] = r0.y;
                qn[kk][4 * (u & 1) + 2] = r1.x;
                qn[kk][4 * (u & 1) + 3] = r1.y;
            }""" % ("nh[K - 1]" if DEP else "0"))
