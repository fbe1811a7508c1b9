// hwid_probe.hip -- SIMD placement of a workgroup's waves (HW_REG_HW_ID bits [5:4] = SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out)
{
    unsigned v = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID, all 32 bits
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = v;
}
int main()
{
    unsigned* d;
    hipMalloc(&d, 64 * 8 * 4);
    for (int waves : {4, 5})
    {
        hipMemset(d, 0, 64 * 8 * 4);
        hipLaunchKernelGGL(k, 6, 64 * waves, 0, 0, d);
        unsigned h[64 * 8];
        hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        for (int b = 0; b < 6; ++b)
        {
            printf("waves %d wg %d:", waves, b);
            for (int w = 0; w < waves; ++w) printf("  w%d simd %u cu %u wave %u", w, (h[b * 8 + w] >> 4) & 3, (h[b * 8 + w] >> 8) & 15, h[b * 8 + w] & 15);
            printf("\n");
        }
    }
    return 0;
}
