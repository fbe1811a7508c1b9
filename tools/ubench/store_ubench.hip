// store_ubench.hip -- store throughput of the write patterns a full-matrix fill can use.
// One wave per workgroup; each wave issues `iters` global_store_dwordx4 (1 KB each) into a
// row-major int32 matrix with row pitch `ld` (10k x 10k: 10001 ints), walking columns like a
// strip sweep.  Pattern P = lanes per row: 4 -> 16 rows x 64 B per instruction, 16 -> 4 rows x
// 256 B, 64 -> 1 row x 1 KB, 1 -> 64 rows x 16 B.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));

template <int P>
__global__ void kern(int* out, long long ld, int iters, int rows_per_wg)
{
    const int lane = threadIdx.x;
    const int rgroup = lane / P, lq = lane % P;      // row within instruction, 16-B piece in row
    constexpr int RPI = 64 / P;                      // rows per instruction
    const long long row0 = (long long)blockIdx.x * rows_per_wg;
    int4a v = {lane, lane + 1, lane + 2, lane + 3};
    for (int it = 0; it < iters; ++it)
    {
        // instruction it: rows block (it % (rows_per_wg/RPI)), columns advance every full row sweep
        const int rb = it % (rows_per_wg / RPI);
        const int cb = it / (rows_per_wg / RPI);
        const long long r = row0 + (long long)rb * RPI + rgroup;
        const long long c = (long long)cb * (4 * P) + 4 * lq + 1;  // +1: 4-byte aligned, like the fill
        *(int4a*)(out + r * ld + c) = v;
        v += 1;
    }
}

int main()
{
    const long long ld = 10001, rows = 10000;
    int* out;
    hipMalloc(&out, (size_t)ld * rows * 4 + 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto k, int P, int wgs, int iters) {
        const int rows_per_wg = (int)(rows / wgs) / 64 * 64;
        hipLaunchKernelGGL(k, wgs, 64, 0, 0, out, ld, iters, rows_per_wg);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, wgs, 64, 0, 0, out, ld, iters, rows_per_wg);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double bytes = (double)wgs * iters * 1024;
        printf("lanes/row %2d  rows/instr %2d  WGs %3d: %8.3f ms  %8.1f GB/s total  %6.2f B/clk/wave @2.4GHz\n", P, 64 / P,
               wgs, ms, bytes / ms / 1e6, bytes / wgs / (ms * 1e-3 * 2.4e9));
    };
    for (int wgs : {1, 40, 256})
    {
        const int iters = 4096;
        run(kern<1>, 1, wgs, iters);
        run(kern<4>, 4, wgs, iters);
        run(kern<16>, 16, wgs, iters);
        run(kern<64>, 64, wgs, iters);
    }
    return 0;
}
