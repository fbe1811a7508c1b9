// store_ubench2.hip -- chip-wide store bandwidth of the strip-sweep write patterns at batch scale.
// Each wave owns 64 consecutive rows of a row-major int32 matrix (row pitch 20001 ints, as a
// 20k-column pair) and sweeps its columns, issuing global_store_dwordx4 (1 KB per instruction):
// P lanes per row -> 64/P rows x 16P bytes per instruction (P = 4: the lane fill's 16 rows x 64 B;
// P = 8: 8 rows x 128 B).  Rows start 4-byte aligned (+1 column), like the fill.
// Build: hipcc --offload-arch=gfx950 -O3 store_ubench2.hip -o store_ubench2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));

template <int P>
__global__ void kern(int* out, long long ld, int iters)
{
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int rgroup = lane / P, lq = lane % P;
    constexpr int RPI = 64 / P;           // rows per instruction
    constexpr int NG = 64 / RPI;          // instructions per column chunk
    const long long row0 = wave * 64;
    int4a v = {lane, lane + 1, lane + 2, lane + 3};
    for (int it = 0; it < iters; ++it)
    {
        const int rb = it % NG, cb = it / NG;
        const long long r = row0 + (long long)rb * RPI + rgroup;
        const long long c = (long long)cb * (4 * P) + 4 * lq + 1;
        *(int4a*)(out + r * ld + c) = v;
        v += 1;
    }
}

int main()
{
    const long long ld = 20001;
    const int waves_per_wg = 4;
    int* out = nullptr;
    const int max_wgs = 2048;
    const size_t bytes_alloc = (size_t)ld * 64 * waves_per_wg * max_wgs * 4 + 4096;
    if (hipMalloc(&out, bytes_alloc) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](auto k, int P, int wgs, int iters) {
        hipLaunchKernelGGL(k, wgs, 64 * waves_per_wg, 0, 0, out, ld, iters);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, wgs, 64 * waves_per_wg, 0, 0, out, ld, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = (double)wgs * waves_per_wg * iters * 1024;
        printf("lanes/row %2d  rows/instr %2d  waves %5d: %8.3f ms  %8.1f GB/s\n", P, 64 / P, wgs * waves_per_wg, ms,
               bytes / ms / 1e6);
    };
    for (int wgs : {256, 512, 1024, 2048})
    {
        const int iters = 4096;  // 4 MB per wave; columns < 4 * iters / 64 * 64 / ... < ld
        run(kern<4>, 4, wgs, iters);
        run(kern<8>, 8, wgs, iters);
        run(kern<16>, 16, wgs, iters);
        run(kern<64>, 64, wgs, iters);
    }
    return 0;
}
