// LDS allocation granule probe: workgroups per CU the runtime reports for a kernel of 64 threads
// at dynamic LDS sizes around 80 KiB (two per CU fit iff 2 x the rounded size <= the CU's LDS).
#include <hip/hip_runtime.h>
#include <cstdio>

extern __shared__ int dsm[];
__global__ void k(int* o)
{
    dsm[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (o) o[threadIdx.x] = dsm[63 - threadIdx.x];
}

int main()
{
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    int lmax = 0;
    hipDeviceGetAttribute(&lmax, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, 0);
    std::printf("max LDS per CU %d\n", lmax);
    const int sizes[] = {53248, 54614, 54615, 55000, 81408, 81664, 81736, 81920, 81921, 82000, 82432};
    for (int s : sizes)
    {
        int n = 0;
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)k, 64, s);
        std::printf("lds %6d B: %d workgroups per CU (%s)\n", s, n, hipGetErrorString(e));
    }
    return 0;
}
