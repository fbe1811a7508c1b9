// Micro-benchmark of the strip kernel's wavefront step on gfx950: which component costs what.
// V0: DPP/max3 chain only; V1: + staging ds_write; V2: + letter ds_read (imm offset);
// V3: + dependent profile ds_read (the full step).  Cycles from s_memtime, per step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

extern __shared__ __attribute__((aligned(16))) char smem[];
__device__ __forceinline__ int lds_ld(unsigned a) { return *(const int*)(smem + a); }
__device__ __forceinline__ void lds_st(unsigned a, int v) { *(int*)(smem + a) = v; }
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

template <int V, int BLK>
__global__ void k(int nblk, unsigned long long* out, int* sink)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned base = w * 32768;
    for (int i = lane; i < 8192; i += 64) lds_st(base + 4 * i, (i * 7) & 255);
    __syncthreads();
    int c0 = lane, c1 = 0;
    int s[BLK];
#pragma unroll
    for (int u = 0; u < BLK; ++u) s[u] = (lane * 13 + u) & 15;
    const unsigned laneoff = base + 4 * lane;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int b = 0; b < nblk; ++b)
    {
        const unsigned xo_base = base + 4 * ((b * BLK) & 1023);
        const unsigned st_base = base + 16384 + 260 * ((b * BLK) & 31) + 4 * lane;
        int xn[BLK], sn[BLK];
#pragma unroll
        for (int u = 0; u < BLK + 4; ++u)
        {
            if (V >= 2 && u < BLK) xn[u] = lds_ld(xo_base + 4 * u);
            if (V >= 3 && u >= 4) sn[u - 4] = lds_ld(((unsigned)xn[u - 4] & 1020) + laneoff);
            if (u < BLK)
            {
                int d = shr1z(c1) + s[u];
                int e = max(d, c0);
                int cn = max(shr1z(c0), e);
                if (V >= 1) lds_st(st_base + 260 * u, cn);
                c1 = c0;
                c0 = cn;
            }
        }
        if (V >= 3)
        {
#pragma unroll
            for (int u = 0; u < BLK; ++u) s[u] = sn[u] & 31;
        }
        else if (V >= 2)
        {
#pragma unroll
            for (int u = 0; u < BLK; ++u) s[u] ^= xn[u] & 1;
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[blockIdx.x * 16 + w] = t1 - t0;
    sink[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1;
}

template <int V>
void run(int waves, int nblk)
{
    unsigned long long* d;
    int* sink;
    hipMalloc(&d, 16 * 8 * sizeof(unsigned long long));
    hipMalloc(&sink, 8 * 1024 * 4);
    hipFuncSetAttribute((const void*)k<V, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 32768 * waves);
    hipLaunchKernelGGL((k<V, 16>), dim3(1), dim3(64 * waves), 32768 * waves, 0, nblk, d, sink);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(16 * 8);
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    double cyc = 0;
    for (int w = 0; w < waves; ++w) cyc += h[w];
    cyc /= waves;
    printf("V%d waves=%d: %.1f cycles/step\n", V, waves, cyc / (nblk * 16.0));
    hipFree(d);
    hipFree(sink);
}

int main()
{
    for (int waves : {1, 4, 5, 8})
    {
        run<0>(waves, 2000);
        run<1>(waves, 2000);
        run<2>(waves, 2000);
        run<3>(waves, 2000);
    }
    return 0;
}
