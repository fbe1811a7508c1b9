// C-wave variants (one wave, no barrier unless noted), cycles per step:
//  A chain only | B + S reads at block start | C + S reads prefetched one block ahead
//  D = B + lane-60 hand-off per group | E = C + hand-off per group | F = C + hand-off once per block (4 writes at end)
//  G = E with BLK 32 | H = E + barrier per block (4 waves) | I = G + barrier per block (4 waves)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
extern __shared__ __attribute__((aligned(16))) char smem[];
typedef int int4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int4v lds_ld4(unsigned a) { return *(const int4v*)(smem + a); }
__device__ __forceinline__ void lds_st4(unsigned a, int4v v) { *(int4v*)(smem + a) = v; }
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int V, int BLK, bool BAR>
__global__ void k(int nblk, unsigned long long* out, int* sink)
{
    constexpr int NG = BLK / 4;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) *(int*)(smem + 4 * i) = (i * 7) & 15;
    __syncthreads();
    const unsigned tab = wid * 16384;
    int c0 = lane, c1 = 0;
    int4v S[NG], Sn[NG];
    for (int q = 0; q < NG; ++q) S[q] = int4v {1, 2, 3, 4};
    const bool pre = (V == 2 || V == 4 || V == 5);
    if (pre)
        for (int q = 0; q < NG; ++q) S[q] = lds_ld4(tab + ((q) * 64 + lane) * 16);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int hb[BLK];
    for (int b = 0; b < nblk; ++b)
    {
        if (V == 1 || V == 3)
        {
#pragma unroll
            for (int q = 0; q < NG; ++q) S[q] = lds_ld4(tab + (((b & 1) * NG + q) * 64 + lane) * 16);
        }
#pragma unroll
        for (int q = 0; q < NG; ++q)
        {
            if (pre) Sn[q] = lds_ld4(tab + ((((b + 1) & 1) * NG + q) * 64 + lane) * 16);
            int h[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                int d = shr1z(c1) + (S[q][u] & 15);
                int e = max(d, c0);
                int cn = max(shr1z(c0), e);
                h[u] = cn;
                hb[4 * q + u] = cn;
                c1 = c0;
                c0 = cn;
            }
            if (V == 3 || V == 4)
            {
                const unsigned addr = tab + 8192 + (((b * NG + q) & 15) << 4);
                if (lane == 60) lds_st4(addr, int4v {h[0], h[1], h[2], h[3]});
            }
        }
        if (V == 5)
        {
            if (lane == 60)
#pragma unroll
                for (int q = 0; q < NG; ++q)
                    lds_st4(tab + 8192 + (((b * NG + q) & 15) << 4), int4v {hb[4 * q], hb[4 * q + 1], hb[4 * q + 2], hb[4 * q + 3]});
        }
        if (pre)
#pragma unroll
            for (int q = 0; q < NG; ++q) S[q] = Sn[q];
        if (BAR) bar();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[wid] = t1 - t0;
    sink[threadIdx.x + blockDim.x * 0] = c0 + c1;
}

template <int V, int BLK, bool BAR>
void run(const char* name, int waves)
{
    const int nblk = 64000 / BLK;
    unsigned long long* d;
    int* sink;
    (void)hipMalloc(&d, 64 * 8);
    (void)hipMalloc(&sink, 4096 * 4);
    (void)hipFuncSetAttribute((const void*)k<V, BLK, BAR>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipLaunchKernelGGL((k<V, BLK, BAR>), dim3(1), dim3(64 * waves), 65536, 0, nblk, d, sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(64);
    (void)hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost);
    double c = 0;
    for (int w = 0; w < waves; ++w) c += h[w];
    printf("%-44s %.1f cycles/step\n", name, c / waves / (nblk * BLK));
    (void)hipFree(d);
    (void)hipFree(sink);
}

int main()
{
    run<0, 16, false>("A chain only", 1);
    run<1, 16, false>("B + S reads at block start", 1);
    run<2, 16, false>("C + S reads prefetched", 1);
    run<3, 16, false>("D = B + hand-off per group", 1);
    run<4, 16, false>("E = C + hand-off per group", 1);
    run<5, 16, false>("F = C + hand-off at block end", 1);
    run<4, 32, false>("G = E, BLK 32", 1);
    run<4, 16, true>("H = E + barrier/block, 4 waves", 4);
    run<4, 32, true>("I = G + barrier/block, 4 waves", 4);
    run<4, 16, false>("E, 4 waves", 4);
    return 0;
}
