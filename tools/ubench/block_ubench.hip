// Micro-benchmark of the v2 block structure on gfx950: C waves (16-step DPP/max3 chain, four
// 16-byte S-table reads per block, one lane-60 16-byte hand-off write) with optional H-style
// helper waves (2 x 16-byte letter reads, 16 dependent profile reads, 4 x 16-byte writes)
// and an optional s_barrier per block.  Reports cycles per block for C and H waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

extern __shared__ __attribute__((aligned(16))) char smem[];
typedef int int4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int lds_ld(unsigned a) { return *(const int*)(smem + a); }
__device__ __forceinline__ int4v lds_ld4(unsigned a) { return *(const int4v*)(smem + a); }
__device__ __forceinline__ void lds_st4(unsigned a, int4v v) { *(int4v*)(smem + a) = v; }
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int NC, int NH, int NIDLE, bool BAR, bool EMPTY>
__global__ void k(int nblk, unsigned long long* out, int* sink)
{
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 16384; i += blockDim.x) *(int*)(smem + 4 * i) = (i * 7) & 255;
    __syncthreads();
    const bool isC = wid < NC, isH = !isC && wid < NC + NH;
    if (isC) __builtin_amdgcn_s_setprio(3);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    int c0 = lane, c1 = 0, acc = 0;
    const unsigned tab = (isC ? wid : wid - NC) * 16384;
    for (int b = 0; b < nblk; ++b)
    {
        if (!EMPTY)
        {
            if (isC)
            {
                int4v S[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) S[q] = lds_ld4(tab + (((b & 3) * 4 + q) * 64 + lane) * 16);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                {
                    int h[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                    {
                        int d = shr1z(c1) + (S[q][u] & 31);
                        int e = max(d, c0);
                        int cn = max(shr1z(c0), e);
                        h[u] = cn;
                        c1 = c0;
                        c0 = cn;
                    }
                    const unsigned addr = tab + (((b + 1) & 15) << 10);
                    if (lane == 60) lds_st4(addr, int4v {h[0], h[1], h[2], h[3]});
                }
            }
            else if (isH)
            {
                const int4v xlo = lds_ld4(tab + 32768 + 32 * lane), xhi = lds_ld4(tab + 32768 + 32 * lane + 16);
                int sv[16];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                {
                    const int word = (u < 8) ? xlo[u >> 1] : xhi[(u - 8) >> 1];
                    const unsigned off = (u & 1) ? ((unsigned)word >> 16) & 0x1f00 : ((unsigned)word & 0x1f00);
                    sv[u] = lds_ld(49152 + off + 4 * lane);
                }
                if (lane >= 1)
                {
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        lds_st4(tab + ((((b + 1) & 3) * 4 + q) * 64 + lane) * 16,
                                int4v {sv[4 * q], sv[4 * q + 1], sv[4 * q + 2], sv[4 * q + 3]} & 31);
                }
                acc += sv[3];
            }
        }
        if (BAR) bar();
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[wid] = t1 - t0;
    sink[threadIdx.x] = c0 + c1 + acc;
}

template <int NC, int NH, int NIDLE, bool BAR, bool EMPTY>
void run(const char* name, int nblk)
{
    constexpr int W = NC + NH + NIDLE;
    unsigned long long* d;
    int* sink;
    (void)hipMalloc(&d, 64 * 8);
    (void)hipMalloc(&sink, 4096 * 4);
    (void)hipFuncSetAttribute((const void*)k<NC, NH, NIDLE, BAR, EMPTY>, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
    hipLaunchKernelGGL((k<NC, NH, NIDLE, BAR, EMPTY>), dim3(1), dim3(64 * W), 65536, 0, nblk, d, sink);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(64);
    (void)hipMemcpy(h.data(), d, 64 * 8, hipMemcpyDeviceToHost);
    double c = 0, hh = 0;
    for (int w = 0; w < NC; ++w) c += h[w];
    for (int w = NC; w < NC + NH; ++w) hh += h[w];
    printf("%-34s C %.0f cyc/block (%.1f /step)   H %.0f cyc/block\n", name, c / NC / nblk, c / NC / nblk / 16,
           NH ? hh / NH / nblk : 0.0);
    (void)hipFree(d);
    (void)hipFree(sink);
}

int main()
{
    const int n = 4000;
    run<1, 0, 0, false, false>("1 C, no barrier", n);
    run<4, 0, 0, false, false>("4 C, no barrier", n);
    run<4, 0, 0, true, false>("4 C, barrier/block", n);
    run<1, 1, 0, false, false>("1 C + 1 H, no barrier", n);
    run<4, 4, 0, false, false>("4 C + 4 H, no barrier", n);
    run<4, 4, 0, true, false>("4 C + 4 H, barrier/block", n);
    run<4, 4, 1, true, false>("4 C + 4 H + 1 idle, barrier/block", n);
    run<0, 4, 0, false, false>("4 H alone, no barrier", n);
    run<4, 0, 1, true, true>("5 waves, empty barrier loop", n);
    run<4, 4, 1, true, true>("9 waves, empty barrier loop", n);
    return 0;
}
