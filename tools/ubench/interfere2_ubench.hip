// interfere2_ubench.hip -- which LDS operations of a strip-like wave slow down while other
// waves of its workgroup stream 16-B stores to HBM?  Wave 0: dependent VALU chain, per 4 steps
// LDSOPS bit 1: 4x ds_write_b128 (staging), bit 2: 1x ds_write_b128 (hand-off),
// bit 4: 4x ds_read_b64 + 1x ds_read_b128 (profile + letters, consumed 4 steps later).
// Waves 1..3 store to HBM when their bit of OMASK is set (wave w and w+2 share a SIMD half).
// One workgroup: no power or clock effect (interfere_ubench.hip shows the clock stays).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int int4a __attribute__((ext_vector_type(4)));
typedef int int2a __attribute__((ext_vector_type(2)));

template <int LDSOPS, int OMASK, int SKIND>
__global__ void __launch_bounds__(256) kern(int4a* buf, long long n16, int iters, unsigned long long* res)
{
    __shared__ int stop;
    __shared__ int4a lds[4096];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) stop = 0;
    for (int k = threadIdx.x; k < 4096; k += 256) lds[k] = int4a {k, 1, 2, 3};
    __syncthreads();
    if (w == 0)
    {
        int v = lane, a = lane * 3, b = lane ^ 5;
        int2a p0 = {0, 0};
        int4a l0 = {0, 0, 0, 0};
        unsigned long long c0 = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < iters; ++i)
        {
#pragma unroll
            for (int k = 0; k < 16; ++k)
            {
                asm volatile("v_add_u32 %0, %0, %1\n v_max3_i32 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b));
                if ((k & 3) == 3)
                {
                    if (LDSOPS & 1)
#pragma unroll
                        for (int q = 0; q < 4; ++q) lds[1024 + ((lane * 8 + q + 4 * (k >> 2)) & 2047)] = int4a {v, a, q, k};
                    if (LDSOPS & 2) lds[3072 + ((lane + 64 * (k >> 2)) & 255)] = int4a {v, b, a, k};
                    if (LDSOPS & 4)
                    {
                        a += p0.x + l0.y;  // consume the previous group's reads
                        const int2a* pp = (const int2a*)lds;
                        p0 = pp[(lane + (v & 7) * 64) & 1023];
#pragma unroll
                        for (int q = 1; q < 4; ++q) p0 += pp[(lane + ((v + q) & 7) * 64 + 512) & 1023];
                        l0 = lds[(lane + i) & 511];
                    }
                }
            }
        }
        unsigned long long c1 = __builtin_amdgcn_s_memtime();
        __hip_atomic_store(&stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane == 0)
        {
            res[0] = c1 - c0;
            res[2] = v + a;
        }
    }
    else if (OMASK & (1 << (w - 1)))
    {
        long long idx = (long long)(w - 1) * 64 * 1024 + lane;
        int it = 0;
        while (!__hip_atomic_load(&stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
        {
#pragma unroll
            for (int k = 0; k < 8; ++k)
            {
                long long j = (idx + (long long)(it * 8 + k) * 64 * 3) % n16;
                if (SKIND == 0) buf[j] = int4a {it, k, lane, w};
                if (SKIND == 1) ((int*)buf)[4 * j] = it;
                if (SKIND == 2) ((int*)buf)[(4 * j) & ~255ll | (lane * 4)] = it;  // 64 lanes -> contiguous 256 B
            }
            ++it;
        }
    }
}

int main()
{
    const long long n16 = 1ll << 26;
    int4a* buf;
    hipMalloc(&buf, n16 * 16);
    hipMemset(buf, 0, n16 * 16);
    unsigned long long* res;
    hipMallocManaged(&res, 64);
    auto run = [&](auto k, const char* name) {
        const int iters = 20000;
        hipLaunchKernelGGL(k, 1, 256, 0, 0, buf, n16, iters, res);
        hipLaunchKernelGGL(k, 1, 256, 0, 0, buf, n16, iters, res);
        hipDeviceSynchronize();
        printf("%-52s %.2f cycles/step\n", name, (double)res[0] / (iters * 16));
    };
#define R(L, M, S) run(kern<L, M, S>, "lds " #L " others " #M " kind " #S)
    R(0, 0, 0); R(0, 7, 0);
    R(1, 0, 0); R(1, 7, 0); R(1, 2, 0); R(1, 5, 0); R(1, 7, 1); R(1, 7, 2);
    R(2, 0, 0); R(2, 7, 0);
    R(4, 0, 0); R(4, 7, 0); R(4, 2, 0); R(4, 5, 0);
    R(7, 0, 0); R(7, 7, 0); R(7, 2, 0); R(7, 5, 0); R(7, 1, 0); R(7, 7, 1);
    return 0;
}
