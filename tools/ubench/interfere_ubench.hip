// interfere_ubench.hip -- does another wave's HBM store stream slow a wave that touches no memory?
// Wave 0 runs a dependent VALU chain (+ optional LDS traffic), timed with s_memtime (core clock)
// and s_memrealtime (100 MHz); waves 1..3 of the same workgroup meanwhile: 0 idle, 1 stream
// 16-B stores to HBM, 2 store into a 16 KB window, 3 stream 16-B loads from HBM.
// cycles/realtime gives the core clock during the run: a clock drop vs a pipeline interaction.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int int4a __attribute__((ext_vector_type(4)));

template <int OTHERS, int LDSOPS>
__global__ void __launch_bounds__(256) kern(int4a* buf, long long n16, int iters, unsigned long long* res)
{
    __shared__ int stop;
    __shared__ int4a lds[1024];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (threadIdx.x == 0) stop = 0;
    __syncthreads();
    if (w == 0)
    {
        int v = lane, a = lane * 3, b = lane ^ 5;
        unsigned long long c0 = __builtin_amdgcn_s_memtime();
        unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < iters; ++i)
        {
#pragma unroll
            for (int k = 0; k < 16; ++k)
            {
                asm volatile("v_add_u32 %0, %0, %1\n v_max3_i32 %0, %0, %1, %2" : "+v"(v) : "v"(a), "v"(b));
                if (LDSOPS && (k & 3) == 0)
                {
                    lds[(lane + 64 * k) & 1023] = int4a {v, a, b, k};
                    a += lds[(lane * 5 + k) & 1023].y & 1;
                }
            }
        }
        unsigned long long c1 = __builtin_amdgcn_s_memtime();
        unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        __hip_atomic_store(&stop, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (lane == 0 && blockIdx.x == 0)
        {
            res[0] = c1 - c0;
            res[1] = r1 - r0;
            res[2] = v;
        }
    }
    else if (OTHERS != 0)
    {
        long long idx = ((long long)blockIdx.x * 3 + (w - 1)) * 64 * 1024 + lane;
        int4a acc = {0, 0, 0, 0};
        int it = 0;
        while (!__hip_atomic_load(&stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
        {
#pragma unroll
            for (int k = 0; k < 8; ++k)
            {
                long long j = (idx + (long long)(it * 8 + k) * 64) % n16;
                if (OTHERS == 1) buf[j] = int4a {it, k, lane, w};
                if (OTHERS == 2) buf[(lane + 64 * k) & 1023] = int4a {it, k, lane, w};
                if (OTHERS == 3) acc += buf[j];
            }
            ++it;
        }
        if (OTHERS == 3 && acc.x == 0x7fffffff) buf[0] = acc;
    }
}

int main()
{
    const long long n16 = 1ll << 26;  // 1 GiB
    int4a* buf;
    hipMalloc(&buf, n16 * 16);
    hipMemset(buf, 0, n16 * 16);
    unsigned long long* res;
    hipMallocManaged(&res, 64);
    const char* names[] = {"idle", "HBM stores", "16KB-window stores", "HBM loads"};
    auto run = [&](auto k, int others, int ldsops, int wgs) {
        const int iters = 20000;
        hipLaunchKernelGGL(k, wgs, 256, 0, 0, buf, n16, iters, res);
        hipLaunchKernelGGL(k, wgs, 256, 0, 0, buf, n16, iters, res);
        hipDeviceSynchronize();
        double cyc = (double)res[0] / (iters * 16), us = res[1] / 100.0;
        printf("WGs %3d lds %d others %-18s: %.2f memtime-ticks/step, %.1f us, clock %.0f MHz (memtime/realtime)\n", wgs,
               ldsops, names[others], cyc, us, res[0] / us);
    };
    for (int wgs : {1, 256})
    {
        run(kern<0, 0>, 0, 0, wgs);
        run(kern<1, 0>, 1, 0, wgs);
        run(kern<2, 0>, 2, 0, wgs);
        run(kern<3, 0>, 3, 0, wgs);
        run(kern<0, 1>, 0, 1, wgs);
        run(kern<1, 1>, 1, 1, wgs);
        run(kern<2, 1>, 2, 1, wgs);
    }
    return 0;
}
