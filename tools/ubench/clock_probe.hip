// clock_probe.hip -- shader clock held under load: G workgroups of 4 waves (one per SIMD) each run
// the same VALU-bound loop (max3/add chains, like the fill's step); every wave records its
// s_memtime (shader clock) and s_memrealtime (100 MHz) deltas, so cycles / (realtime / 100 MHz)
// is the clock it ran at.  Also reports the loop's cycles per iteration.  Diagnostics only.
// Build: hipcc --offload-arch=gfx950 -O3 clock_probe.hip -o clock_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

__global__ void __launch_bounds__(256) spin(int iters, int seed, unsigned long long* out, int* sink)
{
    int h0 = threadIdx.x + seed, h1 = h0 * 3, h2 = h0 * 5, h3 = h0 * 7, d = 0;
    const int q = seed & 7;
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i)
    {
#pragma unroll
        for (int u = 0; u < 16; ++u)
        {
            const int up = __builtin_amdgcn_update_dpp(0, h3, 0x138, 0xF, 0xF, true) + q;
            const int n0 = max(max(d + q, up), h0);
            const int n1 = max(max(h0 + q + u, n0), h1);
            const int n2 = max(max(h1 + q - u, n1), h2);
            const int n3 = max(max(h2 + q ^ u, n2), h3);
            d = up;
            h0 = n0; h1 = n1; h2 = n2; h3 = n3;
        }
    }
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0)
    {
        const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        out[2 * wv] = c1 - c0;
        out[2 * wv + 1] = r1 - r0;
    }
    if (h0 + h1 + h2 + h3 == 0x7fffffff) sink[0] = 1;
}

int main()
{
    const int iters = 20000;
    unsigned long long* d_out;
    int* d_sink;
    hipMalloc(&d_out, 2 * 4 * 1024 * sizeof(unsigned long long));
    hipMalloc(&d_sink, 4);
    for (int G : {1, 8, 32, 64, 98, 128, 196, 256})
    {
        for (int rep = 0; rep < 2; ++rep)
        {
            hipLaunchKernelGGL(spin, dim3(G), dim3(256), 0, 0, iters, rep, d_out, d_sink);
            hipDeviceSynchronize();
        }
        std::vector<unsigned long long> h(2 * 4 * G);
        hipMemcpy(h.data(), d_out, h.size() * 8, hipMemcpyDeviceToHost);
        double mhz = 0, cyc = 0;
        for (int w = 0; w < 4 * G; ++w)
        {
            mhz += (double)h[2 * w] / ((double)h[2 * w + 1] / 100.0);
            cyc += (double)h[2 * w];
        }
        mhz /= 4 * G;
        cyc /= 4 * G;
        printf("G %4d  clock %7.1f MHz  cycles/step %6.2f  (%.3f ms)\n", G, mhz, cyc / (iters * 16.0),
               cyc / mhz / 1000.0);
    }
    return 0;
}
