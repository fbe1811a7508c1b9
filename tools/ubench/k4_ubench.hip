// k4_ubench.hip -- cycles per wavefront step of the 4-rows-per-lane NW-LG step, one wave.
// Variants isolate the cost of SDWA-extracted int16 S, plain int32 S, the chain alone and the
// per-4-step LDS traffic of the strip kernel.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int int2v __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));
extern __shared__ __attribute__((aligned(16))) char smem[];
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int opq(int v) { asm volatile("" : "+v"(v)); return v; }

template <int V>
__global__ void kern(int n, const int* in, int* out, unsigned long long* cyc)
{
    const int lane = threadIdx.x;
    for (int i = lane; i < 8192; i += 64) ((int*)smem)[i] = (i * 2654435761u) & 0x001f001f;
    __syncthreads();
    int A = 0, B = 0, C = 0, D = 0, dA = 0;
    int2v sv[4];
    int s32[4][4];
    for (int u = 0; u < 4; ++u) { sv[u] = int2v{in[lane + u], in[lane + 4 + u]}; for (int k = 0; k < 4; ++k) s32[u][k] = in[lane + 8 * u + k]; }
    int hv[4] = {in[0], in[1], in[2], in[3]};
    int4v lx = {0, 512, 1024, 1536};
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < n; ++it)
    {
        int2v sn[4];
        int4v lx2;
        if constexpr (V >= 4)
        {
            lx2 = *(int4v*)(smem + 16 * ((it * 4 + lane) & 255));
#pragma unroll
            for (int u = 0; u < 4; ++u) sn[u] = *(int2v*)(smem + 8192 + ((lx[u] + 8 * lane) & 8191));
        }
        int Xd[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            const int up = shr1z(D) + hv[u];
            int na, nb, nc, nd;
            if constexpr (V == 1 || V >= 4)
            {
                na = max(max(dA + (int)(short)sv[u].x, up), A);
                nb = max(max(A + (sv[u].x >> 16), na), B);
                nc = max(max(B + (int)(short)sv[u].y, nb), C);
                nd = max(max(C + (sv[u].y >> 16), nc), D);
            }
            else if constexpr (V == 2)
            {
                na = max(max(dA + s32[u][0], up), A);
                nb = max(max(A + s32[u][1], na), B);
                nc = max(max(B + s32[u][2], nb), C);
                nd = max(max(C + s32[u][3], nc), D);
            }
            else  // V == 3: chain only
            {
                na = max(max(dA, up), A);
                nb = max(max(A, na), B);
                nc = max(max(B, nb), C);
                nd = max(max(C, nc), D);
            }
            dA = up; A = na; B = nb; C = nc; D = nd; Xd[u] = nd;
        }
        if constexpr (V >= 4)
        {
            *(int4v*)(smem + 16384 + 16 * ((it - lane) & 127)) = int4v{Xd[0], Xd[1], Xd[2], Xd[3]};
#pragma unroll
            for (int u = 0; u < 4; ++u) sv[u] = sn[u];
            lx = lx2 & 0x1ff8;
        }
        if constexpr (V != 1 && V != 4 && V != 5) { for (int u = 0; u < 4; ++u) sv[u] = int2v{opq(sv[u].x), opq(sv[u].y)}; }
        if constexpr (V == 5) hv[it & 3] = opq(hv[it & 3]);
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[lane] = A + B + C + D + sv[0].x + s32[0][0] + lx[0];
    if (lane == 0) cyc[0] = t1 - t0;
}

int main()
{
    int *in, *out; unsigned long long* cyc;
    hipMalloc(&in, 4096 * 4); hipMalloc(&out, 4096); hipMalloc(&cyc, 8);
    std::vector<int> h(4096); for (int i = 0; i < 4096; ++i) h[i] = (i * 7) % 23;
    hipMemcpy(in, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    const int n = 20000;
    auto run = [&](auto k, const char* name) {
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
        for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k, 1, 64, 65536, 0, n, in, out, cyc);
        unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-58s %6.1f cycles/step\n", name, (double)c / (4.0 * n));
    };
    run(kern<1>, "V1 dpp + 4x(sdwa add + max3)");
    run(kern<2>, "V2 dpp + 4x(add + max3), int32 S");
    run(kern<3>, "V3 dpp + 4x max3 (chain only)");
    run(kern<4>, "V4 V1 + per-4-step LDS (b128 letters, 4 b64 S, b128 write)");
    return 0;
}
