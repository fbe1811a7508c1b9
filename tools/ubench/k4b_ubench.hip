// k4b_ubench.hip -- per-step cost of each LDS component of the 4-rows-per-lane strip step,
// one wave, 16-step blocks unrolled like nw_strip.hip (loads one group ahead, letters two).
// Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef int int2v __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));
extern __shared__ __attribute__((aligned(16))) char smem[];
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

// M: bit0 S reads (ds_read_b64 per step), bit1 letters (ds_read_b128 per 4 steps),
//    bit2 staging ds_write_b128 per 4 steps, bit3 staging ds_write_addtid_b32 per step,
//    bit4 int8 S (ds_read_b32) instead of int16
template <int M>
__global__ void kern(int n, const int* in, int* out, unsigned long long* cyc)
{
    const int lane = threadIdx.x;
    for (int i = lane; i < 16384; i += 64) ((int*)smem)[i] = (i * 2654435761u) & 0x00070007;
    __syncthreads();
    int A = 0, B = 0, C = 0, D = 0, dA = 0;
    int2v sv[4];
    for (int u = 0; u < 4; ++u) sv[u] = int2v{in[lane + u], in[lane + 4 + u]};
    int hv[16];
    for (int u = 0; u < 16; ++u) hv[u] = in[u];
    int4v lx1 = {0, 512, 1024, 1536};
    const uint32_t laneoff = 8192 + 8 * lane;
    unsigned long long t0 = __builtin_readcyclecounter();
    for (int b = 0; b < n; ++b)
    {
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
            const int t = 16 * b + 4 * q;
            int4v lx2 = lx1;
            if constexpr (M & 2) lx2 = *(int4v*)(smem + 16 * ((t / 4 + lane) & 255)) & 0xfc0;
            int2v sn[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                if constexpr (M & 16) { int v = *(int*)(smem + 8192 + 4 * lane + lx1[u]); sn[u] = int2v{v, v}; }
                else if constexpr (M & 1) sn[u] = *(int2v*)(smem + laneoff + lx1[u]);
                else sn[u] = sv[(u + 1) & 3];
            }
            int Xd[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                const int up = shr1z(D) + hv[4 * q + u];
                const int na = max(max(dA + (int)(short)sv[u].x, up), A);
                const int nb = max(max(A + (sv[u].x >> 16), na), B);
                const int nc = max(max(B + (int)(short)sv[u].y, nb), C);
                const int nd = max(max(C + (sv[u].y >> 16), nc), D);
                dA = up; A = na; B = nb; C = nc; D = nd; Xd[u] = nd;
                if constexpr (M & 8)
                {
                    const int m0 = 4 * ((4096 - t - u) & 1023) + 32768;
                    asm volatile("s_mov_b32 m0, %1\n\tds_write_addtid_b32 %0" ::"v"(nd), "s"(m0) : "memory", "m0");
                }
            }
            if constexpr (M & 4)
                *(int4v*)(smem + 49152 + 16 * ((t / 4 - lane) & 127)) = int4v{Xd[0], Xd[1], Xd[2], Xd[3]};
#pragma unroll
            for (int u = 0; u < 4; ++u) sv[u] = sn[u];
            lx1 = lx2;
        }
    }
    unsigned long long t1 = __builtin_readcyclecounter();
    out[lane] = A + B + C + D + sv[0].x + lx1[0];
    if (lane == 0) cyc[0] = t1 - t0;
}

int main()
{
    int *in, *out; unsigned long long* cyc;
    hipMalloc(&in, 4096 * 4); hipMalloc(&out, 4096); hipMalloc(&cyc, 8);
    std::vector<int> h(4096); for (int i = 0; i < 4096; ++i) h[i] = (i * 7) % 23;
    hipMemcpy(in, h.data(), 4096 * 4, hipMemcpyHostToDevice);
    const int n = 4000;
    auto run = [&](auto k, const char* name) {
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536 + 4096);
        for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k, 1, 64, 65536 + 4096, 0, n, in, out, cyc);
        unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
        printf("%-52s %6.1f cycles/step\n", name, (double)c / (16.0 * n));
    };
    run(kern<0>, "no LDS");
    run(kern<1>, "S b64 per step");
    run(kern<16>, "S b32 (int8) per step");
    run(kern<2>, "letters b128 per 4 steps");
    run(kern<4>, "staging b128 per 4 steps");
    run(kern<8>, "staging addtid_b32 per step");
    run(kern<3>, "S b64 + letters");
    run(kern<7>, "S b64 + letters + staging b128 (= kernel)");
    run(kern<11>, "S b64 + letters + staging addtid");
    run(kern<26>, "S b32 + letters + staging addtid");
    return 0;
}
