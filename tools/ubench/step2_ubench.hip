// step2_ubench.hip -- cycles per wavefront step of K-rows NW-LG step variants, one wave (or two
// waves on one SIMD), everything in registers.  Isolates: SDWA int16 operands vs int32 vs
// v_mad_i32_i16 op_sel, the column skew (SK 1: one chain of K+1; SK 2: two chains), K = 2 / 4.
// Build: hipcc --offload-arch=gfx950 -O3 step2_ubench.hip -o step2_ubench
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int opq(int v)
{
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
// a + sext(q.hi) / sext(q.lo) through v_mad_i32_i16 with op_sel (no SDWA)
__device__ __forceinline__ int madlo(int q, int a)
{
    int r;
    asm("v_mad_i32_i16 %0, %1, 1, %2" : "=v"(r) : "v"(q), "v"(a));
    return r;
}
__device__ __forceinline__ int madhi(int q, int a)
{
    int r;
    asm("v_mad_i32_i16 %0, %1, 1, %2 op_sel:[1,0,0,0]" : "=v"(r) : "v"(q), "v"(a));
    return r;
}

// Q: 0 int32 q, 1 SDWA int16 halves, 2 v_mad_i32_i16 op_sel, 3 no q (chain only)
template <int K, int SK, int Q>
__global__ void kern(int n, const int* in, int* out, unsigned long long* cyc)
{
    const int lane = threadIdx.x & 63;
    int H[K], D = 0, DA = 0;
    for (int k = 0; k < K; ++k) H[k] = in[lane + k];
    int q32[K][16], q16[K][8];
    for (int k = 0; k < K; ++k)
    {
        for (int u = 0; u < 16; ++u) q32[k][u] = in[64 + lane + 16 * k + u] & 31;
        for (int j = 0; j < 8; ++j) q16[k][j] = in[256 + lane + 8 * k + j] & 0x001f001f;
    }
    constexpr int KA = SK == 2 ? K / 2 : K;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < n; ++it)
    {
#pragma unroll
        for (int u = 0; u < 16; ++u)
        {
            auto qv = [&](int k) -> int {
                if constexpr (Q == 0) return q32[k][u];
                else if constexpr (Q == 1) return (u & 1) ? (q16[k][u >> 1] >> 16) : (int)(short)q16[k][u >> 1];
                else return 0;
            };
            auto addq = [&](int k, int a) -> int {
                if constexpr (Q == 2) return (u & 1) ? madhi(q16[k][u >> 1], a) : madlo(q16[k][u >> 1], a);
                else if constexpr (Q == 3) return a;
                else return a + qv(k);
            };
            int nh[K];
            const int up = shr1z(H[K - 1]);
            nh[0] = max3i(addq(0, D), up, H[0]);
#pragma unroll
            for (int k = 1; k < K; ++k)
            {
                if (k == KA)
                    nh[k] = max3i(addq(k, DA), H[k - 1], H[k]);
                else
                    nh[k] = max3i(addq(k, H[k - 1]), nh[k - 1], H[k]);
            }
            D = up;
            if constexpr (SK == 2) DA = H[KA - 1];
#pragma unroll
            for (int k = 0; k < K; ++k) H[k] = nh[k];
        }
        // keep q live and unknown across iterations
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
#pragma unroll
            for (int u = 0; u < 16; ++u) q32[k][u] = opq(q32[k][u]);
#pragma unroll
            for (int j = 0; j < 8; ++j) q16[k][j] = opq(q16[k][j]);
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    int s = D + DA;
    for (int k = 0; k < K; ++k) s += H[k];
    out[threadIdx.x] = s;
    if (lane == 0) cyc[threadIdx.x >> 6] = t1 - t0;
}

template <int K, int SK, int Q>
void run(const char* name, int waves, int* in, int* out, unsigned long long* cyc)
{
    const int n = 4000;
    hipLaunchKernelGGL((kern<K, SK, Q>), dim3(1), dim3(64 * waves), 0, 0, 100, in, out, cyc);
    hipLaunchKernelGGL((kern<K, SK, Q>), dim3(1), dim3(64 * waves), 0, 0, n, in, out, cyc);
    unsigned long long h[8];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-44s waves %d: %6.1f cyc/step  (%5.1f cyc/cell-row)\n", name, waves, (double)h[0] / (16.0 * n),
           (double)h[0] / (16.0 * n * K));
}

int main()
{
    int *in, *out;
    unsigned long long* cyc;
    hipMalloc(&in, 4096 * 4);
    hipMalloc(&out, 4096 * 4);
    hipMalloc(&cyc, 64);
    hipMemset(in, 1, 4096 * 4);
    // 4 waves in a 256-thread block land on the 4 SIMDs: one wave per SIMD; 8 waves: two per SIMD
    for (int w : {1, 8})
    {
        run<4, 1, 3>("K4 SK1 chain only", w, in, out, cyc);
        run<4, 1, 0>("K4 SK1 int32 q (v_add)", w, in, out, cyc);
        run<4, 1, 1>("K4 SK1 int16 q (SDWA add)", w, in, out, cyc);
        run<4, 1, 2>("K4 SK1 int16 q (v_mad_i32_i16 op_sel)", w, in, out, cyc);
        run<4, 2, 3>("K4 SK2 chain only", w, in, out, cyc);
        run<4, 2, 0>("K4 SK2 int32 q (v_add)", w, in, out, cyc);
        run<4, 2, 1>("K4 SK2 int16 q (SDWA add)", w, in, out, cyc);
        run<4, 2, 2>("K4 SK2 int16 q (v_mad_i32_i16 op_sel)", w, in, out, cyc);
        run<2, 2, 0>("K2 SK2 int32 q (v_add)", w, in, out, cyc);
        run<2, 2, 1>("K2 SK2 int16 q (SDWA add)", w, in, out, cyc);
        run<8, 2, 0>("K8 SK2 int32 q (v_add)", w, in, out, cyc);
        run<8, 2, 1>("K8 SK2 int16 q (SDWA add)", w, in, out, cyc);
    }
    return 0;
}
