// Ping-pong latency between two workgroups through global memory, same XCD (L2) vs across XCDs, with
// and without a background store stream (the full fill's expansion).  Each workgroup records its
// XCC id (hwreg XCC_ID); the pair is picked among blocks by their ids.  Modes: 0 = agent-scope
// relaxed atomics (sc1), 1 = workgroup-scope (sc0), 2 = L1 invalidate (buffer_inv sc0) + plain load,
// workgroup-scope stores.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/xcc_pingpong.hip -o /tmp/xcc_pp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__device__ unsigned xcc_id() { return __builtin_amdgcn_s_getreg(20 | (3 << 11)); }

template <int MODE>
__device__ unsigned long long ld(unsigned long long* p)
{
    if (MODE == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (MODE == 1) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // 2: the CU's L1 invalidated, then a plain load (served by the XCD's L2)
    asm volatile("buffer_inv sc0" ::: "memory");
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
template <int MODE>
__device__ void st(unsigned long long* p, unsigned long long v)
{
    if (MODE == 0)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ids: per block its xcc id (written first); ctl[0] = start flag set by block a; ctl[1] = stop
template <int MODE>
__global__ void pp(unsigned* ids, unsigned long long* flags, int a, int b, int rounds, unsigned long long* out,
                   int4* bg, size_t bgN, unsigned* stop, int ring)
{
    extern __shared__ int sm[];
    if (threadIdx.x == 0) ids[blockIdx.x] = xcc_id();
    sm[threadIdx.x] = 0;
    if ((int)blockIdx.x == a || (int)blockIdx.x == b)
    {
        if (threadIdx.x != 0) return;
        unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (int i = 1; i <= rounds; ++i)
        {
            // round i's words: line (i mod ring) of a's and b's halves (ring 1: the same lines)
            unsigned long long* fa = flags + 16 * (size_t)(i % ring);
            unsigned long long* fb = flags + (1u << 20) + 16 * (size_t)(i % ring);
            if ((int)blockIdx.x == a)
            {
                st<MODE>(fa, (unsigned long long)i);
                unsigned long long s = __builtin_amdgcn_s_memrealtime();
                while (ld<MODE>(fb) != (unsigned long long)i)
                    if (__builtin_amdgcn_s_memrealtime() - s > 100000000ull) { out[2] = i; goto done; }
            }
            else
            {
                unsigned long long s = __builtin_amdgcn_s_memrealtime();
                while (ld<MODE>(fa) != (unsigned long long)i)
                    if (__builtin_amdgcn_s_memrealtime() - s > 100000000ull) { out[3] = i; goto done; }
                st<MODE>(fb, (unsigned long long)i);
            }
        }
    done:
        if ((int)blockIdx.x == a)
        {
            out[0] = __builtin_amdgcn_s_memrealtime() - t0;
            __hip_atomic_store(stop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (!bg) return;
    // background: stream stores until block a is done
    const size_t per = bgN / gridDim.x;
    int4* base = bg + per * blockIdx.x;
    for (int it = 0; it < 100000; ++it)
    {
        for (size_t k = threadIdx.x; k < per; k += blockDim.x) base[k] = int4 {it, (int)k, 1, 2};
        if (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    }
}

int main(int argc, char** argv)
{
    const int grid = 256, threads = 512;
    unsigned *ids, *stop;
    unsigned long long *flags, *out;
    int4* bg;
    const size_t bgN = (size_t)4 << 30 >> 4;  // 4 GB
    hipMalloc(&ids, grid * 4);
    hipMalloc(&flags, 16 << 20);
    hipMalloc(&out, 64);
    hipMalloc(&stop, 4);
    hipMalloc(&bg, bgN * 16);
    const size_t lds = 100 * 1024;  // one block per CU
    hipFuncSetAttribute((const void*)pp<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipFuncSetAttribute((const void*)pp<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipFuncSetAttribute((const void*)pp<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    // discover the xcc ids of blocks
    std::vector<unsigned> h(grid);
    hipMemset(flags, 0, 16 << 20);
    hipMemset(stop, 0, 4);
    hipLaunchKernelGGL(pp<0>, dim3(grid), dim3(threads), lds, 0, ids, flags, -1, -1, 0, out, (int4*)nullptr, 0, stop, 1);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), ids, grid * 4, hipMemcpyDeviceToHost);
    printf("xcc of blocks 0..15:");
    for (int i = 0; i < 16; ++i) printf(" %u", h[i]);
    printf("\n");
    int same = -1, cross = -1;
    for (int i = 1; i < grid; ++i)
    {
        if (same < 0 && h[i] == h[0]) same = i;
        if (cross < 0 && h[i] != h[0]) cross = i;
    }
    const int rounds = 2000;
    for (int load = 0; load < 2; ++load)
        for (int ring : {1, 64, 65536})
        for (int cfg = 0; cfg < 4; ++cfg)
        {
            if (cfg == 1 || cfg == 3) continue;  // (sc0 / L1-invalidate polls never see the store: measured)
            const int mode = cfg == 1 ? 1 : cfg == 3 ? 2 : 0;
            const int b = cfg == 2 ? cross : same;
            hipMemset(flags, 0, 16 << 20);
            hipMemset(stop, 0, 4);
            hipMemset(out, 0, 64);
            auto kern = mode == 2 ? pp<2> : mode ? pp<1> : pp<0>;
            hipLaunchKernelGGL(kern, dim3(grid), dim3(threads), lds, 0, ids, flags, 0, b, rounds, out,
                               load ? bg : (int4*)nullptr, bgN, stop, ring);
            hipDeviceSynchronize();
            unsigned long long o[4];
            hipMemcpy(o, out, 32, hipMemcpyDeviceToHost);
            hipMemcpy(h.data(), ids, grid * 4, hipMemcpyDeviceToHost);
            printf("ring %6d lines  load %d  %-22s pair (0:xcc%u, %d:xcc%u)  round trip %.3f us  (timeouts a %llu b %llu)\n", ring, load,
                   mode == 2 ? "L1 inv + plain load" : mode ? "sc0 (workgroup scope)" : "sc1 (agent scope)", h[0], b, h[b], o[0] / 100.0 / rounds, o[2], o[3]);
        }
    return 0;
}
