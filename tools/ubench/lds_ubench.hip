// lds_ubench.hip -- what the K-rows strip's per-block LDS traffic costs one wave: the 16-step
// register step (K = 4, SDWA int16 profile) plus, per 16-step block, combinations of
//   P  profile reads for the next block (16 ds_read2_b32, consumed a block later)
//   W  hand-off: 4 ds_write_b128 by every lane (lanes 0..62 into a sink) | by lane 63 only (asm, exec)
//   R  halo: 4 ds_read_b128 by every lane (lanes >= 1 from a zero row) consumed at step 0 (JIT) |
//      read a block ahead
//   F  progress words: 2 ds_write_b32 + 3 ds_read_b32 (mid-block) + readfirstlane at block start
// One wave per SIMD (4 waves), wave 0's s_memtime cycles per 16-step block.
// Build: hipcc --offload-arch=gfx950 -O3 lds_ubench.hip -o lds_ubench
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef int int4v __attribute__((ext_vector_type(4)));
extern __shared__ __attribute__((aligned(16))) char sm[];
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
__device__ __forceinline__ int qlo(int v) { return (int)(short)v; }
__device__ __forceinline__ int qhi(int v) { return v >> 16; }
__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(sm + a); }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(sm + a); }
__device__ __forceinline__ void lds_st4(uint32_t a, int4v v) { *(int4v*)(sm + a) = v; }
__device__ __forceinline__ int raw_ld(uint32_t a)
{
    return __hip_atomic_load((int*)__builtin_assume_aligned(sm + a, 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void flag_st(uint32_t a, int v)
{
    asm volatile("" ::: "memory");
    __hip_atomic_store((int*)__builtin_assume_aligned(sm + a, 4), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// 4 x ds_write_b128 from lane 63 only (exec saved / restored inside one asm block)
__device__ __forceinline__ void st4_lane63(uint32_t a, int4v d0, int4v d1, int4v d2, int4v d3)
{
    uint64_t sv;
    asm volatile(
        "s_mov_b64 %0, exec\n"
        "s_mov_b64 exec, %1\n"
        "ds_write_b128 %2, %3\n"
        "ds_write_b128 %2, %4 offset:16\n"
        "ds_write_b128 %2, %5 offset:32\n"
        "ds_write_b128 %2, %6 offset:48\n"
        "s_mov_b64 exec, %0\n"
        : "=&s"(sv)
        : "s"(1ull << 63), "v"(a), "v"(d0), "v"(d1), "v"(d2), "v"(d3)
        : "memory");
}

constexpr int K = 4, kBlk = 16;
// layout: profile 0..64K, ring 64K..66K, zero row 66K, sink 67K.., flags 80K
constexpr uint32_t kRing = 65536, kZero = 67584, kSink = 68608, kFlags = 81920;

template <int P, int W, int R, int F, int C = 0, int O = 0>
__global__ void __launch_bounds__(256) kern(int nb, const int* in, int* out, unsigned long long* cyc, int* hcol)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < 81920 / 4 + 64; i += 256) ((int*)sm)[i] = (i < 16384) ? ((i * 2654435761u) & 0x001f001f) : 0;
    __syncthreads();
    const uint32_t qrow0 = 4u * (uint32_t)((in[lane] & 15) * 544);
    uint32_t qrow[K];
    for (int k = 0; k < K; ++k) qrow[k] = qrow0 + 4u * 544u * (uint32_t)k;
    int H[K], D = 0;
    for (int k = 0; k < K; ++k) H[k] = in[64 + lane + k];
    int qA[K][8], qB[K][8];
    for (int k = 0; k < K; ++k)
        for (int j = 0; j < 8; ++j) qA[k][j] = qB[k][j] = in[128 + lane + j + 8 * k] & 0x001f001f;
    int4v hA[4], hB[4];
    for (int j = 0; j < 4; ++j) hA[j] = hB[j] = int4v {0, 0, 0, 0};
    int lt[kBlk];
    int rp = 0, acc = 0;
    const uint32_t ring = kRing + 2048u * (uint32_t)w;
    const uint32_t sink = kSink + 1024u * (uint32_t)w + 16u * (uint32_t)lane;
    const uint32_t fl = kFlags + 16u * (uint32_t)w;
    auto halo_addr = [&](int b) { return (lane == 0) ? ring + 4u * (uint32_t)((16 * b + 64) & 511) : (uint32_t)kZero; };
    auto halo = [&](int b, int4v (&h)[4]) {
        const uint32_t hb = halo_addr(b);
#pragma unroll
        for (int j = 0; j < 4; ++j) h[j] = lds_ld4(hb + 16u * (lane == 0 ? j : 0));
    };
    auto handoff = [&](int b) {
        const uint32_t eb = ring + 4u * (uint32_t)((16 * b) & 511);
        if constexpr (W == 1)
        {
            const uint32_t e = (lane == 63) ? eb : sink;
#pragma unroll
            for (int j = 0; j < 4; ++j) lds_st4(e + ((lane == 63) ? 16u * j : 0u), int4v {lt[4 * j], lt[4 * j + 1], lt[4 * j + 2], lt[4 * j + 3]});
        }
        else if constexpr (W == 2)
            st4_lane63(eb, int4v {lt[0], lt[1], lt[2], lt[3]}, int4v {lt[4], lt[5], lt[6], lt[7]},
                       int4v {lt[8], lt[9], lt[10], lt[11]}, int4v {lt[12], lt[13], lt[14], lt[15]});
    };
    int cap[K];
    for (int k = 0; k < K; ++k) cap[k] = 0;
    // C 1: capture a boundary column in 5 of every 16 blocks (tBx 256) with the 16 -> 1 v_cndmask
    // tree over the block's values; C 2: the same with 4 v_cndmask per step into cap[] (one lane
    // per step), flushed by the block's capturing lanes
    auto block = [&](int b, int (&qc)[K][8], int (&qn)[K][8], int4v (&hc)[4], int4v (&hn)[4]) {
        const bool capb = (b & 15) < 5;
        const int base = 16 * (b & 15) - 8;  // first capturing lane (may be < 0)
        int va[C == 1 ? K : 1][C == 1 ? kBlk : 1];
        const uint64_t m0 = (base >= 0 && base < 64) ? (1ull << base) : 0ull;
        if constexpr (F && O == 0)
        {
            acc += __builtin_amdgcn_readfirstlane(rp);
            if (acc == 0x7fffffff) return;  // never: a uniform branch like the progress check
        }
        if constexpr (O == 0)
        {
            if constexpr (R == 1) halo(b, hc);
            if constexpr (R == 2) halo(b + 1, hn);
            if constexpr (W != 0)
                if (b > 0) handoff(b - 1);
        }
        if constexpr (F == 1) flag_st(fl, 16 * b);
        const uint32_t pn = 4u * (uint32_t)((8 * (b + 1) - (lane >> 1)) & 511);
#pragma unroll
        for (int u = 0; u < kBlk; ++u)
        {
            int nh[K];
            const int up = shr1z(H[K - 1]) + ((R != 0) ? hc[u >> 2][u & 3] : 0);
            nh[0] = max3i(D + ((u & 1) ? qhi(qc[0][u >> 1]) : qlo(qc[0][u >> 1])), up, H[0]);
#pragma unroll
            for (int k = 1; k < K; ++k)
                nh[k] = max3i(H[k - 1] + ((u & 1) ? qhi(qc[k][u >> 1]) : qlo(qc[k][u >> 1])), nh[k - 1], H[k]);
            if constexpr (P == 1)
                if (u < 8)
#pragma unroll
                    for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);
            // P 2: the row's 8 dwords as 2 ds_read_b128 at a 4-byte aligned address (gfx950 LDS runs
            // in unaligned mode: tools/ubench/lds_align_probe.hip)
            if constexpr (P == 2)
                if (u < 8 && (u & 1) == 0)
                {
                    const int k = u >> 1;
                    const int4v* pa = (const int4v*)__builtin_assume_aligned(sm + qrow[k] + pn, 16);
                    const int4v x0 = pa[0], x1 = pa[1];
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                    {
                        qn[k][j] = x0[j];
                        qn[k][4 + j] = x1[j];
                    }
                }
            if constexpr (C == 1)
#pragma unroll
                for (int k = 0; k < K; ++k) va[k][u] = nh[k];
            if constexpr (C == 2)
            {
                const uint64_t mu = capb ? (m0 << u) : 0ull;
#pragma unroll
                for (int k = 0; k < K; ++k)
                {
                    int r;
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(cap[k]), "v"(nh[k]), "s"(mu));
                    cap[k] = r;
                }
            }
            lt[u] = H[K - 1];
            D = up;
#pragma unroll
            for (int k = 0; k < K; ++k) H[k] = nh[k];
            if constexpr (F == 1)
                if (u == 8)
                {
                    rp = raw_ld(fl + 4);
                    rp += raw_ld(fl + 8);
                    rp += raw_ld(fl + 12);
                }
            if constexpr (F == 2)
                if (u == 8)
                {
                    const int4v f4 = lds_ld4(fl + 64);
                    rp = f4[0] + f4[1] + f4[2];
                }
        }
        if constexpr (F) flag_st(fl + 4, 16 * b + 16);
        // O 1: the next block's entry (halo, then this block's hand-off) before this block's capture
        if constexpr (O == 1)
        {
            if constexpr (F)
            {
                acc += __builtin_amdgcn_readfirstlane(rp);
                if (acc == 0x7fffffff) return;
            }
            halo(b + 1, hn);
            if constexpr (W != 0) handoff(b);
        }
        if constexpr (C == 1)
            if (capb)
            {
                const int sidx = lane - base;
                if (sidx >= 0 && sidx < 16)
                {
                    const uint64_t m1 = __builtin_amdgcn_ballot_w64((sidx & 1) != 0), m2 = __builtin_amdgcn_ballot_w64((sidx & 2) != 0);
                    const uint64_t m4 = __builtin_amdgcn_ballot_w64((sidx & 4) != 0), m8 = __builtin_amdgcn_ballot_w64((sidx & 8) != 0);
                    int* dst = hcol + (size_t)(b & 1023) * 257 + 4 * lane + 1;
#pragma unroll
                    for (int k = 0; k < K; ++k)
                    {
                        int x[8];
                        auto sel = [](uint64_t m, int a, int c) { int r; asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(c), "s"(m)); return r; };
#pragma unroll
                        for (int i = 0; i < 8; ++i) x[i] = sel(m1, va[k][2 * i], va[k][2 * i + 1]);
#pragma unroll
                        for (int i = 0; i < 4; ++i) x[i] = sel(m2, x[2 * i], x[2 * i + 1]);
#pragma unroll
                        for (int i = 0; i < 2; ++i) x[i] = sel(m4, x[2 * i], x[2 * i + 1]);
                        dst[k] = sel(m8, x[0], x[1]) + (k + b) * 3;
                    }
                }
            }
        if constexpr (C == 2)
            if (capb)
            {
                const int sidx = lane - base;
                if (sidx >= 0 && sidx < 16)
                {
                    int* dst = hcol + (size_t)(b & 1023) * 257 + 4 * lane + 1;
#pragma unroll
                    for (int k = 0; k < K; ++k) dst[k] = cap[k] + (k + b) * 3;
                }
            }
    };
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int b = 0; b < nb; b += 2)
    {
        block(b, qA, qB, hA, hB);
        block(b + 1, qB, qA, hB, hA);
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    int s = D + acc + cap[0];
    for (int k = 0; k < K; ++k) s += H[k] + qA[k][0] + qB[k][7];
    for (int j = 0; j < 4; ++j) s += hA[j][0] + hB[j][3];
    out[threadIdx.x] = s;
    if (lane == 0) cyc[w] = t1 - t0;
}

int* g_hcol;
template <int P, int W, int R, int F, int C = 0, int O = 0>
void run(const char* name, int* in, int* out, unsigned long long* cyc)
{
    const int nb = 4000;
    auto k = kern<P, W, R, F, C, O>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 96 * 1024, 0, 64, in, out, cyc, g_hcol);
    hipLaunchKernelGGL(k, dim3(1), dim3(256), 96 * 1024, 0, nb, in, out, cyc, g_hcol);
    unsigned long long h[4];
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-58s %7.1f cyc/block (%5.1f /step)\n", name, (double)h[0] / nb, (double)h[0] / nb / 16);
}

int main()
{
    int *in, *out;
    unsigned long long* cyc;
    (void)hipMalloc(&in, 4096 * 4);
    (void)hipMalloc(&out, 4096 * 4);
    (void)hipMalloc(&cyc, 64);
    (void)hipMemset(in, 1, 4096 * 4);
    (void)hipMalloc(&g_hcol, 1024 * 257 * 4 + 4096);
    run<0, 0, 0, 0>("step only", in, out, cyc);
    run<1, 0, 0, 0>("+P profile reads", in, out, cyc);
    run<0, 1, 0, 0>("+W hand-off all lanes", in, out, cyc);
    run<0, 2, 0, 0>("+W hand-off lane 63 (asm exec)", in, out, cyc);
    run<0, 0, 1, 0>("+R halo JIT", in, out, cyc);
    run<0, 0, 2, 0>("+R halo a block ahead", in, out, cyc);
    run<0, 0, 0, 1>("+F progress words", in, out, cyc);
    run<1, 1, 1, 1>("P+W(all)+R(JIT)+F  (= the kernel's block)", in, out, cyc);
    run<1, 2, 1, 1>("P+W(lane63)+R(JIT)+F", in, out, cyc);
    run<1, 1, 2, 1>("P+W(all)+R(ahead)+F", in, out, cyc);
    run<1, 2, 2, 1>("P+W(lane63)+R(ahead)+F", in, out, cyc);
    run<2, 0, 0, 0>("+P profile reads as ds_read_b128", in, out, cyc);
    run<0, 0, 0, 2>("+F progress words (1 read b128, 1 write)", in, out, cyc);
    run<2, 2, 2, 2>("P(b128)+W(lane63)+R(ahead)+F(packed)", in, out, cyc);
    run<2, 1, 1, 2>("P(b128)+W(all)+R(JIT)+F(packed)", in, out, cyc);
    run<0, 0, 0, 0, 1>("+C capture, tree (5 of 16 blocks)", in, out, cyc);
    run<0, 0, 0, 0, 2>("+C capture, per-step v_cndmask (5 of 16 blocks)", in, out, cyc);
    run<1, 1, 1, 1, 1>("P+W+R+F+C(tree)  (= the kernel's block)", in, out, cyc);
    run<1, 1, 1, 1, 2>("P+W+R+F+C(per step)", in, out, cyc);
    run<1, 1, 1, 1, 1, 1>("P+W+R+F+C(tree), next entry before capture", in, out, cyc);
    run<1, 1, 1, 1, 0, 1>("P+W+R+F, next entry at block end", in, out, cyc);
    run<1, 2, 1, 1, 1, 1>("P+W(lane63)+R+F+C(tree), next entry before capture", in, out, cyc);
    run<1, 0, 0, 0>("+P profile reads (again)", in, out, cyc);
    run<0, 0, 0, 0>("step only (again)", in, out, cyc);
    return 0;
}
