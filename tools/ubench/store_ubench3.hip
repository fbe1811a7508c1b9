// store_ubench3.hip -- chip-wide store bandwidth vs. bytes written contiguously per row visit.
// Each wave owns 64 consecutive rows of a row-major int32 matrix (pitch LD ints) and writes them
// in column chunks: one "visit" writes W contiguous bytes of one row, the wave visits its 64 rows
// in turn, then moves to the next column chunk (the order a 64-row strip fill produces when it
// buffers W/4 columns per row before storing).  Every instruction is a 1 KB dwordx4 wave store:
// W < 1 KB -> 1024/W rows per instruction; W >= 1 KB -> W/1024 consecutive instructions per row.
// Question answered: the per-visit contiguity the batch full fill needs to pass ~4 TB/s.
// Build: hipcc --offload-arch=gfx950 -O3 store_ubench3.hip -o store_ubench3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));

template <int W, bool NT>
__global__ void kern(int* out, long long ld, long long off, int iters)
{
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const long long row0 = wave * 64;
    int4a v = {lane, lane + 1, lane + 2, lane + 3};
    constexpr int LPR = W >= 1024 ? 64 : W / 16;  // lanes per row in one instruction
    constexpr int RPI = 64 / LPR;                  // rows per instruction
    constexpr int IPV = W >= 1024 ? W / 1024 : 1;  // instructions per visit
    constexpr int IPC = IPV * (64 / RPI);          // instructions per column chunk (all 64 rows)
    for (int it = 0; it < iters; ++it)
    {
        const int chunk = it / IPC, inC = it % IPC;
        const int visit = inC / IPV, part = inC % IPV;
        const long long r = row0 + (long long)visit * RPI + lane / LPR;
        const long long c = (long long)chunk * (W / 4) + part * 256 + 4 * (lane % LPR) + off;
        int4a* p = (int4a*)(out + r * ld + c);
        if (NT)
            __builtin_nontemporal_store(v, p);
        else
            *p = v;
        v += 1;
    }
}

// Lane-fill shaped stores: every instruction writes 16 rows x 64 B (4 lanes per row), aligned.
// PAIR: consecutive instructions write the two 64-B halves of the same 128-B lines (a row's two
// blocks stored together); MASK: only half of the rows (alternating per pair of blocks) store,
// the other half idle (the parity scheme: a row emits its two aligned halves every other block).
template <bool PAIR, bool MASK>
__global__ void kernL(int* out, long long ld, long long off, int iters)
{
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const long long row0 = wave * 64;
    int4a v = {lane, lane + 1, lane + 2, lane + 3};
    // one "block" = 16 columns per row of all 64 rows = 4 instructions (16 rows each)
    for (int it = 0; it < iters; ++it)
    {
        int blk, k;  // block (64-B column chunk) and row group
        if (!PAIR)
        {
            blk = it / 4, k = it % 4;
        }
        else
        {
            // blocks 2q, 2q+1 issued as: k0 b0, k0 b1, k1 b0, k1 b1, ...
            const int q = it / 8, r = it % 8;
            k = r / 2, blk = 2 * q + (r & 1);
        }
        const long long rr = row0 + 16 * k + (lane & 15);
        const long long c = (long long)blk * 16 + 4 * (lane >> 4) + off;
        if (MASK && ((rr + blk / 2) & 1)) continue;
        *(int4a*)(out + rr * ld + c) = v;
        v += 1;
    }
}

int main()
{
    int* out = nullptr;
    const int waves_per_wg = 4;
    const int wgs = 1024;                  // 4096 waves = 16 per CU, as the batch fill
    const long long ldmax = 20032 + 1;
    const size_t bytes_alloc = (size_t)ldmax * 64 * waves_per_wg * wgs * 4 + 4096;  // ~21 GB
    if (hipMalloc(&out, bytes_alloc) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4096;  // 4 MB per wave = 64 rows x 16384 cols... cols used = 4096*1024/64/4 = 16384 < ld
    auto run = [&](auto k, const char* name, int W, long long ld, long long off) {
        hipLaunchKernelGGL(k, wgs, 64 * waves_per_wg, 0, 0, out, ld, off, iters);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, wgs, 64 * waves_per_wg, 0, 0, out, ld, off, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = (double)wgs * waves_per_wg * iters * 1024;
        printf("%-3s W %5d B  ld %5lld off %lld: %8.3f ms  %8.1f GB/s\n", name, W, ld, off, ms, bytes / ms / 1e6);
    };
    {
        auto runL = [&](auto k, const char* name, int mult) {
            const long long ld = 20032;
            hipLaunchKernelGGL(k, wgs, 64 * waves_per_wg, 0, 0, out, ld, 0LL, iters * mult);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, wgs, 64 * waves_per_wg, 0, 0, out, ld, 0LL, iters * mult);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double bytes = (double)wgs * waves_per_wg * iters * 1024;  // MASK: half the lanes over 2x iters
            printf("lane-shaped %-12s: %8.3f ms  %8.1f GB/s\n", name, ms, bytes / ms / 1e6);
        };
        runL(kernL<false, false>, "plain", 1);
        runL(kernL<true, false>, "pair", 1);
        runL(kernL<true, true>, "pair+mask", 2);
        runL(kernL<false, true>, "mask", 2);
    }
    for (long long ld : {20001LL, 20032LL})
    {
        const long long off = ld == 20001 ? 1 : 0;
        run(kern<64, false>, "pl", 64, ld, off);
        run(kern<128, false>, "pl", 128, ld, off);
        run(kern<256, false>, "pl", 256, ld, off);
        run(kern<1024, false>, "pl", 1024, ld, off);
        run(kern<2048, false>, "pl", 2048, ld, off);
        run(kern<4096, false>, "pl", 4096, ld, off);
        run(kern<8192, false>, "pl", 8192, ld, off);
        run(kern<64, true>, "nt", 64, ld, off);
        run(kern<256, true>, "nt", 256, ld, off);
        run(kern<1024, true>, "nt", 1024, ld, off);
        run(kern<4096, true>, "nt", 4096, ld, off);
    }
    return 0;
}
