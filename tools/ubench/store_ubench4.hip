// store_ubench4.hip -- store-only rate of the full-matrix expansion's write pattern on one large
// matrix (pass 2 of the two-pass full fill, nw_expand_dev.h): tasks of W waves x 64 rows x TW
// columns claimed from a counter by persistent workgroups; a wave writes its 64 rows x TW columns
// in pairs of 16-column blocks, each block as 4 dwordx4 instructions of 16 rows x 64 B (the
// transposed lane-fill shape), the even and odd block of a pair back to back so each 128-B line
// leaves whole.  Question answered: how fast can this pattern write a 100k x 100k matrix (400 KB
// row pitch) against a 20k-wide one, by task order, task width and waves per CU.
// Build: hipcc --offload-arch=gfx950 -O3 store_ubench4.hip -o store_ubench4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));

// order 0: row-chunk-major (all tile columns of chunk 0, then chunk 1...); 1: tile-column-major;
// 2: anti-diagonals of (chunk, tile column) weighted as the fused fill's ready time.
// SHAPE 0: 16 rows x 64 B per instruction (pairs); 1: 8 rows x 128 B; 2: 4 rows x 256 B
template <int SHAPE, int DELAY = 0, int RAMP = 0, int NT = 0>
__global__ void kern(int* out, long long ld, int R, int C, int TW, int W, const int* sched, unsigned* counter,
                     int nChunks, int nTiles)
{
    __shared__ int task;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nTasks = nChunks * nTiles;
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) task = (int)atomicAdd(counter, 1u);
        __syncthreads();
        const int t = task;
        if (t >= nTasks) break;
        const int rc = sched[2 * t], jT = sched[2 * t + 1];
        const long long r0 = (long long)rc * W * 64 + w * 64 + 1;
        if (r0 + 63 >= R) continue;
        const long long cb = (long long)jT * TW;
        int4a v = {lane, lane + 1, lane + 2, lane + 3};
        if (RAMP > 0)
        {
            // the expansion's ramp: RAMP blocks of compute before the first store (RAMP / 2 pairs)
            int acc = v[0];
            for (int q = 0; q < RAMP / 2 * DELAY; ++q) acc = __builtin_amdgcn_update_dpp(0, acc, 0x138, 0xF, 0xF, true) + q;
            v[1] += acc;
        }
        for (int b = 0; b + 1 < TW / 16 && cb + 16 * b + 32 <= C; b += 2)
        {
            if (DELAY > 0)
            {
                // a dependent VALU chain between store bursts (the expansion's 2 blocks of compute)
                int acc = v[0];
#pragma unroll
                for (int q = 0; q < DELAY; ++q) acc = __builtin_amdgcn_update_dpp(0, acc, 0x138, 0xF, 0xF, true) + q;
                v[1] += acc;
            }
            if (SHAPE == 0)
            {
#pragma unroll
                for (int k = 0; k < 4; ++k)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                    {
                        const long long rr = r0 + 16 * k + (lane & 15);
                        const long long c = cb + 16 * (b + h) + 4 * (lane >> 4);
                        if (NT)
                            __builtin_nontemporal_store(v, (int4a*)(out + rr * ld + c));
                        else
                            *(int4a*)(out + rr * ld + c) = v;
                        v += 1;
                    }
            }
            else if (SHAPE == 1)
            {
#pragma unroll
                for (int k = 0; k < 8; ++k)
                {
                    const long long rr = r0 + 8 * k + (lane >> 3);
                    const long long c = cb + 16 * b + 4 * (lane & 7);
                    *(int4a*)(out + rr * ld + c) = v;
                    v += 1;
                }
            }
            else if (SHAPE >= 3)
            {
                // 8 rows x 128 B per instruction, lane -> (row, chunk) by SHAPE: 3 row = L & 7, chunk =
                // L >> 3; 4 row bits at lane bits {0, 4, 5}, chunk {1, 2, 3}; 5 row {2, 3, 5}, chunk
                // {0, 1, 4}; 6 row {2, 3, 4}, chunk {0, 1, 5}
                int row, ch;
                if (SHAPE == 7)
                {
                    // 16 rows x 64 B per instruction, each quad 64 contiguous bytes of one row; the
                    // line's other half in the next instruction
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                    {
                        const long long rr = r0 + 16 * (k >> 1) + (lane >> 2);
                        const long long c = cb + 16 * (b + (k & 1)) + 4 * (lane & 3);
                        *(int4a*)(out + rr * ld + c) = v;
                        v += 1;
                    }
                    continue;
                }
                if (SHAPE == 3) { row = lane & 7; ch = lane >> 3; }
                else if (SHAPE == 4) { row = (lane & 1) | ((lane >> 4) << 1); ch = (lane >> 1) & 7; }
                else if (SHAPE == 5) { row = ((lane >> 2) & 3) | ((lane >> 5) << 2); ch = (lane & 3) | (((lane >> 4) & 1) << 2); }
                else { row = (lane >> 2) & 7; ch = (lane & 3) | ((lane >> 5) << 2); }
#pragma unroll
                for (int k = 0; k < 8; ++k)
                {
                    const long long rr = r0 + 8 * k + row;
                    const long long c = cb + 16 * b + 4 * ch;
                    *(int4a*)(out + rr * ld + c) = v;
                    v += 1;
                }
            }
            else if ((b & 3) == 0 && cb + 16 * b + 64 <= C)
            {
#pragma unroll
                for (int k = 0; k < 16; ++k)
                {
                    const long long rr = r0 + 4 * k + (lane >> 4);
                    const long long c = cb + 16 * b + 4 * (lane & 15);
                    *(int4a*)(out + rr * ld + c) = v;
                    v += 1;
                }
            }
        }
        if (RAMP > 0)
        {
            int acc = v[0];
            for (int q = 0; q < RAMP / 2 * DELAY; ++q) acc = __builtin_amdgcn_update_dpp(0, acc, 0x138, 0xF, 0xF, true) + q;
            if (acc == 0x7fffffff) out[0] = acc;
        }
    }
}


// The streamed expansion's task structure (nw_expand_dev.h ex_stream): W waves of which W - 1 store
// (one idle, the loader's slot), per task two workgroup barriers around a PREP-cycle delay (the
// profile build), then per wave 4 ramp blocks (compute only), 32 stored blocks in pairs, 4 tail
// blocks; BLK = dependent-VALU cycles per block (the recurrence).
template <int PREP, int BLK>
__global__ void kernX(int* out, long long ld, int R, int C, int TW, int W, const int* sched, unsigned* counter,
                      int nChunks, int nTiles)
{
    __shared__ int task;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int NW = W - 1;
    const int nTasks = nChunks * nTiles;
    int acc = lane;
    auto delay = [&](int n) {
        for (int q = 0; q < n; ++q) acc = __builtin_amdgcn_update_dpp(0, acc, 0x138, 0xF, 0xF, true) + q;
    };
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) task = (int)atomicAdd(counter, 1u);
        __syncthreads();
        const int t = task;
        if (t >= nTasks) break;
        delay(PREP);
        __syncthreads();
        if (w == NW) continue;
        const int rc = sched[2 * t], jT = sched[2 * t + 1];
        const long long r0 = (long long)rc * NW * 64 + w * 64 + 1;
        if (r0 + 63 >= R) continue;
        const long long cb = (long long)jT * TW;
        int4a v = {lane, lane + 1, lane + 2, lane + 3};
        delay(4 * BLK);
        for (int b = 0; b + 1 < TW / 16 && cb + 16 * b + 32 <= C; b += 2)
        {
            delay(2 * BLK);
            v[1] += acc;
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                {
                    const long long rr = r0 + 16 * k + (lane & 15);
                    const long long c = cb + 16 * (b + h) + 4 * (lane >> 4);
                    *(int4a*)(out + rr * ld + c) = v;
                    v += 1;
                }
        }
        delay(4 * BLK);
    }
    if (acc == 0x7fffffff) out[0] = acc;
}

int main(int argc, char** argv)
{
    const int R = argc > 1 ? atoi(argv[1]) : 99968;
    const int C = argc > 2 ? atoi(argv[2]) : 99968;
    const long long ldAdd = argc > 3 ? atoll(argv[3]) : 32;
    const long long ld = ((C + 31) / 32) * 32 + ldAdd;  // (a multiple of 32 + ldAdd)
    int* out = nullptr;
    const size_t bytes = (size_t)(R + 64) * ld * 4 + 4096;
    if (hipMalloc(&out, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
    unsigned* counter;
    hipMalloc(&counter, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    auto run = [&](auto k, const char* shape, int W, int TW, int order, int wgPerCu, int rowsW = 0, int grid = 0) {
        const int nChunks = (R - 1) / ((rowsW ? rowsW : W) * 64), nTiles = C / TW;
        const size_t lds = wgPerCu == 1 ? 100000 : 0;
        std::vector<int> hs;
        std::vector<std::pair<long long, int>> key;
        for (int rc = 0; rc < nChunks; ++rc)
            for (int j = 0; j < nTiles; ++j)
            {
                const long long kk = order == 0 ? (long long)rc * nTiles + j : order == 1 ? (long long)j * nChunks + rc
                                                                                       : (long long)rc * 400 + (long long)j * TW;
                key.push_back({kk, rc * nTiles + j});
            }
        std::stable_sort(key.begin(), key.end());
        for (auto& q : key) { hs.push_back(q.second / nTiles); hs.push_back(q.second % nTiles); }
        int* sched = nullptr;
        hipMalloc(&sched, hs.size() * 4);
        hipMemcpy(sched, hs.data(), hs.size() * 4, hipMemcpyHostToDevice);
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 100000);
        float best = 1e9;
        for (int rep = 0; rep < 3; ++rep)
        {
            hipMemsetAsync(counter, 0, 4);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, grid ? grid : cus * wgPerCu, 64 * W, lds, 0, out, ld, R, C, TW, W, sched, counter, nChunks, nTiles);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        hipFree(sched);
        const double wbytes = (double)nChunks * (rowsW ? rowsW : W) * 64 * (double)nTiles * TW * 4;
        const int g = grid ? grid : cus * wgPerCu;
        printf("R %d C %d ld %lld shape %s W %2d x %d/CU TW %5d order %d grid %d: %8.3f ms %8.1f GB/s %6.2f GB/s/WG\n", R, C,
               ld, shape, W, wgPerCu, TW, order, g, best, wbytes / best / 1e6, wbytes / best / 1e6 / g);
    };
    // quad-contiguous half lines (16 rows x 64 B, halves in consecutive instructions) against whole lines
    run(kern<7, 0>, "16x64 quad-contig", 8, 512, 2, 1, 0, 64);
    run(kern<6, 0>, "8x128 ch{0,1,5}", 8, 512, 2, 1, 0, 64);
    run(kern<0, 0>, "16x64 pure", 8, 512, 2, 1, 0, 64);
    run(kern<7, 0>, "16x64 quad-contig", 8, 512, 2, 1, 0, 256);
    run(kern<6, 0>, "8x128 ch{0,1,5}", 8, 512, 2, 1, 0, 256);
    return 0;
}
