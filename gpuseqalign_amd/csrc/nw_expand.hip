// nw_expand.hip -- full-matrix expansion, pass 2 of the two-pass full fill, hand-written wave64
// HIP for gfx950 (MI355X).
//
// The plain family (NwAlign_Gpu3..6, nwalign_gpu3_ml_diagdiag.cu:288-596) writes the whole
// (R+1) x (C+1) matrix.  A single wavefront that also stores every cell is bound by its critical
// path and couples its strips to the store stream (nw_lane.hip).  The two-pass fill splits the
// two: pass 1 is the K-rows sparse fill (nw_krow.hip, XR instance: 4 rows per lane, the
// headline's wavefront) and keeps every 256th column (the tile header columns, tBx = kExpHB) and
// every 64th row; pass 2 (this file) recomputes all 64-row x kExpTW-column tiles from their top
// row and left column at once -- tiles are independent, so it is bound by HBM writes, not by a
// dependency chain.  This is the reference's own tile recompute (NwTrace2_AlignTile,
// nwtrace2_sparse.cpp:40-96) run for every tile, into the full matrix.
//
// A wave owns one tile, one row per lane, with the step of nw_lane.hip (unshifted values, 4 VALU
// per cell): lane l owns row r0 + l and at step t works on column cb + t - l; columns <= cb are the
// tile's left boundary (pass-1 header column), lane 0's row above is the tile's top row (pass-1
// row buffer).  The tile is stored as a parallelogram (row r0 + rr over columns cb + 64 - rr ..
// cb + cols + 63 - rr), so every 128-byte line of the pitched layout (gsa_full_pitch) belongs to
// one tile and leaves whole: the transposed stores of nw_lane.hip, 16 rows x 64 bytes per
// instruction, the two halves of each line back to back.  A workgroup = 7 tile waves (a 448-row
// task of one tile column, sharing the column profile Q[y][j] = s(y, X[cb + j]) - g in LDS) and a
// loader wave that stages each task's inputs (nw_expand_dev.h ex_stream).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_expand_dev.h"

namespace gsa {
namespace {

using namespace xdev;

// the streamed expansion (ex_stream): persistent, one workgroup per CU; wave 0 records the
// workgroup's effective clock (gsa_set_full_timing)
__global__ void __launch_bounds__(64 * kExpStreamWaves) nw_expand_stream_kernel(ExpandArgs a)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    uint64_t c0 = 0, r0 = 0;
    if (a.clk && w == 0)
    {
        c0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    ex_stream<kExpStreamWaves, false>(a, a.counter, ExFused {nullptr, 0u, nullptr}, w, lane);
    if (a.clk && w == 0)
    {
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (lane == 0) G(a.clk)[blockIdx.x] = (uint64_t)(uint32_t)(c1 - c0) | ((uint64_t)(uint32_t)(r1 - r0) << 32);
    }
}

}  // namespace

size_t expand_stream_lds_bytes(int substsz) { return (size_t)xdev::ex_stream_lds(substsz, kExpStreamWaves - 1); }

hipError_t launch_expand_stream(const ExpandArgs& a, hipStream_t stream, int grid)
{
    if (a.nTasks <= 0) return hipSuccess;
    if (!a.counter || !a.err || a.substsz > 32) return hipErrorInvalidValue;
    const size_t lds = expand_stream_lds_bytes(a.substsz);
    auto kern = nw_expand_stream_kernel;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (grid <= 0)
    {
        int dev = 0, cus = 0;
        if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
        if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
        grid = std::max(1, cus);
    }
    grid = std::min(grid, a.nTasks);
#ifdef GSA_EXPAND_GRID_PROBE  // (diagnostic builds: the expansion on fewer CUs, its per-CU rate)
    grid = std::min(grid, GSA_EXPAND_GRID_PROBE);
#endif
    if ((e = record_foot((const void*)kern, lds, 64 * kExpStreamWaves, grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kExpStreamWaves), lds, stream, a);
    return hipGetLastError();
}

}  // namespace gsa
