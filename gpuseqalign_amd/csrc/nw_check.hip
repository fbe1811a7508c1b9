// nw_check.hip -- device-side verification of fill outputs.
//
// The reference checks a GPU fill only through what its host consumers read: align_cost,
// the score hash (a CPU recompute, nwtrace2_sparse.cpp:263-340) and the trace hash, so sparse
// header values off the trace path are never compared.  These kernels
// check EVERY output value against the recurrence (nwalign_cpu1_st_row.cpp:4-10), in parallel:
//
//  * sparse (mlsp) headers -- tile consistency.  Tile (iT, jT) is recomputed from its own
//    header row and column alone (as NwTrace2_AlignTile does, nwtrace2_sparse.cpp:40-96, but
//    over the padded tile, padding letter 0), and its last row / last column must equal the
//    header row of tile (iT+1, jT) / header column of tile (iT, jT+1); row 0 and column 0
//    must be j*g and i*g, and every tile's two corner copies must agree.  If all of that
//    holds, every header is the exact matrix value by induction over tile anti-diagonals.
//  * full matrix -- cell consistency: H[i][j] = max3(H[i-1][j-1] + s, H[i-1][j] + g,
//    H[i][j-1] + g) against the stored neighbours, plus row 0 / column 0; same induction.
//
// Tile recompute, one wave per tile, lanes across 64-column panels, rows in sequence:
//   E[j]  = max(H[i-1][j-1] + s(i,j), H[i-1][j] + g)
//   H[i][j] = max(E[j], H[i][j-1] + g)  =>  with H'[j] = H[i][j] - (j-j0)*g,
//   H'[j] = max(H[i][j0], max_{m<=j} E'[m])  -- an inclusive prefix max: 6 DPP steps.
// Values are shifted by the uniform left boundary H[i][j0] so they are >= 0 and the scan's
// out-of-range lanes can read 0.  ~16 VALU + 3 LDS ops per 64 cells; tiles are independent,
// so many waves per CU hide the latencies.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_check.h"

namespace gsa {

namespace {

template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

constexpr int kCheckTileByMax = 4096;  // LDS column buffer of the tile checker

__device__ __forceinline__ void record(const CheckArgs& a, unsigned long long idx)
{
    atomicAdd(a.res + 1, 1ull);
    atomicMin(a.res + 2, idx);
}

// inclusive prefix max over the wave of values >= 0 (out-of-row lanes read 0)
__device__ __forceinline__ int wave_prefix_max(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
    return v;
}

__device__ __forceinline__ int clamp_letter(int x, int substsz) { return ((unsigned)x < (unsigned)substsz) ? x : 0; }

}  // namespace

// one wave per workgroup; tiles handed out grid-stride
__global__ void __launch_bounds__(64) check_sparse_kernel(CheckArgs a)
{
    __shared__ int sub[32 * 32];
    __shared__ int colbuf[kCheckTileByMax + 1];
    __shared__ int yb[kCheckTileByMax + 1];
    const int lane = threadIdx.x;
    const int g = a.g, tBx = a.tBx, tBy = a.tBy;
    const long long W = tBx + 1, H = tBy + 1;
    for (int k = lane; k < a.substsz * a.substsz; k += 64) sub[k] = G(a.subst)[k];
    unsigned long long checked = 0;
    const long long ntiles = (long long)a.trows * a.tcols;
    for (long long k = blockIdx.x; k < ntiles; k += gridDim.x)
    {
        const int iT = (int)(k / a.tcols), jT = (int)(k % a.tcols);
        const gptr<const int> hr = G(a.hrow) + k * W;
        const gptr<const int> hc = G(a.hcol) + k * H;
        const long long rbase = (long long)iT * tBy, cbase = (long long)jT * tBx;
        __syncthreads();  // previous tile's LDS reads are done
        // left header -> colbuf; boundary checks; row letters
        for (int e = lane; e <= tBy; e += 64)
        {
            const int v = hc[e];
            colbuf[e] = v;
            if (jT == 0)
            {
                ++checked;
                if (v != (int)((rbase + e) * g)) record(a, (unsigned long long)(a.hrowElems + k * H + e));
            }
            const long long r = rbase + e;
            yb[e] = clamp_letter(r < a.adjrows ? G(a.seqY)[r] : 0, a.substsz) * a.substsz;
        }
        if (iT == 0)
            for (int c = lane; c <= tBx; c += 64)
            {
                ++checked;
                if (hr[c] != (int)((cbase + c) * g)) record(a, (unsigned long long)(k * W + c));
            }
        if (lane == 0)
        {
            ++checked;
            if (hr[0] != hc[0]) record(a, (unsigned long long)(k * W));
        }
        const bool below = iT + 1 < a.trows, right = jT + 1 < a.tcols;
        if (!below && !right) continue;
        __syncthreads();
        const gptr<const int> hrNext = G(a.hrow) + (k + a.tcols) * W;  // header row of tile (iT+1, jT)
        if (below && lane == 0)
        {
            ++checked;
            if (hrNext[0] != colbuf[tBy]) record(a, (unsigned long long)((k + a.tcols) * W));
        }
        const int nP = (tBx + 63) / 64;
        for (int p = 0; p < nP; ++p)
        {
            const int j0 = 64 * p;
            const int col = j0 + 1 + lane;  // tile-local column of this lane
            const bool valid = col <= tBx;
            const long long gc = cbase + col;
            const int xo = valid ? clamp_letter(gc < a.adjcols ? G(a.seqX)[gc] : 0, a.substsz) : 0;
            int up = valid ? hr[col] : 0;
            const int c1 = -(lane + 1) * g, c2 = -lane * g, c3 = (lane + 1) * g;
            const int last = min(63, tBx - 1 - j0);
            int Lprev = __builtin_amdgcn_readfirstlane(colbuf[0]);  // H[0][j0]
            const int top = __builtin_amdgcn_readlane(up, last);     // H[0][j0+last+1]
            __syncthreads();
            if (lane == 0) colbuf[0] = top;
            int Lnext = __builtin_amdgcn_readfirstlane(colbuf[1]);
            int ynext = __builtin_amdgcn_readfirstlane(yb[1]);
            for (int i = 1; i <= tBy; ++i)
            {
                const int L = Lnext, y = ynext;
                if (i < tBy)
                {
                    Lnext = __builtin_amdgcn_readfirstlane(colbuf[i + 1]);
                    ynext = __builtin_amdgcn_readfirstlane(yb[i + 1]);
                }
                const int s = sub[y + xo];
                const int diag = __builtin_amdgcn_update_dpp(Lprev, up, 0x138, 0xf, 0xf, false);  // wave_shr:1
                const int m = max(max(diag + s + c1, up + c2), L) - L;
                const int h = wave_prefix_max(m) + L + c3;
                if (lane == last) colbuf[i] = h;  // H[i][j0+last+1]: next panel's left boundary
                Lprev = L;
                up = h;
            }
            if (below && valid)
            {
                ++checked;
                if (hrNext[col] != up) record(a, (unsigned long long)((k + a.tcols) * W + col));
            }
        }
        if (right)
        {
            __syncthreads();
            const gptr<const int> hcNext = G(a.hcol) + (k + 1) * H;  // header column of tile (iT, jT+1)
            for (int e = lane; e <= tBy; e += 64)
            {
                ++checked;
                if (hcNext[e] != colbuf[e]) record(a, (unsigned long long)(a.hrowElems + (k + 1) * H + e));
            }
        }
    }
    if (checked) atomicAdd(a.res, checked);
}

// one thread per column; blockIdx.y takes a contiguous range of rows, so the row above (`up`) and
// its left neighbour (`diag`) come from the previous iteration's registers and each cell costs two
// loads from the same lines (its own value and its left neighbour): ~1x the matrix in HBM reads
__global__ void __launch_bounds__(256) check_full_kernel(CheckArgs a)
{
    __shared__ int sub[32 * 32];
    for (int k = threadIdx.x; k < a.substsz * a.substsz; k += 256) sub[k] = G(a.subst)[k];
    __syncthreads();
    const long long j = (long long)blockIdx.x * 256 + threadIdx.x;
    if (j >= a.adjcols) return;
    const int g = a.g;
    const long long ld = a.ld;
    const gptr<const int> S = G(a.score);
    const int xo = clamp_letter(G(a.seqX)[j], a.substsz);
    const long long per = (a.adjrows + gridDim.y - 1) / gridDim.y;
    const long long i0 = (long long)blockIdx.y * per, i1 = min(a.adjrows, i0 + per);
    unsigned long long checked = 0;
    int up = 0, diag = 0;
    if (i0 > 0 && i0 < i1)
    {
        up = S[(i0 - 1) * ld + j];
        if (j > 0) diag = S[(i0 - 1) * ld + j - 1];
    }
    for (long long i = i0; i < i1; ++i)
    {
        const int v = S[i * ld + j];
        const int left = j > 0 ? S[i * ld + j - 1] : 0;
        int e;
        if (i == 0)
            e = (int)(j * g);
        else if (j == 0)
            e = (int)(i * g);
        else
        {
            const int y = clamp_letter(G(a.seqY)[i], a.substsz);
            e = max(max(diag + sub[y * a.substsz + xo], up + g), left + g);
        }
        ++checked;
        if (v != e) record(a, (unsigned long long)(i * a.adjcols + j));
        up = v;
        diag = left;
    }
    atomicAdd(a.res, checked);
}

hipError_t launch_check_sparse(const CheckArgs& a, int cu_count, hipStream_t st)
{
    if (a.tBy > kCheckTileByMax || a.substsz > 32) return hipErrorInvalidValue;
    const long long ntiles = (long long)a.trows * a.tcols;
    const int grid = (int)std::min<long long>(ntiles, (long long)cu_count * 12);
    hipLaunchKernelGGL(check_sparse_kernel, dim3(grid), dim3(64), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_check_full(const CheckArgs& a, hipStream_t st)
{
    if (a.substsz > 32) return hipErrorInvalidValue;
    const int gx = (int)((a.adjcols + 255) / 256);
    if (a.ld < a.adjcols) return hipErrorInvalidValue;
    // ~64k blocks of 256 columns x a contiguous row range
    const int gy = (int)std::min<long long>(a.adjrows, std::max<long long>(1, 65536 / std::max(gx, 1)));
    hipLaunchKernelGGL(check_full_kernel, dim3(gx, gy), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace gsa
