// nw_scan.hip -- score-only NW / SW with linear or affine (Gotoh) gaps (BASELINE configs[4],
// SURVEY.md 8(f)3).  The reference has no implementation (README.md:7-23); the semantics are
// those of oracle/score_oracle.c (header there), which the tests hold this kernel to.
//
// Row scan, lanes across columns.  With go <= ge, opening a gap from a cell that is itself a
// horizontal gap never beats extending it, so along a row
//     F[j] = max(F_up[j] + ge, H_up[j] + go)                     (vertical: per lane)
//     D[j] = max(H_up[j-1] + s(i,j), F[j] [, 0 local])
//     E[j] = max(E[j0+1] + (j-j0-1)*ge, max_{j0<k<j} D[k] + go + (j-k-1)*ge)
//     H[j] = max(D[j], E[j])
// and E - (j-j0-1)*ge is an EXCLUSIVE prefix max over the 64 lanes of a panel: shifted by the
// uniform carry c0 = E[j0+1] it is >= 0, so the scan runs on DPP row_shr / row_bcast with
// zero fill (as nw_check.hip).  About 25 VALU per 64 cells.
//
// Parallel structure: a persistent launch, one wave per workgroup, 64-row tile rows handed out
// by an atomic ticket (a wave only ever waits on the tile row above, which an earlier ticket
// holds, so the launch cannot deadlock).  A tile row sweeps 64-column panels left to right; the
// last row of each panel (H and F, the vertical state) goes to a boundary row in HBM and a
// per-boundary progress word (release / acquire, agent scope) tells the tile row below how far
// it may go.  Rows of a tile row live in lanes: its letters, left boundary (H, E) and the
// carried column are lane-indexed registers read with v_readlane, so a row costs no LDS
// round trip besides the (prefetched) substitution lookup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_scan.h"

namespace gsa {

namespace {

template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

constexpr int kNeg = -(1 << 29);

__device__ __forceinline__ int wave_prefix_max(int v)
{
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31
    return v;
}

__device__ __forceinline__ int clamp_letter(int x, int substsz) { return ((unsigned)x < (unsigned)substsz) ? x : 0; }

__device__ __forceinline__ int hdr(long long k, int go, int ge, bool local)
{
    return (k == 0 || local) ? 0 : (int)(go + (k - 1) * ge);
}

__device__ __forceinline__ bool err_set(const ScoreArgs& a)
{
    return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

}  // namespace

template <bool LOCAL>
__global__ void __launch_bounds__(64) score_scan_kernel(ScoreArgs a)
{
    __shared__ int sub[32 * 32];
    __shared__ int tkt;
    const int lane = threadIdx.x;
    const int go = a.go, ge = a.ge;
    const long long R = a.R, C = a.C, W = C + 1;
    for (int k = lane; k < a.substsz * a.substsz; k += 64) sub[k] = G(a.subst)[k];
    const int nP = (int)((C + 63) / 64);
    const int k1 = go - (lane + 1) * ge;  // V = D + go - (l+1)*ge
    const int k2 = lane * ge;             // E = c0 + excl + l*ge
    // local: best value in this lane and its row-major index (0 = cell (0,0), value 0)
    int bv = 0;
    unsigned long long bidx = 0;
    for (;;)
    {
        __syncthreads();
        if (lane == 0) tkt = err_set(a) ? a.nTR : (int)atomicAdd(a.ticket, 1u);
        __syncthreads();
        const int tk = __builtin_amdgcn_readfirstlane(tkt);
        if (tk >= a.nTR) break;
        const long long r0 = (long long)tk * 64;
        const int nr = (int)min(64ll, R - r0);
        const long long myrow = r0 + 1 + lane;  // the row this lane carries
        const int yoff = (lane < nr) ? clamp_letter(G(a.seqY)[myrow], a.substsz) * a.substsz : 0;
        int Lh = hdr(myrow, go, ge, LOCAL);  // H[row][j0] (column 0 first)
        int Le = kNeg;                       // E[row][j0]
        int topL = hdr(r0, go, ge, LOCAL);   // H[r0][j0]
        const gptr<int> bhIn = G(a.bh) + (long long)tk * W, bfIn = G(a.bf) + (long long)tk * W;
        const gptr<int> bhOut = G(a.bh) + (long long)(tk + 1) * W, bfOut = G(a.bf) + (long long)(tk + 1) * W;
        int seen = 0;  // progress of the boundary row above, as last loaded
        for (int p = 0; p < nP; ++p)
        {
            const long long j0 = 64ll * p;
            const long long col = j0 + 1 + lane;
            const bool valid = col <= C;
            const int last = (int)min(63ll, C - 1 - j0);
            const int need = (int)min(j0 + 65, W);
            if (tk > 0 && seen < need)
            {
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (;;)
                {
                    seen = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(G(a.prog) + tk, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT));
                    if (seen >= need) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || err_set(a))
                    {
                        if (lane == 0) atomicOr(a.err, 1u);
                        return;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            int upH, upF;
            if (tk == 0)
            {
                upH = hdr(col, go, ge, LOCAL);
                upF = kNeg;
            }
            else
            {
                upH = valid ? bhIn[col] : 0;
                upF = valid ? bfIn[col] : kNeg;
            }
            const int xo = valid ? clamp_letter(G(a.seqX)[col], a.substsz) : 0;
            const int topNext = __builtin_amdgcn_readlane(upH, 63);  // H[r0][j0+64]: next panel's corner
            int dg = topL;  // H[i-1][j0] for lane 0's diagonal
            int nLh = 0, nLe = 0;
            int pv = 0, pi = 0;  // LOCAL: best of this lane's column within the panel (first row)
            int s_nx = sub[__builtin_amdgcn_readfirstlane(yoff) + xo];
            for (int r = 0; r < nr; ++r)
            {
                const int s = s_nx;
                if (r + 1 < nr) s_nx = sub[__builtin_amdgcn_readlane(yoff, r + 1) + xo];
                const int lh = __builtin_amdgcn_readlane(Lh, r);
                const int le = __builtin_amdgcn_readlane(Le, r);
                const int diag = __builtin_amdgcn_update_dpp(dg, upH, 0x138, 0xf, 0xf, false);  // H[i-1][j-1]
                const int F = max(upF + ge, upH + go);
                int D = max(diag + s, F);
                if (LOCAL) D = max(D, 0);
                const int c0 = max(le + ge, lh + go);  // E[i][j0+1]
                const int m = max(D + k1, c0) - c0;
                const int ex = __builtin_amdgcn_update_dpp(0, wave_prefix_max(m), 0x138, 0xf, 0xf, true);  // exclusive
                const int E = ex + c0 + k2;
                const int H = max(D, E);
                if (LOCAL)
                {
                    const bool up = H > pv;
                    pv = up ? H : pv;
                    pi = up ? r : pi;
                }
                const int hl = __builtin_amdgcn_readlane(H, last), el = __builtin_amdgcn_readlane(E, last);
                nLh = (lane == r) ? hl : nLh;  // H[i][j0+64]: the next panel's left boundary of row i
                nLe = (lane == r) ? el : nLe;
                dg = lh;
                upH = H;
                upF = F;
            }
            // bottom row of the tile row -> boundary row tk+1, then publish
            if (valid)
            {
                bhOut[col] = upH;
                bfOut[col] = upF;
            }
            if (p == 0 && lane == 0)
            {
                bhOut[0] = hdr(r0 + nr, go, ge, LOCAL);
                bfOut[0] = kNeg;
            }
            if (!LOCAL && tk == a.nTR - 1 && p == nP - 1 && lane == last) G(a.result)[0] = upH;  // H[R][C]
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            if (lane == 0)
                __hip_atomic_store(G(a.prog) + tk + 1, need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (LOCAL && valid && pv > 0)
            {
                const unsigned long long idx = (unsigned long long)(r0 + 1 + pi) * (unsigned long long)W + col;
                if (pv > bv || (pv == bv && idx < bidx))
                {
                    bv = pv;
                    bidx = idx;
                }
            }
            topL = topNext;
            Lh = nLh;
            Le = nLe;
        }
    }
    if (LOCAL)
    {
        const unsigned long long key =
            ((unsigned long long)bv << a.idxBits) | (((1ull << a.idxBits) - 1) - bidx);
        atomicMax(a.best, key);
    }
}

hipError_t launch_score_scan(const ScoreArgs& a, int local, int cu_count, hipStream_t st)
{
    if (a.substsz > 32) return hipErrorInvalidValue;
    const int grid = std::max(1, (int)std::min<long long>(a.nTR, (long long)cu_count * 8));
    if (local)
        hipLaunchKernelGGL(score_scan_kernel<true>, dim3(grid), dim3(64), 0, st, a);
    else
        hipLaunchKernelGGL(score_scan_kernel<false>, dim3(grid), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace gsa
