// nw_expand_dev.h -- device code of the full-matrix expansion (pass 2 of the two-pass full fill),
// shared by the stand-alone expansion kernel (nw_expand.hip) and the single-pair fused kernel
// (nw_krow.hip, XR section): see nw_expand.hip for the algorithm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "nw_expand.h"

#ifndef GSA_EXPAND_PROBE
#define GSA_EXPAND_PROBE 0  // diagnostic builds only (tools/r05_xprobe.sh)
#endif

namespace gsa {
namespace xdev {

constexpr int kBlk = 16;           // steps per block
constexpr int kH = kBlk / 4;       // halo registers (int4) per block
constexpr int kSubRow = 36;        // dwords per subT row (32 letters + 4)
constexpr int kQOff = 64;          // Q[y][kQOff + j], j = 1..kExpTW; reads reach j = -63 .. kExpTW + 15
constexpr int kQS = kQOff + kExpTW + 32;  // Q row stride (dwords), = 0 mod 32: the bank is the column alone
constexpr int kTopS = kExpTW + 80;        // per-wave top row: topw[t] = H(r0 - 1, cb + t) + g, t < kExpTW + 80
static_assert(kQS % 32 == 0 && kTopS % 4 == 0 && kExpTW % kExpHB == 0, "LDS strides");

extern __shared__ __attribute__((aligned(16))) char xsm[];

typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(xsm + a); }
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(xsm + a) = v; }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(xsm + a); }
// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

struct ExLds
{
    uint32_t sub, q, top, gfill;
};
// LDS of a workgroup of `waves` tile waves: the column profile; subT, which only the profile build
// reads, overlaid by one top row per wave; a row of g.  (79.9 KB for 8 waves and 25 letters: two
// workgroups per CU)
__host__ __device__ inline ExLds ex_layout(int substsz, int waves)
{
    ExLds L;
    L.q = 0;
    L.sub = (uint32_t)substsz * kQS * 4u;
    L.top = L.sub;
    const uint32_t subB = (uint32_t)substsz * kSubRow * 4u, topB = (uint32_t)waves * kTopS * 4u;
    L.gfill = L.top + (subB > topB ? subB : topB);
    return L;
}

__device__ __forceinline__ ExpandPair ex_desc(const ExpandPair* p)
{
    constexpr int N = sizeof(ExpandPair) / 4;
    const int* wds = (const int*)p;
    union
    {
        int v[N];
        ExpandPair d;
    } u;
#pragma unroll
    for (int k = 0; k < N; ++k) u.v[k] = __builtin_amdgcn_readfirstlane(G(wds)[k]);
    return u.d;
}

// one 64-row x kExpTW-column tile of the full matrix, one row per lane
__device__ __forceinline__ void ex_tile(const ExpandArgs& a, const ExpandPair& d, const ExLds& L, int w, int lane,
                                        int cb, int cols, int r0)
{
    const int g = a.g;
    // left boundary column cb of the tile, columns cb+1 .. cb+cols (ex_cb, ex_cols)
    const int r = r0 + lane;
    int y = (r <= d.R) ? G(d.seqY)[r] : 0;
    y = ((unsigned)y < (unsigned)a.substsz) ? y : 0;
    // left boundary H(r, cb): column 0, or the pass-1 header column of its tile (iT, cb / kExpHB)
    // (element r - iT tBy; rows up to the last tile row's end are computed there, padding included)
    int lb;
    if (cb == 0)
        lb = r * g;
    else
    {
        const int iT = (r - 1) / kSparseTileBy;
        lb = G(d.hcol)[((size_t)iT * (size_t)d.tcols + (size_t)(cb / kExpHB)) * (size_t)(kSparseTileBy + 1) +
                       (size_t)(r - iT * kSparseTileBy)];
    }
    // top row H(r0 - 1, cb .. cb + kExpTW) + g into LDS: row 0, or pass-1 row 64m (shifted values)
    const uint32_t topw = L.top + 4u * (uint32_t)(kTopS * w);
    {
        const int m = (r0 - 1) / kExpRows;
        for (int j = lane; j <= cols + 3; j += 64)  // (+3: the chunks that straddle the tile's end)
        {
            const int c = cb + j;
            const int v = m == 0 ? c * g
                                 : G(d.rows64)[(size_t)(m - 1) * (size_t)d.rpitch + kRowsPad + c] + (kExpRows * m + c) * g;
            lds_st(topw + 4u * (uint32_t)j, v + g);
        }
    }
    const uint32_t qrow = L.q + 4u * (uint32_t)(y * kQS + kQOff);
    const uint32_t hbase = (lane == 0) ? topw : L.gfill;  // lanes >= 1 read a row of g (no branch)
    // lane 63 reaches column cb + cols + 3 at step cols + 66: a chunk that straddles the tile's end is
    // stored whole by this tile's wave, and skipped by the next tile's, whose ramp stores only the
    // chunks that start inside it -- no per-element stores except at the matrix's own edges
    const int ce = min(cols + 3, d.C - cb);                // last column this wave computes validly
    const int NB = (ce + 64 + kBlk - 1) / kBlk;
    // transposed output (as nw_lane.hip): store k has lane 16h + n write columns 4h .. 4h+3 of the
    // block's 16 for row r0 + 16k + n
    const gptr<int> xbase = G(d.score) + (ptrdiff_t)(r0 + (lane & 15)) * d.ld + cb + 4 * (lane >> 4) - (lane & 15);
    const uint32_t xoff = (uint32_t)(lane & 15) * (uint32_t)(d.ld - 1) + 4u * (uint32_t)(lane >> 4);

    int qA[kBlk], qB[kBlk];
#pragma unroll
    for (int u = 0; u < kBlk; ++u) qA[u] = lds_ld(qrow + 4u * (uint32_t)(u - lane));
    int H = lb, U = lb;
#if GSA_EXPAND_PROBE == 2
    int sink = 0;
#endif
    int tE[kBlk];  // the even block's transposed values, stored with the odd block's
    bool held = false;
#pragma unroll
    for (int e = 0; e < kBlk; ++e) tE[e] = 0;

    auto block = [&](int b, int (&qc)[kBlk], int (&qn)[kBlk], auto rampT) {
        constexpr bool RAMP = decltype(rampT)::value;
        int4v hc[kH];
        {
            const uint32_t hb = hbase + (lane == 0 ? 4u * (uint32_t)(kBlk * b) : 0u);
#pragma unroll
            for (int j = 0; j < kH; ++j) hc[j] = lds_ld4(hb + 16u * (lane == 0 ? j : 0));
        }
        // profile of block b+1: columns 16(b+1) - lane .. + 15
#pragma unroll
        for (int u = 0; u < kBlk; ++u) qn[u] = lds_ld(qrow + 4u * (uint32_t)(kBlk * (b + 1) + u - lane));
        int vals[kBlk];
#pragma unroll
        for (int u = 0; u < kBlk; ++u)
        {
            const int up = shr1z(H) + hc[u >> 2][u & 3];
            const int t1 = U + qc[u];
#if GSA_EXPAND_PROBE == 1
            // diagnostic build (tools/r05_xprobe.sh): no recurrence, one add per cell (results wrong)
            int h = t1;
#else
            int h = max(max(t1, up), H + g);
#endif
            if constexpr (RAMP) h = (lane >= kBlk * b + u) ? lb : h;  // column <= cb: the left boundary
            U = up;
            H = h;
            vals[u] = h;
        }
        int t[kBlk];
#pragma unroll
        for (int e = 0; e < kBlk; ++e) t[e] = vals[e];
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int dd = 0; dd < 4; ++dd)
            {
                const auto sw = __builtin_amdgcn_permlane32_swap(t[4 * k + dd], t[4 * (k + 2) + dd], false, false);
                t[4 * k + dd] = sw[0];
                t[4 * (k + 2) + dd] = sw[1];
            }
#pragma unroll
        for (int k = 0; k < 4; k += 2)
#pragma unroll
            for (int dd = 0; dd < 4; ++dd)
            {
                const auto sw = __builtin_amdgcn_permlane16_swap(t[4 * k + dd], t[4 * (k + 1) + dd], false, false);
                t[4 * k + dd] = sw[0];
                t[4 * (k + 1) + dd] = sw[1];
            }
        // interior blocks (uniform): scalar row bases.  An even interior block's stores wait for the
        // odd block after it and the two go out back to back, so each 128-byte line of the pitched
        // layout is written whole at once (unpaired 64-byte halves of ~400k row streams overflow L2)
        auto interior = [&](int bb) { return kBlk * bb - 63 >= 1 && kBlk * bb + kBlk - 1 <= cols && r0 + 63 <= d.R; };
        auto store4 = [&](int bb, int k, const int (&v)[kBlk]) {
            const gptr<int> ub = G(d.score) + ((ptrdiff_t)(r0 + 16 * k) * d.ld - 16 * k + kBlk * bb + cb);
#if GSA_EXPAND_PROBE == 2
            // diagnostic build: interior stores only into one line per wave (results wrong)
            sink ^= v[4 * k] ^ v[4 * k + 1] ^ v[4 * k + 2] ^ v[4 * k + 3];
            (void)ub;
#else
            *(gptr<int4a>)(ub + xoff) = int4a {v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
#endif
        };
        if (!RAMP && (b & 1) == 0 && b + 1 < NB && interior(b) && interior(b + 1))
        {
#pragma unroll
            for (int e = 0; e < kBlk; ++e) tE[e] = t[e];
            held = true;
        }
        else if (held)
        {
#pragma unroll
            for (int k = 0; k < 4; ++k)
            {
                store4(b - 1, k, tE);
                store4(b, k, t);
            }
            held = false;
        }
        else if (interior(b))
        {
#pragma unroll
            for (int k = 0; k < 4; ++k) store4(b, k, t);
        }
        else
#pragma unroll
            for (int k = 0; k < 4; ++k)
            {
                // edge block: a chunk (row r0 + rr, tile columns xc .. xc+3) is this wave's if it starts
                // in the tile; whole (x4) unless it passes the matrix's last column; the first tile also
                // stores the valid part of the chunk that straddles column 1 (no tile before it)
                const int rr = 16 * k + (lane & 15);
                const int xc = kBlk * b - rr + 4 * (lane >> 4);
                if (r0 + rr <= d.R)
                {
                    const gptr<int> p = xbase + (size_t)k * 16u * (size_t)(d.ld - 1) + kBlk * b;
                    if (xc >= 1 && xc <= cols && xc + 3 <= ce)
                        *(gptr<int4a>)p = int4a {t[4 * k], t[4 * k + 1], t[4 * k + 2], t[4 * k + 3]};
                    else if ((xc >= 1 && xc <= cols) || (cb == 0 && xc + 3 >= 1 && xc <= 0))
                    {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (xc + e >= 1 && xc + e <= ce) p[e] = t[4 * k + e];
                    }
                }
            }
    };
    using T = std::integral_constant<bool, true>;
    using F = std::integral_constant<bool, false>;
    int b = 0;
    for (; b < 64 / kBlk; b += 2)
    {
        block(b, qA, qB, T());
        block(b + 1, qB, qA, T());
    }
    for (; b < NB; b += 2)
    {
        block(b, qA, qB, F());
        if (b + 1 < NB) block(b + 1, qB, qA, F());
    }
#if GSA_EXPAND_PROBE == 2
    if (sink == 0x7fffffff) G(d.score)[0] = sink;
#endif
}


// one task: the tile column jT of the `WAVES * kExpRows * a.mt`-row chunk rc of pair d (all threads
// of the workgroup).  ex_prep: subT and the column profile into LDS, the matrix headers the task
// owns -- none of it reads pass-1 output; ex_tiles: a.mt tiles per wave
template <int WAVES>
__device__ __forceinline__ void ex_prep(const ExpandArgs& a, const ExpandPair& d, int tt)
{
    const ExLds L = ex_layout(a.substsz, WAVES);
    const int jT = tt % d.colTiles, rc = tt / d.colTiles;
    const int cb = ex_cb(d, jT), cols = ex_cols(d, jT);
    for (int k = threadIdx.x; k < a.substsz * kSubRow; k += 64 * WAVES)
    {
        const int x = k / kSubRow, yy = k % kSubRow;
        lds_st(L.sub + 4u * k, yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - a.g : 0);
    }
    if (threadIdx.x < 16) lds_st(L.gfill + 4u * threadIdx.x, a.g);
    __syncthreads();
    // column profile of the tile column: Q[y][kQOff + j] = s(y, X[cb + j]) - g, j = 1..kExpTW + 4
    // (the tile and the 3 columns past it, for the chunks that straddle its end; columns past C:
    // letter 0, never stored)
    constexpr int kQCols = kExpTW + 4;
    for (int k = threadIdx.x; k < a.substsz * kQCols; k += 64 * WAVES)
    {
        const int yy = k / kQCols, j = k % kQCols + 1;
        const int c = cb + j;
        int x = c <= d.C ? G(d.seqX)[c] : 0;
        x = ((unsigned)x < (unsigned)a.substsz) ? x : 0;
        lds_st(L.q + 4u * (uint32_t)(yy * kQS + kQOff + j), lds_ld(L.sub + 4u * (uint32_t)(x * kSubRow + yy)));
    }
    __syncthreads();
    // the matrix headers H(i, 0) = i g, H(0, j) = j g: column 0 of the chunk's rows (first tile
    // column), row 0 of the tile's columns (first row chunk)
    const int kChunk = WAVES * kExpRows * a.mt;
    if (cb == 0)
        for (int r = rc * kChunk + 1 + (int)threadIdx.x; r <= min(d.R, rc * kChunk + kChunk); r += 64 * WAVES)
            G(d.score)[(size_t)r * (size_t)d.ld] = r * a.g;
    if (rc == 0)
    {
        for (int c = cb + 1 + (int)threadIdx.x; c <= cb + cols; c += 64 * WAVES) G(d.score)[c] = c * a.g;
        if (cb == 0 && threadIdx.x == 0) G(d.score)[0] = 0;
    }
}

// the tiles of task tt: wave w's are rows 64 (w + WAVES i) of the chunk, i < mt (no barrier between
// them: each wave has its own top-row buffer).  After ex_prep and a barrier.
template <int WAVES>
__device__ __forceinline__ void ex_tiles(const ExpandArgs& a, const ExpandPair& d, int tt, int w, int lane)
{
    const ExLds L = ex_layout(a.substsz, WAVES);
    const int jT = tt % d.colTiles, rc = tt / d.colTiles;
    const int cb = ex_cb(d, jT), cols = ex_cols(d, jT);
    const int kChunk = WAVES * kExpRows * a.mt;
    for (int i = 0; i < a.mt; ++i)
    {
        const int r0 = rc * kChunk + kExpRows * (w + WAVES * i) + 1;
        if (r0 <= d.R && cb < d.C && !(a.knob & 1)) ex_tile(a, d, L, w, lane, cb, cols, r0);
    }
}

template <int WAVES>
__device__ __forceinline__ void ex_task(const ExpandArgs& a, const ExpandPair& d, int tt, int w, int lane)
{
    ex_prep<WAVES>(a, d, tt);
    ex_tiles<WAVES>(a, d, tt, w, lane);
}

// a word of the expansion's LDS that ex_prep / ex_tiles never write (expand_lds_bytes counts it)
__host__ __device__ inline uint32_t ex_word(int substsz, int waves) { return ex_layout(substsz, waves).gfill + 64u; }

}  // namespace xdev
}  // namespace gsa
