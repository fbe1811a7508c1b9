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
#if GSA_EXPAND_PROBE == 8 || GSA_EXPAND_PROBE == 9
// (8: probe 7 and a loader that loads nothing from HBM; 9: probe 7 without the per-task profile
// build and its two barriers; 10: the full tile work with a loader that loads nothing)
#define GSA_EXPAND_PROBE_STORES_ONLY 1
#else
#define GSA_EXPAND_PROBE_STORES_ONLY (GSA_EXPAND_PROBE == 7)
#endif
#ifndef GSA_EXPAND_STORE
#define GSA_EXPAND_STORE 0  // matrix stores: 0 plain, 1 nontemporal, 2 write-through (sc1)
#endif

namespace gsa {
namespace xdev {

constexpr int kBlk = 16;           // steps per block
constexpr int kH = kBlk / 4;       // halo registers (int4) per block
constexpr int kSubRow = 36;        // dwords per subT row (32 letters + 4)
// A wave computes its tile's columns and kExtra more: its 64 rows are stored as a parallelogram,
// row r0 + rr from column cb + 64 - rr to cb + cols + 63 - rr (ex_tile), so that every 128-byte line
// of the pitched layout belongs to one tile and is written whole, by one wave, at once
constexpr int kExtra = 64;
constexpr int kQOff = 64;          // Q[y][kQOff + j], j = 1..kExpTW + kExtra; reads reach j = -63 .. 16 NB + 15
constexpr int kQS = kQOff + kExpTW + kExtra + 96;  // Q row stride (dwords), = 0 mod 32: the bank is the column alone
constexpr int kTopS = kExpTW + kExtra + 80;        // per-wave top row: topw[t] = H(r0 - 1, cb + t) + g, t < 16 NB
static_assert(kQS % 32 == 0 && kTopS % 4 == 0 && kExpTW % kExpHB == 0, "LDS strides");
static_assert(kQOff + 16 * ((kExpTW + kExtra + 79) / 16) + 15 < kQS && 16 * ((kExpTW + kExtra + 79) / 16) <= kTopS,
              "profile and top-row reads stay in their rows");

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
// one 16-byte chunk of the output matrix (GSA_EXPAND_STORE picks the cache policy)
__device__ __forceinline__ void st_out(gptr<int> p, int4a v)
{
#if GSA_EXPAND_STORE == 1
    __builtin_nontemporal_store(v, (gptr<int4a>)p);
#elif GSA_EXPAND_STORE == 2
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"((int4v)v) : "memory");
#else
    *(gptr<int4a>)p = v;
#endif
}
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(xsm + a) = v; }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(xsm + a); }
// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

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

// the tile's recurrence and stores, its inputs in place: y = the lane's row letter, lb = its left
// boundary H(r0 + lane, cb), topw = LDS byte address of its top row (topw[t] = H(r0 - 1, cb + t) + g,
// t <= ce), qbase / gfill the column profile and the row of g
__device__ __forceinline__ void ex_tile_core(const ExpandArgs& a, const ExpandPair& d, uint32_t qbase, uint32_t gfill,
                                             int lane, int cb, int cols, int r0, int y, int lb, uint32_t topw)
{
    const int g = a.g;
    const uint32_t qrow = qbase + 4u * (uint32_t)(y * kQS + kQOff);
    const uint32_t hbase = (lane == 0) ? topw : gfill;  // lanes >= 1 read a row of g (no branch)
    // Row r0 + rr is stored over columns
    // lo(rr) .. hi(rr) (relative to cb): lo = 64 - rr (1 in the first tile column), hi = min(cols + 63
    // - rr, C - cb): the chunks of blocks 4 .. cols / 16 + 3 of every lane, whole aligned lines, the
    // next tile's parallelogram starting where this one ends -- per-element stores only at the
    // matrix's own edges (its first and last columns, rows past R)
    // the last stored element is lane 63's column cols at step cols + 63: later steps (columns past
    // every row's hi) are not computed
#ifdef GSA_EXPAND_FULLNB
    const int NB = (min(cols + kExtra, d.C - cb) + 64 + kBlk - 1) / kBlk;  // (A/B: the round-5 extent)
#else
    const int NB = (cols + 63) / kBlk + 1;
#endif
    const int hiMax = min(cols + 63, d.C - cb);  // hi(0)
    // transposed output (as nw_lane.hip): store k has lane 16h + n write columns 4h .. 4h+3 of the
    // block's 16 for row r0 + 16k + n
    const gptr<int> xbase = G(d.score) + (ptrdiff_t)(r0 + (lane & 15)) * d.ld + cb + 4 * (lane >> 4) - (lane & 15);

    int qA[kBlk], qB[kBlk];
#pragma unroll
    for (int u = 0; u < kBlk; ++u) qA[u] = lds_ld(qrow + 4u * (uint32_t)(u - lane));
    int H = lb, U = lb;
#if GSA_EXPAND_PROBE == 2
    int sink = 0;
#endif
    int tE[kBlk];  // the even block's transposed values, stored with the odd block's
#pragma unroll
    for (int e = 0; e < kBlk; ++e) tE[e] = 0;

    // the block's stores by phase (compile-time): kRamp = the first 4 blocks (columns <= cb for
    // some lanes; stored only in the first tile column), kHold / kPair = an even / odd interior
    // block (the even one's values held and stored with the odd one's, both halves of every
    // 128-byte line back to back), kEdge = the per-lane path
    enum { kRamp, kHold, kPair, kEdge };
    auto block = [&](int b, int (&qc)[kBlk], int (&qn)[kBlk], auto modeT) {
        constexpr int MODE = decltype(modeT)::value;
        constexpr bool RAMP = MODE == kRamp;
        int4v hc[kH];
#if GSA_EXPAND_PROBE == 6 || GSA_EXPAND_PROBE_STORES_ONLY
        // diagnostic build: no LDS reads and no recurrence, the stores alone (7: no transposes either;
        // results wrong)
#pragma unroll
        for (int j = 0; j < kH; ++j) hc[j] = int4v {b, j, 1, 2};
#pragma unroll
        for (int u = 0; u < kBlk; ++u) qn[u] = u + b;
#else
        {
            const uint32_t hb = hbase + (lane == 0 ? 4u * (uint32_t)(kBlk * b) : 0u);
#pragma unroll
            for (int j = 0; j < kH; ++j) hc[j] = lds_ld4(hb + 16u * (lane == 0 ? j : 0));
        }
        // profile of block b+1: columns 16(b+1) - lane .. + 15
#pragma unroll
        for (int u = 0; u < kBlk; ++u) qn[u] = lds_ld(qrow + 4u * (uint32_t)(kBlk * (b + 1) + u - lane));
#endif
        int vals[kBlk];
#pragma unroll
        for (int u = 0; u < kBlk; ++u)
        {
            const int up = shr1z(H) + hc[u >> 2][u & 3];
            const int t1 = U + qc[u];
#if GSA_EXPAND_PROBE == 1 || GSA_EXPAND_PROBE == 6 || GSA_EXPAND_PROBE_STORES_ONLY
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
        // the per-block transposed shape (ramp and edge blocks): store k has lane 16h + n write
        // columns 4h .. 4h+3 of the block's 16 for row r0 + 16k + n -- lane bits 5, 4 swapped with
        // the chunk index
        auto xpose16 = [&]() {
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
        };
        if constexpr (MODE == kHold)
        {
            // the even block's values, untransposed: stored with the odd block's
#pragma unroll
            for (int e = 0; e < kBlk; ++e) tE[e] = t[e];
        }
        else if constexpr (MODE == kPair)
        {
            // whole 128-byte lines per instruction, each lane quad 64 contiguous bytes: store k
            // (0..7) writes rows rr = 32 (k >> 2) + 4m + (k & 3), m = 0..7, lane 4m + q (+ 32 for the
            // line's second half) columns 4c .. 4c+3 of the pair's 32, chunk c = q + 4 (lane >> 5).  A
            // CU writes 96 GB/s in this shape against 33 in the transposed 16-row x 64-B one (a quad
            // covering 4 rows: tools/ubench/store_ubench4.hip, profiles/r06_store_shape.txt).  Chunk c
            // of the lane's own row: c < 4 the even block's (tE), c >= 4 the odd one's; lane bit 5
            // swaps with chunk bit 2 (permlane32 swaps), lane bits 1 and 0 with chunk bits 1 and 0
            // (quad permutes)
            int A[8][4];
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int dd = 0; dd < 4; ++dd)
                {
                    A[c][dd] = tE[4 * c + dd];
                    A[c + 4][dd] = t[4 * c + dd];
                }
#if !GSA_EXPAND_PROBE_STORES_ONLY && GSA_EXPAND_PROBE != 11  // (11: full tile work, no transposes; results wrong)
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int dd = 0; dd < 4; ++dd)
                {
                    const auto sw = __builtin_amdgcn_permlane32_swap(A[c][dd], A[c + 4][dd], false, false);
                    A[c][dd] = sw[0];
                    A[c + 4][dd] = sw[1];
                }
            // lane bit m (1, then 0) with chunk bit m, per pair of chunks (x: bit m clear, y: set): a
            // lane with lane bit m clear keeps its x and takes its quad partner's x as y, the others
            // keep y and take the partner's y as x -- one v_cndmask_b32 per output, its first operand
            // read across the quad (DPP).  (s_nop 1: the DPP operand may have been written by the
            // instruction before the block.)
            const uint64_t lo1 = 0x3333333333333333ull, lo0 = 0x5555555555555555ull;
            auto qswap = [&](auto mT) {
                constexpr int m = decltype(mT)::value;
                const uint64_t mlo = m ? lo1 : lo0, mhi = ~mlo;
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    if (((c >> m) & 1) == 0)
                    {
                        int* x = A[c];
                        int* y = A[c | (1 << m)];
                        int nx0, nx1, nx2, nx3, ny0, ny1, ny2, ny3;
#define GSA_QSWAP(QP)                                                                                              \
    asm volatile("s_nop 1\n"                                                                                       \
                 "s_mov_b64 vcc, %16\n"                                                                            \
                 "v_cndmask_b32_dpp %0, %12, %8, vcc " QP " row_mask:0xf bank_mask:0xf\n"                          \
                 "v_cndmask_b32_dpp %1, %13, %9, vcc " QP " row_mask:0xf bank_mask:0xf\n"                          \
                 "v_cndmask_b32_dpp %2, %14, %10, vcc " QP " row_mask:0xf bank_mask:0xf\n"                         \
                 "v_cndmask_b32_dpp %3, %15, %11, vcc " QP " row_mask:0xf bank_mask:0xf\n"                         \
                 "s_mov_b64 vcc, %17\n"                                                                            \
                 "v_cndmask_b32_dpp %4, %8, %12, vcc " QP " row_mask:0xf bank_mask:0xf\n"                          \
                 "v_cndmask_b32_dpp %5, %9, %13, vcc " QP " row_mask:0xf bank_mask:0xf\n"                          \
                 "v_cndmask_b32_dpp %6, %10, %14, vcc " QP " row_mask:0xf bank_mask:0xf\n"                         \
                 "v_cndmask_b32_dpp %7, %11, %15, vcc " QP " row_mask:0xf bank_mask:0xf"                            \
                 : "=&v"(nx0), "=&v"(nx1), "=&v"(nx2), "=&v"(nx3), "=&v"(ny0), "=&v"(ny1), "=&v"(ny2), "=&v"(ny3)    \
                 : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(y[0]), "v"(y[1]), "v"(y[2]), "v"(y[3]), "s"(mlo), \
                   "s"(mhi)                                                                                        \
                 : "vcc")
                        if constexpr (m == 1)
                            GSA_QSWAP("quad_perm:[2,3,0,1]");
                        else
                            GSA_QSWAP("quad_perm:[1,0,3,2]");
#undef GSA_QSWAP
                        x[0] = nx0, x[1] = nx1, x[2] = nx2, x[3] = nx3;
                        y[0] = ny0, y[1] = ny1, y[2] = ny2, y[3] = ny3;
                    }
            };
            qswap(std::integral_constant<int, 1>());
            qswap(std::integral_constant<int, 0>());
#endif
            const uint32_t xoffQ = (uint32_t)(4 * ((lane >> 2) & 7)) * (uint32_t)(d.ld - 1) +
                                   4u * (uint32_t)((lane & 3) | ((lane >> 5) << 2));
#pragma unroll
            for (int k = 0; k < 8; ++k)
            {
                const int rk = 32 * (k >> 2) + (k & 3);
                const gptr<int> ub = G(d.score) + ((ptrdiff_t)(r0 + rk) * d.ld - rk + kBlk * (b - 1) + cb);
#if GSA_EXPAND_PROBE == 2
                sink ^= A[k][0] ^ A[k][1] ^ A[k][2] ^ A[k][3];
                (void)ub;
#else
                st_out(ub + xoffQ, int4a {A[k][0], A[k][1], A[k][2], A[k][3]});
#endif
            }
        }
        else if ((MODE == kEdge || cb == 0) && kBlk * b - 63 <= hiMax)
        {
#if !GSA_EXPAND_PROBE_STORES_ONLY
            xpose16();
#endif
#pragma unroll
            for (int k = 0; k < 4; ++k)
            {
                // edge block: the chunk (row r0 + rr, columns xc .. xc+3) is stored where it lies in
                // lo(rr) .. hi(rr): whole, except where the matrix's first or last column cuts it
                const int rr = 16 * k + (lane & 15);
                const int xc = kBlk * b - rr + 4 * (lane >> 4);
                const int lo = cb == 0 ? 1 : 64 - rr, hi = min(cols + 63 - rr, d.C - cb);
                if (r0 + rr <= d.R)
                {
                    const gptr<int> p = xbase + (size_t)k * 16u * (size_t)(d.ld - 1) + kBlk * b;
                    if (xc >= lo && xc + 3 <= hi)
                        st_out(p, int4a {t[4 * k], t[4 * k + 1], t[4 * k + 2], t[4 * k + 3]});
                    else if (xc + 3 >= lo && xc <= hi)
                    {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (xc + e >= lo && xc + e <= hi) p[e] = t[4 * k + e];
                    }
                }
            }
        }
    };
    using MR = std::integral_constant<int, kRamp>;
    using MH = std::integral_constant<int, kHold>;
    using MP = std::integral_constant<int, kPair>;
    using ME = std::integral_constant<int, kEdge>;
    int b = 0;
    for (; b < 64 / kBlk; b += 2)
    {
        block(b, qA, qB, MR());
        block(b + 1, qB, qA, MR());
    }
    // interior blocks (uniform): every lane's chunks inside its row's range, every row <= R
    // (blocks 4 .. (hiMax - 15) / 16); in pairs
    const int bInt = r0 + 63 <= d.R ? (hiMax - (kBlk - 1)) / kBlk : 3;  // last interior block
    for (; b + 1 <= bInt; b += 2)
    {
        block(b, qA, qB, MH());
        block(b + 1, qB, qA, MP());
    }
    for (; b < NB; b += 2)
    {
        block(b, qA, qB, ME());
        if (b + 1 < NB) block(b + 1, qB, qA, ME());
    }
#if GSA_EXPAND_PROBE == 2
    if (sink == 0x7fffffff) G(d.score)[0] = sink;
#endif
}


// ------------------------------------------------------------------------------------
// The streamed expansion (round 6).  A task's inputs -- its column letters and, for each tile wave,
// its 64 row letters, left boundary column and top row -- are global loads, and a wave's global load
// waits for every store that wave issued before it (vmcnt retires in order).  A tile wave that
// fetched its next task's inputs itself drained its whole store queue first, so each CU's store
// stream stopped at every task: at 100k x 100k the fused fill's workgroups spent 25-33 % of the
// expansion between tasks (profiles/r06_fused100k.txt).  Here a workgroup of W waves has W - 1
// tile waves and one loader wave: the loader claims tasks, (FUSED) waits until pass 1 has written
// their rows, and stages their inputs in one of two LDS slots; the tile waves build the task's
// column profile from the slot (LDS only), compute and store -- they never load from global memory
// and never wait for their stores.  A task is (W - 1) x 64 rows of one tile column.
// ------------------------------------------------------------------------------------
constexpr int kSlotHdr = 32;             // dwords: task (-1: no more), pair, tt, then the ExpandPair
constexpr int kSlotX = kExpTW + kExtra;  // letters of columns cb + 1 .. cb + kExpTW + kExtra
constexpr int kTileDw = 2 * kExpRows + kTopS;  // per tile wave: y[64], lb[64], top row[kTopS]
static_assert(sizeof(ExpandPair) % 4 == 0 && 3 + (int)(sizeof(ExpandPair) / 4) <= kSlotHdr, "slot header");

struct ExLdsS
{
    uint32_t q, sub, gfill, ctl, slot, slotB;
};
// profile Q, subT (kept for the launch), the row of g, control words, two task slots
__host__ __device__ inline ExLdsS ex_layout_s(int substsz, int nw)
{
    ExLdsS L;
    L.q = 0;
    L.sub = (uint32_t)substsz * kQS * 4u;
    L.gfill = L.sub + (((uint32_t)substsz * kSubRow * 4u + 15u) & ~15u);
    L.ctl = L.gfill + 64u;
    L.slot = L.ctl + 64u;
    L.slotB = ((uint32_t)(kSlotHdr + kSlotX + nw * kTileDw) * 4u + 15u) & ~15u;
    return L;
}
// task slots: as many as the CU's 160 KB of LDS holds, up to kMaxSlots -- the loader runs that many
// tasks ahead of the tile waves, and its loads wait behind the CU's own store stream (the vector
// memory path is shared), so one task of lead starved the tile waves at 100k
constexpr int kMaxSlots = 4;
constexpr uint32_t kLdsBudget = 160u * 1024u;
__host__ __device__ inline int ex_nslot(int substsz, int nw)
{
    const ExLdsS L = ex_layout_s(substsz, nw);
    const int n = L.slot + 2u * L.slotB > kLdsBudget ? 2 : (int)((kLdsBudget - L.slot) / L.slotB);
    return n < 2 ? 2 : n > kMaxSlots ? kMaxSlots : n;
}
__host__ __device__ inline uint32_t ex_stream_lds(int substsz, int nw)
{
    const ExLdsS L = ex_layout_s(substsz, nw);
    return L.slot + (uint32_t)ex_nslot(substsz, nw) * L.slotB;
}

// LDS words shared by the waves: relaxed workgroup-scope atomics (a single wave's LDS operations
// execute in order, so a word written after the data it publishes is never seen before it)
__device__ __forceinline__ int xs_ld(uint32_t a)
{
    return __builtin_amdgcn_readfirstlane(
        __hip_atomic_load((int*)__builtin_assume_aligned(xsm + a, 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void xs_st(uint32_t a, int v)
{
    asm volatile("" ::: "memory");
    __hip_atomic_store((int*)__builtin_assume_aligned(xsm + a, 4), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ void xs_add(uint32_t a, int v)
{
    asm volatile("" ::: "memory");
    __hip_atomic_fetch_add((int*)__builtin_assume_aligned(xsm + a, 4), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    asm volatile("" ::: "memory");
}
// wait until the LDS word reaches v; false (error word set) after a.spin ticks without it, or when
// another wave has set the error word (a global load: looked at every 256th idle pass only)
__device__ __forceinline__ bool xs_wait(const ExpandArgs& a, uint32_t w, int v)
{
    if (xs_ld(w) >= v) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (unsigned n = 1;; ++n)
    {
        __builtin_amdgcn_s_sleep(1);
        if (xs_ld(w) >= v) return true;
        if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin ||
            ((n & 255) == 0 && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0))
        {
            atomicOr(a.err, 1u);
            return false;
        }
    }
}

__device__ __forceinline__ ExpandPair ex_desc_lds(uint32_t a)
{
    constexpr int N = sizeof(ExpandPair) / 4;
    union
    {
        int v[N];
        ExpandPair d;
    } u;
#pragma unroll
    for (int k = 0; k < N; ++k) u.v[k] = __builtin_amdgcn_readfirstlane(lds_ld(a + 4u * k));
    return u.d;
}

// FUSED: the pass-1 strips' progress words (nw_krow.hip kr_strip, PT 3) and this launch's epoch;
// tstamps: per task [claimed, ready, done] (GSA_STAMPS) or null
struct ExFused
{
    const unsigned long long* xdone;
    unsigned epoch;
    unsigned long long* tstamps;
};

// All W waves of the workgroup (after a barrier: the LDS is reused).  counter: the task claims.
template <int W, bool FUSED>
__device__ __forceinline__ void ex_stream(const ExpandArgs& a, unsigned* counter, const ExFused& f, int w, int lane)
{
    constexpr int NW = W - 1;
    const ExLdsS L = ex_layout_s(a.substsz, NW);
    const int NS = ex_nslot(a.substsz, NW);
    const uint32_t RDY = L.ctl, DONE = L.ctl + 4u * kMaxSlots, BAR = L.ctl + 8u * kMaxSlots;
    for (int k = threadIdx.x; k < a.substsz * kSubRow; k += 64 * W)
    {
        const int x = k / kSubRow, yy = k % kSubRow;
        lds_st(L.sub + 4u * k, yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - a.g : 0);
    }
    if (threadIdx.x < 16)
    {
        lds_st(L.gfill + 4u * threadIdx.x, a.g);
        lds_st(L.ctl + 4u * threadIdx.x, 0);
    }
    __syncthreads();
    if (w == NW)
    {
        // ---- the loader wave ----
        // claims runs of a.run schedule entries (one tile column: the tile waves keep its profile).
        // Its global accesses are round trips that queue behind the CU's own store stream --
        // microseconds each under the full fill, and a loader that made six per task (claim,
        // schedule entry, pair descriptor, one readiness word after the other, inputs) supplied a
        // task every ~37 us, the expansion's whole rate per CU.  So a run's claim is made one run
        // ahead and its schedule entries come in one load, the pair's descriptor is kept while the
        // pair stays, and a task's readiness words are read together: per task one readiness read
        // and one input load.
        int runBase = 0, runLeft = 0, runPos = 0;
        int sv = 0;  // the run's schedule entries: lanes 2i, 2i + 1 = {pair, task} of entry i
        int curLo = -1;
        ExpandPair d {};
        unsigned nextV = 0;  // (lane 0) the next run's claim, in flight
        if (lane == 0) nextV = atomicAdd(counter, 1u);
        for (int k = 0;; ++k)
        {
            const int s = k % NS, gen = k / NS + 1;
            const uint32_t slot = L.slot + (uint32_t)s * L.slotB;
            // the slot's previous task is done with it
            bool ok = k < NS || xs_wait(a, DONE + 4u * s, NW * (gen - 1));
            int task = a.nTasks, lo = -1, tt = 0;
            while (ok && lo < 0)
            {
                if (runLeft == 0)
                {
                    const unsigned t = (unsigned)__builtin_amdgcn_readfirstlane((int)nextV) * (unsigned)a.run;
                    runBase = (int)min(t, (unsigned)a.nTasks);
                    runLeft = runBase < a.nTasks ? min(a.run, a.nTasks - runBase) : 0;
                    if (runLeft == 0) break;  // no more runs
                    sv = lane < 2 * runLeft ? G(a.sched)[2 * runBase + lane] : -1;
                    if (lane == 0) nextV = atomicAdd(counter, 1u);
                    runPos = 0;
                }
                task = runBase + runPos;
                lo = __builtin_amdgcn_readlane(sv, 2 * runPos);
                tt = __builtin_amdgcn_readlane(sv, 2 * runPos + 1);
                ++runPos;
                --runLeft;
            }
            if (lo < 0) task = a.nTasks;
            int jT = 0, rc = 0, cb = 0, cols = 0;
            if (task < a.nTasks)
            {
                if (lo != curLo)
                {
                    d = ex_desc(a.pairs + lo);
                    curLo = lo;
                }
                jT = tt % d.colTiles;
                rc = tt / d.colTiles;
                cb = ex_cb(d, jT);
                cols = ex_cols(d, jT);
                if constexpr (FUSED)
                {
                    // pass 1 has stored rows 64m, m = NW rc .. NW rc + NW - 1, at the columns the
                    // tiles read, and the header column cb for their rows: the words of strips
                    // (NW rc - 1) / 4 .. (NW (rc + 1) - 1) / 4 (256 rows each) reach `need`; lane i
                    // reads strip s0 + i's
                    unsigned long long* ts = f.tstamps ? f.tstamps + 3 * (size_t)task : nullptr;
                    if (ts && lane == 0) ts[0] = __builtin_amdgcn_s_memrealtime();
                    const unsigned need = (unsigned)(min(cb + cols + kExtra, d.C) + 1);
                    const int s0 = rc > 0 ? (NW * rc - 1) / 4 : 0;
                    const int nWords = min((NW * (rc + 1) - 1) / 4, d.p1Strips - 1) - s0 + 1;
                    const unsigned long long* words = f.xdone + d.p1Strip0 + s0;
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    for (unsigned it = 1;; ++it)
                    {
                        bool rdy = true;
                        if (lane < nWords)
                        {
                            const unsigned long long v = __hip_atomic_load(words + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            rdy = (unsigned)(v >> 32) == f.epoch && (unsigned)v >= need;
                        }
                        if (__builtin_amdgcn_ballot_w64(!rdy) == 0) break;
                        __builtin_amdgcn_s_sleep(2);
                        if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin ||
                            ((it & 15) == 0 && __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0))
                        {
                            if (lane == 0) atomicOr(a.err, 1u);
                            ok = false;
                            break;
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    if (ts && lane == 0) ts[1] = __builtin_amdgcn_s_memrealtime();
                }
            }
            if (!ok || task >= a.nTasks)
            {
                // no more tasks (or an error): the tile waves stop at this slot
                if (lane == 0) lds_st(slot, -1);
                xs_st(RDY + 4u * s, gen);
                return;
            }
            // Every input of the task in one round trip: all loads issued (<= 44 per lane, within the
            // 63 that vmcnt tracks) before the first LDS write.  Under the chip's store stream a load
            // takes microseconds, and a loader that waited tile by tile fell behind the tile waves.
            const int ce = min(cols + kExtra, d.C - cb);
            constexpr int kXIt = (kSlotX + 63) / 64;
            constexpr int kTIt = (kExpTW + kExtra + 1 + 255) / 256;  // top-row dwordx4 loads per tile
            int xv[kXIt], yv[NW], lbv[NW];
            int4v tv[NW][kTIt];
#pragma unroll
            for (int i = 0; i < kXIt; ++i)
            {
                const int j = lane + 64 * i, c = cb + 1 + j;
                xv[i] = (GSA_EXPAND_PROBE != 8 && GSA_EXPAND_PROBE != 10 && j < kSlotX && c <= d.C) ? G(d.seqX)[c] : 0;
            }
#pragma unroll
            for (int i = 0; i < NW; ++i)
            {
                const int r0 = rc * NW * kExpRows + kExpRows * i + 1;
                const int r = r0 + lane;
                yv[i] = (GSA_EXPAND_PROBE != 8 && GSA_EXPAND_PROBE != 10 && r <= d.R) ? G(d.seqY)[r] : 0;
                if (cb == 0 || r0 > d.R || GSA_EXPAND_PROBE == 8 || GSA_EXPAND_PROBE == 10)
                    lbv[i] = r * a.g;
                else
                {
                    // (element r - iT tBy of the pass-1 header column; rows up to the last tile row's
                    // end are computed there, padding included)
                    const int iT = (r - 1) / kSparseTileBy;
                    lbv[i] = G(d.hcol)[((size_t)iT * (size_t)d.tcols + (size_t)(cb / kExpHB)) * (size_t)(kSparseTileBy + 1) +
                                       (size_t)(r - iT * kSparseTileBy)];
                }
                // the top row, pass-1 row 64m (m >= 1), 4 columns per lane per load: cb and the row
                // buffer's pitch and pad are multiples of 16 ints, and the chunk that passes ce stays
                // in the row's right pad (columns up to Cp + 63)
                const int m = (r0 - 1) / kExpRows;
                const gptr<const int4v> rowp =
                    (gptr<const int4v>)(G(d.rows64) + (size_t)(m > 0 ? m - 1 : 0) * (size_t)d.rpitch + kRowsPad + cb);
#pragma unroll
                for (int q = 0; q < kTIt; ++q)
                {
                    const int j = 4 * lane + 256 * q;
                    tv[i][q] = (GSA_EXPAND_PROBE == 8 || GSA_EXPAND_PROBE == 10 || m == 0 || r0 > d.R || j > ce) ? int4v {0, 0, 0, 0} : rowp[lane + 64 * q];
                }
            }
#pragma unroll
            for (int i = 0; i < kXIt; ++i)
                if (lane + 64 * i < kSlotX)
                    lds_st(slot + 4u * (uint32_t)(kSlotHdr + lane + 64 * i), ((unsigned)xv[i] < (unsigned)a.substsz) ? xv[i] : 0);
#pragma unroll
            for (int i = 0; i < NW; ++i)
            {
                const int r0 = rc * NW * kExpRows + kExpRows * i + 1;
                if (r0 > d.R) break;
                const uint32_t tb = slot + 4u * (uint32_t)(kSlotHdr + kSlotX + i * kTileDw);
                lds_st(tb + 4u * (uint32_t)lane, ((unsigned)yv[i] < (unsigned)a.substsz) ? yv[i] : 0);
                lds_st(tb + 4u * (uint32_t)(kExpRows + lane), lbv[i]);
                const int m = (r0 - 1) / kExpRows;
#pragma unroll
                for (int q = 0; q < kTIt; ++q)
                {
                    const int j = 4 * lane + 256 * q;
                    if (j <= ce)
                    {
                        int4v o;
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                        {
                            const int c = cb + j + e;
                            o[e] = (m == 0 ? c * a.g : tv[i][q][e] + (kExpRows * m + c) * a.g) + a.g;
                        }
                        *(int4v*)(xsm + tb + 4u * (uint32_t)(2 * kExpRows + j)) = o;
                    }
                }
            }
            {
                constexpr int N = sizeof(ExpandPair) / 4;
                const int* dw = (const int*)&d;
                int dv = 0;
#pragma unroll
                for (int q = 0; q < N; ++q)
                    if (lane == q) dv = dw[q];
                if (lane < N) lds_st(slot + 4u * (uint32_t)(3 + lane), dv);
                if (lane == 0)
                {
                    lds_st(slot, task);
                    lds_st(slot + 4u, lo);
                    lds_st(slot + 8u, tt);
                }
            }
            xs_st(RDY + 4u * s, gen);
        }
    }
    // ---- tile waves ----
    const int tid = w * 64 + lane;
    int barGen = 0;
    int qPair = -1, qCol = -1;  // the pair and tile column the profile in LDS belongs to
    auto bar = [&]() {
        ++barGen;
        if (lane == 0) xs_add(BAR, 1);
        return xs_wait(a, BAR, NW * barGen);
    };
    for (int k = 0;; ++k)
    {
        const int s = k % NS, gen = k / NS + 1;
        const uint32_t slot = L.slot + (uint32_t)s * L.slotB;
        if (!xs_wait(a, RDY + 4u * s, gen)) return;
        const int task = xs_ld(slot);
        if (task < 0) return;
        const int pr = xs_ld(slot + 4u), tt = xs_ld(slot + 8u);
        const ExpandPair d = ex_desc_lds(slot + 12u);
        const int jT = tt % d.colTiles, rc = tt / d.colTiles;
        const int cb = ex_cb(d, jT), cols = ex_cols(d, jT);
        // the profile of the previous task's tile column serves this one too: no rebuild
        const bool same = pr == qPair && jT == qCol;
        qPair = pr;
        qCol = jT;
        // the profile is free once every tile wave is done with the previous task
#if GSA_EXPAND_PROBE != 9
        if (!same)
        {
        if (!bar()) return;
        for (int j = tid + 1; j <= kSlotX; j += NW * 64)
        {
            // subT row x, 4 letters per read (rows are 36 dwords: 16-byte aligned)
            const int x = lds_ld(slot + 4u * (uint32_t)(kSlotHdr + j - 1));
            int4v sv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                if (4 * i < a.substsz) sv[i] = lds_ld4(L.sub + 4u * (uint32_t)(x * kSubRow + 4 * i));
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    if (4 * i + e < a.substsz) lds_st(L.q + 4u * (uint32_t)((4 * i + e) * kQS + kQOff + j), sv[i][e]);
        }
        if (!bar()) return;
        }
#endif
        // the matrix headers H(i, 0) = i g, H(0, j) = j g the task owns
        const int kChunk = NW * kExpRows;
        if (cb == 0)
            for (int r = rc * kChunk + 1 + tid; r <= min(d.R, rc * kChunk + kChunk); r += NW * 64)
                G(d.score)[(size_t)r * (size_t)d.ld] = r * a.g;
        if (rc == 0)
        {
            for (int c = cb + 1 + tid; c <= cb + cols; c += NW * 64) G(d.score)[c] = c * a.g;
            if (cb == 0 && tid == 0) G(d.score)[0] = 0;
        }
        const int r0 = rc * kChunk + kExpRows * w + 1;
        if (r0 <= d.R && cb < d.C)
        {
            const uint32_t tb = slot + 4u * (uint32_t)(kSlotHdr + kSlotX + w * kTileDw);
            ex_tile_core(a, d, L.q, L.gfill, lane, cb, cols, r0, lds_ld(tb + 4u * (uint32_t)lane),
                         lds_ld(tb + 4u * (uint32_t)(kExpRows + lane)), tb + 4u * (uint32_t)(2 * kExpRows));
        }
        if (FUSED && f.tstamps && w == 0 && lane == 0) f.tstamps[3 * (size_t)task + 2] = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) xs_add(DONE + 4u * s, 1);
    }
}

}  // namespace xdev
}  // namespace gsa
