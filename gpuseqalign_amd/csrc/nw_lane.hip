// nw_lane.hip -- NW-LG full-matrix fill with ONE row per lane ("lane strips"), hand-written
// wave64 HIP for gfx950 (MI355X).
//
// Replaces the plain fill family NwAlign_Gpu3..6 (nwalign_gpu3_ml_diagdiag.cu:288-596, the
// per-diagonal kernels :11-287) and has their output contract: nw.score, the (R+1) x (C+1)
// int32 matrix, row-major, unpadded.  Recurrence of UpdateScore (nwalign_cpu1_st_row.cpp:4-10).
//
// Why one row per lane.  A single pair is bounded by its wavefront's critical path,
// (C + nStrips * hop) * t_step, not by HBM: with K rows per lane a step costs ~(a + b*K) cycles
// and the hop is >= 64 steps (the lane skew) per 64*K rows.  The 4-row strips of nw_strip.hip
// run ~200 cycles/step on full fills; one row per lane runs ~25-40 (tools/ubench/k1_ubench.hip),
// which more than pays for 4x the strips.
//
// Step (unshifted values, gap folded into the operands, 4 VALU per cell):
//     up' = dpp_shr1(H) + hv          hv = g; lane 0: H(row above, c) + g         v_add_u32_dpp
//     t1  = U + q                     U = up' of the previous step, q = s(y, X[c]) - g
//     H   = max3(t1, up', H + g)      = max3(H[i-1][j-1]+s, H[i-1][j]+g, H[i][j-1]+g)
//     U   = up'
// Lane l owns row r0 + l and at step t works on column t - l.  Columns <= 0 (the first 64
// steps) are forced to the border r*g.
//
// Substitution scores come from a per-workgroup COLUMN profile Q[y][c] = s(y, X[c]) - g
// (int32, a ring of kLW = 512 or 1024 columns, rows kLW + 32 dwords apart): lane l reads Q[y_l][t-l],
// bank (t - l) mod 32 whatever the row letters (conflict-free), at base + immediate offsets,
// so a step spends no VALU on addressing.  The loader wave builds Q from seqX and the table.
//
// Hand-off: lane 63 of strip w writes its (H + g) values (the "left" operand it computes anyway)
// into ring w+1, element e = column e - 64; lane 0 of strip w+1 reads them 8 at a time, one
// block ahead.  Order is kept with LDS progress words (LDS ops of one wave execute in order).
// Between super-strips (workgroups) the loader moves the last strip's row through 8-byte
// {epoch, H+g} granules in HBM, as nw_strip.hip does.  The strips store their own output: per
// 16-step block the lane's 16 values are transposed across lane bits 5 and 4 (16 permlane32/16
// swaps) so each of the 4 dwordx4 stores writes 16 rows x 64 contiguous bytes.  One row per lane
// per store cost a memory request per lane; with 3-4 strips per CU those requests slowed every
// strip and the granule polls queued behind them (profiles/r01_xpose_probe.txt).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "nw_lane.h"

namespace gsa {
namespace {

// Q ring columns (power of 2).  The ring spans the first strip's frontier back to the last
// strip's oldest column, ~(NS - 1) hops of ~100 columns + the lane skew: 1024 from NS = 5 on.
__host__ __device__ constexpr int lane_lw(int ns) { return ns >= 5 ? 1024 : 512; }
__host__ __device__ constexpr int lane_qrs(int ns) { return lane_lw(ns) + 32; }  // Q row stride in dwords: == 0 mod 32, 32 guard columns
constexpr int kLRing = 512;        // hand-off ring elements per strip boundary (power of 2)
constexpr int kLBlk = 16;          // steps per block
constexpr int kLH = kLBlk / 4;     // halo registers (int4) per block
constexpr int kLBig = 0x3fffffff;  // "everything published"
// Variants measured and not kept (round 1, profiles/): lane-63-only halo reads and hand-off
// writes behind an exec mask (slower by 10-15 cycles/step), the halo prefetched a block ahead
// (one more block of lag per hop), output staged in LDS (114 vs 78 cycles/step), one row per
// lane per store (the CU's requests delay the granule polls), buffer stores (1-4 % slower),
// 8-step blocks.

extern __shared__ __attribute__((aligned(16))) char lsm[];


typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(lsm + a); }
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(lsm + a) = v; }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(lsm + a); }
__device__ __forceinline__ void lds_st4(uint32_t a, int4v v) { *(int4v*)(lsm + a) = v; }
// progress words: relaxed workgroup-scope atomics (no waits; see nw_strip.hip)
__device__ __forceinline__ int raw_ld(uint32_t a)
{
    return __hip_atomic_load((int*)__builtin_assume_aligned(lsm + a, 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int flag_ld(uint32_t a) { return __builtin_amdgcn_readfirstlane(raw_ld(a)); }
__device__ __forceinline__ void flag_st(uint32_t a, int v)
{
    asm volatile("" ::: "memory");  // data writes are issued before the word (LDS executes in order)
    __hip_atomic_store((int*)__builtin_assume_aligned(lsm + a, 4), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool err_set(const StripArgs& a)
{
    return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

// LDS: Q profile, transposed substitution table subT[x][y] = s(y, x) - g (rows of kLSubRow
// dwords, so one lane gathers 4 row letters per ds_read_b128), NS+1 hand-off rings, progress words.
// flags: prog[i] @ 4i (ring i holds elements < prog[i]), cons[i] @ 64+4i (ring i's reader no
// longer needs elements < cons[i]), xo @ 128 (Q holds columns < xo), ticket @ 132.
struct LaneLds
{
    uint32_t q, sub, ring, gfill, sink, flags;
};
constexpr uint32_t kFCons = 64, kFXo = 128, kFTicket = 132;  // prog/cons: NS + 1 <= 16 words each
constexpr int kLSubRow = 36;  // dwords per subT row: 32 letters + 4 (16-byte aligned rows)

__host__ __device__ inline LaneLds lane_layout(int ns, int substsz)
{
    LaneLds L;
    L.q = 0;
    L.sub = (uint32_t)substsz * lane_qrs(ns) * 4u;
    L.ring = L.sub + (uint32_t)substsz * kLSubRow * 4u;
    L.gfill = L.ring + (uint32_t)(ns + 1) * kLRing * 4u;  // 16 x g: the "halo" of lanes >= 1
    L.sink = L.gfill + 64u;                                // lanes 0..62's hand-off writes
    L.flags = L.sink + (uint32_t)ns * 1024u;
    return L;
}

// ------------------------------------------------------------------------------------
// strip wave: 64 rows, one per lane
// ------------------------------------------------------------------------------------
template <int NS, bool PAIR>
__device__ __forceinline__ void lane_strip(const StripArgs& a, const LaneLds& L, int tk, int w, int lane)
{
    const int g = a.g;
    const int C = a.C;
    const int r0 = tk * (kLaneRows * NS) + kLaneRows * w + 1;  // first row of the strip
    const int r = r0 + lane;                                   // this lane's row
    const bool live = r <= a.R;
    int y = live ? G(a.seqY)[r] : 0;
    y = ((unsigned)y < (unsigned)a.substsz) ? y : 0;
    constexpr int kLW = lane_lw(NS), kLQRS = lane_qrs(NS);
    const uint32_t qrow = L.q + (uint32_t)y * (kLQRS * 4u);
    const uint32_t ring_in = L.ring + (uint32_t)w * (kLRing * 4u);
    const uint32_t ring_out = L.ring + (uint32_t)(w + 1) * (kLRing * 4u);
    const uint32_t f_in = L.flags + 4u * w, f_out = L.flags + 4u * (w + 1);
    const uint32_t c_in = L.flags + kFCons + 4u * w, c_out = L.flags + kFCons + 4u * (w + 1);
    const uint32_t f_xo = L.flags + kFXo;
    const uint32_t hsink = L.sink + (uint32_t)w * 1024u + 16u * (uint32_t)lane;
    const int NB = (C + 65 + kLBlk - 1) / kLBlk;  // lane 63 reaches step C+64 (element of column C)
    const int rg = r * g;
    // transposed output: column 16b of row r0 + (lane & 15), shifted by the lane's chunk
    // 4 * (lane >> 4) and the row's skew; + 16k(ld-1) for row r0 + 16k + (lane & 15)
    const gptr<int> xbase = G(a.score) + (ptrdiff_t)(r0 + (lane & 15)) * a.ld + 4 * (lane >> 4) - (lane & 15);
    const uint32_t xoff = (uint32_t)(lane & 15) * (uint32_t)(a.ld - 1) + 4u * (uint32_t)(lane >> 4);  // from row r0 + 16k

    // block b prefetches block b+1's inputs (ring elements < B(b+1)+64+B, Q columns < B(b+1)+B,
    // B = kLBlk) and writes ring elements Bb .. Bb+B-1
    auto ok = [&](int pin, int pco, int pxo, int b) {
        return pin >= kLBlk * b + 64 + kLBlk && pco >= kLBlk * b + kLBlk - kLRing && (w != 0 || pxo >= kLBlk * b + 2 * kLBlk);
    };
    // bounded spin; the error word is a global load, which waits for this wave's outstanding
    // output stores (vmcnt retires in order), so it is polled once per 32 LDS polls
    auto spin = [&](int b) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int it = 1;; ++it)
        {
            const int pin = flag_ld(f_in), pco = flag_ld(c_out), pxo = (w == 0) ? flag_ld(f_xo) : 0;
            if (ok(pin, pco, pxo, b)) return true;
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || ((it & 31) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return false;
            }
        }
    };
    // halo of block bb, read at the start of block bb: ring elements B*bb+64 .. +B-1 (lane 0;
    // lanes >= 1 read a row of g: no exec mask or branch)
    const uint32_t halo_base = (lane != 0) ? L.gfill : ring_in;
    auto halo_load = [&](int bb, int4v (&h)[kLH]) {
        const uint32_t hb = halo_base + (lane == 0 ? 4u * (uint32_t)((kLBlk * bb + 64) & (kLRing - 1)) : 0u);
#pragma unroll
        for (int j = 0; j < kLH; ++j) h[j] = lds_ld4(hb + 16u * (lane == 0 ? j : 0));
    };

    int qA[kLBlk], qB[kLBlk];
    int4v hA[kLH], hB[kLH];
#pragma unroll
    for (int j = 0; j < kLH; ++j) hA[j] = hB[j] = int4v {g, g, g, g};  // lanes >= 1 keep g
    if (!spin(-1)) return;
    {
        const uint32_t qb = qrow + 4u * (uint32_t)((-lane) & (kLW - 1));
#pragma unroll
        for (int u = 0; u < kLBlk; ++u) qA[u] = lds_ld(qb + 4u * u);
    }
    int H = rg, U = rg;
    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in the previous block, checked now
    int tE[kLBlk];                     // PAIR: the even block's transposed values, stored with the odd one's
    bool held = false;
#pragma unroll
    for (int e = 0; e < kLBlk; ++e) tE[e] = 0;

    auto block = [&](int b, int (&qc)[kLBlk], int (&qn)[kLBlk], int4v (&hc)[kLH], int4v (&hn)[kLH], auto rampT) {
        constexpr bool RAMP = decltype(rampT)::value;
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        halo_load(b, hc);
        // prefetch block b+1: Q of columns B(b+1)-l .. +B-1
        {
            const uint32_t qb = qrow + 4u * (uint32_t)((kLBlk * b + kLBlk - lane) & (kLW - 1));
#pragma unroll
            for (int u = 0; u < kLBlk; ++u) qn[u] = lds_ld(qb + 4u * u);
            flag_st(c_in, kLBlk * b + 64 + kLBlk);
        }
        int vals[kLBlk], lt[kLBlk];
#pragma unroll
        for (int u = 0; u < kLBlk; ++u)
        {
            const int up = shr1z(H) + hc[u >> 2][u & 3];
            const int t1 = U + qc[u];
            const int hg = H + g;
            int h = max(max(t1, up), hg);
            if constexpr (RAMP) h = (lane >= kLBlk * b + u) ? rg : h;  // column <= 0: the border
            lt[u] = hg;
            U = up;
            H = h;
            vals[u] = h;
            if (u == kLBlk / 2 - 1)
            {
                rpin = raw_ld(f_in);
                rpco = raw_ld(c_out);
                rpxo = raw_ld(f_xo);
            }
        }
        // hand-off: lane 63's H + g of steps Bb-1 .. Bb+B-2 = ring elements Bb .. Bb+B-1 (columns
        // Bb-64 ..); the last strip's ring is drained into granules by the drain wave.  Every lane
        // writes (no exec mask): lane 63 into the ring, the others into a sink
        {
            const uint32_t eb = (lane == 63) ? ring_out + 4u * (uint32_t)((kLBlk * b) & (kLRing - 1)) : hsink;
#pragma unroll
            for (int j = 0; j < kLH; ++j)
                lds_st4(eb + ((lane == 63) ? 16u * j : 0u), int4v {lt[4 * j], lt[4 * j + 1], lt[4 * j + 2], lt[4 * j + 3]});
        }
        flag_st(f_out, b + 1 == NB ? kLBig : kLBlk * b + kLBlk);
        {
            // output, transposed in registers: the 4 chunks (4 columns each) of the block are
            // exchanged across lane bits 5 and 4 (permlane32/16 swaps, 16 per block), so that
            // store k has lane 16h+n write chunk h of row r0+16k+n: 16 rows x 64 contiguous bytes
            // per store instead of 64 rows x 16 bytes (one row per lane pays one memory request
            // per lane, and the CU's requests are shared by its strips and the granule polls)
            int t[kLBlk];
#pragma unroll
            for (int e = 0; e < kLBlk; ++e) t[e] = vals[e];
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int d = 0; d < 4; ++d)
                {
                    const auto sw = __builtin_amdgcn_permlane32_swap(t[4 * k + d], t[4 * (k + 2) + d], false, false);
                    t[4 * k + d] = sw[0];
                    t[4 * (k + 2) + d] = sw[1];
                }
#pragma unroll
            for (int k = 0; k < 4; k += 2)
#pragma unroll
                for (int d = 0; d < 4; ++d)
                {
                    const auto sw = __builtin_amdgcn_permlane16_swap(t[4 * k + d], t[4 * (k + 1) + d], false, false);
                    t[4 * k + d] = sw[0];
                    t[4 * (k + 1) + d] = sw[1];
                }
            // interior blocks (uniform): every chunk is in the matrix; scalar row bases.  PAIR: an
            // even interior block's stores wait for the odd block after it, and the two blocks' stores
            // of each 16-row group go out back to back, so both 64-byte halves of a 128-byte line
            // (pitched layout, gsa_full_pitch) leave the wave one after the other
            auto interior = [&](int bb) { return kLBlk * bb - 63 >= 1 && kLBlk * bb + kLBlk - 1 <= C && r0 + 63 <= a.R; };
            auto store4 = [&](int bb, int k, const int (&v)[kLBlk]) {
                const gptr<int> ub = G(a.score) + ((ptrdiff_t)(r0 + 16 * k) * a.ld - 16 * k + kLBlk * bb);
                *(gptr<int4a>)(ub + xoff) = int4a {v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]};
            };
            if (PAIR && !RAMP && (b & 1) == 0 && b + 1 < NB && interior(b) && interior(b + 1))
            {
#pragma unroll
                for (int e = 0; e < kLBlk; ++e) tE[e] = t[e];
                held = true;
            }
            else if (PAIR && held)
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
                const int rr = 16 * k + (lane & 15);  // row r0 + rr, columns xc .. xc+3
                const int xc = kLBlk * b - rr + 4 * (lane >> 4);
                if (r0 + rr <= a.R)
                {
                    const gptr<int> p = xbase + (size_t)k * 16u * (size_t)(a.ld - 1) + kLBlk * b;
                    if (xc >= 1 && xc + 3 <= C)
                        *(gptr<int4a>)p = int4a {t[4 * k], t[4 * k + 1], t[4 * k + 2], t[4 * k + 3]};
                    else if (xc + 3 >= 1 && xc <= C)
                    {
#pragma unroll
                        for (int e = 0; e < 4; ++e)
                            if (xc + e >= 1 && xc + e <= C) p[e] = t[4 * k + e];
                    }
                }
            }
        }
        return true;
    };

    int b = 0;
    constexpr int kRampBlocks = 64 / kLBlk;  // columns <= 0 occur only in the first 64 steps
    for (; b < kRampBlocks; b += 2)
    {
        if (!block(b, qA, qB, hA, hB, std::integral_constant<bool, true>())) return;
        if (!block(b + 1, qB, qA, hB, hA, std::integral_constant<bool, true>())) return;
    }
    for (; b < NB; b += 2)
    {
        if (!block(b, qA, qB, hA, hB, std::integral_constant<bool, false>())) return;
        if (b + 1 < NB && !block(b + 1, qB, qA, hB, hA, std::integral_constant<bool, false>())) return;
    }
}

// ------------------------------------------------------------------------------------
// loader wave: Q profile, the row above strip 0 (granules of the previous super-strip, or
// row 0), the drain of the last strip's row into granules for the next super-strip
// ------------------------------------------------------------------------------------
// ROLE 0: both jobs in one wave; 1: the feed only; 2: the profile only.  Single pairs run the
// feed in a wave of its own (FD instance), so a poll is never behind a profile batch: the row
// above strip 0 arrives as soon as its granules are stored
template <int NS, int ROLE>
__device__ __forceinline__ void lane_loader(const StripArgs& a, const LaneLds& L, int tk, int lane)
{
    const int C = a.C, g = a.g;
    constexpr int kLW = lane_lw(NS), kLQRS = lane_qrs(NS);
    const uint32_t F = L.flags;
    const uint32_t ring0 = L.ring;
    const gptr<const unsigned long long> gprev = G((const unsigned long long*)a.gran) + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
    auto letter = [&](int c) {
        int x = (c >= 1 && c <= C) ? G(a.seqX)[c] : 0;
        return ((unsigned)x < (unsigned)a.substsz) ? x : 0;
    };
    int qn = 0;                    // Q holds columns < qn
    int hnext = 0;                 // next column of the row above to feed into ring 0
    int xl = letter(lane);
    int pl = 0, c0 = 0;  // progress words, re-read only when their cached values block
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;  // idle passes (error-word polls)
    while ((ROLE != 1 && qn <= C) || (ROLE != 2 && hnext <= C))
    {
        bool moved = false;
        // (1) the row above strip 0 (H + g) -> ring 0 elements c + 64, as far as granules of the
        //     previous super-strip are published (in column order) and ring 0 has room.  The poll
        //     is issued first and consumed after the Q work below, which runs under its latency;
        //     that latency paces this loop (no sleep while granules are awaited).
        if (ROLE != 2 && hnext <= C && hnext + 128 > c0 + kLRing) c0 = flag_ld(F + kFCons);  // ring 0 consumed
        const bool feed = ROLE != 2 && hnext <= C && hnext + 128 <= c0 + kLRing;
        const int c = hnext + lane;
        const bool in = c <= C;
        unsigned long long q = 0ull;
        if (feed && tk > 0 && in) q = __hip_atomic_load(gprev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (2) Q columns qn .. qn+63: the columns they replace (<= qn+63-kLW) are dead once the
        //     last strip has published elements pl (its next reads start at column pl-55).
        //     Gather the lane's letter column of subT (8 x b128), then 32 straight-line writes.
        if (ROLE != 1 && qn <= C && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);  // last strip's elements
        if (ROLE != 1 && qn <= C && qn <= pl + kLW - 128)
        {
            const uint32_t p = (uint32_t)((qn + lane) & (kLW - 1));
            const uint32_t sb = L.sub + 4u * kLSubRow * (uint32_t)xl;
            int4v v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = lds_ld4(sb + 16u * j);
            const uint32_t qa = L.q + 4u * p;
#pragma unroll
            for (int yy = 0; yy < 32; ++yy)
                if (yy < a.substsz) lds_st(qa + 4u * kLQRS * yy, v[yy >> 2][yy & 3]);
            if ((qn & (kLW - 1)) == 0 && lane < kLBlk)
            {
                // guard copy of columns p < kLBlk at p + kLW: a block's reads run past the wrap
#pragma unroll
                for (int yy = 0; yy < 32; ++yy)
                    if (yy < a.substsz) lds_st(qa + 4u * (kLQRS * yy + kLW), v[yy >> 2][yy & 3]);
            }
            qn += 64;
            xl = letter(qn + lane);
            flag_st(F + kFXo, qn > C ? kLBig : qn);
            moved = true;
        }
        if (feed)
        {
            int v = 0;
            bool good;
            if (tk == 0)
            {
                v = c * g + g;  // row 0: H(0, c) = c*g
                good = in;
            }
            else
            {
                good = in && (uint32_t)(q >> 32) == a.epoch;
                v = (int)(uint32_t)q;
            }
            const uint64_t badm = __ballot(!good);
            const int n = badm ? __builtin_ctzll(badm) : 64;
            if (n > 0)
            {
                if (lane < n) lds_st(ring0 + 4u * (uint32_t)((c + 64) & (kLRing - 1)), v);
                hnext += n;
                flag_st(F, hnext > C ? kLBig : hnext + 64);
                moved = true;
            }
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (moved)
            last = now;
        else
        {
            // the error word is a global load: it would wait for this wave's granule traffic and
            // stretch the idle poll, so another wave's error is looked at every 64th idle pass
            if (now - last > a.spin || ((++idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            if (ROLE == 2 || tk == 0 || hnext > C) __builtin_amdgcn_s_sleep(1);
        }
    }
}

// ------------------------------------------------------------------------------------
// drain wave: the last strip's row (H + g, ring NS) -> granules for the next super-strip.  A
// wave of its own: it issues no global loads, so its stores never wait (vmcnt is in order) and
// the feed wave's granule polls never delay the drain.
// ------------------------------------------------------------------------------------
template <int NS>
__device__ __forceinline__ void lane_drain(const StripArgs& a, const LaneLds& L, int tk, int lane)
{
    const int C = a.C;
    const uint32_t F = L.flags, ringN = L.ring + (uint32_t)NS * (kLRing * 4u);
    if (tk + 1 >= a.nTickets)
    {
        flag_st(F + kFCons + 4u * NS, kLBig);  // nobody reads our last row
        return;
    }
    const gptr<unsigned long long> gout = G(a.gran) + (size_t)tk * a.granStride;
    int dnext = 0;  // next column to drain
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;  // idle passes (error-word polls)
    while (dnext <= C)
    {
        const int avail = min(flag_ld(F + 4u * NS) - 64, C + 1);  // columns < avail are in ring NS
        if (dnext < avail)
        {
            const int c = dnext + lane;
            if (c < avail)
            {
                const int v = lds_ld(ringN + 4u * (uint32_t)((c + 64) & (kLRing - 1)));
                __hip_atomic_store(gout + c, ((unsigned long long)a.epoch << 32) | (uint32_t)v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            dnext = min(dnext + 64, avail);
            flag_st(F + kFCons + 4u * NS, dnext > C ? kLBig : dnext + 64);
            last = __builtin_amdgcn_s_memrealtime();
        }
        else
        {
            // the error word is a global load, which waits for this wave's granule stores (vmcnt
            // retires in order): looked at every 64th idle pass only
            if (__builtin_amdgcn_s_memrealtime() - last > a.spin || ((++idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

__device__ __forceinline__ PairDesc lane_desc(const PairDesc* p)
{
    constexpr int N = sizeof(PairDesc) / 4;
    const int* wds = (const int*)p;
    union
    {
        int v[N];
        PairDesc d;
    } u;
#pragma unroll
    for (int k = 0; k < N; ++k) u.v[k] = __builtin_amdgcn_readfirstlane(G(wds)[k]);
    return u.d;
}

// PAIR: an even block's output stores wait for the odd block after it (lane_strip).  Batches run two
// workgroups per CU (three waves per SIMD): the register budget is held to 168
template <int NS, bool FD, bool PAIR>
__global__ void __launch_bounds__(64 * (NS + 2 + FD), FD ? 2 : 3) nw_lane_kernel(StripArgs a)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const LaneLds L = lane_layout(NS, a.substsz);
    for (int k = threadIdx.x; k < a.substsz * kLSubRow; k += 64 * (NS + 2 + FD))
    {
        const int x = k / kLSubRow, yy = k % kLSubRow;
        lds_st(L.sub + 4u * k, yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - a.g : 0);
    }
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) lds_st(L.flags + kFTicket, err_set(a) ? a.nTicketsTotal : (int)atomicAdd(a.ticket, 1u));
        __syncthreads();
        const int tkg = __builtin_amdgcn_readfirstlane(lds_ld(L.flags + kFTicket));
        if (tkg >= a.nTicketsTotal) break;
        // pair of this ticket: the batch schedule, or the last descriptor with ticketBase <= tkg
        // (binary search, uniform)
        int lo = 0, tks = -1;
        if (a.sched)
        {
            lo = __builtin_amdgcn_readfirstlane(G(a.sched)[2 * tkg]);
            tks = __builtin_amdgcn_readfirstlane(G(a.sched)[2 * tkg + 1]);
        }
        else
        {
            int hi = a.nPairs - 1;
            while (lo < hi)
            {
                const int mid = (lo + hi + 1) >> 1;
                if (__builtin_amdgcn_readfirstlane(G(a.pairs)[mid].ticketBase) <= tkg)
                    lo = mid;
                else
                    hi = mid - 1;
            }
        }
        const PairDesc d = lane_desc(a.pairs + lo);
        StripArgs pa = a;
        pa.seqY = d.seqY;
        pa.seqX = d.seqX;
        pa.R = d.R;
        pa.C = d.C;
        pa.nTickets = d.nTickets;
        pa.score = d.score;
        pa.ld = d.ld;
        pa.gran = a.gran + d.granOff;
        pa.granStride = gran_stride(d.C);
        const int tk = (tks >= 0) ? tks : tkg - d.ticketBase;
        if (threadIdx.x < 32) lds_st(L.flags + 4u * threadIdx.x, 0);  // prog[], cons[]
        if (threadIdx.x < 16) lds_st(L.gfill + 4u * threadIdx.x, a.g);
        if (threadIdx.x == 0) lds_st(L.flags + kFXo, 0);
        __syncthreads();
        if (w == NS + 1)
            lane_drain<NS>(pa, L, tk, lane);
        else if (w == NS)
            lane_loader<NS, FD ? 2 : 0>(pa, L, tk, lane);
        else if (FD && w == NS + 2)
            lane_loader<NS, 1>(pa, L, tk, lane);
        else
        {
            __builtin_amdgcn_s_setprio(3);
            lane_strip<NS, PAIR>(pa, L, tk, w, lane);
            __builtin_amdgcn_s_setprio(0);
        }
    }
}

template <int NS, bool FD = false, bool PAIR = true>
hipError_t launch_lane(const StripArgs& a, int grid, hipStream_t stream)
{
    const size_t lds = lane_lds_bytes(NS, a.substsz);
    auto kern = nw_lane_kernel<NS, FD, PAIR>;
    constexpr int kThreads = 64 * (NS + 2 + FD);
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (grid <= 0)
    {
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, kThreads, lds);
        if (e == hipSuccess) e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        grid = std::max(1, std::min(a.nTicketsTotal, std::max(1, per_cu) * cus));
    }
    if ((e = record_foot((const void*)kern, lds, kThreads, grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

size_t lane_lds_bytes(int ns, int substsz)
{
    return (size_t)lane_layout(ns, substsz).flags + 256;
}

hipError_t launch_lane_fill(const StripArgs& a, int ns, int grid, hipStream_t stream)
{
    if (ns == 1) return launch_lane<1>(a, grid, stream);
    if (ns == 3) return launch_lane<3>(a, grid, stream);
    // a single pair: the feed in a wave of its own (a 7th wave would cost a batch its second
    // workgroup per CU); a.laneFeed (knob GSA_LANE_FEED) overrides
    const bool fd = a.laneFeed >= 0 ? a.laneFeed != 0 : a.nPairs == 1;
    // paired output stores (lane_strip) for batches: 64 x 20k pitched 977-988 -> 1097 GCUPS; a single
    // pair's strips run on their critical path, where the held block costs (10k 100 -> 93 GCUPS,
    // profiles/r04_full_pitch_pair.txt); a.lanePair (knob GSA_LANE_PAIR) overrides
    const bool pair = a.lanePair >= 0 ? a.lanePair != 0 : !fd;
    if (ns == 4)
        return fd ? (pair ? launch_lane<4, true, true>(a, grid, stream) : launch_lane<4, true, false>(a, grid, stream))
                  : (pair ? launch_lane<4, false, true>(a, grid, stream) : launch_lane<4, false, false>(a, grid, stream));
    if (ns == 6) return launch_lane<6>(a, grid, stream);
    if (ns == 8) return launch_lane<8>(a, grid, stream);
    return launch_lane<2>(a, grid, stream);
}

}  // namespace gsa
