// nw_pair2.hip -- NW-LG sparse (mlsp tile-header) fill with TWO rows per lane, hand-written
// wave64 HIP for gfx950 (MI355X).
//
// Replaces the sparse family NwAlign_Gpu7..9 (nwalign_gpu9_mlsp_diagdiagdiag.cu:368-722, kernels
// :15-360) for single pairs and has their output contract: tileHrowMat / tileHcolMat, tile-major
// k = tcols*iT + jT, 1+tBx resp. 1+tBy ints per tile, element 0 the corner, the padded region
// computed with letter 0 (nwalign_gpu9_mlsp_diagdiagdiag.cu:147-171, 471-478).  Recurrence of
// UpdateScore (nwalign_cpu1_st_row.cpp:4-10).
//
// Why two rows per lane.  One pair is bounded by its wavefront: (C + S*L) * t_step, with S strips
// in the chain, L ~ 80 steps of lag per strip (the 64-lane skew + one block) and t_step the cost
// of one step of one wave.  With K rows per lane t_step ~ a + b*K and S = R / (64 K).  Four rows
// per lane (nw_strip.hip) pay a long step (~160 cycles at 100k: 17 VALU + LDS waits per step,
// profiles/r02_pmc_config3.json); one row per lane (nw_lane.hip) doubles the skew term.  Two
// rows per lane with the shifted recurrence is 5 VALU per step and 128 rows per wave.
//
// Step, shifted values H' = H - (i+j)*g (>= 0 for g <= 0; borders 0):
//     up  = dpp_shr1(Hb) + halo        lane 0: H'(row above, c) from the ring; others + 0
//     Ha' = max3(Da + qa, up, Ha)      Da = up of the previous step (= H'(ra-1, c-1))
//     Hb' = max3(Ha + qb, Ha', Hb)     Ha (old) = H'(ra, c-1)
// with q = s(y, X[c]) - 2g from a per-workgroup column profile Q[y][c] (LDS ring, lane l reads
// Q[y_l][t-l] at base + immediate offsets: conflict-free, no VALU addressing).  Lane l owns rows
// r0+2l (a) and r0+2l+1 (b) and at step t works on column t-l.
//
// Sparse output.  Header rows (the last row of a tile row) are the last row of a ticket: the
// drain wave writes them with the granules.  Header columns are captured by the strips: in a
// block whose 79-column window holds a tile boundary, every lane keeps its 16 (Ha, Hb) pairs and
// picks the one at its boundary column with a 4-level v_cndmask tree (one lane per boundary and
// step), then stores 2 ints.  Blocks without a boundary run the bare step.
//
// Hand-off between strips: lane 63 writes its old Hb (column t-64) into the next strip's ring,
// 16 per block (every lane writes, the others into a sink: no exec mask); lane 0 of the next
// strip reads block b's 16 halo values at the start of block b.  LDS progress words keep the
// order (a wave's LDS ops execute in order).  Between super-strips (workgroups) the drain wave
// moves the last row through 8-byte {epoch, H'} granules in HBM (sc1 atomics) and the loader
// wave of the next super-strip polls them (MI355X_MICROARCH.md, handoff-1to1).  Every wait is
// bounded (StripArgs::spin, error word).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_pair2.h"

namespace gsa {
namespace {

__host__ __device__ constexpr int p2_lw(int ns) { return ns >= 5 ? 1024 : 512; }  // Q ring columns
__host__ __device__ constexpr int p2_qrs(int ns) { return p2_lw(ns) + 32; }        // Q row stride (dwords), 32 guard
constexpr int kP2Blk = 16;       // steps per block
constexpr int kP2H = kP2Blk / 4; // halo registers (int4) per block
constexpr int kP2Ring = 512;     // hand-off ring elements per strip boundary (power of 2)
constexpr int kP2Big = 0x3fffffff;
constexpr int kP2SubRow = 36;    // dwords per subT row (32 letters + 4)
constexpr uint32_t kFCons = 64, kFXo = 128, kFTicket = 132;

extern __shared__ __attribute__((aligned(16))) char p2sm[];

// Timing-experiment knobs (tools/build_p2_knobs.sh; any set bit makes results WRONG): 1 no halo
// reads, 2 no Q reads, 4 no hand-off writes, 8 strips never wait, 16 no mid-block progress reads,
// 32 no header-column capture, 64 capture without its global stores, 128 drain without global stores
#ifndef GSA_P2KNOB
#define GSA_P2KNOB 0
#endif
// Diagnostic stamps (separate build, tools/p2_stamps.py): s_memtime at 4 points of blocks
// 64..319 of the strips of tickets 0 and 1, dbg[(tk*NS + w)*1024 + (b-64)*4 + k]
#ifndef GSA_P2STAMP
#define GSA_P2STAMP 0
#endif

typedef int int4v __attribute__((ext_vector_type(4)));
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(p2sm + a); }
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(p2sm + a) = v; }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(p2sm + a); }
__device__ __forceinline__ void lds_st4(uint32_t a, int4v v) { *(int4v*)(p2sm + a) = v; }
// progress words: relaxed workgroup-scope atomics (no vmcnt drains, unlike volatile accesses)
__device__ __forceinline__ int raw_ld(uint32_t a)
{
    return __hip_atomic_load((int*)__builtin_assume_aligned(p2sm + a, 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int flag_ld(uint32_t a) { return __builtin_amdgcn_readfirstlane(raw_ld(a)); }
__device__ __forceinline__ void flag_st(uint32_t a, int v)
{
    asm volatile("" ::: "memory");  // data writes are issued before the word (LDS executes in order)
    __hip_atomic_store((int*)__builtin_assume_aligned(p2sm + a, 4), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool err_set(const StripArgs& a)
{
    return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
// m ? b : a per lane, m a lane mask in an SGPR pair: one v_cndmask (a plain ?: tree over an array
// is turned into a dynamically indexed array in scratch)
__device__ __forceinline__ int sel(uint64_t m, int a, int b)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// LDS: Q profile (substsz rows of p2_qrs dwords), subT[x][y] = s(y, x) - 2g, NS+1 hand-off
// rings, 16 zeros (the halo of lanes >= 1), the hand-off sink, progress words:
// prog[i] @ 4i (ring i holds elements < prog[i]), cons[i] @ 64+4i (ring i's reader no longer
// needs elements < cons[i]), xo @ 128 (Q holds columns < xo), ticket @ 132.
struct P2Lds
{
    uint32_t q, sub, ring, zfill, sink, flags;
};

__host__ __device__ inline P2Lds p2_layout(int ns, int substsz)
{
    P2Lds L;
    L.q = 0;
    L.sub = (uint32_t)substsz * p2_qrs(ns) * 4u;
    L.ring = L.sub + (uint32_t)substsz * kP2SubRow * 4u;
    L.zfill = L.ring + (uint32_t)(ns + 1) * kP2Ring * 4u;
    L.sink = L.zfill + 64u;
    L.flags = L.sink + (uint32_t)ns * 1024u;
    return L;
}

// ------------------------------------------------------------------------------------
// strip wave: 128 rows, two per lane
// ------------------------------------------------------------------------------------
template <int NS>
__device__ __forceinline__ void p2_strip(const StripArgs& a, const P2Lds& L, int tk, int w, int lane)
{
    const int g = a.g;
    const int Cp = a.Cp;
    const int tBx = a.tBx, tBy = a.tBy, tcols = a.tcols;
    const int r0 = tk * (kPair2Rows * NS) + kPair2Rows * w + 1;  // first row of the strip
    const int ra = r0 + 2 * lane, rb = ra + 1;                   // this lane's rows
    auto yl = [&](int r) {
        int y = (r <= a.R) ? G(a.seqY)[r] : 0;
        return ((unsigned)y < (unsigned)a.substsz) ? y : 0;
    };
    constexpr int kLW = p2_lw(NS), kQRS = p2_qrs(NS);
    const uint32_t qrowA = L.q + (uint32_t)yl(ra) * (kQRS * 4u);
    const uint32_t qrowB = L.q + (uint32_t)yl(rb) * (kQRS * 4u);
    const uint32_t ring_in = L.ring + (uint32_t)w * (kP2Ring * 4u);
    const uint32_t ring_out = L.ring + (uint32_t)(w + 1) * (kP2Ring * 4u);
    const uint32_t f_in = L.flags + 4u * w, f_out = L.flags + 4u * (w + 1);
    const uint32_t c_in = L.flags + kFCons + 4u * w, c_out = L.flags + kFCons + 4u * (w + 1);
    const uint32_t f_xo = L.flags + kFXo;
    const uint32_t hsink = L.sink + (uint32_t)w * 1024u + 16u * (uint32_t)lane;
    const int NB = (Cp + 65 + kP2Blk - 1) / kP2Blk;  // lane 63 reaches step Cp+64 (element of column Cp)
    // header column slots of this lane's rows: tile row iT, elements ea, ea+1 (same tile: ra is odd)
    const int iT = (ra - 1) / tBy;
    const int ea = ra - iT * tBy;
    const gptr<int> hcolT = G(a.hcol) + (size_t)iT * (size_t)tcols * (size_t)(tBy + 1) + ea;

    // block b prefetches block b+1's Q (columns < 16b+32) and reads its own halo (ring elements
    // 16b+64 .. 16b+79), writes ring elements 16b .. 16b+15
    auto ok = [&](int pin, int pco, int pxo, int b) {
        if constexpr ((GSA_P2KNOB & 8) != 0) return true;
        return pin >= kP2Blk * b + 64 + kP2Blk && pco >= kP2Blk * b + kP2Blk - kP2Ring &&
               (w != 0 || pxo >= kP2Blk * b + 2 * kP2Blk);
    };
    // the error word is a global load, which waits for this wave's outstanding header stores
    // (vmcnt retires in order): polled once per 32 LDS polls
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
    // halo of block b: lane 0 reads ring elements 16b+64 .. +15, lanes >= 1 a row of zeros (no branch)
    auto halo_load = [&](int b, int4v (&h)[kP2H]) {
        const uint32_t hb = (lane == 0) ? ring_in + 4u * (uint32_t)((kP2Blk * b + 64) & (kP2Ring - 1)) : L.zfill;
#pragma unroll
        for (int j = 0; j < kP2H; ++j) h[j] = lds_ld4(hb + 16u * (lane == 0 ? j : 0));
    };
    auto q_load = [&](int b, int (&qa)[kP2Blk], int (&qb)[kP2Blk]) {
        // columns 16b - lane .. +15 (ring position; reads past the wrap hit the guard copy)
        const uint32_t p = 4u * (uint32_t)((kP2Blk * b - lane) & (kLW - 1));
#pragma unroll
        for (int u = 0; u < kP2Blk; ++u) qa[u] = lds_ld(qrowA + p + 4u * u);
#pragma unroll
        for (int u = 0; u < kP2Blk; ++u) qb[u] = lds_ld(qrowB + p + 4u * u);
    };

    int qA0[kP2Blk], qA1[kP2Blk], qB0[kP2Blk], qB1[kP2Blk];
    int4v hc[kP2H];
#pragma unroll
    for (int j = 0; j < kP2H; ++j) hc[j] = int4v {0, 0, 0, 0};
    if (!spin(-1)) return;
    q_load(0, qA0, qA1);
    int Ha = 0, Hb = 0, Da = 0;
    int lt[kP2Blk];  // lane 63's hand-off values of the last block (Hb of columns t-64)
    // hand-off of block bb: every lane writes (lane 63 into the ring, the others into the sink,
    // no exec mask), then the progress word
    auto handoff = [&](int bb) {
        if constexpr ((GSA_P2KNOB & 4) == 0)
        {
            const uint32_t eb = (lane == 63) ? ring_out + 4u * (uint32_t)((kP2Blk * bb) & (kP2Ring - 1)) : hsink;
#pragma unroll
            for (int j = 0; j < kP2H; ++j)
                lds_st4(eb + ((lane == 63) ? 16u * j : 0u), int4v {lt[4 * j], lt[4 * j + 1], lt[4 * j + 2], lt[4 * j + 3]});
        }
        flag_st(f_out, bb + 1 == NB ? kP2Big : kP2Blk * bb + kP2Blk);
    };
    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block
    int nb0 = tBx, jb0 = 1;             // smallest tile boundary column >= 16b - 63 (uniform)

    // One body for blocks with and without a header-column capture (cap, uniform): separate
    // bodies got different register assignments and ~100 v_mov per block to reconcile them.
    auto block = [&](int b, int (&qca)[kP2Blk], int (&qcb)[kP2Blk], int (&qna)[kP2Blk], int (&qnb)[kP2Blk],
                     auto rampT, bool cap) {
        constexpr bool RAMP = decltype(rampT)::value;
        constexpr bool CAP = !RAMP && (GSA_P2KNOB & 32) == 0;  // ramp blocks hold no boundary (tBx >= 64)
        auto stamp = [&](int k) {
            if constexpr (GSA_P2STAMP != 0)
                if (tk < 2 && b >= 64 && b < 320 && lane == 0 && a.dbg)
                    a.dbg[(size_t)(tk * NS + w) * 1024 + (b - 64) * 4 + k] = __builtin_amdgcn_s_memtime();
        };
        stamp(0);
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        stamp(1);
        if constexpr ((GSA_P2KNOB & 1) == 0) halo_load(b, hc);
        // block b-1's hand-off, behind this block's halo reads (LDS executes a wave's operations in
        // order: written before them, the halo would wait for the writes)
        if (b > 0) handoff(b - 1);
        flag_st(c_in, kP2Blk * b + 64 + kP2Blk);
        // Q of block b+1 (columns 16(b+1) - lane ..), two reads per step: spread over the block,
        // they stay within the 15 outstanding LDS operations lgkmcnt counts
        const uint32_t pn = 4u * (uint32_t)((kP2Blk * (b + 1) - lane) & (kLW - 1));
        int va[CAP ? kP2Blk : 1], vb[CAP ? kP2Blk : 1];
#pragma unroll
        for (int u = 0; u < kP2Blk; ++u)
        {
            const int up = shr1z(Hb) + hc[u >> 2][u & 3];
            int ha = max3i(Da + qca[u], up, Ha);
            int hb = max3i(Ha + qcb[u], ha, Hb);
            if constexpr (RAMP)
            {
                // column t - lane <= 0: the border (H' = 0)
                const bool border = lane >= kP2Blk * b + u;
                ha = border ? 0 : ha;
                hb = border ? 0 : hb;
            }
            // Q of block b+1 in the first half of the block (4 columns per step), so the reads have
            // returned when the next block starts (a wave's LDS operations return in order, and the
            // block start waits on the progress reads issued after them)
            if (u < kP2Blk / 2)
            {
#pragma unroll
                for (int e = 2 * u; e < 2 * u + 2; ++e)
                {
                    if constexpr ((GSA_P2KNOB & 2) == 0)
                    {
                        qna[e] = lds_ld(qrowA + pn + 4u * e);
                        qnb[e] = lds_ld(qrowB + pn + 4u * e);
                    }
                    else
                    {
                        qna[e] = qca[e] ^ 1;
                        qnb[e] = qcb[e] ^ 1;
                    }
                }
            }
            lt[u] = Hb;  // column t-64 of row b: ring element t
            Da = up;
            Ha = ha;
            Hb = hb;
            if constexpr (CAP)
            {
                va[u] = ha;
                vb[u] = hb;
            }
            if ((GSA_P2KNOB & 16) == 0 && u == kP2Blk / 2 - 1)
            {
                rpin = raw_ld(f_in);
                rpco = raw_ld(c_out);
                rpxo = raw_ld(f_xo);
            }
        }
        stamp(2);
        if (CAP && cap)
        {
            // this lane's columns lo .. lo+15; boundaries nb0 (>= 16b-63) and nb0 + tBx
            const int lo = kP2Blk * b - lane;
            int bc = nb0, jT = jb0;
            if (bc < lo)
            {
                bc += tBx;
                ++jT;
            }
            const int s = bc - lo;
            if (s <= kP2Blk - 1 && jT < tcols)
            {
                // 16 -> 1 by the bits of s (v_cndmask tree, 15 per row)
                const uint64_t m1 = __builtin_amdgcn_ballot_w64((s & 1) != 0), m2 = __builtin_amdgcn_ballot_w64((s & 2) != 0);
                const uint64_t m4 = __builtin_amdgcn_ballot_w64((s & 4) != 0), m8 = __builtin_amdgcn_ballot_w64((s & 8) != 0);
                int xa[8], xb[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                {
                    xa[i] = sel(m1, va[2 * i], va[2 * i + 1]);
                    xb[i] = sel(m1, vb[2 * i], vb[2 * i + 1]);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
                {
                    xa[i] = sel(m2, xa[2 * i], xa[2 * i + 1]);
                    xb[i] = sel(m2, xb[2 * i], xb[2 * i + 1]);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
                {
                    xa[i] = sel(m4, xa[2 * i], xa[2 * i + 1]);
                    xb[i] = sel(m4, xb[2 * i], xb[2 * i + 1]);
                }
                const int sa = sel(m8, xa[0], xa[1]);
                const int sb = sel(m8, xb[0], xb[1]);
                const gptr<int> dst = hcolT + (size_t)jT * (size_t)(tBy + 1);
                if constexpr ((GSA_P2KNOB & 64) == 0)
                {
                    dst[0] = sa + (ra + bc) * g;
                    dst[1] = sb + (rb + bc) * g;
                }
                else
                    lds_st(hsink, sa + sb);
            }
        }
        stamp(3);
        return true;
    };

    // the window of block b holds a tile boundary iff nb0 <= 16b+15 (uniform)
    auto advance = [&](int b) {
        if (nb0 < kP2Blk * b - 63)  // the window moves 16 columns per block and tBx >= 64
        {
            nb0 += tBx;
            ++jb0;
        }
        return nb0 <= kP2Blk * b + kP2Blk - 1 && jb0 < tcols;
    };
    using T = std::integral_constant<bool, true>;
    using F = std::integral_constant<bool, false>;
    constexpr int kRampBlocks = 64 / kP2Blk;  // columns <= 0 occur only in the first 64 steps (no boundary there: tBx >= 64)
    int b = 0;
    for (; b < kRampBlocks; b += 2)
    {
        if (!block(b, qA0, qA1, qB0, qB1, T(), false)) return;
        if (!block(b + 1, qB0, qB1, qA0, qA1, T(), false)) return;
    }
    for (; b < NB; b += 2)
    {
        if (!block(b, qA0, qA1, qB0, qB1, F(), advance(b))) return;
        if (b + 1 >= NB) break;
        if (!block(b + 1, qB0, qB1, qA0, qA1, F(), advance(b + 1))) return;
    }
    handoff(NB - 1);
}

// ------------------------------------------------------------------------------------
// loader wave: Q profile and the row above strip 0 (granules of the previous super-strip, or
// row 0)
// ------------------------------------------------------------------------------------
template <int NS>
__device__ __forceinline__ void p2_loader(const StripArgs& a, const P2Lds& L, int tk, int lane)
{
    const int Cp = a.Cp, C = a.C;
    constexpr int kLW = p2_lw(NS), kQRS = p2_qrs(NS);
    const uint32_t F = L.flags;
    const uint32_t ring0 = L.ring;
    const gptr<const unsigned long long> gprev = G((const unsigned long long*)a.gran) + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
    auto letter = [&](int c) {
        int x = (c >= 1 && c <= C) ? G(a.seqX)[c] : 0;  // padded columns: letter 0
        return ((unsigned)x < (unsigned)a.substsz) ? x : 0;
    };
    int qn = 0;     // Q holds columns < qn
    int hnext = 0;  // next column of the row above to feed into ring 0
    int xl = letter(lane);
    int pl = 0, c0 = 0;  // progress words, re-read only when their cached values block
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    while (qn <= Cp || hnext <= Cp)
    {
        bool moved = false;
        // (1) the row above strip 0 -> ring 0 elements c + 64, as far as granules of the previous
        //     super-strip are published (in column order) and ring 0 has room.  The poll is issued
        //     first and consumed after the Q work, which runs under its latency.
        if (hnext <= Cp && hnext + 128 > c0 + kP2Ring) c0 = flag_ld(F + kFCons);
        const bool feed = hnext <= Cp && hnext + 128 <= c0 + kP2Ring;
        const int c = hnext + lane;
        const bool in = c <= Cp;
        unsigned long long q = 0ull;
        if (feed && tk > 0 && in) q = __hip_atomic_load(gprev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (2) Q columns qn .. qn+63: the columns they replace (<= qn+63-kLW) are dead once the last
        //     strip has published elements pl (its next reads start at column pl-55)
        if (qn <= Cp && qn > pl + kLW - 128) pl = flag_ld(F + 4u * NS);
        if (qn <= Cp && qn <= pl + kLW - 128)
        {
            const uint32_t p = (uint32_t)((qn + lane) & (kLW - 1));
            const uint32_t sb = L.sub + 4u * kP2SubRow * (uint32_t)xl;
            int4v v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = lds_ld4(sb + 16u * j);
            const uint32_t qa = L.q + 4u * p;
#pragma unroll
            for (int yy = 0; yy < 32; ++yy)
                if (yy < a.substsz) lds_st(qa + 4u * kQRS * yy, v[yy >> 2][yy & 3]);
            if ((qn & (kLW - 1)) == 0 && lane < kP2Blk)
            {
                // guard copy of columns p < 16 at p + kLW: a block's reads run past the wrap
#pragma unroll
                for (int yy = 0; yy < 32; ++yy)
                    if (yy < a.substsz) lds_st(qa + 4u * (kQRS * yy + kLW), v[yy >> 2][yy & 3]);
            }
            qn += 64;
            xl = letter(qn + lane);
            flag_st(F + kFXo, qn > Cp ? kP2Big : qn);
            moved = true;
        }
        if (feed)
        {
            int v = 0;  // row 0: H' = 0
            bool good = in;
            if (tk > 0)
            {
                good = in && (uint32_t)(q >> 32) == a.epoch;
                v = (int)(uint32_t)q;
            }
            const uint64_t badm = __ballot(!good);
            const int n = badm ? __builtin_ctzll(badm) : 64;
            if (n > 0)
            {
                if (lane < n) lds_st(ring0 + 4u * (uint32_t)((c + 64) & (kP2Ring - 1)), v);
                hnext += n;
                flag_st(F, hnext > Cp ? kP2Big : hnext + 64);
                moved = true;
            }
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (moved)
            last = now;
        else
        {
            if (now - last > a.spin || err_set(a))
            {
                atomicOr(a.err, 1u);
                return;
            }
            if (tk == 0 || hnext > Cp) __builtin_amdgcn_s_sleep(1);
        }
    }
}

// ------------------------------------------------------------------------------------
// drain wave: the last strip's row (ring NS) -> granules for the next super-strip and, when the
// row closes a tile row, the header row of the tiles below (unshifted) with its duplicates: the
// last element of the tile to the left and the corner of the header column
// (nwalign_gpu9_mlsp_diagdiagdiag.cu:214-218, 253-257).  It issues no global loads, so its stores
// never wait behind a poll.
// ------------------------------------------------------------------------------------
template <int NS>
__device__ __forceinline__ void p2_drain(const StripArgs& a, const P2Lds& L, int tk, int lane)
{
    const int Cp = a.Cp, g = a.g, tBx = a.tBx, tBy = a.tBy, tcols = a.tcols;
    const uint32_t F = L.flags, ringN = L.ring + (uint32_t)NS * (kP2Ring * 4u);
    if (tk + 1 >= a.nTickets)
    {
        flag_st(F + kFCons + 4u * NS, kP2Big);  // nobody reads our last row
        return;
    }
    const gptr<unsigned long long> gout = G(a.gran) + (size_t)tk * a.granStride;
    const int rowEnd = (tk + 1) * (kPair2Rows * NS);  // the row this ticket hands down
    const bool hdr = rowEnd % tBy == 0;
    const size_t rowbase = (size_t)(rowEnd / tBy) * (size_t)tcols;  // tile index of (iT+1, 0)
    int dnext = 0;  // next column to drain
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    while (dnext <= Cp)
    {
        const int avail = min(flag_ld(F + 4u * NS) - 64, Cp + 1);  // columns < avail are in ring NS
        if (dnext < avail)
        {
            const int c = dnext + lane;
            if ((GSA_P2KNOB & 128) == 0 && c < avail)
            {
                const int v = lds_ld(ringN + 4u * (uint32_t)((c + 64) & (kP2Ring - 1)));
                __hip_atomic_store(gout + c, ((unsigned long long)a.epoch << 32) | (uint32_t)v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                if (hdr)
                {
                    const int hv = v + (rowEnd + c) * g;
                    const int jT = c / tBx, jj = c - jT * tBx;
                    if (jT < tcols) G(a.hrow)[(rowbase + jT) * (size_t)(tBx + 1) + jj] = hv;
                    if (jj == 0 && jT > 0)
                    {
                        G(a.hrow)[(rowbase + jT - 1) * (size_t)(tBx + 1) + tBx] = hv;
                        if (jT < tcols) G(a.hcol)[(rowbase + jT) * (size_t)(tBy + 1)] = hv;
                    }
                }
            }
            dnext = min(dnext + 64, avail);
            flag_st(F + kFCons + 4u * NS, dnext > Cp ? kP2Big : dnext + 64);
            last = __builtin_amdgcn_s_memrealtime();
        }
        else
        {
            if (__builtin_amdgcn_s_memrealtime() - last > a.spin || err_set(a))
            {
                atomicOr(a.err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

__device__ __forceinline__ PairDesc p2_desc(const PairDesc* p)
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

template <int NS>
__global__ void __launch_bounds__(64 * (NS + 2)) nw_pair2_kernel(StripArgs a)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const P2Lds L = p2_layout(NS, a.substsz);
    for (int k = threadIdx.x; k < a.substsz * kP2SubRow; k += 64 * (NS + 2))
    {
        const int x = k / kP2SubRow, yy = k % kP2SubRow;
        lds_st(L.sub + 4u * k, yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - 2 * a.g : 0);
    }
    if (threadIdx.x < 16) lds_st(L.zfill + 4u * threadIdx.x, 0);
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) lds_st(L.flags + kFTicket, err_set(a) ? a.nTicketsTotal : (int)atomicAdd(a.ticket, 1u));
        __syncthreads();
        const int tkg = __builtin_amdgcn_readfirstlane(lds_ld(L.flags + kFTicket));
        if (tkg >= a.nTicketsTotal) break;
        // pair of this ticket: the batch schedule, or the last descriptor with ticketBase <= tkg
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
        const PairDesc d = p2_desc(a.pairs + lo);
        StripArgs pa = a;
        pa.seqY = d.seqY;
        pa.seqX = d.seqX;
        pa.R = d.R;
        pa.C = d.C;
        pa.Cp = d.Cp;
        pa.nTickets = d.nTickets;
        pa.hrow = d.hrow;
        pa.hcol = d.hcol;
        pa.trows = d.trows;
        pa.tcols = d.tcols;
        pa.gran = a.gran + d.granOff;
        pa.granStride = (long long)d.Cp + 1;
        const int tk = (tks >= 0) ? tks : tkg - d.ticketBase;
        if (threadIdx.x < 32) lds_st(L.flags + 4u * threadIdx.x, 0);  // prog[], cons[]
        if (threadIdx.x == 0) lds_st(L.flags + kFXo, 0);
        __syncthreads();
        if (w == NS + 1)
            p2_drain<NS>(pa, L, tk, lane);
        else if (w == NS)
            p2_loader<NS>(pa, L, tk, lane);
        else
        {
            __builtin_amdgcn_s_setprio(3);
            p2_strip<NS>(pa, L, tk, w, lane);
            __builtin_amdgcn_s_setprio(0);
        }
    }
}

template <int NS>
hipError_t launch_p2(const StripArgs& a, int grid, hipStream_t stream)
{
    const size_t lds = pair2_lds_bytes(NS, a.substsz);
    auto kern = nw_pair2_kernel<NS>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (grid <= 0)
    {
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * (NS + 2), lds);
        if (e == hipSuccess) e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        grid = std::max(1, std::min(a.nTicketsTotal, std::max(1, per_cu) * cus));
    }
    if ((e = record_foot((const void*)kern, lds, 64 * (NS + 2), grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (NS + 2)), lds, stream, a);
    return hipGetLastError();
}

}  // namespace

size_t pair2_lds_bytes(int ns, int substsz) { return (size_t)p2_layout(ns, substsz).flags + 256; }

hipError_t launch_pair2_fill(const StripArgs& a, int ns, int grid, hipStream_t stream)
{
    if (ns == 2) return launch_p2<2>(a, grid, stream);
    return launch_p2<4>(a, grid, stream);
}

}  // namespace gsa
