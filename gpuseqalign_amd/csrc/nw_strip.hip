// nw_strip.hip -- NW-LG score-matrix fill for gfx950 (MI355X), hand-written wave64 HIP.
//
// Replaces the reference's tiled anti-diagonal fill family (gpu3..gpu9, e.g.
// nwalign_gpu9_mlsp_diagdiagdiag.cu:69-360 Kernel B and its per-diagonal launch loop
// :616-660) with ONE persistent launch that sweeps horizontal strips.
//
// Recurrence (nwalign_cpu1_st_row.cpp:4-10) in the shifted space H' = H - (i+j)*g:
//     H'[i][j] = max3(H'[i-1][j-1] + s(i,j) - 2g, H'[i-1][j], H'[i][j-1])
// H' is >= 0 and non-decreasing along rows and columns; one cell = one v_add + one v_max3.
//
// Strip = one wave = 256 rows.  Lane l owns the 4 consecutive rows r0+4l .. r0+4l+3 and at
// step t works on column c = t - l for all four of them (skewed across lanes, not within a
// lane), so one step is
//     up  = DPP wave_shr:1 (row D of lane l-1) [+ halo for lane 0]      v_add_u32_dpp
//     A   = max3(diagA + sA, up, A)                                      v_add_sdwa + v_max3
//     B   = max3(A_prev + sB, A, B) ... D                                 (x3)
// = 9 VALU for 4 cells, chain of 5 dependent ops.  The four s(i,j)-2g values of a lane
// come from ONE ds_read_b64 of a per-wave LDS profile P[x][lane] = 4 x int16 (bank =
// lane, conflict-free); the column letters come as one ds_read_b128 per 4 steps from 4
// pre-shifted copies of a per-workgroup letter ring.
//
// Hand-off between strips (no barriers): every 4 steps each lane writes its 4 row-D values
// with one unconditional ds_write_b128 into a 128-slot "diagonal" ring at slot (group -
// lane); lane 63's values there survive 65 groups before later writes of lower lanes land
// on them.  The next strip's lane 0 reads 5 slots per 16-step block and injects the row
// above through the DPP add.  Producer/consumer order is kept with LDS progress words
// (LDS ops of one wave execute in order, so a progress word written after the data is
// never seen before the data).
//
// Workgroup = NS strip waves + 1 loader wave (letters, the previous super-strip's last row
// from HBM through 8-byte {epoch, value} granules, and the draining of the last strip's
// row to HBM).  Super-strips are handed out by an atomic ticket, so the launch cannot
// deadlock whatever the residency.  Every wait is bounded in wall time (error word set).
//
// Outputs (MODE):
//  * SPARSE : tileHrowMat / tileHcolMat exactly as gpu7/8/9 leave them, for tile height
//             tBy = 256*NS and a tile width tBx (multiple of 16, >= 64); padded cells use
//             letter 0 as the reference does (nwalign_gpu9_mlsp_diagdiagdiag.cu:469-478).
//             Single pairs, batches and mlsppt run on the K-rows kernel (nw_krow.hip);
//             this mode is reached with GSA_SPARSE_KERNEL=strip.
//  * SCORE  : score-only NW / SW with affine gaps (kModeScoreAG / kModeScoreSW, below; with a
//             linear gap: kModeScoreAGL / kModeScoreSWL, the same step without E' and F').
// Full matrices run on the one-row-per-lane kernel (nw_lane.hip).  This kernel's full-matrix
// modes (LDS staging + store waves; L2 output rings drained by copy workgroups) were measured
// slower and removed.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "nw_strip.h"

namespace gsa {

constexpr int kK = 4;               // rows per lane
static_assert(kWaveRows == 64 * kK, "rows per strip");
constexpr int kBLK = 16;            // wavefront steps per block
constexpr int kXR = 1024;           // letter ring (columns), per pre-shifted copy
// Copy m starts at m*kXCopy + kXSkew(m): with these bank offsets the 16 lanes of every
// ds_read_b128 lane group read 16 disjoint 4-bank slots (lane l reads copy (-l)&3).
constexpr int kXCopy = kXR * 4 + 256;
__host__ __device__ constexpr uint32_t xcopy_base(int m) { return (uint32_t)m * kXCopy + (m == 0 ? 0 : m == 1 ? 208 : m == 2 ? 144 : 80); }
constexpr int kRing = 128;          // hand-off ring slots (16 B) per strip boundary
constexpr int kBig = 0x3fffffff;    // "everything published"
// Every spin gives up after StripArgs::spin ticks of s_memrealtime (100 MHz) without progress
// (gsa_set_watchdog; default 1 s) and sets the error word.


extern __shared__ __attribute__((aligned(16))) char smem[];

typedef int int2v __attribute__((ext_vector_type(2)));
typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(smem + a); }
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(smem + a) = v; }
__device__ __forceinline__ int2v lds_ld2(uint32_t a) { return *(const int2v*)(smem + a); }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(smem + a); }
__device__ __forceinline__ void lds_st4(uint32_t a, int4v v) { *(int4v*)(smem + a) = v; }
// progress words: relaxed workgroup-scope atomics (no waits; a volatile access would make the
// compiler drain every outstanding global store around it)
__device__ __forceinline__ int flag_ld(uint32_t a)
{
    int* p = (int*)__builtin_assume_aligned(smem + a, 4);
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void flag_st(uint32_t a, int v)
{
    asm volatile("" ::: "memory");  // data writes are issued before the word (LDS executes in order)
    int* p = (int*)__builtin_assume_aligned(smem + a, 4);
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cbar() { asm volatile("" ::: "memory"); }

// Pointers read from the pair descriptors are global memory: every access goes through a
// pointer of the global address space, or it would become a flat instruction (which also
// counts against lgkmcnt and serialises against the LDS traffic of the hot loop).
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

struct Lds
{
    uint32_t xo, ring, zero, flags, prof, psz;
    uint32_t ring2;  // kModeScoreAG: the F' hand-off rings (same geometry as ring)
};

// flags: prog[i] @ 4i (ring i holds the row above strip i; valid for columns < prog[i]),
//        cons[i] @ 32+4i (ring i's reader no longer needs columns < cons[i]),
//        xo_cols @ 64 (letter ring valid for columns < xo_cols), ticket @ 68.
constexpr uint32_t kFProg = 0, kFCons = 32, kFXo = 64, kFTicket = 68;


template <int NS, int MODE>
__device__ __forceinline__ Lds lds_layout(int substsz)
{
    static_assert(NS >= 1 && NS <= 7, "flag layout");
    Lds L;
    L.psz = (uint32_t)(substsz + 1) * 512u;  // P[x][lane] = 4 x int16; row substsz = NEG
    L.xo = 0;
    L.ring = L.xo + 4 * kXCopy;
    L.ring2 = L.ring + (NS + 1) * kRing * 16;
    L.zero = L.ring2 + (is_score_mode(MODE) ? (NS + 1) * kRing * 16 : 0);
    L.flags = L.zero + 16;
    L.prof = L.flags + 128;
    return L;
}

#ifndef GSA_STRIP_SW
size_t strip_lds_bytes(int ns, int substsz, int mode)
{
    return (size_t)4 * kXCopy + (size_t)(ns + 1) * kRing * 16 * (is_score_mode(mode) ? 2 : 1) + 16 + 128 +
           (size_t)ns * (substsz + 1) * 512;
}
#endif

__device__ __forceinline__ bool err_set(const StripArgs& a)
{
    return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// letter byte-offset into the profile for column c given its loaded letter x
__device__ __forceinline__ int x_offset(const StripArgs& a, int c, int x)
{
    if (c <= 0 || c > a.Cp) return a.substsz * 512;  // NEG row
    if (c > a.C) return 0;                            // padding letter 0
    return ((unsigned)x < (unsigned)a.substsz ? x : 0) * 512;
}

__device__ __forceinline__ int load_letter(const StripArgs& a, int c) { return (c >= 1 && c <= a.C) ? G(a.seqX)[c] : 0; }

// ring slot / element of the lane-63 value of column c (written at step c+63, group (c+63)/4)
__device__ __forceinline__ uint32_t ring_elem(int c)
{
    const int gi = (c + 63) >> 2;
    return 16u * (uint32_t)((gi - 63) & (kRing - 1)) + 4u * (uint32_t)((c + 63) & 3);
}

// Hand-off: the row above is checked (fresh word) and the next block's halo loaded at step group
// kHopQ of a block.
constexpr int kHopQ = 2;

// ------------------------------------------------------------------------------------
// strip wave
// ------------------------------------------------------------------------------------
// Software pipeline (one wave, LDS reads execute in order and a single wave gets a fraction
// of the LDS rate, so every read is issued a whole block before its use):
//   block b computes with  S[b%2]  (issued during block b-1)  and  hv[b%2]  (halo, ditto);
//   during block b it issues  S[(b+1)%2] from letters L[(b+1)%2]  (read during block b-1),
//   letters L[b%2] for block b+2  and  hv[(b+1)%2].
template <int NS, int MODE>
__device__ __forceinline__ void strip_wave(const StripArgs& a, const Lds& L, int tk, int w, int lane)
{
    constexpr int TR = kWaveRows * NS;  // rows per super-strip
    // the lane index made opaque per ticket: otherwise the compiler hoists this wave's per-lane
    // LDS addresses out of the ticket loop into the kernel prologue, where the score modes'
    // register budget (256) cannot hold them all and 3 of them went to scratch
    asm volatile("" : "+v"(lane));
    const int g = a.g;
    const int Cp = a.Cp;
    const int r0 = tk * TR + kWaveRows * w + 1;  // first row of the strip
    const uint32_t F = L.flags;
    if (MODE != kModeSparse && r0 > a.R)
    {
        // nothing below the matrix: pass the (never read) hand-off through
        flag_st(F + kFProg + 4 * (w + 1), kBig);
        flag_st(F + kFCons + 4 * w, kBig);
        return;
    }

    // ---- profile P[x][lane] = 4 x int16 (s(row_k, x) - 2g), row substsz = NEG ----------
    const uint32_t my_prof = L.prof + (uint32_t)w * L.psz;
    {
        gptr<const int> srow[kK];
#pragma unroll
        for (int k = 0; k < kK; ++k)
        {
            const int r = r0 + kK * lane + k;
            int y = (r <= a.R) ? G(a.seqY)[r] : 0;
            y = ((unsigned)y < (unsigned)a.substsz) ? y : 0;
            srow[k] = G(a.subst) + y * a.substsz;
        }
        bool bad = false;
        for (int x = 0; x < a.substsz; ++x)
        {
            int v[kK];
#pragma unroll
            for (int k = 0; k < kK; ++k)
            {
                // LG: s - 2g;  AG (H' = H - (i+j)ge, diagonal carried as Hgo' = H' + d): s - 2ge - d
                v[k] = srow[k][x] - (is_score_mode(MODE) ? a.ge + a.go : 2 * g);
                bad |= (v[k] < -32767) || (v[k] > 32767);
            }
            int2v p;
            p.x = (v[0] & 0xffff) | (v[1] << 16);
            p.y = (v[2] & 0xffff) | (v[3] << 16);
            *(int2v*)(smem + my_prof + 512 * x + 8 * lane) = p;
        }
        *(int2v*)(smem + my_prof + 512 * a.substsz + 8 * lane) = int2v {(int)0x80008000u, (int)0x80008000u};
        if (bad) atomicOr(a.err, 2u);
    }

    const int NB = (Cp + 64 + kBLK - 1) / kBLK;  // blocks: lane 63 reaches column Cp
    const uint32_t laneoff = my_prof + 8u * lane;
    const int xm = (-lane) & 3;
    const uint32_t xo_base = L.xo + xcopy_base(xm);
    const int lanepos = (-lane - xm) >> 2;  // in 16-byte units
    auto xo_addr = [&](int t0) { return xo_base + 16u * (uint32_t)(((t0 >> 2) + lanepos) & (kXR / 4 - 1)); };
    const uint32_t ring_in = L.ring + (uint32_t)w * (kRing * 16);
    const uint32_t ring_out = L.ring + (uint32_t)(w + 1) * (kRing * 16);
    const uint32_t ring2_in = L.ring2 + (uint32_t)w * (kRing * 16);       // AG: F' of the row above
    const uint32_t ring2_out = L.ring2 + (uint32_t)(w + 1) * (kRing * 16);
    const uint32_t fin = F + kFProg + 4 * w, fcout = F + kFCons + 4 * (w + 1);

    // halo window of block b: lane-63 slots of the row above for groups 4b+15 .. 4b+19
    // (steps 16b+60 .. 16b+79 = columns 16b-3 .. 16b+16); lanes >= 1 read zeros.
    auto hv_load = [&](int b, int (&hv)[kBLK]) {
        int4v win[5];
#pragma unroll
        for (int j = 0; j < 5; ++j)
            win[j] = lds_ld4(lane == 0 ? ring_in + 16u * (uint32_t)((4 * b - 48 + j) & (kRing - 1)) : L.zero);
#pragma unroll
        for (int u = 0; u < kBLK; ++u) hv[u] = win[(u + 3) >> 2][(u + 3) & 3];
    };
    auto hvf_load = [&](int b, int (&hv)[kBLK]) {
        if constexpr (is_score_mode(MODE) && !is_lin_mode(MODE))  // F' (linear gaps: unused)
        {
            int4v win[5];
#pragma unroll
            for (int j = 0; j < 5; ++j)
                win[j] = lds_ld4(lane == 0 ? ring2_in + 16u * (uint32_t)((4 * b - 48 + j) & (kRing - 1)) : L.zero);
#pragma unroll
            for (int u = 0; u < kBLK; ++u) hv[u] = win[(u + 3) >> 2][(u + 3) & 3];
        }
    };
    auto letters_load = [&](int b, int4v (&lx)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) lx[q] = lds_ld4(xo_addr(16 * b + 4 * q));
    };
    auto raw_ld = [&](uint32_t ad) {
        return __hip_atomic_load((int*)__builtin_assume_aligned(smem + ad, 4), __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
    };

    // Block b may start once ring_out has room for it and (strip 0) the letters of block b+2 are
    // published.
    // The row above is checked separately, in the middle of block b, right before the halo of
    // block b+1 is loaded (pin_ok): checked late and with a fresh word, it costs the hand-off
    // ~20 steps less lag than a check at block start with a word read a block earlier.
    auto pin_ok = [&](int pin, int b) { return pin >= min(16 * b + 32, Cp + 1); };
    auto start_ok = [&](int pco, int pxo, int b) {
        bool ok = pco >= 16 * b - 307;
        if (w == 0) ok = ok && pxo >= min(16 * b + 48, Cp + 1);
        return ok;
    };
    auto ready = [&](int pin, int pco, int pxo, int b) { return pin_ok(pin, b) && start_ok(pco, pxo, b); };
    // bounded spin until ready(b); false on time-out / error
    auto wait_ready = [&](int& pin, int& pco, int& pxo, int b) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (!ready(pin, pco, pxo, b))
        {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || err_set(a))
            {
                atomicOr(a.err, 1u);
                return false;
            }
            pin = flag_ld(fin);
            pco = flag_ld(fcout);
            if (w == 0) pxo = flag_ld(F + kFXo);
        }
        return true;
    };

    // bounded spin until start_ok(b)
    auto wait_start = [&](int& pco, int& pxo, int b) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (!start_ok(pco, pxo, b))
        {
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || err_set(a))
            {
                atomicOr(a.err, 1u);
                return false;
            }
            pco = flag_ld(fcout);
            if (w == 0) pxo = flag_ld(F + kFXo);
        }
        return true;
    };

    // ---- prologue: halo of block 0, letters of blocks 0 and 1, S of block 0 ----
    int pin = flag_ld(fin), pco = flag_ld(fcout), pxo = (w == 0) ? flag_ld(F + kFXo) : 0;
    if (!wait_ready(pin, pco, pxo, -1)) return;
    cbar();
    int hvA[kBLK], hvB[kBLK], hfA[kBLK], hfB[kBLK];
    int4v lxA[4], lxB[4];
    int2v sA[kBLK], sB[kBLK];
    hv_load(0, hvA);
    hvf_load(0, hfA);
    letters_load(0, lxA);
    letters_load(1, lxB);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int u = 0; u < 4; ++u) sA[4 * q + u] = lds_ld2((uint32_t)lxA[q][u] + laneoff);

    // LG: H' of the 4 rows (0 = the shifted border).  AG: Hgo' of the 4 rows, E' of the 4 rows, F'
    // of row D, all -inf before the matrix (kNegAG: far from overflow, never the maximum)
    constexpr int kNegAG = -(1 << 29);
    constexpr int i0v = is_score_mode(MODE) ? kNegAG : 0;
    int A = i0v, B = i0v, Cc = i0v, D = i0v, dA = i0v;
    int EA = kNegAG, EB = kNegAG, EC = kNegAG, ED = kNegAG, FD = kNegAG;
    const int dd = (is_score_mode(MODE) && !is_lin_mode(MODE)) ? a.go - a.ge : 0;  // linear: d = 0
    // AG: the cell (R, C) lies in this strip iff r0 <= R < r0 + 256: lane, row, step of it
    const int rR = a.R - r0;
    const bool hasR = is_ag_mode(MODE) && rR >= 0 && rR < kWaveRows;
    const int laneR = rR >> 2, kR = rR & 3, tStar = a.C + laneR;
    // SW: floor of row k at the current step, H' >= -(i+j)ge (H >= 0).  Per row, the block's best
    // as H << 4 | (15 - step in block) (one max per step: the larger H, then the earlier step) and,
    // folded at each block end, the best H with the step it first appeared.  Rows below R start at
    // a best nothing beats.  Columns past C are never the maximum: their E/F chains pay go < 0.
    int zA = 0, zB = 0, zC = 0, zD = 0, pA = 0, pB = 0, pC = 0, pD = 0;
    int bA = 0, bB = 0, bC = 0, bD = 0, tA = 0, tB = 0, tC = 0, tD = 0;
    if constexpr (is_sw_mode(MODE))
    {
        const int rb = r0 + kK * lane;  // row of k = A; i + j = rb + k + (t - lane)
        constexpr int kOff = 0x7fffffff;
        zA = -(rb - lane) * a.ge;
        zB = zA - a.ge;
        zC = zB - a.ge;
        zD = zC - a.ge;
        bA = (rb <= a.R) ? 0 : kOff;
        bB = (rb + 1 <= a.R) ? 0 : kOff;
        bC = (rb + 2 <= a.R) ? 0 : kOff;
        bD = (rb + 3 <= a.R) ? 0 : kOff;
    }
    int cap[kK] = {0, 0, 0, 0};
    int rpin = pin, rpco = pco, rpxo = pxo;  // progress words as loaded, checked a block later

    // compute block b with (scur, hvcur); issue snext from lnext (letters of b+1), letters of
    // b+2 into lfree, and hvnext
    auto block = [&](int b, int2v (&scur)[kBLK], int2v (&snext)[kBLK], int4v (&lnext)[4], int4v (&lfree)[4],
                     int (&hvcur)[kBLK], int (&hvnext)[kBLK], int (&hfcur)[kBLK], int (&hfnext)[kBLK], auto capT) {
        constexpr bool CAP = decltype(capT)::value;
        const int cb = (CAP && MODE == kModeSparse) ? ((16 * b) / a.tBx) * a.tBx : 0;
#pragma unroll
        for (int q = 0; q < 4; ++q)
        {
            const int t0 = 16 * b + 4 * q;
            lfree[q] = lds_ld4(xo_addr(t0 + 32));
#pragma unroll
            for (int u = 0; u < 4; ++u) snext[4 * q + u] = lds_ld2((uint32_t)lnext[q][u] + laneoff);
            int Xd[4], Fd[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
            {
                const int2v sv = scur[4 * q + u];
                if constexpr (is_score_mode(MODE))
                {
                    // Gotoh in H' = H - (i+j)ge: E'(k,c) = max(E'(k,c-1), Hgo'(k,c-1)),
                    // F'(k,c) = max(F'(k-1,c), Hgo'(k-1,c)), H' = max3(Hgo'diag + s'', E', F'),
                    // Hgo' = H' + d; the row above comes from lane l-1 (DPP) or the halo
                    const int upH = shr1z(D) + hvcur[4 * q + u];
                    constexpr bool LIN = is_lin_mode(MODE);  // d = 0: E' = H' of the left cell, F' <= Hgo' above
                    const int upF = LIN ? 0 : shr1z(FD) + hfcur[4 * q + u];
                    const int eA = LIN ? A : max(EA, A), eB = LIN ? B : max(EB, B);
                    const int eC = LIN ? Cc : max(EC, Cc), eD = LIN ? D : max(ED, D);
                    // SW: H >= 0 enters as F' >= floor (the max3 that forms F'): H = max(0, diag,
                    // E, F) exactly, and a clamped F passes on at most ge <= 0, below the next floor
                    // linear gaps (d = 0): E' <= H' and F' <= H' hold by induction, so E' is the left
                    // H', F' of a row the H' above it, and only the SW floor stays
                    constexpr bool SW = is_sw_mode(MODE);
                    const int fA = LIN ? (SW ? max(upH, zA) : upH) : SW ? max(max(upF, upH), zA) : max(upF, upH);
                    const int hA = max(max(dA + (int)(short)sv.x, eA), fA);
                    const int nA = hA + dd;
                    const int fB = LIN ? (SW ? max(nA, zB) : nA) : SW ? max(max(fA, nA), zB) : max(fA, nA);
                    const int hB = max(max(A + (sv.x >> 16), eB), fB);
                    const int nB = hB + dd;
                    const int fC = LIN ? (SW ? max(nB, zC) : nB) : SW ? max(max(fB, nB), zC) : max(fB, nB);
                    const int hC = max(max(B + (int)(short)sv.y, eC), fC);
                    const int nC = hC + dd;
                    const int fD = LIN ? (SW ? max(nC, zD) : nC) : SW ? max(max(fC, nC), zD) : max(fC, nC);
                    const int hD = max(max(Cc + (sv.y >> 16), eD), fD);
                    const int nD = hD + dd;
                    if constexpr (SW)
                    {
                        const int bu = 15 - 4 * q - u;
                        pA = max(pA, ((hA - zA) << 4) | bu);
                        pB = max(pB, ((hB - zB) << 4) | bu);
                        pC = max(pC, ((hC - zC) << 4) | bu);
                        pD = max(pD, ((hD - zD) << 4) | bu);
                        zA -= a.ge;
                        zB -= a.ge;
                        zC -= a.ge;
                        zD -= a.ge;
                    }
                    if constexpr (CAP)
                    {
                        if (t0 + u == tStar && lane == laneR)
                            G(a.agResult)[0] = (kR == 0 ? hA : kR == 1 ? hB : kR == 2 ? hC : hD) + (a.R + a.C) * a.ge;
                    }
                    dA = upH;
                    A = nA;
                    B = nB;
                    Cc = nC;
                    D = nD;
                    EA = eA;
                    EB = eB;
                    EC = eC;
                    ED = eD;
                    FD = fD;
                    Xd[u] = nD;
                    Fd[u] = fD;
                    continue;
                }
                const int up = shr1z(D) + hvcur[4 * q + u];
                const int na = max(max(dA + (int)(short)sv.x, up), A);
                const int nb = max(max(A + (sv.x >> 16), na), B);
                const int nc = max(max(B + (int)(short)sv.y, nb), Cc);
                const int nd = max(max(Cc + (sv.y >> 16), nc), D);
                dA = up;
                A = na;
                B = nb;
                Cc = nc;
                D = nd;
                Xd[u] = nd;
                if constexpr (CAP)
                {
                    const bool hit = (t0 + u - lane) == cb;
                    cap[0] = hit ? na : cap[0];
                    cap[1] = hit ? nb : cap[1];
                    cap[2] = hit ? nc : cap[2];
                    cap[3] = hit ? nd : cap[3];
                }
            }
            // hand-off: row D of 4 steps, slot (group - lane)
            lds_st4(ring_out + 16u * (uint32_t)(((t0 >> 2) - lane) & (kRing - 1)), int4v {Xd[0], Xd[1], Xd[2], Xd[3]});
            if constexpr (is_score_mode(MODE) && !is_lin_mode(MODE))
                lds_st4(ring2_out + 16u * (uint32_t)(((t0 >> 2) - lane) & (kRing - 1)), int4v {Fd[0], Fd[1], Fd[2], Fd[3]});
            if (q == kHopQ - 1) rpin = raw_ld(fin);
            // SW reads its halo at block start (one halo buffer live: no spills, 50k 7.64 ->
            // 7.01 ms); NW-AG keeps the prefetch (5.13 vs 5.46 ms; profiles/r01_score_jit.txt)
            if (q == kHopQ && !is_sw_mode(MODE))
            {
                // halo of the next block, once the row above covers it
                int pn = __builtin_amdgcn_readfirstlane(rpin);
                if (!pin_ok(pn, b))
                {
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    while (!pin_ok(pn = flag_ld(fin), b))
                    {
                        __builtin_amdgcn_s_sleep(1);
                        if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || err_set(a))
                        {
                            atomicOr(a.err, 1u);
                            break;
                        }
                    }
                }
                cbar();
                hv_load(b + 1, hvnext);
                hvf_load(b + 1, hfnext);
                flag_st(F + kFCons + 4 * w, 16 * (b + 1) - 3);  // after the halo reads (in order)
            }
            if (q == 0)
            {
                rpco = raw_ld(fcout);
                if (w == 0) rpxo = raw_ld(F + kFXo);
            }
        }
        if constexpr (is_sw_mode(MODE))
        {
            auto fold = [&](int& p, int& best, int& tb) {
                const int v = p >> 4;
                const bool up = v > best;
                best = up ? v : best;
                tb = up ? 16 * b + 15 - (p & 15) : tb;
                p = 0;
            };
            fold(pA, bA, tA);
            fold(pB, bB, tB);
            fold(pC, bC, tC);
            fold(pD, bD, tD);
        }
        if constexpr (CAP && MODE == kModeSparse)
        {
            if (16 * b + 15 == cb + 63)
            {
                // header column of tile (tk, cb/tBx): entries 256w+4l+1 .. +4 (rows r0+4l+k)
                const int jT = cb / a.tBx;
                const int rr = r0 + kK * lane;
                int4a v = int4a {cap[0] + (rr + cb) * g, cap[1] + (rr + 1 + cb) * g, cap[2] + (rr + 2 + cb) * g,
                                 cap[3] + (rr + 3 + cb) * g};
                *(gptr<int4a>)(G(a.hcol) + ((size_t)tk * a.tcols + jT) * (size_t)(a.tBy + 1) + kWaveRows * w + kK * lane + 1) = v;
            }
        }
        flag_st(F + kFProg + 4 * (w + 1), b + 1 == NB ? kBig : 16 * (b + 1) - 63);
    };

    auto run_block = [&](int b, int2v (&scur)[kBLK], int2v (&snext)[kBLK], int4v (&lnext)[4], int4v (&lfree)[4],
                         int (&hvcur)[kBLK], int (&hvnext)[kBLK], int (&hfcur)[kBLK], int (&hfnext)[kBLK]) {
        pco = __builtin_amdgcn_readfirstlane(rpco);
        pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
        if (!start_ok(pco, pxo, b))
        {
            if (!wait_start(pco, pxo, b)) return false;
        }
        if constexpr (is_sw_mode(MODE))
        {
            // halo of this block (block 0's came with the prologue), once the row above covers it
            if (b > 0)
            {
                int pn = __builtin_amdgcn_readfirstlane(rpin);
                if (!pin_ok(pn, b - 1))
                {
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    while (!pin_ok(pn = flag_ld(fin), b - 1))
                    {
                        __builtin_amdgcn_s_sleep(1);
                        if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || err_set(a))
                        {
                            atomicOr(a.err, 1u);
                            return false;
                        }
                    }
                }
                cbar();
                hv_load(b, hvcur);
                hvf_load(b, hfcur);
                flag_st(F + kFCons + 4 * w, 16 * b - 3);  // after the halo reads (in order)
            }
        }
        cbar();
        bool capblk = false;
        if constexpr (MODE == kModeSparse)
        {
            const int jT = (16 * b) / a.tBx;
            capblk = jT >= 1 && jT < a.tcols && 16 * b - jT * a.tBx < 64;
        }
        if constexpr (is_ag_mode(MODE)) capblk = hasR && (tStar >> 4) == b;
        if (capblk)
            block(b, scur, snext, lnext, lfree, hvcur, hvnext, hfcur, hfnext, std::integral_constant<bool, true>());
        else
            block(b, scur, snext, lnext, lfree, hvcur, hvnext, hfcur, hfnext, std::integral_constant<bool, false>());
        return true;
    };

    for (int b = 0; b < NB; b += 2)
    {
        if (!run_block(b, sA, sB, lxB, lxA, hvA, hvB, hfA, hfB)) return;
        if (b + 1 < NB && !run_block(b + 1, sB, sA, lxA, lxB, hvB, hvA, hfB, hfA)) return;
    }
    if constexpr (is_sw_mode(MODE))
    {
        // this lane's best cell, first in row-major order: rows in order, first step per row
        const unsigned long long W = (unsigned long long)a.C + 1, mask = (1ull << a.idxBits) - 1;
        const int bv[kK] = {bA, bB, bC, bD}, tv[kK] = {tA, tB, tC, tD};
        unsigned long long key = 0;
        bool big = false;
#pragma unroll
        for (int k = 0; k < kK; ++k)
        {
            // a score >= 2^26 (before the packing could wrap: one cell adds < 2^16) -> the host's row scan
            big |= bv[k] >= (1 << 26) && r0 + kK * lane + k <= a.R;
            if (bv[k] > 0 && r0 + kK * lane + k <= a.R)
            {
                const unsigned long long idx = (unsigned long long)(r0 + kK * lane + k) * W + (unsigned long long)(tv[k] - lane);
                const unsigned long long kk = ((unsigned long long)bv[k] << a.idxBits) | (mask - idx);
                key = kk > key ? kk : key;
            }
        }
        if (key) atomicMax(a.swBest, key);
        if (big) atomicOr((unsigned*)a.agResult, 1u);  // the AG result word, unused by SW
    }
    flag_st(F + kFCons + 4 * w, kBig);
}

// ------------------------------------------------------------------------------------
// loader wave: letters in, the previous super-strip's last row in, our last row out
// ------------------------------------------------------------------------------------
template <int NS, int MODE>
__device__ __forceinline__ void loader_wave(const StripArgs& a, const Lds& L, int tk, int lane)
{
    const int Cp = a.Cp;
    const int nCh = (Cp + 1 + 63) / 64;  // 64-column chunks covering columns 0..Cp
    const uint32_t F = L.flags;
    const uint32_t ring0 = L.ring;
    // AG: ticket 0 is fed too, from the border row (Hgo' = d at column 0, 2d after it; F' = -inf)
    const bool feed = tk > 0 || is_score_mode(MODE);
    const unsigned long long* gprev = a.gran + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
    unsigned long long* gout = a.gran + (size_t)tk * a.granStride;
    const unsigned long long* gprev2 = a.gran2 + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;  // AG: F'
    unsigned long long* gout2 = a.gran2 + (size_t)tk * a.granStride;
    const uint32_t ring20 = L.ring2;
    const bool pub = tk + 1 < a.nTickets;
    constexpr int TR = kWaveRows * NS;
    const int hrowg = (tk + 1) * TR;  // global row of our last row
    // strips below the matrix (score modes, last super-strip) pass BIG through: the last
    // strip that computes is the one whose progress bounds the letter ring
    const int nAct = (MODE != kModeSparse) ? max(1, min(NS, (a.R - tk * TR + kWaveRows - 1) / kWaveRows)) : NS;
    const uint32_t ringN = L.ring + (uint32_t)nAct * (kRing * 16);
    const uint32_t ringN2 = L.ring2 + (uint32_t)nAct * (kRing * 16);
    int kx = 0;                       // next letter chunk (64 columns)
    int hnext = feed ? 0 : Cp + 1;    // next column of the row above to feed into ring 0
    int dnext = 0;                    // next column of our last row to drain
    int xl = load_letter(a, lane);
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    while (kx < nCh || hnext <= Cp || dnext <= Cp)
    {
        bool moved = false;
        const int pl = flag_ld(F + kFProg + 4 * nAct);
        const int cs0 = flag_ld(F + kFCons + 0);
        // (1) letters of chunk kx, once the last strip no longer reads the columns they replace
        if (kx < nCh && 64 * kx <= pl + 960)
        {
            const int c = 64 * kx + lane;
            const int off = x_offset(a, c, xl);
#pragma unroll
            for (int m = 0; m < 4; ++m) lds_st(L.xo + xcopy_base(m) + 4u * (uint32_t)((c - m) & (kXR - 1)), off);
            ++kx;
            xl = load_letter(a, 64 * kx + lane);
            flag_st(F + kFXo, kx == nCh ? kBig : 64 * kx);
            moved = true;
        }
        // (2) the row above strip 0: the prefix of granules already published by the previous
        //     super-strip -> ring 0 (ring 0 holds 512 columns: stay within 448 of strip 0)
        if (hnext <= Cp && cs0 >= hnext + 63 - 511)
        {
            const int c = hnext + lane;
            const bool in = c <= Cp;
            unsigned long long q = 0ull, q2 = 0ull;
            bool good;
            if (is_score_mode(MODE) && tk == 0)
            {
                // row 0 in the shifted space: global H'(0,c) = d for c >= 1 (0 at c = 0), local
                // H'(0,c) = -c*ge (H = 0); carried as Hgo' = H' + d
                const int dd = a.go - a.ge;
                q = (uint32_t)(is_sw_mode(MODE) ? dd - c * a.ge : (c == 0 ? dd : 2 * dd));
                q2 = (uint32_t)(-(1 << 29));
                good = in;
            }
            else
            {
                q = in ? __hip_atomic_load(gprev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                good = in && (uint32_t)(q >> 32) == a.epoch;
                if constexpr (is_score_mode(MODE) && !is_lin_mode(MODE))
                {
                    q2 = in ? __hip_atomic_load(gprev2 + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
                    good = good && (uint32_t)(q2 >> 32) == a.epoch;
                }
            }
            const uint64_t badm = __ballot(!good);
            const int n = badm ? __builtin_ctzll(badm) : 64;  // granules arrive in column order
            if (n > 0)
            {
                if (lane < n) lds_st(ring0 + ring_elem(c), (int)(uint32_t)q);
                if (is_score_mode(MODE) && !is_lin_mode(MODE) && lane < n) lds_st(ring20 + ring_elem(c), (int)(uint32_t)q2);
                hnext += n;
                flag_st(F + kFProg + 0, hnext > Cp ? kBig : hnext);
                moved = true;
            }
        }
        // (3) drain whatever prefix of our last row is complete: granules for the next
        //     super-strip, sparse hrow
        const int avail = min(pl, Cp + 1);
        if (dnext < avail)
        {
            const int c = dnext + lane;
            if (c < avail)
            {
                const int v = lds_ld(ringN + ring_elem(c));
                if (pub)
                    __hip_atomic_store(gout + c, ((unsigned long long)a.epoch << 32) | (uint32_t)v, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if constexpr (is_score_mode(MODE) && !is_lin_mode(MODE))
                {
                    const int v2 = lds_ld(ringN2 + ring_elem(c));
                    if (pub)
                        __hip_atomic_store(gout2 + c, ((unsigned long long)a.epoch << 32) | (uint32_t)v2, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                }
                if constexpr (MODE == kModeSparse)
                {
                    if (tk + 1 < a.trows)
                    {
                        const int hv = v + (hrowg + c) * a.g;
                        const int jT = c / a.tBx, jj = c - jT * a.tBx;
                        const size_t rowbase = (size_t)(tk + 1) * a.tcols;
                        if (jT < a.tcols) G(a.hrow)[(rowbase + jT) * (size_t)(a.tBx + 1) + jj] = hv;
                        if (jj == 0 && jT > 0) G(a.hrow)[(rowbase + jT - 1) * (size_t)(a.tBx + 1) + a.tBx] = hv;
                        if (jj == 0 && jT > 0 && jT < a.tcols) G(a.hcol)[(rowbase + jT) * (size_t)(a.tBy + 1)] = hv;
                    }
                }
            }
            dnext = min(dnext + 64, avail);
            flag_st(F + kFCons + 4 * NS, dnext > Cp ? kBig : dnext);
            moved = true;
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
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// A pair descriptor into scalar registers: the loads go through the vector path (the compiler
// cannot prove the descriptor array unclobbered after the ticket atomic), every word is then
// made wave-uniform so nothing per-pair lives in VGPRs.
__device__ __forceinline__ PairDesc load_desc(const PairDesc* p)
{
    static_assert(sizeof(PairDesc) % 4 == 0, "descriptor words");
    constexpr int N = sizeof(PairDesc) / 4;
    const int* w = (const int*)p;
    union
    {
        int v[N];
        PairDesc d;
    } u;
#pragma unroll
    for (int k = 0; k < N; ++k) u.v[k] = __builtin_amdgcn_readfirstlane(G(w)[k]);
    return u.d;
}


// waves per workgroup: NS strips + loader
template <int NS>
constexpr int kWaves = NS + 1;

template <int NS, int MODE>
__global__ void __launch_bounds__(64 * (NS + 1)) nw_strip_kernel(StripArgs a)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const Lds L = lds_layout<NS, MODE>(a.substsz);
    const uint32_t F = L.flags;
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) lds_st(F + kFTicket, (err_set(a) ? a.nTicketsTotal : (int)atomicAdd(a.ticket, 1u)));
        __syncthreads();
        const int tkg = __builtin_amdgcn_readfirstlane(lds_ld(F + kFTicket));
        if (tkg >= a.nTicketsTotal) break;
        // pair of this ticket: the batch schedule, or the last descriptor with ticketBase <= tkg
        // (binary search, uniform)
        int lo = 0, tks = -1;
        if (a.sched)
        {
            lo = __builtin_amdgcn_readfirstlane(a.sched[2 * tkg]);
            tks = __builtin_amdgcn_readfirstlane(a.sched[2 * tkg + 1]);
        }
        else
        {
            int hi = a.nPairs - 1;
            while (lo < hi)
            {
                const int mid = (lo + hi + 1) >> 1;
                if (__builtin_amdgcn_readfirstlane(a.pairs[mid].ticketBase) <= tkg)
                    lo = mid;
                else
                    hi = mid - 1;
            }
        }
        const PairDesc d = load_desc(a.pairs + lo);
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
        pa.gran2 = a.gran2 + d.granOff;
        pa.granStride = gran_stride(d.Cp);
        const int tk = (tks >= 0) ? tks : tkg - d.ticketBase;
        // per-super-strip state: letter ring = NEG, ring 0 = row 0 (H' = 0), progress words
        for (int k = threadIdx.x; k < kXCopy; k += 64 * kWaves<NS>) lds_st(L.xo + 4 * k, pa.substsz * 512);
        for (int k = threadIdx.x; k < kRing * 4; k += 64 * kWaves<NS>)
        {
            // score modes: Hgo' and F' of the row above = -inf past the columns the loader feeds
            lds_st(L.ring + 4 * k, is_score_mode(MODE) ? -(1 << 29) : 0);
            if constexpr (is_score_mode(MODE)) lds_st(L.ring2 + 4 * k, -(1 << 29));
        }
        if (threadIdx.x < 4) lds_st(L.zero + 4 * threadIdx.x, 0);
        if (threadIdx.x < 8)
        {
            // nothing valid yet: -64 < every column a lane can touch (lane 63 starts at -63)
            lds_st(F + kFProg + 4 * threadIdx.x, (threadIdx.x == 0 && tk == 0 && !is_score_mode(MODE)) ? kBig : -64);
            lds_st(F + kFCons + 4 * threadIdx.x, 0);
        }
        if (threadIdx.x == 0) lds_st(F + kFXo, 0);
        __syncthreads();
        if (w == NS)
            loader_wave<NS, MODE>(pa, L, tk, lane);
        else
        {
            __builtin_amdgcn_s_setprio(3);
            strip_wave<NS, MODE>(pa, L, tk, w, lane);
            __builtin_amdgcn_s_setprio(0);
        }
    }
}

// Headers: row 0 / column 0 of the full matrix; for the sparse matrices the header row of
// tile row 0 (Kernel A of nwalign_gpu9_mlsp_diagdiagdiag.cu:15-63), the header column of
// tile column 0 and entry 0 of tile row 0's header columns (all plain multiples of g).
// grid.y = pair of the batch.
#ifndef GSA_STRIP_SW
__global__ void nw_headers_kernel(StripArgs a, int mode)
{
    const PairDesc& d = a.pairs[blockIdx.y];
    const gptr<int> score = G(d.score);
    const gptr<int> hrow = G(d.hrow);
    const gptr<int> hcol = G(d.hcol);
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (mode == kModeFull)
    {
        if (tid <= d.C) score[tid] = (int)tid * a.g;
        if (tid >= 1 && tid <= d.R) score[(size_t)tid * (size_t)d.ld] = (int)tid * a.g;
    }
    else
    {
        const int64_t nrow = (int64_t)d.tcols * (a.tBx + 1);
        const int64_t ncol = (int64_t)d.trows * (a.tBy + 1);
        if (tid < nrow)
        {
            const int jT = (int)(tid / (a.tBx + 1)), jj = (int)(tid % (a.tBx + 1));
            hrow[tid] = (jT * a.tBx + jj) * a.g;
            if (jj == 0) hcol[(size_t)jT * (size_t)(a.tBy + 1)] = jT * a.tBx * a.g;
        }
        if (tid < ncol)
        {
            const int iT = (int)(tid / (a.tBy + 1)), e = (int)(tid % (a.tBy + 1));
            hcol[((size_t)iT * d.tcols) * (size_t)(a.tBy + 1) + e] = (iT * a.tBy + e) * a.g;
        }
    }
}
#endif

template <int NS, int MODE>
static hipError_t launch_strip(const StripArgs& a, int grid, hipStream_t stream)
{
    const size_t lds = strip_lds_bytes(NS, a.substsz, MODE);
    auto kern = nw_strip_kernel<NS, MODE>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (grid <= 0)
    {
        // every workgroup that can be resident at once: a batch keeps them all busy
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * kWaves<NS>, lds);
        if (e == hipSuccess) e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        grid = std::max(1, std::min(a.nTicketsTotal, std::max(1, per_cu) * cus));
    }
    if ((e = record_foot((const void*)kern, lds, 64 * kWaves<NS>, grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kWaves<NS>), lds, stream, a);
    return hipGetLastError();
}

#ifndef GSA_STRIP_SW
thread_local LaunchFoot g_last_foot {};

hipError_t record_foot(const void* kern, size_t lds, int threads, int grid)
{
    hipFuncAttributes at {};
    int per_cu = 0, dev = 0, cus = 0;
    hipError_t e = hipFuncGetAttributes(&at, kern);
    if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, threads, lds);
    if (e == hipSuccess) e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    g_last_foot.lds_per_wg = (long long)at.sharedSizeBytes + (long long)lds;
    g_last_foot.scratch_per_lane = (long long)at.localSizeBytes;
    g_last_foot.regs_per_lane = (long long)at.numRegs;
    g_last_foot.threads_per_wg = threads;
    g_last_foot.active_wgs = std::min<long long>(grid, (long long)std::max(1, per_cu) * cus);
    return hipSuccess;
}

hipError_t launch_headers(const StripArgs& a, int mode, long long maxWork, hipStream_t stream)
{
    int blocks = (int)((maxWork + 255) / 256);
    hipLaunchKernelGGL(nw_headers_kernel, dim3(std::max(1, blocks), a.nPairs), dim3(256), 0, stream, a, mode);
    return hipGetLastError();
}

hipError_t launch_strip_sw(const StripArgs& a, int grid, hipStream_t stream);

hipError_t launch_strip_fill(const StripArgs& a, int mode, int grid, hipStream_t stream)
{
    if (mode == kModeScoreAG) return launch_strip<kSparseNS, kModeScoreAG>(a, grid, stream);
    if (mode == kModeScoreAGL) return launch_strip<kSparseNS, kModeScoreAGL>(a, grid, stream);
    if (mode == kModeScoreSWL) return launch_strip<kSparseNS, kModeScoreSWL>(a, grid, stream);
    if (mode == kModeScoreSW) return launch_strip_sw(a, grid, stream);
    if (mode == kModeSparse) return launch_strip<kSparseNS, kModeSparse>(a, grid, stream);
    return hipErrorInvalidValue;  // full matrices: launch_lane_fill (nw_lane.hip)
}
#else
// nw_strip_sw.hip: the SW score instance in a translation unit of its own (its own scheduler flags)
hipError_t launch_strip_sw(const StripArgs& a, int grid, hipStream_t stream)
{
    return launch_strip<kSparseNS, kModeScoreSW>(a, grid, stream);
}
#endif

}  // namespace gsa
