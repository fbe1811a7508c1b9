// nw_krow.hip -- NW-LG sparse (mlsp tile-header) fill with K rows per lane (K = 2 or 4),
// hand-written wave64 HIP for gfx950 (MI355X).
//
// Replaces the sparse family NwAlign_Gpu7..9 (nwalign_gpu9_mlsp_diagdiagdiag.cu:368-722, kernels
// :15-360) for single pairs and has their output contract: tileHrowMat / tileHcolMat, tile-major
// k = tcols*iT + jT, 1+tBx resp. 1+tBy ints per tile, element 0 the corner, the padded region
// computed with letter 0 (nwalign_gpu9_mlsp_diagdiagdiag.cu:147-171, 471-478).  Recurrence of
// UpdateScore (nwalign_cpu1_st_row.cpp:4-10).
//
// Cost model of one pair.  The fill is a wavefront: strip waves of 64K rows (lane l owns rows
// r0+Kl .. r0+Kl+K-1 and at step t works on column t-l) follow each other ~6 blocks of 16 steps
// apart (the 64-lane skew, one block of hand-off granularity, the progress check), so a pair
// takes (C/16 + 6 * R/(64K)) block times.  One wave issues at most one VALU per ~4.5 cycles, so
// the 2K+1 VALU of a step cost ~41 cycles at K = 4 whatever the dependency chain (splitting the
// lane's rows into two groups a column apart halves the chain and changes nothing); the LDS
// side work of a block (16 profile reads, 4 halo reads, 4 hand-off writes, 5 progress words)
// costs ~12-40 cycles per instruction of the wave's time and, with the header-column capture
// and the block's scalar control, about as much as the 16 steps (tools/ubench/lds_ubench.hip,
// profiles/r02_krow_breakdown.txt, profiles/r02_krow_probes.txt).  K = 4 halves the strips of
// K = 2 for a block ~25 % longer.
//
// Step, shifted values H' = H - (i+j)*g (borders 0), K+1 dependent VALU + K adds:
//     up    = dpp_shr1(H[K-1]) + halo    lane 0: H'(row above, c) from the ring; others + 0
//     H[0]' = max3(D + q0, up, H[0])     D = up of the previous step (= H'(r0+Kl-1, c-1))
//     H[k]' = max3(H[k-1] + qk, H[k-1]', H[k])
// q = s(y, X[c]) - 2g (int16) from a per-workgroup column profile in LDS: two copies shifted by
// one column, dword d of copy p holding columns (2d-p, 2d-p+1), so every lane reads its 16 columns
// of a block as 8 aligned dwords at base + immediate offsets (copy = lane parity): no VALU
// addressing, 8*K/2 ds_read2 per block; the halves are taken by SDWA operands of the adds.
//
// Sparse output.  Header rows (the last row of a tile row) are the last row of a ticket: the
// drain wave writes them with the granules.  Header columns are captured by the strips: in a
// block whose 79-column window holds a tile boundary, each lane picks its (H[0..K-1]) at its
// boundary step with a 4-level v_cndmask tree over the block's 16 steps and stores K ints.
//
// Hand-off between strips: at the end of block b lane 63 writes its old H[K-1] (columns t-64 of
// the block's 16 steps) into the next strip's ring; lane 0 of the next strip reads block b's 16
// halo values at the start of block b.  Both run under an exec mask set and restored inside one
// asm block (no divergent branch splits the block).  LDS progress words keep the order (a wave's
// LDS operations execute in order).  Between
// super-strips (workgroups) the drain wave moves the last row through 8-byte {epoch, H'}
// granules in HBM (sc1 atomics), polled by the next super-strip's loader wave
// (MI355X_MICROARCH.md, handoff-1to1).  Every wait is bounded (StripArgs::spin, error word).
#ifndef GSA_PROBE_P1
#define GSA_PROBE_P1 0  // diagnostic builds only (tools/r06_xprobe_build.sh)
#endif
#ifndef GSA_FX_VMCNT
// fused full fill: a strip publishes every 16 blocks what its stores older than its last GSA_FX_VMCNT
// vector-memory operations cover (>= 4 per block: blocks <= b - GSA_FX_VMCNT / 4)
#define GSA_FX_VMCNT 16
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_expand.h"
#include "nw_krow.h"
#ifdef GSA_KROW_XR
#include "nw_expand_dev.h"  // the fused fill's expansion tasks
#endif

namespace gsa {
namespace {

// Column profile, int16 (Q8 = false): 2 copies, dword d of copy p = columns (2d-p, 2d-p+1); int8
// (Q8): 4 copies, dword d of copy p = columns 4d-p .. 4d-p+3, so a lane reads its 16 columns of a row
// as 4 aligned dwords (2 ds_read2_b32 instead of 4: 100k 5.51 -> 5.30 ms) -- used when every
// s - 2g fits int8, the kernel falling back to int16 otherwise (uniform, decided in its prologue).
// dwords per profile row: the ring + a guard, == 0 mod 32 (the row letter never moves a lane's bank)
__host__ __device__ constexpr int kr_qrs(int lw, bool q8 = false) { return (q8 ? lw / 4 : lw / 2) + 32; }
// copy p at p * kr_copy1.  int16: copy 1 starts 16 dwords past a multiple of 32 (lanes 2m and 2m+1
// read the same dword index d, so copy 1 sits in the other half of the banks); int8: copies 8 banks
// apart (lanes 4m+p read the same index in copy p: 8 m's x 4 copies = 32 banks per 32-lane group)
__host__ __device__ constexpr uint32_t kr_copy1(int lw, int substsz, bool q8 = false)
{
    return (uint32_t)substsz * kr_qrs(lw, q8) + (q8 ? 8u : 16u);
}
// dwords of the profile region
__host__ __device__ constexpr uint32_t kr_qdwords(int lw, int substsz, bool q8)
{
    return q8 ? 4u * kr_copy1(lw, substsz, true) : kr_copy1(lw, substsz) + (uint32_t)substsz * kr_qrs(lw) + 16u;
}
constexpr int kBlk = 16;          // steps per block
constexpr int kHalo = kBlk / 4;   // halo registers (int4) per block
constexpr int kRing = 512;        // hand-off ring elements per strip boundary (power of 2)
constexpr int kBig = 0x3fffffff;  // "everything published"
constexpr int kSubRow = 36;       // dwords per subT row (32 letters + 4)
constexpr int kBatch = 128;       // profile columns the loader adds per pass (2 per lane)
// Progress words in 8-byte slots, slot s (s = -1 .. NS) at byte 8(s+1) = {prog[s+1], cons[s]}:
// prog[i] (ring i holds elements < prog[i]) is written by strip i-1 (the loader for i = 0),
// cons[i] (ring i's reader no longer needs elements < cons[i]) by strip i (the drain wave for
// i = NS), so a strip publishes both of its words with ONE 8-byte write, and reads the two it
// waits on -- prog[w] in slot w-1 and cons[w+1] in slot w+1 -- with ONE ds_read2_b64.  Slot -1's
// second word is xo (the profile holds columns < xo), which strip 0 reads in the same read.
__host__ __device__ constexpr uint32_t kr_prog(int i) { return 8u * (uint32_t)i; }
__host__ __device__ constexpr uint32_t kr_cons(int i) { return 8u * (uint32_t)(i + 1) + 4u; }
constexpr uint32_t kFXo = 4, kFTicket = 132;
// mlsppt: strip w's header columns of tile columns < word are in memory (kBig: all), at kFCap + 4w
constexpr uint32_t kFCap = 160;
// the fused fill (PT 3): its strips stage their row-64m segments in LDS (kXD blocks deep per strip,
// after the progress words) for a storer wave, so no strip issues a row-buffer store.  Words at
// kr_xwords: [0, NS) blocks staged, [NS, 2NS) blocks stored (slots free), [2NS, 3NS) header columns
// of boundaries < the word in memory (kXDone: all); the data at kr_xdata: 64 bytes per (strip,
// slot, row 64j).
constexpr int kXD = 32;
constexpr int kLedgerWords = 10;  // GSA_STAMPS words per strip of a K-rows fill (gsa_debug_stamps)
#ifndef GSA_KR_BLOCK_LEDGER
#define GSA_KR_BLOCK_LEDGER 0
#endif
// the strip ledger (GSA_STAMPS=1 in a GSA_KR_LEDGER build, tools/r06_ledger.py): its counters cost the
// production instances SGPRs (the headline's spills 10 -> 24), so they exist in diagnostic builds only
#ifndef GSA_KR_LEDGER
#define GSA_KR_LEDGER GSA_KR_BLOCK_LEDGER
#endif
__host__ __device__ constexpr uint32_t kr_xwords(uint32_t flags) { return flags + 256u; }
__host__ __device__ constexpr uint32_t kr_xdata(uint32_t flags) { return flags + 256u + 64u; }
[[maybe_unused]] __host__ __device__ constexpr uint32_t kr_xstage_bytes(int ns) { return 64u + (uint32_t)ns * kXD * 256u; }

extern __shared__ __attribute__((aligned(16))) char krsm[];


typedef int int4v __attribute__((ext_vector_type(4)));
typedef int int2v __attribute__((ext_vector_type(2)));
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(krsm + a); }
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(krsm + a) = v; }
__device__ __forceinline__ int4v lds_ld4(uint32_t a) { return *(const int4v*)(krsm + a); }
// progress words: relaxed workgroup-scope atomics (no vmcnt drains, unlike volatile accesses)
__device__ __forceinline__ int raw_ld(uint32_t a)
{
    return __hip_atomic_load((int*)__builtin_assume_aligned(krsm + a, 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int flag_ld(uint32_t a) { return __builtin_amdgcn_readfirstlane(raw_ld(a)); }
__device__ __forceinline__ void flag_st(uint32_t a, int v)
{
    asm volatile("" ::: "memory");  // data writes are issued before the word (LDS executes in order)
    __hip_atomic_store((int*)__builtin_assume_aligned(krsm + a, 4), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// two adjacent progress words with one 8-byte write, after the data writes it publishes
__device__ __forceinline__ void flag_st2(uint32_t a, int v0, int v1)
{
    asm volatile("" ::: "memory");
    *(int2v*)(krsm + a) = int2v {v0, v1};
    asm volatile("" ::: "memory");
}
__device__ __forceinline__ bool err_set(const StripArgs& a)
{
    return __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }
// m ? b : a per lane, m a lane mask in an SGPR pair: one v_cndmask (a ?: tree over an array is
// turned into a dynamically indexed array in scratch)
__device__ __forceinline__ int sel(uint64_t m, int a, int b)
{
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
// int16 half of a profile dword: column 2d-p (lo) or 2d-p+1 (hi)
__device__ __forceinline__ int qlo(int v) { return (int)(short)v; }
__device__ __forceinline__ int qhi(int v) { return v >> 16; }

// LDS: profile (2 copies x substsz rows x kr_qrs dwords, copy 1 at kr_copy1), subT[x][y] = s(y, x) - 2g, NS+1
// hand-off rings, progress words (slots kr_prog / kr_cons, xo at kFXo, the ticket at kFTicket).
struct KrLds
{
    uint32_t q, sub, ring, flags;
};

__host__ __device__ inline KrLds kr_layout(int ns, int lw, int substsz, bool q8 = false)
{
    KrLds L;
    L.q = 0;
    L.sub = kr_qdwords(lw, substsz, q8) * 4u;
    L.ring = L.sub + (uint32_t)substsz * kSubRow * 4u;
    L.flags = L.ring + (uint32_t)(ns + 1) * kRing * 4u;
    return L;
}

// ------------------------------------------------------------------------------------
// strip wave: 64K rows, K per lane
// ------------------------------------------------------------------------------------
// PT: 1 = mlsppt (a.done set), 2 = XR, pass 1 of the two-pass full fill (nw_expand.hip): lanes
// 15, 31, 47 and 63 also store their last row (rows 64m of the matrix) into a.rows64; 3 = XR inside
// the fused single-pair fill (nw_full_fused_kernel), which also publishes the strip's progress to
// the expansion workgroups of the same launch (write-through stores, a word per strip).  Each is a
// kernel instance of its own, so the plain fill's strip loop is unchanged.
template <int NS, int K, int LW, int PT, bool Q8>
__device__ __forceinline__ void kr_strip(const StripArgs& a, const KrLds& L, int tk, int w, int lane)
{
    const int g = a.g;
    const int Cp = a.Cp;
    const int tBx = a.tBx, tBy = a.tBy, tcols = a.tcols;
    const int r0 = tk * (64 * K * NS) + 64 * K * w + 1;  // first row of the strip
    const int rl = r0 + K * lane;                          // this lane's first row
    constexpr int kLW = LW, kQRS = kr_qrs(LW, Q8);
    constexpr int kQW = Q8 ? kLW / 4 : kLW / 2;  // profile dwords per copy row (ring)
    constexpr int kQD = Q8 ? 4 : 8;               // profile dwords per row per block
    uint32_t qrow[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
    {
        const int r = rl + k;
        int y = (r <= a.R) ? G(a.seqY)[r] : 0;
        y = ((unsigned)y < (unsigned)a.substsz) ? y : 0;
        qrow[k] = L.q + 4u * ((uint32_t)(lane & (Q8 ? 3 : 1)) * kr_copy1(LW, a.substsz, Q8) + (uint32_t)y * kQRS);
    }
    const uint32_t ring_in = L.ring + (uint32_t)w * (kRing * 4u);
    const uint32_t ring_out = L.ring + (uint32_t)(w + 1) * (kRing * 4u);
    const uint32_t f_in = L.flags + kr_prog(w), f_out = L.flags + kr_prog(w + 1);  // f_out: {prog[w+1], cons[w]}
    const uint32_t c_out = L.flags + kr_cons(w + 1);
    const uint32_t f_xo = L.flags + kFXo;
    const int NB = (Cp + 65 + kBlk - 1) / kBlk;  // lane 63 reaches step Cp+64 (element of column Cp)
    // header-column slots of this lane's rows: tile row iT, elements ea .. ea+K-1 (one tile)
    const int iT = (rl - 1) / tBy;
    const int ea = rl - iT * tBy;
    // header column of the next boundary (tile column jb, starting at jb = 1), advanced per boundary
    gptr<int> hcolP = G(a.hcol) + ((size_t)iT * (size_t)tcols + 1) * (size_t)(tBy + 1) + ea;

    // block b needs its halo (ring elements 16b+64 .. 16b+79), room in ring_out for elements
    // 16b .. 16b+15, and (strip 0; the others trail it) the profile of block b+1 (columns < 16b+32)
    auto ok = [&](int pin, int pco, int pxo, int b) {
        return pin >= kBlk * b + 64 + kBlk && pco >= kBlk * b + kBlk - kRing && (w != 0 || pxo >= kBlk * b + 2 * kBlk);
    };
    // the error word is a global load, which waits for this wave's outstanding header stores
    // (vmcnt retires in order): polled once per 32 LDS polls
    // ledger (GSA_STAMPS=1, plain fills): shader-clock cycles spent waiting here, and the waits
    constexpr bool kLedger = PT < 3 && GSA_KR_LEDGER;
    uint64_t spinCyc = 0;
    unsigned spinN = 0;
#if GSA_KR_BLOCK_LEDGER
    // diagnostic build (tools/r06_ledger.py): s_memtime at each block's start, after its input wait
    // and halo read, after its 16 steps and at its end; per strip the sums of the three spans and of
    // the gaps between blocks (the s_memtime results are awaited where they are subtracted, which
    // adds lgkmcnt waits: the spans are upper bounds)
    uint64_t ldg[4] = {0, 0, 0, 0}, ldgEnd = 0;
    // (sched_barrier: no instruction moves across a stamp)
    auto ldgT = []() {
        __builtin_amdgcn_sched_barrier(0);
        const uint64_t t = __builtin_amdgcn_s_memtime();
        __builtin_amdgcn_sched_barrier(0);
        return t;
    };
#define GSA_LDG_T() ldgT()
#endif
    auto spin = [&](int b) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t c0 = (kLedger && a.stamps) ? __builtin_amdgcn_s_memtime() : 0;
        for (int it = 1;; ++it)
        {
            const int pin = flag_ld(f_in), pco = flag_ld(c_out), pxo = (w == 0) ? flag_ld(f_xo) : 0;
            if (ok(pin, pco, pxo, b))
            {
                if (kLedger && a.stamps)
                {
                    spinCyc += __builtin_amdgcn_s_memtime() - c0;
                    ++spinN;
                }
                return true;
            }
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || ((it & 31) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return false;
            }
        }
    };
    // halo of block b: lane 0 reads ring elements 16b+64 .. +15, lanes >= 1 a row of zeros (no branch)
    int4v hc[kHalo];
#pragma unroll
    for (int j = 0; j < kHalo; ++j) hc[j] = int4v {0, 0, 0, 0};
    auto halo_load = [&](int b) {
        {
            // lane 0 alone (exec set and restored inside the asm: no divergent branch in the
            // block); the other lanes' registers keep their 0; the reads are awaited here (the
            // compiler cannot count them), as the first step needs them anyway
            const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * b + 64) & (kRing - 1));
            uint64_t sv;
            asm volatile(
                "s_mov_b64 %4, exec\n"
                "s_mov_b64 exec, 1\n"
                "ds_read_b128 %0, %5\n"
                "ds_read_b128 %1, %5 offset:16\n"
                "ds_read_b128 %2, %5 offset:32\n"
                "ds_read_b128 %3, %5 offset:48\n"
                "s_mov_b64 exec, %4\n"
                "s_waitcnt lgkmcnt(0)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)
                : "v"(hb)
                : "memory");
        }
    };
    // profile dwords of block b: columns 16b - lane .. +15 are dwords 8b - lane/2 .. +7 of copy
    // (lane & 1) (int8: dwords 4b - lane/4 .. +3 of copy lane & 3); reads past the ring's end hit
    // the guard copy
    auto q_off = [&](int b) {
        return Q8 ? 4u * (uint32_t)((4 * b - (lane >> 2)) & (kQW - 1)) : 4u * (uint32_t)((8 * b - (lane >> 1)) & (kQW - 1));
    };
    int qA[K][kQD], qB[K][kQD];
    {
        const uint32_t p = q_off(0);
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < kQD; ++j) qA[k][j] = 0;
        if (!spin(-1)) return;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < kQD; ++j) qA[k][j] = lds_ld(qrow[k] + p + 4u * j);
    }
    // column u of block's profile dword(s) for row k: int8 byte u & 3 of dword u / 4 (an SDWA
    // BYTE operand of the add), int16 half u & 1 of dword u / 2
    auto qv = [&](const int (&qc)[K][kQD], int k, int u) {
        if constexpr (Q8)
            return (int)(signed char)(qc[k][u >> 2] >> (8 * (u & 3)));
        else
            return (u & 1) ? qhi(qc[k][u >> 1]) : qlo(qc[k][u >> 1]);
    };
    int H[K], D = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) H[k] = 0;
    int lt[kBlk];  // lane 63's hand-off values of the last block (H[K-1] of columns t-64)
    // XR: byte address of block 0's segment of this lane's row 64m (lanes 16j - 1 only)
    // (lanes (64/K) j - 1, j = 1 .. K, hold the strip's rows 64 j - 1 as their last row)
    constexpr int kXL = 64 / K;  // lanes per 64 rows
    // fused (PT 3): this strip's staging words and lane 16j - 1's 64-byte slice of each slot
    const uint32_t xsWords = kr_xwords(L.flags);
    const uint32_t xsData = kr_xdata(L.flags) + (uint32_t)(w * kXD * 256) + 64u * (uint32_t)((lane + 1) / kXL - 1);
    uint64_t xrBase = 0;
    if constexpr (PT >= 2)
    {
        const int j = (lane + 1) / kXL;
        const long long m = (long long)(K * NS) * tk + (long long)K * w + j;  // a ticket holds 64 K NS rows
        xrBase = (uint64_t)(uintptr_t)a.rows64 + 4ull * (uint64_t)((m - 1) * a.rpitch + kRowsPad - kXL * j);
    }
    // hand-off of block bb: lane 63's 16 values, then the progress word
    auto handoff = [&](int bb) {
        {
            // lane 63 alone (exec set and restored inside the asm)
            const uint32_t eb = ring_out + 4u * (uint32_t)((kBlk * bb) & (kRing - 1));
            uint64_t sv;
            asm volatile(
                "s_mov_b64 %0, exec\n"
                "s_mov_b64 exec, %1\n"
                "ds_write_b128 %2, %3\n"
                "ds_write_b128 %2, %4 offset:16\n"
                "ds_write_b128 %2, %5 offset:32\n"
                "ds_write_b128 %2, %6 offset:48\n"
                "s_mov_b64 exec, %0"
                : "=&s"(sv)
                : "s"(1ull << 63), "v"(eb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
                  "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
                : "memory");
        }
        if constexpr (PT >= 2)
        {
            // XR: lanes 16j - 1 (K = 4; 32j - 1 for K = 2) hold row r0 + 64j - 1 = 64m, m = K NS tk
            // + K w + j; their values of the block are columns 16 bb - 16j .. +15 (16 bb - 32j for
            // K = 2; shifted), one 64-byte row segment each (columns < 0 fall in the row buffer's
            // left pad)
            const uint64_t addr = xrBase + 64ull * (uint64_t)bb;
            uint64_t sv;
            // fused fill: write-through (sc1) stores, read by other workgroups of the launch
#define GSA_XR_STORES(MOD)                                                                              \
    asm volatile("s_mov_b64 %0, exec\n"                                                                 \
                 "s_mov_b64 exec, %1\n"                                                                 \
                 "global_store_dwordx4 %2, %3, off" MOD "\n"                                            \
                 "global_store_dwordx4 %2, %4, off offset:16" MOD "\n"                                  \
                 "global_store_dwordx4 %2, %5, off offset:32" MOD "\n"                                  \
                 "global_store_dwordx4 %2, %6, off offset:48" MOD "\n"                                  \
                 "s_mov_b64 exec, %0"                                                                    \
                 : "=&s"(sv)                                                                             \
                 : "s"(K == 4 ? 0x8000800080008000ull : 0x8000000080000000ull), "v"(addr),              \
                   "v"(int4v {lt[0], lt[1], lt[2], lt[3]}),                                              \
                   "v"(int4v {lt[4], lt[5], lt[6], lt[7]}), "v"(int4v {lt[8], lt[9], lt[10], lt[11]}),   \
                   "v"(int4v {lt[12], lt[13], lt[14], lt[15]})                                           \
                 : "memory")
            if constexpr (PT == 3)
                (void)addr;  // the fused fill: staged at the next block's start (halo_stage)
            else if constexpr (PT == 4)
                GSA_XR_STORES(" sc1");  // the fused fill, direct: write-through, read by other workgroups
            else
                GSA_XR_STORES("");
#undef GSA_XR_STORES
        }
        // {prog[w+1], cons[w]}: block bb's 16 elements handed off; ring_in elements < 16bb+80
        // (block bb's halo, read at its start) no longer needed
        flag_st2(f_out, bb + 1 == NB ? kBig : kBlk * bb + kBlk, kBlk * bb + 64 + kBlk);
    };
    // the fused fill (PT 3): block b's halo read together with block b-1's row-64m segments into the
    // storer wave's LDS slot (kr_xstore) and the staged count; only the halo reads are awaited.  The
    // staging writes at the hand-off, in the LDS queue ahead of the next block's halo read, held every
    // block's start behind them: 100k x 100k pass 1 without the expansion 109 -> 98 cycles per step
    // without them (profiles/r06_fused100k.txt)
    auto halo_stage = [&](int b) {
        if constexpr (PT == 3)
        {
            const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * b + 64) & (kRing - 1));
            const uint32_t sa = xsData + 64u * (uint32_t)(4 * ((b - 1) % kXD));
            uint64_t sv;
            asm volatile(
                "s_mov_b64 %4, exec\n"
                "s_mov_b64 exec, 1\n"
                "ds_read_b128 %0, %5\n"
                "ds_read_b128 %1, %5 offset:16\n"
                "ds_read_b128 %2, %5 offset:32\n"
                "ds_read_b128 %3, %5 offset:48\n"
                "s_mov_b64 exec, %6\n"
                "ds_write_b128 %7, %8\n"
                "ds_write_b128 %7, %9 offset:16\n"
                "ds_write_b128 %7, %10 offset:32\n"
                "ds_write_b128 %7, %11 offset:48\n"
                "s_mov_b64 exec, 1\n"
                "ds_write_b32 %12, %13\n"
                "s_mov_b64 exec, %4\n"
                "s_waitcnt lgkmcnt(5)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)
                : "v"(hb), "s"(K == 4 ? 0x8000800080008000ull : 0x8000000080000000ull), "v"(sa),
                  "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
                  "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]}),
                  "v"(xsWords + 4u * (uint32_t)w), "v"(b)
                : "memory");
        }
        else
            halo_load(b);
    };
    int rpin = 0, rpco = 0, rpxo = 0;  // progress words read in mid-block, checked at the next block
    int rsink = 0;                     // the read's 4th dword (unused)
    // Tile boundaries bc = jb*tBx are multiples of 16 columns, and lane l meets column bc at step
    // bc + l: in block bc/16 + l/16, at step l & 15.  So the 4 blocks from bc/16 on capture it, 16
    // lanes each, and every lane picks the block's step (lane & 15): the selection masks are
    // constants.  nbb = bc/16 of the next boundary, jb its tile column (uniform).
    int nbb = tBx / kBlk, jb = 1;
    // mlsppt: tile columns [0, ptPend) captured, to be published once their stores are acknowledged
    // (at the next capture block, or at the strip's end); header stores are then system-scope
    constexpr bool pt = PT == 1;
    // fused: the strip's row-64m segments go to the storer wave through LDS (kr_xstore), and every 16
    // blocks its header-column progress: boundaries < the word stored and acknowledged (kXDone: all)
    constexpr bool fx = PT >= 3;
    int ptPend = 0;

    // One body for blocks with and without a header-column capture (cap, uniform): separate
    // bodies get different register assignments and ~100 v_mov per block to reconcile them.
    auto block = [&](int b, int (&qc)[K][kQD], int (&qn)[K][kQD], auto rampT, bool cap) {
        constexpr bool RAMP = decltype(rampT)::value;
        constexpr bool CAP = !RAMP;  // ramp blocks hold no boundary (tBx >= 64)
#if GSA_KR_BLOCK_LEDGER
        const uint64_t lt0 = GSA_LDG_T();
        if (ldgEnd) ldg[3] += lt0 - ldgEnd;
#endif
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            // every destination register of the progress read stays allocated until here: a dead
            // one reused by the block's last steps is a write-after-write on an LDS load, which
            // the compiler resolves with lgkmcnt(1) there -- a wait for the whole LDS queue (the
            // profile reads and the hand-off writes) on the critical path of every block
            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        if (PT == 3 && b > 0)
            halo_stage(b);
        else
            halo_load(b);
#if GSA_KR_BLOCK_LEDGER
        const uint64_t lt1 = GSA_LDG_T();
#endif
        const uint32_t pn = q_off(b + 1);
        int va[CAP ? K : 1][CAP ? kBlk : 1];
#pragma unroll
        for (int u = 0; u < kBlk; ++u)
        {
            int nh[K];
            const int up = shr1z(H[K - 1]) + hc[u >> 2][u & 3];
            nh[0] = max3i(D + qv(qc, 0, u), up, H[0]);
#pragma unroll
            for (int k = 1; k < K; ++k) nh[k] = max3i(H[k - 1] + qv(qc, k, u), nh[k - 1], H[k]);
            if constexpr (RAMP)
            {
                // column t - lane <= 0: the border (H' = 0)
                const bool border = lane >= kBlk * b + u;
#pragma unroll
                for (int k = 0; k < K; ++k) nh[k] = border ? 0 : nh[k];
            }
            // profile of block b+1: K dwords per step over the first kQD steps of the block
            if (u < kQD)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);
            lt[u] = H[K - 1];  // column t-64 of the lane's last row: ring element t
            D = up;
#pragma unroll
            for (int k = 0; k < K; ++k)
            {
                H[k] = nh[k];
                if constexpr (CAP) va[k][u] = nh[k];
            }
            // read late (step 14): the fresher the words, the rarer the spin at the next block
            // start, where a strip that trails the one above at the minimum lag ends up each block
            // (steps 8 / 12 / 14: 100k 5.95 / 5.97 / 5.87 ms)
            if (u == kBlk - 2)
            {
                // slot w-1 {prog[w], cons[w-1] | xo} and slot w+1 {prog[w+2], cons[w+1]}: one
                // ds_read2_b64 (plain loads, kept in place by the memory clobbers around them)
                asm volatile("" ::: "memory");
                const int2v lo = *(const int2v*)(krsm + f_in), hi = *(const int2v*)(krsm + f_in + 16u);
                asm volatile("" ::: "memory");
                rpin = lo.x;
                rpxo = lo.y;
                rpco = hi.y;
                rsink = hi.x;
            }
        }
        // the block's hand-off at its end (the next strip sees it a block earlier than when it is
        // written behind the next block's halo reads: measured 1 % faster at 100k, slightly slower
        // per block)
#if GSA_KR_BLOCK_LEDGER
        const uint64_t lt2 = GSA_LDG_T();
#endif
        handoff(b);
        if constexpr (PT == 4 && !RAMP)
            if ((b & 15) == 15)
            {
                // direct: every block issues >= 4 stores (its row-buffer segments), so all but the last
                // 16 vector-memory operations complete covers blocks <= b - 4: row 64m columns
                // < 16 (b - 7) (block bb stores columns <= 16 (bb - 4) + 15 of its 4 rows) and the
                // header columns captured by block b - 4 (boundaries <= 16 (b - 7))
                asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                if (lane == 0)
                    __hip_atomic_store(a.xdone + (size_t)tk * NS + w,
                                       ((unsigned long long)a.epoch << 32) | (unsigned)max(0, kBlk * (b - 7)),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        if constexpr (PT == 3 && !RAMP)
            if ((b & 15) == 15)
            {
                // the strip's only global stores are its header columns, 4K per boundary (4 capture
                // blocks x K rows): all but the last 8K vector-memory operations complete covers
                // every boundary but the last two captured (boundaries <= 16 b - 2 tBx)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(8 * K) : "memory");
                flag_st(xsWords + 4u * (uint32_t)(2 * NS + w), max(0, kBlk * (b + 1) - 2 * tBx - 64));
                // room in the staging ring for the next 16 blocks (the storer keeps up: rarely waits)
                const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                for (unsigned it = 1; flag_ld(xsWords + 4u * (uint32_t)(NS + w)) + kXD < b + 1 + 16; ++it)
                {
                    __builtin_amdgcn_s_sleep(1);
                    if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || ((it & 31) == 0 && err_set(a)))
                    {
                        atomicOr(a.err, 1u);
                        return false;
                    }
                }
            }
        if (CAP && cap)
        {
            if (pt && ptPend)
            {
                // the previous boundary's stores, issued blocks ago, are acknowledged: publish them
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                flag_st(L.flags + kFCap + 4u * (uint32_t)w, ptPend);
                ptPend = 0;
            }
            // lanes 16m .. 16m+15 (m = b - nbb) hold column bc at step lane & 15: 16 -> 1 by its
            // bits (v_cndmask tree with constant lane masks, 15 per row)
            constexpr uint64_t m1 = 0xAAAAAAAAAAAAAAAAull, m2 = 0xCCCCCCCCCCCCCCCCull;
            constexpr uint64_t m4 = 0xF0F0F0F0F0F0F0F0ull, m8 = 0xFF00FF00FF00FF00ull;
            int v[K];
#pragma unroll
            for (int k = 0; k < K; ++k)
            {
                int x[8];
#pragma unroll
                for (int i = 0; i < 8; ++i) x[i] = sel(m1, va[k][2 * i], va[k][2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = sel(m2, x[2 * i], x[2 * i + 1]);
#pragma unroll
                for (int i = 0; i < 2; ++i) x[i] = sel(m4, x[2 * i], x[2 * i + 1]);
                v[k] = sel(m8, x[0], x[1]);
            }
            const int gb = (rl + kBlk * nbb) * g;  // un-shift: + (row + bc) g
            if ((lane >> 4) == b - nbb)
            {
                if (pt)
                {
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        __hip_atomic_store(&hcolP[k], v[k] + gb + k * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                else if (fx)
                {
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        __hip_atomic_store(&hcolP[k], v[k] + gb + k * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                else
                {
#pragma unroll
                    for (int k = 0; k < K; ++k) hcolP[k] = v[k] + gb + k * g;
                }
            }
            if (b == nbb + 3)
            {
                nbb += tBx / kBlk;
                ++jb;
                hcolP += (size_t)(tBy + 1);
                if (pt && (jb % a.ptChunk == 0 || jb == tcols)) ptPend = jb;
            }
        }
#if GSA_KR_BLOCK_LEDGER
        ldgEnd = GSA_LDG_T();
        ldg[0] += lt1 - lt0;
        ldg[1] += lt2 - lt1;
        ldg[2] += ldgEnd - lt2;
#endif
        return true;
    };

    // the block captures a header column iff it is one of the 4 blocks from the next boundary's
    // (uniform; tBx >= 64 keeps the boundaries 4 blocks apart)
    // (a two-tile-row ticket's second half past the last tile row computes padding only)
    const bool capRows = 64 * K * NS <= kSparseTileBy || (r0 - 1) / tBy < a.trows;
    auto advance = [&](int b) { return b >= nbb && jb < tcols && capRows; };
    using T = std::integral_constant<bool, true>;
    using F = std::integral_constant<bool, false>;
    constexpr int kRampBlocks = 64 / kBlk;  // columns <= 0 occur only in the first 64 steps
    int b = 0;
    for (; b < kRampBlocks; b += 2)
    {
        if (!block(b, qA, qB, T(), false)) return;
        if (!block(b + 1, qB, qA, T(), false)) return;
    }
    for (; b < NB; b += 2)
    {
        if (!block(b, qA, qB, F(), advance(b))) return;
        if (b + 1 >= NB) break;
        if (!block(b + 1, qB, qA, F(), advance(b + 1))) return;
    }
    if (kLedger && a.stamps && lane == 0)
    {
        a.stamps[kLedgerWords * w + 4] = spinCyc;
        a.stamps[kLedgerWords * w + 5] = spinN;
#if GSA_KR_BLOCK_LEDGER
        for (int q = 0; q < 4; ++q) a.stamps[kLedgerWords * w + 6 + q] = ldg[q];
#endif
    }
    if (pt)
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        flag_st(L.flags + kFCap + 4u * (uint32_t)w, kBig);
    }
    if (PT == 4)
    {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0)
            __hip_atomic_store(a.xdone + (size_t)tk * NS + w, ((unsigned long long)a.epoch << 32) | kXDone,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (PT == 3)
    {
        // block NB-1's segments (halo_stage stages each block at the next one's start)
        {
            const uint32_t sa = xsData + 64u * (uint32_t)(4 * ((NB - 1) % kXD));
            uint64_t sv;
            asm volatile("s_mov_b64 %0, exec\n"
                         "s_mov_b64 exec, %1\n"
                         "ds_write_b128 %2, %3\n"
                         "ds_write_b128 %2, %4 offset:16\n"
                         "ds_write_b128 %2, %5 offset:32\n"
                         "ds_write_b128 %2, %6 offset:48\n"
                         "s_mov_b64 exec, %0"
                         : "=&s"(sv)
                         : "s"(K == 4 ? 0x8000800080008000ull : 0x8000000080000000ull), "v"(sa),
                           "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
                           "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
                         : "memory");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        flag_st(xsWords + 4u * (uint32_t)w, NB);  // (every block staged)
        flag_st(xsWords + 4u * (uint32_t)(2 * NS + w), (int)kXDone);
    }
}

// ------------------------------------------------------------------------------------
// feeder wave (the loader's feed job in a wave of its own, kr_split): the row above strip 0 from
// the previous super-strip's granules, kFeedWin 64-column windows per poll round, all of a round's
// loads in flight together.  A granule read is a memory round trip (sc1 stores, agent-scope
// loads), and one 64-column poll per round trip fed strip 0 at 64 columns per round trip: under
// the full fill's store stream a round trip grew to ~3.5 us, below the ~24 columns/us a strip
// sweeps, and every ticket ran at the feed's pace (100k x 100k fused: inter-ticket lag 6 -> 14-20
// us, first strip's sweep 4.2 -> 4.7-6.4 ms; profiles/r06_fused100k.txt).
// ------------------------------------------------------------------------------------
#ifndef GSA_FEED_WIN  // (A/B builds: windows per poll of the one-poll feed, the fused fill's)
#define GSA_FEED_WIN 4
#endif
constexpr int kFeedWin = GSA_FEED_WIN;
#ifndef GSA_FEED_POLLS  // (A/B builds: polls in flight and windows per poll of the PIPE feed)
#define GSA_FEED_POLLS 2
#endif
#ifndef GSA_FEED_PWIN
#define GSA_FEED_PWIN 4
#endif
constexpr int kFeedPolls = GSA_FEED_POLLS, kFeedPWin = GSA_FEED_PWIN;
#ifndef GSA_FUSED_FEED_PIPE
#define GSA_FUSED_FEED_PIPE false  // (A/B builds: the fused fill's feeder with polls in flight)
#endif
// PIPE: kFeedPolls polls in flight, for the plain fills: 100k sparse, same box, 3 rounds, kernel ms: one
// poll 5.367-5.371 -> three 5.342-5.355; on another box three 5.353-5.374, four 5.402-5.413, three of two
// windows 5.391-5.406, two 5.310-5.326 (kept).  The fused full fill measured 2.5 % slower with three
// (profiles/r06_fused100k.txt)
template <int NS, int K, int LW, bool PIPE = false>
__device__ __forceinline__ void kr_feed(const StripArgs& a, const KrLds& L, int tk, int lane)
{
    const int Cp = a.Cp;
    const uint32_t F = L.flags, ring0 = L.ring;
    const gptr<const unsigned long long> gprev = G((const unsigned long long*)a.gran) + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
    int hnext = 0;  // next column of the row above to feed into ring 0
    int c0 = 0;     // ring 0's consumer word, re-read only when it blocks
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;  // idle passes (error-word polls)
    if (PIPE && tk > 0)
    {
        // kFeedPolls polls in flight, staggered: a granule is fed one load latency after it is
        // visible, plus a fraction of one, instead of up to two (a poll issued just before the store
        // landed, then the next).  Every poll issues all its loads (lanes past the room or Cp read
        // column 0 and drop it), so the vector-memory count the compiler waits on is static.
        constexpr int P = kFeedPolls, W = kFeedPWin;
        unsigned long long q[P][W];
        int qb[P], qr[P];
        auto issue = [&](auto sT) {
            constexpr int s = decltype(sT)::value;
            if (hnext + 64 * W + 64 > c0 + kRing) c0 = flag_ld(F + kr_cons(0));
            qb[s] = hnext;
            qr[s] = max(0, min(W, (c0 + kRing - 64 - hnext) / 64));
#pragma unroll
            for (int j = 0; j < W; ++j)
            {
                const int c = hnext + 64 * j + lane;
                const bool in = j < qr[s] && c <= Cp;
                // (not masked after the load: a select would wait for it here)
                q[s][j] = __hip_atomic_load(gprev + (in ? c : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        // the snapshot's published prefix from hnext on (columns below hnext were fed from an earlier
        // snapshot; past the snapshot's room nothing is taken)
        auto consume = [&](auto sT) {
            constexpr int s = decltype(sT)::value;
            // all of the snapshot's loads awaited here, before any branch: a load the consume skips
            // is otherwise still pending where its register is next written, and the compiler waits
            // there for everything in flight (vmcnt(0))
#pragma unroll
            for (int j = 0; j < W; ++j) asm volatile("" ::"v"(q[s][j]));
            int n = hnext;
            bool stop = false;
#pragma unroll
            for (int j = 0; j < W; ++j)
            {
                if (stop || j >= qr[s]) break;
                const int c = qb[s] + 64 * j + lane;
                const bool good = c > Cp || c < hnext || (uint32_t)(q[s][j] >> 32) == a.epoch;
                const uint64_t badm = __ballot(!good);
                const int nj = badm ? __builtin_ctzll(badm) : 64;
                if (c >= hnext && c <= Cp && lane < nj) lds_st(ring0 + 4u * (uint32_t)((c + 64) & (kRing - 1)), (int)(uint32_t)q[s][j]);
                n = max(n, qb[s] + 64 * j + nj);
                stop = nj < 64;
            }
            if (n > hnext)
            {
                hnext = n;
                flag_st(F, hnext > Cp ? kBig : hnext + 64);
                last = __builtin_amdgcn_s_memrealtime();
            }
            else if ((++idle & 63) == 0)
            {
                // the error word by a scalar load: a vector load here, on some passes only, would
                // leave the compiler unsure which polls are in flight (it then waits for all)
                unsigned e;
                asm volatile("s_load_dword %0, %1, 0x0 glc\n"
                             "s_waitcnt lgkmcnt(0)"
                             : "=s"(e)
                             : "s"(a.err)
                             : "memory");
                if (e != 0 || __builtin_amdgcn_s_memrealtime() - last > a.spin)
                {
                    atomicOr(a.err, 1u);
                    return false;
                }
            }
            return true;
        };
        using S0 = std::integral_constant<int, 0>;
        using S1 = std::integral_constant<int, 1>;
        using S2 = std::integral_constant<int, 2>;
        using S3 = std::integral_constant<int, 3>;
        static_assert(P >= 2 && P <= 4 && W >= 1 && W <= 4, "2-4 polls of 1-4 windows in flight");
        issue(S0());
        issue(S1());
        if constexpr (P > 2) issue(S2());
        if constexpr (P > 3) issue(S3());
        // (straight-line: every pass issues every poll, so the compiler's count of loads in flight
        // is the same on every path)
        bool ok = true;
        for (;;)
        {
            ok &= consume(S0());
            issue(S0());
            ok &= consume(S1());
            issue(S1());
            if constexpr (P > 2)
            {
                ok &= consume(S2());
                issue(S2());
            }
            if constexpr (P > 3)
            {
                ok &= consume(S3());
                issue(S3());
            }
            if (!ok || hnext > Cp) break;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the polls still in flight, unused)
        return;
    }
    while (hnext <= Cp)
    {
        // whole windows whose ring elements (c + 64) strip 0 has released (< c0 + kRing)
        if (hnext + 64 * kFeedWin + 64 > c0 + kRing) c0 = flag_ld(F + kr_cons(0));
        const int room = min(kFeedWin, (c0 + kRing - 64 - hnext) / 64);
        bool moved = false;
        if (room > 0)
        {
            unsigned long long q[kFeedWin];
#pragma unroll
            for (int j = 0; j < kFeedWin; ++j)
            {
                const int c = hnext + 64 * j + lane;
                q[j] = (tk > 0 && j < room && c <= Cp) ? __hip_atomic_load(gprev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                                       : 0ull;
            }
            // the published prefix, in column order (columns past Cp: nothing to feed)
            int n = 0;
            bool stop = false;
#pragma unroll
            for (int j = 0; j < kFeedWin; ++j)
            {
                if (stop || j >= room) break;
                const int c = hnext + 64 * j + lane;
                const bool good = c > Cp || tk == 0 || (uint32_t)(q[j] >> 32) == a.epoch;
                const uint64_t badm = __ballot(!good);
                const int nj = badm ? __builtin_ctzll(badm) : 64;
                if (c <= Cp && lane < nj) lds_st(ring0 + 4u * (uint32_t)((c + 64) & (kRing - 1)), tk > 0 ? (int)(uint32_t)q[j] : 0);
                n += nj;
                stop = nj < 64;
            }
            if (n > 0)
            {
                hnext += n;
                flag_st(F, hnext > Cp ? kBig : hnext + 64);
                moved = true;
            }
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (moved)
            last = now;
        else
        {
            // the error word is a global load; another wave's error is looked at every 64th idle pass
            if (now - last > a.spin || ((++idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            if (tk == 0) __builtin_amdgcn_s_sleep(1);
        }
    }
}

// ------------------------------------------------------------------------------------
// loader wave: the column profile and the row above strip 0 (granules of the previous
// super-strip, or row 0)
// ------------------------------------------------------------------------------------
// ROLE 0: both jobs in one wave; 1: the feed only; 2: the profile only
template <int NS, int K, int LW, int ROLE, bool Q8, bool PIPE = false>
__device__ __forceinline__ void kr_loader(const StripArgs& a, const KrLds& L, int tk, int lane)
{
    if constexpr (ROLE == 1)
    {
        kr_feed<NS, K, LW, PIPE>(a, L, tk, lane);
        return;
    }
    const int Cp = a.Cp, C = a.C;
    constexpr int kLW = LW, kQRS = kr_qrs(LW, Q8), kQW = Q8 ? kLW / 4 : kLW / 2;
    const uint32_t F = L.flags;
    const uint32_t ring0 = L.ring;
    const gptr<const unsigned long long> gprev = G((const unsigned long long*)a.gran) + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
    auto letter = [&](int c) {
#if GSA_PROBE_P1 == 1
        // diagnostic build: no letter loads (results wrong)
        return (c & 7) + 1 < a.substsz ? (c & 7) + 1 : 0;
#else
        int x = (c >= 1 && c <= C) ? G(a.seqX)[c] : 0;  // padded columns: letter 0
        return ((unsigned)x < (unsigned)a.substsz) ? x : 0;
#endif
    };
    int qn = 0;     // the profile holds columns < qn
    int hnext = 0;  // next column of the row above to feed into ring 0
    // letters of the next profile batch, loaded a batch ahead: waited for inside the batch, a global
    // load would stall the granule feed for a round trip every 128 columns, and strip 0's lag
    // ratchets to the worst feed delay.  int16: lane l builds dword qn/2 + l of both copies from
    // columns qn+2l-1 .. qn+2l+1; int8: lane l builds dword qn/4 + (l & 31) of copies 2cp, 2cp+1
    // (cp = l / 32) from the 5 columns from qn + lb
    constexpr int kNX = Q8 ? 5 : 3;
    const int cp = lane >> 5;
    const int lb = Q8 ? 4 * (lane & 31) - 1 - 2 * cp : 2 * lane - 1;
    int xl[kNX], nxl[kNX];  // this batch's letters, the next batch's (loaded in pass 0)
#pragma unroll
    for (int i = 0; i < kNX; ++i)
    {
        xl[i] = letter(lb + i);
        nxl[i] = 0;
    }
    int qsub = 0;                   // next pass (8 letters each) of the batch at qn
    int pl = 0, c0 = 0;  // progress words, re-read only when their cached values block
    // lanes of the next granule poll: the drain stores whole aligned 16-granule lines (gran_stride),
    // so a poll reads one line more than the last one found complete (2 to 4 lines): a 64-lane poll
    // on the producer's edge re-read ~3 unfinished lines per line it found (PMC: reads 1.5x the
    // granule bytes)
    int pw = 64;
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;  // idle passes (error-word polls)
    while ((ROLE != 1 && qn <= Cp) || (ROLE != 2 && hnext <= Cp))
    {
        bool moved = false;
        // (1) the row above strip 0 -> ring 0 elements c + 64, as far as granules of the previous
        //     super-strip are published (in column order) and ring 0 has room.  The poll is issued
        //     first and consumed after the profile work, which runs under its latency.
        if (ROLE != 2 && hnext <= Cp && hnext + 128 > c0 + kRing) c0 = flag_ld(F + kr_cons(0));
        const bool feed = ROLE != 2 && hnext <= Cp && hnext + 128 <= c0 + kRing;
        const int c = hnext + lane;
        const bool in = c <= Cp && lane < pw;
        unsigned long long q = 0ull;
        if (feed && tk > 0 && in) q = __hip_atomic_load(gprev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // (2) profile columns qn .. qn+127 (lane l: qn+2l-1 .. qn+2l+1): the ring slots they take
        //     held columns <= qn+127-kLW, dead once the last strip has published elements pl (it
        //     then reads columns >= pl-47).  Built in 4 passes of 8 letters, one per iteration,
        //     so the poll is consumed and re-issued between them: strip 0's lag ratchets to the
        //     feed delay's tail (one pass per iteration: 100k 5.88 -> 5.70 ms)
        if (ROLE != 1 && qsub == 0 && qn <= Cp && qn + 192 > pl + kLW) pl = flag_ld(F + kr_prog(NS));
        if (ROLE != 1 && (qsub > 0 || (qn <= Cp && qn + 192 <= pl + kLW)))
        {
            // letters yy = 8 qsub .. 8 qsub + 7: dwords 2 qsub, 2 qsub + 1 of the subT rows of the
            // lane's columns
            int4v vx[kNX][2];
            {
                const uint32_t o = 32u * (uint32_t)qsub;
#pragma unroll
                for (int i = 0; i < kNX; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) vx[i][j] = lds_ld4(L.sub + 4u * kSubRow * (uint32_t)xl[i] + o + 16u * j);
            }
            if (qsub == 0)
            {
#pragma unroll
                for (int i = 0; i < kNX; ++i) nxl[i] = letter(qn + kBatch + lb + i);
            }
            // int16: dword of columns (cl, cl+1) / (cl-1, cl); int8: of columns 4d-2cp .. +3 / 4d-2cp-1 .. +2
            const uint32_t d = Q8 ? (uint32_t)((qn / 4 + (lane & 31)) & (kQW - 1)) : (uint32_t)((qn / 2 + lane) & (kQW - 1));
            const bool guard = d < (Q8 ? 4u : 8u);  // ring head: also the guard copy at d + kQW
            const uint32_t ce = L.q + 4u * ((Q8 ? (uint32_t)(2 * cp) * kr_copy1(LW, a.substsz, true) : 0u) + d);
            const uint32_t co = ce + 4u * kr_copy1(LW, a.substsz, Q8);
#pragma unroll
            for (int i = 0; i < 8; ++i)
            {
                const int yy = 8 * qsub + i;
                if (yy < a.substsz)
                {
                    int ev, od;  // the lane's dword of the even / odd copy
                    if constexpr (Q8)
                    {
                        const int w0 = vx[0][i >> 2][i & 3], w1 = vx[1][i >> 2][i & 3], w2 = vx[2][i >> 2][i & 3];
                        const int w3 = vx[3][i >> 2][i & 3], w4 = vx[4][i >> 2][i & 3];
                        od = (w0 & 0xff) | ((w1 & 0xff) << 8) | ((w2 & 0xff) << 16) | (w3 << 24);
                        ev = (int)__builtin_amdgcn_alignbyte((unsigned)w4, (unsigned)od, 1u);
                    }
                    else
                    {
                        const int s0 = vx[1][i >> 2][i & 3];
                        ev = (s0 & 0xffff) | (vx[2][i >> 2][i & 3] << 16);  // copy 0: (cl, cl+1)
                        od = (vx[0][i >> 2][i & 3] & 0xffff) | (s0 << 16);  // copy 1: (cl-1, cl)
                    }
                    const uint32_t ra = 4u * kQRS * (uint32_t)yy;
                    lds_st(ce + ra, ev);
                    lds_st(co + ra, od);
                    if (guard)
                    {
                        lds_st(ce + ra + 4u * kQW, ev);
                        lds_st(co + ra + 4u * kQW, od);
                    }
                }
            }
            if (++qsub == 4 || 8 * qsub >= a.substsz)
            {
                qsub = 0;
#pragma unroll
                for (int i = 0; i < kNX; ++i) xl[i] = nxl[i];
                qn += kBatch;
                flag_st(F + kFXo, qn > Cp ? kBig : qn);
            }
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
            if (tk > 0) pw = max(32, min(64, (n & ~15) + 16));
            if (n > 0)
            {
                if (lane < n) lds_st(ring0 + 4u * (uint32_t)((c + 64) & (kRing - 1)), v);
                hnext += n;
                flag_st(F, hnext > Cp ? kBig : hnext + 64);
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
            if (ROLE == 2 || tk == 0 || hnext > Cp) __builtin_amdgcn_s_sleep(1);
        }
    }
}

// ------------------------------------------------------------------------------------
// drain wave: the last strip's row (ring NS) -> granules for the next super-strip and, when the
// row closes a tile row, the header row of the tiles below (unshifted) with its duplicates: the
// last element of the tile to the left and the corner of the header column
// (nwalign_gpu9_mlsp_diagdiagdiag.cu:214-218, 253-257).  It issues no global loads, so its stores
// never wait behind a poll.  A ticket of two tile rows (NS = 8, K = 4) also has a tile row
// boundary after strip NS/2 - 1: the drain writes that header row from ring NS/2 as strip NS/2
// reads it.  Strip NS/2 - 1 is throttled by strip NS/2's consumption only, so after each read the
// drain checks that the slots it read could not have been rewritten yet (strip NS/2 - 1 rewrites
// element e once it has published e - kRing + 16): it stays within a few columns of the strips, and
// a lag of kRing - 96 elements would end the launch with the error word rather than a wrong header.
// ------------------------------------------------------------------------------------
template <int NS, int K, int LW, int PT>
__device__ __forceinline__ void kr_drain(const StripArgs& a, const KrLds& L, int tk, int lane)
{
    const int Cp = a.Cp, g = a.g, tBx = a.tBx, tBy = a.tBy, tcols = a.tcols;
    const uint32_t F = L.flags, ringN = L.ring + (uint32_t)NS * (kRing * 4u);
    constexpr bool kTwoRows = 64 * K * NS == 2 * kSparseTileBy;
    if constexpr (!kTwoRows)
    {
        // mlsppt (one tile row per ticket): publish to the host the column chunks of this tile row
        // whose headers are in memory -- header columns captured by every strip (their words in
        // LDS follow their acknowledged stores) and the header row below written by this wave
        constexpr bool pt = PT == 1;
        const int cw = pt ? a.ptChunk : 1;
        const int nCh = (tcols + cw - 1) / cw;
        int pub = 0;
        // hrowTiles: tile columns whose header-row stores are complete -- after s_waitcnt vmcnt(0),
        // or vmcnt(60) for stores issued before the wave's last 60 vector-memory instructions
        auto publish = [&](int hrowTiles) {
            int t = hrowTiles;
#pragma unroll
            for (int s = 0; s < NS; ++s)
            {
                const int v = flag_ld(F + kFCap + 4u * (uint32_t)s);
                t = min(t, v == kBig ? tcols : v);
            }
            const int n = t >= tcols ? nCh : t / cw;
            if (n > pub)
            {
                if (lane == 0)
                    __hip_atomic_store(a.done + tk, ((unsigned long long)a.epoch << 32) | (unsigned)n, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                pub = n;
            }
        };
        // after the last column: wait for the strips' last captures
        auto publish_rest = [&]() {
            uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            unsigned spins = 0;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's header-row stores
            while (pt && pub < nCh)
            {
                const int before = pub;
                publish(tcols);
                if (pub > before) t0 = __builtin_amdgcn_s_memrealtime();
                if (pub >= nCh) break;
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.spin || ((++spins & 63) == 0 && err_set(a)))
                {
                    atomicOr(a.err, 1u);
                    return;
                }
            }
        };
        if (tk + 1 >= a.nTickets)
        {
            flag_st(F + kr_cons(NS), kBig);  // nobody reads our last row
            publish_rest();                   // (the last tile row has no header row below)
            return;
        }
        const gptr<unsigned long long> gout = G(a.gran) + (size_t)tk * a.granStride;
        const int rowEnd = (tk + 1) * (64 * K * NS);  // the row this ticket hands down
        const bool hdr = rowEnd % tBy == 0;
        const size_t rowbase = (size_t)(rowEnd / tBy) * (size_t)tcols;  // tile index of (iT+1, 0)
        int dnext = 0;  // next column to drain
        // mlsppt: publication lags the header-row stores by >= 64 loop passes (each issues >= 1
        // vector-memory instruction, the granule store), so vmcnt(60) finds them complete without
        // waiting on the fresh granule stores the next super-strip is polling for
        int passes = 0, markPass = 0, markTiles = 0;
        uint64_t last = __builtin_amdgcn_s_memrealtime();
        unsigned idle = 0;  // idle passes (error-word polls)
        while (dnext <= Cp)
        {
            const int avail = min(flag_ld(F + kr_prog(NS)) - 64, Cp + 1);  // columns < avail are in ring NS
            if (dnext < avail)
            {
                const int c = dnext + lane;
                if (c < avail)
                {
                    const int v = lds_ld(ringN + 4u * (uint32_t)((c + 64) & (kRing - 1)));
                    __hip_atomic_store(gout + c, ((unsigned long long)a.epoch << 32) | (uint32_t)v, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    if (hdr)
                    {
                        const int hv = v + (rowEnd + c) * g;
                        const int jT = c / tBx, jj = c - jT * tBx;
                        auto put = [&](int* p) {
                            if (pt)
                                __hip_atomic_store(p, hv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                            else
                                *G(p) = hv;
                        };
                        if (jT < tcols) put(a.hrow + (rowbase + jT) * (size_t)(tBx + 1) + jj);
                        if (jj == 0 && jT > 0)
                        {
                            put(a.hrow + (rowbase + jT - 1) * (size_t)(tBx + 1) + tBx);
                            if (jT < tcols) put(a.hcol + (rowbase + jT) * (size_t)(tBy + 1));
                        }
                    }
                }
                dnext = min(dnext + 64, avail);
                flag_st(F + kr_cons(NS), dnext > Cp ? kBig : dnext + 64);
                last = __builtin_amdgcn_s_memrealtime();
                if (pt && ++passes - markPass >= 64)
                {
                    asm volatile("s_waitcnt vmcnt(60)" ::: "memory");
                    publish(markTiles);
                    markPass = passes;
                    markTiles = min(tcols, (dnext - 1) / tBx);
                }
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
        publish_rest();
    }
    else
    {
        constexpr int kTicketRows = 64 * K * NS;
        constexpr int kMid = NS / 2;  // ring after the first tile row of a two-row ticket
        const uint32_t ringM = L.ring + (uint32_t)kMid * (kRing * 4u);
        // header row (row, columns c) of the tiles below a tile row boundary, with its duplicates
        auto put_hdr = [&](int row, int c, int hv) {
            const size_t rowbase = (size_t)(row / tBy) * (size_t)tcols;  // tile index of (row / tBy, 0)
            const int jT = c / tBx, jj = c - jT * tBx;
            if (jT < tcols) G(a.hrow)[(rowbase + jT) * (size_t)(tBx + 1) + jj] = hv;
            if (jj == 0 && jT > 0)
            {
                G(a.hrow)[(rowbase + jT - 1) * (size_t)(tBx + 1) + tBx] = hv;
                if (jT < tcols) G(a.hcol)[(rowbase + jT) * (size_t)(tBy + 1)] = hv;
            }
        };
        const bool gr = tk + 1 < a.nTickets;  // a next super-strip reads our last row
        if (!gr) flag_st(F + kr_cons(NS), kBig);  // nobody reads our last row
        const gptr<unsigned long long> gout = G(a.gran) + (size_t)tk * a.granStride;
        const int rowEnd = (tk + 1) * kTicketRows;  // the row this ticket hands down
        const bool hdr = rowEnd % tBy == 0;
        const int rowMid = tk * kTicketRows + kSparseTileBy;
        const bool mid = kTwoRows && rowMid / tBy < a.trows;
        int dnext = gr ? 0 : Cp + 1;   // next column to drain
        int mnext = mid ? 0 : Cp + 1;  // next column of the mid header row
    const int NBs = (Cp + 65 + kBlk - 1) / kBlk;  // blocks of a strip (kr_strip's NB)
        uint64_t last = __builtin_amdgcn_s_memrealtime();
        unsigned idle = 0;  // idle passes (error-word polls)
        while (dnext <= Cp || mnext <= Cp)
        {
            bool moved = false;
            if (dnext <= Cp)
            {
                const int avail = min(flag_ld(F + kr_prog(NS)) - 64, Cp + 1);  // columns < avail are in ring NS
                if (dnext < avail)
                {
                    const int c = dnext + lane;
                    if (c < avail)
                    {
                        const int v = lds_ld(ringN + 4u * (uint32_t)((c + 64) & (kRing - 1)));
                        __hip_atomic_store(gout + c, ((unsigned long long)a.epoch << 32) | (uint32_t)v, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        if (hdr) put_hdr(rowEnd, c, v + (rowEnd + c) * g);
                    }
                    dnext = min(dnext + 64, avail);
                    flag_st(F + kr_cons(NS), dnext > Cp ? kBig : dnext + 64);
                    moved = true;
                }
            }
            if constexpr (kTwoRows)
            {
                if (mnext <= Cp)
                {
                    const int availm = min(flag_ld(F + kr_prog(kMid)) - 64, Cp + 1);  // columns < availm in ring kMid
                    if (mnext < availm)
                    {
                        const int c = mnext + lane;
                        const int v = lds_ld(ringM + 4u * (uint32_t)((c + 64) & (kRing - 1)));
                        asm volatile("" ::: "memory");  // the data reads before the check's read (LDS in order)
                        // (kBig: the strip has finished, having written elements < 16 NBs)
                    const int pm = flag_ld(F + kr_prog(kMid));
                    if ((pm == kBig ? kBlk * NBs : pm) > mnext + 64 + kRing - 32)
                        {
                            atomicOr(a.err, 1u);
                            return;
                        }
                        if (c < availm) put_hdr(rowMid, c, v + (rowMid + c) * g);
                        mnext = min(mnext + 64, availm);
                        moved = true;
                    }
                }
            }
            if (moved)
                last = __builtin_amdgcn_s_memrealtime();
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
}

// ------------------------------------------------------------------------------------
// storer wave (the fused fill, PT 3; the workgroup's eighth wave): the strips' row-64m segments
// from their LDS staging slots to the row buffer, 4 blocks of a strip per store instruction (64
// lanes x 16 bytes: block, row, 16-byte chunk), write-through; then, behind vmcnt(0), the strip's
// progress word for the expansion -- epoch << 32 | X, row 64m columns < X and header columns of
// boundaries < X in memory.  The strips issued these stores themselves before (4 four-lane store
// instructions per block): under the expansion's store stream their write-through stores filled
// each strip's 63 outstanding vector-memory slots and stalled it (100k x 100k: pass 1 6.2 -> 8.4 ms,
// profiles/r06_fused100k.txt).
// ------------------------------------------------------------------------------------
template <int NS, int K>
__device__ __forceinline__ void kr_xstore(const StripArgs& a, const KrLds& L, int tk, int lane)
{
    static_assert(K == 4, "4 rows 64m per strip: a store instruction = 4 blocks x 4 rows x 4 chunks");
    const int NB = (a.Cp + 65 + kBlk - 1) / kBlk;  // blocks of a strip (kr_strip's NB)
    const uint32_t W = kr_xwords(L.flags), D = kr_xdata(L.flags);
    constexpr int kXL = 64 / K;
    const int kk = lane >> 4, jj = (lane >> 2) & 3, c = lane & 3;  // block of the group, row 64(jj+1), chunk
    unsigned long long* const xword = a.xdone + (size_t)tk * NS;
    // this lane's int offset in the row buffer, less 16 bb, per strip
    long long rowOff[NS];
#pragma unroll
    for (int w = 0; w < NS; ++w)
    {
        const long long m = (long long)(K * NS) * tk + K * w + jj + 1;  // row 64m of the matrix
        rowOff[w] = (m - 1) * a.rpitch + kRowsPad - kXL * (jj + 1) + kBlk * kk + 4 * c;
    }
    int sb[NS], pub[NS];
#pragma unroll
    for (int w = 0; w < NS; ++w) sb[w] = pub[w] = 0;
    int since = 0;  // blocks stored since the last publication
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    for (unsigned idle = 1;; ++idle)
    {
        bool moved = false, fin = true;
#pragma unroll
        for (int w = 0; w < NS; ++w)
        {
            const int p = flag_ld(W + 4u * (uint32_t)w);  // blocks staged
            // whole groups of 4 blocks, and the strip's last ones
            while (sb[w] < p && (sb[w] + 4 <= p || p >= NB))
            {
                const int bb = sb[w] + kk;
                if (bb < p)
                {
                    const int4v v =
                        lds_ld4(D + 256u * (uint32_t)(w * kXD + bb % kXD) + 64u * (uint32_t)jj + 16u * (uint32_t)c);
                    const uint64_t addr =
                        (uint64_t)(uintptr_t)a.rows64 + 4ull * (uint64_t)(rowOff[w] + (long long)kBlk * sb[w]);
                    // write-through (sc1): read by other workgroups of the launch
                    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(addr), "v"(v) : "memory");
                }
                const int n = min(4, p - sb[w]);
                sb[w] += n;
                since += n;
                flag_st(W + 4u * (uint32_t)(NS + w), sb[w]);  // slots of blocks < sb[w] free (the reads precede)
                moved = true;
            }
            fin = fin && sb[w] >= NB;
        }
        // publish every 16 blocks per strip (vmcnt(0) waits for this wave's stores only), and at the end
        if (since >= 16 * NS || fin)
        {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            since = 0;
            bool all = true;
#pragma unroll
            for (int w = 0; w < NS; ++w)
            {
                const int hdr = flag_ld(W + 4u * (uint32_t)(2 * NS + w));
                const int x = (sb[w] >= NB && hdr == (int)kXDone) ? (int)kXDone : min(kBlk * sb[w] - 64, hdr);
                if (x > pub[w])
                {
                    if (lane == 0)
                        __hip_atomic_store(xword + w, ((unsigned long long)a.epoch << 32) | (unsigned)x, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    pub[w] = x;
                    moved = true;
                }
                all = all && pub[w] == (int)kXDone;
            }
            if (all) return;
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (moved)
            last = now;
        else
        {
            // idle while the strips wait for their input: the strips' own watchdog is a.spin per wait
            if (now - last > 4 * a.spin || ((idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

__device__ __forceinline__ PairDesc kr_desc(const PairDesc* p)
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

// waves per workgroup: NS strips, the loader (split into a feeder and a profiler wave when the SIMDs
// have room: NS <= 4), the drain
template <int NS, int PT = 0>
constexpr bool kr_split() { return NS <= 4; }
template <int NS, int PT = 0>
constexpr int kr_waves() { return NS + 2 + (kr_split<NS, PT>() ? 1 : 0); }

// Q8: the int8-profile instance.  It declines a table with some s - 2g outside int8 (every
// workgroup exits before taking a ticket and the launch's word in a.q8flag is set to its epoch);
// the host enqueues the int16 instance behind it with a.q8 = 2, which runs only in that case.  Both
// profiles in one kernel (a uniform branch, or the int16 path out of line) cost the int8 path its
// code generation: 5.49 / 5.75 ms against 5.30 for the int8 instance alone.
template <int NS, int K, int LW, int PT, bool Q8>
__global__ void __launch_bounds__((64 * kr_waves<NS, PT>()), 1) nw_krow_kernel(StripArgs a)
{
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const KrLds L = kr_layout(NS, LW, a.substsz, Q8);
    // the int16 fallback behind an int8 launch: nothing to do unless that launch declined the table
    if (!Q8 && a.q8 == 2 && __hip_atomic_load(a.q8flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != a.epoch) return;
    bool bad = false, bad8 = false;
    for (int k = threadIdx.x; k < a.substsz * kSubRow; k += 64 * kr_waves<NS, PT>())
    {
        const int x = k / kSubRow, yy = k % kSubRow;
        const int v = yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - 2 * a.g : 0;
        bad |= v < -32768 || v > 32767;  // the profile holds int16
        bad8 |= v < -128 || v > 127;      // ... or int8
        lds_st(L.sub + 4u * k, v);
    }
    if constexpr (Q8)
    {
        // a table outside int8: decline (every workgroup sees the same table).  Reduced through a
        // word of the dynamic LDS: __syncthreads_or would allocate static LDS, which moves krsm off
        // address 0, and the asm blocks address krsm by raw offsets.
        if (threadIdx.x == 0) lds_st(L.flags + kFTicket, 0);
        __syncthreads();
        if (bad8) atomicOr((int*)(krsm + L.flags + kFTicket), 1);
        __syncthreads();
        if (lds_ld(L.flags + kFTicket) != 0)
        {
            if (threadIdx.x == 0) __hip_atomic_store(a.q8flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    else if (bad)
        atomicOr(a.err, 2u);  // (an int8 table never has this)
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
        const PairDesc d = kr_desc(a.pairs + lo);
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
        pa.granStride = gran_stride(d.Cp);
        pa.rows64 = d.rows64;
        pa.rpitch = d.rpitch;
        const int tk = (tks >= 0) ? tks : tkg - d.ticketBase;
        if (threadIdx.x < 32) lds_st(L.flags + 4u * threadIdx.x, 0);  // prog[], cons[], xo
        if (threadIdx.x >= kFCap / 4 && threadIdx.x < kFCap / 4 + 8) lds_st(L.flags + 4u * threadIdx.x, 0);
        __syncthreads();
        if (w == NS + 1)
            kr_drain<NS, K, LW, PT>(pa, L, tk, lane);
        else if (w == NS)
            kr_loader<NS, K, LW, kr_split<NS, PT>() ? 1 : 0, Q8, true>(pa, L, tk, lane);
        else if (kr_split<NS, PT>() && w == NS + 2)
            kr_loader<NS, K, LW, 2, Q8>(pa, L, tk, lane);
        else
        {
            // ledger (GSA_STAMPS=1): per strip [realtime start, end, shader clock start, end, cycles
            // waiting for input, waits, and in a GSA_KR_BLOCK_LEDGER build the block spans]
            unsigned long long* const lg = (GSA_KR_LEDGER && a.stamps) ? a.stamps + kLedgerWords * ((size_t)tkg * NS + w) : nullptr;
            pa.stamps = lg ? a.stamps + kLedgerWords * (size_t)tkg * NS : nullptr;
            if (lg && lane == 0)
            {
                lg[0] = __builtin_amdgcn_s_memrealtime();
                lg[2] = __builtin_amdgcn_s_memtime();
            }
            __builtin_amdgcn_s_setprio(3);
            kr_strip<NS, K, LW, PT, Q8>(pa, L, tk, w, lane);
            __builtin_amdgcn_s_setprio(0);
            if (lg && lane == 0)
            {
                lg[1] = __builtin_amdgcn_s_memrealtime();
                lg[3] = __builtin_amdgcn_s_memtime();
            }
        }
    }
}

template <int NS, int K, int LW, int PT, bool Q8>
hipError_t launch_kr1(const StripArgs& a, int grid, hipStream_t stream, bool foot = true)
{
    const size_t lds = krow_lds_bytes(NS, LW, a.substsz, Q8);
    auto kern = nw_krow_kernel<NS, K, LW, PT, Q8>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (grid <= 0)
    {
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, 64 * kr_waves<NS, PT>(), lds);
        if (e == hipSuccess) e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        grid = std::max(1, std::min(a.nTicketsTotal, std::max(1, per_cu) * cus));
    }
    if (foot && (e = record_foot((const void*)kern, lds, 64 * kr_waves<NS, PT>(), grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * kr_waves<NS, PT>()), lds, stream, a);
    return hipGetLastError();
}

// a.q8: the int8 instance, then the int16 one behind it (a no-op unless the int8 launch declined
// the table); otherwise the int16 instance alone
template <int NS, int K, int LW, int PT = 0>
hipError_t launch_kr(const StripArgs& a, int grid, hipStream_t stream)
{
    if (!a.q8) return launch_kr1<NS, K, LW, PT, false>(a, grid, stream);
    hipError_t e = launch_kr1<NS, K, LW, PT, true>(a, grid, stream);
    if (e != hipSuccess) return e;
    StripArgs b = a;
    b.q8 = 2;
    return launch_kr1<NS, K, LW, PT, false>(b, grid, stream, false);
}

#ifdef GSA_KROW_SCORE
// ====================================================================================
// Score-only NW / SW, linear or affine gaps, on the K-rows layout (nw_kscore.hip; BASELINE
// configs[4]).  The same workgroup as the sparse fill -- 4 strip waves of K = 4 rows per lane, a
// feeder, a profiler and a drain wave, one 1024-row ticket per workgroup -- with the shifted Gotoh
// recurrence of the strip kernel's score modes (nw_strip.hip kModeScoreAG/SW/AGL/SWL):
//   X' = X - (i+j) ge, d = go - ge, Hgo' = H' + d carried (H' alone when d = 0),
//   E'(k,c) = max(E'(k,c-1), Hgo'(k,c-1)),  F'(k,c) = max(F'(k-1,c), Hgo'(k-1,c)),
//   H'      = max3(Hgo'(k-1,c-1) + s - go - ge, E', F'),
// the SW clamp H >= 0 folded into F' as the floor z = -(i+j) ge, the first maximal cell tracked
// per row.  Two values cross strip boundaries (Hgo' and F' of the last row: two LDS rings, two
// granule arrays between tickets); a linear gap carries H' only.  Column letters past C (and at
// columns <= 0) are a NEG letter whose profile value is -32768: those cells are reached only
// through a gap and never tie a real cell's score.
// ====================================================================================
constexpr int kNegS = -(1 << 29);  // "before the matrix": far from overflow, never the maximum
constexpr int kNegQ = -32768;      // profile value of the NEG column letter
constexpr uint32_t kRing2Off = (uint32_t)(kKrowNSDefault + 1) * kRing * 4u;  // ring2 = ring + this

// LDS: profile as kr_layout, subT with one more row (the NEG letter), NS+1 rings of Hgo' and NS+1
// of F', progress words
struct KsLds
{
    uint32_t q, sub, ring, ring2, flags;
};

__host__ __device__ inline KsLds ks_layout(int substsz, bool q8 = false)
{
    constexpr int LW = 1024;
    KsLds L;
    L.q = 0;
    L.sub = kr_qdwords(LW, substsz, q8) * 4u;
    L.ring = L.sub + (uint32_t)(substsz + 1) * kSubRow * 4u;
    L.ring2 = L.ring + kRing2Off;
    L.flags = L.ring2 + kRing2Off;
    return L;
}

// strip wave (NS = 4): 64 K rows, K (4, or 2) per lane.  TAP: lane tapLane's last row is a.tapRow,
// stored block by block (score_bidi)
template <int MODE, bool Q8, int K, bool TAP = false>
__device__ __forceinline__ void ks_strip(const StripArgs& a, const KsLds& L, int tk, int w, int lane, int tapLane = 0)
{
    constexpr int NS = kKrowNSDefault, LW = 1024;
    constexpr bool AG = !is_lin_mode(MODE);  // E' and F' carried
    constexpr bool SW = is_sw_mode(MODE);
    const int Cp = a.Cp;
    const int ge = a.ge;
    const int dd = AG ? a.go - a.ge : 0;
    const int r0 = tk * (64 * K * NS) + 64 * K * w + 1;
    const int rl = r0 + K * lane;
    // the column profile as the sparse fill's (kr_strip): int16 pairs in 2 shifted copies, or (Q8) int8
    // in 4 byte-shifted copies
    constexpr int kQRS = kr_qrs(LW, Q8), kQW = Q8 ? LW / 4 : LW / 2;
    constexpr int kQD = Q8 ? 4 : 8;  // profile dwords per row per block
    uint32_t qrow[K];
#pragma unroll
    for (int k = 0; k < K; ++k)
    {
        const int r = rl + k;
        int y = (r <= a.R) ? G(a.seqY)[r] : 0;
        y = ((unsigned)y < (unsigned)a.substsz) ? y : 0;
        qrow[k] = L.q + 4u * ((uint32_t)(lane & (Q8 ? 3 : 1)) * kr_copy1(LW, a.substsz, Q8) + (uint32_t)y * kQRS);
    }
    const uint32_t ring_in = L.ring + (uint32_t)w * (kRing * 4u);
    const uint32_t ring_out = L.ring + (uint32_t)(w + 1) * (kRing * 4u);
    const uint32_t f_in = L.flags + kr_prog(w), f_out = L.flags + kr_prog(w + 1);
    const uint32_t c_out = L.flags + kr_cons(w + 1);
    const uint32_t f_xo = L.flags + kFXo;
    const int NB = (Cp + 65 + kBlk - 1) / kBlk;
    auto ok = [&](int pin, int pco, int pxo, int b) {
        return pin >= kBlk * b + 64 + kBlk && pco >= kBlk * b + kBlk - kRing && (w != 0 || pxo >= kBlk * b + 2 * kBlk);
    };
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
    // halo of block b (Hgo' and, affine, F' of the row above): lane 0 reads ring elements
    // 16b+64 .. +15 of both rings, the other lanes keep 0 (exec set and restored in the asm)
    int4v hc[kHalo], hf[kHalo];
#pragma unroll
    for (int j = 0; j < kHalo; ++j)
    {
        hc[j] = int4v {0, 0, 0, 0};
        hf[j] = int4v {0, 0, 0, 0};
    }
    auto halo_load = [&](int b) {
        const uint32_t hb = ring_in + 4u * (uint32_t)((kBlk * b + 64) & (kRing - 1));
        uint64_t sv;
        if constexpr (AG)
            asm volatile(
                "s_mov_b64 %8, exec\n"
                "s_mov_b64 exec, 1\n"
                "ds_read_b128 %0, %9\n"
                "ds_read_b128 %1, %9 offset:16\n"
                "ds_read_b128 %2, %9 offset:32\n"
                "ds_read_b128 %3, %9 offset:48\n"
                "ds_read_b128 %4, %9 offset:%10\n"
                "ds_read_b128 %5, %9 offset:%11\n"
                "ds_read_b128 %6, %9 offset:%12\n"
                "ds_read_b128 %7, %9 offset:%13\n"
                "s_mov_b64 exec, %8\n"
                "s_waitcnt lgkmcnt(0)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "+v"(hf[0]), "+v"(hf[1]), "+v"(hf[2]), "+v"(hf[3]),
                  "=&s"(sv)
                : "v"(hb), "n"(kRing2Off), "n"(kRing2Off + 16), "n"(kRing2Off + 32), "n"(kRing2Off + 48)
                : "memory");
        else
            asm volatile(
                "s_mov_b64 %4, exec\n"
                "s_mov_b64 exec, 1\n"
                "ds_read_b128 %0, %5\n"
                "ds_read_b128 %1, %5 offset:16\n"
                "ds_read_b128 %2, %5 offset:32\n"
                "ds_read_b128 %3, %5 offset:48\n"
                "s_mov_b64 exec, %4\n"
                "s_waitcnt lgkmcnt(0)"
                : "+v"(hc[0]), "+v"(hc[1]), "+v"(hc[2]), "+v"(hc[3]), "=&s"(sv)
                : "v"(hb)
                : "memory");
    };
    auto q_off = [&](int b) {
        return Q8 ? 4u * (uint32_t)((4 * b - (lane >> 2)) & (kQW - 1)) : 4u * (uint32_t)((8 * b - (lane >> 1)) & (kQW - 1));
    };
    int qA[K][kQD], qB[K][kQD];
    {
        const uint32_t p = q_off(0);
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < kQD; ++j) qA[k][j] = 0;
        if (!spin(-1)) return;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int j = 0; j < kQD; ++j) qA[k][j] = lds_ld(qrow[k] + p + 4u * j);
    }
    // Hgo' (H' when linear), E' of the K rows, F' of the last row, the diagonal of row 0
    int H[K], E[K], FD = kNegS, D = kNegS;
#pragma unroll
    for (int k = 0; k < K; ++k)
    {
        H[k] = kNegS;
        E[k] = kNegS;
    }
    // SW: floors z_k = -(i+j) ge of the lane's rows at the current column (column t - lane) and the
    // first maximum per row.  One key per cell, ((h_k - z_0) << 4) + 15 - u = (h_k << 4) + wv with
    // wv = 15 - u - 16 z_0 shared by the rows: h_k - z_0 = H + k |ge| >= 0 is the score of row k
    // plus a per-row constant, so the maximum per row and its first step are those of H; the
    // block's best is folded (score - k |ge|, step) at the block end.  Rows past R never win.
    // (row k's floor at step u is row 0's at step u + k, the same anti-diagonal: one add per step)
    int z0 = 0, p[K], best[K], tb[K];
    uint32_t wv = 0;  // (mod 2^32: the keys themselves stay below 2^31 while scores stay below 2^26)
    if constexpr (SW)
    {
        z0 = -(rl - lane) * ge;
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
            p[k] = 0;
            best[k] = (rl + k <= a.R) ? 0 : 0x7fffffff;
            tb[k] = 0;
        }
    }
    // NW: the cell (R, C) lies in this strip iff r0 <= R < r0 + 64 K; lane laneR reaches column C
    // at step tStar, in block tStar / 16, row kR
    const int rR = a.R - r0;
    const bool hasR = !SW && rR >= 0 && rR < 64 * K;
    const int laneR = rR / K, kR = rR % K, tStar = a.C + laneR;
    int lt[kBlk], lf[kBlk];  // lane 63's hand-off values of the last block (Hgo', F' of columns t-64)
    auto handoff = [&](int bb) {
        const uint32_t eb = ring_out + 4u * (uint32_t)((kBlk * bb) & (kRing - 1));
        uint64_t sv;
        if constexpr (AG)
            asm volatile(
                "s_mov_b64 %0, exec\n"
                "s_mov_b64 exec, %1\n"
                "ds_write_b128 %2, %3\n"
                "ds_write_b128 %2, %4 offset:16\n"
                "ds_write_b128 %2, %5 offset:32\n"
                "ds_write_b128 %2, %6 offset:48\n"
                "ds_write_b128 %2, %7 offset:%11\n"
                "ds_write_b128 %2, %8 offset:%12\n"
                "ds_write_b128 %2, %9 offset:%13\n"
                "ds_write_b128 %2, %10 offset:%14\n"
                "s_mov_b64 exec, %0"
                : "=&s"(sv)
                : "s"(1ull << 63), "v"(eb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
                  "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]}),
                  "v"(int4v {lf[0], lf[1], lf[2], lf[3]}), "v"(int4v {lf[4], lf[5], lf[6], lf[7]}),
                  "v"(int4v {lf[8], lf[9], lf[10], lf[11]}), "v"(int4v {lf[12], lf[13], lf[14], lf[15]}), "n"(kRing2Off),
                  "n"(kRing2Off + 16), "n"(kRing2Off + 32), "n"(kRing2Off + 48)
                : "memory");
        else
            asm volatile(
                "s_mov_b64 %0, exec\n"
                "s_mov_b64 exec, %1\n"
                "ds_write_b128 %2, %3\n"
                "ds_write_b128 %2, %4 offset:16\n"
                "ds_write_b128 %2, %5 offset:32\n"
                "ds_write_b128 %2, %6 offset:48\n"
                "s_mov_b64 exec, %0"
                : "=&s"(sv)
                : "s"(1ull << 63), "v"(eb), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}), "v"(int4v {lt[4], lt[5], lt[6], lt[7]}),
                  "v"(int4v {lt[8], lt[9], lt[10], lt[11]}), "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
                : "memory");
        flag_st2(f_out, bb + 1 == NB ? kBig : kBlk * bb + kBlk, kBlk * bb + 64 + kBlk);
    };
    int rpin = 0, rpco = 0, rpxo = 0, rsink = 0;
    // TAP: byte address of block 0's 16 values of the tap row (lane tapLane: lt[u] and lf[u] are
    // columns 16 b + u - 1 - lane of its last row)
    uint64_t tapB = 0, tapBF = 0;
    if constexpr (TAP)
    {
        tapB = (uint64_t)(uintptr_t)a.tapH + 4ull * (uint64_t)(kTapPad - 1 - lane);
        tapBF = (uint64_t)(uintptr_t)a.tapF + 4ull * (uint64_t)(kTapPad - 1 - lane);
    }
    const uint64_t tapMask = 1ull << (tapLane & 63);

    auto block = [&](int b, int (&qc)[K][kQD], int (&qn)[K][kQD]) {
        {
            const int pin = __builtin_amdgcn_readfirstlane(rpin), pco = __builtin_amdgcn_readfirstlane(rpco);
            const int pxo = (w == 0) ? __builtin_amdgcn_readfirstlane(rpxo) : 0;
            asm volatile("" ::"v"(rpin), "v"(rpco), "v"(rpxo), "v"(rsink));  // (kr_strip: WAW on the read)
            if (!ok(pin, pco, pxo, b) && !spin(b)) return false;
        }
        halo_load(b);
        const uint32_t pn = q_off(b + 1);
        int va[SW ? 1 : K][SW ? 1 : kBlk];  // NW: the block's Hgo' (result cell)
        int zz[SW ? kBlk + K : 1];          // SW: row 0's floor at steps 0 .. 19 of the block
        if constexpr (SW)
        {
            zz[0] = z0;
#pragma unroll
            for (int i = 1; i < kBlk + K; ++i) zz[i] = zz[i - 1] - ge;
        }
#pragma unroll
        for (int u = 0; u < kBlk; ++u)
        {
            const int upH = shr1z(H[K - 1]) + hc[u >> 2][u & 3];
            const int upF = AG ? shr1z(FD) + hf[u >> 2][u & 3] : 0;
            int nh[K], ne[K], h[K];
            int f = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
            {
                int q;
                if constexpr (Q8)
                    q = (int)(signed char)(qc[k][u >> 2] >> (8 * (u & 3)));
                else
                    q = (u & 1) ? qhi(qc[k][u >> 1]) : qlo(qc[k][u >> 1]);
                const int dg = (k == 0 ? D : H[k - 1]) + q;
                const int vup = (k == 0) ? upH : nh[k - 1];
                if constexpr (AG)
                {
                    const int fprev = (k == 0) ? upF : f;
                    f = SW ? max3i(fprev, vup, zz[SW ? u + k : 0]) : max(fprev, vup);
                    ne[k] = max(E[k], H[k]);
                    h[k] = max3i(dg, ne[k], f);
                    nh[k] = h[k] + dd;
                }
                else
                {
                    f = SW ? max(vup, zz[SW ? u + k : 0]) : vup;
                    h[k] = max3i(dg, H[k], f);
                    nh[k] = h[k];
                }
            }
            if constexpr (SW)
            {
#pragma unroll
                for (int k = 0; k < K; ++k)
                {
                    p[k] = max(p[k], (int)(((uint32_t)h[k] << 4) + wv));
                }
                wv += 16u * (uint32_t)ge - 1u;
            }
            if (u < kQD)
#pragma unroll
                for (int k = 0; k < K; ++k) qn[k][u] = lds_ld(qrow[k] + pn + 4u * u);
            lt[u] = H[K - 1];
            if constexpr (AG) lf[u] = FD;
            D = upH;
#pragma unroll
            for (int k = 0; k < K; ++k)
            {
                H[k] = nh[k];
                if constexpr (AG) E[k] = ne[k];
                if constexpr (!SW) va[k][u] = nh[k];
            }
            if constexpr (AG) FD = f;
            if (u == kBlk - 2)
            {
                asm volatile("" ::: "memory");
                const int2v lo = *(const int2v*)(krsm + f_in), hi = *(const int2v*)(krsm + f_in + 16u);
                asm volatile("" ::: "memory");
                rpin = lo.x;
                rpxo = lo.y;
                rpco = hi.y;
                rsink = hi.x;
            }
        }
        handoff(b);
        if constexpr (TAP)
        {
            // the tap lane alone (exec set and restored inside the asm), 64 B per row per block
            uint64_t sv;
            asm volatile("s_mov_b64 %0, exec\n"
                         "s_mov_b64 exec, %1\n"
                         "global_store_dwordx4 %2, %3, off\n"
                         "global_store_dwordx4 %2, %4, off offset:16\n"
                         "global_store_dwordx4 %2, %5, off offset:32\n"
                         "global_store_dwordx4 %2, %6, off offset:48\n"
                         "s_mov_b64 exec, %0"
                         : "=&s"(sv)
                         : "s"(tapMask), "v"(tapB + 64ull * (uint64_t)b), "v"(int4v {lt[0], lt[1], lt[2], lt[3]}),
                           "v"(int4v {lt[4], lt[5], lt[6], lt[7]}), "v"(int4v {lt[8], lt[9], lt[10], lt[11]}),
                           "v"(int4v {lt[12], lt[13], lt[14], lt[15]})
                         : "memory");
            if constexpr (AG)
                asm volatile("s_mov_b64 %0, exec\n"
                             "s_mov_b64 exec, %1\n"
                             "global_store_dwordx4 %2, %3, off\n"
                             "global_store_dwordx4 %2, %4, off offset:16\n"
                             "global_store_dwordx4 %2, %5, off offset:32\n"
                             "global_store_dwordx4 %2, %6, off offset:48\n"
                             "s_mov_b64 exec, %0"
                             : "=&s"(sv)
                             : "s"(tapMask), "v"(tapBF + 64ull * (uint64_t)b), "v"(int4v {lf[0], lf[1], lf[2], lf[3]}),
                               "v"(int4v {lf[4], lf[5], lf[6], lf[7]}), "v"(int4v {lf[8], lf[9], lf[10], lf[11]}),
                               "v"(int4v {lf[12], lf[13], lf[14], lf[15]})
                             : "memory");
        }
        if constexpr (SW)
        {
            // fold the block's best per row: score = key >> 4 - k |ge|, first step 15 - key & 15
#pragma unroll
            for (int k = 0; k < K; ++k)
            {
                const int v = (p[k] >> 4) + k * ge;
                const bool up = v > best[k];
                best[k] = up ? v : best[k];
                tb[k] = up ? kBlk * b + 15 - (p[k] & 15) : tb[k];
                p[k] = 0;
            }
            z0 = zz[SW ? kBlk : 0];
            wv = 15u - 16u * (uint32_t)z0;
        }
        else
        {
            if (hasR && (tStar >> 4) == b)
            {
                // (uniform) the result cell: lane laneR, row kR, step tStar & 15 of this block;
                // that lane parks the block's values in LDS and reads the one back
                const uint32_t scr = L.flags + 256u;
                if (lane == laneR)
                {
#pragma unroll
                    for (int k = 0; k < K; ++k)
#pragma unroll
                        for (int u = 0; u < kBlk; ++u) lds_st(scr + 4u * (uint32_t)(kBlk * k + u), va[k][u]);
                    const int v = lds_ld(scr + 4u * (uint32_t)(kBlk * kR + (tStar & 15)));
                    G(a.agResult)[0] = v - dd + (a.R + a.C) * ge;
                }
            }
        }
        return true;
    };

    if constexpr (SW) wv = 15u - 16u * (uint32_t)z0;
    for (int b = 0; b < NB; b += 2)
    {
        if (!block(b, qA, qB)) return;
        if (b + 1 >= NB) break;
        if (!block(b + 1, qB, qA)) return;
    }
    if constexpr (SW)
    {
        // this lane's best cell, first in row-major order (rows in order, first step per row):
        // key score << idxBits | (2^idxBits - 1 - row-major index); one 64-bit atomicMax per lane
        const unsigned long long W = (unsigned long long)a.C + 1, mask = (1ull << a.idxBits) - 1;
        unsigned long long key = 0;
        bool big = false;
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
            const bool in = rl + k <= a.R;
            // a score >= 2^26 (before the packing could wrap): the host's row scan
            big |= in && best[k] >= (1 << 26);
            if (in && best[k] > 0)
            {
                const unsigned long long idx =
                    (unsigned long long)(rl + k + a.rowOff) * W + (unsigned long long)(tb[k] - lane);
                const unsigned long long kk = ((unsigned long long)best[k] << a.idxBits) | (mask - idx);
                key = kk > key ? kk : key;
            }
        }
        if (key) atomicMax(a.swBest, key);
        if (big) atomicOr((unsigned*)a.agResult, 1u);
    }
}

// feeder wave: the row above strip 0 (Hgo' and F') into ring 0 -- ticket 0 from the border
// generator, later tickets from the previous ticket's granules (both arrays, in column order)
template <int MODE>
__device__ __forceinline__ void ks_feed(const StripArgs& a, const KsLds& L, int tk, int lane)
{
    constexpr bool AG = !is_lin_mode(MODE);
    const int Cp = a.Cp;
    const int dd = AG ? a.go - a.ge : 0;
    const uint32_t F = L.flags;
    const size_t prev = (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
    const gptr<const unsigned long long> gp = G((const unsigned long long*)a.gran) + prev;
    const gptr<const unsigned long long> gp2 = G((const unsigned long long*)a.gran2) + prev;
    int hnext = 0, c0 = 0, pw = 64;
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;
    while (hnext <= Cp)
    {
        bool moved = false;
        if (hnext + 128 > c0 + kRing) c0 = flag_ld(F + kr_cons(0));
        const bool feed = hnext + 128 <= c0 + kRing;
        const int c = hnext + lane;
        const bool in = c <= Cp && lane < pw;
        unsigned long long q = 0ull, q2 = 0ull;
        if (feed && tk > 0 && in)
        {
            q = __hip_atomic_load(gp + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if constexpr (AG) q2 = __hip_atomic_load(gp2 + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (feed)
        {
            int v, v2 = kNegS;
            bool good;
            if (tk == 0)
            {
                // row 0 shifted: global H'(0,c) = d for c >= 1 (0 at c = 0), local -c ge (H = 0);
                // carried as Hgo' = H' + d; F' = -inf
                v = is_sw_mode(MODE) ? dd - c * a.ge : (c == 0 ? dd : 2 * dd);
                good = in;
            }
            else
            {
                good = in && (uint32_t)(q >> 32) == a.epoch && (!AG || (uint32_t)(q2 >> 32) == a.epoch);
                v = (int)(uint32_t)q;
                v2 = (int)(uint32_t)q2;
            }
            const uint64_t badm = __ballot(!good);
            const int n = badm ? __builtin_ctzll(badm) : 64;
            if (tk > 0) pw = max(32, min(64, (n & ~15) + 16));
            if (n > 0)
            {
                if (lane < n)
                {
                    const uint32_t o = 4u * (uint32_t)((c + 64) & (kRing - 1));
                    lds_st(L.ring + o, v);
                    if constexpr (AG) lds_st(L.ring2 + o, v2);
                }
                hnext += n;
                flag_st(F, hnext > Cp ? kBig : hnext + 64);
                moved = true;
            }
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (moved)
            last = now;
        else
        {
            if (now - last > a.spin || ((++idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            if (tk == 0) __builtin_amdgcn_s_sleep(1);
        }
    }
}

// profiler wave: kr_loader's profile job (ROLE 2) with the NEG letter for columns <= 0 and > C; Q8:
// the int8 profile in 4 byte-shifted copies (kr_loader's Q8 build), NEG = -128 (the int8 instance
// runs only for tables whose s - go - ge all lie in [-127, 127])
template <bool Q8>
__device__ __forceinline__ void ks_profile(const StripArgs& a, const KsLds& L, int lane)
{
    constexpr int NS = kKrowNSDefault, LW = 1024;
    const int Cp = a.Cp, C = a.C;
    constexpr int kQRS = kr_qrs(LW, Q8), kQW = Q8 ? LW / 4 : LW / 2;
    const uint32_t F = L.flags;
    const uint32_t copy1 = kr_copy1(LW, a.substsz, Q8);
    auto letter = [&](int c) {
        if (c < 1 || c > C) return a.substsz;  // NEG
        const int x = G(a.seqX)[c];
        return ((unsigned)x < (unsigned)a.substsz) ? x : 0;
    };
    // columns -64 .. -1 (the ring's last dwords of every copy, read by lanes still left of column 0
    // in the first 4 blocks): NEG, or a stale profile there would lift the SW floor's values at
    // negative columns and flow into column 0 through E'.  The first batch that overwrites them
    // (columns 960..) waits until every strip is past them.
    {
        constexpr int kNeg = Q8 ? 17 : 32;  // dwords (int8: 64 columns + the copies' shift)
        constexpr int kCopies = Q8 ? 4 : 2;
        for (int i = lane; i < kCopies * kNeg * a.substsz; i += 64)
        {
            const int yy = i / (kCopies * kNeg), cp = (i / kNeg) % kCopies, dw = kQW - kNeg + i % kNeg;
            lds_st(L.q + 4u * ((uint32_t)cp * copy1 + kQRS * (uint32_t)yy + (uint32_t)dw), Q8 ? (int)0x80808080u : (int)0x80008000u);
        }
    }
    constexpr int kNX = Q8 ? 5 : 3;
    const int cp = lane >> 5;
    const int lb = Q8 ? 4 * (lane & 31) - 1 - 2 * cp : 2 * lane - 1;
    int xl[kNX], nxl[kNX];
#pragma unroll
    for (int i = 0; i < kNX; ++i)
    {
        xl[i] = letter(lb + i);
        nxl[i] = 0;
    }
    int qn = 0;
    int qsub = 0, pl = 0;
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;
    // every column a strip reads (lane 0 reaches column 16 NB - 1), not only those up to Cp: SW tracks
    // the cells right of C too, which the NEG letter keeps below the real maximum, so a stale profile
    // there (another launch's letters, or any bytes) must never be read
    const int qEnd = kBlk * ((Cp + 65 + kBlk - 1) / kBlk);
    while (qn < qEnd)
    {
        bool moved = false;
        if (qsub == 0 && qn + 192 > pl + LW) pl = flag_ld(F + kr_prog(NS));
        if (qsub > 0 || qn + 192 <= pl + LW)
        {
            int4v vx[kNX][2];
            {
                const uint32_t o = 32u * (uint32_t)qsub;
#pragma unroll
                for (int i = 0; i < kNX; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) vx[i][j] = lds_ld4(L.sub + 4u * kSubRow * (uint32_t)xl[i] + o + 16u * j);
            }
            if (qsub == 0)
            {
#pragma unroll
                for (int i = 0; i < kNX; ++i) nxl[i] = letter(qn + kBatch + lb + i);
            }
            // int16: dword of columns (cl, cl+1) / (cl-1, cl); int8: of columns 4d-2cp .. +3 / 4d-2cp-1 .. +2
            const uint32_t d = Q8 ? (uint32_t)((qn / 4 + (lane & 31)) & (kQW - 1)) : (uint32_t)((qn / 2 + lane) & (kQW - 1));
            const bool guard = d < (Q8 ? 4u : 8u);
            const uint32_t ce = L.q + 4u * ((Q8 ? (uint32_t)(2 * cp) * copy1 : 0u) + d);
            const uint32_t co = ce + 4u * copy1;
#pragma unroll
            for (int i = 0; i < 8; ++i)
            {
                const int yy = 8 * qsub + i;
                if (yy < a.substsz)
                {
                    int ev, od;
                    if constexpr (Q8)
                    {
                        const int w0 = vx[0][i >> 2][i & 3], w1 = vx[1][i >> 2][i & 3], w2 = vx[2][i >> 2][i & 3];
                        const int w3 = vx[3][i >> 2][i & 3], w4 = vx[4][i >> 2][i & 3];
                        od = (w0 & 0xff) | ((w1 & 0xff) << 8) | ((w2 & 0xff) << 16) | (w3 << 24);
                        ev = (int)__builtin_amdgcn_alignbyte((unsigned)w4, (unsigned)od, 1u);
                    }
                    else
                    {
                        const int s0 = vx[1][i >> 2][i & 3];
                        ev = (s0 & 0xffff) | (vx[2][i >> 2][i & 3] << 16);  // copy 0: (cl, cl+1)
                        od = (vx[0][i >> 2][i & 3] & 0xffff) | (s0 << 16);  // copy 1: (cl-1, cl)
                    }
                    const uint32_t ra = 4u * kQRS * (uint32_t)yy;
                    lds_st(ce + ra, ev);
                    lds_st(co + ra, od);
                    if (guard)
                    {
                        lds_st(ce + ra + 4u * kQW, ev);
                        lds_st(co + ra + 4u * kQW, od);
                    }
                }
            }
            if (++qsub == 4 || 8 * qsub >= a.substsz)
            {
                qsub = 0;
#pragma unroll
                for (int i = 0; i < kNX; ++i) xl[i] = nxl[i];
                qn += kBatch;
                flag_st(F + kFXo, qn >= qEnd ? kBig : qn);
            }
            moved = true;
        }
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        if (moved)
            last = now;
        else
        {
            if (now - last > a.spin || ((++idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// drain wave: the last strip's Hgo' (and F') -> granules for the next ticket
template <int MODE>
__device__ __forceinline__ void ks_drain(const StripArgs& a, const KsLds& L, int tk, int lane)
{
    constexpr int NS = kKrowNSDefault;
    constexpr bool AG = !is_lin_mode(MODE);
    const int Cp = a.Cp;
    const uint32_t F = L.flags, ringN = L.ring + (uint32_t)NS * (kRing * 4u);
    if (tk + 1 >= a.nTickets && !a.tapGran)
    {
        flag_st(F + kr_cons(NS), kBig);  // nobody reads our last row
        return;
    }
    const size_t off = (size_t)tk * a.granStride;
    const gptr<unsigned long long> go = G(a.gran) + off;
    const gptr<unsigned long long> go2 = G(a.gran2) + off;
    const unsigned long long ep = (unsigned long long)a.epoch << 32;
    int dnext = 0;
    uint64_t last = __builtin_amdgcn_s_memrealtime();
    unsigned idle = 0;
    while (dnext <= Cp)
    {
        const int avail = min(flag_ld(F + kr_prog(NS)) - 64, Cp + 1);
        if (dnext < avail)
        {
            const int c = dnext + lane;
            if (c < avail)
            {
                const uint32_t o = 4u * (uint32_t)((c + 64) & (kRing - 1));
                const int v = lds_ld(ringN + o);
                if constexpr (AG)
                {
                    const int v2 = lds_ld(ringN + kRing2Off + o);
                    __hip_atomic_store(go2 + c, ep | (uint32_t)v2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __hip_atomic_store(go + c, ep | (uint32_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            dnext = min(dnext + 64, avail);
            flag_st(F + kr_cons(NS), dnext > Cp ? kBig : dnext + 64);
            last = __builtin_amdgcn_s_memrealtime();
        }
        else
        {
            if (__builtin_amdgcn_s_memrealtime() - last > a.spin || ((++idle & 63) == 0 && err_set(a)))
            {
                atomicOr(a.err, 1u);
                return;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

// Q8: the int8-profile instance; it declines a table with some s - go - ge outside [-127, 127] as
// nw_krow_kernel's does (a.q8flag), and the int16 instance behind it (a.q8 = 2) runs only then
template <int MODE, bool Q8, int K>
__global__ void __launch_bounds__(64 * kr_waves<kKrowNSDefault>()) nw_kscore_kernel(StripArgs a)
{
    constexpr int NS = kKrowNSDefault;
    constexpr int kThreads = 64 * kr_waves<NS>();
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const KsLds L = ks_layout(a.substsz, Q8);
    if (!Q8 && a.q8 == 2 && __hip_atomic_load(a.q8flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != a.epoch) return;
    // subT[x][y] = s(y, x) - go - ge (int16 range checked), row x = substsz: the NEG letter
    bool bad = false, bad8 = false;
    for (int k = threadIdx.x; k < (a.substsz + 1) * kSubRow; k += kThreads)
    {
        const int x = k / kSubRow, yy = k % kSubRow;
        int v = 0;
        if (yy < a.substsz)
        {
            if (x < a.substsz)
            {
                v = G(a.subst)[yy * a.substsz + x] - a.go - a.ge;
                bad |= v <= kNegQ || v > 32767;
                bad8 |= v <= -128 || v > 127;
            }
            else
                v = Q8 ? -128 : kNegQ;
        }
        lds_st(L.sub + 4u * k, v);
    }
    if constexpr (Q8)
    {
        // decline (every workgroup sees the same table), reduced through a word of the dynamic LDS
        if (threadIdx.x == 0) lds_st(L.flags + kFTicket, 0);
        __syncthreads();
        if (bad8) atomicOr((int*)(krsm + L.flags + kFTicket), 1);
        __syncthreads();
        if (lds_ld(L.flags + kFTicket) != 0)
        {
            if (threadIdx.x == 0) __hip_atomic_store(a.q8flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    else if (bad)
        atomicOr(a.err, 2u);
    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) lds_st(L.flags + kFTicket, err_set(a) ? a.nTicketsTotal : (int)atomicAdd(a.ticket, 1u));
        __syncthreads();
        const int tkg = __builtin_amdgcn_readfirstlane(lds_ld(L.flags + kFTicket));
        if (tkg >= a.nTicketsTotal) break;
        // one pair (gsa_score), or score_bidi's two (three: local) pairs with their tickets
        // round-robin while they have some left (each pair's tickets are still claimed in order)
        int h = 0, tk = tkg + a.tkFirst;
        if (a.bidiTop > 0)
        {
            const int n0 = a.bidiTop, n1 = a.bidiMid > 0 ? a.bidiMid : a.nTicketsTotal - n0;
            const int n2 = a.bidiMid > 0 ? a.nTicketsTotal - n0 - n1 : 0;
            int g = tkg;
            for (int r = 0;; ++r)
            {
                const int c0 = r < n0, c1 = r < n1, c2 = r < n2;
                if (g < c0 + c1 + c2)
                {
                    h = g == 0 ? (c0 ? 0 : c1 ? 1 : 2) : g == 1 ? (c0 && c1 ? 1 : 2) : 2;
                    tk = r;
                    break;
                }
                g -= c0 + c1 + c2;
            }
        }
        const PairDesc d = kr_desc(a.pairs + h);
        StripArgs pa = a;
        pa.seqY = d.seqY;
        pa.seqX = d.seqX;
        pa.R = d.R;
        pa.C = d.C;
        pa.Cp = d.Cp;
        pa.nTickets = d.nTickets;
        pa.granStride = gran_stride(d.Cp);
        pa.gran = a.gran + d.granOff;
        pa.gran2 = a.gran2 + d.granOff;
        pa.tapGran = (a.tapGran >> h) & 1;
        pa.rowOff = d.rowOff;
        if (d.swBest) pa.swBest = d.swBest;
        if (h == 1)
        {
            pa.tapRow = a.tapRowB;
            pa.tapH = a.tapH + a.tapStride;
            pa.tapF = a.tapF + a.tapStride;
        }
        else if (h == 2)
            pa.tapRow = 0;
        if (threadIdx.x < 32) lds_st(L.flags + 4u * threadIdx.x, 0);
        // rings: -inf, so columns no writer reaches (past C at the strips' ends) hold nothing larger
        for (int k = threadIdx.x; k < 2 * (NS + 1) * kRing; k += kThreads) lds_st(L.ring + 4u * k, kNegS);
        __syncthreads();
        if (w == NS + 1)
            ks_drain<MODE>(pa, L, tk, lane);
        else if (w == NS)
            ks_feed<MODE>(pa, L, tk, lane);
        else if (w == NS + 2)
            ks_profile<Q8>(pa, L, lane);
        else
        {
            // score_bidi's tap: the strip with a lane whose last row is a.tapRow (uniform)
            const int r0 = tk * (64 * K * NS) + 64 * K * w + 1;
            const int rt = pa.tapRow - r0;
            __builtin_amdgcn_s_setprio(3);
            if (pa.tapRow > 0 && rt >= 0 && rt < 64 * K && (rt + 1) % K == 0)
                ks_strip<MODE, Q8, K, true>(pa, L, tk, w, lane, (rt + 1) / K - 1);
            else
                ks_strip<MODE, Q8, K>(pa, L, tk, w, lane);
            __builtin_amdgcn_s_setprio(0);
        }
    }
}

template <int MODE, bool Q8, int K>
hipError_t launch_ks1(const StripArgs& a, int grid, hipStream_t stream, bool foot)
{
    const size_t lds = krow_score_lds_bytes(a.substsz, Q8);
    auto kern = nw_kscore_kernel<MODE, Q8, K>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    constexpr int kThreads = 64 * kr_waves<kKrowNSDefault>();
    if (foot && (e = record_foot((const void*)kern, lds, kThreads, grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, stream, a);
    return hipGetLastError();
}

// a.q8: the int8 instance, then the int16 one behind it (a no-op unless the int8 launch declined)
template <int MODE, int K>
hipError_t launch_ks(const StripArgs& a, int grid, hipStream_t stream)
{
    if (!a.q8) return launch_ks1<MODE, false, K>(a, grid, stream, true);
    hipError_t e = launch_ks1<MODE, true, K>(a, grid, stream, true);
    if (e != hipSuccess) return e;
    StripArgs b = a;
    b.q8 = 2;
    return launch_ks1<MODE, false, K>(b, grid, stream, false);
}
#endif  // GSA_KROW_SCORE

}  // namespace

#if defined(GSA_KROW_SCORE) && defined(GSA_KSCORE_AFFINE)
// the affine modes (nw_kscore_ag.hip: its own translation unit, built with the iterative ILP
// scheduler: 50k NW-AG 3.86 -> 3.73 ms, profiles/r04_score_k.txt)
hipError_t launch_krow_score_affine(const StripArgs& a, int mode, int k, int grid, hipStream_t stream)
{
    if (k == 2)
    {
        if (mode == kModeScoreAG) return launch_ks<kModeScoreAG, 2>(a, grid, stream);
        if (mode == kModeScoreSW) return launch_ks<kModeScoreSW, 2>(a, grid, stream);
        return hipErrorInvalidValue;
    }
    if (mode == kModeScoreAG) return launch_ks<kModeScoreAG, 4>(a, grid, stream);
    if (mode == kModeScoreSW) return launch_ks<kModeScoreSW, 4>(a, grid, stream);
    return hipErrorInvalidValue;
}
#elif defined(GSA_KROW_SCORE)
// progress words (256 B) and the NW result cell's scratch (64 ints)
size_t krow_score_lds_bytes(int substsz, bool q8) { return (size_t)ks_layout(substsz, q8).flags + 512; }

hipError_t launch_krow_score(const StripArgs& a, int mode, int k, int grid, hipStream_t stream)
{
    // one pair, or score_bidi's two halves (bidiTop > 0), three with the fresh bottom (bidiMid > 0)
    if (a.nPairs != (a.bidiTop > 0 ? (a.bidiMid > 0 ? 3 : 2) : 1) || grid <= 0 || (k != 2 && k != 4))
        return hipErrorInvalidValue;
    if (mode == kModeScoreAG || mode == kModeScoreSW) return launch_krow_score_affine(a, mode, k, grid, stream);
    if (k == 2)
    {
        if (mode == kModeScoreAGL) return launch_ks<kModeScoreAGL, 2>(a, grid, stream);
        if (mode == kModeScoreSWL) return launch_ks<kModeScoreSWL, 2>(a, grid, stream);
        return hipErrorInvalidValue;
    }
    if (mode == kModeScoreAGL) return launch_ks<kModeScoreAGL, 4>(a, grid, stream);
    if (mode == kModeScoreSWL) return launch_ks<kModeScoreSWL, 4>(a, grid, stream);
    return hipErrorInvalidValue;
}
#elif defined(GSA_KROW_XR)
// pass 1 of the two-pass full fill (nw_krowx.hip): the XR instances, (4, 4) for single pairs and
// (8, 4) for batches
hipError_t launch_krow_fill_xr(const StripArgs& a, int ns, int grid, hipStream_t stream)
{
    return ns == 8 ? launch_kr<8, 4, 1024, 2>(a, grid, stream) : launch_kr<4, 4, 1024, 2>(a, grid, stream);
}

namespace {

// ------------------------------------------------------------------------------------
// The fused single-pair full fill: both passes of the two-pass fill in one launch.  A single pair's
// pass 1 is a chain of ceil(R / 1024) tickets -- ten workgroups for the 10k pair, 98 for 100k -- and
// its pass 2 needs a 64-row tile's rows only once the strips above and beside it have passed its
// columns.  So the first a.xP workgroups of 8 waves take the pass-1 tickets (waves 0..6 the (4, 4)
// K-rows roles, wave 7 the storer in the staged instance) and then expansion tasks; the others take
// expansion tasks only, in the host's ready-time order (nw_expand_dev.h ex_stream): every task's
// producers hold earlier claims, so they are resident and the waits end.  Hand-off, per the guide's
// inter-workgroup rules: row 64m and the header columns are stored write-through (sc1), their
// stores awaited (vmcnt), and a word per strip -- epoch << 32 | X -- published with a relaxed
// agent-scope store; a task's loader polls the words of the strips it reads, then an agent acquire
// precedes its loads.
//   PTF 3 (staged): the strips hand their row-64m segments to the storer wave through LDS
//     (kr_xstore), which stores them and publishes the words.  Under the expansion's store stream a
//     strip's own write-through stores filled its 63 vector-memory slots and stalled it (100k x 100k:
//     pass 1 6.2 -> 8.4 ms).
//   PTF 4 (direct): the strips store the segments and publish every 16 blocks themselves, as round 5
//     did: for small pairs, whose expansion never fills HBM, it saves the staging (10k x 10k: 110 ->
//     105 cycles per step; gsa_capi.hip enqueue_full_twopass picks).
// ------------------------------------------------------------------------------------
template <int NS, int W, bool Q8, int PTF>
__global__ void __launch_bounds__(64 * W) nw_full_fused_kernel(StripArgs a)
{
    constexpr int K = 4, LW = 1024;
    static_assert(kr_waves<NS>() <= W, "the pass-1 roles fit the workgroup");
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const KrLds L = kr_layout(NS, LW, a.substsz, Q8);
    const uint32_t word = L.flags + kFTicket;  // the workgroup's claims, via LDS
    if (!Q8 && a.q8 == 2 && __hip_atomic_load(a.q8flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != a.epoch) return;
    bool bad = false, bad8 = false;
    for (int k = threadIdx.x; k < a.substsz * kSubRow; k += 64 * W)
    {
        const int x = k / kSubRow, yy = k % kSubRow;
        const int v = yy < a.substsz ? G(a.subst)[yy * a.substsz + x] - 2 * a.g : 0;
        bad |= v < -32768 || v > 32767;
        bad8 |= v < -128 || v > 127;
        lds_st(L.sub + 4u * k, v);
    }
    if constexpr (Q8)
    {
        // a table outside int8: decline before claiming anything (nw_krow_kernel)
        if (threadIdx.x == 0) lds_st(word, 0);
        __syncthreads();
        if (bad8) atomicOr((int*)(krsm + word), 1);
        __syncthreads();
        if (lds_ld(word) != 0)
        {
            if (threadIdx.x == 0) __hip_atomic_store(a.q8flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __syncthreads();
    }
    else if (bad)
        atomicOr(a.err, 2u);
    if (threadIdx.x == 0) lds_st(word, (int)atomicAdd(a.xrole, 1u));
    __syncthreads();
    bool p1 = __builtin_amdgcn_readfirstlane(lds_ld(word)) < a.xP;
    // pass 1 (the LDS holds subT until the workgroup's last ticket)
    while (p1)
    {
        __syncthreads();
        if (threadIdx.x == 0) lds_st(word, err_set(a) ? a.nTicketsTotal : (int)atomicAdd(a.ticket, 1u));
        __syncthreads();
        const int tkg = __builtin_amdgcn_readfirstlane(lds_ld(word));
        if (tkg >= a.nTicketsTotal) break;
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
        const PairDesc d = kr_desc(a.pairs + lo);
        const int tk = (tks >= 0) ? tks : tkg - d.ticketBase;
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
        pa.granStride = gran_stride(d.Cp);
        pa.rows64 = d.rows64;
        pa.rpitch = d.rpitch;
        pa.xdone = a.xdone + (size_t)d.ticketBase * NS;  // the pair's strip words
        // (stamps: the ticket's start, and each strip's end -- the strips of a pair sweep the same
        // columns at the same pace, so their ends are spaced by the wavefront's lag)
        unsigned long long* const sst = a.stamps ? a.stamps + 4 * ((size_t)d.ticketBase + tk) * NS : nullptr;
        if (threadIdx.x < 32) lds_st(L.flags + 4u * threadIdx.x, 0);
        if (threadIdx.x >= kFCap / 4 && threadIdx.x < kFCap / 4 + 8) lds_st(L.flags + 4u * threadIdx.x, 0);
        if (PTF == 3 && threadIdx.x >= 64 && threadIdx.x < 64 + 3 * NS) lds_st(kr_xwords(L.flags) + 4u * (threadIdx.x - 64), 0);
        __syncthreads();
        if (PTF == 3 && w == NS + 3)
            kr_xstore<NS, K>(pa, L, tk, lane);
        else if (w == NS + 1)
            kr_drain<NS, K, LW, 3>(pa, L, tk, lane);
        else if (w == NS)
            kr_loader<NS, K, LW, kr_split<NS>() ? 1 : 0, Q8, GSA_FUSED_FEED_PIPE>(pa, L, tk, lane);
        else if (kr_split<NS>() && w == NS + 2)
            kr_loader<NS, K, LW, 2, Q8>(pa, L, tk, lane);
        else if (w < NS)
        {
            if (sst && lane == 0)
            {
                sst[4 * w] = __builtin_amdgcn_s_memrealtime();
                sst[4 * w + 2] = __builtin_amdgcn_s_memtime();
            }
            __builtin_amdgcn_s_setprio(3);
            kr_strip<NS, K, LW, PTF, Q8>(pa, L, tk, w, lane);
            __builtin_amdgcn_s_setprio(0);
            if (sst && lane == 0)
            {
                sst[4 * w + 1] = __builtin_amdgcn_s_memrealtime();
                sst[4 * w + 3] = __builtin_amdgcn_s_memtime();
            }
        }
    }
    // pass 2: the streamed expansion (nw_expand_dev.h ex_stream): W - 1 tile waves and a loader wave
    // that claims the tasks in the host's order, waits until the pass-1 strips of a task's rows have
    // published its columns (their progress words), and stages its inputs in LDS
    __syncthreads();  // (pass 1's LDS is dead)
    ExpandArgs xa {};
    xa.subst = a.subst;
    xa.substsz = a.substsz;
    xa.g = a.g;
    xa.pairs = a.xpair;
    xa.nPairs = a.nPairs;
    xa.nTasks = a.xTasks;
    xa.sched = a.xsched;
    xa.run = a.xrun;
    xa.spin = a.spin;
    xa.err = a.err;
    const xdev::ExFused fx {a.xdone, a.epoch, a.stamps ? a.stamps + 4 * (size_t)a.nTicketsTotal * NS : nullptr};
#ifndef GSA_FUSED_NO_EXPAND  // (diagnostic builds: pass 1 alone inside the fused kernel, results wrong)
    xdev::ex_stream<W, true>(xa, a.xcounter, fx, w, lane);
#endif
}

template <int NS, int W, bool Q8, int PTF>
hipError_t launch_fused1(const StripArgs& a, int grid, hipStream_t stream, bool foot)
{
    static_assert(W == kExpStreamWaves, "the streamed expansion's workgroup");
    static_assert(kr_waves<NS>() < W, "a storer wave beside the pass-1 roles");
    const size_t lds = std::max(krow_lds_bytes(NS, 1024, a.substsz, Q8) + (PTF == 3 ? kr_xstage_bytes(NS) : 0u),
                                expand_stream_lds_bytes(a.substsz));
    auto kern = nw_full_fused_kernel<NS, W, Q8, PTF>;
    constexpr int kThreads = 64 * W;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    if (grid <= 0)
    {
        int per_cu = 0, dev = 0, cus = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, kThreads, lds);
        if (e == hipSuccess) e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        grid = std::max(1, std::min(a.nTicketsTotal + a.xTasks, std::max(1, per_cu) * cus));
    }
    if (foot && (e = record_foot((const void*)kern, lds, kThreads, grid)) != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), lds, stream, a);
    return hipGetLastError();
}

template <int NS, int W, int PTF>
hipError_t launch_fused(const StripArgs& a, int grid, hipStream_t stream)
{
    if (!a.q8) return launch_fused1<NS, W, false, PTF>(a, grid, stream, true);
    hipError_t e = launch_fused1<NS, W, true, PTF>(a, grid, stream, true);
    if (e != hipSuccess) return e;
    StripArgs b = a;
    b.q8 = 2;
    return launch_fused1<NS, W, false, PTF>(b, grid, stream, false);
}

}  // namespace

hipError_t launch_full_fused(const StripArgs& a, int ns, int waves, bool staged, int grid, hipStream_t stream)
{
    if (!a.xpair || !a.xdone || !a.xrole || !a.xcounter) return hipErrorInvalidValue;
    if (ns == 4 && waves == 8) return staged ? launch_fused<4, 8, 3>(a, grid, stream) : launch_fused<4, 8, 4>(a, grid, stream);
    return hipErrorInvalidValue;
}
#elif defined(GSA_KROW_BATCH8)
// nw_krow8.hip: the 8-strip batch instance in a translation unit of its own, so it can be built
// with another instruction scheduler than the single-pair instances (Makefile)
hipError_t launch_krow_fill_b8(const StripArgs& a, int grid, hipStream_t stream)
{
    return launch_kr<8, 4, 1024>(a, grid, stream);
}
#else
hipError_t launch_krow_fill_b8(const StripArgs& a, int grid, hipStream_t stream);

size_t krow_lds_bytes(int ns, int lw, int substsz, bool q8) { return (size_t)kr_layout(ns, lw, substsz, q8).flags + 256; }

hipError_t launch_krow_fill(const StripArgs& a, int ns, int k, int lw, int grid, hipStream_t stream)
{
    if (k == 2) return ns == 2 ? launch_kr<2, 2, 512>(a, grid, stream) : launch_kr<4, 2, 1024>(a, grid, stream);
    (void)lw;  // 512 for (4, 4) measured slower for one pair and for batches (the first strip
               // is throttled by the window): 1024
    if (ns == 8) return launch_krow_fill_b8(a, grid, stream);
    if (a.done) return launch_kr<4, 4, 1024, 1>(a, grid, stream);  // mlsppt: (4, 4) only (enqueue_batch)
    return ns == 2 ? launch_kr<2, 4, 512>(a, grid, stream) : launch_kr<4, 4, 1024>(a, grid, stream);
}
#endif

}  // namespace gsa
