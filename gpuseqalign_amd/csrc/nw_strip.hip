// nw_strip.hip -- NW-LG score-matrix fill for gfx950 (MI355X), hand-written wave64 HIP.
//
// Replaces the reference's tiled anti-diagonal fill family (gpu3..gpu9,
// e.g. nwalign_gpu9_mlsp_diagdiagdiag.cu:69-360 Kernel B and its per-diagonal launch
// loop :616-660) with ONE persistent launch that sweeps horizontal strips:
//
//  * A wave owns a strip of 63 matrix rows.  Lane l>=1 is row (r0-1+l); lane 0 is a
//    HALO lane that replays the row just above the strip.  At local step t lane l
//    works on column (t-l), so one wave instruction advances one anti-diagonal.
//  * The recurrence (nwalign_cpu1_st_row.cpp:4-10) runs in the shifted space
//        H'[i][j] = H[i][j] - (i+j)*g
//    where it becomes  H'[i][j] = max3(H'[i-1][j-1] + s(i,j) - 2g, H'[i-1][j], H'[i][j-1]):
//    three VALU ops per cell (v_add_u32_dpp, v_max3 / v_max_dpp); the up/diag neighbours
//    arrive from lane l-1 through DPP wave_shr:1.  H' is >= 0 and non-decreasing along
//    rows and columns, which is what lets the halo lane replay the row above through
//    the same instruction stream (its diag input is 0 and its S input is the value).
//  * s(i,j)-2g comes from a per-wave LDS profile P[x][lane] (conflict-free: bank = lane);
//    column letters come from a per-workgroup LDS ring of x*256 byte offsets.
//  * A workgroup holds NS strips (a "super-strip" of 63*NS rows = one tile row of the
//    sparse format).  Waves run in lock-step blocks of BLK steps separated by s_barrier;
//    wave w lags wave w-1 by DELTA blocks and reads wave w-1's last row straight from
//    its LDS staging ring (the staging ring holds every computed cell for a few blocks).
//  * Super-strips are handed out by an atomic ticket (so the launch cannot deadlock
//    whatever the residency); super-strip k's wave 0 consumes super-strip k-1's last
//    row from HBM through 8-byte {epoch, value} granules (sc1 stores / sc1 loads,
//    MI355X_MICROARCH.md "R2" form) -- no flags, no fences.
//
// Outputs (MODE):
//  * FULL   : the whole (R+1) x (C+1) int32 matrix, row-major, unpadded
//             (what NwAlign_Gpu3..6 return in nw.score after their 2-D crop).
//  * SPARSE : tileHrowMat / tileHcolMat exactly as gpu7/8/9 leave them, for tile
//             height tBy = 63*NS and a tile width tBx (multiple of 16, >= 64);
//             padded cells use letter 0 as the reference does
//             (nwalign_gpu9_mlsp_diagdiagdiag.cu:469-478).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nw_strip.h"

namespace gsa {

constexpr int kRowsPerWave = 63;  // lane 0 is the halo
constexpr int kSR = 96;           // staging ring depth (steps); multiple of 32 and of BLK
constexpr int kSlot = 65;         // dwords per staging slot (64 lanes + 1 pad: conflict-free column reads)
constexpr int kXR = 1024;         // column-letter ring (entries), plus a BLK mirror
constexpr int kHN = 128;          // inter-workgroup halo ring (entries, power of 2)
constexpr int kRN = 128;          // halo-ramp entries per wave (>= kSR, kHN)
constexpr int kNegS = -(1 << 29); // "minus infinity" profile row for columns <= 0

extern __shared__ __attribute__((aligned(16))) char smem[];

__device__ __forceinline__ int lds_ld(uint32_t a) { return *(const int*)(smem + a); }
__device__ __forceinline__ void lds_st(uint32_t a, int v) { *(int*)(smem + a) = v; }

// lane l <- lane l-1, lane 0 <- 0 (DPP wave_shr:1, bound_ctrl zero)
__device__ __forceinline__ int shr1z(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xF, 0xF, true); }

struct Lds {
    uint32_t st, prof, rmp, xo, hrg, misc, psz;
};

template <int NS>
__device__ __forceinline__ Lds lds_layout(int substsz)
{
    Lds L;
    L.psz = (uint32_t)(substsz + 1) * 256u;
    L.st = 0;
    L.prof = L.st + NS * kSR * kSlot * 4;
    L.rmp = L.prof + NS * L.psz;
    L.xo = L.rmp + NS * kRN * 4;
    L.hrg = L.xo + (kXR + 64) * 4;
    L.misc = L.hrg + kHN * 4;
    return L;
}

size_t strip_lds_bytes(int ns, int substsz)
{
    size_t psz = (size_t)(substsz + 1) * 256u;
    return (size_t)ns * kSR * kSlot * 4 + ns * psz + (size_t)ns * kRN * 4 + (kXR + 64) * 4 + kHN * 4 + 16;
}

// Poll one {epoch, value} granule written by the previous super-strip.  Bounded by wall
// time (s_memrealtime, 100 MHz): on time-out the error word is set and every later poll of
// the launch returns at once, so a broken hand-off ends the kernel instead of hanging it.
__device__ __forceinline__ int poll_granule(const StripArgs& a, const unsigned long long* gp)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;)
    {
        unsigned long long q = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(q >> 32) == a.epoch) return (int)(uint32_t)q;
        if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return 0;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull)  // 0.2 s
        {
            atomicOr(a.err, 1u);
            return 0;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ void xo_store(const Lds& L, int c, int v)
{
    int k = c & (kXR - 1);
    lds_st(L.xo + 4 * k, v);
    if (k < 64) lds_st(L.xo + 4 * (kXR + k), v);  // mirror so a block never wraps
}

// One block of BLK wavefront steps: the whole hot loop.  S values of this block are
// already in registers (s); the next block's letter offsets and S values are fetched
// while this block computes (LAG steps between a letter read and its S read), so no
// LDS latency is exposed on the critical chain.
template <int BLK>
__device__ __forceinline__ void sweep_block(int& c0, int& c1, int (&s)[BLK], uint32_t xo_next, uint32_t laneoff,
                                            uint32_t st_base)
{
    constexpr int LAG = 4;
    int xn[BLK];
    int sn[BLK];
#pragma unroll
    for (int u = 0; u < BLK + LAG; ++u)
    {
        if (u < BLK) xn[u] = lds_ld(xo_next + 4 * u);
        if (u >= LAG) sn[u - LAG] = lds_ld((uint32_t)xn[u - LAG] + laneoff);
        if (u < BLK)
        {
            int d = shr1z(c1) + s[u];      // H'[i-1][j-1] + s - 2g
            int e = max(d, c0);            // vs H'[i][j-1]
            int cn = max(shr1z(c0), e);    // vs H'[i-1][j]
            lds_st(st_base + 4 * kSlot * u, cn);
            c1 = c0;
            c0 = cn;
        }
    }
#pragma unroll
    for (int u = 0; u < BLK; ++u) s[u] = sn[u];
}

template <int BLK>
__device__ __forceinline__ void load_block(int (&s)[BLK], uint32_t xo_cur, uint32_t laneoff)
{
    int x[BLK];
#pragma unroll
    for (int u = 0; u < BLK; ++u) x[u] = lds_ld(xo_cur + 4 * u);
#pragma unroll
    for (int u = 0; u < BLK; ++u) s[u] = lds_ld((uint32_t)x[u] + laneoff);
}

typedef int int4a __attribute__((ext_vector_type(4), aligned(4)));

// letter byte-offset for column c given its loaded letter x
__device__ __forceinline__ int x_offset(const StripArgs& a, int c, int x)
{
    if (c <= 0 || c > a.Cp) return a.substsz * 256;  // NEG row
    if (c > a.C) return 0;                            // padding letter 0
    return ((unsigned)x < (unsigned)a.substsz ? x : 0) * 256;
}

__device__ __forceinline__ int load_letter(const StripArgs& a, int c) { return (c >= 1 && c <= a.C) ? a.seqX[c] : 0; }

// Raw workgroup barrier: waits for this wave's LDS traffic only (global stores stay in
// flight); the "memory" clobber keeps the compiler from moving memory ops across it.
#ifndef GSA_STAMP
#define GSA_STAMP 0
#endif
// Diagnostic stamps (separate build, never in the shipped library): s_memtime at fixed points
// of the first 256 blocks of ticket 0, lane 0 of each wave.
__device__ __forceinline__ void stamp(const StripArgs& a, int tk, int w, int G, int k, int lane)
{
    if constexpr (GSA_STAMP)
    {
        if (tk == 0 && G < 256 && lane == 0 && a.dbg)
        {
            unsigned long long t;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
            a.dbg[((size_t)w * 256 + G) * 4 + k] = t;
        }
    }
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Workgroup = NS compute waves (one 63-row strip each) + 1 loader wave (wave NS) that owns
// every global load of the sweep: column letters and the previous super-strip's last row,
// fetched in 64-column chunks several blocks ahead.  The two roles run separate loops with
// the same barrier count, so the compute loop carries no pending loads (no vmcnt waits).
template <int NS, int BLK, int MODE>
__global__ void __launch_bounds__(64 * (NS + 1)) nw_strip_kernel(StripArgs a)
{
    // block lag between waves: wave w's halo lane prefetches (one block ahead) wave w-1's
    // row-63 cells up to 2*BLK-1+63 steps past its own block start.
    constexpr int DELTA = 2 + (kRowsPerWave + BLK - 1) / BLK;
    constexpr int CPB = 64 / BLK;  // blocks per 64-column chunk
    static_assert(kSR % BLK == 0 && kSR % 32 == 0 && 64 % BLK == 0, "ring geometry");
    const int w = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const bool loader = (w == NS);
    const Lds L = lds_layout<NS>(a.substsz);
    const int g = a.g;
    const int NB = (a.Cp + 64 + BLK - 1) / BLK + 1;  // local blocks per strip
    const int NG = NB + DELTA * (NS - 1);           // global blocks per super-strip
    const uint32_t my_st = L.st + (uint32_t)w * kSR * kSlot * 4;
    const uint32_t my_prof = L.prof + (uint32_t)w * L.psz;
    const uint32_t my_rmp = L.rmp + (uint32_t)w * kRN * 4;
    const int rn = (w == 0) ? kHN : kSR;  // period of this wave's halo ramp

    // Static halo-address ramps: lane 0 of wave w reads, at local step t, the value of the
    // row above at column t.  Wave 0: the inter-workgroup ring; wave w>0: lane 63 of wave
    // w-1's staging slot for its step t+63.
    if (!loader)
        for (int k = lane; k < rn; k += 64)
        {
            uint32_t v = (w == 0) ? L.hrg + 4u * (uint32_t)k
                                  : L.st + (uint32_t)(w - 1) * kSR * kSlot * 4 + 4u * kSlot * (uint32_t)((k + 63) % kSR) +
                                        4u * 63;
            lds_st(my_rmp + 4 * k, (int)v);
        }

    for (;;)
    {
        __syncthreads();
        if (threadIdx.x == 0) lds_st(L.misc, (int)atomicAdd(a.ticket, 1u));
        __syncthreads();
        const int tk = lds_ld(L.misc);
        if (tk >= a.nTickets) break;

        const int rbase = tk * kRowsPerWave * NS;     // halo row of wave 0
        const int r0 = rbase + kRowsPerWave * w + 1;  // first real row of wave w
        const int row = r0 - 1 + lane;                // this lane's row

        for (int k = threadIdx.x; k < kXR + 64; k += 64 * (NS + 1)) lds_st(L.xo + 4 * k, a.substsz * 256);
        if (!loader)
        {
            int y = (lane == 0) ? 0 : (row <= a.R ? a.seqY[row] : 0);
            y = ((unsigned)y < (unsigned)a.substsz) ? y : 0;
            const int* srow = a.subst + y * a.substsz;
            for (int x = 0; x < a.substsz; ++x) lds_st(my_prof + 256 * x + 4 * lane, lane == 0 ? 0 : srow[x] - 2 * g);
            lds_st(my_prof + 256 * a.substsz + 4 * lane, kNegS);
        }
        __syncthreads();

        if (loader)
        {
            // ================= loader wave =================
            const unsigned long long* gprev = a.gran + (size_t)(tk > 0 ? tk - 1 : 0) * a.granStride;
            const bool hand = tk > 0;
            auto gload = [&](int c) -> unsigned long long {
                return (hand && c <= a.Cp) ? __hip_atomic_load(gprev + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                           : 0ull;
            };
            auto publish = [&](int c, int x, unsigned long long q) {
                xo_store(L, c, x_offset(a, c, x));
                int v = 0;
                if (hand && c <= a.Cp) v = ((uint32_t)(q >> 32) == a.epoch) ? (int)(uint32_t)q : poll_granule(a, gprev + c);
                lds_st(L.hrg + 4 * (c & (kHN - 1)), v);
            };
            // chunk 0 now; letters of chunks 1..3 and granules of chunks 1..2 in flight
            publish(lane, load_letter(a, lane), gload(lane));
            int xa = load_letter(a, 64 + lane), xb = load_letter(a, 128 + lane), xc = load_letter(a, 192 + lane);
            unsigned long long qa = gload(64 + lane), qb = gload(128 + lane);
            lds_barrier();
            for (int G = 0; G < NG; ++G)
            {
                stamp(a, tk, w, G, 0, lane);
                if (G % CPB == 0)
                {
                    // chunk n+1 (needed from block 4n+3's prefetch on); fetch chunk n+4 / n+3
                    const int n = G / CPB;
                    publish(64 * (n + 1) + lane, xa, qa);
                    xa = xb;
                    xb = xc;
                    xc = load_letter(a, 64 * (n + 4) + lane);
                    qa = qb;
                    qb = gload(64 * (n + 3) + lane);
                }
                stamp(a, tk, w, G, 2, lane);
                lds_barrier();
            }
        }
        else
        {
            // ================= compute waves =================
            lds_barrier();
            int c0 = 0, c1 = 0;
            int sv[BLK];
            const uint32_t laneoff = (lane == 0) ? 0u : my_prof + 4u * lane;
            const int hgl = (rbase + kRowsPerWave * NS);  // global row of the super-strip's last row
            for (int G = 0; G < NG; ++G)
            {
                stamp(a, tk, w, G, 0, lane);
                const int b = G - DELTA * w;
                if (b >= 0 && b < NB)
                {
                    const int t0 = BLK * b;
                    const uint32_t st_base = my_st + 4u * kSlot * (uint32_t)(t0 % kSR) + 4u * lane;
                    if (b == 0)
                    {
                        const uint32_t xo_cur = (lane == 0) ? my_rmp : L.xo + 4u * (uint32_t)((-lane) & (kXR - 1));
                        load_block<BLK>(sv, xo_cur, laneoff);
                    }
                    const int t1 = t0 + BLK;
                    const uint32_t xo_next = (lane == 0) ? my_rmp + 4u * (uint32_t)(t1 % rn)
                                                         : L.xo + 4u * (uint32_t)((t1 - lane) & (kXR - 1));
                    sweep_block<BLK>(c0, c1, sv, xo_next, laneoff, st_base);
                    stamp(a, tk, w, G, 1, lane);

                    if constexpr (MODE == kModeFull)
                    {
                        // write out columns [c0s, c0s+BLK) of the 63 rows: complete once step
                        // c0s+BLK-1+63 ran.  Lanes hold 4 consecutive columns of one row
                        // (16-byte stores, 4-byte aligned rows).
                        static_assert(BLK == 16, "write-out mapping assumes 16-column blocks");
                        constexpr int LAGB = (kRowsPerWave + BLK) / BLK;
                        const int c0s = BLK * (b - LAGB);
                        if (c0s + BLK > 0 && c0s <= a.C)
                        {
                            const int j0 = c0s + 4 * (lane & 3);
                            // staging slot of (row l, column j0+k) is (j0+k+l) mod kSR; l = 16p + (lane>>2) + 1
                            int sl0 = (j0 + (lane >> 2) + 1) % kSR;
#pragma unroll
                            for (int p = 0; p < 4; ++p)
                            {
                                const int l = 16 * p + (lane >> 2) + 1;
                                const int rr = r0 - 1 + l;
                                if (l < 64 && rr <= a.R && j0 + 3 >= 1 && j0 <= a.C)
                                {
                                    int v[4];
#pragma unroll
                                    for (int k = 0; k < 4; ++k)
                                    {
                                        int sl = sl0 + k;
                                        sl = (sl >= kSR) ? sl - kSR : sl;
                                        v[k] = lds_ld(my_st + 4u * (kSlot * (uint32_t)sl + (uint32_t)l)) + (rr + j0 + k) * g;
                                    }
                                    int* dst = a.score + (size_t)rr * (size_t)a.ld + j0;
                                    if (j0 >= 1 && j0 + 3 <= a.C)
                                        *(int4a*)dst = int4a {v[0], v[1], v[2], v[3]};
                                    else
                                    {
#pragma unroll
                                        for (int k = 0; k < 4; ++k)
                                            if (j0 + k >= 1 && j0 + k <= a.C) dst[k] = v[k];
                                    }
                                }
                                sl0 += 16;
                                sl0 = (sl0 >= kSR) ? sl0 - kSR : sl0;
                            }
                        }
                    }
                    else
                    {
                        // Sparse: header column of tile (tk, jT) at column cb = jT*tBx is
                        // complete after step cb+63.
                        const int lo = t0 - 63, hi = t0 + BLK - 1 - 63;  // cb in [lo, hi]
                        const int cb = (lo <= 0) ? 0 : ((lo + a.tBx - 1) / a.tBx) * a.tBx;
                        if (cb <= hi && cb <= a.Cp - a.tBx && cb >= lo)
                        {
                            const int jT = cb / a.tBx;
                            if (w == 0 || lane >= 1)
                            {
                                int v = lds_ld(my_st + 4u * (kSlot * (uint32_t)((cb + lane) % kSR) + (uint32_t)lane));
                                a.hcol[((size_t)tk * a.tcols + jT) * (size_t)(a.tBy + 1) + kRowsPerWave * w + lane] =
                                    v + (row + cb) * g;
                            }
                        }
                    }

                    if (w == NS - 1 && lane < BLK)
                    {
                        // last row of the super-strip for steps [t0, t0+BLK): column t0+lane-63
                        const int c = t0 + lane - 63;
                        if (c >= 0 && c <= a.Cp)
                        {
                            int v = lds_ld(my_st + 4u * (kSlot * (uint32_t)((t0 + lane) % kSR) + 63u));
                            if (tk + 1 < a.nTickets)
                            {
                                unsigned long long q = ((unsigned long long)a.epoch << 32) | (uint32_t)v;
                                __hip_atomic_store(a.gran + (size_t)tk * a.granStride + c, q, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                            }
                            if constexpr (MODE == kModeSparse)
                            {
                                if (tk + 1 < a.trows)
                                {
                                    const int hv = v + (hgl + c) * g;
                                    const int jT = c / a.tBx, jj = c - jT * a.tBx;
                                    const size_t rowbase = (size_t)(tk + 1) * a.tcols;
                                    if (jT < a.tcols) a.hrow[(rowbase + jT) * (size_t)(a.tBx + 1) + jj] = hv;
                                    if (jj == 0 && jT > 0) a.hrow[(rowbase + jT - 1) * (size_t)(a.tBx + 1) + a.tBx] = hv;
                                }
                            }
                        }
                    }
                }
                stamp(a, tk, w, G, 2, lane);
                lds_barrier();
            }
        }
    }
}

// Headers: row 0 / column 0 of the full matrix, or header row of tile row 0 (Kernel A of
// nwalign_gpu9_mlsp_diagdiagdiag.cu:15-63; column 0 comes out of the strip kernel).
__global__ void nw_headers_kernel(StripArgs a, int mode)
{
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (mode == kModeFull)
    {
        if (tid <= a.C) a.score[tid] = (int)tid * a.g;
        if (tid >= 1 && tid <= a.R) a.score[(size_t)tid * (size_t)a.ld] = (int)tid * a.g;
    }
    else
    {
        const int64_t n = (int64_t)a.tcols * (a.tBx + 1);
        if (tid < n)
        {
            const int jT = (int)(tid / (a.tBx + 1)), jj = (int)(tid % (a.tBx + 1));
            a.hrow[tid] = (jT * a.tBx + jj) * a.g;
        }
    }
}

template <int NS, int BLK, int MODE>
static hipError_t launch_strip(const StripArgs& a, int grid, hipStream_t stream)
{
    const size_t lds = strip_lds_bytes(NS, a.substsz);
    auto kern = nw_strip_kernel<NS, BLK, MODE>;
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * (NS + 1)), lds, stream, a);
    return hipGetLastError();
}

hipError_t launch_headers(const StripArgs& a, int mode, hipStream_t stream)
{
    int64_t n = (mode == kModeFull) ? (int64_t)(a.R > a.C ? a.R : a.C) + 1 : (int64_t)a.tcols * (a.tBx + 1);
    int blocks = (int)((n + 255) / 256);
    hipLaunchKernelGGL(nw_headers_kernel, dim3(blocks), dim3(256), 0, stream, a, mode);
    return hipGetLastError();
}

hipError_t launch_strip_fill(const StripArgs& a, int mode, int grid, hipStream_t stream)
{
    if (mode == kModeFull) return launch_strip<kStripNS, kStripBLK, kModeFull>(a, grid, stream);
    return launch_strip<kStripNS, kStripBLK, kModeSparse>(a, grid, stream);
}

}  // namespace gsa
