// nw_trace_dev.hip -- sparse (mlsp) traceback on the device.
//
// NwTrace2_Sparse (nwtrace2_sparse.cpp:102-257) walks from (adjrows-1, adjcols-1) to (0,0)
// and, each time it enters a tile, recomputes that tile from its header row and column
// (NwTrace2_AlignTile, :40-96).  Here one workgroup does the same walk on the GPU:
//   * the tile recompute is the row scan of nw_check.hip (lanes across 64-column panels,
//     H'[j] = max(H[i][j0], prefix-max E'), 6 DPP steps), over rows 1..iE and columns
//     1..jE only, and instead of the values it keeps, per cell, the move the walk would take
//     there: DIAG if H[i-1][j-1] >= H[i-1][j] and >= H[i][j-1], else UP if H[i-1][j] >=
//     H[i][j-1], else LEFT -- the reference's comparisons in its order (:144-176), 2 bits;
//   * the walk itself is uniform scalar control flow reading those codes back from LDS
//     (global scratch when the tile is wider than 512 columns) and emitting one edit byte per
//     move ('=', 'X', 'I', 'D'), in walk order; the host folds them into the reference's
//     run-length edit string and trace hash.
// Cells outside the real matrix are never visited and never influence a visited cell (all
// dependencies point up / left), so the padded tile (padding letter 0) gives the same moves
// as the reference's zeroed artificial cells.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "nw_trace_dev.h"

namespace gsa {

namespace {

template <typename T>
using gptr = __attribute__((address_space(1))) T*;
template <typename T>
__device__ __forceinline__ gptr<T> G(T* p)
{
    return (gptr<T>)p;
}

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

// move codes: diagonal with equal / different letters ('=' / 'X'), up ('I'), left ('D')
constexpr int kDiagEq = 0, kDiagX = 1, kUp = 2, kLeft = 3;

}  // namespace

extern __shared__ __attribute__((aligned(16))) int tsm[];

__host__ __device__ inline size_t trace_dir_words_dev(int tBy, int tBx)
{
    return (size_t)((tBy + 15) / 16) * ((tBx + 63) / 64) * 64;
}

constexpr int kTW = 4;  // waves per workgroup: the panels of a tile are pipelined over them

__device__ __forceinline__ int lds_flag_ld(int* p)
{
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_flag_st(int* p, int v)
{
    asm volatile("" ::: "memory");  // the boundary values are written before the word (LDS executes in order)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Move codes of tile (iT, jT) for rows 1..iE, columns 1..jE:
// word ((a-1)/16 * nP + (b-1)/64) * 64 + (b-1)%64 holds rows a..a+15 of column b, 2 bits each.
// Wave w takes panels w, w+kTW, ...; panel p reads its left boundary column from slot p % (kTW+1)
// and writes its right one to slot (p+1) % (kTW+1), publishing (panel << 16 | rows) every 16
// rows, so consecutive panels run 16 rows apart.
template <bool DIRS_LDS>
__device__ void tile_moves(const TraceArgs& a, int iT, int jT, int iE, int jE, int* sub, int* bnd, int* yraw,
                           int* xraw, int* bprog, unsigned* dirs, int w, int lane, bool first)
{
    const int g = a.g, tBx = a.tBx, tBy = a.tBy, BS = tBy + 1;
    const long long W = tBx + 1, H = tBy + 1;
    const long long k = (long long)iT * a.tcols + jT;
    const gptr<const int> hr = G(a.hrow) + k * W;
    const gptr<const int> hc = G(a.hcol) + k * H;
    const long long rbase = (long long)iT * tBy, cbase = (long long)jT * tBx;
    const int tid = threadIdx.x;
    __syncthreads();  // the previous walk has read its codes
    for (int e = tid; e <= iE; e += 64 * kTW)
    {
        bnd[e] = hc[e];  // slot 0: the tile's header column = left boundary of panel 0
        const long long r = rbase + e;
        yraw[e] = r < a.adjrows ? G(a.seqY)[r] : 0;
    }
    for (int c = tid; c <= jE; c += 64 * kTW) xraw[c] = G(a.seqX)[cbase + c];  // real columns only (c <= jE)
    if (tid <= kTW) bprog[tid] = (tid == 0) ? iE : -1;  // boundary 0 complete, the others empty
    __syncthreads();
    const int nP = (tBx + 63) / 64;
    const int nPu = (jE + 63) / 64;  // panels the walk can reach
    for (int p = w; p < nPu; p += kTW)
    {
        const int* bin = bnd + (p % (kTW + 1)) * BS;
        int* bout = bnd + ((p + 1) % (kTW + 1)) * BS;
        int* fin = bprog + p % (kTW + 1);
        int* fout = bprog + (p + 1) % (kTW + 1);
        const int j0 = 64 * p;
        const int col = j0 + 1 + lane;
        const bool valid = col <= tBx;
        const long long gc = cbase + col;
        const int xo = valid ? clamp_letter(gc < a.adjcols ? G(a.seqX)[gc] : 0, a.substsz) : 0;
        int up = valid ? hr[col] : 0;
        const int c1 = -(lane + 1) * g, c2 = -lane * g, c3 = (lane + 1) * g;
        const int last = min(63, tBx - 1 - j0);
        int Lprev = __builtin_amdgcn_readfirstlane(hr[j0]);  // H[0][j0]
        const int xr = (col <= jE) ? xraw[col] : -1;         // raw letter of this lane's column
        unsigned word = 0;
        int avail = 0;  // rows of the left boundary known to be written
        for (int i0 = 1; i0 <= iE; i0 += 16)
        {
            const int nr = min(16, iE - i0 + 1);
            const int need = i0 + nr - 1;
            while (avail < need)
            {
                const int v = lds_flag_ld(fin);
                if ((v >> 16) == (p == 0 ? 0 : p) && (v & 0xffff) >= need && v >= 0)
                    avail = v & 0xffff;
                else
                    __builtin_amdgcn_s_sleep(1);
            }
            // left boundary and letters of row i0+r in lane r (readlane, no LDS latency per row)
            const int Lv = (lane < nr) ? bin[i0 + lane] : 0;
            const int yrv = (lane < nr) ? yraw[i0 + lane] : 0;
            int s_nx = sub[clamp_letter(__builtin_amdgcn_readfirstlane(yrv), a.substsz) * a.substsz + xo];
            for (int r = 0; r < nr; ++r)
            {
                const int i = i0 + r;
                const int L = __builtin_amdgcn_readlane(Lv, r);
                const int yr = __builtin_amdgcn_readlane(yrv, r);
                const int s = s_nx;
                if (r + 1 < nr)
                    s_nx = sub[clamp_letter(__builtin_amdgcn_readlane(yrv, r + 1), a.substsz) * a.substsz + xo];
                const int diag = __builtin_amdgcn_update_dpp(Lprev, up, 0x138, 0xf, 0xf, false);  // H[i-1][b-1]
                const int m = max(max(diag + s + c1, up + c2), L) - L;
                const int h = wave_prefix_max(m) + L + c3;
                const int left = __builtin_amdgcn_update_dpp(L, h, 0x138, 0xf, 0xf, false);  // H[i][b-1]
                const int bdu = max(diag, up);
                int code = (diag < up) ? kUp : ((xr == yr) ? kDiagEq : kDiagX);
                code = (bdu < left) ? kLeft : code;
                word |= (unsigned)code << (2 * ((i - 1) & 15));
                if (((i - 1) & 15) == 15 || i == iE)
                {
                    dirs[((size_t)((i - 1) >> 4) * nP + p) * 64 + lane] = word;
                    word = 0;
                }
                if (lane == last) bout[i] = h;
                if (first && i == iE && col == jE) G(a.res)[1] = h;  // H[adjrows-1][adjcols-1] = align_cost
                Lprev = L;
                up = h;
            }
            if (lane == 0) lds_flag_st(fout, ((p + 1) << 16) | need);
        }
    }
    __syncthreads();
    (void)DIRS_LDS;
}

// band slot of tile t (uniform): a load through the scalar cache, so the wait for it counts
// LDS/scalar traffic only, not the walk's outstanding edit-byte stores
__device__ __forceinline__ int band_slot(const TraceArgs& a, long long t)
{
    typedef const __attribute__((address_space(4))) int* cptr;
    return ((cptr)a.tmap)[t];
}

// codes of band slot `slot` -> dst (LDS), by threads t0, t0 + nt, ...: 8 loads in flight per
// thread per round (a loop of single loads pays a round trip per 16 bytes)
__device__ __forceinline__ void copy_codes(const TraceArgs& a, int slot, unsigned* dst, int t, int nt)
{
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const size_t words = trace_dir_words_dev(a.tBy, a.tBx);
    const gptr<const u32x4> src = (gptr<const u32x4>)(a.tcodes + (size_t)slot * words);
    const size_t nq = words / 4;
    for (size_t q0 = 0; q0 < nq; q0 += (size_t)8 * nt)
    {
        u32x4 v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r)
        {
            const size_t q = q0 + (size_t)r * nt + t;
            if (q < nq) v[r] = src[q];
        }
#pragma unroll
        for (int r = 0; r < 8; ++r)
        {
            const size_t q = q0 + (size_t)r * nt + t;
            if (q < nq) ((u32x4*)dst)[q] = v[r];
        }
    }
}

// DBUF: a second LDS code buffer; while wave 0 walks a tile, the other waves copy the band tile
// the walk is predicted to enter next (the one a diagonal path from the entry cell would reach)
template <bool DIRS_LDS, bool DBUF>
__global__ void __launch_bounds__(64 * kTW) trace_sparse_kernel(TraceArgs a)
{
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int tBy = a.tBy;
    const int nP = (a.tBx + 63) / 64;
    int* sub = tsm;
    int* bnd = sub + 32 * 32;
    int* yraw = bnd + (kTW + 1) * (tBy + 1);
    int* xraw = yraw + (tBy + 1);
    int* bprog = xraw + (a.tBx + 1);
    int* state = bprog + 8;  // walk state handed from wave 0 to the others
    unsigned* dirs = DIRS_LDS ? (unsigned*)(state + 8) : a.dirs_scratch;
    unsigned* dnext = dirs + (DBUF ? trace_dir_words_dev(a.tBy, a.tBx) : 0);
    long long pre = -1;  // tile whose codes the other waves copied into dnext during the last walk
    for (int k = tid; k < a.substsz * a.substsz; k += 64 * kTW) sub[k] = G(a.subst)[k];

    int iT = a.iT0, jT = a.jT0, iE = a.iE0, jE = a.jE0;
    const int Wm = a.tBx, Hm = a.tBy;  // hrowLen-1, hcolLen-1
    long long n = 0;  // moves emitted (wave 0)
    bool first = true;
    if (tid == 0 && (iE == 0 || jE == 0))
    {
        // start cell on a header of its tile (empty sequence): the value is stored there
        const long long k = (long long)iT * a.tcols + jT;
        G(a.res)[1] = (iE == 0) ? G(a.hrow)[k * (a.tBx + 1) + jE] : G(a.hcol)[k * (a.tBy + 1) + iE];
    }
    for (;;)
    {
        if (iE > 0 && jE > 0)
        {
            // a tile trace_band precomputed (never the start tile, whose recompute yields the cost):
            // its codes are copied into LDS; any other is recomputed here
            const long long tile = (long long)iT * a.tcols + jT;
            int slot = -1;
            if (DBUF && tile == pre)
                slot = state[5];  // looked up by the copying waves
            else if (a.tmap && !first)
                slot = band_slot(a, tile);
            if (DBUF && slot >= 0 && tile == pre)
            {
                unsigned* t = dirs;  // copied during the last walk (the barrier after it orders the copy)
                dirs = dnext;
                dnext = t;
            }
            else if (slot >= 0 && DIRS_LDS)
            {
                __syncthreads();  // the previous walk has read its codes
                copy_codes(a, slot, dirs, tid, 64 * kTW);
                __syncthreads();
            }
            else if (slot >= 0)
                // codes too large for LDS: the walk reads the band tile where trace_band left it
                dirs = const_cast<unsigned*>(a.tcodes) + (size_t)slot * trace_dir_words_dev(a.tBy, a.tBx);
            else
            {
                if (!DIRS_LDS) dirs = a.dirs_scratch;
                tile_moves<DIRS_LDS>(a, iT, jT, iE, jE, sub, bnd, yraw, xraw, bprog, dirs, w, lane, first);
            }
        }
        first = false;
        int done = 0;
        if (DBUF)
        {
            // the tile a diagonal path from (iE, jE) reaches: left if it meets column 0 first, above
            // if row 0, up-left if both
            const int pi = iT - (iE <= jE ? 1 : 0), pj = jT - (jE <= iE ? 1 : 0);
            pre = -1;
            if (iE > 0 && jE > 0 && pi >= 0 && pj >= 0)
            {
                pre = (long long)pi * a.tcols + pj;
                if (w > 0)
                {
                    // wave 0 walks without waiting for this lookup; the slot reaches it in state[5]
                    const int ps = band_slot(a, pre);
                    if (tid == 64) state[5] = ps;
                    if (ps >= 0) copy_codes(a, ps, dnext, tid - 64, 64 * (kTW - 1));
                }
            }
        }
        if (w == 0)
        {
            // The walk goes by RUNS of equal moves: the move codes of the current 32-row x 64-column
            // window sit in one 64-bit value per lane (lane = column), and every lane l <= c evaluates move
            // k = c - l of a run from (r, c) at once -- a diagonal run reads row r - k of its own
            // column, an up run row r - k of column c, a left run row r of its own column.  One
            // ballot gives the run length, and the run's lanes store its edit bytes in walk order
            // ('=' 'X' 'I' 'D' packed in one word, indexed by the code).  A related pair's path
            // is a few moves to tens of moves per run; the loop is branch-free per run.
            constexpr unsigned kEdits = (unsigned)'=' | ((unsigned)'X' << 8) | ((unsigned)'I' << 16) | ((unsigned)'D' << 24);
            // a.cap >= adjrows + adjcols - 1 >= the moves of any path (the host sizes it so)
            gptr<unsigned char> edits = G(a.edits);
            int ci = __builtin_amdgcn_readfirstlane(iE), cj = __builtin_amdgcn_readfirstlane(jE);
            int dI = 1, dJ = 1;  // row / column step of the last run
            const int nG = (a.tBy + 15) / 16;  // 16-row code groups of a tile
            const int lane2 = 2 * lane;
            for (;;)
            {
                if (ci == 0 && cj == 0)
                {
                    done = 1;
                    break;
                }
                if (ci > 0 && cj > 0)
                {
                    // a window of 32 rows (two 16-row code groups, one 64-bit value per lane)
                    const int gh = (ci - 1) >> 5, pj = (cj - 1) >> 6;
                    const size_t at = ((size_t)(2 * gh) * nP + pj) * 64 + lane;
                    const unsigned lo = dirs[at];
                    const unsigned hi = 2 * gh + 1 < nG ? dirs[at + (size_t)nP * 64] : 0u;
                    const unsigned long long cw = ((unsigned long long)hi << 32) | lo;
                    const int ilo = 32 * gh + 1, jlo = 64 * pj + 1;
                    do
                    {
                        const int r = ci - ilo, c = cj - jlo;
                        const unsigned long long word =
                            ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)hi, c) << 32) |
                            (unsigned)__builtin_amdgcn_readlane((int)lo, c);
                        const int code = (int)((word >> (2 * r)) & 3u);
                        const int cls = code <= kDiagX ? kDiagEq : code;  // diagonal runs mix '=' and 'X'
                        const bool left = cls == kLeft, up = cls == kUp;
                        const unsigned m = cls == kDiagEq ? 1u : 0u;
                        // this lane's move k = c - lane: row r - k of its own column (diagonal), of
                        // column c (up), row r of its own column (left); the shift wraps mod 64 and
                        // lanes past the window's top are cut by the row limit below
                        const unsigned long long src = up ? word : cw;
                        const int sft = (left ? 0 : lane2) + 2 * (left ? r : r - c);
                        const unsigned f = (unsigned)(src >> (sft & 63)) & 3u;
                        const bool in = (f | m) == ((unsigned)cls | m);
                        // run length: the ones from lane c down (lanes above c shift out)
                        const unsigned long long M = __builtin_amdgcn_ballot_w64(in) << (63 - c);
                        const int lim = min(c + 1, left ? 64 : r + 1);
                        const int L = min((unsigned)__builtin_clzll(~M | 1ull), (unsigned)lim);
                        const unsigned k = (unsigned)(c - lane);  // this lane's move in the run
                        if (k < (unsigned)L) ((gptr<unsigned char>)(edits + n))[k] = (unsigned char)(kEdits >> (8 * f));
                        dI = left ? 0 : 1;
                        dJ = up ? 0 : 1;
                        ci -= dI * L;
                        cj -= dJ * L;
                        n += L;
                    } while (ci >= ilo && cj >= jlo);
                }
                else
                {
                    // on the matrix's top row (left moves) or left column (up moves)
                    const bool up = ci > 0;
                    const int L = min(up ? ci : cj, 64);
                    if (lane < L) edits[n + lane] = (unsigned char)(kEdits >> (8 * (up ? kUp : kLeft)));
                    dI = up ? 1 : 0;
                    dJ = up ? 0 : 1;
                    ci -= dI * L;
                    cj -= dJ * L;
                    n += L;
                }
                // into the tile above / left / up-left on reaching its header (nwtrace2_sparse.cpp:195-214)
                if ((ci == 0 && iT > 0) || (cj == 0 && jT > 0))
                {
                    const int diT = (ci == 0 && iT > 0) ? 1 : 0;
                    const int djT = (cj == 0 && jT > 0) ? 1 : 0;
                    iT -= diT;
                    jT -= djT;
                    if (ci == 0 && dI != 0) ci = Hm;
                    if (cj == 0 && dJ != 0) cj = Wm;
                    break;
                }
            }
            iE = ci;
            jE = cj;
            if (lane == 0)
            {
                state[0] = iT;
                state[1] = jT;
                state[2] = iE;
                state[3] = jE;
                state[4] = done;
            }
        }
        __syncthreads();
        iT = state[0];
        jT = state[1];
        iE = state[2];
        jE = state[3];
        done = state[4];
        if (done) break;
    }
    if (tid == 0) G(a.res)[0] = n;
}

// whole tiles, many workgroups: slot s = (list[2s], list[2s+1]), rows 1..min(tBy, rows left),
// columns 1..min(tBx, columns left)
__global__ void __launch_bounds__(64 * kTW) trace_band_kernel(TraceArgs a, const int* list, int n)
{
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int tBy = a.tBy;
    int* sub = tsm;
    int* bnd = sub + 32 * 32;
    int* yraw = bnd + (kTW + 1) * (tBy + 1);
    int* xraw = yraw + (tBy + 1);
    int* bprog = xraw + (a.tBx + 1);
    for (int k = tid; k < a.substsz * a.substsz; k += 64 * kTW) sub[k] = G(a.subst)[k];
    const size_t words = trace_dir_words_dev(a.tBy, a.tBx);
    for (int s = blockIdx.x; s < n; s += gridDim.x)
    {
        const int iT = __builtin_amdgcn_readfirstlane(G(list)[2 * s]);
        const int jT = __builtin_amdgcn_readfirstlane(G(list)[2 * s + 1]);
        const int iE = (int)min((long long)a.tBy, a.adjrows - 1 - (long long)iT * a.tBy);
        const int jE = (int)min((long long)a.tBx, a.adjcols - 1 - (long long)jT * a.tBx);
        if (iE > 0 && jE > 0)
            tile_moves<false>(a, iT, jT, iE, jE, sub, bnd, yraw, xraw, bprog, (unsigned*)a.tcodes + (size_t)s * words,
                              w, lane, false);
    }
}

size_t trace_lds_bytes(int tBy, int tBx, int substsz, bool dirs_lds)
{
    (void)substsz;
    const size_t base = (size_t)4 * (32 * 32 + (kTW + 1) * (tBy + 1) + (tBy + 1) + (tBx + 1) + 16);
    return base + (dirs_lds ? trace_dir_words(tBy, tBx) * 4 : 0);
}

size_t trace_dir_words(int tBy, int tBx) { return trace_dir_words_dev(tBy, tBx); }

hipError_t launch_trace_band(const TraceArgs& a, const int* list, int n, int grid, hipStream_t st)
{
    if (a.substsz > 32) return hipErrorInvalidValue;
    if (n <= 0) return hipSuccess;
    const size_t bytes = trace_lds_bytes(a.tBy, a.tBx, a.substsz, false);
    hipError_t e = hipFuncSetAttribute((const void*)trace_band_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(trace_band_kernel, dim3(std::max(1, std::min(grid, n))), dim3(64 * kTW), bytes, st, a, list, n);
    return hipGetLastError();
}

template <bool DIRS_LDS, bool DBUF>
static hipError_t launch_walk(const TraceArgs& a, size_t bytes, hipStream_t st)
{
    hipError_t e = hipFuncSetAttribute((const void*)trace_sparse_kernel<DIRS_LDS, DBUF>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((trace_sparse_kernel<DIRS_LDS, DBUF>), dim3(1), dim3(64 * kTW), bytes, st, a);
    return hipGetLastError();
}

hipError_t launch_trace_sparse(const TraceArgs& a, hipStream_t st)
{
    if (a.substsz > 32) return hipErrorInvalidValue;
    const bool lds = a.dirs_scratch == nullptr;
    const size_t bytes = trace_lds_bytes(a.tBy, a.tBx, a.substsz, lds);
    if (!lds) return launch_walk<false, false>(a, bytes, st);
    // a second code buffer for the band tile the walk enters next, when it fits
    const size_t bytes2 = bytes + trace_dir_words(a.tBy, a.tBx) * 4;
    if (a.tmap && a.tcodes && bytes2 <= 160 * 1024) return launch_walk<true, true>(a, bytes2, st);
    return launch_walk<true, false>(a, bytes, st);
}

}  // namespace gsa
