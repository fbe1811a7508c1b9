// nw_expand.h -- launch interface of the full-matrix expansion (nw_expand.hip): pass 2 of the
// two-pass full fill.  Pass 1 is the K-rows sparse fill (nw_krow.hip, its XR instance), which
// leaves the tile header columns (tBx = kExpTW) and every 64th row; pass 2 recomputes every
// 64-row x kExpTW-column tile from its top row and left column, all tiles at once.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "nw_strip.h"

namespace gsa {

constexpr int kExpHB = 256;       // pass-1 tile width (tBx): its header columns are every kExpHB columns
constexpr int kExpTW = 512;       // pass-2 tile width, a multiple of kExpHB (the header columns between
                                  // are recomputed: fewer ramp blocks per tile, 8 of 36)
constexpr int kExpRows = 64;      // rows of a wave's tile (one per lane)
constexpr int kRowsPad = 64;      // left pad (columns) of the pass-1 row buffer
constexpr unsigned kXDone = 0x3fffffffu;  // a pass-1 strip's progress word: the strip has finished

// Pass-1 row buffer of a pair: row 64m (m = 1 .. 4 x strips of pass 1) as shifted values
// H' = H - (64m + c) g, column c (-64 <= c <= Cp + 63: the strips' segments past both ends land in
// the pads) at rows64[(m - 1) * rpitch + kRowsPad + c]; rpitch is a multiple of 16 (64-byte segments)
__host__ __device__ inline long long rows64_pitch(int Cp) { return ((long long)kRowsPad + Cp + 64 + 15) & ~15ll; }

struct ExpandPair
{
    const int* seqY;
    const int* seqX;
    int R, C;
    int* score;
    long long ld;
    const int* rows64;  // pass-1 rows (rows64_pitch / rows64_count), shifted values
    long long rpitch;
    const int* hcol;    // pass-1 tile header columns, tile-major, 1 + kSparseTileBy per tile, unshifted
    int tcols;          // pass-1 tile columns (tBx = kExpHB)
    int colTiles;       // ceil(C / kExpTW)
    int rowChunks;      // ceil(R / ((kExpStreamWaves - 1) kExpRows)): tasks of the tile waves' rows
    int taskBase;       // first workgroup task of this pair (colTiles * rowChunks tasks)
    int p1Strip0;       // fused fill: the pair's first pass-1 strip word (ticketBase x ns)
    int p1Strips;       // ... and its strip count (tickets x ns)
    // the last kExpTW tile column is wider than kExpHB: it is split at its pass-1 boundary into
    // two tile columns (colTiles counts both), so the pair's last tiles are at most kExpHB wide
    int lastSplit;
    int pad;
};

// tile column jT of a pair: left boundary column and width
__host__ __device__ inline int ex_cb(const ExpandPair& d, int jT)
{
    return (d.lastSplit && jT == d.colTiles - 1) ? (jT - 1) * kExpTW + kExpHB : jT * kExpTW;
}
__host__ __device__ inline int ex_cols(const ExpandPair& d, int jT)
{
    const int cb = ex_cb(d, jT);
    const int w = (d.lastSplit && jT == d.colTiles - 2) ? kExpHB : kExpTW;
    return d.C - cb < w ? d.C - cb : w;
}

struct ExpandArgs
{
    const int* subst;
    int substsz;
    int g;
    const ExpandPair* pairs;
    int nPairs;
    int nTasks;
    // the schedule: {pair, task within the pair} per entry, in runs of `run` entries of one tile
    // column (a claim takes a run; an entry of pair -1 is padding); nTasks = its entries
    const int* sched;
    int run;
    unsigned* counter;  // the run claims (zeroed before the launch)
    // measurement (gsa_set_full_timing): per workgroup, wave 0's s_memtime cycles (low word) and
    // s_memrealtime ticks (100 MHz, high word) from its start to its end; null = off
    unsigned long long* clk;
    // watchdog ticks (s_memrealtime) and the sticky error word of the context
    unsigned long long spin;
    unsigned* err;
};

// The streamed expansion (nw_expand_dev.h ex_stream): persistent workgroups of kExpStreamWaves waves,
// kExpStreamWaves - 1 tile waves (tasks of (kExpStreamWaves - 1) x 64 rows) and one loader wave that
// claims runs of tasks from a.counter and stages their inputs in LDS, so the tile waves only compute
// and store.  grid <= 0: one workgroup per CU.  Pair arrays and the schedule in device memory.
constexpr int kExpStreamWaves = 8;
size_t expand_stream_lds_bytes(int substsz);
hipError_t launch_expand_stream(const ExpandArgs& a, hipStream_t stream, int grid);

}  // namespace gsa
