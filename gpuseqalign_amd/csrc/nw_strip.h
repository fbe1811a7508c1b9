// nw_strip.h -- launch interface of the strip-wavefront NW-LG fill (nw_strip.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gsa {

struct ExpandPair;  // nw_expand.h

constexpr int kModeFull = 0;  // full matrix (nw_lane.hip; launch_headers)
constexpr int kModeSparse = 1;
// Score-only global alignment with affine gaps on the strip layout (gsa_score_dev, global):
// shifted by (i+j)*gape, H', E', F' follow max recurrences with the constant d = gapo - gape.
constexpr int kModeScoreAG = 3;
// Score-only local alignment (Smith-Waterman) with affine gaps, same layout: the clamp at 0 is
// a per-row floor (i+j)*(-gape) in the shifted space; the best cell goes to a packed atomicMax.
constexpr int kModeScoreSW = 4;
// The same with a linear gap (gapo == gape, so d = 0): E' and F' never exceed H' and drop out, and
// only H' is handed between strips (BASELINE configs[4]'s SW-LG)
constexpr int kModeScoreSWL = 5;
// NW (global) with a linear gap: the AG step without E' and F' (d = 0)
constexpr int kModeScoreAGL = 6;
__host__ __device__ constexpr bool is_sw_mode(int mode) { return mode == kModeScoreSW || mode == kModeScoreSWL; }
__host__ __device__ constexpr bool is_ag_mode(int mode) { return mode == kModeScoreAG || mode == kModeScoreAGL; }
__host__ __device__ constexpr bool is_lin_mode(int mode) { return mode == kModeScoreSWL || mode == kModeScoreAGL; }
__host__ __device__ constexpr bool is_score_mode(int mode) { return is_ag_mode(mode) || is_sw_mode(mode); }
constexpr int kWaveRows = 256;                          // rows per strip (one wave, 4 rows per lane)
constexpr int kSparseNS = 4;                            // strip waves per workgroup, sparse fills
constexpr int kSparseTileBy = kWaveRows * kSparseNS;    // = tile height of the mlsp matrices

// One pair of a batched fill (device-resident array; tickets of pair p are
// [ticketBase, ticketBase + nTickets), pair-major, so every ticket depends only on lower ones).
struct PairDesc
{
    const int* seqY;
    const int* seqX;
    int R, C, Cp, nTickets;
    int ticketBase, trows, tcols;
    int rowOff;  // score_bidi, local: the pair's first row - 1 in the whole matrix (the end-cell key)
    unsigned long long* swBest;  // score_bidi, local: this pair's end-cell keys (null: StripArgs::swBest)
    int* score;
    long long ld;
    int* hrow;
    int* hcol;
    long long granOff;  // first granule of this pair in the hand-off buffer
    int* rows64;        // two-pass full fill, pass 1: rows 64m (nw_expand.h), or null
    long long rpitch;
};

// Granules per super-strip boundary of a pair whose last computed column is Cp: Cp + 1 rounded up
// to 16, so every 16-column chunk a drain stores with one instruction is one aligned 128-B line
__host__ __device__ inline long long gran_stride(int Cp) { return ((long long)Cp + 16) & ~15ll; }

struct StripArgs
{
    const int* seqY;  // adjrows ints, element 0 = header (unused)
    const int* seqX;  // adjcols ints, element 0 = header (unused)
    const int* subst; // substsz*substsz, row = Y letter
    int substsz;
    int g;  // gapoCost
    int R;  // adjrows-1
    int C;  // adjcols-1
    int Cp; // last column computed (sparse: tcols*tBx, full: C)
    int nTickets;
    int ns;  // strip waves per workgroup (super-strip = ns*kWaveRows rows)
    // FULL
    int* score;
    long long ld;  // = adjcols
    // SPARSE
    int* hrow;
    int* hcol;
    int trows, tcols, tBx, tBy;
    int* rows64;          // two-pass full fill, pass 1 (K-rows XR instance): rows 64m, shifted (nw_expand.h)
    long long rpitch;
    // inter-workgroup hand-off + control
    unsigned long long* gran;
    long long granStride;
    unsigned* ticket;
    unsigned* err;      // sticky: set by a spin that gave up, cleared by gsa_sync after reading
    unsigned long long spin;  // watchdog: s_memrealtime ticks (100 MHz) a wait may go without progress
    unsigned epoch;
    // mlsppt (K-rows kernel, one tile row per ticket): host-mapped word per ticket, set to
    // (epoch << 32 | n) once the headers of that tile row's first n column chunks (ptChunk tile
    // columns each) are in memory (system-scope stores, acknowledged); null: no signalling
    unsigned long long* done;
    int ptChunk;
    // K-rows fills (nw_krow.hip): 1 = launch the int8-profile instance, which declines a table with
    // some s - 2g outside int8 by setting *q8flag to its epoch, then the int16 instance with q8 = 2,
    // which runs only then; 0 = the int16 instance alone
    int q8;
    unsigned* q8flag;
    // kModeScoreAG: gap open / extend, the F' hand-off granules (same layout as gran), result H[R][C]
    int go, ge;
    unsigned long long* gran2;
    int* agResult;
    unsigned long long* swBest;  // kModeScoreSW: max of (score << idxBits | (2^idxBits-1 - row-major index))
    int idxBits;
    // batch: the per-pair fields above are loaded from pairs[] for every ticket
    const PairDesc* pairs;
    int nPairs;
    int nTicketsTotal;
    // batch schedule: {pair, ticket within the pair} of every global ticket, round-robin over the
    // pairs (null: pair-major by ticketBase).  Ticket j of a pair always follows its ticket j-1.
    const int* sched;
    // fused full fill (nw_full_fused_kernel): the expansion's descriptors (nPairs) and schedule
    // ({pair, task} per task, or null), its task count, the workgroups that take pass-1 tickets
    // first, the probe knob; claim counters (role, expansion task; zeroed per launch); one progress
    // word per pass-1 strip (epoch << 32 | tile columns published), pair p's at its ticketBase x ns
    const ExpandPair* xpair;
    const int* xsched;
    int xTasks;
    int xP;
    int xrun;  // expansion tasks per claim (a run of one tile column: gsa_capi.hip enqueue_full_twopass)
    int laneFeed, lanePair;  // nw_lane.hip: the feeder wave / paired stores, 0 or 1 (< 0: its own choice)
    unsigned* xrole;
    unsigned* xcounter;
    unsigned long long* xdone;
    // measurement aid (GSA_STAMPS=1, gsa_debug_stamps): s_memrealtime stamps of the fused fill,
    // [start, end] per pass-1 strip (global strip index; start = the ticket's start, before the
    // strip's first wait), then [claimed, ready, done] per expansion task; null otherwise
    unsigned long long* stamps;
    // score-only NW from both ends (gsa_capi.hip score_bidi): the strip with a lane whose last row is
    // tapRow stores that row's Hgo' (tapH) and, affine, F' (tapF), shifted as the hand-off holds
    // them, at tap[kTapPad + column] for every column the lane computes; tapRow <= 0: none.
    // bidiTop > 0: one launch runs both halves, pairs[0] (bidiTop tickets) and pairs[1] (the rest),
    // tickets alternating while both have some, then the longer half's; half 1 taps row tapRowB
    // into tapH / tapF + tapStride
    int* tapH;
    int* tapF;
    int tapRow;
    int tapRowB;
    int tapStride;
    int bidiTop;
    // score_bidi: bit h set -> half h's last ticket ends on its tap row, and that ticket's drain
    // writes its granules like any other ticket's (the combine reads the tap there: no lane tap)
    int tapGran;
    // score_bidi, local: a third pair (bidiMid > 0: pairs[1] has bidiMid tickets, pairs[2] the
    // rest) runs the bottom half forward from a fresh (zero) border, its end-cell keys offset by
    // pairs[2].rowOff rows; each pair's keys go to its PairDesc::swBest
    int bidiMid;
    int rowOff;  // per ticket: the pair's rowOff
    // score_bidi, local, the way back: a one-pair launch that starts at the pair's ticket tkFirst,
    // its row above in that ticket's predecessor's granules (copied there with this epoch)
    int tkFirst;
};
constexpr int kTapPad = 128;  // tap row buffers: columns -kTapPad .. C + 79

// Resource footprint of the last fill launched from this host thread: what the reference's
// updateNwAlgPeakMemUsage (nwalign_shared.cpp:5-25) multiplies out -- kernel attributes
// (hipFuncGetAttributes) and the workgroups resident at once (min(grid, occupancy x CUs)).
struct LaunchFoot
{
    long long lds_per_wg;       // static + dynamic LDS bytes per workgroup
    long long scratch_per_lane; // private (scratch) bytes per lane
    long long regs_per_lane;    // VGPRs per lane (numRegs)
    long long threads_per_wg;
    long long active_wgs;
};
extern thread_local LaunchFoot g_last_foot;
// fill g_last_foot for a launch of `kern` (dynamic LDS `lds`, `threads` per workgroup, `grid`)
hipError_t record_foot(const void* kern, size_t lds, int threads, int grid);

size_t strip_lds_bytes(int ns, int substsz, int mode);
// headers of every pair of the batch (grid.y = pair); maxWork = largest per-pair element count
hipError_t launch_headers(const StripArgs& a, int mode, long long maxWork, hipStream_t stream);
// grid <= 0: as many workgroups as can be co-resident (capped by the ticket count)
hipError_t launch_strip_fill(const StripArgs& a, int mode, int grid, hipStream_t stream);

}  // namespace gsa
