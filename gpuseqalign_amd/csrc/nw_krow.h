// nw_krow.h -- launch interface of the K-rows-per-lane sparse (mlsp) fill (nw_krow.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "nw_strip.h"

namespace gsa {

constexpr int kKrowKDefault = 4;        // rows per lane
constexpr int kKrowNSDefault = 4;       // strip waves per workgroup, single pairs
constexpr int kKrowNSBatchDefault = 8;  // strip waves per workgroup, batches of pairs

// (ns, k) pairs the library instantiates: a ticket = ns * 64 * k rows, which divides the sparse
// tile height kSparseTileBy (1024) or, for (8, 4), spans two tile rows (the drain wave then also
// writes the header row between strips 3 and 4).
__host__ __device__ constexpr bool krow_ok(int ns, int k)
{
    return ((k == 2 || k == 4) && (ns == 2 || ns == 4)) || (k == 4 && ns == 8);
}
__host__ __device__ constexpr int krow_ticket_rows(int ns, int k) { return ns * 64 * k; }
// tickets of a pair with trows tile rows (the last ticket of a two-row geometry may cover one)
__host__ __device__ constexpr int krow_tickets(int trows, int ns, int k)
{
    return (trows * kSparseTileBy + krow_ticket_rows(ns, k) - 1) / krow_ticket_rows(ns, k);
}
// q8: the int8-profile instance's layout (nw_krow.hip)
size_t krow_lds_bytes(int ns, int lw, int substsz, bool q8 = false);
// StripArgs / PairDesc / granule contract as launch_strip_fill (sparse mode, a.tBx, a.tBy,
// per-pair hrow/hcol/trows/tcols/Cp); tickets of a pair = krow_tickets(trows, ns, k).
// Every |s - 2g| must fit int16 (the kernel sets error bit 2 otherwise).  grid <= 0: every resident slot.
// The profile ring holds 512 columns for ns = 2, 1024 otherwise (lw is reserved).
hipError_t launch_krow_fill(const StripArgs& a, int ns, int k, int lw, int grid, hipStream_t stream);
// Pass 1 of the two-pass full fill (nw_expand.h): the sparse fill (K = 4, ns = 4 or 8, a.tBx =
// kExpHB) that also stores rows 64m into each pair's rows64 / rpitch (PairDesc).
hipError_t launch_krow_fill_xr(const StripArgs& a, int ns, int grid, hipStream_t stream);
// Both passes of the two-pass full fill in one launch: the first a.xP workgroups take pass-1
// tickets (the XR fill on (ns, 4) tickets) until none is left, then, like the rest, expansion
// tasks of `waves` x 64 rows (a.xpair, a.xsched, a.xTasks), each task waiting for the progress
// words a.xdone of the strips whose rows and header column it reads.  (ns, waves): (4, 8) or
// (8, 12).  grid <= 0: every resident slot.
// staged: the strips hand row 64m to a storer wave (large pairs); else they store it themselves
hipError_t launch_full_fused(const StripArgs& a, int ns, int waves, bool staged, int grid, hipStream_t stream);

// Score-only NW / SW (modes kModeScoreAG/AGL/SW/SWL of nw_strip.h, same StripArgs contract as
// launch_strip_fill for one pair: go, ge, gran + gran2, agResult, swBest, idxBits) on the K-rows
// layout (nw_kscore.hip): 1024-row tickets, grid > 0 workgroups.  Every s - go - ge must lie in
// (-32768, 32767] (error bit 2 otherwise); SW needs go < 0 and ge <= 0.  a.q8 as launch_kr: the
// int8-profile instance (values in [-127, 127]) with the int16 one behind it.
size_t krow_score_lds_bytes(int substsz, bool q8 = false);
hipError_t launch_krow_score(const StripArgs& a, int mode, int k, int grid, hipStream_t stream);
// (the affine modes' instances, in nw_kscore_ag.hip; called by launch_krow_score)
hipError_t launch_krow_score_affine(const StripArgs& a, int mode, int k, int grid, hipStream_t stream);

}  // namespace gsa
