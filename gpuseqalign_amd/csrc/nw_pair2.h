// nw_pair2.h -- launch interface of the two-rows-per-lane sparse (mlsp) fill (nw_pair2.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "nw_strip.h"

namespace gsa {

constexpr int kPair2Rows = 128;   // rows per strip wave (two per lane)
constexpr int kPair2NSDefault = 4;

// Strip waves per workgroup the library instantiates (a ticket = ns * kPair2Rows rows; it
// must divide the sparse tile height kSparseTileBy).
__host__ __device__ constexpr bool pair2_ns_ok(int ns) { return ns == 2 || ns == 4; }
size_t pair2_lds_bytes(int ns, int substsz);
// StripArgs / PairDesc / granule contract as launch_strip_fill (sparse mode, a.tBx, a.tBy,
// per-pair hrow/hcol/trows/tcols/Cp); tickets of a pair = trows * (tBy / (ns * kPair2Rows)).
// grid <= 0: every resident slot.
hipError_t launch_pair2_fill(const StripArgs& a, int ns, int grid, hipStream_t stream);

}  // namespace gsa
