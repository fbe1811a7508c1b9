// nw_lane.h -- launch interface of the one-row-per-lane NW-LG full fill (nw_lane.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "nw_strip.h"

namespace gsa {

constexpr int kLaneRows = 64;       // rows per lane strip (one wave, one row per lane)
constexpr int kLaneNSDefault = 4;   // lane strips per workgroup (super-strip = 256 rows)

// Workgroup LDS bytes for ns lane strips and a substitution alphabet of substsz letters.
size_t lane_lds_bytes(int ns, int substsz);
// Full fill over the tickets of a.pairs (super-strips of ns*kLaneRows rows, pair-major), same
// StripArgs / PairDesc / granule contract as launch_strip_fill; grid <= 0: every resident slot.
hipError_t launch_lane_fill(const StripArgs& a, int ns, int grid, hipStream_t stream);

}  // namespace gsa
