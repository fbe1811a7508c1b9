// nw_bidi.h -- score-only NW from both ends (gsa_capi.hip score_bidi): the pair's top half runs
// forward and its bottom half, reversed, runs forward at the same time on other CUs; each launch
// taps the row where the halves meet (StripArgs::tapRow), and one workgroup combines the two rows.
#pragma once
#include <hip/hip_runtime.h>

namespace gsa {

// dst[0] = 0, dst[i] = src[last + 1 - i] for i = 1 .. last - first + 1 (a header element, then
// src[first .. last] reversed)
hipError_t launch_reverse(const int* src, int first, int last, int* dst, hipStream_t stream);

// out[0] = max over j = 0 .. C of max(Ht(j) + Hb(C - j), Ft(j) + Fb(C - j) - (go - ge)) (affine), or
// of Ht(j) + Hb(C - j) (linear), where the tapped rows hold shifted values (Hgo' = H - (i+j) ge +
// (go - ge), F' = F - (i+j) ge) of row m (top, forward) and of row mb (bottom, reversed) at
// tap[kTapPad + j]; column 0 is the gap border go + (i-1) ge
hipError_t launch_bidi_combine(const int* topH, const int* topF, const int* botH, const int* botF, int m, int mb,
                               int C, int go, int ge, bool affine, int* out, hipStream_t stream);

}  // namespace gsa
