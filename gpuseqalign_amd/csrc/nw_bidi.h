// nw_bidi.h -- score-only NW from both ends (gsa_capi.hip score_bidi): the pair's top half runs
// forward and its bottom half, reversed, runs forward in the same launch on other CUs (tickets
// interleaved, StripArgs::bidiTop); each half taps the row where the halves meet
// (StripArgs::tapRow / tapRowB), and a combine kernel takes the best crossing.
#pragma once
#include <hip/hip_runtime.h>

#include "nw_strip.h"

namespace gsa {

// One launch before the fill: desc[0..1] = d0, d1; ry[0] = rx[0] = 0, ry[i] = seqY[R + 1 - i]
// (i = 1 .. R - m: rows m+1 .. R reversed), rx[j] = seqX[C + 1 - j]; the launch's ticket word, its
// 8 result / error words and the combine's output (-2^31) reset; substT non-null: substT[x][y] =
// subst[y][x] (substsz x substsz; the pair transposed, when R is odd and C even); d2 non-null (local
// modes): desc[2] = *d2, the bottom half forward from a fresh border.
hipError_t launch_bidi_prep(const PairDesc& d0, const PairDesc& d1, PairDesc* desc, const int* seqY, int m, int R,
                            const int* seqX, int C, int* ry, int* rx, unsigned* ticket,
                            unsigned long long* words, int* out, const int* subst, int substsz, int* substT,
                            hipStream_t stream, const PairDesc* d2 = nullptr);

// out[0] = max over j = 0 .. C of max(Ht(j) + Hb(C - j), Ft(j) + Fb(C - j) - (go - ge)) (affine), or
// of Ht(j) + Hb(C - j) (linear), where the tapped rows hold shifted values (Hgo' = H - (i+j) ge +
// (go - ge), F' = F - (i+j) ge) of row m (top, forward) and of row mb (bottom, reversed), column j
// at topH[ts j] (a lane tap: tap + kTapPad, ts = 1; the last ticket's granules: the low word of each
// 64-bit granule, ts = 2), likewise bottom; column 0 is the gap border go + (i-1) ge (local: H = 0,
// F = -inf; the sum is then the best local alignment through the lattice point (m, j), which
// includes those that end or start there).  Many workgroups, each folding its columns into out[0]
// with an atomic max (out[0] starts at -2^31, launch_bidi_prep).
// The way back of a local pair (score_bidi): dst[c] = epoch << 32 | low word of src[c], c < n, and
// likewise dst2 from src2 when non-null (the top half's last-ticket granules, restamped for the
// continuation launch, which reads them as its first ticket's row above).
hipError_t launch_bidi_seed(const unsigned long long* src, const unsigned long long* src2, unsigned long long* dst,
                            unsigned long long* dst2, long long n, unsigned epoch, hipStream_t stream);

hipError_t launch_bidi_combine(const int* topH, const int* topF, int ts, const int* botH, const int* botF, int bs,
                               int m, int mb, int C, int go, int ge, bool affine, int* out, hipStream_t stream,
                               bool local = false);

}  // namespace gsa
