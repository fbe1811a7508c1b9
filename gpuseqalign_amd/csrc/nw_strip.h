// nw_strip.h -- launch interface of the strip-wavefront NW-LG fill (nw_strip.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gsa {

constexpr int kModeFull = 0;
constexpr int kModeSparse = 1;
constexpr int kWaveRows = 256;                          // rows per strip (one wave, 4 rows per lane)
constexpr int kSparseNS = 4;                            // strip waves per workgroup, sparse fills
constexpr int kSparseTileBy = kWaveRows * kSparseNS;    // = tile height of the mlsp matrices
constexpr int kFullNSDefault = 1;                       // strip waves per workgroup, full fills

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
    // inter-workgroup hand-off + control
    unsigned long long* gran;
    long long granStride;
    unsigned* ticket;
    unsigned* err;
    unsigned epoch;
    unsigned long long* dbg;  // diagnostic builds only (GSA_STAMP): per-wave block time stamps
};

size_t strip_lds_bytes(int ns, int substsz);
hipError_t launch_headers(const StripArgs& a, int mode, hipStream_t stream);
hipError_t launch_strip_fill(const StripArgs& a, int mode, int grid, hipStream_t stream);

}  // namespace gsa
