// nw_trace_dev.h -- sparse traceback on the device (nw_trace_dev.hip); used by gsa_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gsa {

struct TraceArgs
{
    const int* seqY;
    const int* seqX;
    const int* subst;
    int substsz, g;
    long long adjrows, adjcols;
    int tBx, tBy, tcols;
    const int* hrow;
    const int* hcol;
    // starting tile and element (NwTrace2_GetTileAndElemIJ of (adjrows-1, adjcols-1))
    int iT0, jT0, iE0, jE0;
    unsigned char* edits;   // one byte per move, walk order ('=', 'X', 'I', 'D')
    long long cap;          // bytes available in edits
    long long* res;         // [0] moves, [1] align_cost
    unsigned* dirs_scratch; // move codes in global memory when the tile is too wide for LDS (else null)
    // precomputed tiles (trace_band): tmap[iT * tcols + jT] = slot or -1, codes of slot s at
    // tcodes + s * trace_dir_words(tBy, tBx); null: every tile is recomputed on entry
    const int* tmap;
    const unsigned* tcodes;
};

size_t trace_dir_words(int tBy, int tBx);
size_t trace_lds_bytes(int tBy, int tBx, int substsz, bool dirs_lds);
hipError_t launch_trace_sparse(const TraceArgs& a, hipStream_t st);
// move codes of the n tiles list[2s], list[2s+1] (whole tiles) into a.tcodes, slot s; many
// workgroups (the tiles are independent given their headers)
hipError_t launch_trace_band(const TraceArgs& a, const int* list, int n, int grid, hipStream_t st);

}  // namespace gsa
