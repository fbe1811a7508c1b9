// nw_check.h -- device-side verification of fill outputs (nw_check.hip); used by gsa_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsa {

struct CheckArgs
{
    const int* seqY;
    const int* seqX;
    const int* subst;
    int substsz, g;
    long long adjrows, adjcols;
    // sparse geometry (check_sparse) / score matrix (check_full)
    int tBx, tBy, trows, tcols;
    long long hrowElems;
    const int* hrow;
    const int* hcol;
    const int* score;
    long long ld;  // check_full: row pitch of score in ints (>= adjcols)
    // [0] values compared, [1] mismatches, [2] smallest mismatching index (~0 if none)
    unsigned long long* res;
};

hipError_t launch_check_sparse(const CheckArgs& a, int cu_count, hipStream_t st);
hipError_t launch_check_full(const CheckArgs& a, hipStream_t st);

}  // namespace gsa
