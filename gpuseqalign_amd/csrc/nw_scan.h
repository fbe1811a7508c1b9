// nw_scan.h -- score-only NW / SW with linear or affine gaps (nw_scan.hip); used by gsa_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsa {

struct ScoreArgs
{
    const int* seqY;
    const int* seqX;
    const int* subst;
    int substsz;
    int go, ge;
    long long R, C;          // adjrows-1, adjcols-1 (both >= 1)
    int nTR;                 // 64-row tile rows
    int* bh;                 // boundary rows: (nTR+1) x (C+1), H of matrix row 64*b (row R for b = nTR)
    int* bf;                 // ... and F
    int* prog;               // (nTR+1) progress words: boundary row b valid for columns < prog[b]
    unsigned* ticket;
    unsigned* err;
    unsigned long long spin;   // watchdog ticks (100 MHz) without progress
    unsigned long long* best;  // local: max of (score << idxBits | (2^idxBits-1 - row-major index))
    int idxBits;               // local: bits of the row-major index, ceil(log2((R+1)(C+1)))
    int* result;             // global: H[R][C]
};

hipError_t launch_score_scan(const ScoreArgs& a, int local, int cu_count, hipStream_t st);

}  // namespace gsa
