// nw_krow8.hip -- the K-rows fill's 8-strip batch instance (nw_krow_kernel<8, 4, 1024>), compiled
// in a translation unit of its own so the Makefile can give it its own scheduler flags: the
// iterative ILP scheduler that helps the single-pair instances costs this one ~1 %
// (profiles/r03_sched_flags_ab.txt).
#define GSA_KROW_BATCH8
#include "nw_krow.hip"
