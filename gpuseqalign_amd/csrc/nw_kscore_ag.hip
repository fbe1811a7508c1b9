// nw_kscore_ag.hip -- the affine-gap score modes (NW-AG, SW-AG) of nw_kscore_kernel, in a
// translation unit of their own so that the Makefile builds them with the iterative ILP scheduler
// (the linear modes in nw_kscore.hip are faster under the default one).
#define GSA_KROW_SCORE
#define GSA_KSCORE_AFFINE
#include "nw_krow.hip"
