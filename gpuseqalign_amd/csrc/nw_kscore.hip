// nw_kscore.hip -- score-only NW / SW with linear or affine gaps on the K-rows layout
// (nw_kscore_kernel in nw_krow.hip), in a translation unit of its own: the headline sparse fill's
// code generation stays as it is, and the Makefile can give this one its own scheduler flags.
#define GSA_KROW_SCORE
#include "nw_krow.hip"
