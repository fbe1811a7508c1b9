// nw_krowx.hip -- the K-rows fill's XR instances (nw_krow_kernel<NS, 4, 1024, 2>): pass 1 of the
// two-pass full fill (nw_expand.hip), in a translation unit of its own so the sparse instances'
// code generation stays as it is.
#define GSA_KROW_XR
#include "nw_krow.hip"
