// nw_krowco.hip -- pass 1 of the pipelined full batch (nw_krow_kernel<2, 2, 512, 4>): the XR fill in
// 4-wave workgroups that run beside the previous pair group's expansion on the same CUs, in a
// translation unit of its own so the other instances' code generation stays as it is.
#define GSA_KROW_CO
#include "nw_krow.hip"
