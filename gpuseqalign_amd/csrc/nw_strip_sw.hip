// nw_strip_sw.hip -- the strip kernel's SW score instance (nw_strip_kernel<4, kModeScoreSW>),
// compiled in a translation unit of its own so the Makefile can give it its own scheduler flags:
// the iterative ILP scheduler that helps the AG and linear-gap instances costs this one ~1 %
// (profiles/r03_sched_flags_ab.txt).
#define GSA_STRIP_SW
#include "nw_strip.hip"
