// rs_kernels_tb.hip -- the table-of-bases forms of the coding kernels (rs_kernels.hip TB: a
// coalesced group of blocks that each lie in their caller's own page-locked buffer, coded by one
// launch), in a translation unit of their own so the build compiles them beside rs_kernels.hip.
#define RSMI_TB_UNIT 1
#include "rs_kernels.hip"
