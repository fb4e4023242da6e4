// rt_kernels_bvh.hip — the BVH instantiations of the render kernels
// (rt_launch_render_bvh), compiled at -O3 in their own translation unit;
// everything else in rt_kernels.hip is compiled once, at -O1 (see Makefile).
#define RT_TU_BVH
#include "rt_kernels.hip"
