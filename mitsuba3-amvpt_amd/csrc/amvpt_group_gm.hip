/*
 * amvpt_group_gm.hip -- explicit instances of the group-size launchers (launch_primary<G>,
 * launch_splat<G> and their kernels) for G in { -1 }
 * (G = -1: the runtime instance for 257..1024 views, 1024-bit view masks).  Split from
 * amvpt_render.hip so the instances compile in parallel; see "Group-size instances" there.
 */
#define AMVPT_GROUP_TU 1
#define AMVPT_GROUP_LIST(X) X(-1)
#include "amvpt_render.hip"
