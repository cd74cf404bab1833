/*
 * amvpt_group_g8.hip -- explicit instances of the group-size launchers (launch_primary<G>,
 * launch_splat<G> and their kernels) for G in { 8 }
 * (G = 0: the runtime instance for 17..256 views).  Split from amvpt_render.hip so the
 * instances compile in parallel; see "Group-size instances" there.
 */
#define AMVPT_GROUP_TU 1
#define AMVPT_GROUP_LIST(X) X(8)
#include "amvpt_render.hip"
