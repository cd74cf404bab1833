/*
 * amvpt_group_ga.hip -- explicit instances of the group-size launchers (launch_primary<G>,
 * launch_splat<G> and their kernels) for G in { 2 3 5 6 }
 * (G = 0: the runtime instance for 17..256 views).  Split from amvpt_render.hip so the
 * instances compile in parallel; see "Group-size instances" there.
 */
#define AMVPT_GROUP_TU 1
#define AMVPT_GROUP_LIST(X) X(2) X(3) X(5) X(6)
#include "amvpt_render.hip"
