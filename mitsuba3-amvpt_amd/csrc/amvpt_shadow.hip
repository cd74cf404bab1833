/*
 * amvpt_shadow.hip -- the k_shadow kernels (NEE ray tests) and their launcher, compiled
 * with the SLP vectorizer on; everything else in amvpt_render.hip is built without it.
 * See launch_shadow in amvpt_render.hip.
 */
#define AMVPT_SHADOW_TU 1
#include "amvpt_render.hip"
