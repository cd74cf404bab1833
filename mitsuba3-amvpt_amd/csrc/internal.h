/*
 * internal.h -- host-side state shared by the C-ABI (amvpt_capi.cpp) and the
 * kernel launcher (amvpt_render.hip).  Not part of the public interface.
 */
#pragma once
#include <string>
#include <vector>

#include "../../include/amvpt.h"
#include "dscene.h"

struct amvpt_scene {
    amvpt::DScene dev;          /* device pointers */
    void *dev_scene_struct = nullptr; /* device copy of `dev` */
    std::vector<void *> allocations;
    uint32_t n_nodes = 0, n_prims = 0;
    uint32_t n_sph = 0;         /* spheres (<= 64: the wave-uniform walks defer their float64 tests) */
    uint32_t n_outer = 0;       /* rectangles kept out of the BVH (DScene::outer) */
    bool bvh_tri_only = false;  /* every BVH primitive is a triangle (the WALK_LANE_TRI suffix walks) */
    uint32_t n_boxes = 0;       /* box meshes the brute-force walks screen (DScene::boxes) */
    uint32_t n_nodes2 = 0;      /* two-box BVH nodes (DScene::nodes2; 0: the per-lane walks stay threaded) */
    uint32_t bvh2_depth = 0;    /* its depth in inner nodes (<= kStack2 when built) */
    float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};   /* the BVH root box (ray binning's grid) */
    bool has_spheres = false;   /* the brute-force suffix walks take their sphere-free instances otherwise */
    bool all_diffuse = false;   /* every BSDF is plain `diffuse`: kernels take their kDiff instances */
    int device = 0;
};

namespace amvpt {
void set_error(const std::string &msg);
amvpt_status hip_fail(const char *what, int err);
amvpt_status render_impl(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                         const amvpt_lane_set &lanes, const amvpt_film_window &film, void *stream,
                         const amvpt_render_opts &opts, amvpt_counters *counters, float *records,
                         uint32_t record_pass);
amvpt_status develop_impl(const float *film, float *out, uint32_t w, uint32_t h, uint32_t alpha, void *stream);
amvpt_status release_impl(int device);
amvpt_status accumulate_impl(float *quilt, uint32_t qw, uint32_t qh, uint32_t C, const float *win, uint32_t x0,
                             uint32_t y0, uint32_t w, uint32_t h, const uint32_t *ov, uint64_t n_ov, void *stream);
extern uint64_t g_chunk_lanes;
extern uint32_t g_traversal;
extern amvpt_exchange_fn g_exchange;
extern void *g_exchange_ctx;
} // namespace amvpt
