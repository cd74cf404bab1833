/*
 * amvpt_render.hip -- the MI355X wavefront pipeline of the `mvpath` integrator.
 *
 * One frame = n_passes passes (mvpath.cpp:36-41,222-246); one pass = L lanes
 * (lane -> pixel = lane >> log2(spp_per_pass), mvpath.cpp:173-190), processed
 * in chunks of at most g_chunk_lanes lanes (automatic: up to 2^26).  Per chunk:
 *
 *   k_mv_primary<G>  render_multisample + sample_multi up to the suffix
 *                    (jitter, sample_ray_idx, primary hit, emitter sample +
 *                    shadow ray, camera_selection with G-1 visibility rays,
 *                    mis_weights, direct light, mixture pdf)   mvpath_multi.h:8-322
 *                    -> view records (SoA) + compacted suffix queue
 *   k_raygen_single  render_sample: jitter + sample_ray -> queue (G = 1 / `path`)
 *   k_bounce (xN)    one iteration of the shared-suffix / sample_single loop per
 *                    live path; ballot + mbcnt compaction into the next queue
 *                    mvpath_multi.h:563-686, mvpath_single.h:130-275
 *   k_splat_*        indirect accumulation + ImageBlock::put into the film
 *                    (float atomics)          mvpath_multi.h:343-368,61-76; imageblock.cpp:174-559
 *
 * All queues and records are SoA float4 streams in HBM (16 B per lane per
 * stream: one dwordx4 load/store per lane, 1 KiB per wave instruction).
 */
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <type_traits>

#include "internal.h"   /* the C-ABI enums (amvpt.h) before the device headers use them */
#include "dbsdf.h"

/* non-template kernels get internal linkage in the k_shadow translation unit (amvpt_shadow.hip) */
#if defined(AMVPT_SHADOW_TU) || defined(AMVPT_GROUP_TU)
#define AMVPT_TU_LOCAL static
#else
#define AMVPT_TU_LOCAL
#endif

namespace amvpt {

#if !defined(AMVPT_SHADOW_TU) && !defined(AMVPT_GROUP_TU)
/* 0 = automatic: 2^26 lanes, halved while the chunk's arena would exceed 48 GB (of the 288 GB of HBM; config M:
 * 26 GB at 2^26, 1598/1605 -> 1614/1621 Msamples/s against 2^25 chunks, r03zg: fewer fused-suffix tails).
 * Earlier sweep at 24 GB:
 * Fewer, larger chunks mean fewer tails of the fused suffix and fewer kernel boundaries
 * (config M: 2^22 386, 2^23 373, 2^24 364, 2^25 363 ms per frame; r02fd) */
uint64_t g_chunk_lanes = 0;
uint32_t g_traversal = 0;
amvpt_exchange_fn g_exchange = nullptr;
void *g_exchange_ctx = nullptr;
#endif

/* ------------------------------------------------------------------ */
/* Parameters                                                         */
/* ------------------------------------------------------------------ */

/* Walk of the suffix kernels (k_extend, k_shadow), a compile-time choice per scene:
 * per-lane threaded BVH, wave-uniform BVH, or brute force over every primitive
 * (tiny scenes; measured on the Cornell box: k_extend 114 -> 100 ms, k_shadow 103 -> 81 ms
 * per config-M frame; brute force in the coherent primary / visibility walks was slower:
 * k_vis 90 -> 248 ms, k_prim_hit 12 -> 30 ms). */
/* WALK_LANE_NS: the per-lane walk of a scene without spheres (no float64 sphere code in the suffix walks:
 * the sphere branch cost the mesh k_shadow 191 -> 207 ms once the sphere screen grew it, r04g) */
/* WALK_LANE_TRI: the per-lane walk of a BVH of triangles only (no type dispatch in the leaf tests: the mesh scenes,
 * whose rectangles stay out of the BVH, DScene::outer) */
enum : int { WALK_LANE = 0, WALK_UNI = 1, WALK_BRUTE = 2, WALK_BRUTE_NS = 3 /* no spheres */, WALK_LANE_NS = 4, WALK_LANE_TRI = 5 };
#ifndef AMVPT_LANE_TRI
#define AMVPT_LANE_TRI 1   /* triangle-only BVHs take the WALK_LANE_TRI suffix walks (0: WALK_LANE_NS, A/B) */
#endif
/* the per-lane walks' primitive set (dgeom.h trace_closest / trace_any kSph): -1 triangles, 0 no spheres, 1 any */
template <int kWalk> constexpr int walk_sph() { return kWalk == WALK_LANE_TRI ? -1 : kWalk != WALK_LANE_NS ? 1 : 0; }
#ifndef AMVPT_LANE_NS
#define AMVPT_LANE_NS 1   /* sphere-free scenes take the WALK_LANE_NS suffix walks (0: WALK_LANE, A/B) */
#endif
/* the per-lane walks take the two-box BVH when the kernel gave the thread a stack (sc.stk: k_extend / k_shadow with
 * KParams::bvh2), else the threaded one */
template <int kWalk> AD Hit walk_closest(const SceneRef &sc, const Ray &r) {
    if (kWalk == WALK_BRUTE || kWalk == WALK_BRUTE_NS) return brute_closest<kWalk == WALK_BRUTE>(sc, r);
    if (kWalk != WALK_UNI && sc.stk) {
        Hit best{kInf, 0.f, 0.f, -1};
        uint32_t best_orig = 0xffffffffu;
        outer_closest(sc, r, best, best_orig);
        return trace_closest2<walk_sph<kWalk>()>(sc, r, best, best_orig);
    }
    return trace_closest<kWalk == WALK_UNI, AMVPT_WALK_WW, walk_sph<kWalk>()>(sc, r);
}
template <int kWalk> AD bool walk_any(const SceneRef &sc, const Ray &r) {
    if (kWalk == WALK_BRUTE || kWalk == WALK_BRUTE_NS) return brute_any<kWalk == WALK_BRUTE>(sc, r);
    if (kWalk != WALK_UNI && sc.stk) return trace_any2<walk_sph<kWalk>()>(sc, r, outer_any(sc, r, false));
    return trace_any<kWalk == WALK_UNI, AMVPT_WALK_WW, walk_sph<kWalk>()>(sc, r);
}

struct KParams {
    uint32_t W, H, C;
    /* the per-lane suffix walks on the two-box BVH (DScene::nodes2): their LDS stack's byte offset in the dynamic
     * LDS of k_extend / k_shadow (0 / 0 with bvh2 = 0: the threaded walks) */
    uint32_t bvh2, stk_off_ext, stk_off_any;
    uint32_t spp_pp, log_spp, pow2;
    uint32_t max_depth, rr_depth;
    uint32_t sa_mis, fast_mis, debug, n_adapt;
    uint32_t G;
    uint32_t multisensor, batch, n_views, gx, gy, rev_x, rev_y, sres_x, sres_y;
    uint32_t needs_ap;      /* Sensor::needs_aperture_sample: thin-lens views draw a 2-D aperture sample */
    uint32_t box, coalesce_single, path_box_pos, is_mvpath;
    uint32_t seed_value;
    uint32_t trav_mode;     /* amvpt_set_traversal */
    uint32_t sph;           /* spheres in the coherent walks: 0 none (sphere-free instances), 1 tested in place, 2 deferred (dgeom.h) */
    uint32_t win_rs;        /* splat window row stride residue mod 32 (0: stride = width) */
    uint32_t adapt_seed;    /* adaptive pass: seed of the forked sampler (base_seed + wavefront) */
    uint32_t pass_seed;     /* adaptive pass: seed_value of the pass whose lanes are refilled */
    uint64_t range_begin;   /* contiguous lane set: its first lane (lane_of) */
    /* lane set (amvpt_lane_set): chunk offsets are VIRTUAL indices v in [0, span) of the render's
     * lanes; lane_of(v) maps them to global lanes (contiguous, or rect_h runs of run_len lanes) */
    uint32_t rect, rect_x0, rect_y0, run_len;
    /* film window (amvpt_film_window): the film holds quilt pixels [fx0, fx0 + fw) x [fy0, fy0 + fh);
     * cells outside go to the overflow list (header u64 count, then 16-B entries, ov_cap of them) */
    uint32_t fx0, fy0, fw, fh;
    uint32_t *overflow;
    uint64_t ov_cap;
    float inv_w, inv_h;
    /* hdrfilm crop window: pixel offset of the ImageBlock in the film (lane pixels and sample
     * positions are film coordinates), the sample_ray_idx offsets -offset / crop_size
     * (mvpath_multi.h:12-16), and ImageBlock::put's non-coalesced shift (int) -offset - .5f */
    uint32_t off_x, off_y;
    float adj_ox, adj_oy, nc_ox, nc_oy;
    float adapt_w;
    FilterCoeffs filt;
    uint64_t chunk_begin;
    uint32_t chunk_n;
    uint32_t record;      /* write per-lane splat records */
    uint32_t row_splat;   /* row-reduced splat (row_put): lanes in pixel-major order, see slot_lane */
    uint32_t tile_w;      /* != 0: row-splat slots run over 4 x 4 pixel tiles of a tile_w-pixel-wide quilt */
    /* host-computed reciprocals of the kernel-uniform divisors the path-fetch code divides by (udiv_r; 0 when the
     * divisor is 0): tile_w / 4, run_len, n_adapt */
    double rcp_tpr, rcp_run_len, rcp_n_adapt;
    uint32_t adapt_pass;  /* the suffix runs paths of the adaptive wavefront (path_seq) */
    uint32_t valid_ray0;  /* !hide_emitters && environment: escaped camera rays count as valid
                           * (mvpath_multi.h:140, mvpath_single.h:98, path.cpp:114) */
    uint32_t vs_stride;   /* Bufs::vstate: floats between a field's consecutive view slots (the chunk) */
    unsigned long long *film_fx;   /* deterministic mode: 32.32 fixed-point shadow of the film (else null) */
    float *film_base;              /* the film the shadow mirrors (film_fx index = film float index) */
    unsigned long long *fx_drops;  /* deterministic mode: sharded count of finite cell adds out of the 32.32 range */
    /* stock `path` over several passes (integrator.cpp:279-330): the sampler is seeded once and every
     * pass continues each lane's PCG32 stream -- rng_in (passes > 0) holds the state each lane starts the
     * pass with, rng_out (all but the last pass) receives the state its path ends with; both indexed by
     * the lane's virtual index in the render's lane set */
    unsigned long long *rng_in, *rng_out;
    uint32_t box_screen;  /* the brute-force suffix walks screen box meshes (box_walk); 0: AMVPT_OPT_NO_BOX_SCREEN */
    float bin_lo[3], bin_scale[3];   /* ray binning: the scene box's low corner and cells per unit (bin_key) */
};

/* the PCG32 a stock-path lane starts the pass with: TEA-seeded, or the previous pass's state (same
 * stream increment) */
AD Pcg pass_rng(const KParams &P, uint32_t lane, uint64_t v) {
    uint32_t v0, v1;
    tea4(P.seed_value, lane, v0, v1);
    Pcg rng;
    if (P.rng_in) {
        rng.state = P.rng_in[v];
        rng.inc = (((uint64_t) v1) << 1) | 1u;
    } else {
        rng.seed(v0, v1);
    }
    return rng;
}

/* SoA streams of one chunk */
constexpr int kQPlanes = 5;   /* float4 planes of a path state (80 B, see store_state) */
struct Bufs {
    float4 *q_in[kQPlanes];
    float4 *q_out[kQPlanes];
    uint32_t *cnt_in, *cnt_out;  /* kQParts partition counters each, kCntStride words apart */
    uint32_t qcap;               /* entries per queue partition */
    float4 *lane_out;     /* (indirect / result rgb, valid_ray) */
    float4 *lrec[4];      /* k_mv_primary -> splat, per lane: (R0, pdfW), (Dp, lane flags), (Bv, valid mask),
                           * (hit point, indirect mask); R0 = slot 0's result, Dp / Bv = all-diffuse views'
                           * direct light / BSDF value (see k_mv_primary) */
    float4 *vrec;         /* per view [G][n]: all-diffuse scenes one float (weight); otherwise two float4
                           * planes [G][n] (result, weight) and [G][n] (bsdf value, view flags) */
    float *film;
    float *records;       /* optional [n][G][8] */
    unsigned long long *stats; /* [0] vertices [1] reuse lanes [2] visibility rays [3] splats */
    uint8_t *amask;       /* adaptive: per-lane adapt_mask of the pass (virtual index order), or null */
    const uint32_t *asel; /* adaptive: virtual indices of the lanes with adapt_mask (ascending) */
    const uint32_t *run_delta; /* adaptive: per run, (flagged lanes of the pass below the run) - (this
                                * render's flagged lanes below it): entry e of asel is entry
                                * e + run_delta[run] of the pass's compressed array */
    float4 *hit;          /* k_extend / k_prim_hit -> shading: closest hit (t, u, v, prim) per entry */
    float4 *nee[2];       /* k_bounce -> k_shadow: deferred emitter-sample shadow rays (NEE records), */
    float2 *nee_gb;       /* + the visible result's green and blue channels (40 B per record) */
    uint32_t *cnt_nee;
    float4 *vreq[3];      /* k_prim_req -> k_vis: (p, bits), (n, ap.x), (emitter point, ap.y) per lane */
    unsigned long long *occ; /* k_vis -> k_mv_primary: occlusion ballots, word (i >> 6) * G + slot */
    uint4 *vreq_w[8];     /* groups > 16 views (G <= 0 instances): the lane's visibility-request mask (mstore) */
    uint4 *lmask_w[24];   /* groups > 16 views: valid, indirect, wi.z > 0 masks per slot (mask_planes<G>() each) */
    float *vstate;        /* runtime groups whose per-view state exceeds LDS: VS_FIELDS x G x vs_stride floats */
    float4 *sray[2];      /* ray binning (k_bin_sort): a partition's rays in bin order, 32-B records [2 j], [2 j + 1]:
                           * extension rays (o, d.x), (d.yz, entry, -); NEE rays (AMVPT_NEE_CARRY) (o, dest),
                           * (target, result r) with sgb[j] = result g, b; sray[1] unused */
    float2 *sgb;          /* ray binning of NEE rays: the visible result's green and blue channels in bin order */
    uint16_t *key_out, *key_in, *key_nee;   /* ray binning: bin keys of the pushed paths / NEE records (null: off) */
};

/* ------------------------------------------------------------------ */
/* Scene staging                                                      */
/* ------------------------------------------------------------------ */

constexpr int kPrimBlock = 128;
enum { F_PDF, F_JP, F_PDFM, F_WX, F_WY, F_WZ, VS_FIELDS };   /* k_mv_primary's per-view LDS state */
constexpr int kVsFieldsDiff = 2;   /* all-diffuse scenes keep only F_PDF and F_JP in LDS */

/* Small BVHs are walked wave-uniformly from global memory (scalar loads) and not
 * staged; mid-size ones are staged in LDS; large ones stay in global memory. */
/* traversal mode (amvpt_set_traversal): 0 auto, 1 wave-uniform, 2 per-lane */
__host__ __device__ inline bool scene_uniform(uint32_t n_nodes, uint32_t mode) {
    return mode == 1u || (mode == 0u && n_nodes <= kUniformNodeLimit);
}
__host__ __device__ inline bool scene_staged(uint32_t n_nodes, uint32_t lds_bytes, uint32_t mode) {
    return !scene_uniform(n_nodes, mode) && lds_bytes <= kLdsSceneBytes;
}
__host__ __device__ inline uint32_t scene_lds_bytes(const DScene &S, uint32_t mode) {
    return scene_staged(S.n_nodes, S.lds_bytes, mode) ? (S.lds_bytes + 15u) & ~15u : 0u;
}
/* the LDS treelet of the first node ordering (any-hit walks of BVHs read from global memory) */
__host__ __device__ inline uint32_t tree_lds_bytes(const DScene &S, uint32_t mode) {
    return (S.t_stride && !scene_staged(S.n_nodes, S.lds_bytes, mode) && !scene_uniform(S.n_nodes, mode))
               ? S.t_stride * (uint32_t) sizeof(DNode) : 0u;
}
/* the 8 octant treelets (per-lane closest-hit walks) */
__host__ __device__ inline uint32_t oct_tree_lds_bytes(const DScene &S, uint32_t mode) {
    return (S.o_stride && S.oct_stride && !scene_staged(S.n_nodes, S.lds_bytes, mode) && !scene_uniform(S.n_nodes, mode))
               ? 8u * S.o_stride * (uint32_t) sizeof(DNode) : 0u;
}

__host__ __device__ inline uint32_t views_lds_bytes(uint32_t n_views) {
    const uint32_t b = n_views * (uint32_t) sizeof(DView);
    return b <= kViewTabBytes ? tab_round(b) : 0u;
}
/* tables (+ views) go to LDS when both fit */
__host__ __device__ inline bool tables_staged(const DScene &S, uint32_t n_views) {
    return S.tab_bytes != 0 && (n_views == 0 || views_lds_bytes(n_views) != 0);
}
/* dynamic LDS in front of a kernel's own region: [BVH][tables][views] */
__host__ __device__ inline uint32_t staged_lds_bytes(const DScene &S, uint32_t mode, uint32_t n_views) {
    return scene_lds_bytes(S, mode) + (tables_staged(S, n_views) ? S.tab_bytes + views_lds_bytes(n_views) : 0u);
}

template <typename T> AD T *copy_to_lds(const T *src, uint32_t bytes, char *&dst) {
    static_assert(sizeof(T) % 4 == 0, "word-sized records");
    uint32_t *d = (uint32_t *) dst;
    const uint32_t *sp = (const uint32_t *) src;
    for (uint32_t i = threadIdx.x; i < bytes / 4u; i += blockDim.x) d[i] = sp[i];
    T *r = (T *) dst;
    dst += tab_round(bytes);
    return r;
}

/*
 * Per-block staging (one __syncthreads): the BVH when it is walked per lane and
 * fits (<= kLdsSceneBytes), the shape/BSDF/emitter tables when they fit
 * (S.tab_bytes, <= kTabBytes) and the view table (<= kViewTabBytes): their
 * lane-divergent reads then hit LDS instead of L1/L2.  S is the kernel's local
 * copy of the scene header; its table pointers are redirected.
 */
template <bool kTab, bool kBvh = true, bool kTree = false, bool kOct = false>
AD SceneRef stage_scene(DScene &S, char *lds, uint32_t mode, const DView **V = nullptr, uint32_t n_views = 0,
                        bool boxes = false, bool stage_boxes = false) {
    SceneRef sc;
    sc.g = &S;
    /* the brute-force walks' box screening (box_walk) where the kernel asks for it */
    sc.boxes = S.boxes;
    sc.box_prims = S.box_prims;
    sc.box_lds = false;
    sc.loose_prims = S.loose_prims;
    /* off (AMVPT_OPT_NO_BOX_SCREEN, or a kernel without brute-force walks): the plain scan of prims[] */
    sc.n_boxes = boxes ? S.n_boxes : 0u;
    sc.n_loose = boxes ? S.n_loose : 0u;
    sc.n_loose_rect = S.n_loose_rect;
    sc.n_loose_tri = S.n_loose_tri;
    sc.outer = S.outer;   /* every BVH walk tests these (dgeom.h outer_closest / outer_any) */
    sc.n_outer = S.n_outer;
    sc.tnodes = nullptr;
    sc.t_n = 0;
    sc.onodes = nullptr;
    sc.o_n = 0;
    sc.lds_bvh = false;
    sc.nodes2 = S.n_nodes2 ? S.nodes2 : nullptr;
    sc.stk = nullptr;   /* the two-box walks' stack: set by the kernels that run them (k_extend / k_shadow) */
    sc.n_nodes = S.n_nodes;
    sc.gnodes = S.nodes;
    sc.gprims = S.prims;
    sc.uniform = scene_uniform(S.n_nodes, mode);
    sc.oct_stride = sc.uniform ? 0u : S.oct_stride;
    sc.nodes = S.nodes;
    sc.prims = S.prims;
    char *dst = lds;
    bool sync = false;
    if (kBvh && scene_staged(S.n_nodes, S.lds_bytes, mode)) {
        const uint32_t nn = S.n_nodes * (uint32_t) sizeof(DNode) / 16, np = S.n_prims * (uint32_t) sizeof(DPrim) / 16;
        float4 *d4 = (float4 *) lds;
        const float4 *sn = (const float4 *) S.nodes, *spr = (const float4 *) S.prims;
        for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) d4[i] = sn[i];
        for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) d4[nn + i] = spr[i];
        sc.nodes = (const DNode *) lds;
        sc.lds_bvh = true;
        sc.oct_stride = 0;   /* only the first ordering is staged */
        sc.prims = (const DPrim *) (lds + (size_t) nn * 16);
        dst = lds + scene_lds_bytes(S, mode);
        sync = true;
    } else if (kTree && tree_lds_bytes(S, mode)) {
        /* the treelet of the first node ordering (any-hit walks: trace_any_tl / trace_any_uni_tl) */
        const uint32_t n4 = S.t_stride * (uint32_t) sizeof(DNode) / 16;
        float4 *d4 = (float4 *) lds;
        const float4 *st = (const float4 *) S.tnodes;
        for (uint32_t i = threadIdx.x; i < n4; i += blockDim.x) d4[i] = st[i];
        sc.tnodes = (const DNode *) lds;
        sc.t_n = S.t_stride;
        dst = lds + tree_lds_bytes(S, mode);
        sync = true;
    } else if (kOct && oct_tree_lds_bytes(S, mode)) {
        /* the 8 octant treelets (closest-hit walks: trace_closest_tl) */
        const uint32_t n4 = 8u * S.o_stride * (uint32_t) sizeof(DNode) / 16;
        float4 *d4 = (float4 *) lds;
        const float4 *st = (const float4 *) S.onodes;
        for (uint32_t i = threadIdx.x; i < n4; i += blockDim.x) d4[i] = st[i];
        sc.onodes = (const DNode *) lds;
        sc.o_n = S.o_stride;
        dst = lds + oct_tree_lds_bytes(S, mode);
        sync = true;
    }
    /* compile-time choice (the host launches the kTab variant only when the tables fit),
     * so the table pointers are known to be LDS and reads become ds_read, not flat */
    if (kTab) {
        S.shapes = copy_to_lds(S.shapes, S.n_shapes * (uint32_t) sizeof(DShape), dst);
        S.bsdfs = copy_to_lds(S.bsdfs, S.n_bsdfs * (uint32_t) sizeof(DBsdf), dst);
        S.emitters = copy_to_lds(S.emitters, S.n_emitters * (uint32_t) sizeof(DEmitter), dst);
        if (V) *V = copy_to_lds(*V, n_views * (uint32_t) sizeof(DView), dst);
        sync = true;
    }
    /* the box triangles for box_walk's per-lane loads (the caller's dynamic LDS holds box_lds_bytes more) */
    if (stage_boxes && sc.n_boxes) {
        sc.box_prims = copy_to_lds(S.box_prims, sc.n_boxes * 12u * (uint32_t) sizeof(DPrim), dst);
        sc.box_lds = true;
        sync = true;
    }
    if (sync) __syncthreads();
    return sc;
}

AD Hit hit_of(float4 h) { return Hit{h.x, h.y, h.z, (int32_t) fbits(h.w)}; }
AD float4 hit_rec(const Hit &h) { return make_float4(h.t, h.u, h.v, bitsf((uint32_t) h.prim)); }

/* ------------------------------------------------------------------ */
/* Emitters at scene level                                            */
/* ------------------------------------------------------------------ */

/* SurfaceInteraction::emitter: the shape's area emitter, or the scene's environment (constant)
 * emitter for a ray that left the scene */
AD int32_t si_emitter(const SceneRef &sc, const SI &si) {
    return si.valid() ? sc.g->shapes[si.shape].emitter : sc.g->environment;
}

/* AreaLight::eval (area.cpp:82-88: front side only), ConstantBackgroundEmitter::eval
 * (constant.cpp:90-94) */
AD C3 emitter_eval(const SceneRef &sc, int32_t e, const SI &si, bool active) {
    if (e < 0 || !active) return c3(0.f);
    const DEmitter &em = sc.g->emitters[e];
    if (em.type != AMVPT_EMITTER_CONSTANT && !(si.wi.z > 0.f)) return c3(0.f);
    return c3(em.radiance);
}

/* Scene::pdf_emitter (scene.cpp:245-250) */
AD float emitter_pick_pmf(const DScene &S, uint32_t i) {
    return S.distr ? S.emitters[i].weight * S.distr_norm : S.emitter_pmf;
}

/* Scene::sample_emitter (scene.cpp:222-244); non-uniform weights: DiscreteDistribution::
 * sample_reuse_pmf (distr_1d.h:201-215) with the JIT predicate of sample() (:116-134) and
 * dr::binary_search over [0, n - 1] (floor(log2(n - 1)) + 1 halvings) */
AD uint32_t sample_emitter(const DScene &S, float &u, float &weight) {
    const uint32_t n = S.n_emitters;
    weight = 1.f;
    if (n < 2) return 0;
    if (S.distr) {
        const float sample = u * S.distr_sum;
        uint32_t start = 0, end = n - 1u;
        const uint32_t it = 32u - (uint32_t) __builtin_clz(end);
        for (uint32_t k = 0; k < it; ++k) {
            const uint32_t middle = (start + end) >> 1;
            const float c = S.emitters[middle].cdf;
            const bool cond = ((c < sample) || c == 0.f) && c != S.distr_sum;
            start = cond ? min(middle + 1u, end) : start;
            end = cond ? end : middle;
        }
        const float pmf = S.emitters[start].weight * S.distr_norm;
        const float cdf = start > 0 ? S.emitters[start - 1].cdf * S.distr_norm : 0.f;
        u = (u - cdf) / pmf;
        weight = rcp(pmf);
        return start;
    }
    const float scaled = u * (float) n;
    const uint32_t index = min((uint32_t) scaled, n - 1u);
    weight = (float) n;
    u = scaled - (float) index;
    return index;
}

/*
 * Mesh::sample_position (mesh.cpp:765-816) + Shape::sample_direction (shape.cpp:360-377):
 * the face from m_area_pmf.sample_reuse (distr_1d.h: JIT predicate of sample(), binary search
 * over [0, n - 1]), a uniform point on it (warp::square_to_uniform_triangle), the interpolated
 * shading normal when the mesh has vertex normals, else the face normal.
 */
AD DSamp mesh_sample_direction(const DScene &S, const DShape &s, f3 itp, float u1, float u2) {
    DSamp ds = ds_zero();
    const float2 *tab = reinterpret_cast<const float2 *>(S.face_area) + s.fbase;
    const float sum = s.area_sum, norm_ = s.inv_area, sample = u2 * sum;
    uint32_t start = 0, end = s.n_faces - 1u;
    const uint32_t it = end ? 32u - (uint32_t) __builtin_clz(end) : 0u;
    for (uint32_t k = 0; k < it; ++k) {
        const uint32_t middle = (start + end) >> 1;
        const float c = tab[middle].y;
        const bool cond = ((c < sample) || c == 0.f) && c != sum;
        start = cond ? min(middle + 1u, end) : start;
        end = cond ? end : middle;
    }
    const float pmf = tab[start].x * norm_, cdf = start > 0 ? tab[start - 1].y * norm_ : 0.f;
    u2 = (u2 - cdf) / pmf;
    const uint32_t *fi = S.faces + 3 * (size_t) (s.fbase + start);
    const uint32_t i0 = s.vbase + fi[0], i1 = s.vbase + fi[1], i2 = s.vbase + fi[2];
    const f3 p0 = ld3(S.vpos + 3 * (size_t) i0), p1 = ld3(S.vpos + 3 * (size_t) i1), p2 = ld3(S.vpos + 3 * (size_t) i2);
    const f3 e0 = p1 - p0, e1 = p2 - p0;
    const float t = safe_sqrt(1.f - u1), bx = 1.f - t, by = t * u2;
    ds.p = fma3(e0, bx, fma3(e1, by, p0));
    f3 n;
    if (s.has_normals) {
        const f3 n0 = ld3(S.vnrm + 3 * (size_t) i0), n1 = ld3(S.vnrm + 3 * (size_t) i1),
                 n2 = ld3(S.vnrm + 3 * (size_t) i2);
        n = fma3(n0, 1.f - bx - by, fma3(n1, bx, n2 * by));
    } else {
        n = cross(e0, e1);
    }
    ds.n = normalize(n);
    if (s.flip) ds.n = -ds.n;
    ds.pdf = norm_;
    ds.d = ds.p - itp;
    const float d2 = sqnorm(ds.d);
    ds.dist = dsqrt(d2);
    ds.d = ds.d / ds.dist;
    const float x = d2 / absdot(ds.d, ds.n);
    ds.pdf *= finite_(x) ? x : 0.f;
    return ds;
}

/*
 * Scene::sample_emitter_direction (scene.cpp:294-348) up to its ray_test: returns
 * true when the reference would trace the shadow ray spawn_ray_to(ref.p, ref.n,
 * ds.p).  The test itself runs in its own wavefront (k_vis slot 0 for primary
 * vertices, k_shadow / k_bounce for suffix vertices); an occluded sample is then zeroed
 * exactly as the reference does (spec = 0, ds.pdf = 0).
 */
AD bool sample_emitter_direction(const SceneRef &sc, const SI &ref, float u1, float u2, bool active, DSamp &ds,
                                 C3 &spec) {
    ds = ds_zero();
    spec = c3(0.f);
    const DScene &S = *sc.g;
    if (S.n_emitters == 0) return false;
    float weight;
    const uint32_t index = sample_emitter(S, u1, weight);
    if (!active) return false;
    const DEmitter &em = S.emitters[index];
    if (em.type == AMVPT_EMITTER_CONSTANT) {
        /* ConstantBackgroundEmitter::sample_direction (constant.cpp:125-152) */
        const f3 d = uniform_sphere(u1, u2);
        const f3 c = mk(S.bs_center[0], S.bs_center[1], S.bs_center[2]);
        const float radius = vmax(S.bs_radius, norm(ref.p - c)), dist = 2.f * radius;
        ds.p = fma3(d, dist, ref.p);
        ds.n = -d;
        ds.pdf = kInvFourPi;
        ds.delta = false;
        ds.d = d;
        ds.dist = dist;
        spec = c3(em.radiance) / ds.pdf;
    } else {
        const DShape &s = S.shapes[em.shape];
        ds = s.type == PRIM_TRI ? mesh_sample_direction(S, s, ref.p, u1, u2) : shape_sample_direction(s, ref.p, u1, u2);
        bool a = dot(ds.d, ds.n) < 0.f && ds.pdf != 0.f;
        spec = csel(a, c3(em.radiance) / ds.pdf, c3(0.f));
    }
    ds.emitter = (int32_t) index;
    ds.pdf *= emitter_pick_pmf(S, index);
    spec = spec * weight;
    return ds.pdf != 0.f;
}
AD void occlude_emitter_sample(DSamp &ds, C3 &spec) { spec = c3(0.f); ds.pdf = 0.f; }

AD float pdf_emitter_direction(const SceneRef &sc, f3 refp, const DSamp &ds, bool active) {
    if (ds.emitter < 0 || !active) return 0.f;
    const DEmitter &em = sc.g->emitters[ds.emitter];
    const float pick = emitter_pick_pmf(*sc.g, (uint32_t) ds.emitter);
    /* ConstantBackgroundEmitter::pdf_direction (constant.cpp:154-159): the uniform sphere */
    if (em.type == AMVPT_EMITTER_CONSTANT) return kInvFourPi * pick;
    const DShape &s = sc.g->shapes[em.shape];
    bool a = dot(ds.d, ds.n) < 0.f;
    float v = shape_pdf_direction(s, refp, ds);
    return (a ? v : 0.f) * pick;
}

AD float mis_weight(float a, float b) {
    a *= a; b *= b;
    float w = a / (a + b);
    return finite_(w) ? w : 0.f;
}

/* ------------------------------------------------------------------ */
/* Sensors                                                            */
/* ------------------------------------------------------------------ */

AD Ray persp_sample_ray(const DView &v, float x, float y) {
    f3 near_p = xf_point(v.sample_to_camera, mk(x + v.pp[0], y + v.pp[1], 0.f));
    f3 d = normalize(near_p);
    Ray r;
    r.o = mk(v.to_world[3], v.to_world[7], v.to_world[11]);
    r.d = xf_vector(v.to_world, d);
    float inv_z = rcp(d.z);
    float near_t = v.near_clip * inv_z, far_t = v.far_clip * inv_z;
    r.o = r.o + r.d * near_t;
    r.maxt = far_t - near_t;
    return r;
}

/* GridSensor::sample_ray_idx (grid.cpp:269-297) */
/* ThinLensCamera::sample_ray (thinlens.cpp:220-257); ap = the lane's aperture sample */
AD Ray thin_sample_ray(const DView &v, float x, float y, float apx, float apy) {
    f3 near_p = xf_point(v.sample_to_camera, mk(x, y, 0.f));
    float tx, ty;
    disk_concentric(apx, apy, tx, ty);
    const f3 aperture_p = mk(v.aperture_radius * tx, v.aperture_radius * ty, 0.f);
    const f3 focus_p = near_p * (v.focus_distance / near_p.z);
    const f3 d = normalize(focus_p - aperture_p);
    Ray r;
    r.o = xf_point_affine(v.to_world, aperture_p);
    r.d = xf_vector(v.to_world, d);
    float inv_z = rcp(d.z);
    float near_t = v.near_clip * inv_z, far_t = v.far_clip * inv_z;
    r.o = r.o + r.d * near_t;
    r.maxt = far_t - near_t;
    return r;
}
AD Ray camera_sample_ray(const DView &v, float x, float y, float apx, float apy) {
    return v.type == AMVPT_CAMERA_THINLENS ? thin_sample_ray(v, x, y, apx, apy) : persp_sample_ray(v, x, y);
}

AD Ray sample_ray_idx(const KParams &P, const DView *V, float ax, float ay, uint32_t &index, float apx = .5f,
                      float apy = .5f) {
    if (!P.multisensor) { index = 0; return camera_sample_ray(V[0], ax, ay, apx, apy); }
    if (P.batch) {
        /* BatchSensor::sample_ray_idx (batch.cpp:163-181): clamp, then reverse_x */
        const float fx = ax * (float) P.n_views;
        const uint32_t ux = (uint32_t) fx;
        index = min(ux, P.n_views - 1);
        if (P.rev_x) index = (P.n_views - 1) - index;
        return camera_sample_ray(V[index], fx - (float) ux, ay, apx, apy);
    }
    float fx = ax * (float) P.gx, fy = ay * (float) P.gy;
    uint32_t ux = (uint32_t) fx, uy = (uint32_t) fy;
    uint32_t ix = ux, iy = uy;
    if (P.rev_x) ix = (P.gx - 1) - ix;
    if (P.rev_y) iy = (P.gy - 1) - iy;
    index = ix + P.gx * iy;
    index = min(index, P.n_views - 1);
    return camera_sample_ray(V[index], fx - (float) ux, fy - (float) uy, apx, apy);
}

/* the view index part of sample_ray_idx (same arithmetic), for kernels that only need it */
AD uint32_t sensor_index(const KParams &P, float ax, float ay) {
    if (!P.multisensor) return 0;
    if (P.batch) {
        const uint32_t ux = (uint32_t) (ax * (float) P.n_views);
        uint32_t index = min(ux, P.n_views - 1);
        if (P.rev_x) index = (P.n_views - 1) - index;
        return index;
    }
    uint32_t ix = (uint32_t) (ax * (float) P.gx), iy = (uint32_t) (ay * (float) P.gy);
    if (P.rev_x) ix = (P.gx - 1) - ix;
    if (P.rev_y) iy = (P.gy - 1) - iy;
    return min(ix + P.gx * iy, P.n_views - 1);
}

struct Surf { f3 p, d; float uvx, uvy, pdf, Jp; bool face, valid; };

/* Film position of a camera-space point: the raster part of PerspectiveCamera::sample_surface
 * (perspective.cpp:327-385).  Shared by the primary vertex and the splat's reprojection, so
 * both compute the same bits. */
template <class VT> AD void persp_uv(const VT &v, f3 ref_p, float &ux, float &uy, float &uvx, float &uvy) {
    f3 screen = xf_point(v.camera_to_sample, ref_p);
    ux = screen.x - v.pp[0];
    uy = screen.y - v.pp[1];
    uvx = ux * v.res[0];
    uvy = uy * v.res[1];
}
/* the same for ThinLensCamera::sample_surface (thinlens.cpp:358-418) */
template <class VT>
AD void thin_uv(const VT &v, f3 ref_p, float apx, float apy, f3 &aperture_p, f3 &local_d, float &inv_dist, f3 &scr,
                float &uvx, float &uvy) {
    float tx, ty;
    disk_concentric(apx, apy, tx, ty);
    aperture_p = mk(tx * v.aperture_radius, ty * v.aperture_radius, 0.f);
    local_d = ref_p - aperture_p;
    const float dist = norm(local_d);
    inv_dist = rcp(dist);
    local_d = local_d * inv_dist;
    const float inv_f = 1.f / v.focus_distance;
    const f3 film_plane = mk(aperture_p.x * inv_f + local_d.x / local_d.z, aperture_p.y * inv_f + local_d.y / local_d.z,
                             aperture_p.z * inv_f + local_d.z / local_d.z);
    scr = xf_point_affine(v.camera_to_sample, film_plane);
    uvx = scr.x * v.res[0];
    uvy = scr.y * v.res[1];
}
/* Surf::uvx/uvy of camera_sample_surface(v, {p}, active = true, ap): the splat position of a
 * reprojected view sample, recomputed from the primary hit point instead of stored */
template <class VT> AD void camera_uv(const VT &v, f3 p, float apx, float apy, float &uvx, float &uvy) {
    const f3 ref_p = xf_point_affine(v.to_world_inv, p);
    if (v.type == AMVPT_CAMERA_THINLENS) {
        f3 ap, ld, scr;
        float idist;
        thin_uv(v, ref_p, apx, apy, ap, ld, idist, scr, uvx, uvy);
    } else {
        float ux, uy;
        persp_uv(v, ref_p, ux, uy, uvx, uvy);
    }
}

/* PerspectiveCamera::sample_surface under a masked vcall (perspective.cpp:327-385) */
AD Surf persp_sample_surface(const DView &v, const SI &it, bool active) {
    Surf r;
    r.p = mk(0.f, 0.f, 0.f); r.d = mk(0.f, 0.f, 0.f);
    r.uvx = r.uvy = r.pdf = r.Jp = 0.f;
    r.face = false; r.valid = false;
    if (!active) return r;
    f3 ref_p = xf_point_affine(v.to_world_inv, it.p);
    bool a = ref_p.z >= v.near_clip && ref_p.z <= v.far_clip;
    float ux, uy;
    persp_uv(v, ref_p, ux, uy, r.uvx, r.uvy);
    a = a && ux >= 0.f && ux <= 1.f && uy >= 0.f && uy <= 1.f;
    float dist = norm(ref_p), inv_dist = rcp(dist);
    float ctf = ref_p.z;
    a = a && ctf > 0.f;
    float ictf = rcp(ctf), ictf3 = ictf * ictf * ictf;
    r.pdf = v.normalization * ictf3;
    r.p = xf_point_affine(v.to_world, mk(0.f, 0.f, 0.f));
    r.d = (r.p - it.p) * inv_dist;
    float cts = dot(r.d, it.n);
    r.face = cts > 0.f;
    cts = fabs_(cts);
    r.Jp = (cts * inv_dist * inv_dist) * r.pdf;
    r.valid = a;
    return r;
}

/* ThinLensCamera::sample_surface (thinlens.cpp:358-418), JIT semantics */
AD Surf thin_sample_surface(const DView &v, const SI &it, bool active, float apx, float apy) {
    Surf r;
    r.p = mk(0.f, 0.f, 0.f); r.d = mk(0.f, 0.f, 0.f);
    r.uvx = r.uvy = r.pdf = r.Jp = 0.f;
    r.face = false; r.valid = false;
    if (!active) return r;
    const f3 ref_p = xf_point_affine(v.to_world_inv, it.p);
    bool a = ref_p.z >= v.near_clip && ref_p.z <= v.far_clip;
    f3 aperture_p, local_d, scr;
    float inv_dist;
    thin_uv(v, ref_p, apx, apy, aperture_p, local_d, inv_dist, scr, r.uvx, r.uvy);
    const float ictf = rcp(local_d.z), ictf3 = ictf * ictf * ictf;
    a = a && scr.x >= 0.f && scr.y >= 0.f && scr.x <= 1.f && scr.y <= 1.f;
    const float pdf_lens = rcp(sqr(v.aperture_radius) * kPi);
    r.pdf = pdf_lens * (v.normalization * ictf3);
    r.p = xf_point_affine(v.to_world, aperture_p);
    r.d = (r.p - it.p) * inv_dist;
    float cts = dot(r.d, it.n);
    r.face = cts > 0.f;
    cts = fabs_(cts);
    r.Jp = (cts * inv_dist * inv_dist) * r.pdf;
    r.valid = a;
    return r;
}
AD Surf camera_sample_surface(const DView &v, const SI &it, bool active, float apx, float apy) {
    return v.type == AMVPT_CAMERA_THINLENS ? thin_sample_surface(v, it, active, apx, apy)
                                           : persp_sample_surface(v, it, active);
}
/* The raster fields of a DView (floats 12..23, 40..55, 60..67 of the 68-float record):
 * all camera_uv reads.  raster_uniform() fetches them with scalar loads when the view index
 * is wave-uniform (a splat wave = 64 pixels of one view row, so it nearly always is). */
struct DRaster {
    float to_world_inv[12];
    float camera_to_sample[16];
    float res[2], pp[2];
    uint32_t type;
    float aperture_radius, focus_distance, pad1;
};
static_assert(sizeof(DView) == 17 * 16 && sizeof(DRaster) == 9 * 16, "view record layout");
AD DRaster raster_uniform(const DView *V, uint32_t id) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(4))) const v4u cv4u;
    const cv4u *p = (const cv4u *) (uintptr_t) V + (size_t) __builtin_amdgcn_readfirstlane(id) * 17;
    const v4u q[9] = {p[3], p[4], p[5], p[10], p[11], p[12], p[13], p[15], p[16]};
    DRaster r;
    __builtin_memcpy(&r, q, sizeof(r));
    return r;
}
/* camera_uv of view `id` (wave-uniform fast path, per-lane fallback) */
AD void view_uv(const DView *V, uint32_t id, f3 p, float apx, float apy, float &uvx, float &uvy) {
    const uint32_t id0 = __builtin_amdgcn_readfirstlane(id);
    if (__ballot(id != id0) == 0ull) camera_uv(raster_uniform(V, id0), p, apx, apy, uvx, uvy);
    else camera_uv(V[id], p, apx, apy, uvx, uvy);
}

/* Surf::p of camera_sample_surface (the visibility-ray target), bit for bit */
AD f3 camera_point(const DView &v, float apx, float apy) {
    if (v.type != AMVPT_CAMERA_THINLENS) return xf_point_affine(v.to_world, mk(0.f, 0.f, 0.f));
    float tx, ty;
    disk_concentric(apx, apy, tx, ty);
    return xf_point_affine(v.to_world, mk(tx * v.aperture_radius, ty * v.aperture_radius, 0.f));
}

/* ------------------------------------------------------------------ */
/* Film                                                               */
/* ------------------------------------------------------------------ */

/*
 * One film float += v.  Deterministic mode (AMVPT_OPT_DETERMINISTIC, KParams::film_fx): the value goes to
 * the same cell of a 32.32 fixed-point shadow film with an integer atomic -- integer sums do not depend
 * on the order the waves arrive in, so the film is bitwise reproducible (imageblock.cpp:119-133's
 * accumulation, resolved once per render by k_fixed_resolve).  Non-finite values are dropped there.
 */
constexpr double kFixScale = 4294967296.0, kFixLimit = 2147483647.0;
/* kDet = false: a kernel instance that never runs in deterministic mode (the row splat) */
template <bool kDet = true> AD void film_add(const KParams &P, float *p, float v) {
    if (kDet && P.film_fx) {
        const double d = (double) v * kFixScale;
        if (!(fabs(d) < kFixLimit * kFixScale)) {   /* NaN / Inf (counted per sample by check_sample) / out of range */
            if (P.fx_drops && __builtin_isfinite(v)) atomicAdd(P.fx_drops + blockIdx.x % 256u, 1ull);   /* kStatShards */
            return;
        }
        atomicAdd(P.film_fx + (p - P.film_base), (unsigned long long) (long long) __builtin_rint(d));
        return;
    }
    atomicAdd(p, v);
}

/*
 * Film window (amvpt_film_window).  The film buffer holds the quilt rectangle [fx0, fx0 + fw) x
 * [fy0, fy0 + fh); footprints are clipped to the QUILT as ImageBlock::put clips them
 * (imageblock.cpp:265-558), and a cell of the quilt outside the window is appended to the overflow
 * list (a view-group rank's rare lanes whose jittered position rounds into the next tile).  With the
 * whole-quilt window (the single-GPU frame) every cell is inside.
 */
/* kWin = false: the whole-quilt window, known at compile time (the row-splat kernels' instance for
 * single-GPU frames; the runtime test cost 3.5 ms of k_splat per config-M frame, A/B r03d) */
template <bool kWin = true> AD bool in_window(const KParams &P, int x, int y) {
    if (!kWin) return true;
    return (uint32_t) (x - (int) P.fx0) < P.fw && (uint32_t) (y - (int) P.fy0) < P.fh;
}
/* film float of quilt cell (x, y), channel k -- the cell must be inside the window */
template <bool kWin = true> AD float *film_cell(const KParams &P, float *film, int x, int y, int k) {
    if (!kWin) return film + ((size_t) (uint32_t) y * P.W + (uint32_t) x) * P.C + k;
    return film + ((size_t) (uint32_t) (y - (int) P.fy0) * P.fw + (uint32_t) (x - (int) P.fx0)) * P.C + k;
}
/* append quilt float `idx` += v to the overflow list (one returning atomic: rare by construction) */
AD void overflow_push(const KParams &P, uint64_t idx, float v) {
    if (!P.overflow) return;   /* the host requires the list for any window smaller than the quilt */
    const unsigned long long e = atomicAdd(reinterpret_cast<unsigned long long *>(P.overflow), 1ull);
    if (e < P.ov_cap)
        reinterpret_cast<uint4 *>(P.overflow + 4)[e] = make_uint4((uint32_t) idx, (uint32_t) (idx >> 32), __float_as_uint(v), 0u);
}
/* one film float of quilt cell (x, y), channel k: the window, else the overflow list */
template <bool kWin = true, bool kDet = true> AD void film_cell_add(const KParams &P, float *film, int x, int y, int k, float v) {
    if (in_window<kWin>(P, x, y)) film_add<kDet>(P, film_cell<kWin>(P, film, x, y, k), v);
    else overflow_push(P, ((uint64_t) (uint32_t) y * P.W + (uint32_t) x) * P.C + (uint32_t) k, v);
}

/* ------------------------------------------------------------------ */
/* Block-cooperative ImageBlock::put                                   */
/* ------------------------------------------------------------------ */
/*
 * Every thread of a splat block calls block_put() with its own sample (`valid`
 * may be false).  The block's footprints are accumulated in an LDS window and
 * the window is flushed once with global float atomics (skipping cells that
 * received nothing), so the film sees about one atomic per touched
 * pixel-channel per block instead of one per sample.  Footprints that do not
 * fit the window fall back to direct global atomics.  The per-cell weights and
 * the per-cell products value * weight are exactly those of film_put
 * (imageblock.cpp:174-559); only the order of the additions differs.
 *
 * LDS adds on gfx950 (tools/ubench_lds.hip, lane-ops/clk/CU, distinct 8-byte
 * words): ds_add_f32 0.33, a 64-bit compare-and-swap of a float pair 1.55 (3.1
 * channel adds), ds_add_f64 7.4.  The window therefore holds one fp64 word per
 * cell and channel and every contribution is one fire-and-forget ds_add_f64
 * (no return value, no retry loop, NaN/Inf propagate as in fp32).  The f32
 * products are exact in fp64 and the window sum is rounded once to f32 at the
 * flush -- a block's sum is at least as accurate as the reference's sequential
 * fp32 scatter_reduce.
 *
 * The flush writes zeros back, so one put costs two block barriers and no zeroing
 * pass; the window is single-buffered (the next put's first barrier orders its
 * adds after this flush), only the tiny bounding-box exchange alternates buffers.
 */
#ifndef AMVPT_WIN_H
#define AMVPT_WIN_H 8
#endif
#ifndef AMVPT_SPLAT_BLOCK
#define AMVPT_SPLAT_BLOCK 256
#endif
/* Row stride of the window: rows of ww cells are laid out rs cells apart with rs % 32 == 16,
 * so consecutive rows start 32 banks apart for the 64-bit cells (2 * rs mod 64 = 32): lanes
 * whose reprojected footprints straddle a row boundary stop colliding on banks
 * (measured: splat 206 -> 187 ms at config M; rs = ww, or % 32 in {1, 8, 17, 24}: 200-207 ms).
 * The 112-cell width leaves room for the padding (5 blocks per CU either way). */
/* measurement-only attribution builds (wrong images): 1 skips the LDS adds, 2 the flush's
 * film atomics, 4 the filter weights, 8 turns the LDS atomic adds into plain stores, 16 (with 32:
 * the row-half products too) drops the row splat's cross-lane reduce steps */
#ifndef AMVPT_ATTR_SKIP
#define AMVPT_ATTR_SKIP 0
#endif
#ifndef AMVPT_WIN_RS
#define AMVPT_WIN_RS 16
#endif
#ifndef AMVPT_WIN_W
#define AMVPT_WIN_W 112
#endif
constexpr int kWinW = AMVPT_WIN_W, kWinH = AMVPT_WIN_H, kMaxWaves = 16, kMaxFoot = 5;
constexpr int kSplatSuper = 1024;   /* lanes per splat super-block (see slot_lane) */
constexpr int kSplatBlock = AMVPT_SPLAT_BLOCK;   /* threads per splat block (see slot_lane) */
constexpr int kWinCells = kWinW * kWinH;
/*
 * Window cell format.  AMVPT_WIN_FIXED = 0 (default): fp64 cells accumulated with ds_add_f64 --
 * each f32 contribution is exact in f64 and a cell holds at most a few hundred of them, so the
 * window sum is the exact sum to far below the f32 film's resolution.  AMVPT_WIN_FIXED = 1: signed
 * 32.32 fixed point in an int64 word with ds_add_u64 (9.7 lane-ops/clk/CU against 7.5 for
 * ds_add_f64 in isolation, tools/ubench_lds.hip, profiles/r02a_ubench.log; order-independent
 * integer sums, values of magnitude >= 2^20 or non-finite bypass the window) -- but its six-VALU
 * conversion per add costs more than the atomic rate gains now that the row splat is VALU-bound:
 * config-M splat 105.0 ms fixed vs 99.8 ms fp64 (r02fo, r02fp).  AMVPT_WIN_FIXED = 2: fp32 cells
 * with ds_add_f32: 142 ms (the 64-bit bank layout of the row adds no longer spreads).
 */
#ifndef AMVPT_WIN_FIXED
#define AMVPT_WIN_FIXED 0
#endif
#if AMVPT_WIN_FIXED == 2
typedef float WinT;        /* fp32 cells, ds_add_f32 (A/B) */
#elif AMVPT_WIN_FIXED
typedef long long WinT;
#else
typedef double WinT;
#endif
constexpr float kFixMax = 1048576.f;   /* 2^20 */
/* floor(x * 2^32) as a 64-bit two's-complement word, |x| < 2^31: the high dword is floor(x), the
 * low dword the fraction x - floor(x) (exact) times 2^32, truncated (clamped below 2^32, where a
 * tiny negative x rounds the fraction up to 1) -- six VALU ops, no 64-bit arithmetic */
AD long long to_fixed(float x) {
    const float hf = floorf(x);
    const uint32_t lo = (uint32_t) fminf((x - hf) * 4294967296.f, 4294967040.f);
    const uint32_t hi = (uint32_t) (int32_t) hf;
    return (long long) (((unsigned long long) hi << 32) | lo);
}
AD float from_fixed(long long q) { return (float) ((double) q * 2.3283064365386963e-10); }

/* channel planes of the window are `plane` cells apart, plane <= kWinPlane (see window_bbox) */
constexpr int kWinPlane = kWinCells + 32;
/*
 * AMVPT_WAVE_WIN = 1: the row-reduced splat (row_put) gives every wave a window of its own
 * (kWaveWinW x kWaveWinH cells): a wave's bounding box, adds and flush need no block barrier
 * (LDS operations of one wave complete in order).  A wave = 4 pixels x 16 samples, whose
 * footprints span ~8 x 5 cells (view 0) to ~10 x 6 (reprojected views).
 */
#ifndef AMVPT_WAVE_WIN
#define AMVPT_WAVE_WIN 1
#endif
#ifndef AMVPT_WAVE_WIN_W
#define AMVPT_WAVE_WIN_W 32
#endif
constexpr int kWaveWinW = AMVPT_WAVE_WIN_W, kWaveWinH = 6, kWavePlane = kWaveWinW * kWaveWinH + 32;
constexpr int kSplatWaves = AMVPT_SPLAT_BLOCK / 64;
template <int C> struct SplatLds {
    WinT win[kWinPlane * C];                /* channel k of cell c at win[k * plane + c] */
    alignas(16) int bb[2][kMaxWaves][4];
};
/* the wave windows of a row-splat block: wave w's window at win[w * kWavePlane * C] */
template <int C> struct WaveLds {
    WinT win[kSplatWaves * kWavePlane * C];
};
template <int C> AD void wave_lds_init(WaveLds<C> &L) {
    for (int c = threadIdx.x; c < kSplatWaves * kWavePlane * C; c += blockDim.x) L.win[c] = 0;
    __syncthreads();
}

template <int C> AD void splat_lds_init(SplatLds<C> &L) {
    for (int c = threadIdx.x; c < kWinPlane * C; c += blockDim.x) L.win[c] = 0;
    __syncthreads();
}

struct Foot { int x0, y0, nx, ny; float rx, ry; bool ok; };

/* Footprint of ImageBlock::put: first covered pixel (x0, y0), extent (nx, ny) after
 * clipping, and the filter argument rx/ry of pixel (x0, y0). */
AD Foot footprint(const KParams &P, float px, float py, bool coalesce) {
    Foot f;
    const int W = (int) P.W, H = (int) P.H;
    if (P.box) {
        /* imageblock.cpp:211: floor(pos) - offset */
        int ix = (int) floorf(px) - (int) P.off_x, iy = (int) floorf(py) - (int) P.off_y;
        f.ok = (uint32_t) ix < (uint32_t) W && (uint32_t) iy < (uint32_t) H;
        f.x0 = ix; f.y0 = iy; f.nx = f.ny = 1; f.rx = f.ry = 0.f;
        return f;
    }
    const float radius = P.filt.radius;
    if (!coalesce) {
        /* non-coalesced method (imageblock.cpp:265-427): pos + ((int) border - offset - .5f) */
        float pfx = px + P.nc_ox, pfy = py + P.nc_oy;
        int p0x = max((int) ceilf(pfx - radius), 0), p0y = max((int) ceilf(pfy - radius), 0);
        int p1x = min((int) floorf(pfx + radius), W - 1), p1y = min((int) floorf(pfy + radius), H - 1);
        f.ok = (uint32_t) p0x <= (uint32_t) p1x && (uint32_t) p0y <= (uint32_t) p1y;
        const int count = (int) ceilf(2.f * radius);
        f.x0 = p0x; f.y0 = p0y;
        f.nx = min(p1x - p0x + 1, count); f.ny = min(p1y - p0y + 1, count);
        f.rx = (float) (uint32_t) p0x - pfx;
        f.ry = (float) (uint32_t) p0y - pfy;
        return f;
    }
    /* coalesced method (imageblock.cpp:433-558): count = 2n+1 cells from floor(pos) - n, minus the
     * block offset; weights are evaluated at ((pix + .5) - pos) + xs in film coordinates */
    const int n = (int) ceilf(radius - .5f), count = 2 * n + 1;
    const int gx0 = (int) floorf(px) - n, gy0 = (int) floorf(py) - n;
    f.rx = ((float) gx0 + .5f) - px;
    f.ry = ((float) gy0 + .5f) - py;
    const int pix = gx0 - (int) P.off_x, piy = gy0 - (int) P.off_y;
    int sx = max(0, -pix), sy = max(0, -piy);
    f.x0 = pix; f.y0 = piy;
    f.nx = min(count, W - pix);
    f.ny = min(count, H - piy);
    f.ok = f.nx > sx && f.ny > sy;
    return f;
}

AD int wave_min(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
    return v;
}
AD int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

/* ds_add_f64, result unused (the backend emits the no-return form) */
AD void lds_add64(double *p, double v) {
    (void) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
/* ds_add_u64, result unused; one window contribution in the cell format */
AD void lds_add64(long long *p, long long v) {
    (void) __hip_atomic_fetch_add(reinterpret_cast<unsigned long long *>(p), (unsigned long long) v, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_WORKGROUP);
}
AD void win_add(double *p, float x) {
    if (AMVPT_ATTR_SKIP & 8) *p = (double) x;   /* attribution: a plain LDS store instead of ds_add_f64 */
    else lds_add64(p, (double) x);
}
AD void win_add(float *p, float x) {
    (void) __hip_atomic_fetch_add(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
AD void win_add(long long *p, float x) { lds_add64(p, to_fixed(x)); }
/* may the sample go through the window?  (fixed point: finite and below 2^20 in every channel) */
template <int C> AD bool win_fits(const float *vals) {
#if AMVPT_WIN_FIXED == 1
    bool ok = true;
#pragma unroll
    for (int k = 0; k < C; ++k) ok = ok && fabsf(vals[k]) < kFixMax;
    return ok;
#else
    return true;
#endif
}

/* The block's window: union of the active footprints, clamped to kWinW x kWinH. */
struct Win { int bx0, by0, ww, wh, rs, plane; };   /* rs: LDS row stride (cells) >= ww; plane >= rs * wh */
template <int C>
AD Win window_bbox(SplatLds<C> &L, int buf, bool act, int cx0, int cy0, int x1, int y1, int win_rs, bool row_splat) {
    int lx = act ? cx0 : 0x7fffffff, ly = act ? cy0 : 0x7fffffff;
    int hx = act ? x1 : (int) 0x80000000, hy = act ? y1 : (int) 0x80000000;
    lx = wave_min(lx); ly = wave_min(ly); hx = wave_max(hx); hy = wave_max(hy);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        L.bb[buf][wave][0] = lx; L.bb[buf][wave][1] = ly; L.bb[buf][wave][2] = hx; L.bb[buf][wave][3] = hy;
    }
    __syncthreads();
    int bx0 = 0x7fffffff, by0 = 0x7fffffff, bx1 = (int) 0x80000000, by1 = (int) 0x80000000;
    {
        const int l = threadIdx.x & 63;
        if (l < (int) (blockDim.x >> 6)) {
            const int4 q = *reinterpret_cast<const int4 *>(&L.bb[buf][l][0]);
            bx0 = q.x; by0 = q.y; bx1 = q.z; by1 = q.w;
        }
#pragma unroll
        for (int o = kMaxWaves / 2; o > 0; o >>= 1) {
            bx0 = min(bx0, __shfl_xor(bx0, o)); by0 = min(by0, __shfl_xor(by0, o));
            bx1 = max(bx1, __shfl_xor(bx1, o)); by1 = max(by1, __shfl_xor(by1, o));
        }
        bx0 = __shfl(bx0, 0); by0 = __shfl(by0, 0); bx1 = __shfl(bx1, 0); by1 = __shfl(by1, 0);
    }
    const bool any = bx0 != 0x7fffffff && bx0 < bx1;
    Win w;
    w.bx0 = bx0; w.by0 = by0;
    w.ww = any ? min(bx1 - bx0, kWinW) : 0;
    w.wh = any ? min(by1 - by0, kWinH) : 0;
    /* row stride: ww rounded up to rs % 32 == win_rs (2 * rs mod 64 = the bank shift between
     * rows of a 64-bit cell), when that still fits the buffer */
    w.rs = w.ww;
    if (win_rs) {
        const int r = (w.ww & ~31) + win_rs, r2 = r >= w.ww ? r : r + 32;
        w.rs = r2 <= kWinW ? r2 : w.ww;
    }
    /* row_put's atomics of one 16-lane row hit 4 channels x 2 row sets (3 rows apart) x 2 column
     * sets (3 cells apart): with rs % 32 == 16 and plane % 32 == 4 their cell indices are 16
     * distinct residues mod 32, so the 16 lanes of an LDS cycle use 16 distinct bank pairs */
    w.plane = w.rs * w.wh;
    if (row_splat) w.plane += (36 - (w.plane & 31)) & 31;
    return w;
}

/* barrier, then one global float atomic per touched film float of the window; the window
 * is re-zeroed on the way (consecutive threads take consecutive floats of a film row) */
template <int C>
AD void window_flush(const KParams &P, float *film, SplatLds<C> &L, const Win &w) {
    __syncthreads();
    const int plane = w.plane;
    const int rowlen = w.ww * C;
    const float inv_rowlen = 1.f / (float) max(rowlen, 1);
    /* the LDS window's quilt cells inside the film window (uniform): straight film offsets */
    const bool inside = in_window(P, w.bx0, w.by0) && in_window(P, w.bx0 + max(w.ww, 1) - 1, w.by0 + max(w.wh, 1) - 1);
    float *film0 = inside ? film_cell(P, film, w.bx0, w.by0, 0) : film;
    const size_t film_row = (size_t) P.fw * C;
    WinT *win = L.win;
    const int n_elems = w.ww * w.wh * C;                    /* touched film floats (rows of ww cells) */
    for (int e = threadIdx.x; e < n_elems; e += blockDim.x) {
        int cy = (int) ((float) e * inv_rowlen);            /* e < 2^24: off by at most one */
        cy -= (cy * rowlen > e) ? 1 : 0;
        cy += ((cy + 1) * rowlen <= e) ? 1 : 0;
        const int r = e - cy * rowlen, cx = r / C, k = r - cx * C;
        WinT *src = win + k * plane + cy * w.rs + cx;
        const WinT d = *src;
#if AMVPT_WIN_FIXED == 2
        if (__float_as_int(d) != 0) {
            *src = 0.f;
            const float v = d;
#elif AMVPT_WIN_FIXED
        if (d != 0) {
            *src = 0;
            const float v = from_fixed(d);
#else
        if (__double_as_longlong(d) != 0ll) {
            *src = 0.0;
            const float v = (float) d;
#endif
            if ((v != 0.f || v != v) && !(AMVPT_ATTR_SKIP & 2)) {
                if (inside) film_add(P, film0 + (size_t) cy * film_row + r, v);
                else film_cell_add(P, film, w.bx0 + cx, w.by0 + cy, k, v);
            }
        }
    }
}

/* one footprint's cells straight into the window (or the film when it does not fit) */
/* kRolled: the window loop is not unrolled (row_put's rare per-lane path: an unrolled 5 x 5 x C
 * body would set the register allocation of the whole splat kernel) */
template <int C, bool kRolled = false, bool kWin = true, bool kDet = true>
AD void foot_add(const KParams &P, float *film, WinT *const wbase, const Win &wn, const Foot &f, const float *wx,
                 const float *wy, const float *vals, bool coalesce, uint32_t *fallback) {
    const int cx0 = max(f.x0, 0), cy0 = max(f.y0, 0);
    const int plane = wn.plane;
    const bool in_win = cx0 >= wn.bx0 && cy0 >= wn.by0 && f.x0 + f.nx <= wn.bx0 + wn.ww && f.y0 + f.ny <= wn.by0 + wn.wh;
    /* cells per footprint side: uniform over the call (filter radius and method only) */
    const int cnt = P.box ? 1 : (coalesce ? 2 * (int) ceilf(P.filt.radius - .5f) + 1 : (int) ceilf(2.f * P.filt.radius));
    if (in_win && cnt <= kMaxFoot && win_fits<C>(vals)) {
        /* straight-line cnt x cnt cells; clipped cells are masked off (no retry, no branch body) */
        WinT *const c0 = wbase + ((f.y0 - wn.by0) * wn.rs + (f.x0 - wn.bx0));
#pragma unroll(kRolled ? 1 : kMaxFoot)
        for (int ys = 0; ys < kMaxFoot; ++ys) {
            if (ys >= cnt) break;
            const bool rok = ys < f.ny && f.y0 + ys >= 0;
#pragma unroll
            for (int xs = 0; xs < kMaxFoot; ++xs) {
                if (xs >= cnt) break;
                if (rok && xs < f.nx && f.x0 + xs >= 0) {
                    const float w = wx[xs] * wy[ys];
                    WinT *const cp = c0 + ys * wn.rs + xs;
#pragma unroll
                    for (int k = 0; k < C; ++k)
                        if (!(AMVPT_ATTR_SKIP & 1)) win_add(cp + k * plane, P.box ? vals[k] : vals[k] * w);
                }
            }
        }
    } else {
        /* window miss (or a filter wider than kMaxFoot): direct global atomics */
        if (fallback && !in_win) ++*fallback;
        for (int ys = 0; ys < f.ny; ++ys) {
            const int y = f.y0 + ys;
            if (y < 0) continue;
            const float wyv = ys < kMaxFoot ? wy[ys] : (P.box ? 1.f : gaussian_eval(P.filt, f.ry + (float) ys));
            for (int xs = 0; xs < f.nx; ++xs) {
                const int x = f.x0 + xs;
                if (x < 0) continue;
                const float wxv = xs < kMaxFoot ? wx[xs] : (P.box ? 1.f : gaussian_eval(P.filt, f.rx + (float) xs));
                const float w = wxv * wyv;
#pragma unroll
                for (int k = 0; k < C; ++k) film_cell_add<kWin, kDet>(P, film, x, y, k, P.box ? vals[k] : vals[k] * w);
            }
        }
    }
}

/*
 * Deterministic mode's put: every cell of the sample's footprint straight into the fixed-point film,
 * value * (wx * wy) per cell as ImageBlock::put forms it (imageblock.cpp:265-558) -- no LDS window and
 * no row reduction, so no float sum depends on which lanes share a wave, a chunk or a stream.
 */
template <int C, bool kWin = true>
AD void direct_put(const KParams &P, float *film, float px, float py, const float *vals, bool valid, bool coalesce) {
    if (!valid) return;
    const Foot f = footprint(P, px, py, coalesce);
    if (!f.ok) return;
    for (int ys = 0; ys < f.ny; ++ys) {
        const int y = f.y0 + ys;
        if (y < 0) continue;
        const float wyv = P.box ? 1.f : gaussian_eval(P.filt, f.ry + (float) ys);
        for (int xs = 0; xs < f.nx; ++xs) {
            const int x = f.x0 + xs;
            if (x < 0) continue;
            const float w = (P.box ? 1.f : gaussian_eval(P.filt, f.rx + (float) xs)) * wyv;
#pragma unroll
            for (int k = 0; k < C; ++k) film_cell_add<kWin>(P, film, x, y, k, P.box ? vals[k] : vals[k] * w);
        }
    }
}

AD void foot_weights(const KParams &P, const Foot &f, float *wx, float *wy) {
#pragma unroll
    for (int t = 0; t < kMaxFoot; ++t) {
        wx[t] = P.box || (AMVPT_ATTR_SKIP & 4) ? 1.f : gaussian_eval(P.filt, f.rx + (float) t);
        wy[t] = P.box || (AMVPT_ATTR_SKIP & 4) ? 1.f : gaussian_eval(P.filt, f.ry + (float) t);
    }
}

/*
 * Row-reduced put (KParams::row_splat, RGBW films).  Lanes run pixel-major (slot_lane is the
 * identity), so a DPP row of 16 lanes holds 16 samples of one pixel: for view 0 (coalesced
 * method) the 16 footprints are the same 5 x 5 cells, and a reprojected view's 16 footprints
 * usually fall inside one 6 x 6 box.  When every active footprint of a row lies in the window,
 * the union box of the row is at most 6 x 6 and every value is finite and below kFixMax, the
 * row adds its 16 footprints as ONE reduced 6 x 6 x 4 block: every lane forms its products
 * value_c * (wx * wy) (the reference's per-cell products, imageblock.cpp:265-558) for all 36
 * union cells (zero weight outside its own footprint), and a 4-step reduce-scatter over the row
 * (DPP quad xor 1, quad xor 2, row rotate 4, row rotate 8) leaves each lane the row's sum for 9
 * cells of one channel -- 9 ds_add_u64 per lane and view instead of 64 (reprojected) or 100
 * (coalesced).  The products are summed in f32 before the window (the reference's f32 film
 * sums them in some atomic order as well).  Other rows take the per-lane path (foot_add).
 *
 * Ownership: lane bits b0 b1 pick the channel (b0 + 2 b1), b2 the row set (rows 0-2 or 3-5),
 * b3 the column set.  Steps 1-2 and 3 read their partner's values in a lane-permuted order
 * chosen once per sample (channel operands, rows), step 4 selects its column halves.
 */
enum : int { DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_XOR3 = 0x1B, DPP_ROR4 = 0x124, DPP_ROR8 = 0x128 };
template <int kCtrl> AD float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), kCtrl, 0xf, 0xf, true));
}
template <int kCtrl> AD int dpp_i(int v) { return __builtin_amdgcn_update_dpp(0, v, kCtrl, 0xf, 0xf, true); }
/* min / max over the lane's 16-lane row (every lane of the wave active) */
AD int row_min(int v) {
    v = min(v, dpp_i<DPP_XOR1>(v)); v = min(v, dpp_i<DPP_XOR2>(v));
    v = min(v, dpp_i<DPP_ROR4>(v)); return min(v, dpp_i<DPP_ROR8>(v));
}
AD int row_max(int v) {
    v = max(v, dpp_i<DPP_XOR1>(v)); v = max(v, dpp_i<DPP_XOR2>(v));
    v = max(v, dpp_i<DPP_ROR4>(v)); return max(v, dpp_i<DPP_ROR8>(v));
}
/* filter weight of film cell `cell` for a footprint starting at x0 with argument r, zero outside
 * the footprint's cells [lo, hi) -- inside it eval(r + (cell - x0)), the reference's argument */
AD float union_weight(const FilterCoeffs &F, float r, int x0, int cell, int lo, int hi) {
    const float w = gaussian_eval(F, r + (float) (cell - x0));
    return (cell >= lo && cell < hi) ? w : 0.f;
}
#ifndef AMVPT_SPLAT_PKW
/* 1: the row splat evaluates its union weights two at a time with packed-f32 operations (gaussian_eval2: the same
 * bits).  Slower (r06ai: splat 78.3 -> 81.7 ms at M, 320 -> 338 ms at C3 -- the scalar form folds every coefficient
 * into v_fmamk / v_fmaak literals, the packed one moves them through registers), so 0: one gaussian_eval per weight */
#define AMVPT_SPLAT_PKW 0
#endif
/* union_weight of cells a and b (packed evaluation) */
AD f2v_t union_weight2(const FilterCoeffs &F, float r, int x0, int a, int b, int lo, int hi) {
    const f2v_t w = gaussian_eval2(F, f2v_t{r + (float) (a - x0), r + (float) (b - x0)});
    return f2v_t{(a >= lo && a < hi) ? w.x : 0.f, (b >= lo && b < hi) ? w.y : 0.f};
}
/* The row splat runs for the default Gaussian only (rfilter stddev 0.5, the reference's default,
 * gaussian.cpp): its coefficients -- exactly what gaussian_coeffs(0.5) computes on the host, checked
 * there bit for bit before the row splat is chosen -- are compile-time literals, so every Estrin step is
 * one v_fmaak/v_fma with a literal instead of two SGPR operands copied through VGPRs (gfx9 VOP3 reads one
 * SGPR per instruction), and the kernel keeps 11 fewer SGPRs live */
AD FilterCoeffs default_filter() {
    return FilterCoeffs{{0x1.ff9d52p-1f, -0x1.fda5bcp+0f, 0x1.f4a20cp+0f, -0x1.3c9afep+0f, 0x1.181032p-1f, -0x1.604b8ap-3f,
                         0x1.34c5d4p-5f, -0x1.657e54p-8f, 0x1.e9dbd6p-12f, -0x1.2bffdp-16f},
                        0x1p+1f};
}

#ifndef AMVPT_SPLAT_SEL
#define AMVPT_SPLAT_SEL 1   /* row splat: the channel picks as selects on lane masks (0: a pick by lane index, which
                             * compiled to a branch tree; r05v: splat 85.0 -> 83.3 ms at M, 346.8 -> 343.4 at C3) */
#endif
#ifndef AMVPT_SPLAT_PK
#define AMVPT_SPLAT_PK 1   /* row splat: packed-f32 products of the two row halves: config-M splat 101.8 -> 97.7 ms (r03y; 0: A/B) */
#endif
/* union box of the active footprints of the lane's 16-lane row (every lane of the wave active) */
struct RowBox { int x0, y0, x1, y1; };
AD RowBox row_box(const Foot &f, bool act) {
    constexpr int kBig = 0x3fffffff;
    return RowBox{row_min(act ? max(f.x0, 0) : kBig), row_min(act ? max(f.y0, 0) : kBig),
                  row_max(act ? f.x0 + f.nx : -kBig), row_max(act ? f.y0 + f.ny : -kBig)};
}
template <int C, bool kWin = true>
AD void row_put_win(const KParams &P, float *film, WinT *const wbase, const Win &wn, const Foot &f, bool act,
                    const float *vals, bool coalesce, uint32_t *fallback, const RowBox &ub) {
    const int x0c = max(f.x0, 0), y0c = max(f.y0, 0), x1 = f.x0 + f.nx, y1 = f.y0 + f.ny;
    const bool inw = x0c >= wn.bx0 && y0c >= wn.by0 && x1 <= wn.bx0 + wn.ww && y1 <= wn.by0 + wn.wh;
    const bool good = inw && win_fits<C>(vals);
    const int ux0 = ub.x0, uy0 = ub.y0, ux1 = ub.x1, uy1 = ub.y1;
    const int bad = row_max((act && !good) ? 1 : 0);
    const bool fast = C == 4 && ux1 > ux0 && bad == 0 && ux1 - ux0 <= 6 && uy1 - uy0 <= 6;
    if (fast) {
        /* every fast row of the wave within 5 union columns / rows (the common case: a coalesced footprint is 5
         * cells, a reprojected one 4, and a pixel's 16 samples spread less than a cell): the sixth union column /
         * row -- zero weights in every lane -- is skipped (r05za/r05zb: splat 82.0 -> 78.0 ms at M, 330.2 ->
         * 311.7 at C3) */
        const bool u5 = !wave_any(ux1 - ux0 > 5), u5r = !wave_any(uy1 - uy0 > 5);
        const int lane = (int) (__lane_id() & 15u);
        const int b2 = (lane >> 2) & 1, b3 = (lane >> 3) & 1, ch = lane & 3;
        float v[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] = act ? vals[c] : 0.f;
#if AMVPT_SPLAT_SEL
        /* v[ch ^ j] as two selects on lane-constant masks (a pick by a lane-varying index compiled to a
         * branch tree with exec-mask juggling) */
        const bool c0 = (lane & 1) != 0, c1 = (lane & 2) != 0;
        auto pick = [&](int j) {
            const bool s0 = c0 != ((j & 1) != 0), s1 = c1 != ((j & 2) != 0);
            const float lo = s0 ? v[1] : v[0], hi = s0 ? v[3] : v[2];
            return s1 ? hi : lo;
        };
        const float K = pick(0);
        const float B1 = dpp_f<DPP_XOR1>(pick(1)), B2 = dpp_f<DPP_XOR2>(pick(2)), B3 = dpp_f<DPP_XOR3>(pick(3));
#else
        auto pick = [&](int c) { return c == 0 ? v[0] : c == 1 ? v[1] : c == 2 ? v[2] : v[3]; };
        /* K: this lane's value of its channel; Bj: the value of this lane's channel at quad lane
         * (lane ^ j), which hands over its own v[ch ^ j] */
        const float K = pick(ch);
        const float B1 = dpp_f<DPP_XOR1>(pick(ch ^ 1)), B2 = dpp_f<DPP_XOR2>(pick(ch ^ 2)),
                    B3 = dpp_f<DPP_XOR3>(pick(ch ^ 3));
#endif
        /* inactive lanes hand over v = 0, so their (finite) weights need no masking: the weights are
         * straight-line code, not a branch per evaluation */
        const FilterCoeffs F = default_filter();
        float wx[6];
#if AMVPT_SPLAT_PKW
#pragma unroll
        for (int c = 0; c < 6; c += 2) {
            const f2v_t w = union_weight2(F, f.rx, f.x0, ux0 + c, ux0 + c + 1, x0c, x1);
            wx[c] = w.x;
            wx[c + 1] = w.y;
        }
        if (u5) wx[5] = 0.f;
#else
#pragma unroll
        for (int c = 0; c < 5; ++c) wx[c] = union_weight(F, f.rx, f.x0, ux0 + c, x0c, x1);
        wx[5] = 0.f;
        if (!u5) wx[5] = union_weight(F, f.rx, f.x0, ux0 + 5, x0c, x1);
#endif
        WinT *const wch = wbase + ch * wn.plane;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            /* row position r + 3 h holds union row r + 3 (h ^ b2); the quad shares b2 */
            float Ky[2], B1y[2], B2y[2], B3y[2];
            /* union rows r and r + 3 (lane-uniform), row 5 skipped when every fast row of the wave fits 5 */
#if AMVPT_SPLAT_PKW
            const f2v_t wyAB = union_weight2(F, f.ry, f.y0, uy0 + r, uy0 + r + 3, y0c, y1);
            const float wyA = wyAB.x, wyB = (r < 2 || !u5r) ? wyAB.y : 0.f;
#else
            const float wyA = union_weight(F, f.ry, f.y0, uy0 + r, y0c, y1);
            float wyB = 0.f;
            if (r < 2 || !u5r) wyB = union_weight(F, f.ry, f.y0, uy0 + r + 3, y0c, y1);
#endif
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const float wy = (h ^ b2) ? wyB : wyA;
                Ky[h] = K * wy;
                B1y[h] = B1 * dpp_f<DPP_XOR1>(wy);
                B2y[h] = B2 * dpp_f<DPP_XOR2>(wy);
                B3y[h] = B3 * dpp_f<DPP_XOR3>(wy);
            }
            /* steps 1-2: the quad's sum of this lane's channel, sum_j v_j[ch] wy_j wx_j; step 3: plus
             * the rotate-4 partner's quad sum of the other row half */
            float z[6];
#if AMVPT_SPLAT_PK
            /* the two row halves as one packed pair (v_pk_mul_f32 / v_pk_fma_f32: per-element IEEE, the
             * same products and sums bit for bit) */
            typedef float f2v __attribute__((ext_vector_type(2)));
            const f2v Ky2 = {Ky[0], Ky[1]}, B1y2 = {B1y[0], B1y[1]}, B2y2 = {B2y[0], B2y[1]}, B3y2 = {B3y[0], B3y[1]};
            auto col = [&](int c) {
                f2v a = Ky2 * (f2v) wx[c];
                a = __builtin_elementwise_fma((f2v) dpp_f<DPP_XOR1>(wx[c]), B1y2, a);
                a = __builtin_elementwise_fma((f2v) dpp_f<DPP_XOR2>(wx[c]), B2y2, a);
                a = __builtin_elementwise_fma((f2v) dpp_f<DPP_XOR3>(wx[c]), B3y2, a);
                return a.x + dpp_f<DPP_ROR4>(a.y);
            };
#pragma unroll
            for (int c = 0; c < 5; ++c) z[c] = col(c);
            z[5] = 0.f;
            if (!u5) z[5] = col(5);
#else
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                float y[2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    float a = Ky[h] * wx[c];
                    a = fmaf(dpp_f<DPP_XOR1>(wx[c]), B1y[h], a);
                    a = fmaf(dpp_f<DPP_XOR2>(wx[c]), B2y[h], a);
                    y[h] = fmaf(dpp_f<DPP_XOR3>(wx[c]), B3y[h], a);
                }
                z[c] = y[0] + dpp_f<DPP_ROR4>(y[1]);
            }
#endif
            const int row = r + 3 * b2;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float keep = b3 ? z[c + 3] : z[c], send = b3 ? z[c] : z[c + 3];
                const float u = (AMVPT_ATTR_SKIP & 16) ? z[c] : keep + dpp_f<DPP_ROR8>(send);
                const int col = c + 3 * b3;
                if (ux0 + col < ux1 && uy0 + row < uy1 && !(AMVPT_ATTR_SKIP & 1))
                    win_add(wch + (uy0 + row - wn.by0) * wn.rs + (ux0 + col - wn.bx0), u);
            }
        }
    } else if (act) {
        float wx[kMaxFoot], wy[kMaxFoot];
        foot_weights(P, f, wx, wy);
        foot_add<C, true, kWin, false>(P, film, wbase, wn, f, wx, wy, vals, coalesce, fallback);
    }
}

/* the wave's window flush: one global float atomic per touched film float, re-zeroing the
 * window (wave-local, in LDS order after the wave's own adds).  A cell's row comes from a float
 * reciprocal with a one-step correction (e < 2^24), not an integer division.  (Batching four
 * cells per lane -- four LDS reads, one wait -- measured no faster and its live pointers pushed
 * the 5-wave register budget into scratch.) */
template <int C, bool kWin = true>
AD void wave_flush(const KParams &P, float *film, WinT *win, const Win &w) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int rowlen = w.ww * C;
    const int n_elems = rowlen * w.wh;
    const float inv_rowlen = 1.f / (float) max(rowlen, 1);
    /* the wave window's quilt cells inside the film window (uniform; always for the whole quilt) */
    const bool inside = in_window<kWin>(P, w.bx0, w.by0) && in_window<kWin>(P, w.bx0 + w.ww - 1, w.by0 + w.wh - 1);
    float *film0 = inside ? film_cell<kWin>(P, film, w.bx0, w.by0, 0) : film;
    const uint32_t film_row = (kWin ? P.fw : P.W) * (uint32_t) C;
    for (int e = (int) __lane_id(); e < n_elems; e += 64) {
        int cy = (int) ((float) e * inv_rowlen);
        cy -= (cy * rowlen > e) ? 1 : 0;
        cy += ((cy + 1) * rowlen <= e) ? 1 : 0;
        const int r = e - cy * rowlen, cx = r / C, k = r - cx * C;
        WinT *src = win + k * w.plane + cy * w.rs + cx;
        const WinT d = *src;
#if AMVPT_WIN_FIXED == 2
        if (__float_as_int(d) != 0) {
            *src = 0.f;
            const float v = d;
#elif AMVPT_WIN_FIXED
        if (d != 0) {
            *src = 0;
            const float v = from_fixed(d);
#else
        if (__double_as_longlong(d) != 0ll) {
            *src = 0.0;
            const float v = (float) d;
#endif
            if ((v != 0.f || v != v) && !(AMVPT_ATTR_SKIP & 2)) {
                if (inside) atomicAdd(film0 + ((uint32_t) cy * film_row + (uint32_t) r), v);   /* never deterministic */
                else film_cell_add<kWin, false>(P, film, w.bx0 + cx, w.by0 + cy, k, v);
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

/* ImageBlock::put of a wave's samples through its own window (AMVPT_WAVE_WIN, row_splat) */
template <int C, bool kWin = true>
AD void wave_put(const KParams &P, float *film, WaveLds<C> &L, float px, float py, const float *vals, bool valid,
                 bool coalesce, uint32_t *fallback) {
    Foot f;
    f.ok = false;
    f.x0 = f.y0 = 0; f.nx = f.ny = 0; f.rx = f.ry = 0.f;
    if (valid) f = footprint(P, px, py, coalesce);
    const bool act = valid && f.ok;
    /* the rows' union boxes (row_put_win's), then the wave's box from the four row results */
    const RowBox ub = row_box(f, act);
    auto rmin = [](int v) {
        return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                   min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
    };
    auto rmax = [](int v) {
        return max(max(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
                   max(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
    };
    const int bx0 = rmin(ub.x0), by0 = rmin(ub.y0), bx1 = rmax(ub.x1), by1 = rmax(ub.y1);
    if (bx1 <= bx0) return;   /* no active footprint in the wave (uniform) */
    Win wn;
    wn.bx0 = bx0; wn.by0 = by0;
    wn.ww = min(bx1 - bx0, kWaveWinW);
    wn.wh = min(by1 - by0, kWaveWinH);
    wn.rs = wn.ww;
    wn.plane = wn.ww * wn.wh;
    /* row_put's bank spread (see window_bbox): rows 16 mod 32 apart, planes 4 mod 32 apart */
    {
        const int r2 = (wn.ww & ~31) + 16, r3 = r2 >= wn.ww ? r2 : r2 + 32;
        if (r3 * wn.wh + 32 <= kWavePlane) wn.rs = r3;
        wn.plane = wn.rs * wn.wh;
        wn.plane += (36 - (wn.plane & 31)) & 31;
        if (wn.plane > kWavePlane) { wn.rs = wn.ww; wn.plane = wn.ww * wn.wh; }
    }
    WinT *const win = L.win + (threadIdx.x >> 6) * (kWavePlane * C);
    /* row_put reads the window through L.win: hand it this wave's window */
    row_put_win<C, kWin>(P, film, win, wn, f, act, vals, coalesce, fallback, ub);
    wave_flush<C, kWin>(P, film, win, wn);
}

/*
 * Block-cooperative put into window buffer `buf`.  Cells xs in [0, nx) x ys in
 * [0, ny) of the footprint with x0 + xs >= 0 and y0 + ys >= 0 are accumulated (the
 * coalesced footprint may start left/above the film).  Weight of a cell =
 * eval(rx + xs) * eval(ry + ys).  `coalesce` is uniform over the block.
 */
template <int C>
AD void block_put(const KParams &P, float *film, SplatLds<C> &L, int buf, float px, float py, const float *vals,
                  bool valid, bool coalesce, uint32_t *fallback = nullptr) {
    Foot f;
    f.ok = false;
    f.x0 = f.y0 = 0; f.nx = f.ny = 0; f.rx = f.ry = 0.f;
    if (valid) f = footprint(P, px, py, coalesce);
    const bool act = valid && f.ok;
    const Win wn = window_bbox(L, buf, act, max(f.x0, 0), max(f.y0, 0), f.x0 + f.nx, f.y0 + f.ny, (int) P.win_rs,
                               P.row_splat != 0);
    if (C == 4 && P.row_splat) {
        row_put_win<C>(P, film, L.win, wn, f, act, vals, coalesce, fallback, row_box(f, act));
    } else if (act) {
        float wx[kMaxFoot], wy[kMaxFoot];
        foot_weights(P, f, wx, wy);
        foot_add<C>(P, film, L.win, wn, f, wx, wy, vals, coalesce, fallback);
    }
    window_flush<C>(P, film, L, wn);
}

/*
 * Record slots.  Per-lane records (lane_out, lane_rec, view_rec planes) are stored
 * at a SLOT, not at the lane index: lanes are grouped in super-blocks of
 * kSplatSuper = 1024 (= pixels_per_super * spp) and slot (h * 512 + t) of a
 * super-block holds lane (t % ppb) * spp + h * (spp / 2) + t / ppb.  The primary
 * and raygen kernels run one thread per slot (a wave = 64 pixels of one sample:
 * coherent camera rays) and the splat kernels read slot = blockIdx * 512 + tid
 * (fully coalesced), so that a splat wave holds 64 different pixels (no CAS
 * conflicts inside a wave) and the two 512-thread blocks of a super-block write
 * the same small film window.  Partial super-blocks and non power-of-two spp
 * use the identity map.  The map is a bijection on [0, chunk_n).
 */
constexpr int kSplatSplit = kSplatSuper / kSplatBlock;
constexpr uint32_t kSplatSuperLog = __builtin_ctz(kSplatSuper), kSplatSplitLog = __builtin_ctz(kSplatSplit);
static_assert((1 << kSplatSuperLog) == kSplatSuper && (1 << kSplatSplitLog) == kSplatSplit, "powers of two");
#ifndef AMVPT_UDIV_RCP
/* 1: the path fetch of the suffix kernels (path_seq: slot -> lane -> TEA seed) divides by its kernel-uniform runtime
 * divisors through host-computed f64 reciprocals (udiv_r<true>) -- the generic expansion computes each divisor's
 * reciprocal in VGPRs up front, and the fused suffix spilled three of them (a scratch reload and wait at every path
 * fetch).  Elsewhere (k_mv_primary's slot order, the splat) the plain division stays: there the f64 form cost more
 * than it saved (r06am: config-M k_mv_primary 39.7 -> 41.6 ms).  The path-fetch form measured neutral (r06an: M, mesh
 * and C5 within noise, the reloads hide behind the other waves), so 0: plain division everywhere */
#define AMVPT_UDIV_RCP 0
#endif
/* n / d for a kernel-uniform d > 0, exactly: the f64 product n * fl(1/d) lies within 2^-20 of n / d (n, d < 2^32),
 * so its truncation is the quotient or one off, and one step each way corrects it */
template <bool kRcp = true> AD uint32_t udiv_r(uint32_t n, uint32_t d, double rcp) {
    if (!(AMVPT_UDIV_RCP && kRcp)) return n / d;
    uint32_t q = (uint32_t) ((double) n * rcp);
    q -= ((uint64_t) q * d > (uint64_t) n) ? 1u : 0u;
    q += ((uint64_t) (q + 1u) * d <= (uint64_t) n) ? 1u : 0u;
    return q;
}
/* host side of udiv_r */
inline double host_rcp(uint32_t d) { return d ? 1.0 / (double) d : 0.0; }
/*
 * Tiled slot order (KParams::tile_w, 16 samples per pixel and pass): slot block b of 256 = the 4 x 4
 * pixel tile b of the chunk's rows (tile rows of tile_w / 4 tiles), a wave = one pixel row of the
 * tile (64 consecutive lanes), a DPP row = one pixel.  A splat block's footprints then cover ~8 x 8
 * cells instead of 20 x 5, so a block-wide window flushes fewer film cells per sample.
 */
template <bool kRcp = false> AD uint32_t tile_slot_lane(const KParams &P, uint32_t slot) {
    const uint32_t b = slot >> 8, t = slot & 255u, tpr = P.tile_w >> 2;
    const uint32_t trow = udiv_r<kRcp>(b, tpr, P.rcp_tpr), tcol = b - trow * tpr, pt = t >> 4;
    return ((trow * 4u + (pt >> 2)) * P.tile_w + tcol * 4u + (pt & 3u)) * 16u + (t & 15u);
}
AD uint32_t tile_lane_slot(const KParams &P, uint32_t lane) {
    const uint32_t pix = lane >> 4, y = pix / P.tile_w, x = pix - y * P.tile_w, tpr = P.tile_w >> 2;
    return (((y >> 2) * tpr + (x >> 2)) << 8) | ((((y & 3u) << 2) | (x & 3u)) << 4) | (lane & 15u);
}
template <bool kRcp = false> AD uint32_t slot_lane(const KParams &P, uint32_t slot) {
    if (P.tile_w) return tile_slot_lane<kRcp>(P, slot);
    if (P.row_splat) return slot;   /* pixel-major: a 16-lane row = 16 samples of one pixel (row_put) */
    const uint32_t super = slot / (uint32_t) kSplatSuper, within = slot % (uint32_t) kSplatSuper;
    const uint32_t base = super * kSplatSuper;
    const uint32_t remain = P.chunk_n > base ? P.chunk_n - base : 0;
    const uint32_t S = P.spp_pp;
    if (remain >= (uint32_t) kSplatSuper && P.pow2 && S >= (uint32_t) kSplatSplit && S <= (uint32_t) kSplatBlock) {
        const uint32_t h = within / (uint32_t) kSplatBlock, t = within % (uint32_t) kSplatBlock;
        const uint32_t ppb = (uint32_t) kSplatSuper >> P.log_spp;   /* a power of two: mask and shift, not a division */
        return base + (t & (ppb - 1u)) * S + h * (S / kSplatSplit) + (t >> (kSplatSuperLog - P.log_spp));
    }
    return slot;
}
/* inverse of slot_lane */
AD uint32_t lane_slot(const KParams &P, uint32_t lane) {
    if (P.tile_w) return tile_lane_slot(P, lane);
    if (P.row_splat) return lane;
    const uint32_t super = lane / (uint32_t) kSplatSuper, off = lane % (uint32_t) kSplatSuper;
    const uint32_t base = super * kSplatSuper;
    const uint32_t remain = P.chunk_n > base ? P.chunk_n - base : 0;
    const uint32_t S = P.spp_pp;
    if (remain >= (uint32_t) kSplatSuper && P.pow2 && S >= (uint32_t) kSplatSplit && S <= (uint32_t) kSplatBlock) {
        const uint32_t half = S / kSplatSplit, ppb = (uint32_t) kSplatSuper >> P.log_spp;
        const uint32_t p = off >> P.log_spp, smp = off & (S - 1u);
        return base + (smp >> (P.log_spp - kSplatSplitLog)) * (uint32_t) kSplatBlock + (smp & (half - 1u)) * ppb + p;
    }
    return lane;
}

/* ImageBlock::put's sample check (imageblock.cpp:180-204: warn_invalid / warn_negative): an active
 * sample with a non-finite channel, or (finite) with a channel below -1e-5, is counted
 * (amvpt_counters.nonfinite_samples / negative_samples) -- the reference logs a warning. */
template <typename N> AD void check_sample(const KParams &P, const float *vals, bool active, N &nf, N &neg) {
    bool fin = true, nonneg = true;
    for (uint32_t k = 0; k < P.C; ++k) {
        fin = fin && finite_(vals[k]);
        nonneg = nonneg && vals[k] >= -1e-5f;
    }
    nf += (active && !fin) ? 1 : 0;
    neg += (active && fin && !nonneg) ? 1 : 0;
}

AD void pack_vals(const KParams &P, C3 v, float alpha, float weight, float *vals) {
    vals[0] = v.r; vals[1] = v.g; vals[2] = v.b;
    if (P.C == 4) { vals[3] = weight; vals[4] = 0.f; }
    else { vals[3] = alpha; vals[4] = weight; }
}

/* ------------------------------------------------------------------ */
/* Queue                                                              */
/* ------------------------------------------------------------------ */

/* Sum over the wave, result valid in every lane. */
AD unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (unsigned long long) __shfl_xor((long long) v, o);
    return v;
}
/* lane counters: stats[s * kStatShards + shard], one shard per block residue (summed on
 * the host), so the per-wave adds never pile onto one word */
/* [8]: paths pushed into the suffix, [9]: deterministic-film range drops, [10] / [11]: view-record bytes k_mv_primary
 * writes / the splat reads (the byte model's record terms, ABI 10) */
constexpr uint32_t kStatShards = 256, kStats = 12;
static_assert(kStatShards == 256, "film_add shards its range-drop count by blockIdx % 256");
AD void stat_add(unsigned long long *stats, uint32_t which, unsigned long long v) {
    v = wave_sum(v);
    if (__lane_id() == 0 && v) atomicAdd(stats + which * kStatShards + blockIdx.x % kStatShards, v);
}

/*
 * Partitioned queues.  A returning device-scope atomic on ONE word saturates at
 * about 88 per microsecond on MI355X (MI355X_MICROARCH.md, "dequeue"), far below
 * the tens of millions of wave-level pushes a frame makes, so every queue (path
 * queues, NEE queue) is split into kQParts partitions with one counter each, on
 * its own 64-B line.  Block b of a producer appends to partition b % kQParts; block
 * b of a consumer grid (a multiple of kQParts blocks) reads partition b % kQParts,
 * striding over it with the gridDim / kQParts blocks of that partition, and writes
 * its survivors to the same partition of the next queue, so a partition never
 * outgrows its initial fill (<= qcap entries, see render_impl).
 */
constexpr uint32_t kQParts = 256, kCntStride = 16;

/* Wave-aggregated slot allocation: one atomic per wave (ballot + mbcnt). */
AD uint32_t queue_slot(bool want, uint32_t *counter) {
    uint64_t mask = __ballot(want);
    uint32_t lane = __lane_id();
    uint32_t cnt = (uint32_t) __popcll(mask);
    uint32_t leader = mask ? (uint32_t) (__ffsll((unsigned long long) mask) - 1) : 0u;
    uint32_t base = 0;
    if (cnt && lane == leader) base = atomicAdd(counter, cnt);
    base = (uint32_t) __shfl((int) base, (int) leader);
    uint32_t rank = (uint32_t) __popcll(mask & ((1ull << lane) - 1ull));
    return base + rank;
}
/* global index of a new entry in this block's partition */
AD uint32_t push_slot(bool want, uint32_t *counters, uint32_t qcap) {
    const uint32_t p = blockIdx.x % kQParts;
    return p * qcap + queue_slot(want, counters + p * kCntStride);
}

struct PathState {
    Ray ray;
    C3 thr, res;
    bool eta_zero;        /* the eta product is 0 (else 1: every supported BSDF samples eta 1, or 0 when empty) */
    float prev_pdf;
    uint32_t depth;
    bool prev_delta, valid_ray;
    f3 prev_p;
    uint32_t idx;         /* chunk-local slot of the lane (lane_out, slot_lane) */
    uint64_t rng_state;
    uint32_t rng_seq;     /* v1 of TEA -> inc = 2*v1+1 (not stored: path_seq re-derives it) */
};

/*
 * Path state in the queues: 5 float4 planes, 80 B per live path --
 *   q0 (o.xyz, d.x)  q1 (d.yz, thr.rg)  q2 (thr.b, prev_pdf, bits, rng lo)  q3 (prev_p, idx)
 *   q4 (result, rng hi)
 * bits = depth (29 bits) | eta == 0 (bit 29) | prev_delta (30) | valid_ray (31).  eta is a
 * product of BSDF-sample etas, which are 1 for every supported BSDF (diffuse, roughconductor,
 * twosided) and 0 for an empty sample (bs_zero, e.g. a twosided BSDF at wi.z == 0), so one bit
 * holds it exactly.  The PCG increment's seed v1 is re-derived from the slot (path_seq), not
 * stored.  k_shadow adds NEE into q4's xyz in place.
 */
/* the bin key of a ray (ray binning, k_bin_sort): direction octant (major) and the Morton code of the
 * origin's cell in a 2^kBinCellBits-per-axis grid over the scene box */
#ifndef AMVPT_BIN_CELL_BITS
#define AMVPT_BIN_CELL_BITS 2   /* origin cells per axis of the bin key: 2^bits; 3 (4096 keys): walks 3 ms faster, sort 16 ms slower (r05d) */
#endif
constexpr uint32_t kBinCellBits = AMVPT_BIN_CELL_BITS, kBins = 8u << (3 * kBinCellBits), kBinBlock = 1024;
#ifndef AMVPT_BIN_UNROLL
#define AMVPT_BIN_UNROLL 4   /* entries per thread in flight in k_bin_sort's passes (one 1024-thread block per partition) */
#endif
constexpr uint32_t kBinUnroll = AMVPT_BIN_UNROLL;
#ifndef AMVPT_BIN_PREFETCH
/* 1: k_bin_sort's staged scatter loads the next batch during this one's run writes.  Neutral (r06af: k_bin 50.4 ms
 * either way on one box), so 0.  The same change holds the entries in named structs instead of arrays indexed by an
 * unrolled loop, which the compiler had promoted to 32 KB of LDS (each load then waited for its LDS copy): k_bin
 * 57.8 -> 56.9 ms per mesh frame on one box (r06ah; k_bin differs by up to 7 ms between boxes) */
#define AMVPT_BIN_PREFETCH 0
#endif
#ifndef AMVPT_BIN_STAGE
#define AMVPT_BIN_STAGE 1   /* k_bin_sort stages each batch in LDS and writes runs of one bin: sort 54.0 -> 50.3 ms,
                                     * mesh 857 -> 876 Msamples/s (r05h); 0: one scattered write per entry (A/B) */
#endif
AD uint32_t bin_key(const KParams &P, f3 o, f3 d) {
    const uint32_t oct = (fbits(d.x) >> 31) | ((fbits(d.y) >> 31) << 1) | ((fbits(d.z) >> 31) << 2);
    auto cell = [&](float v, int a) {
        const float f = (v - P.bin_lo[a]) * P.bin_scale[a];
        return (uint32_t) min(max((int) f, 0), (int) (1u << kBinCellBits) - 1);
    };
    const uint32_t cx = cell(o.x, 0), cy = cell(o.y, 1), cz = cell(o.z, 2);
    uint32_t m = 0;
#pragma unroll
    for (uint32_t b = 0; b < kBinCellBits; ++b)
        m |= (((cx >> b) & 1u) << (3 * b)) | (((cy >> b) & 1u) << (3 * b + 1)) | (((cz >> b) & 1u) << (3 * b + 2));
    return (oct << (3 * kBinCellBits)) | m;
}
AD void store_state(float4 *const *q, uint32_t slot, const PathState &s) {
    const uint32_t bits = (s.depth & 0x1fffffffu) | (s.eta_zero ? 0x20000000u : 0u) |
                          (s.prev_delta ? 0x40000000u : 0u) | (s.valid_ray ? 0x80000000u : 0u);
    q[0][slot] = make_float4(s.ray.o.x, s.ray.o.y, s.ray.o.z, s.ray.d.x);
    q[1][slot] = make_float4(s.ray.d.y, s.ray.d.z, s.thr.r, s.thr.g);
    q[2][slot] = make_float4(s.thr.b, s.prev_pdf, bitsf(bits), bitsf((uint32_t) s.rng_state));
    q[3][slot] = make_float4(s.prev_p.x, s.prev_p.y, s.prev_p.z, bitsf(s.idx));
    q[4][slot] = make_float4(s.res.r, s.res.g, s.res.b, bitsf((uint32_t) (s.rng_state >> 32)));
}

/* k_bounce's push into the output queue; with ray binning on, also the continuation ray's bin key (k_bin_sort's
 * histogram pass then reads 2 B per entry instead of the 32-B ray).  The primary stage's pushes carry no key
 * (the key code would sit in every primary kernel: k_mv_primary 38.9 -> 41.2 ms at config M, r05f), so the
 * first depth's k_bin_sort forms its keys from the rays */
AD void push_state(const KParams &P, const Bufs &B, uint32_t slot, const PathState &s) {
    store_state(B.q_out, slot, s);
    if (B.key_out) B.key_out[slot] = (uint16_t) bin_key(P, s.ray.o, s.ray.d);
}
AD PathState load_state(float4 *const *q, uint32_t slot) {
    PathState s;
    float4 a = q[0][slot], b = q[1][slot], c = q[2][slot], d = q[3][slot], e = q[4][slot];
    s.ray.o = mk(a.x, a.y, a.z);
    s.ray.d = mk(a.w, b.x, b.y);
    s.ray.maxt = kLargest;
    s.thr = C3{b.z, b.w, c.x};
    s.prev_pdf = c.y;
    const uint32_t bits = fbits(c.z);
    s.depth = bits & 0x1fffffffu;
    s.eta_zero = (bits & 0x20000000u) != 0;
    s.prev_delta = (bits & 0x40000000u) != 0;
    s.valid_ray = (bits & 0x80000000u) != 0;
    s.prev_p = mk(d.x, d.y, d.z);
    s.idx = fbits(d.w);
    s.res = C3{e.x, e.y, e.z};
    s.rng_state = (uint64_t) fbits(c.w) | ((uint64_t) fbits(e.w) << 32);
    s.rng_seq = 0;
    return s;
}

/* ------------------------------------------------------------------ */
/* k_raygen_single: render_sample prologue (mvpath_single.h:50-76)     */
/* ------------------------------------------------------------------ */

/* global lane (mvpath.cpp:173-190 wavefront index) of virtual index v of the render's lane set:
 * a contiguous range, or rect_h runs of run_len lanes (one per pixel row of the rectangle) */
template <bool kRcp = false> AD uint32_t lane_of(const KParams &P, uint64_t v) {
    if (!P.rect) return (uint32_t) (P.range_begin + v);
    const uint32_t vv = (uint32_t) v, r = udiv_r<kRcp>(vv, P.run_len, P.rcp_run_len), o = vv - r * P.run_len;
    return ((P.rect_y0 + r) * P.W + P.rect_x0) * P.spp_pp + o;
}
/* the adaptive fill (mvpath_multi.h:79-115: dr::compress, dr::repeat): index in the PASS's
 * repeated wavefront of entry j of this render's part -- entry e = j / n_adapt of the render's
 * compressed list sits at e + run_delta[run of its lane] of the pass's compressed array */
template <bool kRcp = false> AD uint32_t adapt_index(const KParams &P, const Bufs &B, uint32_t j) {
    const uint32_t e = udiv_r<kRcp>(j, P.n_adapt, P.rcp_n_adapt), rep = j - e * P.n_adapt;
    const uint32_t run = P.rect ? udiv_r<kRcp>(B.asel[e], P.run_len, P.rcp_run_len) : 0u;
    return (e + B.run_delta[run]) * P.n_adapt + rep;
}

/* TEA's v1 of the lane whose path sits in chunk slot `slot` (PCG increment 2 v1 + 1): the main
 * pass seeds lane chunk_begin + slot_lane(slot) with seed_value (k_raygen_single, primary_raygen),
 * the adaptive pass wavefront entry chunk_begin + slot with adapt_seed (k_raygen_adapt) */
AD uint32_t path_seq(const KParams &P, const Bufs &B, uint32_t slot) {
    uint32_t v0, v1;
    if (P.adapt_pass) tea4(P.adapt_seed, adapt_index<true>(P, B, (uint32_t) (P.chunk_begin + slot)), v0, v1);
    else tea4(P.seed_value, lane_of<true>(P, P.chunk_begin + slot_lane<true>(P, slot)), v0, v1);
    return v1;
}

/* film pixel of a lane (mvpath.cpp:173-190: pixel of the crop + crop_offset) */
AD void lane_pixel(const KParams &P, uint32_t lane, int &px, int &py) {
    uint32_t pix = P.pow2 ? (lane >> P.log_spp) : (lane / P.spp_pp);
    uint32_t y = pix / P.W;
    py = (int) (y + P.off_y);
    px = (int) (pix - P.W * y + P.off_x);
}

AMVPT_TU_LOCAL __global__ void __launch_bounds__(256) k_raygen_single(KParams P, const DView *V, Bufs B) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = slot < P.chunk_n;
    PathState s;
    if (ok) {
        const uint32_t i = slot_lane(P, slot);
        const uint32_t lane = lane_of(P, P.chunk_begin + i);
        int px, py;
        lane_pixel(P, lane, px, py);
        Pcg rng = pass_rng(P, lane, P.chunk_begin + i);
        float jx = rng.next_1d(), jy = rng.next_1d();
        float sx = (float) px + jx, sy = (float) py + jy;
        float apx = .5f, apy = .5f;
        if (P.needs_ap) { apx = rng.next_1d(); apy = rng.next_1d(); }
        uint32_t index;
        s.ray = sample_ray_idx(P, V, fmadd(sx, P.inv_w, P.adj_ox), fmadd(sy, P.inv_h, P.adj_oy), index, apx, apy);
        s.thr = c3(1.f); s.res = c3(0.f);
        s.eta_zero = false; s.prev_pdf = 1.f; s.depth = 0; s.prev_delta = true; s.valid_ray = P.valid_ray0 != 0;
        s.prev_p = mk(0.f, 0.f, 0.f);
        s.idx = slot;
        s.rng_state = rng.state;
        s.rng_seq = (uint32_t) (rng.inc >> 1);
        if (P.max_depth == 0) {
            B.lane_out[slot] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (P.rng_out) P.rng_out[P.chunk_begin + i] = rng.state;   /* path.cpp: no draw past the camera's */
            ok = false;
        }
    }
    uint32_t qslot = push_slot(ok, B.cnt_out, B.qcap);
    if (ok) store_state(B.q_out, qslot, s);
    if (B.stats) stat_add(B.stats, 8, ok ? 1ull : 0ull);
}

/* ------------------------------------------------------------------ */
/* Adaptive fill (mvpath_multi.h:79-115): lanes whose primary vertex had at most one
 * indirect-valid view (adapt_mask) are compacted in lane order, each repeated n_adapt
 * times (dr::compress + dr::repeat), re-traced from the same jittered position with
 * sample_single using a forked sampler seeded (wavefront, wavefront), and splatted
 * (non-coalesced) with value adapt_w * L and weight adapt_w.                        */
/* ------------------------------------------------------------------ */

/* jittered sample position of a primary lane of the pass (its first two draws) */
AD void lane_sample_pos(const KParams &P, uint32_t lane, float &sx, float &sy, float &apx, float &apy) {
    int px, py;
    lane_pixel(P, lane, px, py);
    Pcg rng = lane_rng(P.pass_seed, lane);
    const float jx = rng.next_1d(), jy = rng.next_1d();
    sx = (float) px + jx;
    sy = (float) py + jy;
    apx = apy = .5f;
    if (P.needs_ap) { apx = rng.next_1d(); apy = rng.next_1d(); }   /* nested_gather(aperture_sample) */
}

AMVPT_TU_LOCAL __global__ void __launch_bounds__(256) k_raygen_adapt(KParams P, const DView *V, Bufs B) {
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = slot < P.chunk_n;
    PathState s;
    if (ok) {
        const uint32_t j = (uint32_t) (P.chunk_begin + slot);      /* index in this render's part of the fill */
        const uint32_t lane = lane_of(P, B.asel[j / P.n_adapt]);
        float sx, sy, apx, apy;
        lane_sample_pos(P, lane, sx, sy, apx, apy);
        uint32_t v0, v1;
        tea4(P.adapt_seed, adapt_index(P, B, j), v0, v1);
        Pcg rng;
        rng.seed(v0, v1);
        uint32_t index;
        s.ray = sample_ray_idx(P, V, fmadd(sx, P.inv_w, P.adj_ox), fmadd(sy, P.inv_h, P.adj_oy), index, apx, apy);
        s.thr = c3(1.f); s.res = c3(0.f);
        s.eta_zero = false; s.prev_pdf = 1.f; s.depth = 0; s.prev_delta = true; s.valid_ray = P.valid_ray0 != 0;
        s.prev_p = mk(0.f, 0.f, 0.f);
        s.idx = slot;
        s.rng_state = rng.state;
        s.rng_seq = v1;
        if (P.max_depth == 0) {
            B.lane_out[slot] = make_float4(0.f, 0.f, 0.f, 0.f);
            ok = false;
        }
    }
    uint32_t qslot = push_slot(ok, B.cnt_out, B.qcap);
    if (ok) store_state(B.q_out, qslot, s);
    if (B.stats) stat_add(B.stats, 8, ok ? 1ull : 0ull);
}

/* ------------------------------------------------------------------ */
/* k_bounce: one loop iteration (mvpath_multi.h:563-686 == mvpath_single.h:130-275) */
/* ------------------------------------------------------------------ */

/*
 * The suffix loop body (mvpath_multi.h:563-686 == mvpath_single.h:130-275) runs as
 * three wavefronts per depth, so that no kernel holds both a BVH walk and the
 * shading state (each walk runs at high occupancy to hide its node-load latency):
 *   k_extend   closest hit of every live path's ray        (Scene::ray_intersect)
 *   k_bounce   emitter-hit MIS, emitter sample, BSDF eval/sample, Russian roulette,
 *              compaction of the survivors; the emitter sample's shadow ray goes to
 *              the NEE queue with the pre-bounce throughput and its contribution
 *   k_shadow   the NEE ray_test (Scene::sample_emitter_direction's test); if the
 *              light is visible, result = fma(throughput, contribution, result)
 *              in the path's next state (or its final lane record)
 * The accumulation order of a lane's result is the reference's: emitter hit of
 * vertex d, then NEE of vertex d, then vertex d + 1.
 */
/* waves per SIMD the suffix walks' register allocation must allow (latency-bound dependent node loads):
 * k_extend at 6 (80 VGPRs) took the mesh frame 599 -> 609 Msamples/s; 8 (64 VGPRs, 48 B of spills)
 * 606; k_shadow keeps its own allocation (r03k) */
#ifndef AMVPT_EXTEND_WAVES
#define AMVPT_EXTEND_WAVES 6
#endif
#ifndef AMVPT_TREELETS
/* walks of large BVHs that start in an LDS treelet: bit 0 k_shadow (per-lane any hit), bit 1 k_extend (per-lane
 * closest hit, octant treelets), bit 2 k_vis (wave-uniform any hit).  Off: measured slower on the mesh bench
 * (r04c, one-stream kernel ms: k_extend 266 -> 320, k_shadow 191 -> 254, k_vis 80 -> 110; 717 -> 634 / 607
 * Msamples/s) -- the top levels they stage are the nodes every walk already finds in L1 / the scalar cache,
 * and a wave whose lanes are split between treelet and global nodes waits for both loads per step. */
#define AMVPT_TREELETS 0
#endif
#ifndef AMVPT_EXTEND_RAYS
/* per-lane k_extend walks: paths per thread (2: trace_closest_lane2, A/B).  1: the two-path walk measured slower
 * on the mesh bench (k_extend 229.4 -> 254.9 ms at 5 waves/SIMD, r04z_ab_mesh.log) */
#define AMVPT_EXTEND_RAYS 1
#endif
#ifndef AMVPT_EXTEND2_WAVES
#define AMVPT_EXTEND2_WAVES 5   /* the two-path walk: 89 VGPRs, no scratch (at 6: 80 VGPRs and spills inside the walk) */
#endif
#ifndef AMVPT_SHADOW_RAYS
/* per-lane k_shadow walks: records per thread (2: trace_any_lane2, A/B).  1: k_shadow 172.8 -> 182.7 ms with two
 * (r04z_ab_mesh.log) */
#define AMVPT_SHADOW_RAYS 1
#endif
#ifndef AMVPT_SHADOW_WAVES
#define AMVPT_SHADOW_WAVES 1
#endif
/*
 * Ray binning for the per-lane suffix walks of large BVHs (coherence, not more per-lane tricks).
 * The suffix rays of a queue partition arrive in whatever order the producer blocks pushed them: neighbouring
 * lanes of a wave start anywhere and point anywhere, so a wave's walk runs as long as its longest lane and
 * its node loads spread over the whole tree.  Embree restores coherence with ray packets (rtcIntersect16,
 * scene_embree.inl:287-318); here k_bin_sort orders each partition by a key of direction octant (major) and
 * the Morton code of the origin's cell in an 8 x 8 x 8 grid over the scene box -- a counting sort in LDS,
 * one 1024-thread block per partition: an LDS histogram of the 4096 keys, a block scan, and a scatter whose
 * returning LDS atomics hand out the positions -- and writes the rays in that order (32 B each, with the
 * entry they came from).  k_extend / k_shadow then walk the binned rays: consecutive lanes share an octant
 * (the same node ordering) and start nearby, and write their hit / verdict back to the entry.  The result of
 * each ray does not depend on which lane walks it, so records stay bit-identical.  NEE rays are keyed the
 * same way (direction to the light sample).
 */
#ifndef AMVPT_BIN
#define AMVPT_BIN 3   /* bit 0: bin the extension rays (k_extend), bit 1: the NEE rays (k_shadow); 0: off (A/B) */
#endif
#ifndef AMVPT_NEE_CARRY
/* 1: a binned NEE record carries the visible result itself (red in the record's last word, green and blue in a
 * bin-order plane, sgb) instead of the entry it came from: k_shadow's visible write then reads it with the sorted
 * record (coalesced) instead of two scattered loads from the unsorted records (nee[1][entry].w, nee_gb[entry]) --
 * the mesh frame's k_shadow fetched 270 GB from HBM for ~50 GB of sorted records (r06y_traffic_mesh.json); 0: A/B */
#define AMVPT_NEE_CARRY 1
#endif
#ifndef AMVPT_BIN_UNI
#define AMVPT_BIN_UNI 0   /* 1: binned waves take the wave-uniform walk (scalar node loads) instead of the per-lane one */
#endif
template <bool kNee, bool kFromRays = false>
__global__ void __launch_bounds__(kBinBlock) k_bin_sort(KParams P, Bufs B) {
    /* NEE records carry their visible result (AMVPT_NEE_CARRY): k_shadow then reads it in bin order */
    constexpr bool nee_carry = kNee && AMVPT_NEE_CARRY;
    __shared__ uint32_t h[kBins];
    __shared__ uint32_t wsum[kBinBlock / 64];
    const uint32_t part = blockIdx.x;
    const uint32_t count = (kNee ? B.cnt_nee : B.cnt_in)[part * kCntStride], pbase = part * B.qcap;
    float4 *const *src = kNee ? B.nee : B.q_in;
    const uint16_t *const keys = kNee ? B.key_nee : B.key_in;
    for (uint32_t k = threadIdx.x; k < kBins; k += kBinBlock) h[k] = 0u;
    __syncthreads();
    /* the histogram of the producers' keys (2 B per entry), kBinUnroll loads in flight per thread */
    for (uint32_t e0 = threadIdx.x; e0 < count; e0 += kBinUnroll * kBinBlock) {
        uint32_t k[kBinUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kBinUnroll; ++u) {
            const uint32_t e = e0 + u * kBinBlock;
            if (kFromRays) {
                k[u] = kBins;
                if (e < count) {
                    const float4 a = src[0][pbase + e], b = src[1][pbase + e];
                    k[u] = bin_key(P, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y));
                }
            } else {
                k[u] = e < count ? keys[pbase + e] : kBins;
            }
        }
#pragma unroll
        for (uint32_t u = 0; u < kBinUnroll; ++u)
            if (k[u] < kBins) (void) atomicAdd(&h[k[u]], 1u);
    }
    __syncthreads();
    /* exclusive scan of the histogram: thread t owns bins [t * per, t * per + per) */
    constexpr uint32_t per = kBins >= kBinBlock ? kBins / kBinBlock : 1u;
    uint32_t v[per], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < per; ++k) {
        v[k] = threadIdx.x * per + k < kBins ? h[threadIdx.x * per + k] : 0u;
        sum += v[k];
    }
    const int lane = (int) __lane_id(), wave = (int) (threadIdx.x >> 6);
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (int w = 0; w < wave; ++w) run += wsum[w];
#pragma unroll
    for (uint32_t k = 0; k < per; ++k) {
        if (threadIdx.x * per + k < kBins) h[threadIdx.x * per + k] = run;
        run += v[k];
    }
    __syncthreads();
    /* the scatter, two entries per thread in flight: each ray (32 B) to its bin's next position */
    auto place = [&](uint32_t i, const float4 &a, const float4 &b, uint32_t key) {
        /* one 32-B record per ray (a whole memory sector per scattered write, not two 16-B halves in two planes) */
        const uint32_t j = pbase + atomicAdd(&h[key], 1u);
        B.sray[0][2 * (size_t) j] = a;
        B.sray[0][2 * (size_t) j + 1] = nee_carry ? b : kNee ? make_float4(b.x, b.y, b.z, bitsf(i)) : make_float4(b.x, b.y, bitsf(i), 0.f);
        if (nee_carry) B.sgb[j] = B.nee_gb[i];
    };
#if AMVPT_BIN_STAGE
    /* staged scatter: batches of kStage entries are counting-sorted in LDS first, so the global writes go out
     * as runs of consecutive records of one bin (consecutive threads, consecutive addresses) */
    constexpr uint32_t kStage = 2 * kBinBlock;
    __shared__ float4 stg[2 * kStage];
    __shared__ float2 sgb[kNee && AMVPT_NEE_CARRY ? kStage : 1];
    __shared__ uint16_t skey[kStage];
    __shared__ uint32_t lh[kBins], lbase[kBins];
    /* the batch's global loads (rays, producer keys, carried green / blue): with AMVPT_BIN_PREFETCH the next batch's
     * are issued before this batch's run writes, so their latency overlaps them (one block per CU leaves nothing
     * else to hide it).  Two entries per thread as named structs, not arrays: an array indexed by the unrolled
     * entry loop is promoted to LDS before the loop is unrolled, and the load then waits for its LDS copy. */
    struct Ent { float4 a, b; uint32_t k, r; float2 g; };
    auto load = [&](uint32_t e, Ent &x) {
        const uint32_t i = pbase + min(e, count - 1u);
        x.a = src[0][i]; x.b = src[1][i];
        if (!kFromRays) x.k = keys[i];
        if (nee_carry) x.g = B.nee_gb[i];
    };
    Ent x0, x1, n0, n1;
    x0.k = x1.k = n0.k = n1.k = 0u;
    x0.g = x1.g = n0.g = n1.g = make_float2(0.f, 0.f);
    if (AMVPT_BIN_PREFETCH && count > 0) { load(threadIdx.x, x0); load(threadIdx.x + kBinBlock, x1); }
    for (uint32_t b0 = 0; b0 < count; b0 += kStage) {
        const uint32_t n = min(kStage, count - b0);
        for (uint32_t q = threadIdx.x; q < kBins; q += kBinBlock) lh[q] = 0u;
        __syncthreads();
        if (!AMVPT_BIN_PREFETCH) { load(b0 + threadIdx.x, x0); load(b0 + threadIdx.x + kBinBlock, x1); }
        auto rank = [&](Ent &x, uint32_t e) {
            if (kFromRays) x.k = bin_key(P, mk(x.a.x, x.a.y, x.a.z), mk(x.a.w, x.b.x, x.b.y));
            x.r = e < count ? atomicAdd(&lh[x.k], 1u) : 0u;
        };
        rank(x0, b0 + threadIdx.x);
        rank(x1, b0 + threadIdx.x + kBinBlock);
        __syncthreads();
        /* the batch's run of each bin: its position in the batch (a scan of lh) and in the partition */
        for (uint32_t q = threadIdx.x; q < kBins; q += kBinBlock) {
            const uint32_t c = lh[q];
            lbase[q] = c ? atomicAdd(&h[q], c) : 0u;   /* the partition position of the run */
        }
        uint32_t vv[per], sm = 0;
#pragma unroll
        for (uint32_t q = 0; q < per; ++q) {
            vv[q] = threadIdx.x * per + q < kBins ? lh[threadIdx.x * per + q] : 0u;
            sm += vv[q];
        }
        uint32_t in2 = sm;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(in2, o);
            if (lane >= o) in2 += t;
        }
        __syncthreads();   /* (lh read above, wsum reused) */
        if (lane == 63) wsum[wave] = in2;
        __syncthreads();
        uint32_t run2 = in2 - sm;
        for (int w = 0; w < wave; ++w) run2 += wsum[w];
#pragma unroll
        for (uint32_t q = 0; q < per; ++q) {
            if (threadIdx.x * per + q < kBins) lh[threadIdx.x * per + q] = run2;   /* batch offset of bin q */
            run2 += vv[q];
        }
        __syncthreads();
        auto stage = [&](const Ent &x, uint32_t e) {
            if (e < count) {
                const uint32_t sp = lh[x.k] + x.r, i = pbase + e;
                stg[2 * sp] = x.a;
                stg[2 * sp + 1] = nee_carry ? x.b : kNee ? make_float4(x.b.x, x.b.y, x.b.z, bitsf(i)) : make_float4(x.b.x, x.b.y, bitsf(i), 0.f);
                if (nee_carry) sgb[sp] = x.g;
                skey[sp] = (uint16_t) x.k;
            }
        };
        stage(x0, b0 + threadIdx.x);
        stage(x1, b0 + threadIdx.x + kBinBlock);
        /* the next batch's loads (registers of their own, live across the run writes) */
        const bool more = AMVPT_BIN_PREFETCH && b0 + kStage < count;
        if (more) { load(b0 + kStage + threadIdx.x, n0); load(b0 + kStage + threadIdx.x + kBinBlock, n1); }
        __syncthreads();
        for (uint32_t sp = threadIdx.x; sp < n; sp += kBinBlock) {
            const uint32_t q = skey[sp], j = pbase + lbase[q] + (sp - lh[q]);
            B.sray[0][2 * (size_t) j] = stg[2 * sp];
            B.sray[0][2 * (size_t) j + 1] = stg[2 * sp + 1];
            if (nee_carry) B.sgb[j] = sgb[sp];
        }
        if (more) { x0 = n0; x1 = n1; }
        __syncthreads();
    }
#else
    for (uint32_t e0 = threadIdx.x; e0 < count; e0 += kBinUnroll * kBinBlock) {
        float4 a[kBinUnroll], b[kBinUnroll];
        uint32_t k[kBinUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kBinUnroll; ++u) {
            const uint32_t e = min(e0 + u * kBinBlock, count - 1u), i = pbase + e;
            a[u] = src[0][i]; b[u] = src[1][i];
            k[u] = kFromRays ? bin_key(P, mk(a[u].x, a[u].y, a[u].z), mk(a[u].w, b[u].x, b[u].y)) : keys[i];
        }
#pragma unroll
        for (uint32_t u = 0; u < kBinUnroll; ++u)
            if (e0 + u * kBinBlock < count) place(pbase + e0 + u * kBinBlock, a[u], b[u], k[u]);
    }
#endif
}

template <int kWalk, bool kBin = false>
__global__ void __launch_bounds__(256, (AMVPT_EXTEND_RAYS == 2 && (kWalk == WALK_LANE || kWalk == WALK_LANE_NS)) ? AMVPT_EXTEND2_WAVES
                                                                                                                  : AMVPT_EXTEND_WAVES)
k_extend(KParams P, const DScene *Sp, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<false, true, false, (AMVPT_TREELETS & 2) != 0>(S, lds, P.trav_mode, nullptr, 0, P.box_screen != 0);
    if (P.bvh2) sc.stk = reinterpret_cast<uint32_t *>(lds + P.stk_off_ext) + threadIdx.x;
    const uint32_t part = blockIdx.x % kQParts, pstride = gridDim.x / kQParts * blockDim.x;
    const uint32_t count = B.cnt_in[part * kCntStride], pbase = part * B.qcap;
    /* the counters k_bounce fills are zeroed here (the previous k_bounce / k_shadow are done) */
    if (blockIdx.x == 0) {
        for (uint32_t q = threadIdx.x; q < kQParts; q += blockDim.x) { B.cnt_out[q * kCntStride] = 0u; B.cnt_nee[q * kCntStride] = 0u; }
    }
    if constexpr (kBin) {
        /* the partition's rays in bin order (k_bin_sort); the hit goes back to the ray's entry */
        for (uint32_t e0 = blockIdx.x / kQParts * blockDim.x; e0 < count; e0 += pstride) {
            const uint32_t j = pbase + e0 + threadIdx.x;
            if (e0 + threadIdx.x < count) {
                const float4 a = B.sray[0][2 * (size_t) j], b = B.sray[0][2 * (size_t) j + 1];
                const Ray r{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), kLargest};
                const Hit h = AMVPT_BIN_UNI ? trace_closest<true, 0, kWalk != WALK_LANE_NS>(sc, r) : walk_closest<kWalk>(sc, r);
                B.hit[fbits(b.z)] = hit_rec(h);
            }
        }
        return;
    }
    if constexpr (AMVPT_EXTEND_RAYS == 2 && (kWalk == WALK_LANE || kWalk == WALK_LANE_NS)) {
        /* two paths per thread (trace_closest_lane2): entries e0 + t and e0 + t + blockDim.x */
        for (uint32_t e0 = blockIdx.x / kQParts * 2u * blockDim.x; e0 < count; e0 += 2u * pstride) {
            const uint32_t e_0 = e0 + threadIdx.x, e_1 = e_0 + blockDim.x;
            const bool act0 = e_0 < count, act1 = e_1 < count;
            Ray r0{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), kLargest}, r1 = r0;
            if (act0) { const float4 a = B.q_in[0][pbase + e_0], b = B.q_in[1][pbase + e_0]; r0 = Ray{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), kLargest}; }
            if (act1) { const float4 a = B.q_in[0][pbase + e_1], b = B.q_in[1][pbase + e_1]; r1 = Ray{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), kLargest}; }
            Hit h0, h1;
            trace_closest_lane2<kWalk == WALK_LANE_NS ? 0 : 1>(sc, r0, act0, r1, act1, h0, h1);
            if (act0) B.hit[pbase + e_0] = hit_rec(h0);
            if (act1) B.hit[pbase + e_1] = hit_rec(h1);
        }
        return;
    }
    for (uint32_t e0 = blockIdx.x / kQParts * blockDim.x; e0 < count; e0 += pstride) {
        const uint32_t i = pbase + e0 + threadIdx.x;
        if (e0 + threadIdx.x < count) {
            const float4 a = B.q_in[0][i], b = B.q_in[1][i];
            const Ray r{mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), kLargest};
            B.hit[i] = hit_rec(walk_closest<kWalk>(sc, r));
        }
    }
}

template <int kWalk, bool kBin = false>
__global__ void __launch_bounds__(256, AMVPT_SHADOW_WAVES) k_shadow(KParams P, const DScene *Sp, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<false, true, (AMVPT_TREELETS & 1) != 0>(S, lds, P.trav_mode, nullptr, 0, P.box_screen != 0);
    if (P.bvh2) sc.stk = reinterpret_cast<uint32_t *>(lds + P.stk_off_any) + threadIdx.x;
    const uint32_t part = blockIdx.x % kQParts, pstride = gridDim.x / kQParts * blockDim.x;
    const uint32_t count = B.cnt_nee[part * kCntStride], pbase = part * B.qcap;
    /* the visible-light write of a record (the path's result becomes fma(throughput, contribution, result),
     * formed by k_bounce; its .w -- valid_ray / rng hi -- stays) */
    auto visible = [&](uint32_t i, const float4 &a, const float4 &b) {
        const float2 gb = B.nee_gb[i];
        const uint32_t dest = fbits(a.w);
        float *const dp = (float *) ((dest & 0x80000000u) ? &B.lane_out[dest & 0x7fffffffu] : &B.q_out[4][dest]);
        dp[0] = b.w;
        dp[1] = gb.x;
        dp[2] = gb.y;
    };
    auto nee_ray = [&](const float4 &a, const float4 &b) {
        /* spawn_ray_to's direction and extent from its origin and target (same operations) */
        const f3 o = mk(a.x, a.y, a.z);
        f3 d = mk(b.x, b.y, b.z) - o;
        const float dist = norm(d);
        d = d / dist;
        return Ray{o, d, dist * (1.f - kShadowEps)};
    };
    if constexpr (kBin) {
        /* the partition's NEE rays in bin order (k_bin_sort): (origin, destination), (target, entry); a visible
         * light's result is read from the entry's record */
        for (uint32_t e0 = blockIdx.x / kQParts * blockDim.x; e0 < count; e0 += pstride) {
            const uint32_t j = pbase + e0 + threadIdx.x;
            if (e0 + threadIdx.x < count) {
                const float4 a = B.sray[0][2 * (size_t) j], b = B.sray[0][2 * (size_t) j + 1];
                const Ray r = nee_ray(a, b);
                const bool occ = AMVPT_BIN_UNI ? trace_any<true, 0, kWalk != WALK_LANE_NS>(sc, r) : walk_any<kWalk>(sc, r);
                if (!occ) {
                    if (AMVPT_NEE_CARRY) {
                        /* the record's own result: red in b.w, green and blue in sgb[j] */
                        const float2 gb = B.sgb[j];
                        const uint32_t dest = fbits(a.w);
                        float *const dp = (float *) ((dest & 0x80000000u) ? &B.lane_out[dest & 0x7fffffffu] : &B.q_out[4][dest]);
                        dp[0] = b.w;
                        dp[1] = gb.x;
                        dp[2] = gb.y;
                    } else {
                        const uint32_t i = fbits(b.w);
                        visible(i, a, make_float4(0.f, 0.f, 0.f, B.nee[1][i].w));
                    }
                }
            }
        }
        return;
    }
    if constexpr (AMVPT_SHADOW_RAYS == 2 && (kWalk == WALK_LANE || kWalk == WALK_LANE_NS)) {
        /* two records per thread (trace_any_lane2): entries e0 + t and e0 + t + blockDim.x */
        for (uint32_t e0 = blockIdx.x / kQParts * 2u * blockDim.x; e0 < count; e0 += 2u * pstride) {
            const uint32_t e_0 = e0 + threadIdx.x, e_1 = e_0 + blockDim.x;
            const bool act0 = e_0 < count, act1 = e_1 < count;
            float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), b0 = make_float4(0.f, 0.f, 1.f, 0.f), a1 = a0, b1 = b0;
            if (act0) { a0 = B.nee[0][pbase + e_0]; b0 = B.nee[1][pbase + e_0]; }
            if (act1) { a1 = B.nee[0][pbase + e_1]; b1 = B.nee[1][pbase + e_1]; }
            bool occ0, occ1;
            trace_any_lane2<kWalk == WALK_LANE_NS ? 0 : 1>(sc, nee_ray(a0, b0), act0, nee_ray(a1, b1), act1, occ0, occ1);
            if (act0 && !occ0) visible(pbase + e_0, a0, b0);
            if (act1 && !occ1) visible(pbase + e_1, a1, b1);
        }
        return;
    }
    for (uint32_t e0 = blockIdx.x / kQParts * blockDim.x; e0 < count; e0 += pstride) {
        const uint32_t i = pbase + e0 + threadIdx.x;
        if (e0 + threadIdx.x < count) {
            const float4 a = B.nee[0][i], b = B.nee[1][i];
            /* spawn_ray_to's direction and extent from its origin and target (same operations) */
            const f3 o = mk(a.x, a.y, a.z);
            f3 d = mk(b.x, b.y, b.z) - o;
            const float dist = norm(d);
            d = d / dist;
            const Ray r{o, d, dist * (1.f - kShadowEps)};
            if (!walk_any<kWalk>(sc, r)) visible(i, a, b);   /* the light is visible */
        }
    }
}

/* waves per SIMD k_bounce's register allocation must allow: 5 (<= 96 VGPRs, from 101 at 4) hides
 * more of the state loads and the fused NEE walk (109.7 vs 118.3 ms per config-M frame, A/B r02z) */
#ifndef AMVPT_BOUNCE_WAVES
#define AMVPT_BOUNCE_WAVES 5
#endif
/* bounce_vertex's state hooks when the whole path state stays in registers (k_bounce) */
struct NoPark {
    AD void in(PathState &, Pcg &) const {}
    AD void res_out(const PathState &) const {}
    AD void nee_out(C3 &, f3 &) const {}
    AD void nee_to_in(f3 &) const {}
    AD void out(const PathState &, const Pcg &) const {}
};

/*
 * One suffix vertex (mvpath_multi.h:563-686 == mvpath_single.h:130-275): emitter-hit MIS at the
 * ray's hit, emitter sample, BSDF eval/sample, Russian roulette.  s advances in place; returns
 * whether the path continues; nee = the emitter sample's shadow ray shr (to nee_to) leaves the path
 * with result res_nee if unoccluded.  Shared by k_bounce and k_suffix_fused.  pk moves the fields
 * the vertex does not touch between its phases out of registers (k_suffix_fused's LdsPark): in()
 * brings them in before the emitter-hit term, res_out() takes the result out once the NEE term is
 * formed, out() the rest at the end.
 */
template <bool kDiff, class Pk = NoPark>
AD bool bounce_vertex(const KParams &P, const DScene &S, const SceneRef &sc, PathState &s, Pcg &rng, const Hit &hit,
                      bool &nee, Ray &shr, f3 &nee_to, C3 &res_nee, const Pk &pk = Pk()) {
    SI si = compute_si(sc, s.ray, hit);
    int32_t em = si_emitter(sc, si);
    pk.in(s, rng);
    {
        DSamp ds = ds_zero();
        ds.p = si.p; ds.n = si.sh.n;
        f3 rel = si.p - s.prev_p;
        ds.dist = norm(rel);
        ds.d = si.valid() ? rel / ds.dist : -si.wi;
        ds.emitter = em;
        float em_pdf = pdf_emitter_direction(sc, s.prev_p, ds, !s.prev_delta);
        float mis_bsdf = mis_weight(s.prev_pdf, em_pdf);
        s.res = cfma(s.thr, emitter_eval(sc, em, si, s.prev_pdf > 0.f) * mis_bsdf, s.res);
    }
    bool active_next = (s.depth + 1 < P.max_depth) && si.valid();
    int32_t b = si.valid() ? S.shapes[si.shape].bsdf : -1;
    bool active_em = active_next && (bsdf_flags(S.bsdfs, b) & BF_Smooth);
    float e1 = rng.next_1d(), e2 = rng.next_1d();
    {
        DSamp ds;
        C3 em_w;
        sample_emitter_direction(sc, si, e1, e2, active_em, ds, em_w);
        active_em = active_em && ds.pdf != 0.f;   /* ds.pdf != 0 <=> the reference traces the ray */
        f3 wo = si.sh.to_local(ds.d);
        C3 bval;
        float bpdf;
        bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, si.wi, wo, true, bval, bpdf);
        /* the NEE term is settled before the BSDF sample (which does not read it), so the emitter
         * sample, the BSDF value and pdf die here instead of living across the sample and the
         * shadow walk: the caller keeps only the result the path has if the light is visible,
         * fma(throughput, contribution, result) -- the reference's accumulation, evaluated early
         * (s.res does not change again in this vertex) */
        if (active_em) {
            float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, bpdf);
            nee = true;
            res_nee = cfma(s.thr, bval * em_w * mis_em, s.res);
            nee_to = ds.p;
            pk.nee_out(res_nee, nee_to);
        }
    }
    pk.res_out(s);
    float s1 = rng.next_1d();
    float s2a = rng.next_1d(), s2b = rng.next_1d();
    (void) s1;
    BSample bs;
    C3 bw;
    bsdf_sample<kDiff>(S.bsdfs, b, CTX_ALL, si.wi, s2a, s2b, true, bs, bw);
    s.ray = spawn_ray(si.p, si.n, si.sh.to_world(bs.wo));
    if (nee) {
        pk.nee_to_in(nee_to);
        shr = spawn_ray_to(si.p, si.n, nee_to);
    }
    s.thr = s.thr * bw;
    s.eta_zero = s.eta_zero || bs.eta == 0.f;
    s.prev_p = si.p;
    s.prev_pdf = bs.pdf;
    s.prev_delta = (bs.type & BF_Delta) != 0;
    if (si.valid()) s.depth += 1;
    float tmax = cmax(s.thr);
    const float eta = s.eta_zero ? 0.f : 1.f;
    float rr_prob = vmin(tmax * sqr(eta), .95f);
    bool rractive = s.depth >= P.rr_depth;
    bool rr_continue = rng.next_1d() < rr_prob;
    s.valid_ray = s.valid_ray || (si.valid() && !(bs.type & BF_Null));
    if (rractive) s.thr = s.thr * rcp(rr_prob);
    pk.out(s, rng);
    return active_next && (!rractive || rr_continue) && (tmax != 0.f);
}

/*
 * kNee >= 0: the NEE shadow ray is traced inside k_bounce with walk kNee (the brute-force walks of
 * tiny scenes, which are ALU-bound and need no occupancy to hide node-load latency): no NEE
 * record goes through HBM, no k_shadow launch, and the visible light's contribution is added to
 * the path's result right after the vertex's emitter-hit term -- the order k_shadow keeps.
 * kNee < 0: NEE records for k_shadow.
 */
template <bool kTab, bool kDiff, int kNee>
__global__ void __launch_bounds__(256, AMVPT_BOUNCE_WAVES) k_bounce(KParams P, const DScene *Sp, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<kTab, false>(S, lds, P.trav_mode, nullptr, 0, P.box_screen != 0);
    const uint32_t part = blockIdx.x % kQParts, pstride = gridDim.x / kQParts * blockDim.x;
    const uint32_t count = B.cnt_in[part * kCntStride], pbase = part * B.qcap;
    unsigned long long verts = 0, shadows = 0;
    for (uint32_t e0 = blockIdx.x / kQParts * blockDim.x; e0 < count; e0 += pstride) {
        const uint32_t i = pbase + e0 + threadIdx.x;
        bool ok = e0 + threadIdx.x < count;
        PathState s;
        bool keep = false, nee = false;
        Ray shr;
        f3 nee_to;
        C3 res_nee;
        if (ok) {
            s = load_state(B.q_in, i);
            Pcg rng;
            rng.state = s.rng_state;
            rng.inc = (((uint64_t) path_seq(P, B, s.idx)) << 1) | 1u;
            ++verts;
            keep = bounce_vertex<kDiff>(P, S, sc, s, rng, hit_of(B.hit[i]), nee, shr, nee_to, res_nee);
            s.rng_state = rng.state;
            if (!keep && P.rng_out) P.rng_out[P.chunk_begin + slot_lane(P, s.idx)] = rng.state;
            if (kNee < 0 && !keep) B.lane_out[s.idx] = make_float4(s.res.r, s.res.g, s.res.b, s.valid_ray ? 1.f : 0.f);
        }
        shadows += nee ? 1 : 0;
        if constexpr (kNee >= 0) {
            /* every lane of the wave walks (wave-uniform brute force); lanes without a shadow ray
             * start as found */
            const bool occluded = brute_any<kNee == WALK_BRUTE>(sc, shr, !nee);
            if (nee && !occluded) s.res = res_nee;
            if (ok && !keep) B.lane_out[s.idx] = make_float4(s.res.r, s.res.g, s.res.b, s.valid_ray ? 1.f : 0.f);
        }
        const uint32_t slot = push_slot(keep, B.cnt_out, B.qcap);
        if (keep) push_state(P, B, slot, s);
        if constexpr (kNee >= 0) continue;
        const uint32_t ns = push_slot(nee, B.cnt_nee, B.qcap);
        if (nee) {
            const uint32_t dest = keep ? slot : (0x80000000u | s.idx);
            /* (origin, destination), (light point, visible result .r), visible result .gb: k_shadow
             * re-derives the direction and extent exactly as spawn_ray_to did */
            B.nee[0][ns] = make_float4(shr.o.x, shr.o.y, shr.o.z, bitsf(dest));
            B.nee[1][ns] = make_float4(nee_to.x, nee_to.y, nee_to.z, res_nee.r);
            B.nee_gb[ns] = make_float2(res_nee.g, res_nee.b);
            if (B.key_nee) B.key_nee[ns] = (uint16_t) bin_key(P, shr.o, nee_to - shr.o);
        }
    }
    if (B.stats) { stat_add(B.stats, 0, verts); stat_add(B.stats, 5, shadows); }
}

/*
 * k_suffix_fused: the whole shared suffix of the brute-force-walk scenes in ONE launch, paths
 * resident in registers.  Every wave iteration is one vertex for each of its lanes -- closest
 * hit (brute force), bounce_vertex, the NEE any-hit walk -- whatever depth each lane's path is
 * at; a lane whose path ended takes the partition's next queued path (the primary kernel's
 * output queue, one returning atomic per wave on the partition's work counter).  No per-depth
 * launches, no path state or hit through HBM (80 B in once per path, 16 B out): the walks are
 * wave-uniform brute force, ALU-bound, so they need no occupancy of their own.  Lane results
 * are the same operations in the same order as the k_extend / k_bounce wavefronts.
 * The work counters (cnt_out of the queue pair) are zeroed by the host before the launch.
 */
#ifndef AMVPT_BOX_LDS
#define AMVPT_BOX_LDS 1   /* k_suffix_fused stages the box triangles in LDS for box_walk's per-lane loads (0: L1/L2, A/B) */
#endif
#ifndef AMVPT_FUSE_BVH
/* 1: BVH scenes run k_suffix_fused too (per-lane / wave-uniform walks inside the fused loop).  Off:
 * on the 3.6 k-triangle mesh it measured 519 vs 608 Msamples/s for the wavefront suffix (r03m) --
 * the walks, latency-bound on dependent node loads, lose more at the fused kernel's register budget
 * (80 VGPRs + 144 B of spills) than the fused loop saves in state traffic and launches */
#define AMVPT_FUSE_BVH 0
#endif
#ifndef AMVPT_FUSED_BLOCKS
/* blocks per queue partition (x kQParts blocks of 256 threads), more than are resident at once:
 * blocks that start late find their partition partly drained, which evens out the tail
 * (config M, 2^23-lane chunks, suffix ms: 5 -> 163.7, 8 -> 149.0, 16 -> 144.8, 24..64 -> 144.8,
 * r02fb; 2^25-lane chunks: 12 -> 135.2, 16 -> 133.5, 24 -> 132.4, 32 -> 132.7, r02fm) */
#define AMVPT_FUSED_BLOCKS 24
#endif
#ifndef AMVPT_FUSED_WAVES
/* 6 waves/SIMD (80 VGPRs, 68 B of spills): suffix 146.4 -> 143.2 ms per config-M frame; 4 waves 157.8 (r02fc);
 * 5 waves (no spills) 1480 vs 1510 Msamples/s at 6 (r03m) */
#define AMVPT_FUSED_WAVES 6
#endif
#ifndef AMVPT_FUSED_PARK
/* path-state groups k_suffix_fused keeps in LDS between the phases that use them (LdsPark) */
#define AMVPT_FUSED_PARK 0x2f
#endif
enum : int { PK_RES = 1, PK_PREV = 2, PK_THR = 4, PK_RNG = 8, PK_RAY = 16, PK_NEE = 32 };
/* LDS slots (floats) of a parked path: field f of block thread t at base[f * 256 + t] */
enum : int { PF_RES = 0, PF_IDX = 3, PF_PREVP = 4, PF_PREVPDF = 7, PF_THR = 8, PF_DEPTH = 11, PF_RNG = 12, PF_RESNEE = 16,
             PF_NEETO = 19, PF_RAY = 22 };
/* slots in use: the ray's only with PK_RAY */
constexpr int park_fields(int m) { return (m & PK_RAY) ? 28 : (m & PK_NEE) ? 22 : 16; }
constexpr uint32_t kFusedBlock = 256;
/*
 * The fused suffix's path state between phases, one LDS slot per field and lane (field-major, so a
 * wave's 64 accesses of one field hit 64 distinct banks).  A vertex needs its previous point and pdf
 * only for the emitter-hit term, its result only there and for the NEE term, its lane slot only when
 * the path ends, its throughput, depth and sampler state only inside bounce_vertex, and its ray only
 * for the closest-hit walk: kept in registers across the walks and the BSDF sample, they made the
 * 6-wave allocation spill to scratch (config M 60 B, the glossy C3 instance 120 B per lane, 1.8x /
 * 5.6x the kernel's algorithmic HBM bytes, round 3).  Volatile accesses: the compiler must not keep a
 * register copy of a value it stored (store-to-load forwarding would make the register live again).
 */
typedef __attribute__((address_space(3))) float lds_float;
template <int kMask> struct LdsPark {
    lds_float *b;   /* an LDS-space pointer: a generic one becomes 64-bit flat accesses */
    AD void put(int f, float v) const { *(volatile lds_float *) (b + f * (int) kFusedBlock) = v; }
    AD float get(int f) const { return *(volatile lds_float *) (b + f * (int) kFusedBlock); }
    AD void put3(int f, f3 v) const { put(f, v.x); put(f + 1, v.y); put(f + 2, v.z); }
    AD f3 get3(int f) const { return mk(get(f), get(f + 1), get(f + 2)); }
    AD void putc(int f, C3 v) const { put(f, v.r); put(f + 1, v.g); put(f + 2, v.b); }
    AD C3 getc(int f) const { return C3{get(f), get(f + 1), get(f + 2)}; }
    AD void put_u64(int f, uint64_t v) const { put(f, bitsf((uint32_t) v)); put(f + 1, bitsf((uint32_t) (v >> 32))); }
    AD uint64_t get_u64(int f) const { return (uint64_t) fbits(get(f)) | ((uint64_t) fbits(get(f + 1)) << 32); }
    /* a path fetched from the queue: everything parked goes to LDS */
    AD void fetch(const PathState &s, const Pcg &rng) const {
        if (kMask & PK_RES) { putc(PF_RES, s.res); put(PF_IDX, bitsf(s.idx)); }
        if (kMask & PK_PREV) { put3(PF_PREVP, s.prev_p); put(PF_PREVPDF, s.prev_pdf); }
        if (kMask & PK_THR) { putc(PF_THR, s.thr); put(PF_DEPTH, bitsf(s.depth)); }
        if (kMask & PK_RNG) { put_u64(PF_RNG, rng.state); put_u64(PF_RNG + 2, rng.inc); }
    }
    AD void in(PathState &s, Pcg &rng) const {
        if (kMask & PK_PREV) { s.prev_p = get3(PF_PREVP); s.prev_pdf = get(PF_PREVPDF); }
        if (kMask & PK_THR) { s.thr = getc(PF_THR); s.depth = fbits(get(PF_DEPTH)); }
        if (kMask & PK_RES) s.res = getc(PF_RES);
        if (kMask & PK_RNG) { rng.state = get_u64(PF_RNG); rng.inc = get_u64(PF_RNG + 2); }
    }
    AD void res_out(const PathState &s) const { if (kMask & PK_RES) putc(PF_RES, s.res); }
    /* the NEE term waits in LDS during the BSDF sample (its result until the shadow walk's verdict) */
    AD void nee_out(C3 &res_nee, f3 &nee_to) const {
        if (kMask & PK_NEE) { putc(PF_RESNEE, res_nee); put3(PF_NEETO, nee_to); }
    }
    AD void nee_to_in(f3 &nee_to) const { if (kMask & PK_NEE) nee_to = get3(PF_NEETO); }
    AD C3 res_nee(C3 r) const { return (kMask & PK_NEE) ? getc(PF_RESNEE) : r; }
    AD void out(const PathState &s, const Pcg &rng) const {
        if (kMask & PK_PREV) { put3(PF_PREVP, s.prev_p); put(PF_PREVPDF, s.prev_pdf); }
        if (kMask & PK_THR) { putc(PF_THR, s.thr); put(PF_DEPTH, bitsf(s.depth)); }
        if (kMask & PK_RNG) { put_u64(PF_RNG, rng.state); put_u64(PF_RNG + 2, rng.inc); }
    }
    /* the result after the NEE walk, and the lane slot, when the path ends */
    AD C3 res(const PathState &s) const { return (kMask & PK_RES) ? getc(PF_RES) : s.res; }
    AD void set_res(PathState &s, C3 v) const { if (kMask & PK_RES) putc(PF_RES, v); else s.res = v; }
    AD uint32_t idx(const PathState &s) const { return (kMask & PK_RES) ? fbits(get(PF_IDX)) : s.idx; }
    AD uint64_t rng_state(const Pcg &rng) const { return (kMask & PK_RNG) ? get_u64(PF_RNG) : rng.state; }
};
template <int kMask> constexpr uint32_t park_lds_bytes() { return kMask ? park_fields(kMask) * 4u * kFusedBlock : 0u; }
constexpr uint32_t kFusedParkBytes = park_lds_bytes<AMVPT_FUSED_PARK>();

#ifndef AMVPT_FUSED_WAVES_GLOSSY
/* the instance with microfacet BSDFs (kDiff = false): its own register budget.  5 waves/SIMD (96 VGPRs, no
 * scratch) and 6 (80 VGPRs, 44 B of scratch) run the C3 suffix in the same time (305.1 vs 303.9 ms, r04b);
 * at 6 its PMC bytes are 1.54x the algorithmic ones (r04d_traffic_C3.json), so 5 */
#define AMVPT_FUSED_WAVES_GLOSSY 5
#endif
template <bool kTab, bool kDiff, int kW>
__global__ void __launch_bounds__(kFusedBlock, kDiff ? AMVPT_FUSED_WAVES : AMVPT_FUSED_WAVES_GLOSSY)
    k_suffix_fused(KParams P, const DScene *Sp, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int kPk = AMVPT_FUSED_PARK;
    /* the parked state sits in front of the staged tables (dynamic LDS: [park][tables]) */
    const LdsPark<kPk> pk{(lds_float *) (uint32_t) (uintptr_t) lds + threadIdx.x};
    DScene S = *Sp;
    SceneRef sc = stage_scene<kTab, false>(S, lds + kFusedParkBytes, P.trav_mode, nullptr, 0, P.box_screen != 0,
                                           AMVPT_BOX_LDS != 0);
    const uint32_t part = blockIdx.x % kQParts;
    const uint32_t count = B.cnt_in[part * kCntStride], pbase = part * B.qcap;
    uint32_t *const work = B.cnt_out + part * kCntStride;
    uint64_t verts = 0, shadows = 0;
    PathState s;
    s.ray = Ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), kLargest};
    if (kPk & PK_RAY) { pk.put3(PF_RAY, s.ray.o); pk.put3(PF_RAY + 3, s.ray.d); }
    Pcg rng;
    bool live = false, drained = false;
    for (;;) {
        if (!drained) {
            const uint32_t j = queue_slot(!live, work);
            const bool got = !live && j < count;
            if (wave_any(!live && j >= count)) drained = true;   /* later entries are larger still */
            if (got) {
                s = load_state(B.q_in, pbase + j);
                rng.state = s.rng_state;
                rng.inc = (((uint64_t) path_seq(P, B, s.idx)) << 1) | 1u;
                pk.fetch(s, rng);
                if (kPk & PK_RAY) { pk.put3(PF_RAY, s.ray.o); pk.put3(PF_RAY + 3, s.ray.d); }
                live = true;
            }
        }
        if (!wave_any(live)) break;
        constexpr bool kBruteW = kW == WALK_BRUTE || kW == WALK_BRUTE_NS;
        if (kPk & PK_RAY) s.ray = Ray{pk.get3(PF_RAY), pk.get3(PF_RAY + 3), kLargest};
        Hit h{kInf, 0.f, 0.f, -1};
        if (kBruteW || live) h = walk_closest<kW>(sc, s.ray);   /* brute force: every lane of the wave walks */
        bool keep = false, nee = false;
        Ray shr;
        f3 nee_to;
        C3 res_nee;
        if (live) keep = bounce_vertex<kDiff>(P, S, sc, s, rng, h, nee, shr, nee_to, res_nee, pk);
        /* the continuation ray waits in LDS during the shadow walk */
        if ((kPk & PK_RAY) && live) { pk.put3(PF_RAY, s.ray.o); pk.put3(PF_RAY + 3, s.ray.d); }
        /* wave-level counts in scalar registers (no per-lane 64-bit counters across the loop) */
        verts += (uint32_t) __popcll(__ballot(live));
        shadows += (uint32_t) __popcll(__ballot(nee));
        bool occluded = true;
        if constexpr (kBruteW) occluded = brute_any<kW == WALK_BRUTE>(sc, shr, !nee);
        else if (nee) occluded = walk_any<kW>(sc, shr);
        if (nee && !occluded) pk.set_res(s, pk.res_nee(res_nee));
        if (live && !keep) {
            const C3 r = pk.res(s);
            const uint32_t idx = pk.idx(s);
            B.lane_out[idx] = make_float4(r.r, r.g, r.b, s.valid_ray ? 1.f : 0.f);
            if (P.rng_out) P.rng_out[P.chunk_begin + slot_lane(P, idx)] = pk.rng_state(rng);
            live = false;
        }
    }
    if (B.stats && __lane_id() == 0) {
        if (verts) atomicAdd(B.stats + 0 * kStatShards + blockIdx.x % kStatShards, (unsigned long long) verts);
        if (shadows) atomicAdd(B.stats + 5 * kStatShards + blockIdx.x % kStatShards, (unsigned long long) shadows);
    }
}

/* ------------------------------------------------------------------ */
/* k_splat_single: ImageBlock::put of render_sample                    */
/* ------------------------------------------------------------------ */

template <int C>
__global__ void __launch_bounds__(kSplatBlock) k_splat_single(KParams P, Bufs B) {
    __shared__ SplatLds<C> L;
    splat_lds_init(L);
    const uint32_t slot = blockIdx.x * kSplatBlock + threadIdx.x;
    const bool ok = slot < P.chunk_n;
    const uint32_t i = ok ? slot_lane(P, slot) : 0u;
    float vals[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float putx = 0.f, puty = 0.f;
    if (ok) {
        const uint32_t lane = lane_of(P, P.chunk_begin + i);
        int px, py;
        lane_pixel(P, lane, px, py);
        Pcg rng = pass_rng(P, lane, P.chunk_begin + i);
        float jx = rng.next_1d(), jy = rng.next_1d();
        float sx = (float) px + jx, sy = (float) py + jy;
        float4 lo = B.lane_out[slot];
        bool valid = lo.w != 0.f;
        C3 spec = csel(valid, C3{lo.x, lo.y, lo.z}, c3(0.f));
        float alpha = valid ? 1.f : 0.f;
        pack_vals(P, spec, alpha, 1.f, vals);
        putx = P.path_box_pos ? (float) px : sx;
        puty = P.path_box_pos ? (float) py : sy;
        if (P.record) {
            float *r = B.records + (size_t) i * 8;
            r[0] = sx; r[1] = sy; r[2] = spec.r; r[3] = spec.g; r[4] = spec.b; r[5] = alpha; r[6] = 1.f; r[7] = 1.f;
        }
    }
    unsigned long long nonfinite = 0, negative = 0;
    check_sample(P, vals, ok, nonfinite, negative);
    if (P.film_fx) direct_put<C>(P, B.film, putx, puty, vals, ok, P.coalesce_single != 0);
    else block_put<C>(P, B.film, L, 0, putx, puty, vals, ok, P.coalesce_single != 0);
    if (B.stats) { stat_add(B.stats, 6, nonfinite); stat_add(B.stats, 7, negative); }
}

template <int C>
__global__ void __launch_bounds__(kSplatBlock) k_splat_adapt(KParams P, Bufs B) {
    __shared__ SplatLds<C> L;
    splat_lds_init(L);
    const uint32_t slot = blockIdx.x * kSplatBlock + threadIdx.x;
    const bool ok = slot < P.chunk_n;
    float vals[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    float sx = 0.f, sy = 0.f;
    if (ok) {
        const uint32_t j = (uint32_t) (P.chunk_begin + slot);
        float apx, apy;
        lane_sample_pos(P, lane_of(P, B.asel[j / P.n_adapt]), sx, sy, apx, apy);
        const float4 lo = B.lane_out[slot];
        const float w = P.adapt_w;
        pack_vals(P, C3{w * lo.x, w * lo.y, w * lo.z}, 1.f, w, vals);
    }
    unsigned long long nonfinite = 0, negative = 0;
    check_sample(P, vals, ok, nonfinite, negative);
    if (P.film_fx) direct_put<C>(P, B.film, sx, sy, vals, ok, false);
    else block_put<C>(P, B.film, L, 0, sx, sy, vals, ok, false);
    if (B.stats) { stat_add(B.stats, 6, nonfinite); stat_add(B.stats, 7, negative); }
}

/* ------------------------------------------------------------------ */
/* Primary vertex of render_multisample (mvpath_multi.h:8-38)          */
/* ------------------------------------------------------------------ */

/* jitter, [aperture], sample_ray_idx of lane-order thread i of the chunk */
struct PrimRay {
    Pcg rng;
    uint32_t v1, p_idx;
    float sx, sy, apx, apy;
    Ray ray;
};
AD PrimRay primary_raygen(const KParams &P, const DView *V, uint32_t i) {
    PrimRay r;
    const uint32_t lane = lane_of(P, P.chunk_begin + i);
    int px, py;
    lane_pixel(P, lane, px, py);
    uint32_t v0;
    tea4(P.seed_value, lane, v0, r.v1);
    r.rng.seed(v0, r.v1);
    const float jx = r.rng.next_1d(), jy = r.rng.next_1d();
    r.sx = (float) px + jx;
    r.sy = (float) py + jy;
    r.apx = r.apy = .5f;   /* aperture sample: raygen and every view's sample_surface */
    if (P.needs_ap) { r.apx = r.rng.next_1d(); r.apy = r.rng.next_1d(); }
    r.ray = sample_ray_idx(P, V, fmadd(r.sx, P.inv_w, P.adj_ox), fmadd(r.sy, P.inv_h, P.adj_oy), r.p_idx, r.apx, r.apy);
    return r;
}
/*
 * Group sizes.  G = 2..16 are compile-time instances; G = 0 and G = -1 are the runtime instances for
 * groups of 17..256 and 257..1024 views (KParams::G): 256- / 1024-bit per-view masks (WMask<4>,
 * WMask<16>) kept in their own planes (vreq_w, lmask_w), 64-thread primary blocks with the per-view
 * state in LDS while it fits in 64 KB and in a global plane per chunk beyond (Bufs::vstate), k_vis waves
 * that walk several slots.  The reference has no cap (mvpath.cpp:192-217); groups beyond 1024 views
 * (over a million MIS pair terms per lane) are refused.
 */
constexpr uint32_t kMaxGWide = 256, kMaxGHuge = 1024;
template <int G> AD int group_size(const KParams &P) { return G > 0 ? G : (int) P.G; }
/* per-view bit masks: 32 bits for G <= 16 (bits 16+ carry other fields), NW 64-bit words for the
 * runtime instances, indexed with a wave-uniform view slot k */
template <int NW> struct WMask {
    unsigned long long w[NW];
    AD WMask(uint32_t v = 0u) {
#pragma unroll
        for (int q = 0; q < NW; ++q) w[q] = q ? 0ull : (unsigned long long) v;
    }
};
template <int G> constexpr int mask_words() { return G == 0 ? 4 : 16; }
template <int G> using VMask = typename std::conditional<(G > 0), uint32_t, WMask<mask_words<G>()>>::type;
/* uint4 planes per runtime-instance mask (two 64-bit words each) */
template <int G> constexpr int mask_planes() { return G > 0 ? 0 : mask_words<G>() / 2; }
constexpr int kMaxMaskPlanes = 8;
AD bool mget(uint32_t m, int k) { return (m >> k) & 1u; }
template <int NW> AD bool mget(const WMask<NW> &m, int k) {
    unsigned long long x = 0ull;
#pragma unroll
    for (int q = 0; q < NW; ++q) x = (k >> 6) == q ? m.w[q] : x;
    return (x >> (k & 63)) & 1ull;
}
AD uint32_t mpopc(uint32_t m) { return (uint32_t) __popc(m & 0xffffu); }   /* G <= 16: bits 16+ are other fields */
template <int NW> AD uint32_t mpopc(const WMask<NW> &m) {
    uint32_t c = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) c += (uint32_t) __popcll(m.w[q]);
    return c;
}
AD void mset(uint32_t &m, int k, bool b) { m |= b ? 1u << k : 0u; }
template <int NW> AD void mset(WMask<NW> &m, int k, bool b) {
#pragma unroll
    for (int q = 0; q < NW; ++q) m.w[q] |= (b && (k >> 6) == q) ? 1ull << (k & 63) : 0ull;
}
AD void mclr(uint32_t &m, int k) { m &= ~(1u << k); }
/* a compile-time group's mask in bits 16..31 of a record word (0 for the runtime instances) */
AD uint32_t mlow16(uint32_t m) { return m << 16; }
template <int NW> AD uint32_t mlow16(const WMask<NW> &) { return 0u; }
template <int NW> AD void mclr(WMask<NW> &m, int k) {
#pragma unroll
    for (int q = 0; q < NW; ++q) m.w[q] &= (k >> 6) == q ? ~(1ull << (k & 63)) : ~0ull;
}
/* a runtime-instance mask through NW / 2 uint4 planes (words 2j, 2j + 1 in plane j) */
template <int NW> AD void mstore(uint4 *const *pl, uint32_t slot, const WMask<NW> &m) {
#pragma unroll
    for (int j = 0; j < NW / 2; ++j)
        pl[j][slot] = make_uint4((uint32_t) m.w[2 * j], (uint32_t) (m.w[2 * j] >> 32), (uint32_t) m.w[2 * j + 1],
                                 (uint32_t) (m.w[2 * j + 1] >> 32));
}
template <int NW> AD WMask<NW> mload(const uint4 *const *pl, uint32_t slot) {
    WMask<NW> m;
#pragma unroll
    for (int j = 0; j < NW / 2; ++j) {
        const uint4 a = pl[j][slot];
        m.w[2 * j] = ((unsigned long long) a.y << 32) | a.x;
        m.w[2 * j + 1] = ((unsigned long long) a.w << 32) | a.z;
    }
    return m;
}
/* view index of group slot k of a lane whose primary view is p_idx (mvpath_multi.h:31-38) */
AD uint32_t group_view_n(uint32_t Gn, uint32_t p_idx, int k) {
    const uint32_t max_idx = Gn * (p_idx / Gn + 1u), id = p_idx + (uint32_t) k;
    return id < max_idx ? id : id - Gn;
}
template <int G> AD uint32_t group_view(uint32_t p_idx, int k) { return group_view_n((uint32_t) G, p_idx, k); }
/* k_vis's verdict for slot k of lane-order thread i (0: emitter shadow ray, k >= 1: view k) */
AD bool occluded_n(const Bufs &B, uint32_t Gn, uint32_t i, int k) {
    return (B.occ[(size_t) (i >> 6) * Gn + (uint32_t) k] >> (i & 63u)) & 1ull;
}

/*
 * The primary vertex runs as four wavefronts (the BVH walks get their own launches):
 *   k_prim_hit   raygen + closest hit                         -> hit
 *   k_prim_req   the rays the reference traces at this vertex: the emitter sample's
 *                shadow ray (scene.cpp:338) and one visibility ray per view of the
 *                group that passes sensors_visible's geometric tests (mvpath.h:243-256)
 *   k_vis        those rays, one wave per (64 lanes, slot): any-hit -> occlusion ballots
 *   k_mv_primary the whole vertex (camera_selection, mis_weights, direct light,
 *                mixture pdf) with the ray tests read from the ballots
 * k_prim_req and k_mv_primary evaluate the same functions on the same inputs, so the
 * traced rays are exactly the reference's.
 */
template <bool kUni>
__global__ void __launch_bounds__(256) k_prim_hit(KParams P, const DScene *Sp, const DView *V, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<false>(S, lds, P.trav_mode);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < P.chunk_n && P.max_depth != 0) {
        const PrimRay pr = primary_raygen(P, V, i);
        B.hit[i] = hit_rec(trace_closest<kUni>(sc, pr.ray));
    }
}

/* k_prim_req's body for lane-order thread i: the primary vertex (pr, hit) -> visibility requests */
template <int G, bool kTab, bool kDiff>
AD void prim_requests(const KParams &P, const SceneRef &sc, const DScene &S, const DView *V, const Bufs &B, uint32_t i,
                      PrimRay pr, const Hit &hit) {
    const int Gn = group_size<G>(P);
    VMask<G> bits = 0;
    f3 p = mk(0.f, 0.f, 0.f), n = p, dsp = p;
    if (P.max_depth != 0) {
        const SI si = compute_si(sc, pr.ray, hit);
        const bool p_hit = si.valid();
        const bool direct_em = si_emitter(sc, si) >= 0;
        const int32_t b = p_hit ? S.shapes[si.shape].bsdf : -1;
        const bool bsdf_smooth = (bsdf_flags(S.bsdfs, b) & BF_Smooth) != 0;
        const float e1 = pr.rng.next_1d(), e2 = pr.rng.next_1d();
        DSamp ds;
        C3 em_w;
        if (sample_emitter_direction(sc, si, e1, e2, p_hit && bsdf_smooth, ds, em_w)) mset(bits, 0, true);
        (void) pr.rng.next_1d();   /* rand_1 */
        const float r2a = pr.rng.next_1d(), r2b = pr.rng.next_1d();
        BSample bsmp;
        C3 bsdf_weight;
        bsdf_sample<kDiff>(S.bsdfs, b, CTX_ALL, si.wi, r2a, r2b, true, bsmp, bsdf_weight);
        const bool delta = (bsmp.type & BF_Delta) != 0 || (bsmp.type & BF_Null) != 0;
        const bool reuse = !direct_em && !delta && p_hit && bsdf_smooth;
        const bool p_face = si.wi.z > 0.f;
#pragma unroll 1
        for (int k = 1; k < Gn; ++k) {
            const Surf r = camera_sample_surface(V[group_view_n((uint32_t) Gn, pr.p_idx, k)], si, reuse, pr.apx, pr.apy);
            mset(bits, k, r.valid && (r.face == p_face) && r.Jp > 0.f);
        }
        p = si.p; n = si.n; dsp = ds.p;
    }
    uint32_t w0 = 0;
    if constexpr (G <= 0) {
        mstore(B.vreq_w, i, bits);
        w0 = pr.p_idx;   /* the runtime instance keeps the primary view in the first plane */
    } else {
        w0 = bits | (pr.p_idx << 16);
    }
    B.vreq[0][i] = make_float4(p.x, p.y, p.z, bitsf(w0));
    B.vreq[1][i] = make_float4(n.x, n.y, n.z, pr.apx);
    B.vreq[2][i] = make_float4(dsp.x, dsp.y, dsp.z, pr.apy);
}

template <int G, bool kTab, bool kDiff>
__global__ void __launch_bounds__(256) k_prim_req(KParams P, const DScene *Sp, const DView *V, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<kTab, false>(S, lds, P.trav_mode, &V, P.n_views);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.chunk_n) return;
    const PrimRay pr = primary_raygen(P, V, i);
    prim_requests<G, kTab, kDiff>(P, sc, S, V, B, i, pr, P.max_depth != 0 ? hit_of(B.hit[i]) : Hit{kInf, 0.f, 0.f, -1});
}

/*
 * k_prim_hit + k_prim_req in one launch (wave-uniform BVHs, whose walk needs no LDS): the raygen
 * is computed once and the hit goes straight into the request code (it is still stored for
 * k_mv_primary).  AMVPT_FUSE_PRIM=0 keeps the two launches (A/B).
 */
#ifndef AMVPT_PRIM_HIT_WAVES_DEFER
#define AMVPT_PRIM_HIT_WAVES_DEFER 8   /* as AMVPT_VIS_WAVES_DEFER, for the primary closest-hit walk */
#endif
template <int G, bool kTab, bool kDiff, int kSph = 1>
__global__ void __launch_bounds__(256, kSph == 2 ? AMVPT_PRIM_HIT_WAVES_DEFER : 1) k_prim_hit_req(KParams P, const DScene *Sp, const DView *V, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<kTab, false>(S, lds, P.trav_mode, &V, P.n_views);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.chunk_n) return;
    const PrimRay pr = primary_raygen(P, V, i);
    Hit h{kInf, 0.f, 0.f, -1};
    if (P.max_depth != 0) {
        h = trace_closest<true, 0, kSph>(sc, pr.ray);
        B.hit[i] = hit_rec(h);
    }
    prim_requests<G, kTab, kDiff>(P, sc, S, V, B, i, pr, h);
}

/* one block = 64 lanes x G slots, wave k traces slot k of the block's 64 lanes (G = 0: 16 waves,
 * wave w traces slots w, w + 16, ... of the runtime group size).  Wave-uniform walks with G > 0
 * (vis_pairs): one block = 128 lanes, wave k traces slot k of both 64-lane groups at once
 * (trace_any2_uni).  AMVPT_VIS_PAIRS = 0 turns that off (A/B). */
#ifndef AMVPT_VIS_PAIRS
#define AMVPT_VIS_PAIRS 1
#endif
template <int G> constexpr int vis_waves() { return G > 0 ? G : 16; }
template <int G, bool kUni> constexpr bool vis_pairs() { return AMVPT_VIS_PAIRS && kUni && G > 0; }
#ifndef AMVPT_VIS_RAYS
/* rays per lane of the pair walk (trace_any2_uni; > 2: trace_anyN_uni, A/B -- 4 rays: config-M k_vis 43.5 ->
 * 50.5 ms, C3 165 -> 238 ms, r04z_ab_*.log) */
#define AMVPT_VIS_RAYS 2
#endif
/* waves per SIMD the paired walk's register allocation must allow (0: no bound).  Measured at
 * config M (r02ac): unbounded 96 VGPRs / 5 waves 69.3 ms, 6 waves (80 VGPRs, 12 B scratch)
 * 63.5 ms, 8 waves (64 VGPRs, 52 B scratch) 74.1 ms; one ray per lane, 8 waves: 72.3 ms */
#ifndef AMVPT_VIS_WAVES
#define AMVPT_VIS_WAVES 6
#endif
template <int G, bool kUni> constexpr int vis_min_waves() { return vis_pairs<G, kUni>() ? AMVPT_VIS_WAVES : 0; }
#ifndef AMVPT_VIS_WAVES_DEFER
/* k_vis with deferred sphere tests: the walk needs what the sphere-free walk needs (41 VGPRs), so the register
 * budget is that of 8 waves/SIMD; the float64 tests after the walk -- rare, after the screen -- may spill */
#define AMVPT_VIS_WAVES_DEFER 8
#endif
template <int G, bool kUni, int kSph = 1>
__global__ void __launch_bounds__(64 * vis_waves<G>(), (kSph == 2 && vis_pairs<G, kUni>() ? AMVPT_VIS_WAVES_DEFER : vis_min_waves<G, kUni>())) k_vis(KParams P, const DScene *Sp, const DView *V, Bufs B) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    SceneRef sc = stage_scene<false, true, (AMVPT_TREELETS & 4) != 0>(S, lds, P.trav_mode);
    const int Gn = group_size<G>(P);
    if constexpr (vis_pairs<G, kUni>()) {
        /* kVR = AMVPT_VIS_RAYS rays per lane: 64-lane groups h of the block's 64 x kVR lanes, one view slot k per wave */
        constexpr int kVR = AMVPT_VIS_RAYS;
        const int k = (int) (threadIdx.x >> 6);
        Ray r[kVR];
        bool act[kVR];
#pragma unroll
        for (int h = 0; h < kVR; ++h) {
            const uint32_t i = blockIdx.x * (64u * kVR) + 64u * (uint32_t) h + (threadIdx.x & 63u);
            act[h] = false;
            r[h] = Ray{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 1.f), 0.f};
            if (i < P.chunk_n) {
                const float4 a = B.vreq[0][i];
                const uint32_t bits = fbits(a.w);
                if ((bits >> k) & 1u) {
                    const float4 nn = B.vreq[1][i], d = B.vreq[2][i];
                    const f3 target = k == 0 ? mk(d.x, d.y, d.z) : camera_point(V[group_view<G>(bits >> 16, k)], nn.w, d.w);
                    r[h] = spawn_ray_to(mk(a.x, a.y, a.z), mk(nn.x, nn.y, nn.z), target);
                    act[h] = true;
                }
            }
        }
        bool occ[kVR];
        if constexpr (kVR == 2) trace_any2_uni<kSph>(sc, r[0], act[0], r[1], act[1], occ[0], occ[1]);
        else trace_anyN_uni<kSph, kVR>(sc, r, act, occ);
#pragma unroll
        for (int h = 0; h < kVR; ++h) {
            const unsigned long long m = __ballot(occ[h]);
            const uint32_t grp = kVR * blockIdx.x + (uint32_t) h;
            if ((threadIdx.x & 63u) == 0u && (h == 0 || grp * 64u < P.chunk_n)) B.occ[(size_t) grp * Gn + (uint32_t) k] = m;
        }
        return;
    }
    const uint32_t i = blockIdx.x * 64u + (threadIdx.x & 63u);
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f), nn = a, d = a;
    VMask<G> bits = 0;
    uint32_t p_idx = 0;
    if (i < P.chunk_n) {
        a = B.vreq[0][i];
        if constexpr (G <= 0) {
            bits = mload<mask_words<G>()>(B.vreq_w, i);
            p_idx = fbits(a.w);
        } else {
            bits = fbits(a.w);
            p_idx = (uint32_t) bits >> 16;
        }
    }
    /* G > 0: exactly one slot per wave (block = 64 x G threads), a straight-line body */
#pragma unroll 1
    for (int k = (int) (threadIdx.x >> 6); G > 0 ? true : k < Gn; k += vis_waves<G>()) {
        bool occ = false;
        if (i < P.chunk_n && mget(bits, k)) {
            nn = B.vreq[1][i]; d = B.vreq[2][i];
            const f3 target = k == 0 ? mk(d.x, d.y, d.z) : camera_point(V[group_view_n((uint32_t) Gn, p_idx, k)], nn.w, d.w);
            occ = trace_any<kUni, 0, kSph>(sc, spawn_ray_to(mk(a.x, a.y, a.z), mk(nn.x, nn.y, nn.z), target));
        }
        const unsigned long long m = __ballot(occ);
        if ((threadIdx.x & 63u) == 0u) B.occ[(size_t) blockIdx.x * Gn + (uint32_t) k] = m;
        if (G > 0) break;
    }
}

/* ------------------------------------------------------------------ */
/* k_mv_primary<G>: sample_multi up to the shared suffix               */
/* ------------------------------------------------------------------ */

enum : uint32_t { VF_VALID = 1u, VF_INDIRECT = 2u };
/* generic stage (AMVPT_WAVE_DIFF): the all-diffuse waves' compact records, one weight per view [G][n], after
 * the two float4 planes of the generic view records */
AD float *vrec_compact(const Bufs &B, int Gn, uint32_t n) { return reinterpret_cast<float *>(B.vrec + (size_t) 2 * Gn * n); }
enum : uint32_t { LF_VALIDRAY = 1u, LF_ADAPT = 2u, LF_REUSE = 4u, LF_MIS = 8u, LF_DIRECT = 16u,
                  LF_DIFFW = 32u /* an all-diffuse wave of the generic stage: compact view records, vrec_compact */ };

struct SD {        /* SampleData (mvpath.h:150-167) without the derived fields */
    C3 result, bsdf_val;
    f3 wi;
    float px, py, weight, pdfM, pdf, pdf_lk, Jp, iJp;
    uint32_t idx;
    bool indirect, valid;
};

struct BD { int32_t bsdf; float alpha, sqr_a, rsqrt_a; bool diffuse, reuse; };

AD float tv_pdf(const DBsdf *T, f3 wo_l, f3 wi_k, float p_k, const BD &bd, bool active) {
    active = active && p_k > 0.f;
    float p_l = bsdf_pdf(T, bd.bsdf, CTX_GLOSSY, wi_k, wo_l, active);
    active = active && p_l > 0.f;
    float p_max = vmax(p_l, p_k), p_min = vmin(p_l, p_k);
    float q = p_min * rcp(p_max);
    float p = fmadd(q - 1.f, bd.rsqrt_a, 1.f);
    p = sqr(vmax(p, 0.f));
    p = lerp_(p, q, bd.alpha);
    return active ? p : 0.f;
}
/* tv_pdf with wi_k's pdf row hoisted out of a loop over wo_l (same value bit for bit) */
AD float tv_pdf_row(const PdfRow &R, f3 wo_l, float p_k, const BD &bd, bool active) {
    active = active && p_k > 0.f;
    float p_l = row_pdf(R, wo_l, active);
    active = active && p_l > 0.f;
    float p_max = vmax(p_l, p_k), p_min = vmin(p_l, p_k);
    float q = p_min * rcp(p_max);
    float p = fmadd(q - 1.f, bd.rsqrt_a, 1.f);
    p = sqr(vmax(p, 0.f));
    p = lerp_(p, q, bd.alpha);
    return active ? p : 0.f;
}
AD float tv_pdf_fast(f3 wo_l, f3 wi_k, float p_k, const BD &bd, bool active) {
    float p_l = sqr(normalize(wi_k + wo_l).z);
    float N = fmadd(bd.sqr_a, vmax(p_k, p_l), 1.f), D = fmadd(bd.sqr_a, vmin(p_k, p_l), 1.f);
    float q = sqr(N * rcp(D));
    float p = fmadd(q - 1.f, bd.rsqrt_a, 1.f);
    p = sqr(vmax(p, 0.f));
    p = lerp_(p, q, bd.alpha);
    return active ? p : 0.f;
}
AD f3 reflect_l(f3 w) { return mk(-w.x, -w.y, w.z); }

/*
 * Per-view state lives in LDS (VS_FIELDS floats per view slot, thread-minor so
 * every access is bank-conflict free) and the per-view loops are not unrolled, so
 * each per-view body (a visibility ray, three BSDF evaluations, ...) is emitted
 * once: the unrolled form with register arrays needed > 256 VGPRs and spilled.
 * View records are written as soon as each part is final:
 *   rec0[k] = (splat x, splat y, weight, flags), rec1[k] = result, rec2[k] = bsdf_val.
 */
#ifndef AMVPT_BOUNCE_TAB
#define AMVPT_BOUNCE_TAB 1
#endif
#ifndef AMVPT_PRIM_TAB
#define AMVPT_PRIM_TAB 1
#endif
#ifndef AMVPT_PRIM_SLOT_ORDER
#define AMVPT_PRIM_SLOT_ORDER 1
#endif
#ifndef AMVPT_DEFER_SAMPLE
/* camera_selection's per-view BSDF samples: the loop takes each view's sample type (no sampling)
 * and one bsdf_sample runs for the last replacing view (0: a sample per view, A/B) */
#define AMVPT_DEFER_SAMPLE 1
#endif
#ifndef AMVPT_PAIR_REGS
/* pair-sum operands of views j >= 1 in registers for G <= 8: k_mv_primary 459 -> 427 ms per C3 frame
 * (0: read from LDS per pair, A/B r03g); reading view k's own fields from the register copies too
 * (uniform dynamic index) measured slower, 444 ms (r03h) */
#define AMVPT_PAIR_REGS 1
#endif
#ifndef AMVPT_PDF_REGS
/* 1: with the pair registers, the views' F_PDF lives in registers only (written under a uniform view index in
 * camera_selection, read the same way in mis_weights), so the generic instance's per-view LDS state drops from 6
 * to 5 fields: 29.4 -> 25.3 KB per 128-thread block at C3, 6 blocks (12 waves, its VGPR limit) per CU instead of
 * 5 (0: A/B) */
#define AMVPT_PDF_REGS 1
#endif
#ifndef AMVPT_DIFF_REGS
/* 1: the all-diffuse body (kDiff: the all-diffuse scenes' k_mv_primary and the mixed scenes' all-diffuse waves) of
 * the compile-time groups up to 8 views keeps both per-view fields, F_PDF and F_JP, in registers (written and read
 * under a uniform view index, the MIS pair sums unrolled over register operands), so it has no per-view LDS state
 * and no LDS read per pair term.  Measured slower (r06ad: config-M k_mv_primary 40.0 -> 41.7 ms, C3 and mesh neutral --
 * the uniform-index select chains cost more issue than the LDS reads they replace), so 0: the two LDS fields */
#define AMVPT_DIFF_REGS 0
#endif
/* the all-diffuse body keeps F_PDF and F_JP in registers (see AMVPT_DIFF_REGS) */
template <int G, bool kDiff> __host__ __device__ constexpr bool diff_regs() {
    return AMVPT_DIFF_REGS && AMVPT_PAIR_REGS && kDiff && G >= 2 && G <= 8;
}
/* the generic compile-time groups keep F_PDF out of LDS (see AMVPT_PDF_REGS) */
template <int G, bool kDiff> __host__ __device__ constexpr bool pdf_in_regs() {
    return (AMVPT_PAIR_REGS && AMVPT_PDF_REGS && !kDiff && G >= 2 && G <= 8) || diff_regs<G, kDiff>();
}
template <int G, bool kDiff> __host__ __device__ constexpr int vs_fields() {
    return kDiff ? (diff_regs<G, kDiff>() ? 0 : kVsFieldsDiff) : VS_FIELDS - (pdf_in_regs<G, kDiff>() ? 1 : 0);
}
#ifndef AMVPT_FUSED_TWO_STREAMS
#define AMVPT_FUSED_TWO_STREAMS 0   /* 1: fused-suffix scenes alternate chunks over two streams too (A/B) */
#endif
#ifndef AMVPT_CHUNK_STREAMS
#define AMVPT_CHUNK_STREAMS 4   /* chunk streams of a per-depth-suffix render (1: every chunk on the render stream; mesh
                                 * 962-973 / 984-988 / 1001-1002 Msamples/s with 2 / 3 / 4, r05zi; A/B) */
#endif
#ifndef AMVPT_TILE_SLOTS
/* 4 x 4 pixel tiles per row-splat block (see tile_slot_lane): config M 1472 -> 1521 Msamples/s (splat
 * 106.3 -> 100.7 ms, and the fused suffix 134 -> 129.6 ms: its queue drains spatially coherent paths);
 * with block-wide windows instead of wave windows it lost (splat 122 ms, r03s) */
#define AMVPT_TILE_SLOTS 1
#endif
#ifndef AMVPT_PDF_ROW
#define AMVPT_PDF_ROW 1   /* the pairwise MIS sum hoists wi_k's pdf row (0: per-pair bsdf_pdf, A/B) */
#endif
#ifndef AMVPT_COH_UNI
/* 1: k_prim_hit(_req) and k_vis walk wave-uniformly (scalar node loads, the wave enters a node when
 * any lane's ray hits its box) on BVHs of any size -- a wave's camera / visibility rays are nearly
 * identical (4 pixels x 16 samples, one target view per wave), and the primary walk fuses with the
 * request code (k_prim_hit_req).  3.6 k-triangle mesh: 629.9 -> 663.8 Msamples/s (r03v); 0: per-lane
 * walks above kUniformNodeLimit nodes (A/B) */
#define AMVPT_COH_UNI 1
#endif
#ifndef AMVPT_WAVE_DIFF
/* 1: the generic k_mv_primary runs the all-diffuse body for waves whose primary hits are all plain
 * diffuse (mixed-material scenes; A/B 0) */
#define AMVPT_WAVE_DIFF 1
#endif
#ifndef AMVPT_PRIM_WAVES
#define AMVPT_PRIM_WAVES 1
#endif
/*
 * kDiff (every BSDF of the scene is plain `diffuse`): pdf_Mat is 1 and eval/pdf depend
 * on a direction only through the sign of its z, a view's BSDF sample is the primary's
 * own (cosine_hemisphere(rand_2) whatever wi), so the per-view state reduces to F_PDF,
 * F_JP and one sign bit per view -- same values, a third of the LDS per thread.
 */
template <int G> constexpr int prim_block() { return G > 0 ? kPrimBlock : 64; }   /* G <= 0: LDS state grows with G */
/*
 * The per-lane body of k_mv_primary.  kDiff: the all-diffuse computation (see below); kGenRec (with
 * kDiff): a wave of a mixed scene's generic stage whose primary hits are all plain `diffuse` runs the
 * all-diffuse computation -- it reads the hit's BSDF only, so the values are the generic path's -- and
 * writes the compact records (one weight per view, vrec_compact) with LF_DIFFW in its lane flags;
 * k_splat_multi reads such a wave's records the all-diffuse way.
 */
template <int G, bool kTab, bool kDiff, bool kGenRec>
AD void mv_primary_lane(const KParams &P, const DScene &S, const SceneRef &sc, const DView *V, const Bufs &B,
                        float *const vs, const uint32_t vs_stride, const uint32_t slot, const uint32_t i, const bool ok) {
    const int Gn = group_size<G>(P);
    constexpr bool kPdfRegs = pdf_in_regs<G, kDiff>();
    constexpr bool kJpRegs = diff_regs<G, kDiff>();   /* F_JP in registers as well: no per-view LDS state */
    /* field f of view slot k (kPdfRegs: F_PDF is not stored, the other fields move down one) */
#define VSF(f, k) vs[(((f) - (kPdfRegs ? 1 : 0)) * Gn + (k)) * vs_stride]
    PathState ps;
    bool push = false;
    unsigned long long st_reuse = 0, st_vis = 0;
    if (ok) {
        /* every global load first: a load issued after the record stores would wait
         * for them (vmcnt counts loads and stores in issue order) */
        const float4 hitv = B.hit[i];
        VMask<G> occm = 0;   /* bit k: k_vis found slot k occluded */
#pragma unroll
        for (int k = 0; k < Gn; ++k) mset(occm, k, occluded_n(B, (uint32_t) Gn, i, k));
        const uint32_t n = P.chunk_n;
        const PrimRay pr = primary_raygen(P, V, i);
        Pcg rng = pr.rng;
        const uint32_t v1 = pr.v1, p_idx = pr.p_idx;
        const float apx = pr.apx, apy = pr.apy;
        const Ray pray = pr.ray;
        /* view records (see Bufs): kDiff -> one weight per view; generic -> (result, weight) and
         * (bsdf value, flags) per view.  Splat positions are not stored: k_splat_multi recomputes
         * them from the hit point (camera_uv) and the lane's jitter. */
        float *const vw = kGenRec ? vrec_compact(B, Gn, n) : reinterpret_cast<float *>(B.vrec);
        float4 *const vR = B.vrec, *const vB = B.vrec + (size_t) Gn * n;
        auto view_of = [&](int k) -> uint32_t { return group_view_n((uint32_t) Gn, p_idx, k); };
        auto put_view = [&](int k, float w, C3 res, C3 bv, uint32_t vf) {
            const size_t o = (size_t) k * n + slot;
            if (kDiff) {
                vw[o] = w;
            } else {
                vR[o] = make_float4(res.r, res.g, res.b, w);
                vB[o] = make_float4(bv.r, bv.g, bv.b, bitsf(vf));
            }
        };
        VMask<G> vmask = 0, imask = 0;   /* bit k: view k valid / indirect */
        float w0 = 1.f;                  /* slot 0's splat weight */
        C3 R0 = c3(0.f);                 /* slot 0's result: emission + direct light */
        C3 Dp = c3(0.f);                 /* kDiff: direct light through a valid view k >= 1 */
        C3 Bv = c3(0.f);                 /* kDiff: BSDF value of every indirect view */
        f3 hp = mk(0.f, 0.f, 0.f);       /* primary hit point (reprojection in the splat) */
        bool records_done = false, reuse_l = false, direct_l = false;
        uint32_t nf_bits = 0;   /* kDiff: non-finite emis_mis channels */
        VMask<G> smask = 0;     /* kDiff: wi_k.z > 0 views */

        /* ---- sample_multi (mvpath_multi.h:130-369) ---- */
        bool valid_ray = P.valid_ray0 != 0 && P.max_depth != 0, adapt_mask = false;
        float pdfW = 1.f;
        bool should_mis = P.sa_mis != 0;
        if (P.max_depth != 0) {
            SI si = compute_si(sc, pray, hit_of(hitv));
            bool p_hit = si.valid();
            hp = si.p;
            int32_t em = si_emitter(sc, si);
            bool direct_em = em >= 0;
            C3 emitted = c3(0.f);
            if (direct_em) emitted = emitter_eval(sc, em, si, true);
            int32_t b = p_hit ? S.shapes[si.shape].bsdf : -1;
            bool bsdf_smooth = (bsdf_flags(S.bsdfs, b) & BF_Smooth) != 0;
            bool active_em = p_hit && bsdf_smooth;
            float e1 = rng.next_1d(), e2 = rng.next_1d();
            DSamp ds;
            C3 em_w;
            if (sample_emitter_direction(sc, si, e1, e2, active_em, ds, em_w) && mget(occm, 0))
                occlude_emitter_sample(ds, em_w);
            active_em = active_em && ds.pdf != 0.f;
            direct_l = active_em;
            f3 wo = si.sh.to_local(ds.d);
            float rand_1 = rng.next_1d();
            float r2a = rng.next_1d(), r2b = rng.next_1d();
            (void) rand_1;
            C3 bsdf_val;
            float direct_pdf;
            bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, si.wi, wo, true, bsdf_val, direct_pdf);
            BSample bsmp;
            C3 bsdf_weight;
            bsdf_sample<kDiff>(S.bsdfs, b, CTX_ALL, si.wi, r2a, r2b, true, bsmp, bsdf_weight);
            bool flag_delta = (bsmp.type & BF_Delta) != 0, flag_null = (bsmp.type & BF_Null) != 0;
            bool flag_diff = (bsmp.type & BF_Diffuse) != 0;
            bool delta = flag_delta || flag_null, p_not_delta = !delta && p_hit;
            bool reuse = !direct_em && p_not_delta && bsdf_smooth;
            reuse_l = reuse;
            st_reuse += reuse ? 1 : 0;
            bool p_face = si.wi.z > 0.f;
            if (should_mis) {
                BD bd;
                bd.bsdf = b;
                bd.alpha = bsdf_roughness<kDiff>(S.bsdfs, b, si.wi);
                bd.sqr_a = fmsub(bd.alpha, bd.alpha, 1.f);
                bd.rsqrt_a = rsqrt_(bd.alpha);
                bd.diffuse = flag_diff;
                bd.reuse = reuse;
                /* ---- camera_selection (mvpath_multi.h:371-464) ---- */
                Surf p0 = camera_sample_surface(V[view_of(0)], si, p_hit, apx, apy);
                const float pdf0 = p0.pdf, Jp0 = p0.Jp, iJp0 = p_hit ? rcp(p0.Jp) : 0.f;
                if (!kPdfRegs) VSF(F_PDF, 0) = pdf0;
                /* kJpRegs: the views' F_JP (slot 0 and slots 1..G-1) */
                float rJp[kJpRegs ? G : 1];
                if constexpr (kJpRegs) {
                    rJp[0] = Jp0;
#pragma unroll
                    for (int j = 1; j < G; ++j) rJp[j] = 0.f;
                } else {
                    VSF(F_JP, 0) = Jp0;
                }
                mset(vmask, 0, p_hit);
                mset(imask, 0, p_hit);
                const f3 wo_r0 = reflect_l(si.wi);
                VMask<G> wpos = p_face ? 1u : 0u;   /* kDiff: bit k = (wi_k.z > 0) */
                if (!kDiff) {
                    VSF(F_WX, 0) = si.wi.x; VSF(F_WY, 0) = si.wi.y; VSF(F_WZ, 0) = si.wi.z;
                    VSF(F_PDFM, 0) = bd.diffuse ? 1.f : (P.fast_mis ? sqr(normalize(si.wi + wo_r0).z)
                                                                   : bsdf_pdf(S.bsdfs, b, CTX_GLOSSY, si.wi, wo_r0, p_hit));
                }
                /* view k's wi (kDiff: diffuse eval / pdf read wi only through the sign of its z) */
                auto wi_of = [&](int k) -> f3 {
                    if (kDiff) return k == 0 ? si.wi : mk(0.f, 0.f, mget(wpos, k) ? 1.f : -1.f);
                    return mk(VSF(F_WX, k), VSF(F_WY, k), VSF(F_WZ, k));
                };
                /* pdf_Mat of view k toward view 0 (tv_pdf, camera_selection) */
                auto mat_pdf = [&](f3 wik, float pdfM, bool active) -> float {
                    if (bd.diffuse) return 1.f;
                    return P.fast_mis ? tv_pdf_fast(wo_r0, wik, pdfM, bd, active)
                                      : tv_pdf(S.bsdfs, wo_r0, wik, pdfM, bd, active);
                };
                /* kPdfRegs: the views' F_PDF (slots 1..G-1) */
                float rPdf[kPdfRegs ? G : 1];
                if constexpr (kPdfRegs) {
#pragma unroll
                    for (int j = 0; j < G; ++j) rPdf[j] = 0.f;
                }
                float n_direct = 1.f, n_indir = 2.f;
                int rep_k = 0;   /* AMVPT_DEFER_SAMPLE: the view whose BSDF sample replaces the primary's */
                (void) rep_k;
#pragma unroll 1
                for (int k = 1; k < Gn; ++k) {
                    Surf r = camera_sample_surface(V[view_of(k)], si, bd.reuse, apx, apy);
                    bool valid = r.valid && (r.face == p_face) && r.Jp > 0.f;
                    if (valid) {
                        ++st_vis;
                        valid = !mget(occm, k);
                    }
                    f3 wik = si.sh.to_local(r.d);
                    float pdf_Mat = 1.f;   /* kDiff: valid implies a diffuse hit (mat_pdf = 1) */
                    if (!kDiff) {
                        VSF(F_WX, k) = wik.x; VSF(F_WY, k) = wik.y; VSF(F_WZ, k) = wik.z;
                        f3 wor = reflect_l(wik);
                        float pdfM = P.fast_mis ? sqr(normalize(wik + wor).z)
                                                : bsdf_pdf(S.bsdfs, b, CTX_GLOSSY, wik, wor, valid);
                        VSF(F_PDFM, k) = pdfM;
                        pdf_Mat = mat_pdf(wik, pdfM, valid);
                    } else {
                        mset(wpos, k, wik.z > 0.f);
                    }
                    float J = r.Jp * iJp0;
                    float pdf_J = J > 1.f ? rcp(J) : J;
                    float pdf_Sel = pdf_Mat * pdf_J;
                    valid = valid && (rng.next_1d() < pdf_Sel);
                    if constexpr (kJpRegs) {
#pragma unroll
                        for (int j = 1; j < G; ++j) rJp[j] = j == k ? r.Jp : rJp[j];
                    } else {
                        VSF(F_JP, k) = r.Jp;
                    }
                    if constexpr (kPdfRegs) {
                        const float pk = valid ? r.pdf : 0.f;
#pragma unroll
                        for (int j = 1; j < G; ++j) rPdf[j] = j == k ? pk : rPdf[j];
                    } else {
                        VSF(F_PDF, k) = valid ? r.pdf : 0.f;
                    }
                    bool indirect = valid, direct = valid;
                    bool replace = n_indir * rng.next_1d() < 1.f;
                    C3 bvk;
                    float bpk;
                    BSample bsk;
                    C3 bwk;
                    bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, wik, wo, valid, bvk, bpk);
                    direct = direct && bpk > 0.f;
                    direct_pdf += direct ? bpk : 0.f;
                    n_direct += (float) direct;
                    if (!kDiff) {
#if AMVPT_DEFER_SAMPLE
                        /* only the last replacing view's sampled direction survives the loop: its type
                         * decides here, the one bsdf_sample runs after the loop */
                        indirect = indirect && bsdf_sample_type(S.bsdfs, b, CTX_ALL, wik, valid) == bsmp.type;
                        if (indirect && replace) rep_k = k;
#else
                        bsdf_sample(S.bsdfs, b, CTX_ALL, wik, r2a, r2b, valid, bsk, bwk);
                        indirect = indirect && bsk.type == bsmp.type;
                        if (indirect && replace) bsmp.wo = bsk.wo;
#endif
                    }
                    /* kDiff: a valid view's sample is the primary's (same type, same wo) */
                    (void) replace;
                    n_indir += (float) indirect;
                    mset(vmask, k, valid);
                    mset(imask, k, indirect);
                }
#if AMVPT_DEFER_SAMPLE
                if (!kDiff && rep_k > 0) {
                    BSample bsk;
                    C3 bwk;
                    bsdf_sample(S.bsdfs, b, CTX_ALL, wi_of(rep_k), r2a, r2b, true, bsk, bwk);
                    bsmp.wo = bsk.wo;
                }
#endif
                direct_pdf /= n_direct;
                const float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, direct_pdf);
                const C3 emis_mis = em_w * mis_em;
                /* kDiff lane values.  A diffuse eval sees wi only through sign(wi.z) and is zero
                 * for wi.z <= 0, so every view's value is one of two per lane: the direct light
                 * of a valid view k >= 1 is Dp (wi_k.z > 0) or cfma(0, emis_mis, 0) (= 0, or NaN
                 * where emis_mis is not finite: bit 8 + c of the lane flags), and an indirect view
                 * (pdf > 0, so wi_k.z > 0) has Bv = eval(+z, wo) with pdf bp_d. */
                float bp_d = 0.f;
                if (kDiff) {
                    R0 = emitted;
                    if (active_em && mget(vmask, 0)) R0 = cfma(bsdf_val, emis_mis, emitted);
                    if (active_em) {
                        C3 ep;
                        float epd;
                        bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, mk(0.f, 0.f, 1.f), wo, true, ep, epd);
                        Dp = cfma(ep, emis_mis, c3(0.f));
                        nf_bits = (finite_(emis_mis.r) ? 0u : 1u) | (finite_(emis_mis.g) ? 0u : 2u) |
                                  (finite_(emis_mis.b) ? 0u : 4u);
                    }
                    bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, mk(0.f, 0.f, 1.f), bsmp.wo, true, Bv, bp_d);
                    smask = wpos;
                }
                /* ---- per view: mis_weights (mvpath_multi.h:466-523), direct light and
                 *      the multi-view mixture pdf (mvpath_multi.h:245-317) ---- */
                float n_ind = 0.f, pdf = 0.f;
                /* the pair sums' operands of views j >= 1 (same for every k): registers for the
                 * compile-time groups up to 8 views, LDS otherwise */
                constexpr int kPR = (AMVPT_PAIR_REGS && (!kDiff || kJpRegs) && G >= 2 && G <= 8) ? G : 1;
                constexpr int kPW = kDiff ? 1 : kPR;   /* the all-diffuse body reads no wi_j */
                float pJp[kPR], pPdf[kPR], pWx[kPW], pWy[kPW], pWz[kPW];
                if constexpr (kPR > 1) {
#pragma unroll
                    for (int j = 1; j < kPR; ++j) {
                        if constexpr (kJpRegs) pJp[j] = rJp[j < G ? j : 0];
                        else pJp[j] = VSF(F_JP, j);
                        if constexpr (kPdfRegs) pPdf[j] = rPdf[j < G ? j : 0];
                        else pPdf[j] = VSF(F_PDF, j);
                        if constexpr (!kDiff) { pWx[j] = VSF(F_WX, j); pWy[j] = VSF(F_WY, j); pWz[j] = VSF(F_WZ, j); }
                    }
                }
#pragma unroll 1
                for (int k = 0; k < Gn; ++k) {
                    const bool vk = mget(vmask, k);
                    float Jpk;
                    if constexpr (kJpRegs) {
                        Jpk = rJp[0];
#pragma unroll
                        for (int j = 1; j < G; ++j) Jpk = j == k ? rJp[j] : Jpk;
                    } else {
                        Jpk = VSF(F_JP, k);
                    }
                    const float iJpk = k == 0 ? iJp0 : (vk ? rcp(Jpk) : 0.f);
                    const f3 wik = wi_of(k);
                    const float pdfMk = kDiff ? 1.f : VSF(F_PDFM, k);
                    /* pdf_lk of camera_selection, re-derived: valid_k implies it was active */
                    float pdf_lk = pdf0;
                    if (k > 0) {
                        const float J = Jpk * iJp0, pdf_J = J > 1.f ? rcp(J) : J;
                        pdf_lk = vk ? pdf0 * J * ((kDiff ? 1.f : mat_pdf(wik, pdfMk, true)) * pdf_J) : 0.f;
                    }
                    float pdfSum = pdf_lk;
                    if (k > 0) {
                        if constexpr (kPdfRegs) {
                            float pk = 0.f;
#pragma unroll
                            for (int j = 1; j < G; ++j) pk = j == k ? pPdf[j] : pk;
                            pdfSum += pk;
                        } else {
                            pdfSum += VSF(F_PDF, k);
                        }
                    }
                    bool cond = k > 0 ? vk : bd.reuse;
                    float acc = 0.f;
                    if (!kDiff && cond && !bd.diffuse) {
#if AMVPT_PDF_ROW
                        const PdfRow row = pdf_row(S.bsdfs, b, CTX_GLOSSY, wik);
#endif
                        if constexpr (kPR > 1) {
#pragma unroll
                            for (int j = 1; j < kPR; ++j) {
                                if (j == k) continue;
                                const float pdf_J = vmin(sqr(pJp[j] * iJpk), 1.f);
                                const int jw = kDiff ? 0 : j;   /* (the all-diffuse body never runs this branch) */
                                const f3 worj = reflect_l(mk(pWx[jw], pWy[jw], pWz[jw]));
                                const bool vj = mget(vmask, j);
#if AMVPT_PDF_ROW
                                const float pdf_Mat = P.fast_mis ? tv_pdf_fast(worj, wik, pdfMk, bd, vj)
                                                                 : tv_pdf_row(row, worj, pdfMk, bd, vj);
#else
                                const float pdf_Mat = P.fast_mis ? tv_pdf_fast(worj, wik, pdfMk, bd, vj)
                                                                 : tv_pdf(S.bsdfs, worj, wik, pdfMk, bd, vj);
#endif
                                acc = fmadd(pPdf[j], pdf_J * pdf_Mat, acc);
                            }
                        } else
#pragma unroll 1
                        for (int j = 1; j < Gn; ++j) {
                            if (j == k) continue;
                            float pdf_J = vmin(sqr(VSF(F_JP, j) * iJpk), 1.f);
                            f3 worj = reflect_l(mk(VSF(F_WX, j), VSF(F_WY, j), VSF(F_WZ, j)));
                            const bool vj = mget(vmask, j);
#if AMVPT_PDF_ROW
                            float pdf_Mat = P.fast_mis ? tv_pdf_fast(worj, wik, pdfMk, bd, vj)
                                                       : tv_pdf_row(row, worj, pdfMk, bd, vj);
#else
                            float pdf_Mat = P.fast_mis ? tv_pdf_fast(worj, wik, pdfMk, bd, vj)
                                                       : tv_pdf(S.bsdfs, worj, wik, pdfMk, bd, vj);
#endif
                            acc = fmadd(VSF(F_PDF, j), pdf_J * pdf_Mat, acc);
                        }
                    } else if constexpr (kPR > 1) {
#pragma unroll
                        for (int j = 1; j < kPR; ++j) {
                            if (j == k) continue;
                            const float pdf_J = vmin(sqr(pJp[j] * iJpk), 1.f);
                            acc = fmadd(pPdf[j], pdf_J, acc);
                        }
                        acc = cond ? acc : 0.f;
                    } else {
#pragma unroll 1
                        for (int j = 1; j < Gn; ++j) {
                            if (j == k) continue;
                            float pdf_J = vmin(sqr(VSF(F_JP, j) * iJpk), 1.f);
                            acc = fmadd(VSF(F_PDF, j), pdf_J, acc);
                        }
                        acc = cond ? acc : 0.f;
                    }
                    pdfSum += acc;
                    const float wk = pdf_lk / pdfSum;
                    bool valid = mget(imask, k);
                    C3 res = c3(0.f), bv = c3(0.f);
                    float bp;
                    if (kDiff) {
                        bp = (valid && mget(wpos, k)) ? bp_d : 0.f;
                    } else {
                        /* result: emission (slot 0) + direct light through this view's BSDF value */
                        res = csel(k == 0, emitted, c3(0.f));
                        if (active_em && vk) {
                            C3 bvk = bsdf_val;
                            if (k > 0) {   /* the value camera_selection evaluated for view k */
                                float bpk;
                                bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, wik, wo, true, bvk, bpk);
                            }
                            res = cfma(bvk, emis_mis, res);
                        }
                        if (k == 0) R0 = res;
                        bsdf_eval_pdf<kDiff>(S.bsdfs, b, CTX_ALL, wik, bsmp.wo, valid, bv, bp);
                        if (k == 0) {
                            bv = csel(p_not_delta, bv, bsdf_weight);
                            bp = p_not_delta ? bp : bsmp.pdf;
                            valid = valid && (bp > 0.f || delta);
                        }
                    }
                    bool pvalid = bp > 0.f;
                    valid = valid && ((k == 0 && !kDiff) ? (pvalid || delta) : pvalid);
                    bp = valid ? bp : 0.f;
                    bv = csel(valid, bv, c3(0.f));
                    pdf += bp;
                    n_ind += (float) valid;
                    if (!valid) mclr(imask, k);
                    if (k == 0) w0 = wk;
                    else put_view(k, wk, res, bv, (vk ? VF_VALID : 0u) | (valid ? VF_INDIRECT : 0u));
                    if (k == 0 && !kDiff) Bv = bv;   /* slot 0's (bsdf value), stored with slot 0 below */
                }
                bsmp.pdf = p_not_delta ? pdf / n_ind : bsmp.pdf;
                adapt_mask = p_hit && !flag_null && (n_ind <= 1.f);
                records_done = true;
            } else {
                mset(vmask, 0, p_hit);
#pragma unroll 1
                for (int k = 1; k < Gn; ++k) {
                    Surf r = camera_sample_surface(V[view_of(k)], si, reuse, apx, apy);
                    bool valid = r.valid && (r.face == p_face) && r.Jp > 0.f;
                    if (valid) {
                        ++st_vis;
                        valid = !mget(occm, k);
                    }
                    mset(vmask, k, valid);
                }
                float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, direct_pdf);
                R0 = emitted;
                if (active_em) R0 = cfma(bsdf_val, em_w * mis_em, R0);
            }
            /* ---- BSDF sampling continuation ---- */
            Ray pd_ray = spawn_ray(si.p, si.n, si.sh.to_world(bsmp.wo));
            C3 thr = csel(should_mis, c3(1.f), bsdf_weight);
            valid_ray = valid_ray || (p_hit && !flag_null);
            bool pd_active = p_hit;
            if (!should_mis) pd_active = pd_active && (cmax(thr) != 0.f);
            if (P.max_depth <= 1) pd_active = false;
            pdfW = p_not_delta ? rcp(bsmp.pdf) : 1.f;
            if (pd_active) {
                ps.ray = pd_ray;
                ps.thr = thr;
                ps.res = c3(0.f);
                ps.eta_zero = bsmp.eta == 0.f;
                ps.prev_pdf = bsmp.pdf;
                ps.depth = p_hit ? 1u : 0u;
                ps.prev_delta = flag_delta;
                ps.valid_ray = false;
                ps.prev_p = si.p;
                ps.idx = slot;
                ps.rng_state = rng.state;
                ps.rng_seq = v1;
                push = true;
            }
            /* p_sample.weight/valid finalisation happens after the suffix */
            if (!p_hit) w0 = 1.f;
            mset(vmask, 0, true);
        }
        if (!push) B.lane_out[slot] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (P.max_depth == 0) {
            /* no intersection at all: every slot keeps weight 0 and is invalid */
            vmask = 0u;
            imask = 0u;
            w0 = 0.f;
        }
        const uint32_t lflags = (valid_ray ? LF_VALIDRAY : 0u) | (adapt_mask ? LF_ADAPT : 0u) |
                                (should_mis ? LF_MIS : 0u) | (reuse_l ? LF_REUSE : 0u) | (direct_l ? LF_DIRECT : 0u) |
                                (nf_bits << 8) | mlow16(smask) | (kGenRec ? LF_DIFFW : 0u);
        B.lrec[0][slot] = make_float4(R0.r, R0.g, R0.b, pdfW);
        B.lrec[1][slot] = make_float4(Dp.r, Dp.g, Dp.b, bitsf(lflags));
        B.lrec[2][slot] = make_float4(Bv.r, Bv.g, Bv.b, bitsf(mlow16(vmask) >> 16 | mlow16(imask)));
        if constexpr (G <= 0) {   /* planes: valid, indirect, wi.z > 0 (mask_planes<G>() each) */
            constexpr int NP = mask_planes<G>();
            mstore(B.lmask_w, slot, vmask);
            mstore(B.lmask_w + NP, slot, imask);
            mstore(B.lmask_w + 2 * NP, slot, smask);
        }
        B.lrec[3][slot] = make_float4(hp.x, hp.y, hp.z, 0.f);
        /* slot 0 (generic: its bsdf value rides in L2), and the views the MIS loop did not write */
        put_view(0, w0, R0, Bv, (mget(vmask, 0) ? VF_VALID : 0u) | (mget(imask, 0) ? VF_INDIRECT : 0u));
        if (!records_done) {
#pragma unroll 1
            for (int k = 1; k < Gn; ++k)
                put_view(k, P.max_depth != 0 ? 1.f : 0.f, c3(0.f), c3(0.f), (mget(vmask, k)) ? VF_VALID : 0u);
        }
    }
    const uint32_t qslot = push_slot(push, B.cnt_out, B.qcap);
    if (push) store_state(B.q_out, qslot, ps);
    if (B.stats) {
        stat_add(B.stats, 1, st_reuse);
        stat_add(B.stats, 2, st_vis);
        stat_add(B.stats, 0, (ok && P.max_depth != 0) ? 1ull : 0ull);
        stat_add(B.stats, 8, push ? 1ull : 0ull);
        stat_add(B.stats, 10, ok ? (unsigned long long) ((kDiff ? 4 : 32) * Gn) : 0ull);
    }
}
#undef VSF

/* every primary hit of the wave is on a plain `diffuse` BSDF, or a miss (wave-uniform) */
AD bool wave_diffuse(const KParams &P, const DScene &S, const SceneRef &sc, const Bufs &B, uint32_t i, bool ok) {
    bool dl = true;
    if (ok && P.max_depth != 0) {
        const int32_t prim = (int32_t) fbits(B.hit[i].w);
        if (prim >= 0) {
            const int32_t b = S.shapes[sc.prims[prim].shape].bsdf;
            dl = b < 0 || S.bsdfs[b].type == BSDF_DIFFUSE;
        }
    }
    return !wave_any(!dl);
}
/* kDiff: the all-diffuse scenes' kernel.  Otherwise (AMVPT_WAVE_DIFF) two launches of the generic stage:
 * kDW = true runs the waves whose primary hits are all diffuse with the all-diffuse body at its own
 * register budget (generic records), kDW = false the others with the generic body */
template <int G, bool kTab, bool kDiff, bool kDW = false>
__global__ void __launch_bounds__(prim_block<G>(), AMVPT_PRIM_WAVES) k_mv_primary(KParams P, const DScene *Sp, const DView *V, Bufs B) {
    constexpr int kPB = prim_block<G>();
    extern __shared__ __attribute__((aligned(16))) char lds[];
    DScene S = *Sp;
    const uint32_t vs_off = kTab ? S.tab_bytes + views_lds_bytes(P.n_views) : 0u;
    SceneRef sc = stage_scene<kTab, false>(S, lds, P.trav_mode, &V, P.n_views);
    /* per-view state: field f of view slot k of this thread at vs[(f * G + k) * kPB] */
    /* (runtime groups too large for LDS: the chunk's global per-view state, field-major, slot-minor) */
    const bool vs_glob = G <= 0 && B.vstate != nullptr;
    const uint32_t vs_stride = vs_glob ? P.vs_stride : (uint32_t) kPB;
    float *const vs = vs_glob ? B.vstate + (blockIdx.x * blockDim.x + threadIdx.x)
                              : reinterpret_cast<float *>(lds + vs_off) + threadIdx.x;
#if AMVPT_PRIM_SLOT_ORDER
    /* threads run in slot order (a wave = 64 pixels of one sample, see slot_lane), so every
     * record store of a wave is 64 contiguous slots; the hit and the ballots are read at the
     * lane (16-B loads 256 B apart) */
    const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = slot < P.chunk_n;
    const uint32_t i = ok ? slot_lane(P, slot) : 0u;
#else
    /* threads run in lane order (a wave = 4 pixels x 16 samples); records go to the
     * lane's slot (see slot_lane) */
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = i < P.chunk_n;
    const uint32_t slot = ok ? lane_slot(P, i) : 0u;
#endif
    if constexpr (kDiff) {
        mv_primary_lane<G, kTab, true, false>(P, S, sc, V, B, vs, vs_stride, slot, i, ok);
    } else if (kDW) {
        /* the waves whose primary hits are all plain diffuse (or misses): the all-diffuse body */
        if (wave_diffuse(P, S, sc, B, i, ok)) mv_primary_lane<G, kTab, true, true>(P, S, sc, V, B, vs, vs_stride, slot, i, ok);
    } else {
        /* the other waves (all of them without AMVPT_WAVE_DIFF) */
        if (!(AMVPT_WAVE_DIFF && wave_diffuse(P, S, sc, B, i, ok)))
            mv_primary_lane<G, kTab, false, false>(P, S, sc, V, B, vs, vs_stride, slot, i, ok);
    }
}


/* ------------------------------------------------------------------ */
/* k_splat_multi<G>: indirect accumulation + splats (mvpath_multi.h:343-368,44-76) */
/* ------------------------------------------------------------------ */

/* waves per SIMD the register allocation must allow: the 30-KB window admits 5 blocks (20 waves)
 * per CU, and 5 (<= 96 VGPRs) no longer spills (113.8 vs 117.9 ms per config-M frame, A/B r02z) */
#ifndef AMVPT_SPLAT_SKIP
#define AMVPT_SPLAT_SKIP 1   /* skip views without a valid splat in the wave (0: off, A/B) */
#endif
#ifndef AMVPT_SPLAT_BVW
#define AMVPT_SPLAT_BVW 1   /* all-diffuse waves form Bv * pdfW inside the view loop (0: hoisted by the compiler, A/B) */
#endif
#ifndef AMVPT_SPLAT_WAVES
#define AMVPT_SPLAT_WAVES 5
#endif
/* kRow: the row-reduced splat with wave windows (P.row_splat, RGBW), else the block window;
 * kWin = false (kRow only): the film is the whole quilt */
/* kRec = false: an instance without the record and debug paths (the bench's and every plain render's
 * row splat; 96 -> 95 VGPRs, no scratch, a third less code) */
template <int G, int C, bool kDiff, bool kRow, bool kWin = true, bool kRec = true>
__global__ void __launch_bounds__(kSplatBlock, AMVPT_SPLAT_WAVES) k_splat_multi(KParams P, const DView *V, Bufs B) {
    const bool rec_ = kRec && P.record != 0, dbg_ = kRec && P.debug != 0;
    __shared__ typename std::conditional<kRow, WaveLds<C>, SplatLds<C>>::type L;
    if (kRow) wave_lds_init(reinterpret_cast<WaveLds<C> &>(L));
    else splat_lds_init(reinterpret_cast<SplatLds<C> &>(L));
    /* one put of this kernel's kind */
    auto put = [&](float x, float y, const float *vals, bool valid, bool coalesce, int buf, uint32_t *fb) {
        if constexpr (kRow) {
            wave_put<C, kWin>(P, B.film, L, x, y, vals, valid, coalesce, fb);
        } else {
            /* deterministic mode runs these instances only (launch_splat) */
            if (P.film_fx) direct_put<C, kWin>(P, B.film, x, y, vals, valid, coalesce);
            else block_put<C>(P, B.film, L, buf, x, y, vals, valid, coalesce, fb);
        }
    };
    const uint32_t slot = blockIdx.x * kSplatBlock + threadIdx.x;
    const bool ok = slot < P.chunk_n;
    const uint32_t i = ok ? slot_lane(P, slot) : 0u;   /* chunk-local lane */
    const uint32_t n = P.chunk_n;
    float4 l0 = make_float4(0.f, 0.f, 0.f, 0.f), l1 = l0, l2 = l0, l3 = l0, lo = l0;
    if (ok) { l0 = B.lrec[0][slot]; l1 = B.lrec[1][slot]; l2 = B.lrec[2][slot]; l3 = B.lrec[3][slot]; lo = B.lane_out[slot]; }
    const int Gn = group_size<G>(P);
    const uint32_t lflags = fbits(l1.w);
    VMask<G> vmask = 0u, imask = 0u, smask = 0u;
    if constexpr (G <= 0) {
        constexpr int NP = mask_planes<G>(), NW = mask_words<G>();
        if (ok) { vmask = mload<NW>(B.lmask_w, slot); imask = mload<NW>(B.lmask_w + NP, slot); smask = mload<NW>(B.lmask_w + 2 * NP, slot); }
    } else {
        vmask = fbits(l2.w) & 0xffffu; imask = fbits(l2.w) >> 16; smask = lflags >> 16;
    }
    const float qnan = __builtin_nanf("");
    const float pdfW = l0.w;
    const C3 R0 = C3{l0.x, l0.y, l0.z}, Dp = C3{l1.x, l1.y, l1.z}, Bv = C3{l2.x, l2.y, l2.z};
    const f3 hp = mk(l3.x, l3.y, l3.z);
    if (ok && B.amask) B.amask[P.chunk_begin + i] = (lflags & LF_ADAPT) ? 1u : 0u;
    const bool valid_ray = (lflags & LF_VALIDRAY) || lo.w != 0.f;
    const bool mis = (lflags & LF_MIS) != 0, adapt_mask = (lflags & LF_ADAPT) != 0;
    const bool reuse = (lflags & LF_REUSE) != 0, direct = (lflags & LF_DIRECT) != 0;
    const C3 indirect = C3{lo.x, lo.y, lo.z};
    const float alpha = valid_ray ? 1.f : 0.f;
    const C3 res0 = R0 + indirect;   /* sa_mis = false: every view splats the primary's radiance */
    /* slot 0's position = the jittered sample (the lane's first two draws), aperture sample, and
     * the primary view (sample_ray_idx) -- recomputed, not stored */
    float sx = 0.f, sy = 0.f, apx = .5f, apy = .5f;
    uint32_t p_idx = 0;
    if (ok) {
        const uint32_t lane = lane_of(P, P.chunk_begin + i);
        int px, py;
        lane_pixel(P, lane, px, py);
        Pcg rng = lane_rng(P.seed_value, lane);
        const float jx = rng.next_1d(), jy = rng.next_1d();
        sx = (float) px + jx;
        sy = (float) py + jy;
        if (P.needs_ap) { apx = rng.next_1d(); apy = rng.next_1d(); }
        p_idx = sensor_index(P, fmadd(sx, P.inv_w, P.adj_ox), fmadd(sy, P.inv_h, P.adj_oy));
    }
    /* an all-diffuse wave of a mixed scene's generic stage (AMVPT_WAVE_DIFF) carries the compact
     * records (vrec_compact): the all-diffuse reads below, at run time */
    const bool kd = kDiff || (AMVPT_WAVE_DIFF && !wave_any(ok && !(lflags & LF_DIFFW)) && wave_any(ok));
    const float *const vw = kDiff ? reinterpret_cast<const float *>(B.vrec) : vrec_compact(B, Gn, n);
    const float4 *const vR = B.vrec, *const vB = B.vrec + (size_t) Gn * n;
    uint32_t splats = 0, fallback = 0, nonfinite = 0, negative = 0;   /* per lane, <= G each */
    uint32_t views_read = 0;   /* views the loop reads records of (wave-uniform) */
#pragma unroll 1
    for (int k = 0; k < Gn; ++k) {
        /* a view no lane of the wave splats into: no reprojection, no put (the lane record carries the
         * valid bits of every view, both record formats; records / debug mode write every view's entry) */
        if (AMVPT_SPLAT_SKIP && k > 0 && !rec_ && !dbg_) {
            /* wave windows skip per wave; the block window's put has block barriers, so its skip must be
             * block-uniform (a wave skipping alone would pair its next barriers with the wrong view's) */
            const bool any = kRow ? wave_any(ok && mget(vmask, k)) : __syncthreads_or(ok && mget(vmask, k));
            if (!any) continue;
        }
        ++views_read;
        const size_t o = (size_t) k * n + slot;
        float weight = 0.f;
        bool valid = false;
        C3 result = c3(0.f);
        float x = sx, y = sy;
        if (k > 0) {
            /* reprojected position in view k (camera_sample_surface, inactive -> 0) + quilt offset */
            const uint32_t id = group_view_n((uint32_t) Gn, p_idx, k);
            float ux = 0.f, uy = 0.f;
            view_uv(V, id, hp, apx, apy, ux, uy);
            x = reuse ? ux : 0.f;
            y = reuse ? uy : 0.f;
            uint32_t yy = id / P.gx, xx = id - yy * P.gx;
            if (P.rev_x) xx = (P.gx - 1) - xx;
            if (P.rev_y) yy = (P.gy - 1) - yy;
            x += (float) (xx * P.sres_x);
            y += (float) (yy * P.sres_y);
        }
        if (ok) {
            if (kd) {
                weight = vw[o];
                valid = mget(vmask, k);
                if (mis) {
                    /* cfma(0, emis_mis, 0) of a valid view whose wi.z <= 0 (kDiff, see k_mv_primary): three
                     * selects per view from the lane flags instead of three registers held across the view
                     * loop (the 5-wave allocation spilled them; the asm keeps the compiler from hoisting them) */
                    uint32_t lf = lflags;
                    asm volatile("" : "+v"(lf));
                    const C3 Dn = {(lf & 0x100u) ? qnan : 0.f, (lf & 0x200u) ? qnan : 0.f, (lf & 0x400u) ? qnan : 0.f};
                    result = k == 0 ? R0 : csel(direct && valid, csel(mget(smask, k), Dp, Dn), c3(0.f));
                    if (mget(imask, k)) {
#if AMVPT_SPLAT_BVW
                        /* Bv * pdfW formed here, per view: hoisted out of the view loop, the generic instance kept the
                         * three products in registers it did not have and spilled two of them (a scratch reload and
                         * wait per indirect view of every all-diffuse wave) */
                        float pw = pdfW;
                        asm volatile("" : "+v"(pw));
                        result = cfma(Bv * pw, indirect, result);
#else
                        result = cfma(Bv * pdfW, indirect, result);
#endif
                    }
                } else {
                    result = res0;
                }
            } else {
                /* the lane masks are the records' VF_VALID / VF_INDIRECT bits (k_mv_primary writes both from
                 * the same vmask / imask): a view's (result, weight) is read only when it splats (or is
                 * recorded), its BSDF value only when it adds the indirect term -- 32 B per view otherwise */
                valid = mget(vmask, k);
                const bool ind = mis && mget(imask, k);
                float4 r = make_float4(0.f, 0.f, 0.f, 0.f), bv = r;
                if (valid || rec_) r = vR[o];
                if (ind) bv = vB[o];
                weight = r.w;
                if (mis) {
                    result = C3{r.x, r.y, r.z};
                    if (ind) result = cfma(C3{bv.x, bv.y, bv.z} * pdfW, indirect, result);
                } else {
                    result = res0;
                }
            }
        }
        if (k == 0 && P.n_adapt && adapt_mask) weight = weight * P.adapt_w;
        C3 v = {weight * result.r, weight * result.g, weight * result.b};
        float vals[5];
        if (dbg_) {
            if (k > 0) break; /* uniform: every thread breaks at k == 1 */
            pack_vals(P, c3(adapt_mask ? 1.f : 0.f), alpha, 1.f, vals);
            put(x, y, vals, ok, true, 0, nullptr);
            continue;
        }
        pack_vals(P, v, alpha, weight, vals);
        check_sample(P, vals, valid, nonfinite, negative);
        put(x, y, vals, valid, k == 0, k & 1, &fallback);
        splats += valid ? 1 : 0;
        if (ok && rec_) {
            float *rr = B.records + ((size_t) i * Gn + k) * 8;
            rr[0] = x; rr[1] = y; rr[2] = v.r; rr[3] = v.g; rr[4] = v.b; rr[5] = alpha; rr[6] = weight;
            rr[7] = valid ? 1.f : 0.f;
        }
    }
    if (B.stats) {
        stat_add(B.stats, 3, splats); stat_add(B.stats, 4, fallback);
        stat_add(B.stats, 6, nonfinite); stat_add(B.stats, 7, negative);
        /* view-record bytes read: a weight per visited view (all-diffuse records), else (result, weight) per
         * valid view (every visited view when recording) and the BSDF value per indirect view */
        const uint32_t vb = !ok ? 0u : kd ? 4u * views_read
                                          : 16u * ((rec_ ? views_read : mpopc(vmask)) + (mis ? mpopc(imask) : 0u));
        stat_add(B.stats, 11, vb);
    }
}

/* develop: rgb / W (hdrfilm.cpp:400) */
AMVPT_TU_LOCAL __global__ void k_develop(const float *film, float *out, uint32_t npx, uint32_t alpha) {
    uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= npx) return;
    uint32_t C = alpha ? 5u : 4u, T = alpha ? 4u : 3u;
    const float *src = film + (size_t) p * C;
    float w = src[C - 1];
    float d = w == 0.f ? 1.f : w;
    for (uint32_t c = 0; c < T; ++c) out[(size_t) p * T + c] = src[c] / d;
}

/*
 * k_shadow launcher.  It is defined in its own translation unit (amvpt_shadow.hip
 * includes this file with AMVPT_SHADOW_TU), which is compiled WITH the SLP vectorizer:
 * k_shadow is the one kernel that is faster with it (71 vs 80 ms per config-M frame),
 * while the rest of this file is built with -fno-slp-vectorize (see Makefile).
 */
void launch_shadow(int walk, bool bin, dim3 grid, size_t lds, hipStream_t st, const KParams &P, const DScene *dS, const Bufs &B)
#ifdef AMVPT_SHADOW_TU
{
    if (bin && walk == WALK_LANE_TRI) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_LANE_TRI, true>), grid, dim3(256), lds, st, P, dS, B);
    else if (bin && walk == WALK_LANE_NS) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_LANE_NS, true>), grid, dim3(256), lds, st, P, dS, B);
    else if (bin && walk == WALK_LANE) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_LANE, true>), grid, dim3(256), lds, st, P, dS, B);
    else if (walk == WALK_BRUTE_NS) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_BRUTE_NS>), grid, dim3(256), lds, st, P, dS, B);
    else if (walk == WALK_BRUTE) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_BRUTE>), grid, dim3(256), lds, st, P, dS, B);
    else if (walk == WALK_UNI) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_UNI>), grid, dim3(256), lds, st, P, dS, B);
    else if (walk == WALK_LANE_TRI) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_LANE_TRI>), grid, dim3(256), lds, st, P, dS, B);
    else if (walk == WALK_LANE_NS) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_LANE_NS>), grid, dim3(256), lds, st, P, dS, B);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_shadow<WALK_LANE>), grid, dim3(256), lds, st, P, dS, B);
}
#else
;
#endif

/* A/B knobs: kernel-path choices fixed in release builds.  A build with -DAMVPT_AB_KNOBS (tools/ab.sh
 * variant libraries) reads them once from the environment; results are identical in every setting.
 * Per-call path selection for tests goes through amvpt_render_opts.flags instead. */
struct AbKnobs {
    bool fuse_prim = true, row_splat = true, brute = true, fuse_nee = true, fuse_suffix = true;
    uint32_t win_rs = AMVPT_WIN_RS, fused_blocks = AMVPT_FUSED_BLOCKS;
};
inline const AbKnobs &ab_knobs() {
    static const AbKnobs k = [] {
        AbKnobs r;
#ifdef AMVPT_AB_KNOBS
        auto off = [](const char *n) { const char *e = std::getenv(n); return e && e[0] == '0'; };
        r.fuse_prim = !off("AMVPT_FUSE_PRIM");
        r.row_splat = !off("AMVPT_ROW_SPLAT");
        r.brute = !off("AMVPT_BRUTE");
        r.fuse_nee = !off("AMVPT_FUSE_NEE");
        r.fuse_suffix = !off("AMVPT_FUSE_SUFFIX");
        if (const char *e = std::getenv("AMVPT_WIN_RS")) r.win_rs = (uint32_t) std::strtoul(e, nullptr, 0) % 32u;
        if (const char *e = std::getenv("AMVPT_FUSED_BLOCKS"))
            r.fused_blocks = std::max<uint32_t>(1, std::min<uint32_t>(64, (uint32_t) std::strtoul(e, nullptr, 0)));
#endif
        return r;
    }();
    return k;
}

/* Per-kernel HIP-event timing of an instrumented render (amvpt_counters given): an
 * event pair around every launch on the render stream, resolved in batches. */
#ifndef AMVPT_FLUSH_MARKS
#define AMVPT_FLUSH_MARKS 1
#endif
struct KTimer {
    static constexpr size_t kPairs = 128;
    bool on = false;
    hipError_t err = hipSuccess;
    hipEvent_t ev[2 * kPairs] = {};
    int kid[kPairs] = {};
    size_t n = 0;
    double ms[AMVPT_K_COUNT] = {};
    uint64_t launches[AMVPT_K_COUNT] = {};
    void init(bool enable) {
        on = enable;
        if (!on) return;
        for (auto &e : ev)
            if (err == hipSuccess) err = hipEventCreate(&e);
    }
    void flush() {
        if (!on || n == 0 || err != hipSuccess) return;
        for (size_t i = 0; i < n && err == hipSuccess; ++i) {
            err = hipEventSynchronize(ev[2 * i + 1]);   /* pairs may sit on either chunk stream */
            if (err != hipSuccess) break;
            float t = 0.f;
            err = hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]);
            ms[kid[i]] += t;
            launches[kid[i]] += 1;
        }
        n = 0;
    }
    void begin(int k, hipStream_t st) {
        if (!on || err != hipSuccess) return;
        if (n == kPairs) flush();
        kid[n] = k;
        err = hipEventRecord(ev[2 * n], st);
    }
    void end(hipStream_t st) {
        if (!on || err != hipSuccess) return;
        err = hipEventRecord(ev[2 * n + 1], st);
        ++n;
    }
    /* stage markers when not timing: a timing-enabled event record after each stage
     * (measured: a frame without them, or with hipEventDisableTiming markers, ran ~2 %
     * slower; AMVPT_FLUSH_MARKS A/B) */
    hipEvent_t mark_ev = nullptr;
    void mark(hipStream_t st) {
        if (on || !AMVPT_FLUSH_MARKS) return;
        if (!mark_ev && hipEventCreate(&mark_ev) != hipSuccess) return;
        (void) hipEventRecord(mark_ev, st);
    }
    ~KTimer() {
        for (auto &e : ev)
            if (e) (void) hipEventDestroy(e);
        if (mark_ev) (void) hipEventDestroy(mark_ev);
    }
};

/*
 * Group-size instances.  The G-dependent launchers (and the ~20 kernels each pulls in) are
 * explicitly instantiated in the translation units csrc/amvpt_group_*.hip (this file included
 * with AMVPT_GROUP_TU and AMVPT_GROUP_LIST), so the instances compile in parallel; this unit
 * only declares them.  k_prim_hit does not depend on G: its launcher lives here.
 */
void launch_prim_hit(bool uni, dim3 grid, size_t lds_bvh, hipStream_t st, const KParams &P, const DScene *S,
                     const DView *V, const Bufs &B)
#if !defined(AMVPT_SHADOW_TU) && !defined(AMVPT_GROUP_TU)
{
    if (uni) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit<true>), grid, dim3(256), lds_bvh, st, P, S, V, B);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit<false>), grid, dim3(256), lds_bvh, st, P, S, V, B);
}
#else
;
#endif
#ifdef AMVPT_GROUP_TU
template <int G> inline int group_size_host(const KParams &P) { return G > 0 ? G : (int) P.G; }
/* the primary wavefronts of one chunk: k_prim_hit -> k_prim_req -> k_vis -> k_mv_primary */
template <int G>
void launch_primary(uint32_t cn, size_t lds_tab, size_t lds_bvh, hipStream_t st, const KParams &P,
                           const DScene *S, const DView *V, const Bufs &B, bool tab, bool uni, bool diff, KTimer &T) {
    constexpr int kPB = prim_block<G>(), kVW = vis_waves<G>();
    const dim3 g256((cn + 255) / 256), g64((cn + 63) / 64), gp((cn + kPB - 1) / kPB);
    const size_t lds_view = B.vstate ? 0u : (size_t) (diff ? vs_fields<G, true>() : vs_fields<G, false>()) * group_size_host<G>(P) * kPB * sizeof(float);
    if (uni && ab_knobs().fuse_prim) {
        T.begin(AMVPT_K_PRIM_HIT, st);
        /* sphere-free scenes: the instances without float64 sphere code (the Cornell and mesh benches); scenes of
         * <= 64 spheres: the deferred sphere tests (P.sph, dgeom.h) */
        if (tab && diff && P.sph == 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, true, true, 0>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (tab && P.sph == 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, true, false, 0>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (tab && diff && P.sph == 2) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, true, true, 2>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (tab && P.sph == 2) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, true, false, 2>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (tab && diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, true, true>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (tab) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, true, false>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, false, true>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_hit_req<G, false, false>), g256, dim3(256), lds_tab, st, P, S, V, B);
        T.end(st);
    } else {
        T.begin(AMVPT_K_PRIM_HIT, st);
        launch_prim_hit(uni, g256, lds_bvh, st, P, S, V, B);
        T.end(st);
        T.begin(AMVPT_K_PRIM_REQ, st);
        if (tab && diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_req<G, true, true>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (tab) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_req<G, true, false>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else if (diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_req<G, false, true>), g256, dim3(256), lds_tab, st, P, S, V, B);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_prim_req<G, false, false>), g256, dim3(256), lds_tab, st, P, S, V, B);
        T.end(st);
    }
    T.begin(AMVPT_K_VIS, st);
    constexpr bool kVisPairs = vis_pairs<G, true>();
    const dim3 gvis = kVisPairs ? dim3((cn + 64 * AMVPT_VIS_RAYS - 1) / (64 * AMVPT_VIS_RAYS)) : g64;
    if (uni && P.sph == 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_vis<G, true, 0>), gvis, dim3(64 * kVW), lds_bvh, st, P, S, V, B);
    else if (uni && P.sph == 2) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_vis<G, true, 2>), gvis, dim3(64 * kVW), lds_bvh, st, P, S, V, B);
    else if (uni) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_vis<G, true>), gvis, dim3(64 * kVW), lds_bvh, st, P, S, V, B);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_vis<G, false>), g64, dim3(64 * kVW), lds_bvh, st, P, S, V, B);
    T.end(st);
    T.begin(AMVPT_K_MV_PRIMARY, st);
    if (tab && diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mv_primary<G, true, true>), gp, dim3(kPB), lds_tab + lds_view, st, P, S, V, B);
    else if (diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mv_primary<G, false, true>), gp, dim3(kPB), lds_tab + lds_view, st, P, S, V, B);
    else {
        if (AMVPT_WAVE_DIFF) {
            /* the all-diffuse waves first, with the all-diffuse body's smaller per-view LDS state */
            const size_t lds_dw = B.vstate ? 0u : (size_t) vs_fields<G, true>() * group_size_host<G>(P) * kPB * sizeof(float);
            if (tab) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mv_primary<G, true, false, true>), gp, dim3(kPB), lds_tab + lds_dw, st, P, S, V, B);
            else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mv_primary<G, false, false, true>), gp, dim3(kPB), lds_tab + lds_dw, st, P, S, V, B);
        }
        if (tab) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mv_primary<G, true, false>), gp, dim3(kPB), lds_tab + lds_view, st, P, S, V, B);
        else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_mv_primary<G, false, false>), gp, dim3(kPB), lds_tab + lds_view, st, P, S, V, B);
    }
    T.end(st);
}
template <int G>
void launch_splat(dim3 grid, hipStream_t st, const KParams &P, const DView *V, const Bufs &B, bool diff) {
    const bool row = AMVPT_WAVE_WIN && P.row_splat && P.C == 4 && !P.film_fx;   /* deterministic: direct puts */
    const bool whole = P.fx0 == 0u && P.fy0 == 0u && P.fw == P.W && P.fh == P.H;
    if (P.C == 5 && diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 5, true, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (P.C == 5) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 5, false, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (diff && row && whole && !P.record && !P.debug) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, true, true, false, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (row && whole && !P.record && !P.debug) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, false, true, false, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (diff && row && whole) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, true, true, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (row && whole) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, false, true, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (diff && row) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, true, true>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (row) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, false, true>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else if (diff) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, true, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
    else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_multi<G, 4, false, false>), grid, dim3(kSplatBlock), 0, st, P, V, B);
}
#define AMVPT_GROUP_INST(G_)                                                                                      \
    template void launch_primary<G_>(uint32_t, size_t, size_t, hipStream_t, const KParams &, const DScene *,            \
                                     const DView *, const Bufs &, bool, bool, bool, KTimer &);                          \
    template void launch_splat<G_>(dim3, hipStream_t, const KParams &, const DView *, const Bufs &, bool);
AMVPT_GROUP_LIST(AMVPT_GROUP_INST)
#undef AMVPT_GROUP_INST
#else
template <int G>
void launch_primary(uint32_t cn, size_t lds_tab, size_t lds_bvh, hipStream_t st, const KParams &P, const DScene *S,
                    const DView *V, const Bufs &B, bool tab, bool uni, bool diff, KTimer &T);
template <int G>
void launch_splat(dim3 grid, hipStream_t st, const KParams &P, const DView *V, const Bufs &B, bool diff);
#endif

#if !defined(AMVPT_SHADOW_TU) && !defined(AMVPT_GROUP_TU) && !defined(AMVPT_KERNEL_PROBE)
/* ------------------------------------------------------------------ */
/* Host orchestration                                                 */
/* ------------------------------------------------------------------ */

static void plan(const amvpt_params &P, uint32_t &spp, uint32_t &spp_pp, uint32_t &n_passes, uint64_t &L) {
    uint32_t s = P.spp ? P.spp : 1;
    uint64_t px = (uint64_t) P.film_width * P.film_height;
    if (P.integrator == AMVPT_INTEGRATOR_MVPATH) {
        spp_pp = P.spp_pass_lim ? std::min(P.spp_pass_lim, s) : s;
        n_passes = s / spp_pp;
        s = n_passes * spp_pp;
    } else {
        /* SamplingIntegrator::render (integrator.cpp:137-146): samples_per_pass travels in spp_pass_lim
         * (0 = unset); render_impl refuses an spp it does not divide, as the reference throws */
        spp_pp = P.spp_pass_lim ? std::min(P.spp_pass_lim, s) : s;
        n_passes = s / spp_pp;
    }
    uint64_t wf = px * spp_pp;
    if (wf > 0xffffffffull) {
        spp_pp /= (uint32_t) ((wf + 0xffffffffull - 1) / 0xffffffffull);
        n_passes = s / spp_pp;
        wf = px * spp_pp;
    }
    spp = s;
    L = wf;
}

static uint32_t group_size(const amvpt_params &P) {
    uint32_t N = P.n_views, G = std::min(P.reuse_count, N);
    if (G == 0 || N % G) {
        G = 0;
        for (uint32_t p = 8; p < N; p++) if (N % p == 0) { G = p; break; }
        if (!G) {
            for (uint32_t p = 8; p > 1; p--) if (N % p == 0) { G = p; break; }
            G = G ? G : N;
        }
        G = G ? G : N;
    }
    return G;
}

/* default_filter()'s literals, for the host-side check */
static const float kDefaultFilterHost[10] = {0x1.ff9d52p-1f, -0x1.fda5bcp+0f, 0x1.f4a20cp+0f, -0x1.3c9afep+0f,
                                             0x1.181032p-1f, -0x1.604b8ap-3f, 0x1.34c5d4p-5f, -0x1.657e54p-8f,
                                             0x1.e9dbd6p-12f, -0x1.2bffdp-16f};
static void gaussian_coeffs(float stddev, FilterCoeffs &f) {
    static const double cd[10] = {9.992604880e-1, -4.977025247e-1, 1.222248550e-1, -1.932406282e-2,
                                  2.136713061e-3, -1.679873860e-4, 9.202145248e-6, -3.329417433e-7,
                                  7.128382794e-9, -6.821193280e-11};
    f.radius = 4.f * stddev;
    double scale = 1;
    for (int i = 0; i < 10; ++i) {
        f.c[i] = (float) (cd[i] * scale);
        scale /= ((double) stddev * (double) stddev);
    }
    /* coeff[0] -= estrin(radius^2, coeff): same Estrin levels as the device */
    float x = f.radius * f.radius;
    const float *c = f.c;
    float r0 = std::fmaf(x, c[1], c[0]), r1 = std::fmaf(x, c[3], c[2]), r2 = std::fmaf(x, c[5], c[4]),
          r3 = std::fmaf(x, c[7], c[6]), r4 = std::fmaf(x, c[9], c[8]);
    float x2 = x * x;
    float q0 = std::fmaf(x2, r1, r0), q1 = std::fmaf(x2, r3, r2), q2 = r4;
    float x4 = x2 * x2;
    float w0 = std::fmaf(x4, q1, q0), w1 = q2;
    float x8 = x4 * x4;
    f.c[0] -= std::fmaf(x8, w1, w0);
}

/* roctx range over a host scope (the reference's ScopedPhase, profiler.h:20-110): the render,
 * each pass and each chunk's stages show up on rocprofv3's marker trace (--marker-trace) */
struct RoctxScope {
    explicit RoctxScope(const char *name) { roctxRangePushA(name); }
    ~RoctxScope() { roctxRangePop(); }
    RoctxScope(const RoctxScope &) = delete;
    RoctxScope &operator=(const RoctxScope &) = delete;
};

#define HIPCHK(x)                                                    \
    do {                                                             \
        hipError_t e_ = (x);                                         \
        if (e_ != hipSuccess) return hip_fail(#x, (int) e_);         \
    } while (0)

/*
 * Device buffers of amvpt_render, one set per device.  A render holds its device's
 * lock while it enqueues (calls from several host threads on one device serialise;
 * threads driving different devices run concurrently), and records `done` on its
 * stream when it returns: the next render waits on that event before it touches the
 * buffers (hipStreamWaitEvent when it runs on another stream), and a buffer is only
 * freed for a larger one after the event completed.
 */
constexpr int kMaxChunkStreams = 4;
struct DevArena {
    std::mutex mu;
    void *base = nullptr, *adapt = nullptr;
    size_t bytes = 0, abytes = 0;
    hipEvent_t done = nullptr;
    hipStream_t last = nullptr;
    bool pending = false;
    /* the other chunk streams (AMVPT_CHUNK_STREAMS > 1): created once per device; fork / join
     * order them after / before the render stream */
    hipStream_t side[kMaxChunkStreams - 1] = {};
    hipEvent_t fork = nullptr, join[kMaxChunkStreams - 1] = {};
    void *fx = nullptr;   /* deterministic mode's fixed-point film */
    size_t fxbytes = 0;
    void *carry = nullptr;   /* multi-pass stock path: two per-lane PCG32 state planes (rng_in / rng_out) */
    size_t cbytes = 0;
};
static std::mutex g_arenas_mu;
static std::map<int, std::unique_ptr<DevArena>> g_arenas;
static DevArena &dev_arena(int dev) {
    std::lock_guard<std::mutex> g(g_arenas_mu);
    std::unique_ptr<DevArena> &a = g_arenas[dev];
    if (!a) a.reset(new DevArena());
    return *a;
}
/* (re)allocate one of the arena's buffers; the previous contents may still be in use */
static amvpt_status arena_reserve(DevArena &A, void *&buf, size_t &have, size_t need, const char *what) {
    if (have >= need) return AMVPT_OK;
    if (buf) {
        if (A.pending) HIPCHK(hipEventSynchronize(A.done));
        (void) hipFree(buf);
    }
    buf = nullptr;
    have = 0;
    if (hipMalloc(&buf, need) != hipSuccess) {
        set_error(std::string("amvpt_render: device allocation of the ") + what + " failed");
        return AMVPT_ERR_OOM;
    }
    have = need;
    return AMVPT_OK;
}


static void launch_suffix_fused(bool tab, bool diff, int walk, dim3 grid, size_t lds, hipStream_t st, const KParams &P,
                                const DScene *S, const Bufs &B) {
#define AMVPT_FUSED(T_, D_)                                                                                           \
    do {                                                                                                              \
        if (walk == WALK_BRUTE_NS)                                                                                    \
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_suffix_fused<T_, D_, WALK_BRUTE_NS>), grid, dim3(256), lds, st, P, S, B); \
        else if (walk == WALK_BRUTE)                                                                                  \
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_suffix_fused<T_, D_, WALK_BRUTE>), grid, dim3(256), lds, st, P, S, B); \
        else if (AMVPT_FUSE_BVH && walk == WALK_UNI)                                                                  \
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_suffix_fused<T_, D_, WALK_UNI>), grid, dim3(256), lds, st, P, S, B); \
        else if (AMVPT_FUSE_BVH)                                                                                      \
            hipLaunchKernelGGL(HIP_KERNEL_NAME(k_suffix_fused<T_, D_, WALK_LANE>), grid, dim3(256), lds, st, P, S, B); \
    } while (0)
    if (tab && diff) AMVPT_FUSED(true, true);
    else if (tab) AMVPT_FUSED(true, false);
    else if (diff) AMVPT_FUSED(false, true);
    else AMVPT_FUSED(false, false);
#undef AMVPT_FUSED
}

static void launch_bounce(bool tab, bool diff, int nee_walk, dim3 grid, size_t lds, hipStream_t st, const KParams &P,
                          const DScene *S, const Bufs &B) {
#define AMVPT_BOUNCE(T_, D_, N_) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_bounce<T_, D_, N_>), grid, dim3(256), lds, st, P, S, B)
#define AMVPT_BOUNCE_N(T_, D_)                                            \
    do {                                                                 \
        if (nee_walk == WALK_BRUTE_NS) AMVPT_BOUNCE(T_, D_, WALK_BRUTE_NS); \
        else if (nee_walk == WALK_BRUTE) AMVPT_BOUNCE(T_, D_, WALK_BRUTE);  \
        else AMVPT_BOUNCE(T_, D_, -1);                                    \
    } while (0)
    if (tab && diff) AMVPT_BOUNCE_N(true, true);
    else if (tab) AMVPT_BOUNCE_N(true, false);
    else if (diff) AMVPT_BOUNCE_N(false, true);
    else AMVPT_BOUNCE_N(false, false);
#undef AMVPT_BOUNCE_N
#undef AMVPT_BOUNCE
}


typedef void (*primary_fn)(uint32_t, size_t, size_t, hipStream_t, const KParams &, const DScene *, const DView *,
                           const Bufs &, bool, bool, bool, KTimer &);
typedef void (*splat_fn)(dim3, hipStream_t, const KParams &, const DView *, const Bufs &, bool);
/* group sizes 2..16: the per-view bit masks (k_prim_req's request bits below the view index at
 * bit 16, k_mv_primary's valid / indirect flags at bits k and 16 + k) hold 16 views; entry 0 is
 * the runtime instance for 17..256 views (256-bit masks in vreq_w / lmask_w), entry 1 the one for
 * 257..1024 views (1024-bit masks) */
static const primary_fn kPrimary[] = {launch_primary<0>, launch_primary<-1>, launch_primary<2>, launch_primary<3>, launch_primary<4>,
                                      launch_primary<5>, launch_primary<6>, launch_primary<7>, launch_primary<8>,
                                      launch_primary<9>, launch_primary<10>, launch_primary<11>, launch_primary<12>,
                                      launch_primary<13>, launch_primary<14>, launch_primary<15>, launch_primary<16>};
static const splat_fn kSplat[] = {launch_splat<0>, launch_splat<-1>, launch_splat<2>, launch_splat<3>, launch_splat<4>,
                                  launch_splat<5>, launch_splat<6>, launch_splat<7>, launch_splat<8>,
                                  launch_splat<9>, launch_splat<10>, launch_splat<11>, launch_splat<12>,
                                  launch_splat<13>, launch_splat<14>, launch_splat<15>, launch_splat<16>};
constexpr uint32_t kMaxG = 16;
static uint32_t dispatch_g(uint32_t G) { return G > kMaxGWide ? 1u : G > kMaxG ? 0u : G; }
/*
 * The adaptive fill's compaction (dr::compress, mvpath_multi.h:79-88): the virtual indices of the pass's
 * adapt_mask lanes, in lane order, in ONE pass over the mask with decoupled look-back.
 *  - A block takes the next tile of kSelTile lanes by ticket (one returning atomic per block), so every earlier
 *    tile belongs to a block that is already running and will publish: the look-back always ends.
 *  - Each thread reads 16 mask bytes (one 16-B load) into a 16-bit flag word; a wave inclusive scan of the
 *    per-thread counts and a 4-wave sum in LDS give the block's count and every thread's offset in it.
 *  - The block publishes its count (kSelAgg), then wave 0 reads the predecessors' status words 64 tiles per
 *    step (a ballot finds the nearest published inclusive prefix, kSelInc; an unpublished word in front of it
 *    is read again) and sums them; the tile publishes its inclusive prefix.
 *  - Every thread writes its flagged lanes' indices at tile prefix + wave prefix + thread prefix: ascending
 *    lane order, as dr::compress keeps it.  The last tile writes the total.
 * Status words are 64-bit (2 flag bits, 62 value bits), zeroed with the ticket before the launch.
 */
constexpr uint32_t kSelTile = 256 * 16;
constexpr unsigned long long kSelAgg = 1ull << 62, kSelInc = 2ull << 62, kSelVal = kSelAgg - 1;
AMVPT_TU_LOCAL __global__ void __launch_bounds__(256) k_select_flagged(const uint8_t *amask, uint64_t n, uint32_t *out,
                                                                      uint32_t *count, unsigned long long *status,
                                                                      uint32_t *ticket, uint32_t n_tiles) {
    __shared__ uint32_t s_tile, s_wave[4];
    __shared__ unsigned long long s_prefix;
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t base = (uint64_t) tile * kSelTile + (uint64_t) threadIdx.x * 16u;
    uint32_t bits = 0;   /* bit i: lane base + i is flagged */
    if (base + 16 <= n) {
        const uint4 q = *reinterpret_cast<const uint4 *>(amask + base);
        const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int b = 0; b < 4; ++b) bits |= (((w[k] >> (8 * b)) & 0xffu) != 0u ? 1u : 0u) << (4 * k + b);
    } else {
        for (int i = 0; i < 16; ++i)
            if (base + i < n && amask[base + i]) bits |= 1u << i;
    }
    const uint32_t c = (uint32_t) __builtin_popcount(bits);
    const int lane = (int) __lane_id(), wave = (int) (threadIdx.x >> 6);
    uint32_t inc = c;   /* wave inclusive scan */
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t wpre = 0, total = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t t = s_wave[k];
        wpre += k < wave ? t : 0u;
        total += t;
    }
    if (wave == 0) {
        unsigned long long excl = 0;
        if (tile == 0) {
            if (lane == 0) __hip_atomic_store(status, kSelInc | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0) __hip_atomic_store(status + tile, kSelAgg | total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = (int64_t) tile - 1;   /* the nearest predecessor not summed yet */
            for (;;) {
                const int64_t t = j - lane;
                const unsigned long long v =
                    t >= 0 ? __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kSelInc;
                const unsigned long long inc_m = __ballot((v >> 62) == 2ull), zero_m = __ballot((v >> 62) == 0ull);
                /* lanes up to and including the nearest inclusive prefix (all 64 when there is none) */
                const unsigned long long upto = inc_m ? ((inc_m & (~inc_m + 1ull)) << 1) - 1ull : ~0ull;
                if (zero_m & upto) continue;   /* a predecessor has not published yet: read again */
                excl += wave_sum(((upto >> lane) & 1ull) ? (v & kSelVal) : 0ull);
                if (inc_m) break;
                j -= 64;
            }
            if (lane == 0) __hip_atomic_store(status + tile, kSelInc | (excl + total), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            s_prefix = excl;
            if (tile == n_tiles - 1) *count = (uint32_t) (excl + total);
        }
    }
    __syncthreads();
    uint32_t o = (uint32_t) s_prefix + wpre + (inc - c);
    while (bits) {
        const int i = __builtin_ctz(bits);
        bits &= bits - 1u;
        out[o++] = (uint32_t) (base + (uint64_t) i);
    }
}

/* adaptive fill: flagged lanes of each run of a rectangular lane set (one block per run) */
AMVPT_TU_LOCAL __global__ void __launch_bounds__(256) k_run_counts(const uint8_t *amask, uint32_t run_len, uint32_t *counts) {
    __shared__ unsigned long long part[4];
    const uint8_t *m = amask + (size_t) blockIdx.x * run_len;
    unsigned long long c = 0;
    for (uint32_t i = threadIdx.x; i < run_len; i += blockDim.x) c += m[i];
    c = wave_sum(c);
    if (__lane_id() == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = (uint32_t) (part[0] + part[1] + part[2] + part[3]);
}

/* deterministic mode: film += fixed-point sums (one thread per float, a fixed conversion per cell) */
AMVPT_TU_LOCAL __global__ void k_fixed_resolve(float *film, const unsigned long long *fx, uint64_t n) {
    const uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    film[i] += (float) ((double) (long long) fx[i] * (1.0 / kFixScale));
}

amvpt_status render_impl(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                         const amvpt_lane_set &lanes, const amvpt_film_window &fwin, void *stream,
                         const amvpt_render_opts &opts, amvpt_counters *counters, float *records,
                         uint32_t record_pass) {
    float *const film = fwin.film;
    if (!scene || !views || !params || !film) { set_error("amvpt_render: null argument"); return AMVPT_ERR_INVALID; }
    RoctxScope range_render("amvpt_render");
    const amvpt_params &Pp = *params;
    hipStream_t st = (hipStream_t) stream;
    const AbKnobs &K = ab_knobs();
    const bool diffuse_spec = !(opts.flags & AMVPT_OPT_GENERIC_KERNELS);
    const uint32_t trav = opts.traversal;
    if (trav > 2) { set_error("amvpt_render: traversal must be 0 (auto), 1 (wave-uniform) or 2 (per-lane)"); return AMVPT_ERR_INVALID; }
    if (Pp.n_views == 0) { set_error("amvpt_render: n_views == 0"); return AMVPT_ERR_INVALID; }
    if (Pp.multisensor && !Pp.batch && Pp.n_views != Pp.grid_x * Pp.grid_y) {
        set_error("amvpt_render: a grid MultiSensor needs n_views == grid_x * grid_y");
        return AMVPT_ERR_INVALID;
    }
    if (Pp.multisensor && Pp.batch && (Pp.grid_y != 1 || Pp.grid_x != Pp.n_views)) {
        set_error("amvpt_render: a batch MultiSensor needs grid_x == n_views and grid_y == 1");
        return AMVPT_ERR_INVALID;
    }
    uint32_t spp, spp_pp, n_passes;
    uint64_t L;
    plan(Pp, spp, spp_pp, n_passes, L);
    const bool is_mv = Pp.integrator == AMVPT_INTEGRATOR_MVPATH;
    const bool reuse = is_mv && Pp.sa_reuse && Pp.n_views > 1 && Pp.reuse_count != 1;
    const uint32_t G = reuse ? group_size(Pp) : 1;
    if (G > kMaxGHuge) { set_error("amvpt_render: group size > 1024 not implemented"); return AMVPT_ERR_UNSUPPORTED; }
    const uint32_t n_adapt = reuse ? std::min(Pp.adaptive, G - 1) : 0;
    if (!is_mv && Pp.spp_pass_lim && (Pp.spp ? Pp.spp : 1) % std::min(Pp.spp_pass_lim, Pp.spp ? Pp.spp : 1u)) {
        set_error("sample_count (" + std::to_string(Pp.spp ? Pp.spp : 1) + ") must be a multiple of spp_per_pass (" +
                  std::to_string(std::min(Pp.spp_pass_lim, Pp.spp ? Pp.spp : 1u)) + ").");
        return AMVPT_ERR_INVALID;
    }
    /* the stock path's passes continue each lane's sampler (rng_in / rng_out) */
    const bool rng_carry = !is_mv && n_passes > 1;
    if (Pp.multisensor && (Pp.grid_x == 0 || Pp.grid_y == 0 || Pp.film_width % Pp.grid_x || Pp.film_height % Pp.grid_y)) {
        set_error("Film size must be divisible by grid dimensions !");
        return AMVPT_ERR_INVALID;
    }
    for (uint32_t v = 0; v < Pp.n_views; ++v)
        if (views[v].type != AMVPT_CAMERA_PERSPECTIVE && views[v].type != AMVPT_CAMERA_THINLENS) {
            set_error("amvpt_render: unknown camera type");
            return AMVPT_ERR_INVALID;
        }
    /* ---- lane set: contiguous [lane_begin, lane_end), or a pixel rectangle (runs of pixel rows) ---- */
    const uint32_t QW = Pp.film_width, QH = Pp.film_height;
    bool rect = lanes.rect_width != 0;
    uint64_t lane_begin = lanes.lane_begin, lane_end = lanes.lane_end;
    uint32_t rx0 = 0, ry0 = 0, rw = 0, rh = 0;
    if (rect) {
        rx0 = lanes.rect_x0; ry0 = lanes.rect_y0; rw = lanes.rect_width; rh = lanes.rect_height;
        if ((uint64_t) rx0 + rw > QW || (uint64_t) ry0 + rh > QH) {
            set_error("amvpt_render: lane rectangle outside the quilt");
            return AMVPT_ERR_INVALID;
        }
        /* whole pixel rows are one contiguous range */
        if (rx0 == 0 && rw == QW) {
            rect = false;
            lane_begin = (uint64_t) ry0 * QW * spp_pp;
            lane_end = (uint64_t) (ry0 + rh) * QW * spp_pp;
        } else {
            lane_begin = 0;
            lane_end = (uint64_t) rw * rh * spp_pp;   /* virtual span */
        }
    }
    if (!rect && lane_end > L) lane_end = L;
    const uint64_t span = lane_begin < lane_end ? lane_end - lane_begin : 0;
    const uint32_t n_runs = span == 0 ? 0u : (rect ? rh : 1u);
    /* ---- film window ---- */
    if ((uint64_t) fwin.x0 + fwin.width > QW || (uint64_t) fwin.y0 + fwin.height > QH) {
        set_error("amvpt_render: film window outside the quilt");
        return AMVPT_ERR_INVALID;
    }
    const bool whole_film = fwin.x0 == 0 && fwin.y0 == 0 && fwin.width == QW && fwin.height == QH;
    const bool deterministic = (opts.flags & AMVPT_OPT_DETERMINISTIC) != 0;
    if (deterministic && !whole_film) {
        set_error("amvpt_render: AMVPT_OPT_DETERMINISTIC needs a whole-quilt film window");
        return AMVPT_ERR_UNSUPPORTED;
    }
    if (!whole_film && !fwin.overflow) {
        set_error("amvpt_render: a film window smaller than the quilt needs an overflow list");
        return AMVPT_ERR_INVALID;
    }
    /* the adaptive fill compacts the whole pass (its RNG seeds depend on the global
     * wavefront): a partial lane set needs the host's count exchange */
    const bool do_fill = n_adapt && !Pp.debug;
    const bool partial = rect || lane_begin != 0 || lane_end != L;
    const amvpt_run_exchange_fn exchange = opts.exchange;
    void *const exchange_ctx = opts.exchange_ctx;
    if (do_fill && partial && !exchange) {
        set_error("amvpt_render: adaptive > 0 over a lane range needs amvpt_set_adaptive_exchange "
                  "(or the whole frame: lane_begin = 0, lane_end = all lanes)");
        return AMVPT_ERR_UNSUPPORTED;
    }
    if (span == 0) {
        /* an empty lane set still takes part in every pass's count exchange (an all-gather on
         * the host side: the other ranks would wait for it forever) */
        if (do_fill && partial)
            for (uint32_t pass = 0; pass < n_passes; ++pass) {
                uint64_t total = 0;
                if (exchange(exchange_ctx, 0, nullptr, nullptr, nullptr, &total) != 0) {
                    set_error("amvpt_render: adaptive count exchange failed");
                    return AMVPT_ERR_INVALID;
                }
            }
        if (counters) *counters = amvpt_counters{};
        return AMVPT_OK;
    }

    KParams P{};
    P.W = Pp.film_width; P.H = Pp.film_height; P.C = Pp.film_alpha ? 5 : 4;
    P.spp_pp = spp_pp;
    uint32_t log_spp = 0;
    while ((1u << log_spp) < spp_pp) ++log_spp;
    P.log_spp = log_spp;
    P.pow2 = (1u << log_spp) == spp_pp;
    P.max_depth = Pp.max_depth; P.rr_depth = Pp.rr_depth;
    P.sa_mis = Pp.sa_mis; P.fast_mis = Pp.fast_mis; P.debug = Pp.debug; P.n_adapt = n_adapt;
    P.G = G;
    P.multisensor = Pp.multisensor; P.batch = Pp.batch; P.n_views = Pp.n_views;
    /* grid: its first sub-sensor decides (grid.cpp:228); batch: any child (batch.cpp:127) */
    P.needs_ap = 0;
    for (uint32_t v = 0; v < (Pp.multisensor && Pp.batch ? Pp.n_views : 1u); ++v)
        P.needs_ap |= views[v].type == AMVPT_CAMERA_THINLENS ? 1u : 0u;
    P.gx = Pp.grid_x ? Pp.grid_x : 1; P.gy = Pp.grid_y ? Pp.grid_y : 1;
    P.rev_x = Pp.reverse_x; P.rev_y = Pp.reverse_y;
    /* quilt tile pitch of reprojected views: film->size() / grid (mvpath_multi.h:62), the full film */
    const uint32_t fullW = Pp.full_width ? Pp.full_width : P.W, fullH = Pp.full_height ? Pp.full_height : P.H;
    P.sres_x = fullW / P.gx; P.sres_y = fullH / P.gy;
    P.box = Pp.rfilter == AMVPT_RFILTER_BOX;
    P.coalesce_single = spp_pp >= 4;
    P.path_box_pos = (!is_mv && P.box) ? 1 : 0;
    P.is_mvpath = is_mv;
    P.inv_w = 1.f / (float) P.W;
    P.inv_h = 1.f / (float) P.H;
    P.off_x = Pp.crop_offset_x; P.off_y = Pp.crop_offset_y;
    P.adj_ox = -(float) P.off_x * P.inv_w;   /* -ScalarVector2f(crop_offset) * scale */
    P.adj_oy = -(float) P.off_y * P.inv_h;
    P.nc_ox = (float) (-(int) P.off_x) - .5f;
    P.nc_oy = (float) (-(int) P.off_y) - .5f;
    P.adapt_w = 1.f / (float) (n_adapt + 1);
    P.trav_mode = trav;
    P.box_screen = (opts.flags & AMVPT_OPT_NO_BOX_SCREEN) ? 0u : 1u;
    for (int a = 0; a < 3; ++a) {
        const float ext = scene->root_hi[a] - scene->root_lo[a];
        P.bin_lo[a] = scene->root_lo[a];
        P.bin_scale[a] = ext > 0.f ? (float) (1u << kBinCellBits) / ext : 0.f;
    }
    P.sph = !scene->has_spheres ? 0u : (AMVPT_SPHERE_DEFER && scene->n_sph <= 64u) ? 2u : 1u;
    P.win_rs = K.win_rs;
    P.range_begin = rect ? 0 : lane_begin;
    P.rect = rect ? 1u : 0u;
    P.rect_x0 = rx0; P.rect_y0 = ry0;
    P.run_len = rect ? rw * spp_pp : 0u;
    P.fx0 = fwin.x0; P.fy0 = fwin.y0; P.fw = fwin.width; P.fh = fwin.height;
    P.overflow = whole_film ? nullptr : fwin.overflow;
    P.ov_cap = whole_film ? 0 : fwin.overflow_capacity;
    /* the list's count before this render: renders append (amvpt_film_window), film_overflow reports the
     * cells this one added */
    uint64_t overflow_before = 0, overflow_added = 0;
    if (P.overflow) {
        HIPCHK(hipMemcpyAsync(&overflow_before, P.overflow, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    P.valid_ray0 = (!Pp.hide_emitters && scene->dev.environment >= 0) ? 1u : 0u;
    if (!P.box) gaussian_coeffs(Pp.rfilter_stddev, P.filt);
    /* row-reduced splat (row_put): RGBW film, Gaussian filter, >= 16 samples per pixel and pass
     * (a 16-lane row = one pixel); AMVPT_ROW_SPLAT=0 keeps the per-lane splat (A/B) */
    {
        /* ... and the default Gaussian (its coefficients are literals in the row kernels, default_filter) */
        FilterCoeffs d;
        gaussian_coeffs(0.5f, d);
        const bool def_filt = !P.box && std::memcmp(&d, &P.filt, sizeof(d)) == 0 &&
                              std::memcmp(&d.c[0], &kDefaultFilterHost[0], sizeof(d.c)) == 0;
        P.row_splat = (K.row_splat && P.C == 4 && def_filt && P.pow2 && spp_pp >= 16) ? 1u : 0u;
    }
    /* tiled slots: whole 4-row bands of a quilt row width divisible by 4, 16 samples per pixel and pass,
     * contiguous lane sets whose chunks start and end on band boundaries */
    {
        const uint64_t band = 4ull * QW * 16ull;
        P.tile_w = (AMVPT_TILE_SLOTS && P.row_splat && spp_pp == 16 && QW % 4 == 0 && !rect && lane_begin % band == 0 &&
                    span % band == 0 && span <= 0xffffffffull) ? QW : 0u;
    }

    /* views to device (tiny) */
    std::vector<DView> hv(Pp.n_views);
    for (uint32_t v = 0; v < Pp.n_views; ++v) {
        const amvpt_view_desc &d = views[v];
        DView &o = hv[v];
        std::memcpy(o.to_world, d.to_world, 12 * sizeof(float));
        std::memcpy(o.to_world_inv, d.to_world_inv, 12 * sizeof(float));
        std::memcpy(o.sample_to_camera, d.sample_to_camera, 16 * sizeof(float));
        std::memcpy(o.camera_to_sample, d.camera_to_sample, 16 * sizeof(float));
        o.near_clip = d.near_clip; o.far_clip = d.far_clip; o.normalization = d.normalization; o.pad0 = 0.f;
        o.res[0] = d.resolution[0]; o.res[1] = d.resolution[1];
        o.pp[0] = d.pp_offset[0]; o.pp[1] = d.pp_offset[1];
        o.type = d.type;
        o.aperture_radius = d.aperture_radius;
        o.focus_distance = d.focus_distance;
        o.pad1 = 0.f;
    }

    /* lane arena: queues (2 x 5 x 16 B), lane_out + hit (32 B), NEE queue (52 B), visibility requests
     * (48 B), lane records (64 B), view records (4 B x G all-diffuse, else 32 B x G), ballots (G / 8 B) */
    const bool wide = G > kMaxG;   /* the runtime group-size instances (256- / 1024-bit view masks) */
    const int mplanes = G > kMaxGWide ? mask_planes<-1>() : mask_planes<0>();   /* uint4 planes per mask */
    const bool diff_rec = scene->all_diffuse && diffuse_spec && !wide;   /* kDiff instances, compact view records */
    /* the runtime instance's per-view state: LDS (64-thread blocks) while it fits, else a global
     * VS_FIELDS x G float plane per lane */
    const size_t lds_tab_views = (AMVPT_PRIM_TAB && tables_staged(scene->dev, Pp.n_views))
                                     ? scene->dev.tab_bytes + views_lds_bytes(Pp.n_views) : 0u;
    const bool vs_global = wide && lds_tab_views + (size_t) VS_FIELDS * G * 64 * sizeof(float) > 65536;
    const size_t per_lane = 2 * kQPlanes * 16 + 32 + 52 + 48 + 64 + 32 + 8 + 6 /* binned rays, binned NEE results, keys */ +
                            (size_t) (diff_rec ? 4 : (AMVPT_WAVE_DIFF ? 36 : 32)) * G + (G + 7) / 8 +
                            (wide ? (size_t) 4 * 16 * mplanes : 0) + (vs_global ? (size_t) VS_FIELDS * 4 * G : 0);
    uint64_t chunk_max = opts.chunk_lanes ? std::max<uint64_t>(256, opts.chunk_lanes) : 0;
    if (chunk_max == 0) {
        chunk_max = 1ull << 26;
        while (chunk_max > (1ull << 16) && chunk_max * per_lane > (48ull << 30)) chunk_max >>= 1;
    }
    uint64_t chunk = std::min<uint64_t>(chunk_max, span);
    const size_t views_bytes = ((hv.size() * sizeof(DView)) + 255) & ~(size_t) 255;
    /* one partition holds the pushes of every kQParts-th producer block (<= 256 lanes each) */
    auto qcap_of = [](uint64_t c) { return (uint32_t) (((c + kQParts - 1) / kQParts + 512 + 63) & ~(uint64_t) 63); };
    const size_t stats_bytes = (size_t) kStats * kStatShards * 8, cnt_bytes = (size_t) 3 * kQParts * kCntStride * 4;
    const bool tab_b = AMVPT_BOUNCE_TAB && tables_staged(scene->dev, 0), tab_p = AMVPT_PRIM_TAB && tables_staged(scene->dev, Pp.n_views);
    const bool uni = scene_uniform(scene->dev.n_nodes, trav);
    /* the coherent primary and visibility rays walk wave-uniformly on every BVH in automatic mode
     * (AMVPT_COH_UNI, see launch_primary); the incoherent suffix rays keep the per-lane walk */
    const bool uni_coh = uni || (AMVPT_COH_UNI && trav == 0u);
    /* suffix walk: brute force for tiny scenes in auto mode */
    int walk = uni ? WALK_UNI : (scene->has_spheres || !AMVPT_LANE_NS) ? WALK_LANE
                              : (scene->bvh_tri_only && AMVPT_LANE_TRI) ? WALK_LANE_TRI : WALK_LANE_NS;
    if (uni && trav == 0u && K.brute && scene->dev.n_prims <= kBrutePrims) walk = scene->has_spheres ? WALK_BRUTE : WALK_BRUTE_NS;
    const bool diff = diff_rec;                                                                           /* kDiff instances */
    /* NEE traced inside k_bounce (brute-force walks; AMVPT_OPT_SPLIT_NEE keeps k_shadow) */
    const bool fuse_nee = (walk == WALK_BRUTE || walk == WALK_BRUTE_NS) && K.fuse_nee && !(opts.flags & AMVPT_OPT_SPLIT_NEE);
    /* the whole suffix in one launch, paths in registers (brute-force walks with fused NEE;
     * AMVPT_OPT_WAVEFRONT_SUFFIX keeps the per-depth k_extend / k_bounce wavefronts) */
    const bool fuse_suffix = (fuse_nee || (AMVPT_FUSE_BVH && K.fuse_nee && !(opts.flags & AMVPT_OPT_SPLIT_NEE))) &&
                             K.fuse_suffix && !(opts.flags & AMVPT_OPT_WAVEFRONT_SUFFIX);
    /* chunks of the per-depth wavefront suffix (BVH scenes) take turns over up to four buffer sets on as many
     * streams (the render stream and the arena's side streams): one chunk's short deep-bounce launches and
     * tails leave CUs idle that the other chunks' kernels fill (mesh 550 -> 599 Msamples/s with two, round 2;
     * 967 -> 1001 with four, r05zi).  The
     * fused-suffix scenes gain 0.0-0.5 % (r03i) and keep one stream, so their per-kernel HIP-event
     * times are not overlapped (AMVPT_OPT_ONE_STREAM forces one stream everywhere) */
    /* ray binning (k_bin_sort) for the per-lane suffix walks of BVHs read from device memory */
    const bool lane_walk = (walk == WALK_LANE || walk == WALK_LANE_NS || walk == WALK_LANE_TRI) && !fuse_suffix && scene_lds_bytes(scene->dev, trav) == 0u;
    const bool bin_ext = lane_walk && (AMVPT_BIN & 1) && !(opts.flags & AMVPT_OPT_NO_BINNING);
    const bool bin_nee = lane_walk && (AMVPT_BIN & 2) && !fuse_nee && !(opts.flags & AMVPT_OPT_NO_BINNING);
    auto set_bytes_of = [&](uint64_t c) {
        return cnt_bytes + per_lane * std::max<uint64_t>(c, (uint64_t) qcap_of(c) * kQParts) + 8192;
    };
    /* as many buffer sets as chunk streams, at most one per chunk of the render (chunk i on set i mod n across
     * the passes) and 192 GB of sets in all */
    auto sets_for = [&](uint64_t c) {
        int n = (AMVPT_CHUNK_STREAMS > 1 && span > c && (!fuse_suffix || AMVPT_FUSED_TWO_STREAMS) &&
                 !(opts.flags & AMVPT_OPT_ONE_STREAM)) ? std::min(AMVPT_CHUNK_STREAMS, kMaxChunkStreams) : 1;
        n = (int) std::min<uint64_t>((uint64_t) n, (uint64_t) n_passes * ((span + c - 1) / c));
        while (n > 2 && set_bytes_of(c) * (size_t) n > (192ull << 30)) --n;
        return n;
    };
    int n_sets = sets_for(chunk);
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    DevArena &A = dev_arena(dev);
    std::unique_lock<std::mutex> arena_lock(A.mu);
    if (!A.done) HIPCHK(hipEventCreateWithFlags(&A.done, hipEventDisableTiming));
    /* the previous render's buffers may still be in flight on another stream */
    if (A.pending && A.last != st) HIPCHK(hipStreamWaitEvent(st, A.done, 0));
    /* every return below joins the side streams into this one and records `done` (also the error paths) */
    struct ArenaRelease {
        DevArena &A; hipStream_t st; int n_side; bool side = false;
        void join() {
            if (!side) return;
            side = false;
            for (int k = 0; k < n_side; ++k)
                if (hipEventRecord(A.join[k], A.side[k]) == hipSuccess) (void) hipStreamWaitEvent(st, A.join[k], 0);
        }
        ~ArenaRelease() {
            join();
            if (hipEventRecord(A.done, st) == hipSuccess) { A.pending = true; A.last = st; }
        }
    } arena_release{A, st, 0};
    /* Device-memory budget (ABI 10; the reference bounds a pass's memory with spp_pass_lim and its wavefront
     * cap, mvpath.cpp:36-41,133-147): opts.budget_mib, else this device's free memory plus what the arena
     * already holds, less max(2 GiB, 1/64 of the device).  Sizing drops chunk streams' buffer sets first, then
     * halves the chunk (records and films do not depend on either); a failing allocation takes the same steps
     * before the render reports AMVPT_ERR_OOM. */
    const size_t held = A.bytes + A.abytes + A.fxbytes + A.cbytes;
    size_t budget = 0;
    if (opts.budget_mib) {
        budget = (size_t) opts.budget_mib << 20;
    } else {
        size_t fr = 0, tot = 0;
        HIPCHK(hipMemGetInfo(&fr, &tot));
        const size_t headroom = std::max<size_t>(2ull << 30, tot / 64);
        budget = fr + held > headroom ? fr + held - headroom : 0;
    }
    /* the span-sized buffers below (deterministic film, sampler states, adaptive fill) */
    const size_t other_need = (deterministic ? (size_t) QW * QH * (Pp.film_alpha ? 5 : 4) * 8 : 0) +
                              (rng_carry ? (size_t) 16 * span : 0) + (do_fill ? (size_t) 6 * span + (1u << 20) : 0);
    const uint64_t min_chunk = std::min<uint64_t>(span, 1ull << 16);
    auto need_of = [&](uint64_t c, int n) { return views_bytes + stats_bytes + set_bytes_of(c) * (size_t) n; };
    auto shrink = [&]() {   /* one step down: a buffer set less, then half the chunk (256-lane multiples) */
        if (n_sets > 1) { --n_sets; return true; }
        if (chunk <= min_chunk) return false;
        chunk = std::max<uint64_t>(min_chunk, ((chunk / 2) + 255) & ~(uint64_t) 255);
        return true;
    };
    size_t need = 0;
    for (;;) {
        need = need_of(chunk, n_sets);
        if (need + other_need > budget) {
            if (shrink()) continue;
            set_error("amvpt_render: the device-memory budget (" + std::to_string(budget >> 20) + " MiB) cannot hold "
                      "the smallest lane chunk (" + std::to_string((need + other_need) >> 20) + " MiB)");
            return AMVPT_ERR_OOM;
        }
        /* an arena held from an earlier, larger render is trimmed to this one's budget */
        if (A.base && A.bytes >= need && held - A.bytes + need + other_need <= budget && A.bytes + other_need > budget) {
            if (A.pending) HIPCHK(hipEventSynchronize(A.done));
            (void) hipFree(A.base);
            A.base = nullptr;
            A.bytes = 0;
        }
        const amvpt_status as_ = arena_reserve(A, A.base, A.bytes, need, "lane arena");
        if (as_ == AMVPT_OK) break;
        if (as_ != AMVPT_ERR_OOM || !shrink()) return as_;
        (void) hipGetLastError();
    }
    if (P.tile_w && chunk % (4ull * QW * 16ull) != 0) P.tile_w = 0;   /* chunks must hold whole tile bands */
    P.rcp_tpr = host_rcp(P.tile_w >> 2);   /* udiv_r's reciprocals of the final divisors */
    P.rcp_run_len = host_rcp(P.run_len);
    P.rcp_n_adapt = host_rcp(P.n_adapt);
    P.vs_stride = (uint32_t) chunk;
    const uint32_t qcap = qcap_of(chunk);
    const uint64_t qlen = (uint64_t) qcap * kQParts;
    for (int k = 0; k + 1 < n_sets; ++k)
        if (!A.side[k]) {
            HIPCHK(hipStreamCreateWithFlags(&A.side[k], hipStreamNonBlocking));
            HIPCHK(hipEventCreateWithFlags(&A.join[k], hipEventDisableTiming));
        }
    if (n_sets > 1 && !A.fork) HIPCHK(hipEventCreateWithFlags(&A.fork, hipEventDisableTiming));
    arena_release.n_side = n_sets - 1;
    /* the side stream starts after `st`'s work so far (views upload, counters) */
    auto fork_side = [&]() -> amvpt_status {
        if (n_sets < 2 || arena_release.side) return AMVPT_OK;
        HIPCHK(hipEventRecord(A.fork, st));
        for (int k = 0; k + 1 < n_sets; ++k) HIPCHK(hipStreamWaitEvent(A.side[k], A.fork, 0));
        arena_release.side = true;
        return AMVPT_OK;
    };
    char *base = (char *) A.base;
    DView *dviews = (DView *) base;
    unsigned long long *dstats = (unsigned long long *) (base + views_bytes);
    char *p = base + views_bytes + stats_bytes;
    auto carve = [&](size_t bytes) { char *r = p; p += (bytes + 255) & ~(size_t) 255; return r; };
    HIPCHK(hipMemcpyAsync(dviews, hv.data(), hv.size() * sizeof(DView), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(dstats, 0, stats_bytes, st));

    /* deterministic mode: the zeroed 32.32 fixed-point film the splats add into (k_fixed_resolve at the end) */
    const size_t film_floats = (size_t) QW * QH * (Pp.film_alpha ? 5 : 4);
    if (deterministic) {
        { const amvpt_status as_ = arena_reserve(A, A.fx, A.fxbytes, film_floats * 8, "deterministic film"); if (as_ != AMVPT_OK) return as_; }
        HIPCHK(hipMemsetAsync(A.fx, 0, film_floats * 8, st));
        P.film_fx = (unsigned long long *) A.fx;
        P.film_base = film;
        P.fx_drops = dstats + 9 * kStatShards;
    }

    /* multi-pass stock path: the per-lane sampler states between passes, two planes used in turn */
    unsigned long long *carry[2] = {nullptr, nullptr};
    if (rng_carry) {
        { const amvpt_status as_ = arena_reserve(A, A.carry, A.cbytes, (size_t) 16 * span, "sampler states"); if (as_ != AMVPT_OK) return as_; }
        carry[0] = (unsigned long long *) A.carry;
        carry[1] = carry[0] + span;
    }

    /* adaptive fill buffers: per-lane mask + compacted lane list for a whole pass */
    uint8_t *d_amask = nullptr;
    uint32_t *d_asel = nullptr, *d_anum = nullptr, *d_runs = nullptr, *d_delta = nullptr;
    unsigned long long *d_sel_status = nullptr;
    uint32_t *d_sel_ticket = nullptr;
    const uint64_t span_all = span;
    const size_t runs_bytes = 4 * (((size_t) n_runs + 63) & ~(size_t) 63);
    /* k_select_flagged: one status word per tile + the ticket */
    const uint32_t sel_tiles = (uint32_t) ((span_all + kSelTile - 1) / kSelTile);
    const size_t sel_bytes = 8 * (((size_t) sel_tiles + 31) & ~(size_t) 31) + 256;
    if (do_fill && span_all > 0xffffffffull) {
        set_error("amvpt_render: adaptive fill over a lane set of 2^32 or more lanes (32-bit lane indices)");
        return AMVPT_ERR_UNSUPPORTED;
    }
    if (do_fill) {
        const size_t abytes = ((span_all + 255) & ~(uint64_t) 255) + 4 * ((span_all + 63) & ~(uint64_t) 63) + 256 +
                              2 * runs_bytes + sel_bytes;
        { const amvpt_status as_ = arena_reserve(A, A.adapt, A.abytes, abytes, "adaptive buffers"); if (as_ != AMVPT_OK) return as_; }
        char *ap = (char *) A.adapt;
        d_amask = (uint8_t *) ap; ap += (span_all + 255) & ~(uint64_t) 255;
        d_asel = (uint32_t *) ap; ap += 4 * ((span_all + 63) & ~(uint64_t) 63);
        d_anum = (uint32_t *) ap; ap += 256;
        d_runs = (uint32_t *) ap; ap += runs_bytes;     /* flagged lanes per run (rect lane sets) */
        d_delta = (uint32_t *) ap; ap += runs_bytes;    /* run_delta */
        d_sel_status = (unsigned long long *) ap;
        d_sel_ticket = (uint32_t *) (ap + sel_bytes - 256);
    }

    /* one buffer set per chunk stream: queues A / B and their counters, the chunk's lane arena */
    struct ChunkSet {
        Bufs B{};
        float4 *qa[kQPlanes], *qb[kQPlanes];
        uint16_t *ka, *kb;              /* ray binning: bin keys of queues A / B (null: off) */
        uint32_t *cntA, *cntB, *cntN;   /* [kQParts * kCntStride] each */
        hipStream_t st;
    } sets[kMaxChunkStreams];
    for (int si = 0; si < n_sets; ++si) {
        ChunkSet &cs = sets[si];
        Bufs &B = cs.B;
        cs.st = si == 0 ? st : A.side[si - 1];
        uint32_t *dcnt = (uint32_t *) carve(cnt_bytes);
        cs.cntA = dcnt; cs.cntB = dcnt + kQParts * kCntStride; cs.cntN = dcnt + 2 * kQParts * kCntStride;
        for (int k = 0; k < kQPlanes; ++k) cs.qa[k] = (float4 *) carve(16 * qlen);
        for (int k = 0; k < kQPlanes; ++k) cs.qb[k] = (float4 *) carve(16 * qlen);
        B.lane_out = (float4 *) carve(16 * chunk);
        for (int k = 0; k < 4; ++k) B.lrec[k] = (float4 *) carve(16 * chunk);
        B.hit = (float4 *) carve(16 * std::max<uint64_t>(chunk, qlen));
        for (int k = 0; k < 2; ++k) B.nee[k] = (float4 *) carve(16 * qlen);
        B.nee_gb = (float2 *) carve(8 * qlen);
        for (int k = 0; k < 3; ++k) B.vreq[k] = (float4 *) carve(16 * chunk);
        B.occ = (unsigned long long *) carve((size_t) 8 * G * ((chunk + 63) / 64));
        B.cnt_nee = cs.cntN;
        B.qcap = qcap;
        B.vrec = (float4 *) carve((size_t) (diff_rec ? 4 : (AMVPT_WAVE_DIFF ? 36 : 32)) * G * chunk);
        cs.ka = cs.kb = nullptr;
        B.key_out = B.key_in = B.key_nee = nullptr;
        if (bin_ext || bin_nee) { B.sray[0] = (float4 *) carve(32 * qlen); B.sray[1] = nullptr; }
        B.sgb = (bin_nee && AMVPT_NEE_CARRY) ? (float2 *) carve(8 * qlen) : nullptr;
        if (bin_ext) { cs.ka = (uint16_t *) carve(2 * qlen); cs.kb = (uint16_t *) carve(2 * qlen); }
        if (bin_nee) B.key_nee = (uint16_t *) carve(2 * qlen);
        if (wide) {
            for (int k = 0; k < mplanes; ++k) B.vreq_w[k] = (uint4 *) carve(16 * chunk);
            for (int k = 0; k < 3 * mplanes; ++k) B.lmask_w[k] = (uint4 *) carve(16 * chunk);
            if (vs_global) B.vstate = (float *) carve((size_t) VS_FIELDS * 4 * G * chunk);
        }
        B.film = film;
        B.records = records;
        B.stats = dstats;
        B.amask = d_amask;
        B.asel = d_asel;
        B.run_delta = d_delta;
    }

    const DScene *dS = (const DScene *) scene->dev_scene_struct;
    const uint32_t fused_blocks = K.fused_blocks;
    const size_t lds = tab_b ? scene->dev.tab_bytes : 0u;                                           /* k_bounce */
    /* k_suffix_fused: the box triangles staged for box_walk (AMVPT_BOX_LDS) */
    const size_t box_lds = (AMVPT_BOX_LDS && P.box_screen) ? (size_t) scene->n_boxes * 12u * sizeof(DPrim) : 0u;
    const size_t lds_ext = scene_lds_bytes(scene->dev, trav);                                       /* BVH walks */
    const size_t lds_any0 = lds_ext + ((AMVPT_TREELETS & 1) ? tree_lds_bytes(scene->dev, trav) : 0u);    /* k_shadow: + any-hit treelet */
    const size_t lds_vis = lds_ext + ((AMVPT_TREELETS & 4) ? tree_lds_bytes(scene->dev, trav) : 0u);     /* k_vis */
    const size_t lds_close0 = lds_ext + ((AMVPT_TREELETS & 2) ? oct_tree_lds_bytes(scene->dev, trav) : 0u); /* k_extend: + octant treelets */
    /* the two-box BVH walks (DScene::nodes2) for the per-lane suffix walks of BVHs read from device memory: a stack
     * of kStack2 u32 entries per thread after the kernels' other LDS (AMVPT_OPT_THREADED_BVH keeps the threaded walks) */
    P.bvh2 = (scene->n_nodes2 && lane_walk && !(AMVPT_TREELETS & 3) && !(opts.flags & AMVPT_OPT_THREADED_BVH)) ? 1u : 0u;
    const size_t stk_bytes = P.bvh2 ? (size_t) kStack2 * kStk2Stride * 4u : 0u;
    P.stk_off_ext = (uint32_t) ((lds_close0 + 15u) & ~(size_t) 15u);
    P.stk_off_any = (uint32_t) ((lds_any0 + 15u) & ~(size_t) 15u);
    const size_t lds_close = P.bvh2 ? P.stk_off_ext + stk_bytes : lds_close0;
    const size_t lds_any = P.bvh2 ? P.stk_off_any + stk_bytes : lds_any0;
    const size_t lds_prim = tab_p ? scene->dev.tab_bytes + views_lds_bytes(Pp.n_views) : 0u;        /* primary shading */
    KTimer T;
    T.init(counters != nullptr);
    HIPCHK(T.err);
    auto t0 = std::chrono::steady_clock::now();
    const uint32_t max_bounces = P.max_depth == 0xffffffffu ? 0xffffffffu : P.max_depth + 1;

    /* the shared suffix (sample_suffix / sample_single loop) over the queue the raygen
     * or primary kernel filled: one k_bounce launch per depth, ping-pong A <-> B */
    auto run_suffix = [&](ChunkSet &cs, uint32_t cn) -> amvpt_status {
        Bufs &B = cs.B;
        hipStream_t st = cs.st;
        float4 *const *qa = cs.qa, *const *qb = cs.qb;
        uint32_t *const cntA = cs.cntA, *const cntB = cs.cntB;
        if (fuse_suffix) {
            /* one k_suffix_fused launch over the primary queue (A); B's counters are its work counters */
            for (int k = 0; k < kQPlanes; ++k) { B.q_in[k] = qa[k]; B.q_out[k] = qb[k]; }
            B.cnt_in = cntA;
            B.cnt_out = cntB;
            HIPCHK(hipMemsetAsync(cntB, 0, (size_t) kQParts * kCntStride * 4, st));
            T.begin(AMVPT_K_SUFFIX, st);
            launch_suffix_fused(tab_b, diff, walk, dim3(kQParts * fused_blocks), kFusedParkBytes + lds + box_lds, st, P, dS, B);
            T.end(st);
            HIPCHK(hipGetLastError());
            HIPCHK(T.err);
            return AMVPT_OK;
        }
        /* a multiple of kQParts blocks: 1..16 per partition */
        const uint32_t bgrid = kQParts * std::max<uint32_t>(1, std::min<uint32_t>(16, (cn + 256 * kQParts - 1) / (256 * kQParts)));
        bool a_is_in = true;
        for (uint32_t bnc = 0; bnc < max_bounces; ++bnc) {
            for (int k = 0; k < kQPlanes; ++k) {
                B.q_in[k] = a_is_in ? qa[k] : qb[k];
                B.q_out[k] = a_is_in ? qb[k] : qa[k];
            }
            B.cnt_in = a_is_in ? cntA : cntB;
            B.cnt_out = a_is_in ? cntB : cntA;
            B.key_in = a_is_in ? cs.ka : cs.kb;
            B.key_out = a_is_in ? cs.kb : cs.ka;
            /* k_extend zeroes cnt_out and cnt_nee */
            if (bin_ext) {
                T.begin(AMVPT_K_BIN, st);
                if (bnc == 0) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_bin_sort<false, true>), dim3(kQParts), dim3(kBinBlock), 0, st, P, B);
                else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_bin_sort<false>), dim3(kQParts), dim3(kBinBlock), 0, st, P, B);
                T.end(st);
            }
            T.begin(AMVPT_K_EXTEND, st);
            if (bin_ext && walk == WALK_LANE_TRI) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_LANE_TRI, true>), dim3(bgrid), dim3(256), lds_close, st, P, dS, B);
            else if (bin_ext && walk == WALK_LANE_NS) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_LANE_NS, true>), dim3(bgrid), dim3(256), lds_close, st, P, dS, B);
            else if (bin_ext) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_LANE, true>), dim3(bgrid), dim3(256), lds_close, st, P, dS, B);
            else if (walk == WALK_BRUTE_NS) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_BRUTE_NS>), dim3(bgrid), dim3(256), lds_ext, st, P, dS, B);
            else if (walk == WALK_BRUTE) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_BRUTE>), dim3(bgrid), dim3(256), lds_ext, st, P, dS, B);
            else if (walk == WALK_UNI) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_UNI>), dim3(bgrid), dim3(256), lds_ext, st, P, dS, B);
            else if (walk == WALK_LANE_TRI) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_LANE_TRI>), dim3(bgrid), dim3(256), lds_close, st, P, dS, B);
            else if (walk == WALK_LANE_NS) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_LANE_NS>), dim3(bgrid), dim3(256), lds_close, st, P, dS, B);
            else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_extend<WALK_LANE>), dim3(bgrid), dim3(256), lds_close, st, P, dS, B);
            T.end(st);
            T.begin(AMVPT_K_BOUNCE, st);
            launch_bounce(tab_b, diff, fuse_nee ? walk : -1, dim3(bgrid), lds, st, P, dS, B);
            T.end(st);
            if (!fuse_nee) {
                if (bin_nee) {
                    T.begin(AMVPT_K_BIN, st);
                    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_bin_sort<true>), dim3(kQParts), dim3(kBinBlock), 0, st, P, B);
                    T.end(st);
                }
                T.begin(AMVPT_K_SHADOW, st);
                launch_shadow(walk, bin_nee, dim3(bgrid), lds_any, st, P, dS, B);
                T.end(st);
            }
            HIPCHK(hipGetLastError());
            HIPCHK(T.err);
            a_is_in = !a_is_in;
            if (bnc >= 15 && (bnc & 7) == 7) { /* unbounded depth: poll the live count */
                std::vector<uint32_t> hc((size_t) kQParts * kCntStride);
                HIPCHK(hipMemcpyAsync(hc.data(), B.cnt_out, hc.size() * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                uint64_t live = 0;
                for (uint32_t q = 0; q < kQParts; ++q) live += hc[(size_t) q * kCntStride];
                if (live == 0) break;
            }
        }
        return AMVPT_OK;
    };
    uint64_t adaptive_lanes = 0;

    uint64_t chunk_index = 0;
    for (uint32_t pass = 0; pass < n_passes; ++pass) {
        RoctxScope range_pass("amvpt pass");
        P.seed_value = Pp.base_seed + (is_mv ? (spp_pp * pass + Pp.seed) : Pp.seed);
        P.record = (records && pass == record_pass) ? 1u : 0u;
        P.rng_in = rng_carry && pass > 0 ? carry[pass & 1u] : nullptr;
        P.rng_out = rng_carry && pass + 1 < n_passes ? carry[(pass + 1) & 1u] : nullptr;
        for (uint64_t c0 = 0; c0 < span; c0 += chunk, ++chunk_index) {   /* virtual indices of the lane set */
            const uint32_t cn = (uint32_t) std::min<uint64_t>(chunk, span - c0);
            /* chunk i on set i mod n_sets: the side streams start once the first chunk's primary stage is queued
             * (the streams then run offset from each other) */
            ChunkSet &cs = sets[chunk_index % (uint64_t) n_sets];
            Bufs &B = cs.B;
            hipStream_t st = cs.st;
            uint32_t *const cntA = cs.cntA, *const cntB = cs.cntB;
            float4 *const *qa = cs.qa, *const *qb = cs.qb;
            if (&cs != &sets[0]) {   /* a side chunk never runs before the fork (e.g. after a pass's join) */
                const amvpt_status fs_ = fork_side();
                if (fs_ != AMVPT_OK) return fs_;
            }
            P.chunk_begin = c0;
            P.chunk_n = cn;
            B.records = P.record ? records + (size_t) c0 * G * 8 : records;
            const dim3 grid((cn + 255) / 256);
            /* counters: [0] = queue A, [1] = queue B */
            HIPCHK(hipMemsetAsync(cntA, 0, (size_t) kQParts * kCntStride * 4, st));
            for (int k = 0; k < kQPlanes; ++k) { B.q_out[k] = qa[k]; B.q_in[k] = qb[k]; }
            B.cnt_out = cntA; B.cnt_in = cntB;
            B.key_out = cs.ka; B.key_in = cs.kb;
            T.mark(st);
            {
                RoctxScope range_primary("amvpt primary vertex (raygen, visibility, camera selection, MIS)");
                if (G == 1) {
                    T.begin(AMVPT_K_RAYGEN, st);
                    hipLaunchKernelGGL(k_raygen_single, grid, dim3(256), 0, st, P, dviews, B);
                    T.end(st);
                } else {
                    kPrimary[dispatch_g(G)](cn, lds_prim, lds_vis, st, P, dS, dviews, B, tab_p, uni_coh, diff, T);
                }
            }
            HIPCHK(hipGetLastError());
            HIPCHK(T.err);
            T.mark(st);
            if (n_sets > 1 && chunk_index % (uint64_t) n_sets == 0) {   /* the side streams' start: after this primary stage */
                const amvpt_status fs_ = fork_side();
                if (fs_ != AMVPT_OK) return fs_;
            }
            /* suffix bounces: ping-pong A <-> B */
            {
                RoctxScope range_suffix("amvpt shared suffix (extend, bounce, NEE)");
                const amvpt_status rs_ = run_suffix(cs, cn);
                if (rs_ != AMVPT_OK) return rs_;
            }
            T.mark(st);
            RoctxScope range_splat("amvpt splat (ImageBlock::put)");
            const dim3 sgrid((cn + kSplatBlock - 1) / kSplatBlock);
            T.begin(AMVPT_K_SPLAT, st);
            if (G == 1 && P.C == 5) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_single<5>), sgrid, dim3(kSplatBlock), 0, st, P, B);
            else if (G == 1) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_single<4>), sgrid, dim3(kSplatBlock), 0, st, P, B);
            else kSplat[dispatch_g(G)](sgrid, st, P, dviews, B, diff_rec);
            T.end(st);
            T.mark(st);
            HIPCHK(hipGetLastError());
            if (n_sets < 2) T.flush();
            HIPCHK(T.err);
        }
        /* the stock path's next pass reads the sampler states this pass writes (and writes the plane this
         * pass read): with two chunk streams, chunk c of the next pass may run on the other stream than chunk
         * c of this one, so both streams meet at every pass boundary (the next side chunk forks again) */
        if (rng_carry) arena_release.join();
        if (do_fill) {
            /* the fill reads the whole pass's adapt_mask: both chunk streams first */
            arena_release.join();
            RoctxScope range_fill("amvpt adaptive fill");
            /* compact the pass's adapt_mask lanes in lane order (virtual indices of the lane set,
             * ascending = lane order), then n_adapt re-traces each */
            uint64_t n_sel = 0;
            {
                HIPCHK(hipMemsetAsync(d_sel_status, 0, sel_bytes, st));   /* status words + ticket */
                T.begin(AMVPT_K_SELECT, st);
                hipLaunchKernelGGL(k_select_flagged, dim3(sel_tiles), dim3(256), 0, st, (const uint8_t *) d_amask, span_all,
                                   d_asel, d_anum, d_sel_status, d_sel_ticket, sel_tiles);
                T.end(st);
                HIPCHK(hipGetLastError());
                uint32_t got = 0;
                HIPCHK(hipMemcpyAsync(&got, d_anum, 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
                n_sel = got;
            }
            /* this render's place in the pass's compressed array: per run, the flagged lanes of the
             * whole pass below it (one exchange per pass), as run_delta = global - local prefix */
            uint64_t total = n_sel;
            std::vector<uint32_t> delta(n_runs, 0u);
            if (partial) {
                std::vector<uint64_t> run_begin(n_runs), run_count(n_runs, 0), run_prefix(n_runs, 0);
                if (rect) {
                    hipLaunchKernelGGL(k_run_counts, dim3(n_runs), dim3(256), 0, st, (const uint8_t *) d_amask, P.run_len, d_runs);
                    HIPCHK(hipGetLastError());
                    std::vector<uint32_t> rc(n_runs);
                    HIPCHK(hipMemcpyAsync(rc.data(), d_runs, 4 * (size_t) n_runs, hipMemcpyDeviceToHost, st));
                    HIPCHK(hipStreamSynchronize(st));
                    for (uint32_t r = 0; r < n_runs; ++r) {
                        run_count[r] = rc[r];
                        run_begin[r] = ((uint64_t) (ry0 + r) * QW + rx0) * spp_pp;
                    }
                } else {
                    run_count[0] = n_sel;
                    run_begin[0] = lane_begin;
                }
                if (exchange(exchange_ctx, n_runs, run_begin.data(), run_count.data(), run_prefix.data(), &total) != 0) {
                    set_error("amvpt_render: adaptive count exchange failed");
                    return AMVPT_ERR_INVALID;
                }
                uint64_t local = 0;
                for (uint32_t r = 0; r < n_runs; ++r) {
                    if (run_prefix[r] < local || run_prefix[r] + run_count[r] > total) {
                        set_error("amvpt_render: adaptive count exchange returned inconsistent prefixes");
                        return AMVPT_ERR_INVALID;
                    }
                    delta[r] = (uint32_t) (run_prefix[r] - local);
                    local += run_count[r];
                }
                if (local != n_sel) {
                    set_error("amvpt_render: per-run adaptive counts disagree with the compaction");
                    return AMVPT_ERR_INVALID;
                }
            }
            if (total * n_adapt > 0xffffffffull) { set_error("amvpt_render: adaptive wavefront over 2^32 lanes"); return AMVPT_ERR_UNSUPPORTED; }
            HIPCHK(hipMemcpyAsync(d_delta, delta.data(), 4 * (size_t) n_runs, hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));   /* `delta` is a host temporary */
            const uint64_t wf = n_sel * n_adapt;
            adaptive_lanes += wf;
            KParams Ps = P;
            P.pass_seed = P.seed_value;
            P.adapt_seed = Pp.base_seed + (uint32_t) (total * n_adapt);   /* sampler->fork(); seed(wavefront, wavefront) */
            P.adapt_pass = 1;
            P.record = 0;
            ChunkSet &cs = sets[0];
            Bufs &B = cs.B;
            uint32_t *const cntA = cs.cntA, *const cntB = cs.cntB;
            float4 *const *qa = cs.qa, *const *qb = cs.qb;
            for (uint64_t c0 = 0; c0 < wf; c0 += chunk) {
                const uint32_t cn = (uint32_t) std::min<uint64_t>(chunk, wf - c0);
                P.chunk_begin = c0;
                P.chunk_n = cn;
                HIPCHK(hipMemsetAsync(cntA, 0, (size_t) kQParts * kCntStride * 4, st));
                for (int k = 0; k < kQPlanes; ++k) { B.q_out[k] = qa[k]; B.q_in[k] = qb[k]; }
                B.cnt_out = cntA; B.cnt_in = cntB;
                B.key_out = cs.ka; B.key_in = cs.kb;
                T.begin(AMVPT_K_RAYGEN, st);
                hipLaunchKernelGGL(k_raygen_adapt, dim3((cn + 255) / 256), dim3(256), 0, st, P, dviews, B);
                T.end(st);
                HIPCHK(hipGetLastError());
                { const amvpt_status rs_ = run_suffix(cs, cn); if (rs_ != AMVPT_OK) return rs_; }
                const dim3 sgrid((cn + kSplatBlock - 1) / kSplatBlock);
                T.begin(AMVPT_K_SPLAT, st);
                if (P.C == 5) hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_adapt<5>), sgrid, dim3(kSplatBlock), 0, st, P, B);
                else hipLaunchKernelGGL(HIP_KERNEL_NAME(k_splat_adapt<4>), sgrid, dim3(kSplatBlock), 0, st, P, B);
                T.end(st);
                HIPCHK(hipGetLastError());
                T.flush();
                HIPCHK(T.err);
            }
            P = Ps;
        }
    }
    arena_release.join();
    if (deterministic) {
        hipLaunchKernelGGL(k_fixed_resolve, dim3((uint32_t) ((film_floats + 255) / 256)), dim3(256), 0, st, film,
                           (const unsigned long long *) A.fx, (uint64_t) film_floats);
        HIPCHK(hipGetLastError());
    }
    uint64_t overflow_cells = 0;
    if (P.overflow) {
        /* the caller sums the list; a list that ran out of room lost cells: fail loudly */
        HIPCHK(hipMemcpyAsync(&overflow_cells, P.overflow, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        overflow_added = overflow_cells - std::min(overflow_cells, overflow_before);
        if (overflow_cells > P.ov_cap) {
            set_error("amvpt_render: film overflow list full (" + std::to_string(overflow_cells) + " cells > capacity " +
                      std::to_string(P.ov_cap) + "): widen the film window or the list");
            return AMVPT_ERR_OOM;
        }
    }
    if (counters) {
        std::vector<unsigned long long> hsh((size_t) kStats * kStatShards);
        HIPCHK(hipMemcpyAsync(hsh.data(), dstats, stats_bytes, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        unsigned long long hs[kStats] = {0};
        for (uint32_t k = 0; k < kStats; ++k)
            for (uint32_t q = 0; q < kStatShards; ++q) hs[k] += hsh[(size_t) k * kStatShards + q];
        amvpt_counters &c = *counters;
        c = amvpt_counters{};
        c.lanes = span * n_passes;
        c.passes = n_passes;
        c.vertices = hs[0];
        c.reuse_lanes = hs[1];
        c.visibility_rays = hs[2];
        c.view_splats = hs[3];
        c.splat_fallback = hs[4];
        c.adaptive_lanes = adaptive_lanes;
        c.shadow_rays = hs[5];
        c.record_bytes = G > 1 ? 64 + 16 + (diff_rec ? 4 : 32) * (uint64_t) G : 0;
        c.nonfinite_samples = hs[6];
        c.negative_samples = hs[7];
        c.pushed_paths = hs[8];
        c.film_overflow = overflow_added;   /* this render's cells (renders append to the list) */
        c.film_range_drops = hs[9];
        c.primary_record_bytes = hs[10];
        c.splat_record_bytes = hs[11];
        c.chunk_lanes = chunk;
        c.buffer_sets = (uint64_t) n_sets;
        c.arena_bytes = A.bytes + A.abytes + A.fxbytes + A.cbytes;
        T.flush();
        HIPCHK(T.err);
        for (int k = 0; k < AMVPT_K_COUNT; ++k) { c.kernel_ms[k] = T.ms[k]; c.kernel_launches[k] = T.launches[k]; }
        c.kernel_ms_primary = T.ms[AMVPT_K_PRIM_HIT] + T.ms[AMVPT_K_PRIM_REQ] + T.ms[AMVPT_K_VIS] +
                              T.ms[AMVPT_K_MV_PRIMARY] + T.ms[AMVPT_K_RAYGEN];
        c.kernel_ms_bounce = T.ms[AMVPT_K_EXTEND] + T.ms[AMVPT_K_BOUNCE] + T.ms[AMVPT_K_SHADOW] + T.ms[AMVPT_K_SUFFIX];
        c.kernel_ms_splat = T.ms[AMVPT_K_SPLAT];
        c.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return AMVPT_OK;
}

/* amvpt_film_accumulate: window rows into the quilt (one thread per float; a window's floats are
 * distinct quilt floats, so plain adds), then the overflow entries (float atomics: entries repeat) */
AMVPT_TU_LOCAL __global__ void k_accumulate(float *quilt, uint32_t qw, uint32_t C, const float *win, uint32_t x0,
                                            uint32_t y0, uint32_t w) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (i >= w * C) return;
    quilt[((size_t) (y0 + y) * qw + x0) * C + i] += win[(size_t) y * w * C + i];
}
AMVPT_TU_LOCAL __global__ void k_overflow_apply(float *quilt, uint64_t n_floats, const uint4 *e, uint64_t n) {
    const uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 v = e[i];
    const uint64_t idx = (uint64_t) v.x | ((uint64_t) v.y << 32);
    if (idx < n_floats) atomicAdd(quilt + idx, __uint_as_float(v.z));
}
amvpt_status accumulate_impl(float *quilt, uint32_t qw, uint32_t qh, uint32_t C, const float *win, uint32_t x0,
                             uint32_t y0, uint32_t w, uint32_t h, const uint32_t *ov, uint64_t n_ov, void *stream) {
    if (!quilt || (w && h && !win) || (n_ov && !ov) || (C != 4 && C != 5)) {
        set_error("amvpt_film_accumulate: bad argument");
        return AMVPT_ERR_INVALID;
    }
    if ((uint64_t) x0 + w > qw || (uint64_t) y0 + h > qh) {
        set_error("amvpt_film_accumulate: window outside the quilt");
        return AMVPT_ERR_INVALID;
    }
    hipStream_t st = (hipStream_t) stream;
    if (w && h) hipLaunchKernelGGL(k_accumulate, dim3((w * C + 255) / 256, h), dim3(256), 0, st, quilt, qw, C, win, x0, y0, w);
    if (n_ov)
        hipLaunchKernelGGL(k_overflow_apply, dim3((uint32_t) ((n_ov + 255) / 256)), dim3(256), 0, st, quilt,
                           (uint64_t) qw * qh * C, (const uint4 *) ov, n_ov);
    HIPCHK(hipGetLastError());
    return AMVPT_OK;
}

/* amvpt_release_device_memory: the device's lane arena and span buffers, after the last render that used them */
amvpt_status release_impl(int device) {
    DevArena *a = nullptr;
    {
        std::lock_guard<std::mutex> g(g_arenas_mu);
        auto it = g_arenas.find(device);
        if (it != g_arenas.end()) a = it->second.get();
    }
    if (!a) return AMVPT_OK;
    std::lock_guard<std::mutex> g(a->mu);
    int cur = 0;
    HIPCHK(hipGetDevice(&cur));
    HIPCHK(hipSetDevice(device));
    hipError_t e = a->pending ? hipEventSynchronize(a->done) : hipSuccess;
    a->pending = false;
    void **bufs[4] = {&a->base, &a->adapt, &a->fx, &a->carry};
    for (void **b : bufs) {
        if (*b) (void) hipFree(*b);
        *b = nullptr;
    }
    a->bytes = a->abytes = a->fxbytes = a->cbytes = 0;
    (void) hipSetDevice(cur);
    if (e != hipSuccess) return hip_fail("hipEventSynchronize (release)", (int) e);
    return AMVPT_OK;
}

amvpt_status develop_impl(const float *film, float *out, uint32_t w, uint32_t h, uint32_t alpha, void *stream) {
    uint32_t npx = w * h;
    hipLaunchKernelGGL(k_develop, dim3((npx + 255) / 256), dim3(256), 0, (hipStream_t) stream, film, out, npx, alpha);
    HIPCHK(hipGetLastError());
    return AMVPT_OK;
}

#endif /* !AMVPT_SHADOW_TU && !AMVPT_GROUP_TU && !AMVPT_KERNEL_PROBE */
} // namespace amvpt
