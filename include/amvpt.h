/*
 * amvpt.h -- C-ABI of the MI355X-native AMVPT (`mvpath`) hot path.
 *
 * This is the drop-in boundary: the `mvpath` integrator plugin's render()
 * (reference: src/integrators/mvpath.cpp:7-278, `MVPathIntegrator::render`)
 * flattens its Scene / MultiSensor / Film / Sampler objects into the plain
 * descriptors below and calls `amvpt_render()`; the pass loop, the per-lane
 * `render_multisample` / `render_sample` work and the ImageBlock splat all run
 * on the GPU behind this interface.  No torch or HIP types appear here: every
 * buffer is a plain pointer + size, every failure an integer status plus
 * `amvpt_last_error()`.
 *
 * Reference interfaces replaced (file:line in xacond00/mitsuba3-amvpt):
 *   amvpt_scene_create   <- Scene ctor + accel_init_cpu (Embree BVH build)
 *                           src/render/scene.cpp:30-96, scene_embree.inl:114-116
 *   amvpt_render         <- MVPathIntegrator::render JIT branch
 *                           src/integrators/mvpath.cpp:132-272
 *                           (and SamplingIntegrator::render, integrator.cpp:236-330,
 *                           for the stock `path` integrator, C1)
 *   amvpt_develop        <- HDRFilm::develop, src/films/hdrfilm.cpp:304-418
 *   amvpt_last_error     <- Throw() / C++ exceptions (mvpath.cpp:17,25,46)
 *
 * Matrices are row-major 4x4 (m[r*4+c]), matching mitsuba::Transform4f::matrix.
 */
#ifndef AMVPT_H
#define AMVPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMVPT_ABI_VERSION 10

typedef enum amvpt_status {
    AMVPT_OK = 0,
    AMVPT_ERR_INVALID = 1,     /* bad descriptor / argument */
    AMVPT_ERR_HIP = 2,         /* HIP runtime failure (see amvpt_last_error) */
    AMVPT_ERR_OOM = 3,         /* device allocation failed */
    AMVPT_ERR_UNSUPPORTED = 4, /* feature outside the implemented path */
    AMVPT_ERR_NO_DEVICE = 5    /* no GPU visible: the product path never falls back to CPU */
} amvpt_status;

/* ------------------------------------------------------------------ */
/* Scene description                                                  */
/* ------------------------------------------------------------------ */

enum {
    AMVPT_SHAPE_RECTANGLE = 0, /* src/shapes/rectangle.cpp  */
    AMVPT_SHAPE_MESH = 1,      /* src/render/mesh.cpp (cube.cpp, obj.cpp, ...) */
    AMVPT_SHAPE_SPHERE = 2     /* src/shapes/sphere.cpp     */
};

typedef struct amvpt_shape_desc {
    uint32_t type;
    int32_t bsdf;         /* index into bsdfs[] (host loader assigns the default diffuse) */
    int32_t emitter;      /* index into emitters[] or -1 */
    uint32_t flip_normals;
    float to_world[16];   /* rectangle / sphere object-to-world */
    float to_object[16];  /* inverse of to_world */
    /* mesh: world-space attributes exactly as Mesh stores them after its ctor */
    uint32_t vertex_count;
    uint32_t face_count;
    const float *positions; /* vertex_count*3 */
    const float *normals;   /* vertex_count*3 or NULL */
    const float *texcoords; /* vertex_count*2 or NULL */
    const uint32_t *faces;  /* face_count*3 */
    /* sphere */
    float center[3];
    float radius;
} amvpt_shape_desc;

enum {
    AMVPT_BSDF_DIFFUSE = 0,        /* src/bsdfs/diffuse.cpp        */
    AMVPT_BSDF_ROUGHCONDUCTOR = 1, /* src/bsdfs/roughconductor.cpp */
    AMVPT_BSDF_TWOSIDED = 2        /* src/bsdfs/twosided.cpp       */
};
enum { AMVPT_MICROFACET_BECKMANN = 0, AMVPT_MICROFACET_GGX = 1 };

typedef struct amvpt_bsdf_desc {
    uint32_t type;
    int32_t nested[2];        /* twosided: front / back (== front if single) */
    float reflectance[3];     /* diffuse */
    uint32_t distribution;    /* roughconductor */
    uint32_t sample_visible;
    float alpha_u, alpha_v;
    float eta[3], k[3];
    uint32_t has_specular_reflectance;
    float specular_reflectance[3];
} amvpt_bsdf_desc;

enum {
    AMVPT_EMITTER_AREA = 0,     /* src/emitters/area.cpp: attached to a rectangle / sphere / mesh shape */
    AMVPT_EMITTER_CONSTANT = 1  /* src/emitters/constant.cpp: environment, shape = -1 */
};

/* emitters[] is Scene::m_emitters: the order in which the scene lists them (an area emitter at
 * its shape's position, a constant emitter at its own), which emitter sampling indexes */
typedef struct amvpt_emitter_desc {
    uint32_t type;
    int32_t shape;          /* shape the area emitter is attached to; -1 for AMVPT_EMITTER_CONSTANT */
    float radiance[3];
    float sampling_weight;  /* Emitter 'sampling_weight' (>= 0); any != 1 -> DiscreteDistribution
                               emitter sampling (scene.cpp:100-119, 222-244) */
} amvpt_emitter_desc;

typedef struct amvpt_scene_desc {
    const amvpt_shape_desc *shapes;
    uint32_t shape_count;
    const amvpt_bsdf_desc *bsdfs;
    uint32_t bsdf_count;
    const amvpt_emitter_desc *emitters;
    uint32_t emitter_count;
    uint32_t has_environment; /* number of AMVPT_EMITTER_CONSTANT entries in emitters[] (0 or 1:
                                 Scene::m_environment); its bounding sphere is the scene bbox's */
} amvpt_scene_desc;

/* ------------------------------------------------------------------ */
/* Sensors: one projective view per sub-sensor of the MultiSensor      */
/* (grid.cpp:84-236 builds them; perspective.cpp:173-203 transforms)  */
/* ------------------------------------------------------------------ */

enum { AMVPT_CAMERA_PERSPECTIVE = 0, AMVPT_CAMERA_THINLENS = 1 };

typedef struct amvpt_view_desc {
    uint32_t type;
    float to_world[16];          /* camera-to-world */
    float to_world_inv[16];      /* world-to-camera (Transform::inverse(), exact shuffle) */
    float sample_to_camera[16];  /* includes lens_shift (perspective.cpp:179) */
    float camera_to_sample[16];
    float near_clip, far_clip;
    float normalization;         /* 1 / image_rect.volume() */
    float resolution[2];         /* sub-film crop size (m_resolution) */
    float pp_offset[2];          /* film.size * principal_point_offset / crop_size */
    float aperture_radius;       /* thinlens */
    float focus_distance;        /* thinlens */
} amvpt_view_desc;

/* ------------------------------------------------------------------ */
/* Integrator / film / sampler parameters                             */
/* ------------------------------------------------------------------ */

enum { AMVPT_INTEGRATOR_MVPATH = 0, AMVPT_INTEGRATOR_PATH = 1 };
enum { AMVPT_RFILTER_BOX = 0, AMVPT_RFILTER_GAUSSIAN = 1 };

typedef struct amvpt_params {
    uint32_t integrator;     /* AMVPT_INTEGRATOR_* */
    /* mvpath Properties (mvpath.h:120-129) + MonteCarloIntegrator (integrator.cpp:505-522) */
    uint32_t max_depth;      /* -1 maps to 0xffffffff */
    uint32_t rr_depth;
    uint32_t hide_emitters;
    uint32_t sa_reuse, sa_mis, fast_mis, debug;
    uint32_t adaptive;
    /* mvpath: spp_pass_lim (mvpath.h:127, default 16).  The stock path integrator: its samples_per_pass
     * (integrator.cpp:107, 0 = unset): a frame of several passes continues every lane's sampler stream
     * from pass to pass as the reference's JIT render does (integrator.cpp:279-330); an spp it does not
     * divide is refused with the reference's message.  Either integrator also splits a pass of more than
     * 2^32 - 1 lanes (integrator.cpp:249-265). */
    uint32_t spp_pass_lim;
    uint32_t reuse_count;
    /* sampler (independent.cpp) */
    uint32_t spp;            /* requested spp (0 -> sampler sample_count) */
    uint32_t seed;           /* render(seed=...) */
    uint32_t base_seed;      /* sampler 'seed' property */
    /* MultiSensor (grid.cpp) */
    uint32_t n_views;
    uint32_t multisensor;    /* 1: grid sensor (sample_ray_idx); 0: single projective camera */
    uint32_t grid_x, grid_y;
    uint32_t reverse_x, reverse_y;
    /* film (hdrfilm.cpp) */
    uint32_t film_width, film_height; /* quilt crop size */
    uint32_t film_alpha;     /* 1 -> RGBAW (5 channels), 0 -> RGBW */
    uint32_t rfilter;        /* AMVPT_RFILTER_* */
    float rfilter_stddev;    /* gaussian stddev (radius = 4*stddev) */
    /* MultiSensor layout: 0 grid (grid.cpp:268-297), 1 batch (batch.cpp:163-181:
     * a horizontal strip, grid_y = 1, index clamped before reverse_x) */
    uint32_t batch;
    /* ABI 8: hdrfilm crop window (hdrfilm.cpp:245-291).  film_width / film_height above are the
     * crop size (the ImageBlock and the lane space, mvpath.cpp:28-30,173-190); crop_offset is the
     * ImageBlock's offset in the film (sample positions are film coordinates, ImageBlock::put
     * subtracts it, imageblock.cpp:211,266,447) and full_width / full_height the film size (the
     * quilt tile pitch of reprojected views is film->size() / grid, mvpath_multi.h:62).  Zeros: no crop. */
    uint32_t crop_offset_x, crop_offset_y;
    uint32_t full_width, full_height;
} amvpt_params;

/* Per-render counters (device-side lane statistics; SURVEY 8(d) byte model). */
typedef struct amvpt_counters {
    uint64_t lanes;            /* primary lanes processed */
    uint64_t passes;
    uint64_t vertices;         /* path vertices processed (primary + suffix bounces) */
    uint64_t reuse_lanes;      /* lanes whose primary hit was reusable (h-bar numerator) */
    uint64_t visibility_rays;  /* camera-visibility rays traced in camera_selection */
    uint64_t view_splats;      /* valid view samples splatted */
    uint64_t adaptive_lanes;   /* lanes re-traced by the adaptive pass */
    double kernel_ms_primary;  /* HIP-event time per stage: primary wavefronts (or raygen), */
    double kernel_ms_bounce;   /* the suffix (extend + bounce + shadow, all depths), */
    double kernel_ms_splat;    /* the splat */
    double total_ms;
    uint64_t splat_fallback;   /* view samples splatted with direct global atomics (LDS window miss) */
    /* ABI 4: per-kernel HIP-event time and launch count, indexed by amvpt_kernel_id */
    uint64_t shadow_rays;      /* suffix NEE rays traced by k_shadow */
    double kernel_ms[12];
    uint64_t kernel_launches[12];
    /* ABI 5 */
    uint64_t record_bytes;     /* bytes of per-lane records k_mv_primary writes and the splat reads (lane + views) */
    uint64_t nonfinite_samples; /* splatted view samples with a NaN/Inf value (ImageBlock::put's check, imageblock.cpp:180-204) */
    uint64_t negative_samples;  /* splatted view samples with a negative RGB component (same check) */
    /* ABI 8 */
    uint64_t pushed_paths;      /* paths that left the primary vertex into the shared suffix (byte model of the suffix) */
    uint64_t film_overflow;     /* film floats added to the overflow list (cells outside an amvpt_film_window) */
    /* ABI 9 */
    uint64_t film_range_drops;  /* AMVPT_OPT_DETERMINISTIC: finite footprint-cell adds of |v| >= 2^31 the fixed-point
                                 * film cannot hold, dropped (ImageBlock::put would add them; 0 otherwise) */
    /* ABI 10: the render's memory plan (amvpt_render_opts.budget_mib) */
    uint64_t chunk_lanes;       /* lanes per chunk the render ran (the automatic or requested chunk, after the budget) */
    uint64_t buffer_sets;       /* chunk buffer sets (= chunk streams) */
    uint64_t arena_bytes;       /* device bytes the device's arena holds after the render (amvpt_release_device_memory) */
    uint64_t primary_record_bytes; /* view-record bytes k_mv_primary wrote (4 per view all-diffuse, else 32) */
    uint64_t splat_record_bytes;   /* view-record bytes the splat read (only the views it visits / that splat) */
} amvpt_counters;

/* kernels of the pipeline, for amvpt_counters.kernel_ms */
typedef enum amvpt_kernel_id {
    AMVPT_K_PRIM_HIT = 0,      /* raygen + primary closest hit            */
    AMVPT_K_PRIM_REQ = 1,      /* shadow / visibility ray requests        */
    AMVPT_K_VIS = 2,           /* visibility + primary shadow any-hit     */
    AMVPT_K_MV_PRIMARY = 3,    /* camera selection, MIS, direct light     */
    AMVPT_K_RAYGEN = 4,        /* G = 1 / adaptive raygen                 */
    AMVPT_K_EXTEND = 5,        /* suffix closest hit                      */
    AMVPT_K_BOUNCE = 6,        /* suffix shading                          */
    AMVPT_K_SHADOW = 7,        /* suffix NEE any-hit                      */
    AMVPT_K_SPLAT = 8,         /* ImageBlock::put                         */
    AMVPT_K_SUFFIX = 9,        /* ABI 7: the whole suffix in one launch (closest hit + shading + NEE, brute-force scenes) */
    AMVPT_K_SELECT = 10,       /* ABI 9: the adaptive fill's compaction of the adapt_mask lanes (k_select_flagged) */
    AMVPT_K_BIN = 11,          /* ABI 9: ray binning of the per-lane suffix walks (k_bin_sort) */
    AMVPT_K_COUNT = 12
} amvpt_kernel_id;

typedef struct amvpt_scene amvpt_scene; /* opaque device-resident scene */

/* Library / device */
const char *amvpt_last_error(void);
uint32_t amvpt_abi_version(void);
amvpt_status amvpt_device_count(int *count);
amvpt_status amvpt_set_device(int device);

/* Upload the scene (shapes, BSDFs, emitters) and build the BVH. */
amvpt_status amvpt_scene_create(const amvpt_scene_desc *desc, amvpt_scene **out);
amvpt_status amvpt_scene_destroy(amvpt_scene *scene);
/* BVH statistics for tests / DESIGN: node and primitive count. */
amvpt_status amvpt_scene_stats(const amvpt_scene *scene, uint32_t *n_nodes, uint32_t *n_prims);
/* ABI 9, host only (no device needed): the box meshes amvpt_scene_create recognises in a descriptor (a `cube`,
 * or any 12-triangle mesh tiling the faces of a parallelepiped; used by the brute-force walks of scenes of at
 * most 48 primitives, DESIGN.md "Box meshes") */
amvpt_status amvpt_scene_desc_boxes(const amvpt_scene_desc *d, uint32_t *n_boxes);

/* Number of channels of the ImageBlock (4 = RGBW, 5 = RGBAW). */
uint32_t amvpt_film_channels(const amvpt_params *params);

/*
 * Render all passes of one frame into a device-resident film of
 * film_height*film_width*channels fp32 (row-major, channel-minor, exactly the
 * ImageBlock tensor layout).  The film is accumulated into (not cleared).
 *
 * Lanes [lane_begin, lane_end) of every pass are processed (lane = global
 * wavefront index, mvpath.cpp:174); passing [0, UINT64_MAX) renders the whole
 * frame.  Lanes keep their global index for TEA seeding, so results are
 * identical for any sharding.  `stream` is a hipStream_t (NULL: default).
 */
amvpt_status amvpt_render(amvpt_scene *scene, const amvpt_view_desc *views,
                          const amvpt_params *params, uint64_t lane_begin,
                          uint64_t lane_end, float *film_device, void *stream,
                          amvpt_counters *counters);

/*
 * Test hook (parity): like amvpt_render, and additionally writes the per-lane,
 * per-view ImageBlock::put arguments of pass `pass` to records_device as
 * 8 floats [pos.x, pos.y, r, g, b, alpha, weight, valid] laid out
 * [(lane - lane_begin) * G + view_slot], G = group size (1 without reuse).
 */
amvpt_status amvpt_render_records(amvpt_scene *scene, const amvpt_view_desc *views,
                                  const amvpt_params *params, uint32_t pass,
                                  uint64_t lane_begin, uint64_t lane_end, float *film_device,
                                  float *records_device, void *stream);

/* Frame geometry the render will use: spp after rounding, passes, lanes per pass. */
amvpt_status amvpt_plan(const amvpt_params *params, uint32_t *spp, uint32_t *spp_per_pass,
                        uint32_t *n_passes, uint64_t *lanes_per_pass);

/* hdrfilm develop: rgb[h*w*c_out] = film[...]/W (W==0 -> 1); c_out = 3 (+1 alpha). */
amvpt_status amvpt_develop(const float *film_device, float *out_device, uint32_t width,
                           uint32_t height, uint32_t film_alpha, void *stream);

/* Tuning knobs (0 keeps the default). chunk_lanes bounds the lanes per chunk; 0 restores the automatic
 * chunk: 2^26 lanes, halved while one buffer set would exceed 48 GB (about 700 B per lane for a mesh scene at
 * G = 8, 46 GB per set; 26 GB at config M).  BVH scenes run up to four buffer sets on as many streams (192 GB
 * at most).  Every render then fits its chunk and sets to a device-memory budget (amvpt_render_opts.budget_mib;
 * automatic: the device's free memory plus what the arena holds, less max(2 GiB, 1/64 of the device)) by
 * dropping buffer sets, then halving the chunk; results do not depend on either.  The arena is kept per device
 * for the next render until amvpt_release_device_memory. */
amvpt_status amvpt_set_chunk_lanes(uint64_t chunk_lanes);
/* BVH walk: 0 auto (wave-uniform for <= 255 nodes, else per-lane; scenes of <= 48
 * primitives test every primitive in the suffix walks instead), 1 force the wave-uniform
 * BVH walk, 2 force per-lane.  Results are identical in every mode (closest hit = min (t, prim)). */
amvpt_status amvpt_set_traversal(uint32_t mode);
/* BVH build of later amvpt_scene_create calls: leaves keep up to max_leaf_prims (1..15,
 * default 4) primitives unless splitting is cheaper; a split costs traversal_cost
 * primitive tests per unit area (default 0).  Hits are identical for every shape. */
amvpt_status amvpt_set_bvh_build(uint32_t max_leaf_prims, float traversal_cost);

/*
 * Adaptive fill over a lane range (adaptive > 0 with lane_begin/lane_end not the
 * whole pass).  The fill re-traces the pass's flagged lanes in compressed order
 * and seeds its sampler from the size of the WHOLE pass's compressed array
 * (mvpath_multi.h:81-90: dr::compress, dr::repeat, sampler->seed(wavefront,
 * wavefront)), so a rank rendering [lane_begin, lane_end) must learn, once per
 * pass, how many flagged lanes lie in lower ranges (`prefix`) and in the whole
 * pass (`total`).  The host supplies that exchange (an all-gather of one
 * integer per rank: MPI, RCCL, torch.distributed, ...); it receives this
 * range's flagged-lane count and returns 0 on success.  Every rank calls
 * amvpt_render with the same params and disjoint ranges; NULL clears it, and
 * without it a partial-range adaptive render is refused.
 */
typedef int (*amvpt_exchange_fn)(void *ctx, uint64_t local_count, uint64_t *prefix, uint64_t *total);
amvpt_status amvpt_set_adaptive_exchange(amvpt_exchange_fn fn, void *ctx);

/* ------------------------------------------------------------------ */
/* ABI 8: one rank's share of a frame, with per-call options           */
/* ------------------------------------------------------------------ */

/*
 * The lanes of one render (a rank's share of the frame).  Lane = global
 * wavefront index (mvpath.cpp:173-190: pixel = lane / spp_per_pass, pixel = y * W + x).
 *   rect_width == 0: the contiguous lanes [lane_begin, lane_end) of every pass (a band of
 *                    quilt rows: the strong-scaling lane shards of configs M / C3 / C4);
 *   rect_width  > 0: the lanes of the quilt pixels [rect_x0, rect_x0 + rect_width) x
 *                    [rect_y0, rect_y0 + rect_height) -- one RUN of rect_width * spp_per_pass
 *                    consecutive lanes per pixel row.  A view group's tiles (mvpath_multi.h:31-38,
 *                    grid.cpp:269-297) form such a rectangle: the view-group partition of C5
 *                    ("4 views per GPU"), whose reprojected splats stay inside the group's tiles.
 */
typedef struct amvpt_lane_set {
    uint64_t lane_begin, lane_end;
    uint32_t rect_x0, rect_y0, rect_width, rect_height;
} amvpt_lane_set;

/*
 * The film of one render: a device RGBW (RGBAW) fp32 buffer of height x width pixels holding
 * the quilt rectangle [x0, x0 + width) x [y0, y0 + height) (row-major, channel-minor, the
 * ImageBlock layout; 0, 0, W, H = the whole ImageBlock).  Splats are clipped to the quilt as
 * ImageBlock::put does (imageblock.cpp:265-558); a footprint cell of the quilt outside the
 * window is appended to `overflow` (device): a 16-byte header whose first u64 counts the cells,
 * then entries of 4 u32 {quilt float index lo, hi, f32 value bits, 0}, at most overflow_capacity
 * of them (the count keeps counting past it).  Renders APPEND to the list: the caller zeroes the
 * 16-byte header before the first render into it; a render fails with AMVPT_ERR_OOM when the list's
 * count passes its capacity, and counters.film_overflow reports the cells this render added.  A window
 * smaller than the quilt needs an overflow buffer.  Summing every window into its rectangle and
 * every overflow entry into its float gives the whole-quilt ImageBlock (float summation order aside).
 */
typedef struct amvpt_film_window {
    float *film;
    uint32_t x0, y0, width, height;
    uint32_t *overflow;
    uint64_t overflow_capacity;
} amvpt_film_window;

/*
 * Adaptive fill over a lane set that is not the whole pass (ABI 8).  The fill re-traces the
 * pass's flagged lanes in compressed order and seeds from the WHOLE pass's compressed array
 * (mvpath_multi.h:79-115), so every run of every rank's lane set needs the number of flagged
 * lanes of the whole pass below its first lane.  Called once per pass with this render's runs
 * (ascending lane_begin; a contiguous lane set is one run) and their flagged-lane counts; fills
 * run_prefix[i] = flagged lanes of the pass with a lane index < run_lane_begin[i] (all ranks)
 * and *total = flagged lanes of the pass.  Runs of different ranks must not interleave.  Every
 * rank calls it once per pass (an empty lane set with n_runs = 0).  Returns 0 on success.
 */
typedef int (*amvpt_run_exchange_fn)(void *ctx, uint32_t n_runs, const uint64_t *run_lane_begin,
                                     const uint64_t *run_count, uint64_t *run_prefix, uint64_t *total);

/* Per-call options (ABI 8; NULL = defaults): replace the process-global knobs above, so
 * concurrent renders (two scenes, or several ranks in one process) do not share state. */
enum {
    /* amvpt_render_opts.flags: kernel-path selection for tests and A/B runs (results are identical) */
    AMVPT_OPT_GENERIC_KERNELS = 1u,   /* no all-diffuse kernel instances (kDiff) */
    AMVPT_OPT_WAVEFRONT_SUFFIX = 2u,  /* per-depth k_extend / k_bounce instead of k_suffix_fused */
    AMVPT_OPT_SPLIT_NEE = 4u,         /* suffix NEE rays in k_shadow instead of inside k_bounce */
    AMVPT_OPT_ONE_STREAM = 8u,        /* every chunk on the render stream (no second chunk stream) */
    AMVPT_OPT_NO_BINNING = 32u,       /* ABI 9: the per-lane suffix walks of large BVHs take the rays in queue order
                                       * (no k_bin_sort); results are identical */
    AMVPT_OPT_NO_BOX_SCREEN = 64u,    /* ABI 9: the brute-force walks of small scenes test every triangle of a box
                                       * mesh (no per-lane face screening); results are identical */
    AMVPT_OPT_THREADED_BVH = 128u,    /* ABI 10: the per-lane suffix walks of large BVHs take the threaded (skip-link)
                                       * tree instead of the two-box one; results are identical */
    AMVPT_OPT_DETERMINISTIC = 16u     /* bitwise-reproducible film: splats summed as 32.32 fixed point with
                                       * integer atomics (order-independent), added to the film once at the
                                       * end; each footprint-cell add is rounded to a multiple of 2^-32 and
                                       * must stay below 2^31 in magnitude: non-finite values (counted by
                                       * nonfinite_samples) and finite ones of |v| >= 2^31 (counted per cell
                                       * add by film_range_drops) are dropped; needs a whole-quilt film window */
};
typedef struct amvpt_render_opts {
    uint64_t chunk_lanes;             /* 0: automatic (see amvpt_set_chunk_lanes) */
    uint32_t traversal;               /* 0 auto, 1 wave-uniform, 2 per-lane (see amvpt_set_traversal) */
    uint32_t flags;                   /* AMVPT_OPT_* */
    amvpt_run_exchange_fn exchange;   /* adaptive fill over a partial lane set */
    void *exchange_ctx;
    float *records;                   /* test hook (parity), NULL: off -- as amvpt_render_records: [v * G + slot][8] */
    uint32_t record_pass;             /*   of pass record_pass, v = the lane's index in the lane set (lane order) */
    uint32_t budget_mib;              /* ABI 10: device memory (MiB) the render's buffers may hold; 0 = automatic (see
                                       * amvpt_set_chunk_lanes).  A budget below the smallest chunk: AMVPT_ERR_OOM */
} amvpt_render_opts;

/*
 * amvpt_render over a lane set into a film window, with per-call options.  amvpt_render(...,
 * lane_begin, lane_end, film, ...) is amvpt_render_ex with the contiguous lane set, the
 * whole-quilt window and the process-global knobs.
 */
amvpt_status amvpt_render_ex(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                             const amvpt_lane_set *lanes, const amvpt_film_window *film, void *stream,
                             const amvpt_render_opts *opts, amvpt_counters *counters);

/*
 * The gather side of a windowed render (ABI 8): add a film window -- height x width x channels fp32
 * holding quilt pixels [x0, x0 + width) x [y0, y0 + height) -- and n_entries overflow entries (the
 * 16-byte entries that follow an overflow list's header) into a whole-quilt film of quilt_height x
 * quilt_width x channels.  Device pointers; the adds are ordered on `stream`.
 */
amvpt_status amvpt_film_accumulate(float *quilt, uint32_t quilt_width, uint32_t quilt_height, uint32_t channels,
                                   const float *window, uint32_t x0, uint32_t y0, uint32_t width, uint32_t height,
                                   const uint32_t *overflow_entries, uint64_t n_entries, void *stream);

/*
 * ABI 10: free the lane arena (chunk buffer sets, adaptive / deterministic / sampler-state buffers) renders keep
 * on `device` between frames, once the last render that used it has finished.  Dr.Jit frees a render's
 * wavefront buffers when the render returns; here the arena is kept for the next frame (a frame of config M
 * reuses 26 GB) until this call.  The host scene's destructor calls it for every device it rendered on.  A later
 * render allocates again.
 */
amvpt_status amvpt_release_device_memory(int device);

/*
 * ABI 10: the two-box BVH of a scene (dscene.h DNode2) its per-lane suffix walks take: node count (0: the scene
 * keeps the threaded walks -- a BVH small enough for the wave-uniform or LDS-staged walks, or one deeper than the
 * walks' 16-entry stack) and the tree's depth in inner nodes (also when not built).
 */
amvpt_status amvpt_scene_bvh2(const amvpt_scene *scene, uint32_t *n_nodes2, uint32_t *depth);

#ifdef __cplusplus
}
#endif

#endif /* AMVPT_H */
