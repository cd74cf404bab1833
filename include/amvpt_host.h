/*
 * amvpt_host.h -- C entry points of libamvpt_host.so, the Mitsuba-style host
 * framework around the hot path (XML scene subset, Properties, plugin
 * registry, MVPathIntegrator / PathIntegrator::render()).
 *
 * These mirror what the reference exposes to its front-ends:
 *   amvpt_host_load_file / _load_string  <- xml::load_file / load_string
 *                                           (src/core/xml.cpp; mitsuba_render.cpp:347)
 *   amvpt_host_render                    <- Integrator::render(scene, sensor_index, seed,
 *                                           spp, develop, evaluate)  integrator.cpp:30-42,
 *                                           dispatching to MVPathIntegrator::render mvpath.cpp:7-278
 *   amvpt_host_write_exr                 <- Film::write (hdrfilm.cpp, OpenEXR float32)
 *   amvpt_host_parse_fov / _perspective_projection
 *                                        <- parse_fov sensor.cpp:163-214,
 *                                           perspective_projection sensor.h:319-356
 * Errors: non-zero return + amvpt_host_last_error() carrying the reference's
 * Throw() message text.
 */
#ifndef AMVPT_HOST_H
#define AMVPT_HOST_H

#include "amvpt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct amvpt_host_scene amvpt_host_scene;

const char *amvpt_host_last_error(void);

/* Load a scene; defines are `-D key=value` substitutions for <default>/$key. */
amvpt_host_scene *amvpt_host_load_file(const char *path, const char *const *keys,
                                       const char *const *values, int n_defines);
amvpt_host_scene *amvpt_host_load_string(const char *xml, const char *const *keys,
                                         const char *const *values, int n_defines);
void amvpt_host_scene_free(amvpt_host_scene *scene);

/* Film geometry of a sensor: quilt width/height, developed channels (3 or 4). */
int amvpt_host_film_info(amvpt_host_scene *scene, uint32_t sensor_index, uint32_t *width,
                         uint32_t *height, uint32_t *channels, uint32_t *sample_count);
uint32_t amvpt_host_sensor_count(amvpt_host_scene *scene);

/*
 * Integrator::render(scene, sensor, seed, spp, develop=true).  Writes the developed
 * H x W x channels image to out_host (or the raw ImageBlock H x W x (4|5) when
 * raw != 0).  spp = 0 uses the sampler's sample_count.  Runs on the current HIP device.
 */
int amvpt_host_render(amvpt_host_scene *scene, uint32_t sensor_index, uint32_t seed, uint32_t spp,
                      int raw, float *out_host, amvpt_counters *counters);

/*
 * amvpt_host_render on a caller stream (hipStream_t; NULL: the default stream).  Both run through
 * amvpt_render_ex with explicit default options (no process-global knob), keep the device scene
 * (BVH build + upload) and the film / image buffers on the host scene per device for the next frame,
 * and serialise renders of one host scene (its cached buffers); renders of different host scenes from
 * different threads are independent.  Returns once the image is in out_host.
 */
int amvpt_host_render_stream(amvpt_host_scene *scene, uint32_t sensor_index, uint32_t seed, uint32_t spp,
                             int raw, float *out_host, void *stream, amvpt_counters *counters);
/* amvpt_host_render's cache counters: device-scene creations, buffer allocations, renders */
int amvpt_host_render_stats(amvpt_host_scene *scene, uint64_t *scene_creates, uint64_t *buffer_allocs,
                            uint64_t *renders);

/*
 * Integrator::render over n_devices GPUs of one node, one host thread per device.
 * View groups, when they divide among the devices (C5): devices[r] renders the lanes of its groups'
 * quilt tiles into a film window (tiles + filter border), the windows and overflow cells go to
 * devices[0] (ncclSend / ncclRecv) and are summed into the ImageBlock there (amvpt_film_accumulate).
 * Otherwise lane bands: devices[r] renders amvpt_host_lane_shard(L, r, n_devices) of every pass into
 * its own RGBW ImageBlock and the blocks are summed onto devices[0] with one ncclReduce.  Developed on
 * devices[0].  The adaptive fill's per-run count exchange runs between the threads (per-call option).
 * Communicators, per-device scenes and films are cached on the scene for the next frame.  The image
 * equals amvpt_host_render's up to float summation order.  Counters: lane statistics summed, times of
 * the slowest device.  A list naming ONE device several times is a shared-device rehearsal (one rank per
 * entry on that device, the films summed on it with amvpt_film_accumulate instead of RCCL; adaptive renders
 * are refused there, their count exchange needs concurrent renders); other repeated devices are an error.
 */
int amvpt_host_render_multi(amvpt_host_scene *scene, uint32_t sensor_index, uint32_t seed, uint32_t spp,
                            int raw, const int *devices, int n_devices, float *out_host,
                            amvpt_counters *counters);

/* [begin, end) of rank's contiguous lane range (sizes differ by at most one; amvpt.dist.lane_shard) */
void amvpt_host_lane_shard(uint64_t lanes, uint32_t rank, uint32_t world, uint64_t *begin, uint64_t *end);

/* The view-group partition of amvpt_host_render_multi (amvpt.dist.view_group_partition): rank's lane
 * rectangle and film window {x0, y0, width, height}; returns 1, or 0 when the view groups do not
 * divide among `world` devices as rectangles of quilt tiles (lane bands are used then). */
int amvpt_host_view_group_partition(const amvpt_params *params, uint32_t rank, uint32_t world, uint32_t *rect,
                                    uint32_t *window);

/* render_multi's per-scene cache (communicators, per-device scene copies, streams, films): how many
 * scene creations, communicator initialisations and completed multi-GPU renders it has seen. */
int amvpt_host_multi_stats(amvpt_host_scene *scene, uint64_t *scene_creates, uint64_t *comm_inits, uint64_t *renders);

/*
 * Test hook (CPU, no device): amvpt_host_render_multi's rank coordination (host/ranks.h: phase barriers,
 * the in-process count exchange and its abort) with n rank threads that each make `passes` count
 * exchanges in the render phase; rank fail_rank fails in phase fail_phase (0 setup, 1 render before its
 * exchanges, 2 render between them, 3 render after them, 4 before the gather, 5 finish; -1 none).
 * Returns 0 when every rank succeeded, 1 with the reported (first own) failure in
 * amvpt_host_last_error(), 2 if an exchange returned a wrong prefix.  Never leaves a thread blocked.
 */
int amvpt_host_test_ranks(int n, int passes, int fail_rank, int fail_phase);

/*
 * The exact descriptors render() hands to the C-ABI (for the parity tests: the oracle
 * consumes the same scene, views and params).  Pointers stay valid until the scene is freed.
 */
int amvpt_host_describe(amvpt_host_scene *scene, uint32_t sensor_index, uint32_t seed, uint32_t spp,
                        const amvpt_scene_desc **scene_desc, const amvpt_view_desc **views,
                        amvpt_params *params);

/* Text summary of the integrator (Integrator::to_string). */
const char *amvpt_host_integrator_string(amvpt_host_scene *scene);

/* OpenEXR (uncompressed float32 scanlines) writer / reader: channels 3 (RGB) or 4 (RGBA). */
int amvpt_host_write_exr(const char *path, const float *data, uint32_t width, uint32_t height,
                         uint32_t channels);
int amvpt_host_read_exr(const char *path, float *data, uint32_t width, uint32_t height,
                        uint32_t channels);

/* Known-answer hooks (sensor.cpp / sensor.h). fov_axis: "x","y","smaller","larger","diagonal". */
double amvpt_host_parse_fov(double fov, const char *fov_axis, const char *focal_length, double aspect);
void amvpt_host_perspective_projection(const int *film_size, const int *crop_size,
                                       const int *crop_offset, float fov_x, float near_clip,
                                       float far_clip, float *matrix16);

#ifdef __cplusplus
}
#endif

#endif /* AMVPT_HOST_H */
