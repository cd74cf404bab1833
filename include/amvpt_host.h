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
 * Integrator::render over n_devices GPUs of one node, one host thread per device:
 * device devices[r] renders the lane range amvpt_host_lane_shard(L, r, n_devices) of every pass
 * (L = lanes per pass, amvpt_plan) into its own RGBW ImageBlock; the blocks are summed onto
 * devices[0] with one RCCL reduce (ncclReduce, sum, fp32, communicators from ncclCommInitAll) and
 * developed there.  The adaptive fill's per-pass count exchange runs between the threads.  The
 * image equals amvpt_host_render's up to float summation order.  Counters: lane statistics summed,
 * times of the slowest device.
 */
int amvpt_host_render_multi(amvpt_host_scene *scene, uint32_t sensor_index, uint32_t seed, uint32_t spp,
                            int raw, const int *devices, int n_devices, float *out_host,
                            amvpt_counters *counters);

/* [begin, end) of rank's contiguous lane range (sizes differ by at most one; amvpt.dist.lane_shard) */
void amvpt_host_lane_shard(uint64_t lanes, uint32_t rank, uint32_t world, uint64_t *begin, uint64_t *end);

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
