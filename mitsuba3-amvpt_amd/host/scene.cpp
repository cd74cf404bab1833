/*
 * scene.cpp -- plugin layer of the host framework: turns the loaded scene
 * graph into the C-ABI descriptors and implements Integrator::render() for
 * the `mvpath` and `path` plugins on top of libamvpt_hip.so.
 *
 * Plugin constructors restated (reference file:line):
 *   MVPathIntegrator        src/integrators/mvpath.h:120-129, integrator.cpp:22-28,505-522
 *   MVPathIntegrator::render checks (MultiSensor, subsensor type)  mvpath.cpp:15-46
 *   GridSensor              src/sensors/grid.cpp:84-236
 *   PerspectiveCamera       src/sensors/perspective.cpp:140-203; parse_fov sensor.cpp:163-214
 *   Sensor (film / sampler / wrap lookup)  src/render/sensor.cpp:15-88
 *   Film / HDRFilm          src/render/film.cpp:7-52, src/films/hdrfilm.cpp:130-300
 *   GaussianFilter          src/rfilters/gaussian.cpp:46-52
 *   IndependentSampler      src/render/sampler.cpp:10-16
 *   Rectangle / Cube / Sphere src/shapes/rectangle.cpp:98-123, cube.cpp:105-160, sphere.cpp:126-169
 *   default BSDF            src/render/shape.cpp:64-70
 *   SmoothDiffuse / RoughConductor / TwoSided  diffuse.cpp:88-93, roughconductor.cpp:160-211, twosided.cpp:60-100
 *   AreaLight               src/emitters/area.cpp:40-80
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/amvpt.h"
#include "../../include/amvpt_host.h"
#include "xml.h"
#include "meshio.h"

namespace mi {

static std::string lower(std::string s) {
    for (auto &c : s) c = (char) std::tolower((unsigned char) c);
    return s;
}

[[noreturn]] static void Throw(const std::string &m) { throw std::runtime_error(m); }

/* parse_fov (src/render/sensor.cpp:163-214) */
double parse_fov(const Properties &props, double aspect) {
    if (props.has("fov") && props.has("focal_length"))
        Throw("Please specify either a focal length ('focal_length') or a field of view ('fov')!");
    double fov;
    std::string fov_axis;
    if (props.has("fov")) {
        fov = props.get_float("fov", 0.0);
        fov_axis = lower(props.get_string("fov_axis", "x"));
        if (fov_axis == "smaller") fov_axis = aspect > 1 ? "y" : "x";
        else if (fov_axis == "larger") fov_axis = aspect > 1 ? "x" : "y";
    } else {
        std::string f = props.get_string("focal_length", "50mm");
        if (f.size() > 2 && f.substr(f.size() - 2) == "mm") f = f.substr(0, f.size() - 2);
        char *end = nullptr;
        double value = std::strtod(f.c_str(), &end);
        if (end == f.c_str())
            Throw("Could not parse the focal length (must be of the form <x>mm, where <x> is a positive integer)!");
        fov = 2.0 * (180.0 / M_PI) * std::atan(std::sqrt(double(36 * 36 + 24 * 24)) / (2.0 * value));
        fov_axis = "diagonal";
    }
    double result;
    if (fov_axis == "x") result = fov;
    else if (fov_axis == "y") result = (180.0 / M_PI) * (2.0 * std::atan(std::tan(0.5 * fov * (M_PI / 180.0)) * aspect));
    else if (fov_axis == "diagonal") {
        double diagonal = 2.0 * std::tan(0.5 * fov * (M_PI / 180.0));
        double width = diagonal / std::sqrt(1.0 + 1.0 / (aspect * aspect));
        result = (180.0 / M_PI) * (2.0 * std::atan(width * 0.5));
    } else {
        Throw("The 'fov_axis' parameter must be set to one of 'smaller', 'larger', 'diagonal', 'x', or 'y'!");
    }
    if (result <= 0.0 || result >= 180.0) Throw("The horizontal field of view must be in the range [0, 180]!");
    return result;
}

/* ------------------------------------------------------------------ */
/* Films / samplers / sensors                                          */
/* ------------------------------------------------------------------ */

struct FilmInfo {
    uint32_t w = 768, h = 576;
    uint32_t cw = 768, ch = 576, cx = 0, cy = 0;   /* crop window (film.cpp:16-27; Film::set_size resets it) */
    void reset_crop() { cw = w; ch = h; cx = cy = 0; }
    bool alpha = false;
    uint32_t rfilter = AMVPT_RFILTER_GAUSSIAN;
    float stddev = 0.5f;
};

static FilmInfo make_film(const Properties &p) {
    if (lower(p.plugin) != "hdrfilm") Throw("Film plugin \"" + p.plugin + "\" is not implemented (hdrfilm only)");
    FilmInfo f;
    f.w = (uint32_t) p.get_int("width", 768);
    f.h = (uint32_t) p.get_int("height", 576);
    /* Film ctor (film.cpp:16-27) + set_crop_window (film.cpp:91-100) */
    f.cw = (uint32_t) p.get_int("crop_width", f.w);
    f.ch = (uint32_t) p.get_int("crop_height", f.h);
    f.cx = (uint32_t) p.get_int("crop_offset_x", 0);
    f.cy = (uint32_t) p.get_int("crop_offset_y", 0);
    if ((uint64_t) f.cx + f.cw > f.w || (uint64_t) f.cy + f.ch > f.h)
        Throw("Invalid crop window specification: crop_offset(" + std::to_string(f.cx) + ", " + std::to_string(f.cy) +
              ") + crop_size(" + std::to_string(f.cw) + ", " + std::to_string(f.ch) + ") > size(" +
              std::to_string(f.w) + ", " + std::to_string(f.h) + ")");
    if (p.get_bool("sample_border", false)) Throw("hdrfilm: sample_border is not implemented");
    std::string pf = lower(p.get_string("pixel_format", "rgb"));
    if (pf == "rgb") f.alpha = false;
    else if (pf == "rgba") f.alpha = true;
    else Throw("hdrfilm: pixel_format \"" + pf + "\" is not implemented (rgb, rgba)");
    /* output-file keys of hdrfilm (hdrfilm.cpp:172-215): they shape the written file, not the
     * ImageBlock; the EXR writer (exr.cpp) writes float32 OpenEXR */
    const std::string ff = lower(p.get_string("file_format", "openexr"));
    if (ff != "openexr" && ff != "exr") Throw("hdrfilm: file_format \"" + ff + "\" is not implemented (openexr)");
    (void) p.get_string("component_format", "float16");
    (void) p.get_bool("banner", true);
    (void) p.get_bool("compensate", false);
    int n_filters = 0;
    for (auto &e : p.entries) {
        if (e.second.kind != Properties::Obj || e.second.o->tag != "rfilter") continue;
        if (n_filters++) Throw("A film can only have one reconstruction filter.");
        p.mark_queried(e.first);   /* film.cpp:34-42 */
        const Properties &rp = e.second.o->props;
        std::string t = lower(rp.plugin);
        if (t == "gaussian") { f.rfilter = AMVPT_RFILTER_GAUSSIAN; f.stddev = (float) rp.get_float("stddev", 0.5); }
        else if (t == "box") f.rfilter = AMVPT_RFILTER_BOX;
        else Throw("rfilter \"" + t + "\" is not implemented (gaussian, box)");
    }
    return f;
}

struct SamplerInfo { uint32_t sample_count = 4, seed = 0; };
static SamplerInfo make_sampler(const Properties &p) {
    if (lower(p.plugin) != "independent")
        Throw("Sampler \"" + p.plugin + "\" is not implemented (mvpath optimises the independent sampler, mvpath.cpp:43)");
    SamplerInfo s;
    s.sample_count = (uint32_t) p.get_int("sample_count", 4);
    s.seed = (uint32_t) p.get_int("seed", 0);
    return s;
}

/* Wrap (src/render/wrap.cpp:6-22): its Properties become a plugin of class wrap_class / type wrap_type */
static Properties unwrap(const Object &w) {
    Properties p = w.props;
    p.plugin = p.get_string("wrap_type");
    p.remove("wrap_class");
    p.remove("wrap_type");
    return p;
}
static std::string wrap_class(const Object &w) { return w.props.get_string("wrap_class"); }

/* Sensor base: film / sampler lookup (sensor.cpp:25-75) */
static void sensor_parts(const Properties &p, FilmInfo &film, SamplerInfo &samp) {
    bool hf = false, hs = false;
    for (auto &e : p.entries) {
        if (e.second.kind != Properties::Obj) continue;
        const Object &o = *e.second.o;
        if (o.tag == "film") {
            if (hf) Throw("Only one film can be specified per sensor.");
            film = make_film(o.props); hf = true;
            p.mark_queried(e.first);   /* sensor.cpp:25-41 */
        } else if (o.tag == "sampler") {
            if (hs) Throw("Only one sampler can be specified per sensor.");
            samp = make_sampler(o.props); hs = true;
            p.mark_queried(e.first);
        } else if (o.tag == "wrap") {
            std::string c = wrap_class(o);
            if (c == "film") { if (hf) Throw("Only one film can be specified per sensor."); film = make_film(unwrap(o)); hf = true; }
            else if (c == "sampler") { if (hs) Throw("Only one sampler can be specified per sensor."); samp = make_sampler(unwrap(o)); hs = true; }
            else continue;
            p.mark_queried(e.first);   /* the sensor read its film / sampler, wrapped or not */
        }
    }
    if (!hf) film = FilmInfo();
    if (!hs) samp = SamplerInfo();
}

static void store3x4(const Mat4 &m, float *out16) { m.store(out16); }

/* PerspectiveCamera ctor + update_camera_transforms (perspective.cpp:140-203) for a film of size (w,h)
 * with the crop window (cw, ch) at (cx, cy) (0 / 0: the whole film) */
static amvpt_view_desc make_perspective_view(const Properties &p, const Transform4f &to_world, uint32_t w, uint32_t h,
                                             double fov_x_override, bool use_override, float lens_shift,
                                             uint32_t cw = 0, uint32_t ch = 0, uint32_t cx = 0, uint32_t cy = 0) {
    if (!cw) { cw = w; ch = h; cx = cy = 0; }
    amvpt_view_desc v;
    std::memset(&v, 0, sizeof(v));
    std::string t = lower(p.plugin);
    if (t == "thinlens") v.type = AMVPT_CAMERA_THINLENS;
    else if (t == "perspective") v.type = AMVPT_CAMERA_PERSPECTIVE;
    else Throw("Subsensor must be of type ThinLensCamera or PerspectiveCamera !");
    /* Sensor base (sensor.cpp:14-22, 72-80): no time sample on the implemented path, no spectral response */
    const float shutter_open = (float) p.get_float("shutter_open", 0.0);
    const float shutter_time = (float) p.get_float("shutter_close", 0.0) - shutter_open;
    if (shutter_time < 0.f) Throw("Shutter opening time must be less than or equal to the shutter closing time!");
    if (shutter_time > 0.f) Throw("A shutter interval (time sample, motion blur) is not implemented");
    if (p.has("srf")) Throw("A sensor response function ('srf') is not implemented (rgb variants)");
    float near_clip = (float) p.get_float("near_clip", 1e-2), far_clip = (float) p.get_float("far_clip", 1e4);
    if (near_clip <= 0.f) Throw("The 'near_clip' parameter must be greater than zero!");
    if (near_clip >= far_clip) Throw("The 'near_clip' parameter must be smaller than 'far_clip'.");
    if (to_world.has_scale()) Throw("Scale factors in the camera-to-world transformation are not allowed!");
    float x_fov = use_override ? (float) fov_x_override : (float) parse_fov(p, (double) w / (double) h);
    int size[2] = {(int) w, (int) h}, crop[2] = {(int) cw, (int) ch}, off[2] = {(int) cx, (int) cy};
    Transform4f c2s = perspective_projection(size, crop, off, x_fov, near_clip, far_clip);
    c2s.matrix.m[0][2] += lens_shift;
    c2s.inverse_transpose = c2s.matrix.inverse().transpose();
    Transform4f s2c = c2s.inverse();
    V3f pmin = s2c.apply_point_h({0.f, 0.f, 0.f}), pmax = s2c.apply_point_h({1.f, 1.f, 0.f});
    float ax = pmin.x / pmin.z, ay = pmin.y / pmin.z, bx = pmax.x / pmax.z, by = pmax.y / pmax.z;
    float lx = std::min(ax, bx), hx = std::max(ax, bx), ly = std::min(ay, by), hy = std::max(ay, by);
    v.normalization = 1.f / ((hx - lx) * (hy - ly));
    store3x4(to_world.matrix, v.to_world);
    store3x4(to_world.inverse().matrix, v.to_world_inv);
    s2c.matrix.store(v.sample_to_camera);
    c2s.matrix.store(v.camera_to_sample);
    v.near_clip = near_clip;
    v.far_clip = far_clip;
    v.resolution[0] = (float) cw;   /* m_resolution = film->crop_size() (sensor.cpp:69) */
    v.resolution[1] = (float) ch;
    float ppx = (float) p.get_float("principal_point_offset_x", 0.0), ppy = (float) p.get_float("principal_point_offset_y", 0.0);
    v.pp_offset[0] = (float) w * ppx / (float) cw;   /* film.size * principal_point_offset / crop_size */
    v.pp_offset[1] = (float) h * ppy / (float) ch;
    v.focus_distance = (float) p.get_float("focus_distance", far_clip);
    v.aperture_radius = v.type == AMVPT_CAMERA_THINLENS ? (float) p.get_float("aperture_radius", 0.0) : 0.f;
    if (v.type == AMVPT_CAMERA_THINLENS) {
        /* thinlens.cpp:156-162 */
        if (!p.has("aperture_radius")) Throw("Property \"aperture_radius\" has not been specified!");
        if (v.aperture_radius == 0.f) v.aperture_radius = 5.9604645e-8f; /* dr::Epsilon<float> */
    }
    return v;
}

struct SensorInfo {
    bool multisensor = false;
    bool batch = false;
    uint32_t gx = 1, gy = 1;
    bool rev_x = false, rev_y = false;
    FilmInfo film;           /* quilt film */
    SamplerInfo sampler;
    std::vector<amvpt_view_desc> views;
};

static SensorInfo make_sensor(const Object &o) {
    SensorInfo s;
    const Properties &p = o.props;
    std::string t = lower(p.plugin);
    sensor_parts(p, s.film, s.sampler);
    Transform4f to_world = p.get_transform("to_world");
    if (t == "perspective" || t == "thinlens") {
        s.views.push_back(make_perspective_view(p, to_world, s.film.w, s.film.h, 0.0, false,
                                                (float) p.get_float("lens_shift", 0.0), s.film.cw, s.film.ch, s.film.cx,
                                                s.film.cy));
        return s;
    }
    if (t == "batch") {
        /* BatchSensor (batch.cpp:94-131): child sensors side by side on one film */
        s.multisensor = true;
        s.batch = true;
        s.rev_x = p.get_bool("reverse_x", false);
        s.rev_y = p.get_bool("reverse_y", false);
        std::vector<const Object *> kids;
        for (auto &e : p.objects()) {   /* batch.cpp:96: props.objects() */
            const Object &c = *e.second;
            if (c.tag == "sensor") kids.push_back(&c);
            else if (c.tag == "shape")
                Throw("BatchSensor: shapes can only be specified as children if a sensor is associated with them!");
        }
        if (kids.empty()) Throw("BatchSensor: at least one child sensor must be specified!");
        const uint32_t n = (uint32_t) kids.size(), sub = s.film.w / n;
        if (sub * n != s.film.w)
            Throw("BatchSensor: the horizontal resolution (currently " + std::to_string(s.film.w) +
                  ") must be divisible by the number of child sensors (" + std::to_string(n) + ")!");
        s.gx = n;
        s.gy = 1;
        for (const Object *c : kids) {
            const Properties &cp = c->props;
            std::string ct = lower(cp.plugin);
            if (ct != "perspective" && ct != "thinlens") Throw("Sensor \"" + cp.plugin + "\" is not implemented (perspective)");
            /* the child computes its fov from ITS OWN film at construction, then the batch
             * resizes that film to (sub, h) and rebuilds the projection (batch.cpp:122-126) */
            FilmInfo cf;
            SamplerInfo cs;
            sensor_parts(cp, cf, cs);
            const double x_fov = parse_fov(cp, (double) cf.w / (double) cf.h);
            s.views.push_back(make_perspective_view(cp, cp.get_transform("to_world"), sub, s.film.h, x_fov, true,
                                                    (float) cp.get_float("lens_shift", 0.0)));
        }
        return s;
    }
    if (t != "grid") Throw("Sensor \"" + p.plugin + "\" is not implemented (perspective, grid, batch)");
    /* GridSensor (grid.cpp:84-236) */
    s.multisensor = true;
    s.rev_x = p.get_bool("reverse_x", false);
    s.rev_y = p.get_bool("reverse_y", true);
    s.gx = (uint32_t) p.get_int("grid_x", 1);
    s.gy = (uint32_t) p.get_int("grid_y", 1);
    uint32_t res_x = (uint32_t) p.get_int("res_x", 0), res_y = (uint32_t) p.get_int("res_y", 0);
    res_x = res_x ? res_x : s.film.w * s.gx;
    res_y = res_y ? res_y : s.film.h * s.gy;
    if (res_x % s.gx || res_y % s.gy) Throw("Film size must be divisible by grid dimensions !");
    uint32_t sub_x = res_x / s.gx, sub_y = res_y / s.gy;
    double sub_asp = sub_x / double(sub_y);
    uint32_t n = s.gx * s.gy;
    bool used_cone = false, cam_center = false;
    float cone_deg = 0.f, cam_dist = 0.1f;
    V3f cam_dir{1.f, 0.f, 0.f};
    if (p.has("cone_deg")) {
        used_cone = true;
        cone_deg = (float) p.get_float("cone_deg", 0.0);
    } else if (p.has("cam_dir")) {
        cam_dir = p.get_vec3("cam_dir", {1, 0, 0});
        cam_dist = std::sqrt(dot3(cam_dir, cam_dir));
        cam_dist = (float) p.get_float("cam_dist", cam_dist);
        cam_center = p.get_bool("cam_center", true);
    } else if (p.has("cam_end")) {
        V3f beg = to_world.translation(), end = p.get_vec3("cam_end", {0, 0, 0});
        cam_dir = to_world.inverse().apply_vector({end.x - beg.x, end.y - beg.y, end.z - beg.z});
        cam_dist = std::sqrt(dot3(cam_dir, cam_dir));
        cam_dir = {cam_dir.x / cam_dist, cam_dir.y / cam_dist, cam_dir.z / cam_dist};
        cam_center = false;
    }
    V3f cam_off = p.get_vec3("cam_off", {0, 0, 0});
    cam_off.y = -cam_off.y;
    cam_off.z = -cam_off.z;
    const Object *w_sens = nullptr;
    for (auto &e : p.entries) {
        if (e.second.kind != Properties::Obj || e.second.o->tag != "wrap") continue;
        std::string c = wrap_class(*e.second.o);
        if (c == "sensor") {
            if (w_sens) Throw("Only one Wrap of type Sensor can be specified !");
            w_sens = e.second.o.get();
        }
    }
    bool has_film_wrap = false, has_samp_wrap = false;
    for (auto &e : p.entries)
        if (e.second.kind == Properties::Obj && e.second.o->tag == "wrap") {
            std::string c = wrap_class(*e.second.o);
            has_film_wrap |= c == "film";
            has_samp_wrap |= c == "sampler";
        }
    if (!w_sens || !has_film_wrap || !has_samp_wrap) Throw("Need to specify wraps for sensor, film and sampler !");
    Properties sub = unwrap(*w_sens);
    double fov_x = parse_fov(p.has("fov") ? p : sub, sub_asp);
    float foc = (float) sub.get_float("focus_distance", 1.0);
    foc = (float) p.get_float("focus_distance", foc);
    s.views.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        float dt = (float) i / (float) (n - 1);
        Mat4 it = to_world.inverse_transpose;
        float shift = 0.f;
        if (used_cone) {
            float tan_off = std::tan((dt - 0.5f) * (cone_deg * (3.14159265358979323846f / 180.f)));
            float offset = foc * tan_off;
            shift = (float) (0.5 * double(tan_off) / std::tan((fov_x * (M_PI / 180.0)) * 0.5));
            it.m[3][0] += offset + cam_off.x;
            it.m[3][1] += cam_off.y;
            it.m[3][2] += cam_off.z;
        } else {
            float f = cam_dist * (dt - 0.5f * (float) cam_center);
            V3f off{cam_off.x + cam_dir.x * f, cam_off.y + cam_dir.y * f, cam_off.z + cam_dir.z * f};
            it.m[3][0] += off.x;
            it.m[3][1] += off.y;
            it.m[3][2] += off.z;
        }
        Mat4 nt = it.transpose().inverse();
        Transform4f trafo(nt, it);
        s.views.push_back(make_perspective_view(sub, trafo, sub_x, sub_y, fov_x, true, shift));
        s.views.back().focus_distance = foc;
    }
    s.film.w = res_x;
    s.film.h = res_y;
    s.film.reset_crop();
    p.mark_all_queried();   /* grid.cpp:231-232 */   /* m_film->set_size(m_film_res) resets the crop window (grid.cpp:230, film.cpp:102-106) */
    return s;
}

/* ------------------------------------------------------------------ */
/* Scene                                                               */
/* ------------------------------------------------------------------ */

struct IntegratorInfo {
    std::string type = "path";
    amvpt_params p{};
    std::string text;
    float timeout = -1.f;                    /* accepted; unused by the JIT renders (see build) */
    uint32_t samples_per_pass = 0xffffffffu; /* SamplingIntegrator::m_samples_per_pass */
};

struct MeshStore { std::vector<float> pos, nrm, uv; std::vector<uint32_t> faces; };

} // namespace mi

struct amvpt_multi_cache;   /* multi.cpp: communicators, per-device scenes and films of render_multi */
struct amvpt_host_scene {
    std::shared_ptr<mi::Object> root;
    mi::IntegratorInfo integrator;
    std::vector<mi::SensorInfo> sensors;
    std::vector<amvpt_shape_desc> shapes;
    std::vector<amvpt_bsdf_desc> bsdfs;
    std::vector<amvpt_emitter_desc> emitters;
    std::vector<std::unique_ptr<mi::MeshStore>> meshes;
    amvpt_scene_desc desc{};
    bool has_env = false;
    /* amvpt_host_render's per-device state, kept for the next frame: the device scene (BVH build +
     * upload happen once per device, not per frame) and the ImageBlock / developed-image buffers */
    struct DeviceCache {
        int device = -1;
        amvpt_scene *scene = nullptr;
        float *film = nullptr, *image = nullptr;
        size_t film_bytes = 0, image_bytes = 0;
    };
    std::mutex render_mu;                 /* one render of this scene at a time (its cached buffers) */
    std::vector<DeviceCache> devices;
    uint64_t scene_creates = 0, buffer_allocs = 0, renders = 0;
    std::vector<amvpt_view_desc> last_views;
    std::shared_ptr<amvpt_multi_cache> multi;
    ~amvpt_host_scene() {
        multi.reset();
        for (auto &d : devices) {
            int cur = 0;
            const bool have = hipGetDevice(&cur) == hipSuccess;
            if (have) (void) hipSetDevice(d.device);
            if (d.scene) amvpt_scene_destroy(d.scene);
            if (d.film) (void) hipFree(d.film);
            if (d.image) (void) hipFree(d.image);
            (void) amvpt_release_device_memory(d.device);   /* the renders' lane arena on this device (ABI 10) */
            if (have) (void) hipSetDevice(cur);
        }
    }
};

/* multi.cpp's cache slot on the host scene */
std::shared_ptr<amvpt_multi_cache> &amvpt_host_multi_slot(amvpt_host_scene *s) { return s->multi; }

namespace mi {

static void fill_xform(const Transform4f &t, float *to_world, float *to_object) {
    t.matrix.store(to_world);
    t.inverse().matrix.store(to_object);
}

static int add_bsdf(amvpt_host_scene &S, std::map<const Object *, int> &seen, const Object &o) {
    auto it = seen.find(&o);
    if (it != seen.end()) return it->second;
    const Properties &p = o.props;
    std::string t = lower(p.plugin);
    amvpt_bsdf_desc d;
    std::memset(&d, 0, sizeof(d));
    d.nested[0] = d.nested[1] = -1;
    if (t == "diffuse") {
        d.type = AMVPT_BSDF_DIFFUSE;
        float r[3] = {.5f, .5f, .5f};
        p.get_rgb("reflectance", r);
        std::memcpy(d.reflectance, r, 12);
    } else if (t == "roughconductor") {
        d.type = AMVPT_BSDF_ROUGHCONDUCTOR;
        std::string material = p.get_string("material", "none");
        if (p.has("eta") || material == "none") {
            float eta[3] = {0, 0, 0}, k[3] = {1, 1, 1};
            p.get_rgb("eta", eta);
            p.get_rgb("k", k);
            if (material != "none") Throw("Should specify either (eta, k) or material, not both.");
            std::memcpy(d.eta, eta, 12);
            std::memcpy(d.k, k, 12);
        } else {
            Throw("roughconductor: named materials need data/ior/*.spd, absent from the reference checkout; pass eta/k");
        }
        std::string distr = lower(p.get_string("distribution", "beckmann"));
        if (distr == "beckmann") d.distribution = AMVPT_MICROFACET_BECKMANN;
        else if (distr == "ggx") d.distribution = AMVPT_MICROFACET_GGX;
        else Throw("Specified an invalid distribution \"" + distr + "\", must be \"beckmann\" or \"ggx\"!");
        d.sample_visible = p.get_bool("sample_visible", true);
        if (p.has("alpha_u") || p.has("alpha_v")) {
            if (!p.has("alpha_u") || !p.has("alpha_v"))
                Throw("Microfacet model: both 'alpha_u' and 'alpha_v' must be specified.");
            if (p.has("alpha")) Throw("Microfacet model: please specifyeither 'alpha' or 'alpha_u'/'alpha_v'.");
            d.alpha_u = (float) p.get_float("alpha_u", 0.1);
            d.alpha_v = (float) p.get_float("alpha_v", 0.1);
        } else {
            d.alpha_u = d.alpha_v = (float) p.get_float("alpha", 0.1);
        }
        float sr[3];
        if (p.get_rgb("specular_reflectance", sr)) { d.has_specular_reflectance = 1; std::memcpy(d.specular_reflectance, sr, 12); }
    } else if (t == "twosided") {
        d.type = AMVPT_BSDF_TWOSIDED;
        std::vector<const Object *> nested;
        for (auto &e : p.objects())   /* twosided.cpp:75: props.objects() */
            if (e.second->tag == "bsdf") nested.push_back(e.second);
            else Throw("twosided: nested object of type \"" + e.second->tag + "\" is not a BSDF");
        if (nested.empty()) Throw("A nested one-sided material is required!");
        if (nested.size() > 2) Throw("At most two nested BSDFs can be specified!");
        int a = add_bsdf(S, seen, *nested[0]);
        int b = nested.size() == 2 ? add_bsdf(S, seen, *nested[1]) : a;
        d.nested[0] = a;
        d.nested[1] = b;
    } else {
        Throw("BSDF \"" + p.plugin + "\" is not implemented (diffuse, roughconductor, twosided)");
    }
    int idx = (int) S.bsdfs.size();
    S.bsdfs.push_back(d);
    seen[&o] = idx;
    return idx;
}

/* a BSDF add_bsdf can build (its nested BSDFs too) */
static bool bsdf_implemented(const Object &o) {
    const std::string t = lower(o.props.plugin);
    if (t == "diffuse" || t == "roughconductor") return true;
    if (t != "twosided") return false;
    for (auto &e : o.props.objects())
        if (e.second->tag == "bsdf" && !bsdf_implemented(*e.second)) return false;
    return true;
}
static void mark_tree_queried(const Object &o) {
    o.props.mark_all_queried();
    for (auto &e : o.props.objects()) mark_tree_queried(*e.second);
}

/* Cube geometry (src/shapes/cube.cpp:105-160) */
static void cube_mesh(const Transform4f &T, MeshStore &m) {
    static const float V[24][3] = {{1, -1, -1}, {1, -1, 1}, {-1, -1, 1}, {-1, -1, -1}, {1, 1, -1}, {-1, 1, -1},
                                   {-1, 1, 1}, {1, 1, 1}, {1, -1, -1}, {1, 1, -1}, {1, 1, 1}, {1, -1, 1},
                                   {1, -1, 1}, {1, 1, 1}, {-1, 1, 1}, {-1, -1, 1}, {-1, -1, 1}, {-1, 1, 1},
                                   {-1, 1, -1}, {-1, -1, -1}, {1, 1, -1}, {1, -1, -1}, {-1, -1, -1}, {-1, 1, -1}};
    static const float N[24][3] = {{0, -1, 0}, {0, -1, 0}, {0, -1, 0}, {0, -1, 0}, {0, 1, 0}, {0, 1, 0},
                                   {0, 1, 0}, {0, 1, 0}, {1, 0, 0}, {1, 0, 0}, {1, 0, 0}, {1, 0, 0},
                                   {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {0, 0, 1}, {-1, 0, 0}, {-1, 0, 0},
                                   {-1, 0, 0}, {-1, 0, 0}, {0, 0, -1}, {0, 0, -1}, {0, 0, -1}, {0, 0, -1}};
    static const float UV[24][2] = {{0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0},
                                    {0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0},
                                    {0, 1}, {1, 1}, {1, 0}, {0, 0}, {0, 1}, {1, 1}, {1, 0}, {0, 0}};
    static const uint32_t F[12][3] = {{0, 1, 2}, {3, 0, 2}, {4, 5, 6}, {7, 4, 6}, {8, 9, 10}, {11, 8, 10},
                                      {12, 13, 14}, {15, 12, 14}, {16, 17, 18}, {19, 16, 18}, {20, 21, 22}, {23, 20, 22}};
    for (int i = 0; i < 24; ++i) {
        V3f p = T.apply_point({V[i][0], V[i][1], V[i][2]});
        V3f n = normalize3(T.apply_normal({N[i][0], N[i][1], N[i][2]}));
        m.pos.insert(m.pos.end(), {p.x, p.y, p.z});
        m.nrm.insert(m.nrm.end(), {n.x, n.y, n.z});
        m.uv.insert(m.uv.end(), {UV[i][0], UV[i][1]});
    }
    for (auto &f : F) m.faces.insert(m.faces.end(), {f[0], f[1], f[2]});
}

static void build(amvpt_host_scene &S) {
    std::map<const Object *, int> seen;
    const Properties &rp = S.root->props;
    bool have_integrator = false;
    for (auto &e : rp.objects()) {   /* scene.cpp:23: props.objects() */
        const Object &o = *e.second;
        if (o.tag == "integrator") {
            if (have_integrator) Throw("Only one integrator can be specified per scene.");
            have_integrator = true;
            IntegratorInfo &I = S.integrator;
            const Properties &p = o.props;
            I.type = lower(p.plugin);
            std::memset(&I.p, 0, sizeof(I.p));
            long long md = p.get_int("max_depth", -1);
            if (md < 0 && md != -1) Throw("\"max_depth\" must be set to -1 (infinite) or a value >= 0");
            I.p.max_depth = (uint32_t) md;
            long long rr = p.get_int("rr_depth", 5);
            if (rr <= 0) Throw("\"rr_depth\" must be set to a value greater than zero!");
            I.p.rr_depth = (uint32_t) rr;
            I.p.hide_emitters = p.get_bool("hide_emitters", false);
            /* Integrator / SamplingIntegrator keys (integrator.cpp:22-28, 96-116): the JIT render of both
             * integrators never reads `timeout` or `block_size` (the scalar block renderer does);
             * `samples_per_pass` splits the stock path integrator's frame into passes (integrator.cpp:137-146)
             * and is ignored by mvpath, whose pass size is spp_pass_lim (mvpath.cpp:36) */
            I.timeout = (float) p.get_float("timeout", -1.0);
            long long bs = p.get_int("block_size", 0);
            if (bs < 0) Throw("\"block_size\" must be a non-negative integer");
            long long spp_pass = p.get_int("samples_per_pass", -1);
            if (spp_pass < -1 || spp_pass == 0 || spp_pass > 0xffffffffll)
                Throw("\"samples_per_pass\" must be a positive integer");
            I.samples_per_pass = spp_pass == -1 ? 0xffffffffu : (uint32_t) spp_pass;
            if (I.type == "mvpath") {
                I.p.integrator = AMVPT_INTEGRATOR_MVPATH;
                I.p.sa_reuse = p.get_bool("sa_reuse", false);
                I.p.sa_mis = p.get_bool("sa_mis", false);
                I.p.fast_mis = p.get_bool("fast_mis", false);
                I.p.debug = p.get_bool("debug", false);
                I.p.adaptive = (uint32_t) p.get_int("adaptive", 0);
                I.p.spp_pass_lim = (uint32_t) p.get_int("spp_pass_lim", 16);
                I.p.reuse_count = (uint32_t) p.get_int("reuse_count", 1);
                (void) p.get_bool("force_eval", true);
                std::ostringstream os;
                os << "MVPathIntegrator[\n  max_depth = " << I.p.max_depth << ",\n  rr_depth = " << I.p.rr_depth
                   << "\n  sa_reuse = " << I.p.sa_reuse << "\n  sa_mis = " << I.p.sa_mis << "\n  fast_mis = "
                   << I.p.fast_mis << "\n  reuse_count = " << I.p.reuse_count << "\n  adaptive = " << I.p.adaptive
                   << "\n  spp_pass_lim = " << I.p.spp_pass_lim << "\n]";
                I.text = os.str();
            } else if (I.type == "path") {
                I.p.integrator = AMVPT_INTEGRATOR_PATH;
                /* the path integrator's pass size travels in spp_pass_lim (amvpt.h) */
                I.p.spp_pass_lim = I.samples_per_pass == 0xffffffffu ? 0u : I.samples_per_pass;
                std::ostringstream os;
                os << "PathIntegrator[\n  max_depth = " << (int) I.p.max_depth << ",\n  rr_depth = " << I.p.rr_depth << "\n]";
                I.text = os.str();
            } else {
                Throw("Integrator \"" + p.plugin + "\" is not implemented (mvpath, path)");
            }
        } else if (o.tag == "sensor") {
            S.sensors.push_back(make_sensor(o));
        } else if (o.tag == "emitter") {
            std::string t = lower(o.props.plugin);
            if (t == "area") Throw("Emitter \"area\" must be attached to a shape");
            if (t == "constant") {
                /* ConstantBackgroundEmitter (constant.cpp:52-65): radiance (default 1), infinite */
                if (S.has_env) Throw("Only one environment emitter can be specified per scene.");
                amvpt_emitter_desc ed;
                std::memset(&ed, 0, sizeof(ed));
                ed.type = AMVPT_EMITTER_CONSTANT;
                ed.shape = -1;
                float rad[3] = {1.f, 1.f, 1.f};
                (void) o.props.get_rgb("radiance", rad);
                std::memcpy(ed.radiance, rad, 12);
                ed.sampling_weight = (float) o.props.get_float("sampling_weight", 1.0);
                S.emitters.push_back(ed);
                S.has_env = true;
            } else if (t == "envmap") {
                Throw("Emitter \"envmap\" is outside the implemented path (constant, area)");
            } else {
                Throw("Emitter \"" + o.props.plugin + "\" must be attached to a shape (area) on the implemented path");
            }
        } else if (o.tag == "shape") {
            const Properties &p = o.props;
            std::string t = lower(p.plugin);
            amvpt_shape_desc d;
            std::memset(&d, 0, sizeof(d));
            d.emitter = -1;
            d.bsdf = -1;
            Transform4f T = p.get_transform("to_world");
            bool flip = p.get_bool("flip_normals", false);
            const Object *bsdf = nullptr, *emit = nullptr;
            (void) p.get_float("silhouette_sampling_weight", 1.0);   /* shape.cpp: only used by differentiable rendering */
            for (auto &c : p.objects(false)) {   /* shape.cpp:26-64 */
                const std::string &ct = c.second->tag;
                if (ct == "bsdf") { if (bsdf) Throw("Only a single BSDF child object can be specified per shape."); bsdf = c.second; }
                else if (ct == "emitter") { if (emit) Throw("Only a single Emitter child object can be specified per shape."); emit = c.second; }
                else if (ct == "sensor" || ct == "medium" || ct == "texture")
                    Throw("Shape: a child " + ct + " is outside the implemented path");
                else continue;
                p.mark_queried(c.first);
            }
            if (t == "rectangle") {
                d.type = AMVPT_SHAPE_RECTANGLE;
                if (flip) T = T * Transform4f::scale({1.f, 1.f, -1.f});
                fill_xform(T, d.to_world, d.to_object);
            } else if (t == "cube") {
                d.type = AMVPT_SHAPE_MESH;
                d.flip_normals = flip;
                auto m = std::make_unique<MeshStore>();
                cube_mesh(T, *m);
                d.vertex_count = 24;
                d.face_count = 12;
                d.positions = m->pos.data();
                /* Mesh::m_face_normals (mesh.cpp): shading with the face normals, vertex normals dropped */
                d.normals = p.get_bool("face_normals", false) ? nullptr : m->nrm.data();
                d.texcoords = m->uv.data();
                d.faces = m->faces.data();
                fill_xform(T, d.to_world, d.to_object);
                S.meshes.push_back(std::move(m));
            } else if (t == "obj" || t == "ply") {
                /* OBJMesh / PLYMesh (obj.cpp:148-406, ply.cpp:150-450) */
                d.type = AMVPT_SHAPE_MESH;
                d.flip_normals = flip;
                std::string fn = p.get_string("filename");
                if (fn.empty()) Throw("\"" + t + "\": property \"filename\" has not been specified");
                if (fn[0] != '/') fn = (S.root->base_dir.empty() ? std::string(".") : S.root->base_dir) + "/" + fn;
                const bool fnorm = p.get_bool("face_normals", false);
                MeshData md = t == "obj" ? load_obj(fn, T, fnorm, p.get_bool("flip_tex_coords", true))
                                         : load_ply(fn, T, fnorm, p.get_bool("flip_tex_coords", false));
                if (md.faces.empty()) Throw("\"" + fn + "\": mesh has no faces");
                auto m = std::make_unique<MeshStore>();
                m->pos = std::move(md.pos);
                m->nrm = std::move(md.nrm);
                m->uv = std::move(md.uv);
                m->faces = std::move(md.faces);
                d.vertex_count = (uint32_t) (m->pos.size() / 3);
                d.face_count = (uint32_t) (m->faces.size() / 3);
                d.positions = m->pos.data();
                d.normals = m->nrm.empty() ? nullptr : m->nrm.data();
                d.texcoords = m->uv.empty() ? nullptr : m->uv.data();
                d.faces = m->faces.data();
                fill_xform(T, d.to_world, d.to_object);
                S.meshes.push_back(std::move(m));
            } else if (t == "sphere") {
                d.type = AMVPT_SHAPE_SPHERE;
                V3f c = p.get_vec3("center", {0, 0, 0});
                float r = (float) p.get_float("radius", 1.0);
                Transform4f W = T * Transform4f::translate(c) * Transform4f::scale({r, r, r});
                V3f rv = W.apply_vector({1.f, 0.f, 0.f});
                d.radius = std::sqrt(dot3(rv, rv));
                V3f ctr = W.apply_point({0.f, 0.f, 0.f});
                d.center[0] = ctr.x; d.center[1] = ctr.y; d.center[2] = ctr.z;
                d.flip_normals = flip;
                fill_xform(W, d.to_world, d.to_object);
            } else {
                Throw("Shape \"" + p.plugin + "\" is not implemented (rectangle, cube, sphere, obj, ply)");
            }
            if (emit) {
                std::string et = lower(emit->props.plugin);
                if (et != "area") Throw("Emitter \"" + emit->props.plugin + "\" cannot be attached to a shape (area only)");
                if (emit->props.has("to_world"))
                    Throw("Found a 'to_world' transformation -- this is not allowed. The area light inherits this "
                          "transformation from its parent shape.");
                amvpt_emitter_desc ed;
                std::memset(&ed, 0, sizeof(ed));
                ed.type = AMVPT_EMITTER_AREA;
                ed.shape = (int32_t) S.shapes.size();
                float rad[3] = {1, 1, 1};
                if (!emit->props.get_rgb("radiance", rad)) Throw("area: property \"radiance\" has not been specified");
                std::memcpy(ed.radiance, rad, 12);
                ed.sampling_weight = (float) emit->props.get_float("sampling_weight", 1.0);
                d.emitter = (int32_t) S.emitters.size();
                S.emitters.push_back(ed);
            }
            if (bsdf) d.bsdf = add_bsdf(S, seen, *bsdf);
            else {
                /* shape.cpp:64-70: default diffuse, black when the shape emits */
                amvpt_bsdf_desc bd;
                std::memset(&bd, 0, sizeof(bd));
                bd.type = AMVPT_BSDF_DIFFUSE;
                bd.nested[0] = bd.nested[1] = -1;
                float v = emit ? 0.f : .5f;
                bd.reflectance[0] = bd.reflectance[1] = bd.reflectance[2] = v;
                d.bsdf = (int) S.bsdfs.size();
                S.bsdfs.push_back(bd);
            }
            S.shapes.push_back(d);
        }
    }
    /* the reference's loader instantiates every child of the scene, so a top-level BSDF no shape uses (or only
     * a removed <ref> did) still has its constructor read its keys: build such BSDFs into a scratch scene (their
     * keys marked read, their errors raised) without adding them to the device tables */
    {
        amvpt_host_scene scratch;
        std::map<const Object *, int> scratch_seen;
        /* ... except a BSDF of a plugin this port does not implement (dielectric, plastic, ...): the scene never
         * renders it, so it loads as the reference's does, its keys unchecked */
        for (auto &e : rp.objects())
            if (e.second->tag == "bsdf" && !seen.count(e.second)) {
                if (bsdf_implemented(*e.second)) (void) add_bsdf(scratch, scratch_seen, *e.second);
                else mark_tree_queried(*e.second);
            }
    }
    if (!have_integrator) {
        /* Scene default: path integrator */
        S.integrator.type = "path";
        std::memset(&S.integrator.p, 0, sizeof(S.integrator.p));
        S.integrator.p.integrator = AMVPT_INTEGRATOR_PATH;
        S.integrator.p.max_depth = 0xffffffffu;
        S.integrator.p.rr_depth = 5;
    }
    /* emitter indices point into shapes[] which moved while building: re-link */
    S.desc.shapes = S.shapes.data();
    S.desc.shape_count = (uint32_t) S.shapes.size();
    S.desc.bsdfs = S.bsdfs.data();
    S.desc.bsdf_count = (uint32_t) S.bsdfs.size();
    S.desc.emitters = S.emitters.data();
    S.desc.emitter_count = (uint32_t) S.emitters.size();
    S.desc.has_environment = S.has_env;
}

/* amvpt_params for one render call (mvpath.cpp:32-41 spp handling happens in amvpt_plan) */
static amvpt_params params_for(const amvpt_host_scene &S, const SensorInfo &sn, uint32_t seed, uint32_t spp) {
    amvpt_params p = S.integrator.p;
    if (p.integrator == AMVPT_INTEGRATOR_MVPATH && !sn.multisensor)
        Throw("This integrator can only be used with MultiSensor !");
    if (p.integrator == AMVPT_INTEGRATOR_PATH && sn.multisensor)
        Throw("The stock `path` integrator on a grid sensor is outside the implemented path");
    p.spp = spp ? spp : sn.sampler.sample_count;
    if (p.integrator == AMVPT_INTEGRATOR_PATH && p.spp_pass_lim) {
        /* SamplingIntegrator::render (integrator.cpp:137-143) */
        const uint32_t spp_per_pass = std::min(p.spp_pass_lim, p.spp);
        if (p.spp % spp_per_pass)
            Throw("sample_count (" + std::to_string(p.spp) + ") must be a multiple of spp_per_pass (" +
                  std::to_string(spp_per_pass) + ").");
    }
    p.seed = seed;
    p.base_seed = sn.sampler.seed;
    p.n_views = (uint32_t) sn.views.size();
    p.multisensor = sn.multisensor;
    p.grid_x = sn.gx;
    p.grid_y = sn.gy;
    p.reverse_x = sn.rev_x;
    p.batch = sn.batch ? 1u : 0u;
    p.reverse_y = sn.rev_y;
    p.film_width = sn.film.cw;    /* the ImageBlock / lane space: the crop (mvpath.cpp:28) */
    p.film_height = sn.film.ch;
    p.crop_offset_x = sn.film.cx;
    p.crop_offset_y = sn.film.cy;
    p.full_width = sn.film.w;
    p.full_height = sn.film.h;
    p.film_alpha = sn.film.alpha;
    p.rfilter = sn.film.rfilter;
    p.rfilter_stddev = sn.film.stddev;
    return p;
}

} // namespace mi

/* ====================================================================== */
/* C API                                                                   */
/* ====================================================================== */

static thread_local std::string g_host_err;
/* shared with exr.cpp */
void amvpt_host_set_error(const std::string &msg) { g_host_err = msg; }

template <class F> static int guarded(F &&f) {
    try {
        return f();
    } catch (const std::exception &e) {
        g_host_err = e.what();
        return -1;
    }
}

/* guarded() for the other translation units of the host library (multi.cpp) */
int amvpt_host_guarded_call(int (*fn)(void *), void *ctx) {
    return guarded([&] { return fn(ctx); });
}

static std::map<std::string, std::string> defines_of(const char *const *k, const char *const *v, int n) {
    std::map<std::string, std::string> d;
    for (int i = 0; i < n; ++i) d[k[i]] = v[i];
    return d;
}

extern "C" {

const char *amvpt_host_last_error(void) { return g_host_err.c_str(); }

static amvpt_host_scene *load_common(std::shared_ptr<mi::Object> root) {
    auto *S = new amvpt_host_scene();
    S->root = root;
    try {
        mi::build(*S);
        mi::check_unqueried(*root);   /* xml.cpp:1089-1107 */
    } catch (...) {
        delete S;
        throw;
    }
    return S;
}

amvpt_host_scene *amvpt_host_load_file(const char *path, const char *const *keys, const char *const *values, int n) {
    amvpt_host_scene *out = nullptr;
    guarded([&] {
        out = load_common(mi::load_scene_file(path, defines_of(keys, values, n)));
        return 0;
    });
    return out;
}

amvpt_host_scene *amvpt_host_load_string(const char *xml, const char *const *keys, const char *const *values, int n) {
    amvpt_host_scene *out = nullptr;
    guarded([&] {
        out = load_common(mi::load_scene_string(xml, defines_of(keys, values, n)));
        return 0;
    });
    return out;
}

void amvpt_host_scene_free(amvpt_host_scene *s) { delete s; }

uint32_t amvpt_host_sensor_count(amvpt_host_scene *s) { return s ? (uint32_t) s->sensors.size() : 0u; }

int amvpt_host_film_info(amvpt_host_scene *s, uint32_t si, uint32_t *w, uint32_t *h, uint32_t *c, uint32_t *spp) {
    return guarded([&] {
        if (!s || si >= s->sensors.size()) throw std::runtime_error("Scene::render(): sensor index out of bounds!");
        const mi::SensorInfo &sn = s->sensors[si];
        if (w) *w = sn.film.cw;   /* develop() returns the crop (hdrfilm.cpp:304-418) */
        if (h) *h = sn.film.ch;
        if (c) *c = sn.film.alpha ? 4u : 3u;
        if (spp) *spp = sn.sampler.sample_count;
        return 0;
    });
}

int amvpt_host_describe(amvpt_host_scene *s, uint32_t si, uint32_t seed, uint32_t spp, const amvpt_scene_desc **sd,
                        const amvpt_view_desc **views, amvpt_params *params) {
    return guarded([&] {
        if (!s || si >= s->sensors.size()) throw std::runtime_error("Scene::render(): sensor index out of bounds!");
        const mi::SensorInfo &sn = s->sensors[si];
        amvpt_params p = mi::params_for(*s, sn, seed, spp);
        if (sd) *sd = &s->desc;
        if (views) *views = sn.views.data();
        if (params) *params = p;
        return 0;
    });
}

const char *amvpt_host_integrator_string(amvpt_host_scene *s) { return s ? s->integrator.text.c_str() : ""; }

/* a device buffer of at least `bytes`, grown (never shrunk) across frames */
static void ensure_buffer(float *&buf, size_t &have, size_t bytes, uint64_t &allocs) {
    if (have >= bytes) return;
    if (buf) (void) hipFree(buf);
    buf = nullptr;
    have = 0;
    if (hipMalloc(&buf, bytes) != hipSuccess) throw std::runtime_error("hipMalloc of the film failed");
    have = bytes;
    ++allocs;
}

int amvpt_host_render_stream(amvpt_host_scene *s, uint32_t si, uint32_t seed, uint32_t spp, int raw, float *out,
                             void *stream, amvpt_counters *counters) {
    return guarded([&] {
        if (!s || si >= s->sensors.size()) throw std::runtime_error("Scene::render(): sensor index out of bounds!");
        const mi::SensorInfo &sn = s->sensors[si];
        amvpt_params p = mi::params_for(*s, sn, seed, spp);
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
        std::lock_guard<std::mutex> lock(s->render_mu);
        amvpt_host_scene::DeviceCache *dc = nullptr;
        for (auto &d : s->devices)
            if (d.device == dev) dc = &d;
        if (!dc) {
            s->devices.emplace_back();
            dc = &s->devices.back();
            dc->device = dev;
        }
        if (!dc->scene) {
            if (amvpt_scene_create(&s->desc, &dc->scene) != AMVPT_OK) throw std::runtime_error(amvpt_last_error());
            ++s->scene_creates;
        }
        const hipStream_t st = (hipStream_t) stream;
        const uint32_t C = amvpt_film_channels(&p);
        const size_t npx = (size_t) p.film_width * p.film_height;
        ensure_buffer(dc->film, dc->film_bytes, npx * C * sizeof(float), s->buffer_allocs);
        if (hipMemsetAsync(dc->film, 0, npx * C * sizeof(float), st) != hipSuccess)
            throw std::runtime_error("hipMemsetAsync(film) failed");
        /* the whole frame with explicit per-call options: no process-global knob takes part */
        amvpt_lane_set lanes{};
        lanes.lane_begin = 0;
        lanes.lane_end = UINT64_MAX;
        amvpt_film_window win{};
        win.film = dc->film;
        win.width = p.film_width;
        win.height = p.film_height;
        amvpt_render_opts opts{};
        if (amvpt_render_ex(dc->scene, sn.views.data(), &p, &lanes, &win, stream, &opts, counters) != AMVPT_OK)
            throw std::runtime_error(amvpt_last_error());
        ++s->renders;
        const float *src = dc->film;
        size_t bytes = npx * C * sizeof(float);
        if (!raw) {
            const uint32_t T = p.film_alpha ? 4u : 3u;
            bytes = npx * T * sizeof(float);
            ensure_buffer(dc->image, dc->image_bytes, bytes, s->buffer_allocs);
            if (amvpt_develop(dc->film, dc->image, p.film_width, p.film_height, p.film_alpha, stream) != AMVPT_OK)
                throw std::runtime_error(amvpt_last_error());
            src = dc->image;
        }
        if (hipMemcpyAsync(out, src, bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            throw std::runtime_error("copying the image to the host failed");
        return 0;
    });
}

int amvpt_host_render(amvpt_host_scene *s, uint32_t si, uint32_t seed, uint32_t spp, int raw, float *out,
                      amvpt_counters *counters) {
    return amvpt_host_render_stream(s, si, seed, spp, raw, out, nullptr, counters);
}

int amvpt_host_render_stats(amvpt_host_scene *s, uint64_t *scene_creates, uint64_t *buffer_allocs, uint64_t *renders) {
    return guarded([&] {
        if (!s) throw std::runtime_error("amvpt_host_render_stats: null scene");
        std::lock_guard<std::mutex> lock(s->render_mu);
        if (scene_creates) *scene_creates = s->scene_creates;
        if (buffer_allocs) *buffer_allocs = s->buffer_allocs;
        if (renders) *renders = s->renders;
        return 0;
    });
}

double amvpt_host_parse_fov(double fov, const char *fov_axis, const char *focal_length, double aspect) {
    double r = -1.0;
    guarded([&] {
        mi::Properties p;
        if (fov > 0) p.set_float("fov", fov);
        if (fov_axis) p.set_string("fov_axis", fov_axis);
        if (focal_length) p.set_string("focal_length", focal_length);
        r = mi::parse_fov(p, aspect);
        return 0;
    });
    return r;
}

void amvpt_host_perspective_projection(const int *film_size, const int *crop_size, const int *crop_offset, float fov_x,
                                       float near_clip, float far_clip, float *m16) {
    mi::Transform4f t = mi::perspective_projection(film_size, crop_size, crop_offset, fov_x, near_clip, far_clip);
    t.matrix.store(m16);
}

} // extern "C"
