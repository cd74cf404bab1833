/*
 * amvpt_oracle.cpp -- TEST INFRASTRUCTURE ONLY: the parity oracle.
 *
 * A scalar, per-lane CPU restatement of the reference's `mvpath` hot path
 * (xacond00/mitsuba3-amvpt, Mitsuba 3.6.4 fork) under the semantics of its
 * JIT (llvm_rgb) variant: every `if (dr::any_or<true>(..))` is taken, every
 * `if (dr::none_or<false>(..)) return/continue` is not, masked virtual calls
 * return zeros on masked lanes, and RNG draws happen unconditionally outside
 * loops (per active iteration inside `dr::while_loop`).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  It is never part of the product path.
 *
 * It consumes the same plain descriptors as the product C-ABI (include/amvpt.h)
 * and has no code in common with the HIP implementation.
 *
 * Reference functions restated (file:line):
 *   render (pass split, lane->pixel, group size)   src/integrators/mvpath.cpp:7-278
 *   render_multisample / sample_multi / camera_selection / mis_weights /
 *   sample_suffix                                  src/integrators/mvpath_multi.h:8-689
 *   render_sample / sample_single                  src/integrators/mvpath_single.h:50-278
 *   tv_pdf / tv_pdf_fast / mis_weight / sensors_visible  mvpath.h:243-311
 *   GridSensor::sample_ray_idx                     src/sensors/grid.cpp:269-297
 *   BatchSensor::sample_ray_idx                    src/sensors/batch.cpp:163-181
 *   ThinLensCamera::sample_ray / sample_surface    src/sensors/thinlens.cpp:220-257,358-418
 *   PerspectiveCamera::sample_ray / sample_surface src/sensors/perspective.cpp:205-241,327-385
 *   PCG32Sampler::seed / IndependentSampler        src/render/sampler.cpp:125-144, independent.cpp:77-97
 *   sample_tea_32                                  include/mitsuba/core/random.h:77-90
 *   ImageBlock::put (coalesced / non-coalesced)    src/render/imageblock.cpp:174-559
 *   GaussianFilter::eval                           src/rfilters/gaussian.cpp:48-100
 *   Scene::sample_emitter_direction / pdf          src/render/scene.cpp:223-361
 *   AreaLight::eval / sample_direction / pdf       src/emitters/area.cpp:82-190
 *   Shape::sample_direction / pdf_direction        src/render/shape.cpp:360-390
 *   Rectangle (intersect, SI, sample_position)     src/shapes/rectangle.cpp:112-178,447-563
 *   Mesh SI, Moeller-Trumbore, face_normal         src/render/mesh.cpp:1393-1560, mesh.h:156-164,467-488
 *   Sphere (intersect, SI, sampling)               src/shapes/sphere.cpp:200-330,520-620
 *   Interaction spawn_ray / spawn_ray_to / offset_p include/mitsuba/render/interaction.h:140-169
 *   initialize_sh_frame / finalize                 interaction.h:278-288,497-517
 *   SmoothDiffuse                                  src/bsdfs/diffuse.cpp:100-188
 *   RoughConductor + MicrofacetDistribution        src/bsdfs/roughconductor.cpp:225-523,
 *                                                  include/mitsuba/render/microfacet.h:185-431
 *   fresnel_conductor / reflect                    include/mitsuba/render/fresnel.h:93-116,276-284
 *   TwoSidedBRDF                                   src/bsdfs/twosided.cpp:112-296
 *   warps (concentric disk, cosine hemisphere, cone, sphere)  include/mitsuba/core/warp.h
 */
#include "oracle_math.h"
#include "../include/amvpt.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>
#include <functional>
#include <array>

using namespace orc;

namespace {

/* BSDFFlags (include/mitsuba/render/bsdf.h:37-86) */
enum : uint32_t {
    F_Null = 0x1, F_DiffuseReflection = 0x2, F_DiffuseTransmission = 0x4,
    F_GlossyReflection = 0x8, F_GlossyTransmission = 0x10,
    F_DeltaReflection = 0x20, F_DeltaTransmission = 0x40,
    F_Anisotropic = 0x1000, F_FrontSide = 0x8000, F_BackSide = 0x10000,
    F_Diffuse = F_DiffuseReflection | F_DiffuseTransmission,
    F_Glossy = F_GlossyReflection | F_GlossyTransmission,
    F_Smooth = F_Diffuse | F_Glossy,
    F_Delta = F_DeltaReflection | F_DeltaTransmission,
};
static const uint32_t CTX_ALL = 0xffffffffu;      /* BSDFContext() */
static const uint32_t CTX_GLOSSY = F_Glossy;      /* BSDFContext(Radiance, Glossy) */
static inline bool ctx_enabled(uint32_t mask, uint32_t type) {
    return mask == 0xffffffffu || (mask & type) == type;
}

struct Spec { float r, g, b; };
static inline Spec sp(float v) { return {v, v, v}; }
static inline Spec operator*(Spec a, Spec b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
static inline Spec operator*(Spec a, float s) { return {a.r * s, a.g * s, a.b * s}; }
static inline Spec operator*(float s, Spec a) { return {s * a.r, s * a.g, s * a.b}; }
static inline Spec operator+(Spec a, Spec b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }
static inline Spec operator/(Spec a, float s) { return {a.r / s, a.g / s, a.b / s}; }
static inline Spec spec_fma(Spec a, Spec b, Spec c) { return {fmadd(a.r, b.r, c.r), fmadd(a.g, b.g, c.g), fmadd(a.b, b.b, c.b)}; }
static inline Spec sel(bool m, Spec a, Spec b) { return m ? a : b; }
static inline float smax(Spec a) { return fmaxf_(fmaxf_(a.r, a.g), a.b); }

struct Ray { V3 o, d; float maxt; };
static inline V3 ray_at(const Ray &r, float t) { return fmadd(r.d, t, r.o); }

struct SI {
    float t = Infinity;
    V3 p{0, 0, 0}, n{0, 0, 0};
    V2 uv{0, 0};
    Frame sh{{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    V3 dp_du{0, 0, 0}, dp_dv{0, 0, 0};
    V3 wi{0, 0, 0};
    int shape = -1;
    bool valid() const { return t != Infinity; }
    V3 to_local(V3 v) const { return sh.to_local(v); }
    V3 to_world(V3 v) const { return sh.to_world(v); }
};

/* Interaction::offset_p / spawn_ray / spawn_ray_to (interaction.h:140-169) */
static inline V3 offset_p(V3 p, V3 n, V3 d) {
    float mag = (1.f + hmax(v3(std::fabs(p.x), std::fabs(p.y), std::fabs(p.z)))) * RayEpsilon;
    mag = mulsign(mag, dot(n, d));
    return fmadd(n, mag, p);
}
static inline Ray spawn_ray(V3 p, V3 n, V3 d) { return Ray{offset_p(p, n, d), d, Largest}; }
static inline Ray spawn_ray_to(V3 p, V3 n, V3 t) {
    V3 o = offset_p(p, n, t - p);
    V3 d = t - o;
    float dist = norm(d);
    d = d / dist;
    return Ray{o, d, dist * (1.f - ShadowEpsilon)};
}

/* warps (warp.h) */
static inline V2 square_to_uniform_disk_concentric(V2 s) {
    float x = fmsub(2.f, s.x, 1.f), y = fmsub(2.f, s.y, 1.f);
    bool is_zero = x == 0.f && y == 0.f, q13 = std::fabs(x) < std::fabs(y);
    float r = q13 ? y : x, rp = q13 ? x : y;
    float phi = (0.25f * Pi) * rp / r;
    if (q13) phi = (0.5f * Pi) - phi;
    if (is_zero) phi = 0.f;
    float sn, cs;
    sincos_(phi, sn, cs);
    return {r * cs, r * sn};
}
static inline V3 square_to_cosine_hemisphere(V2 s) {
    V2 p = square_to_uniform_disk_concentric(s);
    float z = safe_sqrt(1.f - fmadd(p.y, p.y, p.x * p.x));
    return {p.x, p.y, z};
}
static inline float cosine_hemisphere_pdf(V3 v) { return InvPi * v.z; }
/* warp::square_to_uniform_sphere (warp.h:249-255): z = 1 - 2 y, r = circ(z), phi = 2 pi x */
static inline V3 square_to_uniform_sphere(V2 s) {
    float z = fmadd(-2.f, s.y, 1.f);
    float r = safe_sqrt(fmadd(-z, z, 1.f));
    float sn, cs;
    sincos_(s.x * (2.f * Pi), sn, cs);
    return {r * cs, r * sn, z};
}
static inline float uniform_cone_pdf(float cos_cutoff) { return InvTwoPi / (1.f - cos_cutoff); }

/* --------------------------------------------------------------------- */
/* Scene                                                                 */
/* --------------------------------------------------------------------- */

struct Prim { uint32_t type, shape, face; };

struct Shape {
    uint32_t type;
    int bsdf, emitter;
    bool flip;
    float to_world[16], to_object[16];
    Frame frame;         /* rectangle m_frame */
    float inv_area;
    std::vector<float> pos, nrm, uv;
    std::vector<uint32_t> faces;
    float center[3];
    float radius;
    /* Mesh::m_area_pmf (mesh.cpp:444-485): face areas and their inclusive float prefix sums */
    std::vector<float> area_pmf, area_cdf;
    float area_sum = 0.f;
};

struct Scene {
    std::vector<Shape> shapes;
    std::vector<amvpt_bsdf_desc> bsdfs;
    std::vector<amvpt_emitter_desc> emitters;
    std::vector<Prim> prims;
    float emitter_pmf = 0.f;
    /* non-uniform sampling weights: DiscreteDistribution (distr_1d.h:218-231, JIT compute_cdf) */
    bool distr = false;
    std::vector<float> cdf;       /* inclusive prefix sums of the weights (float) */
    float distr_sum = 0.f, distr_norm = 0.f;
    int environment = -1;         /* the constant emitter (Scene::m_environment), or -1 */
    V3 bs_center{0, 0, 0};        /* ConstantBackgroundEmitter::m_bsphere after set_scene */
    float bs_radius = 0.f;
    /* optional acceleration (oracle_set_bvh, the CPU-baseline timing only; the parity tests keep the brute-force
     * scans): a binary median-split BVH over padded primitive boxes, leaves of <= 4 primitive indices */
    struct BNode { double lo[3], hi[3]; uint32_t first, count, right, axis; };
    std::vector<BNode> bvh;
    std::vector<uint32_t> bvh_idx;
};

/* PreliminaryIntersection */
struct PI { float t = Infinity; float u = 0, v = 0; int prim = -1; };

static inline bool rect_hit(const Shape &s, const Ray &ray_w, float &t, float &lx, float &ly) {
    V3 o = xform_point_affine(s.to_object, ray_w.o);
    V3 d = xform_vector(s.to_object, ray_w.d);
    t = -o.z / d.z;
    V3 local = fmadd(d, t, o);
    lx = local.x; ly = local.y;
    return t >= 0.f && t <= ray_w.maxt && std::fabs(local.x) <= 1.f && std::fabs(local.y) <= 1.f;
}

static inline V3 vtx(const Shape &s, uint32_t i) { return {s.pos[3 * i], s.pos[3 * i + 1], s.pos[3 * i + 2]}; }

static inline bool tri_hit(const Shape &s, uint32_t f, const Ray &ray, float &t, float &u, float &v) {
    V3 p0 = vtx(s, s.faces[3 * f]), p1 = vtx(s, s.faces[3 * f + 1]), p2 = vtx(s, s.faces[3 * f + 2]);
    V3 e1 = p1 - p0, e2 = p2 - p0;
    V3 pvec = cross(ray.d, e2);
    float inv_det = rcp(dot(e1, pvec));
    V3 tvec = ray.o - p0;
    u = dot(tvec, pvec) * inv_det;
    bool active = u >= 0.f && u <= 1.f;
    V3 qvec = cross(tvec, e1);
    v = dot(ray.d, qvec) * inv_det;
    active = active && v >= 0.f && u + v <= 1.f;
    t = dot(e2, qvec) * inv_det;
    return active && t >= 0.f && t <= ray.maxt;
}

/* sphere.cpp ray_intersect_preliminary_impl (float64 on llvm variants) */
static inline bool sphere_hit(const Shape &s, const Ray &ray, float &t_out) {
    double cx = s.center[0], cy = s.center[1], cz = s.center[2], r = s.radius;
    double ox = ray.o.x, oy = ray.o.y, oz = ray.o.z, dx = ray.d.x, dy = ray.d.y, dz = ray.d.z;
    double maxt = ray.maxt;
    double lx = ox - cx, ly = oy - cy, lz = oz - cz;
    double dn = std::sqrt(std::fma(dz, dz, std::fma(dy, dy, dx * dx)));
    double plane_t = std::fma(-lz, dz, std::fma(-ly, dy, -lx * dx)) / dn;
    bool no_hit = plane_t == 0.0 && (ray.o.x != s.center[0] && ray.o.y != s.center[1] && ray.o.z != s.center[2]);
    /* plane_p = ray(FloatP(plane_t)) in float, then widened */
    float pt_f = (float) plane_t;
    V3 pp = ray_at(ray, pt_f);
    double ppx = (double) pp.x - cx, ppy = (double) pp.y - cy, ppz = (double) pp.z - cz;
    no_hit = no_hit && (std::sqrt(std::fma(ppz, ppz, std::fma(ppy, ppy, ppx * ppx))) > r);
    double A = std::fma(dz, dz, std::fma(dy, dy, dx * dx));
    double B = 2.0 * std::fma(ppz, dz, std::fma(ppy, dy, ppx * dx));
    double C = std::fma(ppz, ppz, std::fma(ppy, ppy, ppx * ppx)) - r * r;
    /* math::solve_quadratic (math.h:360-400) */
    bool linear = A == 0.0, valid_linear = linear && B != 0.0;
    double x0 = -C / B, x1 = x0;
    double discrim = std::fma(B, B, -(4.0 * A * C));
    bool valid_quad = !linear && discrim >= 0.0;
    {
        double sq = std::sqrt(discrim);
        double temp = -0.5 * (B + std::copysign(sq, B));
        double x0p = temp / A, x1p = C / temp;
        double x0m = std::min(x0p, x1p), x1m = std::max(x0p, x1p);
        x0 = linear ? x0 : x0m;
        x1 = linear ? x0 : x1m;
    }
    bool found = valid_linear || valid_quad;
    double near_t = x0 + plane_t, far_t = x1 + plane_t;
    bool out_bounds = !(near_t <= maxt && far_t >= 0.0);
    bool in_bounds = near_t < 0.0 && far_t > maxt;
    bool active = found && !no_hit && !out_bounds && !in_bounds;
    t_out = active ? (near_t < 0.0 ? (float) far_t : (float) near_t) : Infinity;
    return active;
}

static inline bool prim_hit_any_type(const Scene &sc, size_t i, const Ray &ray, float &t, float &u, float &v) {
    const Prim &pr = sc.prims[i];
    const Shape &s = sc.shapes[pr.shape];
    u = v = 0.f;
    if (pr.type == AMVPT_SHAPE_RECTANGLE) return rect_hit(s, ray, t, u, v);
    if (pr.type == AMVPT_SHAPE_MESH) return tri_hit(s, pr.face, ray, t, u, v);
    return sphere_hit(s, ray, t);
}
/* slab test of a padded box in double (conservative for every hit the float tests report) */
static inline bool bvh_box_hit(const Scene::BNode &n, const Ray &ray, float tmax) {
    double t0 = 0.0, t1 = (double) tmax;
    const double o[3] = {ray.o.x, ray.o.y, ray.o.z}, d[3] = {ray.d.x, ray.d.y, ray.d.z};
    for (int a = 0; a < 3; ++a) {
        if (d[a] == 0.0) {
            if (o[a] < n.lo[a] || o[a] > n.hi[a]) return false;
            continue;
        }
        const double inv = 1.0 / d[a];
        double ta = (n.lo[a] - o[a]) * inv, tb = (n.hi[a] - o[a]) * inv;
        if (ta > tb) std::swap(ta, tb);
        t0 = std::max(t0, ta);
        t1 = std::min(t1, tb);
        if (t0 > t1) return false;
    }
    return true;
}
/* the BVH walk: every primitive whose box the ray crosses, closest by the (t, index) rule (= the brute-force scan's
 * lowest-index-first tie break), or any hit */
template <bool kAny> static PI bvh_walk(const Scene &sc, const Ray &ray) {
    PI best;
    uint32_t stack[128], sp = 0;
    stack[sp++] = 0;
    while (sp) {
        const Scene::BNode &n = sc.bvh[stack[--sp]];
        /* closest hit: boxes beyond the best hit so far are skipped (inclusive: a tie may still win on the index) */
        if (!bvh_box_hit(n, ray, kAny ? ray.maxt : std::min(ray.maxt, best.t))) continue;
        if (n.count) {
            for (uint32_t k = 0; k < n.count; ++k) {
                const uint32_t i = sc.bvh_idx[n.first + k];
                float t, u, v;
                if (prim_hit_any_type(sc, i, ray, t, u, v) && (t < best.t || (t == best.t && (int) i < best.prim))) {
                    best.t = t; best.u = u; best.v = v; best.prim = (int) i;
                    if (kAny) return best;
                }
            }
        } else if (sp + 2 <= 128) {
            /* the child on the ray's side of the split first (popped first) */
            const uint32_t left = (uint32_t) (&n - sc.bvh.data()) + 1u;
            const float da = n.axis == 0 ? ray.d.x : n.axis == 1 ? ray.d.y : ray.d.z;
            stack[sp++] = da < 0.f ? left : n.right;
            stack[sp++] = da < 0.f ? n.right : left;
        } else {
            /* (never at these depths) the rest by brute force */
            for (size_t i = 0; i < sc.prims.size(); ++i) {
                float t, u, v;
                if (prim_hit_any_type(sc, i, ray, t, u, v) && (t < best.t || (t == best.t && (int) i < best.prim))) {
                    best.t = t; best.u = u; best.v = v; best.prim = (int) i;
                }
            }
            return best;
        }
    }
    return best;
}
static void build_bvh(Scene &sc) {
    const size_t n = sc.prims.size();
    std::vector<std::array<double, 6>> box(n);
    std::vector<std::array<double, 3>> cen(n);
    for (size_t i = 0; i < n; ++i) {
        const Prim &pr = sc.prims[i];
        const Shape &s = sc.shapes[pr.shape];
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        auto grow = [&](V3 p) {
            const double q[3] = {p.x, p.y, p.z};
            for (int a = 0; a < 3; ++a) { lo[a] = std::min(lo[a], q[a]); hi[a] = std::max(hi[a], q[a]); }
        };
        if (pr.type == AMVPT_SHAPE_RECTANGLE) {
            for (int c = 0; c < 4; ++c) grow(xform_point_affine(s.to_world, v3((c & 1) ? 1.f : -1.f, (c & 2) ? 1.f : -1.f, 0.f)));
        } else if (pr.type == AMVPT_SHAPE_MESH) {
            for (int k = 0; k < 3; ++k) grow(vtx(s, s.faces[3 * pr.face + k]));
        } else {
            grow(v3(s.center[0] - s.radius, s.center[1] - s.radius, s.center[2] - s.radius));
            grow(v3(s.center[0] + s.radius, s.center[1] + s.radius, s.center[2] + s.radius));
        }
        double m = 0.0;
        for (int a = 0; a < 3; ++a) m = std::max(m, std::max(std::fabs(lo[a]), std::fabs(hi[a])));
        const double e = 1e-4 * (1.0 + m);
        for (int a = 0; a < 3; ++a) {
            box[i][a] = lo[a] - e; box[i][3 + a] = hi[a] + e;
            cen[i][a] = .5 * (lo[a] + hi[a]);
        }
    }
    sc.bvh_idx.resize(n);
    for (size_t i = 0; i < n; ++i) sc.bvh_idx[i] = (uint32_t) i;
    sc.bvh.clear();
    std::function<uint32_t(uint32_t, uint32_t)> build = [&](uint32_t b, uint32_t e) -> uint32_t {
        const uint32_t at = (uint32_t) sc.bvh.size();
        sc.bvh.push_back({});
        Scene::BNode nd{};
        double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int a = 0; a < 3; ++a) { nd.lo[a] = INFINITY; nd.hi[a] = -INFINITY; }
        for (uint32_t k = b; k < e; ++k) {
            const uint32_t i = sc.bvh_idx[k];
            for (int a = 0; a < 3; ++a) {
                nd.lo[a] = std::min(nd.lo[a], box[i][a]); nd.hi[a] = std::max(nd.hi[a], box[i][3 + a]);
                clo[a] = std::min(clo[a], cen[i][a]); chi[a] = std::max(chi[a], cen[i][a]);
            }
        }
        if (e - b <= 4) {
            nd.first = b; nd.count = e - b;
        } else {
            int ax = 0;
            for (int a = 1; a < 3; ++a) if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
            const uint32_t mid = (b + e) / 2;
            std::nth_element(sc.bvh_idx.begin() + b, sc.bvh_idx.begin() + mid, sc.bvh_idx.begin() + e,
                             [&](uint32_t x, uint32_t y) { return cen[x][ax] < cen[y][ax]; });
            build(b, mid);                  /* left child: at + 1 */
            nd.right = build(mid, e);
            nd.count = 0;
            nd.axis = (uint32_t) ax;
        }
        sc.bvh[at] = nd;
        return at;
    };
    if (n) build(0, (uint32_t) n);
}
static bool g_use_bvh = false;   /* oracle_set_bvh */

/* closest hit: minimum (t, prim index) over all primitives (brute force; or the BVH walk, oracle_set_bvh). */
static PI intersect_pi(const Scene &sc, const Ray &ray) {
    if (!sc.bvh.empty()) return bvh_walk<false>(sc, ray);
    PI best;
    for (size_t i = 0; i < sc.prims.size(); ++i) {
        const Prim &pr = sc.prims[i];
        const Shape &s = sc.shapes[pr.shape];
        float t, u = 0, v = 0;
        bool hit;
        if (pr.type == AMVPT_SHAPE_RECTANGLE) hit = rect_hit(s, ray, t, u, v);
        else if (pr.type == AMVPT_SHAPE_MESH) hit = tri_hit(s, pr.face, ray, t, u, v);
        else hit = sphere_hit(s, ray, t);
        if (hit && t < best.t) { best.t = t; best.u = u; best.v = v; best.prim = (int) i; }
    }
    return best;
}

static bool ray_test(const Scene &sc, const Ray &ray) {
    if (!sc.bvh.empty()) return bvh_walk<true>(sc, ray).prim >= 0;
    for (size_t i = 0; i < sc.prims.size(); ++i) {
        const Prim &pr = sc.prims[i];
        const Shape &s = sc.shapes[pr.shape];
        float t, u, v;
        bool hit;
        if (pr.type == AMVPT_SHAPE_RECTANGLE) hit = rect_hit(s, ray, t, u, v);
        else if (pr.type == AMVPT_SHAPE_MESH) hit = tri_hit(s, pr.face, ray, t, u, v);
        else hit = sphere_hit(s, ray, t);
        if (hit) return true;
    }
    return false;
}

/* Shape::compute_surface_interaction + finalize_surface_interaction */
static SI compute_si(const Scene &sc, const Ray &ray, const PI &pi) {
    SI si;
    if (pi.prim < 0) {
        si.t = Infinity;
        si.wi = -ray.d;
        return si;
    }
    const Prim &pr = sc.prims[pi.prim];
    const Shape &s = sc.shapes[pr.shape];
    si.shape = (int) pr.shape;
    si.t = pi.t;
    if (pr.type == AMVPT_SHAPE_RECTANGLE) {
        V3 p = ray_at(ray, pi.t);
        V3 tr = v3(s.to_world[3], s.to_world[7], s.to_world[11]);
        float dist = dot(tr - p, s.frame.n);
        si.p = p + dist * s.frame.n;
        si.n = s.frame.n;
        si.sh.n = s.frame.n;
        si.dp_du = s.frame.s;
        si.dp_dv = s.frame.t;
        si.uv = {fmadd(pi.u, 0.5f, 0.5f), fmadd(pi.v, 0.5f, 0.5f)};
    } else if (pr.type == AMVPT_SHAPE_MESH) {
        uint32_t i0 = s.faces[3 * pr.face], i1 = s.faces[3 * pr.face + 1], i2 = s.faces[3 * pr.face + 2];
        V3 p0 = vtx(s, i0), p1 = vtx(s, i1), p2 = vtx(s, i2);
        float b1 = pi.u, b2 = pi.v, b0 = 1.f - b1 - b2;
        si.p = fmadd(p0, b0, fmadd(p1, b1, p2 * b2));
        si.n = normalize(cross(p1 - p0, p2 - p0));
        si.uv = {b1, b2};
        coordinate_system(si.n, si.dp_du, si.dp_dv);
        V3 dp0 = p1 - p0, dp1 = p2 - p0;
        if (!s.uv.empty()) {
            V2 uv0{s.uv[2 * i0], s.uv[2 * i0 + 1]}, uv1{s.uv[2 * i1], s.uv[2 * i1 + 1]}, uv2{s.uv[2 * i2], s.uv[2 * i2 + 1]};
            si.uv = {fmadd(uv2.x, b2, fmadd(uv1.x, b1, uv0.x * b0)), fmadd(uv2.y, b2, fmadd(uv1.y, b1, uv0.y * b0))};
            V2 duv0{uv1.x - uv0.x, uv1.y - uv0.y}, duv1{uv2.x - uv0.x, uv2.y - uv0.y};
            float det = fmsub(duv0.x, duv1.y, duv0.y * duv1.x), inv_det = rcp(det);
            if (det != 0.f) {
                for (int c = 0; c < 3; ++c) {
                    si.dp_du[c] = fmsub(duv1.y, dp0[c], duv0.y * dp1[c]) * inv_det;
                    si.dp_dv[c] = fnmadd(duv1.x, dp0[c], duv0.x * dp1[c]) * inv_det;
                }
            }
        }
        if (!s.nrm.empty()) {
            V3 n0{s.nrm[3 * i0], s.nrm[3 * i0 + 1], s.nrm[3 * i0 + 2]};
            V3 n1{s.nrm[3 * i1], s.nrm[3 * i1 + 1], s.nrm[3 * i1 + 2]};
            V3 n2{s.nrm[3 * i2], s.nrm[3 * i2 + 1], s.nrm[3 * i2 + 2]};
            V3 n = fmadd(n2, b2, fmadd(n1, b1, n0 * b0));
            float il = rsqrt(squared_norm(n));
            si.sh.n = n * il;
        } else {
            si.sh.n = si.n;
        }
        if (s.flip) { si.n = -si.n; si.sh.n = -si.sh.n; }
    } else { /* sphere.cpp:607-718 compute_surface_interaction (non-diff branch) */
        V3 c{s.center[0], s.center[1], s.center[2]};
        si.sh.n = normalize(ray_at(ray, pi.t) - c);
        si.p = fmadd(si.sh.n, s.radius, c);
        V3 local = xform_point_affine(s.to_object, si.p);
        float rd_2 = sqr(local.x) + sqr(local.y);
        /* si.uv (atan2 / unit_angle_z) only feeds textures: none on the implemented path */
        si.uv = {0.f, 0.f};
        si.dp_du = v3(-local.y, local.x, 0.f);
        float rd = std::sqrt(rd_2), inv_rd = rcp(rd), cos_phi = local.x * inv_rd, sin_phi = local.y * inv_rd;
        si.dp_dv = v3(local.z * cos_phi, local.z * sin_phi, -rd);
        if (rd == 0.f) si.dp_dv = v3(1.f, 0.f, 0.f);
        si.dp_du = xform_vector(s.to_world, si.dp_du) * (2.f * Pi);
        si.dp_dv = xform_vector(s.to_world, si.dp_dv) * Pi;
        if (s.flip) si.sh.n = -si.sh.n;
        si.n = si.sh.n;
    }
    /* finalize_surface_interaction: initialize_sh_frame (interaction.h:278-288) */
    si.sh.s = normalize(fmadd(si.sh.n, -dot(si.sh.n, si.dp_du), si.dp_du));
    if (si.dp_du.x == 0.f && si.dp_du.y == 0.f && si.dp_du.z == 0.f) {
        V3 s0, t0;
        coordinate_system(si.sh.n, s0, t0);
        si.sh.s = s0;
    }
    si.sh.t = cross(si.sh.n, si.sh.s);
    si.wi = si.to_local(-ray.d);
    return si;
}

static SI intersect(const Scene &sc, const Ray &ray) { return compute_si(sc, ray, intersect_pi(sc, ray)); }

/* --------------------------------------------------------------------- */
/* Emitters / shape sampling                                             */
/* --------------------------------------------------------------------- */

struct DS {            /* DirectionSample3f */
    V3 p{0, 0, 0}, n{0, 0, 0};
    V2 uv{0, 0};
    float pdf = 0.f;
    bool delta = false;
    V3 d{0, 0, 0};
    float dist = 0.f;
    int emitter = -1;
};

/* SurfaceInteraction::emitter (interaction.h): the shape's area emitter, or the scene's
 * environment emitter for a ray that left the scene */
static int si_emitter(const Scene &sc, const SI &si) {
    if (!si.valid()) return sc.environment;
    return sc.shapes[si.shape].emitter;
}

/* AreaLight::eval (area.cpp:82-88), ConstantBackgroundEmitter::eval (constant.cpp:90-94);
 * masked vcall -> 0 when !active */
static Spec emitter_eval(const Scene &sc, int e, const SI &si, bool active) {
    if (e < 0 || !active) return sp(0.f);
    const amvpt_emitter_desc &ed = sc.emitters[e];
    if (ed.type != AMVPT_EMITTER_CONSTANT && !(si.wi.z > 0.f)) return sp(0.f);
    return {ed.radiance[0], ed.radiance[1], ed.radiance[2]};
}

/* Scene::pdf_emitter (scene.cpp:245-250): the probability of picking emitter `i` */
static float emitter_pick_pmf(const Scene &sc, uint32_t i) {
    return sc.distr ? sc.emitters[i].sampling_weight * sc.distr_norm : sc.emitter_pmf;
}

/* DiscreteDistribution::sample (distr_1d.h:116-134, JIT predicate) with dr::binary_search over
 * [0, n - 1]: iterations = floor(log2(n - 1)) + 1, middle = (start + end) >> 1, a true predicate
 * moves start to min(middle + 1, end), a false one moves end to middle */
static uint32_t distr_sample(const Scene &sc, float value) {
    const uint32_t n = (uint32_t) sc.cdf.size();
    const float sample = value * sc.distr_sum;
    uint32_t start = 0, end = n - 1, it = 0;
    if (end > 0) { uint32_t x = end; while (x) { ++it; x >>= 1; } }
    for (uint32_t i = 0; i < it; ++i) {
        const uint32_t middle = (start + end) >> 1;
        const float c = sc.cdf[middle];
        const bool cond = ((c < sample) || c == 0.f) && c != sc.distr_sum;
        if (cond) start = std::min(middle + 1u, end);
        else end = middle;
    }
    return start;
}

/* Scene::sample_emitter (scene.cpp:222-244): (index, weight, re-used sample) */
static uint32_t sample_emitter(const Scene &sc, float &u, float &weight) {
    const size_t n = sc.emitters.size();
    weight = 1.f;
    if (n < 2) return 0;
    if (sc.distr) {
        /* sample_reuse_pmf (distr_1d.h:201-215) */
        const uint32_t index = distr_sample(sc, u);
        const float pmf = sc.emitters[index].sampling_weight * sc.distr_norm;
        const float cdf = index > 0 ? sc.cdf[index - 1] * sc.distr_norm : 0.f;
        u = (u - cdf) / pmf;
        weight = rcp(pmf);
        return index;
    }
    float scaled = u * (float) n;
    uint32_t index = std::min((uint32_t) scaled, (uint32_t) n - 1u);
    weight = (float) n;
    u = scaled - (float) index;
    return index;
}

/* Shape::sample_direction (shape.cpp:360-377) / Sphere::sample_direction (sphere.cpp:234-309) */
static DS shape_sample_direction(const Shape &s, V3 itp, V2 sample) {
    DS ds;
    if (s.type == AMVPT_SHAPE_RECTANGLE) {
        ds.p = xform_point_affine(s.to_world, v3(sample.x * 2.f - 1.f, sample.y * 2.f - 1.f, 0.f));
        ds.n = s.frame.n;
        ds.pdf = s.inv_area;
        ds.uv = sample;
        ds.delta = false;
        ds.d = ds.p - itp;
        float dist_squared = squared_norm(ds.d);
        ds.dist = std::sqrt(dist_squared);
        ds.d = ds.d / ds.dist;
        float dp = absdot(ds.d, ds.n);
        float x = dist_squared / dp;
        ds.pdf *= isfinite_(x) ? x : 0.f;
        return ds;
    }
    if (s.type == AMVPT_SHAPE_SPHERE) {
        V3 c{s.center[0], s.center[1], s.center[2]};
        V3 dc_v = c - itp;
        float dc_2 = squared_norm(dc_v);
        float radius_adj = s.radius * (s.flip ? (1.f + RayEpsilon) : (1.f - RayEpsilon));
        bool outside = dc_2 > sqr(radius_adj);
        DS res;
        if (outside) {
            float inv_dc = rsqrt(dc_2), sin_theta_max = s.radius * inv_dc,
                  sin_theta_max_2 = sqr(sin_theta_max), inv_sin_theta_max = rcp(sin_theta_max),
                  cos_theta_max = safe_sqrt(1.f - sin_theta_max_2);
            float sin_theta_2 = sin_theta_max_2 > 0.00068523f
                                    ? 1.f - sqr(fmadd(cos_theta_max - 1.f, sample.x, 1.f))
                                    : sin_theta_max_2 * sample.x;
            float cos_theta = safe_sqrt(1.f - sin_theta_2);
            float cos_alpha = sin_theta_2 * inv_sin_theta_max +
                              cos_theta * safe_sqrt(fnmadd(sin_theta_2, sqr(inv_sin_theta_max), 1.f));
            float sin_alpha = safe_sqrt(fnmadd(cos_alpha, cos_alpha, 1.f));
            float sin_phi, cos_phi;
            sincos_(sample.y * (2.f * Pi), sin_phi, cos_phi);
            Frame f = frame_from(dc_v * -inv_dc);
            V3 d = f.to_world(v3(cos_phi * sin_alpha, sin_phi * sin_alpha, cos_alpha));
            ds.p = fmadd(d, s.radius, c);
            ds.n = d;
            ds.d = ds.p - itp;
            float dist2 = squared_norm(ds.d);
            ds.dist = std::sqrt(dist2);
            ds.d = ds.d / ds.dist;
            ds.pdf = uniform_cone_pdf(cos_theta_max);
            if (ds.dist == 0.f) ds.pdf = 0.f;
            res = ds;
        } else {
            V3 d = square_to_uniform_sphere(sample);
            ds.p = fmadd(d, s.radius, c);
            ds.n = d;
            ds.d = ds.p - itp;
            float dist2 = squared_norm(ds.d);
            ds.dist = std::sqrt(dist2);
            ds.d = ds.d / ds.dist;
            ds.pdf = s.inv_area * dist2 / absdot(ds.d, ds.n);
            res = ds;
        }
        res.delta = s.radius == 0.f;
        if (s.flip) res.n = -res.n;
        return res;
    }
    /* Mesh::sample_position (mesh.cpp:765-816): DiscreteDistribution::sample_reuse over the face
     * areas (JIT predicate of sample(), distr_1d.h:116-134), warp::square_to_uniform_triangle */
    const uint32_t n = (uint32_t) s.area_pmf.size();
    const float norm_ = s.inv_area, value = sample.y * s.area_sum;
    uint32_t start = 0, end = n - 1u;
    const uint32_t iters = end ? 32u - (uint32_t) __builtin_clz(end) : 0u;
    for (uint32_t k = 0; k < iters; ++k) {
        const uint32_t middle = (start + end) >> 1;
        const float c = s.area_cdf[middle];
        const bool cond = ((c < value) || c == 0.f) && c != s.area_sum;
        start = cond ? std::min(middle + 1u, end) : start;
        end = cond ? end : middle;
    }
    const float pmf = s.area_pmf[start] * norm_, cdf = start > 0 ? s.area_cdf[start - 1] * norm_ : 0.f;
    sample.y = (sample.y - cdf) / pmf;
    const uint32_t i0 = s.faces[3 * start], i1 = s.faces[3 * start + 1], i2 = s.faces[3 * start + 2];
    V3 p0 = vtx(s, i0), p1 = vtx(s, i1), p2 = vtx(s, i2);
    V3 e0 = p1 - p0, e1 = p2 - p0;
    float t = safe_sqrt(1.f - sample.x), bx = 1.f - t, by = t * sample.y;
    ds.p = fmadd(e0, bx, fmadd(e1, by, p0));
    V3 n3;
    if (!s.nrm.empty()) {
        V3 n0{s.nrm[3 * i0], s.nrm[3 * i0 + 1], s.nrm[3 * i0 + 2]}, n1{s.nrm[3 * i1], s.nrm[3 * i1 + 1], s.nrm[3 * i1 + 2]},
            n2{s.nrm[3 * i2], s.nrm[3 * i2 + 1], s.nrm[3 * i2 + 2]};
        n3 = fmadd(n0, 1.f - bx - by, fmadd(n1, bx, n2 * by));
    } else {
        n3 = cross(e0, e1);
    }
    ds.n = normalize(n3);
    if (s.flip) ds.n = -ds.n;
    ds.pdf = norm_;
    ds.uv = V2{bx, by};
    ds.delta = false;
    /* Shape::sample_direction (shape.cpp:360-377) */
    ds.d = ds.p - itp;
    float dist_squared = squared_norm(ds.d);
    ds.dist = std::sqrt(dist_squared);
    ds.d = ds.d / ds.dist;
    float x = dist_squared / absdot(ds.d, ds.n);
    ds.pdf *= isfinite_(x) ? x : 0.f;
    return ds;
}

static float shape_pdf_direction(const Shape &s, V3 itp, const DS &ds) {
    if (s.type == AMVPT_SHAPE_SPHERE) {
        V3 c{s.center[0], s.center[1], s.center[2]};
        float sin_alpha = s.radius * rcp(norm(c - itp)), cos_alpha = safe_sqrt(1.f - sin_alpha * sin_alpha);
        return sin_alpha < OneMinusEpsilon ? uniform_cone_pdf(cos_alpha)
                                           : s.inv_area * sqr(ds.dist) / absdot(ds.d, ds.n);
    }
    float pdf = s.inv_area, dp = absdot(ds.d, ds.n);
    pdf *= dp != 0.f ? (ds.dist * ds.dist) / dp : 0.f;
    return pdf;
}

/* Scene::sample_emitter_direction, JIT branch (scene.cpp:294-348) */
static std::pair<DS, Spec> sample_emitter_direction(const Scene &sc, const SI &ref, V2 sample, bool active) {
    DS ds;
    Spec spec = sp(0.f);
    size_t n = sc.emitters.size();
    if (n == 0) return {ds, spec};
    float weight = 1.f;
    const uint32_t index = sample_emitter(sc, sample.x, weight);
    if (!active) return {ds, spec}; /* masked vcall: zeros */
    const amvpt_emitter_desc &ed = sc.emitters[index];
    Spec rad{ed.radiance[0], ed.radiance[1], ed.radiance[2]};
    if (ed.type == AMVPT_EMITTER_CONSTANT) {
        /* ConstantBackgroundEmitter::sample_direction (constant.cpp:125-152) */
        V3 d = square_to_uniform_sphere(sample);
        float radius = std::max(sc.bs_radius, norm(ref.p - sc.bs_center)), dist = 2.f * radius;
        ds.p = fmadd(d, dist, ref.p);
        ds.n = -d;
        ds.uv = sample;
        ds.pdf = InvFourPi;
        ds.delta = false;
        ds.d = d;
        ds.dist = dist;
        spec = rad / ds.pdf;
    } else {
        /* AreaLight::sample_direction (area.cpp:117-167) */
        const Shape &s = sc.shapes[ed.shape];
        ds = shape_sample_direction(s, ref.p, sample);
        bool a = dot(ds.d, ds.n) < 0.f && ds.pdf != 0.f;
        spec = a ? rad / ds.pdf : sp(0.f);
    }
    ds.emitter = (int) index;
    ds.pdf *= emitter_pick_pmf(sc, index);
    spec = spec * weight;
    bool act = ds.pdf != 0.f;
    if (act) {
        Ray r = spawn_ray_to(ref.p, ref.n, ds.p);
        if (ray_test(sc, r)) { spec = sp(0.f); ds.pdf = 0.f; }
    }
    return {ds, spec};
}

/* Scene::pdf_emitter_direction (scene.cpp:350-361), masked vcall */
static float pdf_emitter_direction(const Scene &sc, V3 refp, const DS &ds, bool active) {
    if (ds.emitter < 0 || !active) return 0.f;
    const amvpt_emitter_desc &ed = sc.emitters[ds.emitter];
    const float pick = emitter_pick_pmf(sc, (uint32_t) ds.emitter);
    /* ConstantBackgroundEmitter::pdf_direction (constant.cpp:154-159): uniform sphere */
    if (ed.type == AMVPT_EMITTER_CONSTANT) return InvFourPi * pick;
    const Shape &s = sc.shapes[ed.shape];
    float dp = dot(ds.d, ds.n);
    bool a = dp < 0.f;
    float value = shape_pdf_direction(s, refp, ds);
    return (a ? value : 0.f) * pick;
}

/* --------------------------------------------------------------------- */
/* BSDFs                                                                 */
/* --------------------------------------------------------------------- */

struct BSample { V3 wo{0, 0, 0}; float pdf = 0.f, eta = 0.f; uint32_t type = 0; uint32_t comp = 0; };

static uint32_t bsdf_flags(const Scene &sc, int b) {
    if (b < 0) return 0;
    const amvpt_bsdf_desc &d = sc.bsdfs[b];
    if (d.type == AMVPT_BSDF_DIFFUSE) return F_DiffuseReflection | F_FrontSide;
    if (d.type == AMVPT_BSDF_ROUGHCONDUCTOR) {
        uint32_t f = F_GlossyReflection | F_FrontSide;
        if (d.alpha_u != d.alpha_v) f |= F_Anisotropic;
        return f;
    }
    uint32_t f0 = bsdf_flags(sc, d.nested[0]), f1 = bsdf_flags(sc, d.nested[1]);
    return ((f0 & ~F_BackSide) | F_FrontSide) | ((f1 & ~F_FrontSide) | F_BackSide);
}

/* MicrofacetDistribution (microfacet.h) */
struct Microfacet {
    uint32_t type; float au, av; bool visible;
    Microfacet(const amvpt_bsdf_desc &d) : type(d.distribution), visible(d.sample_visible != 0) {
        au = fmaxf_(d.alpha_u, 1e-4f);
        av = fmaxf_(d.alpha_v, 1e-4f);
    }
    float eval(V3 m) const {
        float alpha_uv = au * av, ct = m.z, ct2 = sqr(ct), result;
        if (type == AMVPT_MICROFACET_BECKMANN) {
            result = exp_(-(sqr(m.x / au) + sqr(m.y / av)) / ct2) / (Pi * alpha_uv * sqr(ct2));
        } else {
            result = rcp(Pi * alpha_uv * sqr(sqr(m.x / au) + sqr(m.y / av) + sqr(m.z)));
        }
        return result * ct > 1e-20f ? result : 0.f;
    }
    float smith_g1(V3 v, V3 m) const {
        float xy_alpha_2 = sqr(au * v.x) + sqr(av * v.y), tan_theta_alpha_2 = xy_alpha_2 / sqr(v.z), result;
        if (type == AMVPT_MICROFACET_BECKMANN) {
            float a = rsqrt(tan_theta_alpha_2), a_sqr = sqr(a);
            result = a >= 1.6f ? 1.f : (3.535f * a + 2.181f * a_sqr) / (1.f + 2.276f * a + 2.577f * a_sqr);
        } else {
            result = 2.f / (1.f + std::sqrt(1.f + tan_theta_alpha_2));
        }
        if (xy_alpha_2 == 0.f) result = 1.f;
        if (dot(v, m) * v.z <= 0.f) result = 0.f;
        return result;
    }
    V2 sample_visible_11(float cos_theta_i, V2 s) const {
        if (type == AMVPT_MICROFACET_BECKMANN) {
            /* numerical inversion with three Newton steps (microfacet.h:372-403) */
            float tan_theta_i = safe_sqrt(fnmadd(cos_theta_i, cos_theta_i, 1.f)) / cos_theta_i;
            float cot_theta_i = rcp(tan_theta_i);
            float maxval = erf_(cot_theta_i);
            s.x = fmaxf_(fminf_(s.x, 1.f - 1e-6f), 1e-6f);
            s.y = fmaxf_(fminf_(s.y, 1.f - 1e-6f), 1e-6f);
            float x = maxval - (maxval + 1.f) * erf_(std::sqrt(-log_(s.x)));
            s.x *= 1.f + maxval + InvSqrtPi * tan_theta_i * exp_(-sqr(cot_theta_i));
            for (int i = 0; i < 3; ++i) {
                float slope = erfinv_(x),
                      value = 1.f + x + InvSqrtPi * tan_theta_i * exp_(-sqr(slope)) - s.x,
                      derivative = 1.f - slope * tan_theta_i;
                x -= value / derivative;
            }
            return {erfinv_(x), erfinv_(fmsub(2.f, s.y, 1.f))};
        }
        /* GGX branch (microfacet.h:404-418) */
        V2 p = square_to_uniform_disk_concentric(s);
        float ss = 0.5f * (1.f + cos_theta_i);
        p.y = lerp(safe_sqrt(1.f - sqr(p.x)), p.y, ss);
        float x = p.x, y = p.y, z = safe_sqrt(1.f - fmadd(p.y, p.y, p.x * p.x));
        float sin_theta_i = safe_sqrt(1.f - sqr(cos_theta_i));
        float nrm = rcp(fmadd(sin_theta_i, y, cos_theta_i * z));
        return {fmsub(cos_theta_i, y, sin_theta_i * z) * nrm, x * nrm};
    }
    void sample(V3 wi, V2 s, V3 &m, float &pdf) const {
        if (!visible) {
            /* microfacet.h:244-300: azimuth (isotropic: uniform; anisotropic: tan inversion),
             * then the elevation of the distribution */
            float sin_phi, cos_phi, alpha_2;
            if (au == av) {
                sincos_((2.f * Pi) * s.y, sin_phi, cos_phi);
                alpha_2 = au * au;
            } else {
                float ratio = av / au, tmp = ratio * tan_((2.f * Pi) * s.y);
                cos_phi = rsqrt(fmadd(tmp, tmp, 1.f));
                cos_phi = mulsign(cos_phi, std::fabs(s.y - .5f) - .25f);
                sin_phi = cos_phi * tmp;
                alpha_2 = rcp(sqr(cos_phi / au) + sqr(sin_phi / av));
            }
            float cos_theta, cos_theta_2;
            if (type == AMVPT_MICROFACET_BECKMANN) {
                cos_theta = rsqrt(fnmadd(alpha_2, log_(1.f - s.x), 1.f));
                cos_theta_2 = sqr(cos_theta);
                float cos_theta_3 = fmaxf_(cos_theta_2 * cos_theta, 1e-20f);
                pdf = (1.f - s.x) / (Pi * au * av * cos_theta_3);
            } else {
                float tan_theta_m_2 = alpha_2 * s.x / (1.f - s.x);
                cos_theta = rsqrt(1.f + tan_theta_m_2);
                cos_theta_2 = sqr(cos_theta);
                float temp = 1.f + tan_theta_m_2 / alpha_2, cos_theta_3 = fmaxf_(cos_theta_2 * cos_theta, 1e-20f);
                pdf = rcp(Pi * au * av * cos_theta_3 * sqr(temp));
            }
            float sin_theta = std::sqrt(1.f - cos_theta_2);
            m = v3(cos_phi * sin_theta, sin_phi * sin_theta, cos_theta);
            return;
        }
        V3 wi_p = normalize(v3(au * wi.x, av * wi.y, wi.z));
        /* Frame::sincos_phi (frame.h:111-122) */
        float st2 = fmadd(wi_p.x, wi_p.x, sqr(wi_p.y)), inv_st = rsqrt(st2);
        float rx = wi_p.x * inv_st, ry = wi_p.y * inv_st;
        if (std::fabs(st2) <= 4.f * Epsilon) { rx = 1.f; ry = 0.f; }
        else { rx = fminf_(fmaxf_(rx, -1.f), 1.f); ry = fminf_(fmaxf_(ry, -1.f), 1.f); }
        float sin_phi = ry, cos_phi = rx, cos_theta = wi_p.z;
        V2 slope = sample_visible_11(cos_theta, s);
        slope = {fmsub(cos_phi, slope.x, sin_phi * slope.y) * au, fmadd(sin_phi, slope.x, cos_phi * slope.y) * av};
        m = normalize(v3(-slope.x, -slope.y, 1.f));
        pdf = eval(m) * smith_g1(wi, m) * absdot(wi, m) / wi.z;
    }
};

static float fresnel_conductor(float ci, float er, float ei) {
    float ci2 = ci * ci, si2 = 1.f - ci2, si4 = si2 * si2;
    float temp_1 = er * er - ei * ei - si2,
          a_2_pb_2 = safe_sqrt(temp_1 * temp_1 + 4.f * ei * ei * er * er),
          a = safe_sqrt(.5f * (a_2_pb_2 + temp_1));
    float term_1 = a_2_pb_2 + ci2, term_2 = 2.f * ci * a;
    float r_s = (term_1 - term_2) / (term_1 + term_2);
    float term_3 = a_2_pb_2 * ci2 + si4, term_4 = term_2 * si2;
    float r_p = r_s * (term_3 - term_4) / (term_3 + term_4);
    return 0.5f * (r_s + r_p);
}
static Spec fresnel_c(const amvpt_bsdf_desc &d, float ci) {
    return {fresnel_conductor(ci, d.eta[0], d.k[0]), fresnel_conductor(ci, d.eta[1], d.k[1]),
            fresnel_conductor(ci, d.eta[2], d.k[2])};
}

/* All BSDF entry points: masked vcalls return zeros for b < 0 or !active. */
struct EvalPdf { Spec val; float pdf; };

static EvalPdf bsdf_eval_pdf(const Scene &sc, int b, uint32_t ctx, const SI &si, V3 wi, V3 wo, bool active);
static float bsdf_pdf(const Scene &sc, int b, uint32_t ctx, V3 wi, V3 wo, bool active);
static std::pair<BSample, Spec> bsdf_sample(const Scene &sc, int b, uint32_t ctx, V3 wi, float s1, V2 s2, bool active);

static EvalPdf bsdf_eval_pdf(const Scene &sc, int b, uint32_t ctx, const SI &si, V3 wi, V3 wo, bool active) {
    if (b < 0 || !active) return {sp(0.f), 0.f};
    const amvpt_bsdf_desc &d = sc.bsdfs[b];
    if (d.type == AMVPT_BSDF_DIFFUSE) {
        if (!ctx_enabled(ctx, F_DiffuseReflection)) return {sp(0.f), 0.f};
        float cti = wi.z, cto = wo.z;
        bool a = active && cti > 0.f && cto > 0.f;
        Spec refl{d.reflectance[0], d.reflectance[1], d.reflectance[2]};
        Spec value = refl * InvPi * cto;
        float pdf = cosine_hemisphere_pdf(wo);
        return {a ? value : sp(0.f), a ? pdf : 0.f};
    }
    if (d.type == AMVPT_BSDF_ROUGHCONDUCTOR) {
        float cti = wi.z, cto = wo.z;
        V3 H = normalize(wo + wi);
        bool a = active && cti > 0.f && cto > 0.f && dot(wi, H) > 0.f && dot(wo, H) > 0.f;
        if (!ctx_enabled(ctx, F_GlossyReflection)) return {sp(0.f), 0.f};
        Microfacet distr(d);
        float D = distr.eval(H);
        a = a && D != 0.f;
        float g1wi = distr.smith_g1(wi, H);
        float G = g1wi * distr.smith_g1(wo, H);
        float value = D * G / (4.f * wi.z);
        Spec F = fresnel_c(d, dot(wi, H));
        Spec v = F * value;
        if (d.has_specular_reflectance)
            v = F * (value * Spec{d.specular_reflectance[0], d.specular_reflectance[1], d.specular_reflectance[2]});
        float pdf;
        if (distr.visible) pdf = D * g1wi / (4.f * cti);
        else pdf = distr.eval(H) * H.z / (4.f * dot(wo, H));
        return {a ? v : sp(0.f), a ? pdf : 0.f};
    }
    /* twosided (twosided.cpp:215-262) */
    if (d.nested[0] == d.nested[1]) {
        V3 wo2 = wo, wi2 = wi;
        wo2.z = mulsign(wo.z, wi.z);
        wi2.z = std::fabs(wi.z);
        return bsdf_eval_pdf(sc, d.nested[0], ctx, si, wi2, wo2, active);
    }
    bool front = wi.z > 0.f && active, back = wi.z < 0.f && active;
    EvalPdf r = bsdf_eval_pdf(sc, d.nested[0], ctx, si, wi, wo, front);
    if (back) r = bsdf_eval_pdf(sc, d.nested[1], ctx, si, v3(wi.x, wi.y, -wi.z), v3(wo.x, wo.y, -wo.z), back);
    return r;
}

static float bsdf_pdf(const Scene &sc, int b, uint32_t ctx, V3 wi, V3 wo, bool active) {
    if (b < 0 || !active) return 0.f;
    const amvpt_bsdf_desc &d = sc.bsdfs[b];
    if (d.type == AMVPT_BSDF_DIFFUSE) {
        if (!ctx_enabled(ctx, F_DiffuseReflection)) return 0.f;
        float pdf = cosine_hemisphere_pdf(wo);
        return (wi.z > 0.f && wo.z > 0.f) ? pdf : 0.f;
    }
    if (d.type == AMVPT_BSDF_ROUGHCONDUCTOR) {
        float cti = wi.z, cto = wo.z;
        V3 m = normalize(wo + wi);
        bool a = active && cti > 0.f && cto > 0.f && dot(wi, m) > 0.f && dot(wo, m) > 0.f;
        if (!ctx_enabled(ctx, F_GlossyReflection)) return 0.f;
        Microfacet distr(d);
        float result;
        if (distr.visible) result = distr.eval(m) * distr.smith_g1(wi, m) / (4.f * cti);
        else result = distr.eval(m) * m.z / (4.f * dot(wo, m));
        return a ? result : 0.f;
    }
    if (d.nested[0] == d.nested[1]) {
        V3 wo2 = wo, wi2 = wi;
        wo2.z = mulsign(wo.z, wi.z);
        wi2.z = std::fabs(wi.z);
        return bsdf_pdf(sc, d.nested[0], ctx, wi2, wo2, active);
    }
    bool front = wi.z > 0.f && active, back = wi.z < 0.f && active;
    float r = bsdf_pdf(sc, d.nested[0], ctx, wi, wo, front);
    if (back) r = bsdf_pdf(sc, d.nested[1], ctx, v3(wi.x, wi.y, -wi.z), v3(wo.x, wo.y, -wo.z), back);
    return r;
}

static std::pair<BSample, Spec> bsdf_sample(const Scene &sc, int b, uint32_t ctx, V3 wi, float s1, V2 s2, bool active) {
    BSample bs;
    if (b < 0 || !active) return {bs, sp(0.f)};
    const amvpt_bsdf_desc &d = sc.bsdfs[b];
    if (d.type == AMVPT_BSDF_DIFFUSE) {
        float cti = wi.z;
        bool a = active && cti > 0.f;
        if (!ctx_enabled(ctx, F_DiffuseReflection)) return {bs, sp(0.f)};
        bs.wo = square_to_cosine_hemisphere(s2);
        bs.pdf = cosine_hemisphere_pdf(bs.wo);
        bs.eta = 1.f;
        bs.type = F_DiffuseReflection;
        bs.comp = 0;
        Spec refl{d.reflectance[0], d.reflectance[1], d.reflectance[2]};
        return {bs, (a && bs.pdf > 0.f) ? refl : sp(0.f)};
    }
    if (d.type == AMVPT_BSDF_ROUGHCONDUCTOR) {
        float cti = wi.z;
        bool a = active && cti > 0.f;
        if (!ctx_enabled(ctx, F_GlossyReflection)) return {bs, sp(0.f)};
        Microfacet distr(d);
        V3 m;
        distr.sample(wi, s2, m, bs.pdf);
        bs.wo = fmsub(m, 2.f * dot(wi, m), wi); /* reflect(wi, m) */
        bs.eta = 1.f;
        bs.comp = 0;
        bs.type = F_GlossyReflection;
        a = a && bs.pdf != 0.f && bs.wo.z > 0.f;
        float weight;
        if (distr.visible) weight = distr.smith_g1(bs.wo, m);
        else weight = distr.smith_g1(wi, m) * distr.smith_g1(bs.wo, m) * dot(wi, m) / (cti * m.z);
        bs.pdf /= 4.f * dot(bs.wo, m);
        Spec F = fresnel_c(d, dot(wi, m));
        Spec w = sp(weight);
        if (d.has_specular_reflectance)
            w = w * Spec{d.specular_reflectance[0], d.specular_reflectance[1], d.specular_reflectance[2]};
        return {bs, a ? F * w : sp(0.f)};
    }
    /* twosided (twosided.cpp:112-146) */
    if (d.nested[0] == d.nested[1]) {
        V3 wi2 = wi;
        wi2.z = std::fabs(wi.z);
        auto r = bsdf_sample(sc, d.nested[0], ctx, wi2, s1, s2, active);
        r.first.wo.z = mulsign(r.first.wo.z, wi.z);
        return r;
    }
    bool front = wi.z > 0.f && active, back = wi.z < 0.f && active;
    std::pair<BSample, Spec> r{BSample(), sp(0.f)};
    if (front) r = bsdf_sample(sc, d.nested[0], ctx, wi, s1, s2, front);
    if (back) {
        r = bsdf_sample(sc, d.nested[1], ctx, v3(wi.x, wi.y, -wi.z), s1, s2, back);
        r.first.wo.z *= -1.f;
    }
    return r;
}

static float bsdf_eval_roughness(const Scene &sc, int b, V3 wi, bool active) {
    if (b < 0 || !active) return 0.f;
    const amvpt_bsdf_desc &d = sc.bsdfs[b];
    if (d.type == AMVPT_BSDF_DIFFUSE) return 1.f; /* diffuse.cpp:186-188 */
    if (d.type == AMVPT_BSDF_ROUGHCONDUCTOR)     /* roughconductor.cpp:518-523 */
        return std::sqrt(0.5f * (sqr(d.alpha_u) + sqr(d.alpha_v)));
    if (d.nested[0] == d.nested[1]) return bsdf_eval_roughness(sc, d.nested[0], v3(wi.x, wi.y, std::fabs(wi.z)), active);
    bool front = wi.z > 0.f && active, back = wi.z < 0.f && active;
    float r = bsdf_eval_roughness(sc, d.nested[0], wi, front);
    if (back) r = bsdf_eval_roughness(sc, d.nested[1], v3(wi.x, wi.y, -wi.z), back);
    return r;
}

/* BSDF::eval_pdf_sample (bsdf.cpp:28-37) */
struct EPS { Spec val; float pdf; BSample bs; Spec weight; };
static EPS bsdf_eval_pdf_sample(const Scene &sc, int b, const SI &si, V3 wi, V3 wo, float s1, V2 s2, bool active) {
    EPS r;
    EvalPdf ep = bsdf_eval_pdf(sc, b, CTX_ALL, si, wi, wo, active);
    auto sm = bsdf_sample(sc, b, CTX_ALL, wi, s1, s2, active);
    r.val = ep.val; r.pdf = ep.pdf; r.bs = sm.first; r.weight = sm.second;
    return r;
}

/* --------------------------------------------------------------------- */
/* Sensors                                                               */
/* --------------------------------------------------------------------- */

/* PerspectiveCamera::sample_ray (perspective.cpp:205-241) */
static Ray persp_sample_ray(const amvpt_view_desc &v, V2 pos) {
    V3 near_p = xform_point(v.sample_to_camera, v3(pos.x + v.pp_offset[0], pos.y + v.pp_offset[1], 0.f));
    V3 d = normalize(near_p);
    Ray r;
    r.o = v3(v.to_world[3], v.to_world[7], v.to_world[11]);
    r.d = xform_vector(v.to_world, d);
    float inv_z = rcp(d.z);
    float near_t = v.near_clip * inv_z, far_t = v.far_clip * inv_z;
    r.o = r.o + r.d * near_t;
    r.maxt = far_t - near_t;
    return r;
}

/* ThinLensCamera::sample_ray (thinlens.cpp:220-257) */
static Ray thin_sample_ray(const amvpt_view_desc &v, V2 pos, V2 ap) {
    V3 near_p = xform_point(v.sample_to_camera, v3(pos.x, pos.y, 0.f));
    V2 t = square_to_uniform_disk_concentric(ap);
    V3 aperture_p = v3(v.aperture_radius * t.x, v.aperture_radius * t.y, 0.f);
    V3 focus_p = near_p * (v.focus_distance / near_p.z);
    V3 d = normalize(focus_p - aperture_p);
    Ray r;
    r.o = xform_point_affine(v.to_world, aperture_p);
    r.d = xform_vector(v.to_world, d);
    float inv_z = rcp(d.z);
    float near_t = v.near_clip * inv_z, far_t = v.far_clip * inv_z;
    r.o = r.o + r.d * near_t;
    r.maxt = far_t - near_t;
    return r;
}

static Ray camera_sample_ray(const amvpt_view_desc &v, V2 pos, V2 ap) {
    return v.type == AMVPT_CAMERA_THINLENS ? thin_sample_ray(v, pos, ap) : persp_sample_ray(v, pos);
}

struct SurfSample { DS ds; float Jp; bool face; bool valid; };

/* ThinLensCamera::sample_surface (thinlens.cpp:358-418), JIT semantics (none_or<false>
 * early-outs never taken); `ap` = the primary lane's aperture sample, shared by all views. */
static SurfSample thin_sample_surface(const amvpt_view_desc &v, const SI &it, bool active, V2 ap) {
    SurfSample r;
    r.Jp = 0.f; r.face = false; r.valid = false;
    if (!active) return r;
    V3 ref_p = xform_point_affine(v.to_world_inv, it.p);
    DS ds;
    bool a = ref_p.z >= v.near_clip && ref_p.z <= v.far_clip;
    V2 t = square_to_uniform_disk_concentric(ap);
    V3 aperture_p = v3(t.x * v.aperture_radius, t.y * v.aperture_radius, 0.f);
    V3 local_d = ref_p - aperture_p;
    float dist = norm(local_d), inv_dist = rcp(dist);
    local_d = local_d * inv_dist;
    float ctf = local_d.z, ictf = rcp(ctf), ictf3 = ictf * ictf * ictf;
    float inv_f = 1.f / v.focus_distance;
    /* aperture_p * (1 / f) + local_d / local_d.z: separate multiply and add (no contraction) */
    V3 film_plane = v3(aperture_p.x * inv_f + local_d.x / local_d.z, aperture_p.y * inv_f + local_d.y / local_d.z,
                       aperture_p.z * inv_f + local_d.z / local_d.z);
    V3 scr = xform_point_affine(v.camera_to_sample, film_plane);
    a = a && scr.x >= 0.f && scr.y >= 0.f && scr.x <= 1.f && scr.y <= 1.f;
    float pdf_lens = rcp(sqr(v.aperture_radius) * Pi);
    float pdf_film = v.normalization * ictf3;
    ds.pdf = pdf_lens * pdf_film;
    ds.uv = {scr.x * v.resolution[0], scr.y * v.resolution[1]};
    ds.p = xform_point_affine(v.to_world, aperture_p);
    ds.d = (ds.p - it.p) * inv_dist;
    ds.dist = dist;
    ds.n = xform_vector(v.to_world, v3(0.f, 0.f, 1.f));
    float cts = dot(ds.d, it.n);
    bool face = cts > 0.f;
    cts = std::fabs(cts);
    r.ds = ds;
    r.Jp = (cts * inv_dist * inv_dist) * ds.pdf;
    r.face = face;
    r.valid = a;
    return r;
}

/* PerspectiveCamera::sample_surface (perspective.cpp:327-385), JIT semantics;
 * reached through GridSensor::sample_surface's masked vcall (grid.cpp:331-336). */
static SurfSample persp_sample_surface(const amvpt_view_desc &v, const SI &it, bool active) {
    SurfSample r;
    r.Jp = 0.f; r.face = false; r.valid = false;
    if (!active) return r;
    V3 ref_p = xform_point_affine(v.to_world_inv, it.p);
    DS ds;
    ds.pdf = 0.f;
    bool a = ref_p.z >= v.near_clip && ref_p.z <= v.far_clip;
    V3 screen = xform_point(v.camera_to_sample, ref_p);
    ds.uv = {screen.x - v.pp_offset[0], screen.y - v.pp_offset[1]};
    a = a && ds.uv.x >= 0.f && ds.uv.x <= 1.f && ds.uv.y >= 0.f && ds.uv.y <= 1.f;
    ds.uv = {ds.uv.x * v.resolution[0], ds.uv.y * v.resolution[1]};
    V3 local_d = ref_p;
    float dist = norm(local_d), inv_dist = rcp(dist);
    float ctf = local_d.z;
    a = a && ctf > 0.f;
    float ictf = rcp(ctf), ictf3 = ictf * ictf * ictf;
    float pdf_film = v.normalization * ictf3;
    ds.pdf = pdf_film;
    ds.p = xform_point_affine(v.to_world, v3(0.f, 0.f, 0.f));
    ds.d = (ds.p - it.p) * inv_dist;
    ds.dist = dist;
    ds.n = xform_vector(v.to_world, v3(0.f, 0.f, 1.f));
    float cts = dot(ds.d, it.n);
    bool face = cts > 0.f;
    cts = std::fabs(cts);
    float Jp = (cts * inv_dist * inv_dist) * ds.pdf;
    r.ds = ds; r.Jp = Jp; r.face = face; r.valid = a;
    return r;
}

static SurfSample camera_sample_surface(const amvpt_view_desc &v, const SI &it, bool active, V2 ap) {
    return v.type == AMVPT_CAMERA_THINLENS ? thin_sample_surface(v, it, active, ap) : persp_sample_surface(v, it, active);
}

/* --------------------------------------------------------------------- */
/* Film (ImageBlock)                                                     */
/* --------------------------------------------------------------------- */

struct Film {
    uint32_t W, H, C;
    bool box;
    Gaussian g;
    float *data;
    int ox = 0, oy = 0;   /* ImageBlock offset (the hdrfilm crop offset, mvpath.cpp:168) */
    /* fixed-point film (oracle_set_fixed_film; the device's AMVPT_OPT_DETERMINISTIC film, include/amvpt.h):
     * each cell add is rounded to a multiple of 2^-32 and summed as an integer, so the sum does not depend
     * on the order of the adds; finite adds of |v| >= 2^31 are dropped and counted, non-finite ones dropped */
    int64_t *fx = nullptr;
    uint64_t *drops = nullptr;
    void add(float *ptr, float v) const {
        if (!fx) { *ptr += v; return; }
        const double d = (double) v * 4294967296.0;
        if (!(std::fabs(d) < 2147483647.0 * 4294967296.0)) {
            if (std::isfinite(v)) ++*drops;
            return;
        }
        int64_t &c = fx[ptr - data];
        c = (int64_t) ((uint64_t) c + (uint64_t) (int64_t) std::rint(d));   /* two's-complement wrap, as the device's u64 atomics */
    }
    void put(V2 pos, const float *values, bool active, bool coalesce) const {
        if (!active) return;
        if (box) {
            /* imageblock.cpp:211: floor(pos) - offset */
            int px = (int) std::floor(pos.x) - ox, py = (int) std::floor(pos.y) - oy;
            uint32_t ux = (uint32_t) px, uy = (uint32_t) py;
            if (!(ux < W && uy < H)) return;
            float *ptr = data + ((size_t) uy * W + ux) * C;
            for (uint32_t k = 0; k < C; ++k) add(ptr + k, values[k]);
            return;
        }
        float radius = g.radius;
        if (!coalesce) {
            /* imageblock.cpp:265-427 (recorded-loop form 1.2): pos + ((int) border - offset - .5f) */
            V2 pos_f{pos.x + ((float) (-ox) - 0.5f), pos.y + ((float) (-oy) - 0.5f)};
            V2 pos_0_f{pos_f.x - radius, pos_f.y - radius}, pos_1_f{pos_f.x + radius, pos_f.y + radius};
            int p0x = std::max((int) std::ceil(pos_0_f.x), 0), p0y = std::max((int) std::ceil(pos_0_f.y), 0);
            int p1x = std::min((int) std::floor(pos_1_f.x), (int) W - 1), p1y = std::min((int) std::floor(pos_1_f.y), (int) H - 1);
            uint32_t u0x = (uint32_t) p0x, u0y = (uint32_t) p0y, u1x = (uint32_t) p1x, u1y = (uint32_t) p1y;
            uint32_t count = (uint32_t) std::ceil(2.f * radius);
            if (!(u0x <= u1x && u0y <= u1y)) return;
            V2 rel_f{(float) u0x - pos_f.x, (float) u0y - pos_f.y};
            for (uint32_t ys = 0; ys < count; ++ys) {
                float wy = g.eval(rel_f.y + (float) ys);
                bool a1 = u0y + ys <= u1y;
                for (uint32_t xs = 0; xs < count; ++xs) {
                    float wx = g.eval(rel_f.x + (float) xs);
                    float w = wx * wy;
                    bool a2 = a1 && (u0x + xs <= u1x);
                    if (!a2) continue;
                    float *ptr = data + ((size_t) (u0y + ys) * W + (u0x + xs)) * C;
                    for (uint32_t k = 0; k < C; ++k) add(ptr + k, values[k] * w);
                }
            }
            return;
        }
        /* coalesced (imageblock.cpp:433-558, recorded-loop form 2.2) */
        uint32_t n = (uint32_t) std::ceil(radius - .5f), count = 2 * n + 1;
        int pix = (int) std::floor(pos.x) - (int) n, piy = (int) std::floor(pos.y) - (int) n;
        uint32_t x = (uint32_t) (pix - ox), y = (uint32_t) (piy - oy);   /* pos_i_local (imageblock.cpp:447) */
        V2 rel_f{((float) pix + .5f) - pos.x, ((float) piy + .5f) - pos.y};
        for (uint32_t ys = 0; ys < count; ++ys) {
            float wy = g.eval(rel_f.y + (float) ys);
            bool a1 = y + ys < H;
            for (uint32_t xs = 0; xs < count; ++xs) {
                float wx = g.eval(rel_f.x + (float) xs);
                float w = wx * wy;
                bool a2 = a1 && (x + xs < W);
                if (!a2) continue;
                float *ptr = data + ((size_t) (y + ys) * W + (x + xs)) * C;
                for (uint32_t k = 0; k < C; ++k) add(ptr + k, values[k] * w);
            }
        }
    }
};

/* --------------------------------------------------------------------- */
/* Integrator                                                            */
/* --------------------------------------------------------------------- */

static inline float mis_weight(float a, float b) {
    a *= a; b *= b;
    float w = a / (a + b);
    return isfinite_(w) ? w : 0.f;
}

struct SampleData {
    Spec result{0, 0, 0}, bsdf_val{0, 0, 0};
    V3 wi{0, 0, 0}, wo_r{0, 0, 0};
    V2 pos{0, 0};
    float weight = 0, pdfM = 0, pdf = 0, pdf_lk = 0, Jp = 0, iJp = 0;
    uint32_t idx = 0;
    bool indirect = false, valid = false;
};

struct BSDFData { int bsdf; float alpha, sqr_a, rsqrt_a; bool diffuse, reuse; };

struct Renderer {
    const Scene &sc;
    const amvpt_view_desc *views;
    amvpt_params P;
    uint32_t G;                 /* group size */
    uint32_t spp_pp, n_passes;
    uint64_t L;                 /* lanes per pass */
    uint32_t fw, fh;
    uint64_t stat_vertices = 0, stat_reuse = 0, stat_vis = 0, stat_splats = 0;

    V2 ap{.5f, .5f};            /* aperture sample of the current lane */
    bool needs_ap = false;      /* Sensor::needs_aperture_sample (thin-lens views) */

    Renderer(const Scene &s, const amvpt_view_desc *v, const amvpt_params &p) : sc(s), views(v), P(p) {
        /* grid: its first sub-sensor decides (grid.cpp:228); batch: any child (batch.cpp:127) */
        uint32_t nv = p.multisensor ? (p.batch ? p.n_views : 1u) : 1u;
        for (uint32_t i = 0; i < nv; ++i) needs_ap = needs_ap || v[i].type == AMVPT_CAMERA_THINLENS;
    }

    /* GridSensor::sample_ray_idx (grid.cpp:269-297) / single camera */
    Ray sample_ray_idx(V2 pos01, uint32_t &index) const {
        if (!P.multisensor) {
            index = 0;
            return camera_sample_ray(views[0], pos01, ap);
        }
        if (P.batch) {
            /* BatchSensor::sample_ray_idx (batch.cpp:163-181): clamp, then reverse_x */
            float idx_f = pos01.x * (float) P.n_views;
            uint32_t idx_u = (uint32_t) idx_f;
            index = std::min(idx_u, P.n_views - 1);
            if (P.reverse_x) index = (P.n_views - 1) - index;
            return camera_sample_ray(views[index], V2{idx_f - (float) idx_u, pos01.y}, ap);
        }
        float gx = (float) P.grid_x, gy = (float) P.grid_y;
        V2 idx_f{pos01.x * gx, pos01.y * gy};
        uint32_t ux = (uint32_t) idx_f.x, uy = (uint32_t) idx_f.y;
        uint32_t ix = ux, iy = uy;
        if (P.reverse_x) ix = (P.grid_x - 1) - ix;
        if (P.reverse_y) iy = (P.grid_y - 1) - iy;
        index = ix + P.grid_x * iy;
        index = std::min(index, P.n_views - 1);
        V2 p2{idx_f.x - (float) ux, idx_f.y - (float) uy};
        return camera_sample_ray(views[index], p2, ap);
    }

    /* sample_single (mvpath_single.h:82-278) == PathIntegrator::sample */
    std::pair<Spec, bool> sample_single(PCG32 &rng, Ray ray, uint64_t &verts) const {
        if (P.max_depth == 0) return {sp(0.f), false};
        Spec throughput = sp(1.f), result = sp(0.f);
        float eta = 1.f;
        uint32_t depth = 0;
        bool valid_ray = !P.hide_emitters && sc.environment >= 0;   /* mvpath_single.h:98, path.cpp:114 */
        SI prev_si; prev_si.t = 0.f; /* dr::zeros<Interaction3f> */
        float prev_bsdf_pdf = 1.f;
        bool prev_bsdf_delta = true;
        bool active = true;
        while (active) {
            ++verts;
            SI si = intersect(sc, ray);
            int em = si_emitter(sc, si);
            {
                DS ds;
                ds.p = si.p; ds.n = si.sh.n;
                V3 rel = si.p - prev_si.p;
                ds.dist = norm(rel);
                ds.d = si.valid() ? rel / ds.dist : -si.wi;
                ds.emitter = em;
                float em_pdf = pdf_emitter_direction(sc, prev_si.p, ds, !prev_bsdf_delta);
                float mis_bsdf = mis_weight(prev_bsdf_pdf, em_pdf);
                result = spec_fma(throughput, emitter_eval(sc, em, si, prev_bsdf_pdf > 0.f) * mis_bsdf, result);
            }
            bool active_next = (depth + 1 < P.max_depth) && si.valid();
            int b = si.valid() ? sc.shapes[si.shape].bsdf : -1;
            bool active_em = active_next && (bsdf_flags(sc, b) & F_Smooth);
            V2 es{rng.next_1d(), 0.f}; es.y = rng.next_1d();
            auto [ds, em_weight] = sample_emitter_direction(sc, si, es, active_em);
            active_em = active_em && ds.pdf != 0.f;
            V3 wo = si.to_local(ds.d);
            float s1 = rng.next_1d();
            V2 s2{rng.next_1d(), 0.f}; s2.y = rng.next_1d();
            EPS e = bsdf_eval_pdf_sample(sc, b, si, si.wi, wo, s1, s2, true);
            {
                float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, e.pdf);
                if (active_em) result = spec_fma(throughput, e.val * em_weight * mis_em, result);
            }
            ray = spawn_ray(si.p, si.n, si.to_world(e.bs.wo));
            throughput = throughput * e.weight;
            eta *= e.bs.eta;
            valid_ray = valid_ray || (active && si.valid() && !(e.bs.type & F_Null));
            prev_si = si;
            prev_bsdf_pdf = e.bs.pdf;
            prev_bsdf_delta = (e.bs.type & F_Delta) != 0;
            if (si.valid()) depth += 1;
            float tmax = smax(throughput);
            float rr_prob = fminf_(tmax * sqr(eta), .95f);
            bool rractive = depth >= P.rr_depth;
            bool rr_continue = rng.next_1d() < rr_prob;
            if (rractive) throughput = throughput * rcp(rr_prob);
            active = active_next && (!rractive || rr_continue) && (tmax != 0.f);
        }
        return {valid_ray ? result : sp(0.f), valid_ray};
    }

    /* sample_suffix (mvpath_multi.h:526-689) */
    std::pair<Spec, bool> sample_suffix(PCG32 &rng, Ray ray, Spec throughput, float eta, uint32_t depth,
                                        SI prev_si, float prev_bsdf_pdf, bool prev_bsdf_delta, bool active,
                                        uint64_t &verts) const {
        if (P.max_depth <= 1) return {sp(0.f), false};
        Spec result = sp(0.f);
        bool valid_ray = false;
        while (active) {
            ++verts;
            SI si = intersect(sc, ray);
            int em = si_emitter(sc, si);
            {
                DS ds;
                ds.p = si.p; ds.n = si.sh.n;
                V3 rel = si.p - prev_si.p;
                ds.dist = norm(rel);
                ds.d = si.valid() ? rel / ds.dist : -si.wi;
                ds.emitter = em;
                float em_pdf = pdf_emitter_direction(sc, prev_si.p, ds, !prev_bsdf_delta);
                float mis_bsdf = mis_weight(prev_bsdf_pdf, em_pdf);
                result = spec_fma(throughput, emitter_eval(sc, em, si, prev_bsdf_pdf > 0.f) * mis_bsdf, result);
            }
            bool active_next = (depth + 1 < P.max_depth) && si.valid();
            int b = si.valid() ? sc.shapes[si.shape].bsdf : -1;
            bool active_em = active_next && (bsdf_flags(sc, b) & F_Smooth);
            V2 es{rng.next_1d(), 0.f}; es.y = rng.next_1d();
            auto [ds, em_weight] = sample_emitter_direction(sc, si, es, active_em);
            active_em = active_em && ds.pdf != 0.f;
            V3 wo = si.to_local(ds.d);
            float s1 = rng.next_1d();
            V2 s2{rng.next_1d(), 0.f}; s2.y = rng.next_1d();
            EPS e = bsdf_eval_pdf_sample(sc, b, si, si.wi, wo, s1, s2, true);
            {
                float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, e.pdf);
                if (active_em) result = spec_fma(throughput, e.val * em_weight * mis_em, result);
            }
            ray = spawn_ray(si.p, si.n, si.to_world(e.bs.wo));
            throughput = throughput * e.weight;
            eta *= e.bs.eta;
            prev_si = si;
            prev_bsdf_pdf = e.bs.pdf;
            prev_bsdf_delta = (e.bs.type & F_Delta) != 0;
            if (si.valid()) depth += 1;
            float tmax = smax(throughput);
            float rr_prob = fminf_(tmax * sqr(eta), .95f);
            bool rractive = depth >= P.rr_depth;
            bool rr_continue = rng.next_1d() < rr_prob;
            valid_ray = valid_ray || (active && si.valid() && !(e.bs.type & F_Null));
            if (rractive) throughput = throughput * rcp(rr_prob);
            active = active_next && (!rractive || rr_continue) && (tmax != 0.f);
        }
        return {result, valid_ray};
    }

    /* tv_pdf / tv_pdf_fast (mvpath.h:259-293) */
    float tv_pdf(V3 wo_l, V3 si_k_wi, float p_k, const BSDFData &bd, bool active) const {
        active = active && p_k > 0.f;
        float p_l = bsdf_pdf(sc, bd.bsdf, CTX_GLOSSY, si_k_wi, wo_l, active);
        active = active && p_l > 0.f;
        float p_max = fmaxf_(p_l, p_k), p_min = fminf_(p_l, p_k);
        float q = p_min * rcp(p_max);
        float p = fmadd(q - 1.f, bd.rsqrt_a, 1.f);
        p = sqr(fmaxf_(p, 0.f));
        p = lerp(p, q, bd.alpha);
        return active ? p : 0.f;
    }
    float tv_pdf_fast(V3 wo_l, V3 wi_k, float p_k, const BSDFData &bd, bool active) const {
        float p_l = sqr(normalize(wi_k + wo_l).z);
        float N = fmadd(bd.sqr_a, fmaxf_(p_k, p_l), 1.f), D = fmadd(bd.sqr_a, fminf_(p_k, p_l), 1.f);
        float q = sqr(N * rcp(D));
        float p = fmadd(q - 1.f, bd.rsqrt_a, 1.f);
        p = sqr(fmaxf_(p, 0.f));
        p = lerp(p, q, bd.alpha);
        return active ? p : 0.f;
    }

    /* sensors_visible<primary> (mvpath.h:243-256) */
    SurfSample sensors_visible(bool primary, const SI &si, bool prim_face, uint32_t idx, bool active, bool count) {
        SurfSample r = camera_sample_surface(views[idx], si, active, ap);
        if (!primary) {
            r.valid = r.valid && (r.face == prim_face) && r.Jp > 0.f;
            if (r.valid) { /* ray_test result only matters where valid */
                if (count) stat_vis++;
                Ray ray = spawn_ray_to(si.p, si.n, r.ds.p);
                r.valid = r.valid && !ray_test(sc, ray);
            }
        }
        return r;
    }

    /* camera_selection (mvpath_multi.h:371-464) */
    void camera_selection(PCG32 &rng, SampleData *S, const SI &si, const BSDFData &bd, V3 wo, float rand_1,
                          V2 rand_2, bool p_hit, BSample &bsdf_sample, float &direct_pdf) {
        SampleData &p = S[0];
        bool p_face = si.wi.z > 0.f;
        SurfSample ps = sensors_visible(true, si, p_face, p.idx, p_hit, false);
        p.pdf = ps.ds.pdf;
        p.pdf_lk = ps.ds.pdf;
        p.Jp = ps.Jp;
        p.iJp = p_hit ? rcp(ps.Jp) : 0.f;
        p.wi = si.wi;
        p.wo_r = v3(-si.wi.x, -si.wi.y, si.wi.z);
        p.valid = p_hit;
        p.indirect = p_hit;
        p.pdfM = P.fast_mis ? sqr(normalize(p.wi + p.wo_r).z) : bsdf_pdf(sc, bd.bsdf, CTX_GLOSSY, si.wi, p.wo_r, p_hit);
        if (bd.diffuse) p.pdfM = 1.f;
        float n_direct = 1.f, n_indir = 2.f;
        for (uint32_t k = 1; k < G; ++k) {
            SampleData &s = S[k];
            SurfSample r = sensors_visible(false, si, p_face, s.idx, bd.reuse, true);
            bool valid = r.valid;
            s.wi = si.to_local(r.ds.d);
            s.wo_r = v3(-s.wi.x, -s.wi.y, s.wi.z);
            V3 si_k_wi = s.wi;
            s.pdfM = P.fast_mis ? sqr(normalize(si_k_wi + s.wo_r).z) : bsdf_pdf(sc, bd.bsdf, CTX_GLOSSY, si_k_wi, s.wo_r, valid);
            float pdf_Mat = P.fast_mis ? tv_pdf_fast(p.wo_r, si_k_wi, s.pdfM, bd, valid) : tv_pdf(p.wo_r, si_k_wi, s.pdfM, bd, valid);
            if (bd.diffuse) pdf_Mat = 1.f;
            float J = r.Jp * p.iJp;
            float pdf_J = J > 1.f ? rcp(J) : J;
            float pdf_Sel = pdf_Mat * pdf_J;
            valid = valid && (rng.next_1d() < pdf_Sel);
            s.Jp = r.Jp;
            s.iJp = valid ? rcp(r.Jp) : 0.f;
            s.pos = r.ds.uv;
            s.pdf = valid ? r.ds.pdf : 0.f;
            s.pdf_lk = valid ? p.pdf * J * pdf_Sel : 0.f;
            s.valid = valid;
            bool indirect = valid, direct = valid;
            bool replace = n_indir * rng.next_1d() < 1.f;
            EPS e = bsdf_eval_pdf_sample(sc, bd.bsdf, si, si_k_wi, wo, rand_1, rand_2, valid);
            direct = direct && e.pdf > 0.f;
            s.bsdf_val = e.val;
            direct_pdf += direct ? e.pdf : 0.f;
            n_direct += (float) direct;
            indirect = indirect && e.bs.type == bsdf_sample.type;
            if (indirect && replace) bsdf_sample.wo = e.bs.wo;
            n_indir += (float) indirect;
            s.indirect = indirect;
        }
        direct_pdf /= n_direct;
    }

    /* mis_weights (mvpath_multi.h:466-523) */
    void mis_weights(SampleData *S, const BSDFData &bd) const {
        for (uint32_t k = 0; k < G; ++k) {
            SampleData &s = S[k];
            bool nf = k > 0;
            float pdfSum = s.pdf_lk;
            if (nf) pdfSum += s.pdf;
            bool cond = nf ? s.valid : bd.reuse;
            float add;
            if (cond && !bd.diffuse) {
                float acc = 0.f;
                for (uint32_t j = 1; j < G; ++j) {
                    if (j == k) continue;
                    const SampleData &sj = S[j];
                    float pdf_J = fminf_(sqr(sj.Jp * s.iJp), 1.f);
                    float pdf_Mat = P.fast_mis ? tv_pdf_fast(sj.wo_r, s.wi, s.pdfM, bd, sj.valid)
                                               : tv_pdf(sj.wo_r, s.wi, s.pdfM, bd, sj.valid);
                    acc = fmadd(sj.pdf, pdf_J * pdf_Mat, acc);
                }
                add = acc;
            } else {
                float acc = 0.f;
                for (uint32_t j = 1; j < G; ++j) {
                    if (j == k) continue;
                    const SampleData &sj = S[j];
                    float pdf_J = fminf_(sqr(sj.Jp * s.iJp), 1.f);
                    acc = fmadd(sj.pdf, pdf_J, acc);
                }
                add = cond ? acc : 0.f;
            }
            pdfSum += add;
            s.weight = s.pdf_lk / pdfSum;
        }
    }

    /* sample_multi (mvpath_multi.h:130-369) -> (valid_ray, adapt_mask) */
    std::pair<bool, bool> sample_multi(PCG32 &rng, SampleData *S, const Ray &p_ray, uint64_t &verts) {
        bool adapt_mask = false;
        if (P.max_depth == 0) return {false, adapt_mask};
        SampleData &p = S[0];
        bool valid_ray = !P.hide_emitters && sc.environment >= 0;   /* mvpath_multi.h:140 */
        ++verts;
        SI si = intersect(sc, p_ray);
        bool p_hit = si.valid();
        int em = si_emitter(sc, si);
        bool direct_em = em >= 0;
        if (direct_em) p.result = emitter_eval(sc, em, si, true);
        int b = p_hit ? sc.shapes[si.shape].bsdf : -1;
        bool bsdf_smooth = (bsdf_flags(sc, b) & F_Smooth) != 0;
        bool active_em = p_hit && bsdf_smooth;
        V2 es{rng.next_1d(), 0.f}; es.y = rng.next_1d();
        auto [ds, em_weight] = sample_emitter_direction(sc, si, es, active_em);
        active_em = active_em && ds.pdf != 0.f;
        V3 wo = si.to_local(ds.d);
        float rand_1 = rng.next_1d();
        V2 rand_2{rng.next_1d(), 0.f}; rand_2.y = rng.next_1d();
        EPS e = bsdf_eval_pdf_sample(sc, b, si, si.wi, wo, rand_1, rand_2, true);
        Spec bsdf_val = e.val;
        float direct_pdf = e.pdf;
        BSample bsdf_sample = e.bs;
        Spec bsdf_weight = e.weight;
        bool flag_delta = (bsdf_sample.type & F_Delta) != 0, flag_null = (bsdf_sample.type & F_Null) != 0;
        bool flag_diff = (bsdf_sample.type & F_Diffuse) != 0;
        bool delta = flag_delta || flag_null, not_delta = !delta, p_not_delta = not_delta && p_hit;
        bool reuse = !direct_em && p_not_delta && bsdf_smooth;
        if (reuse) stat_reuse++;
        bool should_reuse = G > 1;  /* JIT: any_or<true>(reuse) */
        bool should_mis = P.sa_mis && should_reuse;
        if (should_mis) {
            BSDFData bd;
            bd.bsdf = b;
            bd.alpha = bsdf_eval_roughness(sc, b, si.wi, true);
            bd.sqr_a = fmsub(bd.alpha, bd.alpha, 1.f);
            bd.rsqrt_a = rsqrt(bd.alpha);
            bd.diffuse = flag_diff;
            bd.reuse = reuse;
            p.bsdf_val = bsdf_val;
            camera_selection(rng, S, si, bd, wo, rand_1, rand_2, p_hit, bsdf_sample, direct_pdf);
            mis_weights(S, bd);
        } else if (should_reuse) {
            p.valid = p_hit;
            bool p_face = si.wi.z > 0.f;
            for (uint32_t k = 1; k < G; ++k) {
                SurfSample r = sensors_visible(false, si, p_face, S[k].idx, reuse, true);
                S[k].pos = r.ds.uv;
                S[k].valid = r.valid;
            }
        }
        /* emitter sampling contribution */
        {
            float mis_em = ds.delta ? 1.f : mis_weight(ds.pdf, direct_pdf);
            Spec emis_mis = em_weight * mis_em;
            if (should_mis) {
                for (uint32_t k = 0; k < G; ++k)
                    if (active_em && S[k].valid) S[k].result = spec_fma(S[k].bsdf_val, emis_mis, S[k].result);
            } else {
                if (active_em) p.result = spec_fma(bsdf_val, emis_mis, p.result);
            }
        }
        /* BSDF sampling */
        Ray pd_ray = spawn_ray(si.p, si.n, si.to_world(bsdf_sample.wo));
        if (should_mis) {
            float n_indir = 0.f, pdf = 0.f;
            for (uint32_t k = 0; k < G; ++k) {
                SampleData &s = S[k];
                bool valid = s.indirect;
                EvalPdf ep = bsdf_eval_pdf(sc, b, CTX_ALL, si, s.wi, bsdf_sample.wo, valid);
                Spec bv = ep.val;
                float bp = ep.pdf;
                if (k == 0) {
                    bv = p_not_delta ? bv : bsdf_weight;
                    bp = p_not_delta ? bp : bsdf_sample.pdf;
                    valid = valid && (bp > 0.f || delta);
                }
                bool pvalid = bp > 0.f;
                valid = valid && ((k == 0) ? (pvalid || delta) : pvalid);
                bp = valid ? bp : 0.f;
                s.bsdf_val = valid ? bv : sp(0.f);
                pdf += bp;
                n_indir += (float) valid;
                s.indirect = s.indirect && valid;
            }
            bsdf_sample.pdf = p_not_delta ? pdf / n_indir : bsdf_sample.pdf;
            adapt_mask = p_hit && !flag_null && (n_indir <= 1.f);
        }
        Spec thr = should_mis ? sp(1.f) : bsdf_weight;
        valid_ray = valid_ray || (p_hit && !flag_null);
        bool pd_active = p_hit;
        if (!should_mis) pd_active = pd_active && (smax(thr) != 0.f);
        auto [indirect, valid] = sample_suffix(rng, pd_ray, thr, bsdf_sample.eta, (uint32_t) p_hit, si,
                                               bsdf_sample.pdf, flag_delta, pd_active, verts);
        valid_ray = valid_ray || valid;
        if (should_mis) {
            float pdfW = p_not_delta ? rcp(bsdf_sample.pdf) : 1.f;
            for (uint32_t k = 0; k < G; ++k) {
                SampleData &s = S[k];
                if (s.indirect) s.result = spec_fma(s.bsdf_val * pdfW, indirect, s.result);
            }
        } else {
            p.result = p.result + indirect;
            p.weight = 1.f;
            if (should_reuse)
                for (uint32_t k = 1; k < G; ++k) { S[k].weight = 1.f; S[k].result = p.result; }
        }
        p.weight = p_hit ? p.weight : 1.f;
        p.valid = true;
        return {valid_ray, adapt_mask};
    }

    void splat(const Film &film, V2 pos, Spec v, float alpha, float weight, bool active, bool coalesce) const {
        float values[5] = {v.r, v.g, v.b, 0.f, 0.f};
        if (film.C == 4) values[3] = weight;
        else { values[3] = alpha; values[4] = weight; }
        film.put(pos, values, active, coalesce);
    }
};

bool build_scene(const amvpt_scene_desc *d, Scene &sc) {
    sc.bsdfs.assign(d->bsdfs, d->bsdfs + d->bsdf_count);
    sc.emitters.assign(d->emitters, d->emitters + d->emitter_count);
    sc.emitter_pmf = sc.emitters.empty() ? 0.f : 1.f / (float) sc.emitters.size();
    /* Scene::update_emitter_sampling_distribution (scene.cpp:100-119) */
    for (auto &e : sc.emitters) sc.distr = sc.distr || e.sampling_weight != 1.f;
    if (sc.distr) {
        float acc = 0.f;
        for (auto &e : sc.emitters) { acc += e.sampling_weight; sc.cdf.push_back(acc); }
        sc.distr_sum = sc.cdf.back();
        sc.distr_norm = rcp(sc.distr_sum);
    }
    for (uint32_t i = 0; i < d->emitter_count; ++i)
        if (d->emitters[i].type == AMVPT_EMITTER_CONSTANT) sc.environment = (int) i;
    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        Shape sh;
        sh.type = s.type; sh.bsdf = s.bsdf; sh.emitter = s.emitter; sh.flip = s.flip_normals != 0;
        std::memcpy(sh.to_world, s.to_world, sizeof(sh.to_world));
        std::memcpy(sh.to_object, s.to_object, sizeof(sh.to_object));
        sh.inv_area = 0.f;
        if (s.type == AMVPT_SHAPE_RECTANGLE) {
            /* Rectangle::update (rectangle.cpp:112-123) */
            V3 dp_du = xform_vector(sh.to_world, v3(2.f, 0.f, 0.f));
            V3 dp_dv = xform_vector(sh.to_world, v3(0.f, 2.f, 0.f));
            V3 nn = normalize(xform_normal_inv(sh.to_object, v3(0.f, 0.f, 1.f)));
            sh.frame = Frame{dp_du, dp_dv, nn};
            sh.inv_area = rcp(norm(cross(sh.frame.s, sh.frame.t)));
            sc.prims.push_back({AMVPT_SHAPE_RECTANGLE, i, 0});
        } else if (s.type == AMVPT_SHAPE_MESH) {
            sh.pos.assign(s.positions, s.positions + 3 * s.vertex_count);
            if (s.normals) sh.nrm.assign(s.normals, s.normals + 3 * s.vertex_count);
            if (s.texcoords) sh.uv.assign(s.texcoords, s.texcoords + 2 * s.vertex_count);
            sh.faces.assign(s.faces, s.faces + 3 * s.face_count);
            float acc = 0.f;
            for (uint32_t f = 0; f < s.face_count; ++f) {
                V3 p0 = vtx(sh, sh.faces[3 * f]), p1 = vtx(sh, sh.faces[3 * f + 1]), p2 = vtx(sh, sh.faces[3 * f + 2]);
                const float a = .5f * norm(cross(p1 - p0, p2 - p0)); /* mesh.cpp:470 */
                acc += a;
                sh.area_pmf.push_back(a);
                sh.area_cdf.push_back(acc);
            }
            sh.area_sum = acc;
            sh.inv_area = acc != 0.f ? 1.f / acc : 0.f;
            for (uint32_t f = 0; f < s.face_count; ++f) sc.prims.push_back({AMVPT_SHAPE_MESH, i, f});
        } else {
            std::memcpy(sh.center, s.center, sizeof(sh.center));
            sh.radius = s.radius;
            sh.inv_area = rcp((4.f * Pi) * sqr(s.radius));
            sc.prims.push_back({AMVPT_SHAPE_SPHERE, i, 0});
        }
        sc.shapes.push_back(std::move(sh));
    }
    if (g_use_bvh && sc.prims.size() > 64) build_bvh(sc);
    if (sc.environment >= 0) {
        /* ConstantBackgroundEmitter::set_scene (constant.cpp:73-88): the bounding sphere of the scene's
         * bounding box (union of Shape::bbox: rectangle corners rectangle.cpp bbox(), mesh vertices,
         * sphere center -+ radius), radius enlarged by (1 + RayEpsilon) */
        V3 lo{Infinity, Infinity, Infinity}, hi{-Infinity, -Infinity, -Infinity};
        bool any = false;
        auto expand = [&](V3 p) {
            lo = {std::min(lo.x, p.x), std::min(lo.y, p.y), std::min(lo.z, p.z)};
            hi = {std::max(hi.x, p.x), std::max(hi.y, p.y), std::max(hi.z, p.z)};
            any = true;
        };
        for (const Shape &sh : sc.shapes) {
            if (sh.type == AMVPT_SHAPE_RECTANGLE) {
                expand(xform_point_affine(sh.to_world, v3(-1.f, -1.f, 0.f)));
                expand(xform_point_affine(sh.to_world, v3(1.f, -1.f, 0.f)));
                expand(xform_point_affine(sh.to_world, v3(1.f, 1.f, 0.f)));
                expand(xform_point_affine(sh.to_world, v3(-1.f, 1.f, 0.f)));
            } else if (sh.type == AMVPT_SHAPE_MESH) {
                for (size_t v = 0; v + 2 < sh.pos.size(); v += 3) expand(v3(sh.pos[v], sh.pos[v + 1], sh.pos[v + 2]));
            } else {
                expand(v3(sh.center[0] - sh.radius, sh.center[1] - sh.radius, sh.center[2] - sh.radius));
                expand(v3(sh.center[0] + sh.radius, sh.center[1] + sh.radius, sh.center[2] + sh.radius));
            }
        }
        if (any) {
            sc.bs_center = (hi + lo) * .5f;
            sc.bs_radius = norm(sc.bs_center - hi);
            sc.bs_radius = std::max(RayEpsilon, sc.bs_radius * (1.f + RayEpsilon));
        } else {
            sc.bs_center = v3(0.f, 0.f, 0.f);
            sc.bs_radius = RayEpsilon;
        }
    }
    return true;
}

/* render plan (mvpath.cpp:32-41,133-147; integrator.cpp for `path`) */
static void plan(const amvpt_params &P, uint32_t &spp, uint32_t &spp_pp, uint32_t &n_passes, uint64_t &L) {
    uint32_t s = P.spp ? P.spp : 1;
    uint64_t px = (uint64_t) P.film_width * P.film_height;
    if (P.integrator == AMVPT_INTEGRATOR_MVPATH) {
        spp_pp = P.spp_pass_lim ? std::min(P.spp_pass_lim, s) : s;
        n_passes = s / spp_pp;
        s = n_passes * spp_pp;
    } else {
        /* SamplingIntegrator::render (integrator.cpp:137-146): samples_per_pass (spp_pass_lim here,
         * 0 = unset); the host refuses an spp it does not divide */
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

/* group size rule (mvpath.cpp:192-217) */
static uint32_t group_size(const amvpt_params &P, bool reuse) {
    uint32_t N = P.n_views;
    uint32_t G = reuse ? P.reuse_count : 1;
    G = std::min(G, N);
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

} // namespace

/* ====================================================================== */
/* Exported C API (test infrastructure)                                    */
/* ====================================================================== */
extern "C" {

typedef int (*oracle_exchange_fn)(void *ctx, uint64_t local, uint64_t *prefix, uint64_t *total);
static oracle_exchange_fn g_exchange = nullptr;
static void *g_exchange_ctx = nullptr;
/* adaptive fill over a lane range: per pass, (local flagged-lane count) -> (prefix, total) */
void oracle_set_exchange(oracle_exchange_fn fn, void *ctx) { g_exchange = fn; g_exchange_ctx = ctx; }
/* the same over the runs of a lane rectangle (amvpt_run_exchange_fn of include/amvpt.h): per pass,
 * (run lane begins, run flagged counts) -> (flagged lanes of the pass below each run, pass total) */
typedef int (*oracle_run_exchange_fn)(void *ctx, uint32_t n_runs, const uint64_t *run_lane_begin,
                                      const uint64_t *run_count, uint64_t *run_prefix, uint64_t *total);
static oracle_run_exchange_fn g_run_exchange = nullptr;
static void *g_run_exchange_ctx = nullptr;
void oracle_set_run_exchange(oracle_run_exchange_fn fn, void *ctx) { g_run_exchange = fn; g_run_exchange_ctx = ctx; }

struct oracle_stats { uint64_t lanes, vertices, reuse_lanes, visibility_rays, adaptive_lanes; double seconds; uint64_t range_drops; };
/* the device's deterministic film (AMVPT_OPT_DETERMINISTIC) restated: 32.32 fixed-point cell sums, resolved
 * into the f32 film once at the end (k_fixed_resolve); 0: the f32 film of ImageBlock::put */
static bool g_fixed_film = false;
void oracle_set_fixed_film(int on) { g_fixed_film = on != 0; }
/* closest-hit / any-hit queries through a BVH instead of the brute-force scans (scenes of more than 64 primitives):
 * the same hits by the (t, index) rule -- bench.py's CPU baseline on the mesh config; the parity tests keep it off */
void oracle_set_bvh(int on) { g_use_bvh = on != 0; }

/*
 * Render [lane_begin, lane_end) of every pass into `film` (host memory, H*W*C
 * floats, accumulated).  `records` (optional): per-lane per-view splat records
 * of pass `record_pass` (8 floats: pos.x, pos.y, r, g, b, alpha, weight, valid)
 * laid out [lane - lane_begin][view slot].  Returns 0 on success.
 */
/* the lanes of a render: contiguous [lane_begin, lane_end), or (rect) the lanes of the quilt pixels
 * [x0, x0 + w) x [y0, y0 + h) -- virtual index v -> lane, runs of w * spp_per_pass lanes per row */
struct LaneMap {
    bool rect = false;
    uint32_t x0 = 0, y0 = 0, w = 0, h = 0;
};
static int render_core(const amvpt_scene_desc *sd, const amvpt_view_desc *views, const amvpt_params *params,
                       uint64_t lane_begin, uint64_t lane_end, const LaneMap &lm, float *film, int n_threads,
                       float *records, uint32_t record_pass, oracle_stats *stats);

int oracle_render(const amvpt_scene_desc *sd, const amvpt_view_desc *views, const amvpt_params *params,
                  uint64_t lane_begin, uint64_t lane_end, float *film, int n_threads,
                  float *records, uint32_t record_pass, oracle_stats *stats) {
    return render_core(sd, views, params, lane_begin, lane_end, LaneMap{}, film, n_threads, records, record_pass, stats);
}

/* the lanes of a pixel rectangle of the quilt (a view-group rank's share, amvpt_lane_set rect form) */
int oracle_render_rect(const amvpt_scene_desc *sd, const amvpt_view_desc *views, const amvpt_params *params,
                       uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float *film, int n_threads, oracle_stats *stats) {
    LaneMap lm;
    lm.rect = true;
    lm.x0 = x0; lm.y0 = y0; lm.w = w; lm.h = h;
    if ((uint64_t) x0 + w > params->film_width || (uint64_t) y0 + h > params->film_height) return 4;
    return render_core(sd, views, params, 0, 0, lm, film, n_threads, nullptr, 0, stats);
}

static int render_core(const amvpt_scene_desc *sd, const amvpt_view_desc *views, const amvpt_params *params,
                       uint64_t lane_begin, uint64_t lane_end, const LaneMap &lm, float *film, int n_threads,
                       float *records, uint32_t record_pass, oracle_stats *stats) {
    auto t0 = std::chrono::steady_clock::now();
    Scene sc;
    if (!build_scene(sd, sc)) return 4;
    for (auto &e : sc.emitters)
        if (e.type == AMVPT_EMITTER_AREA && sc.shapes[e.shape].type == AMVPT_SHAPE_MESH &&
            !(sc.shapes[e.shape].area_sum > 0.f))
            return 4; /* Mesh::build_pmf: "no probability mass found" */
    amvpt_params P = *params;
    uint32_t spp, spp_pp, n_passes;
    uint64_t L;
    plan(P, spp, spp_pp, n_passes, L);
    bool is_mv = P.integrator == AMVPT_INTEGRATOR_MVPATH;
    bool reuse = is_mv && P.sa_reuse && P.n_views > 1 && P.reuse_count != 1;
    uint32_t G = reuse ? group_size(P, true) : 1;
    uint32_t C = P.film_alpha ? 5 : 4;
    uint32_t W = P.film_width, H = P.film_height;
    if (lm.rect) { lane_begin = 0; lane_end = (uint64_t) lm.w * lm.h * spp_pp; }   /* virtual indices */
    else if (lane_end > L) lane_end = L;
    if (lane_begin >= lane_end) lane_begin = lane_end;
    const uint64_t run_len = (uint64_t) lm.w * spp_pp;
    auto lane_of = [&](uint64_t v) -> uint64_t {
        if (!lm.rect) return v;
        const uint64_t r = v / run_len;
        return ((uint64_t) (lm.y0 + r) * P.film_width + lm.x0) * spp_pp + (v - r * run_len);
    };
    uint32_t log_spp = 0;
    while ((1u << log_spp) < spp_pp) ++log_spp;
    bool pow2 = (1u << log_spp) == spp_pp;
    bool coalesce_single = spp_pp >= 4;
    uint32_t gx = P.grid_x ? P.grid_x : 1, gy = P.grid_y ? P.grid_y : 1;
    /* tile pitch of reprojected views: film->size() / grid (mvpath_multi.h:62), the full film */
    const uint32_t fullW = P.full_width ? P.full_width : W, fullH = P.full_height ? P.full_height : H;
    uint32_t sres_x = fullW / gx, sres_y = fullH / gy;
    const int ox = (int) P.crop_offset_x, oy = (int) P.crop_offset_y;
    /* render_multisample / render_sample: scale = 1 / crop_size, offset = -crop_offset * scale */
    const float scale_x = 1.f / (float) W, scale_y = 1.f / (float) H;
    const float off_x = -(float) ox * scale_x, off_y = -(float) oy * scale_y;
    uint32_t n_adapt = std::min(P.adaptive, G - 1);
    /* stock path over several passes (integrator.cpp:279-330): the sampler is seeded once, every pass
     * continues each lane's PCG32 stream where the previous pass left it (advance() only moves the
     * sample index, which the independent sampler does not read) */
    const bool carry = !is_mv && n_passes > 1;
    if (carry && (lm.rect || spp % spp_pp)) return 4;
    std::vector<uint64_t> carried(carry ? lane_end - lane_begin : 0);
    const bool partial = lm.rect || lane_begin != 0 || lane_end != L;
    if (n_adapt && partial && !(lm.rect ? (bool) g_run_exchange : (bool) g_exchange))
        return 4; /* adaptive needs the full frame or a count exchange */
    if (n_threads <= 0) n_threads = (int) std::max(1u, std::thread::hardware_concurrency());

    std::atomic<uint64_t> a_vert{0}, a_reuse{0}, a_vis{0}, a_adapt{0};
    std::vector<std::vector<float>> films(n_threads);
    const bool fixed = g_fixed_film;
    std::vector<std::vector<int64_t>> fxs(fixed ? n_threads : 0);
    std::vector<uint64_t> drops(n_threads, 0);

    for (uint32_t pass = 0; pass < n_passes; ++pass) {
        uint32_t seed_value = P.base_seed + (is_mv ? (spp_pp * pass + P.seed) : P.seed);
        uint64_t span = lane_end - lane_begin;
        std::vector<uint8_t> amask(n_adapt ? L : 0, 0);
        std::vector<float> spos(n_adapt ? 2 * L : 0, 0.f), sap(n_adapt ? 2 * L : 0, .5f);
        auto worker = [&](int tid) {
            std::vector<float> &tf = films[tid];
            if (tf.empty()) tf.assign((size_t) W * H * C, 0.f);
            Film film{W, H, C, P.rfilter == AMVPT_RFILTER_BOX, {}, tf.data(), ox, oy};
            film.g.init(P.rfilter_stddev);
            if (fixed) {
                if (fxs[tid].empty()) fxs[tid].assign((size_t) W * H * C, 0);
                film.fx = fxs[tid].data();
                film.drops = &drops[tid];
            }
            Renderer R(sc, views, P);
            R.G = G;
            uint64_t verts = 0;
            uint64_t b0 = lane_begin + span * tid / n_threads, b1 = lane_begin + span * (tid + 1) / n_threads;
            std::vector<SampleData> S(G);
            for (uint64_t vi = b0; vi < b1; ++vi) {
                const uint64_t lane = lane_of(vi);
                uint32_t idx32 = (uint32_t) lane;
                uint32_t pix = pow2 ? (idx32 >> log_spp) : (idx32 / spp_pp);
                int py = (int) (pix / W);
                int px = (int) (pix - W * (uint32_t) py);
                px += ox;   /* pos += film->crop_offset() (mvpath.cpp:190) */
                py += oy;
                uint32_t v0, v1;
                tea(seed_value, idx32, 4, v0, v1);
                PCG32 rng;
                rng.seed(v0, v1);
                if (carry && pass > 0) rng.state = carried[vi - lane_begin];
                V2 jit{rng.next_1d(), 0.f};
                jit.y = rng.next_1d();
                V2 sample_pos{(float) px + jit.x, (float) py + jit.y};
                R.ap = V2{.5f, .5f};
                if (R.needs_ap) { R.ap.x = rng.next_1d(); R.ap.y = rng.next_1d(); }
                V2 adj{fmadd(sample_pos.x, scale_x, off_x), fmadd(sample_pos.y, scale_y, off_y)};
                float *rec = (records && pass == record_pass) ? records + (vi - lane_begin) * (size_t) G * 8 : nullptr;
                if (!reuse) {
                    /* render_sample (mvpath_single.h:50-80) / SamplingIntegrator::render_sample */
                    uint32_t index;
                    Ray ray = R.sample_ray_idx(adj, index);
                    auto [spec, valid] = R.sample_single(rng, ray, verts);
                    if (carry) carried[vi - lane_begin] = rng.state;
                    float alpha = valid ? 1.f : 0.f;
                    /* SamplingIntegrator::render_sample puts at the integer pixel under a box filter */
                    V2 put_pos = (!is_mv && film.box) ? V2{(float) px, (float) py} : sample_pos;
                    R.splat(film, put_pos, spec, alpha, 1.f, true, coalesce_single);
                    if (rec) {
                        float r8[8] = {sample_pos.x, sample_pos.y, spec.r, spec.g, spec.b, alpha, 1.f, 1.f};
                        std::memcpy(rec, r8, sizeof(r8));
                    }
                    continue;
                }
                /* render_multisample (mvpath_multi.h:8-116) */
                uint32_t p_idx;
                Ray ray = R.sample_ray_idx(adj, p_idx);
                uint32_t max_idx = G * (p_idx / G + 1u);
                for (uint32_t s = 0; s < G; ++s) {
                    S[s] = SampleData();
                    uint32_t id = p_idx + s;
                    S[s].idx = id < max_idx ? id : id - G;
                }
                S[0].pos = sample_pos;
                auto [valid_ray, adapt_mask] = R.sample_multi(rng, S.data(), ray, verts);
                float alpha = valid_ray ? 1.f : 0.f;
                float adapt_w = 1.f / (float) (n_adapt + 1);
                if (P.debug) {
                    R.splat(film, S[0].pos, sp(adapt_mask ? 1.f : 0.f), alpha, 1.f, true, true);
                    continue;
                } else if (n_adapt) {
                    if (adapt_mask) S[0].weight = S[0].weight * adapt_w;
                    amask[lane] = adapt_mask;
                    spos[2 * lane] = sample_pos.x;
                    spos[2 * lane + 1] = sample_pos.y;
                    if (R.needs_ap) { sap[2 * lane] = R.ap.x; sap[2 * lane + 1] = R.ap.y; }
                }
                for (uint32_t i = 0; i < G; ++i) {
                    SampleData &s = S[i];
                    if (i > 0) {
                        uint32_t y = s.idx / gx, x = s.idx - y * gx;
                        if (P.reverse_x) x = (gx - 1) - x;
                        if (P.reverse_y) y = (gy - 1) - y;
                        s.pos.x += (float) (x * sres_x);
                        s.pos.y += (float) (y * sres_y);
                    }
                    Spec v = {s.weight * s.result.r, s.weight * s.result.g, s.weight * s.result.b};
                    R.splat(film, s.pos, v, alpha, s.weight, s.valid, i == 0);
                    if (rec) {
                        float r8[8] = {s.pos.x, s.pos.y, v.r, v.g, v.b, alpha, s.weight, s.valid ? 1.f : 0.f};
                        std::memcpy(rec + i * 8, r8, sizeof(r8));
                    }
                }
            }
            a_vert += verts;
            a_reuse += R.stat_reuse;
            a_vis += R.stat_vis;
        };
        std::vector<std::thread> th;
        for (int t = 0; t < n_threads; ++t) th.emplace_back(worker, t);
        for (auto &t : th) t.join();

        if (n_adapt) {
            /* adaptive fill (mvpath_multi.h:79-115): compress + repeat, new sampler seeded (W, W) */
            std::vector<uint32_t> idx;
            std::vector<uint64_t> run_count(lm.rect ? lm.h : 1, 0);
            for (uint64_t v = lane_begin; v < lane_end; ++v) {
                const uint64_t l = lane_of(v);
                if (amask[l]) {
                    for (uint32_t r = 0; r < n_adapt; ++r) idx.push_back((uint32_t) l);
                    run_count[lm.rect ? v / run_len : 0] += 1;
                }
            }
            uint64_t wf = idx.size();
            /* sharded frame: the fill's index space is the whole pass's compressed array, so ask
             * the other ranks how many flagged lanes precede each run of this one */
            uint64_t total = wf / n_adapt;
            std::vector<uint64_t> run_prefix(run_count.size(), 0);
            if (lm.rect) {
                std::vector<uint64_t> run_begin(lm.h);
                for (uint32_t r = 0; r < lm.h; ++r) run_begin[r] = lane_of((uint64_t) r * run_len);
                const uint32_t n_runs = lane_end > lane_begin ? lm.h : 0u;   /* an empty set still joins */
                if (g_run_exchange(g_run_exchange_ctx, n_runs, run_begin.data(), run_count.data(), run_prefix.data(), &total) != 0)
                    return 5;
            } else if (partial) {
                if (g_exchange(g_exchange_ctx, wf / n_adapt, &run_prefix[0], &total) != 0) return 5;
            }
            /* entry e of the local compressed list -> its index in the pass's compressed array */
            std::vector<uint32_t> gidx;
            for (size_t r = 0, e = 0; r < run_count.size(); ++r)
                for (uint64_t k = 0; k < run_count[r]; ++k, ++e) gidx.push_back((uint32_t) (run_prefix[r] + k));
            a_adapt += wf;
            if (wf > 0) {
                uint32_t sv = P.base_seed + (uint32_t) (total * n_adapt);
                float adapt_w = 1.f / (float) (n_adapt + 1);
                auto aworker = [&](int tid) {
                    Film film{W, H, C, P.rfilter == AMVPT_RFILTER_BOX, {}, films[tid].data(), ox, oy};
                    film.g.init(P.rfilter_stddev);
                    if (fixed) { film.fx = fxs[tid].data(); film.drops = &drops[tid]; }
                    Renderer R(sc, views, P);
                    R.G = G;
                    uint64_t verts = 0;
                    uint64_t b0 = wf * tid / n_threads, b1 = wf * (tid + 1) / n_threads;
                    for (uint64_t j = b0; j < b1; ++j) {
                        uint32_t v0, v1;
                        tea(sv, gidx[j / n_adapt] * n_adapt + (uint32_t) (j % n_adapt), 4, v0, v1);
                        PCG32 rng;
                        rng.seed(v0, v1);
                        uint32_t lane = idx[j];
                        V2 sample_pos{spos[2 * lane], spos[2 * lane + 1]};
                        R.ap = V2{sap[2 * lane], sap[2 * lane + 1]};   /* nested_gather(aperture_sample, idx) */
                        V2 adj{fmadd(sample_pos.x, scale_x, off_x), fmadd(sample_pos.y, scale_y, off_y)};
                        uint32_t index;
                        Ray ray = R.sample_ray_idx(adj, index);
                        auto [spec, valid] = R.sample_single(rng, ray, verts);
                        (void) valid;
                        Spec v = {adapt_w * spec.r, adapt_w * spec.g, adapt_w * spec.b};
                        R.splat(film, sample_pos, v, 1.f, adapt_w, true, false);
                    }
                    a_vert += verts;
                };
                std::vector<std::thread> th2;
                for (int t = 0; t < n_threads; ++t) th2.emplace_back(aworker, t);
                for (auto &t : th2) t.join();
            }
        }
    }
    size_t n = (size_t) W * H * C;
    if (fixed) {
        /* integer sums (order-free), then the device's k_fixed_resolve conversion */
        std::vector<uint64_t> tot(n, 0);
        for (int t = 0; t < n_threads; ++t)
            if (!fxs[t].empty())
                for (size_t i = 0; i < n; ++i) tot[i] += (uint64_t) fxs[t][i];
        for (size_t i = 0; i < n; ++i) film[i] += (float) ((double) (int64_t) tot[i] * (1.0 / 4294967296.0));
    } else {
        for (int t = 0; t < n_threads; ++t)
            if (!films[t].empty())
                for (size_t i = 0; i < n; ++i) film[i] += films[t][i];
    }
    if (stats) {
        stats->lanes = (lane_end - lane_begin) * (uint64_t) n_passes;
        stats->vertices = a_vert;
        stats->reuse_lanes = a_reuse;
        stats->visibility_rays = a_vis;
        stats->adaptive_lanes = a_adapt;
        stats->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        stats->range_drops = 0;
        for (uint64_t d : drops) stats->range_drops += d;
    }
    return 0;
}

/*
 * Test hook (the unbiasedness gate's geometric edge mask): the primary hit through the centre of every
 * quilt pixel -- sample_ray_idx at (x + .5, y + .5) / quilt size, closest hit -- as 8 floats per
 * pixel: shape index (-1 for a miss), geometric normal, hit point, view index.  Scene geometry only;
 * no sampling.
 */
int oracle_primary_hits(const amvpt_scene_desc *sd, const amvpt_view_desc *views, const amvpt_params *params,
                        float *out) {
    Scene sc;
    if (!build_scene(sd, sc)) return 4;
    const amvpt_params P = *params;
    Renderer R(sc, views, P);
    const uint32_t W = P.film_width, H = P.film_height;
    const float sx = 1.f / (float) W, sy = 1.f / (float) H;
    const float ox = -(float) P.crop_offset_x * sx, oy = -(float) P.crop_offset_y * sy;
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            /* crop pixel (x, y) = film pixel + crop offset, mapped as render_sample maps it */
            const V2 adj{fmadd((float) (x + P.crop_offset_x) + .5f, sx, ox), fmadd((float) (y + P.crop_offset_y) + .5f, sy, oy)};
            uint32_t index = 0;
            const Ray ray = R.sample_ray_idx(adj, index);
            const SI si = intersect(sc, ray);
            float *o = out + ((size_t) y * W + x) * 8;
            o[0] = si.valid() ? (float) si.shape : -1.f;
            o[1] = si.n.x; o[2] = si.n.y; o[3] = si.n.z;
            o[4] = si.p.x; o[5] = si.p.y; o[6] = si.p.z;
            o[7] = (float) index;
        }
    return 0;
}

int oracle_plan(const amvpt_params *p, uint32_t *spp, uint32_t *spp_pp, uint32_t *n_passes, uint64_t *L, uint32_t *G) {
    plan(*p, *spp, *spp_pp, *n_passes, *L);
    bool is_mv = p->integrator == AMVPT_INTEGRATOR_MVPATH;
    bool reuse = is_mv && p->sa_reuse && p->n_views > 1 && p->reuse_count != 1;
    *G = reuse ? group_size(*p, true) : 1;
    return 0;
}

/* ---- known-answer hooks for the golden tests ---- */
void oracle_tea(uint32_t v0, uint32_t v1, int rounds, uint32_t *o0, uint32_t *o1) { tea(v0, v1, rounds, *o0, *o1); }
float oracle_tea_float32(uint32_t v0, uint32_t v1, int rounds) {
    uint32_t a, b;
    tea(v0, v1, rounds, a, b);
    return u2f((b >> 9) | 0x3f800000u) - 1.f;
}
double oracle_tea_float64(uint32_t v0, uint32_t v1, int rounds) {
    uint32_t a, b;
    tea(v0, v1, rounds, a, b);
    uint64_t u = (uint64_t) a + ((uint64_t) b << 32);
    uint64_t bits = (u >> 12) | 0x3ff0000000000000ull;
    double d;
    std::memcpy(&d, &bits, 8);
    return d - 1.0;
}
void oracle_pcg32_u32(uint64_t initstate, uint64_t initseq, uint32_t n, uint32_t *out) {
    PCG32 r;
    r.seed(initstate, initseq);
    for (uint32_t i = 0; i < n; ++i) out[i] = r.next_u32();
}
void oracle_sampler_1d(uint32_t seed_value, uint32_t lane, uint32_t n, float *out) {
    uint32_t v0, v1;
    tea(seed_value, lane, 4, v0, v1);
    PCG32 r;
    r.seed(v0, v1);
    for (uint32_t i = 0; i < n; ++i) out[i] = r.next_1d();
}
float oracle_gaussian_eval(float stddev, float x) { Gaussian g; g.init(stddev); return g.eval(x); }
void oracle_sincos(float x, float *s, float *c) { sincos_(x, *s, *c); }
/* the Beckmann path's transcendentals (oracle_math.h), checked against libm by the CPU tests */
void oracle_math(uint32_t fn, const float *x, float *y, uint32_t n) {
    for (uint32_t i = 0; i < n; ++i)
        y[i] = fn == 0 ? exp_(x[i]) : fn == 1 ? log_(x[i]) : fn == 2 ? erf_(x[i]) : fn == 3 ? erfinv_(x[i]) : tan_(x[i]);
}
void oracle_square_to_cosine_hemisphere(float u, float v, float *out) {
    V3 r = square_to_cosine_hemisphere({u, v});
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
void oracle_square_to_uniform_disk_concentric(float u, float v, float *out) {
    V2 r = square_to_uniform_disk_concentric({u, v});
    out[0] = r.x; out[1] = r.y;
}
/* diffuse eval/pdf for wi/wo in local frame (test_diffuse.py) */
void oracle_diffuse_eval_pdf(const float *refl, const float *wi, const float *wo, float *val3, float *pdf) {
    Scene sc;
    amvpt_bsdf_desc d{};
    d.type = AMVPT_BSDF_DIFFUSE;
    std::memcpy(d.reflectance, refl, 12);
    sc.bsdfs.push_back(d);
    SI si;
    EvalPdf e = bsdf_eval_pdf(sc, 0, CTX_ALL, si, v3(wi[0], wi[1], wi[2]), v3(wo[0], wo[1], wo[2]), true);
    val3[0] = e.val.r; val3[1] = e.val.g; val3[2] = e.val.b; *pdf = e.pdf;
}
/* microfacet distribution KAT hooks (test_microfacet.py) */
float oracle_microfacet_eval(uint32_t type, float au, float av, const float *m) {
    amvpt_bsdf_desc d{}; d.distribution = type; d.alpha_u = au; d.alpha_v = av; d.sample_visible = 1;
    return Microfacet(d).eval(v3(m[0], m[1], m[2]));
}
float oracle_microfacet_smith_g1(uint32_t type, float au, float av, const float *v, const float *m) {
    amvpt_bsdf_desc d{}; d.distribution = type; d.alpha_u = au; d.alpha_v = av; d.sample_visible = 1;
    return Microfacet(d).smith_g1(v3(v[0], v[1], v[2]), v3(m[0], m[1], m[2]));
}
float oracle_microfacet_pdf(uint32_t type, float au, float av, uint32_t visible, const float *wi, const float *m) {
    amvpt_bsdf_desc d{}; d.distribution = type; d.alpha_u = au; d.alpha_v = av; d.sample_visible = visible;
    Microfacet mf(d);
    V3 w = v3(wi[0], wi[1], wi[2]), mm = v3(m[0], m[1], m[2]);
    float r = mf.eval(mm);
    if (mf.visible) r *= mf.smith_g1(w, mm) * absdot(w, mm) / w.z;
    else r *= mm.z;
    return r;
}
void oracle_microfacet_sample(uint32_t type, float au, float av, uint32_t visible, const float *wi, float u, float v,
                              float *m_out, float *pdf) {
    amvpt_bsdf_desc d{}; d.distribution = type; d.alpha_u = au; d.alpha_v = av; d.sample_visible = visible;
    V3 m;
    Microfacet(d).sample(v3(wi[0], wi[1], wi[2]), {u, v}, m, *pdf);
    m_out[0] = m.x; m_out[1] = m.y; m_out[2] = m.z;
}
float oracle_fresnel_conductor(float ci, float er, float ei) { return fresnel_conductor(ci, er, ei); }
/* ImageBlock::put of one sample into a W x H x C film (test_imageblock.py) */
void oracle_film_put(uint32_t W, uint32_t H, uint32_t C, uint32_t box, float stddev, float *data, float x, float y,
                     const float *values, uint32_t coalesce) {
    Film f;
    f.W = W; f.H = H; f.C = C; f.box = box != 0; f.data = data;
    if (!f.box) f.g.init(stddev);
    f.put({x, y}, values, true, coalesce != 0);
}

} // extern "C"
