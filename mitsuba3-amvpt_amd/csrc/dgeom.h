/*
 * dgeom.h -- ray/primitive intersection, BVH traversal and surface
 * interactions on gfx950.
 *
 * Closest hit = minimum (t, BVH primitive index); BVH boxes are built with a
 * relative outward pad so that the box test never culls a primitive whose hit
 * distance is <= the current best.  The hit record is therefore the same as a
 * brute-force scan and independent of traversal order.
 *
 * Reference (file:line): Rectangle ray_intersect_preliminary / SI
 * src/shapes/rectangle.cpp:447-563; Mesh SI src/render/mesh.cpp:1393-1560 and
 * moeller_trumbore include/mitsuba/render/mesh.h:467-488; Sphere
 * src/shapes/sphere.cpp:460-718; finalize/initialize_sh_frame
 * include/mitsuba/render/interaction.h:278-288,497-517; spawn_ray*
 * interaction.h:140-169.
 */
#pragma once
#include <type_traits>
#include "dmath.h"
#include "dscene.h"

namespace amvpt {

struct Ray { f3 o, d; float maxt; };
AD f3 ray_at(const Ray &r, float t) { return fma3(r.d, t, r.o); }

/* Scene tables as seen by a kernel; nodes/prims may point into LDS. */
struct SceneRef {
    const DNode *nodes;       /* LDS copy when staged, else global */
    const DPrim *prims;
    const DNode *gnodes;      /* global tables (scalar loads on the wave-uniform path) */
    const DPrim *gprims;
    const DScene *g;
    uint32_t n_nodes;
    uint32_t oct_stride;      /* per-lane walks: octant copy o of the nodes at nodes + o * oct_stride (0: one copy) */
    bool uniform;             /* small BVH: the kernels run their kUni = true instance (see trace_closest) */
    const DNode *tnodes;      /* LDS treelet of the first node ordering (stage_scene kTree), t_n nodes; 0: none */
    uint32_t t_n;
    const DNode *onodes;      /* LDS treelets of the 8 octant orderings (stage_scene kOct), o_n nodes each; 0: none */
    uint32_t o_n;
    bool lds_bvh;             /* nodes / prims are the block's LDS copy (stage_scene), else device memory */
    /* brute-force walks: box meshes screened per lane (DScene::boxes, box_walk) and the other primitives;
     * n_boxes = 0: scan gprims[] (no boxes, or AMVPT_OPT_NO_BOX_SCREEN) */
    const DBox *boxes;
    const DPrim *box_prims;
    const DPrim *loose_prims;
    uint32_t n_boxes, n_loose, n_loose_rect, n_loose_tri;
    bool box_lds;             /* box_prims points into the block's LDS (stage_scene stage_boxes) */
    /* BVH scenes: rectangles kept out of the BVH (DScene::outer), tested by every walk before its BVH */
    const DPrim *outer;
    uint32_t n_outer;
    /* the two-box BVH (DScene::nodes2) and this thread's LDS stack for its walks (trace_closest2 / trace_any2):
     * entry k at stk[k * kStk2Stride]; null: none */
    const DNode2 *nodes2;
    uint32_t *stk;
};
constexpr uint32_t kStk2Stride = 256;   /* the suffix walks' block size: entry k of every thread's stack in one row */


struct Hit { float t, u, v; int32_t prim; };
constexpr uint32_t kNoEnd = 0xffffffffu;   /* treelet walks: the portal's subtree end, not read yet */

AD bool rect_hit(const DPrim &p, const Ray &r, float &t, float &lx, float &ly) {
    /* to_object.transform_affine(ray) then plane z=0 (rectangle.cpp:447-467) */
    f3 o = {fmadd(p.a[2], r.o.z, fmadd(p.a[1], r.o.y, fmadd(p.a[0], r.o.x, p.a[3]))),
            fmadd(p.b[2], r.o.z, fmadd(p.b[1], r.o.y, fmadd(p.b[0], r.o.x, p.b[3]))),
            fmadd(p.c[2], r.o.z, fmadd(p.c[1], r.o.y, fmadd(p.c[0], r.o.x, p.c[3])))};
    f3 d = {fmadd(p.a[2], r.d.z, fmadd(p.a[1], r.d.y, p.a[0] * r.d.x)),
            fmadd(p.b[2], r.d.z, fmadd(p.b[1], r.d.y, p.b[0] * r.d.x)),
            fmadd(p.c[2], r.d.z, fmadd(p.c[1], r.d.y, p.c[0] * r.d.x))};
    t = -o.z / d.z;
    f3 local = fma3(d, t, o);
    lx = local.x; ly = local.y;
    return t >= 0.f && t <= r.maxt && fabs_(local.x) <= 1.f && fabs_(local.y) <= 1.f;
}

/*
 * Does rect_hit certainly miss (for an any-hit segment)?  With the object-space o.z and d.z formed exactly as
 * rect_hit forms them, rect_hit's t = -o.z / d.z (correctly rounded) is negative when o.z and d.z are nonzero
 * with the same sign, and exceeds maxt when |o.z| > maxt |d.z| (1 + 2^-20) -- the quotient then exceeds
 * maxt (1 + 2^-21) before rounding, so its rounded value does too.  Zero or NaN operands never count as a miss.
 */
#ifndef AMVPT_RECT_CULL
#define AMVPT_RECT_CULL 1   /* brute_any skips rectangles its wave certainly misses (A/B) */
#endif
AD bool rect_plane_miss(const DPrim &p, const Ray &r) {
    const float oz = fmadd(p.c[2], r.o.z, fmadd(p.c[1], r.o.y, fmadd(p.c[0], r.o.x, p.c[3])));
    const float dz = fmadd(p.c[2], r.d.z, fmadd(p.c[1], r.d.y, p.c[0] * r.d.x));
    const bool nz = oz != 0.f && dz != 0.f && oz == oz && dz == dz;
    const bool behind = (fbits(oz) >> 31) == (fbits(dz) >> 31);
    const bool beyond = fabs_(oz) > (r.maxt * fabs_(dz)) * (1.f + 0x1p-20f);
    return nz && (behind || beyond);
}
AD bool tri_hit(const DPrim &p, const Ray &r, float &t, float &u, float &v) {
    const f3 p0 = ld3(p.a), e1 = ld3(p.b), e2 = ld3(p.c);   /* edges precomputed by the host */
    f3 pvec = cross(r.d, e2);
    float inv_det = rcp(dot(e1, pvec));
    f3 tvec = r.o - p0;
    u = dot(tvec, pvec) * inv_det;
    bool active = u >= 0.f && u <= 1.f;
    f3 qvec = cross(tvec, e1);
    v = dot(r.d, qvec) * inv_det;
    active = active && v >= 0.f && u + v <= 1.f;
    t = dot(e2, qvec) * inv_det;
    return active && t >= 0.f && t <= r.maxt;
}

/*
 * Packed intersection tests: two (primitive, ray) tests of one primitive type with their arithmetic in
 * v_pk_* pairs -- two primitives against one ray (AMVPT_PAIR_PRIMS) or one primitive against two rays
 * (AMVPT_PAIR_RAYS, the two visibility rays per lane of k_vis).  Element e performs exactly rect_hit's /
 * tri_hit's IEEE operations in the same order (packed FMA, multiply, add and subtract are per-element IEEE;
 * the divisions stay per element), so the hits, t, u and v are the same bits.
 */
typedef float f2v __attribute__((ext_vector_type(2)));
AD f2v fma2(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
struct Hit2 { bool h[2]; float t[2], u[2], v[2]; };
struct PrimPair { f2v a[4], b[4], c[4]; };
struct RayPair { f2v ox, oy, oz, dx, dy, dz; float maxt[2]; };
AD PrimPair prim_pair(const DPrim &p, const DPrim &q) {
    PrimPair o;
#pragma unroll
    for (int k = 0; k < 4; ++k) { o.a[k] = f2v{p.a[k], q.a[k]}; o.b[k] = f2v{p.b[k], q.b[k]}; o.c[k] = f2v{p.c[k], q.c[k]}; }
    return o;
}
AD PrimPair prim_pair(const DPrim &p) {
    PrimPair o;
#pragma unroll
    for (int k = 0; k < 4; ++k) { o.a[k] = (f2v) p.a[k]; o.b[k] = (f2v) p.b[k]; o.c[k] = (f2v) p.c[k]; }
    return o;
}
AD RayPair ray_pair(const Ray &r) {
    return RayPair{(f2v) r.o.x, (f2v) r.o.y, (f2v) r.o.z, (f2v) r.d.x, (f2v) r.d.y, (f2v) r.d.z, {r.maxt, r.maxt}};
}
AD RayPair ray_pair(const Ray &r0, const Ray &r1) {
    return RayPair{f2v{r0.o.x, r1.o.x}, f2v{r0.o.y, r1.o.y}, f2v{r0.o.z, r1.o.z},
                   f2v{r0.d.x, r1.d.x}, f2v{r0.d.y, r1.d.y}, f2v{r0.d.z, r1.d.z}, {r0.maxt, r1.maxt}};
}
AD Hit2 rect_hit2(const PrimPair &P, const RayPair &R) {
    const f2v lox = fma2(P.a[2], R.oz, fma2(P.a[1], R.oy, fma2(P.a[0], R.ox, P.a[3])));
    const f2v loy = fma2(P.b[2], R.oz, fma2(P.b[1], R.oy, fma2(P.b[0], R.ox, P.b[3])));
    const f2v loz = fma2(P.c[2], R.oz, fma2(P.c[1], R.oy, fma2(P.c[0], R.ox, P.c[3])));
    const f2v ldx = fma2(P.a[2], R.dz, fma2(P.a[1], R.dy, P.a[0] * R.dx));
    const f2v ldy = fma2(P.b[2], R.dz, fma2(P.b[1], R.dy, P.b[0] * R.dx));
    const f2v ldz = fma2(P.c[2], R.dz, fma2(P.c[1], R.dy, P.c[0] * R.dx));
    Hit2 o;
#pragma unroll
    for (int e = 0; e < 2; ++e) o.t[e] = -loz[e] / ldz[e];
    /* the local hit point (lx = fma(dx, t, ox) per element) */
    const f2v tt = {o.t[0], o.t[1]};
    const f2v lx = fma2(ldx, tt, lox), ly = fma2(ldy, tt, loy);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        o.u[e] = lx[e];
        o.v[e] = ly[e];
        o.h[e] = o.t[e] >= 0.f && o.t[e] <= R.maxt[e] && fabs_(lx[e]) <= 1.f && fabs_(ly[e]) <= 1.f;
    }
    return o;
}
AD Hit2 tri_hit2(const PrimPair &P, const RayPair &R) {
    /* p0 = a, e1 = b, e2 = c; pvec = cross(d, e2) with fmsub(a, b, c) = fma(a, b, -c) */
    const f2v pvx = fma2(R.dy, P.c[2], -(R.dz * P.c[1])), pvy = fma2(R.dz, P.c[0], -(R.dx * P.c[2])),
              pvz = fma2(R.dx, P.c[1], -(R.dy * P.c[0]));
    const f2v det = fma2(P.b[2], pvz, fma2(P.b[1], pvy, P.b[0] * pvx));
    f2v inv;
    inv[0] = 1.0f / det[0];
    inv[1] = 1.0f / det[1];
    const f2v tvx = R.ox - P.a[0], tvy = R.oy - P.a[1], tvz = R.oz - P.a[2];
    const f2v u = fma2(tvz, pvz, fma2(tvy, pvy, tvx * pvx)) * inv;
    const f2v qx = fma2(tvy, P.b[2], -(tvz * P.b[1])), qy = fma2(tvz, P.b[0], -(tvx * P.b[2])),
              qz = fma2(tvx, P.b[1], -(tvy * P.b[0]));
    const f2v v = fma2(R.dz, qz, fma2(R.dy, qy, R.dx * qx)) * inv;
    const f2v t = fma2(P.c[2], qz, fma2(P.c[1], qy, P.c[0] * qx)) * inv;
    const f2v uv = u + v;
    Hit2 o;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        o.t[e] = t[e]; o.u[e] = u[e]; o.v[e] = v[e];
        o.h[e] = u[e] >= 0.f && u[e] <= 1.f && v[e] >= 0.f && uv[e] <= 1.f && t[e] >= 0.f && t[e] <= R.maxt[e];
    }
    return o;
}

/*
 * f32 screen in front of the float64 sphere test (AMVPT_SPHERE_SCREEN): false only when the exact test
 * cannot hit, so a dropped ray returns what the exact test would (no hit, t = inf) and the results are the
 * same bits; NaN keeps the ray.
 * Line: the exact test hits only if its discriminant B^2 - 4AC >= 0, i.e. (up to f64 rounding, ~1e-16
 * relative) only if the line through pp (the f32 point o + d * plane_t) along d passes within r of the
 * center; pp lies within eps <= 8u (|o| + |l|) of the ray's own line (u = 2^-24, l = o - c).  Here
 * h^2 |d|^2 = |l x d|^2 -- the cross-product form, whose f32 error near h = r is <~ 8u |l| r |d|^2 (no
 * cancellation of |l|^2 terms) -- and the ray is dropped only if h^2 > R2 = r^2 (1 + 1e-5) +
 * 2e-5 r s + 4e-12 s^2 (s = sqrt(2 (|o|^2 + |l|^2)) >= |o| + |l|): over 10x the error and eps terms.
 * Segment (AMVPT_SPHERE_SCREEN 2): the sphere of radius^2 R2 meets the line over the parameters tc -+ th
 * (tc = -l.d / |d|^2, th = sqrt(R2 - h^2) / |d|), which contain the exact test's entry and exit parameters
 * (plane_t + x0 / x1) up to errors below m = 2e-5 (|tc| + |l| / |d|); the ray is dropped when that range
 * lies beyond [0, maxt] by m.  A shadow ray toward a point on a sphere light stops ShadowEpsilon ~ 9e-4 of
 * its length short of it (spawn_ray_to), so the target light's own exact test is dropped too.
 */
#ifndef AMVPT_SPHERE_SCREEN
#define AMVPT_SPHERE_SCREEN 2   /* 1: the line test only, 0: off (A/B) */
#endif
#ifndef AMVPT_SPHERE_DEFER
/* 1: the wave-uniform walks of scenes with <= 64 spheres and the brute-force walks defer the float64 tests
 * past the walk (kSph = 2 below, brute_closest / brute_any); 0: in place (A/B) */
#define AMVPT_SPHERE_DEFER 1
#endif
AD bool sphere_maybe(const DPrim &p, const Ray &ray) {
    const float lx = ray.o.x - p.a[0], ly = ray.o.y - p.a[1], lz = ray.o.z - p.a[2], r = p.a[3];
    const f3 d = ray.d;
    const float dd = fmadd(d.z, d.z, fmadd(d.y, d.y, d.x * d.x));
    const float ll = fmadd(lz, lz, fmadd(ly, ly, lx * lx));
    const float oo = fmadd(ray.o.z, ray.o.z, fmadd(ray.o.y, ray.o.y, ray.o.x * ray.o.x));
    const float cx = fmsub(ly, d.z, lz * d.y), cy = fmsub(lz, d.x, lx * d.z), cz = fmsub(lx, d.y, ly * d.x);
    const float E = fmadd(cz, cz, fmadd(cy, cy, cx * cx));   /* h^2 |d|^2 */
    const float sc = __builtin_amdgcn_sqrtf(2.f * (oo + ll));
    const float R2 = fmadd(r * r, 1.00001f, fmadd(2e-5f * r, sc, 4e-12f * (sc * sc)));
    if (E > dd * R2) return false;
    if (AMVPT_SPHERE_SCREEN >= 2) {
        const float ld = fmadd(lz, d.z, fmadd(ly, d.y, lx * d.x));
        const float idd = __builtin_amdgcn_rcpf(dd);
        const float tc = -ld * idd;
        const float th = __builtin_amdgcn_sqrtf(fmaxf(fmadd(dd, R2, -E), 0.f)) * idd * 1.0001f;
        const float m = 2e-5f * (fabs_(tc) + __builtin_amdgcn_sqrtf(ll * idd));
        if (tc - th > ray.maxt + m || tc + th < -m) return false;
    }
    return true;
}

/* float64 sphere test, as the llvm variants compute it (sphere.cpp:460-518) */
AD bool sphere_hit(const DPrim &p, const Ray &ray, float &t_out) {
    if (AMVPT_SPHERE_SCREEN && !sphere_maybe(p, ray)) {
        t_out = kInf;
        return false;
    }
    double cx = p.a[0], cy = p.a[1], cz = p.a[2], r = p.a[3];
    double ox = ray.o.x, oy = ray.o.y, oz = ray.o.z, dx = ray.d.x, dy = ray.d.y, dz = ray.d.z;
    double maxt = ray.maxt;
    double lx = ox - cx, ly = oy - cy, lz = oz - cz;
    double dn = __builtin_sqrt(__builtin_fma(dz, dz, __builtin_fma(dy, dy, dx * dx)));
    double plane_t = __builtin_fma(-lz, dz, __builtin_fma(-ly, dy, -lx * dx)) / dn;
    bool no_hit = plane_t == 0.0 && (ray.o.x != p.a[0] && ray.o.y != p.a[1] && ray.o.z != p.a[2]);
    f3 pp = ray_at(ray, (float) plane_t);
    double ppx = (double) pp.x - cx, ppy = (double) pp.y - cy, ppz = (double) pp.z - cz;
    no_hit = no_hit && (__builtin_sqrt(__builtin_fma(ppz, ppz, __builtin_fma(ppy, ppy, ppx * ppx))) > r);
    double A = __builtin_fma(dz, dz, __builtin_fma(dy, dy, dx * dx));
    double B = 2.0 * __builtin_fma(ppz, dz, __builtin_fma(ppy, dy, ppx * dx));
    double C = __builtin_fma(ppz, ppz, __builtin_fma(ppy, ppy, ppx * ppx)) - r * r;
    bool linear = A == 0.0, valid_linear = linear && B != 0.0;
    double x0 = -C / B, x1 = x0;
    double discrim = __builtin_fma(B, B, -(4.0 * A * C));
    bool valid_quad = !linear && discrim >= 0.0;
    {
        double sq = __builtin_sqrt(discrim);
        double temp = -0.5 * (B + __builtin_copysign(sq, B));
        double x0p = temp / A, x1p = C / temp;
        /* std::min / std::max operand order (NaN handling) as Dr.Jit evaluates them */
        double x0m = x1p < x0p ? x1p : x0p, x1m = x0p < x1p ? x1p : x0p;
        x0 = linear ? x0 : x0m;
        x1 = linear ? x0 : x1m;
    }
    bool found = valid_linear || valid_quad;
    double near_t = x0 + plane_t, far_t = x1 + plane_t;
    bool out_bounds = !(near_t <= maxt && far_t >= 0.0);
    bool in_bounds = near_t < 0.0 && far_t > maxt;
    bool active = found && !no_hit && !out_bounds && !in_bounds;
    t_out = active ? (near_t < 0.0 ? (float) far_t : (float) near_t) : kInf;
    return active;
}

AD bool prim_hit(const DPrim &p, const Ray &r, float &t, float &u, float &v) {
    if (p.type == PRIM_RECT) return rect_hit(p, r, t, u, v);
    if (p.type == PRIM_TRI) return tri_hit(p, r, t, u, v);
    u = v = 0.f;
    return sphere_hit(p, r, t);
}

/*
 * Slab test with inclusive bounds; boxes carry a relative pad from the builder (1e-4 of the
 * scene's coordinate magnitude).  The test only has to be conservative -- it decides which
 * primitives get the exact test, never a hit -- so it runs on a 1-ulp reciprocal and the fused
 * form t = lo * inv - o * inv (one rounding of o * inv: an error far below the pad in t units
 * for origins within 1000x the scene's extent); a NaN slab (0 * inf) drops out of the min/max
 * and only widens the box.  AMVPT_EXACT_BOX=1 restores (lo - o) / d (A/B).
 */
#ifndef AMVPT_EXACT_BOX
#define AMVPT_EXACT_BOX 0
#endif
struct BoxRay { f3 o, inv, oinv; };
/* per-lane walk of the suffix kernels (k_extend, k_shadow): 2 speculative while-while, 1 plain
 * while-while, 0 one loop (A/B) */
#ifndef AMVPT_WALK_WW
#define AMVPT_WALK_WW 2
#endif
/* the while-while node step's leaf bookkeeping as selects instead of nested branches (0: branches, A/B) */
#ifndef AMVPT_WALK_SEL
#define AMVPT_WALK_SEL 1
#endif
AD float box_rcp(float d) {
#if AMVPT_EXACT_BOX
    return 1.f / (d != 0.f ? d : mulsign(1e-30f, d));
#else
    return __builtin_amdgcn_rcpf(fabs_(d) >= 1e-30f ? d : mulsign(1e-30f, d));
#endif
}
AD BoxRay box_ray(const Ray &r) {
    BoxRay b;
    b.o = r.o;
    b.inv = mk(box_rcp(r.d.x), box_rcp(r.d.y), box_rcp(r.d.z));
    b.oinv = mk(r.o.x * b.inv.x, r.o.y * b.inv.y, r.o.z * b.inv.z);
    return b;
}
AD bool box_hit(const DNode &n, const BoxRay &b, float tmax) {
#if AMVPT_EXACT_BOX
    float tx0 = (n.lo[0] - b.o.x) * b.inv.x, tx1 = (n.hi[0] - b.o.x) * b.inv.x;
    float ty0 = (n.lo[1] - b.o.y) * b.inv.y, ty1 = (n.hi[1] - b.o.y) * b.inv.y;
    float tz0 = (n.lo[2] - b.o.z) * b.inv.z, tz1 = (n.hi[2] - b.o.z) * b.inv.z;
#else
    float tx0 = fmaf(n.lo[0], b.inv.x, -b.oinv.x), tx1 = fmaf(n.hi[0], b.inv.x, -b.oinv.x);
    float ty0 = fmaf(n.lo[1], b.inv.y, -b.oinv.y), ty1 = fmaf(n.hi[1], b.inv.y, -b.oinv.y);
    float tz0 = fmaf(n.lo[2], b.inv.z, -b.oinv.z), tz1 = fmaf(n.hi[2], b.inv.z, -b.oinv.z);
#endif
    float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
    float tm = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    return tmin <= tm;
}

AD uint32_t ufirst(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

/* the node array of the ray's direction octant (bit a = sign of d[a]; -0 counts as negative,
 * any order gives the same hit) */
AD const DNode *octant_nodes(const SceneRef &sc, f3 d) {
    const uint32_t o = (fbits(d.x) >> 31) | ((fbits(d.y) >> 31) << 1) | ((fbits(d.z) >> 31) << 2);
    return sc.nodes + (size_t) o * sc.oct_stride;
}

/* Scalar (s_load) reads of read-only scene records at a wave-uniform index: the
 * constant address space tells the backend the bytes are not written by the kernel. */
template <typename T> AD T load_uniform(const T *base, uint32_t idx) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(4))) const v4u cv4u;
    static_assert(sizeof(T) % 16 == 0, "16-byte records");
    constexpr int W = (int) (sizeof(T) / 16);
    const cv4u *p = (const cv4u *) (uintptr_t) base + (size_t) ufirst(idx) * W;
    T out;
    v4u *o = reinterpret_cast<v4u *>(&out);
#pragma unroll
    for (int k = 0; k < W; ++k) o[k] = p[k];
    return out;
}
AD bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0ull; }

/* Per-lane reads of 16-byte records through an explicit address space.  A treelet walk reads a node from
 * its LDS treelet or from the global array, lane by lane; through the generic SceneRef pointers the two
 * became one flat load (every node read paying the flat path, and flat loads count against both the
 * vector-memory and the LDS wait counters).  load_lds takes a generic pointer into the block's LDS (its
 * low 32 bits are the LDS offset), load_global a pointer into device memory. */
template <typename T, int AS> AD T load_as(const T *base, uint32_t idx) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(AS))) const v4u av4u;
    static_assert(sizeof(T) % 16 == 0, "16-byte records");
    constexpr int W = (int) (sizeof(T) / 16);
    const av4u *p;
    if constexpr (AS == 3) p = (const av4u *) (uint32_t) (uintptr_t) base + idx * (uint32_t) W;
    else p = (const av4u *) (uintptr_t) base + (size_t) idx * W;
    T out;
    v4u *o = reinterpret_cast<v4u *>(&out);
#pragma unroll
    for (int k = 0; k < W; ++k) o[k] = p[k];
    return out;
}
template <typename T> AD T load_lds(const T *base, uint32_t idx) { return load_as<T, 3>(base, idx); }
#ifndef AMVPT_WALK_AS
#define AMVPT_WALK_AS 1   /* per-lane walks read nodes / primitives through explicit address spaces (0: generic, A/B) */
#endif
template <typename T> AD T load_global(const T *base, uint32_t idx) { return load_as<T, 1>(base, idx); }

/* Primitive test with a wave-uniform primitive type (no divergence between shapes). */
/*
 * Spheres in the wave-uniform walks, kSph: 0 the scene has none (no float64 code in the walk: k_vis 80 -> 41
 * VGPRs), 1 tested in place, 2 deferred (scenes of <= 64 spheres): the walk only screens a sphere
 * (sphere_maybe) and, when a lane may hit it, sets the sphere's bit in a wave-uniform 64-bit mask (the
 * record's `face` field holds its ordinal, DScene::sph_prims maps it back); the float64 tests run after the
 * walk, where the walk's own registers are free -- the walk loop then allocates like a sphere-free one.
 * Hits are order-independent (any hit; closest by the (t, scene-order index) rule), so the results are the
 * same bits.
 */
template <int kSph = 1> AD bool prim_hit_u(const DPrim &p, uint32_t type, const Ray &r, float &t, float &u, float &v) {
    if (kSph < 0) return tri_hit(p, r, t, u, v);   /* a BVH of triangles only (WALK_LANE_TRI) */
    if (type == PRIM_RECT) return rect_hit(p, r, t, u, v);
    if (kSph != 1 || type == PRIM_TRI) return tri_hit(p, r, t, u, v);
    u = v = 0.f;
    return sphere_hit(p, r, t);
}
/* the k-th sphere's primitive record (a scalar load of DScene::sph_prims) */
AD DPrim deferred_sphere(const SceneRef &sc, uint32_t k) {
    typedef __attribute__((address_space(4))) const uint32_t cu32;
    return load_uniform(sc.gprims, ufirst(((cu32 *) (uintptr_t) sc.g->sph_prims)[k]));
}
AD uint32_t mask_pop(uint64_t &m) {
    const uint32_t k = (uint32_t) __builtin_ctzll(m);
    m &= m - 1ull;
    return k;
}

/*
 * Closest hit over the threaded BVH (dscene.h), no traversal stack (nothing is
 * spilled to scratch).  Ties resolve toward the lower scene-order primitive
 * index, so the hit equals a brute-force scan whatever the traversal visits.
 *
 * Small BVHs (kUni, chosen per scene by the host) are walked wave-uniformly: the wave enters a node if
 * any active lane's ray hits its box and every active lane tests the leaf's
 * primitives.  Node and primitive records are then wave-uniform scalar loads,
 * the primitive type is a uniform branch, and there is no per-lane divergence.
 * Testing a primitive for a lane whose own box test failed cannot change that
 * lane's result (its box is padded and inclusive), so both walks are exact.
 */
/*
 * The rectangles a BVH scene keeps out of its BVH (DScene::outer: a room's walls and lights, whose boxes
 * span the scene -- every ray crossing the room descended to their leaves).  Each walk tests them first,
 * wave-uniformly (scalar record loads, no divergence): the closest-hit walks start their BVH walk with the
 * nearest wall's t as the box-test bound, the any-hit walks skip a rectangle whose plane the wave's open
 * segments do not cross (rect_plane_miss) and walk the BVH only for the lanes still open.  The (t,
 * scene-order index) rule and any-hit do not depend on the order of the tests: the same hits.
 */
AD void outer_closest(const SceneRef &sc, const Ray &ray, Hit &best, uint32_t &best_orig) {
    const uint32_t n = ufirst(sc.n_outer);
    for (uint32_t j = 0; j < n; ++j) {
        const DPrim p = load_uniform(sc.outer, j);
        float t, u, v;
        if (rect_hit(p, ray, t, u, v)) {
            const uint32_t orig = ufirst(p.pad);
            if (t < best.t || (t == best.t && orig < best_orig)) {
                best.t = t; best.u = u; best.v = v; best.prim = (int32_t) (ufirst(p.type) >> 8);
                best_orig = orig;
            }
        }
    }
}
/* skip: the lane needs no test (no ray, or already found) */
AD bool outer_any(const SceneRef &sc, const Ray &ray, bool skip) {
    const uint32_t n = ufirst(sc.n_outer);
    bool found = false;
    for (uint32_t j = 0; j < n; ++j) {
        const DPrim p = load_uniform(sc.outer, j);
        if (!wave_any(!skip && !found && !rect_plane_miss(p, ray))) continue;
        float t, u, v;
        const bool h = !skip && rect_hit(p, ray, t, u, v);
        found = found || h;
    }
    return found;
}

/*
 * Closest hit over the octant treelets (per-lane walks of large BVHs): the ray's direction-octant
 * ordering starts in its LDS treelet and continues at a portal in the same ordering's global copy
 * (indices local to the copy), returning to the treelet at the end of the portal's subtree.  The node
 * sequence is the global walk's, so the hit is the same; speculative while-while as trace_closest.
 */
AD Hit trace_closest_tl(const SceneRef &sc, const Ray &ray, Hit best, uint32_t best_orig) {
    const BoxRay br = box_ray(ray);
    float tmax_box = fminf(ray.maxt, best.t);
    const uint32_t o = (fbits(ray.d.x) >> 31) | ((fbits(ray.d.y) >> 31) << 1) | ((fbits(ray.d.z) >> 31) << 2);
    const DNode *const tn = sc.onodes + (size_t) o * sc.o_n;
    const DNode *const gn = sc.gnodes + (size_t) o * sc.oct_stride;
    auto leaf_test = [&](uint32_t first, uint32_t count) {
        for (uint32_t i = 0; i < count; ++i) {
            const uint32_t pi = first + i;
            const DPrim p = load_global(sc.gprims, pi);
            float t, u, v;
            if (prim_hit(p, ray, t, u, v)) {
                if (t < best.t || (t == best.t && p.pad < best_orig)) {
                    best.t = t; best.u = u; best.v = v; best.prim = (int32_t) pi;
                    best_orig = p.pad;
                    tmax_box = t;
                }
            }
        }
    };
    const uint32_t nt = sc.o_n;
    uint32_t node = 0, gend = 0, tres = 0;
    bool glob = false;
    for (;;) {
        uint32_t lf = 0, lc = 0;
        bool stop = false;
        for (;;) {
            const bool open = glob || node < nt;
            if (!wave_any(open && lc == 0u)) break;
            if (open && !stop) {
                DNode n;
                if (glob) n = load_global(gn, node);
                else n = load_lds(tn, node);
                if (glob && gend == kNoEnd) gend = n.skip_count & kNodeSkipMask;   /* the portal's own node */
                const bool hit = box_hit(n, br, tmax_box);
                const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
                uint32_t next;
                if (hit && count) {
                    if (lc == 0u) { lf = n.first; lc = count; next = skip; }
                    else { stop = true; next = node; }
                } else if (hit && !glob && (n.first & kPortal)) {
                    tres = skip;
                    glob = true;
                    gend = kNoEnd;
                    next = n.first & ~kPortal;
                } else {
                    next = hit ? node + 1 : skip;
                }
                if (glob && next == gend) { glob = false; next = tres; }
                node = next;
            }
        }
        if (!wave_any(lc != 0u)) break;
        leaf_test(lf, lc);
    }
    return best;
}

template <bool kSph> AD bool prim_hit_b(const DPrim &p, uint32_t type, const Ray &r, float &t, float &u, float &v);
/* the per-lane walks' leaf test: kSph -1 a triangle-only BVH (no type dispatch), 0 no spheres, 1 any */
template <int kSph> AD bool prim_hit_l(const DPrim &p, const Ray &r, float &t, float &u, float &v) {
    if constexpr (kSph < 0) return tri_hit(p, r, t, u, v);
    else return prim_hit_b<kSph != 0>(p, p.type, r, t, u, v);
}
/* kSph = false (per-lane walks): the scene has no sphere, the primitive tests carry no float64 code */
template <bool kUni, int kWW = 0, int kSph = 1> AD Hit trace_closest(const SceneRef &sc, const Ray &ray) {
    Hit best{kInf, 0.f, 0.f, -1};
    uint32_t best_orig = 0xffffffffu;
    outer_closest(sc, ray, best, best_orig);
    if (!kUni && sc.o_n) return trace_closest_tl(sc, ray, best, best_orig);
    const BoxRay br = box_ray(ray);
    float tmax_box = fminf(ray.maxt, best.t);
    if (kUni) {
        const uint32_t nn = ufirst(sc.n_nodes);
        /* BVHs with direction-octant copies (large ones, walked uniformly by the coherent primary
         * rays): the copy of the first lane's octant (any copy gives the same hit) */
        const DNode *const gn = sc.oct_stride ? sc.gnodes + (size_t) ufirst(
                                    (fbits(ray.d.x) >> 31) | ((fbits(ray.d.y) >> 31) << 1) | ((fbits(ray.d.z) >> 31) << 2)) * sc.oct_stride
                                              : sc.gnodes;
        uint32_t node = 0;
        uint64_t dm = 0;   /* kSph = 2: deferred spheres */
        while (node < nn) {
            const DNode n = load_uniform(gn, node);
            const bool enter = wave_any(box_hit(n, br, tmax_box));
            const uint32_t skc = ufirst(n.skip_count);
            const uint32_t count = skc >> kNodeCountShift, skip = skc & kNodeSkipMask;
            if (enter && count) {
                const uint32_t first = ufirst(n.first);
                for (uint32_t i = 0; i < count; ++i) {
                    const uint32_t pi = first + i;
                    const DPrim p = load_uniform(sc.gprims, pi);
                    const uint32_t type = ufirst(p.type);
                    if (kSph == 2 && type == PRIM_SPHERE) {
                        if (wave_any(sphere_maybe(p, ray))) dm |= 1ull << ufirst(p.face);
                        continue;
                    }
                    float t, u, v;
                    const bool h = prim_hit_u<kSph>(p, type, ray, t, u, v);
                    const uint32_t orig = ufirst(p.pad);
                    const bool better = h && (t < best.t || (t == best.t && orig < best_orig));
                    best.t = better ? t : best.t;
                    best.u = better ? u : best.u;
                    best.v = better ? v : best.v;
                    best.prim = better ? (int32_t) pi : best.prim;
                    best_orig = better ? orig : best_orig;
                    tmax_box = better ? t : tmax_box;
                }
            }
            node = (enter && !count) ? node + 1 : skip;
        }
        if constexpr (kSph == 2) {
            while (dm) {
                const uint32_t k = mask_pop(dm);
                const DPrim p = deferred_sphere(sc, k);
                float t;
                const bool h = sphere_hit(p, ray, t);
                const uint32_t orig = ufirst(p.pad);
                const bool better = h && (t < best.t || (t == best.t && orig < best_orig));
                best.t = better ? t : best.t;
                best.u = better ? 0.f : best.u;
                best.v = better ? 0.f : best.v;
                best.prim = better ? (int32_t) ufirst(sc.g->sph_prims[k]) : best.prim;
                best_orig = better ? orig : best_orig;
            }
        }
        return best;
    }
    const DNode *const nodes = octant_nodes(sc, ray.d);
    /* kL: the BVH is staged in LDS (stage_scene), else it is read from device memory; explicit address
     * spaces (not the generic SceneRef pointers, which made every node and primitive read a flat load) */
    auto walk = [&](auto lds_tag) -> Hit {
        constexpr bool kL = decltype(lds_tag)::value;
        auto ld_node = [&](uint32_t i) {
            if (!AMVPT_WALK_AS) return nodes[i];
            return kL ? load_lds(nodes, i) : load_global(nodes, i);
        };
        auto leaf_test = [&](uint32_t first, uint32_t count) {
            for (uint32_t i = 0; i < count; ++i) {
                const uint32_t pi = first + i;
                const DPrim p = !AMVPT_WALK_AS ? sc.prims[pi] : kL ? load_lds(sc.prims, pi) : load_global(sc.prims, pi);
                float t, u, v;
                if (prim_hit_l<kSph>(p, ray, t, u, v)) {
                    if (t < best.t || (t == best.t && p.pad < best_orig)) {
                        best.t = t; best.u = u; best.v = v; best.prim = (int32_t) pi;
                        best_orig = p.pad;
                        tmax_box = t;
                    }
                }
            }
        };
        const uint32_t nn = sc.n_nodes;
        uint32_t node = 0;
        if constexpr (kWW != 0) {
        /* while-while (per-lane walks of large BVHs): the node loop runs until every lane holds a hit
         * leaf or has finished, then the wave tests its leaves together -- the primitive code runs
         * once per round for all lanes instead of once per divergent leaf visit.  kWW = 2: a lane
         * that holds a leaf keeps stepping speculatively until the others have one (it stops at a
         * second leaf and keeps it for the next round).  Incoherent rays only (the suffix walks):
         * coherent primary / visibility waves lose with it (mesh k_vis 122 -> 138 ms). */
        for (;;) {
            uint32_t lf = 0, lc = 0;
            bool stop = false;
            for (;;) {
                if (!wave_any(lc == 0u && node < nn)) break;
                if (node < nn && !stop && (kWW == 2 || lc == 0u)) {
                    const DNode n = ld_node(node);
                    const bool hit = box_hit(n, br, tmax_box);
                    const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
#if AMVPT_WALK_SEL
                    /* one branch per step: the leaf bookkeeping as selects */
                    const bool leaf = hit && count != 0u, take = leaf && lc == 0u;
                    stop = leaf && !take;   /* the second leaf: revisit it next round */
                    lf = take ? n.first : lf;
                    lc = take ? count : lc;
                    node = (hit && count == 0u) ? node + 1 : (stop ? node : skip);
#else
                    if (hit && count) {
                        if (lc == 0u) { lf = n.first; lc = count; node = skip; }
                        else stop = true;   /* the second leaf: revisit it next round */
                    } else {
                        node = hit ? node + 1 : skip;
                    }
#endif
                }
            }
            if (!wave_any(lc != 0u)) break;
            leaf_test(lf, lc);
        }
        return best;
        }
        while (node < nn) {
            const DNode n = ld_node(node);
            const bool hit = box_hit(n, br, tmax_box);
            const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
            if (hit && count) leaf_test(n.first, count);
            node = (hit && !count) ? node + 1 : skip;
        }
        return best;
    };
    return sc.lds_bvh ? walk(std::true_type{}) : walk(std::false_type{});
}

/*
 * Any-hit walks over an LDS treelet (large BVHs, DScene::tnodes): the top levels of the first node
 * ordering sit in LDS (staged per block), so the first node visits of a walk -- the ones every ray makes
 * -- are LDS reads instead of dependent loads from L2; a portal (a treelet node whose children lie below
 * the cut) continues the threaded walk in the global array at the same node, whose skip link is the end
 * of its subtree, and the walk returns to the treelet there.  The nodes tested are the same as the
 * global walk's (same boxes, same order), so the verdict is the same.
 */
AD bool trace_any_tl(const SceneRef &sc, const Ray &ray, bool found = false) {
    const BoxRay br = box_ray(ray);
    auto leaf_any = [&](uint32_t first, uint32_t count) {
        bool f = false;
        for (uint32_t i = 0; i < count && !f; ++i) {
            const DPrim p = load_global(sc.gprims, first + i);
            float t, u, v;
            f = prim_hit(p, ray, t, u, v);
        }
        return f;
    };
    const uint32_t nt = sc.t_n;
    uint32_t node = 0, gend = 0, tres = 0;
    bool glob = false;
    /* speculative while-while (trace_any kWW = 2): a lane holding a leaf steps on until the wave's
     * other lanes hold one too, and stops at a second leaf */
    for (;;) {
        uint32_t lf = 0, lc = 0;
        bool stop = false;
        for (;;) {
            const bool open = !found && (glob || node < nt);
            if (!wave_any(open && lc == 0u)) break;
            if (open && !stop) {
                DNode n;
                if (glob) n = load_global(sc.gnodes, node);
                else n = load_lds(sc.tnodes, node);
                if (glob && gend == kNoEnd) gend = n.skip_count & kNodeSkipMask;   /* the portal's own node */
                const bool hit = box_hit(n, br, ray.maxt);
                const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
                uint32_t next;
                if (hit && count) {
                    if (lc == 0u) { lf = n.first; lc = count; next = skip; }
                    else { stop = true; next = node; }   /* the second leaf: revisit it next round */
                } else if (hit && !glob && (n.first & kPortal)) {
                    tres = skip;
                    glob = true;
                    gend = kNoEnd;
                    next = n.first & ~kPortal;
                } else {
                    next = hit ? node + 1 : skip;
                }
                if (glob && next == gend) { glob = false; next = tres; }
                node = next;
            }
        }
        if (!wave_any(lc != 0u)) break;
        if (lc) found = found || leaf_any(lf, lc);
    }
    return found;
}

/* the wave-uniform any-hit walk over the treelet for one or two rays per lane (trace_any<true> /
 * trace_any2_uni): the treelet node is one LDS broadcast read per wave */
AD void trace_any_uni_tl(const SceneRef &sc, const Ray &r0, bool act0, const Ray &r1, bool act1, bool two, bool &f0,
                         bool &f1) {
    const BoxRay b0 = box_ray(r0), b1 = box_ray(r1);
    f0 = !act0;
    f1 = !act1 || !two;
    f0 = f0 || outer_any(sc, r0, f0);
    f1 = f1 || outer_any(sc, r1, f1);
    const uint32_t nt = ufirst(sc.t_n);
    uint32_t t = 0, g = 0, gend = 0, tres = 0;
    bool glob = false;
    for (;;) {
        DNode n;
        if (!glob) {
            if (t >= nt) break;
            n = load_lds(sc.tnodes, t);
        } else {
            n = load_uniform(sc.gnodes, g);
            if (gend == kNoEnd) gend = ufirst(n.skip_count) & kNodeSkipMask;
        }
        const bool enter = wave_any((!f0 && box_hit(n, b0, r0.maxt)) || (!f1 && box_hit(n, b1, r1.maxt)));
        const uint32_t skc = ufirst(n.skip_count), first = ufirst(n.first);
        const uint32_t count = skc >> kNodeCountShift, skip = skc & kNodeSkipMask;
        if (enter && count) {
            for (uint32_t i = 0; i < count; ++i) {
                const DPrim p = load_uniform(sc.gprims, first + i);
                const uint32_t type = ufirst(p.type);
                float tt, u, v;
                const bool h0 = prim_hit_u(p, type, r0, tt, u, v);
                f0 = f0 || h0;
                if (two) {
                    const bool h1 = prim_hit_u(p, type, r1, tt, u, v);
                    f1 = f1 || h1;
                }
            }
            if (!wave_any(!f0 || !f1)) break;
        }
        if (enter && !count && !glob && (first & kPortal)) {
            tres = skip;
            glob = true;
            gend = kNoEnd;
            g = first & ~kPortal;
            continue;
        }
        const uint32_t cur = glob ? g : t;
        const uint32_t next = (enter && !count) ? cur + 1 : skip;
        if (glob) {
            if (next == gend) { glob = false; t = tres; }
            else g = next;
        } else {
            t = next;
        }
    }
    f0 = f0 && act0;
    f1 = f1 && act1 && two;
}

/* Any hit in [0, maxt] (Scene::ray_test); same two walks as trace_closest. */
template <bool kUni, int kWW = 0, int kSph = 1> AD bool trace_any(const SceneRef &sc, const Ray &ray) {
    if (sc.t_n) {
        if (kUni) {
            bool f0, f1;
            trace_any_uni_tl(sc, ray, true, ray, false, false, f0, f1);
            return f0;
        }
        return trace_any_tl(sc, ray, outer_any(sc, ray, false));
    }
    const BoxRay br = box_ray(ray);
    const bool outer_found = outer_any(sc, ray, false);
    if (kUni) {
        const uint32_t nn = ufirst(sc.n_nodes);
        bool found = outer_found;
        uint32_t node = 0;
        uint64_t dm = 0;   /* kSph = 2: deferred spheres */
        while (node < nn) {
            const DNode n = load_uniform(sc.gnodes, node);
            const bool enter = wave_any(!found && box_hit(n, br, ray.maxt));
            const uint32_t skc = ufirst(n.skip_count);
            const uint32_t count = skc >> kNodeCountShift, skip = skc & kNodeSkipMask;
            if (enter && count) {
                const uint32_t first = ufirst(n.first);
                for (uint32_t i = 0; i < count; ++i) {
                    const DPrim p = load_uniform(sc.gprims, first + i);
                    const uint32_t type = ufirst(p.type);
                    if (kSph == 2 && type == PRIM_SPHERE) {
                        if (wave_any(!found && sphere_maybe(p, ray))) dm |= 1ull << ufirst(p.face);
                        continue;
                    }
                    float t, u, v;
                    const bool h = prim_hit_u<kSph>(p, type, ray, t, u, v);
                    found = found || h;
                }
                if (!wave_any(!found)) break;
            }
            node = (enter && !count) ? node + 1 : skip;
        }
        if constexpr (kSph == 2) {
            while (dm && wave_any(!found)) {
                const DPrim p = deferred_sphere(sc, mask_pop(dm));
                float t;
                const bool h = !found && sphere_hit(p, ray, t);
                found = found || h;
            }
        }
        return found;
    }
    /* the first ordering: an any-hit walk gains nothing from near-first order (an unoccluded
     * ray visits every box it crosses either way) and one copy keeps the cache footprint small
     * (k_shadow on the 3.6 k-triangle mesh: 280 ms with it, 301 ms with the octant copies).
     * kL: LDS-staged BVH, else device memory (explicit address spaces, see trace_closest) */
    auto walk = [&](auto lds_tag) -> bool {
        constexpr bool kL = decltype(lds_tag)::value;
        auto ld_node = [&](uint32_t i) {
            if (!AMVPT_WALK_AS) return sc.nodes[i];
            return kL ? load_lds(sc.nodes, i) : load_global(sc.nodes, i);
        };
        auto leaf_any = [&](uint32_t first, uint32_t count) {
            bool f = false;
            for (uint32_t i = 0; i < count && !f; ++i) {
                const DPrim p = !AMVPT_WALK_AS ? sc.prims[first + i]
                                : kL ? load_lds(sc.prims, first + i) : load_global(sc.prims, first + i);
                float t, u, v;
                f = prim_hit_l<kSph>(p, ray, t, u, v);
            }
            return f;
        };
        const uint32_t nn = sc.n_nodes;
        uint32_t node = 0;
        if constexpr (kWW != 0) {
        bool found = outer_found;
        for (;;) {
            uint32_t lf = 0, lc = 0;
            bool stop = false;
            for (;;) {
                if (!wave_any(!found && lc == 0u && node < nn)) break;
                if (!found && node < nn && !stop && (kWW == 2 || lc == 0u)) {
                    const DNode n = ld_node(node);
                    const bool hit = box_hit(n, br, ray.maxt);
                    const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
#if AMVPT_WALK_SEL
                    const bool leaf = hit && count != 0u, take = leaf && lc == 0u;
                    stop = leaf && !take;
                    lf = take ? n.first : lf;
                    lc = take ? count : lc;
                    node = (hit && count == 0u) ? node + 1 : (stop ? node : skip);
#else
                    if (hit && count) {
                        if (lc == 0u) { lf = n.first; lc = count; node = skip; }
                        else stop = true;
                    } else {
                        node = hit ? node + 1 : skip;
                    }
#endif
                }
            }
            if (!wave_any(lc != 0u)) break;
            if (lc) found = found || leaf_any(lf, lc);
        }
        return found;
        }
        if (outer_found) return true;
        while (node < nn) {
            const DNode n = ld_node(node);
            const bool hit = box_hit(n, br, ray.maxt);
            const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
            if (hit && count && leaf_any(n.first, count)) return true;
            node = (hit && !count) ? node + 1 : skip;
        }
        return false;
    };
    return sc.lds_bvh ? walk(std::true_type{}) : walk(std::false_type{});
}

/*
 * Walks of the two-box BVH (dscene.h DNode2; round 6), per lane, for the suffix rays of large
 * BVHs.  A node holds both children's boxes, so the walk loads a node only when it enters it -- one dependent load
 * per inner node entered, where the threaded walk loads every node it TESTS (both children of each node entered)
 * -- and orders the children by the ray's own entry distances, nearer first, the farther one on a per-lane stack of
 * kStack2 entries in LDS (entry k of thread t at stk[k * kStk2Stride + t]: the lanes of a wave hit distinct banks
 * whatever their stack depths).  The host builds the tree only when it is at most kStack2 inner nodes deep, so
 * the stack never overflows (a walk pushes at most one entry per inner node on its path).  Leaves are references
 * in their parent; a leaf reached is held and tested in the speculative while-while rounds of the threaded walks
 * (the wave tests its lanes' leaves together; a lane holding one keeps stepping until it meets a second).  The
 * boxes are the threaded tree's padded ones, tested with box_hit's operations; the primitives, their tests and
 * the (t, scene-order index) rule are the same, so the hits and verdicts are the same bits.
 */
AD bool box2_hit(const float *b, const BoxRay &br, float tmax, float &tmin_out) {
    const float tx0 = fmaf(b[0], br.inv.x, -br.oinv.x), tx1 = fmaf(b[3], br.inv.x, -br.oinv.x);
    const float ty0 = fmaf(b[1], br.inv.y, -br.oinv.y), ty1 = fmaf(b[4], br.inv.y, -br.oinv.y);
    const float tz0 = fmaf(b[2], br.inv.z, -br.oinv.z), tz1 = fmaf(b[5], br.inv.z, -br.oinv.z);
    const float tmin = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.f));
    const float tm = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    tmin_out = tmin;
    return tmin <= tm;
}
AD uint32_t stk_load(const uint32_t *stk, uint32_t k) {
    typedef __attribute__((address_space(3))) const uint32_t lu32;
    return ((lu32 *) (uint32_t) (uintptr_t) stk)[k * kStk2Stride];
}
AD void stk_store(uint32_t *stk, uint32_t k, uint32_t v) {
    typedef __attribute__((address_space(3))) uint32_t lu32;
    ((lu32 *) (uint32_t) (uintptr_t) stk)[k * kStk2Stride] = v;
}
constexpr uint32_t kRef2End = 0x7fffffffu;   /* no node (an inner index never reaches it) */
/* the 32-B float16 nodes (dscene.h DNode2h) instead of the 64-B float ones: half the bytes per node step (A/B) */
#ifndef AMVPT_TRI_LOAD48
#define AMVPT_TRI_LOAD48 1   /* the two-box walks of triangle-only BVHs load 48 / 52 B of a leaf triangle (0: 64, A/B) */
#endif
#ifndef AMVPT_BVH2_HALF
#define AMVPT_BVH2_HALF 1
#endif
AD void half2_unpack(uint32_t w, float &a, float &b) {
    a = (float) __builtin_bit_cast(_Float16, (uint16_t) (w & 0xffffu));
    b = (float) __builtin_bit_cast(_Float16, (uint16_t) (w >> 16));
}
/* the walk's ray: in the float16 nodes' normalized frame (same t: origin and direction scale together) */
AD BoxRay box2_ray(const SceneRef &sc, const Ray &r) {
    if (!AMVPT_BVH2_HALF) return box_ray(r);
    const DScene &S = *sc.g;
    const float s = S.n2_scale;
    const Ray q{mk((r.o.x - S.n2_center[0]) * s, (r.o.y - S.n2_center[1]) * s, (r.o.z - S.n2_center[2]) * s),
                mk(r.d.x * s, r.d.y * s, r.d.z * s), r.maxt};
    return box_ray(q);
}
/* one step of a two-box walk at inner node `cur`: enter the nearer hit child, stack the farther one */
AD uint32_t node2_step(const SceneRef &sc, uint32_t cur, const BoxRay &br, float tmax, uint32_t &sp) {
    float bx[12];
    uint32_t r0, r1;
    if (AMVPT_BVH2_HALF) {
        const DNode2h n = load_global(sc.g->nodes2h, cur);
#pragma unroll
        for (int w = 0; w < 6; ++w) half2_unpack(n.h[w], bx[2 * w], bx[2 * w + 1]);
        r0 = n.ref[0]; r1 = n.ref[1];
    } else {
        const DNode2 n = load_global(sc.nodes2, cur);
#pragma unroll
        for (int k = 0; k < 12; ++k) bx[k] = n.b[k];
        r0 = n.ref[0]; r1 = n.ref[1];
    }
    float t0, t1;
    const bool h0 = box2_hit(bx, br, tmax, t0), h1 = box2_hit(bx + 6, br, tmax, t1);
    const bool sw = h1 && (!h0 || t1 < t0);
    const uint32_t a = sw ? r1 : r0, b = sw ? r0 : r1;
    if (h0 && h1) stk_store(sc.stk, sp++, b);
    if (h0 || h1) return a;
    return sp ? stk_load(sc.stk, --sp) : kRef2End;
}
/* a leaf primitive of the two-box walks: a triangle-only BVH (kSph < 0) reads the record's three vertex vectors and
 * (closest hit: kPad) the scene-order index only -- 48 / 52 of its 64 B (the walks are bound by the bytes their
 * divergent gathers return, see above); other BVHs read the whole record */
template <int kSph, bool kPad> AD DPrim leaf_prim(const SceneRef &sc, uint32_t i) {
    if constexpr (kSph < 0 && AMVPT_TRI_LOAD48) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(1))) const v4f gv4f;
        typedef __attribute__((address_space(1))) const uint32_t gu32;
        const gv4f *q = (const gv4f *) (uintptr_t) (sc.gprims + i);
        DPrim p;
        const v4f a = q[0], b = q[1], c = q[2];
#pragma unroll
        for (int k = 0; k < 4; ++k) { p.a[k] = a[k]; p.b[k] = b[k]; p.c[k] = c[k]; }
        p.type = PRIM_TRI; p.shape = 0; p.face = 0;
        p.pad = kPad ? ((gu32 *) (uintptr_t) (sc.gprims + i))[15] : 0u;
        return p;
    } else {
        return load_global(sc.gprims, i);
    }
}
template <int kSph> AD Hit trace_closest2(const SceneRef &sc, const Ray &ray, Hit best, uint32_t best_orig) {
    const BoxRay br = box2_ray(sc, ray);
    float tmax_box = fminf(ray.maxt, best.t);
    uint32_t cur = 0, sp = 0;
    for (;;) {
        uint32_t lf = 0, lc = 0;
        bool stop = false;
        for (;;) {
            if (!wave_any(lc == 0u && cur != kRef2End)) break;
            if (cur != kRef2End && !stop) {
                if (cur & kRef2Leaf) {
                    /* a leaf: held for this round's tests, or (a second one) kept for the next round */
                    stop = lc != 0u;
                    if (!stop) {
                        lf = cur & kRef2FirstMask;
                        lc = (cur >> kRef2CountShift) & 15u;
                        cur = sp ? stk_load(sc.stk, --sp) : kRef2End;
                    }
                } else {
                    cur = node2_step(sc, cur, br, tmax_box, sp);
                }
            }
        }
        if (!wave_any(lc != 0u)) break;
        for (uint32_t i = 0; i < lc; ++i) {
            const uint32_t pi = lf + i;
            const DPrim p = leaf_prim<kSph, true>(sc, pi);
            float t, u, v;
            if (prim_hit_l<kSph>(p, ray, t, u, v)) {
                if (t < best.t || (t == best.t && p.pad < best_orig)) {
                    best.t = t; best.u = u; best.v = v; best.prim = (int32_t) pi;
                    best_orig = p.pad;
                    tmax_box = t;
                }
            }
        }
    }
    return best;
}
template <int kSph> AD bool trace_any2(const SceneRef &sc, const Ray &ray, bool found) {
    const BoxRay br = box2_ray(sc, ray);
    uint32_t cur = found ? kRef2End : 0u, sp = 0;
    for (;;) {
        uint32_t lf = 0, lc = 0;
        bool stop = false;
        for (;;) {
            if (!wave_any(lc == 0u && cur != kRef2End)) break;
            if (cur != kRef2End && !stop) {
                if (cur & kRef2Leaf) {
                    stop = lc != 0u;
                    if (!stop) {
                        lf = cur & kRef2FirstMask;
                        lc = (cur >> kRef2CountShift) & 15u;
                        cur = sp ? stk_load(sc.stk, --sp) : kRef2End;
                    }
                } else {
                    cur = node2_step(sc, cur, br, ray.maxt, sp);
                }
            }
        }
        if (!wave_any(lc != 0u)) break;
        bool f = false;
        for (uint32_t i = 0; i < lc && !f; ++i) {
            const DPrim p = leaf_prim<kSph, false>(sc, lf + i);
            float t, u, v;
            f = prim_hit_l<kSph>(p, ray, t, u, v);
        }
        if (f) { found = true; cur = kRef2End; }
    }
    return found;
}

/*
 * Two any-hit rays per lane on the wave-uniform walk (k_vis: the same view's visibility rays of
 * two adjacent 64-lane groups, near-identical paths through the tree): the wave enters a node if
 * any lane's first or second ray hits its box, so every node record is loaded and waited for
 * once per two rays.  Lanes without a ray pass act = false (they count as found).  Exact for the
 * same reason as trace_any: a primitive tested for a ray whose box test failed cannot hit it.
 */
#ifndef AMVPT_PAIR_RAYS
/* 1: trace_any2_uni tests a primitive against both rays as one packed test -- off: config-M k_vis 63.2 ->
 * 79.0 ms, C3 232 -> 284 ms (r04e; 48 B of scratch and the pair moves outweigh the packed arithmetic) */
#define AMVPT_PAIR_RAYS 0
#endif
template <int kSph = 1>
AD void trace_any2_uni(const SceneRef &sc, const Ray &r0, bool act0, const Ray &r1, bool act1, bool &f0, bool &f1) {
    if (sc.t_n) { trace_any_uni_tl(sc, r0, act0, r1, act1, true, f0, f1); return; }
    const BoxRay b0 = box_ray(r0), b1 = box_ray(r1);
    const RayPair R2 = ray_pair(r0, r1);
    const uint32_t nn = ufirst(sc.n_nodes);
    f0 = !act0; f1 = !act1;
    f0 = f0 || outer_any(sc, r0, f0);
    f1 = f1 || outer_any(sc, r1, f1);
    uint32_t node = 0;
    uint64_t dm = 0;   /* kSph = 2: deferred spheres */
    while (node < nn) {
        const DNode n = load_uniform(sc.gnodes, node);
        const bool enter = wave_any((!f0 && box_hit(n, b0, r0.maxt)) || (!f1 && box_hit(n, b1, r1.maxt)));
        const uint32_t skc = ufirst(n.skip_count);
        const uint32_t count = skc >> kNodeCountShift, skip = skc & kNodeSkipMask;
        if (enter && count) {
            const uint32_t first = ufirst(n.first);
            for (uint32_t i = 0; i < count; ++i) {
                const DPrim p = load_uniform(sc.gprims, first + i);
                const uint32_t type = ufirst(p.type);
                if (kSph == 2 && type == PRIM_SPHERE) {
                    if (wave_any((!f0 && sphere_maybe(p, r0)) || (!f1 && sphere_maybe(p, r1)))) dm |= 1ull << ufirst(p.face);
                    continue;
                }
                if (AMVPT_PAIR_RAYS && type != PRIM_SPHERE) {
                    /* both rays against the primitive as one packed test */
                    const Hit2 h = type == PRIM_RECT ? rect_hit2(prim_pair(p), R2) : tri_hit2(prim_pair(p), R2);
                    f0 = f0 || h.h[0];
                    f1 = f1 || h.h[1];
                    continue;
                }
                float t, u, v;
                const bool h0 = prim_hit_u<kSph>(p, type, r0, t, u, v);
                const bool h1 = prim_hit_u<kSph>(p, type, r1, t, u, v);
                f0 = f0 || h0;
                f1 = f1 || h1;
            }
            if (!wave_any(!f0 || !f1)) break;
        }
        node = (enter && !count) ? node + 1 : skip;
    }
    if constexpr (kSph == 2) {
        while (dm && wave_any(!f0 || !f1)) {
            const DPrim p = deferred_sphere(sc, mask_pop(dm));
            float t;
            const bool h0 = !f0 && sphere_hit(p, r0, t);
            const bool h1 = !f1 && sphere_hit(p, r1, t);
            f0 = f0 || h0;
            f1 = f1 || h1;
        }
    }
    f0 = f0 && act0;
    f1 = f1 && act1;
}

/*
 * Per-lane walks of two rays per thread (AMVPT_SHADOW_RAYS / AMVPT_EXTEND_RAYS = 2, the suffix walks of large
 * BVHs): the speculative while-while walk of trace_any / trace_closest for each ray, stepped together -- the
 * two node loads of a step are issued back to back, so a thread keeps two dependent-load chains in flight.
 * Each ray visits exactly the nodes and primitives its single walk visits, so the results are the same.
 */
struct LaneWalk { uint32_t node, lf, lc; bool stop; };
AD void lane_step(const DNode &n, const BoxRay &b, float tmax, LaneWalk &w) {
    const bool hit = box_hit(n, b, tmax);
    const uint32_t count = n.skip_count >> kNodeCountShift, skip = n.skip_count & kNodeSkipMask;
    if (hit && count) {
        if (w.lc == 0u) { w.lf = n.first; w.lc = count; w.node = skip; }
        else w.stop = true;   /* the second leaf: revisit it next round */
    } else {
        w.node = hit ? w.node + 1 : skip;
    }
}
template <int kSph = 1>
AD void trace_any_lane2(const SceneRef &sc, const Ray &r0, bool act0, const Ray &r1, bool act1, bool &f0, bool &f1) {
    const BoxRay b0 = box_ray(r0), b1 = box_ray(r1);
    auto walk = [&](auto lds_tag) {
        constexpr bool kL = decltype(lds_tag)::value;
        auto ld_node = [&](uint32_t i) { return kL ? load_lds(sc.nodes, i) : load_global(sc.nodes, i); };
        auto leaf_any = [&](const Ray &ray, uint32_t first, uint32_t count) {
            bool f = false;
            for (uint32_t i = 0; i < count && !f; ++i) {
                const DPrim p = kL ? load_lds(sc.prims, first + i) : load_global(sc.prims, first + i);
                float t, u, v;
                f = prim_hit_l<kSph>(p, ray, t, u, v);
            }
            return f;
        };
        const uint32_t nn = sc.n_nodes;
        LaneWalk w0{act0 ? 0u : nn, 0u, 0u, false}, w1{act1 ? 0u : nn, 0u, 0u, false};
        bool h0 = outer_any(sc, r0, !act0), h1 = outer_any(sc, r1, !act1);
        for (;;) {
            w0.lf = w0.lc = w1.lf = w1.lc = 0u;
            w0.stop = w1.stop = false;
            for (;;) {
                const bool need = (!h0 && w0.lc == 0u && w0.node < nn) || (!h1 && w1.lc == 0u && w1.node < nn);
                if (!wave_any(need)) break;
                const bool s0 = !h0 && w0.node < nn && !w0.stop, s1 = !h1 && w1.node < nn && !w1.stop;
                DNode n0, n1;
                if (s0) n0 = ld_node(w0.node);
                if (s1) n1 = ld_node(w1.node);
                if (s0) lane_step(n0, b0, r0.maxt, w0);
                if (s1) lane_step(n1, b1, r1.maxt, w1);
            }
            if (!wave_any(w0.lc != 0u || w1.lc != 0u)) break;
            if (w0.lc) h0 = h0 || leaf_any(r0, w0.lf, w0.lc);
            if (w1.lc) h1 = h1 || leaf_any(r1, w1.lf, w1.lc);
        }
        f0 = h0 && act0;
        f1 = h1 && act1;
    };
    if (sc.lds_bvh) walk(std::true_type{});
    else walk(std::false_type{});
}

template <int kSph = 1>
AD void trace_closest_lane2(const SceneRef &sc, const Ray &r0, bool act0, const Ray &r1, bool act1, Hit &o0, Hit &o1) {
    const BoxRay b0 = box_ray(r0), b1 = box_ray(r1);
    const DNode *const nodes0 = octant_nodes(sc, r0.d), *const nodes1 = octant_nodes(sc, r1.d);
    Hit best0{kInf, 0.f, 0.f, -1}, best1{kInf, 0.f, 0.f, -1};
    uint32_t orig0 = 0xffffffffu, orig1 = 0xffffffffu;
    outer_closest(sc, r0, best0, orig0);
    outer_closest(sc, r1, best1, orig1);
    float tmax0 = fminf(r0.maxt, best0.t), tmax1 = fminf(r1.maxt, best1.t);
    auto walk = [&](auto lds_tag) {
        constexpr bool kL = decltype(lds_tag)::value;
        auto ld_node = [&](const DNode *nodes, uint32_t i) { return kL ? load_lds(nodes, i) : load_global(nodes, i); };
        auto leaf_test = [&](const Ray &ray, uint32_t first, uint32_t count, Hit &best, uint32_t &best_orig, float &tmax) {
            for (uint32_t i = 0; i < count; ++i) {
                const uint32_t pi = first + i;
                const DPrim p = kL ? load_lds(sc.prims, pi) : load_global(sc.prims, pi);
                float t, u, v;
                if (prim_hit_l<kSph>(p, ray, t, u, v)) {
                    if (t < best.t || (t == best.t && p.pad < best_orig)) {
                        best.t = t; best.u = u; best.v = v; best.prim = (int32_t) pi;
                        best_orig = p.pad;
                        tmax = t;
                    }
                }
            }
        };
        const uint32_t nn = sc.n_nodes;
        LaneWalk w0{act0 ? 0u : nn, 0u, 0u, false}, w1{act1 ? 0u : nn, 0u, 0u, false};
        for (;;) {
            w0.lf = w0.lc = w1.lf = w1.lc = 0u;
            w0.stop = w1.stop = false;
            for (;;) {
                const bool need = (w0.lc == 0u && w0.node < nn) || (w1.lc == 0u && w1.node < nn);
                if (!wave_any(need)) break;
                const bool s0 = w0.node < nn && !w0.stop, s1 = w1.node < nn && !w1.stop;
                DNode n0, n1;
                if (s0) n0 = ld_node(nodes0, w0.node);
                if (s1) n1 = ld_node(nodes1, w1.node);
                if (s0) lane_step(n0, b0, tmax0, w0);
                if (s1) lane_step(n1, b1, tmax1, w1);
            }
            if (!wave_any(w0.lc != 0u || w1.lc != 0u)) break;
            if (w0.lc) leaf_test(r0, w0.lf, w0.lc, best0, orig0, tmax0);
            if (w1.lc) leaf_test(r1, w1.lf, w1.lc, best1, orig1, tmax1);
        }
    };
    if (sc.lds_bvh) walk(std::true_type{});
    else walk(std::false_type{});
    o0 = best0;
    o1 = best1;
}

/* trace_any2_uni for N rays per lane (AMVPT_VIS_RAYS = N > 2 in k_vis): the wave enters a node when any lane's
 * ray of any of its N hits its box -- N times the rays in flight per wave on the latency-bound walk */
template <int kSph, int N>
AD void trace_anyN_uni(const SceneRef &sc, const Ray *r, const bool *act, bool *f) {
    BoxRay b[N];
#pragma unroll
    for (int h = 0; h < N; ++h) { b[h] = box_ray(r[h]); f[h] = !act[h]; f[h] = f[h] || outer_any(sc, r[h], f[h]); }
    const uint32_t nn = ufirst(sc.n_nodes);
    uint32_t node = 0;
    uint64_t dm = 0;   /* kSph = 2: deferred spheres */
    auto open = [&]() {
        bool o = false;
#pragma unroll
        for (int h = 0; h < N; ++h) o = o || !f[h];
        return o;
    };
    while (node < nn) {
        const DNode n = load_uniform(sc.gnodes, node);
        bool hit = false;
#pragma unroll
        for (int h = 0; h < N; ++h) hit = hit || (!f[h] && box_hit(n, b[h], r[h].maxt));
        const bool enter = wave_any(hit);
        const uint32_t skc = ufirst(n.skip_count);
        const uint32_t count = skc >> kNodeCountShift, skip = skc & kNodeSkipMask;
        if (enter && count) {
            const uint32_t first = ufirst(n.first);
            for (uint32_t i = 0; i < count; ++i) {
                const DPrim p = load_uniform(sc.gprims, first + i);
                const uint32_t type = ufirst(p.type);
                if (kSph == 2 && type == PRIM_SPHERE) {
                    bool m = false;
#pragma unroll
                    for (int h = 0; h < N; ++h) m = m || (!f[h] && sphere_maybe(p, r[h]));
                    if (wave_any(m)) dm |= 1ull << ufirst(p.face);
                    continue;
                }
#pragma unroll
                for (int h = 0; h < N; ++h) {
                    float t, u, v;
                    const bool hh = prim_hit_u<kSph>(p, type, r[h], t, u, v);
                    f[h] = f[h] || hh;
                }
            }
            if (!wave_any(open())) break;
        }
        node = (enter && !count) ? node + 1 : skip;
    }
    if constexpr (kSph == 2) {
        while (dm && wave_any(open())) {
            const DPrim p = deferred_sphere(sc, mask_pop(dm));
#pragma unroll
            for (int h = 0; h < N; ++h) {
                float t;
                const bool hh = !f[h] && sphere_hit(p, r[h], t);
                f[h] = f[h] || hh;
            }
        }
    }
#pragma unroll
    for (int h = 0; h < N; ++h) f[h] = f[h] && act[h];
}

/*
 * Brute-force walks for tiny scenes (n_prims <= kBrutePrims, wave-uniform kernels only):
 * every primitive is tested in BVH order with the next record's scalar load issued
 * before the current test, so there are no dependent node loads and no box tests.
 * For incoherent rays (suffix extension / NEE) a wave enters nearly every node of a
 * Cornell-sized BVH anyway.  Same (t, scene-order index) rule -> the same hit.
 */
constexpr uint32_t kBrutePrims = 48;
/* kSph = false: the scene has no sphere (no f64 sphere code, fewer registers) */
template <bool kSph> AD bool prim_hit_b(const DPrim &p, uint32_t type, const Ray &r, float &t, float &u, float &v) {
    if (!kSph || type != PRIM_SPHERE) {
        if (type == PRIM_RECT) return rect_hit(p, r, t, u, v);
        return tri_hit(p, r, t, u, v);
    }
    u = v = 0.f;
    return sphere_hit(p, r, t);
}

/* closest-hit update of the brute-force walks: (t, scene-order index) as trace_closest.  Branchy:
 * a select per field instead measured 1-2 ms slower per config-M frame (k_suffix 133.3 vs
 * 133.7..135.2 ms, A/B r03d) */
template <bool kSph> AD void brute_test(const DPrim &p, uint32_t pi, const Ray &ray, Hit &best, uint32_t &best_orig) {
    float t, u, v;
    if (prim_hit_b<kSph>(p, ufirst(p.type), ray, t, u, v)) {
        const uint32_t orig = ufirst(p.pad);
        if (t < best.t || (t == best.t && orig < best_orig)) {
            best.t = t; best.u = u; best.v = v; best.prim = (int32_t) pi;
            best_orig = orig;
        }
    }
}
#ifndef AMVPT_PAIR_PRIMS
/* 1: the brute-force walks test two same-type primitives as one packed pair -- off: at the fused suffix's
 * 80-VGPR budget the pairs spill (240 B of scratch, k_suffix_fused<true, true, 3>) */
#define AMVPT_PAIR_PRIMS 0
#endif
/* the pair (a, b) = primitives (pi, pi + 1): one packed test when both are rectangles or both triangles */
template <bool kSph> AD void brute_pair(const DPrim &a, const DPrim &b, uint32_t pi, const Ray &ray, Hit &best,
                                        uint32_t &best_orig) {
    const uint32_t ta = ufirst(a.type), tb = ufirst(b.type);
    if (AMVPT_PAIR_PRIMS && ta == tb && ta != PRIM_SPHERE) {
        Hit2 h;
        if (ta == PRIM_RECT) h = rect_hit2(prim_pair(a, b), ray_pair(ray));
        else h = tri_hit2(prim_pair(a, b), ray_pair(ray));
        const uint32_t orig[2] = {ufirst(a.pad), ufirst(b.pad)};
#pragma unroll
        for (int e = 0; e < 2; ++e)
            if (h.h[e] && (h.t[e] < best.t || (h.t[e] == best.t && orig[e] < best_orig))) {
                best.t = h.t[e]; best.u = h.u[e]; best.v = h.v[e]; best.prim = (int32_t) (pi + e);
                best_orig = orig[e];
            }
    } else {
        brute_test<kSph>(a, pi, ray, best, best_orig);
        brute_test<kSph>(b, pi + 1, ray, best, best_orig);
    }
}
template <bool kSph> AD bool brute_pair_any(const DPrim &a, const DPrim &b, const Ray &ray) {
    const uint32_t ta = ufirst(a.type), tb = ufirst(b.type);
    if (AMVPT_PAIR_PRIMS && ta == tb && ta != PRIM_SPHERE) {
        Hit2 h;
        if (ta == PRIM_RECT) h = rect_hit2(prim_pair(a, b), ray_pair(ray));
        else h = tri_hit2(prim_pair(a, b), ray_pair(ray));
        return h.h[0] || h.h[1];
    }
    float t, u, v;
    const bool ha = prim_hit_b<kSph>(a, ta, ray, t, u, v);
    const bool hb = prim_hit_b<kSph>(b, tb, ray, t, u, v);
    return ha || hb;
}
/*
 * Box meshes in the brute-force walks (the fused suffix's instruction count).  A `cube` is 12
 * triangles, 24 of the Cornell box's 30 primitives, and a wave-uniform scan tests all of them for every ray.
 * box_walk screens each box per lane in box space ([-1, 1]^3, DBox::m): for each of the six faces the ray's
 * crossing of the face plane (an approximate reciprocal is enough) decides whether the face's two triangles
 * can report a hit at all; only those are tested -- with the exact tri_hit and the same (t, scene-order index)
 * rule as the scan, so the walk's hit is the scan's hit, bit for bit.  A face is skipped only when that is
 * certain:
 *   - the crossing point lies more than kBoxEps (box units) outside the face square -- its t lies outside
 *     one of the other two axes' slabs widened by kBoxEps -- or its t lies outside [0, maxt] by more than
 *     kBoxEpsT (1 + |t|), AND the ray is not grazing the face plane (|d_axis| >= kBoxGraze |d|_max): then
 *     tri_hit's own rounding (relative ~1e-7 / sin of the angle to the plane, below 1e-4 here) cannot move its
 *     barycentrics or t across the boundary; a NaN anywhere keeps the face;
 *   - in the closest-hit walk, its crossing t exceeds the best hit so far by more than kBoxEpsT (1 + |t|): any
 *     hit on it is farther.
 * A grazing face is always tested (first).  Lanes take their
 * candidate faces in ascending crossing order, one face (two per-lane triangle loads) per round, so a lane
 * that hits its entry face is done after one round; the wave runs until its last lane is.
 */
constexpr float kBoxEps = 1e-3f, kBoxEpsT = 1e-3f, kBoxGraze = 1e-3f;
AD void box_candidates(const DBox &B, const Ray &r, float maxt, float *key, uint32_t &cand) {
    const f3 o = mk(fmaf(B.m[2], r.o.z, fmaf(B.m[1], r.o.y, fmaf(B.m[0], r.o.x, B.m[3]))),
                    fmaf(B.m[6], r.o.z, fmaf(B.m[5], r.o.y, fmaf(B.m[4], r.o.x, B.m[7]))),
                    fmaf(B.m[10], r.o.z, fmaf(B.m[9], r.o.y, fmaf(B.m[8], r.o.x, B.m[11]))));
    const f3 d = mk(fmaf(B.m[2], r.d.z, fmaf(B.m[1], r.d.y, B.m[0] * r.d.x)),
                    fmaf(B.m[6], r.d.z, fmaf(B.m[5], r.d.y, B.m[4] * r.d.x)),
                    fmaf(B.m[10], r.d.z, fmaf(B.m[9], r.d.y, B.m[8] * r.d.x)));
    const float oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
    const float dmax = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    /* per axis: the crossings of its two face planes (t0: x = -1, t1: x = +1), and the interval of t over which
     * the ray lies within the axis's slab widened by kBoxEps ([lo, hi]; empty or unbounded for d = 0) */
    float t0[3], t1[3], lo[3], hi[3];
    bool graze[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        /* box_rcp: a zero component gives +-1e30, not inf -- with inf, (1 + eps) inf - o inf would be NaN and drop
         * the slab of a ray running parallel to it (AMVPT r05e: one lane in 37 k) */
        const float inv = box_rcp(da[a]), oi = -oa[a] * inv;
        t0[a] = fmaf(-1.f, inv, oi);
        t1[a] = fmaf(1.f, inv, oi);
        const float e0 = fmaf(-1.f - kBoxEps, inv, oi), e1 = fmaf(1.f + kBoxEps, inv, oi);
        lo[a] = fminf(e0, e1);
        hi[a] = fmaxf(e0, e1);
        graze[a] = !(fabsf(da[a]) >= kBoxGraze * dmax);
    }
    cand = 0u;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int b = (a + 1) % 3, c = (a + 2) % 3;
        /* a face's crossing lies within kBoxEps of its square iff it lies in the other two widened slabs */
        const float l = fmaxf(lo[b], lo[c]), h = fminf(hi[b], hi[c]);
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const float t = side ? t1[a] : t0[a];
            const float et = kBoxEpsT * (1.f + fabsf(t));
            const bool in_sq = !(t < l) && !(t > h) && !(t < -et) && !(t > maxt + et);
            /* a grazing face is always a candidate, tested first (its crossing's t is unreliable) */
            key[2 * a + side] = graze[a] ? -kInf : t;
            cand |= (graze[a] || in_sq) ? 1u << (2 * a + side) : 0u;
        }
    }
}
/* loose primitives [j0, j1) of one type, two records in flight (each reloaded right after its own test, as
 * brute_closest's scan) */
template <class F> AD void loose_scan(const SceneRef &sc, uint32_t j0, uint32_t j1, F test) {
    if (j0 >= j1) return;
    const uint32_t last = j1 - 1u;
    DPrim a = load_uniform(sc.loose_prims, j0), b = load_uniform(sc.loose_prims, min(j0 + 1u, last));
    for (uint32_t j = j0; j < j1; j += 2) {
        test(a);
        a = load_uniform(sc.loose_prims, min(j + 2u, last));
        if (j + 1 < j1) test(b);
        b = load_uniform(sc.loose_prims, min(j + 3u, last));
    }
}
/* kAny: any hit in [0, ray.maxt] (found); else the closest hit (best, best_orig) */
template <bool kAny>
AD void box_walk(const SceneRef &sc, const Ray &ray, Hit &best, uint32_t &best_orig, bool &found) {
    const uint32_t nb = ufirst(sc.n_boxes);
    for (uint32_t bi = 0; bi < nb; ++bi) {
        const DBox B = load_uniform(sc.boxes, bi);
        float key[6];
        uint32_t cand;
        box_candidates(B, ray, ray.maxt, key, cand);
        if (kAny && found) cand = 0u;
        const DPrim *const bt = sc.box_prims + 12u * bi;
        for (;;) {
            /* the lane's next face: the candidate with the smallest crossing */
            uint32_t k = 0u;
            float kmin = kInf;
#pragma unroll
            for (uint32_t f = 0; f < 6; ++f) {
                const bool take = ((cand >> f) & 1u) && !(key[f] >= kmin);
                kmin = take ? key[f] : kmin;
                k = take ? f : k;
            }
            bool act = cand != 0u;
            if (!kAny) act = act && !(kmin > best.t + kBoxEpsT * (1.f + fabsf(best.t)));
            if (!wave_any(act)) break;
            if (act) {
                cand &= ~(1u << k);
#pragma unroll
                for (uint32_t j = 0; j < 2; ++j) {
                    const DPrim p = sc.box_lds ? load_lds(bt, 2u * k + j) : load_global(bt, 2u * k + j);
                    float t, u, v;
                    if (tri_hit(p, ray, t, u, v)) {
                        if (kAny) {
                            found = true;
                        } else if (t < best.t || (t == best.t && p.pad < best_orig)) {
                            best.t = t; best.u = u; best.v = v; best.prim = (int32_t) (p.type >> 8);
                            best_orig = p.pad;
                        }
                    }
                }
                if (kAny && found) cand = 0u;
            }
        }
    }
}

/* Two records in flight (a, b), each reloaded in place right after its own test: the next
 * record's scalar load overlaps the current test and no record is copied between registers
 * (a one-record prefetch made the compiler move all 16 SGPRs of the record every iteration). */
/* kSph with AMVPT_SPHERE_DEFER: the float64 sphere tests run after the loop over the primitives (a brute-force
 * scene has <= kBrutePrims < 64 spheres), so the loop allocates like a sphere-free one (see prim_hit_u) */
template <bool kSph> AD Hit brute_closest(const SceneRef &sc, const Ray &ray) {
    Hit best{kInf, 0.f, 0.f, -1};
    uint32_t best_orig = 0xffffffffu;
    if (sc.n_loose) {
        /* the loose primitives (their BVH index in `type`'s upper bits) by type -- rectangles, triangles, then
         * spheres, each group with its own test (one uniform type branch per primitive let the compiler
         * if-convert both tests into every iteration) -- then the boxes */
        const uint32_t nl = ufirst(sc.n_loose), nr = ufirst(sc.n_loose_rect), nt = nr + ufirst(sc.n_loose_tri);
        uint64_t dm = 0;
        auto upd = [&](const DPrim &p, bool h, float t, float u, float v) {
            if (h) {
                const uint32_t orig = ufirst(p.pad);
                if (t < best.t || (t == best.t && orig < best_orig)) {
                    best.t = t; best.u = u; best.v = v; best.prim = (int32_t) (ufirst(p.type) >> 8);
                    best_orig = orig;
                }
            }
        };
        loose_scan(sc, 0u, nr, [&](const DPrim &p) { float t, u, v; const bool h = rect_hit(p, ray, t, u, v); upd(p, h, t, u, v); });
        loose_scan(sc, nr, nt, [&](const DPrim &p) { float t, u, v; const bool h = tri_hit(p, ray, t, u, v); upd(p, h, t, u, v); });
        if constexpr (kSph)
            for (uint32_t j = nt; j < nl; ++j) {
                const DPrim p = load_uniform(sc.loose_prims, j);
                if (wave_any(sphere_maybe(p, ray))) dm |= 1ull << ufirst(p.face);
            }
        bool found = false;
        box_walk<false>(sc, ray, best, best_orig, found);
        if constexpr (kSph) {
            while (dm) {
                const uint32_t k = mask_pop(dm);
                const DPrim p = deferred_sphere(sc, k);
                float t;
                if (sphere_hit(p, ray, t)) {
                    const uint32_t orig = ufirst(p.pad);
                    if (t < best.t || (t == best.t && orig < best_orig)) {
                        best.t = t; best.u = 0.f; best.v = 0.f; best.prim = (int32_t) ufirst(sc.g->sph_prims[k]);
                        best_orig = orig;
                    }
                }
            }
        }
        return best;
    }
    constexpr bool kDefer = kSph && AMVPT_SPHERE_DEFER && !AMVPT_PAIR_PRIMS;
    uint64_t dm = 0;
    auto test = [&](const DPrim &p, uint32_t pi) {
        if (ufirst(p.type) == PRIM_SPHERE) {
            if (wave_any(sphere_maybe(p, ray))) dm |= 1ull << ufirst(p.face);
            return;
        }
        brute_test<false>(p, pi, ray, best, best_orig);
    };
    const uint32_t np = ufirst(sc.g->n_prims);
    const uint32_t last = np - 1u;
    DPrim a = load_uniform(sc.gprims, 0), b = load_uniform(sc.gprims, min(1u, last));
    for (uint32_t pi = 0; pi < np; pi += 2) {
        /* unconditional reloads (index clamped to the table): a conditional one would merge two
         * values of the record and cost a register copy per primitive */
        if (AMVPT_PAIR_PRIMS && pi + 1 < np) {
            brute_pair<kSph>(a, b, pi, ray, best, best_orig);
            a = load_uniform(sc.gprims, min(pi + 2u, last));
            b = load_uniform(sc.gprims, min(pi + 3u, last));
            continue;
        }
        if constexpr (kDefer) {
            test(a, pi);
            a = load_uniform(sc.gprims, min(pi + 2u, last));
            if (pi + 1 < np) test(b, pi + 1);
            b = load_uniform(sc.gprims, min(pi + 3u, last));
            continue;
        }
        brute_test<kSph>(a, pi, ray, best, best_orig);
        a = load_uniform(sc.gprims, min(pi + 2u, last));
        if (pi + 1 < np) brute_test<kSph>(b, pi + 1, ray, best, best_orig);
        b = load_uniform(sc.gprims, min(pi + 3u, last));
    }
    if constexpr (kDefer) {
        while (dm) {
            const uint32_t k = mask_pop(dm);
            const DPrim p = deferred_sphere(sc, k);
            float t;
            if (sphere_hit(p, ray, t)) {
                const uint32_t orig = ufirst(p.pad);
                if (t < best.t || (t == best.t && orig < best_orig)) {
                    best.t = t; best.u = 0.f; best.v = 0.f; best.prim = (int32_t) ufirst(sc.g->sph_prims[k]);
                    best_orig = orig;
                }
            }
        }
    }
    return best;
}

/* skip: the lane has no ray (it counts as found, so the wave stops when every real ray is) */
template <bool kSph> AD bool brute_any(const SceneRef &sc, const Ray &ray, bool skip = false) {
    const uint32_t np = ufirst(sc.g->n_prims);
    bool found = skip;
    if (sc.n_loose) {
        const uint32_t nl = ufirst(sc.n_loose), nr = ufirst(sc.n_loose_rect), nt = nr + ufirst(sc.n_loose_tri);
        uint64_t dm = 0;
        loose_scan(sc, 0u, nr, [&](const DPrim &p) {
            /* a rectangle the wave's open segments certainly do not cross is skipped (rect_plane_miss: its plane
             * lies behind every origin or beyond every segment's end) -- the NEE segments of a closed room stay
             * inside it, so its walls drop out; the exact test otherwise */
            if (AMVPT_RECT_CULL && !wave_any(!found && !rect_plane_miss(p, ray))) return;
            float t, u, v;
            const bool h = rect_hit(p, ray, t, u, v);
            found = found || h;
        });
        if (!wave_any(!found)) return found;
        loose_scan(sc, nr, nt, [&](const DPrim &p) { float t, u, v; const bool h = tri_hit(p, ray, t, u, v); found = found || h; });
        if (!wave_any(!found)) return found;
        if constexpr (kSph)
            for (uint32_t j = nt; j < nl; ++j) {
                const DPrim p = load_uniform(sc.loose_prims, j);
                if (wave_any(!found && sphere_maybe(p, ray))) dm |= 1ull << ufirst(p.face);
            }
        Hit best_unused{kInf, 0.f, 0.f, -1};
        uint32_t orig_unused = 0u;
        box_walk<true>(sc, ray, best_unused, orig_unused, found);
        if constexpr (kSph) {
            while (dm && wave_any(!found)) {
                const DPrim p = deferred_sphere(sc, mask_pop(dm));
                float t;
                const bool h = !found && sphere_hit(p, ray, t);
                found = found || h;
            }
        }
        return found;
    }
    constexpr bool kDefer = kSph && AMVPT_SPHERE_DEFER && !AMVPT_PAIR_PRIMS;
    uint64_t dm = 0;
    auto test = [&](const DPrim &p) {
        const uint32_t type = ufirst(p.type);
        if (type == PRIM_SPHERE) {
            if (wave_any(!found && sphere_maybe(p, ray))) dm |= 1ull << ufirst(p.face);
            return;
        }
        float t, u, v;
        const bool h = prim_hit_b<false>(p, type, ray, t, u, v);
        found = found || h;
    };
    const uint32_t last = np - 1u;
    DPrim a = load_uniform(sc.gprims, 0), b = load_uniform(sc.gprims, min(1u, last));
    for (uint32_t pi = 0; pi < np; pi += 2) {
        /* branch-free: every lane tests (the wave runs the test anyway while any lane is open) */
        if (AMVPT_PAIR_PRIMS && pi + 1 < np) {
            const bool hab = brute_pair_any<kSph>(a, b, ray);
            found = found || hab;
            a = load_uniform(sc.gprims, min(pi + 2u, last));
            b = load_uniform(sc.gprims, min(pi + 3u, last));
        } else if constexpr (kDefer) {
            test(a);
            a = load_uniform(sc.gprims, min(pi + 2u, last));
            if (pi + 1 < np) test(b);
            b = load_uniform(sc.gprims, min(pi + 3u, last));
        } else {
            float t, u, v;
            const bool ha = prim_hit_b<kSph>(a, ufirst(a.type), ray, t, u, v);
            found = found || ha;
            a = load_uniform(sc.gprims, min(pi + 2u, last));
            if (pi + 1 < np) {
                const bool hb = prim_hit_b<kSph>(b, ufirst(b.type), ray, t, u, v);
                found = found || hb;
            }
            b = load_uniform(sc.gprims, min(pi + 3u, last));
        }
        if (!wave_any(!found)) break;
    }
    if constexpr (kDefer) {
        while (dm && wave_any(!found)) {
            const DPrim p = deferred_sphere(sc, mask_pop(dm));
            float t;
            const bool h = !found && sphere_hit(p, ray, t);
            found = found || h;
        }
    }
    return found;
}

/* SurfaceInteraction3f restricted to what the path reads. */
struct SI {
    float t;
    f3 p, n;
    Frame3 sh;
    f3 wi;
    int32_t shape;
    AD bool valid() const { return t != kInf; }
};

AD SI compute_si(const SceneRef &sc, const Ray &ray, const Hit &h) {
    SI si;
    si.shape = -1;
    if (h.prim < 0) {
        si.t = kInf;
        si.p = mk(0.f, 0.f, 0.f);
        si.n = mk(0.f, 0.f, 0.f);
        si.sh = Frame3{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f)};
        si.wi = -ray.d;
        return si;
    }
    const DPrim pr = sc.prims[h.prim];
    const DShape &s = sc.g->shapes[pr.shape];
    si.shape = (int32_t) pr.shape;
    si.t = h.t;
    f3 dp_du;
    if (pr.type == PRIM_RECT) {
        f3 p = ray_at(ray, h.t);
        f3 tr = mk(s.to_world[3], s.to_world[7], s.to_world[11]);
        f3 fn = ld3(s.frame_n);
        float dist = dot(tr - p, fn);
        si.p = p + dist * fn;
        si.n = fn;
        si.sh.n = fn;
        dp_du = ld3(s.frame_s);
    } else if (pr.type == PRIM_TRI) {
        /* the record's fourth words: vbase + faces[3 (fbase + face) + k] (amvpt_capi.cpp) */
        const uint32_t i0 = fbits(pr.a[3]), i1 = fbits(pr.b[3]), i2 = fbits(pr.c[3]);
        f3 p0 = ld3(sc.g->vpos + 3 * (size_t) i0), p1 = ld3(sc.g->vpos + 3 * (size_t) i1),
           p2 = ld3(sc.g->vpos + 3 * (size_t) i2);
        float b1 = h.u, b2 = h.v, b0 = 1.f - b1 - b2;
        si.p = fma3(p0, b0, fma3(p1, b1, p2 * b2));
        si.n = normalize(cross(p1 - p0, p2 - p0));
        f3 dpdv;
        coord_sys(si.n, dp_du, dpdv);
        if (s.has_uv) {
            const float *uv = sc.g->vuv;
            float u0x = uv[2 * i0], u0y = uv[2 * i0 + 1], u1x = uv[2 * i1], u1y = uv[2 * i1 + 1],
                  u2x = uv[2 * i2], u2y = uv[2 * i2 + 1];
            float d0x = u1x - u0x, d0y = u1y - u0y, d1x = u2x - u0x, d1y = u2y - u0y;
            float det = fmsub(d0x, d1y, d0y * d1x), inv_det = rcp(det);
            if (det != 0.f) {
                f3 dp0 = p1 - p0, dp1 = p2 - p0;
                dp_du = mk(fmsub(d1y, dp0.x, d0y * dp1.x) * inv_det, fmsub(d1y, dp0.y, d0y * dp1.y) * inv_det,
                           fmsub(d1y, dp0.z, d0y * dp1.z) * inv_det);
            }
        }
        if (s.has_normals) {
            f3 n0 = ld3(sc.g->vnrm + 3 * (size_t) i0), n1 = ld3(sc.g->vnrm + 3 * (size_t) i1),
               n2 = ld3(sc.g->vnrm + 3 * (size_t) i2);
            f3 n = fma3(n2, b2, fma3(n1, b1, n0 * b0));
            float il = rsqrt_(sqnorm(n));
            si.sh.n = n * il;
        } else {
            si.sh.n = si.n;
        }
        if (s.flip) { si.n = -si.n; si.sh.n = -si.sh.n; }
    } else {
        f3 c = ld3(s.center);
        si.sh.n = normalize(ray_at(ray, h.t) - c);
        si.p = fma3(si.sh.n, s.radius, c);
        const float *to = s.to_object;
        f3 local = {fmadd(to[2], si.p.z, fmadd(to[1], si.p.y, fmadd(to[0], si.p.x, to[3]))),
                    fmadd(to[6], si.p.z, fmadd(to[5], si.p.y, fmadd(to[4], si.p.x, to[7]))),
                    fmadd(to[10], si.p.z, fmadd(to[9], si.p.y, fmadd(to[8], si.p.x, to[11])))};
        dp_du = mk(-local.y, local.x, 0.f);
        const float *tw = s.to_world;
        dp_du = mk(fmadd(tw[2], dp_du.z, fmadd(tw[1], dp_du.y, tw[0] * dp_du.x)),
                   fmadd(tw[6], dp_du.z, fmadd(tw[5], dp_du.y, tw[4] * dp_du.x)),
                   fmadd(tw[10], dp_du.z, fmadd(tw[9], dp_du.y, tw[8] * dp_du.x))) * (2.f * kPi);
        if (s.flip) si.sh.n = -si.sh.n;
        si.n = si.sh.n;
    }
    /* initialize_sh_frame */
    si.sh.s = normalize(fma3(si.sh.n, -dot(si.sh.n, dp_du), dp_du));
    if (dp_du.x == 0.f && dp_du.y == 0.f && dp_du.z == 0.f) {
        f3 s0, t0;
        coord_sys(si.sh.n, s0, t0);
        si.sh.s = s0;
    }
    si.sh.t = cross(si.sh.n, si.sh.s);
    si.wi = si.sh.to_local(-ray.d);
    return si;
}

AD f3 offset_p(f3 p, f3 n, f3 d) {
    float mag = (1.f + hmax3(mk(fabs_(p.x), fabs_(p.y), fabs_(p.z)))) * kRayEps;
    mag = mulsign(mag, dot(n, d));
    return fma3(n, mag, p);
}
AD Ray spawn_ray(f3 p, f3 n, f3 d) { return Ray{offset_p(p, n, d), d, kLargest}; }
AD Ray spawn_ray_to(f3 p, f3 n, f3 t) {
    f3 o = offset_p(p, n, t - p);
    f3 d = t - o;
    float dist = norm(d);
    d = d / dist;
    return Ray{o, d, dist * (1.f - kShadowEps)};
}

} // namespace amvpt
