/*
 * amvpt_capi.cpp -- C-ABI of libamvpt_hip.so (include/amvpt.h).
 *
 * Scene upload replaces the reference's Scene constructor + Embree BVH build
 * (src/render/scene.cpp:30-96, src/render/scene_embree.inl:114-116): the host
 * builds a binned-SAH binary BVH over rectangles, triangles and spheres, lays
 * out the primitives in BVH order and uploads the small read-only tables once.
 * The product path has no CPU fallback: without a GPU every render entry
 * point returns AMVPT_ERR_NO_DEVICE.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "internal.h"

namespace amvpt {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
amvpt_status hip_fail(const char *what, int err) {
    g_err = std::string(what) + ": " + hipGetErrorString((hipError_t) err);
    return err == (int) hipErrorOutOfMemory ? AMVPT_ERR_OOM : AMVPT_ERR_HIP;
}

/* ---- host arithmetic for per-shape constants (same sequences as the kernels) ---- */
static inline float hdot(const float *a, const float *b) { return std::fmaf(a[2], b[2], std::fmaf(a[1], b[1], a[0] * b[0])); }
static inline void hvec(const float *m, const float *v, float *o) { /* Transform4f * Vector3f */
    for (int i = 0; i < 3; ++i) o[i] = std::fmaf(m[i * 4 + 2], v[2], std::fmaf(m[i * 4 + 1], v[1], m[i * 4 + 0] * v[0]));
}
static inline void hpoint(const float *m, const float *p, float *o) { /* transform_affine(Point3f) */
    for (int i = 0; i < 3; ++i)
        o[i] = std::fmaf(m[i * 4 + 2], p[2], std::fmaf(m[i * 4 + 1], p[1], std::fmaf(m[i * 4 + 0], p[0], m[i * 4 + 3])));
}
static inline void hcross(const float *a, const float *b, float *o) {
    o[0] = std::fmaf(a[1], b[2], -(a[2] * b[1]));
    o[1] = std::fmaf(a[2], b[0], -(a[0] * b[2]));
    o[2] = std::fmaf(a[0], b[1], -(a[1] * b[0]));
}
/* x as an IEEE float16 bit pattern rounded toward -inf (up = false) or +inf (up = true); magnitudes past the
 * float16 range go to -+inf / the largest finite value on the conservative side */
static uint16_t half_dir(double x, bool up) {
    auto to_d = [](uint16_t h) -> double {
        const int e = (h >> 10) & 31, m = h & 1023;
        const double v = e == 0 ? std::ldexp((double) m, -24) : e == 31 ? INFINITY : std::ldexp((double) (1024 + m), e - 25);
        return (h & 0x8000) ? -v : v;
    };
    /* the nearest representable by bisection over the ordered bit patterns (monotone in value) */
    auto key = [](uint16_t h) -> int { return (h & 0x8000) ? -(int) (h & 0x7fff) : (int) (h & 0x7fff); };
    auto from_key = [](int k) -> uint16_t { return k < 0 ? (uint16_t) (0x8000 | (-k)) : (uint16_t) k; };
    int lo = key(0xfc00), hi = key(0x7c00);   /* -inf .. +inf */
    /* largest pattern with value <= x (down), or smallest with value >= x (up) */
    if (!up) {
        while (hi - lo > 1) { const int mid = lo + (hi - lo) / 2; if (to_d(from_key(mid)) <= x) lo = mid; else hi = mid; }
        return from_key(to_d(from_key(hi)) <= x ? hi : lo);
    }
    while (hi - lo > 1) { const int mid = lo + (hi - lo) / 2; if (to_d(from_key(mid)) >= x) hi = mid; else lo = mid; }
    return from_key(to_d(from_key(lo)) >= x ? lo : hi);
}

/* .5 * dr::norm(dr::cross(p1 - p0, p2 - p0)) (mesh.cpp:470) */
static inline float tri_area(const float *p0, const float *p1, const float *p2) {
    const float e0[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
    const float e1[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
    float c[3];
    hcross(e0, e1, c);
    return .5f * std::sqrt(hdot(c, c));
}

/* ---------------------------------------------------------------- */
/* Binned SAH BVH                                                    */
/* ---------------------------------------------------------------- */

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const float *p) { for (int i = 0; i < 3; ++i) { lo[i] = std::min(lo[i], p[i]); hi[i] = std::max(hi[i], p[i]); } }
    void grow(const Box &b) { grow(b.lo); grow(b.hi); }
    float area() const {
        float d[3];
        for (int i = 0; i < 3; ++i) d[i] = std::max(hi[i] - lo[i], 0.f);
        return 2.f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
    bool empty() const { return lo[0] > hi[0]; }
};

struct BuildPrim { Box box; float c[3]; uint32_t idx; };

/* Binary SAH tree as built (children of inner node i at left, left + 1). */
struct BNode { Box box; uint32_t left_or_first, count, axis = 0; };

/* SAH shape: leaves of up to g_bvh_max_leaf primitives are kept when the split is
 * not cheaper; a split costs g_bvh_trav_cost primitive tests per unit of area on top
 * of the children's tests (amvpt_set_bvh_build). */
#ifndef AMVPT_SAH_BINS
#define AMVPT_SAH_BINS 16   /* centroid bins per axis of the binned SAH build */
#endif
static uint32_t g_bvh_max_leaf = 4;
static float g_bvh_trav_cost = 0.f;
/* depth of the LDS treelets (dscene.h DScene::tnodes), 0: none (A/B builds: EXTRA=-DAMVPT_TREELET_DEPTH=n);
 * 2^depth - 1 nodes at most, 32 B each */
#ifndef AMVPT_TREELETS
#define AMVPT_TREELETS 0   /* the walks that stage treelets (amvpt_render.hip); 0: none, so none are built */
#endif
#ifndef AMVPT_TREELET_DEPTH
#define AMVPT_TREELET_DEPTH ((AMVPT_TREELETS & 5) ? 8 : 0)   /* any-hit walks (k_shadow, k_vis): 255 nodes, 8 KB */
#endif
#ifndef AMVPT_OCT_TREELET_DEPTH
#define AMVPT_OCT_TREELET_DEPTH ((AMVPT_TREELETS & 2) ? 6 : 0)   /* closest hit: 8 octant treelets, 8 x 63 nodes, 16 KB */
#endif
/* direction-octant node orderings for the per-lane closest-hit walks of large BVHs (A/B builds:
 * EXTRA=-DAMVPT_OCT_BVH=0 keeps one copy); a build-time choice, never a process-global knob */
/* the two-box BVH (dscene.h DNode2) for the per-lane suffix walks of large BVHs (A/B builds: EXTRA=-DAMVPT_BVH2=0
 * keeps the threaded walks) */
#ifndef AMVPT_BVH2
#define AMVPT_BVH2 1
#endif
#ifndef AMVPT_OCT_BVH
#define AMVPT_OCT_BVH 1
#endif
static const uint32_t g_treelet_depth = AMVPT_TREELET_DEPTH, g_oct_treelet_depth = AMVPT_OCT_TREELET_DEPTH;

struct Builder {
    std::vector<BuildPrim> &prims;
    std::vector<BNode> nodes;
    explicit Builder(std::vector<BuildPrim> &p) : prims(p) {}

    static void pad(Box &b) {
        float m = 0.f;
        for (int i = 0; i < 3; ++i) m = std::max(m, std::max(std::fabs(b.lo[i]), std::fabs(b.hi[i])));
        float e = 1e-4f * (1.f + m);
        for (int i = 0; i < 3; ++i) { b.lo[i] -= e; b.hi[i] += e; }
    }
    void set(uint32_t ni, const Box &b) {
        Box pb = b;
        pad(pb);
        nodes[ni].box = pb;
    }
    /* every split leaves both halves non-empty, so the recursion ends with leaves of <= 4 prims */
    void build(uint32_t ni, uint32_t begin, uint32_t end, int depth) {
        Box b, cb;
        for (uint32_t i = begin; i < end; ++i) { b.grow(prims[i].box); cb.grow(prims[i].c); }
        set(ni, b);
        uint32_t n = end - begin;
        if (n <= 2) { nodes[ni].left_or_first = begin; nodes[ni].count = n; return; }
        const int NB = AMVPT_SAH_BINS;
        float best_cost = INFINITY;
        int best_axis = -1, best_split = -1;
        for (int ax = 0; ax < 3; ++ax) {
            float ext = cb.hi[ax] - cb.lo[ax];
            if (!(ext > 0.f)) continue;
            Box bins[NB];
            uint32_t cnt[NB] = {0};
            for (uint32_t i = begin; i < end; ++i) {
                int k = std::min(NB - 1, (int) (NB * (prims[i].c[ax] - cb.lo[ax]) / ext));
                bins[k].grow(prims[i].box);
                cnt[k]++;
            }
            Box lb[NB], rb[NB];
            uint32_t lc[NB], rc[NB];
            Box acc;
            uint32_t ac = 0;
            for (int k = 0; k < NB; ++k) { if (cnt[k]) acc.grow(bins[k]); ac += cnt[k]; lb[k] = acc; lc[k] = ac; }
            acc = Box();
            ac = 0;
            for (int k = NB - 1; k >= 0; --k) { if (cnt[k]) acc.grow(bins[k]); ac += cnt[k]; rb[k] = acc; rc[k] = ac; }
            for (int k = 0; k < NB - 1; ++k) {
                if (!lc[k] || !rc[k + 1]) continue;
                float cost = lb[k].area() * lc[k] + rb[k + 1].area() * rc[k + 1];
                if (cost < best_cost) { best_cost = cost; best_axis = ax; best_split = k; }
            }
        }
        float leaf_cost = b.area() * n;
        best_cost += g_bvh_trav_cost * b.area();
        if (best_axis < 0 || (n <= g_bvh_max_leaf && best_cost >= leaf_cost)) {
            if (best_axis < 0) {
                /* degenerate centroids: median split on the index */
                if (n <= g_bvh_max_leaf) { nodes[ni].left_or_first = begin; nodes[ni].count = n; return; }
                uint32_t mid = begin + n / 2;
                uint32_t l = (uint32_t) nodes.size();
                nodes.resize(nodes.size() + 2);
                nodes[ni].left_or_first = l; nodes[ni].count = 0; nodes[ni].axis = 0;
                build(l, begin, mid, depth + 1);
                build(l + 1, mid, end, depth + 1);
                return;
            }
            nodes[ni].left_or_first = begin; nodes[ni].count = n;
            return;
        }
        float ext = cb.hi[best_axis] - cb.lo[best_axis];
        auto it = std::partition(prims.begin() + begin, prims.begin() + end, [&](const BuildPrim &p) {
            int k = std::min(NB - 1, (int) (NB * (p.c[best_axis] - cb.lo[best_axis]) / ext));
            return k <= best_split;
        });
        uint32_t mid = (uint32_t) (it - prims.begin());
        if (mid == begin || mid == end) mid = begin + n / 2;
        uint32_t l = (uint32_t) nodes.size();
        nodes.resize(nodes.size() + 2);
        nodes[ni].left_or_first = l; nodes[ni].count = 0; nodes[ni].axis = (uint32_t) best_axis;
        build(l, begin, mid, depth + 1);
        build(l + 1, mid, end, depth + 1);
    }
    /*
     * Depth-first pre-order with skip links (DNode), children in the order a ray of direction
     * octant `oct` (bit a: negative along axis a) meets them: the lower child along the split
     * axis first for a positive direction, the upper one first for a negative direction.  The
     * skip links are local to the copy, so octant copy o is the array at o * n_nodes.
     */
    void flatten(uint32_t ni, std::vector<DNode> &out, uint32_t oct = 0, uint32_t base = 0,
                 std::vector<uint32_t> *pos = nullptr) const {
        const BNode &bn = nodes[ni];
        const uint32_t at = (uint32_t) out.size();
        if (pos) (*pos)[ni] = at;
        DNode d{};
        for (int i = 0; i < 3; ++i) { d.lo[i] = bn.box.lo[i]; d.hi[i] = bn.box.hi[i]; }
        d.first = bn.count ? bn.left_or_first : 0u;
        out.push_back(d);
        if (!bn.count) {
            const uint32_t near = (oct >> bn.axis) & 1u;
            flatten(bn.left_or_first + near, out, oct, base, pos);
            flatten(bn.left_or_first + (near ^ 1u), out, oct, base, pos);
        }
        out[at].skip_count = (((uint32_t) out.size() - base) & kNodeSkipMask) | (bn.count << kNodeCountShift);
    }
    /* the two-box BVH (dscene.h DNode2) of the subtree under inner node ni, depth-first (a node, then its first
     * child's subtree, then its second's); returns ni's index in out; depth: inner nodes on the path to ni */
    uint32_t flatten2(uint32_t ni, std::vector<DNode2> &out, uint32_t depth, uint32_t &max_depth) const {
        const uint32_t at = (uint32_t) out.size();
        out.push_back(DNode2{});
        max_depth = std::max(max_depth, depth);
        uint32_t refs[2];
        for (int c = 0; c < 2; ++c) {
            const BNode &ch = nodes[nodes[ni].left_or_first + c];
            refs[c] = ch.count ? (kRef2Leaf | (ch.count << kRef2CountShift) | ch.left_or_first)
                               : flatten2(nodes[ni].left_or_first + c, out, depth + 1, max_depth);
            for (int k = 0; k < 3; ++k) {
                out[at].b[6 * c + k] = ch.box.lo[k];
                out[at].b[6 * c + 3 + k] = ch.box.hi[k];
            }
        }
        out[at].ref[0] = refs[0];
        out[at].ref[1] = refs[1];
        return at;
    }
    /* the treelet of one ordering: the nodes of depth < depth_cut in the same depth-first order, skip links
     * local to the treelet; an inner node at depth depth_cut - 1 is a portal to its subtree in the global
     * copy (gpos: each builder node's index in that copy's array, including the copy's base) */
    void flatten_top(uint32_t ni, std::vector<DNode> &out, uint32_t oct, uint32_t depth, uint32_t depth_cut,
                     const std::vector<uint32_t> &gpos, uint32_t gbase, uint32_t base) const {
        const BNode &bn = nodes[ni];
        const uint32_t at = (uint32_t) out.size();
        DNode d{};
        for (int i = 0; i < 3; ++i) { d.lo[i] = bn.box.lo[i]; d.hi[i] = bn.box.hi[i]; }
        d.first = bn.count ? bn.left_or_first : 0u;
        const bool portal = !bn.count && depth + 1 >= depth_cut;
        if (portal) d.first = kPortal | (gpos[ni] - gbase);   /* index local to the copy, as its skip links */
        out.push_back(d);
        if (!bn.count && !portal) {
            const uint32_t near = (oct >> bn.axis) & 1u;
            flatten_top(bn.left_or_first + near, out, oct, depth + 1, depth_cut, gpos, gbase, base);
            flatten_top(bn.left_or_first + (near ^ 1u), out, oct, depth + 1, depth_cut, gpos, gbase, base);
        }
        out[at].skip_count = (((uint32_t) out.size() - base) & kNodeSkipMask) | (bn.count << kNodeCountShift);
    }
};

static bool device_ok() {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

static uint32_t leaf_flags(const amvpt_bsdf_desc &d) {
    if (d.type == AMVPT_BSDF_DIFFUSE) return 0x2u | 0x8000u;
    uint32_t f = 0x8u | 0x8000u;
    if (d.alpha_u != d.alpha_v) f |= 0x1000u;
    return f;
}

} // namespace amvpt

using namespace amvpt;

extern "C" {

const char *amvpt_last_error(void) { return g_err.c_str(); }
uint32_t amvpt_abi_version(void) { return AMVPT_ABI_VERSION; }

amvpt_status amvpt_device_count(int *count) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    if (count) *count = n;
    return AMVPT_OK;
}

amvpt_status amvpt_set_device(int device) {
    if (!device_ok()) { set_error("no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) return hip_fail("hipSetDevice", (int) e);
    return AMVPT_OK;
}

uint32_t amvpt_film_channels(const amvpt_params *p) { return p && p->film_alpha ? 5u : 4u; }

amvpt_status amvpt_set_chunk_lanes(uint64_t chunk_lanes) {
    g_chunk_lanes = chunk_lanes ? std::max<uint64_t>(256, chunk_lanes) : 0;   /* 0: automatic */
    return AMVPT_OK;
}

amvpt_status amvpt_set_traversal(uint32_t mode) {
    if (mode > 2) { set_error("amvpt_set_traversal: mode must be 0 (auto), 1 (wave-uniform) or 2 (per-lane)"); return AMVPT_ERR_INVALID; }
    g_traversal = mode;
    return AMVPT_OK;
}

amvpt_status amvpt_set_bvh_build(uint32_t max_leaf_prims, float traversal_cost) {
    if (max_leaf_prims < 1 || max_leaf_prims > kMaxLeafPrims || !(traversal_cost >= 0.f)) {
        set_error("amvpt_set_bvh_build: max_leaf_prims in [1, 15], traversal_cost >= 0");
        return AMVPT_ERR_INVALID;
    }
    g_bvh_max_leaf = max_leaf_prims;
    g_bvh_trav_cost = traversal_cost;
    return AMVPT_OK;
}

amvpt_status amvpt_set_adaptive_exchange(amvpt_exchange_fn fn, void *ctx) {
    g_exchange = fn;
    g_exchange_ctx = fn ? ctx : nullptr;
    return AMVPT_OK;
}

amvpt_status amvpt_plan(const amvpt_params *P, uint32_t *spp, uint32_t *spp_pp, uint32_t *n_passes,
                        uint64_t *lanes) {
    if (!P) { set_error("amvpt_plan: null params"); return AMVPT_ERR_INVALID; }
    uint32_t s = P->spp ? P->spp : 1, spl;
    uint32_t np;
    if (P->integrator == AMVPT_INTEGRATOR_MVPATH) {
        spl = P->spp_pass_lim ? std::min(P->spp_pass_lim, s) : s;
        np = s / spl;
        s = np * spl;
    } else {
        spl = s;
        np = 1;
    }
    uint64_t wf = (uint64_t) P->film_width * P->film_height * spl;
    if (wf > 0xffffffffull) {
        spl /= (uint32_t) ((wf + 0xffffffffull - 1) / 0xffffffffull);
        np = s / spl;
        wf = (uint64_t) P->film_width * P->film_height * spl;
    }
    if (spp) *spp = s;
    if (spp_pp) *spp_pp = spl;
    if (n_passes) *n_passes = np;
    if (lanes) *lanes = wf;
    return AMVPT_OK;
}

/* Descriptor checks of amvpt_scene_create (run before any device work, so malformed
 * input fails with AMVPT_ERR_INVALID even on a host without a GPU). */
static amvpt_status validate_scene(const amvpt_scene_desc *d) {
    if ((d->shape_count && !d->shapes) || (d->bsdf_count && !d->bsdfs) || (d->emitter_count && !d->emitters)) {
        set_error("amvpt_scene_create: null table with a non-zero count");
        return AMVPT_ERR_INVALID;
    }
    {
        uint32_t n_env = 0;
        bool positive = false;
        for (uint32_t i = 0; i < d->emitter_count; ++i) {
            n_env += d->emitters[i].type == AMVPT_EMITTER_CONSTANT ? 1u : 0u;
            const float w = d->emitters[i].sampling_weight;
            if (!(w >= 0.f) || !std::isfinite(w)) {
                set_error("DiscreteDistribution: entries must be non-negative!");
                return AMVPT_ERR_INVALID;
            }
            positive = positive || w > 0.f;
        }
        if (d->emitter_count && !positive) { set_error("DiscreteDistribution: no probability mass found!"); return AMVPT_ERR_INVALID; }
        if (n_env > 1) { set_error("Only one environment emitter can be specified per scene."); return AMVPT_ERR_INVALID; }
        if (d->has_environment != n_env) {
            set_error("amvpt_scene_create: has_environment must count the AMVPT_EMITTER_CONSTANT emitters");
            return AMVPT_ERR_INVALID;
        }
    }
    for (uint32_t i = 0; i < d->bsdf_count; ++i) {
        const amvpt_bsdf_desc &b = d->bsdfs[i];
        if (b.type == AMVPT_BSDF_ROUGHCONDUCTOR && b.distribution != AMVPT_MICROFACET_GGX &&
            b.distribution != AMVPT_MICROFACET_BECKMANN) {
            set_error("roughconductor: unknown microfacet distribution");
            return AMVPT_ERR_INVALID;
        }
        if (b.type == AMVPT_BSDF_TWOSIDED) {
            for (int k = 0; k < 2; ++k) {
                int32_t nb = b.nested[k];
                if (nb < 0 || (uint32_t) nb >= d->bsdf_count || d->bsdfs[nb].type == AMVPT_BSDF_TWOSIDED) {
                    set_error("twosided: invalid nested BSDF");
                    return AMVPT_ERR_INVALID;
                }
            }
        } else if (b.type > AMVPT_BSDF_TWOSIDED) {
            set_error("unknown BSDF type");
            return AMVPT_ERR_INVALID;
        }
    }
    for (uint32_t i = 0; i < d->emitter_count; ++i) {
        const amvpt_emitter_desc &e = d->emitters[i];
        if (e.type == AMVPT_EMITTER_CONSTANT) {
            if (e.shape != -1) { set_error("a constant emitter is not attached to a shape (shape must be -1)"); return AMVPT_ERR_INVALID; }
            continue;
        }
        if (e.type != AMVPT_EMITTER_AREA) { set_error("unknown emitter type"); return AMVPT_ERR_INVALID; }
        if (e.shape < 0 || (uint32_t) e.shape >= d->shape_count) { set_error("emitter without a valid shape"); return AMVPT_ERR_INVALID; }
    }

    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        if (s.bsdf < 0 || (uint32_t) s.bsdf >= d->bsdf_count) { set_error("shape without a valid BSDF"); return AMVPT_ERR_INVALID; }
        if (s.emitter < -1 || (s.emitter >= 0 && (uint32_t) s.emitter >= d->emitter_count)) {
            set_error("shape.emitter outside [-1, emitter_count)");
            return AMVPT_ERR_INVALID;
        }
        /* the area emitter and its shape must point at each other (Shape::set_emitter) */
        if (s.emitter >= 0 && d->emitters[s.emitter].shape != (int32_t) i) {
            set_error("shape.emitter and emitter.shape disagree");
            return AMVPT_ERR_INVALID;
        }
        if (s.type == AMVPT_SHAPE_MESH) {
            if (!s.positions || !s.faces) { set_error("mesh without positions/faces"); return AMVPT_ERR_INVALID; }
            for (size_t f = 0; f < 3 * (size_t) s.face_count; ++f)
                if (s.faces[f] >= s.vertex_count) { set_error("mesh face index >= vertex_count"); return AMVPT_ERR_INVALID; }
            if (s.emitter >= 0) {
                /* Mesh::build_pmf (mesh.cpp:448-449) / DiscreteDistribution::compute_cdf (distr_1d.h) */
                if (s.face_count == 0) { set_error("Cannot create sampling table for an empty mesh"); return AMVPT_ERR_INVALID; }
                float acc = 0.f;
                for (uint32_t f = 0; f < s.face_count; ++f)
                    acc += tri_area(s.positions + 3 * s.faces[3 * f], s.positions + 3 * s.faces[3 * f + 1],
                                    s.positions + 3 * s.faces[3 * f + 2]);
                if (!(acc > 0.f)) { set_error("DiscreteDistribution: no probability mass found!"); return AMVPT_ERR_INVALID; }
            }
        } else if (s.type != AMVPT_SHAPE_RECTANGLE && s.type != AMVPT_SHAPE_SPHERE) {
            set_error("unknown shape type");
            return AMVPT_ERR_INVALID;
        }
    }
    for (uint32_t i = 0; i < d->emitter_count; ++i)
        if (d->emitters[i].type == AMVPT_EMITTER_AREA && d->shapes[d->emitters[i].shape].emitter != (int32_t) i) {
            set_error("shape.emitter and emitter.shape disagree");
            return AMVPT_ERR_INVALID;
        }
    return AMVPT_OK;
}

/* Transform::transform_affine of a point with the reference's fmadd chains (row-major 4x4) */
static void xform_affine(const float *m, const float p[3], float out[3]) {
    for (int i = 0; i < 3; ++i)
        out[i] = std::fmaf(m[i * 4 + 2], p[2], std::fmaf(m[i * 4 + 1], p[1], std::fmaf(m[i * 4 + 0], p[0], m[i * 4 + 3])));
}

/* ConstantBackgroundEmitter::set_scene (constant.cpp:73-88): the bounding sphere of Scene::bbox()
 * (union of Shape::bbox(): rectangle corners, mesh vertices, sphere center -+ radius), center =
 * (min + max) / 2, radius = |center - max| enlarged by (1 + RayEpsilon), at least RayEpsilon */
static void scene_bsphere(const amvpt_scene_desc *d, float center[3], float &radius) {
    const float ray_eps = 1500.f * 5.9604644775390625e-8f;   /* math.h:18-23: 1500 * 2^-24 */
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    bool any = false;
    auto expand = [&](const float p[3]) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
        any = true;
    };
    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        if (s.type == AMVPT_SHAPE_RECTANGLE) {
            const float corners[4][3] = {{-1.f, -1.f, 0.f}, {1.f, -1.f, 0.f}, {1.f, 1.f, 0.f}, {-1.f, 1.f, 0.f}};
            for (auto &c : corners) { float w[3]; xform_affine(s.to_world, c, w); expand(w); }
        } else if (s.type == AMVPT_SHAPE_MESH) {
            for (uint32_t v = 0; v < s.vertex_count; ++v) expand(s.positions + 3 * (size_t) v);
        } else {
            const float a[3] = {s.center[0] - s.radius, s.center[1] - s.radius, s.center[2] - s.radius};
            const float b[3] = {s.center[0] + s.radius, s.center[1] + s.radius, s.center[2] + s.radius};
            expand(a); expand(b);
        }
    }
    if (!any) { center[0] = center[1] = center[2] = 0.f; radius = ray_eps; return; }
    for (int k = 0; k < 3; ++k) center[k] = (hi[k] + lo[k]) * .5f;
    const float dx = center[0] - hi[0], dy = center[1] - hi[1], dz = center[2] - hi[2];
    radius = std::sqrt(std::fmaf(dz, dz, std::fmaf(dy, dy, dx * dx)));
    radius = std::max(ray_eps, radius * (1.f + ray_eps));
}

#ifndef AMVPT_BVH_OUTER
#define AMVPT_BVH_OUTER 2    /* up to kOuterMax rectangles stay out of the BVH: 2 in every scene (the brute-force
                                     * scenes' coherent walks too: config-M k_vis 44.2 -> 35.3 ms, r05u), 1 in scenes of
                                     * more than kBrutePrims primitives only, 0 none (A/B) */
#endif
static constexpr uint32_t kBrutePrimsHost = 48;   /* dgeom.h kBrutePrims: brute-force scenes have no BVH walk */
static constexpr float kInf32 = std::numeric_limits<float>::infinity();
#ifndef AMVPT_BOX_SCREEN
#define AMVPT_BOX_SCREEN 1   /* box meshes of brute-force scenes get DBox records (0: none, A/B) */
#endif
/*
 * Box meshes (dscene.h DBox): a mesh shape of 12 triangles whose vertices map, through the shape's
 * to_object (in double), to corners of [-1, 1]^3 within 1e-5, every triangle lying in one face plane, two
 * triangles per face covering its four corners -- the `cube` plugin's mesh (cube.cpp:105-160) under any
 * affine to_world.  Boxes whose box-space coordinates would magnify the walks' rounding are left to the plain
 * scan: the screen maps a ray's ORIGIN into box space, and the suffix rays start anywhere on the scene's
 * surfaces, so the bound is the box's conditioning (largest row norm of to_object) times (1 + the largest
 * coordinate magnitude of the whole scene, desc_extent), not of the box's own vertices: a small
 * cube on a ground plane 1000 units wide would have its box-space origins at ~1e4 and f32 rounding near kBoxEps.
 * prims[] is in BVH order; box_prims / loose_prims hold copies with the BVH index in `type`'s upper bits.
 */
/* the largest coordinate magnitude of any primitive of the scene (world space): mesh vertices, rectangle corners
 * (to_world of (+-1, +-1, 0)), sphere centres +- radius */
static double desc_extent(const amvpt_scene_desc *d) {
    double e = 0.0;
    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        if (s.type == AMVPT_SHAPE_MESH && s.positions) {
            for (size_t k = 0; k < (size_t) 3 * s.vertex_count; ++k) e = std::max(e, (double) std::fabs(s.positions[k]));
        } else if (s.type == AMVPT_SHAPE_RECTANGLE) {
            for (int c = 0; c < 4; ++c) {
                const double x = (c & 1) ? 1.0 : -1.0, y = (c & 2) ? 1.0 : -1.0;
                for (int r = 0; r < 3; ++r)
                    e = std::max(e, std::fabs(s.to_world[4 * r] * x + s.to_world[4 * r + 1] * y + s.to_world[4 * r + 3]));
            }
        } else if (s.type == AMVPT_SHAPE_SPHERE) {
            for (int r = 0; r < 3; ++r) e = std::max(e, (double) std::fabs(s.center[r]) + (double) std::fabs(s.radius));
        }
    }
    return e;
}
static void find_boxes(const amvpt_scene_desc *d, const std::vector<DPrim> &prims, std::vector<DBox> &boxes,
                       std::vector<DPrim> &box_prims, std::vector<DPrim> &loose) {
    const double extent = desc_extent(d);
    std::vector<int> in_box(prims.size(), 0);
    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        if (s.type != AMVPT_SHAPE_MESH || s.face_count != 12 || !s.positions || !s.faces) continue;
        std::vector<uint32_t> tris;
        for (uint32_t pi = 0; pi < (uint32_t) prims.size(); ++pi)
            if (prims[pi].type == PRIM_TRI && prims[pi].shape == i) tris.push_back(pi);
        if (tris.size() != 12) continue;
        double M[12], cond = 0.0, wmax = 0.0;
        for (int k = 0; k < 12; ++k) M[k] = (double) s.to_object[k];
        for (int r = 0; r < 3; ++r)
            cond = std::max(cond, std::sqrt(M[4 * r] * M[4 * r] + M[4 * r + 1] * M[4 * r + 1] + M[4 * r + 2] * M[4 * r + 2]));
        bool ok = true;
        int n_on[6] = {0, 0, 0, 0, 0, 0};
        uint32_t ftri[12];
        uint32_t corners[6] = {0, 0, 0, 0, 0, 0};   /* per face: the (b, c) corners its triangles touch, 4 bits */
        for (uint32_t pi : tris) {
            const uint32_t f = prims[pi].face;
            double b[3][3];
            for (int v = 0; v < 3; ++v) {
                const float *w = s.positions + 3 * (size_t) s.faces[3 * f + v];
                for (int r = 0; r < 3; ++r) {
                    b[v][r] = M[4 * r] * w[0] + M[4 * r + 1] * w[1] + M[4 * r + 2] * w[2] + M[4 * r + 3];
                    wmax = std::max(wmax, (double) std::fabs(w[r]));
                    if (std::fabs(std::fabs(b[v][r]) - 1.0) > 1e-5) ok = false;
                }
            }
            int axis = -1;
            for (int a = 0; a < 3; ++a)
                if ((b[0][a] > 0) == (b[1][a] > 0) && (b[0][a] > 0) == (b[2][a] > 0)) { axis = a; break; }
            if (!ok || axis < 0) { ok = false; break; }
            const int face = 2 * axis + (b[0][axis] > 0 ? 1 : 0);
            if (n_on[face] >= 2) { ok = false; break; }
            ftri[2 * face + n_on[face]++] = pi;
            const int bx = (axis + 1) % 3, cx = (axis + 2) % 3;
            for (int v = 0; v < 3; ++v) corners[face] |= 1u << ((b[v][bx] > 0 ? 1 : 0) + (b[v][cx] > 0 ? 2 : 0));
        }
        for (int f = 0; ok && f < 6; ++f) ok = n_on[f] == 2 && corners[f] == 15u;
        if (!ok || cond * (1.0 + std::max(wmax, extent)) >= 100.0) continue;
        DBox B{};
        for (int k = 0; k < 12; ++k) B.m[k] = (float) M[k];
        for (int k = 0; k < 12; ++k) {
            DPrim q = prims[ftri[k]];
            q.type = PRIM_TRI | (ftri[k] << 8);
            box_prims.push_back(q);
            in_box[ftri[k]] = 1;
        }
        boxes.push_back(B);
    }
    /* (with no box, every primitive is loose: the typed scans and the rectangle cull still apply) */
    /* grouped by type (rectangles, triangles, spheres), BVH order within a group: the walks loop over each
     * group with its own test (the closest-hit rule does not depend on the order) */
    for (uint32_t type : {(uint32_t) PRIM_RECT, (uint32_t) PRIM_TRI, (uint32_t) PRIM_SPHERE})
        for (uint32_t pi = 0; pi < (uint32_t) prims.size(); ++pi)
            if (!in_box[pi] && prims[pi].type == type) {
                DPrim q = prims[pi];
                q.type |= pi << 8;
                loose.push_back(q);
            }
}

amvpt_status amvpt_scene_create(const amvpt_scene_desc *d, amvpt_scene **out) {
    if (!d || !out) { set_error("amvpt_scene_create: null argument"); return AMVPT_ERR_INVALID; }
    *out = nullptr;
    /* validate the whole descriptor first (also without a device): every index the host
     * tables or the kernels follow must be in range */
    {
        const amvpt_status vs = validate_scene(d);
        if (vs != AMVPT_OK) return vs;
    }
    if (!device_ok()) { set_error("amvpt_scene_create: no HIP device visible (the product path has no CPU fallback)"); return AMVPT_ERR_NO_DEVICE; }
    bool has_spheres = false;
    std::vector<DShape> shapes(d->shape_count);
    std::vector<float> vpos, vnrm, vuv, face_area;
    std::vector<uint32_t> faces;
    std::vector<BuildPrim> bprims;
    std::vector<DPrim> scene_prims; /* scene order */
    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        DShape &o = shapes[i];
        std::memset(&o, 0, sizeof(o));
        o.type = s.type;
        o.flip = s.flip_normals;
        o.bsdf = s.bsdf;
        o.emitter = s.emitter;
        std::memcpy(o.to_world, s.to_world, 12 * sizeof(float));
        std::memcpy(o.to_object, s.to_object, 12 * sizeof(float));
        if (s.bsdf < 0 || (uint32_t) s.bsdf >= d->bsdf_count) { set_error("shape without a valid BSDF"); return AMVPT_ERR_INVALID; }
        if (s.type == AMVPT_SHAPE_RECTANGLE) {
            /* Rectangle::update (rectangle.cpp:112-123) */
            const float ex[3] = {2.f, 0.f, 0.f}, ey[3] = {0.f, 2.f, 0.f};
            hvec(s.to_world, ex, o.frame_s);
            hvec(s.to_world, ey, o.frame_t);
            /* normal through inverse_transpose = transpose(to_object) */
            float nn[3];
            for (int r = 0; r < 3; ++r)
                nn[r] = std::fmaf(s.to_object[2 * 4 + r], 1.f, std::fmaf(s.to_object[1 * 4 + r], 0.f, s.to_object[0 * 4 + r] * 0.f));
            float inv = 1.f / std::sqrt(hdot(nn, nn));
            for (int r = 0; r < 3; ++r) o.frame_n[r] = nn[r] * inv;
            float cr[3];
            hcross(o.frame_s, o.frame_t, cr);
            o.inv_area = 1.f / std::sqrt(hdot(cr, cr));
            DPrim p{};
            std::memcpy(p.a, s.to_object + 0, 16);
            std::memcpy(p.b, s.to_object + 4, 16);
            std::memcpy(p.c, s.to_object + 8, 16);
            p.type = PRIM_RECT; p.shape = i; p.face = 0;
            BuildPrim bp;
            const float corners[4][3] = {{-1, -1, 0}, {-1, 1, 0}, {1, -1, 0}, {1, 1, 0}};
            for (auto &c : corners) { float w[3]; hpoint(s.to_world, c, w); bp.box.grow(w); }
            p.pad = (uint32_t) scene_prims.size();
            scene_prims.push_back(p);
            bp.idx = p.pad;
            for (int k = 0; k < 3; ++k) bp.c[k] = 0.5f * (bp.box.lo[k] + bp.box.hi[k]);
            bprims.push_back(bp);
        } else if (s.type == AMVPT_SHAPE_MESH) {
            if (!s.positions || !s.faces) { set_error("mesh without positions/faces"); return AMVPT_ERR_INVALID; }
            o.vbase = (uint32_t) (vpos.size() / 3);
            o.fbase = (uint32_t) (faces.size() / 3);
            o.has_normals = s.normals != nullptr;
            o.has_uv = s.texcoords != nullptr;
            vpos.insert(vpos.end(), s.positions, s.positions + 3 * (size_t) s.vertex_count);
            if (s.normals) {
                vnrm.resize(vpos.size() - 3 * (size_t) s.vertex_count, 0.f);
                vnrm.insert(vnrm.end(), s.normals, s.normals + 3 * (size_t) s.vertex_count);
            }
            if (s.texcoords) {
                vuv.resize(2 * (vpos.size() / 3 - s.vertex_count), 0.f);
                vuv.insert(vuv.end(), s.texcoords, s.texcoords + 2 * (size_t) s.vertex_count);
            }
            faces.insert(faces.end(), s.faces, s.faces + 3 * (size_t) s.face_count);
            /* Mesh::build_pmf (mesh.cpp:444-485): face areas .5 |(p1 - p0) x (p2 - p0)|, float prefix sum */
            float acc = 0.f;
            for (uint32_t f = 0; f < s.face_count; ++f) {
                const float a = tri_area(s.positions + 3 * s.faces[3 * f], s.positions + 3 * s.faces[3 * f + 1],
                                         s.positions + 3 * s.faces[3 * f + 2]);
                acc += a;
                face_area.push_back(a);
                face_area.push_back(acc);
            }
            o.n_faces = s.face_count;
            o.area_sum = acc;
            o.inv_area = acc != 0.f ? 1.f / acc : 0.f;
            for (uint32_t f = 0; f < s.face_count; ++f) {
                DPrim p{};
                const float *P0 = s.positions + 3 * s.faces[3 * f], *P1 = s.positions + 3 * s.faces[3 * f + 1],
                            *P2 = s.positions + 3 * s.faces[3 * f + 2];
                /* p0 and the two edges (the f32 differences tri_hit would form: same bits) */
                for (int k = 0; k < 3; ++k) { p.a[k] = P0[k]; p.b[k] = P1[k] - P0[k]; p.c[k] = P2[k] - P0[k]; }
                /* the spare fourth words: the face's absolute vertex indices (compute_si reads the vertices without
                 * a dependent load of the face table) */
                for (int k = 0; k < 3; ++k) {
                    const uint32_t vi = o.vbase + s.faces[3 * f + k];
                    std::memcpy(k == 0 ? &p.a[3] : k == 1 ? &p.b[3] : &p.c[3], &vi, 4);
                }
                p.type = PRIM_TRI; p.shape = i; p.face = f;
                p.pad = (uint32_t) scene_prims.size();
                BuildPrim bp;
                bp.box.grow(P0); bp.box.grow(P1); bp.box.grow(P2);
                bp.idx = p.pad;
                for (int k = 0; k < 3; ++k) bp.c[k] = 0.5f * (bp.box.lo[k] + bp.box.hi[k]);
                scene_prims.push_back(p);
                bprims.push_back(bp);
            }
        } else if (s.type == AMVPT_SHAPE_SPHERE) {
            std::memcpy(o.center, s.center, 12);
            o.radius = s.radius;
            o.inv_area = 1.f / ((4.f * 3.14159265358979323846f) * (s.radius * s.radius));
            DPrim p{};
            p.a[0] = s.center[0]; p.a[1] = s.center[1]; p.a[2] = s.center[2]; p.a[3] = s.radius;
            p.type = PRIM_SPHERE; p.shape = i; p.face = 0;
            has_spheres = true;
            p.pad = (uint32_t) scene_prims.size();
            BuildPrim bp;
            for (int k = 0; k < 3; ++k) { bp.box.lo[k] = s.center[k] - s.radius; bp.box.hi[k] = s.center[k] + s.radius; }
            bp.idx = p.pad;
            for (int k = 0; k < 3; ++k) bp.c[k] = s.center[k];
            scene_prims.push_back(p);
            bprims.push_back(bp);
        } else {
            set_error("unknown shape type");
            return AMVPT_ERR_INVALID;
        }
    }
    if (!vnrm.empty()) vnrm.resize(vpos.size(), 0.f);
    if (!vuv.empty()) vuv.resize(2 * (vpos.size() / 3), 0.f);

    /* the scene's bounds (all primitives): the ray-binning grid (render_impl) */
    float scene_lo[3] = {kInf32, kInf32, kInf32}, scene_hi[3] = {-kInf32, -kInf32, -kInf32};
    for (const BuildPrim &bp : bprims)
        for (int k = 0; k < 3; ++k) { scene_lo[k] = std::min(scene_lo[k], bp.box.lo[k]); scene_hi[k] = std::max(scene_hi[k], bp.box.hi[k]); }
    /* BVH scenes with a few rectangles (a room's walls and lights): the rectangles stay out of the BVH and
     * every walk tests them first (DScene::outer, dgeom.h outer_closest / outer_any) -- their boxes span the
     * scene, so every ray crossing it descended to their leaves and tested them in divergent leaf code */
    std::vector<uint32_t> outer_idx;
    if (AMVPT_BVH_OUTER && (scene_prims.size() > kBrutePrimsHost || AMVPT_BVH_OUTER >= 2)) {
        std::vector<BuildPrim> keep;
        for (const BuildPrim &bp : bprims) {
            if (scene_prims[bp.idx].type == PRIM_RECT) outer_idx.push_back(bp.idx);
            else keep.push_back(bp);
        }
        if (outer_idx.size() <= kOuterMax && !keep.empty()) bprims.swap(keep);
        else outer_idx.clear();
    }
    std::vector<DNode> nodes, tnodes, onodes;
    std::vector<DNode2> nodes2;   /* the two-box BVH (empty: none) */
    std::vector<DNode2h> nodes2h; /* its float16 form */
    float n2_center[3] = {0.f, 0.f, 0.f}, n2_scale = 1.f;
    uint32_t bvh2_depth = 0;
    std::vector<DPrim> prims;
    uint32_t oct_stride = 0;   /* nodes per octant copy (0: one copy) */
    uint32_t t_stride = 0;     /* nodes of the first ordering's treelet (0: none) */
    uint32_t o_stride = 0;     /* nodes per octant treelet (0: none) */
    if (bprims.empty()) {
        /* one inner node with an empty box: every ray misses it and skips to the end */
        DNode root{};
        root.lo[0] = root.lo[1] = root.lo[2] = 1.f;
        root.hi[0] = root.hi[1] = root.hi[2] = -1.f;
        root.first = 0;
        root.skip_count = 1u;
        nodes.push_back(root);
    } else {
        Builder b(bprims);
        b.nodes.resize(1);
        b.build(0, 0, (uint32_t) bprims.size(), 0);
        nodes.reserve(b.nodes.size());
        /* per-ordering positions of the build nodes: only the treelet builds read them */
        const bool want_pos = g_treelet_depth > 0 || g_oct_treelet_depth > 0;
        std::vector<std::vector<uint32_t>> gpos(want_pos ? 8 : 1);
        if (want_pos) for (auto &g : gpos) g.assign(b.nodes.size(), 0u);
        b.flatten(0, nodes, 0, 0, want_pos ? &gpos[0] : nullptr);
        if (nodes.size() > kNodeSkipMask) {
            set_error("BVH too large (more than 2^28 nodes)");
            return AMVPT_ERR_INVALID;
        }
        /* per-lane walks of BVHs that are neither wave-uniform nor LDS-staged read the copy of
         * their ray's direction octant: nearest child first, so the closest hit shrinks the
         * box-test range early */
        const uint32_t n0 = (uint32_t) nodes.size();
        const uint64_t lds_b = (uint64_t) n0 * sizeof(DNode) + bprims.size() * sizeof(DPrim);
        if (AMVPT_OCT_BVH && n0 > kUniformNodeLimit && lds_b > kLdsSceneBytes && (uint64_t) n0 * 8 <= kNodeSkipMask) {
            nodes.reserve((size_t) n0 * 8);
            for (uint32_t o = 1; o < 8; ++o) b.flatten(0, nodes, o, o * n0, want_pos ? &gpos[o] : nullptr);
            oct_stride = n0;
        }
        /* LDS treelets for BVHs the walks read from global memory (neither wave-uniform-small nor staged
         * whole): one per node ordering */
        if (g_treelet_depth > 0 && n0 > kUniformNodeLimit && lds_b > kLdsSceneBytes) {
            b.flatten_top(0, tnodes, 0, 0, g_treelet_depth, gpos[0], 0, 0);
            t_stride = (uint32_t) tnodes.size();
        }
        if (g_oct_treelet_depth > 0 && oct_stride) {
            for (uint32_t o = 0; o < 8; ++o) {
                const uint32_t base = (uint32_t) onodes.size();
                b.flatten_top(0, onodes, o, 0, g_oct_treelet_depth, gpos[o], o * n0, base);
                if (o == 0) o_stride = (uint32_t) onodes.size();
            }
        }
        /* the two-box BVH of the per-lane suffix walks (BVHs read from device memory, leaves addressable in a
         * reference, at most kStack2 inner nodes deep) */
        if (AMVPT_BVH2 && n0 > kUniformNodeLimit && lds_b > kLdsSceneBytes && bprims.size() <= kRef2FirstMask) {
            uint32_t depth = 0;
            if (b.nodes[0].count) {
                /* a root leaf: one node with the leaf and an empty second child */
                DNode2 r{};
                for (int k = 0; k < 3; ++k) {
                    r.b[k] = b.nodes[0].box.lo[k]; r.b[3 + k] = b.nodes[0].box.hi[k];
                    r.b[6 + k] = 1.f; r.b[9 + k] = -1.f;
                }
                r.ref[0] = kRef2Leaf | (b.nodes[0].count << kRef2CountShift) | b.nodes[0].left_or_first;
                r.ref[1] = r.ref[0];
                nodes2.push_back(r);
                depth = 1;
            } else {
                b.flatten2(0, nodes2, 1, depth);
            }
            bvh2_depth = depth;
            if (depth > kStack2) nodes2.clear();
            /* the float16 form (dscene.h DNode2h): the root box's centre and half extent set the frame */
            const Box &rb = b.nodes[0].box;
            double hmax = 0.0;
            for (int k = 0; k < 3; ++k) {
                n2_center[k] = (float) (.5 * ((double) rb.lo[k] + (double) rb.hi[k]));
                hmax = std::max(hmax, .5 * ((double) rb.hi[k] - (double) rb.lo[k]));
            }
            n2_scale = hmax > 0.0 ? (float) (1.0 / hmax) : 1.f;
            for (const DNode2 &n : nodes2) {
                DNode2h q{};
                uint16_t hv[12];
                for (int c = 0; c < 2; ++c)
                    for (int k = 0; k < 3; ++k) {
                        const double lo = ((double) n.b[6 * c + k] - (double) n2_center[k]) * (double) n2_scale;
                        const double hi = ((double) n.b[6 * c + 3 + k] - (double) n2_center[k]) * (double) n2_scale;
                        hv[6 * c + k] = half_dir(lo, false);
                        hv[6 * c + 3 + k] = half_dir(hi, true);
                    }
                for (int w = 0; w < 6; ++w) q.h[w] = (uint32_t) hv[2 * w] | ((uint32_t) hv[2 * w + 1] << 16);
                q.ref[0] = n.ref[0];
                q.ref[1] = n.ref[1];
                nodes2h.push_back(q);
            }
        }
        prims.resize(bprims.size());
        for (size_t i = 0; i < bprims.size(); ++i) prims[i] = scene_prims[bprims[i].idx];
    }
    std::vector<DPrim> outer;
    for (uint32_t idx : outer_idx) {
        DPrim q = scene_prims[idx];
        q.type |= (uint32_t) prims.size() << 8;
        outer.push_back(q);
        prims.push_back(scene_prims[idx]);
    }
    const uint32_t n_outer = (uint32_t) outer.size();
    if (outer.empty()) outer.resize(1);
    if (prims.empty()) prims.resize(1); /* keep a valid pointer */

    std::vector<DBsdf> bsdfs(d->bsdf_count);
    for (uint32_t i = 0; i < d->bsdf_count; ++i) {
        const amvpt_bsdf_desc &s = d->bsdfs[i];
        DBsdf &o = bsdfs[i];
        std::memset(&o, 0, sizeof(o));
        o.type = s.type;
        o.distribution = s.distribution;
        o.sample_visible = s.sample_visible;
        o.has_spec = s.has_specular_reflectance;
        o.nested0 = s.nested[0];
        o.nested1 = s.nested[1];
        std::memcpy(o.refl, s.reflectance, 12);
        o.alpha_u = s.alpha_u; o.alpha_v = s.alpha_v;
        std::memcpy(o.eta, s.eta, 12);
        std::memcpy(o.k, s.k, 12);
        std::memcpy(o.spec, s.specular_reflectance, 12);
        if (s.type == AMVPT_BSDF_TWOSIDED) {
            uint32_t f0 = leaf_flags(d->bsdfs[s.nested[0]]), f1 = leaf_flags(d->bsdfs[s.nested[1]]);
            o.flags = ((f0 & ~0x10000u) | 0x8000u) | ((f1 & ~0x8000u) | 0x10000u);
        } else {
            o.flags = leaf_flags(s);
        }
    }
    std::vector<DEmitter> emitters(std::max<uint32_t>(1, d->emitter_count));
    bool distr = false;
    int32_t environment = -1;
    float cdf_acc = 0.f;
    for (uint32_t i = 0; i < d->emitter_count; ++i) {
        DEmitter &e = emitters[i];
        std::memset(&e, 0, sizeof(e));
        e.shape = d->emitters[i].shape;
        e.type = d->emitters[i].type;
        std::memcpy(e.radiance, d->emitters[i].radiance, 12);
        e.weight = d->emitters[i].sampling_weight;
        cdf_acc += e.weight;   /* DiscreteDistribution::compute_cdf: dr::prefix_sum in float */
        e.cdf = cdf_acc;
        distr = distr || e.weight != 1.f;
        if (e.type == AMVPT_EMITTER_CONSTANT) environment = (int32_t) i;
    }
    if (vpos.empty()) vpos.resize(3, 0.f);
    if (vnrm.empty()) vnrm.resize(3, 0.f);
    if (vuv.empty()) vuv.resize(2, 0.f);
    if (faces.empty()) faces.resize(3, 0);
    if (face_area.empty()) face_area.resize(2, 0.f);

    amvpt_scene *sc = new amvpt_scene();
    sc->has_spheres = has_spheres;
    sc->bvh_tri_only = !bprims.empty();
    for (const BuildPrim &bp : bprims) sc->bvh_tri_only = sc->bvh_tri_only && scene_prims[bp.idx].type == PRIM_TRI;
    (void) hipGetDevice(&sc->device);
    auto upload = [&](const void *src, size_t bytes, void **dst) -> amvpt_status {
        hipError_t e = hipMalloc(dst, bytes);
        if (e != hipSuccess) return hip_fail("hipMalloc(scene)", (int) e);
        sc->allocations.push_back(*dst);
        e = hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return hip_fail("hipMemcpy(scene)", (int) e);
        return AMVPT_OK;
    };
    /* sphere ordinals (DScene::sph_prims): the record's `face` field, unused by spheres otherwise */
    std::vector<uint32_t> sph_prims;
    for (uint32_t i = 0; i < (uint32_t) prims.size(); ++i)
        if (prims[i].type == PRIM_SPHERE) {
            prims[i].face = (uint32_t) sph_prims.size();
            sph_prims.push_back(i);
        }
    const uint32_t n_sph = (uint32_t) sph_prims.size();
    if (sph_prims.empty()) sph_prims.resize(1, 0u);
    /* box meshes of brute-force scenes (dscene.h DBox; dgeom.h box_walk) */
    std::vector<DBox> boxes;
    std::vector<DPrim> box_prims, loose_prims;
    if (AMVPT_BOX_SCREEN && prims.size() <= 48) find_boxes(d, prims, boxes, box_prims, loose_prims);
    const uint32_t n_boxes = (uint32_t) boxes.size(), n_loose = (uint32_t) loose_prims.size();
    if (boxes.empty()) boxes.resize(1);
    if (box_prims.empty()) box_prims.resize(1);
    if (loose_prims.empty()) loose_prims.resize(1);
    void *p_nodes, *p_prims, *p_shapes, *p_bsdfs, *p_emit, *p_vpos, *p_vnrm, *p_vuv, *p_faces, *p_farea, *p_tnodes, *p_onodes, *p_sph;
    void *p_boxes, *p_box_prims, *p_loose, *p_outer, *p_nodes2, *p_nodes2h;
    if (tnodes.empty()) tnodes.resize(1);   /* keep a valid pointer */
    const uint32_t n_nodes2 = (uint32_t) nodes2.size();
    if (nodes2.empty()) nodes2.resize(1);
    if (nodes2h.empty()) nodes2h.resize(1);
    if (onodes.empty()) onodes.resize(1);
    amvpt_status st;
#define UP(vec, ptr)                                                                      \
    if ((st = upload(vec.data(), vec.size() * sizeof(vec[0]), &ptr)) != AMVPT_OK) {       \
        amvpt_scene_destroy(sc);                                                          \
        return st;                                                                        \
    }
    UP(nodes, p_nodes) UP(prims, p_prims) UP(shapes, p_shapes) UP(bsdfs, p_bsdfs) UP(emitters, p_emit)
    UP(vpos, p_vpos) UP(vnrm, p_vnrm) UP(vuv, p_vuv) UP(faces, p_faces) UP(face_area, p_farea) UP(tnodes, p_tnodes) UP(onodes, p_onodes)
    UP(sph_prims, p_sph) UP(boxes, p_boxes) UP(box_prims, p_box_prims) UP(loose_prims, p_loose) UP(outer, p_outer)
    UP(nodes2, p_nodes2) UP(nodes2h, p_nodes2h)
#undef UP
    DScene &D = sc->dev;
    D.nodes = (const DNode *) p_nodes;
    D.prims = (const DPrim *) p_prims;
    D.shapes = (const DShape *) p_shapes;
    D.bsdfs = (const DBsdf *) p_bsdfs;
    D.emitters = (const DEmitter *) p_emit;
    D.vpos = (const float *) p_vpos;
    D.vnrm = (const float *) p_vnrm;
    D.vuv = (const float *) p_vuv;
    D.faces = (const uint32_t *) p_faces;
    D.face_area = (const float *) p_farea;
    D.n_nodes = oct_stride ? oct_stride : (uint32_t) nodes.size();
    D.oct_stride = oct_stride;
    D.tnodes = (const DNode *) p_tnodes;
    D.t_stride = t_stride;
    D.onodes = (const DNode *) p_onodes;
    D.o_stride = o_stride;
    D.sph_prims = (const uint32_t *) p_sph;
    D.n_sph = n_sph;
    sc->n_sph = n_sph;
    D.boxes = (const DBox *) p_boxes;
    D.box_prims = (const DPrim *) p_box_prims;
    D.loose_prims = (const DPrim *) p_loose;
    D.n_boxes = n_boxes;
    D.n_loose = n_loose;
    D.n_loose_rect = D.n_loose_tri = 0;
    for (uint32_t j = 0; j < n_loose; ++j) {
        D.n_loose_rect += (loose_prims[j].type & 0xffu) == PRIM_RECT ? 1u : 0u;
        D.n_loose_tri += (loose_prims[j].type & 0xffu) == PRIM_TRI ? 1u : 0u;
    }
    sc->n_boxes = n_boxes;
    D.outer = (const DPrim *) p_outer;
    D.n_outer = n_outer;
    D.nodes2 = (const DNode2 *) p_nodes2;
    D.n_nodes2 = n_nodes2;
    D.nodes2h = (const DNode2h *) p_nodes2h;
    for (int k = 0; k < 3; ++k) D.n2_center[k] = n2_center[k];
    D.n2_scale = n2_scale;
    sc->n_nodes2 = n_nodes2;
    sc->bvh2_depth = bvh2_depth;
    sc->n_outer = n_outer;
    for (int a = 0; a < 3; ++a) {
        sc->root_lo[a] = bprims.empty() ? nodes[0].lo[a] : scene_lo[a];
        sc->root_hi[a] = bprims.empty() ? nodes[0].hi[a] : scene_hi[a];
    }
    D.n_prims = (uint32_t) prims.size();
    D.n_shapes = d->shape_count;
    D.n_emitters = d->emitter_count;
    D.emitter_pmf = d->emitter_count ? 1.f / (float) d->emitter_count : 0.f;
    D.environment = environment;
    D.distr = distr ? 1u : 0u;
    D.distr_sum = d->emitter_count ? emitters[d->emitter_count - 1].cdf : 0.f;
    D.distr_norm = D.distr_sum != 0.f ? 1.f / D.distr_sum : 0.f;
    if (environment >= 0) scene_bsphere(d, D.bs_center, D.bs_radius);
    else { D.bs_center[0] = D.bs_center[1] = D.bs_center[2] = 0.f; D.bs_radius = 0.f; }
    D.n_bsdfs = d->bsdf_count;
    {
        const uint32_t tb = tab_round(d->shape_count * (uint32_t) sizeof(DShape)) +
                            tab_round(d->bsdf_count * (uint32_t) sizeof(DBsdf)) +
                            tab_round(d->emitter_count * (uint32_t) sizeof(DEmitter));
        D.tab_bytes = tb <= kTabBytes ? tb : 0u;
    }
    D.lds_bytes = (uint32_t) ((size_t) D.n_nodes * sizeof(DNode) + prims.size() * sizeof(DPrim));
    sc->n_nodes = D.n_nodes;
    sc->n_prims = (uint32_t) (bprims.size() + n_outer);
    sc->all_diffuse = d->bsdf_count > 0;
    for (uint32_t i = 0; i < d->bsdf_count; ++i) sc->all_diffuse = sc->all_diffuse && d->bsdfs[i].type == AMVPT_BSDF_DIFFUSE;
    std::vector<DScene> one(1, D);
    if ((st = upload(one.data(), sizeof(DScene), &sc->dev_scene_struct)) != AMVPT_OK) {
        amvpt_scene_destroy(sc);
        return st;
    }
    *out = sc;
    return AMVPT_OK;
}

amvpt_status amvpt_scene_desc_boxes(const amvpt_scene_desc *d, uint32_t *n_boxes) {
    if (!d || !n_boxes) { set_error("amvpt_scene_desc_boxes: null argument"); return AMVPT_ERR_INVALID; }
    const amvpt_status vs = validate_scene(d);
    if (vs != AMVPT_OK) return vs;
    /* the primitives in scene order (find_boxes reads type, shape and face only) */
    std::vector<DPrim> prims;
    for (uint32_t i = 0; i < d->shape_count; ++i) {
        const amvpt_shape_desc &s = d->shapes[i];
        const uint32_t n = s.type == AMVPT_SHAPE_MESH ? s.face_count : 1u;
        for (uint32_t f = 0; f < n; ++f) {
            DPrim p{};
            p.type = s.type == AMVPT_SHAPE_MESH ? PRIM_TRI : s.type == AMVPT_SHAPE_SPHERE ? PRIM_SPHERE : PRIM_RECT;
            p.shape = i;
            p.face = f;
            prims.push_back(p);
        }
    }
    std::vector<DBox> boxes;
    std::vector<DPrim> bp, lp;
    find_boxes(d, prims, boxes, bp, lp);
    *n_boxes = (uint32_t) boxes.size();
    return AMVPT_OK;
}

amvpt_status amvpt_scene_destroy(amvpt_scene *scene) {
    if (!scene) return AMVPT_OK;
    for (void *p : scene->allocations) (void) hipFree(p);
    delete scene;
    return AMVPT_OK;
}

amvpt_status amvpt_scene_bvh2(const amvpt_scene *scene, uint32_t *n_nodes2, uint32_t *depth) {
    if (!scene || !n_nodes2 || !depth) { set_error("amvpt_scene_bvh2: null argument"); return AMVPT_ERR_INVALID; }
    *n_nodes2 = scene->n_nodes2;
    *depth = scene->bvh2_depth;
    return AMVPT_OK;
}

amvpt_status amvpt_scene_stats(const amvpt_scene *scene, uint32_t *n_nodes, uint32_t *n_prims) {
    if (!scene) { set_error("null scene"); return AMVPT_ERR_INVALID; }
    if (n_nodes) *n_nodes = scene->n_nodes;
    if (n_prims) *n_prims = scene->n_prims;
    return AMVPT_OK;
}

} // extern "C"

namespace {
/* amvpt_set_adaptive_exchange's one-count exchange as a run exchange: a contiguous lane set is
 * one run (or none, for an empty range) */
struct LegacyExchange { amvpt_exchange_fn fn; void *ctx; };
int legacy_run_exchange(void *ctx, uint32_t n_runs, const uint64_t *, const uint64_t *run_count, uint64_t *run_prefix,
                        uint64_t *total) {
    const LegacyExchange *x = static_cast<const LegacyExchange *>(ctx);
    if (n_runs > 1) return 1;
    uint64_t prefix = 0;
    const int rc = x->fn(x->ctx, n_runs ? run_count[0] : 0, &prefix, total);
    if (n_runs) run_prefix[0] = prefix;
    return rc;
}
/* amvpt_render / amvpt_render_records: contiguous lanes, whole-quilt film, process-global knobs */
amvpt_status render_legacy(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                           uint64_t lane_begin, uint64_t lane_end, float *film, void *stream, amvpt_counters *counters,
                           float *records, uint32_t pass) {
    if (!params) { set_error("amvpt_render: null argument"); return AMVPT_ERR_INVALID; }
    amvpt_lane_set lanes{};
    lanes.lane_begin = lane_begin;
    lanes.lane_end = lane_end;
    amvpt_film_window w{};
    w.film = film;
    w.width = params->film_width;
    w.height = params->film_height;
    LegacyExchange lx{g_exchange, g_exchange_ctx};
    amvpt_render_opts o{};
    o.chunk_lanes = g_chunk_lanes;
    o.traversal = g_traversal;
    if (g_exchange) { o.exchange = legacy_run_exchange; o.exchange_ctx = &lx; }
    return render_impl(scene, views, params, lanes, w, stream, o, counters, records, pass);
}
} // namespace

extern "C" {

amvpt_status amvpt_render(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                          uint64_t lane_begin, uint64_t lane_end, float *film_device, void *stream,
                          amvpt_counters *counters) {
    if (!device_ok()) { set_error("amvpt_render: no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    return render_legacy(scene, views, params, lane_begin, lane_end, film_device, stream, counters, nullptr, 0);
}

amvpt_status amvpt_render_records(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                                  uint32_t pass, uint64_t lane_begin, uint64_t lane_end, float *film_device,
                                  float *records_device, void *stream) {
    if (!device_ok()) { set_error("amvpt_render_records: no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    return render_legacy(scene, views, params, lane_begin, lane_end, film_device, stream, nullptr, records_device, pass);
}

amvpt_status amvpt_render_ex(amvpt_scene *scene, const amvpt_view_desc *views, const amvpt_params *params,
                             const amvpt_lane_set *lanes, const amvpt_film_window *film, void *stream,
                             const amvpt_render_opts *opts, amvpt_counters *counters) {
    if (!lanes || !film) { set_error("amvpt_render_ex: null lane set or film window"); return AMVPT_ERR_INVALID; }
    if (!device_ok()) { set_error("amvpt_render_ex: no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    const amvpt_render_opts defaults{};
    const amvpt_render_opts &o = opts ? *opts : defaults;
    return render_impl(scene, views, params, *lanes, *film, stream, o, counters, o.records, o.record_pass);
}

amvpt_status amvpt_film_accumulate(float *quilt, uint32_t quilt_width, uint32_t quilt_height, uint32_t channels,
                                   const float *window, uint32_t x0, uint32_t y0, uint32_t width, uint32_t height,
                                   const uint32_t *overflow_entries, uint64_t n_entries, void *stream) {
    if (!device_ok()) { set_error("amvpt_film_accumulate: no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    return accumulate_impl(quilt, quilt_width, quilt_height, channels, window, x0, y0, width, height, overflow_entries,
                           n_entries, stream);
}

amvpt_status amvpt_develop(const float *film_device, float *out_device, uint32_t width, uint32_t height,
                           uint32_t film_alpha, void *stream) {
    if (!device_ok()) { set_error("amvpt_develop: no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    return develop_impl(film_device, out_device, width, height, film_alpha, stream);
}

amvpt_status amvpt_release_device_memory(int device) {
    if (!device_ok()) { set_error("amvpt_release_device_memory: no HIP device visible"); return AMVPT_ERR_NO_DEVICE; }
    return release_impl(device);
}

} // extern "C"
