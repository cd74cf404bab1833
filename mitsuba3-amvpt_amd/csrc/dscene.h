/*
 * dscene.h -- device-resident scene layout of the AMVPT hot path (HBM).
 *
 * Everything the per-lane kernels read about the scene lives in a handful of
 * small, read-only tables that fit the Infinity Cache / L2 (Cornell box: ~6 KB)
 * and are staged into LDS at kernel start when they fit (kLdsSceneBytes):
 *   nodes[]   binary BVH, 32 B per node                (replaces Embree, scene_embree.inl)
 *   prims[]   BVH-ordered primitives, 64 B each        (rectangle / triangle / sphere)
 *   shapes[]  per-shape transforms, frames, mesh bases (rectangle.cpp, mesh.cpp, sphere.cpp)
 *   bsdfs[]   flattened BSDF parameters                (diffuse / roughconductor / twosided)
 *   emitters[] area lights                             (area.cpp)
 *   views[]   per-sub-sensor projective transforms     (grid.cpp + perspective.cpp)
 *   mesh vertex / normal / texcoord / face streams     (mesh.cpp)
 */
#pragma once
#include <stdint.h>

namespace amvpt {

enum : uint32_t { PRIM_RECT = 0, PRIM_TRI = 1, PRIM_SPHERE = 2 };

/*
 * Threaded (stackless) BVH node, nodes stored in depth-first pre-order: the
 * first child of an inner node is the next node, and `skip` is the node that
 * follows the whole subtree (n_nodes for the last one).  Traversal is
 * "hit -> descend (node + 1) or test the leaf, miss/leaf -> skip": no stack.
 */
struct alignas(16) DNode {
    float lo[3];
    uint32_t first;          /* leaf: first prim; inner: unused */
    float hi[3];
    uint32_t skip_count;     /* bits 0..27: skip node index; bits 28..31: prim count (0 = inner node) */
};
constexpr uint32_t kNodeSkipMask = 0x0fffffffu, kNodeCountShift = 28, kMaxLeafPrims = 15;
/*
 * Two-box BVH node (round 6) for the per-lane suffix walks of large BVHs: an inner node of the same binary SAH
 * tree holding BOTH children's (padded) boxes and their references, so a walk loads a node only when it enters it
 * -- one dependent load per inner node entered instead of one per node tested -- and orders the two children by
 * the ray's own entry distances (near first) with the far one on a short per-lane LDS stack.  A reference is an
 * inner node's index in nodes2[], or kRef2Leaf | count << 27 | first for a leaf of prims[first, first + count)
 * (the threaded BVH's leaves, the same BVH-order prims[]).  4 x 16 B: (lo0.xyz, hi0.x), (hi0.yz, lo1.xy),
 * (lo1.z, hi1.xyz), (ref0, ref1, -, -).
 */
struct alignas(16) DNode2 {
    float b[12];             /* lo0[3], hi0[3], lo1[3], hi1[3] */
    uint32_t ref[2];
    uint32_t pad[2];
};
constexpr uint32_t kRef2Leaf = 0x80000000u, kRef2FirstMask = 0x07ffffffu, kRef2CountShift = 27;
/*
 * The same node in 32 B (AMVPT_BVH2_HALF): the two child boxes as float16 in the scene's normalized frame
 * (x' = (x - n2_center) * n2_scale, the BVH root box mapped into [-1, 1]^3), each plane rounded outward (lo down, hi
 * up) from the padded float box, so every box contains its float box: a cull test only, never a hit, so the walk
 * finds the same hits.  h[0..5] = (lo0.xy), (lo0.z, hi0.x), (hi0.yz), (lo1.xy), (lo1.z, hi1.x), (hi1.yz), two halves
 * per word, low half first; then the two references.
 */
struct alignas(16) DNode2h {
    uint32_t h[6];
    uint32_t ref[2];
};
constexpr uint32_t kStack2 = 16;   /* per-lane stack entries of the two-box walks: a tree deeper than this keeps the
                                    * threaded walks (a walk pushes at most one entry per inner node on its path) */
/* BVHs up to this many nodes are traversed wave-uniformly; per-lane walks stage nodes + prims
 * in LDS up to kLdsSceneBytes. */
constexpr uint32_t kUniformNodeLimit = 255, kLdsSceneBytes = 48 * 1024;

struct alignas(16) DPrim {
    /* rect: rows 0..2 of to_object; tri: p0, p1 - p0, p2 - p0 (xyz) and the three absolute vertex indices (the
     * fourth words, as bits); sphere: a = (center, radius) */
    float a[4], b[4], c[4];
    uint32_t type, shape, face;
    uint32_t pad;            /* scene-order primitive index: closest-hit tie-break */
};

struct DShape {
    uint32_t type, flip;
    int32_t bsdf, emitter;
    float to_world[12];     /* rows 0..2 of the 4x4 */
    float to_object[12];
    float frame_s[3], frame_t[3], frame_n[3]; /* rectangle m_frame */
    float inv_area;
    uint32_t vbase, fbase, has_normals, has_uv;
    float center[3], radius;
    uint32_t n_faces;       /* mesh: face count of its area distribution (Mesh::m_area_pmf) */
    float area_sum;         /* mesh: m_area_pmf.sum(); inv_area holds its normalization() */
};

struct DBsdf {
    uint32_t type, distribution, sample_visible, has_spec;
    int32_t nested0, nested1;
    uint32_t flags;         /* BSDFFlags of the whole BSDF (bsdf.h:37-86) */
    uint32_t pad;
    float refl[3];
    float alpha_u, alpha_v; /* raw (eval_roughness) */
    float eta[3], k[3], spec[3];
};

struct DEmitter {
    int32_t shape;          /* area: its shape; constant (environment): -1 */
    uint32_t type;          /* AMVPT_EMITTER_AREA / AMVPT_EMITTER_CONSTANT */
    float radiance[3];
    float weight;           /* sampling_weight (DiscreteDistribution pmf entry) */
    float cdf;              /* inclusive prefix sum of the weights (float, compute_cdf) */
    float pad[3];
};

struct DView {
    float to_world[12];
    float to_world_inv[12];
    float sample_to_camera[16];
    float camera_to_sample[16];
    float near_clip, far_clip, normalization, pad0;
    float res[2], pp[2];
    uint32_t type;          /* AMVPT_CAMERA_PERSPECTIVE / _THINLENS */
    float aperture_radius, focus_distance, pad1;
};

/* Small material/shape/emitter/view tables are copied to LDS by every kernel. */
constexpr uint32_t kTabBytes = 8192, kViewTabBytes = 8192;
inline __host__ __device__ uint32_t tab_round(uint32_t b) { return (b + 15u) & ~15u; }

/*
 * A box mesh (a `cube` shape, or any 12-triangle mesh whose triangles tile the faces of a parallelepiped):
 * m maps world space to box space, where the box is [-1, 1]^3.  Its triangles are copied in face order to
 * DScene::box_prims[12 * box + 2 * face + j] (face = 2 * axis + (side > 0)), each record's `type` holding
 * PRIM_TRI | (its index in prims[] << 8).  The brute-force walks screen a box per lane and test only the
 * triangles of the faces a ray can reach (dgeom.h box_walk).
 */
struct alignas(16) DBox {
    float m[12];
    uint32_t pad[4];
};

struct DScene {
    const DNode *nodes;
    const DPrim *prims;
    const DShape *shapes;
    const DBsdf *bsdfs;
    const DEmitter *emitters;
    const float *vpos;      /* xyz per vertex */
    const float *vnrm;
    const float *vuv;
    const uint32_t *faces;  /* 3 per face, indices relative to the shape's vbase */
    const float *face_area; /* (pmf, inclusive cdf) per face at 2 * (fbase + f): Mesh::m_area_pmf */
    uint32_t n_nodes, n_prims, n_shapes, n_emitters;
    float emitter_pmf;
    int32_t environment;    /* the constant emitter's index, or -1 */
    uint32_t distr;         /* non-uniform emitter sampling (scene.cpp:100-119) */
    float distr_sum, distr_norm;
    float bs_center[3], bs_radius;  /* the constant emitter's bounding sphere (constant.cpp:73-88) */
    uint32_t lds_bytes;     /* nodes+prims footprint (LDS staging when small) */
    uint32_t n_bsdfs;
    uint32_t tab_bytes;     /* shapes+bsdfs+emitters footprint if <= kTabBytes (staged in LDS), else 0 */
    uint32_t oct_stride;    /* != 0: nodes[] holds 8 direction-octant orderings of n_nodes each (amvpt_capi.cpp) */
    /* LDS treelets of large BVHs (the walks stage them per block, dgeom.h trace_*_tl): the nodes of depth
     * < treelet_depth of each node ordering in depth-first order with treelet-local skip links; a node whose
     * children lie below the cut is a portal (count 0, first = kPortal | its index in `nodes`), where the walk
     * continues in the global copy.  t_stride nodes per ordering (1 or 8 of them, as oct_stride); 0: none */
    const DNode *tnodes;
    uint32_t t_stride;
    /* the same for the 8 direction-octant orderings (closest-hit walks, trace_closest_tl): o_stride nodes
     * each, a shallower cut (all 8 are staged together); 0: none */
    const DNode *onodes;
    uint32_t o_stride;
    /* the spheres' primitive indices in scene order of their ordinals (a sphere record's `face` field holds its
     * ordinal): the wave-uniform walks' deferred sphere tests (dgeom.h, kSph = 2) */
    const uint32_t *sph_prims;
    uint32_t n_sph;
    /* box meshes of brute-force scenes (DBox): the boxes, their triangles in face order, and every other
     * primitive ("loose", in BVH order, `type` | index << 8); n_boxes = 0: none (the walks scan prims[]) */
    const DBox *boxes;
    const DPrim *box_prims;
    const DPrim *loose_prims;
    uint32_t n_boxes, n_loose;
    uint32_t n_loose_rect, n_loose_tri;   /* loose_prims: rectangles, then triangles, then spheres */
    /* BVH scenes: the rectangles kept out of the BVH (amvpt_capi.cpp, at most kOuterMax), each record's
     * `type` | its index in prims[] << 8 (they follow the BVH's primitives there); n_outer = 0: none */
    const DPrim *outer;
    uint32_t n_outer;
    /* the two-box BVH of the per-lane suffix walks (DNode2; nodes2[0] is the root); n_nodes2 = 0: none (small or
     * LDS-staged BVHs, a tree deeper than kStack2, or AMVPT_BVH2 off) */
    const DNode2 *nodes2;
    uint32_t n_nodes2;
    const DNode2h *nodes2h;       /* the float16 form of nodes2 (AMVPT_BVH2_HALF), in the normalized frame: */
    float n2_center[3], n2_scale; /*   x' = (x - n2_center) * n2_scale */
};
constexpr uint32_t kOuterMax = 8;
constexpr uint32_t kPortal = 0x80000000u;

} // namespace amvpt
