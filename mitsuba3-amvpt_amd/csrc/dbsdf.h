/*
 * dbsdf.h -- BSDFs, area emitters and projective sensors for the AMVPT kernels.
 *
 * Every entry point follows Dr.Jit's masked-virtual-call convention of the
 * reference's JIT variants: a null BSDF/emitter or a masked lane returns zeros.
 *
 * Reference (file:line): SmoothDiffuse src/bsdfs/diffuse.cpp:100-188;
 * RoughConductor src/bsdfs/roughconductor.cpp:225-523; MicrofacetDistribution
 * include/mitsuba/render/microfacet.h:185-431; fresnel_conductor fresnel.h:93-116;
 * TwoSidedBRDF src/bsdfs/twosided.cpp:112-296; AreaLight src/emitters/area.cpp:82-190;
 * Shape::sample_direction / pdf_direction src/render/shape.cpp:360-390;
 * Sphere::sample_direction / pdf_direction src/shapes/sphere.cpp:234-330;
 * Scene::sample_emitter_direction / pdf_emitter_direction src/render/scene.cpp:294-361;
 * PerspectiveCamera::sample_ray / sample_surface src/sensors/perspective.cpp:205-241,327-385.
 */
#pragma once
#include "dgeom.h"

namespace amvpt {

enum : uint32_t {
    BF_Null = 0x1, BF_DiffuseReflection = 0x2, BF_GlossyReflection = 0x8,
    BF_Diffuse = 0x2 | 0x4, BF_Glossy = 0x8 | 0x10, BF_Smooth = 0x2 | 0x4 | 0x8 | 0x10,
    BF_Delta = 0x20 | 0x40
};
enum : uint32_t { BSDF_DIFFUSE = 0, BSDF_ROUGHCONDUCTOR = 1, BSDF_TWOSIDED = 2 };
constexpr uint32_t CTX_ALL = 0xffffffffu, CTX_GLOSSY = BF_Glossy;
AD bool ctx_on(uint32_t mask, uint32_t type) { return mask == 0xffffffffu || (mask & type) == type; }

struct C3 { float r, g, b; };
AD C3 c3(float v) { return {v, v, v}; }
AD C3 c3(const float *p) { return {p[0], p[1], p[2]}; }
AD C3 operator*(C3 a, C3 b) { return {a.r * b.r, a.g * b.g, a.b * b.b}; }
AD C3 operator*(C3 a, float s) { return {a.r * s, a.g * s, a.b * s}; }
AD C3 operator*(float s, C3 a) { return {s * a.r, s * a.g, s * a.b}; }
AD C3 operator+(C3 a, C3 b) { return {a.r + b.r, a.g + b.g, a.b + b.b}; }
AD C3 operator/(C3 a, float s) { return {a.r / s, a.g / s, a.b / s}; }
AD C3 cfma(C3 a, C3 b, C3 c) { return {fmadd(a.r, b.r, c.r), fmadd(a.g, b.g, c.g), fmadd(a.b, b.b, c.b)}; }
AD float cmax(C3 a) { return vmax(vmax(a.r, a.g), a.b); }
/* component-wise select: a ternary on the structs makes clang select between two stack
 * temporaries' addresses, which SROA cannot always undo (scratch loads in k_mv_primary) */
AD C3 csel(bool m, C3 a, C3 b) { return {m ? a.r : b.r, m ? a.g : b.g, m ? a.b : b.b}; }

struct BSample { f3 wo; float pdf, eta; uint32_t type; };
AD BSample bs_zero() { return BSample{mk(0.f, 0.f, 0.f), 0.f, 0.f, 0u}; }

/* ---------------- microfacet (microfacet.h:185-431): GGX and Beckmann ---------------- */
constexpr float kInvSqrtPi = 0.56418958354775628695f;
struct Mf {
    float au, av;
    bool visible, beckmann;
    AD Mf() : au(1.f), av(1.f), visible(false), beckmann(false) {}
    AD Mf(const DBsdf &b)
        : au(vmax(b.alpha_u, 1e-4f)), av(vmax(b.alpha_v, 1e-4f)), visible(b.sample_visible != 0),
          beckmann(b.distribution == AMVPT_MICROFACET_BECKMANN) {}
    AD float eval(f3 m) const {
        float alpha_uv = au * av, ct = m.z, result;
        if (beckmann) {
            const float ct2 = sqr(ct);
            result = exp_(-(sqr(m.x / au) + sqr(m.y / av)) / ct2) / (kPi * alpha_uv * sqr(ct2));
        } else {
            result = rcp(kPi * alpha_uv * sqr(sqr(m.x / au) + sqr(m.y / av) + sqr(m.z)));
        }
        return result * ct > 1e-20f ? result : 0.f;
    }
    AD float smith_g1(f3 v, f3 m) const {
        float xy = sqr(au * v.x) + sqr(av * v.y), ta2 = xy / sqr(v.z), result;
        if (beckmann) {
            /* rational approximation of the shadowing-masking function (microfacet.h:332-339) */
            float a = rsqrt_(ta2), a_sqr = sqr(a);
            result = a >= 1.6f ? 1.f : (3.535f * a + 2.181f * a_sqr) / (1.f + 2.276f * a + 2.577f * a_sqr);
        } else {
            result = 2.f / (1.f + dsqrt(1.f + ta2));
        }
        if (xy == 0.f) result = 1.f;
        if (dot(v, m) * v.z <= 0.f) result = 0.f;
        return result;
    }
    /* sample_visible_11 (microfacet.h:362-420) */
    AD void visible_11(float cti, float u1, float u2, float &slx, float &sly) const {
        if (beckmann) {
            /* numerical inversion, three Newton steps */
            float tan_theta_i = safe_sqrt(fnmadd(cti, cti, 1.f)) / cti;
            float cot_theta_i = rcp(tan_theta_i);
            float maxval = erf_(cot_theta_i);
            u1 = vmax(vmin(u1, 1.f - 1e-6f), 1e-6f);
            u2 = vmax(vmin(u2, 1.f - 1e-6f), 1e-6f);
            float x = maxval - (maxval + 1.f) * erf_(dsqrt(-log_(u1)));
            u1 *= 1.f + maxval + kInvSqrtPi * tan_theta_i * exp_(-sqr(cot_theta_i));
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                float slope = erfinv_(x),
                      value = 1.f + x + kInvSqrtPi * tan_theta_i * exp_(-sqr(slope)) - u1,
                      derivative = 1.f - slope * tan_theta_i;
                x -= value / derivative;
            }
            slx = erfinv_(x);
            sly = erfinv_(fmsub(2.f, u2, 1.f));
            return;
        }
        float px, py;
        disk_concentric(u1, u2, px, py);
        float s = 0.5f * (1.f + cti);
        py = lerp_(safe_sqrt(1.f - sqr(px)), py, s);
        float x = px, y = py, z = safe_sqrt(1.f - fmadd(py, py, px * px));
        float sti = safe_sqrt(1.f - sqr(cti));
        float nrm = rcp(fmadd(sti, y, cti * z));
        slx = fmsub(cti, y, sti * z) * nrm;
        sly = x * nrm;
    }
    AD void sample(f3 wi, float u1, float u2, f3 &m, float &pdf) const {
        if (!visible) {
            /* azimuth: uniform (isotropic) or the tan inversion (anisotropic), then the
             * distribution's elevation (microfacet.h:244-300) */
            float sin_phi, cos_phi, alpha_2;
            if (au == av) {
                sincos_c((2.f * kPi) * u2, sin_phi, cos_phi);
                alpha_2 = au * au;
            } else {
                float ratio = av / au, tmp = ratio * tan_((2.f * kPi) * u2);
                cos_phi = rsqrt_(fmadd(tmp, tmp, 1.f));
                cos_phi = mulsign(cos_phi, fabs_(u2 - .5f) - .25f);
                sin_phi = cos_phi * tmp;
                alpha_2 = rcp(sqr(cos_phi / au) + sqr(sin_phi / av));
            }
            float ct, ct2;
            if (beckmann) {
                ct = rsqrt_(fnmadd(alpha_2, log_(1.f - u1), 1.f));
                ct2 = sqr(ct);
                float ct3 = vmax(ct2 * ct, 1e-20f);
                pdf = (1.f - u1) / (kPi * au * av * ct3);
            } else {
                float tan2 = alpha_2 * u1 / (1.f - u1);
                ct = rsqrt_(1.f + tan2);
                ct2 = sqr(ct);
                float temp = 1.f + tan2 / alpha_2, ct3 = vmax(ct2 * ct, 1e-20f);
                pdf = rcp(kPi * au * av * ct3 * sqr(temp));
            }
            float st = dsqrt(1.f - ct2);
            m = mk(cos_phi * st, sin_phi * st, ct);
            return;
        }
        f3 wp = normalize(mk(au * wi.x, av * wi.y, wi.z));
        float st2 = fmadd(wp.x, wp.x, sqr(wp.y)), inv_st = rsqrt_(st2);
        float rx = wp.x * inv_st, ry = wp.y * inv_st;
        if (fabs_(st2) <= 4.f * kEps) { rx = 1.f; ry = 0.f; }
        else { rx = vmin(vmax(rx, -1.f), 1.f); ry = vmin(vmax(ry, -1.f), 1.f); }
        float sin_phi = ry, cos_phi = rx, cti = wp.z;
        float slx, sly;
        visible_11(cti, u1, u2, slx, sly);
        float sx = fmsub(cos_phi, slx, sin_phi * sly) * au, sy = fmadd(sin_phi, slx, cos_phi * sly) * av;
        m = normalize(mk(-sx, -sy, 1.f));
        pdf = eval(m) * smith_g1(wi, m) * absdot(wi, m) / wi.z;
    }
};

AD float fresnel_cond(float ci, float er, float ei) {
    float ci2 = ci * ci, si2 = 1.f - ci2, si4 = si2 * si2;
    float temp_1 = er * er - ei * ei - si2, a2pb2 = safe_sqrt(temp_1 * temp_1 + 4.f * ei * ei * er * er),
          a = safe_sqrt(.5f * (a2pb2 + temp_1));
    float term_1 = a2pb2 + ci2, term_2 = 2.f * ci * a;
    float r_s = (term_1 - term_2) / (term_1 + term_2);
    float term_3 = a2pb2 * ci2 + si4, term_4 = term_2 * si2;
    float r_p = r_s * (term_3 - term_4) / (term_3 + term_4);
    return 0.5f * (r_s + r_p);
}
AD C3 fresnel3(const DBsdf &b, float ci) {
    return {fresnel_cond(ci, b.eta[0], b.k[0]), fresnel_cond(ci, b.eta[1], b.k[1]), fresnel_cond(ci, b.eta[2], b.k[2])};
}

/* ---------------- leaf BSDFs ---------------- */
/* diffuse.cpp:100-188 */
AD void diffuse_eval_pdf(const DBsdf &d, uint32_t ctx, f3 wi, f3 wo, C3 &val, float &pdf) {
    if (!ctx_on(ctx, BF_DiffuseReflection)) { val = c3(0.f); pdf = 0.f; return; }
    bool a = wi.z > 0.f && wo.z > 0.f;
    C3 v = c3(d.refl) * kInvPi * wo.z;
    float p = kInvPi * wo.z;
    val = csel(a, v, c3(0.f));
    pdf = a ? p : 0.f;
}
AD float diffuse_pdf(uint32_t ctx, f3 wi, f3 wo) {
    if (!ctx_on(ctx, BF_DiffuseReflection)) return 0.f;
    float p = kInvPi * wo.z;
    return (wi.z > 0.f && wo.z > 0.f) ? p : 0.f;
}
AD void diffuse_sample(const DBsdf &d, uint32_t ctx, f3 wi, float u1, float u2, BSample &bs, C3 &w) {
    bool a = wi.z > 0.f;
    if (!ctx_on(ctx, BF_DiffuseReflection)) { w = c3(0.f); return; }
    bs.wo = cosine_hemisphere(u1, u2);
    bs.pdf = kInvPi * bs.wo.z;
    bs.eta = 1.f;
    bs.type = BF_DiffuseReflection;
    w = csel(a && bs.pdf > 0.f, c3(d.refl), c3(0.f));
}

AD void leaf_eval_pdf(const DBsdf &d, uint32_t ctx, f3 wi, f3 wo, C3 &val, float &pdf) {
    if (d.type == BSDF_DIFFUSE) { diffuse_eval_pdf(d, ctx, wi, wo, val, pdf); return; }
    f3 H = normalize(wo + wi);
    bool a = wi.z > 0.f && wo.z > 0.f && dot(wi, H) > 0.f && dot(wo, H) > 0.f;
    if (!ctx_on(ctx, BF_GlossyReflection)) { val = c3(0.f); pdf = 0.f; return; }
    Mf mf(d);
    float D = mf.eval(H);
    a = a && D != 0.f;
    float g1 = mf.smith_g1(wi, H);
    float G = g1 * mf.smith_g1(wo, H);
    float value = D * G / (4.f * wi.z);
    C3 F = fresnel3(d, dot(wi, H));
    C3 v = d.has_spec ? F * (value * c3(d.spec)) : F * value;
    float p = mf.visible ? D * g1 / (4.f * wi.z) : mf.eval(H) * H.z / (4.f * dot(wo, H));
    val = csel(a, v, c3(0.f));
    pdf = a ? p : 0.f;
}

AD float leaf_pdf(const DBsdf &d, uint32_t ctx, f3 wi, f3 wo) {
    if (d.type == BSDF_DIFFUSE) return diffuse_pdf(ctx, wi, wo);
    f3 m = normalize(wo + wi);
    bool a = wi.z > 0.f && wo.z > 0.f && dot(wi, m) > 0.f && dot(wo, m) > 0.f;
    if (!ctx_on(ctx, BF_GlossyReflection)) return 0.f;
    Mf mf(d);
    float r = mf.visible ? mf.eval(m) * mf.smith_g1(wi, m) / (4.f * wi.z) : mf.eval(m) * m.z / (4.f * dot(wo, m));
    return a ? r : 0.f;
}

AD void leaf_sample(const DBsdf &d, uint32_t ctx, f3 wi, float u1, float u2, BSample &bs, C3 &w) {
    bs = bs_zero();
    if (d.type == BSDF_DIFFUSE) { diffuse_sample(d, ctx, wi, u1, u2, bs, w); return; }
    bool a = wi.z > 0.f;
    if (!ctx_on(ctx, BF_GlossyReflection)) { w = c3(0.f); return; }
    Mf mf(d);
    f3 m;
    mf.sample(wi, u1, u2, m, bs.pdf);
    bs.wo = fms3(m, 2.f * dot(wi, m), wi);
    bs.eta = 1.f;
    bs.type = BF_GlossyReflection;
    a = a && bs.pdf != 0.f && bs.wo.z > 0.f;
    float weight = mf.visible ? mf.smith_g1(bs.wo, m)
                              : mf.smith_g1(wi, m) * mf.smith_g1(bs.wo, m) * dot(wi, m) / (wi.z * m.z);
    bs.pdf /= 4.f * dot(bs.wo, m);
    C3 F = fresnel3(d, dot(wi, m));
    C3 ww = csel(d.has_spec, c3(weight) * c3(d.spec), c3(weight));
    w = csel(a, F * ww, c3(0.f));
}

/* ---------------- dispatch incl. twosided ---------------- */
AD uint32_t bsdf_flags(const DBsdf *T, int32_t b) { return b < 0 ? 0u : T[b].flags; }

/*
 * twosided (twosided.cpp:149-296) resolved to ONE leaf call: the leaf BSDF and the
 * frame flip are chosen first, so each dispatch site inlines a single copy of the
 * leaf code instead of one per twosided branch (code size: the hot kernels must
 * fit the instruction cache).  flip: 0 none, 1 back side (negate z), 2 shared
 * nested BSDF (|wi.z|, wo.z carries wi.z's sign).  leaf < 0: the result is zero.
 */
struct TwoSided { int32_t leaf; uint32_t flip; };
AD TwoSided resolve_twosided(const DBsdf *T, int32_t b, f3 wi) {
    const DBsdf &d = T[b];
    if (d.type != BSDF_TWOSIDED) return TwoSided{b, 0u};
    if (d.nested0 == d.nested1) return TwoSided{d.nested0, 2u};
    if (wi.z > 0.f) return TwoSided{d.nested0, 0u};
    if (wi.z < 0.f) return TwoSided{d.nested1, 1u};
    return TwoSided{-1, 0u};   /* wi.z == 0 or NaN: neither side */
}
AD f3 ts_wi(const TwoSided &r, f3 wi) {
    return r.flip == 1u ? mk(wi.x, wi.y, -wi.z) : (r.flip == 2u ? mk(wi.x, wi.y, fabs_(wi.z)) : wi);
}
AD f3 ts_wo(const TwoSided &r, f3 wi, f3 wo) {
    return r.flip == 1u ? mk(wo.x, wo.y, -wo.z) : (r.flip == 2u ? mk(wo.x, wo.y, mulsign(wo.z, wi.z)) : wo);
}

/*
 * Dispatch.  kDiff: the scene's BSDFs are all plain `diffuse` (the host checks), so
 * the call is diffuse.cpp alone -- no twosided resolve, no microfacet code in the
 * kernel (fewer registers), same arithmetic.
 */
template <bool kDiff = false>
AD void bsdf_eval_pdf(const DBsdf *T, int32_t b, uint32_t ctx, f3 wi, f3 wo, bool active, C3 &val, float &pdf) {
    val = c3(0.f); pdf = 0.f;
    if (b < 0 || !active) return;
    if (kDiff) { diffuse_eval_pdf(T[b], ctx, wi, wo, val, pdf); return; }
    const TwoSided r = resolve_twosided(T, b, wi);
    if (r.leaf < 0) return;
    leaf_eval_pdf(T[r.leaf], ctx, ts_wi(r, wi), ts_wo(r, wi, wo), val, pdf);
}

template <bool kDiff = false>
AD float bsdf_pdf(const DBsdf *T, int32_t b, uint32_t ctx, f3 wi, f3 wo, bool active) {
    if (b < 0 || !active) return 0.f;
    if (kDiff) return diffuse_pdf(ctx, wi, wo);
    const TwoSided r = resolve_twosided(T, b, wi);
    if (r.leaf < 0) return 0.f;
    return leaf_pdf(T[r.leaf], ctx, ts_wi(r, wi), ts_wo(r, wi, wo));
}

/*
 * bsdf_pdf with wi fixed, for loops over many wo (the pairwise MIS sums): the twosided
 * resolve, the leaf's microfacet parameters, smith_g1(wi) and 4 wi.z are taken once.
 * smith_g1(wi, m) is G1(wi) unless dot(wi, m) wi.z <= 0, which leaf_pdf's own validity
 * test already zeroes, so row_pdf returns leaf_pdf's value bit for bit (same operations
 * in the same order).
 */
struct PdfRow {
    int32_t leaf;     /* < 0: every pdf is zero */
    uint32_t flip;
    f3 wi, twi;       /* wi and its twosided-resolved form */
    Mf mf;
    float g1, den;    /* smith_g1(twi, .) before its orientation test; 4 twi.z */
    bool diffuse, on; /* leaf type; ctx enables the leaf's lobe */
};
AD PdfRow pdf_row(const DBsdf *T, int32_t b, uint32_t ctx, f3 wi) {
    PdfRow R{-1, 0u, wi, wi, Mf(), 0.f, 1.f, false, false};
    if (b < 0) return R;
    const TwoSided r = resolve_twosided(T, b, wi);
    R.leaf = r.leaf;
    if (r.leaf < 0) return R;
    R.flip = r.flip;
    R.twi = ts_wi(r, wi);
    const DBsdf &d = T[r.leaf];
    R.diffuse = d.type == BSDF_DIFFUSE;
    R.on = ctx_on(ctx, R.diffuse ? BF_DiffuseReflection : BF_GlossyReflection);
    R.mf = Mf(d);
    R.g1 = R.mf.smith_g1(R.twi, R.twi);   /* m = wi passes the orientation test when wi.z != 0 */
    R.den = 4.f * R.twi.z;
    return R;
}
AD float row_pdf(const PdfRow &R, f3 wo, bool active) {
    if (R.leaf < 0 || !active || !R.on) return 0.f;
    const f3 two = ts_wo(TwoSided{R.leaf, R.flip}, R.wi, wo);
    if (R.diffuse) {
        float p = kInvPi * two.z;
        return (R.twi.z > 0.f && two.z > 0.f) ? p : 0.f;
    }
    f3 m = normalize(two + R.twi);
    bool a = R.twi.z > 0.f && two.z > 0.f && dot(R.twi, m) > 0.f && dot(two, m) > 0.f;
    float r = R.mf.visible ? R.mf.eval(m) * R.g1 / R.den : R.mf.eval(m) * m.z / (4.f * dot(two, m));
    return a ? r : 0.f;
}

template <bool kDiff = false>
AD void bsdf_sample(const DBsdf *T, int32_t b, uint32_t ctx, f3 wi, float u1, float u2, bool active, BSample &bs,
                    C3 &w) {
    bs = bs_zero(); w = c3(0.f);
    if (b < 0 || !active) return;
    if (kDiff) { diffuse_sample(T[b], ctx, wi, u1, u2, bs, w); return; }
    const TwoSided r = resolve_twosided(T, b, wi);
    if (r.leaf < 0) return;
    leaf_sample(T[r.leaf], ctx, ts_wi(r, wi), u1, u2, bs, w);
    if (r.flip == 1u) bs.wo.z *= -1.f;
    if (r.flip == 2u) bs.wo.z = mulsign(bs.wo.z, wi.z);
}

/* bsdf_sample(...).type without the sample: leaf_sample sets the lobe's type whether or not the
 * sample is valid, and zero when the BSDF is null, the lane masked, the lobe off in ctx or the
 * twosided resolve finds no side */
template <bool kDiff = false>
AD uint32_t bsdf_sample_type(const DBsdf *T, int32_t b, uint32_t ctx, f3 wi, bool active) {
    if (b < 0 || !active) return 0u;
    int32_t leaf = b;
    if (!kDiff) {
        const TwoSided r = resolve_twosided(T, b, wi);
        if (r.leaf < 0) return 0u;
        leaf = r.leaf;
    }
    const uint32_t lobe = (kDiff || T[leaf].type == BSDF_DIFFUSE) ? BF_DiffuseReflection : BF_GlossyReflection;
    return ctx_on(ctx, lobe) ? lobe : 0u;
}

AD float leaf_roughness(const DBsdf &d) {
    return d.type == BSDF_DIFFUSE ? 1.f : dsqrt(0.5f * (sqr(d.alpha_u) + sqr(d.alpha_v)));
}
template <bool kDiff = false>
AD float bsdf_roughness(const DBsdf *T, int32_t b, f3 wi) {
    if (b < 0) return 0.f;
    if (kDiff) return 1.f;
    const DBsdf &d = T[b];
    if (d.type != BSDF_TWOSIDED) return leaf_roughness(d);
    if (d.nested0 == d.nested1) return leaf_roughness(T[d.nested0]);
    float r = 0.f;
    if (wi.z > 0.f) r = leaf_roughness(T[d.nested0]);
    if (wi.z < 0.f) r = leaf_roughness(T[d.nested1]);
    return r;
}

/* ---------------- emitters ---------------- */
struct DSamp { f3 p, n, d; float pdf, dist; bool delta; int32_t emitter; };
AD DSamp ds_zero() { return DSamp{mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), mk(0.f, 0.f, 0.f), 0.f, 0.f, false, -1}; }

AD DSamp shape_sample_direction(const DShape &s, f3 itp, float u1, float u2) {
    DSamp ds = ds_zero();
    if (s.type == PRIM_RECT) {
        ds.p = xf_point_affine(s.to_world, mk(u1 * 2.f - 1.f, u2 * 2.f - 1.f, 0.f));
        ds.n = ld3(s.frame_n);
        ds.pdf = s.inv_area;
        ds.d = ds.p - itp;
        float d2 = sqnorm(ds.d);
        ds.dist = dsqrt(d2);
        ds.d = ds.d / ds.dist;
        float dp = absdot(ds.d, ds.n);
        float x = d2 / dp;
        ds.pdf *= finite_(x) ? x : 0.f;
        return ds;
    }
    /* sphere */
    f3 c = ld3(s.center);
    f3 dc_v = c - itp;
    float dc_2 = sqnorm(dc_v);
    float radius_adj = s.radius * (s.flip ? (1.f + kRayEps) : (1.f - kRayEps));
    if (dc_2 > sqr(radius_adj)) {
        float inv_dc = rsqrt_(dc_2), stm = s.radius * inv_dc, stm2 = sqr(stm), inv_stm = rcp(stm),
              ctm = safe_sqrt(1.f - stm2);
        float st2 = stm2 > 0.00068523f ? 1.f - sqr(fmadd(ctm - 1.f, u1, 1.f)) : stm2 * u1;
        float ct = safe_sqrt(1.f - st2);
        float ca = st2 * inv_stm + ct * safe_sqrt(fnmadd(st2, sqr(inv_stm), 1.f));
        float sa = safe_sqrt(fnmadd(ca, ca, 1.f));
        float sp, cp;
        sincos_c(u2 * (2.f * kPi), sp, cp);
        Frame3 f;
        f.n = dc_v * -inv_dc;
        coord_sys(f.n, f.s, f.t);
        f3 d = f.to_world(mk(cp * sa, sp * sa, ca));
        ds.p = fma3(d, s.radius, c);
        ds.n = d;
        ds.d = ds.p - itp;
        float d2 = sqnorm(ds.d);
        ds.dist = dsqrt(d2);
        ds.d = ds.d / ds.dist;
        ds.pdf = kInvTwoPi / (1.f - ctm);
        if (ds.dist == 0.f) ds.pdf = 0.f;
    } else {
        f3 d = uniform_sphere(u1, u2);
        ds.p = fma3(d, s.radius, c);
        ds.n = d;
        ds.d = ds.p - itp;
        float d2 = sqnorm(ds.d);
        ds.dist = dsqrt(d2);
        ds.d = ds.d / ds.dist;
        ds.pdf = s.inv_area * d2 / absdot(ds.d, ds.n);
    }
    ds.delta = s.radius == 0.f;
    if (s.flip) ds.n = -ds.n;
    return ds;
}

AD float shape_pdf_direction(const DShape &s, f3 itp, const DSamp &ds) {
    if (s.type == PRIM_SPHERE) {
        f3 c = ld3(s.center);
        float sa = s.radius * rcp(norm(c - itp)), ca = safe_sqrt(1.f - sa * sa);
        return sa < kOneMinusEps ? kInvTwoPi / (1.f - ca) : s.inv_area * sqr(ds.dist) / absdot(ds.d, ds.n);
    }
    float pdf = s.inv_area, dp = absdot(ds.d, ds.n);
    pdf *= dp != 0.f ? (ds.dist * ds.dist) / dp : 0.f;
    return pdf;
}

} // namespace amvpt
