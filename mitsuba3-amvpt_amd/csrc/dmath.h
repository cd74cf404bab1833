/*
 * dmath.h -- device arithmetic for the AMVPT kernels (gfx950).
 *
 * Floating-point contract (see DESIGN.md "Numerics"): the kernels are built
 * with -ffp-contract=off and correctly-rounded f32 divide/sqrt; an FMA is
 * issued exactly where the reference writes dr::fmadd / fmsub / fnmadd, so a
 * lane's arithmetic is a fixed sequence of IEEE operations.  Transcendentals
 * come from the single-precision Cephes sincos below (the algorithm of the
 * reference's pinned Dr.Jit 1.0.5 llvm backend), never from ocml, so the
 * result does not depend on the device math library.
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amvpt {

#define AD __device__ __forceinline__

AD float fmadd(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
AD float fmsub(float a, float b, float c) { return __builtin_fmaf(a, b, -c); }
AD float fnmadd(float a, float b, float c) { return __builtin_fmaf(-a, b, c); }
AD float rcp(float x) { return 1.0f / x; }
AD float dsqrt(float x) { return __builtin_sqrtf(x); }
AD float rsqrt_(float x) { return 1.0f / __builtin_sqrtf(x); }
AD float safe_sqrt(float x) { return __builtin_sqrtf(x > 0.f ? x : 0.f); }
AD float sqr(float x) { return x * x; }
AD float vmax(float a, float b) { return a > b ? a : b; }   /* dr::maximum */
AD float vmin(float a, float b) { return a < b ? a : b; }   /* dr::minimum */
AD float fabs_(float x) { return __builtin_fabsf(x); }
AD uint32_t fbits(float f) { return __float_as_uint(f); }
AD float bitsf(uint32_t u) { return __uint_as_float(u); }
AD float mulsign(float a, float b) { return bitsf(fbits(a) ^ (fbits(b) & 0x80000000u)); }
AD float mulsign_neg(float a, float b) { return bitsf(fbits(a) ^ (~fbits(b) & 0x80000000u)); }
AD float lerp_(float a, float b, float t) { return fmadd(b, t, fnmadd(a, t, a)); }
AD bool finite_(float x) { return (fbits(x) & 0x7f800000u) != 0x7f800000u; }

constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.31830988618379067154f;
constexpr float kInvTwoPi = 0.15915494309189533577f;
constexpr float kInvFourPi = 0.07957747154594766788f;
constexpr float kEps = 5.9604644775390625e-08f;
constexpr float kRayEps = kEps * 1500.f;
constexpr float kShadowEps = kRayEps * 10.f;
constexpr float kLargest = 3.40282346638528859812e+38f;
constexpr float kOneMinusEps = 0.99999994039535522461f;
#define kInf __builtin_huge_valf()

/* Cephes single-precision sincos with bit-level quadrant / sign handling. */
AD void sincos_c(float x, float &s_out, float &c_out) {
    float xa = fabs_(x);
    int32_t j = (int32_t) (xa * 1.27323954473516268615f);
    j = (j + 1) & ~1;
    float y = (float) j;
    uint32_t sign_sin = (((uint32_t) j) << 29) ^ fbits(x);
    uint32_t sign_cos = ((uint32_t) ~(j - 2)) << 29;
    float r = fnmadd(y, 0.78515625f, xa);
    r = fnmadd(y, 2.4187564849853515625e-4f, r);
    r = fnmadd(y, 3.77489497744594108e-8f, r);
    float z = r * r;
    float s = fmadd(z * z, -1.9515295891e-4f, fmadd(z, 8.3321608736e-3f, -1.6666654611e-1f)) * z;
    float c = fmadd(z * z, 2.443315711809948e-5f, fmadd(z, -1.388731625493765e-3f, 4.166664568298827e-2f)) * z;
    s = fmadd(s, r, r);
    c = fmadd(c, z, fmadd(z, -0.5f, 1.f));
    bool poly = (j & 2) == 0;
    float rs = poly ? s : c, rc = poly ? c : s;
    s_out = bitsf(fbits(rs) ^ (sign_sin & 0x80000000u));
    c_out = bitsf(fbits(rc) ^ (sign_cos & 0x80000000u));
    if (!(xa < kInf)) { s_out = __builtin_nanf(""); c_out = __builtin_nanf(""); }
}

/*
 * exp / log / erf / erfinv / tan for the Beckmann distribution and anisotropic microfacet
 * sampling (microfacet.h:185-431): Cephes expf / logf, a fitted erf (|x| < 1: x P(x^2), below 4:
 * 1 - exp(-x^2) Q(1/x^2) / |x|, |error| < 2.1e-7), M. Giles' single-precision erfinv and
 * tan = sin / cos -- the same operation sequences as the CPU parity checker's restatements, so
 * the two agree bit for bit.
 */
AD float ldexp_(float y, int n) {
    const int h = n / 2, l = n - h;
    return (y * bitsf((uint32_t) (h + 127) << 23)) * bitsf((uint32_t) (l + 127) << 23);
}
AD float exp_(float x) {
    if (x != x) return x;
    if (x > 88.3762626647949f) return kInf;
    if (x < -88.3762626647949f) return 0.f;
    const float n = __builtin_floorf(fmadd(1.44269504088896341f, x, .5f));
    float r = fnmadd(n, 0.693359375f, x);
    r = fnmadd(n, -2.12194440e-4f, r);
    float p = fmadd(r, 1.9875691500e-4f, 1.3981999507e-3f);
    p = fmadd(p, r, 8.3334519073e-3f);
    p = fmadd(p, r, 4.1665795894e-2f);
    p = fmadd(p, r, 1.6666665459e-1f);
    p = fmadd(p, r, 5.0000001201e-1f);
    const float y = fmadd(p, r * r, r + 1.f);
    return ldexp_(y, (int) n);
}
AD float log_(float x) {
    if (x != x || x < 0.f) return __builtin_nanf("");
    if (x == 0.f) return -kInf;
    if (x == kInf) return kInf;
    int e_adj = 0;
    if (x < 1.17549435e-38f) { x *= 8388608.f; e_adj = -23; }
    const uint32_t u = fbits(x);
    int e = (int) ((u >> 23) & 0xffu) - 126 + e_adj;
    float m = bitsf((u & 0x007fffffu) | 0x3f000000u);   /* [0.5, 1) */
    if (m < 0.707106781186547524f) { e -= 1; m = m + m - 1.f; }
    else m = m - 1.f;
    const float z = m * m;
    float p = fmadd(m, 7.0376836292e-2f, -1.1514610310e-1f);
    p = fmadd(p, m, 1.1676998740e-1f);
    p = fmadd(p, m, -1.2420140846e-1f);
    p = fmadd(p, m, 1.4249322787e-1f);
    p = fmadd(p, m, -1.6668057665e-1f);
    p = fmadd(p, m, 2.0000714765e-1f);
    p = fmadd(p, m, -2.4999993993e-1f);
    p = fmadd(p, m, 3.3333331174e-1f);
    const float fe = (float) e;
    float y = (p * m) * z;
    y = fmadd(fe, -2.12194440e-4f, y);
    y = fmadd(z, -0.5f, y);
    return fmadd(fe, 0.693359375f, m + y);
}
AD float erf_(float x) {
    const float a = fabs_(x);
    float r;
    if (a < 1.f) {
        const float t = x * x;
        float p = fmadd(t, 7.93334984e-05f, -0.000803480507f);
        p = fmadd(p, t, 0.00519121392f);
        p = fmadd(p, t, -0.026855398f);
        p = fmadd(p, t, 0.112836257f);
        p = fmadd(p, t, -0.376126289f);
        p = fmadd(p, t, 1.12837923f);
        return p * x;
    }
    if (a < 4.f) {
        const float s = 1.f / (a * a);
        float q = fmadd(s, 0.208238602f, -1.215765f);
        q = fmadd(q, s, 3.14549613f);
        q = fmadd(q, s, -4.78043795f);
        q = fmadd(q, s, 4.79150534f);
        q = fmadd(q, s, -3.40518451f);
        q = fmadd(q, s, 1.84398246f);
        q = fmadd(q, s, -0.850101471f);
        q = fmadd(q, s, 0.407034457f);
        q = fmadd(q, s, -0.281359404f);
        q = fmadd(q, s, 0.564175129f);
        r = 1.f - exp_(-(a * a)) * q / a;
    } else {
        r = a == a ? 1.f : a;
    }
    return mulsign(r, x);
}
AD float erfinv_(float x) {
    float w = -log_((1.f - x) * (1.f + x)), p;
    if (w < 5.f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = fmadd(p, w, 3.43273939e-07f);
        p = fmadd(p, w, -3.5233877e-06f);
        p = fmadd(p, w, -4.39150654e-06f);
        p = fmadd(p, w, 0.00021858087f);
        p = fmadd(p, w, -0.00125372503f);
        p = fmadd(p, w, -0.00417768164f);
        p = fmadd(p, w, 0.246640727f);
        p = fmadd(p, w, 1.50140941f);
    } else {
        w = __builtin_sqrtf(w) - 3.f;
        p = -0.000200214257f;
        p = fmadd(p, w, 0.000100950558f);
        p = fmadd(p, w, 0.00134934322f);
        p = fmadd(p, w, -0.00367342844f);
        p = fmadd(p, w, 0.00573950773f);
        p = fmadd(p, w, -0.0076224613f);
        p = fmadd(p, w, 0.00943887047f);
        p = fmadd(p, w, 1.00167406f);
        p = fmadd(p, w, 2.83297682f);
    }
    return p * x;
}
AD float tan_(float x) {
    float s, c;
    sincos_c(x, s, c);
    return s / c;
}

struct f3 { float x, y, z; };
AD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
AD f3 operator+(f3 a, f3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
AD f3 operator-(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
AD f3 operator-(f3 a) { return {-a.x, -a.y, -a.z}; }
AD f3 operator*(f3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
AD f3 operator*(float s, f3 a) { return {s * a.x, s * a.y, s * a.z}; }
AD f3 operator*(f3 a, f3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
AD f3 operator/(f3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
AD f3 fma3(f3 a, float b, f3 c) { return {fmadd(a.x, b, c.x), fmadd(a.y, b, c.y), fmadd(a.z, b, c.z)}; }
AD f3 fma3(f3 a, f3 b, f3 c) { return {fmadd(a.x, b.x, c.x), fmadd(a.y, b.y, c.y), fmadd(a.z, b.z, c.z)}; }
AD f3 fms3(f3 a, float b, f3 c) { return {fmsub(a.x, b, c.x), fmsub(a.y, b, c.y), fmsub(a.z, b, c.z)}; }
AD float dot(f3 a, f3 b) { return fmadd(a.z, b.z, fmadd(a.y, b.y, a.x * b.x)); }
AD float absdot(f3 a, f3 b) { return fabs_(dot(a, b)); }
AD float sqnorm(f3 a) { return dot(a, a); }
AD float norm(f3 a) { return dsqrt(sqnorm(a)); }
AD f3 normalize(f3 a) { return a * rsqrt_(sqnorm(a)); }
AD f3 cross(f3 a, f3 b) {
    return {fmsub(a.y, b.z, a.z * b.y), fmsub(a.z, b.x, a.x * b.z), fmsub(a.x, b.y, a.y * b.x)};
}
AD float hmax3(f3 a) { return vmax(vmax(a.x, a.y), a.z); }
AD f3 ld3(const float *p) { return {p[0], p[1], p[2]}; }

/* Transform4f (transform.h:117-170); m holds rows (4 floats each). */
AD f3 xf_point_affine(const float *m, f3 p) {
    return {fmadd(m[2], p.z, fmadd(m[1], p.y, fmadd(m[0], p.x, m[3]))),
            fmadd(m[6], p.z, fmadd(m[5], p.y, fmadd(m[4], p.x, m[7]))),
            fmadd(m[10], p.z, fmadd(m[9], p.y, fmadd(m[8], p.x, m[11])))};
}
AD f3 xf_point(const float *m, f3 p) {
    float r0 = fmadd(m[2], p.z, fmadd(m[1], p.y, fmadd(m[0], p.x, m[3])));
    float r1 = fmadd(m[6], p.z, fmadd(m[5], p.y, fmadd(m[4], p.x, m[7])));
    float r2 = fmadd(m[10], p.z, fmadd(m[9], p.y, fmadd(m[8], p.x, m[11])));
    float r3 = fmadd(m[14], p.z, fmadd(m[13], p.y, fmadd(m[12], p.x, m[15])));
    return {r0 / r3, r1 / r3, r2 / r3};
}
AD f3 xf_vector(const float *m, f3 v) {
    return {fmadd(m[2], v.z, fmadd(m[1], v.y, m[0] * v.x)),
            fmadd(m[6], v.z, fmadd(m[5], v.y, m[4] * v.x)),
            fmadd(m[10], v.z, fmadd(m[9], v.y, m[8] * v.x))};
}

/* coordinate_system (vector.h:116-136) */
AD void coord_sys(f3 n, f3 &s, f3 &t) {
    float sg = mulsign(1.f, n.z), a = -rcp(sg + n.z), b = n.x * n.y * a;
    s = {mulsign(sqr(n.x) * a, n.z) + 1.f, mulsign(b, n.z), mulsign_neg(n.x, n.z)};
    t = {b, fmadd(n.y, n.y * a, sg), -n.y};
}

struct Frame3 {
    f3 s, t, n;
    AD f3 to_local(f3 v) const { return {dot(v, s), dot(v, t), dot(v, n)}; }
    AD f3 to_world(f3 v) const { return fma3(n, v.z, fma3(t, v.y, s * v.x)); }
};

/* Sample generation: TEA (random.h:77-90) and Dr.Jit PCG32. */
AD void tea4(uint32_t v0, uint32_t v1, uint32_t &o0, uint32_t &o1) {
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    o0 = v0; o1 = v1;
}

struct Pcg {
    uint64_t state, inc;
    AD uint32_t next_u32() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t) (((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t) (old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    AD float next_1d() { return bitsf((next_u32() >> 9) | 0x3f800000u) - 1.f; }
    AD void seed(uint32_t initstate, uint32_t initseq) {
        state = 0;
        inc = (((uint64_t) initseq) << 1) | 1u;
        next_u32();
        state += (uint64_t) initstate;
        next_u32();
    }
};

/* Sampler for lane `lane` of a pass seeded with `seed_value` (sampler.cpp:125-144). */
AD Pcg lane_rng(uint32_t seed_value, uint32_t lane) {
    uint32_t v0, v1;
    tea4(seed_value, lane, v0, v1);
    Pcg r;
    r.seed(v0, v1);
    return r;
}

/* Gaussian filter: Remez polynomial of x^2 by Dr.Jit's Estrin levels (gaussian.cpp:94-101). */
struct FilterCoeffs { float c[10]; float radius; };
AD float gaussian_eval(const FilterCoeffs &f, float x) {
    float x2 = x * x;
    const float *c = f.c;
    float r0 = fmadd(x2, c[1], c[0]), r1 = fmadd(x2, c[3], c[2]), r2 = fmadd(x2, c[5], c[4]),
          r3 = fmadd(x2, c[7], c[6]), r4 = fmadd(x2, c[9], c[8]);
    float x4 = x2 * x2;
    float q0 = fmadd(x4, r1, r0), q1 = fmadd(x4, r3, r2), q2 = r4;
    float x8 = x4 * x4;
    float w0 = fmadd(x8, q1, q0), w1 = q2;
    float x16 = x8 * x8;
    return vmax(fmadd(x16, w1, w0), 0.f);
}
/* gaussian_eval at two arguments as packed-f32 operations (v_pk_mul_f32 / v_pk_fma_f32 are per-element IEEE, so
 * each element is gaussian_eval's value bit for bit): the row splat's filter weights, two per instruction */
typedef float f2v_t __attribute__((ext_vector_type(2)));
AD f2v_t gaussian_eval2(const FilterCoeffs &f, f2v_t x) {
    const f2v_t x2 = x * x;
    const float *c = f.c;
    auto pf = [](f2v_t a, f2v_t b, f2v_t d) { return __builtin_elementwise_fma(a, b, d); };
    const f2v_t r0 = pf(x2, (f2v_t) c[1], (f2v_t) c[0]), r1 = pf(x2, (f2v_t) c[3], (f2v_t) c[2]),
                r2 = pf(x2, (f2v_t) c[5], (f2v_t) c[4]), r3 = pf(x2, (f2v_t) c[7], (f2v_t) c[6]),
                r4 = pf(x2, (f2v_t) c[9], (f2v_t) c[8]);
    const f2v_t x4 = x2 * x2;
    const f2v_t q0 = pf(x4, r1, r0), q1 = pf(x4, r3, r2), q2 = r4;
    const f2v_t x8 = x4 * x4;
    const f2v_t w0 = pf(x8, q1, q0), w1 = q2;
    const f2v_t x16 = x8 * x8;
    const f2v_t v = pf(x16, w1, w0);
    return f2v_t{vmax(v.x, 0.f), vmax(v.y, 0.f)};
}

/* Warps (warp.h) */
AD void disk_concentric(float u, float v, float &ox, float &oy) {
    float x = fmsub(2.f, u, 1.f), y = fmsub(2.f, v, 1.f);
    bool is_zero = x == 0.f && y == 0.f, q13 = fabs_(x) < fabs_(y);
    float r = q13 ? y : x, rp = q13 ? x : y;
    float phi = (0.25f * kPi) * rp / r;
    if (q13) phi = (0.5f * kPi) - phi;
    if (is_zero) phi = 0.f;
    float s, c;
    sincos_c(phi, s, c);
    ox = r * c; oy = r * s;
}
AD f3 cosine_hemisphere(float u, float v) {
    float x, y;
    disk_concentric(u, v, x, y);
    return {x, y, safe_sqrt(1.f - fmadd(y, y, x * x))};
}
/* warp::square_to_uniform_sphere (warp.h:249-255): z = 1 - 2 v, r = circ(z), phi = 2 pi u */
AD f3 uniform_sphere(float u, float v) {
    const float z = fmadd(-2.f, v, 1.f);
    const float q = fmadd(-z, z, 1.f);
    const float r = dsqrt(q > 0.f ? q : 0.f);   /* circ = safe_sqrt(1 - z^2) */
    float s, c;
    sincos_c(u * (2.f * kPi), s, c);
    return {r * c, r * s, z};
}

} // namespace amvpt
