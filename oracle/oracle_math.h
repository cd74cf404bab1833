/*
 * oracle_math.h -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * Scalar CPU restatement of the arithmetic primitives the reference's hot path
 * uses.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load the oracle; the product path never links or calls it.
 *
 * Floating-point contract (shared by oracle and product, written separately):
 *   - no FMA contraction (built with -ffp-contract=off); fmaf() exactly where
 *     the reference calls dr::fmadd / fmsub / fnmadd;
 *   - division and sqrt IEEE-correctly rounded; rcp(x) = 1/x, rsqrt = 1/sqrt;
 *   - sincos: Cephes single-precision polynomial (the algorithm Dr.Jit 1.0.5,
 *     the reference's pinned dependency (pyproject.toml:5,17), uses for
 *     llvm_* variants; Dr.Jit is not vendored under /root/reference, so the
 *     exact bits of this restatement vs Dr.Jit are "parity unpinned").
 */
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

namespace orc {

static inline uint32_t f2u(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

static inline float fmadd(float a, float b, float c) { return std::fmaf(a, b, c); }
static inline float fmsub(float a, float b, float c) { return std::fmaf(a, b, -c); }
static inline float fnmadd(float a, float b, float c) { return std::fmaf(-a, b, c); }
static inline float rcp(float x) { return 1.0f / x; }
static inline float rsqrt(float x) { return 1.0f / std::sqrt(x); }
static inline float safe_sqrt(float x) { return std::sqrt(x > 0.f ? x : 0.f); }
static inline float sqr(float x) { return x * x; }
static inline float fmaxf_(float a, float b) { return a > b ? a : b; }  // dr::maximum
static inline float fminf_(float a, float b) { return a < b ? a : b; }  // dr::minimum
/* dr::mulsign(a, b): a with its sign flipped where b's sign bit is set */
static inline float mulsign(float a, float b) { return u2f(f2u(a) ^ (f2u(b) & 0x80000000u)); }
/* dr::mulsign_neg(a, b) = mulsign(a, -b) */
static inline float mulsign_neg(float a, float b) { return u2f(f2u(a) ^ (~f2u(b) & 0x80000000u)); }
static inline float sign(float x) { return mulsign(1.f, x); }
/* dr::lerp(a, b, t) = fmadd(b, t, fnmadd(a, t, a)) */
static inline float lerp(float a, float b, float t) { return fmadd(b, t, fnmadd(a, t, a)); }
static inline bool isfinite_(float x) { return (f2u(x) & 0x7f800000u) != 0x7f800000u; }

static const float Pi = 3.14159265358979323846f;
static const float InvPi = 0.31830988618379067154f;
static const float InvTwoPi = 0.15915494309189533577f;
static const float InvFourPi = 0.07957747154594766788f;
static const float InvSqrtPi = 0.56418958354775628695f;
static const float Epsilon = 5.9604644775390625e-08f;       /* 2^-24 */
static const float RayEpsilon = Epsilon * 1500.f;            /* math.h:18-23 */
static const float ShadowEpsilon = RayEpsilon * 10.f;
static const float Largest = 3.40282346638528859812e+38f;
static const float Infinity = INFINITY;
static const float OneMinusEpsilon = 0.99999994039535522461f;

/* Cephes sincosf (single precision), sign/quadrant logic by bit arithmetic. */
static inline void sincos_(float x, float &s_out, float &c_out) {
    float xa = std::fabs(x);
    int32_t j = (int32_t) (xa * 1.27323954473516268615f);
    j = (j + 1) & ~1;
    float y = (float) j;
    uint32_t sign_sin = (((uint32_t) j) << 29) ^ f2u(x);
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
    s_out = u2f(f2u(rs) ^ (sign_sin & 0x80000000u));
    c_out = u2f(f2u(rc) ^ (sign_cos & 0x80000000u));
    if (!(xa < Infinity)) { s_out = NAN; c_out = NAN; }
}

/*
 * exp / log / erf / erfinv / tan for the Beckmann distribution and anisotropic microfacet
 * sampling (microfacet.h:185-431).  Dr.Jit's own single-precision versions are not vendored,
 * so these are restatements of the published algorithms -- parity unpinned at the last ulp
 * against the reference, pinned by tests/test_oracle_golden.py against libm / math.erf within
 * a few ulp, and bit-identical between this oracle and the device (dmath.h, same operations).
 *   exp    Cephes expf: n = floor(x log2 e + 1/2), two-constant Cody-Waite reduction, degree-5
 *          polynomial, ldexp in two exact halves; 0 below -88.376, inf above +88.376
 *   log    Cephes logf: frexp to [sqrt(1/2), sqrt 2), degree-8 polynomial, Cody-Waite ln 2
 *   erf    |x| < 1: x P(x^2); 1 <= |x| < 4: 1 - exp(-x^2) Q(1/x^2) / |x|; else +-1
 *          (least-squares fits, |error| < 2.1e-7)
 *   erfinv M. Giles, "Approximating the erfinv function" (GPU Computing Gems, 2010), single
 *   tan    sin / cos of the Cephes sincos above
 */
static inline float ldexp_(float y, int n) {
    const int h = n / 2, l = n - h;
    return (y * u2f((uint32_t) (h + 127) << 23)) * u2f((uint32_t) (l + 127) << 23);
}
static inline float exp_(float x) {
    if (x != x) return x;
    if (x > 88.3762626647949f) return Infinity;
    if (x < -88.3762626647949f) return 0.f;
    const float n = std::floor(fmadd(1.44269504088896341f, x, .5f));
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
static inline float log_(float x) {
    if (x != x || x < 0.f) return NAN;
    if (x == 0.f) return -Infinity;
    if (x == Infinity) return Infinity;
    int e_adj = 0;
    if (x < 1.17549435e-38f) { x *= 8388608.f; e_adj = -23; }
    const uint32_t u = f2u(x);
    int e = (int) ((u >> 23) & 0xffu) - 126 + e_adj;
    float m = u2f((u & 0x007fffffu) | 0x3f000000u);   /* [0.5, 1) */
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
static inline float erf_(float x) {
    const float a = std::fabs(x);
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
static inline float erfinv_(float x) {
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
        w = std::sqrt(w) - 3.f;
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
static inline float tan_(float x) {
    float s, c;
    sincos_(x, s, c);
    return s / c;
}

/* ---------------- vectors ---------------- */
struct V2 { float x, y; };
struct V3 {
    float x, y, z;
    float &operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
static inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
static inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
static inline V3 operator*(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
static inline V3 operator*(float s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
static inline V3 operator*(V3 a, V3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static inline V3 operator/(V3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
static inline V3 fmadd(V3 a, float b, V3 c) { return {fmadd(a.x, b, c.x), fmadd(a.y, b, c.y), fmadd(a.z, b, c.z)}; }
static inline V3 fmadd(V3 a, V3 b, V3 c) { return {fmadd(a.x, b.x, c.x), fmadd(a.y, b.y, c.y), fmadd(a.z, b.z, c.z)}; }
static inline V3 fmsub(V3 a, float b, V3 c) { return {fmsub(a.x, b, c.x), fmsub(a.y, b, c.y), fmsub(a.z, b, c.z)}; }
/* dr::dot: a.x*b.x, then fmadd over the remaining components */
static inline float dot(V3 a, V3 b) { return fmadd(a.z, b.z, fmadd(a.y, b.y, a.x * b.x)); }
static inline float absdot(V3 a, V3 b) { return std::fabs(dot(a, b)); }
static inline float squared_norm(V3 a) { return dot(a, a); }
static inline float norm(V3 a) { return std::sqrt(squared_norm(a)); }
static inline V3 normalize(V3 a) { return a * rsqrt(squared_norm(a)); }
/* dr::cross with fmsub */
static inline V3 cross(V3 a, V3 b) {
    return {fmsub(a.y, b.z, a.z * b.y), fmsub(a.z, b.x, a.x * b.z), fmsub(a.x, b.y, a.y * b.x)};
}
static inline float hmax(V3 a) { return fmaxf_(fmaxf_(a.x, a.y), a.z); }

/* Transform4f applied with the reference's fmadd chains (transform.h:117-170).
 * m is row-major 4x4. */
static inline V3 xform_point_affine(const float *m, V3 p) {
    V3 r;
    for (int i = 0; i < 3; ++i)
        r[i] = fmadd(m[i * 4 + 2], p.z, fmadd(m[i * 4 + 1], p.y, fmadd(m[i * 4 + 0], p.x, m[i * 4 + 3])));
    return r;
}
static inline V3 xform_point(const float *m, V3 p) { /* with homogeneous divide */
    float r[4];
    for (int i = 0; i < 4; ++i)
        r[i] = fmadd(m[i * 4 + 2], p.z, fmadd(m[i * 4 + 1], p.y, fmadd(m[i * 4 + 0], p.x, m[i * 4 + 3])));
    return {r[0] / r[3], r[1] / r[3], r[2] / r[3]};
}
static inline V3 xform_vector(const float *m, V3 v) {
    V3 r;
    for (int i = 0; i < 3; ++i)
        r[i] = fmadd(m[i * 4 + 2], v.z, fmadd(m[i * 4 + 1], v.y, m[i * 4 + 0] * v.x));
    return r;
}
/* normal: multiply by inverse_transpose = transpose(to_object) */
static inline V3 xform_normal_inv(const float *to_object, V3 n) {
    V3 r;
    for (int i = 0; i < 3; ++i)
        r[i] = fmadd(to_object[2 * 4 + i], n.z, fmadd(to_object[1 * 4 + i], n.y, to_object[0 * 4 + i] * n.x));
    return r;
}

/* vector.h:116-136 */
static inline void coordinate_system(V3 n, V3 &s, V3 &t) {
    float sg = sign(n.z), a = -rcp(sg + n.z), b = n.x * n.y * a;
    s = {mulsign(sqr(n.x) * a, n.z) + 1.f, mulsign(b, n.z), mulsign_neg(n.x, n.z)};
    t = {b, fmadd(n.y, n.y * a, sg), -n.y};
}

struct Frame {
    V3 s, t, n;
    V3 to_local(V3 v) const { return {dot(v, s), dot(v, t), dot(v, n)}; }
    V3 to_world(V3 v) const { return fmadd(n, v.z, fmadd(t, v.y, s * v.x)); }
};
static inline Frame frame_from(V3 n) { Frame f; f.n = n; coordinate_system(n, f.s, f.t); return f; }

/* ---------------- RNG: TEA (random.h:77-90) + PCG32 (Dr.Jit) ---------------- */
static inline void tea(uint32_t v0, uint32_t v1, int rounds, uint32_t &o0, uint32_t &o1) {
    uint32_t sum = 0;
    for (int i = 0; i < rounds; ++i) {
        sum += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    o0 = v0; o1 = v1;
}

struct PCG32 {
    uint64_t state = 0x853c49e6748fea9bULL, inc = 0xda3e39cb94b95bdbULL;
    uint32_t next_u32() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dULL + inc;
        uint32_t xs = (uint32_t) (((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t) (old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    float next_1d() { return u2f((next_u32() >> 9) | 0x3f800000u) - 1.f; }
    void seed(uint64_t initstate, uint64_t initseq) {
        state = 0;
        inc = (initseq << 1) | 1u;
        next_u32();
        state += initstate;
        next_u32();
    }
};

/* ---------------- Gaussian reconstruction filter (gaussian.cpp:48-100) ---------------- */
/* Dr.Jit estrin_impl restated: pairwise fmadd levels in x, x^2, x^4, ... */
template <int N> static inline float estrin(float x, const float *c) {
    constexpr int n_rec = (N - 1) / 2, n_fma = N / 2;
    float rec[n_rec + 1];
    for (int i = 0; i < n_fma; ++i) rec[i] = fmadd(x, c[2 * i + 1], c[2 * i]);
    if (n_rec == n_fma) rec[n_rec] = c[N - 1];
    if constexpr (n_rec == 0) return rec[0];
    else return estrin<n_rec + 1>(x * x, rec);
}
template <> inline float estrin<1>(float, const float *c) { return c[0]; }

struct Gaussian {
    float stddev, radius, coeff[10];
    void init(float sd) {
        stddev = sd; radius = 4.f * sd;
        static const double cd[10] = {9.992604880e-1, -4.977025247e-1, 1.222248550e-1,
                                      -1.932406282e-2, 2.136713061e-3, -1.679873860e-4,
                                      9.202145248e-6, -3.329417433e-7, 7.128382794e-9,
                                      -6.821193280e-11};
        double scale = 1;
        for (int i = 0; i < 10; ++i) {
            coeff[i] = (float) (cd[i] * scale);
            scale /= ((double) stddev * (double) stddev);
        }
        coeff[0] -= estrin<10>(radius * radius, coeff);
    }
    float eval(float x) const { return fmaxf_(estrin<10>(x * x, coeff), 0.f); }
};

} // namespace orc
