/*
 * transform.h -- mitsuba::Transform4f restated for the host framework:
 * a float matrix and its inverse transpose, composed pairwise exactly as
 * include/mitsuba/core/transform.h:25-330 does (translate / scale / rotate /
 * perspective / look_at keep an analytic inverse; composition multiplies both).
 */
#pragma once
#include <array>
#include <cmath>

namespace mi {

struct Mat4 {
    float m[4][4];
    static Mat4 identity() {
        Mat4 r{};
        for (int i = 0; i < 4; ++i) r.m[i][i] = 1.f;
        return r;
    }
    static Mat4 zero() { Mat4 r{}; return r; }
    Mat4 transpose() const {
        Mat4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.m[i][j] = m[j][i];
        return r;
    }
    Mat4 operator*(const Mat4 &b) const {
        Mat4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j)
                r.m[i][j] = std::fmaf(m[i][3], b.m[3][j], std::fmaf(m[i][2], b.m[2][j], std::fmaf(m[i][1], b.m[1][j], m[i][0] * b.m[0][j])));
        return r;
    }
    /* general 4x4 inverse (cofactor expansion, double internally) */
    Mat4 inverse() const {
        double a[16], inv[16];
        for (int i = 0; i < 16; ++i) a[i] = m[i / 4][i % 4];
        inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] + a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
        inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] - a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
        inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] + a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
        inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] - a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
        inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] - a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
        inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] + a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
        inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] - a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
        inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] + a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
        inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] + a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
        inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] - a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
        inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] + a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
        inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] - a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
        inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] - a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
        inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] + a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
        inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] - a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
        inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] + a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
        double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
        Mat4 r;
        for (int i = 0; i < 16; ++i) r.m[i / 4][i % 4] = (float) (inv[i] / det);
        return r;
    }
    void store(float *out) const {
        for (int i = 0; i < 16; ++i) out[i] = m[i / 4][i % 4];
    }
};

struct V3f { float x, y, z; };

static inline float dot3(V3f a, V3f b) { return std::fmaf(a.z, b.z, std::fmaf(a.y, b.y, a.x * b.x)); }
static inline V3f normalize3(V3f a) {
    float s = 1.f / std::sqrt(dot3(a, a));
    return {a.x * s, a.y * s, a.z * s};
}
static inline V3f cross3(V3f a, V3f b) {
    return {std::fmaf(a.y, b.z, -(a.z * b.y)), std::fmaf(a.z, b.x, -(a.x * b.z)), std::fmaf(a.x, b.y, -(a.y * b.x))};
}

struct Transform4f {
    Mat4 matrix = Mat4::identity();
    Mat4 inverse_transpose = Mat4::identity();

    Transform4f() = default;
    Transform4f(const Mat4 &m, const Mat4 &it) : matrix(m), inverse_transpose(it) {}
    explicit Transform4f(const Mat4 &m) : matrix(m), inverse_transpose(m.inverse().transpose()) {}

    Transform4f operator*(const Transform4f &o) const {
        return Transform4f(matrix * o.matrix, inverse_transpose * o.inverse_transpose);
    }
    Transform4f inverse() const { return Transform4f(inverse_transpose.transpose(), matrix.transpose()); }
    V3f translation() const { return {matrix.m[0][3], matrix.m[1][3], matrix.m[2][3]}; }

    V3f apply_point(V3f p) const { /* transform_affine(Point3f) */
        float r[3];
        for (int i = 0; i < 3; ++i)
            r[i] = std::fmaf(matrix.m[i][2], p.z, std::fmaf(matrix.m[i][1], p.y, std::fmaf(matrix.m[i][0], p.x, matrix.m[i][3])));
        return {r[0], r[1], r[2]};
    }
    V3f apply_point_h(V3f p) const { /* operator*(Point3f) with the homogeneous divide */
        float r[4];
        for (int i = 0; i < 4; ++i)
            r[i] = std::fmaf(matrix.m[i][2], p.z, std::fmaf(matrix.m[i][1], p.y, std::fmaf(matrix.m[i][0], p.x, matrix.m[i][3])));
        return {r[0] / r[3], r[1] / r[3], r[2] / r[3]};
    }
    V3f apply_vector(V3f v) const {
        float r[3];
        for (int i = 0; i < 3; ++i)
            r[i] = std::fmaf(matrix.m[i][2], v.z, std::fmaf(matrix.m[i][1], v.y, matrix.m[i][0] * v.x));
        return {r[0], r[1], r[2]};
    }
    V3f apply_normal(V3f n) const {
        Mat4 inv = inverse_transpose.transpose();
        float r[3];
        for (int i = 0; i < 3; ++i)
            r[i] = std::fmaf(inv.m[2][i], n.z, std::fmaf(inv.m[1][i], n.y, inv.m[0][i] * n.x));
        return {r[0], r[1], r[2]};
    }

    static Transform4f translate(V3f v) {
        Mat4 m = Mat4::identity(), mi = Mat4::identity();
        m.m[0][3] = v.x; m.m[1][3] = v.y; m.m[2][3] = v.z;
        mi.m[0][3] = -v.x; mi.m[1][3] = -v.y; mi.m[2][3] = -v.z;
        return Transform4f(m, mi.transpose());
    }
    static Transform4f scale(V3f v) {
        Mat4 m = Mat4::identity(), mi = Mat4::identity();
        m.m[0][0] = v.x; m.m[1][1] = v.y; m.m[2][2] = v.z;
        mi.m[0][0] = 1.f / v.x; mi.m[1][1] = 1.f / v.y; mi.m[2][2] = 1.f / v.z;
        return Transform4f(m, mi);
    }
    /* dr::rotate<Matrix>(axis, deg_to_rad(angle)) */
    static Transform4f rotate(V3f a, float angle_deg) {
        float ang = angle_deg * (3.14159265358979323846f / 180.f);
        float s = std::sin(ang), c = std::cos(ang), cm = 1.f - c;
        float ax[3] = {a.x, a.y, a.z};
        float sh1[3] = {a.y, a.z, a.x}, sh2[3] = {a.z, a.x, a.y};
        float t0[3], t1[3], t2[3];
        for (int i = 0; i < 3; ++i) {
            t0[i] = std::fmaf(ax[i] * ax[i], cm, c);
            t1[i] = std::fmaf(ax[i] * sh1[i], cm, sh2[i] * s);
            t2[i] = std::fmaf(ax[i] * sh1[i], cm, -(sh2[i] * s));
        }
        Mat4 m = Mat4::identity();
        m.m[0][0] = t0[0]; m.m[0][1] = t2[0]; m.m[0][2] = t1[2];
        m.m[1][0] = t1[0]; m.m[1][1] = t0[1]; m.m[1][2] = t2[1];
        m.m[2][0] = t2[2]; m.m[2][1] = t1[1]; m.m[2][2] = t0[2];
        return Transform4f(m, m);
    }
    static Transform4f perspective(float fov, float near_, float far_) {
        float recip = 1.f / (far_ - near_);
        float tn = std::tan((fov * .5f) * (3.14159265358979323846f / 180.f)), cot = 1.f / tn;
        Mat4 t = Mat4::zero(), it = Mat4::zero();
        t.m[0][0] = cot; t.m[1][1] = cot; t.m[2][2] = far_ * recip; t.m[3][3] = 0.f;
        t.m[2][3] = -near_ * far_ * recip;
        t.m[3][2] = 1.f;
        it.m[0][0] = tn; it.m[1][1] = tn; it.m[2][2] = 0.f; it.m[3][3] = 1.f / near_;
        it.m[2][3] = 1.f;
        it.m[3][2] = (near_ - far_) / (far_ * near_);
        return Transform4f(t, it.transpose());
    }
    static Transform4f look_at(V3f origin, V3f target, V3f up) {
        V3f dir = normalize3({target.x - origin.x, target.y - origin.y, target.z - origin.z});
        V3f left = normalize3(cross3(up, dir));
        V3f new_up = cross3(dir, left);
        Mat4 r = Mat4::identity();
        r.m[0][0] = left.x; r.m[1][0] = left.y; r.m[2][0] = left.z;
        r.m[0][1] = new_up.x; r.m[1][1] = new_up.y; r.m[2][1] = new_up.z;
        r.m[0][2] = dir.x; r.m[1][2] = dir.y; r.m[2][2] = dir.z;
        r.m[0][3] = origin.x; r.m[1][3] = origin.y; r.m[2][3] = origin.z;
        /* inverse_transpose: rows 0..2 hold (left|up|dir) columns, row 3 = -R^T o */
        Mat4 inv = Mat4::identity();
        inv.m[0][0] = left.x; inv.m[0][1] = new_up.x; inv.m[0][2] = dir.x; inv.m[0][3] = 0.f;
        inv.m[1][0] = left.y; inv.m[1][1] = new_up.y; inv.m[1][2] = dir.y; inv.m[1][3] = 0.f;
        inv.m[2][0] = left.z; inv.m[2][1] = new_up.z; inv.m[2][2] = dir.z; inv.m[2][3] = 0.f;
        V3f no = {-origin.x, -origin.y, -origin.z};
        inv.m[3][0] = dot3(left, no);
        inv.m[3][1] = dot3(new_up, no);
        inv.m[3][2] = dot3(dir, no);
        inv.m[3][3] = 1.f;
        return Transform4f(r, inv);
    }
    bool has_scale() const {
        for (int i = 0; i < 3; ++i) {
            float s = 0.f;
            for (int j = 0; j < 3; ++j) s += matrix.m[j][i] * matrix.m[j][i];
            if (std::fabs(s - 1.f) > 1e-3f) return true;
        }
        return false;
    }
};

/* perspective_projection (include/mitsuba/render/sensor.h:319-356) */
static inline Transform4f perspective_projection(const int film_size[2], const int crop_size[2],
                                                 const int crop_offset[2], float fov_x, float near_clip,
                                                 float far_clip) {
    float fsx = (float) film_size[0], fsy = (float) film_size[1];
    float rsx = (float) crop_size[0] / fsx, rsy = (float) crop_size[1] / fsy;
    float rox = (float) crop_offset[0] / fsx, roy = (float) crop_offset[1] / fsy;
    float aspect = fsx / fsy;
    return Transform4f::scale({1.f / rsx, 1.f / rsy, 1.f}) * Transform4f::translate({-rox, -roy, 0.f}) *
           Transform4f::scale({-0.5f, -0.5f * aspect, 1.f}) * Transform4f::translate({-1.f, -1.f / aspect, 0.f}) *
           Transform4f::perspective(fov_x, near_clip, far_clip);
}

} // namespace mi
