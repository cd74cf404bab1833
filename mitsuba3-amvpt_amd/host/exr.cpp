/*
 * exr.cpp -- OpenEXR writer/reader for developed films (float32, uncompressed
 * scanlines, channels Y or R,G,B[,A]).  Replaces the reference's Bitmap/OpenEXR path
 * used by Film::write (src/films/hdrfilm.cpp:420-546, OpenEXR submodule not vendored).
 */
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/amvpt_host.h"

void amvpt_host_set_error(const std::string &msg);

namespace {
void put_bytes(std::vector<uint8_t> &b, const void *p, size_t n) {
    const uint8_t *c = (const uint8_t *) p;
    b.insert(b.end(), c, c + n);
}
void put_i32(std::vector<uint8_t> &b, int32_t v) { put_bytes(b, &v, 4); }
void put_str(std::vector<uint8_t> &b, const char *s) { put_bytes(b, s, std::strlen(s) + 1); }
void attr(std::vector<uint8_t> &b, const char *name, const char *type, const std::vector<uint8_t> &v) {
    put_str(b, name);
    put_str(b, type);
    put_i32(b, (int32_t) v.size());
    b.insert(b.end(), v.begin(), v.end());
}
const char *kNames1[] = {"Y"};
const char *kNames3[] = {"B", "G", "R"};
const char *kNames4[] = {"A", "B", "G", "R"};
/* channel index in the interleaved (R,G,B[,A]) source for each sorted EXR channel */
const int kSrc1[] = {0};
const int kSrc3[] = {2, 1, 0};
const int kSrc4[] = {3, 2, 1, 0};
const char *name_of(uint32_t c, uint32_t k) { return c == 1 ? kNames1[k] : c == 3 ? kNames3[k] : kNames4[k]; }
int src_of(uint32_t c, uint32_t k) { return c == 1 ? kSrc1[k] : c == 3 ? kSrc3[k] : kSrc4[k]; }
int fail(const std::string &msg) {
    amvpt_host_set_error(msg);
    return -1;
}
} // namespace

extern "C" int amvpt_host_write_exr(const char *path, const float *data, uint32_t w, uint32_t h, uint32_t c) {
    if (c != 1 && c != 3 && c != 4) return fail("write_exr: channel count must be 1, 3 or 4");
    if (!w || !h) return fail("write_exr: empty image");
    std::vector<uint8_t> b;
    put_i32(b, 20000630);
    put_i32(b, 2);
    std::vector<uint8_t> v;
    for (uint32_t k = 0; k < c; ++k) {
        put_str(v, name_of(c, k));
        put_i32(v, 2);                 /* FLOAT */
        uint8_t lin[4] = {0, 0, 0, 0}; /* pLinear + reserved */
        put_bytes(v, lin, 4);
        put_i32(v, 1);
        put_i32(v, 1);
    }
    v.push_back(0);
    attr(b, "channels", "chlist", v);
    attr(b, "compression", "compression", std::vector<uint8_t>{0});
    v.clear();
    put_i32(v, 0); put_i32(v, 0); put_i32(v, (int32_t) w - 1); put_i32(v, (int32_t) h - 1);
    attr(b, "dataWindow", "box2i", v);
    attr(b, "displayWindow", "box2i", v);
    attr(b, "lineOrder", "lineOrder", std::vector<uint8_t>{0});
    v.clear();
    float one = 1.f, zero[2] = {0.f, 0.f};
    put_bytes(v, &one, 4);
    attr(b, "pixelAspectRatio", "float", v);
    v.clear();
    put_bytes(v, zero, 8);
    attr(b, "screenWindowCenter", "v2f", v);
    v.clear();
    put_bytes(v, &one, 4);
    attr(b, "screenWindowWidth", "float", v);
    b.push_back(0);
    const size_t line_bytes = (size_t) w * c * 4;
    uint64_t off = b.size() + 8ull * h;
    for (uint32_t y = 0; y < h; ++y) {
        put_bytes(b, &off, 8);
        off += 8 + line_bytes;
    }
    std::vector<float> line((size_t) w * c);
    for (uint32_t y = 0; y < h; ++y) {
        put_i32(b, (int32_t) y);
        put_i32(b, (int32_t) line_bytes);
        for (uint32_t k = 0; k < c; ++k) {
            int src = src_of(c, k);
            for (uint32_t x = 0; x < w; ++x) line[(size_t) k * w + x] = data[((size_t) y * w + x) * c + src];
        }
        put_bytes(b, line.data(), line_bytes);
    }
    FILE *f = std::fopen(path, "wb");
    if (!f) return fail(std::string("write_exr: cannot open ") + path);
    size_t n = std::fwrite(b.data(), 1, b.size(), f);
    std::fclose(f);
    return n == b.size() ? 0 : fail(std::string("write_exr: short write to ") + path);
}

/* Reads files produced by amvpt_host_write_exr (same layout). */
extern "C" int amvpt_host_read_exr(const char *path, float *data, uint32_t w, uint32_t h, uint32_t c) {
    if (c != 1 && c != 3 && c != 4) return fail("read_exr: channel count must be 1, 3 or 4");
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(std::string("read_exr: cannot open ") + path);
    std::vector<uint8_t> b;
    uint8_t buf[65536];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) b.insert(b.end(), buf, buf + n);
    std::fclose(f);
    if (b.size() < 8) return fail("read_exr: truncated file");
    int32_t magic;
    std::memcpy(&magic, b.data(), 4);
    if (magic != 20000630) return fail("read_exr: not an OpenEXR file");
    size_t p = 8;
    while (p < b.size() && b[p] != 0) {
        std::string name((const char *) &b[p]);
        p += name.size() + 1;
        std::string type((const char *) &b[p]);
        p += type.size() + 1;
        int32_t sz;
        std::memcpy(&sz, &b[p], 4);
        p += 4 + (size_t) sz;
    }
    p += 1 + 8ull * h;
    const size_t line_bytes = (size_t) w * c * 4;
    for (uint32_t y = 0; y < h; ++y) {
        if (p + 8 + line_bytes > b.size()) return fail("read_exr: truncated scanline data");
        p += 8;
        const float *line = (const float *) &b[p];
        for (uint32_t k = 0; k < c; ++k) {
            int dst = src_of(c, k);
            for (uint32_t x = 0; x < w; ++x) data[((size_t) y * w + x) * c + dst] = line[(size_t) k * w + x];
        }
        p += line_bytes;
    }
    return 0;
}
