/*
 * meshio.cpp -- triangle-mesh files for the `obj` and `ply` shape plugins.
 *
 * OBJ follows src/shapes/obj.cpp:148-406: positions through to_world
 * (transform_affine), normals through its inverse transpose and normalised,
 * texture coordinates flipped vertically unless flip_tex_coords = false,
 * vertices de-duplicated by their (v, vt, vn) index triple in first-use order,
 * polygons fan-triangulated as (v0, v[k-1], v[k]); face_normals = true drops the
 * vertex normals.
 * PLY follows src/shapes/ply.cpp:150-450: ascii / binary_little_endian /
 * binary_big_endian, vertex x y z [nx ny nz] [u v | s t | texture_u texture_v],
 * triangle faces (vertex_indices / vertex_index lists of 3), flip_tex_coords
 * default false.
 * Missing vertex normals (and face_normals = false) are recomputed with the
 * angle-weighted scheme of Mesh::recompute_vertex_normals (mesh.cpp:331-410,
 * JIT branch); that path is unpinned (Dr.Jit's acos is not vendored).
 */
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "meshio.h"

namespace mi {

static V3f nrm3(V3f v) {
    float l2 = std::fmaf(v.z, v.z, std::fmaf(v.y, v.y, v.x * v.x));
    float r = 1.f / std::sqrt(l2);
    return {v.x * r, v.y * r, v.z * r};
}
static V3f sub3(V3f a, V3f b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }

void recompute_vertex_normals(MeshData &m) {
    const size_t nv = m.pos.size() / 3, nf = m.faces.size() / 3;
    std::vector<float> acc(nv * 3, 0.f);
    auto P = [&](uint32_t i) { return V3f{m.pos[3 * i], m.pos[3 * i + 1], m.pos[3 * i + 2]}; };
    for (size_t f = 0; f < nf; ++f) {
        const uint32_t fi[3] = {m.faces[3 * f], m.faces[3 * f + 1], m.faces[3 * f + 2]};
        const V3f v[3] = {P(fi[0]), P(fi[1]), P(fi[2])};
        const V3f e1 = sub3(v[1], v[0]), e2 = sub3(v[2], v[0]);
        const V3f n = nrm3({std::fmaf(e1.y, e2.z, -(e1.z * e2.y)), std::fmaf(e1.z, e2.x, -(e1.x * e2.z)),
                            std::fmaf(e1.x, e2.y, -(e1.y * e2.x))});
        for (int i = 0; i < 3; ++i) {
            const V3f d0 = nrm3(sub3(v[(i + 1) % 3], v[i])), d1 = nrm3(sub3(v[(i + 2) % 3], v[i]));
            float c = std::fmaf(d0.z, d1.z, std::fmaf(d0.y, d1.y, d0.x * d1.x));
            c = std::fmin(std::fmax(c, -1.f), 1.f); /* safe_acos */
            const float a = std::acos(c);
            acc[3 * fi[i]] += n.x * a;
            acc[3 * fi[i] + 1] += n.y * a;
            acc[3 * fi[i] + 2] += n.z * a;
        }
    }
    m.nrm.resize(nv * 3);
    for (size_t i = 0; i < nv; ++i) {
        const V3f n = nrm3({acc[3 * i], acc[3 * i + 1], acc[3 * i + 2]});
        m.nrm[3 * i] = n.x; m.nrm[3 * i + 1] = n.y; m.nrm[3 * i + 2] = n.z;
    }
}

static std::string read_all(const std::string &path, const char *kind) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error(std::string("Error while loading ") + kind + " file \"" + path + "\": file not found");
    std::ostringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

MeshData load_obj(const std::string &path, const Transform4f &to_world, bool face_normals, bool flip_tex_coords) {
    const std::string name = path.substr(path.find_last_of('/') + 1);
    auto fail = [&](const std::string &d) {
        throw std::runtime_error("Error while loading OBJ file \"" + name + "\": " + d);
    };
    const std::string text = read_all(path, "OBJ");
    std::vector<V3f> vs, ns;
    std::vector<float> ts;
    struct Key { uint32_t v, t, n; bool operator<(const Key &o) const { return v != o.v ? v < o.v : t != o.t ? t < o.t : n < o.n; } };
    std::map<Key, uint32_t> ids;
    std::vector<Key> order;
    MeshData m;
    size_t pos = 0;
    while (pos < text.size()) {
        size_t eol = text.find('\n', pos);
        if (eol == std::string::npos) eol = text.size();
        std::string line = text.substr(pos, eol - pos);
        pos = eol + 1;
        const char *cur = line.c_str();
        while (*cur == ' ' || *cur == '\t' || *cur == '\r') ++cur;
        bool err = false;
        auto rd = [&](float &x) { char *e; x = std::strtof(cur, &e); err |= e == cur; cur = e; };
        if (cur[0] == 'v' && (cur[1] == ' ' || cur[1] == '\t')) {
            cur += 2;
            V3f p; rd(p.x); rd(p.y); rd(p.z);
            p = to_world.apply_point(p);
            if (!std::isfinite(p.x) || !std::isfinite(p.y) || !std::isfinite(p.z)) fail("mesh contains invalid vertex position data");
            vs.push_back(p);
        } else if (cur[0] == 'v' && cur[1] == 'n' && (cur[2] == ' ' || cur[2] == '\t')) {
            if (!face_normals) {
                cur += 3;
                V3f n; rd(n.x); rd(n.y); rd(n.z);
                n = nrm3(to_world.apply_normal(n));
                if (!std::isfinite(n.x) || !std::isfinite(n.y) || !std::isfinite(n.z)) fail("mesh contains invalid vertex normal data");
                ns.push_back(n);
            }
        } else if (cur[0] == 'v' && cur[1] == 't' && (cur[2] == ' ' || cur[2] == '\t')) {
            cur += 3;
            float u, v; rd(u); rd(v);
            if (flip_tex_coords) v = 1.f - v;
            ts.push_back(u); ts.push_back(v);
        } else if (cur[0] == 'f' && (cur[1] == ' ' || cur[1] == '\t')) {
            cur += 2;
            uint32_t key[3] = {0, 0, 0}, tri[3] = {0, 0, 0};
            size_t vi = 0, ti = 0;
            while (true) {
                char *next;
                unsigned long val = std::strtoul(cur, &next, 10);
                if (cur == next) break;
                if (ti < 3) key[ti] = (uint32_t) val;
                else { err = true; break; }
                while (*next == '/') { ++ti; ++next; }
                if (*next == ' ' || *next == '\t' || *next == '\0' || *next == '\r') {
                    ti = 0;
                    if (key[0] == 0 || key[0] > vs.size()) fail("reference to invalid vertex " + std::to_string(key[0]) + "!");
                    Key k{key[0], key[1], key[2]};
                    auto it = ids.find(k);
                    uint32_t id;
                    if (it != ids.end()) id = it->second;
                    else { id = (uint32_t) order.size(); ids.emplace(k, id); order.push_back(k); }
                    if (vi < 3) tri[vi] = id;
                    else { tri[1] = tri[2]; tri[2] = id; }
                    ++vi;
                    if (vi >= 3) m.faces.insert(m.faces.end(), {tri[0], tri[1], tri[2]});
                    /* key is not reset between the vertices of a face (obj.cpp:275-330) */
                }
                cur = next;
            }
        }
        if (err) fail("could not parse line \"" + line + "\"");
    }
    m.pos.resize(order.size() * 3);
    if (!ts.empty()) m.uv.assign(order.size() * 2, 0.f);
    if (!face_normals && !ns.empty()) m.nrm.assign(order.size() * 3, 0.f);
    for (size_t i = 0; i < order.size(); ++i) {
        const Key &k = order[i];
        const V3f p = vs[k.v - 1];
        m.pos[3 * i] = p.x; m.pos[3 * i + 1] = p.y; m.pos[3 * i + 2] = p.z;
        if (k.t) {
            if (k.t > ts.size() / 2) fail("reference to invalid texture coordinate " + std::to_string(k.t) + "!");
            m.uv[2 * i] = ts[2 * (k.t - 1)]; m.uv[2 * i + 1] = ts[2 * (k.t - 1) + 1];
        }
        if (!face_normals && k.n) {
            if (k.n > ns.size()) fail("reference to invalid normal " + std::to_string(k.n) + "!");
            const V3f n = ns[k.n - 1];
            m.nrm[3 * i] = n.x; m.nrm[3 * i + 1] = n.y; m.nrm[3 * i + 2] = n.z;
        }
    }
    if (!face_normals && ns.empty() && !m.faces.empty()) recompute_vertex_normals(m);
    return m;
}

/* ------------------------------------------------------------------ PLY */

namespace {
struct PlyProp { std::string name, type, count_type; bool list = false; };
struct PlyElem { std::string name; size_t count = 0; std::vector<PlyProp> props; };

size_t type_size(const std::string &t) {
    if (t == "char" || t == "uchar" || t == "int8" || t == "uint8") return 1;
    if (t == "short" || t == "ushort" || t == "int16" || t == "uint16") return 2;
    if (t == "int" || t == "uint" || t == "float" || t == "int32" || t == "uint32" || t == "float32") return 4;
    if (t == "double" || t == "float64") return 8;
    throw std::runtime_error("PLY: unknown property type \"" + t + "\"");
}

struct Reader {
    const std::string &buf;
    size_t p;
    int fmt;   /* 0 ascii, 1 binary LE, 2 binary BE */
    std::istringstream ascii;
    Reader(const std::string &b, size_t start, int f) : buf(b), p(start), fmt(f) {
        if (fmt == 0) ascii.str(buf.substr(start));
    }
    double value(const std::string &t) {
        if (fmt == 0) {
            double v;
            if (!(ascii >> v)) throw std::runtime_error("PLY: truncated ascii data");
            return v;
        }
        const size_t n = type_size(t);
        if (p + n > buf.size()) throw std::runtime_error("PLY: truncated binary data");
        unsigned char b[8];
        std::memcpy(b, buf.data() + p, n);
        p += n;
        if (fmt == 2) for (size_t i = 0; i < n / 2; ++i) std::swap(b[i], b[n - 1 - i]);
        if (t == "char" || t == "int8") { int8_t v; std::memcpy(&v, b, 1); return v; }
        if (t == "uchar" || t == "uint8") return b[0];
        if (t == "short" || t == "int16") { int16_t v; std::memcpy(&v, b, 2); return v; }
        if (t == "ushort" || t == "uint16") { uint16_t v; std::memcpy(&v, b, 2); return v; }
        if (t == "int" || t == "int32") { int32_t v; std::memcpy(&v, b, 4); return v; }
        if (t == "uint" || t == "uint32") { uint32_t v; std::memcpy(&v, b, 4); return v; }
        if (t == "float" || t == "float32") { float v; std::memcpy(&v, b, 4); return v; }
        double v; std::memcpy(&v, b, 8); return v;
    }
    bool at_end() {
        if (fmt == 0) { ascii >> std::ws; return ascii.eof(); }
        return p == buf.size();
    }
};
} // namespace

MeshData load_ply(const std::string &path, const Transform4f &to_world, bool face_normals, bool flip_tex_coords) {
    const std::string name = path.substr(path.find_last_of('/') + 1);
    auto fail = [&](const std::string &d) {
        throw std::runtime_error("Error while loading PLY file \"" + name + "\": " + d);
    };
    const std::string buf = read_all(path, "PLY");
    if (buf.compare(0, 3, "ply") != 0) fail("invalid PLY header");
    size_t he = buf.find("end_header");
    if (he == std::string::npos) fail("invalid PLY header");
    size_t data = buf.find('\n', he);
    if (data == std::string::npos) fail("invalid PLY header");
    ++data;
    std::istringstream hs(buf.substr(0, he));
    std::string tok;
    int fmt = -1;
    std::vector<PlyElem> elems;
    std::string line;
    while (std::getline(hs, line)) {
        std::istringstream ls(line);
        ls >> tok;
        if (tok == "format") {
            std::string f; ls >> f;
            fmt = f == "ascii" ? 0 : f == "binary_little_endian" ? 1 : f == "binary_big_endian" ? 2 : -1;
            if (fmt < 0) fail("unknown format \"" + f + "\"");
        } else if (tok == "element") {
            PlyElem e; ls >> e.name >> e.count; elems.push_back(e);
        } else if (tok == "property") {
            if (elems.empty()) fail("property before element");
            PlyProp pr; std::string t; ls >> t;
            if (t == "list") { pr.list = true; ls >> pr.count_type >> pr.type >> pr.name; }
            else { pr.type = t; ls >> pr.name; }
            elems.back().props.push_back(pr);
        }
    }
    if (fmt < 0) fail("missing format line");
    Reader rd(buf, data, fmt);
    MeshData m;
    bool has_n = false, has_uv = false;
    for (const PlyElem &e : elems) {
        if (e.name == "vertex") {
            auto idx = [&](const char *n) { for (size_t i = 0; i < e.props.size(); ++i) if (e.props[i].name == n) return (int) i; return -1; };
            int ix = idx("x"), iy = idx("y"), iz = idx("z"), inx = idx("nx"), iny = idx("ny"), inz = idx("nz");
            int iu = idx("u"), iv = idx("v");
            if (iu < 0 || iv < 0) { iu = idx("texture_u"); iv = idx("texture_v"); }
            if (iu < 0 || iv < 0) { iu = idx("s"); iv = idx("t"); }
            if (ix < 0 || iy < 0 || iz < 0) fail("vertex element without x/y/z");
            has_n = !face_normals && inx >= 0 && iny >= 0 && inz >= 0;
            has_uv = iu >= 0 && iv >= 0;
            std::vector<double> vals(e.props.size());
            for (size_t k = 0; k < e.count; ++k) {
                for (size_t i = 0; i < e.props.size(); ++i) {
                    if (e.props[i].list) fail("list property in the vertex element");
                    vals[i] = rd.value(e.props[i].type);
                }
                V3f p = to_world.apply_point({(float) vals[ix], (float) vals[iy], (float) vals[iz]});
                m.pos.insert(m.pos.end(), {p.x, p.y, p.z});
                if (has_n) {
                    V3f n = nrm3(to_world.apply_normal({(float) vals[inx], (float) vals[iny], (float) vals[inz]}));
                    m.nrm.insert(m.nrm.end(), {n.x, n.y, n.z});
                }
                if (has_uv) {
                    float u = (float) vals[iu], v = (float) vals[iv];
                    if (flip_tex_coords) v = 1.f - v;
                    m.uv.insert(m.uv.end(), {u, v});
                }
            }
        } else if (e.name == "face") {
            int il = -1;
            for (size_t i = 0; i < e.props.size(); ++i)
                if (e.props[i].list && (e.props[i].name == "vertex_indices" || e.props[i].name == "vertex_index")) il = (int) i;
            if (il < 0) fail("vertex_index/vertex_indices property not found");
            for (size_t k = 0; k < e.count; ++k) {
                for (size_t i = 0; i < e.props.size(); ++i) {
                    const PlyProp &pr = e.props[i];
                    if (!pr.list) { (void) rd.value(pr.type); continue; }
                    const size_t n = (size_t) rd.value(pr.count_type);
                    if ((int) i == il && n != 3) fail("incompatible contents -- is this a triangle mesh?");
                    for (size_t j = 0; j < n; ++j) {
                        const double v = rd.value(pr.type);
                        if ((int) i == il) m.faces.push_back((uint32_t) v);
                    }
                }
            }
        } else {
            for (size_t k = 0; k < e.count; ++k)
                for (const PlyProp &pr : e.props) {
                    if (!pr.list) { (void) rd.value(pr.type); continue; }
                    const size_t n = (size_t) rd.value(pr.count_type);
                    for (size_t j = 0; j < n; ++j) (void) rd.value(pr.type);
                }
        }
    }
    if (!rd.at_end()) fail("invalid file -- trailing content");
    const size_t nv = m.pos.size() / 3;
    for (uint32_t f : m.faces)
        if (f >= nv) fail("face references vertex " + std::to_string(f) + " of " + std::to_string(nv));
    if (!face_normals && !has_n && !m.faces.empty()) recompute_vertex_normals(m);
    return m;
}

} // namespace mi
