/*
 * xml.cpp -- XML reader and the Mitsuba scene-format loader (subset).
 * Reference behaviour: src/core/xml.cpp (tags, <default>/$param, transform
 * ops applied as `op * current`, <ref>, ids, <wrap> at xml.cpp:79-81).
 */
#include "xml.h"

#include <cctype>
#include <cstring>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <stdexcept>

namespace mi {

/* ------------------------------------------------------------------ */
/* XML reader                                                          */
/* ------------------------------------------------------------------ */

namespace {
struct Reader {
    const std::string &s;
    size_t i = 0;
    int line = 1;
    explicit Reader(const std::string &t) : s(t) {}
    [[noreturn]] void fail(const std::string &m) {
        throw std::runtime_error("XML parse error (line " + std::to_string(line) + "): " + m);
    }
    bool eof() const { return i >= s.size(); }
    char peek() const { return i < s.size() ? s[i] : '\0'; }
    void adv(size_t n = 1) {
        for (size_t k = 0; k < n && i < s.size(); ++k, ++i)
            if (s[i] == '\n') ++line;
    }
    bool starts(const char *p) const { return s.compare(i, std::strlen(p), p) == 0; }
    void ws() { while (!eof() && std::isspace((unsigned char) peek())) adv(); }
    void skip_misc() {
        for (;;) {
            ws();
            if (starts("<!--")) {
                size_t e = s.find("-->", i + 4);
                if (e == std::string::npos) fail("unterminated comment");
                adv(e + 3 - i);
            } else if (starts("<?")) {
                size_t e = s.find("?>", i + 2);
                if (e == std::string::npos) fail("unterminated processing instruction");
                adv(e + 2 - i);
            } else if (starts("<!DOCTYPE")) {
                size_t e = s.find('>', i);
                if (e == std::string::npos) fail("unterminated doctype");
                adv(e + 1 - i);
            } else {
                break;
            }
        }
    }
    std::string name() {
        size_t b = i;
        while (!eof() && (std::isalnum((unsigned char) peek()) || peek() == '_' || peek() == '-' || peek() == ':' || peek() == '.')) adv();
        if (b == i) fail("expected a name");
        return s.substr(b, i - b);
    }
    static std::string unescape(const std::string &v) {
        std::string o;
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] == '&') {
                size_t e = v.find(';', k);
                std::string ent = v.substr(k + 1, e - k - 1);
                if (ent == "lt") o += '<'; else if (ent == "gt") o += '>'; else if (ent == "amp") o += '&';
                else if (ent == "quot") o += '"'; else if (ent == "apos") o += '\''; else o += "&" + ent + ";";
                k = e;
            } else o += v[k];
        }
        return o;
    }
    std::unique_ptr<XmlNode> element() {
        if (peek() != '<') fail("expected '<'");
        adv();
        auto n = std::make_unique<XmlNode>();
        n->line = line;
        n->tag = name();
        for (;;) {
            ws();
            if (starts("/>")) { adv(2); return n; }
            if (peek() == '>') { adv(); break; }
            std::string k = name();
            ws();
            if (peek() != '=') fail("expected '=' after attribute " + k);
            adv();
            ws();
            char q = peek();
            if (q != '"' && q != '\'') fail("expected a quoted attribute value");
            adv();
            size_t e = s.find(q, i);
            if (e == std::string::npos) fail("unterminated attribute value");
            std::string v = s.substr(i, e - i);
            adv(e + 1 - i);
            n->attrs.push_back({k, unescape(v)});
        }
        for (;;) {
            skip_misc();
            if (eof()) fail("unterminated element <" + n->tag + ">");
            if (starts("</")) {
                adv(2);
                std::string cn = name();
                if (cn != n->tag) fail("mismatched closing tag </" + cn + "> for <" + n->tag + ">");
                ws();
                if (peek() != '>') fail("expected '>'");
                adv();
                return n;
            }
            if (peek() == '<') n->children.push_back(element());
            else {
                /* character data is not used by the scene format: skip */
                while (!eof() && peek() != '<') adv();
            }
        }
    }
};
} // namespace

std::unique_ptr<XmlNode> parse_xml(const std::string &text) {
    Reader r(text);
    r.skip_misc();
    auto root = r.element();
    r.skip_misc();
    return root;
}

/* ------------------------------------------------------------------ */
/* Properties                                                          */
/* ------------------------------------------------------------------ */

static std::runtime_error prop_err(const std::string &k, const std::string &what) {
    return std::runtime_error("Property \"" + k + "\": " + what);
}

long long Properties::get_int(const std::string &k, long long def) const {
    const Value *v = find(k);
    if (!v) return def;
    if (v->kind == Int) return v->i;
    throw prop_err(k, "expected an integer");
}
double Properties::get_float(const std::string &k, double def) const {
    const Value *v = find(k);
    if (!v) return def;
    if (v->kind == Float) return v->f;
    if (v->kind == Int) return (double) v->i;
    throw prop_err(k, "expected a float");
}
bool Properties::get_bool(const std::string &k, bool def) const {
    const Value *v = find(k);
    if (!v) return def;
    if (v->kind == Bool) return v->b;
    throw prop_err(k, "expected a boolean");
}
std::string Properties::get_string(const std::string &k, const std::string &def) const {
    const Value *v = find(k);
    if (!v) return def;
    if (v->kind == String) return v->s;
    throw prop_err(k, "expected a string");
}
std::string Properties::get_string(const std::string &k) const {
    const Value *v = find(k);
    if (!v) throw prop_err(k, "property not specified");
    return get_string(k, "");
}
V3f Properties::get_vec3(const std::string &k, V3f def) const {
    const Value *v = find(k);
    if (!v) return def;
    if (v->kind == Vec3 || v->kind == Rgb) return {v->v[0], v->v[1], v->v[2]};
    if (v->kind == Float || v->kind == Int) {
        float f = (float) (v->kind == Float ? v->f : (double) v->i);
        return {f, f, f};
    }
    throw prop_err(k, "expected a vector");
}
bool Properties::get_rgb(const std::string &k, float out[3]) const {
    const Value *v = find(k);
    if (!v) return false;
    if (v->kind == Rgb || v->kind == Vec3) { out[0] = v->v[0]; out[1] = v->v[1]; out[2] = v->v[2]; return true; }
    if (v->kind == Float || v->kind == Int) {
        float f = (float) (v->kind == Float ? v->f : (double) v->i);
        out[0] = out[1] = out[2] = f;
        return true;
    }
    throw prop_err(k, "expected an rgb value or a float (textures other than constant rgb are not implemented)");
}
Transform4f Properties::get_transform(const std::string &k) const {
    const Value *v = find(k);
    if (!v) return Transform4f();
    if (v->kind == Xform) return v->t;
    throw prop_err(k, "expected a transform");
}
void Properties::set_float(const std::string &k, double f) { Value v; v.kind = Float; v.f = f; set(k, v); }
void Properties::set_string(const std::string &k, const std::string &s) { Value v; v.kind = String; v.s = s; set(k, v); }
void Properties::set_transform(const std::string &k, const Transform4f &t) { Value v; v.kind = Xform; v.t = t; set(k, v); }
void Properties::set_object(const std::string &k, std::shared_ptr<Object> o) { Value v; v.kind = Obj; v.o = o; set(k, v); }

/* ------------------------------------------------------------------ */
/* Scene loader                                                        */
/* ------------------------------------------------------------------ */

namespace {

const char *kObjectTags[] = {"scene", "integrator", "sensor", "film", "rfilter", "sampler", "bsdf",
                             "emitter", "shape", "wrap", "texture", "medium", "phase", "volume", "spectrum"};

bool is_object_tag(const std::string &t) {
    for (auto *o : kObjectTags)
        if (t == o) return true;
    return false;
}

struct Loader {
    std::string src = "<string>";   /* the scene file, for error messages */
    std::map<std::string, std::string> params;
    std::map<std::string, std::shared_ptr<Object>> ids;
    int unnamed = 0;

    [[noreturn]] void fail(const XmlNode &n, const std::string &m) {
        throw std::runtime_error("Error while loading scene (line " + std::to_string(n.line) + ", <" + n.tag + ">): " + m);
    }
    std::string sub(const std::string &v) {
        /* $name substitution (xml.cpp: parameter substitution) */
        std::string o;
        for (size_t k = 0; k < v.size(); ++k) {
            if (v[k] == '$') {
                size_t e = k + 1;
                while (e < v.size() && (std::isalnum((unsigned char) v[e]) || v[e] == '_')) ++e;
                std::string key = v.substr(k + 1, e - k - 1);
                auto it = params.find(key);
                if (it == params.end()) throw std::runtime_error("Undefined parameter \"$" + key + "\"");
                o += it->second;
                k = e - 1;
            } else o += v[k];
        }
        return o;
    }
    std::string attr(const XmlNode &n, const char *k, bool required = true) {
        const std::string *a = n.attr(k);
        if (!a) {
            if (required) fail(n, std::string("missing attribute \"") + k + "\"");
            return "";
        }
        return sub(*a);
    }
    static std::vector<float> floats(const std::string &s) {
        std::vector<float> r;
        std::string t = s;
        for (char &c : t) if (c == ',') c = ' ';
        std::istringstream is(t);
        double d;
        while (is >> d) r.push_back((float) d);
        return r;
    }
    V3f vec_attr(const XmlNode &n, float def) {
        if (n.attr("value")) {
            auto f = floats(attr(n, "value"));
            if (f.size() == 1) return {f[0], f[0], f[0]};
            if (f.size() != 3) fail(n, "expected 3 components");
            return {f[0], f[1], f[2]};
        }
        V3f r{def, def, def};
        if (n.attr("x")) r.x = (float) std::atof(attr(n, "x").c_str());
        if (n.attr("y")) r.y = (float) std::atof(attr(n, "y").c_str());
        if (n.attr("z")) r.z = (float) std::atof(attr(n, "z").c_str());
        return r;
    }

    Transform4f transform(const XmlNode &n) {
        Transform4f t;
        for (auto &c : n.children) {
            const XmlNode &o = *c;
            if (o.tag == "translate") t = Transform4f::translate(vec_attr(o, 0.f)) * t;
            else if (o.tag == "scale") {
                V3f v = vec_attr(o, 1.f);
                t = Transform4f::scale(v) * t;
            } else if (o.tag == "rotate") {
                V3f axis = vec_attr(o, 0.f);
                float angle = (float) std::atof(attr(o, "angle").c_str());
                t = Transform4f::rotate(axis, angle) * t;
            } else if (o.tag == "lookat" || o.tag == "look_at") {
                auto org = floats(attr(o, "origin")), tgt = floats(attr(o, "target"));
                std::vector<float> up = o.attr("up") ? floats(attr(o, "up")) : std::vector<float>{0.f, 1.f, 0.f};
                if (org.size() != 3 || tgt.size() != 3 || up.size() != 3) fail(o, "lookat expects 3-vectors");
                t = Transform4f::look_at({org[0], org[1], org[2]}, {tgt[0], tgt[1], tgt[2]}, {up[0], up[1], up[2]}) * t;
            } else if (o.tag == "matrix") {
                auto f = floats(attr(o, "value"));
                if (f.size() != 16 && f.size() != 9) fail(o, "matrix expects 16 (or 9) values");
                Mat4 m = Mat4::identity();
                if (f.size() == 16) for (int k = 0; k < 16; ++k) m.m[k / 4][k % 4] = f[k];
                else for (int k = 0; k < 9; ++k) m.m[k / 3][k % 3] = f[k];
                t = Transform4f(m) * t;
            } else {
                fail(o, "unsupported transform operation");
            }
        }
        return t;
    }

    std::shared_ptr<Object> object(const XmlNode &n) {
        auto obj = std::make_shared<Object>();
        obj->tag = n.tag;
        obj->src = src;
        obj->line = n.line;
        if (n.tag != "scene") obj->props.plugin = attr(n, "type", n.tag != "wrap" || true);
        obj->props.id = n.attr("id") ? attr(n, "id") : "_unnamed_" + std::to_string(unnamed++);
        for (auto &cp : n.children) {
            const XmlNode &c = *cp;
            std::string name = c.attr("name") ? attr(c, "name") : "";
            Properties::Value v;
            if (c.tag == "default") {
                std::string k = attr(c, "name");
                if (!params.count(k)) params[k] = attr(c, "value");
                continue;
            } else if (c.tag == "integer") {
                v.kind = Properties::Int;
                v.i = std::atoll(attr(c, "value").c_str());
            } else if (c.tag == "float") {
                v.kind = Properties::Float;
                v.f = std::atof(attr(c, "value").c_str());
            } else if (c.tag == "boolean") {
                std::string b = attr(c, "value");
                for (auto &ch : b) ch = (char) std::tolower((unsigned char) ch);
                if (b != "true" && b != "false") fail(c, "boolean must be true or false");
                v.kind = Properties::Bool;
                v.b = b == "true";
            } else if (c.tag == "string") {
                v.kind = Properties::String;
                v.s = attr(c, "value");
            } else if (c.tag == "vector" || c.tag == "point") {
                v.kind = Properties::Vec3;
                V3f p = vec_attr(c, 0.f);
                v.v[0] = p.x; v.v[1] = p.y; v.v[2] = p.z;
            } else if (c.tag == "rgb" || c.tag == "color") {
                v.kind = Properties::Rgb;
                auto f = floats(attr(c, "value"));
                if (f.size() == 1) f = {f[0], f[0], f[0]};
                if (f.size() != 3) fail(c, "rgb expects 1 or 3 values");
                v.v[0] = f[0]; v.v[1] = f[1]; v.v[2] = f[2];
            } else if (c.tag == "transform") {
                v.kind = Properties::Xform;
                v.t = transform(c);
            } else if (c.tag == "ref") {
                std::string id = attr(c, "id");
                auto it = ids.find(id);
                if (it == ids.end()) fail(c, "reference to unknown object \"" + id + "\"");
                v.kind = Properties::Obj;
                v.o = it->second;
                if (name.empty()) name = "_ref_" + id + "_" + std::to_string(unnamed++);
            } else if (is_object_tag(c.tag)) {
                v.kind = Properties::Obj;
                v.o = object(c);
                if (name.empty()) name = "_arg_" + std::to_string(unnamed++);
            } else if (c.tag == "include") {
                fail(c, "<include> is not supported");
            } else {
                fail(c, "unsupported tag");
            }
            if (name.empty()) fail(c, "missing attribute \"name\"");
            obj->props.set(name, v);
        }
        if (n.attr("id")) {
            std::string id = attr(n, "id");
            if (ids.count(id)) fail(n, "duplicate id \"" + id + "\"");
            ids[id] = obj;
        }
        return obj;
    }
};

} // namespace

static std::shared_ptr<Object> load_scene(const std::string &xml, const std::map<std::string, std::string> &defines,
                                          const std::string &src) {
    auto root = parse_xml(xml);
    if (root->tag != "scene") throw std::runtime_error("XML root must be <scene>");
    Loader L;
    L.src = src;
    L.params = defines;
    /* <default> must be visible before use: pre-scan the root's <default> tags */
    for (auto &c : root->children)
        if (c->tag == "default") {
            const std::string *k = c->attr("name"), *v = c->attr("value");
            /* values may use earlier parameters ($name is substituted in every attribute, xml.cpp) */
            if (k && v && !L.params.count(*k)) L.params[*k] = L.sub(*v);
        }
    return L.object(*root);
}

std::shared_ptr<Object> load_scene_string(const std::string &xml, const std::map<std::string, std::string> &defines) {
    return load_scene(xml, defines, "<string>");
}

std::shared_ptr<Object> load_scene_file(const std::string &path, const std::map<std::string, std::string> &defines) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("Unable to open scene file \"" + path + "\"");
    std::stringstream ss;
    ss << f.rdbuf();
    auto root = load_scene(ss.str(), defines, path);
    const size_t slash = path.find_last_of('/');
    root->base_dir = slash == std::string::npos ? std::string(".") : path.substr(0, slash);
    return root;
}

/* ------------------------------------------------------------------ */
/* Unreferenced properties (xml.cpp:1089-1107)                         */
/* ------------------------------------------------------------------ */

/* the plugin class as the reference names it: string::to_lower(Class::name()) */
static std::string class_name(const std::string &tag) {
    if (tag == "rfilter") return "reconstructionfilter";
    return tag;
}

static void check_object(const Object &o, std::vector<const Object *> &seen) {
    for (const Object *s : seen)
        if (s == &o) return;
    seen.push_back(&o);
    /* children first: the loader instantiates (and checks) them before their parent */
    for (auto &e : o.props.entries)
        if (e.second.kind == Properties::Obj) check_object(*e.second.o, seen);
    /* Wrap marks its own properties queried (wrap.cpp:12-14); the plugin it creates reads a copy of them
     * (unwrap), and its XML children were instantiated, and are checked, as any other */
    if (o.tag == "wrap") return;
    const std::string near = "\"" + o.src + "\" (near line " + std::to_string(o.line) + ")";
    const std::string type = o.tag == "scene" ? "scene" : o.props.plugin;
    std::vector<std::string> names;
    for (auto &e : o.props.entries) {
        if (e.second.queried) continue;
        if (e.second.kind == Properties::Obj) {
            const Object &c = *e.second.o;
            throw std::runtime_error("Error while loading " + near + ": unreferenced object " + c.tag + " of type \"" +
                                     c.props.plugin + "\" (within " + class_name(o.tag) + " of type \"" + type + "\")");
        }
        names.push_back("\"" + e.first + "\"");
    }
    if (names.empty()) return;
    std::string list = "[";
    for (size_t i = 0; i < names.size(); ++i) list += (i ? ", " : "") + names[i];
    list += "]";
    throw std::runtime_error("Error while loading " + near + ": unreferenced " +
                             (names.size() > 1 ? "properties" : "property") + " \"" + list + "\" in " +
                             class_name(o.tag) + " plugin of type \"" + type + "\"");
}

void check_unqueried(const Object &root) {
    std::vector<const Object *> seen;
    check_object(root, seen);
}

} // namespace mi
