/*
 * xml.h -- minimal XML reader + Mitsuba scene-format front end.
 *
 * Accepts the subset of the Mitsuba 3 scene format the hot path needs
 * (reference src/core/xml.cpp): <scene>, <default>,
 * $var substitution, objects (<integrator> <sensor> <film> <rfilter> <sampler>
 * <bsdf> <emitter> <shape> <wrap>), properties (<integer> <float> <boolean>
 * <string> <rgb> <vector> <point> <transform>), transform ops (<translate>
 * <rotate> <scale> <lookat> <matrix>), ids and <ref>.
 */
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "transform.h"

namespace mi {

struct XmlNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XmlNode>> children;
    int line = 0;
    const std::string *attr(const std::string &k) const {
        for (auto &a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
};

/* Parse an XML document; throws std::runtime_error with a line number on error. */
std::unique_ptr<XmlNode> parse_xml(const std::string &text);

struct Object;

/* Typed property store (include/mitsuba/core/properties.h). */
struct Properties {
    enum Kind { Bool, Int, Float, String, Vec3, Rgb, Xform, Obj };
    struct Value {
        Kind kind;
        bool b = false;
        long long i = 0;
        double f = 0;
        std::string s;
        float v[3] = {0, 0, 0};
        Transform4f t;
        std::shared_ptr<Object> o;
        /* read by the plugin that consumed these Properties (Properties::Entry::queried); the XML
         * loader's check refuses unread ones (xml.cpp:1089-1107) */
        mutable bool queried = false;
    };
    std::string plugin;   /* type="..." */
    std::string id;
    std::vector<std::pair<std::string, Value>> entries;  /* insertion order */

    /* lookup that counts as a query (the typed getters), and one that does not (has_property) */
    const Value *find(const std::string &k) const {
        const Value *v = peek(k);
        if (v) v->queried = true;
        return v;
    }
    const Value *peek(const std::string &k) const {
        for (auto &e : entries)
            if (e.first == k) return &e.second;
        return nullptr;
    }
    bool has(const std::string &k) const { return peek(k) != nullptr; }
    void mark_queried(const std::string &k) const { (void) find(k); }
    void mark_all_queried() const { for (auto &e : entries) e.second.queried = true; }
    /* Properties::objects(mark_queried): the object-valued entries in insertion order */
    std::vector<std::pair<std::string, const Object *>> objects(bool mark = true) const {
        std::vector<std::pair<std::string, const Object *>> r;
        for (auto &e : entries)
            if (e.second.kind == Obj) {
                r.push_back({e.first, e.second.o.get()});
                if (mark) e.second.queried = true;
            }
        return r;
    }
    std::vector<std::string> unqueried() const {
        std::vector<std::string> r;
        for (auto &e : entries)
            if (!e.second.queried) r.push_back(e.first);
        return r;
    }
    void set(const std::string &k, const Value &v) {
        for (auto &e : entries)
            if (e.first == k) { e.second = v; return; }
        entries.push_back({k, v});
    }
    void remove(const std::string &k) {
        for (size_t i = 0; i < entries.size(); ++i)
            if (entries[i].first == k) { entries.erase(entries.begin() + i); return; }
    }
    long long get_int(const std::string &k, long long def) const;
    double get_float(const std::string &k, double def) const;
    bool get_bool(const std::string &k, bool def) const;
    std::string get_string(const std::string &k, const std::string &def) const;
    std::string get_string(const std::string &k) const;
    V3f get_vec3(const std::string &k, V3f def) const;
    /* rgb / float texture constant */
    bool get_rgb(const std::string &k, float out[3]) const;
    Transform4f get_transform(const std::string &k) const;
    void set_float(const std::string &k, double v);
    void set_string(const std::string &k, const std::string &v);
    void set_transform(const std::string &k, const Transform4f &t);
    void set_object(const std::string &k, std::shared_ptr<Object> o);
};

/* A node of the instantiated scene graph: tag ("bsdf", "shape", ...) + Properties. */
struct Object {
    std::string tag;       /* object class: integrator, sensor, film, rfilter, sampler, bsdf, emitter, shape, wrap, scene */
    Properties props;
    std::string base_dir;  /* root only: directory of the scene file (FileResolver for `filename`) */
    std::string src;       /* the scene file (or "<string>") and the line of the object's tag, for error messages */
    int line = 0;
    virtual ~Object() = default;
};

/* The XML loader's check after instantiating the scene (xml.cpp:1089-1107): every property and child
 * object of every object the loader instantiated must have been read by its plugin, else the
 * reference's "unreferenced property" / "unreferenced object" error. */
void check_unqueried(const Object &root);

std::shared_ptr<Object> load_scene_file(const std::string &path, const std::map<std::string, std::string> &defines);
std::shared_ptr<Object> load_scene_string(const std::string &xml, const std::map<std::string, std::string> &defines);

} // namespace mi
