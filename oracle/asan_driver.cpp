/*
 * TEST INFRASTRUCTURE ONLY: the CPU oracle under AddressSanitizer + UBSan (oracle/Makefile `asan`).
 * Loads each scene with the host framework (XML -> the C-ABI descriptors the product receives),
 * renders a small frame with per-lane records on 4 threads and checks that film and records are
 * finite where they must be.  Run by tests/test_oracle_asan.py; a sanitizer report aborts with a
 * non-zero exit.
 *   asan_driver <scene.xml> [key=value ...]
 */
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/amvpt_host.h"

extern "C" int oracle_render(const amvpt_scene_desc *sd, const amvpt_view_desc *views, const amvpt_params *params,
                             uint64_t lane_begin, uint64_t lane_end, float *film, int n_threads, float *records,
                             uint32_t record_pass, void *stats);
extern "C" int oracle_plan(const amvpt_params *p, uint32_t *spp, uint32_t *spp_pp, uint32_t *n_passes, uint64_t *L,
                           uint32_t *G);

int main(int argc, char **argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: %s scene.xml [key=value ...]\n", argv[0]); return 2; }
    std::vector<std::string> keys, vals;
    for (int i = 2; i < argc; ++i) {
        const char *eq = std::strchr(argv[i], '=');
        if (!eq) return 2;
        keys.emplace_back(argv[i], eq - argv[i]);
        vals.emplace_back(eq + 1);
    }
    std::vector<const char *> kp, vp;
    for (size_t i = 0; i < keys.size(); ++i) { kp.push_back(keys[i].c_str()); vp.push_back(vals[i].c_str()); }
    amvpt_host_scene *s = amvpt_host_load_file(argv[1], kp.data(), vp.data(), (int) kp.size());
    if (!s) { std::fprintf(stderr, "load: %s\n", amvpt_host_last_error()); return 3; }
    const amvpt_scene_desc *sd = nullptr;
    const amvpt_view_desc *vd = nullptr;
    amvpt_params p;
    if (amvpt_host_describe(s, 0, 0, 0, &sd, &vd, &p) != 0) { std::fprintf(stderr, "describe failed\n"); return 3; }
    uint32_t spp, spp_pp, n_passes, G;
    uint64_t L;
    oracle_plan(&p, &spp, &spp_pp, &n_passes, &L, &G);
    const uint32_t C = p.film_alpha ? 5 : 4;
    std::vector<float> film((size_t) p.film_width * p.film_height * C, 0.f);
    std::vector<float> rec((size_t) L * G * 8, 0.f);
    const int rc = oracle_render(sd, vd, &p, 0, L, film.data(), 4, rec.data(), 0, nullptr);
    if (rc != 0) { std::fprintf(stderr, "oracle_render: %d\n", rc); return 4; }
    size_t bad = 0;
    for (float f : film) bad += std::isfinite(f) ? 0 : 1;
    double sum = 0.0;
    for (size_t i = 0; i < film.size(); i += C) sum += film[i + C - 1];
    std::printf("%s: %ux%u, %llu lanes x %u passes, G=%u, weight sum %.6g, non-finite film values %zu\n", argv[1],
                p.film_width, p.film_height, (unsigned long long) L, n_passes, G, sum, bad);
    amvpt_host_scene_free(s);
    return bad == 0 && sum > 0.0 ? 0 : 5;
}
