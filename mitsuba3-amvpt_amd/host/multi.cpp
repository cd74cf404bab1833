/*
 * multi.cpp -- Integrator::render over several GPUs of one node, without torch.
 *
 * Every lane seeds its sampler from its global index (TEA(seed_value, lane), mvpath.cpp:227-235), so a
 * frame shards across devices with results bit-for-bit the single-GPU ones (float summation order
 * aside).  Two partitions, as bench.py / amvpt.dist:
 *   view groups (C5, "4 views per GPU"): device r owns whole view groups (mvpath_multi.h:31-38), a
 *     rectangle of quilt tiles; it renders the lanes of those pixels (amvpt_lane_set rect form) into a
 *     film window of its tiles + a 4-px filter border, and the windows (and the few overflow cells)
 *     are sent to devices[0] (ncclSend / ncclRecv over xGMI) and summed into the quilt there
 *     (amvpt_film_accumulate);
 *   lane bands (otherwise): device r renders the contiguous range amvpt_host_lane_shard(L, r, n) of
 *     every pass into a whole-quilt ImageBlock, summed onto devices[0] with one ncclReduce.
 * Then develop on devices[0] (hdrfilm.cpp:304-418).  With adaptive > 0 the fill compacts the whole
 * pass (mvpath_multi.h:79-115): the device threads exchange their per-run flagged-lane counts through
 * the per-call amvpt_render_opts.exchange (an in-process all-gather) -- no process-global state.
 *
 * Per-frame cost: the RCCL communicators, the per-device scene copies (scene upload + BVH build),
 * streams and film buffers are cached on the host scene, keyed by the device list, and reused by the
 * next frame (amvpt_host_multi_stats counts scene creations and communicator initialisations).
 *
 * A device list naming ONE device several times is a shared-device rehearsal of the same code (a box with one GPU):
 * every rank renders its share on that device through its own scene copy, stream and film, and devices[0]'s thread
 * sums the others' films / windows and overflow cells with amvpt_film_accumulate instead of RCCL (renders on one
 * device serialise on its lane arena, so the adaptive fill's cross-rank count exchange is refused there).
 *
 * Failure handling: the device threads meet at in-process barriers after setup and after the render;
 * the collectives run only when every device reached them healthy, so a failing device (bad id, OOM,
 * a failed render) never leaves a peer blocked inside RCCL, and a failed render aborts the count
 * exchange so no peer waits in it either.  The call then reports the first error.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <array>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/amvpt.h"
#include "../../include/amvpt_host.h"
#include "ranks.h"

namespace {

using amvpt_ranks::RunExchange;
struct RankExchange { RunExchange *ex; int rank; };
int run_exchange_cb(void *ctx, uint32_t n, const uint64_t *b, const uint64_t *c, uint64_t *prefix, uint64_t *total) {
    const RankExchange *x = static_cast<const RankExchange *>(ctx);
    return x->ex->exchange(x->rank, n, b, c, prefix, total);
}

/* device buffers of one device, grown on demand and kept across frames */
struct DevState {
    int device = -1;
    amvpt_scene *scene = nullptr;
    hipStream_t st = nullptr;
    float *film = nullptr;  size_t film_bytes = 0;       /* window (view groups) or whole quilt (lane bands) */
    uint32_t *ovf = nullptr; size_t ovf_bytes = 0;       /* overflow list (view groups) */
    float *quilt = nullptr; size_t quilt_bytes = 0;      /* devices[0], view groups: the assembled ImageBlock */
    float *out = nullptr;   size_t out_bytes = 0;        /* devices[0]: developed image */
    std::vector<float *> recv; std::vector<size_t> recv_bytes;     /* devices[0]: peers' windows */
    std::vector<uint32_t *> recv_ov; std::vector<size_t> recv_ov_bytes;
};

bool grow(void *&p, size_t &have, size_t need) {
    if (have >= need) return true;
    if (p) (void) hipFree(p);
    p = nullptr;
    have = 0;
    if (hipMalloc(&p, need) != hipSuccess) return false;
    have = need;
    return true;
}
template <class T> bool grow(T *&p, size_t &have, size_t need) {
    void *v = p;
    const bool ok = grow(v, have, need);
    p = static_cast<T *>(v);
    return ok;
}

}  // namespace

/* the per-scene multi-GPU cache (opaque to scene.cpp) */
struct amvpt_multi_cache {
    std::mutex mu;   /* one render_multi at a time per scene */
    std::vector<int> devices;
    std::vector<ncclComm_t> comms;
    std::vector<DevState> dev;
    uint64_t scene_creates = 0, comm_inits = 0, renders = 0;
    void release() {
        int cur = -1;
        const bool restore = hipGetDevice(&cur) == hipSuccess;
        for (auto c : comms) if (c) (void) ncclCommDestroy(c);
        comms.clear();
        for (DevState &d : dev) {
            if (d.device >= 0) (void) hipSetDevice(d.device);
            if (d.st) (void) hipStreamSynchronize(d.st);
            for (void *p : {(void *) d.film, (void *) d.ovf, (void *) d.quilt, (void *) d.out}) if (p) (void) hipFree(p);
            for (float *p : d.recv) if (p) (void) hipFree(p);
            for (uint32_t *p : d.recv_ov) if (p) (void) hipFree(p);
            if (d.scene) amvpt_scene_destroy(d.scene);
            if (d.st) (void) hipStreamDestroy(d.st);
        }
        dev.clear();
        devices.clear();
        if (restore) (void) hipSetDevice(cur);   /* the caller's current device stays as it was */
    }
    ~amvpt_multi_cache() { release(); }
};

/* scene.cpp: the host scene's cache slot and the exception guard */
std::shared_ptr<amvpt_multi_cache> &amvpt_host_multi_slot(amvpt_host_scene *s);
int amvpt_host_guarded_call(int (*fn)(void *), void *ctx);
template <class F> static int amvpt_host_guarded(F &&f) {
    return amvpt_host_guarded_call([](void *c) { return (*static_cast<F *>(c))(); }, &f);
}

namespace {

/* MVPathIntegrator::render's group size (mvpath.cpp:192-217) */
uint32_t group_size(const amvpt_params &p) {
    const bool reuse = p.integrator == AMVPT_INTEGRATOR_MVPATH && p.sa_reuse && p.n_views > 1 && p.reuse_count != 1;
    if (!reuse) return 1;
    const uint32_t N = p.n_views;
    uint32_t G = std::min(p.reuse_count, N);
    if (G == 0 || N % G) {
        G = 0;
        for (uint32_t q = 8; q < N; ++q) if (N % q == 0) { G = q; break; }
        if (!G) for (uint32_t q = 8; q > 1; --q) if (N % q == 0) { G = q; break; }
        if (!G) G = N;
    }
    return G;
}

/* pixels around a rank's tiles its splats can reach (amvpt.dist.filter_border): ImageBlock::put's footprint
 * around a sample in the tile reaches ceil(radius - 1/2) cells (coalesced) or ceil(radius + 1/2) (not
 * coalesced), radius = 4 stddev for the Gaussian (gaussian.cpp:48-60); the box filter stays in its pixel.
 * At least 4, the default filter's border (radius 2) with a cell to spare. */
static uint32_t filter_border(const amvpt_params &p) {
    if (p.rfilter == AMVPT_RFILTER_BOX) return 4;
    const float radius = 4.f * (p.rfilter_stddev > 0.f ? p.rfilter_stddev : .5f);
    return std::max<uint32_t>(4, (uint32_t) std::ceil(radius + .5f));
}

}  // namespace

extern "C" {

void amvpt_host_lane_shard(uint64_t lanes, uint32_t rank, uint32_t world, uint64_t *begin, uint64_t *end) {
    const uint64_t q = world ? lanes / world : 0, r = world ? lanes % world : 0;
    const uint64_t b = rank * q + std::min<uint64_t>(rank, r);
    *begin = b;
    *end = b + q + (rank < r ? 1u : 0u);
}

int amvpt_host_view_group_partition(const amvpt_params *p, uint32_t rank, uint32_t world, uint32_t *rect,
                                    uint32_t *window) {
    if (!p || !p->multisensor || world == 0 || rank >= world) return 0;
    const uint32_t G = group_size(*p);
    if (G < 1 || p->n_views % G) return 0;
    const uint32_t n_groups = p->n_views / G;
    if (n_groups < world || n_groups % world) return 0;
    const uint32_t gx = std::max(1u, p->grid_x), gy = std::max(1u, p->grid_y);
    const uint32_t sx = p->film_width / gx, sy = p->film_height / gy;
    const uint32_t per = n_groups / world, v0 = rank * per * G, v1 = (rank + 1) * per * G;
    /* tiles of views [v0, v1): the inverse of GridSensor::sample_ray_idx's index (grid.cpp:269-297) */
    uint32_t tx0 = gx, ty0 = gy, tx1 = 0, ty1 = 0;
    std::vector<uint8_t> seen((size_t) gx * gy, 0);
    for (uint32_t v = v0; v < v1; ++v) {
        uint32_t ix = v % gx, iy = v / gx;
        if (p->reverse_x) ix = gx - 1 - ix;
        if (p->reverse_y) iy = gy - 1 - iy;
        if (iy >= gy) return 0;
        seen[(size_t) iy * gx + ix] = 1;
        tx0 = std::min(tx0, ix); ty0 = std::min(ty0, iy); tx1 = std::max(tx1, ix + 1); ty1 = std::max(ty1, iy + 1);
    }
    if ((tx1 - tx0) * (ty1 - ty0) != v1 - v0) return 0;   /* not a rectangle of tiles */
    rect[0] = tx0 * sx; rect[1] = ty0 * sy; rect[2] = (tx1 - tx0) * sx; rect[3] = (ty1 - ty0) * sy;
    const uint32_t border = filter_border(*p);
    const uint32_t wx0 = rect[0] > border ? rect[0] - border : 0;
    const uint32_t wy0 = rect[1] > border ? rect[1] - border : 0;
    const uint32_t wx1 = std::min(p->film_width, rect[0] + rect[2] + border);
    const uint32_t wy1 = std::min(p->film_height, rect[1] + rect[3] + border);
    window[0] = wx0; window[1] = wy0; window[2] = wx1 - wx0; window[3] = wy1 - wy0;
    return 1;
}

int amvpt_host_multi_stats(amvpt_host_scene *s, uint64_t *scene_creates, uint64_t *comm_inits, uint64_t *renders) {
    return amvpt_host_guarded([&] {
        if (!s) throw std::runtime_error("amvpt_host_multi_stats: null scene");
        std::shared_ptr<amvpt_multi_cache> &slot = amvpt_host_multi_slot(s);
        if (scene_creates) *scene_creates = slot ? slot->scene_creates : 0;
        if (comm_inits) *comm_inits = slot ? slot->comm_inits : 0;
        if (renders) *renders = slot ? slot->renders : 0;
        return 0;
    });
}

int amvpt_host_render_multi(amvpt_host_scene *s, uint32_t si, uint32_t seed, uint32_t spp, int raw,
                            const int *devices, int n_devices, float *out, amvpt_counters *counters) {
    return amvpt_host_guarded([&] {
        if (!s || si >= amvpt_host_sensor_count(s)) throw std::runtime_error("Scene::render(): sensor index out of bounds!");
        if (!devices || n_devices < 1) throw std::runtime_error("amvpt_host_render_multi: no devices");
        const amvpt_scene_desc *sd = nullptr;
        const amvpt_view_desc *views = nullptr;
        amvpt_params p;
        if (amvpt_host_describe(s, si, seed, spp, &sd, &views, &p) != 0) throw std::runtime_error(amvpt_host_last_error());
        uint32_t spp_all, spp_pp, n_passes;
        uint64_t L;
        if (amvpt_plan(&p, &spp_all, &spp_pp, &n_passes, &L) != AMVPT_OK) throw std::runtime_error(amvpt_last_error());
        const uint32_t C = amvpt_film_channels(&p);
        const size_t npx = (size_t) p.film_width * p.film_height, nfloat = npx * C;
        const int n = n_devices;
        {
            int visible = 0;
            if (hipGetDeviceCount(&visible) != hipSuccess) visible = 0;
            for (int r = 0; r < n; ++r)
                if (devices[r] < 0 || devices[r] >= visible)
                    throw std::runtime_error("amvpt_host_render_multi: device " + std::to_string(devices[r]) +
                                             " is not visible (" + std::to_string(visible) + " devices)");
        }

        /* one device named n > 1 times: the shared-device rehearsal (header comment); other repeats are refused */
        bool shared = false;
        if (n > 1) {
            std::vector<int> u(devices, devices + n);
            std::sort(u.begin(), u.end());
            const size_t distinct = (size_t) (std::unique(u.begin(), u.end()) - u.begin());
            if (distinct == 1) shared = true;
            else if (distinct < (size_t) n)
                throw std::runtime_error("amvpt_host_render_multi: a device list repeats a device (only a list of one "
                                         "device repeated is a shared-device rehearsal)");
            if (shared && p.adaptive > 0 && p.sa_reuse)
                throw std::runtime_error("amvpt_host_render_multi: a shared-device rehearsal cannot run the adaptive "
                                         "fill's count exchange (renders on one device serialise on its lane arena)");
        }

        /* ---- the cache: communicators, per-device scenes, streams and buffers for this device list ---- */
        std::shared_ptr<amvpt_multi_cache> &slot = amvpt_host_multi_slot(s);
        if (!slot) slot = std::make_shared<amvpt_multi_cache>();
        std::shared_ptr<amvpt_multi_cache> cache = slot;
        std::lock_guard<std::mutex> cache_lock(cache->mu);
        const std::vector<int> devs(devices, devices + n);
        if (cache->devices != devs) {
            cache->release();
            cache->devices = devs;
            cache->dev.resize((size_t) n);
            for (int r = 0; r < n; ++r) cache->dev[(size_t) r].device = devs[(size_t) r];
        }
        if (cache->comms.empty() && n > 1 && !shared) {
            cache->comms.assign((size_t) n, nullptr);
            if (ncclCommInitAll(cache->comms.data(), n, devices) != ncclSuccess) {
                cache->comms.clear();
                throw std::runtime_error("ncclCommInitAll failed");
            }
            ++cache->comm_inits;
        }

        /* ---- partition: view groups when they divide among the devices, else lane bands ---- */
        std::vector<std::array<uint32_t, 4>> rects((size_t) n), wins((size_t) n);
        bool groups = n > 1;
        for (int r = 0; r < n && groups; ++r)
            groups = amvpt_host_view_group_partition(&p, (uint32_t) r, (uint32_t) n, rects[(size_t) r].data(),
                                                     wins[(size_t) r].data()) == 1;
        const uint64_t ov_cap = 1u << 20;

        amvpt_ranks::Ranks ranks;
        RunExchange &ex = ranks.ex;
        std::vector<RankExchange> rx((size_t) n);
        std::vector<amvpt_counters> cnt((size_t) n);
        std::vector<uint64_t> ov_count((size_t) n, 0);
        std::mutex stat_mu;
        auto wfloats_of = [&](int r) { return groups ? (size_t) wins[(size_t) r][2] * wins[(size_t) r][3] * C : nfloat; };
        const std::string failure = ranks.run(n, [&](int r, int ph) -> std::string {
            DevState &D = cache->dev[(size_t) r];
            const size_t wfloats = wfloats_of(r);
            switch (ph) {
            case amvpt_ranks::SETUP: {   /* nothing collective */
                if (hipSetDevice(D.device) != hipSuccess) return "hipSetDevice failed";
                if (!D.st && hipStreamCreateWithFlags(&D.st, hipStreamNonBlocking) != hipSuccess) return "hipStreamCreate failed";
                if (!D.scene) {
                    if (amvpt_scene_create(sd, &D.scene) != AMVPT_OK) return amvpt_last_error();
                    std::lock_guard<std::mutex> lk(stat_mu);
                    ++cache->scene_creates;
                }
                if (!grow(D.film, D.film_bytes, wfloats * sizeof(float))) return "hipMalloc(film) failed";
                if (groups && !grow(D.ovf, D.ovf_bytes, 16 * (ov_cap + 1))) return "hipMalloc(overflow) failed";
                if (hipMemsetAsync(D.film, 0, wfloats * sizeof(float), D.st) != hipSuccess) return "hipMemset(film) failed";
                if (groups && hipMemsetAsync(D.ovf, 0, 16, D.st) != hipSuccess) return "hipMemset(overflow) failed";
                if (r == 0 && groups) {
                    if (!grow(D.quilt, D.quilt_bytes, nfloat * sizeof(float))) return "hipMalloc(quilt) failed";
                    D.recv.resize((size_t) n, nullptr); D.recv_bytes.resize((size_t) n, 0);
                    D.recv_ov.resize((size_t) n, nullptr); D.recv_ov_bytes.resize((size_t) n, 0);
                    for (int q = 1; q < n; ++q)
                        if (!grow(D.recv[(size_t) q], D.recv_bytes[(size_t) q], wfloats_of(q) * sizeof(float)))
                            return "hipMalloc(window receive) failed";
                }
                return "";
            }
            case amvpt_ranks::RENDER: {   /* this device's share; the count exchange is the only cross-device step */
                if (hipSetDevice(D.device) != hipSuccess) return "hipSetDevice failed";
                amvpt_lane_set lanes{};
                amvpt_film_window fw{};
                fw.film = D.film;
                if (groups) {
                    lanes.rect_x0 = rects[(size_t) r][0]; lanes.rect_y0 = rects[(size_t) r][1];
                    lanes.rect_width = rects[(size_t) r][2]; lanes.rect_height = rects[(size_t) r][3];
                    fw.x0 = wins[(size_t) r][0]; fw.y0 = wins[(size_t) r][1];
                    fw.width = wins[(size_t) r][2]; fw.height = wins[(size_t) r][3];
                    fw.overflow = D.ovf;
                    fw.overflow_capacity = ov_cap;
                } else {
                    amvpt_host_lane_shard(L, (uint32_t) r, (uint32_t) n, &lanes.lane_begin, &lanes.lane_end);
                    fw.width = p.film_width; fw.height = p.film_height;
                }
                rx[(size_t) r] = RankExchange{&ex, r};
                amvpt_render_opts o{};
                if (n > 1) { o.exchange = run_exchange_cb; o.exchange_ctx = &rx[(size_t) r]; }
                if (amvpt_render_ex(D.scene, views, &p, &lanes, &fw, D.st, &o, counters ? &cnt[(size_t) r] : nullptr) != AMVPT_OK)
                    return amvpt_last_error();
                if (groups && (hipMemcpyAsync(&ov_count[(size_t) r], D.ovf, 8, hipMemcpyDeviceToHost, D.st) != hipSuccess ||
                               hipStreamSynchronize(D.st) != hipSuccess))
                    return "overflow count read failed";
                return "";
            }
            case amvpt_ranks::PREPARE:   /* devices[0]: room for the peers' overflow cells */
                /* shared device: devices[0]'s thread reads every rank's film in COMBINE, so each one's is complete */
                if (shared && hipStreamSynchronize(D.st) != hipSuccess) return "hipStreamSynchronize failed";
                if (groups && r == 0 && !shared)
                    for (int q = 1; q < n; ++q)
                        if (!grow(D.recv_ov[(size_t) q], D.recv_ov_bytes[(size_t) q], 16 * std::max<uint64_t>(1, ov_count[(size_t) q])))
                            return "hipMalloc(overflow receive) failed";
                return "";
            case amvpt_ranks::COMBINE: {   /* every device is healthy here, so every collective completes */
                if (shared) {
                    /* one device: devices[0]'s thread sums the others' films (lane bands) or assembles the quilt from
                     * every rank's window and overflow cells (view groups), as the RCCL forms below do */
                    if (r == 0) {
                        if (groups && hipMemsetAsync(D.quilt, 0, nfloat * sizeof(float), D.st) != hipSuccess)
                            return "hipMemset(quilt) failed";
                        for (int q = groups ? 0 : 1; q < n; ++q) {
                            const DevState &E = cache->dev[(size_t) q];
                            const auto &w = wins[(size_t) q];
                            const amvpt_status st = groups
                                ? amvpt_film_accumulate(D.quilt, p.film_width, p.film_height, C, E.film, w[0], w[1], w[2],
                                                        w[3], E.ovf + 4, ov_count[(size_t) q], D.st)
                                : amvpt_film_accumulate(D.film, p.film_width, p.film_height, C, E.film, 0, 0, p.film_width,
                                                        p.film_height, nullptr, 0, D.st);
                            if (st != AMVPT_OK) return amvpt_last_error();
                        }
                    }
                } else if (groups) {
                    ncclComm_t comm = cache->comms[(size_t) r];
                    bool ok = ncclGroupStart() == ncclSuccess;
                    if (r == 0) {
                        for (int q = 1; q < n; ++q) {
                            ok = ok && ncclRecv(D.recv[(size_t) q], wfloats_of(q), ncclFloat, q, comm, D.st) == ncclSuccess;
                            if (ov_count[(size_t) q])
                                ok = ok && ncclRecv(D.recv_ov[(size_t) q], 4 * ov_count[(size_t) q], ncclUint32, q, comm, D.st) == ncclSuccess;
                        }
                    } else {
                        ok = ok && ncclSend(D.film, wfloats, ncclFloat, 0, comm, D.st) == ncclSuccess;
                        if (ov_count[(size_t) r])
                            ok = ok && ncclSend(D.ovf + 4, 4 * ov_count[(size_t) r], ncclUint32, 0, comm, D.st) == ncclSuccess;
                    }
                    ok = (ncclGroupEnd() == ncclSuccess) && ok;
                    if (!ok) return "ncclSend / ncclRecv of the film windows failed";
                    if (r == 0) {
                        if (hipMemsetAsync(D.quilt, 0, nfloat * sizeof(float), D.st) != hipSuccess) return "hipMemset(quilt) failed";
                        for (int q = 0; q < n; ++q) {
                            const auto &w = wins[(size_t) q];
                            const float *win = q == 0 ? D.film : D.recv[(size_t) q];
                            const uint32_t *ov = q == 0 ? D.ovf + 4 : D.recv_ov[(size_t) q];
                            if (amvpt_film_accumulate(D.quilt, p.film_width, p.film_height, C, win, w[0], w[1], w[2], w[3], ov,
                                                      ov_count[(size_t) q], D.st) != AMVPT_OK)
                                return amvpt_last_error();
                        }
                    }
                } else if (n > 1) {
                    if (ncclReduce(D.film, D.film, nfloat, ncclFloat, ncclSum, 0, cache->comms[(size_t) r], D.st) != ncclSuccess)
                        return "ncclReduce failed";
                }
                if (D.st && hipStreamSynchronize(D.st) != hipSuccess) return "hipStreamSynchronize failed";
                return "";
            }
            default: {   /* FINISH: develop / copy out on devices[0] */
                if (r != 0) return "";
                const float *frame = groups ? D.quilt : D.film;
                if (raw) {
                    if (hipMemcpy(out, frame, nfloat * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) return "hipMemcpy(film) failed";
                    return "";
                }
                const uint32_t T = p.film_alpha ? 4u : 3u;
                if (!grow(D.out, D.out_bytes, npx * T * sizeof(float))) return "hipMalloc(out) failed";
                if (amvpt_develop(frame, D.out, p.film_width, p.film_height, p.film_alpha, D.st) != AMVPT_OK)
                    return amvpt_last_error();
                if (hipStreamSynchronize(D.st) != hipSuccess ||
                    hipMemcpy(out, D.out, npx * T * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
                    return "develop / copy-out failed";
                return "";
            }
            }
        });
        if (!failure.empty()) {
            /* name the device of the failing rank */
            const size_t sp = failure.find(':');
            const int fr = std::atoi(failure.c_str() + 5);
            throw std::runtime_error("device " + std::to_string(devices[fr]) + failure.substr(sp));
        }
        ++cache->renders;
        if (counters) {
            /* lane statistics sum over the shards; per-kernel and wall times: the slowest device */
            amvpt_counters c = cnt[0];
            for (int r = 1; r < n; ++r) {
                const amvpt_counters &o = cnt[(size_t) r];
                c.lanes += o.lanes; c.vertices += o.vertices; c.reuse_lanes += o.reuse_lanes;
                c.visibility_rays += o.visibility_rays; c.view_splats += o.view_splats;
                c.splat_fallback += o.splat_fallback; c.adaptive_lanes += o.adaptive_lanes;
                c.shadow_rays += o.shadow_rays; c.nonfinite_samples += o.nonfinite_samples;
                c.negative_samples += o.negative_samples; c.pushed_paths += o.pushed_paths;
                c.film_overflow += o.film_overflow;
                c.film_range_drops += o.film_range_drops;
                c.total_ms = std::max(c.total_ms, o.total_ms);
                c.kernel_ms_primary = std::max(c.kernel_ms_primary, o.kernel_ms_primary);
                c.kernel_ms_bounce = std::max(c.kernel_ms_bounce, o.kernel_ms_bounce);
                c.kernel_ms_splat = std::max(c.kernel_ms_splat, o.kernel_ms_splat);
                for (int k = 0; k < AMVPT_K_COUNT; ++k) {
                    c.kernel_ms[k] = std::max(c.kernel_ms[k], o.kernel_ms[k]);
                    c.kernel_launches[k] = std::max(c.kernel_launches[k], o.kernel_launches[k]);
                }
            }
            *counters = c;
        }
        return 0;
    });
}

int amvpt_host_test_ranks(int n, int passes, int fail_rank, int fail_phase) {
    int status = 0;
    const int rc = amvpt_host_guarded([&] {
        if (n < 1 || n > 64 || passes < 0) throw std::runtime_error("amvpt_host_test_ranks: 1 <= n <= 64, passes >= 0");
        amvpt_ranks::Ranks ranks;
        std::mutex mu;
        bool bad_prefix = false;
        const std::string failure = ranks.run(n, [&](int r, int ph) -> std::string {
            const bool fails = r == fail_rank;
            switch (ph) {
            case amvpt_ranks::SETUP:
                return fails && fail_phase == 0 ? "injected setup failure" : "";
            case amvpt_ranks::RENDER:
                if (fails && fail_phase == 1) return "injected render failure before the exchanges";
                for (int k = 0; k < passes; ++k) {
                    if (fails && fail_phase == 2 && k == passes / 2) return "injected render failure between exchanges";
                    /* one run per rank: begin 1000 r, (r + 1)(k + 1) flagged lanes */
                    const uint64_t b = 1000ull * (uint64_t) r, c = (uint64_t) (r + 1) * (uint64_t) (k + 1);
                    uint64_t prefix = 0, total = 0;
                    if (ranks.ex.exchange(r, 1, &b, &c, &prefix, &total) != 0) return "amvpt_render: adaptive count exchange failed";
                    const uint64_t want_p = (uint64_t) r * (uint64_t) (r + 1) / 2 * (uint64_t) (k + 1);
                    const uint64_t want_t = (uint64_t) n * (uint64_t) (n + 1) / 2 * (uint64_t) (k + 1);
                    if (prefix != want_p || total != want_t) {
                        std::lock_guard<std::mutex> lk(mu);
                        bad_prefix = true;
                    }
                }
                return fails && fail_phase == 3 ? "injected render failure after the exchanges" : "";
            case amvpt_ranks::PREPARE:
                return fails && fail_phase == 4 ? "injected failure before the gather" : "";
            case amvpt_ranks::COMBINE:
                return "";
            default:
                return fails && fail_phase == 5 ? "injected finish failure" : "";
            }
        });
        if (bad_prefix) { status = 2; throw std::runtime_error("amvpt_host_test_ranks: wrong exchange prefix"); }
        if (!failure.empty()) { status = 1; throw std::runtime_error(failure); }
        return 0;
    });
    return rc == 0 ? 0 : (status ? status : 1);
}

}  // extern "C"
