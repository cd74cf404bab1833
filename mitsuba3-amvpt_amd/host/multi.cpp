/*
 * multi.cpp -- Integrator::render over several GPUs of one node, without torch.
 *
 * The path shards by lanes: every pass is the lane space [0, W*H*spp_per_pass) and a lane seeds its
 * sampler from its global index (TEA(seed_value, lane), mvpath.cpp:227-235), so device r renders the
 * contiguous range amvpt_host_lane_shard(L, r, n) of every pass (a band of quilt rows) and the frame
 * is bit-for-bit the single-GPU one up to float summation order.  The only data-path collective is
 * the sum of the per-device RGBW ImageBlocks: one RCCL reduce (sum, fp32) onto devices[0] over
 * xGMI, then develop there (hdrfilm.cpp:304-418).  With adaptive > 0 the fill compacts the whole
 * pass (mvpath_multi.h:79-115), so the devices exchange their per-pass flagged-lane counts through
 * amvpt_set_adaptive_exchange: an in-process all-gather between the device threads.
 *
 * One host thread per device drives its own scene copy, stream and film (8(b) "Threading").  A
 * device whose render fails still joins the reduce with its (zeroed) film, so no peer blocks in
 * the collective; the call then reports the first error.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/amvpt.h"
#include "../../include/amvpt_host.h"

namespace {

/* per-pass all-gather of the adaptive fill's local counts between the device threads */
struct CountExchange {
    std::mutex mu;
    std::condition_variable cv;
    int world = 1;
    int arrived = 0;
    bool aborted = false;     /* a device failed: the others' exchanges fail instead of waiting */
    uint64_t generation = 0;
    std::vector<uint64_t> counts, published;

    int exchange(int rank, uint64_t local, uint64_t *prefix, uint64_t *total) {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return -1;
        const uint64_t gen = generation;
        counts[(size_t) rank] = local;
        if (++arrived == world) {
            published = counts;
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen || aborted; });
            if (generation == gen) return -1;
        }
        uint64_t p = 0, t = 0;
        for (int r = 0; r < world; ++r) {
            if (r < rank) p += published[(size_t) r];
            t += published[(size_t) r];
        }
        *prefix = p;
        *total = t;
        return 0;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

thread_local int t_rank = 0;

int exchange_cb(void *ctx, uint64_t local, uint64_t *prefix, uint64_t *total) {
    return static_cast<CountExchange *>(ctx)->exchange(t_rank, local, prefix, total);
}

struct DeviceResult {
    std::string error;
    amvpt_counters counters{};
};

}  // namespace

int amvpt_host_guarded_call(int (*fn)(void *), void *ctx);   /* scene.cpp: exception -> status + last_error */
template <class F> static int amvpt_host_guarded(F &&f) {
    return amvpt_host_guarded_call([](void *c) { return (*static_cast<F *>(c))(); }, &f);
}

extern "C" {

void amvpt_host_lane_shard(uint64_t lanes, uint32_t rank, uint32_t world, uint64_t *begin, uint64_t *end) {
    const uint64_t q = world ? lanes / world : 0, r = world ? lanes % world : 0;
    const uint64_t b = rank * q + std::min<uint64_t>(rank, r);
    *begin = b;
    *end = b + q + (rank < r ? 1u : 0u);
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

        std::vector<ncclComm_t> comms((size_t) n);
        if (ncclCommInitAll(comms.data(), n, devices) != ncclSuccess) throw std::runtime_error("ncclCommInitAll failed");
        struct Comms {
            std::vector<ncclComm_t> &c;
            ~Comms() { for (auto x : c) if (x) (void) ncclCommDestroy(x); }
        } comms_guard{comms};

        CountExchange ex;
        ex.world = n;
        ex.counts.assign((size_t) n, 0);
        (void) amvpt_set_adaptive_exchange(n > 1 ? exchange_cb : nullptr, n > 1 ? &ex : nullptr);
        struct ResetExchange { ~ResetExchange() { (void) amvpt_set_adaptive_exchange(nullptr, nullptr); } } reset_ex;

        std::vector<DeviceResult> res((size_t) n);
        std::vector<std::thread> threads;
        for (int r = 0; r < n; ++r) {
            threads.emplace_back([&, r] {
                t_rank = r;
                DeviceResult &R = res[(size_t) r];
                amvpt_scene *dsc = nullptr;
                hipStream_t st = nullptr;
                float *film = nullptr, *dev_out = nullptr;
                auto fail = [&](const std::string &m) { if (R.error.empty()) R.error = m; };
                if (hipSetDevice(devices[r]) != hipSuccess) fail("hipSetDevice failed");
                if (R.error.empty() && hipStreamCreate(&st) != hipSuccess) fail("hipStreamCreate failed");
                if (R.error.empty() && hipMalloc(&film, nfloat * sizeof(float)) != hipSuccess) fail("hipMalloc(film) failed");
                if (R.error.empty() && hipMemsetAsync(film, 0, nfloat * sizeof(float), st) != hipSuccess) fail("hipMemset(film) failed");
                if (R.error.empty() && amvpt_scene_create(sd, &dsc) != AMVPT_OK) fail(amvpt_last_error());
                uint64_t b, e;
                amvpt_host_lane_shard(L, (uint32_t) r, (uint32_t) n, &b, &e);
                if (R.error.empty() &&
                    amvpt_render(dsc, views, &p, b, e, film, st, counters ? &R.counters : nullptr) != AMVPT_OK) {
                    fail(amvpt_last_error());
                    ex.abort();
                    (void) hipMemsetAsync(film, 0, nfloat * sizeof(float), st);
                }
                /* every device joins the reduce (a missing peer would block the others in it) */
                if (film && ncclReduce(film, film, nfloat, ncclFloat, ncclSum, 0, comms[(size_t) r], st) != ncclSuccess)
                    fail("ncclReduce failed");
                if (st && hipStreamSynchronize(st) != hipSuccess) fail("hipStreamSynchronize failed");
                if (r == 0 && film) {
                    if (raw) {
                        if (hipMemcpy(out, film, nfloat * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
                            fail("hipMemcpy(film) failed");
                    } else {
                        const uint32_t T = p.film_alpha ? 4u : 3u;
                        if (hipMalloc(&dev_out, npx * T * sizeof(float)) != hipSuccess) fail("hipMalloc(out) failed");
                        else if (amvpt_develop(film, dev_out, p.film_width, p.film_height, p.film_alpha, st) != AMVPT_OK)
                            fail(amvpt_last_error());
                        else if (hipStreamSynchronize(st) != hipSuccess ||
                                 hipMemcpy(out, dev_out, npx * T * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess)
                            fail("develop / copy-out failed");
                    }
                }
                if (dev_out) (void) hipFree(dev_out);
                if (film) (void) hipFree(film);
                if (dsc) amvpt_scene_destroy(dsc);
                if (st) (void) hipStreamDestroy(st);
            });
        }
        for (auto &t : threads) t.join();
        for (int r = 0; r < n; ++r)
            if (!res[(size_t) r].error.empty()) throw std::runtime_error("device " + std::to_string(devices[r]) + ": " + res[(size_t) r].error);
        if (counters) {
            /* lane statistics sum over the shards; per-kernel and wall times: the slowest device */
            amvpt_counters c = res[0].counters;
            for (int r = 1; r < n; ++r) {
                const amvpt_counters &o = res[(size_t) r].counters;
                c.lanes += o.lanes; c.vertices += o.vertices; c.reuse_lanes += o.reuse_lanes;
                c.visibility_rays += o.visibility_rays; c.view_splats += o.view_splats;
                c.splat_fallback += o.splat_fallback; c.adaptive_lanes += o.adaptive_lanes;
                c.shadow_rays += o.shadow_rays; c.nonfinite_samples += o.nonfinite_samples;
                c.negative_samples += o.negative_samples;
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

}  // extern "C"
