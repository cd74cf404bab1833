/*
 * ranks.h -- the host-side coordination of amvpt_host_render_multi's device threads, free of HIP and
 * RCCL so that its failure handling can be exercised on the CPU (amvpt_host_test_ranks).
 *
 * One thread per rank walks the phases SETUP -> RENDER -> PREPARE -> COMBINE -> FINISH.  The first three
 * end at an in-process barrier where every rank reports whether it is healthy; a rank continues only
 * when all were, so the collective phase (COMBINE: ncclReduce / ncclSend + ncclRecv) is entered by
 * every rank or by none and no peer is ever left blocked inside RCCL.  During RENDER the adaptive fill's
 * per-pass count exchange (RunExchange, an all-gather between the threads) is the only cross-rank step;
 * a rank whose render fails aborts it, which releases every peer waiting in it.  The error the caller
 * sees is the first rank's own failure, not the "a peer failed" echoes it caused in the others.
 */
#pragma once
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace amvpt_ranks {

/* in-process barrier; each thread reports whether it is healthy and learns whether all were */
struct Barrier {
    std::mutex mu;
    std::condition_variable cv;
    int world = 1, arrived = 0;
    uint64_t generation = 0;
    bool all_ok = true, published_ok = true;
    bool wait(bool ok) {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t gen = generation;
        all_ok = all_ok && ok;
        if (++arrived == world) {
            published_ok = all_ok;
            all_ok = true;
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
        return published_ok;
    }
};

/* per-pass all-gather of the adaptive fill's per-run counts (amvpt_run_exchange_fn): a run's prefix is
 * every count of every rank whose run starts below it (runs of different ranks are disjoint); a failed
 * rank aborts it so no peer waits */
struct RunExchange {
    std::mutex mu;
    std::condition_variable cv;
    int world = 1, arrived = 0;
    bool aborted = false;
    uint64_t generation = 0;
    std::vector<std::vector<uint64_t>> begins, counts, pub_b, pub_c;

    void reset(int n) {
        world = n;
        arrived = 0;
        aborted = false;
        begins.assign((size_t) n, {});
        counts.assign((size_t) n, {});
    }
    int exchange(int rank, uint32_t n, const uint64_t *b, const uint64_t *c, uint64_t *prefix, uint64_t *total) {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return -1;
        const uint64_t gen = generation;
        begins[(size_t) rank].assign(b, b + n);
        counts[(size_t) rank].assign(c, c + n);
        if (++arrived == world) {
            pub_b = begins;
            pub_c = counts;
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen || aborted; });
            if (generation == gen) return -1;
        }
        uint64_t t = 0;
        for (int r = 0; r < world; ++r)
            for (uint64_t x : pub_c[(size_t) r]) t += x;
        for (uint32_t i = 0; i < n; ++i) {
            uint64_t p = 0;
            for (int r = 0; r < world; ++r)
                for (size_t j = 0; j < pub_b[(size_t) r].size(); ++j)
                    if (pub_b[(size_t) r][j] < b[i]) p += pub_c[(size_t) r][j];
            prefix[i] = p;
        }
        *total = t;
        return 0;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

enum Phase : int { SETUP = 0, RENDER = 1, PREPARE = 2, COMBINE = 3, FINISH = 4, N_PHASES = 5 };
inline const char *phase_name(int ph) {
    static const char *k[] = {"setup", "the render", "the gather's preparation", "the combine", "the finish"};
    return ph >= 0 && ph < N_PHASES ? k[ph] : "?";
}

/*
 * Run n rank threads through the phases; phase(rank, ph) returns "" on success or the rank's error.
 * Returns "" when every rank succeeded, else the first rank's own error as "rank r: <error>".
 */
struct Ranks {
    Barrier bar;
    RunExchange ex;
    std::string run(int n, const std::function<std::string(int, int)> &phase) {
        bar.world = n;
        bar.arrived = 0;
        ex.reset(n);
        std::vector<std::string> err((size_t) n);
        /* the error only reports a peer's failure; one byte per rank (vector<bool> packs the ranks' flags into
         * shared words, and the threads' concurrent writes lost each other's updates) */
        std::vector<uint8_t> echo((size_t) n, 0);
        std::vector<std::thread> threads;
        for (int r = 0; r < n; ++r)
            threads.emplace_back([&, r] {
                std::string &e = err[(size_t) r];
                for (int ph = SETUP; ph < N_PHASES; ++ph) {
                    bool aborted_before = false;
                    if (ph == RENDER) {
                        std::lock_guard<std::mutex> lk(ex.mu);
                        aborted_before = ex.aborted;
                    }
                    std::string m = phase(r, ph);
                    if (!m.empty() && e.empty()) {
                        e = m;
                        if (ph == RENDER) {
                            std::lock_guard<std::mutex> lk(ex.mu);
                            echo[(size_t) r] = aborted_before || ex.aborted;   /* a peer aborted the exchange first */
                        }
                    }
                    if (ph == RENDER && !e.empty() && !echo[(size_t) r]) ex.abort();
                    if (ph <= PREPARE && !bar.wait(e.empty())) {
                        if (e.empty()) {
                            e = std::string("a peer device failed during ") + phase_name(ph);
                            echo[(size_t) r] = true;
                        }
                        return;
                    }
                    if (!e.empty()) return;
                }
            });
        for (auto &t : threads) t.join();
        for (int pass = 0; pass < 2; ++pass)   /* own failures first, then echoes */
            for (int r = 0; r < n; ++r)
                if (!err[(size_t) r].empty() && (echo[(size_t) r] != 0) == (pass == 1))
                    return "rank " + std::to_string(r) + ": " + err[(size_t) r];
        return "";
    }
};

}  // namespace amvpt_ranks
