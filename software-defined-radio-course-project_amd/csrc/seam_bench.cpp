// seam_bench.cpp -- bin/fmrx_seam: the per-block seam timed from C++, the way the reference's own
// program drives its stages (src/project.cpp): one 12,800-byte mode-0 block a call,
// fmrx_rf_block then fmrx_audio_block (rf_thread :48-84, audio_thread :132-196).
//
//   serial       one context, both stages per block on one thread
//   two_threads  two contexts, project.cpp's producer / consumer: thread A runs fmrx_rf_block and
//                queues the demod block (a bounded queue of QUEUE_CAPACITY = 3, project.cpp:17),
//                thread B runs fmrx_audio_block on it
//
// The synthetic stream (fmrx_synth_host seed 5, as tools/bench_seam.py) is generated first; the
// two legs' PCM must be equal.  One JSON line on stdout.  Measurement tooling, not the product.
//
//   fmrx_seam [--blocks 3000] [--warmup 100] [--start 0]
#include <fmrx.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

double secs(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

[[noreturn]] void die(const char* what) {
    std::fprintf(stderr, "fmrx_seam: %s: %s\n", what, fmrx_last_error());
    std::exit(1);
}

struct Stats {
    double mean, median, p99, max;
};
Stats stats_ms(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    double s = 0;
    for (double x : v) s += x;
    const size_t n = v.size();
    return {1e3 * s / n, 1e3 * (n % 2 ? v[n / 2] : 0.5 * (v[n / 2 - 1] + v[n / 2])),
            1e3 * v[std::min(n - 1, (size_t)(0.99 * n))], 1e3 * v[n - 1]};
}
std::string json(const Stats& s) {
    char b[160];
    std::snprintf(b, sizeof b, "{\"mean\": %.4f, \"median\": %.4f, \"p99\": %.4f, \"max\": %.4f}", s.mean, s.median,
                  s.p99, s.max);
    return b;
}

fmrx_ctx* make_ctx() {
    fmrx_config cfg;
    if (fmrx_config_default(&cfg, 0, FMRX_STEREO)) die("config");
    fmrx_ctx* c = nullptr;
    if (fmrx_create(&cfg, &c)) die("create");
    return c;
}

}  // namespace

int main(int argc, char** argv) {
    long blocks = 3000, warmup = 100, start = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!std::strcmp(argv[i], "--blocks")) blocks = std::atol(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--warmup")) warmup = std::atol(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--start")) start = std::atol(argv[i + 1]);
    }
    fmrx_config cfg;
    fmrx_geometry_t geo;
    if (fmrx_config_default(&cfg, 0, FMRX_STEREO) || fmrx_geometry(&cfg, &geo)) die("geometry");
    const size_t bb = geo.block_bytes, nif = geo.if_samples, npcm = geo.pcm_samples;
    const long nb = start + warmup + blocks;
    std::vector<uint8_t> iq((size_t)nb * bb);
    if (fmrx_synth_host(5, geo.rf_fs, 0, iq.size() / 2, iq.data())) die("synth");
    const double budget = (double)(bb / 2) / geo.rf_fs;  // seconds of signal a block

    // serial: one context
    std::vector<int16_t> pcm1((size_t)nb * npcm), pcm2((size_t)nb * npcm);
    std::vector<float> demod((size_t)nb * nif);
    std::vector<double> t_rf, t_au, t_blk;
    fmrx_ctx* c = make_ctx();
    if (start > 0 && fmrx_process(c, iq.data(), (size_t)start, pcm1.data())) die("process");
    for (long b = start; b < nb; b++) {
        const auto t0 = Clock::now();
        if (fmrx_rf_block(c, iq.data() + (size_t)b * bb, 1, demod.data() + (size_t)b * nif)) die("rf_block");
        const auto t1 = Clock::now();
        if (fmrx_audio_block(c, demod.data() + (size_t)b * nif, 1, pcm1.data() + (size_t)b * npcm)) die("audio_block");
        const auto t2 = Clock::now();
        if (b >= start + warmup) {
            t_rf.push_back(secs(t0, t1));
            t_au.push_back(secs(t1, t2));
            t_blk.push_back(secs(t0, t2));
        }
    }
    fmrx_destroy(c);
    double tot = 0;
    for (double x : t_blk) tot += x;

    // two threads, two contexts, project.cpp's bounded queue between them
    fmrx_ctx* ca = make_ctx();
    fmrx_ctx* cb = make_ctx();
    if (start > 0 && (fmrx_process(ca, iq.data(), (size_t)start, pcm2.data()) ||
                      fmrx_process(cb, iq.data(), (size_t)start, pcm2.data())))
        die("process");
    std::deque<long> q;
    std::mutex mu;
    std::condition_variable cv;
    Clock::time_point t_start{}, t_end{};
    std::thread rf([&] {
        for (long b = start; b < nb; b++) {
            if (b == start + warmup) t_start = Clock::now();
            if (fmrx_rf_block(ca, iq.data() + (size_t)b * bb, 1, demod.data() + (size_t)b * nif)) die("rf_block");
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return q.size() < 3; });  // QUEUE_CAPACITY (project.cpp:17, :73)
            q.push_back(b);
            cv.notify_all();
        }
        std::unique_lock<std::mutex> lk(mu);
        q.push_back(-1);
        cv.notify_all();
    });
    std::thread au([&] {
        for (;;) {
            long b;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return !q.empty(); });
                b = q.front();
                q.pop_front();
                cv.notify_all();
            }
            if (b < 0) break;
            if (fmrx_audio_block(cb, demod.data() + (size_t)b * nif, 1, pcm2.data() + (size_t)b * npcm))
                die("audio_block");
        }
        t_end = Clock::now();
    });
    rf.join();
    au.join();
    fmrx_destroy(ca);
    fmrx_destroy(cb);
    const double span = secs(t_start, t_end);
    const bool equal = std::memcmp(pcm1.data() + (size_t)start * npcm, pcm2.data() + (size_t)start * npcm,
                                   (size_t)(nb - start) * npcm * sizeof(int16_t)) == 0;
    std::printf("{\"driver\": \"bin/fmrx_seam (C++, project.cpp's call pattern)\", \"blocks\": %ld, \"warmup\": %ld, "
                "\"start_block\": %ld, \"block_budget_ms\": %.4f, "
                "\"serial\": {\"rf_block_ms\": %s, \"audio_block_ms\": %s, \"block_ms\": %s, \"x_realtime\": %.2f}, "
                "\"two_threads\": {\"x_realtime\": %.2f, \"seconds\": %.4f, \"pcm_equals_serial\": %s}}\n",
                blocks, warmup, start, 1e3 * budget, json(stats_ms(t_rf)).c_str(), json(stats_ms(t_au)).c_str(),
                json(stats_ms(t_blk)).c_str(), blocks * budget / tot, blocks * budget / span, span,
                equal ? "true" : "false");
    return equal ? 0 : 2;
}
