// cli.cpp — `fmrx [mode channels] [--batch N] [--device D]`: the drop-in for the reference's
// `project` executable (src/project.cpp:273-390).  Reads u8 I/Q from stdin, writes raw S16LE
// to stdout: stereo = 2 channels interleaved R,L exactly like project.cpp:179-195; mono =
// 1 channel (the private-history mono product; project.cpp logs `channels` but ignores it).
//
// Threading mirrors project.cpp's producer/consumer split: a reader thread fills batches of
// whole blocks into a bounded queue of depth 3 (QUEUE_CAPACITY, project.cpp:17) and the main
// thread runs each batch through libfmrx on the GPU and writes the PCM.  Unlike the reference
// (project.cpp:51-54, which exit(1)s while blocks are still queued) every full block read is
// processed before the process exits 0; a trailing partial block is dropped, as in the
// reference.
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "fmrx.h"

namespace {

struct Batch {
    std::vector<uint8_t> bytes;
    size_t blocks = 0;
    bool last = false;
};

class BoundedQueue {
  public:
    explicit BoundedQueue(size_t cap) : cap_(cap) {}
    void push(Batch&& b) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return q_.size() < cap_; });
        q_.push_back(std::move(b));
        cv_.notify_all();
    }
    Batch pop() {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        Batch b = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return b;
    }

  private:
    size_t cap_;
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<Batch> q_;
};

void usage(const char* argv0) {
    std::fprintf(stderr,
                 "Usage: %s [<mode> <channels>] [--batch N] [--device D] [--rf-taps T]\n"
                 "\t<mode> is a value from 0 to 3, <channels> is either 1 or 2\n",
                 argv0);
}

}  // namespace

int main(int argc, char** argv) {
    int mode = 0, channels = 1, batch = 16, device = 0, rf_taps = 51;
    std::vector<const char*> pos;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--batch") && i + 1 < argc) batch = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rf-taps") && i + 1 < argc) rf_taps = std::atoi(argv[++i]);
        else if (argv[i][0] == '-') { usage(argv[0]); return 1; }
        else pos.push_back(argv[i]);
    }
    if (pos.size() == 2) {
        mode = std::atoi(pos[0]);
        channels = std::atoi(pos[1]);
    } else if (!pos.empty()) {
        usage(argv[0]);
        return 1;
    } else {
        std::fprintf(stderr, "Operating in default mode 0, mono\n");
    }
    if (mode < 0 || mode > 3) { std::fprintf(stderr, "Invalid mode: %d!\n", mode); return 1; }
    if (channels < 1 || channels > 2) { std::fprintf(stderr, "Invalid channel: %d!\n", channels); return 1; }
    if (batch < 1) batch = 1;
    std::fprintf(stderr, "Operating in mode %d, %s\n", mode, channels == 1 ? "mono" : "stereo");

    fmrx_config cfg;
    if (fmrx_config_default(&cfg, mode, channels) != FMRX_OK) {
        std::fprintf(stderr, "fmrx: %s\n", fmrx_last_error());
        return 1;
    }
    cfg.device = device;
    cfg.rf_taps = rf_taps;
    fmrx_geometry_t geo;
    fmrx_ctx* ctx = nullptr;
    if (fmrx_geometry(&cfg, &geo) != FMRX_OK || fmrx_create(&cfg, &ctx) != FMRX_OK) {
        std::fprintf(stderr, "fmrx: %s\n", fmrx_last_error());
        return 1;
    }

    BoundedQueue queue(3);
    std::thread reader([&] {
        for (;;) {
            Batch b;
            b.bytes.resize(geo.block_bytes * (size_t)batch);
            size_t got = 0;
            while (got < b.bytes.size()) {
                const size_t r = std::fread(b.bytes.data() + got, 1, b.bytes.size() - got, stdin);
                if (r == 0) break;
                got += r;
            }
            b.blocks = got / geo.block_bytes;
            b.last = got < b.bytes.size();
            queue.push(std::move(b));
            if (got < geo.block_bytes * (size_t)batch) return;
        }
    });

    int rc = 0;
    std::vector<int16_t> pcm;
    for (;;) {
        Batch b = queue.pop();
        if (b.blocks > 0) {
            pcm.resize(b.blocks * geo.pcm_samples);
            if (fmrx_process(ctx, b.bytes.data(), b.blocks, pcm.data()) != FMRX_OK) {
                std::fprintf(stderr, "fmrx: %s\n", fmrx_last_error());
                rc = 1;
                break;
            }
            std::fwrite(pcm.data(), sizeof(int16_t), pcm.size(), stdout);
        }
        if (b.last) break;
    }
    std::fflush(stdout);
    if (rc) {
        reader.detach();
        fmrx_destroy(ctx);
        std::_Exit(rc);
    }
    reader.join();
    fmrx_destroy(ctx);
    std::fprintf(stderr, "End of input stream reached!\n");
    return 0;
}
