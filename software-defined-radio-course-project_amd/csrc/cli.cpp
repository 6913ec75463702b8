// cli.cpp — `fmrx [<mode> <channels>] [--batch N] [--device D] [--rf-taps T] [--mono-product]`:
// the drop-in for the reference's `project` executable (src/project.cpp:273-390).  Reads u8 I/Q
// from stdin and writes raw S16LE to stdout under project's process contract:
//   * arguments as project.cpp:278-299: fewer than two positional arguments run the default
//     mode 0 (a lone one is ignored, as `project 3` ignores it), exactly two are <mode>
//     <channels> (atoi; out of range -> message, exit 1), more print the usage and exit 1;
//   * the output is ALWAYS the 2-channel interleaved R,L stream of project.cpp:179-195:
//     `channels` is only logged (:301-302), the reference has no mono-only output;
//   * --mono-product (an fmrx extension, not a project argument) writes the 1-channel mono
//     product instead (project.cpp:146's mono resample with a private history, quantised like
//     :187) -- the BASELINE headline path.
//
// Streaming runtime.  The reference splits the work into a producer thread
// (read + RF front end, project.cpp:48-84) and a consumer thread (audio back end, :132-196)
// joined by a bounded queue of depth 3 (QUEUE_CAPACITY, :17).  Here the whole receive runs on
// the GPU and the queue becomes a ring of 3 batch slots, each a pinned host input/output pair
// and a device input/output pair, cycled by three agents:
//   reader thread : fread whole blocks straight into a free slot's pinned input;
//   main thread   : H2D on a copy stream -> (event) -> fmrx_process_device on the context's
//                   stream -> (event) -> D2H on an output stream, all asynchronous;
//   writer thread : waits for the slot's D2H event, writes its PCM, frees the slot.
// so the upload of batch i+1, the receive of batch i and the write of batch i-1 overlap.
// Stream order keeps the receiver state sequential (one context, one compute stream).
// Unlike the reference (project.cpp:51-54, which exit(1)s while blocks are still queued) every
// full block read is processed before the process exits 0; a trailing partial block is
// dropped, as in the reference.
#include <hip/hip_runtime_api.h>

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

constexpr int kSlots = 3;  // project.cpp:17 QUEUE_CAPACITY

class IndexQueue {
  public:
    void push(int v) {
        std::lock_guard<std::mutex> lk(m_);
        q_.push_back(v);
        cv_.notify_all();
    }
    int pop() {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        const int v = q_.front();
        q_.pop_front();
        return v;
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<int> q_;
};

struct Slot {
    uint8_t* h_in = nullptr;   // pinned
    int16_t* h_out = nullptr;  // pinned
    uint8_t* d_in = nullptr;
    int16_t* d_out = nullptr;
    hipEvent_t uploaded{}, computed{}, downloaded{};
    size_t blocks = 0;
    bool last = false;
};

void usage(const char* argv0) {
    std::fprintf(stderr,
                 "Usage: %s\nor \nUsage %s <mode> <channels>\n"
                 "\t\t<mode> is a value from 0 to 3\n\t\t   <channels> is either 1 or 2\n"
                 "options (fmrx): [--batch N] [--device D] [--rf-taps T] [--mono-product]\n",
                 argv0, argv0);
}

[[noreturn]] void die_hip(hipError_t e, const char* what) {
    std::fprintf(stderr, "fmrx: %s: %s\n", what, hipGetErrorString(e));
    std::fflush(stdout);
    std::_Exit(1);
}

#define CLI_HIP(x)                              \
    do {                                        \
        const hipError_t e_ = (x);              \
        if (e_ != hipSuccess) die_hip(e_, #x);  \
    } while (0)

}  // namespace

int main(int argc, char** argv) {
    int mode = 0, channels = 1, batch = 16, device = 0, rf_taps = 51;
    bool mono_product = false;
    std::vector<const char*> pos;
    for (int i = 1; i < argc; i++) {
        if (!std::strcmp(argv[i], "--batch") && i + 1 < argc) batch = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rf-taps") && i + 1 < argc) rf_taps = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--mono-product")) mono_product = true;
        else if (argv[i][0] == '-' && argv[i][1] != '\0' && !(argv[i][1] >= '0' && argv[i][1] <= '9')) {
            usage(argv[0]);
            return 1;
        } else pos.push_back(argv[i]);  // "-1" is a (negative, invalid) mode as in project
    }
    if (pos.size() < 2) {  // project.cpp:278-279 (argc < 3): argv[1] alone is not parsed
        std::fprintf(stderr, "Operating in default mode 0, mono\n");
    } else if (pos.size() == 2) {  // :280-291
        mode = std::atoi(pos[0]);
        channels = std::atoi(pos[1]);
        if (mode < 0 || mode > 3) { std::fprintf(stderr, "Invalid mode: %d!\n", mode); return 1; }
        if (channels < 1 || channels > 2) { std::fprintf(stderr, "Invaild channel: %d!\n", channels); return 1; }  // project.cpp:289, verbatim
    } else {  // :292-298
        usage(argv[0]);
        return 1;
    }
    if (batch < 1) batch = 1;
    std::fprintf(stderr, "Operating in mode %d, %s\n", mode, channels == 1 ? "mono" : "stereo");

    // project.cpp always writes the stereo R,L stream whatever `channels` says (:179-195).
    const int out_channels = mono_product ? FMRX_MONO : FMRX_STEREO;
    fmrx_config cfg;
    if (fmrx_config_default(&cfg, mode, out_channels) != FMRX_OK) {
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
    const size_t in_cap = geo.block_bytes * (size_t)batch;
    const size_t out_cap = geo.pcm_samples * (size_t)batch;

    CLI_HIP(hipSetDevice(device));
    hipStream_t compute = static_cast<hipStream_t>(fmrx_stream(ctx));
    hipStream_t up, down;
    CLI_HIP(hipStreamCreateWithFlags(&up, hipStreamNonBlocking));
    CLI_HIP(hipStreamCreateWithFlags(&down, hipStreamNonBlocking));
    Slot slots[kSlots];
    for (Slot& s : slots) {
        CLI_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_in), in_cap, hipHostMallocDefault));
        CLI_HIP(hipHostMalloc(reinterpret_cast<void**>(&s.h_out), out_cap * sizeof(int16_t), hipHostMallocDefault));
        CLI_HIP(hipMalloc(reinterpret_cast<void**>(&s.d_in), in_cap));
        CLI_HIP(hipMalloc(reinterpret_cast<void**>(&s.d_out), out_cap * sizeof(int16_t)));
        CLI_HIP(hipEventCreateWithFlags(&s.uploaded, hipEventDisableTiming));
        CLI_HIP(hipEventCreateWithFlags(&s.computed, hipEventDisableTiming));
        CLI_HIP(hipEventCreateWithFlags(&s.downloaded, hipEventDisableTiming));
    }

    IndexQueue free_q, filled_q, done_q;
    for (int i = 0; i < kSlots; i++) free_q.push(i);

    std::thread reader([&] {
        for (;;) {
            const int i = free_q.pop();
            Slot& s = slots[i];
            size_t got = 0;
            while (got < in_cap) {
                const size_t r = std::fread(s.h_in + got, 1, in_cap - got, stdin);
                if (r == 0) break;
                got += r;
            }
            s.blocks = got / geo.block_bytes;
            s.last = got < in_cap;
            filled_q.push(i);
            if (s.last) return;
        }
    });
    std::thread writer([&] {
        for (;;) {
            const int i = done_q.pop();
            Slot& s = slots[i];
            if (s.blocks > 0) {
                CLI_HIP(hipEventSynchronize(s.downloaded));
                std::fwrite(s.h_out, sizeof(int16_t), s.blocks * geo.pcm_samples, stdout);
            }
            if (s.last) return;
            free_q.push(i);
        }
    });

    for (;;) {
        const int i = filled_q.pop();
        Slot& s = slots[i];
        if (s.blocks > 0) {
            CLI_HIP(hipMemcpyAsync(s.d_in, s.h_in, s.blocks * geo.block_bytes, hipMemcpyHostToDevice, up));
            CLI_HIP(hipEventRecord(s.uploaded, up));
            CLI_HIP(hipStreamWaitEvent(compute, s.uploaded, 0));
            if (fmrx_process_device(ctx, s.d_in, s.blocks, s.d_out) != FMRX_OK) {
                std::fprintf(stderr, "fmrx: %s\n", fmrx_last_error());
                std::fflush(stdout);
                std::_Exit(1);
            }
            CLI_HIP(hipEventRecord(s.computed, compute));
            CLI_HIP(hipStreamWaitEvent(down, s.computed, 0));
            CLI_HIP(hipMemcpyAsync(s.h_out, s.d_out, s.blocks * geo.pcm_samples * sizeof(int16_t),
                                   hipMemcpyDeviceToHost, down));
            CLI_HIP(hipEventRecord(s.downloaded, down));
        }
        done_q.push(i);
        if (s.last) break;
    }
    reader.join();
    writer.join();
    std::fflush(stdout);
    for (Slot& s : slots) {
        (void)hipHostFree(s.h_in);
        (void)hipHostFree(s.h_out);
        (void)hipFree(s.d_in);
        (void)hipFree(s.d_out);
        (void)hipEventDestroy(s.uploaded);
        (void)hipEventDestroy(s.computed);
        (void)hipEventDestroy(s.downloaded);
    }
    (void)hipStreamDestroy(up);
    (void)hipStreamDestroy(down);
    fmrx_destroy(ctx);
    std::fprintf(stderr, "End of input stream reached!\n");
    return 0;
}
