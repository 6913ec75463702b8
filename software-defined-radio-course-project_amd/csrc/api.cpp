// api.cpp — the C ABI of include/fmrx.h: context lifetime, per-stream state, the block-
// streaming entry points and the filter.h primitive mirror.  Host C++ driving the HIP
// kernels of mono_fused.hip / stereo.hip / prims.hip on one device and one HIP stream per
// context.  No CPU compute path exists: every numeric result comes from a GPU kernel.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fmrx.h"
#include "fmrx_internal.h"
#include "synth.h"

using namespace fmrx;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIPCHK(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess)                                                          \
            return fail(FMRX_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                        __FILE__, __LINE__);                                           \
    } while (0)

constexpr int kDemodHist = 64;   // demod samples kept in front of each call (>= bp_taps-1)
constexpr int kMixTail = 64;     // must match stereo.hip kTail
constexpr uint32_t kStateMagic = 0x46524D58u;  // "FMRX"
constexpr uint32_t kStateVersion = 2;  // 2: + flags word (bit 0: audio history stale after fmrx_seek)
constexpr int kStateHdrWords = 10;  // magic, version, mode, channels, rf_taps, n_streams, halo, audio_hist, flags, 0

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int ensure(size_t count) {
        if (count <= n) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(T)) != hipSuccess) {
            p = nullptr;
            return fail(FMRX_ENOMEM, "hipMalloc of %zu bytes failed", count * sizeof(T));
        }
        n = count;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

// Pinned host memory, mapped into the device's address space (hipHostMalloc: kernels read and
// write it through the same pointer): the staging of the host-buffer entry points' small calls
// (the reference's per-block seam, project.cpp:48-84 / 132-196): the input goes to the device by
// DMA from it, the kernels write their output into it in place -- one copy operation on the stream
// and one host memcpy each way.
template <class T>
struct PinnedBuf {
    T* p = nullptr;
    size_t n = 0;
    int ensure(size_t count) {
        if (count <= n) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T), hipHostMallocDefault) !=
            hipSuccess) {
            p = nullptr;
            return fail(FMRX_ENOMEM, "hipHostMalloc of %zu bytes failed", count * sizeof(T));
        }
        n = count;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

// calls up to this many input bytes go through the pinned staging (larger ones: device buffers
// and hipMemcpyAsync, whose DMA beats kernels reading host memory at that size)
constexpr size_t kPinnedCallBytes = (size_t)4 << 20;

}  // namespace

struct fmrx_ctx {
    mutable std::recursive_mutex mu;  // every entry point holds it: one call on a context at a time
    fmrx_config cfg{};
    fmrx_geometry_t geo{};
    ModeConstants mc{};
    hipStream_t stream = nullptr;
    // taps (host) and device copies
    std::vector<float> rf, audio, ch, ca;
    MonoTaps mono_taps{};
    DevBuf<float> d_audio, d_rf;
    DevBuf<float> d_audio_rows;   // modes 2/3: the audio prototype by phase (kAudioRow floats per row)
    // RF state: the raw bytes preceding the next call, double-buffered
    size_t halo_bytes = 0;
    DevBuf<uint8_t> d_halo[2];
    int halo_cur = 0;
    // audio state of the mono product: last (audio_taps_total - 1) demod samples
    int audio_hist = 0;
    DevBuf<float> d_audio_hist;
    bool audio_hist_stale = false;  // after fmrx_seek, until a fused call refreshes it
    // stereo engine state
    DevBuf<float> d_demod;        // n_streams x (kDemodHist + cap_if)
    size_t demod_stride = 0;
    DevBuf<float> d_channel, d_carrier;
    DevBuf<float> d_pll;          // n_streams x 8
    DevBuf<float> d_mix_tail;     // n_streams x kMixTail
    DevBuf<float> d_mono_state;   // n_streams x 8
    // RDS front half state (project.cpp:200-271; not part of the checkpoint blob)
    DevBuf<float> d_rds_taps;     // 54-60 kHz taps, then 113.5-114.5 kHz taps
    DevBuf<float> d_rds_dhist;    // n_streams x kRdsDemodHist
    DevBuf<float> d_rds_chan;     // n_streams x (kRdsChanHist + cap)
    size_t rds_chan_stride = 0;
    DevBuf<float> d_rds_car;      // n_streams x cap
    DevBuf<float> d_rds_pll;      // n_streams x 8
    // staging for the host-buffer entry points
    DevBuf<uint8_t> d_in;
    DevBuf<int16_t> d_out;
    PinnedBuf<uint8_t> h_in, h_out;  // the small host calls' staging (kPinnedCallBytes)
    DevBuf<float> d_f32;
    DevBuf<float> d_scratch;
    DevBuf<double> d_pll_side;    // PLL side data of one segment (pll_side_doubles)
    DevBuf<double> d_pll_side2;   // the pipelined engine's second one (odd chunks: their NCO runs
                                  //   on the audio stream while the next chunk's PLL fills the first)
    DevBuf<int16_t> d_sintab;
    DevBuf<uint8_t> d_synth_params;  // fmrx_synth_device_streams: SynthParams per stream
    // kernel timing: pairs of HIP events recorded around each fused-kernel launch on the
    // context stream (no host sync inside the timed loop); read by fmrx_kernel_timing
    std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
    size_t ev_used = 0;
    bool timing = false;
    unsigned long long* stamps = nullptr;  // fmrx_debug_mono_stamps (diagnostic)
    unsigned long long* pll_stats = nullptr;  // fmrx_debug_pll_stats (diagnostic)
    unsigned* pll_redos = nullptr;            // fmrx_debug_pll_redos (diagnostic)
    StageTimer stage_timer;                   // fmrx_debug_stage_timing (diagnostic)
    // the pipelined stereo engine (run_stereo_pipelined): front-end / band-pass stream, audio
    // stream and their events, created at the first pipelined call
    hipStream_t s_front = nullptr, s_audio = nullptr;
    std::vector<hipEvent_t> pipe_ev;
    int n_simd = 1024;                        // SIMDs of cfg.device (4 per CU), set at creation
    // switches (fmrx_debug_set_knob): the tuning ones from the environment once, at creation;
    // none of them changes the output (the PLL test hooks make the runners redo work)
    struct Knobs {
        PllKnobs pll;
        int stereo_chunks = 0;  // 0: by stream count and call length; k: k chunks (1: serial engine)
        int stereo_head = 8;    // the first chunk's blocks in 16ths of a middle chunk's
        int stereo_tail = 8;    // the last chunk's blocks in 16ths of a middle chunk's
        int stereo_lead = 0;    // n > 0: chunk k's front end waits for chunk k - n's PLL; 0: none
        int audio_defer = 2;    // 2: chunks 0 .. K-2's audio beside the last PLL; 1: all after it; 0: beside the next
                                // (2 + e: chunks 0 .. e-1 beside the PLL before the last)
        int mono_split = -1;    // -1: kOlderShare; 0: equal spans; n: the older wave's n / 1024
        int bpf_tile = 1;       // 0: the per-output band-pass kernel
        int halo_kernel = 0;    // 1: the separate halo_kernel after the fused one
    } knobs;
    // bounds on the streams' trigOffset (PllHint) of the stereo and the RDS PLL: 0 after a reset,
    // advanced by every call's samples (the float increments stick at 2^24), re-read from the
    // blob by fmrx_set_state; unknown after a failed launch
    struct TrigTrack {
        bool known = true;
        double lo = 0.0, hi = 0.0;
        void advance(size_t n) {
            lo = std::min(lo + (double)n, 16777216.0);
            hi = std::min(hi + (double)n, 16777216.0);
        }
    } pll_trig, rds_trig;
    PllHint hint(const TrigTrack& t) const {
        PllHint h;
        h.n_simd = n_simd;
        h.knobs = knobs.pll;
        h.redos = pll_redos;
        h.known = t.known;
        h.trig_lo = t.lo;
        h.trig_hi = t.hi;
        h.timer = stage_timer.on ? const_cast<StageTimer*>(&stage_timer) : nullptr;
        return h;
    }
};

namespace {

constexpr int kAudioHist50 = 50;
// stereo calls of up to this many blocks a stream take launch_stereo_audio_small (modes 0/1)
constexpr int kSmallAudioBlocks = 4;  // demod samples a resampler output reads before its base

// Serialises the entry points of one context (rf and audio stages may be driven from two
// threads, as project.cpp does; they share the context's stream and scratch buffers).
class CtxLock {
  public:
    explicit CtxLock(const fmrx_ctx* c) : c_(c) {
        if (c_) c_->mu.lock();
    }
    ~CtxLock() {
        if (c_) c_->mu.unlock();
    }
    CtxLock(const CtxLock&) = delete;
    CtxLock& operator=(const CtxLock&) = delete;

  private:
    const fmrx_ctx* c_;
};

bool fused_rf_supported(const fmrx_ctx* c) {
    const int t = c->geo.rf_taps, d = c->geo.rf_decim;
    return (t == 51 || t == 101) && (d == 10 || d == 4 || d == 9);
}

int set_device(const fmrx_ctx* c) {
    HIPCHK(hipSetDevice(c->cfg.device));
    return 0;
}

int reset_state(fmrx_ctx* c) {
    const int ns = c->cfg.n_streams;
    c->pll_trig = fmrx_ctx::TrigTrack{};
    c->rds_trig = fmrx_ctx::TrigTrack{};
    HIPCHK(hipMemsetAsync(c->d_halo[0].p, 0x80, c->halo_bytes * ns, c->stream));
    HIPCHK(hipMemsetAsync(c->d_halo[1].p, 0x80, c->halo_bytes * ns, c->stream));
    c->halo_cur = 0;
    HIPCHK(hipMemsetAsync(c->d_audio_hist.p, 0, sizeof(float) * c->audio_hist * ns, c->stream));
    c->audio_hist_stale = false;
    if (c->d_demod.p)  // the history in front of each stream (every call overwrites the rest)
        HIPCHK(hipMemset2DAsync(c->d_demod.p, c->demod_stride * sizeof(float), 0, sizeof(float) * kDemodHist, ns,
                                c->stream));
    // project.cpp:106-111: integrator 0, phaseEst 0, feedbackI 1, feedbackQ 0,
    // ncoOut_state 1, trigOffset 0
    std::vector<float> pll(8 * ns, 0.0f);
    for (int s = 0; s < ns; s++) {
        pll[8 * s + 2] = 1.0f;
        pll[8 * s + 4] = 1.0f;
    }
    HIPCHK(hipMemcpyAsync(c->d_pll.p, pll.data(), sizeof(float) * pll.size(),
                          hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->d_mix_tail.p, 0, sizeof(float) * kMixTail * ns, c->stream));
    HIPCHK(hipMemsetAsync(c->d_mono_state.p, 0, sizeof(float) * 8 * ns, c->stream));
    // RDS (project.cpp:206-226): zero histories, the same PLL start as the pilot PLL
    HIPCHK(hipMemsetAsync(c->d_rds_dhist.p, 0, sizeof(float) * kRdsDemodHist * ns, c->stream));
    if (c->d_rds_chan.p) HIPCHK(hipMemsetAsync(c->d_rds_chan.p, 0, sizeof(float) * c->d_rds_chan.n, c->stream));
    HIPCHK(hipMemcpyAsync(c->d_rds_pll.p, pll.data(), sizeof(float) * pll.size(), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

// RDS front half over n_if new demod samples per stream (d_demod: ns x n_if, stride
// demod_stride).  Optional copies of the NCO and the channel (ns x n_if each).
int run_rds(fmrx_ctx* c, const float* d_demod, size_t demod_stride, size_t n_if, float* d_out,
            float* d_nco, float* d_channel) {
    const int ns = c->cfg.n_streams;
    if (kRdsChanHist + n_if > c->rds_chan_stride) {
        const size_t stride = kRdsChanHist + n_if;
        DevBuf<float> nb;
        int rc = nb.ensure(stride * ns);
        if (rc) return rc;
        HIPCHK(hipMemsetAsync(nb.p, 0, sizeof(float) * nb.n, c->stream));
        if (c->d_rds_chan.p) {
            HIPCHK(hipMemcpy2DAsync(nb.p, stride * sizeof(float), c->d_rds_chan.p,
                                    c->rds_chan_stride * sizeof(float), kRdsChanHist * sizeof(float), ns,
                                    hipMemcpyDeviceToDevice, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            c->d_rds_chan.release();
        }
        c->d_rds_chan = nb;
        c->rds_chan_stride = stride;
    }
    int rc = c->d_rds_car.ensure(n_if * ns);
    if (!rc) rc = c->d_pll_side.ensure(pll_side_doubles((int)n_if, ns));
    if (rc) return rc;
    RdsLaunch L{};
    L.demod = d_demod;
    L.demod_stride = demod_stride;
    L.dhist = c->d_rds_dhist.p;
    L.chan = c->d_rds_chan.p;
    L.chan_stride = c->rds_chan_stride;
    L.carrier = c->d_rds_car.p;
    L.car_stride = n_if;
    L.out = d_out;
    L.out_stride = n_if;
    L.pll = c->d_rds_pll.p;
    L.pll_side = c->d_pll_side.p;
    L.ex = c->d_rds_taps.p;
    L.ca = c->d_rds_taps.p + kRdsTaps;
    L.bp_fs = (float)c->geo.bp_fs;
    L.n_if = (int)n_if;
    L.hint = c->hint(c->rds_trig);
    L.hint.redos = nullptr;  // fmrx_debug_pll_redos counts the stereo PLL's streams only
    if (launch_rds(L, ns, c->stream)) {
        c->rds_trig.known = false;
        return fail(FMRX_EHIP, "RDS launch failed");
    }
    c->rds_trig.advance(n_if);
    if (d_nco)
        HIPCHK(hipMemcpyAsync(d_nco, c->d_rds_car.p, sizeof(float) * n_if * ns, hipMemcpyDeviceToDevice,
                              c->stream));
    if (d_channel)
        HIPCHK(hipMemcpy2DAsync(d_channel, n_if * sizeof(float), c->d_rds_chan.p + kRdsChanHist,
                                c->rds_chan_stride * sizeof(float), n_if * sizeof(float), ns,
                                hipMemcpyDeviceToDevice, c->stream));
    return 0;
}

// Segments per stream for the fused kernel: enough workgroups to fill the chip
// (2 resident per CU on 256 CUs) without making segments so short that the pre-roll chunk
// dominates.
int mono_segments(const fmrx_ctx* c, long long n_if, int wg_per_cu = 0) {
    const long long chunks = mono_chunks(n_if, c->geo.rf_taps, c->geo.rf_decim, c->geo.audio_down);
    // one full wave of workgroups (or wg_per_cu a CU: the pipelined stereo front end, which
    // leaves the rest of each CU's LDS and SIMDs to the PLL runners beside it)
    const long long target_wg = 256LL * (wg_per_cu > 0 ? wg_per_cu : mono_wg_per_cu(c->geo.rf_decim));
    long long segs = std::max<long long>(1, target_wg / std::max(1, c->cfg.n_streams));
    // a call too short to fill the grid even at one chunk a segment (the per-block seam: 4-5
    // chunks a stream) takes one chunk a segment: twice the chunks, but all of them at once
    if ((long long)c->cfg.n_streams * chunks <= target_wg) return (int)std::max<long long>(1, chunks);
    segs = std::min(segs, std::max<long long>(1, chunks / 4));
    return (int)std::max<long long>(1, segs);
}

// Unequal shares for the two waves of a SIMD (mono_fused.hip mono_share): when the grid is
// two resident waves per SIMD (segs even, >= 15/16 of 2 x the SIMD count, 8 workgroups per
// CU), the first-dispatched wave takes kOlderShare/1024 of each span.  Knob mono_split = n
// (FMRX_MONO_SPLIT at creation) overrides it (0 = equal segments; timing sweeps).  660 since round 3's latency cuts (sweeps of
// 580-700 on two boxes, profiles/r03/split_sweep*/: 660 fastest on both, 1.2-1.6 % ahead of 620).
constexpr int kOlderShare = 660;
int mono_older_share(const fmrx_ctx* c, int segs) {
    const int n_simd = c->n_simd;
    const int share = c->knobs.mono_split < 0 ? kOlderShare : c->knobs.mono_split;
    if (share <= 0 || share >= 1024) return 0;
    const long long wgs = (long long)segs * c->cfg.n_streams;
    if ((segs & 1) != 0 || mono_wg_per_cu(c->geo.rf_decim) != 8 || wgs * 16 < 2LL * n_simd * 15 || wgs > 2LL * n_simd)
        return 0;
    return share;
}

// Workgroups a CU of the pipelined stereo front end past the first chunk (two of the fused
// kernel's 18.8 KB and one wave each): a full grid (8 a CU) holds every CU's LDS for its whole
// span, and a PLL launch queued behind it on the context stream waits until it drains.  The first
// chunk's front end runs alone (full grid).
constexpr int kPipeFrontWgPerCu = 2;

// RF front end (+ the mono audio stage when `pcm` is non-null and the mode allows it).
// Chunk form (the stereo pipeline, run_stereo_pipelined): blocks [b0, b0 + n_blocks) of a call of
// call_blocks blocks a stream starting at d_iq, on stream `st`; the halo of a chunk past the first
// is the call's own bytes in front of it, and only the last chunk (`last`) moves the context's halo.
int run_fused(fmrx_ctx* c, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm, float* d_mono,
              float* d_demod, size_t demod_stride, int demod_hist, bool with_audio, size_t b0 = 0,
              size_t call_blocks = 0, hipStream_t st = nullptr, bool last = true) {
    const int ns = c->cfg.n_streams;
    const size_t bb = c->geo.block_bytes;
    if (call_blocks == 0) call_blocks = n_blocks;
    if (!st) st = c->stream;
    MonoLaunch L{};
    L.iq = d_iq + b0 * bb;
    L.iq_stride = call_blocks * bb;
    L.halo = b0 == 0 ? c->d_halo[c->halo_cur].p : d_iq + b0 * bb - c->halo_bytes;
    L.halo_stride = b0 == 0 ? c->halo_bytes : L.iq_stride;
    L.pcm = d_pcm;
    L.mono = d_mono;
    L.demod = d_demod ? d_demod + b0 * c->geo.if_samples : nullptr;
    L.demod_stride = demod_stride;
    L.demod_hist = demod_hist;
    // When this call produces the mono audio itself, the mono product's audio history stays in
    // step with the stream, so a later fmrx_audio_block continues from it: its last 50 samples
    // are all a resampler output reads back (51 taps per phase in every mode).  The RF-only
    // calls (fmrx_rf_block, the stereo engine) leave it alone: the audio stage they feed owns it.
    L.demod_tail = with_audio ? c->d_audio_hist.p + (c->audio_hist - kAudioHist50) : nullptr;
    L.demod_tail_stride = (size_t)c->audio_hist;
    L.audio_coeff = c->d_audio.p;
    L.audio_rows = c->d_audio_rows.p;
    L.stream_bytes = n_blocks * c->geo.block_bytes;
    L.halo_bytes = c->halo_bytes;
    L.n_if = (long long)(n_blocks * c->geo.if_samples);
    L.segs = mono_segments(c, L.n_if, b0 > 0 ? kPipeFrontWgPerCu : 0);
    L.older_share = mono_older_share(c, L.segs);
    L.stamps = c->stamps;
    L.audio = with_audio ? 1 : 0;
    // the halo update rides in the fused kernel when every stream row is 16-B aligned (halo
    // bytes and block bytes are multiples of 16); otherwise halo_kernel runs after it
    const bool fused_halo = (reinterpret_cast<uintptr_t>(L.iq) & 15) == 0 && L.stream_bytes % 16 == 0 &&
                            L.iq_stride % 16 == 0 && c->halo_bytes % 16 == 0 &&
                            c->knobs.halo_kernel != 1;  // knob halo_kernel = 1: the separate kernel (A/B)
    L.halo_next = (last && fused_halo) ? c->d_halo[c->halo_cur ^ 1].p : nullptr;
    const int ad = c->geo.audio_up == 1 ? c->geo.audio_down : 5;
    std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
    if (c->timing) {
        if (c->ev_used == c->evs.size()) {
            std::pair<hipEvent_t, hipEvent_t> e{nullptr, nullptr};
            HIPCHK(hipEventCreate(&e.first));
            HIPCHK(hipEventCreate(&e.second));
            c->evs.push_back(e);
        }
        ev = &c->evs[c->ev_used++];
        HIPCHK(hipEventRecord(ev->first, st));
    }
    const int st_t = (!with_audio && d_demod) ? c->stage_timer.begin(st) : -1;
    int rc = launch_mono_fused(L, ns, c->geo.rf_taps, c->geo.rf_decim, c->geo.audio_up,
                               c->geo.audio_up == 1 ? ad : c->geo.audio_down, c->mono_taps, st);
    c->stage_timer.end(st_t, kStFront, 0.0, st);
    if (rc != 0) return fail(rc == -1 ? FMRX_EINVAL : FMRX_EHIP, "fused kernel launch failed (%d)", rc);
    if (ev) HIPCHK(hipEventRecord(ev->second, st));
    if (with_audio) c->audio_hist_stale = false;  // demod_tail rewrote the audio history
    if (!last) return 0;
    if (!L.halo_next) {  // the whole call's tail (every chunk's bytes are in d_iq)
        rc = launch_halo_update(d_iq, call_blocks * bb, c->d_halo[c->halo_cur].p, c->d_halo[c->halo_cur ^ 1].p,
                                c->halo_bytes, ns, st);
        if (rc != 0) return fail(FMRX_EHIP, "halo update failed");
    }
    c->halo_cur ^= 1;
    return 0;
}

// Mono product audio stage on a demod buffer (generic polyphase path: modes 2/3 and the
// split API).  demod: ns x n_if contiguous.  Advances d_audio_hist.
int run_mono_audio(fmrx_ctx* c, const float* d_demod, size_t demod_stride, size_t n_if,
                   int16_t* d_pcm, float* d_mono) {
    const int ns = c->cfg.n_streams;
    const int at = c->geo.audio_taps_total;
    const size_t na = n_if * c->geo.audio_up / c->geo.audio_down;
    // every stream in one launch: the resampler (+ the quantiser) over (output, stream), then
    // the history move of every stream (after all reads of the old history)
    PolyStreams P{};
    P.in = d_demod;
    P.in_stride = demod_stride;
    P.state = c->d_audio_hist.p;
    P.state_stride = c->audio_hist;
    P.coeff = c->d_audio.p;
    P.taps = at;
    P.up = c->geo.audio_up;
    P.down = c->geo.audio_down;
    P.n_out = (int)na;
    P.out = d_mono;
    P.out_stride = na;
    P.pcm = d_pcm;
    P.pcm_stride = na;
    int rc = launch_polyphase(P, ns, c->stream);
    if (rc == 0 && n_if >= (size_t)(at - 1))
        rc = launch_copy_streams(c->d_audio_hist.p, c->audio_hist, d_demod + (n_if - (at - 1)), demod_stride,
                                 at - 1, ns, c->stream);
    if (rc) return fail(FMRX_EHIP, "mono audio stage launch failed");
    return 0;
}

// Stereo engine on c->d_demod (history in front, n_if new samples per stream).
// src (may be null): the call's new demod, n_if a stream contiguous, not yet in c->d_demod --
// the band-pass kernel reads it from there (pinned host memory: no copy launch) and stores it.
int run_stereo_audio(fmrx_ctx* c, size_t n_blocks, int16_t* d_pcm, float* d_mono, const float* src = nullptr) {
    const int ns = c->cfg.n_streams;
    const size_t n_if = n_blocks * c->geo.if_samples;
    int rc = c->d_channel.ensure(n_if * ns);
    if (!rc) rc = c->d_carrier.ensure(n_if * ns);
    if (rc) return rc;
    StereoLaunch S{};
    S.demod = c->d_demod.p;
    S.channel = c->d_channel.p;
    S.carrier = c->d_carrier.p;
    S.n_if = (int)n_if;
    S.out_stride = n_if;
    S.hist = kDemodHist;
    S.demod_stride = c->demod_stride;
    S.ch_c = c->ch.data();
    S.ca_c = c->ca.data();
    S.bp_taps = c->geo.bp_taps;
    S.src = src;
    const int t_bp = c->stage_timer.begin(c->stream);
    if (launch_bpf_pair(S, ns, c->stream, c->knobs.bpf_tile != 0)) return fail(FMRX_EHIP, "band-pass launch failed");
    c->stage_timer.end(t_bp, kStBpf, 0.0, c->stream);
    // project.cpp:166: PLL(carrier, 19000, if_fs, 2, 0, 0.01, ...)
    if ((rc = c->d_pll_side.ensure(pll_side_doubles((int)n_if, ns)))) return rc;
    // a call of a few blocks (the per-block seam): the NCO, audio, state carry and demod history in
    // one launch after the PLL (launch_stereo_audio_small); longer calls: the parallel kernels
    const bool small = c->geo.audio_up == 1 && n_blocks <= (size_t)kSmallAudioBlocks;
    if (launch_pll(c->d_carrier.p, (int)n_if, ns, n_if, 19000.0f, (float)c->geo.if_fs, 2.0f, 0.0f,
                   0.01f, c->d_pll.p, c->d_pll_side.p, c->stream, c->hint(c->pll_trig), c->pll_stats, !small)) {
        c->pll_trig.known = false;
        return fail(FMRX_EHIP, "PLL launch failed");
    }
    c->pll_trig.advance(n_if);
    AudioLaunch A{};
    A.demod = c->d_demod.p;
    A.demod_stride = c->demod_stride;
    A.hist = kDemodHist;
    A.channel = c->d_channel.p;
    A.nco = c->d_carrier.p;
    A.mix_tail = c->d_mix_tail.p;
    A.mono_state = c->d_mono_state.p;
    A.pcm = d_pcm;
    A.mono_out = d_mono;
    A.n_blocks = (int)n_blocks;
    A.if_per_block = (int)c->geo.if_samples;
    A.frames_per_block = (int)c->geo.audio_frames;
    A.up = c->geo.audio_up;
    A.down = c->geo.audio_down;
    A.at = c->geo.audio_taps_total;
    A.audio_c = c->d_audio.p;
    const int t_au = c->stage_timer.begin(c->stream);
    if (small) {
        if (launch_stereo_audio_small(A, ns, pll_trig_args(c->d_pll_side.p, (int)n_if, ns), n_if, 2.0f, 0.0f,
                                      c->d_pll.p, kDemodHist, c->stream))
            return fail(FMRX_EHIP, "stereo audio launch failed");
        c->stage_timer.end(t_au, kStAudio, 0.0, c->stream);
        return 0;
    }
    if (launch_stereo_audio(A, ns, c->stream)) return fail(FMRX_EHIP, "stereo audio launch failed");
    c->stage_timer.end(t_au, kStAudio, 0.0, c->stream);
    // demod history for the next call: last kDemodHist samples -> front, every stream in one
    // launch (n_if >= one block of IF samples > kDemodHist: the ranges never overlap)
    if (launch_copy_streams(c->d_demod.p, c->demod_stride, c->d_demod.p + n_if, c->demod_stride, kDemodHist, ns,
                            c->stream))
        return fail(FMRX_EHIP, "demod history copy failed");
    return 0;
}

// First block of chunk k of K (k = K: n_blocks).  The first chunk is head / 16 of the others and
// the last tail / 16 (knobs stereo_head, stereo_tail; default 8: half): the first chunk's front
// end and the last chunk's NCO and audio stage have no PLL beside them.
size_t chunk_begin(size_t n_blocks, int k, int K, int head = 8, int tail = 8) {
    if (K <= 1 || k <= 0) return k <= 0 ? 0 : n_blocks;
    if (k >= K) return n_blocks;
    const unsigned long long h = (unsigned long long)std::max(1, std::min(head, 64));
    const unsigned long long tl = (unsigned long long)std::max(1, std::min(tail, 64));
    return (size_t)(((unsigned long long)n_blocks * (h + 16ULL * (unsigned long long)(k - 1))) /
                    (h + 16ULL * (unsigned long long)(K - 2) + tl));
}

// Chunks of the stereo pipeline for a call of n_blocks blocks a stream: the stage work beside
// the serial PLL (front end, band-pass pair, NCO, audio) grows with the streams, the PLL's with
// the samples a stream, so a call pipelines from 16 streams on when a chunk holds enough blocks.
// Knob stereo_chunks = k (FMRX_STEREO_CHUNKS at creation) forces k chunks (1: the serial engine).
int stereo_chunks(const fmrx_ctx* c, size_t n_blocks) {
    int k = c->cfg.n_streams >= 16 ? 8 : 1;  // 32 streams x 60 s: 0.423 vs 0.430 s (profiles/r04/g9)
    if (c->knobs.stereo_chunks > 0) k = c->knobs.stereo_chunks;
    else
        while (k > 1 && n_blocks * c->geo.if_samples / (size_t)k < 16384) k--;  // >= 2^14 samples a chunk
    // a chunk past the first reads its RF halo from the call's own bytes in front of it: every
    // chunk holds at least the halo's blocks
    const size_t hb = (c->halo_bytes + c->geo.block_bytes - 1) / c->geo.block_bytes;
    auto short_chunk = [&](int kk) {  // a chunk of the partition shorter than the halo
        for (int j = 0; j < kk; j++)
            if (chunk_begin(n_blocks, j + 1, kk, c->knobs.stereo_head, c->knobs.stereo_tail) -
                    chunk_begin(n_blocks, j, kk, c->knobs.stereo_head, c->knobs.stereo_tail) < hb)
                return true;
        return false;
    };
    while (k > 1 && short_chunk(k)) k--;  // the short first and last chunks too
    return k;
}


// The stereo engine over the call's blocks in K chunks, pipelined like project.cpp's two threads
// and their queue (rf_thread / audio_thread, project.cpp:17,71-80,133-141): the context stream
// runs the serial PLL of chunk k (launch_pll over its samples, the state carried in d_pll),
// s_front the front end and band-pass pair of chunk k + 1 ahead of it, s_audio the audio stage of
// chunk k - 1 behind it.  Every chunk reads the call's buffers (demod with its history, channel,
// carrier/NCO) at its offset, so each stage sees exactly the serial engine's inputs: the same
// bits.  Events order chunk k's PLL after its band-pass and its audio after its PLL; the call
// ends with the context stream waiting for the audio stream.
int run_stereo_pipelined_body(fmrx_ctx* c, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm, float* d_mono,
                              int K);
int run_stereo_pipelined(fmrx_ctx* c, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm, float* d_mono, int K) {
    const int rc = run_stereo_pipelined_body(c, d_iq, n_blocks, d_pcm, d_mono, K);
    if (rc != 0 && c->s_front) {
        // a launch failed part-way: the context stream still waits for whatever the side streams
        // hold, so a later call (or fmrx_synchronize) never races them
        c->pll_trig.known = false;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (hipEventCreateWithFlags(&e0, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&e1, hipEventDisableTiming) == hipSuccess) {
            (void)hipEventRecord(e0, c->s_front);
            (void)hipEventRecord(e1, c->s_audio);
            (void)hipStreamWaitEvent(c->stream, e0, 0);
            (void)hipStreamWaitEvent(c->stream, e1, 0);
            (void)hipStreamSynchronize(c->stream);
        }
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
    }
    return rc;
}

int run_stereo_pipelined_body(fmrx_ctx* c, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm, float* d_mono,
                              int K) {
    // first block of chunk j of K
    auto cb = [&](int j) { return chunk_begin(n_blocks, j, K, c->knobs.stereo_head, c->knobs.stereo_tail); };
    const int ns = c->cfg.n_streams;
    const size_t ipb = c->geo.if_samples, n_if = n_blocks * ipb;
    for (int k = 0; k < K; k++)
        if ((cb(k + 1) - cb(k)) * c->geo.block_bytes < c->halo_bytes)
            return fail(FMRX_EINVAL, "chunks shorter than the halo");
    int rc = c->d_channel.ensure(n_if * ns);
    if (!rc) rc = c->d_carrier.ensure(n_if * ns);
    if (rc) return rc;
    if (!c->s_front) {  // the lowest priority: the PLL's launches go first when a CU frees up
        int lo = 0, hi = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPCHK(hipStreamCreateWithPriority(&c->s_front, hipStreamNonBlocking, lo));
        HIPCHK(hipStreamCreateWithPriority(&c->s_audio, hipStreamNonBlocking, lo));
    }
    const size_t n_ev = 3 * (size_t)K + 3;
    while (c->pipe_ev.size() < n_ev) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        c->pipe_ev.push_back(e);
    }
    hipEvent_t ev_start = c->pipe_ev[0], ev_end = c->pipe_ev[1], ev_lane = c->pipe_ev[2 * (size_t)K + 2];
    auto ev_bp = [&](int k) { return c->pipe_ev[2 + 2 * (size_t)k]; };
    auto ev_pll = [&](int k) { return c->pipe_ev[3 + 2 * (size_t)k]; };
    auto ev_nco = [&](int k) { return c->pipe_ev[2 * (size_t)K + 3 + (size_t)k]; };
    // both side streams start after everything enqueued on the context stream so far
    HIPCHK(hipEventRecord(ev_start, c->stream));
    HIPCHK(hipStreamWaitEvent(c->s_front, ev_start, 0));
    HIPCHK(hipStreamWaitEvent(c->s_audio, ev_start, 0));
    size_t max_m = 0;
    for (int k = 0; k < K; k++)
        max_m = std::max(max_m, (cb(k + 1) - cb(k)) * ipb);
    if ((rc = c->d_pll_side.ensure(pll_side_doubles((int)max_m, ns)))) return rc;
    if ((rc = c->d_pll_side2.ensure(pll_side_doubles((int)max_m, ns)))) return rc;
    AudioLaunch A{};
    A.demod = c->d_demod.p;
    A.demod_stride = c->demod_stride;
    A.hist = kDemodHist;
    A.channel = c->d_channel.p;
    A.nco = c->d_carrier.p;
    A.mix_tail = c->d_mix_tail.p;
    A.mono_state = c->d_mono_state.p;
    A.pcm = d_pcm;
    A.mono_out = d_mono;
    A.n_blocks = (int)n_blocks;
    A.if_per_block = (int)ipb;
    A.frames_per_block = (int)c->geo.audio_frames;
    A.up = c->geo.audio_up;
    A.down = c->geo.audio_down;
    A.at = c->geo.audio_taps_total;
    A.audio_c = c->d_audio.p;
    // the PLL of chunk 0 in two launches when its streams start below 2^18: the lane runner's
    // segments and the index runner's [2^17, 2^18) form first (issue-bound: a front-end wave
    // sharing a chain's SIMD halves its rate), then the rest; chunk 1's front end waits for the
    // first part
    size_t lane_m = 0;
    if (c->pll_trig.known && c->pll_trig.lo == c->pll_trig.hi && c->pll_trig.lo < (double)kPllIdxMin)
        lane_m = (size_t)((double)kPllIdxMin - c->pll_trig.lo);
    // a chunk's PLL leaves its NCO (filter.cpp:170, a parallel pass) to the audio stream, so the
    // context stream goes on to the next chunk's runners; chunk k's trigArgs stay in side buffer
    // k & 1 until that NCO has read them (the context stream waits for it before chunk k + 2)
    auto side_of = [&](int k) { return (k & 1) ? c->d_pll_side2.p : c->d_pll_side.p; };
    auto pll = [&](size_t off, size_t m, double* side, bool nco) -> int {
        if (m == 0) return 0;
        PllHint h = c->hint(c->pll_trig);
        h.demote_once = true;  // one demoted-kernel launch a chunk (beside the stage kernels)
        if (launch_pll(c->d_carrier.p + off, (int)m, ns, n_if, 19000.0f, (float)c->geo.if_fs, 2.0f, 0.0f, 0.01f,
                       c->d_pll.p, side, c->stream, h, c->pll_stats, nco)) {
            c->pll_trig.known = false;
            return fail(FMRX_EHIP, "PLL launch failed");
        }
        c->pll_trig.advance(m);
        return 0;
    };
    // the audio stage of chunk j (s_audio, after chunk j's NCO)
    auto audio = [&](int j) -> int {
        const int t_au = c->stage_timer.begin(c->s_audio);
        if (launch_stereo_audio_range(A, (int)cb(j), (int)cb(j + 1), j == K - 1, ns, c->s_audio))
            return fail(FMRX_EHIP, "stereo audio launch failed");
        c->stage_timer.end(t_au, kStAudio, 0.0, c->s_audio);
        return 0;
    };
    for (int k = 0; k < K; k++) {
        const size_t b0 = cb(k), b1 = cb(k + 1);
        const size_t nb = b1 - b0, m = nb * ipb, off = b0 * ipb;
        const bool last = k == K - 1;
        if (k == 1 && lane_m > 0) HIPCHK(hipStreamWaitEvent(c->s_front, ev_lane, 0));
        // paced: chunk k's front end runs beside chunk k - lead + 1's PLL, not all of them at the start
        const int lead = c->knobs.stereo_lead;
        if (lead > 0 && k >= lead) HIPCHK(hipStreamWaitEvent(c->s_front, ev_pll(k - lead), 0));
        // s_front: front end and band-pass pair of chunk k
        if ((rc = run_fused(c, d_iq, nb, nullptr, nullptr, c->d_demod.p, c->demod_stride, kDemodHist, false, b0,
                            n_blocks, c->s_front, last)))
            return rc;
        StereoLaunch S{};
        S.demod = c->d_demod.p + off;
        S.channel = c->d_channel.p + off;
        S.carrier = c->d_carrier.p + off;
        S.n_if = (int)m;
        S.out_stride = n_if;
        S.hist = kDemodHist;
        S.demod_stride = c->demod_stride;
        S.ch_c = c->ch.data();
        S.ca_c = c->ca.data();
        S.bp_taps = c->geo.bp_taps;
        const int t_bp = c->stage_timer.begin(c->s_front);
        if (launch_bpf_pair(S, ns, c->s_front, c->knobs.bpf_tile != 0)) return fail(FMRX_EHIP, "band-pass launch failed");
        c->stage_timer.end(t_bp, kStBpf, 0.0, c->s_front);
        HIPCHK(hipEventRecord(ev_bp(k), c->s_front));
        // the context stream: the PLL of chunk k (project.cpp:166)
        HIPCHK(hipStreamWaitEvent(c->stream, ev_bp(k), 0));
        if (k >= 2) HIPCHK(hipStreamWaitEvent(c->stream, ev_nco(k - 2), 0));  // side buffer k & 1 read
        const size_t m0 = k == 0 ? std::min(lane_m, m) : 0;
        if ((rc = pll(off, m0, side_of(k), true))) return rc;  // (the lane part: its NCO in place)
        if (k == 0 && lane_m > 0) HIPCHK(hipEventRecord(ev_lane, c->stream));
        if ((rc = pll(off + m0, m - m0, side_of(k), false))) return rc;
        HIPCHK(hipEventRecord(ev_pll(k), c->stream));
        // s_audio: the NCO and the audio stage of chunk k (and the state carry after the last)
        HIPCHK(hipStreamWaitEvent(c->s_audio, ev_pll(k), 0));
        const int t_nco = c->stage_timer.begin(c->s_audio);
        if (launch_pll_nco(c->d_carrier.p + off + m0, (int)(m - m0), ns, n_if, 2.0f, 0.0f, c->d_pll.p, side_of(k),
                           c->s_audio))
            return fail(FMRX_EHIP, "NCO launch failed");
        c->stage_timer.end(t_nco, kStNco, 0.0, c->s_audio);
        HIPCHK(hipEventRecord(ev_nco(k), c->s_audio));
        // audio_defer (tools/ubench_noise.hip: the audio stages' LDS tiles slow the PLL chains they
        // run beside): 0 each chunk's audio after its NCO, beside the next chunk's PLL; 1 every
        // chunk's after the last chunk's PLL (configs[4] 0.4168 -> 0.4113 s,
        // profiles/r05/ab_audio_defer/); 2, the default, chunks 0 .. K - 2 beside the LAST chunk's
        // PLL only and chunk K - 1's after it: a short tail, one chunk's chains disturbed
        // (0.4058 -> 0.3955 s, profiles/r05/ab_audio_defer2/); 2 + e, chunks 0 .. e - 1 of those
        // beside chunk K - 2's PLL instead (a shorter queue beside the last PLL).  Everything here is
        // on s_audio in issue order, so NCO(K - 1) and audio(K - 1) queue behind all deferred audio
        // stages (the intended tail); e is clamped to K - 2, so with K <= 3 the 2 + e forms are 2
        // (same bits either way: only the order on s_audio changes)
        const int ad = c->knobs.audio_defer;
        const int early = ad >= 2 ? std::min(ad - 2, K - 2) : 0;
        if (ad == 0 && (rc = audio(k))) return rc;
        if (ad >= 2 && early > 0 && k == K - 3)
            for (int j = 0; j < early; j++)
                if ((rc = audio(j))) return rc;
        if (ad >= 2 && k == K - 2)
            for (int j = early; j <= K - 2; j++)
                if ((rc = audio(j))) return rc;
        if (ad >= 2 && k == K - 1 && (rc = audio(k))) return rc;
    }
    if (c->knobs.audio_defer == 1)
        for (int j = 0; j < K; j++)
            if ((rc = audio(j))) return rc;
    // demod history for the next call (after every read of this call's demod: the last audio
    // launch follows every band-pass launch through the events)
    if (launch_copy_streams(c->d_demod.p, c->demod_stride, c->d_demod.p + n_if, c->demod_stride, kDemodHist, ns,
                            c->s_audio))
        return fail(FMRX_EHIP, "demod history copy failed");
    HIPCHK(hipEventRecord(ev_end, c->s_audio));
    HIPCHK(hipStreamWaitEvent(c->stream, ev_end, 0));
    return 0;
}

int ensure_demod(fmrx_ctx* c, size_t n_if) {
    const size_t stride = kDemodHist + n_if;
    if (stride <= c->demod_stride) return 0;
    // grow, preserving the history of every stream
    DevBuf<float> nb;
    int rc = nb.ensure(stride * c->cfg.n_streams);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(nb.p, 0, sizeof(float) * nb.n, c->stream));
    if (c->d_demod.p) {
        HIPCHK(hipMemcpy2DAsync(nb.p, stride * sizeof(float), c->d_demod.p,
                                c->demod_stride * sizeof(float), kDemodHist * sizeof(float),
                                c->cfg.n_streams, hipMemcpyDeviceToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        c->d_demod.release();
    }
    c->d_demod = nb;
    c->demod_stride = stride;
    return 0;
}

}  // namespace

extern "C" {

const char* fmrx_last_error(void) { return g_err.c_str(); }
const char* fmrx_version(void) { return "fmrx 0.1 (gfx950)"; }

int fmrx_config_default(fmrx_config* cfg, int mode, int channels) {
    if (!cfg) return fail(FMRX_EINVAL, "null config");
    ModeConstants m;
    if (!mode_constants(mode, &m)) return fail(FMRX_EINVAL, "invalid mode %d", mode);
    if (channels != FMRX_MONO && channels != FMRX_STEREO)
        return fail(FMRX_EINVAL, "invalid channels %d", channels);
    cfg->mode = mode;
    cfg->channels = channels;
    cfg->rf_taps = 51;     // src/project.cpp:306
    cfg->bp_taps = 51;     // src/project.cpp:307
    cfg->audio_taps = 51;  // src/project.cpp:319
    cfg->n_streams = 1;
    cfg->device = 0;
    return FMRX_OK;
}

int fmrx_geometry(const fmrx_config* cfg, fmrx_geometry_t* g) {
    if (!cfg || !g) return fail(FMRX_EINVAL, "null argument");
    ModeConstants m;
    if (!mode_constants(cfg->mode, &m)) return fail(FMRX_EINVAL, "invalid mode %d", cfg->mode);
    if (cfg->channels != FMRX_MONO && cfg->channels != FMRX_STEREO)
        return fail(FMRX_EINVAL, "invalid channels %d", cfg->channels);
    const int rf_taps = cfg->rf_taps ? cfg->rf_taps : 51;
    const int bp_taps = cfg->bp_taps ? cfg->bp_taps : 51;
    const int audio_taps = cfg->audio_taps ? cfg->audio_taps : 51;
    if (rf_taps < 3 || rf_taps > kMaxRfTaps) return fail(FMRX_EINVAL, "rf_taps %d out of range", rf_taps);
    if (bp_taps < 3 || bp_taps > 64) return fail(FMRX_EINVAL, "bp_taps %d out of range", bp_taps);
    // The fused audio stages (mono window, rational resampler rows, stereo LPFs' shared
    // 50-sample history) are compiled for the reference's 51 taps per phase (project.cpp:319).
    if (audio_taps != 51) return fail(FMRX_EINVAL, "audio_taps %d unsupported (51 per phase)", audio_taps);
    g->rf_fs = m.rf_fs;
    g->rf_decim = m.rf_decim;
    g->if_fs = m.if_fs;
    g->bp_fs = m.bp_fs;
    g->audio_up = m.audio_up;
    g->audio_down = m.audio_down;
    g->rf_taps = rf_taps;
    g->bp_taps = bp_taps;
    g->audio_taps_total = audio_taps * m.audio_up;  // project.cpp:347,356
    g->block_bytes = (size_t)256 * m.rf_decim * m.audio_down;  // project.cpp:364
    g->iq_pairs = g->block_bytes / 2;
    g->if_samples = g->iq_pairs / m.rf_decim;
    g->audio_frames = g->if_samples * m.audio_up / m.audio_down;
    g->pcm_samples = g->audio_frames * cfg->channels;
    if ((size_t)g->audio_taps_total - 1 > g->if_samples || (size_t)rf_taps - 1 > g->iq_pairs)
        return fail(FMRX_EINVAL, "filter longer than a block");
    return FMRX_OK;
}

// The tuning switches of a new context from the environment (A/B measurements: which runner or
// kernel form runs, never what it computes).  The PLL test hooks are not read here: only
// fmrx_debug_set_knob sets them, per context.
// Every knob's accepted range (include/fmrx.h): a value outside it is refused (FMRX_EINVAL from
// fmrx_debug_set_knob; fmrx_create refuses a bad environment variable), so no setting can reach
// an untested kernel form.  Integer knobs take integer values only.
struct KnobSpec {
    int id;
    const char* env;  // the tuning knobs' environment variable (null: test hooks, never from there)
    double lo, hi;
    bool integer;
};
constexpr KnobSpec kKnobs[] = {
    {FMRX_KNOB_PLL_SPEC, "FMRX_PLL_SPEC", 0, 1, true},
    {FMRX_KNOB_PLL_SAT, "FMRX_PLL_SAT", 0, 1, true},
    {FMRX_KNOB_PLL_PRED, "FMRX_PLL_PRED", 0, 2, true},
    {FMRX_KNOB_PLL_PIPE, "FMRX_PLL_PIPE", 0, 1, true},
    {FMRX_KNOB_PLL_IDX, "FMRX_PLL_IDX", 0, 2, true},
    {FMRX_KNOB_STEREO_CHUNKS, "FMRX_STEREO_CHUNKS", 0, 64, true},
    {FMRX_KNOB_MONO_SPLIT, "FMRX_MONO_SPLIT", -1, 1023, true},
    {FMRX_KNOB_BPF_TILE, "FMRX_BPF_TILE", 0, 1, true},
    {FMRX_KNOB_HALO_KERNEL, "FMRX_HALO_KERNEL", 0, 1, true},
    {FMRX_KNOB_PLL_INJECT, nullptr, -1, 1 << 30, true},
    {FMRX_KNOB_PLL_PIPE_MISS, nullptr, -(1 << 30), 1 << 30, true},
    {FMRX_KNOB_PLL_HINT_SKEW, nullptr, -16777216.0, 16777216.0, false},
    {FMRX_KNOB_PLL_CNT, "FMRX_PLL_CNT", 0, 31, true},
    {FMRX_KNOB_PLL_STICK, "FMRX_PLL_STICK", 0, 1, true},
    {FMRX_KNOB_STEREO_HEAD, "FMRX_STEREO_HEAD", 1, 64, true},
    {FMRX_KNOB_STEREO_LEAD, "FMRX_STEREO_LEAD", 0, 64, true},
    {FMRX_KNOB_AUDIO_DEFER, "FMRX_AUDIO_DEFER", 0, 64, true},
    {FMRX_KNOB_STEREO_TAIL, "FMRX_STEREO_TAIL", 1, 64, true},
};

const KnobSpec* knob_spec(int knob) {
    for (const KnobSpec& k : kKnobs)
        if (k.id == knob) return &k;
    return nullptr;
}

// value into the context's knobs (range already checked)
void knob_set(fmrx_ctx::Knobs& k, int knob, double value) {
    const int v = (int)value;
    switch (knob) {
        case FMRX_KNOB_PLL_SPEC: k.pll.spec = v; break;
        case FMRX_KNOB_PLL_SAT: k.pll.sat = v; break;
        case FMRX_KNOB_PLL_PRED: k.pll.pred = v; break;
        case FMRX_KNOB_PLL_PIPE: k.pll.pipe = v; break;
        case FMRX_KNOB_PLL_IDX: k.pll.idx = v; break;
        case FMRX_KNOB_STEREO_CHUNKS: k.stereo_chunks = v; break;
        case FMRX_KNOB_STEREO_HEAD: k.stereo_head = v; break;
        case FMRX_KNOB_STEREO_TAIL: k.stereo_tail = v; break;
        case FMRX_KNOB_STEREO_LEAD: k.stereo_lead = v; break;
        case FMRX_KNOB_AUDIO_DEFER: k.audio_defer = v; break;
        case FMRX_KNOB_MONO_SPLIT: k.mono_split = v; break;
        case FMRX_KNOB_BPF_TILE: k.bpf_tile = v; break;
        case FMRX_KNOB_HALO_KERNEL: k.halo_kernel = v; break;
        case FMRX_KNOB_PLL_INJECT: k.pll.inject = v; break;
        case FMRX_KNOB_PLL_PIPE_MISS: k.pll.pipe_miss = v; break;
        case FMRX_KNOB_PLL_HINT_SKEW: k.pll.skew = value; break;
        case FMRX_KNOB_PLL_CNT: k.pll.cnt = v; break;
        case FMRX_KNOB_PLL_STICK: k.pll.stick = v; break;
        default: break;
    }
}

bool knob_ok(const KnobSpec& s, double v) {
    return v == v && v >= s.lo && v <= s.hi && (!s.integer || v == std::floor(v));
}

// the tuning knobs from the environment, read once by fmrx_create; a set variable must be an
// integer in its knob's range (otherwise the context is refused, naming the variable)
int knobs_from_env(fmrx_ctx::Knobs* out) {
    fmrx_ctx::Knobs k;
    for (const KnobSpec& s : kKnobs) {
        if (!s.env) continue;
        const char* e = std::getenv(s.env);
        if (!e || !*e) continue;
        char* end = nullptr;
        const long v = std::strtol(e, &end, 10);
        if (*end != '\0' || !knob_ok(s, (double)v))
            return fail(FMRX_EINVAL, "%s=%s: not an integer in [%g, %g]", s.env, e, s.lo, s.hi);
        knob_set(k, s.id, (double)v);
    }
    *out = k;
    return FMRX_OK;
}

int fmrx_create(const fmrx_config* cfg, fmrx_ctx** out) {
    if (!out) return fail(FMRX_EINVAL, "null output pointer");
    *out = nullptr;
    fmrx_geometry_t g;
    int rc = fmrx_geometry(cfg, &g);
    if (rc) return rc;
    if (cfg->n_streams < 1) return fail(FMRX_EINVAL, "n_streams must be >= 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(FMRX_EHIP, "no HIP device available (libfmrx has no CPU path)");
    if (cfg->device < 0 || cfg->device >= ndev) return fail(FMRX_EINVAL, "bad device %d", cfg->device);
    // every per-stream launch puts the streams on grid.y (band-pass, PLL check / NCO / pre-pass,
    // halo update, the multi-stream audio and copy kernels): refuse what cannot launch here
    // rather than fail at the first call
    int max_y = 0;
    if (hipDeviceGetAttribute(&max_y, hipDeviceAttributeMaxGridDimY, cfg->device) == hipSuccess && max_y > 0 &&
        cfg->n_streams > max_y)
        return fail(FMRX_EINVAL, "n_streams %d exceeds the device's grid.y limit %d", cfg->n_streams, max_y);
    fmrx_ctx* c = new fmrx_ctx();
    c->cfg = *cfg;
    c->cfg.rf_taps = g.rf_taps;
    c->cfg.bp_taps = g.bp_taps;
    c->geo = g;
    mode_constants(cfg->mode, &c->mc);
    if (!fused_rf_supported(c)) {
        delete c;
        return fail(FMRX_EINVAL, "no compiled RF kernel for rf_taps=%d rf_decim=%d", g.rf_taps,
                    g.rf_decim);
    }
    if ((rc = set_device(c))) { delete c; return rc; }
    if ((rc = knobs_from_env(&c->knobs))) {
        delete c;
        return rc;
    }
    {
        int cus = 0;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cfg->device) == hipSuccess && cus > 0)
            c->n_simd = 4 * cus;
    }
    // taps, exactly as the reference designs them (project.cpp:37, 97, 104, 117)
    c->rf.resize(g.rf_taps);
    design_lpf(c->rf.data(), (float)g.rf_fs, (float)kRfFc, g.rf_taps, 1);
    c->audio.resize(g.audio_taps_total);
    design_lpf(c->audio.data(), (float)g.if_fs, (float)kAudioFc, g.audio_taps_total, g.audio_up);
    c->ch.resize(g.bp_taps);
    design_bpf(c->ch.data(), (float)g.bp_fs, 22000.0f, 54000.0f, g.bp_taps);
    c->ca.resize(g.bp_taps);
    design_bpf(c->ca.data(), (float)g.bp_fs, 18500.0f, 19500.0f, g.bp_taps);
    std::memset(&c->mono_taps, 0, sizeof c->mono_taps);
    std::copy(c->rf.begin(), c->rf.end(), c->mono_taps.rf);
    if (g.audio_up == 1) std::copy(c->audio.begin(), c->audio.end(), c->mono_taps.audio);

    const int ns = cfg->n_streams;
    auto cleanup = [&](int code) { fmrx_destroy(c); return code; };
    // the context stream at the highest priority (the serial PLL of the pipelined stereo engine
    // runs on it, its stage streams at the lowest)
    int prio_lo = 0, prio_hi = 0;
    if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess ||
        hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, prio_hi) != hipSuccess)
        return cleanup(fail(FMRX_EHIP, "hipStreamCreate failed"));
    c->halo_bytes = mono_halo_bytes(g.rf_taps, g.rf_decim, g.audio_down);
    c->audio_hist = g.audio_taps_total - 1;
    if ((rc = c->d_halo[0].ensure(c->halo_bytes * ns)) || (rc = c->d_halo[1].ensure(c->halo_bytes * ns)) ||
        (rc = c->d_audio_hist.ensure((size_t)c->audio_hist * ns)) ||
        (rc = c->d_audio.ensure(c->audio.size())) || (rc = c->d_rf.ensure(c->rf.size())) ||
        (rc = c->d_pll.ensure(8 * (size_t)ns)) || (rc = c->d_mix_tail.ensure((size_t)kMixTail * ns)) ||
        (rc = c->d_mono_state.ensure(8 * (size_t)ns)) || (rc = c->d_sintab.ensure(kSinSize)) ||
        (rc = c->d_rds_taps.ensure(2 * kRdsTaps)) || (rc = c->d_rds_dhist.ensure((size_t)kRdsDemodHist * ns)) ||
        (rc = c->d_rds_pll.ensure(8 * (size_t)ns)))
        return cleanup(rc);
    // RDS taps, project.cpp:211 and :217 (bp_taps = 51 at bp_fs)
    std::vector<float> rds_taps(2 * kRdsTaps);
    design_bpf(rds_taps.data(), (float)g.bp_fs, 54000.0f, 60000.0f, kRdsTaps);
    design_bpf(rds_taps.data() + kRdsTaps, (float)g.bp_fs, 113500.0f, 114500.0f, kRdsTaps);
    if (hipMemcpy(c->d_rds_taps.p, rds_taps.data(), sizeof(float) * rds_taps.size(), hipMemcpyHostToDevice) != hipSuccess)
        return cleanup(fail(FMRX_EHIP, "RDS tap upload failed"));
    if (hipMemcpy(c->d_audio.p, c->audio.data(), sizeof(float) * c->audio.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_rf.p, c->rf.data(), sizeof(float) * c->rf.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(c->d_sintab.p, synth_sintab(), sizeof(int16_t) * kSinSize, hipMemcpyHostToDevice) != hipSuccess)
        return cleanup(fail(FMRX_EHIP, "tap upload failed"));
    if (g.audio_up > 1) {
        // the rational resampler's prototype by phase: row k0 holds the 51 taps an output of
        // phase k0 reads, in the order filter.cpp:84 visits them (k = k0, k0 + up, ...)
        const int up = g.audio_up;
        std::vector<float> rows((size_t)up * kAudioRow, 0.0f);
        for (int k0 = 0; k0 < up; k0++)
            for (int i = 0; i < 51; i++) rows[(size_t)k0 * kAudioRow + i] = c->audio[(size_t)k0 + (size_t)i * up];
        if ((rc = c->d_audio_rows.ensure(rows.size()))) return cleanup(rc);
        if (hipMemcpy(c->d_audio_rows.p, rows.data(), sizeof(float) * rows.size(), hipMemcpyHostToDevice) != hipSuccess)
            return cleanup(fail(FMRX_EHIP, "tap upload failed"));
    }
    if ((rc = reset_state(c))) return cleanup(rc);
    *out = c;
    return FMRX_OK;
}

void fmrx_destroy(fmrx_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->cfg.device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->d_audio.release(); c->d_rf.release(); c->d_audio_rows.release(); c->d_halo[0].release(); c->d_halo[1].release();
    c->d_audio_hist.release(); c->d_demod.release(); c->d_channel.release(); c->d_carrier.release();
    c->d_pll.release(); c->d_mix_tail.release(); c->d_mono_state.release(); c->d_in.release();
    c->d_out.release(); c->d_f32.release(); c->d_scratch.release(); c->d_sintab.release();
    c->h_in.release(); c->h_out.release();
    c->d_pll_side.release(); c->d_pll_side2.release();
    c->d_rds_taps.release(); c->d_rds_dhist.release(); c->d_rds_chan.release(); c->d_rds_car.release();
    c->d_rds_pll.release();
    for (auto& e : c->evs) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    c->stage_timer.release();
    if (c->s_front) (void)hipStreamSynchronize(c->s_front);
    if (c->s_audio) (void)hipStreamSynchronize(c->s_audio);
    for (auto e : c->pipe_ev) (void)hipEventDestroy(e);
    if (c->s_front) (void)hipStreamDestroy(c->s_front);
    if (c->s_audio) (void)hipStreamDestroy(c->s_audio);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int fmrx_history_bytes(const fmrx_ctx* c, size_t* bytes) {
    CtxLock lock_(c);
    if (!c || !bytes) return fail(FMRX_EINVAL, "null argument");
    *bytes = c->halo_bytes;
    return FMRX_OK;
}

// The fused kernel rebuilds every float state of the mono product from the raw bytes in the
// halo by a pre-roll chunk (mono_fused.hip), so seeking is setting the halo: the last
// halo_bytes of prev, 0x80 (x = 0.0, the reference's zero-initialised state) in front of a
// shorter prev.
int fmrx_seek(fmrx_ctx* c, const uint8_t* prev, size_t n, int prev_on_device) {
    CtxLock lock_(c);
    if (!c || (!prev && n > 0)) return fail(FMRX_EINVAL, "bad argument");
    if (c->cfg.channels != FMRX_MONO) return fail(FMRX_ESTATE, "fmrx_seek: mono product only (the PLL is serial)");
    int rc = set_device(c);
    if (rc) return rc;
    const size_t ns = c->cfg.n_streams, hb = c->halo_bytes, m = std::min(n, hb);
    uint8_t* h = c->d_halo[c->halo_cur].p;
    if (m < hb) HIPCHK(hipMemset2DAsync(h, hb, 0x80, hb - m, ns, c->stream));
    if (m > 0)
        HIPCHK(hipMemcpy2DAsync(h + (hb - m), hb, prev + (n - m), n, m, ns,
                                prev_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
    if (!prev_on_device) HIPCHK(hipStreamSynchronize(c->stream));  // prev may be freed on return
    c->audio_hist_stale = true;
    return FMRX_OK;
}

int fmrx_reset(fmrx_ctx* c) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    int rc = set_device(c);
    return rc ? rc : reset_state(c);
}

// ---- state blob: header + halo bytes + audio history + stereo state ------------------
int fmrx_state_size(const fmrx_ctx* c, size_t* bytes) {
    CtxLock lock_(c);
    if (!c || !bytes) return fail(FMRX_EINVAL, "null argument");
    const size_t ns = c->cfg.n_streams;
    *bytes = kStateHdrWords * sizeof(uint32_t) + ns * (c->halo_bytes + sizeof(float) * (c->audio_hist + kDemodHist + 8 + kMixTail + 8));
    return FMRX_OK;
}

namespace {
struct BlobIO {
    uint8_t* p;
    bool put;
    int io(fmrx_ctx* c, void* dev, size_t n) {
        if (n == 0) return 0;
        if (put) HIPCHK(hipMemcpyAsync(dev, p, n, hipMemcpyHostToDevice, c->stream));
        else HIPCHK(hipMemcpyAsync(p, dev, n, hipMemcpyDeviceToHost, c->stream));
        p += n;
        return 0;
    }
};

int state_io(fmrx_ctx* c, uint8_t* buf, size_t bytes, bool put) {
    size_t need;
    fmrx_state_size(c, &need);
    if (bytes < need) return fail(FMRX_ESTATE, "state buffer too small (%zu < %zu)", bytes, need);
    int rc = set_device(c);
    if (rc) return rc;
    // words 0-7 identify the context shape and must match; word 8 carries the audio-history
    // staleness of a context taken between fmrx_seek and its next fused call (restored with
    // the blob, so fmrx_audio_block refuses the stale history there too)
    uint32_t hdr[kStateHdrWords] = {kStateMagic, kStateVersion, (uint32_t)c->cfg.mode, (uint32_t)c->cfg.channels,
                                    (uint32_t)c->geo.rf_taps, (uint32_t)c->cfg.n_streams, (uint32_t)c->halo_bytes,
                                    (uint32_t)c->audio_hist, c->audio_hist_stale ? 1u : 0u, 0u};
    if (put) {
        uint32_t got[kStateHdrWords];
        std::memcpy(got, buf, sizeof got);
        if (got[0] != kStateMagic) return fail(FMRX_ESTATE, "not an fmrx state blob (magic 0x%08x)", got[0]);
        if (got[1] != kStateVersion)
            return fail(FMRX_ESTATE, "state blob version %u, expected %u (INTEGRATION.md: blob versions)", got[1],
                        kStateVersion);
        if (std::memcmp(hdr + 2, got + 2, 6 * sizeof(uint32_t)) != 0)
            return fail(FMRX_ESTATE, "state blob is for another context shape (mode %u, channels %u, rf_taps %u, "
                        "%u streams)", got[2], got[3], got[4], got[5]);
        if (got[8] > 1u) return fail(FMRX_ESTATE, "state blob: unknown flags 0x%x", got[8]);
        if (got[9] != 0u) return fail(FMRX_ESTATE, "state blob: reserved word 9 is 0x%x, must be 0", got[9]);
    } else {
        std::memcpy(buf, hdr, sizeof hdr);
    }
    const size_t ns = c->cfg.n_streams;
    if (put && (rc = ensure_demod(c, 1))) return rc;
    if (!put && !c->d_demod.p && (rc = ensure_demod(c, 1))) return rc;
    BlobIO b{buf + sizeof hdr, put};
    if ((rc = b.io(c, c->d_halo[c->halo_cur].p, ns * c->halo_bytes))) return rc;
    if ((rc = b.io(c, c->d_audio_hist.p, ns * sizeof(float) * c->audio_hist))) return rc;
    // demod history: kDemodHist floats in front of each stream's row (one 2-D copy)
    {
        const size_t w = sizeof(float) * kDemodHist, pitch = sizeof(float) * c->demod_stride;
        if (put) HIPCHK(hipMemcpy2DAsync(c->d_demod.p, pitch, b.p, w, w, ns, hipMemcpyHostToDevice, c->stream));
        else HIPCHK(hipMemcpy2DAsync(b.p, w, c->d_demod.p, pitch, w, ns, hipMemcpyDeviceToHost, c->stream));
        b.p += w * ns;
    }
    if ((rc = b.io(c, c->d_pll.p, ns * sizeof(float) * 8))) return rc;
    // (slots 6-7 of each stream's PLL state are the runners' hand-off within a call, 0 between
    // calls: a blob's values there are not trusted)
    if (put)
        HIPCHK(hipMemset2DAsync(c->d_pll.p + 6, 8 * sizeof(float), 0, 2 * sizeof(float), ns, c->stream));
    if ((rc = b.io(c, c->d_mix_tail.p, ns * sizeof(float) * kMixTail))) return rc;
    if ((rc = b.io(c, c->d_mono_state.p, ns * sizeof(float) * 8))) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}
}  // namespace

int fmrx_get_state(fmrx_ctx* c, void* buf, size_t bytes) {
    CtxLock lock_(c);
    if (!c || !buf) return fail(FMRX_EINVAL, "null argument");
    return state_io(c, static_cast<uint8_t*>(buf), bytes, false);
}

int fmrx_set_state(fmrx_ctx* c, const void* buf, size_t bytes) {
    CtxLock lock_(c);
    if (!c || !buf) return fail(FMRX_EINVAL, "null argument");
    const uint8_t* p = static_cast<const uint8_t*>(buf);
    const int rc = state_io(c, const_cast<uint8_t*>(p), bytes, true);
    if (rc == 0) {
        uint32_t flags;
        std::memcpy(&flags, p + 8 * sizeof(uint32_t), sizeof flags);
        c->audio_hist_stale = (flags & 1u) != 0;
        // the streams' trigOffsets (state_io order: halo, audio history, demod history, PLL x 8)
        const size_t ns = c->cfg.n_streams;
        const uint8_t* pll = p + kStateHdrWords * sizeof(uint32_t) +
                             ns * (c->halo_bytes + sizeof(float) * (c->audio_hist + kDemodHist));
        fmrx_ctx::TrigTrack t;
        t.lo = 16777216.0;
        t.hi = 0.0;
        for (size_t s = 0; s < ns; s++) {
            float v;
            std::memcpy(&v, pll + (8 * s + 5) * sizeof(float), sizeof v);
            if (!(v >= 0.0f && v <= 16777216.0f && v == std::floor(v))) t.known = false;
            t.lo = std::min(t.lo, (double)v);
            t.hi = std::max(t.hi, (double)v);
        }
        if (!t.known) t.lo = t.hi = 0.0;
        c->pll_trig = t;
    }
    return rc;
}

// ---- fused device-resident path ----------------------------------------------------------
int fmrx_process_device_ex(fmrx_ctx* c, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm,
                           float* d_mono) {
    CtxLock lock_(c);
    if (!c || !d_iq || !d_pcm) return fail(FMRX_EINVAL, "null argument");
    if (n_blocks == 0) return FMRX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t n_if = n_blocks * c->geo.if_samples;
    if (c->cfg.channels == FMRX_MONO)  // every mode: RF + demod + audio resampler in one launch
        return run_fused(c, d_iq, n_blocks, d_pcm, d_mono, nullptr, 0, 0, true);
    if ((rc = ensure_demod(c, n_if))) return rc;
    const int K = stereo_chunks(c, n_blocks);
    if (K > 1) return run_stereo_pipelined(c, d_iq, n_blocks, d_pcm, d_mono, K);
    if ((rc = run_fused(c, d_iq, n_blocks, nullptr, nullptr, c->d_demod.p, c->demod_stride,
                        kDemodHist, false)))
        return rc;
    return run_stereo_audio(c, n_blocks, d_pcm, d_mono);
}

int fmrx_process_device(fmrx_ctx* c, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm) {
    return fmrx_process_device_ex(c, d_iq, n_blocks, d_pcm, nullptr);
}

int fmrx_synchronize(fmrx_ctx* c) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    const hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) {
        // an asynchronous fault of an enqueued launch: the device state no longer follows the
        // host's trigOffset bounds, so the runner choice falls back to "unknown" until a reset
        c->pll_trig.known = false;
        c->rds_trig.known = false;
        return fail(FMRX_EHIP, "stream synchronize failed: %s", hipGetErrorString(e));
    }
    return FMRX_OK;
}

void* fmrx_stream(fmrx_ctx* c) { return c ? (void*)c->stream : nullptr; }

int fmrx_kernel_timing(fmrx_ctx* c, int reset, double* avg_ms, long* launches) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    int rc = set_device(c);
    if (rc) return rc;
    double total = 0.0;
    if (c->ev_used) HIPCHK(hipEventSynchronize(c->evs[c->ev_used - 1].second));
    for (size_t i = 0; i < c->ev_used; i++) {
        float ms = 0.0f;
        HIPCHK(hipEventElapsedTime(&ms, c->evs[i].first, c->evs[i].second));
        total += ms;
    }
    if (avg_ms) *avg_ms = c->ev_used ? total / (double)c->ev_used : 0.0;
    if (launches) *launches = (long)c->ev_used;
    if (reset > 0) {  // reset > 0: clear and arm event timing of the fused kernel
        c->ev_used = 0;
        c->timing = true;
    } else if (reset < 0) {  // reset < 0: clear and disarm
        c->ev_used = 0;
        c->timing = false;
    }
    return FMRX_OK;
}

// ---- host-buffer entry points ---------------------------------------------------------------
// End of a small host call: poll the stream instead of hipStreamSynchronize, whose blocking wait
// wakes the thread ~10 us after the last kernel of a 20-80 us call (the per-block seam's
// calls); after kSpinNs the call is not small after all and blocks.
constexpr long long kSpinNs = 2000000;
int wait_small(fmrx_ctx* c) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0;; k++) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) return FMRX_OK;
        if (e != hipErrorNotReady) return fail(FMRX_EHIP, "stream query: %s", hipGetErrorString(e));
        if ((k & 63) == 63 && std::chrono::duration_cast<std::chrono::nanoseconds>(
                                  std::chrono::steady_clock::now() - t0).count() > kSpinNs)
            break;
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return FMRX_OK;
}

int fmrx_process(fmrx_ctx* c, const uint8_t* iq, size_t n_blocks, int16_t* pcm) {
    CtxLock lock_(c);
    if (!c || !iq || !pcm) return fail(FMRX_EINVAL, "null argument");
    if (n_blocks == 0) return FMRX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t ns = c->cfg.n_streams;
    const size_t in_bytes = ns * n_blocks * c->geo.block_bytes;
    const size_t out_n = ns * n_blocks * c->geo.pcm_samples;
    if (in_bytes <= kPinnedCallBytes) {  // pinned staging: the input by DMA, the PCM written in place
        if ((rc = c->h_in.ensure(in_bytes)) || (rc = c->h_out.ensure(out_n * sizeof(int16_t))) ||
            (rc = c->d_in.ensure(in_bytes)))
            return rc;
        std::memcpy(c->h_in.p, iq, in_bytes);
        HIPCHK(hipMemcpyAsync(c->d_in.p, c->h_in.p, in_bytes, hipMemcpyHostToDevice, c->stream));
        if ((rc = fmrx_process_device(c, c->d_in.p, n_blocks, reinterpret_cast<int16_t*>(c->h_out.p)))) return rc;
        if ((rc = wait_small(c))) return rc;
        std::memcpy(pcm, c->h_out.p, out_n * sizeof(int16_t));
        return FMRX_OK;
    }
    if ((rc = c->d_in.ensure(in_bytes)) || (rc = c->d_out.ensure(out_n))) return rc;
    HIPCHK(hipMemcpyAsync(c->d_in.p, iq, in_bytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = fmrx_process_device(c, c->d_in.p, n_blocks, c->d_out.p))) return rc;
    HIPCHK(hipMemcpyAsync(pcm, c->d_out.p, out_n * sizeof(int16_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return FMRX_OK;
}

// rf_thread body (project.cpp:48-70): u8 blocks -> demod floats.
int fmrx_rf_block(fmrx_ctx* c, const uint8_t* iq, size_t n_blocks, float* demod) {
    CtxLock lock_(c);
    if (!c || !iq || !demod) return fail(FMRX_EINVAL, "null argument");
    if (n_blocks == 0) return FMRX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t ns = c->cfg.n_streams;
    const size_t in_bytes = ns * n_blocks * c->geo.block_bytes;
    const size_t n_if = n_blocks * c->geo.if_samples;
    if (in_bytes <= kPinnedCallBytes) {  // pinned staging: the input by DMA (the fused kernel's
                                         // staging reads host memory 4x slower), the demod in place
        if ((rc = c->h_in.ensure(in_bytes)) || (rc = c->h_out.ensure(sizeof(float) * ns * n_if)) ||
            (rc = c->d_in.ensure(in_bytes)))
            return rc;
        std::memcpy(c->h_in.p, iq, in_bytes);
        HIPCHK(hipMemcpyAsync(c->d_in.p, c->h_in.p, in_bytes, hipMemcpyHostToDevice, c->stream));
        float* h_demod = reinterpret_cast<float*>(c->h_out.p);
        if ((rc = run_fused(c, c->d_in.p, n_blocks, nullptr, nullptr, h_demod, n_if, 0, false))) return rc;
        if ((rc = wait_small(c))) return rc;
        std::memcpy(demod, h_demod, sizeof(float) * ns * n_if);
        return FMRX_OK;
    }
    if ((rc = c->d_in.ensure(in_bytes)) || (rc = c->d_f32.ensure(ns * n_if))) return rc;
    HIPCHK(hipMemcpyAsync(c->d_in.p, iq, in_bytes, hipMemcpyHostToDevice, c->stream));
    if ((rc = run_fused(c, c->d_in.p, n_blocks, nullptr, nullptr, c->d_f32.p, n_if, 0, false))) return rc;
    HIPCHK(hipMemcpyAsync(demod, c->d_f32.p, sizeof(float) * ns * n_if, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return FMRX_OK;
}

// audio_thread body (project.cpp:132-195): demod floats -> S16.
int fmrx_audio_block(fmrx_ctx* c, const float* demod, size_t n_blocks, int16_t* pcm) {
    CtxLock lock_(c);
    if (!c || !demod || !pcm) return fail(FMRX_EINVAL, "null argument");
    if (n_blocks == 0) return FMRX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t ns = c->cfg.n_streams;
    const size_t n_if = n_blocks * c->geo.if_samples;
    const size_t out_n = ns * n_blocks * c->geo.pcm_samples;
    if (c->cfg.channels == FMRX_MONO && c->audio_hist_stale)
        return fail(FMRX_ESTATE, "no audio history after fmrx_seek (run a fused call first)");
    // small calls: the demod through the pinned staging (stereo: read there by the band-pass
    // kernel; mono: one copy), the PCM written by the audio kernel into pinned memory in place
    const bool pinned = sizeof(float) * ns * n_if <= kPinnedCallBytes;
    const float* src = demod;
    int16_t* d_pcm = nullptr;
    if (pinned) {
        if ((rc = c->h_in.ensure(sizeof(float) * ns * n_if)) || (rc = c->h_out.ensure(out_n * sizeof(int16_t))))
            return rc;
        std::memcpy(c->h_in.p, demod, sizeof(float) * ns * n_if);
        src = reinterpret_cast<const float*>(c->h_in.p);
        d_pcm = reinterpret_cast<int16_t*>(c->h_out.p);
    } else {
        if ((rc = c->d_out.ensure(out_n))) return rc;
        d_pcm = c->d_out.p;
    }
    if (c->cfg.channels == FMRX_MONO) {
        if ((rc = c->d_f32.ensure(ns * n_if))) return rc;
        HIPCHK(hipMemcpyAsync(c->d_f32.p, src, sizeof(float) * ns * n_if, hipMemcpyHostToDevice, c->stream));
        if ((rc = run_mono_audio(c, c->d_f32.p, n_if, n_if, d_pcm, nullptr))) return rc;
    } else {
        if ((rc = ensure_demod(c, n_if))) return rc;
        if (!pinned)
            HIPCHK(hipMemcpy2DAsync(c->d_demod.p + kDemodHist, c->demod_stride * sizeof(float), src,
                                    n_if * sizeof(float), n_if * sizeof(float), ns,
                                    hipMemcpyHostToDevice, c->stream));
        // pinned: the band-pass kernel reads the staging buffer itself (one launch fewer)
        if ((rc = run_stereo_audio(c, n_blocks, d_pcm, nullptr, pinned ? src : nullptr))) return rc;
    }
    if (!pinned)
        HIPCHK(hipMemcpyAsync(pcm, c->d_out.p, out_n * sizeof(int16_t), hipMemcpyDeviceToHost, c->stream));
    if (pinned) {
        if ((rc = wait_small(c))) return rc;
        std::memcpy(pcm, c->h_out.p, out_n * sizeof(int16_t));
    } else {
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return FMRX_OK;
}

// ---- RDS front half (rds_thread body, project.cpp:200-271) -------------------------------
int fmrx_rds_block(fmrx_ctx* c, const float* demod, size_t n_blocks, float* rds, float* nco,
                   float* channel) {
    CtxLock lock_(c);
    if (!c || !demod || !rds) return fail(FMRX_EINVAL, "null argument");
    if (n_blocks == 0) return FMRX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t ns = c->cfg.n_streams;
    const size_t n = ns * n_blocks * c->geo.if_samples;
    if ((rc = c->d_f32.ensure(n)) || (rc = c->d_scratch.ensure(3 * n))) return rc;
    float* d_rds = c->d_scratch.p;
    float* d_nco = nco ? c->d_scratch.p + n : nullptr;
    float* d_ch = channel ? c->d_scratch.p + 2 * n : nullptr;
    HIPCHK(hipMemcpyAsync(c->d_f32.p, demod, sizeof(float) * n, hipMemcpyHostToDevice, c->stream));
    if ((rc = run_rds(c, c->d_f32.p, n / ns, n / ns, d_rds, d_nco, d_ch))) return rc;
    HIPCHK(hipMemcpyAsync(rds, d_rds, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    if (nco) HIPCHK(hipMemcpyAsync(nco, d_nco, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    if (channel) HIPCHK(hipMemcpyAsync(channel, d_ch, sizeof(float) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return FMRX_OK;
}

int fmrx_rds_device(fmrx_ctx* c, const float* d_demod, size_t n_blocks, float* d_rds, float* d_nco,
                    float* d_channel) {
    CtxLock lock_(c);
    if (!c || !d_demod || !d_rds) return fail(FMRX_EINVAL, "null argument");
    if (n_blocks == 0) return FMRX_OK;
    int rc = set_device(c);
    if (rc) return rc;
    const size_t n_if = n_blocks * c->geo.if_samples;
    return run_rds(c, d_demod, n_if, n_if, d_rds, d_nco, d_channel);
}

// ---- arctan demodulator and PSD estimate ------------------------------
int fmrx_fm_demod_arctan(fmrx_ctx* c, float* d_out, double* d_prev_phase, const float* d_i,
                         const float* d_q, int n) {
    CtxLock lock_(c);
    if (!c || !d_out || !d_prev_phase || !d_i || !d_q || n < 0) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    if (launch_demod_arctan(d_out, d_prev_phase, d_i, d_q, n, c->stream)) return fail(FMRX_EHIP, "launch failed");
    return FMRX_OK;
}

namespace {
// estimatePSD's window (fourier.cpp:57-61): pow(sin(i*PI/N), 2) in double, stored as float.
int psd_run(fmrx_ctx* c, const float* d_x, size_t n, int freq_bins, float fs, float* d_psd) {
    const int N = freq_bins;
    if (N < 2 || N > kPsdMaxBins || (N & (N - 1)) != 0)
        return fail(FMRX_EINVAL, "freq_bins must be a power of two in [2, %d]", kPsdMaxBins);
    const size_t nseg = n / (size_t)N;
    if (nseg < 1) return fail(FMRX_EINVAL, "need at least freq_bins samples");
    int rc = c->d_scratch.ensure((size_t)N + nseg * (N / 2));
    if (rc) return rc;
    std::vector<float> hann(N);
    for (int i = 0; i < N; i++) {
        const double s = std::sin(i * 3.14159265358979323846 / N);  // PI, dy4.h:14
        hann[i] = (float)(s * s);
    }
    HIPCHK(hipMemcpyAsync(c->d_scratch.p, hann.data(), sizeof(float) * N, hipMemcpyHostToDevice, c->stream));
    // psd_seg = (4 / (Fs * freq_bins)) * |X|^2 (fourier.cpp:103)
    const double scale = 4.0 / ((double)fs * (double)N);
    if (launch_psd(d_x, (int)nseg, N, c->d_scratch.p, scale, c->d_scratch.p + N, d_psd, c->stream))
        return fail(FMRX_EHIP, "PSD launch failed");
    HIPCHK(hipStreamSynchronize(c->stream));  // the window lives in host memory until here
    return 0;
}
}  // namespace

int fmrx_psd_device(fmrx_ctx* c, const float* d_samples, size_t n, int freq_bins, float fs, float* d_psd) {
    CtxLock lock_(c);
    if (!c || !d_samples || !d_psd) return fail(FMRX_EINVAL, "null argument");
    int rc = set_device(c);
    return rc ? rc : psd_run(c, d_samples, n, freq_bins, fs, d_psd);
}

int fmrx_estimate_psd(fmrx_ctx* c, const float* samples, size_t n, int freq_bins, float fs, float* freq,
                      float* psd) {
    CtxLock lock_(c);
    if (!c || !samples || !freq || !psd) return fail(FMRX_EINVAL, "null argument");
    int rc = set_device(c);
    if (rc) return rc;
    if (freq_bins < 2) return fail(FMRX_EINVAL, "freq_bins must be >= 2");
    const size_t used = n / (size_t)freq_bins * (size_t)freq_bins;
    if ((rc = c->d_f32.ensure(used + (size_t)freq_bins / 2))) return rc;
    HIPCHK(hipMemcpyAsync(c->d_f32.p, samples, sizeof(float) * used, hipMemcpyHostToDevice, c->stream));
    if ((rc = psd_run(c, c->d_f32.p, used, freq_bins, fs, c->d_f32.p + used))) return rc;
    HIPCHK(hipMemcpy(psd, c->d_f32.p + used, sizeof(float) * (freq_bins / 2), hipMemcpyDeviceToHost));
    const float df = fs / (float)freq_bins;  // fourier.cpp:42-50
    for (int i = 0; i < freq_bins / 2; i++) freq[i] = (float)i * df;
    return FMRX_OK;
}

// ---- filter.h primitives ---------------------------------------------------------------
int fmrx_impulse_response_lpf(float* h, float fs, float fc, int taps, int gain) {
    if (!h || taps < 1) return fail(FMRX_EINVAL, "bad argument");
    design_lpf(h, fs, fc, taps, gain);
    return FMRX_OK;
}

int fmrx_impulse_response_bpf(float* h, float fs, float fb, float fe, int taps) {
    if (!h || taps < 1) return fail(FMRX_EINVAL, "bad argument");
    design_bpf(h, fs, fb, fe, taps);
    return FMRX_OK;
}

int fmrx_resample(fmrx_ctx* c, float* d_out, float* d_state, const float* d_in, int n_in,
                  const float* d_coeff, int taps, int up, int down, int* n_out) {
    CtxLock lock_(c);
    if (!c || !d_out || !d_state || !d_in || !d_coeff || taps < 1 || up < 1 || down < 1)
        return fail(FMRX_EINVAL, "bad argument");
    if (n_in < taps - 1) return fail(FMRX_EINVAL, "input shorter than the filter history");
    int rc = set_device(c);
    if (rc) return rc;
    const int no = (int)((long long)n_in * up / down);  // filter.cpp:77
    if (launch_resample(d_out, d_state, d_in, n_in, d_coeff, taps, up, down, no, c->stream) ||
        launch_tail_copy(d_state, d_in + (n_in - (taps - 1)), taps - 1, c->stream))
        return fail(FMRX_EHIP, "resample launch failed");
    if (n_out) *n_out = no;
    return FMRX_OK;
}

int fmrx_fm_demod(fmrx_ctx* c, float* d_out, float* d_prev, const float* d_i, const float* d_q, int n) {
    CtxLock lock_(c);
    if (!c || !d_out || !d_prev || !d_i || !d_q || n < 0) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    return launch_fm_demod(d_out, d_prev, d_i, d_q, n, c->stream) ? fail(FMRX_EHIP, "launch failed") : 0;
}

int fmrx_pll(fmrx_ctx* c, float* d_io, int n, float freq, float fs, float nco_scale, float phase_adjust,
             float norm_bw, float* d_st) {
    CtxLock lock_(c);
    if (!c || !d_io || !d_st || n < 0) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    // single stream with a 6-float state: stage through the 8-float layout of the kernel
    rc = c->d_scratch.ensure(8);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(c->d_scratch.p, d_st, 6 * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
    // slots 6-7 are the runners' (6: the demoted hand-off, read by every runner launch): zero
    HIPCHK(hipMemsetAsync(c->d_scratch.p + 6, 0, 2 * sizeof(float), c->stream));
    if ((rc = c->d_pll_side.ensure(pll_side_doubles(n, 1)))) return rc;
    // the state is the caller's: its trigOffset (read back, 4 bytes) is the hint when it is in the
    // float increments' domain (an integer in [0, 2^24]); unknown otherwise (every runner launched
    // for every segment, each taking its own streams)
    float trig = -1.0f;
    HIPCHK(hipMemcpyAsync(&trig, d_st + 5, sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    PllHint hint;
    hint.n_simd = c->n_simd;
    hint.knobs = c->knobs.pll;
    hint.known = trig >= 0.0f && trig <= 16777216.0f && trig == std::floor(trig);
    hint.trig_lo = hint.trig_hi = hint.known ? (double)trig : 0.0;
    hint.timer = c->stage_timer.on ? &c->stage_timer : nullptr;
    hint.redos = c->pll_redos;  // fmrx_debug_pll_redos: as stream 0
    if (launch_pll(d_io, n, 1, (size_t)n, freq, fs, nco_scale, phase_adjust, norm_bw, c->d_scratch.p,
                   c->d_pll_side.p, c->stream, hint, c->pll_stats))
        return fail(FMRX_EHIP, "launch failed");
    HIPCHK(hipMemcpyAsync(d_st, c->d_scratch.p, 6 * sizeof(float), hipMemcpyDeviceToDevice, c->stream));
    return FMRX_OK;
}

int fmrx_mixer(fmrx_ctx* c, float* d_out, const float* d_a, const float* d_b, int n) {
    CtxLock lock_(c);
    if (!c || !d_out || !d_a || !d_b || n < 0) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    return launch_mixer(d_out, d_a, d_b, n, c->stream) ? fail(FMRX_EHIP, "launch failed") : 0;
}

int fmrx_lr_extraction(fmrx_ctx* c, float* d_l, float* d_r, const float* d_m, const float* d_s, int n) {
    CtxLock lock_(c);
    if (!c || !d_l || !d_r || !d_m || !d_s || n < 0) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    return launch_lr(d_l, d_r, d_m, d_s, n, c->stream) ? fail(FMRX_EHIP, "launch failed") : 0;
}

int fmrx_normalize_iq(fmrx_ctx* c, const uint8_t* d_iq, size_t n_pairs, float* d_i, float* d_q) {
    CtxLock lock_(c);
    if (!c || !d_iq || !d_i || !d_q) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    return launch_normalize(d_iq, n_pairs, d_i, d_q, c->stream) ? fail(FMRX_EHIP, "launch failed") : 0;
}

int fmrx_quantize(fmrx_ctx* c, const float* d_x, size_t n, int16_t* d_out) {
    CtxLock lock_(c);
    if (!c || !d_x || !d_out) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    return launch_quantize(d_x, n, d_out, c->stream) ? fail(FMRX_EHIP, "launch failed") : 0;
}

int fmrx_test_pll_fallback(fmrx_ctx* c, int kind, const float* d_a, const float* d_b, size_t n, float* d_out) {
    CtxLock lock_(c);
    if (!c || kind < 0 || kind > 2 || (n && (!d_a || !d_out || (kind == 1 && !d_b))))
        return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    return launch_pll_fallback_test(kind, d_a, d_b, n, d_out, c->stream) ? fail(FMRX_EHIP, "launch failed") : 0;
}

// ---- synthetic input --------------------------------------------------------------------
int fmrx_synth_host(uint64_t seed, int rf_fs, uint64_t first_pair, size_t n_pairs, uint8_t* out) {
    if (!out || rf_fs <= 0) return fail(FMRX_EINVAL, "bad argument");
    SynthParams p;
    synth_setup(seed, rf_fs, &p);
    const int16_t* tab = synth_sintab();
    for (size_t k = 0; k < n_pairs; k++) synth_pair(p, tab, first_pair + k, out + 2 * k);
    return FMRX_OK;
}

int fmrx_synth_device(fmrx_ctx* c, uint64_t seed, int rf_fs, uint64_t first_pair, size_t n_pairs,
                      uint8_t* d_out) {
    CtxLock lock_(c);
    if (!c || !d_out || rf_fs <= 0) return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    SynthParams p;
    synth_setup(seed, rf_fs, &p);
    return launch_synth(p, c->d_sintab.p, first_pair, n_pairs, d_out, c->stream)
               ? fail(FMRX_EHIP, "synth launch failed")
               : 0;
}

int fmrx_synth_device_streams(fmrx_ctx* c, const uint64_t* seeds, size_t n_seeds, int rf_fs, uint64_t first_pair,
                              size_t n_pairs, uint8_t* d_out, size_t stride_bytes) {
    CtxLock lock_(c);
    // synth_streams_kernel stores 16-bit (I, Q) pairs at d_out + k stride: both must be even
    if (!c || !d_out || !seeds || rf_fs <= 0 || n_seeds == 0 || n_seeds > 65535 ||
        (n_seeds > 1 && stride_bytes < 2 * n_pairs) || (stride_bytes & 1) ||
        (reinterpret_cast<uintptr_t>(d_out) & 1))
        return fail(FMRX_EINVAL, "bad argument");
    int rc = set_device(c);
    if (rc) return rc;
    std::vector<SynthParams> ps(n_seeds);
    for (size_t k = 0; k < n_seeds; k++) synth_setup(seeds[k], rf_fs, &ps[k]);
    if ((rc = c->d_synth_params.ensure(sizeof(SynthParams) * n_seeds))) return rc;
    // ps is pageable host memory: the stream is drained before it goes out of scope
    HIPCHK(hipMemcpyAsync(c->d_synth_params.p, ps.data(), sizeof(SynthParams) * n_seeds, hipMemcpyHostToDevice,
                          c->stream));
    if (launch_synth_streams(reinterpret_cast<const SynthParams*>(c->d_synth_params.p), (int)n_seeds,
                             c->d_sintab.p, first_pair, n_pairs, d_out, stride_bytes, c->stream)) {
        (void)hipStreamSynchronize(c->stream);  // the copy from ps may still be in flight
        return fail(FMRX_EHIP, "synth launch failed");
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return FMRX_OK;
}

}  // extern "C"

// Diagnostic: per-workgroup clock stamps of the fused mono kernel (default variant, mode 0,
// 101-tap RF); the kernel's results are unchanged.  d_stamps = null turns them off.
int fmrx_debug_mono_stamps(fmrx_ctx* c, unsigned long long* d_stamps, size_t n_workgroups, size_t* needed) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    if (needed) *needed = (size_t)c->cfg.n_streams * 256 * (size_t)mono_wg_per_cu(c->geo.rf_decim);
    if (d_stamps && needed && n_workgroups < *needed)
        return fail(FMRX_EINVAL, "stamp buffer holds %zu workgroups, up to %zu launch", n_workgroups, *needed);
    c->stamps = d_stamps;
    return FMRX_OK;
}

// Diagnostic: per-stage device time of the stereo engine (StageTimer).  op 1 arms (and clears),
// 0 reads, -1 reads and disarms; the read waits for the last recorded event.
int fmrx_debug_stage_timing(fmrx_ctx* c, int op, double* ms, double* steps, long* launches, int n_kinds) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    int rc = set_device(c);
    if (rc) return rc;
    StageTimer& T = c->stage_timer;
    if (op == 1) {
        T.on = true;
        T.used = 0;
        return FMRX_OK;
    }
    if (n_kinds < 0 || (n_kinds > 0 && (!ms || !steps || !launches))) return fail(FMRX_EINVAL, "bad argument");
    for (int k = 0; k < n_kinds; k++) {
        ms[k] = steps[k] = 0.0;
        launches[k] = 0;
    }
    if (T.used) HIPCHK(hipEventSynchronize(T.recs[T.used - 1].b));
    for (size_t i = 0; i < T.used; i++) {
        const StageTimer::Rec& r = T.recs[i];
        if (r.kind >= n_kinds) continue;
        float t = 0.0f;
        HIPCHK(hipEventSynchronize(r.b));
        HIPCHK(hipEventElapsedTime(&t, r.a, r.b));
        ms[r.kind] += t;
        steps[r.kind] += r.steps;
        launches[r.kind] += 1;
    }
    if (op == -1) {
        T.on = false;
        T.used = 0;
    }
    return FMRX_OK;
}

int fmrx_debug_set_knob(fmrx_ctx* c, int knob, double value) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    const KnobSpec* s = knob_spec(knob);
    if (!s) return fail(FMRX_EINVAL, "unknown knob %d", knob);
    if (!knob_ok(*s, value)) return fail(FMRX_EINVAL, "knob %d: %g outside [%g, %g]", knob, value, s->lo, s->hi);
    knob_set(c->knobs, knob, value);
    return FMRX_OK;
}

// Diagnostic: per-stream redo counts of the self-certifying PLL runners (stereo calls).
int fmrx_debug_pll_redos(fmrx_ctx* c, unsigned* d_counts) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    c->pll_redos = d_counts;
    return FMRX_OK;
}

// Diagnostic: speculative-PLL counters of the stereo and PLL calls (launch_pll's spec_stats).
int fmrx_debug_pll_stats(fmrx_ctx* c, unsigned long long* d_counts) {
    CtxLock lock_(c);
    if (!c) return fail(FMRX_EINVAL, "null context");
    c->pll_stats = d_counts;
    return FMRX_OK;
}
