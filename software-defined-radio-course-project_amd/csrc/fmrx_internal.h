// fmrx_internal.h — shared declarations between the host runtime (api.cpp) and the HIP
// kernels (kernels.hip).  Not part of the public ABI (include/fmrx.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "mono_launch.h"
#include "synth.h"

namespace fmrx {

struct ModeConstants {
    int rf_fs, rf_decim, if_fs, bp_fs, audio_up, audio_down;
};

bool mode_constants(int mode, ModeConstants* m);
void design_lpf(float* h, float fs, float fc, int taps, int gain);
void design_bpf(float* h, float fs, float fb, float fe, int taps);

constexpr int kMonoDelay = 5;   // src/project.cpp:308
constexpr int kRfFc = 100000;   // src/project.cpp:304
constexpr int kAudioFc = 16000; // src/project.cpp:305

// Halo bookkeeping: new_halo = last halo_bytes of (old_halo ++ iq), per stream.
int launch_halo_update(const uint8_t* iq, size_t stream_bytes, const uint8_t* old_halo,
                       uint8_t* new_halo, size_t halo_bytes, int n_streams, hipStream_t s);

// ---- stereo engine (REF_EXACT) kernels -----------------------------------------------
struct StereoLaunch {
    const float* demod;     // n_streams x (hist + n_if): hist demod samples precede each call
    float* channel;         // n_streams x out_stride
    float* carrier;         // n_streams x out_stride (PLL in place -> NCO)
    int n_if;               // IF samples this launch per stream
    size_t out_stride;      // floats between streams in channel / carrier (n_if, or the whole
                            //   call's when this launch is a chunk of a longer call)
    int hist;               // demod history length kept in front (>= taps-1)
    size_t demod_stride;    // floats between streams in demod
    const float* ch_c;      // bp taps, HOST memory (passed to the kernel by value)
    const float* ca_c;
    int bp_taps;
    const float* src = nullptr;  // non-null (tiled kernel only): the call's n_if new demod samples a
                                 //   stream (stride n_if, e.g. pinned host memory) are read from here
                                 //   and written into demod behind the history -- no separate copy
};
// tiled = false: the per-output kernel (A/B measurements; same bits)
int launch_bpf_pair(const StereoLaunch& L, int n_streams, hipStream_t s, bool tiled = true);
// PLL over n samples of n_streams streams (state st, 8 floats per stream), then the NCO
// (filter.cpp:136-174).  side: device scratch of pll_side_doubles(n, n_streams) doubles.
// spec_stats (diagnostic, may be null): the speculative path adds the runner batches that did
// not verify to spec_stats[0] and the batches checked to spec_stats[1].
constexpr size_t kPllSeg = (size_t)1 << 18;  // at most this many samples per stream per PLL segment
size_t pll_side_doubles(int n, int n_streams);
// What the host knows when it launches a PLL (api.cpp tracks it per context): the device's SIMD
// count (streams per wave) and, when `known`, bounds on every stream's trigOffset at the call's
// start (integer-valued, <= 2^24: the reference's float increments from a reset), so that
// launch_pll enqueues only the runners some segment can use.  Unknown (the fmrx_pll primitive's
// state lives in caller memory): every runner is launched and each takes its own waves.
// Per-stage device time of the stereo engine (fmrx_debug_stage_timing; diagnostic): HIP event
// pairs recorded on the stream each stage is launched on, read after the call.  Runner records
// carry the serial steps they ran when they were the only runner of their segment (the host's
// trigOffset bounds put every stream in that runner's regime), so ns per step per regime is
// measured, not modelled.
enum StageKind {
    kStFront, kStBpf, kStPrep, kStLane, kStPred, kStSat, kStPipe20, kStPipe21, kStPipe22, kStCheck, kStTail,
    kStNco, kStAudio, kStIdx17, kStIdx18, kStIdx19, kStCnt17, kStCnt18, kStCnt19, kStCnt20, kStCnt21, kStStick, kStKinds
};
struct StageTimer {
    bool on = false;
    struct Rec {
        int kind;
        double steps;
        hipEvent_t a, b;
    };
    std::vector<Rec> recs;
    size_t used = 0;
    int begin(hipStream_t s) {
        if (!on) return -1;
        if (used == recs.size()) {
            Rec r{0, 0.0, nullptr, nullptr};
            if (hipEventCreate(&r.a) != hipSuccess || hipEventCreate(&r.b) != hipSuccess) return -1;
            recs.push_back(r);
        }
        if (hipEventRecord(recs[used].a, s) != hipSuccess) return -1;
        return (int)used++;
    }
    void end(int i, int kind, double steps, hipStream_t s) {
        if (i < 0) return;
        recs[i].kind = kind;
        recs[i].steps = steps;
        (void)hipEventRecord(recs[i].b, s);
    }
    void release() {
        for (auto& r : recs) {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
        recs.clear();
        used = 0;
    }
};

// The count runner's forms by default: [2^19, 2^20) and [2^20, 2^21) (bits 2, 3).  Same-box A/B,
// two alternating rounds (profiles/r05/ab_cnt12/): one 10 s stream 0.1093 -> 0.0923 s, configs[4]
// 0.430 -> 0.418 s, configs[2] 1.240 -> 1.222 s.  [2^17, 2^19) stay on the index runner (the
// count form's 31-candidate evaluators bound it: 68-73 ns a step against 55), [2^21, 2^22) on the
// three-wave runner (profiles/r05/rprof/).
constexpr int kPllCntDefault = 12;

// Per-context switches of the PLL launch (api.cpp fmrx_ctx::knobs; fmrx_debug_set_knob).  The
// tuning ones pick which runners run (same bits either way) and are read from the environment
// once, when the context is created; the test hooks make the runners do extra (redone) work --
// the output stays the exact path's -- and are set only through fmrx_debug_set_knob.
struct PllKnobs {
    int spec = 1;        // 0: the plain certified launch (FMRX_PLL_SPEC)
    int sat = 1;         // 0: no saturated-segment runner (FMRX_PLL_SAT)
    int pred = 1;        // 0: no predicted runners; 2: the two-wave one even where waves share SIMDs
    int pipe = 1;        // 0: no three-wave runner (FMRX_PLL_PIPE)
    int idx = 2;         // index runner from 2^17 (2), from 2^18 (1), off (0) (FMRX_PLL_IDX)
    int cnt = kPllCntDefault;  // bit f - 17: the count runner takes form f's range (FMRX_PLL_CNT)
    int stick = 1;       // the three-candidate runner's stick form past trigOffset 2^24 (FMRX_PLL_STICK)
    int inject = -1;     // test hook: the runners corrupt batch 1 + (k + s) % (nb - 1) of stream s
    int pipe_miss = -1;  // test hook: the self-certifying runners report interval k as missed
    double skew = 0.0;   // test hook: the host's trigOffset bounds shifted by this many samples
};
struct PllHint {
    int n_simd = 1024;
    PllKnobs knobs;
    unsigned* redos = nullptr;  // fmrx_debug_pll_redos (diagnostic): n_streams x kPllRedoSlots
    bool known = false;
    double trig_lo = 0.0, trig_hi = 0.0;
    StageTimer* timer = nullptr;  // diagnostic stage timing (null: off)
    // pll_demoted_kernel once after the call's runner launches (a demoted stream's later launches
    // skip it) instead of after each runner range: the pipelined engine's chunks, where each of its
    // launches waited ~0.3 ms for CUs the stage kernels beside the chains hold
    bool demote_once = false;
};
// nco = false: the NCO pass is left to the caller (launch_pll_nco with the same io, n, stride,
// side and st, on any stream ordered after this launch and before `side` is reused).
int launch_pll(float* io, int n, int n_streams, size_t stride, float freq, float fs,
               float nco_scale, float phase_adjust, float norm_bw, float* st, double* side, hipStream_t s,
               const PllHint& hint, unsigned long long* spec_stats = nullptr, bool nco = true);
int launch_pll_nco(float* io, int n, int n_streams, size_t stride, float nco_scale, float phase_adjust, float* st,
                   const double* side, hipStream_t s);

// pll_sat.hip: the saturated-segment runner over a launch_pll segment (pll_spec_lane_kernel's grid
// and arguments; it runs the streams that one leaves to it)
void launch_pll_sat(dim3 grid, dim3 block, hipStream_t s, const float* io, int n, int n_streams, int spw,
                    size_t stride, const double* side, size_t seg, double step, float norm_bw, const float* st,
                    float* out, size_t ostride, int* fail, float2* rec, size_t rb, int inject);

// pll_pred.hip: the predicted-trigArg runner (segments from trigOffset 2^20, the stick included),
// pll_spec_lane_kernel's arguments, one two-wave workgroup per group of spw streams; it runs the
// groups that kernel leaves to it (pll_pred_wave)
void launch_pll_pred(int waves, hipStream_t s, const float* io, int n, int n_streams, int spw, size_t stride,
                     const double* side, size_t seg, double step, float norm_bw, const float* st, float* out,
                     size_t ostride, int* fail, float2* rec, size_t rb, int inject, int sat_ok, int pipe_on);
// pll_pred.hip: the three-wave runner for one stream a workgroup (spw == 1) from trigOffset 2^20,
// the stick included (pll_pipe_stream), self-certifying (no check / resume kernel): one launch runs
// samples [0, n) of io (stream stride `stride`) from the state st and writes their trigArgs to out
// (stride ostride) and the exact end state to st.  form 22: 3 candidates, 64-step intervals
// (trigOffset from 2^22); 21: 5 candidates, 64 steps ([2^21, 2^22)); 20: 5 candidates, 16 steps
// ([2^20, 2^21)).  A stream whose trigOffset is outside the form's domain runs the range on the
// exact path (a wrong host hint costs speed, not bits).  miss >= 1 / inject >= 0 (test hooks):
// a forced miss on interval `miss` / interval 1 + (inject + s) % intervals, so the exact redo
// runs.  stats (may be null): += batches redone exactly, batches run.
void launch_pll_pipe(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step, float norm_bw,
                     float* st, float* out, size_t ostride, int inject, int miss, int form,
                     unsigned long long* stats, unsigned* redos = nullptr);

// pll_pred.hip: the index runner (one stream a workgroup: the chain and four evaluator waves
// for forms 17 / 18, three for form 19 -- a CU a stream, two of the five waves sharing a SIMD),
// self-certifying like launch_pll_pipe, same arguments; form 17: 32 candidates ([2^17, 2^18)),
// 18: 32 ([2^18, 2^19)), 19: 16 ([2^19, 2^20)).  A stream outside the form's domain runs the
// range exactly.  Returns non-zero when the form's workgroup cannot be resident on one CU (its
// registers) or the launch fails.
int launch_pll_idx(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step, float norm_bw,
                   float* st, float* out, size_t ostride, int inject, int miss, int form, unsigned long long* stats,
                   unsigned* redos = nullptr);
// pll_pred.hip: the count runner (pll_cnt_kernel: the chain picks each step's e by one compare of
// the phase against a row of exact thresholds and a bit count), one stream a workgroup of five
// waves (a CU), self-certifying, same arguments as launch_pll_idx; form 17 / 18: [2^17, 2^18) /
// [2^18, 2^19), 31 candidates, 16-step intervals; 19: [2^19, 2^20), 15, 32 steps; 20: [2^20,
// 2^21), 15, 64 steps; 21: [2^21, 2^22), 7, 64 steps.
int launch_pll_cnt(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step, float norm_bw,
                   float* st, float* out, size_t ostride, int inject, int miss, int form, unsigned long long* stats,
                   unsigned* redos = nullptr);
// pll_demote.hip: the rest of a self-certifying runner launch's range for the streams it demoted
// (pll_device.h pll_demote): the same arguments as the runner launch it follows on stream s.  That
// launch leaves each stream's first step for this kernel in the PLL state's slot 6 (int bits; 0:
// not demoted), which this kernel clears.  One stream a workgroup: a speculative chain
// (pll_spec_lane_kernel's step) checked a sub-segment behind by the other waves, which also form
// its side data; a batch that does not verify is recomputed exactly and the chain resumes after it.
// steps an interval of launch_pll's form (17-23) on the count runner (cnt) or the index / three-wave
// runner: a range of fewer than 24 intervals cannot demote (launch_pll skips pll_demoted_kernel)
int pll_form_interval(int form, bool cnt);
// launch_pll: a range of fewer than kPllShortIntervals of its form's long intervals runs on the
// 16-step forms (in a call of fewer than kPllShortCall steps a stream, to the call's end); a long
// form's tail past its last whole interval of at least kPllShortTail steps runs on the 16-step form
// (three 16-step intervals; a long launch needs two whole intervals or it runs exactly)
constexpr size_t kPllShortCall = 4096, kPllShortIntervals = 2, kPllShortTail = 48;
int launch_pll_demoted(hipStream_t s, const float* io, int n, int n_streams, size_t stride, double step,
                       float norm_bw, float* st, float* out, size_t ostride, int inject, unsigned long long* stats);
// fmrx_debug_pll_redos: per stream kPllRedoSlots u32, by the trigOffset range r of the runner's
// launch (0 [2^17, 2^20), 1 [2^20, 2^21), 2 [2^21, 2^22), 3 from 2^22, the stick included):
// slot r the intervals the self-certifying runners redid exactly, slot 4 + r the steps they ran
// demoted (pll_demote: the rest of a range on the exact path after most intervals missed)
constexpr int kPllRedoSlots = 8;
constexpr int kPllIdxSimds = 4;  // SIMDs a stream takes: one CU (launch_pll admits n_simd / 4 streams)
// the index runner's lowest trigOffset: 2^17 (kPllIdxMin64; 2^18, kPllIdxMin, with FMRX_PLL_IDX=1).  In
// [2^17, 2^18) 32 candidates (c0 - 16 .. c0 + 15) run 62 ns a step with their misses redone,
// against the lane runner's 75; 64 took 113 (1,024 candidate evaluations an interval on three
// evaluator waves, profiles/r04/val/stages.json; profiles/r04/ab_idx17_nc32/)
constexpr float kPllIdxMin = 262144.0f;
constexpr float kPllIdxMin64 = 131072.0f;

// test hook: the PLL's fallback libm on device (kind 0 sincos, 1 atan2, 2 NCO cos)
int launch_pll_fallback_test(int kind, const float* a, const float* b, size_t n, float* out, hipStream_t s);

struct AudioLaunch {
    const float* demod;     // with hist samples in front (per stream stride demod_stride)
    size_t demod_stride;
    int hist;
    const float* channel;   // n_streams x n_if
    const float* nco;       // n_streams x n_if
    float* mix_tail;        // n_streams x (at-1): last mixer samples of the previous block
    float* mono_state;      // n_streams x 5
    int16_t* pcm;           // n_streams x n_blocks*2*frames
    float* mono_out;        // optional REF_EXACT mono floats
    int n_blocks, if_per_block, frames_per_block;
    int up, down, at;       // audio resampler
    const float* audio_c;
};
// The audio stage of blocks [b0, b1) of the call (the blocks before b0 already computed: their
// demod / channel / NCO feed b0's histories), then, when `last`, the state carry of the call's
// last block.  launch_stereo_audio: all of them.
int launch_stereo_audio_range(const AudioLaunch& L, int b0, int b1, bool last, int n_streams, hipStream_t s);
int launch_stereo_audio(const AudioLaunch& L, int n_streams, hipStream_t s);
// A few blocks a stream in ONE launch (modes 0/1, the per-block seam): the NCO from the PLL's
// trigArgs (args, astride floats a stream: pll_trig_args of a launch_pll with nco = false), the audio
// of every block in order, the state carry and the demod history move (the last demod_hist samples
// of the call to the front of its buffer); -1 when the geometry does not fit the tile.
const float* pll_trig_args(const double* side, int n, int n_streams);
int launch_stereo_audio_small(const AudioLaunch& L, int n_streams, const float* args, size_t astride, float nco_scale,
                              float phase_adjust, float* pll_st, int demod_hist, hipStream_t s);

// ---- RDS front half (project.cpp:200-271) ----------------------------------------------
constexpr int kRdsTaps = 51;        // bp_taps, project.cpp:307
constexpr int kRdsDelay = 5;        // rds_delay, project.cpp:309 (commented constant)
constexpr int kRdsDemodHist = 2 * (kRdsTaps - 1);  // both FIRs' history, in demod samples
constexpr int kRdsChanHist = 8;     // >= kRdsDelay channel samples kept in front
struct RdsLaunch {
    const float* demod;     // n_streams x n_if (stride demod_stride), the call's demod
    size_t demod_stride;
    float* dhist;           // n_streams x kRdsDemodHist: demod samples before this call
    float* chan;            // n_streams x (kRdsChanHist + n_if): channel, its tail in front
    size_t chan_stride;
    float* carrier;         // n_streams x n_if: BPF output, then (PLL in place) the NCO
    size_t car_stride;
    float* out;             // n_streams x n_if: mixer output
    size_t out_stride;
    float* pll;             // n_streams x 8 PLL state
    double* pll_side;       // pll_side_doubles(n_if, n_streams) scratch
    const float* ex;        // 54-60 kHz taps (device)
    const float* ca;        // 113.5-114.5 kHz taps (device)
    float bp_fs;
    int n_if;
    PllHint hint;           // the RDS PLL's (launch_pll)
};
int launch_rds(const RdsLaunch& L, int n_streams, hipStream_t s);

// ---- spectrum tooling and the arctan demodulator ------------------
constexpr int kPsdMaxBins = 8192;  // N complex doubles in LDS per segment
int launch_demod_arctan(float* out, double* prev, const float* i, const float* q, int n, hipStream_t s);
int launch_psd(const float* x, int nseg, int N, const float* hann, double scale, float* seg_db, float* psd,
               hipStream_t s);

// ---- generic filter.h primitives ------------------------------------------------------
int launch_resample(float* out, const float* state, const float* in, int n_in,
                    const float* coeff, int taps, int up, int down, int n_out, hipStream_t s);
// mono audio stage of every stream in one launch (project.cpp:146 + the S16 quantiser)
struct PolyStreams {
    const float* in;        // stream s: in + s in_stride, n_out outputs' inputs
    size_t in_stride;
    const float* state;     // stream s: state + s state_stride, taps - 1 floats of history
    size_t state_stride;
    const float* coeff;     // taps
    int taps, up, down, n_out;
    float* out;             // optional float output (stream s at out + s out_stride)
    size_t out_stride;
    int16_t* pcm;           // S16 output (stream s at pcm + s pcm_stride)
    size_t pcm_stride;
};
int launch_polyphase(const PolyStreams& P, int n_streams, hipStream_t s);
int launch_copy_streams(float* dst, size_t dst_stride, const float* src, size_t src_stride, int n, int n_streams,
                        hipStream_t s);
int launch_tail_copy(float* dst, const float* src, int n, hipStream_t s);
int launch_fm_demod(float* out, float* prev, const float* i, const float* q, int n,
                    hipStream_t s);
int launch_mixer(float* out, const float* a, const float* b, int n, hipStream_t s);
int launch_lr(float* l, float* r, const float* m, const float* st, int n, hipStream_t s);
int launch_normalize(const uint8_t* iq, size_t n_pairs, float* i, float* q, hipStream_t s);
int launch_quantize(const float* x, size_t n, int16_t* out, hipStream_t s);
int launch_synth(const SynthParams& p, const int16_t* d_sintab, uint64_t first, size_t n,
                 uint8_t* out, hipStream_t s);
// n_streams streams in one launch: stream k (params d_params[k]) at out + k * stride
int launch_synth_streams(const SynthParams* d_params, int n_streams, const int16_t* d_sintab,
                         uint64_t first, size_t n, uint8_t* out, size_t stride, hipStream_t s);

}  // namespace fmrx
