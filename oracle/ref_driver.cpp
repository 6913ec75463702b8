// oracle/ref_driver.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A sequential driver around the REFERENCE's own DSP code.  It is compiled together
// with /root/reference/src/filter.cpp and /root/reference/src/iofunc.cpp (unmodified,
// in place, by oracle/Makefile) into oracle/_ref/libfmref.so.  It calls the reference
// functions in exactly the order of the two thread bodies of src/project.cpp:
//
//   rf_thread    src/project.cpp:48-84   readStdinBlockData -> deinterleave -> resample(I,Q)
//                                         -> FMDemod
//   audio_thread src/project.cpp:132-196 resample(mono, SHARED audio_state) -> mono delay ->
//                                         resample(channel) -> resample(carrier) -> PLL ->
//                                         mixer -> resample(stereo, SHARED audio_state) ->
//                                         LRExtraction -> S16 quantise (R then L)
//
// with one deliberate difference: every full block is processed, i.e. the
// EOF race of project.cpp:51-54 (exit(1) while audio blocks are still queued) is not
// reproduced.  Partial trailing blocks are dropped exactly like the reference.
//
// It additionally runs the "mono product" (MONO_INDEPENDENT): the same mono resample call
// (project.cpp:146) but with a private history vector, i.e. the mono receiver one gets
// from the reference's primitives without the shared-state coupling of project.cpp:172.
//
// Only tests/, tests/golden/make_golden.py and bench.py's cpu_baseline leg load this.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <streambuf>
#include <vector>

#include "dy4.h"
#include "filter.h"
#include "fourier.h"
#include "iofunc.h"

namespace {

// project.cpp:304-364 (mode table), restated as data.
struct RefMode {
    int rf_fs, rf_decim, if_fs, bp_fs, audio_decim, audio_interp, audio_taps;
};

bool ref_mode(int mode, RefMode* m) {
    const int audio_taps_base = 51;  // project.cpp:319
    switch (mode) {
        case 0: *m = {2400000, 10, 240000, 240000, 5, 1, audio_taps_base}; return true;
        case 1: *m = {1152000, 4, 288000, 288000, 6, 1, audio_taps_base}; return true;
        case 2: *m = {2400000, 10, 240000 * 147, 240000, 800, 147, audio_taps_base * 147}; return true;
        case 3: *m = {2304000, 9, 256000 * 441, 256000, 2560, 441, audio_taps_base * 441}; return true;
        default: return false;
    }
}

// A read-only streambuf so the reference's readStdinBlockData (iofunc.cpp:62-69), which
// reads std::cin, can be fed from memory.
struct MemBuf : std::streambuf {
    MemBuf(const uint8_t* p, size_t n) {
        char* c = reinterpret_cast<char*>(const_cast<uint8_t*>(p));
        setg(c, c, c + n);
    }
};

struct CinRedirect {
    MemBuf buf;
    std::streambuf* old;
    CinRedirect(const uint8_t* p, size_t n) : buf(p, n) {
        old = std::cin.rdbuf(&buf);
        std::cin.clear();
    }
    ~CinRedirect() {
        std::cin.rdbuf(old);
        std::cin.clear();
    }
};

// project.cpp:185-191: NaN -> 0, else static_cast<short int>(x * 16384).
// Compiled with g++ -O3 (no -march) like the reference, so the float->short conversion
// lowers to the same cvttss2si + 16-bit store.
inline short quant(float x) {
    if (std::isnan(x)) return 0;
    return static_cast<short int>(x * 16384);
}

template <class T>
void put(T* dst, size_t off, const std::vector<T>& v) {
    if (dst) std::memcpy(dst + off, v.data(), v.size() * sizeof(T));
}

}  // namespace

extern "C" {

// Optional output pointers (NULL = not wanted).  Sizes per block follow SURVEY table M.
struct ref_outputs {
    float* demod;          // if_samples per block        (project.cpp:69)
    float* mono_exact;     // audio_frames per block      (project.cpp:146, shared state)
    float* mono_indep;     // audio_frames per block      (private-state mono product)
    int16_t* pcm;          // 2*audio_frames per block    (project.cpp:179-195, R,L)
    int16_t* pcm_mono;     // audio_frames per block      (quantised mono_indep)
    float* channel;        // if_samples per block        (project.cpp:162)
    float* carrier;        // if_samples per block        (project.cpp:165, before PLL)
    float* nco;            // if_samples per block        (project.cpp:166, PLL output)
    float* mixer;          // if_samples per block        (project.cpp:169)
    float* stereo;         // audio_frames per block      (project.cpp:172)
    float* left;           // audio_frames per block      (project.cpp:175)
    float* right;          // audio_frames per block
    float* pll_state;      // 6 floats per block after the block: integrator, phaseEst,
                           // feedbackI, feedbackQ, ncoOut_state, trigOffset
};

int ref_geometry(int mode, int* block_bytes, int* if_samples, int* audio_frames) {
    RefMode m;
    if (!ref_mode(mode, &m)) return -1;
    const int block_size = 256 * m.rf_decim * m.audio_decim;  // project.cpp:364
    *block_bytes = block_size;
    *if_samples = block_size / 2 / m.rf_decim;
    *audio_frames = int((long long)(*if_samples) * m.audio_interp / m.audio_decim);
    return 0;
}

// impulseResponseLPF (filter.cpp:14-37)
int ref_lpf(float* h, float fs, float fc, int taps, int gain) {
    std::vector<float> v;
    impulseResponseLPF(v, fs, fc, taps, gain);
    std::memcpy(h, v.data(), v.size() * sizeof(float));
    return (int)v.size();
}

// impulseResponseBPF (filter.cpp:39-64)
int ref_bpf(float* h, float fs, float fb, float fe, int taps) {
    std::vector<float> v;
    impulseResponseBPF(v, fs, fb, fe, taps);
    std::memcpy(h, v.data(), v.size() * sizeof(float));
    return (int)v.size();
}

// resample (filter.cpp:67-103).  state has taps-1 entries on entry and on exit.
int ref_resample(float* out, float* state, const float* in, int n_in, const float* coeff,
                 int taps, int up, int down) {
    std::vector<float> o, s(state, state + taps - 1), x(in, in + n_in), c(coeff, coeff + taps);
    resample(o, s, x, c, up, down);
    std::memcpy(out, o.data(), o.size() * sizeof(float));
    std::memcpy(state, s.data(), s.size() * sizeof(float));
    return (int)o.size();
}

// FMDemod (filter.cpp:106-133).  prev[0]=prev_i, prev[1]=prev_q (in/out).
int ref_fmdemod(float* out, float* prev, const float* i_ds, const float* q_ds, int n) {
    std::vector<float> o, vi(i_ds, i_ds + n), vq(q_ds, q_ds + n);
    FMDemod(o, prev[0], prev[1], vi, vq);
    std::memcpy(out, o.data(), o.size() * sizeof(float));
    return (int)o.size();
}

// PLL (filter.cpp:136-174); io is overwritten with the NCO output like the reference.
// st = {integrator, phaseEst, feedbackI, feedbackQ, ncoOut_state, trigOffset}.
int ref_pll(float* io, int n, float freq, float fs, float ncoScale, float phaseAdjust,
            float normBW, float* st) {
    std::vector<float> v(io, io + n);
    PLL(v, freq, fs, ncoScale, phaseAdjust, normBW, st[0], st[1], st[2], st[3], st[4], st[5]);
    std::memcpy(io, v.data(), n * sizeof(float));
    return n;
}

// readStdinBlockData (iofunc.cpp:62-69) on a memory buffer.
int ref_normalize(const uint8_t* bytes, int n, float* out) {
    CinRedirect r(bytes, (size_t)n);
    std::vector<float> v(n);
    readStdinBlockData((unsigned)n, 0, v);
    std::memcpy(out, v.data(), n * sizeof(float));
    return n;
}

// audio_thread locals (project.cpp:93-130) and body (:143-195) for one demod block, plus the
// private-state mono product (the mono resample of :146 with its own history vector).
struct AudioStage {
    RefMode m;
    const int audio_fc = 16000, bp_taps = 51, mono_delay = 5;  // project.cpp:304-308
    std::vector<float> channel, channel_state, channel_coeff;
    std::vector<float> carrier, carrier_state, carrier_coeff;
    float integrator = 0.0, phaseEst = 0.0, feedbackI = 1.0, feedbackQ = 0.0, trigOffset = 0.0,
          ncoOut_state = 1.0;
    std::vector<float> audio_state, audio_coeff;
    std::vector<float> mono_shift, mono, mono_state;
    std::vector<float> mixer_v, left, right, stereo;
    std::vector<float> indep_state, mono_indep;

    explicit AudioStage(const RefMode& mm)
        : m(mm), channel_state(bp_taps - 1, 0.0), carrier_state(bp_taps - 1, 0.0),
          audio_state(mm.audio_taps - 1, 0.0), mono_state(mono_delay, 0.0),
          indep_state(mm.audio_taps - 1, 0.0) {
        impulseResponseBPF(channel_coeff, m.bp_fs, 22000.0, 54000.0, bp_taps);
        impulseResponseBPF(carrier_coeff, m.bp_fs, 18500, 19500, bp_taps);
        impulseResponseLPF(audio_coeff, m.if_fs, audio_fc, m.audio_taps, m.audio_interp);
    }

    void block(const std::vector<float>& demod, long b, ref_outputs* o) {
        const size_t nif = demod.size();
        // mono product with its own history
        resample(mono_indep, indep_state, demod, audio_coeff, m.audio_interp, m.audio_decim);
        const size_t na = mono_indep.size();
        put(o->mono_indep, b * na, mono_indep);
        if (o->pcm_mono)
            for (size_t k = 0; k < na; k++) o->pcm_mono[b * na + k] = quant(mono_indep[k]);

        // ---- audio_thread body
        resample(mono, audio_state, demod, audio_coeff, m.audio_interp, m.audio_decim);
        put(o->mono_exact, b * na, mono);
        mono_shift.clear();
        mono_shift.insert(mono_shift.end(), mono_state.begin(), mono_state.end());
        mono_shift.insert(mono_shift.end(), mono.begin(), mono.end() - mono_delay);
        mono_state.assign(mono.end() - mono_delay, mono.end());

        resample(channel, channel_state, demod, channel_coeff, 1, 1);
        put(o->channel, b * nif, channel);
        resample(carrier, carrier_state, demod, carrier_coeff, 1, 1);
        put(o->carrier, b * nif, carrier);
        PLL(carrier, 19000, m.if_fs, 2, 0, 0.01, integrator, phaseEst, feedbackI, feedbackQ,
            ncoOut_state, trigOffset);
        put(o->nco, b * nif, carrier);
        if (o->pll_state) {
            float* s = o->pll_state + 6 * b;
            s[0] = integrator; s[1] = phaseEst; s[2] = feedbackI; s[3] = feedbackQ;
            s[4] = ncoOut_state; s[5] = trigOffset;
        }
        mixer(mixer_v, channel, carrier);
        put(o->mixer, b * nif, mixer_v);
        resample(stereo, audio_state, mixer_v, audio_coeff, m.audio_interp, m.audio_decim);
        put(o->stereo, b * na, stereo);
        LRExtraction(left, right, mono_shift, stereo);
        put(o->left, b * na, left);
        put(o->right, b * na, right);
        if (o->pcm) {
            int16_t* p = o->pcm + b * 2 * na;
            for (size_t k = 0; k < left.size(); k++) {
                p[2 * k] = quant(right[k]);
                p[2 * k + 1] = quant(left[k]);
            }
        }
    }
};

// Sequential project.cpp (all full blocks) + the private-state mono product.
// Returns the number of blocks processed, or -1 on a bad mode.
long ref_run(int mode, int rf_taps, const uint8_t* iq, size_t nbytes, ref_outputs* o) {
    RefMode m;
    if (!ref_mode(mode, &m)) return -1;
    const int rf_fc = 100000;                                  // project.cpp:304
    const int block_size = 256 * m.rf_decim * m.audio_decim;  // :364
    const long n_blocks = (long)(nbytes / (size_t)block_size);
    CinRedirect cin_from(iq, nbytes);

    // ---- rf_thread locals (project.cpp:26-46)
    std::vector<float> iq_block(block_size);
    const int half = int(iq_block.size() * 0.5);
    std::vector<float> i_block(half), q_block(half);
    std::vector<float> state_i(rf_taps - 1, 0.0), state_q(rf_taps - 1, 0.0);
    std::vector<float> rf_coeff;
    impulseResponseLPF(rf_coeff, m.rf_fs, rf_fc, rf_taps, 1);
    std::vector<float> i_ds, q_ds, demod;
    float prev_i = 0.0, prev_q = 0.0;
    AudioStage audio(m);

    for (long b = 0; b < n_blocks; b++) {
        readStdinBlockData(block_size, (unsigned)b, iq_block);
        int j = 0;
        for (int i = 0; i < (int)iq_block.size(); i += 2) {
            i_block[j] = iq_block[i];
            q_block[j] = iq_block[i + 1];
            j++;
        }
        resample(i_ds, state_i, i_block, rf_coeff, 1, m.rf_decim);
        resample(q_ds, state_q, q_block, rf_coeff, 1, m.rf_decim);
        FMDemod(demod, prev_i, prev_q, i_ds, q_ds);
        put(o->demod, b * demod.size(), demod);
        audio.block(demod, b, o);
    }
    return n_blocks;
}

// audio_thread alone (project.cpp:132-196) over given demod blocks (if_samples floats each),
// e.g. the reference's own data/fm_demod_10.bin; o->demod is ignored.  Returns the blocks run.
long ref_run_audio(int mode, const float* demod, size_t n_blocks, ref_outputs* o) {
    RefMode m;
    if (!ref_mode(mode, &m)) return -1;
    const size_t nif = (size_t)(256 * m.rf_decim * m.audio_decim) / 2 / m.rf_decim;
    AudioStage audio(m);
    for (size_t b = 0; b < n_blocks; b++) {
        std::vector<float> d(demod + b * nif, demod + (b + 1) * nif);
        audio.block(d, (long)b, o);
    }
    return (long)n_blocks;
}

// CPU baseline: the reference's sequential mono-only receive path (rf_thread body +
// the mono resample with a private history + quantise), one core.
long ref_run_mono(int mode, int rf_taps, const uint8_t* iq, size_t nbytes, int16_t* pcm) {
    RefMode m;
    if (!ref_mode(mode, &m)) return -1;
    const int rf_fc = 100000, audio_fc = 16000;
    const int block_size = 256 * m.rf_decim * m.audio_decim;
    const long n_blocks = (long)(nbytes / (size_t)block_size);
    CinRedirect cin_from(iq, nbytes);
    std::vector<float> iq_block(block_size);
    const int half = int(iq_block.size() * 0.5);
    std::vector<float> i_block(half), q_block(half);
    std::vector<float> state_i(rf_taps - 1, 0.0), state_q(rf_taps - 1, 0.0), rf_coeff;
    impulseResponseLPF(rf_coeff, m.rf_fs, rf_fc, rf_taps, 1);
    std::vector<float> i_ds, q_ds, demod, mono;
    float prev_i = 0.0, prev_q = 0.0;
    std::vector<float> audio_state(m.audio_taps - 1, 0.0), audio_coeff;
    impulseResponseLPF(audio_coeff, m.if_fs, audio_fc, m.audio_taps, m.audio_interp);
    for (long b = 0; b < n_blocks; b++) {
        readStdinBlockData(block_size, (unsigned)b, iq_block);
        int j = 0;
        for (int i = 0; i < (int)iq_block.size(); i += 2) {
            i_block[j] = iq_block[i];
            q_block[j] = iq_block[i + 1];
            j++;
        }
        resample(i_ds, state_i, i_block, rf_coeff, 1, m.rf_decim);
        resample(q_ds, state_q, q_block, rf_coeff, 1, m.rf_decim);
        FMDemod(demod, prev_i, prev_q, i_ds, q_ds);
        resample(mono, audio_state, demod, audio_coeff, m.audio_interp, m.audio_decim);
        for (size_t k = 0; k < mono.size(); k++) pcm[b * mono.size() + k] = quant(mono[k]);
    }
    return n_blocks;
}

// RDS front half, rds_thread body (src/project.cpp:200-271; dead code in the reference: the
// thread launch is commented out at :380-382, its constants at :308-309): per demod block
//   resample(channel, BPF 54-60 kHz) -> square -> resample(carrier, BPF 113.5-114.5 kHz) ->
//   PLL(114 kHz, bp_fs, ncoScale 0.5, phaseAdjust 0, normBW 0.01) -> channel delay (5) ->
//   mixer(carrier, delayed channel).
// The 3 kHz LPF it designs (:229-230) is never applied and is not reproduced.  Outputs (all
// optional, if_samples per block each): channel, carrier (before the PLL), nco (PLL output),
// rds (mixer output).  Returns the number of blocks, -1 on a bad mode.
long ref_rds(int mode, const float* demod, size_t n_blocks, float* channel, float* carrier,
             float* nco, float* rds) {
    RefMode m;
    if (!ref_mode(mode, &m)) return -1;
    const int bp_taps = 51, channel_delay = 5;  // project.cpp:307, :309 (rds_delay)
    const size_t nif = (size_t)(256 * m.rf_decim * m.audio_decim) / 2 / m.rf_decim;  // IF samples/block
    std::vector<float> channel_shift, channel_shift_state(channel_delay, 0.0f), channel_data;
    std::vector<float> channel_state(bp_taps - 1, 0.0f), extract_coeff;
    impulseResponseBPF(extract_coeff, m.bp_fs, 54000, 60000, bp_taps);
    std::vector<float> channel_squared, carrier_data, carrier_state(bp_taps - 1, 0.0f), carrier_coeff;
    impulseResponseBPF(carrier_coeff, m.bp_fs, 113500, 114500, bp_taps);
    float integrator = 0.0f, phaseEst = 0.0f, feedbackI = 1.0f, feedbackQ = 0.0f, trigOffset = 0.0f;
    float ncoOut_state = 1.0f;
    std::vector<float> mixer_data;
    for (size_t b = 0; b < n_blocks; b++) {
        std::vector<float> demod_data(demod + b * nif, demod + (b + 1) * nif);
        resample(channel_data, channel_state, demod_data, extract_coeff, 1, 1);
        channel_squared.assign(channel_data.size(), 0.0f);
        for (size_t i = 0; i < channel_data.size(); i++) channel_squared[i] = channel_data[i] * channel_data[i];
        resample(carrier_data, carrier_state, channel_squared, carrier_coeff, 1, 1);
        put(carrier, b * nif, carrier_data);
        PLL(carrier_data, 114000, m.bp_fs, 0.5, 0, 0.01, integrator, phaseEst, feedbackI, feedbackQ,
            ncoOut_state, trigOffset);
        channel_shift.clear();
        channel_shift.insert(channel_shift.end(), channel_shift_state.begin(), channel_shift_state.end());
        channel_shift.insert(channel_shift.end(), channel_data.begin(), channel_data.end() - channel_delay);
        channel_shift_state.assign(channel_data.end() - channel_delay, channel_data.end());
        mixer(mixer_data, carrier_data, channel_shift);
        put(channel, b * nif, channel_data);
        put(nco, b * nif, carrier_data);
        put(rds, b * nif, mixer_data);
    }
    return (long)n_blocks;
}

// estimatePSD (src/fourier.cpp:35-117): Hann window, per-segment DFT, 10 log10 of
// 4/(Fs N) |X|^2 over the positive half, averaged in dB over the whole segments.  freq and
// psd hold freq_bins/2 floats.  Returns the number of segments.
int ref_estimate_psd(const float* samples, size_t n, int freq_bins, float fs, float* freq, float* psd) {
    std::vector<float> f, p, x(samples, samples + n);
    estimatePSD(f, p, x, freq_bins, fs);
    std::memcpy(freq, f.data(), f.size() * sizeof(float));
    std::memcpy(psd, p.data(), p.size() * sizeof(float));
    return (int)(n / (size_t)freq_bins);
}

}  // extern "C"
