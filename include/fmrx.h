/* include/fmrx.h — C ABI of the MI355X-native FM receive chain (libfmrx.so).
 *
 * Drop-in boundary for the per-block processing stage of the reference
 * (mehtas30/Software-Defined-Radio-Course-Project).  Plain C types only: pointers, sizes,
 * ints.  Every entry point returns an int status (FMRX_OK == 0, < 0 on error) instead of
 * calling exit() like the reference does.
 *
 * Reference interfaces replaced (file:line under the reference tree):
 *   fmrx_impulse_response_lpf  <- impulseResponseLPF   include/filter.h:15, src/filter.cpp:14-37
 *   fmrx_impulse_response_bpf  <- impulseResponseBPF   include/filter.h:17, src/filter.cpp:39-64
 *   fmrx_resample              <- resample             include/filter.h:19, src/filter.cpp:67-103
 *   fmrx_fm_demod              <- FMDemod              include/filter.h:21, src/filter.cpp:106-133
 *   fmrx_pll                   <- PLL                  include/filter.h:23, src/filter.cpp:136-174
 *   fmrx_mixer                 <- mixer                include/filter.h:25, src/filter.cpp:176-184
 *   fmrx_lr_extraction         <- LRExtraction         include/filter.h:27, src/filter.cpp:186-199
 *   fmrx_normalize_iq          <- readStdinBlockData   include/iofunc.h:28, src/iofunc.cpp:62-69
 *                                 + deinterleave       src/project.cpp:56-62
 *   fmrx_rf_block              <- rf_thread loop body  src/project.cpp:48-70
 *   fmrx_audio_block           <- audio_thread body    src/project.cpp:132-195
 *   fmrx_process               <- both bodies fused (host buffers in, host PCM out)
 *   fmrx_process_device        <- both bodies fused, device-resident buffers, async
 *   fmrx_rds_block / _device   <- rds_thread body      src/project.cpp:200-271 (RDS front half;
 *                                 never launched by the reference, :380-382)
 *   fmrx_fm_demod_arctan       <- fmDemodArctan        model/fmSupportLib.py:34-63
 *   fmrx_estimate_psd          <- estimatePSD          include/fourier.h:27-31, src/fourier.cpp:35-117
 *   fmrx_psd_device               (model/fmSupportLib.py:83-157)
 *
 * Buffers: functions named *_device / fmrx_resample etc. take DEVICE pointers and enqueue on
 * the context's HIP stream; fmrx_rf_block / fmrx_audio_block / fmrx_process take HOST
 * pointers and return when the result is in host memory.  The caller owns every buffer.
 */
#ifndef FMRX_H
#define FMRX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FMRX_OK 0
#define FMRX_EINVAL (-1)   /* bad argument / configuration */
#define FMRX_EHIP (-2)     /* HIP runtime error (no device, launch failure, ...) */
#define FMRX_ENOMEM (-3)   /* device or host allocation failed */
#define FMRX_ESTATE (-4)   /* state blob size/version mismatch */

/* Output semantics (SURVEY §7 hard part 3). */
#define FMRX_STEREO 2        /* project.cpp output: S16 interleaved R,L; shared audio_state  */
#define FMRX_MONO 1          /* mono S16 with a private audio history (project.cpp:146 with  */
                             /* its own state vector: fmMonoBlock-style receiver)            */

typedef struct {
    int mode;        /* 0..3, src/project.cpp:327-362                                         */
    int channels;    /* FMRX_MONO or FMRX_STEREO                                              */
    int rf_taps;     /* RF LPF taps, reference 51 (project.cpp:306); 0 = default              */
    int bp_taps;     /* stereo band-pass taps, reference 51 (project.cpp:307); 0 = default   */
    int audio_taps;  /* audio LPF taps per phase: 51 only (project.cpp:319; x up in 2/3)    */
    int n_streams;   /* independent IQ streams processed per call (>=1, <= the device's grid.y */
                     /* limit; fmrx_create refuses more with FMRX_EINVAL).  Device memory per   */
                     /* stream: 2 halos (~26 KiB) + the audio history; stereo adds the demod /  */
                     /* channel / carrier rows (3 x 4 B per IF sample of a call) and the PLL    */
                     /* scratch: ~32.5 B per sample of a segment (2^18 samples per stream, fewer */
                     /* past 32 streams: segment x streams ~2^23, >= 2^14 -- ~0.5 MB a stream at */
                     /* 2,048 streams) plus the call's trigArgs, 4 B per IF sample of a call (the */
                     /* NCO reads them after the runners; one 1 GiB mode-0 call: ~200 MB; the    */
                     /* pipelined engine from 16 streams holds two such side buffers).           */
    int device;      /* HIP device ordinal                                                     */
} fmrx_config;

typedef struct {
    int rf_fs, rf_decim, if_fs, bp_fs, audio_up, audio_down;
    int rf_taps, bp_taps, audio_taps_total; /* audio_taps_total = audio_taps * audio_up      */
    size_t block_bytes;   /* u8 per block, project.cpp:364 (256 * rf_decim * audio_decim)     */
    size_t iq_pairs;      /* block_bytes / 2                                                  */
    size_t if_samples;    /* demod floats per block                                           */
    size_t audio_frames;  /* audio frames per block                                           */
    size_t pcm_samples;   /* int16 per block = audio_frames * channels                        */
} fmrx_geometry_t;

typedef struct fmrx_ctx fmrx_ctx;

/* ---- configuration & lifetime ------------------------------------------------------- */
int fmrx_config_default(fmrx_config* cfg, int mode, int channels);
int fmrx_geometry(const fmrx_config* cfg, fmrx_geometry_t* geo);
int fmrx_create(const fmrx_config* cfg, fmrx_ctx** out);
void fmrx_destroy(fmrx_ctx* ctx);
int fmrx_reset(fmrx_ctx* ctx);                         /* back to the power-on state        */
const char* fmrx_last_error(void);                     /* thread-local message              */
const char* fmrx_version(void);

/* ---- stream state (checkpoint / resume) ---------------------------------------------- */
int fmrx_state_size(const fmrx_ctx* ctx, size_t* bytes);
int fmrx_get_state(fmrx_ctx* ctx, void* buf, size_t bytes);
int fmrx_set_state(fmrx_ctx* ctx, const void* buf, size_t bytes);

/* ---- time shards of one recording (mono product) ------------------------- */
/* The mono product has finite memory: the RF FIR (rf_taps - 1 I/Q pairs), the demodulator's
 * previous sample and the audio FIR depend only on a bounded run of raw bytes.  fmrx_seek
 * makes the NEXT call continue a stream whose bytes before it are `prev` (per stream, the n
 * bytes ending right before the call's first byte; stream-major, n_streams x n; n may be
 * anything -- fewer than fmrx_history_bytes means the stream began inside them), so a shard
 * of a recording that starts at a block boundary yields exactly the mono PCM the whole
 * recording yields there.  prev_on_device: 0 host pointer, 1 device pointer.  MONO contexts
 * only (the stereo PLL is a serial recurrence: FMRX_ESTATE); until the next fused call,
 * fmrx_audio_block has no valid history and returns FMRX_ESTATE.                        */
int fmrx_history_bytes(const fmrx_ctx* ctx, size_t* bytes);
int fmrx_seek(fmrx_ctx* ctx, const uint8_t* prev, size_t n, int prev_on_device);

/* ---- block-streaming entry points (host buffers; stream-major for n_streams > 1) ------ */
/* iq: n_streams x (n_blocks * block_bytes) u8; pcm: n_streams x (n_blocks * pcm_samples).  */
int fmrx_process(fmrx_ctx* ctx, const uint8_t* iq, size_t n_blocks, int16_t* pcm);
/* Split stages, the reference's thread split (project.cpp:19-85 | 87-197).
 * demod: n_streams x (n_blocks * if_samples) float.                                        */
int fmrx_rf_block(fmrx_ctx* ctx, const uint8_t* iq, size_t n_blocks, float* demod);
int fmrx_audio_block(fmrx_ctx* ctx, const float* demod, size_t n_blocks, int16_t* pcm);

/* ---- device-resident fused path (async on the context stream) ------------------------ */
int fmrx_process_device(fmrx_ctx* ctx, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm);
/* Optional float taps of the mono product (n_streams x n_blocks*audio_frames), may be NULL */
int fmrx_process_device_ex(fmrx_ctx* ctx, const uint8_t* d_iq, size_t n_blocks, int16_t* d_pcm,
                           float* d_mono);
int fmrx_synchronize(fmrx_ctx* ctx);
void* fmrx_stream(fmrx_ctx* ctx);                       /* the hipStream_t used               */
/* Device time of the fused RF/demod/audio kernel, from HIP event pairs recorded around each
 * launch on the context stream (no host sync in between).  Returns the average over the
 * launches recorded since the last reset.  reset > 0: clear and arm recording; reset < 0:
 * clear and disarm; 0: just read.                                                         */
int fmrx_kernel_timing(fmrx_ctx* ctx, int reset, double* avg_ms, long* launches);

/* ---- filter.h primitives on device buffers (context stream; s = per-call state) ------- */
int fmrx_impulse_response_lpf(float* h, float fs, float fc, int taps, int gain);      /* host */
int fmrx_impulse_response_bpf(float* h, float fs, float fb, float fe, int taps);      /* host */
/* d_state: taps-1 floats (in/out).  Returns the output count in *n_out.                    */
int fmrx_resample(fmrx_ctx* ctx, float* d_out, float* d_state, const float* d_in, int n_in,
                  const float* d_coeff, int taps, int up, int down, int* n_out);
/* d_prev: 2 floats {prev_i, prev_q} (in/out).                                              */
int fmrx_fm_demod(fmrx_ctx* ctx, float* d_out, float* d_prev, const float* d_i,
                  const float* d_q, int n);
/* d_io: PLL input, overwritten by the NCO output.  d_st: 6 floats {integrator, phaseEst,
 * feedbackI, feedbackQ, ncoOut_state, trigOffset} (in/out).  Every PLL (this call, stereo,
 * RDS) runs speculatively with the same bits as the certified recurrence: below trigOffset
 * 2^17 (and without a known trigOffset) the serial loop runs uncertified and every 16-sample
 * batch is re-verified exactly in parallel, the certified path resuming from the first batch
 * that differs; from 2^17 the self-certifying runners (index, three-wave) prove each step as
 * they go and redo a missed interval exactly themselves.  Knob FMRX_KNOB_PLL_SPEC 0 selects the
 * plain certified launch.  fmrx_pll reads d_st's trigOffset back (4 bytes, a host
 * synchronisation on the context stream) to choose the runners.                             */
int fmrx_pll(fmrx_ctx* ctx, float* d_io, int n, float freq, float fs, float nco_scale,
             float phase_adjust, float norm_bw, float* d_st);
int fmrx_mixer(fmrx_ctx* ctx, float* d_out, const float* d_a, const float* d_b, int n);
int fmrx_lr_extraction(fmrx_ctx* ctx, float* d_left, float* d_right, const float* d_mono,
                       const float* d_stereo, int n);
/* u8 interleaved I,Q -> float I and Q (n_pairs each), iofunc.cpp:67 normalisation.        */
int fmrx_normalize_iq(fmrx_ctx* ctx, const uint8_t* d_iq, size_t n_pairs, float* d_i, float* d_q);
/* S16 quantiser of project.cpp:185-191 (NaN -> 0, x86 truncation + 16-bit wrap).           */
int fmrx_quantize(fmrx_ctx* ctx, const float* d_x, size_t n, int16_t* d_out);

/* ---- RDS front half (rds_thread body, src/project.cpp:200-271) ------------------------- */
/* demod (IF rate, as fmrx_rf_block returns it) -> BPF 54-60 kHz -> square -> BPF
 * 113.5-114.5 kHz -> PLL(114 kHz, bp_fs, ncoScale 0.5, 0, 0.01) -> 5-sample channel delay ->
 * mixer.  Every buffer is n_streams x (n_blocks * if_samples) float; rds is the mixer output
 * (project.cpp:271 mixer_data), nco the PLL output (:259), channel the 54-60 kHz band (:247);
 * nco and channel may be NULL.  The RDS state (filter histories, PLL, delay line) lives in the
 * context, starts as the reference's (:206-226), is cleared by fmrx_reset and is not part of
 * the fmrx_get_state blob.  Block-size invariant: any n_blocks per call.                     */
int fmrx_rds_block(fmrx_ctx* ctx, const float* demod, size_t n_blocks, float* rds, float* nco,
                   float* channel);
int fmrx_rds_device(fmrx_ctx* ctx, const float* d_demod, size_t n_blocks, float* d_rds,
                    float* d_nco, float* d_channel);

/* ---- arctan demodulator and PSD estimate (floating-point diagnostics) ------ */
/* fmDemodArctan: out[k] = atan2(Q,I) phase difference to the previous sample, wrapped into
 * [-pi, pi] as np.unwrap does; computed in double, stored as float.  d_prev_phase (one double,
 * in/out) is the phase before d_i[0]; on return the principal phase of the last sample (the
 * model returns the unwrapped one: equal mod 2 pi).  Device buffers, async.                  */
int fmrx_fm_demod_arctan(fmrx_ctx* ctx, float* d_out, double* d_prev_phase, const float* d_i,
                         const float* d_q, int n);
/* estimatePSD: Hann window, floor(n / freq_bins) segments, 10 log10(4/(Fs N) |X|^2) for the
 * freq_bins/2 positive bins, averaged in dB over segments.  freq_bins: power of two in
 * [2, 8192] (FFT in double; the reference's O(N^2) float DFT allows any N); n >= freq_bins.
 * Host buffers: freq and psd_db hold freq_bins/2 floats (freq[i] = i * fs / freq_bins).    */
int fmrx_estimate_psd(fmrx_ctx* ctx, const float* samples, size_t n, int freq_bins, float fs,
                      float* freq, float* psd_db);
int fmrx_psd_device(fmrx_ctx* ctx, const float* d_samples, size_t n, int freq_bins, float fs,
                    float* d_psd_db);

/* ---- deterministic synthetic FM-stereo IQ; identical bytes host/device ---- */
/* Stream `seed`, samples [first_pair, first_pair+n_pairs) of a stream at rf_fs.            */
int fmrx_synth_host(uint64_t seed, int rf_fs, uint64_t first_pair, size_t n_pairs, uint8_t* out);
int fmrx_synth_device(fmrx_ctx* ctx, uint64_t seed, int rf_fs, uint64_t first_pair,
                      size_t n_pairs, uint8_t* d_out);
/* n_seeds streams in ONE launch: stream k (seed seeds[k], host array) is written at
 * d_out + k * stride_bytes, samples [first_pair, first_pair + n_pairs) each (stride_bytes even
 * and >= 2 n_pairs).  Returns after the launch has completed (the seed table is uploaded).    */
int fmrx_synth_device_streams(fmrx_ctx* ctx, const uint64_t* seeds, size_t n_seeds, int rf_fs,
                              uint64_t first_pair, size_t n_pairs, uint8_t* d_out, size_t stride_bytes);

/* ---- test hook: the PLL's fallback libm (src/filter.cpp:161,168-170 on refused args) ---- */
/* Runs the device functions the PLL calls where its certified fast paths refuse, on device
 * buffers (context stream, async): kind 0 -> d_out[2i] = float(sin a_i), d_out[2i+1] =
 * float(cos a_i); kind 1 -> d_out[i] = float(atan2(a_i, b_i)); kind 2 -> d_out[i] = the NCO's
 * float(cos a_i).  tests/test_gpu_parity.py checks them against glibc's floats
 * (tests/golden/pll_fallback.npz).                                                         */
int fmrx_test_pll_fallback(fmrx_ctx* ctx, int kind, const float* d_a, const float* d_b, size_t n,
                           float* d_out);

/* ---- diagnostic: clock stamps of the fused mono kernel ---------------------------------- */
/* With d_stamps set, the mode-0 101-tap fused kernel (default variant) also writes, per     *
 * workgroup w, 6 u64 at d_stamps[6w..]: shader-clock counter at start and end, the 100 MHz  *
 * counter at start and end, HW_ID, XCC_ID (tools/mono_stamps.py: effective clock, wave       *
 * lifetimes, per-XCD balance).  Results are unchanged.  *needed = the largest grid a call    *
 * can launch (n_streams x 256 x resident workgroups per CU).  d_stamps = NULL turns it off. */
int fmrx_debug_mono_stamps(fmrx_ctx* ctx, unsigned long long* d_stamps, size_t n_workgroups, size_t* needed);

/* ---- diagnostic: speculative PLL counters ------------------------------------------------ */
/* With d_counts set (2 u64 on the device, zeroed and owned by the caller), every speculative  *
 * PLL segment of the stereo path and of fmrx_pll adds the runner's 16-step batches that did    *
 * not verify (resumed on the certified path) to d_counts[0] and the batches checked to         *
 * d_counts[1].  Results are unchanged.  d_counts = NULL turns it off.                          */
int fmrx_debug_pll_stats(fmrx_ctx* ctx, unsigned long long* d_counts);

/* ---- diagnostic: per-stream redos of the self-certifying PLL runners ----------------------- */
/* With d_counts set (n_streams x 8 u32 on the device, zeroed and owned by the caller), the stereo *
 * calls and fmrx_pll (as stream 0) add, per stream s and trigOffset range r of a runner launch    *
 * (r = 0 [2^17, 2^20), 1 [2^20, 2^21), 2 [2^21, 2^22), 3 from 2^22, the stuck 2^24 included):     *
 * d_counts[8 s + r] += the intervals the runner redid on the exact path (a trigArg outside its    *
 * candidates or an uncertified step), d_counts[8 s + 4 + r] += the steps it ran demoted (most of   *
 * its last 32 intervals missed, as on an unlocked loop: the rest of the range on the exact path). *
 * Results are unchanged.  d_counts = NULL turns it off.                                           */
int fmrx_debug_pll_redos(fmrx_ctx* ctx, unsigned* d_counts);

/* ---- diagnostic: per-stage device time of the stereo engine ------------------------------ */
/* op 1 arms (and clears) HIP event pairs around every stage launch of the following stereo     *
 * calls (ms of overlapping stages add up); op 0 reads, op -1 reads and disarms.  Stage k of     *
 * n_kinds: 0 RF front end, 1 band-pass pair, 2 PLL pre-pass, 3 lane runner, 4 two-wave          *
 * predicted runner, 5 saturated runner, 6/7/8 three-wave runner forms from trigOffset 2^20 /   *
 * 2^21 / 2^22, 9 check, 10 resume/tail, 11 NCO, 12 audio, 13/14/15 index runner forms from     *
 * trigOffset 2^17 / 2^18 / 2^19, 16-20 count runner forms from 2^17 / 2^18 / 2^19 / 2^20 /      *
 * 2^21 (FMRX_KNOB_PLL_CNT), 21 the three-candidate stick form (trigOffset stuck at 2^24).      *
 * ms[k] = summed device time,                                                                    *
 * launches[k] = launches, steps[k] = serial PLL steps a runner kind ran as its segment's only  *
 * runner (per stream chain; for ns per step of each regime).  Results are unchanged.           */
int fmrx_debug_stage_timing(fmrx_ctx* ctx, int op, double* ms, double* steps, long* launches, int n_kinds);

/* ---- diagnostic / test knobs of one context ----------------------------------------------- */
/* None of them changes the output.  The tuning knobs pick which kernel form runs (A/B
 * measurements); a new context takes them from the environment variable named beside each
 * (read once, at fmrx_create).  The PLL test hooks make the runners do extra work that their
 * exact paths then redo (bit-identical output, counted by fmrx_debug_pll_stats); they are set
 * only here, never from the environment.  value: the knob's integer (the skew: samples).
 * Accepted range [lo, hi] in brackets: fmrx_debug_set_knob returns FMRX_EINVAL for a value
 * outside it (or a fraction for an integer knob), fmrx_create for such an environment variable
 * (tests/test_gpu_parity.py test_knob_sweep_bit_exact sweeps every value of every range).      */
#define FMRX_KNOB_PLL_SPEC 0          /* [0,1] 1 speculative runners, 0 the certified launch FMRX_PLL_SPEC */
#define FMRX_KNOB_PLL_SAT 1           /* [0,1] 0: no saturated-segment runner            FMRX_PLL_SAT  */
#define FMRX_KNOB_PLL_PRED 2          /* [0,2] 0 no predicted runners, 2 forced on       FMRX_PLL_PRED */
#define FMRX_KNOB_PLL_PIPE 3          /* [0,1] 0: no three-wave runner                   FMRX_PLL_PIPE */
#define FMRX_KNOB_PLL_IDX 4           /* [0,2] 2 index runner from 2^17, 1 from 2^18, 0 off FMRX_PLL_IDX */
#define FMRX_KNOB_STEREO_CHUNKS 5     /* [0,64] 0 auto, k chunks (1 the serial engine)  FMRX_STEREO_CHUNKS */
#define FMRX_KNOB_MONO_SPLIT 6        /* [-1,1023] -1 default, 0 equal, n/1024 older wave's FMRX_MONO_SPLIT */
#define FMRX_KNOB_BPF_TILE 7          /* [0,1] 0: the per-output band-pass kernel        FMRX_BPF_TILE */
#define FMRX_KNOB_HALO_KERNEL 8       /* [0,1] 1: the separate halo kernel            FMRX_HALO_KERNEL */
#define FMRX_KNOB_PLL_INJECT 9        /* [-1,2^30] test hook: runners corrupt batch 1+(k+s)%(nb-1) of stream s */
#define FMRX_KNOB_PLL_PIPE_MISS 10    /* [-2^30,2^30] test hook: self-certifying runners miss interval k
                                         (k >= 1), every interval from -k - 1 on (k <= -2: the demotion
                                         runs), none (-1, 0)                                            */
#define FMRX_KNOB_PLL_HINT_SKEW 11    /* [-2^24,2^24] test hook: host trigOffset bounds shifted by value */
#define FMRX_KNOB_PLL_CNT 12          /* [0,31] bit f-17: count runner for form f's range (12) FMRX_PLL_CNT */
#define FMRX_KNOB_PLL_STICK 13        /* [0,1] 1: the stick form past trigOffset 2^24    FMRX_PLL_STICK */
#define FMRX_KNOB_STEREO_HEAD 14      /* [1,64] first chunk in 16ths of a chunk (8)    FMRX_STEREO_HEAD */
#define FMRX_KNOB_STEREO_LEAD 15      /* [0,64] n: chunk k's front end after chunk k-n's PLL FMRX_STEREO_LEAD */
#define FMRX_KNOB_AUDIO_DEFER 16      /* [0,64] 0 beside the next PLL, 1 after the last, 2 (default) all but
                                         the last chunk's beside the last PLL, 2 + e: the first e of those
                                         beside the PLL before it (e past the chunks: all of them)
                                                                                     FMRX_AUDIO_DEFER */
#define FMRX_KNOB_STEREO_TAIL 17      /* [1,64] last chunk in 16ths of a chunk (8)     FMRX_STEREO_TAIL */
int fmrx_debug_set_knob(fmrx_ctx* ctx, int knob, double value);

#ifdef __cplusplus
}
#endif
#endif /* FMRX_H */
