/* oracle/fmrx_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Independent plain-C restatement of the reference FM receive path
 * (/root/reference/src/filter.cpp, src/project.cpp, src/iofunc.cpp).  It is the checker
 * for the HIP product: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  It is pinned bit-for-bit against fixtures produced by the reference itself
 * (oracle/_ref/libfmref.so, see tests/golden/make_golden.py).
 */
#ifndef FMRX_ORACLE_H
#define FMRX_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int rf_fs, rf_decim, if_fs, bp_fs, audio_decim, audio_interp, audio_taps;
    int block_bytes, if_samples, audio_frames;
} orc_mode;

/* same layout as ref_outputs in ref_driver.cpp */
typedef struct {
    float* demod;
    float* mono_exact;
    float* mono_indep;
    int16_t* pcm;
    int16_t* pcm_mono;
    float* channel;
    float* carrier;
    float* nco;
    float* mixer;
    float* stereo;
    float* left;
    float* right;
    float* pll_state;
} orc_outputs;

int orc_geometry(int mode, orc_mode* m);
int orc_lpf(float* h, float Fs, float Fc, int taps, int gain);
int orc_bpf(float* h, float fs, float fb, float fe, int taps);
int orc_normalize(const uint8_t* bytes, int n, float* out);
int orc_resample(float* out, float* state, const float* in, int n_in, const float* coeff, int taps,
                 int up, int down);
int orc_fmdemod(float* out, float* prev, const float* i_ds, const float* q_ds, int n);
int orc_pll(float* io, int n, float freq, float fs, float ncoScale, float phaseAdjust, float normBW,
            float* st);
int orc_mixer(float* out, const float* a, const float* b, int n);
int orc_lr(float* left, float* right, const float* mono, const float* stereo, int n);
int16_t orc_quant(float x);
long orc_run(int mode, int rf_taps, const uint8_t* iq, size_t nbytes, orc_outputs* o);
long orc_run_audio(int mode, const float* demod, size_t n_blocks, orc_outputs* o);
int orc_fm_demod_arctan(double* out, double* prev_phase, const double* i_in, const double* q_in, int n);
int orc_estimate_psd(const float* samples, size_t n, int freq_bins, float fs, float* freq, float* psd);
long orc_rds(int mode, const float* demod, size_t n_blocks, float* channel, float* carrier,
             float* nco, float* rds);

#ifdef __cplusplus
}
#endif
#endif
