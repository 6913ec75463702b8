/* oracle/fmrx_oracle.c — TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C restatement of the reference receive path, written from the reference's
 * semantics (each function cites the file:line it follows) with every implicit C++
 * float/double promotion of the reference spelled out explicitly.  Built with
 * gcc -O2 -ffp-contract=off (no FMA), like the reference's g++ -O3 without -march.
 *
 * Pinned: tests/test_oracle.py checks every function bit-for-bit against fixtures that the
 * reference itself produced (oracle/_ref/libfmref.so, fixtures under tests/golden).
 */
#include "fmrx_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PI 3.14159265358979323846 /* include/dy4.h:14 — a DOUBLE literal */

/* src/project.cpp:304-364 — per-mode constants; block size in bytes at :364. */
int orc_geometry(int mode, orc_mode* m) {
    switch (mode) {
        case 0: m->rf_fs = 2400000; m->rf_decim = 10; m->if_fs = 240000; m->bp_fs = 240000;
                m->audio_decim = 5; m->audio_interp = 1; break;
        case 1: m->rf_fs = 1152000; m->rf_decim = 4; m->if_fs = 288000; m->bp_fs = 288000;
                m->audio_decim = 6; m->audio_interp = 1; break;
        case 2: m->rf_fs = 2400000; m->rf_decim = 10; m->if_fs = 240000 * 147; m->bp_fs = 240000;
                m->audio_decim = 800; m->audio_interp = 147; break;
        case 3: m->rf_fs = 2304000; m->rf_decim = 9; m->if_fs = 256000 * 441; m->bp_fs = 256000;
                m->audio_decim = 2560; m->audio_interp = 441; break;
        default: return -1;
    }
    m->audio_taps = 51 * m->audio_interp;
    m->block_bytes = 256 * m->rf_decim * m->audio_decim;
    m->if_samples = m->block_bytes / 2 / m->rf_decim;
    m->audio_frames = (int)((long long)m->if_samples * m->audio_interp / m->audio_decim);
    return 0;
}

/* src/filter.cpp:14-37 impulseResponseLPF.
 * norm_fc and 1/N are float; the centre test and the sinc argument are double; sin() is the
 * double libm call; pow(x,2) is folded by g++ into a double square. */
int orc_lpf(float* h, float Fs, float Fc, int taps, int gain) {
    const float norm_fc = Fc / (Fs / 2.0f);
    const float inv_taps = 1.0f / (float)taps;
    const double centre = (double)(taps - 1) * 0.5;
    for (int i = 0; i < taps; i++) {
        float v;
        if ((double)i == centre) {
            v = norm_fc;
        } else {
            const float den = (float)((ORC_PI * (double)norm_fc) * ((double)i - centre));
            const float num = (float)sin((double)den);
            v = norm_fc * (num / den);
        }
        const double w = sin(((double)i * ORC_PI) * (double)inv_taps);
        v = (float)((double)v * (w * w));
        if (gain != 1) v = v * (float)gain;
        h[i] = v;
    }
    return taps;
}

/* src/filter.cpp:39-64 impulseResponseBPF.  Here the sinc quotient and both window
 * factors stay in double until the float store. */
int orc_bpf(float* h, float fs, float fb, float fe, int taps) {
    const float norm_cent = (fe + fb) / fs;
    const float norm_pass = 2.0f * (fe - fb) / fs;
    const double centre = (double)(taps - 1) * 0.5;
    for (int i = 0; i < taps; i++) {
        float v;
        if (i == (taps - 1) / 2) {
            v = norm_pass;
        } else {
            const float den = (float)((ORC_PI * ((double)norm_pass * 0.5)) * ((double)i - centre));
            v = (float)(((double)norm_pass * sin((double)den)) / (double)den);
        }
        v = (float)((double)v * cos(((double)i * ORC_PI) * (double)norm_cent));
        const double w = sin(((double)i * ORC_PI) / (double)taps);
        v = (float)((double)v * (w * w));
        h[i] = v;
    }
    return taps;
}

/* src/iofunc.cpp:67 — (u8 - 128.0) / 128.0 evaluated in double, stored as float (exact). */
int orc_normalize(const uint8_t* bytes, int n, float* out) {
    for (int k = 0; k < n; k++) out[k] = (float)(((double)(float)bytes[k] - 128.0) / 128.0);
    return n;
}

/* src/filter.cpp:67-103 resample: polyphase up/down FIR over [state ++ input].
 * Each output is a SEQUENTIAL float sum in ascending tap order, mul and add rounded
 * separately; afterwards the state is the last taps-1 inputs. */
int orc_resample(float* out, float* state, const float* in, int n_in, const float* coeff, int taps,
                 int up, int down) {
    const int state_size = taps - 1;
    const int n_out = (int)((long long)n_in * up / down);
    for (int n = 0; n < n_out; n++) {
        float acc = 0.0f;
        const long long nd = (long long)n * down;
        for (int k = (int)(nd % up); k < taps; k += up) {
            const long long j = (nd - k) / up;
            const float x = j >= 0 ? in[j] : state[state_size + j];
            acc = acc + coeff[k] * x;
        }
        out[n] = acc;
    }
    memmove(state, in + (n_in - state_size), (size_t)state_size * sizeof(float));
    return n_out;
}

/* src/filter.cpp:106-133 FMDemod: derivative discriminator (I dQ - Q dI)/(I^2+Q^2),
 * the denominator via std::pow(float,2) i.e. double squares summed in double. */
int orc_fmdemod(float* out, float* prev, const float* i_ds, const float* q_ds, int n) {
    float pi = prev[0], pq = prev[1];
    for (int k = 0; k < n; k++) {
        const float ci = i_ds[k], cq = q_ds[k];
        const float di = ci - pi, dq = cq - pq;
        const float den = (float)((double)ci * (double)ci + (double)cq * (double)cq);
        if (den != 0.0f) {
            const float num = (ci * dq) - (cq * di);
            out[k] = num / den;
        } else {
            out[k] = 0.0f;
        }
        pi = ci;
        pq = cq;
    }
    prev[0] = pi;
    prev[1] = pq;
    return n;
}

/* src/filter.cpp:136-174 PLL, output in place.  st = {integrator, phaseEst, feedbackI,
 * feedbackQ, ncoOut_state, trigOffset}.  Float state; atan2/cos/sin in double. */
int orc_pll(float* io, int n, float freq, float fs, float ncoScale, float phaseAdjust, float normBW,
            float* st) {
    const float Cp = (float)2.666, Ci = (float)3.555;
    const float Kp = normBW * Cp;
    const float Ki = (normBW * normBW) * Ci;
    float integ = st[0], phase = st[1], fbI = st[2], fbQ = st[3], trig = st[5];
    const double step = (2.0 * ORC_PI) * (double)(freq / fs);
    for (int i = 0; i < n; i++) {
        const float x = io[i];
        const float eI = x * fbI;
        const float eQ = x * (-fbQ);
        const float e = (float)atan2((double)eQ, (double)eI);
        integ = integ + Ki * e;
        phase = phase + ((Kp * e) + integ);
        trig = trig + 1.0f;
        const float arg = (float)(step * (double)trig + (double)phase);
        fbI = (float)cos((double)arg);
        fbQ = (float)sin((double)arg);
        io[i] = (float)cos((double)(arg * ncoScale + phaseAdjust));
    }
    st[0] = integ; st[1] = phase; st[2] = fbI; st[3] = fbQ; st[5] = trig;
    if (n > 0) st[4] = io[n - 1];
    return n;
}

/* src/filter.cpp:176-184 mixer: 2 * (a * b), float. */
int orc_mixer(float* out, const float* a, const float* b, int n) {
    for (int i = 0; i < n; i++) out[i] = 2.0f * (a[i] * b[i]);
    return n;
}

/* src/filter.cpp:186-199 LRExtraction: (mono +/- stereo) * 0.5 (double 0.5, exact). */
int orc_lr(float* left, float* right, const float* mono, const float* stereo, int n) {
    for (int i = 0; i < n; i++) {
        left[i] = (float)((double)(mono[i] + stereo[i]) * 0.5);
        right[i] = (float)((double)(mono[i] - stereo[i]) * 0.5);
    }
    return n;
}

/* src/project.cpp:185-191: NaN -> 0, else static_cast<short>(x * 16384) as x86-64 g++ lowers
 * it: cvttss2si to int32 (out-of-range/inf -> INT32_MIN) then the low 16 bits are stored. */
int16_t orc_quant(float x) {
    if (isnan(x)) return 0;
    const float v = x * 16384.0f;
    int32_t t;
    if (!(v < 2147483648.0f) || v < -2147483648.0f) t = INT32_MIN;
    else t = (int32_t)v;
    return (int16_t)(uint16_t)((uint32_t)t & 0xFFFFu);
}

/* Sequential src/project.cpp (rf_thread :48-84 then audio_thread :132-196 per block; all
 * full blocks, no EOF race) plus the private-history mono product.  With demod_in set, the
 * rf_thread half is skipped and block b's demod is demod_in + b * if_samples. */
static long run_blocks(const orc_mode* mp, int rf_taps, const uint8_t* iq, const float* demod_in,
                       long n_blocks, orc_outputs* o) {
    const orc_mode m = *mp;
    const int bp_taps = 51, mono_delay = 5;
    const int B = m.block_bytes, H = B / 2, NIF = m.if_samples, NA = m.audio_frames;
    const int at = m.audio_taps;

    float* rf_c = malloc(sizeof(float) * rf_taps);
    float* ch_c = malloc(sizeof(float) * bp_taps);
    float* ca_c = malloc(sizeof(float) * bp_taps);
    float* au_c = malloc(sizeof(float) * at);
    orc_lpf(rf_c, (float)m.rf_fs, 100000.0f, rf_taps, 1);
    orc_bpf(ch_c, (float)m.bp_fs, 22000.0f, 54000.0f, bp_taps);
    orc_bpf(ca_c, (float)m.bp_fs, 18500.0f, 19500.0f, bp_taps);
    orc_lpf(au_c, (float)m.if_fs, 16000.0f, at, m.audio_interp);

    float* xb = malloc(sizeof(float) * B);
    float* ib = malloc(sizeof(float) * H);
    float* qb = malloc(sizeof(float) * H);
    float* ids = malloc(sizeof(float) * NIF);
    float* qds = malloc(sizeof(float) * NIF);
    float* dem = malloc(sizeof(float) * NIF);
    float* chn = malloc(sizeof(float) * NIF);
    float* car = malloc(sizeof(float) * NIF);
    float* mix = malloc(sizeof(float) * NIF);
    float* mono = malloc(sizeof(float) * NA);
    float* mind = malloc(sizeof(float) * NA);
    float* ster = malloc(sizeof(float) * NA);
    float* shift = malloc(sizeof(float) * NA);
    float* left = malloc(sizeof(float) * NA);
    float* right = malloc(sizeof(float) * NA);
    float* st_i = calloc((size_t)rf_taps - 1, sizeof(float));
    float* st_q = calloc((size_t)rf_taps - 1, sizeof(float));
    float* st_ch = calloc((size_t)bp_taps - 1, sizeof(float));
    float* st_ca = calloc((size_t)bp_taps - 1, sizeof(float));
    float* st_au = calloc((size_t)at - 1, sizeof(float)); /* SHARED mono/stereo history */
    float* st_in = calloc((size_t)at - 1, sizeof(float)); /* private mono history */
    float st_mono[5] = {0, 0, 0, 0, 0};
    float prev[2] = {0.0f, 0.0f};
    float pll[6] = {0.0f, 0.0f, 1.0f, 0.0f, 1.0f, 0.0f}; /* project.cpp:106-111 */

    for (long b = 0; b < n_blocks; b++) {
        if (demod_in) {
            memcpy(dem, demod_in + (size_t)b * NIF, sizeof(float) * NIF);
        } else {
            orc_normalize(iq + (size_t)b * B, B, xb);
            for (int k = 0; k < H; k++) {
                ib[k] = xb[2 * k];
                qb[k] = xb[2 * k + 1];
            }
            orc_resample(ids, st_i, ib, H, rf_c, rf_taps, 1, m.rf_decim);
            orc_resample(qds, st_q, qb, H, rf_c, rf_taps, 1, m.rf_decim);
            orc_fmdemod(dem, prev, ids, qds, NIF);
        }
        if (o->demod) memcpy(o->demod + b * NIF, dem, sizeof(float) * NIF);

        orc_resample(mind, st_in, dem, NIF, au_c, at, m.audio_interp, m.audio_decim);
        if (o->mono_indep) memcpy(o->mono_indep + b * NA, mind, sizeof(float) * NA);
        if (o->pcm_mono)
            for (int k = 0; k < NA; k++) o->pcm_mono[b * NA + k] = orc_quant(mind[k]);

        orc_resample(mono, st_au, dem, NIF, au_c, at, m.audio_interp, m.audio_decim);
        if (o->mono_exact) memcpy(o->mono_exact + b * NA, mono, sizeof(float) * NA);
        /* project.cpp:152-159 five-sample delay line */
        for (int k = 0; k < NA; k++) shift[k] = k < mono_delay ? st_mono[k] : mono[k - mono_delay];
        for (int k = 0; k < mono_delay; k++) st_mono[k] = mono[NA - mono_delay + k];

        orc_resample(chn, st_ch, dem, NIF, ch_c, bp_taps, 1, 1);
        if (o->channel) memcpy(o->channel + b * NIF, chn, sizeof(float) * NIF);
        orc_resample(car, st_ca, dem, NIF, ca_c, bp_taps, 1, 1);
        if (o->carrier) memcpy(o->carrier + b * NIF, car, sizeof(float) * NIF);
        /* project.cpp:166 — note Fs = if_fs, the UPSAMPLED rate in modes 2/3 */
        orc_pll(car, NIF, 19000.0f, (float)m.if_fs, 2.0f, 0.0f, 0.01f, pll);
        if (o->nco) memcpy(o->nco + b * NIF, car, sizeof(float) * NIF);
        if (o->pll_state) memcpy(o->pll_state + 6 * b, pll, sizeof(float) * 6);
        orc_mixer(mix, chn, car, NIF);
        if (o->mixer) memcpy(o->mixer + b * NIF, mix, sizeof(float) * NIF);
        orc_resample(ster, st_au, mix, NIF, au_c, at, m.audio_interp, m.audio_decim);
        if (o->stereo) memcpy(o->stereo + b * NA, ster, sizeof(float) * NA);
        orc_lr(left, right, shift, ster, NA);
        if (o->left) memcpy(o->left + b * NA, left, sizeof(float) * NA);
        if (o->right) memcpy(o->right + b * NA, right, sizeof(float) * NA);
        if (o->pcm)
            for (int k = 0; k < NA; k++) {
                o->pcm[b * 2 * NA + 2 * k] = orc_quant(right[k]);
                o->pcm[b * 2 * NA + 2 * k + 1] = orc_quant(left[k]);
            }
    }
    free(rf_c); free(ch_c); free(ca_c); free(au_c); free(xb); free(ib); free(qb); free(ids);
    free(qds); free(dem); free(chn); free(car); free(mix); free(mono); free(mind); free(ster);
    free(shift); free(left); free(right); free(st_i); free(st_q); free(st_ch); free(st_ca);
    free(st_au); free(st_in);
    return n_blocks;
}

long orc_run(int mode, int rf_taps, const uint8_t* iq, size_t nbytes, orc_outputs* o) {
    orc_mode m;
    if (orc_geometry(mode, &m) != 0 || rf_taps < 2) return -1;
    return run_blocks(&m, rf_taps, iq, NULL, (long)(nbytes / (size_t)m.block_bytes), o);
}

/* audio_thread alone (project.cpp:132-196) over n_blocks demod blocks of if_samples floats. */
long orc_run_audio(int mode, const float* demod, size_t n_blocks, orc_outputs* o) {
    orc_mode m;
    if (orc_geometry(mode, &m) != 0) return -1;
    return run_blocks(&m, 51, NULL, demod, (long)n_blocks, o);
}

/* RDS front half, the rds_thread body (src/project.cpp:200-271, dead code in the reference):
 * per demod block BPF 54-60 kHz (:211, :247) -> square (:250-254) -> BPF 113.5-114.5 kHz
 * (:217, :257) -> PLL(114 kHz, bp_fs, 0.5, 0, 0.01) (:259) -> 5-sample channel delay
 * (:262-268, rds_delay :309) -> mixer(carrier, delayed channel) (:271).  Outputs (optional,
 * if_samples per block): channel, carrier (PLL input), nco (PLL output), rds (mixer). */
long orc_rds(int mode, const float* demod, size_t n_blocks, float* channel, float* carrier,
             float* nco, float* rds) {
    orc_mode m;
    if (orc_geometry(mode, &m) != 0) return -1;
    enum { T = 51, DLY = 5 };
    const int NIF = m.if_samples;
    float ex_c[T], ca_c[T], st_ex[T - 1], st_ca[T - 1], shift_st[DLY], pll[6] = {0, 0, 1, 0, 1, 0};
    orc_bpf(ex_c, (float)m.bp_fs, 54000.0f, 60000.0f, T);
    orc_bpf(ca_c, (float)m.bp_fs, 113500.0f, 114500.0f, T);
    memset(st_ex, 0, sizeof st_ex);
    memset(st_ca, 0, sizeof st_ca);
    memset(shift_st, 0, sizeof shift_st);
    float* ch = (float*)malloc(sizeof(float) * NIF);
    float* sq = (float*)malloc(sizeof(float) * NIF);
    float* ca = (float*)malloc(sizeof(float) * NIF);
    float* sh = (float*)malloc(sizeof(float) * NIF);
    for (size_t b = 0; b < n_blocks; b++) {
        orc_resample(ch, st_ex, demod + b * NIF, NIF, ex_c, T, 1, 1);
        for (int i = 0; i < NIF; i++) sq[i] = ch[i] * ch[i];
        orc_resample(ca, st_ca, sq, NIF, ca_c, T, 1, 1);
        if (carrier) memcpy(carrier + b * NIF, ca, sizeof(float) * NIF);
        orc_pll(ca, NIF, 114000.0f, (float)m.bp_fs, 0.5f, 0.0f, 0.01f, pll);
        memcpy(sh, shift_st, sizeof shift_st);
        memcpy(sh + DLY, ch, sizeof(float) * (NIF - DLY));
        memcpy(shift_st, ch + NIF - DLY, sizeof shift_st);
        if (channel) memcpy(channel + b * NIF, ch, sizeof(float) * NIF);
        if (nco) memcpy(nco + b * NIF, ca, sizeof(float) * NIF);
        if (rds) orc_mixer(rds + b * NIF, ca, sh, NIF);
    }
    free(ch); free(sq); free(ca); free(sh);
    return (long)n_blocks;
}

/* fmDemodArctan (model/fmSupportLib.py:34-63), float64 like the model: per sample
 * current_phase = atan2(Q, I); [prev, current] = np.unwrap([prev, current]); demod = current -
 * prev; prev = current (the UNWRAPPED phase, which keeps growing).  np.unwrap (numpy 2.x):
 * dd = cur - prev; ddmod = mod(dd + pi, 2 pi) - pi (numpy's floored mod); ddmod = pi where
 * ddmod == -pi and dd > 0; correction ddmod - dd, zeroed when |dd| < pi. */
static double np_mod(double x, double y) {
    double m = fmod(x, y);
    if (m != 0.0 && ((y < 0.0) != (m < 0.0))) m += y;
    return m;
}

int orc_fm_demod_arctan(double* out, double* prev_phase, const double* i_in, const double* q_in, int n) {
    const double pi = 3.141592653589793, two_pi = 2.0 * pi;
    double prev = *prev_phase;
    for (int k = 0; k < n; k++) {
        const double cur = atan2(q_in[k], i_in[k]);
        const double dd = cur - prev;
        double ddmod = np_mod(dd + pi, two_pi) - pi;
        if (ddmod == -pi && dd > 0.0) ddmod = pi;
        double corr = ddmod - dd;
        if (fabs(dd) < pi) corr = 0.0;
        const double unwrapped = cur + corr;
        out[k] = unwrapped - prev;
        prev = unwrapped;
    }
    *prev_phase = prev;
    return n;
}

/* estimatePSD (src/fourier.cpp:35-117; model/fmSupportLib.py:83-157) restated accurately:
 * float Hann window sin(i pi / N)^2 (double, rounded to float, as fourier.cpp:59-61), float
 * windowed samples, DFT in double with exact twiddle angles 2 pi (k m mod N) / N,
 * 10 log10(4/(Fs N) |X|^2) per positive bin, float mean over segments in segment order. */
int orc_estimate_psd(const float* samples, size_t n, int freq_bins, float fs, float* freq, float* psd) {
    const int N = freq_bins, half = N / 2;
    const int nseg = (int)(n / (size_t)N);
    if (N < 2 || nseg < 1) return -1;
    const double pi = 3.14159265358979323846;
    const float df = fs / (float)N;
    for (int i = 0; i < half; i++) freq[i] = (float)i * df;
    float* hann = (float*)malloc(sizeof(float) * N);
    float* w = (float*)malloc(sizeof(float) * N);
    double* cs = (double*)malloc(sizeof(double) * N);
    double* sn = (double*)malloc(sizeof(double) * N);
    for (int i = 0; i < N; i++) {
        const double s = sin(i * pi / N);
        hann[i] = (float)(s * s);
        cs[i] = cos(2.0 * pi * i / N);
        sn[i] = -sin(2.0 * pi * i / N);
    }
    for (int k = 0; k < half; k++) psd[k] = 0.0f;
    float* seg = (float*)malloc(sizeof(float) * (size_t)half * nseg);
    for (int l = 0; l < nseg; l++) {
        for (int i = 0; i < N; i++) w[i] = samples[(size_t)l * N + i] * hann[i];
        for (int m = 0; m < half; m++) {
            double re = 0.0, im = 0.0;
            for (int k = 0; k < N; k++) {
                const int idx = (int)(((long long)k * m) % N);
                re += w[k] * cs[idx];
                im += w[k] * sn[idx];
            }
            seg[(size_t)l * half + m] = (float)(10.0 * log10(4.0 / ((double)fs * N) * (re * re + im * im)));
        }
    }
    for (int k = 0; k < half; k++) {
        float acc = 0.0f;
        for (int l = 0; l < nseg; l++) acc += seg[(size_t)l * half + k];
        psd[k] = acc / (float)nseg;
    }
    free(hann); free(w); free(cs); free(sn); free(seg);
    return nseg;
}
