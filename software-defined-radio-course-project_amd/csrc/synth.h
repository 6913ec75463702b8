// synth.h — deterministic synthetic FM-stereo u8 I/Q generator.
//
// Integer-only evaluation so the host and the GPU produce IDENTICAL bytes, and random
// access in the sample index so any slice of a stream can be generated independently
// (each GPU / workgroup generates its own part of a 1 GiB stream).
//
// Signal (per stream `seed`, sample n at rate rf_fs):
//   L = 0.5 sin(2 pi fL t), R = 0.5 sin(2 pi fR t)
//   m = 0.45 (L+R) + 0.1 cos(2 pi 19k t) + 0.45 (L-R) cos(2 pi 38k t)
//   phi(t) = 2 pi 75k * integral(m)  -- closed form: a sum of 7 tones, each term
//            a_k (75k / f_k) * {-cos | sin}(2 pi f_k t)
//   I,Q = cos(phi), sin(phi);  u8 = clamp(128 + round(100 x) + noise), noise ~ N(0, 2 LSB)
//   (sigma 0.02 of full scale), from a counter-based hash of (seed, n).
//
// Variants for the PLL's unlocked regimes, selected by the seed's top byte (seeds below 2^56 are
// the plain signal; the tones follow the low 56 bits): kSynthNoPilot drops the 19 kHz pilot (a
// mono broadcast: the reference PLL, filter.cpp:157-171, then never locks), and noise shift k
// (bits 57-59) scales the noise by 2^k (k = 3: sigma ~16 LSB against a carrier of 100).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fmrx {

constexpr int kSynthTones = 7;
constexpr int kSinBits = 14;  // 16384-entry Q15 sine table
constexpr int kSinSize = 1 << kSinBits;
constexpr uint64_t kSynthNoPilot = 1ull << 56;
constexpr int kSynthNoiseShiftBit = 57;  // 3 bits

struct SynthParams {
    uint64_t seed;
    int noise_shift;              // noise x 2^noise_shift (seed bits 57-59)
    int64_t amp[kSynthTones];     // phase amplitude in 2^-32-turn units, Q15-scaled table
    uint64_t inc[kSynthTones];    // phase increment per sample, 2^-32 turn units (64-bit)
    uint32_t off[kSynthTones];    // phase offset (0 for sin, -pi/2 for -cos)
};

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Approximately Gaussian integer noise, sigma ~ 2 LSB: sum of four bytes (var 21845) scaled.
__host__ __device__ inline int synth_noise(uint32_t r) {
    const int s = (int)(r & 0xFF) + (int)((r >> 8) & 0xFF) + (int)((r >> 16) & 0xFF) +
                  (int)(r >> 24) - 510;
    return (s * 887 + (1 << 15)) >> 16;  // arithmetic shift, rounds to nearest-ish
}

__host__ __device__ inline uint8_t synth_quant(int v_q15, int noise) {
    // 128 + round(100 * v / 32768) + noise, clamped to u8
    int x = 128 + ((100 * v_q15 + (1 << 14)) >> 15) + noise;
    x = x < 0 ? 0 : (x > 255 ? 255 : x);
    return (uint8_t)x;
}

// One I/Q pair of stream `p` at absolute sample index n.  `sintab` is the Q15 table.
__host__ __device__ inline void synth_pair(const SynthParams& p, const int16_t* sintab,
                                           uint64_t n, uint8_t* iq) {
    int64_t phase = 0;
#pragma unroll
    for (int k = 0; k < kSynthTones; k++) {
        const uint32_t ph = (uint32_t)(n * p.inc[k]) + p.off[k];
        phase += p.amp[k] * (int64_t)sintab[ph >> (32 - kSinBits)];
    }
    const uint32_t phi = (uint32_t)((uint64_t)phase >> 15);
    const int c = sintab[(uint32_t)(phi + 0x40000000u) >> (32 - kSinBits)];  // cos = sin(+pi/2)
    const int s = sintab[phi >> (32 - kSinBits)];
    const uint64_t h = splitmix64(p.seed * 0xD1B54A32D192ED03ull ^ n);
    iq[0] = synth_quant(c, synth_noise((uint32_t)h) * (1 << p.noise_shift));
    iq[1] = synth_quant(s, synth_noise((uint32_t)(h >> 32)) * (1 << p.noise_shift));
}

// Host-side parameter setup (double math, done once per stream).
void synth_setup(uint64_t seed, int rf_fs, SynthParams* p);
const int16_t* synth_sintab();  // host copy, kSinSize entries

}  // namespace fmrx
