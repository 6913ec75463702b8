// mono_launch.h — the fused mono kernel's launch interface (mono_fused.hip): its argument
// structs and host entry points.  Its own header so that the kernel's sources -- this file,
// mono_fused.hip and dsp_device.h, which bench.py hashes to stamp the PMC traffic record
// (profiles/traffic_mono101.json) -- change only when the kernel does.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace fmrx {

constexpr int kMaxRfTaps = 256;

constexpr int kMaxAudioTaps = 64;
constexpr int kAudioRow = 52;   // one polyphase phase of the 51-taps-per-phase audio prototype, 16-B rows

// Coefficient tables handed to kernels by value (kernarg segment -> scalar registers).
struct MonoTaps {
    float rf[kMaxRfTaps];
    float audio[kMaxAudioTaps];
};

// ---- fused mono receiver (a1 a4 a5 a6 a12; MONO semantics) ---------------------------
struct MonoLaunch {
    const uint8_t* iq;          // n_streams x stream_bytes
    const uint8_t* halo;        // n_streams x halo_bytes: bytes preceding this call
    int16_t* pcm;               // n_streams x n_blocks*audio_frames
    float* mono;                // optional float output (same shape), may be null
    float* demod;               // optional demod output, written at demod[s*demod_stride +
                                //   demod_hist + g] for IF index g (stereo engine input)
    size_t demod_stride;
    int demod_hist;
    float* demod_tail;          // optional: the last AH demod samples, at demod_tail +
                                //   s * demod_tail_stride for stream s
    size_t demod_tail_stride;
    const float* audio_coeff;   // modes 2/3: the rational resampler's prototype (device)
    const float* audio_rows;    // modes 2/3: the same taps as `up` rows of kAudioRow floats,
                                //   row k0 = coeff[k0 + i up] for i < 51 (then zeros)
    size_t stream_bytes;        // n_blocks * block_bytes
    size_t halo_bytes;
    long long n_if;             // IF samples per stream this call
    int segs;                   // workgroups (segments) per stream
    int audio;                  // 1: run the audio stage (pcm / mono outputs)
    unsigned long long* stamps; // diagnostic (fmrx_debug_mono_stamps): 6 u64 per workgroup, else null
    int older_share;            // 0: equal segments; else (even segs, two waves per SIMD) the
                                //   first-dispatched wave's share of a SIMD's span, in 1/1024
    uint8_t* halo_next;         // optional: the halo after this call (last halo_bytes of halo ++
                                //   iq per stream), written by the kernel in 16-B words; the
                                //   caller guarantees 16-B aligned iq rows (else null + halo_kernel)
    size_t iq_stride;           // bytes between streams in iq (stream_bytes, or the whole call's
                                //   when this launch is a chunk of a longer call)
    size_t halo_stride;         // bytes between streams in halo (halo_bytes, or iq_stride when the
                                //   halo is the call's own bytes in front of the chunk)
};

// Halo bytes the fused kernel needs in front of a call (pre-roll chunk + RF history).
size_t mono_halo_bytes(int rf_taps, int rf_decim, int audio_down);
// Chunks (work units) per stream for n_if IF samples, used to size the grid.
long long mono_chunks(long long n_if, int rf_taps, int rf_decim, int audio_down);
// Resident workgroups per CU of the selected variant (grid sizing).
int mono_wg_per_cu(int rf_decim);
// Returns 0 on success, FMRX_EINVAL if no compiled variant matches.
int launch_mono_fused(const MonoLaunch& L, int n_streams, int rf_taps, int rf_decim,
                      int audio_up, int audio_down, const MonoTaps& taps, hipStream_t s);

}  // namespace fmrx
