// pll_device.h — device pieces of the stereo pilot PLL (src/filter.cpp:136-174) shared by
// stereo.hip (the runners, check and resume kernels) and pll_sat.hip (the saturated-segment
// runner, built as its own translation unit: see the Makefile).
#pragma once
#include <hip/hip_runtime.h>

#include <utility>

#include "pll_cr.h"
#include "pll_math.h"

namespace fmrx {
namespace {

// src/filter.cpp:136-174 PLL.  A nonlinear recurrence: strictly serial in time, so one lane
// per stream.  Float state; the reference's double atan2 / cos / sin results rounded to
// float come from pll_math.h's certified fast path (fallback: the full library call).
// st = {integrator, phaseEst, feedbackI, feedbackQ, ncoOut_state, trigOffset} (stride 8).
//
// The recurrence only needs atan2 and sincos; the NCO output cos(trigArg * ncoScale +
// phaseAdjust) (filter.cpp:170) depends on nothing later, so the serial loop stores trigArg
// in place and pll_nco_kernel evaluates the NCO for all samples in parallel afterwards.
// Fallbacks where a certified fast path refuses (~1e-6 of steps), out of line: pll_cr.h's
// double-double evaluation rounded like glibc (float of the correctly rounded double), pinned to
// glibc on every refusable sincos argument of the PLL's domain (tools/check_pll_cr.cpp,
// tests/golden/pll_fallback.npz).  HIP's double sin/cos only beyond |x| >= 2^31, a trigArg no
// PLL state reaches (|trigArg| < 1e9 wherever the step's product is finite).
__device__ __noinline__ float atan2_lib(float y, float x) {
    float e;
    if (fast_atan2_f(y, x, &e)) return e;
    return cr::atan2_f(y, x);
}
__device__ __noinline__ float2 sincos_lib(float a) {
    if (!cr::sincos_domain(a))
        return make_float2(static_cast<float>(sin(static_cast<double>(a))),
                           static_cast<float>(cos(static_cast<double>(a))));
    float sv, cv;
    cr::sincos_f(a, &sv, &cv);
    return make_float2(sv, cv);
}

struct DeviceLib {
    __device__ float atan2f_(float y, float x) const { return atan2_lib(y, x); }
    __device__ void sincosf_(float a, float* s, float* c) const {
        const float2 r = sincos_lib(a);
        *s = r.x;
        *c = r.y;
    }
};

// n exact steps (pll_step with the library fallbacks), out of line: the kernel then holds no
// calls, so the batch loop's registers are not saved and restored around them.
struct PllPair {
    PllState p;
    PllCtx ctx;
};
// `wr` false: compute only.  Lanes of the grid's padding waves (s_lane >= n_streams) recompute
// the last stream but do not run in lockstep with its own wave, which in the plain launch
// overwrites the input in place: they must not write what they derived from it.
__device__ __noinline__ PllPair pll_redo(PllState p, PllCtx ctx, const float* xb, float* ob, int n, float Ki,
                                         float Kp, double step, bool wr) {
    const DeviceLib lib;
#pragma unroll 1
    for (int j = 0; j < n; j++) {
        const float a = pll_step(p, ctx, xb[j], Ki, Kp, step, lib);
        if (wr) ob[j] = a;
    }
    return PllPair{p, ctx};
}

// NB samples per optimistic batch.  Measured (10 s mode-0 stereo): NB = 16 beats 8 and 12.  The
// certification is ~23 % of the step: without it the loop runs 0.31 s instead of 0.40 s.
constexpr int kPllBatch = 16;

// Demotion of a self-certifying runner's stream (pll_pred.hip): the chain keeps the verdicts of
// its last 32 intervals as bits; past kPllDemoteMisses misses among them the trigArgs are not
// where the candidates are predicted (an unlocked loop: no pilot, noise, mode 2/3's if_fs, whose
// phase moves many candidate cells an interval) and the runner leaves the rest of its range to
// pll_demoted_kernel (pll_demote.hip: a speculative chain checked behind it, ~lane-runner speed)
// instead of paying a failed interval plus its redo each time.  Locked streams miss <= ~1 % of
// intervals (profiles/r05 redos); unlocked ones 75-100 % (profiles/r06/unlocked.json).
constexpr int kPllDemoteMisses = 24;
// the index forms ([2^17, 2^20), 16-step intervals, the tightest candidate windows) want 28: there
// locked streams miss in bursts -- at 24, 20 of configs[4]'s 256 synth streams demoted and their
// demoted steps ran after the runner launch (0.4206 vs 0.4098 s at 28, none demoted at 28 or 32;
// profiles/r06/demote_probe/); the unlocked streams still demote within their first ~30 intervals
constexpr int kPllDemoteMissesIdx = 28;
// only a runner launch of at least this many intervals demotes (launch_pll queues the demoted kernel
// after exactly those: a shorter range cannot pay for it, e.g. the per-block seam's 640 steps)
constexpr int kPllDemoteMinIntervals = 64;
// test hook (knob pll_pipe_miss = m): m >= 1 a forced miss on interval m (past the last: the last),
// m <= -2 on every interval from -m - 1 on (an unlocked loop's pattern: the demotion runs), -1 off
__device__ inline bool pll_hook_miss(int i, int miss, int ni) {
    return miss >= 1 ? i == min(miss, ni) : (miss <= -2 && i >= -miss - 1);
}
__device__ inline bool pll_demote(uint32_t& hist, bool miss) {
    hist = (hist << 1) | (miss ? 1u : 0u);
    return __builtin_popcount(hist) >= kPllDemoteMisses;
}

template <int L>
__device__ inline double row_bcast(double v) {
    const long long bits = __builtin_bit_cast(long long, v);
    return __builtin_bit_cast(double, (long long)__builtin_amdgcn_mov_dpp(bits, 0x150 + L, 0xF, 0xF, false));
}

// f(integral_constant<int, 0>), ..., f(integral_constant<int, N - 1>): a loop whose index is a
// compile-time constant in the body (row_bcast's lane)
template <class F, int... J>
__device__ inline void unroll_ic(F&& f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}

// A segment for pll_sat_kernel: one stream a wave and trigOffset stuck at 2^24 from its start
// (filter.cpp:165-166: trigOffset + 1.0f == trigOffset from there, 69.9 s into a stream at
// 240 kS/s), so every step's pr is the constant step 2^24 (pll_side).  pll_spec_lane_kernel
// leaves exactly these streams to it.
__device__ inline bool pll_sat_segment(int spw, float trig0, double step) {
    return spw == 1 && trig0 == kPllTrigStick && fabs(step * (double)kPllTrigStick) < kPllMaxPr;
}

// A stream for pll_pred_kernel: trigOffset in [2^20, 2^24] at the segment start (integer-valued,
// as pll_side needs), where the predicted trigArgs almost always hit (pll_pred.hip).  The wave
// takes the predicted runner only if every stream of it qualifies (ballot: all lanes alike), and
// pll_spec_lane_kernel makes the same test to leave exactly those waves to it; saturated waves go
// to pll_sat_kernel first when it is launched.
constexpr float kPllPredMin = 1048576.0f;  // 2^20
__device__ inline bool pll_pred_wave(float trig0, double step) {
    const bool ok = trig0 >= kPllPredMin && trig0 <= kPllTrigStick && trig0 == floorf(trig0) &&
                    fabs(step * (double)kPllTrigStick) < kPllMaxPr;
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// A stream for pll_pipe_kernel (one stream a workgroup, spw == 1): trigOffset in [2^20, 2^24] at
// the segment start, where the predicted trigArgs of the bench stream hit their candidates
// (tools/pll_predict.cpp): three candidates in 64-step intervals from 2^22 (every interval), five
// in 64-step intervals in [2^21, 2^22) (99.97 %), five in 16-step intervals in [2^20, 2^21)
// (99.7 %; a miss costs an exact redo).  pll_pred_kernel and pll_sat_kernel leave these streams
// to it when it is launched.
constexpr float kPllPipeMin = 4194304.0f;     // 2^22
constexpr float kPllPipeMin5 = 2097152.0f;    // 2^21
constexpr float kPllPipeMinLow = 1048576.0f;  // 2^20
__device__ inline bool pll_pipe_stream(float trig0, double step, float lo = kPllPipeMinLow,
                                       float hi = kPllTrigStick) {
    return trig0 >= lo && trig0 <= hi && trig0 == floorf(trig0) && fabs(step * (double)kPllTrigStick) < kPllMaxPr;
}

// the fmrx_debug_pll_redos slot of a runner launch whose range starts at trigOffset t0
// (fmrx_internal.h kPllRedoSlots)
__device__ inline int pll_redo_range(float t0) {
    return t0 < kPllPipeMinLow ? 0 : t0 < kPllPipeMin5 ? 1 : t0 < kPllPipeMin ? 2 : 3;
}

}  // namespace
}  // namespace fmrx
