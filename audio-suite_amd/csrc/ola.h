// ola.h — the overlap-add's per-frame pieces shared by k_ola_env (kernels_core.h,
// TU msgpu.hip) and k_fir8p's fused segment loads (fir8_fft.h, TU k_fir.hip):
// the ADSR envelope (make_adsr, MS:172-195) and the sorted-event search.
#pragma once
#include "rt.h"

// x^c for x in [0, 1] (hardware log2/exp2; exact at 0 and 1)
MSG_DEV float env_pow(float x, float c) { return x > 0.f ? exp2f(c * __log2f(x)) : 0.f; }

// make_adsr (MS:172-195) at frame t < n; region bounds and reciprocals precomputed on the host
MSG_DEV float adsr_at(const PresetRt& r, int t) {
    const float c = r.envC, S = r.envS;
    if (t < r.envA) return env_pow((float)t * r.envInvA, c);
    if (t < r.envJ) return 1.0f - (1.0f - S) * env_pow((float)(t - r.envA) * r.envInvD, c);
    if (t < r.envS1) return S;
    const int n = (int)r.out_n;
    const float u = (n - r.envS1 == 1) ? 0.f : (t == n - 1 ? 1.f : (float)(t - r.envS1) * r.envInvR);
    return S * (1.0f - env_pow(u, c));
}

// Number of events (sorted by start) with start <= lim: a 64-ary ballot search,
// one dependent load for up to 64 events instead of a log2 n binary search.
// Call from every lane of a wave.
MSG_DEV int events_starting_by(const msg_event* __restrict__ ev, int n, int64_t lim) {
    const int lane = (int)(threadIdx.x & 63);
    int lo = 0, len = n;
    while (len > 0) {
        const int step = (len + 63) >> 6;
        const int nseg = (len + step - 1) / step;
        const int last = min((lane + 1) * step, len) - 1;       // last element of this lane's segment
        const bool ok = lane < nseg && (int64_t)ev[lo + last].start <= lim;
        const int c = __popcll(__ballot(ok));                   // sorted: a prefix of the segments
        if (c == nseg) { lo += len; break; }
        lo += c * step;
        if (step == 1) break;
        len = min(step, len - c * step) - 1;                    // segment c ends above lim
    }
    return lo;
}

