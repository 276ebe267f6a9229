// kernels_spectral.h — LDS-resident spectral chain per event (TU: k_spectral.hip).
#pragma once
#include "rt.h"

// Phase timing (debug builds with -DMSG_STAMPS): block-summed clock64 deltas
// per phase, read back with msg_debug_stamps.
#ifdef MSG_STAMPS
__device__ unsigned long long g_spec_stamps[16];
#define SPEC_STAMP(i)                                                            \
    do {                                                                         \
        __syncthreads();                                                         \
        if (threadIdx.x == 0) {                                                  \
            const long long now_ = wall_clock64();                               \
            atomicAdd(&g_spec_stamps[i], (unsigned long long)(now_ - stamp_));   \
            stamp_ = now_;                                                       \
        }                                                                        \
    } while (0)
#define SPEC_STAMP_INIT long long stamp_ = wall_clock64()
#define SPEC_STAMP_RESET stamp_ = wall_clock64()
__device__ int g_spec_skip;   // debug: bit 0 skip lowpass, bit 1 skip gathers, bit 2 skip transforms
#define SPEC_SKIP(b) ((g_spec_skip >> (b)) & 1)
#else
#define SPEC_SKIP(b) 0
#define SPEC_STAMP(i) do {} while (0)
#define SPEC_STAMP_INIT do {} while (0)
#define SPEC_STAMP_RESET do {} while (0)
#endif

// ---------------------------------------------------------------------------
// Spectral chain, one workgroup per event, grain resident in LDS.
//
// The chain (MS:219-269 tilt/envelope, MS:39-128 band-limit / warp / stretch)
// is written once over an LDS layout policy L and a transform functor, and
// instantiated twice: the runtime-plan engine (fft_lds.h, XOR-swizzled
// layout) for any length, and compile-time plans for hot lengths
// (spec_ct.h, identity layout).
// ---------------------------------------------------------------------------
struct LaySwz { static MSG_DEV int c(int k) { return lp(k); } };
struct LayId { static MSG_DEV int c(int k) { return k; } };

template <class L> MSG_DEV float2& cxl(float2* b, int k) { return b[L::c(k)]; }
template <class L> MSG_DEV float rxl_get(const float2* b, bool even, int t) {
    return reinterpret_cast<const float*>(b)[even ? 2 * L::c(t >> 1) + (t & 1) : 2 * L::c(t)];
}
template <class L> MSG_DEV void rxl_set(float2* b, bool even, int t, float v) {
    if (even) reinterpret_cast<float*>(b)[2 * L::c(t >> 1) + (t & 1)] = v;
    else b[L::c(t)] = make_float2(v, 0.f);
}

// x[s0 + u] for u < N into the LDS real view, read as 16-byte aligned float4
// quads, Q4 quads in flight per thread per round (a whole 150 KB grain in one
// round trip at T = 512).  Loads are unconditional (clamped index) so no
// branch splits them: x + [floor4(s0), ceil4(s0 + N)) must lie inside the
// allocation (16-byte aligned regions padded to whole quads).
template <class L, int T, int Q4>
MSG_DEV void load_real_segment(float2* lds, bool evn, const float* __restrict__ x, int64_t s0, int N, int tid) {
    const int64_t a0 = (s0 >> 2) << 2;
    const int shift = (int)(s0 - a0);
    const int nq = (N + shift + 3) >> 2;
    const float4* xq = reinterpret_cast<const float4*>(x + a0);
    for (int v0 = 0; v0 < nq; v0 += Q4 * T) {
        float4 q[Q4];
#pragma unroll
        for (int i = 0; i < Q4; ++i) {
            const int v = v0 + i * T + tid;
            q[i] = xq[v < nq ? v : nq - 1];
        }
#pragma unroll
        for (int i = 0; i < Q4; ++i) {
            const int v = v0 + i * T + tid;
            if (v >= nq) continue;
            const int u = 4 * v - shift;
            const float e[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (u + c >= 0 && u + c < N) rxl_set<L>(lds, evn, u + c, e[c]);
        }
    }
}

// lowpass_fft weights (MS:39-58): float64 thresholds exactly as rfftfreq
// (f = k * (1 / (n * (1 / sr)))), per-event constants hoisted.
struct Lowpass {
    double val, c, r, f1, inv_band;
    MSG_DEV Lowpass(int n, int sr, double cutoff, double roll) {
        const double nyq = 0.5 * (double)sr;
        c = fmin(fmax(cutoff, 1.0), nyq);
        r = fmax(0.0, roll);
        val = 1.0 / ((double)n * (1.0 / (double)sr));
        f1 = fmin(nyq, c + r);
        inv_band = 1.0 / fmax(1e-12, (f1 - c));
    }
    MSG_DEV float w(int k) const {
        const double f = (double)k * val;
        if (r <= 0) return f > c ? 0.f : 1.f;
        if (f > f1) return 0.f;
        if (f >= c) return (float)(0.5 * (1.0 + cos(3.141592653589793 * ((f - c) * inv_band))));
        return 1.f;
    }
};

// Smallest k in [0, K] with k * val >= x / > x (k * val as rfftfreq builds it).
MSG_DEV int first_bin_at_least(double val, double x, int K) {
    double g = floor(x / val);
    int k = g < 0.0 ? 0 : (g > (double)K ? K : (int)g);
    while (k > 0 && (double)(k - 1) * val >= x) --k;
    while (k < K && (double)k * val < x) ++k;
    return k;
}
MSG_DEV int first_bin_above(double val, double x, int K) {
    double g = floor(x / val);
    int k = g < 0.0 ? 0 : (g > (double)K ? K : (int)g);
    while (k > 0 && (double)(k - 1) * val > x) --k;
    while (k < K && (double)k * val <= x) ++k;
    return k;
}

// Y[k] = interp(src(k), arange(K), X) for re/im, zero outside (np.interp, MS:112-127),
// in place.  Every source lies on one side of its bin (ascending: src(k) >= k,
// else src(k) <= k), so chunks of CH*T bins processed in that order -- read the
// chunk's sources, barrier, write the chunk, barrier -- never read a bin that
// was already overwritten.  Bins >= kz are zero (a band limit whose zeroing
// was deferred): they are never read, and a chunk whose first (smallest,
// src is increasing) source is >= kz is written as zeros without reading.
template <class L, int T, int CH, class Src>
MSG_DEV void spectral_gather(float2* buf, int K, bool ascending, Src src, int kz) {
    constexpr int C = CH * T;
    const int nch = (K + C - 1) / C;
    const int tid = otid();
    for (int c = 0; c < nch; ++c) {
        const int base = (ascending ? c : nch - 1 - c) * C;
        if (src(base) >= (double)kz) {             // chunk-uniform: all sources past the band
#pragma unroll
            for (int b = 0; b < CH; ++b) {
                const int k = base + tid + b * T;
                if (k < K) cxl<L>(buf, k) = make_float2(0.f, 0.f);
            }
            __syncthreads();
            continue;
        }
        float2 y[CH];
#pragma unroll
        for (int b = 0; b < CH; ++b) {
            const int k = base + tid + b * T;
            y[b] = make_float2(0.f, 0.f);
            if (k < K) {
                const double xs = src(k);
                if (xs >= 0.0 && xs <= (double)(K - 1) && xs < (double)kz) {
                    const int j = (int)xs;
                    if (j >= K - 1) {
                        y[b] = cxl<L>(buf, K - 1);
                    } else {
                        const float fr = (float)(xs - (double)j);
                        const float2 a = cxl<L>(buf, j);
                        const float2 e = j + 1 < kz ? cxl<L>(buf, j + 1) : make_float2(0.f, 0.f);
                        y[b] = make_float2((e.x - a.x) * fr + a.x, (e.y - a.y) * fr + a.y);
                    }
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < CH; ++b) {
            const int k = base + tid + b * T;
            if (k < K) cxl<L>(buf, k) = y[b];
        }
        __syncthreads();
    }
}

// irfft drops the imaginary part of the DC bin (and of the Nyquist bin for even n);
// reproduce that between fused spectral stages.
template <class L> MSG_DEV void drop_edge_imag(float2* buf, bool even, int n) {
    if (threadIdx.x == 0) {
        cxl<L>(buf, 0).y = 0.f;
        if (even) cxl<L>(buf, n / 2).y = 0.f;
    }
    __syncthreads();
}

// Transform sequence: [tilt F, tilt I] for noise/skew generators, then
// [chain F, chain I] for the band-limit / warp / stretch chain.  One call site
// of the transform keeps one copy of the FFT engine in the kernel.  Per-step
// constants are re-read through opaque pointers: computed before the step
// loop (LICM) they stay live across the FFT engine's register peak and spill.
template <class L, int T, class XF>
MSG_DEV void spectral_chain(float2* lds, bool evn, const EventRt* __restrict__ ert, int ei, int n,
                            float* micro, XF&& xf) {
    SPEC_STAMP_INIT;
    const int ops = ert[ei].ops;
    const bool tilt = (ops & (SPEC_TILT_NOISE | SPEC_TILT_SKEW)) != 0;
    const bool chain = (ops & (SPEC_LOWPASS | SPEC_STRETCH | SPEC_WARP)) != 0;
    const int first = tilt ? 0 : 2;
    const int last = chain ? 4 : 2;
    for (int step = first; step < last; ++step) {
        const bool inv = (step & 1) != 0;
        if (!SPEC_SKIP(2)) xf(inv);
        const int tid = otid();
        const EventRt& ex = *opaque_ptr(ert + ei);
        const int nn = opaque(n);
        const int KK = nn / 2 + 1;
        if (step == 0) {
            // tilted_noise (MS:224-233): W *= (f/f1)^alpha with f[0] := f[1]
            const double val = 1.0 / ((double)nn * (1.0 / (double)ex.gen_sr));
            const double ival = 1.0 / fmax(1e-12, val);
            const double alpha = ex.tilt_alpha;
            for (int k = tid; k < KK; k += T) {
                double sh = 1.0;
                if (KK > 1 && k > 0) sh = pow(((double)k * val) * ival, alpha);
                cxl<L>(lds, k) = cscale(cxl<L>(lds, k), (float)sh);
            }
            __syncthreads();
        } else if (step == 1) {
            // envelope, skew, fade (MS:246-255, 265-268); the result is micro_last
            const int fade = (int)(0.01 * nn) > 8 ? (int)(0.01 * nn) : 8;
            const double k_env = -(1.0 / (double)ex.gen_sr) / ex.env_tau;
            if (ex.ops & SPEC_TILT_SKEW) {
                // d = diff(max(0, w), prepend=w[0]) in place: d[j] reads w[j-1], w[j],
                // so chunks run top-down with read -> barrier -> write -> barrier
                constexpr int CH = 8, C = CH * T;
                const int nch = (nn + C - 1) / C;
                for (int c = nch - 1; c >= 0; --c) {
                    float d[CH];
#pragma unroll
                    for (int b = 0; b < CH; ++b) {
                        const int j = c * C + tid + b * T;
                        d[b] = 0.f;
                        if (j < nn && j > 0)
                            d[b] = fmaxf(0.f, rxl_get<L>(lds, evn, j)) - fmaxf(0.f, rxl_get<L>(lds, evn, j - 1));
                    }
                    __syncthreads();
#pragma unroll
                    for (int b = 0; b < CH; ++b) {
                        const int j = c * C + tid + b * T;
                        if (j < nn)
                            rxl_set<L>(lds, evn, j, d[b] * (float)exp((double)j * k_env) * fade_w(j, nn, fade));
                    }
                    __syncthreads();
                }
            } else {
                for (int j = tid; j < nn; j += T)
                    rxl_set<L>(lds, evn, j,
                               rxl_get<L>(lds, evn, j) * (float)exp((double)j * k_env) * fade_w(j, nn, fade));
                __syncthreads();
            }
            float* mo = opaque_ptr(micro);
            for (int j = tid; j < nn; j += T) mo[j] = rxl_get<L>(lds, evn, j);
        } else if (step == 2) {
            const int ops2 = ex.ops;
            int kz = KK;          // bins >= kz are zero, zeroing deferred to the next gather
            if ((ops2 & SPEC_LOWPASS) && !SPEC_SKIP(0)) {
                // lowpass_fft (MS:48-58): weight 1 below c, the cosine band [c, f1],
                // zero above (f1 = c without roll); f = k * val is increasing in k,
                // so the band and the zero range are index ranges
                const Lowpass lpw(nn, ex.gen_sr, ex.cutoff_gen, ex.roll);
                const double lim = lpw.r <= 0 ? lpw.c : lpw.f1;
                const int kb = first_bin_at_least(lpw.val, lpw.c, KK);          // f(kb) >= c
                kz = first_bin_above(lpw.val, lim, KK);                         // f(kz) > lim
                for (int k = kb + tid; k < kz; k += T) {
                    const float wk = lpw.w(k);
                    if (wk != 1.f) cxl<L>(lds, k) = cscale(cxl<L>(lds, k), wk);
                }
                if (!(ops2 & (SPEC_WARP | SPEC_STRETCH))) {
                    for (int k = kz + tid; k < KK; k += T) cxl<L>(lds, k) = make_float2(0.f, 0.f);
                    kz = KK;
                }
                __syncthreads();
            }
            if (ops2 & SPEC_WARP) {   // fft_warp_power (MS:103-115)
                drop_edge_imag<L>(lds, evn, nn);
                const double kmax = fmax(1.0, (double)(KK - 1));
                const double ikmax = 1.0 / kmax;
                const double ip = 1.0 / fmax(1e-6, ex.warp_power);
                spectral_gather<L, T, 8>(lds, KK, ip <= 1.0,
                                         [&](int k) { return pow((double)k * ikmax, ip) * kmax; }, kz);
                kz = KK;
            }
            if ((ops2 & SPEC_STRETCH) && !SPEC_SKIP(1)) {   // fft_partial_stretch (MS:117-128)
                drop_edge_imag<L>(lds, evn, nn);
                const double f = fmax(1e-12, ex.stretch);
                const double inv_f = 1.0 / f;
                spectral_gather<L, T, 8>(lds, KK, f < 1.0, [&](int k) { return (double)k * inv_f; }, kz);
            }
        }
        SPEC_STAMP(2 + step);
    }
}

// Runtime-plan kernel: any grain length (Bluestein for non-7-smooth lengths).
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_spectral(const msg_preset* __restrict__ presets, const msg_event* __restrict__ events,
           const EventRt* __restrict__ ert, const PresetRt* __restrict__ rt,
           const RealPlan* __restrict__ plans, const int32_t* __restrict__ ev_list, int n_list,
           float* __restrict__ micro_pool, float* __restrict__ grain_pool) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int li = blockIdx.x;
    if (li >= n_list) return;
    SPEC_STAMP_INIT;
    const int ei = ev_list[li];
    const msg_event& e = events[ei];
    const PresetRt& r = rt[e.preset];
    const int n = e.n;
    float* micro = micro_pool + r.pool_base + e.pool_off;
    float* grain = grain_pool + r.pool_base + e.pool_off;
    if (ert[ei].ops == 0) {   // no spectral stage: grain = micro
        for (int j = threadIdx.x; j < n; j += T) grain[j] = micro[j];
        return;
    }
    const RealPlan& rp = plans[ert[ei].plan];
    const bool evn = rp.even != 0;
    // the whole grain in flight at once (float4 loads from the 16-byte aligned preset pool)
    load_real_segment<LaySwz, T, (2 * MAXM + 4 * T - 1) / (4 * T)>(lds, evn, micro_pool + r.pool_base,
                                                                   e.pool_off, n, threadIdx.x);
    SPEC_STAMP(0);
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);   // includes the barrier
    SPEC_STAMP(1);
    spectral_chain<LaySwz, T>(lds, evn, ert, ei, n, micro,
                              [&](bool inv) { rtransform<T, MAXM, RSET_ALL>(lds, rp, tw, inv); });
    SPEC_STAMP_RESET;
    for (int j = threadIdx.x; j < n; j += T) grain[j] = rxl_get<LaySwz>(lds, evn, j);
    SPEC_STAMP(10);
}
