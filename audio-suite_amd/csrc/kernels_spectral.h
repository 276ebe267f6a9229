// kernels_spectral.h — LDS-resident spectral chain per event (TU: k_spectral.hip).
#pragma once
#include "rt.h"

// ---------------------------------------------------------------------------
// Spectral chain, one workgroup per event, grain resident in LDS.
// ---------------------------------------------------------------------------
// lowpass_fft weight of bin k (MS:39-58), float64 thresholds exactly as rfftfreq.
MSG_DEV float lowpass_w(int k, int n, int sr, double cutoff, double roll) {
    const double nyq = 0.5 * (double)sr;
    const double c = fmin(fmax(cutoff, 1.0), nyq);
    const double r = fmax(0.0, roll);
    const double f = (double)k * (1.0 / ((double)n * (1.0 / (double)sr)));
    if (r <= 0) return f > c ? 0.f : 1.f;
    const double f1 = fmin(nyq, c + r);
    if (f > f1) return 0.f;
    if (f >= c) {
        const double t = (f - c) / fmax(1e-12, (f1 - c));
        return (float)(0.5 * (1.0 + cos(3.141592653589793 * t)));
    }
    return 1.f;
}

// Y[k] = interp(src(k), arange(K), X) for re/im, zero outside (np.interp, MS:112-127).
template <int T, int MAXK, class Src>
MSG_DEV void spectral_gather(float2* buf, int K, Src src) {
    constexpr int PER = (MAXK + T - 1) / T;
    const int tid = otid();
    float2 y[PER];
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int k = tid + b * T;
        y[b] = make_float2(0.f, 0.f);
        if (k < K) {
            const double xs = src(k);
            if (xs >= 0.0 && xs <= (double)(K - 1)) {
                const int j = (int)xs;
                if (j >= K - 1) {
                    y[b] = cx(buf, K - 1);
                } else {
                    const float fr = (float)(xs - (double)j);
                    const float2 a = cx(buf, j), c = cx(buf, j + 1);
                    y[b] = make_float2((c.x - a.x) * fr + a.x, (c.y - a.y) * fr + a.y);
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int k = tid + b * T;
        if (k < K) cx(buf, k) = y[b];
    }
    __syncthreads();
}

// irfft drops the imaginary part of the DC bin (and of the Nyquist bin for even n);
// reproduce that between fused spectral stages.
MSG_DEV void drop_edge_imag(float2* buf, const RealPlan& rp) {
    if (threadIdx.x == 0) {
        cx(buf, 0).y = 0.f;
        if (rp.even) cx(buf, rp.n / 2).y = 0.f;
    }
    __syncthreads();
}

template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_spectral(const msg_preset* __restrict__ presets, const msg_event* __restrict__ events,
           const EventRt* __restrict__ ert, const PresetRt* __restrict__ rt,
           const RealPlan* __restrict__ plans, const int32_t* __restrict__ ev_list, int n_list,
           float* __restrict__ micro_pool, float* __restrict__ grain_pool) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int li = blockIdx.x;
    if (li >= n_list) return;
    const int ei = ev_list[li];
    const msg_event& e = events[ei];
    const EventRt er = ert[ei];
    const PresetRt& r = rt[e.preset];
    const int n = e.n;
    float* micro = micro_pool + r.pool_base + e.pool_off;
    float* grain = grain_pool + r.pool_base + e.pool_off;
    const int ops = er.ops;
    if (ops == 0) {   // no spectral stage: grain = micro
        for (int j = threadIdx.x; j < n; j += T) grain[j] = micro[j];
        return;
    }
    const RealPlan& rp = plans[er.plan];
    const int K = n / 2 + 1;
    // the whole grain in flight at once (float4 loads from the 16-byte aligned preset pool)
    load_real_segment<T, (2 * MAXM + 4 * T - 1) / (4 * T)>(lds, rp, micro_pool + r.pool_base, e.pool_off + n,
                                                           e.pool_off, n, threadIdx.x);
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);   // includes the barrier

    // Transform sequence: [tilt F, tilt I] for noise/skew generators, then
    // [chain F, chain I] for the band-limit / warp / stretch chain.  One call
    // site of rtransform keeps one copy of the FFT engine in the kernel.
    const bool tilt = (ops & (SPEC_TILT_NOISE | SPEC_TILT_SKEW)) != 0;
    const bool chain = (ops & (SPEC_LOWPASS | SPEC_STRETCH | SPEC_WARP)) != 0;
    const int first = tilt ? 0 : 2;
    const int last = chain ? 4 : 2;
    for (int step = first; step < last; ++step) {
        const bool inv = (step & 1) != 0;
        const int tid = otid();
        rtransform<T, MAXM, RSET_ALL>(lds, rp, tw, inv);
        if (step == 0) {
            // tilted_noise (MS:224-233): W *= (f/f1)^alpha with f[0] := f[1]
            const double val = 1.0 / ((double)n * (1.0 / (double)er.gen_sr));
            for (int k = tid; k < K; k += T) {
                double sh = 1.0;
                if (K > 1 && k > 0) sh = pow(((double)k * val) / fmax(1e-12, val), er.tilt_alpha);
                cx(lds, k) = cscale(cx(lds, k), (float)sh);
            }
            __syncthreads();
        } else if (step == 1) {
            // envelope, skew, fade (MS:246-255, 265-268); the result is micro_last
            const int fade = (int)(0.01 * n) > 8 ? (int)(0.01 * n) : 8;
            const double inv_sr = 1.0 / (double)er.gen_sr;
            if (ops & SPEC_TILT_SKEW) {
                // d = diff(max(0, w), prepend=w[0]): needs neighbours -> via registers
                constexpr int PER = (2 * MAXM + T - 1) / T;
                float d[PER];
#pragma unroll
                for (int b = 0; b < PER; ++b) {
                    const int j = tid + b * T;
                    d[b] = 0.f;
                    if (j < n && j > 0) d[b] = fmaxf(0.f, rx_get(lds, rp, j)) - fmaxf(0.f, rx_get(lds, rp, j - 1));
                }
                __syncthreads();
#pragma unroll
                for (int b = 0; b < PER; ++b) {
                    const int j = tid + b * T;
                    if (j < n) {
                        const float env = (float)exp(-((double)j * inv_sr) / er.env_tau);
                        rx_set(lds, rp, j, d[b] * env * fade_w(j, n, fade));
                    }
                }
            } else {
                for (int j = tid; j < n; j += T) {
                    const float env = (float)exp(-((double)j * inv_sr) / er.env_tau);
                    rx_set(lds, rp, j, rx_get(lds, rp, j) * env * fade_w(j, n, fade));
                }
            }
            __syncthreads();
            for (int j = tid; j < n; j += T) micro[j] = rx_get(lds, rp, j);
        } else if (step == 2) {
            if (ops & SPEC_LOWPASS) {
                for (int k = tid; k < K; k += T)
                    cx(lds, k) = cscale(cx(lds, k), lowpass_w(k, n, er.gen_sr, er.cutoff_gen, er.roll));
                __syncthreads();
            }
            if (ops & SPEC_WARP) {   // fft_warp_power (MS:103-115)
                drop_edge_imag(lds, rp);
                const double kmax = fmax(1.0, (double)(K - 1));
                const double ip = 1.0 / fmax(1e-6, er.warp_power);
                spectral_gather<T, MAXM + 1>(lds, K, [&](int k) { return pow((double)k / kmax, ip) * kmax; });
            }
            if (ops & SPEC_STRETCH) {   // fft_partial_stretch (MS:117-128)
                drop_edge_imag(lds, rp);
                const double f = fmax(1e-12, er.stretch);
                spectral_gather<T, MAXM + 1>(lds, K, [&](int k) { return (double)k / f; });
            }
        }
    }
    for (int j = threadIdx.x; j < n; j += T) grain[j] = rx_get(lds, rp, j);
}
