// spec_ct.h — compile-time FFT plans for hot grain lengths (TU: k_spectral_ct.hip).
//
// Grain lengths are fixed per design rate (n = round(gen_sr * micro_ms), MS:221),
// so a batch usually holds a handful of distinct n.  For the lengths of the
// benchmark configurations the real transform is instantiated with its radix
// sequence, butterfly counts and strides as constants: every LDS offset is an
// immediate, divisions by the pass stride are multiply-shifts, there is no
// radix switch, and the identity LDS layout is conflict-free for the strided
// Stockham stores because the first radix is odd.  The spectral chain itself
// (spectral_chain in kernels_spectral.h) is shared with the runtime-plan kernel.
#pragma once
#include <cmath>
#include <vector>
#include "kernels_spectral.h"

template <int M_, int T_, int... Rs>
struct SpecPlan {
    static constexpr int M = M_, T = T_;
    static constexpr int NP = sizeof...(Rs);
    static constexpr int RADS[NP] = {Rs...};
    static constexpr int rad(int p) { return RADS[p]; }
    static constexpr int ns(int p) { return p == 0 ? 1 : ns(p - 1) * rad(p - 1); }
    static_assert((Rs * ...) == M_, "radix product");
    static_assert(RADS[0] % 2 == 1, "odd first radix: conflict-free identity layout");
    // twiddles, at LDS offset 0: w_M two-level (x = hi*128 + lo), post w_2M two-level
    static constexpr int HI_M = (M + 127) / 128;
    static constexpr int HI_P = (M / 2) / 128 + 2;
    static constexpr int OFF_MLO = 0, OFF_MHI = 128, OFF_PLO = 128 + HI_M, OFF_PHI = OFF_PLO + 128;
    static constexpr int TAB_USED = OFF_PHI + HI_P;
    static constexpr int TAB = (TAB_USED + 15) & ~15;
    static constexpr int BUF = M + 16;             // M complex + bin M of the half spectrum
    static constexpr int LDS_BYTES = (TAB + BUF) * 8;
    static constexpr int Q4 = (2 * M + 4 * T - 1) / (4 * T);   // float4 loads per thread
    static_assert(LDS_BYTES <= 163840, "LDS budget");
};

template <class P> MSG_DEV float2 ct_wM(const float2* tab, int x) {   // exp(-2 pi i x / M)
    return cmul(tab[P::OFF_MHI + (x >> 7)], tab[P::OFF_MLO + (x & 127)]);
}
template <class P> MSG_DEV float2 ct_w2M(const float2* tab, int x) {  // exp(-2 pi i x / 2M)
    return cmul(tab[P::OFF_PHI + (x >> 7)], tab[P::OFF_PLO + (x & 127)]);
}

// Stockham pass p, in place: all loads, barrier, twiddle w_{NS R}^{k r} (power
// tree from one table value) + DFT_R, stores, barrier.
template <class P, int p>
MSG_DEV void ct_pass(float2* buf, const float2* tab) {
    constexpr int M = P::M, T = P::T, R = P::rad(p), NS = P::ns(p), NB = M / R;
    constexpr int BP = (NB + T - 1) / T;
    constexpr int TWS = M / (NS * R);              // w_{NS R} = w_M^TWS
    const int t = otid();
    float2 v[BP][R];
#pragma unroll
    for (int b = 0; b < BP; ++b) {
        const int j = t + b * T;
        if (NB % T == 0 || j < NB) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = buf[j + r * NB];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BP; ++b) {
        const int j = t + b * T;
        if (NB % T == 0 || j < NB) {
            const int k = j % NS, q = j / NS;
            if (NS > 1) {
                constexpr int B = tw_base<R>();          // k TWS B < M: B <= R, k < NS
                twiddle_pow_ab<R, B>(v[b], ct_wM<P>(tab, k * TWS), ct_wM<P>(tab, k * TWS * B));
            }
            Dft<R, false>::run(v[b]);
#pragma unroll
            for (int r = 0; r < R; ++r) buf[q * NS * R + k + r * NS] = v[b][r];
        }
    }
    __syncthreads();
}

template <class P, int p = 0> MSG_DEV void ct_fft(float2* buf, const float2* tab) {
    ct_pass<P, p>(buf, tab);
    if constexpr (p + 1 < P::NP) ct_fft<P, p + 1>(buf, tab);
}

// Real transform of n = 2M samples in place (identity layout), same contract
// as rtransform (fft_lds.h): forward rfft, or irfft with numpy normalisation
// ignoring the imaginary parts of bins 0 and M; the inverse runs the forward
// engine on the conjugated packed spectrum.
template <class P>
MSG_DEV void ct_rtransform(float2* buf, const float2* tab, bool inverse) {
    constexpr int M = P::M, T = P::T;
    const int tid = otid();
    if (inverse) {
        for (int k = tid; k <= M / 2; k += T) {
            if (k == 0) {
                const float y0 = buf[0].x, ym = buf[M].x;
                buf[0] = make_float2(0.5f * (y0 + ym), -0.5f * (y0 - ym));
                continue;
            }
            const float2 yk = buf[k], ym = buf[M - k];
            const float2 w = ct_w2M<P>(tab, k);
            const float2 e1 = cscale(cadd(yk, cconj(ym)), 0.5f);
            const float2 o1 = cscale(cmulc(csub(yk, cconj(ym)), w), 0.5f);
            buf[k] = make_float2(e1.x - o1.y, -(e1.y + o1.x));
            buf[M - k] = make_float2(e1.x + o1.y, e1.y - o1.x);     // conj Z'[M-k]
        }
        __syncthreads();
    }
    ct_fft<P>(buf, tab);
    if (!inverse) {
        for (int k = tid; k <= M / 2; k += T) {
            if (k == 0) {
                const float2 z0 = buf[0];
                buf[0] = make_float2(z0.x + z0.y, 0.f);
                buf[M] = make_float2(z0.x - z0.y, 0.f);
                continue;
            }
            const float2 zk = buf[k], zm = buf[M - k];
            const float2 w = ct_w2M<P>(tab, k);
            const float2 e = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
            const float2 d = make_float2(zk.x - zm.x, zk.y + zm.y);
            const float2 wo = cmul(w, make_float2(0.5f * d.y, -0.5f * d.x));
            buf[k] = cadd(e, wo);
            buf[M - k] = make_float2(e.x - wo.x, wo.y - e.y);       // conj(e - w o)
        }
        __syncthreads();
    } else {
        const float s = 1.0f / (float)M;
        for (int j = tid; j < M; j += T) { const float2 z = buf[j]; buf[j] = make_float2(z.x * s, -z.y * s); }
        __syncthreads();
    }
}

template <class P>
__global__ void __launch_bounds__(P::T)
k_spectral_ct(const msg_event* __restrict__ events, const EventRt* __restrict__ ert,
              const PresetRt* __restrict__ rt, const float2* __restrict__ tables,
              const int32_t* __restrict__ ev_list, int n_list,
              float* __restrict__ micro_pool, float* __restrict__ grain_pool) {
    constexpr int T = P::T;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + P::TAB;
    const int li = blockIdx.x;
    if (li >= n_list) return;
    SPEC_STAMP_INIT;
    const int ei = ev_list[li];
    const msg_event& e = events[ei];
    const PresetRt& r = rt[e.preset];
    const int n = 2 * P::M;
    float* micro = micro_pool + r.pool_base + e.pool_off;
    float* grain = grain_pool + r.pool_base + e.pool_off;
    { TabCopy<P::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }   // one memory latency, not one per T entries
    load_real_segment<LayId, T, P::Q4>(buf, true, micro_pool + r.pool_base, e.pool_off, n, threadIdx.x);
    __syncthreads();
    SPEC_STAMP(0);
    spectral_chain<LayId, T>(buf, true, ert, ei, n, micro, [&](bool inv) { ct_rtransform<P>(buf, tab, inv); });
    SPEC_STAMP_RESET;
    // grain out: packed pairs, 8-byte stores when the grain is 8-byte aligned
    if ((((uintptr_t)grain) & 7) == 0) {
        float2* g2 = reinterpret_cast<float2*>(grain);
        for (int j = threadIdx.x; j < P::M; j += T) g2[j] = buf[j];
    } else {
        for (int j = threadIdx.x; j < n; j += T) grain[j] = rxl_get<LayId>(buf, true, j);
    }
    SPEC_STAMP(10);
}

// Host: the plan's twiddle tables (float64-built, rounded once).
template <class P>
inline void spec_ct_tables(std::vector<float>& out) {
    out.assign(2 * (size_t)P::TAB_USED, 0.f);
    const long double PI = 3.14159265358979323846264338327950288L;
    auto put = [&](int at, long double num, long double den) {
        const long double a = -2.0L * PI * num / den;
        out[2 * at] = (float)cosl(a);
        out[2 * at + 1] = (float)sinl(a);
    };
    for (int x = 0; x < 128; ++x) put(P::OFF_MLO + x, x, P::M);
    for (int x = 0; x < P::HI_M; ++x) put(P::OFF_MHI + x, 128.0L * x, P::M);
    for (int x = 0; x < 128; ++x) put(P::OFF_PLO + x, x, 2.0L * P::M);
    for (int x = 0; x < P::HI_P; ++x) put(P::OFF_PHI + x, 128.0L * x, 2.0L * P::M);
}

// The hot lengths: C3/C4 (37500), C5 reading B (30000), C2 (2400), C5 reading A
// (1920), the factory default (1500) and H48 (480: 384 kHz x 1.25 ms).
using SpecP18750 = SpecPlan<18750, 768, 25, 5, 5, 5, 6>;
using SpecP15000 = SpecPlan<15000, 640, 25, 5, 5, 6, 4>;
using SpecP1200 = SpecPlan<1200, 64, 25, 6, 8>;
using SpecP960 = SpecPlan<960, 64, 15, 8, 8>;
using SpecP750 = SpecPlan<750, 64, 25, 5, 6>;
using SpecP240 = SpecPlan<240, 64, 5, 6, 8>;
