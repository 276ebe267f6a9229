// kernels.h — gfx950 kernels of the Microsound render path.
//
//   k_plan_sizes / k_plan_events   per-preset planner (one thread per preset)      MS:589-646, 409-417
//   k_gen_normal                   grain generator, one wave per event              MS:219-269
//   k_spectral<T>                  LDS-resident spectral chain, one WG per event    MS:39-128, 224-233, 690-702
//   k_ola_env                      grain overlap-add x ADSR, one WG per tile        MS:742-764
//   k_fir_h                        (delta + ER) * IR kernel spectra per partition   MS:409-445
//   k_fir                          partitioned FFT overlap-save FIR                 MS:766-773
//   k_stereo_max / k_stereo_out    25-tap Bessel stereo, tanh, peak normalise       MS:423-436, 775-781
#pragma once
#include "msg_common.h"
#include "nprng.h"
#include "plan.h"
#include "fft_lds.h"

// Per-preset runtime record, built on the host after planning.
struct PresetRt {
    int64_t out_n;
    int64_t out_off;       // first output frame of this preset
    int64_t pool_base;     // grain pool offset (floats)
    int64_t y_off;         // mono buffers offset (floats)
    int32_t ev_begin;      // first event slot
    int32_t n_events;
    int32_t er_base;       // first ER tap
    int32_t n_taps;        // ER taps (0 when ER off)
    int32_t tile_begin;    // first overlap-add tile
    int32_t max_n;
    // ADSR (MS:172-195), in samples
    int32_t envA, envD, envR;
    float envS, envC;
    // FIR (combined ER + IR), 0 = identity
    int32_t fir_on, fir_N, fir_P, fir_Q, fir_B;
    int32_t fir_block_begin;
    int32_t h_block_begin;
    int32_t ir_len;        // taps of the IR (0 -> delta)
    int64_t ir_off;        // offset of the IR in the device IR bank (float64)
    int64_t h_off;         // offset of the Q partition spectra (float2)
    // stereo / saturation / normalisation
    int32_t stereo_fir;    // 1: 25-tap Bessel FIR, 0: L = R = y
    int32_t dl, dr;
    float bess[25];        // J_m(0.9 w), m = -12..12
    float drive, peak;
    int32_t pad2;
};

// Per-event spectral work descriptor (host-built after planning).
struct EventRt {
    int32_t plan;          // RealPlan index for n
    int32_t ops;           // bit mask of SPEC_* below
    int32_t n, gen_sr;
    double cutoff_gen, roll;
    double stretch;
    double tilt_alpha;     // log2 of the per-octave gain (MS:229-230)
    double env_tau;        // noise/skewed envelope time constant (s)
    double warp_power;     // fft_warp_power exponent (MS:103-115)
};
enum : int32_t {
    SPEC_TILT_NOISE = 1, SPEC_TILT_SKEW = 2, SPEC_LOWPASS = 4, SPEC_STRETCH = 8, SPEC_WARP = 16,
};

constexpr int GEN_T = 64;          // one wave per event
constexpr int OLA_T = 256;
constexpr int OLA_TILE = 2048;
constexpr int ST_T = 256;
constexpr int ST_TILE = 4096;

// ---------------------------------------------------------------------------
// Planner (one thread per preset).
// ---------------------------------------------------------------------------
__global__ void k_plan_sizes(const msg_preset* __restrict__ presets, int n_presets,
                             const int64_t* __restrict__ frag_len, nprng::Zig z,
                             msg_plan_info* __restrict__ info) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_presets) return;
    msg_plan_info inf;
    msgplan::plan_sizes(presets[p], z, frag_len[p], inf);
    info[p] = inf;
}

__global__ void k_plan_events(const msg_preset* __restrict__ presets, int n_presets,
                              const int64_t* __restrict__ frag_len, nprng::Zig z,
                              const int32_t* __restrict__ slot_base, const int32_t* __restrict__ tap_base,
                              msg_event* __restrict__ events, int32_t* __restrict__ er_off,
                              double* __restrict__ er_gain, msg_plan_info* __restrict__ info) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_presets) return;
    msg_plan_info inf;
    const msg_preset& pr = presets[p];
    const bool er = (pr.flags & MSG_F_ER_CLOUD) != 0;
    msgplan::plan_events(pr, z, frag_len[p], p, inf, events + slot_base[p],
                         er ? er_off + tap_base[p] : nullptr, er ? er_gain + tap_base[p] : nullptr);
    info[p] = inf;
}

// ---------------------------------------------------------------------------
// Generators driven by standard_normal(n): parallel ziggurat walk.
//
// The stream of raw PCG64 draws is consumed 64 at a time: lane l holds the
// state of draw base+l (jump-ahead), classifies it as a fast ziggurat accept,
// and a wave ballot locates the rare draws that start a slow (rejection)
// normal.  That lane finishes the slow normal sequentially from its own
// state and reports how many draws it consumed, which moves the parse
// position.  The emitted sequence is exactly NumPy's standard_normal(n).
// ---------------------------------------------------------------------------
struct JumpTab { nprng::u128 a[GEN_T]; nprng::u128 s[GEN_T]; nprng::u128 a64, s64; };

MSG_DEV double slow_normal(nprng::u128 st, nprng::u128 inc, uint64_t rabs, int idx, double x,
                           const nprng::Zig& z, int& consumed) {
    nprng::Pcg64 g;
    g.state = st; g.inc = inc; g.has_u32 = 0; g.u32 = 0;
    int c = 1;
    for (;;) {
        if (idx == 0) {
            for (;;) {
                const double xx = -nprng::ZIG_NOR_INV_R * log1p(-nprng::next_double(g));
                const double yy = -log1p(-nprng::next_double(g));
                c += 2;
                if (yy + yy > xx * xx) {
                    consumed = c;
                    return ((rabs >> 8) & 1) ? -(nprng::ZIG_NOR_R + xx) : nprng::ZIG_NOR_R + xx;
                }
            }
        }
        const double u = nprng::next_double(g);
        c += 1;
        if (((z.fi[idx - 1] - z.fi[idx]) * u + z.fi[idx]) < exp(-0.5 * x * x)) { consumed = c; return x; }
        uint64_t r = nprng::next_u64(g);
        c += 1;
        idx = (int)(r & 0xff);
        r >>= 8;
        const int sign = (int)(r & 1);
        rabs = (r >> 1) & 0x000fffffffffffffULL;
        x = (double)rabs * z.wi[idx];
        if (sign) x = -x;
        if (rabs < z.ki[idx]) { consumed = c; return x; }
    }
}

// Closed-form part of gen_basic for sample j given its normal N_j (MS:235-268).
struct GenBasicConst {
    int mode;            // MSG_GEN_*
    int n, fade;
    double inv_sr;
    double f_ring, inv_tau, inv_tau_exc;   // resonant
    double inv_sigma;                       // gaussian
};
MSG_DEV float fade_w(int j, int n, int fade) {
    double w = 1.0;
    if (j < fade) w *= (double)j * (1.0 / (double)fade);
    if (j >= n - fade) w *= (double)(j - (n - fade)) * (-1.0 / (double)fade) + 1.0;
    return (float)w;
}
MSG_DEV float gen_basic_sample(const GenBasicConst& c, int j, double nrm) {
    float x;
    if (c.mode == MSG_GEN_RESONANT) {
        const double t = (double)j * c.inv_sr;
        const double cyc = c.f_ring * t;                      // sin(2 pi f t), reduced in float64
        const float ph = (float)(cyc - floor(cyc));
        const float ring = sinpif(2.0f * ph) * expf((float)(-t * c.inv_tau));
        const float exc = (float)nrm * expf((float)(-t * c.inv_tau_exc));
        x = 0.9f * ring + 0.25f * exc;
    } else if (c.mode == MSG_GEN_GAUSSIAN_CLICK) {
        const double u = (double)j * c.inv_sigma;
        x = (float)(exp(-0.5 * (u * u)) * (nrm * 0.12 + 1.0));
    } else if (c.mode == MSG_GEN_NOISE_BURST || c.mode == MSG_GEN_SKEWED) {
        return (float)nrm;                                    // raw normals; tilt/env in k_spectral
    } else {
        x = (float)(nrm * 0.1);                               // fallback (MS:263)
    }
    return x * fade_w(j, c.n, c.fade);
}

__global__ void __launch_bounds__(GEN_T)
k_gen_normal(const msg_preset* __restrict__ presets, const msg_event* __restrict__ events,
             const PresetRt* __restrict__ rt, const int32_t* __restrict__ ev_list, int n_list,
             nprng::Zig z, const JumpTab* __restrict__ jt, float* __restrict__ pool) {
    const int li = blockIdx.x;
    if (li >= n_list) return;
    const msg_event& e = events[ev_list[li]];
    const msg_preset& pr = presets[e.preset];
    const PresetRt& r = rt[e.preset];
    const int lane = threadIdx.x;
    const int n = e.n;
    float* out = pool + r.pool_base + e.pool_off;

    GenBasicConst c;
    c.mode = pr.gen_mode == MSG_GEN_FALLBACK ? MSG_GEN_NOISE_BURST : pr.gen_mode;   // MS:686
    c.n = n;
    c.fade = (int)(0.01 * n) > 8 ? (int)(0.01 * n) : 8;
    c.inv_sr = 1.0 / (double)e.gen_sr;
    c.f_ring = fmax(10.0, pr.ring_hz);
    c.inv_tau = 1.0 / fmax(1e-6, pr.ring_decay_ms / 1000.0);
    c.inv_tau_exc = 1.0 / fmax(1e-6, (pr.micro_ms / 1000.0) * 0.15);
    const int sigma = (int)(0.0025 * n) > 1 ? (int)(0.0025 * n) : 1;
    c.inv_sigma = 1.0 / (double)sigma;

    // default_rng(seed + i): every lane computes the (uniform) seed state.
    const nprng::Pcg64 g0 = nprng::default_rng((uint64_t)(pr.seed + e.index));
    const nprng::u128 inc = g0.inc;
    const nprng::u128 c64 = inc * jt->s64;
    nprng::u128 st = jt->a[lane] * g0.state + inc * jt->s[lane];   // state after lane+1 steps

    int produced = 0;
    int local = 0;   // parse position within the current chunk
    while (produced < n) {
        const uint64_t raw = nprng::xsl_rr(st);
        const int idx = (int)(raw & 0xff);
        const uint64_t rr = raw >> 8;
        const uint64_t rabs = (rr >> 1) & 0x000fffffffffffffULL;
        double x = (double)rabs * z.wi[idx];
        if (rr & 1) x = -x;
        const bool fast = rabs < z.ki[idx];
        const uint64_t F = __ballot(fast);
        while (local < 64 && produced < n) {
            const uint64_t S = ~F & (~0ULL << local);
            const int q = S ? __builtin_ctzll(S) : 64;
            if (lane >= local && lane < q) {
                const int j = produced + lane - local;
                if (j < n) out[j] = gen_basic_sample(c, j, x);
            }
            produced += q - local;
            if (q == 64) { local = 64; break; }
            int consumed = 1;
            double v = 0.0;
            if (lane == q) v = slow_normal(st, inc, rabs, idx, x, z, consumed);
            v = __shfl(v, q);
            consumed = __shfl(consumed, q);
            if (produced < n && lane == 0) out[produced] = gen_basic_sample(c, produced, v);
            ++produced;
            local = q + consumed;
        }
        do {   // advance all lanes by one chunk; skip chunks a slow normal consumed
            st = jt->a64 * st + c64;
            local -= 64;
        } while (local >= 64);
    }
}

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
    float2 y[PER];
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int k = (int)threadIdx.x + b * T;
        y[b] = make_float2(0.f, 0.f);
        if (k < K) {
            const double xs = src(k);
            if (xs >= 0.0 && xs <= (double)(K - 1)) {
                const int j = (int)xs;
                if (j >= K - 1) {
                    y[b] = buf[K - 1];
                } else {
                    const float fr = (float)(xs - (double)j);
                    const float2 a = buf[j], c = buf[j + 1];
                    y[b] = make_float2((c.x - a.x) * fr + a.x, (c.y - a.y) * fr + a.y);
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < PER; ++b) {
        const int k = (int)threadIdx.x + b * T;
        if (k < K) buf[k] = y[b];
    }
    __syncthreads();
}

// irfft drops the imaginary part of the DC bin (and of the Nyquist bin for even n);
// reproduce that between fused spectral stages.
MSG_DEV void drop_edge_imag(float2* buf, const RealPlan& rp) {
    if (threadIdx.x == 0) {
        buf[0].y = 0.f;
        if (rp.even) buf[rp.n / 2].y = 0.f;
    }
    __syncthreads();
}

template <int T, int MAXC>
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
    const RealPlan rp = plans[er.plan];
    const int K = n / 2 + 1;
    for (int j = threadIdx.x; j < n; j += T) rx_set(lds, rp, j, micro[j]);
    __syncthreads();

    if (ops & (SPEC_TILT_NOISE | SPEC_TILT_SKEW)) {
        // tilted_noise (MS:224-233): W *= (f/f1)^alpha with f[0] := f[1]
        rfft_lds<T, MAXC>(lds, rp);
        const double val = 1.0 / ((double)n * (1.0 / (double)er.gen_sr));
        for (int k = threadIdx.x; k < K; k += T) {
            double sh = 1.0;
            if (K > 1 && k > 0) sh = pow(((double)k * val) / fmax(1e-12, val), er.tilt_alpha);
            lds[k] = cscale(lds[k], (float)sh);
        }
        __syncthreads();
        irfft_lds<T, MAXC>(lds, rp);
        // envelope, skew, fade (MS:246-255, 265-268)
        const int fade = (int)(0.01 * n) > 8 ? (int)(0.01 * n) : 8;
        const double inv_sr = 1.0 / (double)er.gen_sr;
        if (ops & SPEC_TILT_SKEW) {
            // d = diff(max(0, w), prepend=w[0]): needs neighbours -> via registers
            constexpr int PER = (2 * MAXC + T - 1) / T;
            float d[PER];
#pragma unroll
            for (int b = 0; b < PER; ++b) {
                const int j = (int)threadIdx.x + b * T;
                d[b] = 0.f;
                if (j < n && j > 0) d[b] = fmaxf(0.f, rx_get(lds, rp, j)) - fmaxf(0.f, rx_get(lds, rp, j - 1));
            }
            __syncthreads();
#pragma unroll
            for (int b = 0; b < PER; ++b) {
                const int j = (int)threadIdx.x + b * T;
                if (j < n) {
                    const float env = (float)exp(-((double)j * inv_sr) / er.env_tau);
                    rx_set(lds, rp, j, d[b] * env * fade_w(j, n, fade));
                }
            }
        } else {
            for (int j = threadIdx.x; j < n; j += T) {
                const float env = (float)exp(-((double)j * inv_sr) / er.env_tau);
                rx_set(lds, rp, j, rx_get(lds, rp, j) * env * fade_w(j, n, fade));
            }
        }
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += T) micro[j] = rx_get(lds, rp, j);
        if (!(ops & (SPEC_LOWPASS | SPEC_STRETCH | SPEC_WARP))) {
            for (int j = threadIdx.x; j < n; j += T) grain[j] = rx_get(lds, rp, j);
            return;
        }
        __syncthreads();
    }

    rfft_lds<T, MAXC>(lds, rp);
    if (ops & SPEC_LOWPASS) {
        for (int k = threadIdx.x; k < K; k += T)
            lds[k] = cscale(lds[k], lowpass_w(k, n, er.gen_sr, er.cutoff_gen, er.roll));
        __syncthreads();
    }
    if (ops & SPEC_WARP) {   // fft_warp_power (MS:103-115)
        drop_edge_imag(lds, rp);
        const double kmax = fmax(1.0, (double)(K - 1));
        const double ip = 1.0 / fmax(1e-6, er.warp_power);
        spectral_gather<T, MAXC + 1>(lds, K, [&](int k) { return pow((double)k / kmax, ip) * kmax; });
    }
    if (ops & SPEC_STRETCH) {   // fft_partial_stretch (MS:117-128)
        drop_edge_imag(lds, rp);
        const double f = fmax(1e-12, er.stretch);
        spectral_gather<T, MAXC + 1>(lds, K, [&](int k) { return (double)k / f; });
    }
    irfft_lds<T, MAXC>(lds, rp);
    for (int j = threadIdx.x; j < n; j += T) grain[j] = rx_get(lds, rp, j);
}

// ---------------------------------------------------------------------------
// Overlap-add of placed grains (event order) x ADSR -> mono a[t].
// ---------------------------------------------------------------------------
MSG_DEV float adsr_at(const PresetRt& r, int64_t t) {
    const int64_t n = r.out_n;
    const int64_t A = r.envA, D = r.envD, R = r.envR;
    const int64_t i = A;
    const int64_t j = n < i + D ? n : i + D;
    const int64_t s1 = (j > n - R) ? j : n - R;
    const float c = r.envC, S = r.envS;
    if (A > 0 && t < A) return powf((float)((double)t * (1.0 / (double)A)), c);
    if (D > 0 && j > i && t >= i && t < j) {
        const float d = (float)((double)(t - i) * (1.0 / (double)(j - i)));
        return 1.0f - (1.0f - S) * powf(d, c);
    }
    if (t >= j && t < s1) return S;
    if (R > 0 && n > s1 && t >= s1) {
        const int64_t num = n - s1;
        float u;
        if (num == 1) u = 0.f;
        else if (t == n - 1) u = 1.f;
        else u = (float)((double)(t - s1) * (1.0 / (double)(num - 1)));
        return S * (1.0f - powf(u, c));
    }
    return 1.0f;
}

__device__ __forceinline__ int find_preset(const int32_t* __restrict__ begin, int n_presets, int b) {
    int lo = 0, hi = n_presets - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (begin[mid] <= b) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__global__ void __launch_bounds__(OLA_T)
k_ola_env(const msg_event* __restrict__ events, const PresetRt* __restrict__ rt,
          const int32_t* __restrict__ tile_begin, int n_presets,
          const float* __restrict__ grain_pool, float* __restrict__ mono) {
    const int b = blockIdx.x;
    const int p = find_preset(tile_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int64_t t0 = (int64_t)(b - r.tile_begin) * OLA_TILE;
    const int64_t t1 = t0 + OLA_TILE < r.out_n ? t0 + OLA_TILE : r.out_n;
    constexpr int PER = OLA_TILE / OLA_T;
    float acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = 0.f;
    // events sorted by start: first event whose start > t0 - max_n
    const msg_event* ev = events + r.ev_begin;
    int lo = 0, hi = r.n_events;
    const int64_t lim = t0 - (int64_t)r.max_n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if ((int64_t)ev[mid].start <= lim) lo = mid + 1; else hi = mid;
    }
    for (int k = lo; k < r.n_events; ++k) {
        const msg_event& e = ev[k];
        if ((int64_t)e.start >= t1) break;
        if (e.len <= 0) continue;
        const int64_t s = e.start, L = e.len;
        if (s + L <= t0) continue;
        const float amp = (float)e.amp;
        const float* g = grain_pool + r.pool_base + e.pool_off + e.offset;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int64_t t = t0 + threadIdx.x + u * OLA_T;
            const int64_t q = t - s;
            if (t < t1 && q >= 0 && q < L) acc[u] += amp * g[q];
        }
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t t = t0 + threadIdx.x + u * OLA_T;
        if (t < t1) mono[r.y_off + t] = acc[u] * adsr_at(r, t);
    }
}

// ---------------------------------------------------------------------------
// Combined space FIR h = (delta + ER) * IR, partition spectra (one WG per partition).
// ---------------------------------------------------------------------------
template <int T, int MAXC>
__global__ void __launch_bounds__(T)
k_fir_h(const PresetRt* __restrict__ rt, const int32_t* __restrict__ hblk_begin, int n_presets,
        const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
        const int32_t* __restrict__ er_off, const double* __restrict__ er_gain,
        const double* __restrict__ ir_bank, float2* __restrict__ hspec) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int p = find_preset(hblk_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int q = b - r.h_block_begin;
    const RealPlan rp = fir_plans[fir_plan_of[p]];
    const int N = r.fir_N, P = r.fir_P;
    const double* ir = ir_bank + r.ir_off;
    const int irl = r.ir_len;
    for (int u = threadIdx.x; u < N; u += T) {
        double h = 0.0;
        const int64_t t = (int64_t)q * P + u;
        if (u < P) {
            h = irl > 0 ? (t < irl ? ir[t] : 0.0) : (t == 0 ? 1.0 : 0.0);
            for (int k = 0; k < r.n_taps; ++k) {
                const int64_t o = er_off[r.er_base + k];
                if (o <= 0 || o >= r.out_n) continue;              // MS:418-420
                const int64_t s = t - o;
                if (irl > 0) { if (s >= 0 && s < irl) h += er_gain[r.er_base + k] * ir[s]; }
                else if (s == 0) h += er_gain[r.er_base + k];
            }
        }
        rx_set(lds, rp, u, (float)h);
    }
    __syncthreads();
    rfft_lds<T, MAXC>(lds, rp);
    const int K = N / 2 + 1;
    float2* dst = hspec + r.h_off + (int64_t)q * K;
    for (int k = threadIdx.x; k < K; k += T) dst[k] = lds[k];
}

// Partitioned FFT overlap-save: block outputs B samples; Q forward FFTs
// accumulate X_q * H_q in registers, one inverse FFT (MS:438-445 arithmetic,
// with the ER taps of MS:409-421 folded into h).
template <int T, int MAXC>
__global__ void __launch_bounds__(T)
k_fir(const PresetRt* __restrict__ rt, const int32_t* __restrict__ fblk_begin, int n_presets,
      const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
      const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int p = find_preset(fblk_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const RealPlan rp = fir_plans[fir_plan_of[p]];
    const int N = r.fir_N, P = r.fir_P, Q = r.fir_Q, B = r.fir_B;
    const int64_t n = r.out_n;
    const int64_t t0 = (int64_t)(b - r.fir_block_begin) * B;
    const float* x = x_in + r.y_off;
    const int K = N / 2 + 1;
    constexpr int PER = (MAXC + 1 + T - 1) / T;
    float2 acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = make_float2(0.f, 0.f);
    for (int q = 0; q < Q; ++q) {
        const int64_t s0 = t0 - (int64_t)q * P - (P - 1);
        for (int u = threadIdx.x; u < N; u += T) {
            const int64_t s = s0 + u;
            rx_set(lds, rp, u, (s >= 0 && s < n) ? x[s] : 0.f);
        }
        __syncthreads();
        rfft_lds<T, MAXC>(lds, rp);
        const float2* H = hspec + r.h_off + (int64_t)q * K;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = (int)threadIdx.x + u * T;
            if (k < K) {
                const float2 v = cmul(lds[k], H[k]);
                acc[u] = cadd(acc[u], v);
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int k = (int)threadIdx.x + u * T;
        if (k < K) lds[k] = acc[u];
    }
    __syncthreads();
    irfft_lds<T, MAXC>(lds, rp);
    float* y = y_out + r.y_off;
    for (int u = threadIdx.x + (P - 1); u < N; u += T) {
        const int64_t t = t0 + (u - (P - 1));
        if (t < n) y[t] = rx_get(lds, rp, u);
    }
}

// ---------------------------------------------------------------------------
// Stereo (even n: exact 25-tap Bessel FIR form of the spectral rotation),
// tanh saturation and peak normalisation.
// ---------------------------------------------------------------------------
MSG_DEV void stereo_pair(const PresetRt& r, const float* __restrict__ y, int64_t t, float& L, float& R) {
    const int64_t n = r.out_n;
    if (!r.stereo_fir) { L = R = y[t]; return; }
    int64_t il = t - r.dl;
    il %= n; if (il < 0) il += n;
    L = y[il];
    float acc = 0.f;
    int64_t base = (t + r.dr - 24) % n;
    if (base < 0) base += n;
#pragma unroll
    for (int m = 0; m < 25; ++m) {
        int64_t idx = base + 2 * m;
        if (idx >= n) idx -= n;
        if (idx >= n) idx -= n;
        acc = fmaf(r.bess[m], y[idx], acc);
    }
    R = acc;
}

__global__ void __launch_bounds__(ST_T)
k_stereo_max(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_begin, int n_presets,
             const float* __restrict__ ybuf, unsigned* __restrict__ maxbits) {
    const int b = blockIdx.x;
    const int p = find_preset(st_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int64_t t0 = (int64_t)(b - st_begin[p]) * ST_TILE;
    const float* y = ybuf + r.y_off;
    float m = 0.f;
    for (int u = threadIdx.x; u < ST_TILE; u += ST_T) {
        const int64_t t = t0 + u;
        if (t >= r.out_n) break;
        float L, R;
        stereo_pair(r, y, t, L, R);
        m = fmaxf(m, fmaxf(fabsf(L), fabsf(R)));
    }
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    __shared__ float wm[ST_T / 64];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        float v = wm[0];
        for (int w = 1; w < ST_T / 64; ++w) v = fmaxf(v, wm[w]);
        atomicMax(maxbits + p, __float_as_uint(v));
    }
}

MSG_DEV float sat(float v, float d, float inv_td) { return d > 0.f ? tanhf(v * d) * inv_td : v; }

__global__ void __launch_bounds__(ST_T)
k_stereo_out(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_begin, int n_presets,
             const float* __restrict__ ybuf, const unsigned* __restrict__ maxbits, float* __restrict__ out) {
    const int b = blockIdx.x;
    const int p = find_preset(st_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int64_t t0 = (int64_t)(b - st_begin[p]) * ST_TILE;
    const float* y = ybuf + r.y_off;
    const float d = r.drive;
    const float inv_td = d > 0.f ? 1.0f / tanhf(d) : 1.f;
    const float M = __uint_as_float(maxbits[p]);
    const float mc = sat(M, d, inv_td);
    const float scale = mc > 0.f ? r.peak / mc : 1.f;
    float2* o = reinterpret_cast<float2*>(out) + r.out_off;
    for (int u = threadIdx.x; u < ST_TILE; u += ST_T) {
        const int64_t t = t0 + u;
        if (t >= r.out_n) break;
        float L, R;
        stereo_pair(r, y, t, L, R);
        o[t] = make_float2(sat(L, d, inv_td) * scale, sat(R, d, inv_td) * scale);
    }
}
