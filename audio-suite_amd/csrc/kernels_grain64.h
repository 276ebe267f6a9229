// kernels_grain64.h — the float64 grain chain (TUs: k_grain64_lds.hip and
// k_grain64_glb.hip for k_grain64<false/true>, k_grain64.hip for the rest).
//
// Presets that use a stage whose reference result hinges on float64 decisions
// or float64 noise floors run every event through this chain instead of the
// float32 one (kernels_spectral.h):
//   generators   Dust (MS:239-245), Crackle (MS:271-281), Stick-slip
//                (MS:283-301), Micro-chaos (MS:303-315), Wavelet atoms
//                (MS:317-331), IR fragment (MS:333-348), Image scanline
//                (MS:350-362), and the normal-driven modes (MS:219-269)
//   spectral     band-limit (MS:39-59), power warp (MS:103-115), cepstral warp
//                (MS:150-163), partial lock (MS:130-148), stretch (MS:117-128)
//   physics      resonator bank (MS:369-384), waveguide splinters (MS:386-402)
//   unfold       multi-band (MS:492-500, 61-101)
//   chain        event feedback (MS:731-734), spectral imprint (MS:565-581)
//
// k_grain64: one workgroup per event; the grain lives in LDS as float64 from
// generation to the end of the multi-band unfold, every spectral stage working
// on one resident spectrum (the reference's irfft -> rfft between stages is an
// identity up to the dropped imaginary DC/Nyquist parts, reproduced here).
// k_chain64: one workgroup per preset walks its events in order for the
// feedback/imprint recurrences (state: previous grain and the imprint memory).
#pragma once
#include "rt.h"
#include "fft64.h"

constexpr int G64_T = 512;
constexpr int G64_MAXE = 16;
constexpr int G64_CAP = G64_T * G64_MAXE;      // 8192 double2 slots = 128 KiB of LDS
constexpr int G64_MAXPAR = 256;                // modes / atoms / lines / peaks

#if defined(__HIPCC__)
constexpr double G64_PI = 3.141592653589793;

struct G64Shared {
    double red[G64_T / 64];
    int ired[G64_T / 64];
    double par[4][G64_MAXPAR];
    int ipar[G64_MAXPAR];
    double2 peak_x[G64_MAXPAR];
    int peak_k2[G64_MAXPAR];
    uint32_t mask[(G64_CAP + 1 + 31) / 32 + 1];
    int scal[4];
};

MSG_DEV double block_max(double v, G64Shared& sh) {
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh.red[threadIdx.x >> 6] = v;
    __syncthreads();
    double r = sh.red[0];
    for (int k = 1; k < G64_T / 64; ++k) r = fmax(r, sh.red[k]);
    return r;
}

// hann(n) (MS:17-21) and the gen_basic edge fade (MS:265-268), float64
MSG_DEV double hann64(int j, int n) {
    if (n <= 1) return 1.0;
    return 0.5 - 0.5 * cos(2.0 * G64_PI * (double)j / (double)(n - 1));
}
MSG_DEV double fade64(int j, int n, int fade) {
    double w = 1.0;
    if (j < fade) w *= (double)j * (1.0 / (double)fade);
    if (j >= n - fade) w *= (double)(j - (n - fade)) * (-1.0 / (double)fade) + 1.0;
    return w;
}
// np.linspace(0, 1, m)[i]
MSG_DEV double lin01(int i, int m) {
    if (m <= 1) return 0.0;
    if (i == m - 1) return 1.0;
    return (double)i * (1.0 / (double)(m - 1));
}
// np.interp(x, linspace(0, 1, m), fp) with fp(i) a functor
template <class F>
MSG_DEV double interp_lin01(double x, int m, F&& fp) {
    if (m == 1) return fp(0);
    if (x < 0.0) return fp(0);
    if (x > 1.0) return fp(m - 1);
    int j = (int)(x * (double)(m - 1));
    if (j > m - 1) j = m - 1;
    while (j > 0 && lin01(j, m) > x) --j;
    while (j < m - 1 && lin01(j + 1, m) <= x) ++j;
    if (j >= m - 1) return fp(m - 1);
    const double xj = lin01(j, m);
    if (xj == x) return fp(j);
    const double slope = (fp(j + 1) - fp(j)) / (lin01(j + 1, m) - xj);
    return slope * (x - xj) + fp(j);
}

// np.convolve(x, exp(-linspace(0, E, K)), mode="same") with x = s[0..n0) ->
// d[0..L), L = max(n0, K) (the arrays swap when the kernel is longer).
MSG_DEV void conv_same_exp(double* d, const double* s, int n0, int K, double E) {
    const int L = n0 > K ? n0 : K;
    const int S = n0 < K ? n0 : K;
    const int off = (S - 1) / 2;
    const double step = E / (double)(K - 1);
    for (int t = threadIdx.x; t < L; t += G64_T) {
        const int i = t + off;               // index into the full convolution
        int j0 = i - (K - 1); if (j0 < 0) j0 = 0;
        int j1 = i; if (j1 > n0 - 1) j1 = n0 - 1;
        double acc = 0.0;
        for (int j = j0; j <= j1; ++j) {
            const int k = i - j;
            const double h = exp(-(k == K - 1 ? E : (double)k * step));
            acc += s[j] * h;
        }
        d[t] = acc;
    }
    __syncthreads();
}

// copy d[0..n) -> s[0..n) (scratch), ends with a barrier
MSG_DEV void copy_to(double* s, const double* d, int n) {
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += G64_T) s[j] = d[j];
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Generators -> d[0..n) (float64), MS:219-362.
// ---------------------------------------------------------------------------
MSG_DEV void gen64(const msg_preset& pr, const PresetRt& r, const Ev64& ev, const Real64Plan& rp,
                   const double* __restrict__ normals, const double* __restrict__ irbank,
                   const uint8_t* __restrict__ imgbank, const nprng::Zig& z, double2* buf, double2* scr,
                   G64Shared& sh) {
    double* d = reinterpret_cast<double*>(buf);
    const int n = ev.n;
    double* s = d + n;                      // scratch: n doubles after the signal
    const int tid = threadIdx.x;
    const uint64_t seed = (uint64_t)(pr.seed + ev.index);
    const double sr = (double)ev.gen_sr;
    const int mode = pr.gen_mode == MSG_GEN_FALLBACK ? MSG_GEN_NOISE_BURST : pr.gen_mode;
    const double tilt_db = pr.gen_mode == MSG_GEN_FALLBACK ? -3.0 : pr.noise_tilt;
    const int fade = (int)(0.01 * n) > 8 ? (int)(0.01 * n) : 8;
    switch (mode) {
    case MSG_GEN_GAUSSIAN_CLICK: case MSG_GEN_RESONANT: {
        const int sigma = (int)(0.0025 * n) > 1 ? (int)(0.0025 * n) : 1;
        const double f = fmax(10.0, pr.ring_hz);
        const double tau = fmax(1e-6, pr.ring_decay_ms / 1000.0);
        const double tau_e = fmax(1e-6, (pr.micro_ms / 1000.0) * 0.15);
        const double w2 = 2.0 * G64_PI * f;
        for (int j = tid; j < n; j += G64_T) {
            const double N = normals[j];
            double x;
            if (mode == MSG_GEN_GAUSSIAN_CLICK) {
                const double u = (double)j / (double)sigma;
                x = exp(-0.5 * (u * u)) * (N * 0.12 + 1.0);
            } else {
                const double t = (double)j / sr;
                x = 0.9 * (sin(w2 * t) * exp(-t / tau)) + 0.25 * (N * exp(-t / tau_e));
            }
            d[j] = x * fade64(j, n, fade);
        }
        __syncthreads();
        return;
    }
    case MSG_GEN_NOISE_BURST: case MSG_GEN_SKEWED: {
        // tilted_noise (MS:224-233)
        for (int j = tid; j < n; j += G64_T) d[j] = normals[j];
        f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
        const double val = 1.0 / ((double)n * (1.0 / sr));
        const double alpha = log(pow(10.0, tilt_db / 20.0)) / log(2.0);
        const int K = n / 2 + 1;
        for (int k = tid; k < K; k += G64_T) {
            const double fk = (K > 1 && k == 0) ? val : (double)k * val;
            buf[k] = dscale(buf[k], pow(fk / fmax(1e-12, val), alpha));
        }
        f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);
        const bool skew = mode == MSG_GEN_SKEWED;
        const double tau = fmax(1e-6, (pr.micro_ms / 1000.0) * (skew ? 0.2 : 0.25));
        if (skew) copy_to(s, d, n);
        for (int j = tid; j < n; j += G64_T) {
            double x;
            if (skew) x = (j == 0) ? 0.0 : fmax(0.0, s[j]) - fmax(0.0, s[j - 1]);
            else x = d[j];
            const double t = (double)j / sr;
            d[j] = x * exp(-t / tau) * fade64(j, n, fade);
        }
        __syncthreads();
        return;
    }
    case MSG_GEN_DUST: {
        for (int j = tid; j < n; j += G64_T) s[j] = 0.0;
        __syncthreads();
        if (tid == 0) {
            const double kr = rint(pr.dust_density * (double)n);
            const int64_t k = kr > 1.0 ? (int64_t)kr : 1;
            nprng::Pcg64 gi = nprng::default_rng(seed);
            nprng::Pcg64 gu = gi;
            for (int64_t q = 0; q < k; ++q) (void)nprng::integers(gu, 0, n);   // idx = integers(0, n, size=k)
            for (int64_t q = 0; q < k; ++q) {                                 // x[idx] = uniform(-1, 1, size=k)
                const int64_t idx = nprng::integers(gi, 0, n);
                s[idx] = nprng::uniform(gu, -1.0, 1.0);
            }
        }
        __syncthreads();
        const int K = (int)(0.01 * n) > 8 ? (int)(0.01 * n) : 8;
        conv_same_exp(d, s, n, K, 6.0);
        for (int j = tid; j < n; j += G64_T) d[j] *= fade64(j, n, fade);
        __syncthreads();
        return;
    }
    case MSG_GEN_CRACKLE: {
        const int n0 = ev.n0;
        const int K = pr.crackle_kernel > 8 ? pr.crackle_kernel : 8;
        for (int j = tid; j < n0; j += G64_T) s[j] = 0.0;
        __syncthreads();
        if (tid == 0) {
            const int64_t cnt = (int64_t)fmax(8.0, pr.crackle_density);
            nprng::Pcg64 gp = nprng::default_rng(seed);
            nprng::Pcg64 gu = gp;
            for (int64_t q = 0; q < cnt; ++q) (void)nprng::pareto(gu, z, pr.crackle_alpha);
            double cs = 0.0;
            for (int64_t q = 0; q < cnt; ++q) {
                cs += nprng::pareto(gp, z, pr.crackle_alpha);       // times = cumsum(steps)
                if (cs < (double)n0) {
                    const int ti = (int)cs;
                    s[ti] += nprng::uniform(gu, -1.0, 1.0);
                }
            }
        }
        __syncthreads();
        conv_same_exp(d, s, n0, K, 6.0);
        return;
    }
    case MSG_GEN_STICK_SLIP: {
        if (tid == 0) {
#pragma clang fp contract(off)
            nprng::Pcg64 g = nprng::default_rng(seed);
            bool sticking = true;
            double force = 0.0;
            for (int i = 0; i < n; ++i) {
                double x = 0.0;
                if (sticking) {
                    const double N = nprng::standard_normal(g, z);
                    const double a = N * pr.ss_noise;
                    const double b = a + 0.2;
                    const double c = pr.ss_build * b;
                    force = force + c;
                    if (fabs(force) > pr.ss_threshold) sticking = false;
                } else {
                    const double N = nprng::standard_normal(g, z);
                    const double a = 0.25 * N;
                    x = force + a;
                    force = force * pr.ss_decay;
                    if (fabs(force) < 0.02) { sticking = true; force = 0.0; }
                }
                d[i] = x;
            }
        }
        __syncthreads();
        for (int j = tid; j < n; j += G64_T) d[j] *= hann64(j, n);
        __syncthreads();
        return;
    }
    case MSG_GEN_MICRO_CHAOS: {
        if (tid == 0) {
#pragma clang fp contract(off)
            nprng::Pcg64 g = nprng::default_rng(seed);
            const int64_t sd = pr.seed + ev.index;
            double y = (double)(((sd % 10000) + 10000) % 10000) / 10000.0;
            for (int i = 0; i < n; ++i) {
                const double ry = pr.chaos_r * y;
                y = ry * (1.0 - y);
                const double v = y - 0.5;
                s[i] = (nprng::next_double(g) < pr.chaos_gate) ? v : 0.0;
            }
        }
        __syncthreads();
        conv_same_exp(d, s, n, 48, 5.0);
        for (int j = tid; j < n; j += G64_T) d[j] *= hann64(j, n);
        __syncthreads();
        return;
    }
    case MSG_GEN_WAVELET: {
        // any atom count: the atoms' parameters are drawn G64_MAXPAR at a time by
        // lane 0 from the one stream (MS:322-327), and every sample's sum runs on
        // in d[j] across the chunks, in the reference's k order (MS:329)
        const int cnt = pr.wav_count > 1 ? pr.wav_count : 1;
        const double dur = pr.micro_ms;
        const double half = (double)n / 2.0;
        nprng::Pcg64 g = nprng::default_rng(seed);
        const int64_t lo = -(int64_t)((n + 7) / 8);       // Python -n//8 (floor)
        const int64_t hi = n / 8;
        for (int k0 = 0; k0 < cnt; k0 += G64_MAXPAR) {
            const int kn = cnt - k0 < G64_MAXPAR ? cnt - k0 : G64_MAXPAR;
            if (tid == 0) {
                for (int k = 0; k < kn; ++k) {
                    const double f0 = pr.wav_base_hz * pow(2.0, nprng::uniform(g, -pr.wav_spread, pr.wav_spread));
                    const double sig_ms = fmax(0.03, dur * nprng::uniform(g, 0.04, 0.18));
                    const double ph = nprng::uniform(g, 0.0, 2.0 * G64_PI);
                    const int64_t sh_ = nprng::integers(g, lo, hi);
                    sh.par[0][k] = f0;
                    sh.par[1][k] = fmax(1e-9, sig_ms / 1000.0);
                    sh.par[2][k] = ph;
                    sh.ipar[k] = (int)sh_;
                }
            }
            __syncthreads();
            for (int j = tid; j < n; j += G64_T) {
                double x = k0 == 0 ? 0.0 : d[j];
                for (int k = 0; k < kn; ++k) {
                    int i = (j - sh.ipar[k]) % n;
                    if (i < 0) i += n;
                    const double t = ((double)i - half) / sr;
                    const double u = t / sh.par[1][k];
                    const double a = exp(-0.5 * (u * u)) * cos(2.0 * G64_PI * sh.par[0][k] * t + sh.par[2][k]);
                    x += (1.0 / (1.0 + (double)(k0 + k) * 0.6)) * a;
                }
                d[j] = x;
            }
            __syncthreads();                              // the chunk's parameters are read up
        }
        for (int j = tid; j < n; j += G64_T) d[j] *= hann64(j, n);
        __syncthreads();
        return;
    }
    case MSG_GEN_IR_FRAGMENT: {
        if (r.frag_len < 32) {                     // "No IR loaded": zeros (MS:335-336)
            for (int j = tid; j < n; j += G64_T) d[j] = 0.0;
            __syncthreads();
            return;
        }
        if (tid == 0) {
            nprng::Pcg64 g = nprng::default_rng(seed);
            const int64_t hi = r.frag_len - 256 > 1 ? r.frag_len - 256 : 1;
            const int64_t st = nprng::integers(g, 0, hi);
            sh.scal[0] = (int)st;
            sh.scal[1] = (int)(r.frag_len - st < 256 ? r.frag_len - st : 256);
        }
        __syncthreads();
        const double* sl = irbank + r.frag_off + sh.scal[0];
        const int L = sh.scal[1];
        double m = 0.0;
        for (int j = tid; j < n; j += G64_T) {
            const double x = interp_lin01(lin01(j, n), L, [&](int i) { return sl[i]; }) * hann64(j, n);
            d[j] = x;
            m = fmax(m, fabs(x));
        }
        m = block_max(m, sh);
        if (m > 0.0) {
            const double sc = 0.9 / m;
            for (int j = tid; j < n; j += G64_T) d[j] *= sc;
        }
        __syncthreads();
        return;
    }
    case MSG_GEN_IMAGE: {
        if (r.img_h <= 0) {                        // "No image loaded": zeros (MS:353-354)
            for (int j = tid; j < n; j += G64_T) d[j] = 0.0;
            __syncthreads();
            return;
        }
        const int w = r.img_w;
        if (tid == 0) {
            nprng::Pcg64 g = nprng::default_rng(seed);
            const int y = (int)nprng::integers(g, 0, r.img_h);
            const uint8_t* row = imgbank + r.img_off + (int64_t)y * w;
            double sum = 0.0;
            for (int i = 0; i < w; ++i) sum += (double)row[i] / 255.0;
            sh.scal[0] = y;
            sh.par[0][0] = sum / (double)w;
        }
        __syncthreads();
        const uint8_t* row = imgbank + r.img_off + (int64_t)sh.scal[0] * w;
        const double mean = sh.par[0][0];
        for (int j = tid; j < n; j += G64_T) {
            const double x = interp_lin01(lin01(j, n), w,
                                          [&](int i) { return ((double)row[i] / 255.0 - mean) * 2.0; });
            s[j] = x * hann64(j, n);
        }
        __syncthreads();
        conv_same_exp(d, s, n, 48, 5.0);
        return;
    }
    default:
        for (int j = tid; j < n; j += G64_T) d[j] = 0.0;
        __syncthreads();
        return;
    }
}

// ---------------------------------------------------------------------------
// Spectral stages on the resident spectrum X[0..K) (MS:39-163).
// ---------------------------------------------------------------------------
MSG_DEV void drop_edge_imag64(double2* buf, const Real64Plan& rp) {
    __syncthreads();
    if (threadIdx.x == 0) {
        buf[0].y = 0.0;
        if (rp.even) buf[rp.n / 2].y = 0.0;
    }
    __syncthreads();
}

// rfftfreq(n, 1/sr)[k] exactly as NumPy builds it
struct Freq64 {
    double val;
    MSG_DEV Freq64(int n, double sr) { val = 1.0 / ((double)n * (1.0 / sr)); }
    MSG_DEV double f(int k) const { return (double)k * val; }
};

// lowpass_fft weight (MS:48-58)
MSG_DEV double lowpass_w64(double f, double c, double r, double f1) {
    if (r <= 0) return f > c ? 0.0 : 1.0;
    if (f > f1) return 0.0;
    if (f >= c) return 0.5 * (1.0 + cos(G64_PI * ((f - c) / fmax(1e-12, (f1 - c)))));
    return 1.0;
}

// bandpass_fft weight of one band (MS:61-101); zero band when hi <= 0
MSG_DEV double bandpass_w64(double f, double lo, double hi, double roll, double nyq) {
    lo = fmax(0.0, lo);
    hi = fmax(lo, hi);
    hi = fmin(hi, nyq);
    if (hi <= 0) return 0.0;
    const double r = fmax(0.0, roll);
    double w = 1.0;
    if (lo > 0) {
        if (r <= 0) { if (f < lo) w = 0.0; }
        else {
            const double f0 = fmax(0.0, lo - r), f1 = lo;
            if (f < f0) w = 0.0;
            else if (f >= f0 && f <= f1) w *= 0.5 * (1.0 - cos(G64_PI * ((f - f0) / fmax(1e-12, (f1 - f0)))));
        }
    }
    if (hi < nyq) {
        if (r <= 0) { if (f > hi) w = 0.0; }
        else {
            const double f0 = hi, f1 = fmin(nyq, hi + r);
            if (f > f1) w = 0.0;
            else if (f >= f0 && f <= f1) w *= 0.5 * (1.0 + cos(G64_PI * ((f - f0) / fmax(1e-12, (f1 - f0)))));
        }
    }
    return w;
}

// np.interp's slope form: (fp[j+1] - fp[j]) / 1 * (x - j) + fp[j]
MSG_DEV double lerp64(double a, double b, double fr) { return (b - a) * fr + a; }
MSG_DEV double2 lerp64(double2 a, double2 b, double fr) { return d2((b.x - a.x) * fr + a.x, (b.y - a.y) * fr + a.y); }

// In-place Y[k] = interp(src(k), arange(K), X) (np.interp, left = right = 0).
// Sources lie on one side of their bin: chunks run in the safe order with
// read -> barrier -> write -> barrier.  Works for real arrays too (C = double).
template <class C, class Src>
MSG_DEV void gather64(C* buf, int K, bool ascending, Src src) {
    constexpr int CH = 4, CW = CH * G64_T;
    const int nch = (K + CW - 1) / CW;
    for (int c = 0; c < nch; ++c) {
        const int base = (ascending ? c : nch - 1 - c) * CW;
        C y[CH];
#pragma unroll
        for (int b = 0; b < CH; ++b) {
            const int k = base + threadIdx.x + b * G64_T;
            y[b] = C{};
            if (k < K) {
                const double xs = src(k);
                if (xs >= 0.0 && xs <= (double)(K - 1)) {
                    const int j = (int)xs;
                    if (j >= K - 1) {
                        y[b] = buf[K - 1];
                    } else if ((double)j == xs) {
                        y[b] = buf[j];
                    } else {
                        const double fr = xs - (double)j;
                        y[b] = lerp64(buf[j], buf[j + 1], fr);
                    }
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int b = 0; b < CH; ++b) {
            const int k = base + threadIdx.x + b * G64_T;
            if (k < K) buf[k] = y[b];
        }
        __syncthreads();
    }
}
// partial_lock_stretch (MS:130-148) on the resident spectrum.  Peaks are taken by
// repeated block arg-max (descending |X|, ties to the larger bin) and applied in
// argsort order (ascending: selection p is entry cnt-1-p).  Up to G64_MAXPAR
// peaks are held at once; beyond that the entries are applied G64_MAXPAR at a
// time in argsort order, each chunk re-running the selection down to its own
// entries, with every bin's sum carried across the chunks (registers in the LDS
// engine, where K <= G64_T * G64_MAXE; acc_g, the FFT scratch, in the global one).
MSG_DEV void partial_lock64(double2* buf, int K, double factor, int top_n, int neigh, G64Shared& sh,
                            uint32_t* mask, double2* acc_g) {
    const int nb = K - 1;                   // candidates: bins 1..K-1
    int cnt;
    if (top_n > 0) cnt = top_n < nb ? top_n : nb;
    else if (top_n == 0) cnt = nb;          // a[-0:] is the whole array
    else cnt = nb + top_n > 0 ? nb + top_n : 0;
    const double inv = 1.0 / (double)(neigh + 1);
    double2 accr[G64_MAXE];
#pragma unroll
    for (int b = 0; b < G64_MAXE; ++b) accr[b] = d2(0.0, 0.0);
    if (acc_g)
        for (int k = threadIdx.x; k < K; k += G64_T) acc_g[k] = d2(0.0, 0.0);
    for (int c0 = 0; c0 < cnt || c0 == 0; c0 += G64_MAXPAR) {
        const int c1 = cnt - c0 < G64_MAXPAR ? cnt : c0 + G64_MAXPAR;   // entries [c0, c1) of the argsort
        for (int i = threadIdx.x; i < (K + 31) / 32 + 1; i += G64_T) mask[i] = 0u;
        __syncthreads();
        // descending selection: pick the largest |X| not yet taken, down to entry c0
        for (int p = 0; p < cnt - c0; ++p) {
            double bv = -1.0;
            int bk = -1;
            for (int k = 1 + threadIdx.x; k < K; k += G64_T) {
                if ((mask[k >> 5] >> (k & 31)) & 1u) continue;
                const double m = hypot(buf[k].x, buf[k].y);
                if (m > bv || (m == bv && k > bk)) { bv = m; bk = k; }
            }
            for (int off = 32; off > 0; off >>= 1) {
                const double ov = __shfl_xor(bv, off);
                const int ok = __shfl_xor(bk, off);
                if (ov > bv || (ov == bv && ok > bk)) { bv = ov; bk = ok; }
            }
            if ((threadIdx.x & 63) == 0) { sh.red[threadIdx.x >> 6] = bv; sh.ired[threadIdx.x >> 6] = bk; }
            __syncthreads();
            if (threadIdx.x == 0) {
                double v = sh.red[0];
                int kk = sh.ired[0];
                for (int w = 1; w < G64_T / 64; ++w)
                    if (sh.red[w] > v || (sh.red[w] == v && sh.ired[w] > kk)) { v = sh.red[w]; kk = sh.ired[w]; }
                const int slot = cnt - 1 - p;
                if (slot < c1) {
                    sh.peak_x[slot - c0] = buf[kk];
                    sh.peak_k2[slot - c0] = (int)rint((double)kk * factor);
                }
                mask[kk >> 5] |= 1u << (kk & 31);
            }
            __syncthreads();
        }
        // Y[kk] += X[k] w(d) over this chunk's peaks, in argsort order
        const int np = c1 - c0;
        auto add = [&](int k, double2 acc) -> double2 {
            if (k >= 1) {
                for (int q = 0; q < np; ++q) {
                    const int k2 = sh.peak_k2[q];
                    if (k2 < 1 || k2 >= K) continue;
                    const int dd = k - k2;
                    if (dd < -neigh || dd > neigh) continue;
                    const double w = 1.0 - ((double)(dd < 0 ? -dd : dd) * inv);
                    acc = dadd(acc, dscale(sh.peak_x[q], w));
                }
            }
            return acc;
        };
        if (acc_g) {
            for (int k = threadIdx.x; k < K; k += G64_T) acc_g[k] = add(k, acc_g[k]);
        } else {
#pragma unroll
            for (int b = 0; b < G64_MAXE; ++b) {
                const int k = threadIdx.x + b * G64_T;
                if (k < K) accr[b] = add(k, accr[b]);
            }
        }
        __syncthreads();                      // the chunk's peaks are read up
    }
    // then + 0.12 X (MS:147)
    if (acc_g) {
        for (int k = threadIdx.x; k < K; k += G64_T) buf[k] = dadd(acc_g[k], dscale(buf[k], 0.12));
    } else {
#pragma unroll
        for (int b = 0; b < G64_MAXE; ++b) {
            const int k = threadIdx.x + b * G64_T;
            if (k < K) buf[k] = dadd(accr[b], dscale(buf[k], 0.12));
        }
    }
    __syncthreads();
}

// cepstral_warp (MS:150-163): the spectrum X is saved per thread (same bins
// read back by the same thread), the cepstrum round trip runs in the buffer.
MSG_DEV void cepstral64(double2* buf, const Real64Plan& rp, double factor, double2* __restrict__ save,
                        double2* scr) {
    const int n = rp.n, K = n / 2 + 1;
    for (int k = threadIdx.x; k < K; k += G64_T) {
        const double2 x = buf[k];
        save[k] = x;
        buf[k] = d2(log(hypot(x.x, x.y) + 1e-12), 0.0);
    }
    f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);                  // cep (n real)
    double* d = reinterpret_cast<double*>(buf);
    const double inv_f = 1.0 / fmax(1e-12, factor);
    gather64<double>(d, n, inv_f > 1.0, [&](int t) { return (double)t * inv_f; });
    f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
    for (int k = threadIdx.x; k < K; k += G64_T) {
        const double mag2 = exp(buf[k].x);
        const double2 x = save[k];
        const double a = atan2(x.y, x.x);
        double sa, ca;
        sincos(a, &sa, &ca);
        buf[k] = d2(mag2 * ca, mag2 * sa);
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// Physics (MS:369-402) on d[0..n).
// ---------------------------------------------------------------------------
// Any mode / line count: lane 0 draws the parameters G64_MAXPAR at a time from
// the one stream (MS:377-380, 391-396); the per-sample mode sum runs on in s[j]
// across the chunks in the reference's k order (MS:382), the lines stay
// sequential (MS:391-401).
MSG_DEV void resonator64(double* d, int n, double sr, const msg_preset& pr, uint64_t seed, const nprng::Zig& z,
                         G64Shared& sh) {
    (void)z;
    const int modes = pr.res_modes > 1 ? pr.res_modes : 1;
    double* s = d + n;
    nprng::Pcg64 g = nprng::default_rng(seed + 321);
    const double ratio = pr.res_fmax / fmax(1.0, pr.res_fmin);
    const int den = pr.res_modes - 1 > 1 ? pr.res_modes - 1 : 1;
    const double tau = fmax(1e-6, pr.res_decay_ms / 1000.0);
    double m = 0.0;
    for (int k0 = 0; k0 < modes; k0 += G64_MAXPAR) {
        const int kn = modes - k0 < G64_MAXPAR ? modes - k0 : G64_MAXPAR;
        if (threadIdx.x == 0) {
            for (int k = 0; k < kn; ++k) {
                double f = pr.res_fmin * pow(ratio, (double)(k0 + k) / (double)den);
                f *= pow(2.0, nprng::uniform(g, -0.02, 0.02));
                sh.par[0][k] = f;
                sh.par[1][k] = nprng::uniform(g, 0.0, 2.0 * G64_PI);
            }
        }
        __syncthreads();
        const bool last = k0 + kn >= modes;
        for (int j = threadIdx.x; j < n; j += G64_T) {
            const double t = (double)j / sr;
            const double env = exp(-t / tau);
            double acc = k0 == 0 ? 0.0 : s[j];
            for (int k = 0; k < kn; ++k) {
                const double carrier = sin(2.0 * G64_PI * sh.par[0][k] * t + sh.par[1][k]);
                acc += (1.0 / (1.0 + (double)(k0 + k) * 0.35)) * carrier * env;
            }
            s[j] = acc;
            if (last) m = fmax(m, fabs(acc));
        }
        __syncthreads();
    }
    m = block_max(m, sh);
    const double dn = fmax(1e-12, m);
    for (int j = threadIdx.x; j < n; j += G64_T) {
        const double x = d[j];
        const double sg = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0);
        d[j] = 0.55 * x + 0.45 * (s[j] / dn) * sg;
    }
    __syncthreads();
}

MSG_DEV void waveguide64(double* d, int n, double sr, const msg_preset& pr, uint64_t seed, G64Shared& sh) {
    const int lines = pr.wg_lines > 1 ? pr.wg_lines : 1;
    nprng::Pcg64 g = nprng::default_rng(seed + 777);
    for (int l0 = 0; l0 < lines; l0 += G64_MAXPAR) {
        const int ln = lines - l0 < G64_MAXPAR ? lines - l0 : G64_MAXPAR;
        if (threadIdx.x == 0) {
            for (int l = 0; l < ln; ++l) {
                const double dl = rint((nprng::uniform(g, 0.4, pr.wg_max_ms) / 1000.0) * sr);
                sh.ipar[l] = dl > 1.0 ? (int)fmin(dl, 2.0e9) : 1;
                sh.par[0][l] = pr.wg_fb * nprng::uniform(g, 0.6, 0.98);
                sh.par[1][l] = nprng::uniform(g, 0.15, 0.45);
            }
        }
        __syncthreads();
        for (int l = 0; l < ln; ++l) {
            const int dly = sh.ipar[l];
            const double gn = sh.par[0][l], mix = sh.par[1][l];
            const int lanes = dly < n ? dly : n;
            // v[t] = y[t] + g v[t - d]: independent recursions per residue t mod d
            for (int r0 = threadIdx.x; r0 < lanes; r0 += G64_T) {
                double v = 0.0;
                for (int t = r0; t < n; t += dly) {
                    const double yt = d[t];
                    v = yt + gn * v;
                    d[t] = (1.0 - mix) * yt + mix * v;
                }
            }
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------
// k_grain64: one event, generator -> spectral stages -> physics -> multi-band.
// ---------------------------------------------------------------------------
// GLOBAL = false: the grain in LDS, one event per workgroup.  GLOBAL = true:
// grains beyond the LDS engine; each workgroup walks events li = blockIdx.x +
// k gridDim.x with its own global slot (buffer gA, FFT ping-pong scratch gB,
// partial-lock mask gmask).
template <bool GLOBAL>
__global__ void __launch_bounds__(G64_T)
k_grain64(const msg_preset* __restrict__ presets, const Ev64* __restrict__ ev64, const PresetRt* __restrict__ rt,
          const Real64Plan* __restrict__ plans, const int32_t* __restrict__ list, int n_list,
          const double* __restrict__ irbank, const uint8_t* __restrict__ imgbank, nprng::Zig z,
          double* __restrict__ micro64, double* __restrict__ grain64, double2* __restrict__ save,
          float* __restrict__ grain_pool, double2* gA, double2* gB, uint32_t* gmask, int64_t slot_cap,
          int64_t mask_words) {
    extern __shared__ __attribute__((aligned(16))) double2 lds_buf[];
    __shared__ G64Shared sh;
    double2* buf = GLOBAL ? gA + (int64_t)blockIdx.x * slot_cap : lds_buf;
    double2* scr = GLOBAL ? gB + (int64_t)blockIdx.x * slot_cap : nullptr;
    uint32_t* mask = GLOBAL ? gmask + (int64_t)blockIdx.x * mask_words : sh.mask;
    for (int li = blockIdx.x; li < n_list; li += GLOBAL ? (int)gridDim.x : n_list) {
    __syncthreads();
    const Ev64 ev = ev64[list[li]];
    const msg_preset& pr = presets[ev.preset];
    const PresetRt& r = rt[ev.preset];
    const Real64Plan& rp = plans[ev.plan];
    const int n = ev.n;
    double* d = reinterpret_cast<double*>(buf);
    const uint64_t seed = (uint64_t)(pr.seed + ev.index);
    const double sr = (double)ev.gen_sr;

    gen64(pr, r, ev, rp, micro64 + ev.off64, irbank, imgbank, z, buf, scr, sh);
    for (int j = threadIdx.x; j < n; j += G64_T) micro64[ev.off64 + j] = d[j];   // micro_last (MS:688)

    const int ops = ev.ops;
    if (ops & G64_SPEC) {
        const int K = n / 2 + 1;
        f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
        if (ops & G64_LOWPASS) {                                // MS:690-692
            const Freq64 fq(n, sr);
            const double nyq = 0.5 * sr;
            const double c = fmin(fmax(ev.cutoff_gen, 1.0), nyq);
            const double rr = fmax(0.0, pr.bandlimit_roll_hz);
            const double f1 = fmin(nyq, c + rr);
            for (int k = threadIdx.x; k < K; k += G64_T) {
                const double w = lowpass_w64(fq.f(k), c, rr, f1);
                if (w != 1.0) buf[k] = dscale(buf[k], w);
            }
            __syncthreads();
        }
        // Stage boundaries: the reference leaves every stage through irfft and
        // enters the next through rfft.  Fused, that is an identity up to the
        // dropped imaginary DC/Nyquist parts -- except for the rounding floor it
        // leaves in masked bins, which the cepstral warp's log(|X| + 1e-12) and the
        // imprint's angle(X) read (MS:154, 580).  Grains that reach either run
        // the round trip itself so that floor has the reference's statistics.
        const bool faithful = (ops & G64_CEP) || (pr.flags & MSG_F_IMPRINT);
        auto boundary = [&]() {
            if (faithful) {
                f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);
                f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
            } else {
                drop_edge_imag64(buf, rp);
            }
        };
        if (ops & G64_WARP) {                                   // MS:694-695
            boundary();
            const double kmax = fmax(1.0, (double)(K - 1));
            const double ip = 1.0 / fmax(1e-6, pr.nl_warp_power);
            gather64<double2>(buf, K, ip <= 1.0, [&](int k) { return pow((double)k / kmax, ip) * kmax; });
        }
        if (ops & G64_CEP) {                                    // MS:696-697
            boundary();
            cepstral64(buf, rp, pr.cep_factor, save + ev.save_off, scr);
        }
        if (ops & G64_LOCK) {                                   // MS:699-700
            boundary();
            partial_lock64(buf, K, ev.stretch, pr.pl_top_n, pr.pl_neigh, sh, mask, GLOBAL ? scr : nullptr);
        } else if (ops & G64_STRETCH) {                         // MS:701-702
            boundary();
            const double inv_f = 1.0 / fmax(1e-12, ev.stretch);
            gather64<double2>(buf, K, inv_f > 1.0, [&](int k) { return (double)k * inv_f; });
        }
        f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);
    }
    if (ops & G64_RES) resonator64(d, n, sr, pr, seed, z, sh);  // MS:704-710
    if (ops & G64_WG) waveguide64(d, n, sr, pr, seed, sh);      // MS:712-717
    if (ops & G64_MB) {                                         // MS:722-727
        f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
        const Freq64 fq(n, sr);
        const double nyq = 0.5 * sr;
        const int K = n / 2 + 1;
        for (int k = threadIdx.x; k < K; k += G64_T) {
            const double f = fq.f(k);
            double w = 0.0;
            double lo = 0.0;
            for (int b = 0; b < 3; ++b) {
                const double hi = pr.mb_b[b];
                w += bandpass_w64(f, lo * pr.mb_u[b], hi * pr.mb_u[b], pr.mb_roll, nyq);
                lo = hi;
            }
            buf[k] = dscale(buf[k], w);
        }
        f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += G64_T) {
        grain64[ev.off64 + j] = d[j];                          // grain_last (MS:729)
        if (!(ops & G64_CHAIN)) grain_pool[ev.grain_off + j] = (float)d[j];
    }
    }   // events
}

// ---------------------------------------------------------------------------
// k_chain64: event feedback + spectral imprint, events of one preset in order.
// ---------------------------------------------------------------------------

template <bool GLOBAL>
__global__ void __launch_bounds__(G64_T)
k_chain64(const msg_preset* __restrict__ presets, const Ev64* __restrict__ ev64, const Chain64* __restrict__ chains,
          int n_chains, const Real64Plan* __restrict__ plans, const double* __restrict__ grain64,
          double* __restrict__ state, float* __restrict__ grain_pool, double2* gA, double2* gB, int64_t slot_cap) {
    extern __shared__ __attribute__((aligned(16))) double2 lds_buf[];
    double2* buf = GLOBAL ? gA + (int64_t)blockIdx.x * slot_cap : lds_buf;
    double2* scr = GLOBAL ? gB + (int64_t)blockIdx.x * slot_cap : nullptr;
    for (int ci = blockIdx.x; ci < n_chains; ci += GLOBAL ? (int)gridDim.x : n_chains) {
    __syncthreads();
    const Chain64 ch = chains[ci];
    const msg_preset& pr = presets[ch.preset];
    double* prev = state + ch.prev_off;
    double* mem = state + ch.mem_off;
    double* d = reinterpret_cast<double*>(buf);
    const bool fb_on = (pr.flags & MSG_F_EVENT_FEEDBACK) != 0;
    const bool imp_on = (pr.flags & MSG_F_IMPRINT) != 0;
    const double fb = pr.event_feedback_amt;
    const double amount = pr.spectral_imprint_amt, smooth = pr.spectral_imprint_smooth;
    int prev_n = 0, mem_k = 0;
    for (int q = 0; q < ch.n_events; ++q) {
        const Ev64& ev = ev64[ch.ev_begin + q];
        const int n = ev.n;
        const Real64Plan& rp = plans[ev.plan];
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += G64_T) {
            double x = grain64[ev.off64 + j];
            if (fb_on && prev_n > 0 && j < prev_n) x = (1.0 - fb) * x + fb * prev[j];   // MS:731-734
            d[j] = x;
        }
        if (imp_on && n >= 64 && amount > 0) {                 // MS:569-581
            const int K = n / 2 + 1;
            f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
            const bool reset = (mem_k != K);
            for (int k = threadIdx.x; k < K; k += G64_T) {
                const double2 x = buf[k];
                const double mag = hypot(x.x, x.y);
                const double mk = reset ? mag : smooth * mem[k] + (1.0 - smooth) * mag;
                mem[k] = mk;
                const double mag2 = (1.0 - amount) * mag + amount * mk;
                const double a = atan2(x.y, x.x);
                double sa, ca;
                sincos(a, &sa, &ca);
                buf[k] = d2(mag2 * ca, mag2 * sa);
            }
            mem_k = K;
            f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);
        }
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += G64_T) {
            prev[j] = d[j];
            grain_pool[ev.grain_off + j] = (float)d[j];
        }
        prev_n = n;
    }
    }   // chains
}
#endif  // __HIPCC__

#if defined(__HIPCC__)
// ---------------------------------------------------------------------------
// k_stft64: the app's spectrogram, stft_mag_db (MS:197-212), one workgroup per
// frame: (mono or the L/R mean of an interleaved buffer) x hann(win) -> rfft
// (float64 engine in LDS) -> 20 log10(max(|X|, 1e-12)).  A signal shorter
// than win is one frame of x * hann(n), zero-padded to win (MS:199-202).
// x is float32 (render output) or float64; S is frames x (win/2 + 1), row-major.
// ---------------------------------------------------------------------------
template <typename TX>
__global__ void __launch_bounds__(G64_T)
k_stft64(const Real64Plan* __restrict__ plans, int plan, const TX* __restrict__ x, int64_t n, int channels,
         int win, int hop, double* __restrict__ S) {
    extern __shared__ __attribute__((aligned(16))) double2 buf[];
    const Real64Plan& rp = plans[plan];
    double* d = reinterpret_cast<double*>(buf);
    const int f = blockIdx.x;
    const int64_t a = (int64_t)f * hop;
    const int nseg = n < win ? (int)n : win;
    for (int j = threadIdx.x; j < win; j += G64_T) {
        double v = 0.0;
        if (j < nseg) {
            const int64_t i = a + j;
            const double s = channels == 2 ? ((double)x[2 * i] + (double)x[2 * i + 1]) / 2.0 : (double)x[i];
            v = s * hann64(j, nseg);
        }
        d[j] = v;
    }
    __syncthreads();
    f64_rfft<G64_T, G64_MAXE>(buf, rp);
    const int K = win / 2 + 1;
    for (int k = threadIdx.x; k < K; k += G64_T)
        S[(int64_t)f * K + k] = 20.0 * log10(fmax(hypot(buf[k].x, buf[k].y), 1e-12));
}
#endif
