// fft64.h — float64 mixed-radix Stockham FFT (+ Bluestein) over an LDS
// buffer, one workgroup per transform: the engine of the float64 grain chain
// (kernels_grain64.h).
//
// Why float64: the reference's cepstral warp takes log(|X| + 1e-12)
// (MS:150-163).  Bins that are exactly zero in float64 (after the band-limit
// mask, or in the far tail of a Gaussian atom's spectrum) sit at the 1e-17
// rounding floor in NumPy and at the 1e-8 floor in float32, so the log
// spectrum — and with it the whole grain — diverges (0.11 RMS measured, SURVEY
// §0).  Partial-lock's top-k selection (MS:137) and the spectral imprint's
// phase (MS:580) are also decisions taken on float64 magnitudes.  Grains of
// presets that use those stages therefore run this engine end to end.
//
// Layout: the buffer holds complex double2 slots.  A real signal of n samples
// is kept as n contiguous doubles at the start of the buffer (the packed
// complex view of an even-length signal, so rfft needs no copy).
//
// Passes: radix R in {2,3,4,5,7,8,11,13,16}; each pass loads every operand of
// the thread's butterflies into registers, barrier, twiddle + register DFT,
// Stockham autosort store, barrier (in place, no ping-pong buffer).  Lengths
// with another prime factor run Bluestein through a power-of-two length.
// Twiddles come from float64 tables in global memory (L2-resident).
#pragma once
#include "msg_common.h"

constexpr int F64_MAXRAD = 20;

struct Fft64 {
    int32_t m;            // complex length of the transform
    int32_t size;         // m, or the power-of-two Bluestein length
    int32_t blue;         // 1 -> Bluestein through `size`
    int32_t nrad;         // Stockham passes over `size`
    int32_t rad[F64_MAXRAD];
    const double2* tw;    // exp(-2 pi i j / size), j < size
    const double2* chirp; // Bluestein: exp(-pi i (j*j mod 2m) / m), j < m
    const double2* bspec; // Bluestein: FFT_size(wrapped conj chirp) / size
};

// Real transform of n samples.  even n: packed m = n/2 complex + post-twiddles;
// odd n: m = n complex with zero imaginary parts.
struct Real64Plan {
    int32_t n;
    int32_t even;
    int32_t cap;          // complex slots of buffer the grain chain needs
    int32_t pad;
    Fft64 c;
    const double2* rt;    // even n: exp(-2 pi i k / n), k <= n/2
};

#if defined(__HIPCC__)
MSG_DEV double2 d2(double x, double y) { double2 r; r.x = x; r.y = y; return r; }
MSG_DEV double2 dadd(double2 a, double2 b) { return d2(a.x + b.x, a.y + b.y); }
MSG_DEV double2 dsub(double2 a, double2 b) { return d2(a.x - b.x, a.y - b.y); }
MSG_DEV double2 dmul(double2 a, double2 b) { return d2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
MSG_DEV double2 dconj(double2 a) { return d2(a.x, -a.y); }
MSG_DEV double2 dscale(double2 a, double s) { return d2(a.x * s, a.y * s); }
template <bool INV> MSG_DEV double2 dmul_mi(double2 a) { return INV ? d2(-a.y, a.x) : d2(a.y, -a.x); }

// a * exp(-+2 pi i e / N) for a compile-time e (after unrolling)
template <bool INV> MSG_DEV double2 dtwc(double2 a, int e, int N) {
    e %= N;
    if (e == 0) return a;
    if (4 * e == N) return dmul_mi<INV>(a);
    if (2 * e == N) return d2(-a.x, -a.y);
    if (4 * e == 3 * N) return dmul_mi<!INV>(a);
    const double c = __builtin_cos(2.0 * 3.14159265358979323846 * e / N);
    const double s = __builtin_sin(2.0 * 3.14159265358979323846 * e / N);
    return dmul(a, d2(c, INV ? s : -s));
}

// ---- register DFTs (forward sign -1, inverse +1), in place ----
template <int R, bool INV> struct D64;
template <bool INV> struct D64<2, INV> {
    static MSG_DEV void run(double2* v) { const double2 a = v[0], b = v[1]; v[0] = dadd(a, b); v[1] = dsub(a, b); }
};
template <bool INV> struct D64<4, INV> {
    static MSG_DEV void run(double2* v) {
        const double2 a0 = dadd(v[0], v[2]), a1 = dsub(v[0], v[2]);
        const double2 b0 = dadd(v[1], v[3]), b1 = dmul_mi<INV>(dsub(v[1], v[3]));
        v[0] = dadd(a0, b0); v[2] = dsub(a0, b0);
        v[1] = dadd(a1, b1); v[3] = dsub(a1, b1);
    }
};
// odd radices, symmetric-pair form (constants folded after unrolling)
template <int R, bool INV> struct D64Odd {
    static MSG_DEV void run(double2* v) {
        constexpr int H = (R - 1) / 2;
        double2 a[H], b[H];
        const double2 x0 = v[0];
        double2 s0 = x0;
#pragma unroll
        for (int j = 1; j <= H; ++j) {
            a[j - 1] = dadd(v[j], v[R - j]);
            b[j - 1] = dsub(v[j], v[R - j]);
            s0 = dadd(s0, a[j - 1]);
        }
        double2 out[R];
        out[0] = s0;
#pragma unroll
        for (int k = 1; k <= H; ++k) {
            double2 re = x0, im = d2(0.0, 0.0);
#pragma unroll
            for (int j = 1; j <= H; ++j) {
                const int jk = (j * k) % R;
                const double c = __builtin_cos(2.0 * 3.14159265358979323846 * jk / R);
                const double s = __builtin_sin(2.0 * 3.14159265358979323846 * jk / R);
                re = d2(a[j - 1].x * c + re.x, a[j - 1].y * c + re.y);
                im = d2(b[j - 1].x * s + im.x, b[j - 1].y * s + im.y);
            }
            const double2 t = INV ? d2(-im.y, im.x) : d2(im.y, -im.x);
            out[k] = dadd(re, t);
            out[R - k] = dsub(re, t);
        }
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = out[k];
    }
};
template <bool INV> struct D64<3, INV> { static MSG_DEV void run(double2* v) { D64Odd<3, INV>::run(v); } };
template <bool INV> struct D64<5, INV> { static MSG_DEV void run(double2* v) { D64Odd<5, INV>::run(v); } };
template <bool INV> struct D64<7, INV> { static MSG_DEV void run(double2* v) { D64Odd<7, INV>::run(v); } };
template <bool INV> struct D64<11, INV> { static MSG_DEV void run(double2* v) { D64Odd<11, INV>::run(v); } };
template <bool INV> struct D64<13, INV> { static MSG_DEV void run(double2* v) { D64Odd<13, INV>::run(v); } };
// R = R1 * R2 in registers: inner DFT_R1 over x[R2 n1 + n2], twiddle W_R^(n2 k1),
// outer DFT_R2 -> X[k1 + R1 k2]
template <int R1, int R2, bool INV> struct D64Comp {
    static MSG_DEV void run(double2* v) {
        constexpr int R = R1 * R2;
        double2 t[R];
#pragma unroll
        for (int n2 = 0; n2 < R2; ++n2) {
            double2 u[R1];
#pragma unroll
            for (int n1 = 0; n1 < R1; ++n1) u[n1] = v[R2 * n1 + n2];
            D64<R1, INV>::run(u);
#pragma unroll
            for (int k1 = 0; k1 < R1; ++k1) t[n2 * R1 + k1] = dtwc<INV>(u[k1], n2 * k1, R);
        }
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) {
            double2 u[R2];
#pragma unroll
            for (int n2 = 0; n2 < R2; ++n2) u[n2] = t[n2 * R1 + k1];
            D64<R2, INV>::run(u);
#pragma unroll
            for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = u[k2];
        }
    }
};
template <bool INV> struct D64<8, INV> { static MSG_DEV void run(double2* v) { D64Comp<4, 2, INV>::run(v); } };
template <bool INV> struct D64<16, INV> { static MSG_DEV void run(double2* v) { D64Comp<4, 4, INV>::run(v); } };

// One Stockham pass of radix R over buf[0..N), Ns = product of the earlier
// radices.  Butterfly idx (< N/R) reads buf[idx + q N/R], multiplies operand q
// by W_{Ns R}^(j q) (j = idx mod Ns), and stores DFT_R to
// buf[(idx - j) R + j + q Ns].  MAXE bounds N / T.
template <int R, bool INV, int T, int MAXE>
MSG_DEV void f64_pass(double2* buf, int N, int Ns, const double2* __restrict__ tw) {
    constexpr int B = (MAXE + R - 1) / R;
    const int nb = N / R;
    const int mul = N / (Ns * R);
    const int tid = threadIdx.x;
    double2 v[B][R];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int idx = tid + b * T;
        if (idx < nb) {
            const int j = idx % Ns;
#pragma unroll
            for (int q = 0; q < R; ++q) v[b][q] = buf[idx + q * nb];
            if (Ns > 1) {
#pragma unroll
                for (int q = 1; q < R; ++q) {
                    double2 w = tw[j * q * mul];
                    if (INV) w.y = -w.y;
                    v[b][q] = dmul(v[b][q], w);
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int idx = tid + b * T;
        if (idx < nb) {
            D64<R, INV>::run(v[b]);
            const int j = idx % Ns;
            const int base = (idx - j) * R + j;
#pragma unroll
            for (int q = 0; q < R; ++q) buf[base + q * Ns] = v[b][q];
        }
    }
    __syncthreads();
}

// Global-memory variant of one pass (grains beyond the LDS engine): reads
// src, writes dst (ping-pong), any number of butterflies per thread.
template <int R, bool INV, int T>
MSG_DEV void f64_pass_ping(const double2* src, double2* dst, int N, int Ns, const double2* __restrict__ tw) {
    const int nb = N / R;
    const int mul = N / (Ns * R);
    for (int idx = threadIdx.x; idx < nb; idx += T) {
        const int j = idx % Ns;
        double2 v[R];
#pragma unroll
        for (int q = 0; q < R; ++q) v[q] = src[idx + q * nb];
        if (Ns > 1) {
#pragma unroll
            for (int q = 1; q < R; ++q) {
                double2 w = tw[(int64_t)j * q * mul];
                if (INV) w.y = -w.y;
                v[q] = dmul(v[q], w);
            }
        }
        D64<R, INV>::run(v);
        const int base = (idx - j) * R + j;
#pragma unroll
        for (int q = 0; q < R; ++q) dst[base + q * Ns] = v[q];
    }
    __syncthreads();
}

// Unscaled DFT of buf[0..p.size) through the radix plan.  scr == nullptr:
// in place through registers (LDS buffers, MAXE >= size / T); otherwise
// ping-pong through the global scratch scr (same size), result back in buf.
template <bool INV, int T, int MAXE>
MSG_DEV void f64_stockham(double2* buf, const Fft64& p, double2* scr = nullptr) {
    __syncthreads();
    const int N = p.size;
    int Ns = 1;
    if (scr) {
        double2* src = buf;
        double2* dst = scr;
        for (int s = 0; s < p.nrad; ++s) {
            const int R = p.rad[s];
            switch (R) {
                case 2: f64_pass_ping<2, INV, T>(src, dst, N, Ns, p.tw); break;
                case 3: f64_pass_ping<3, INV, T>(src, dst, N, Ns, p.tw); break;
                case 4: f64_pass_ping<4, INV, T>(src, dst, N, Ns, p.tw); break;
                case 5: f64_pass_ping<5, INV, T>(src, dst, N, Ns, p.tw); break;
                case 7: f64_pass_ping<7, INV, T>(src, dst, N, Ns, p.tw); break;
                case 8: f64_pass_ping<8, INV, T>(src, dst, N, Ns, p.tw); break;
                case 11: f64_pass_ping<11, INV, T>(src, dst, N, Ns, p.tw); break;
                case 13: f64_pass_ping<13, INV, T>(src, dst, N, Ns, p.tw); break;
                default: f64_pass_ping<16, INV, T>(src, dst, N, Ns, p.tw); break;
            }
            Ns *= R;
            double2* t = src; src = dst; dst = t;
        }
        if (src != buf) {
            for (int j = threadIdx.x; j < N; j += T) buf[j] = src[j];
            __syncthreads();
        }
        return;
    }
    for (int s = 0; s < p.nrad; ++s) {
        const int R = p.rad[s];
        switch (R) {
            case 2: f64_pass<2, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 3: f64_pass<3, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 4: f64_pass<4, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 5: f64_pass<5, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 7: f64_pass<7, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 8: f64_pass<8, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 11: f64_pass<11, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            case 13: f64_pass<13, INV, T, MAXE>(buf, N, Ns, p.tw); break;
            default: f64_pass<16, INV, T, MAXE>(buf, N, Ns, p.tw); break;
        }
        Ns *= R;
    }
}

// Unscaled complex DFT of length p.m in place (Bluestein when p.blue).
// Ends with a barrier.
template <bool INV, int T, int MAXE>
MSG_DEV void f64_cfft(double2* buf, const Fft64& p, double2* scr = nullptr) {
    if (!p.blue) { f64_stockham<INV, T, MAXE>(buf, p, scr); return; }
    const int m = p.m, M = p.size;
    const int tid = threadIdx.x;
    __syncthreads();
    // a_j = x_j w_j (inverse: conj in, conj out), zero padded to M
    for (int j = tid; j < M; j += T) {
        double2 a = d2(0.0, 0.0);
        if (j < m) {
            a = buf[j];
            if (INV) a.y = -a.y;
            a = dmul(a, p.chirp[j]);
        }
        buf[j] = a;
    }
    f64_stockham<false, T, MAXE>(buf, p, scr);
    for (int j = tid; j < M; j += T) buf[j] = dmul(buf[j], p.bspec[j]);
    f64_stockham<true, T, MAXE>(buf, p, scr);
    for (int k = tid; k < m; k += T) {
        double2 a = dmul(buf[k], p.chirp[k]);
        if (INV) a.y = -a.y;
        buf[k] = a;
    }
    __syncthreads();
}

// Real samples d[0..n) (contiguous doubles) <-> complex slots (x, 0), via
// registers (LDS) or through the global scratch scr.
template <int T, int MAXE>
MSG_DEV void f64_real_to_complex(double2* buf, int n, double2* scr = nullptr) {
    const double* d = reinterpret_cast<const double*>(buf);
    __syncthreads();
    if (scr) {
        double* sd = reinterpret_cast<double*>(scr);
        for (int j = threadIdx.x; j < n; j += T) sd[j] = d[j];
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += T) buf[j] = d2(sd[j], 0.0);
        __syncthreads();
        return;
    }
    double v[MAXE];
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
        const int j = threadIdx.x + i * T;
        v[i] = j < n ? d[j] : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
        const int j = threadIdx.x + i * T;
        if (j < n) buf[j] = d2(v[i], 0.0);
    }
    __syncthreads();
}
template <int T, int MAXE>
MSG_DEV void f64_complex_to_real(double2* buf, int n, double scale, double2* scr = nullptr) {
    double* d = reinterpret_cast<double*>(buf);
    __syncthreads();
    if (scr) {
        double* sd = reinterpret_cast<double*>(scr);
        for (int j = threadIdx.x; j < n; j += T) sd[j] = buf[j].x * scale;
        __syncthreads();
        for (int j = threadIdx.x; j < n; j += T) d[j] = sd[j];
        __syncthreads();
        return;
    }
    double v[MAXE];
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
        const int j = threadIdx.x + i * T;
        v[i] = j < n ? buf[j].x * scale : 0.0;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
        const int j = threadIdx.x + i * T;
        if (j < n) d[j] = v[i];
    }
    __syncthreads();
}

// np.fft.rfft: real d[0..n) -> X[0..n/2] in buf.  Ends with a barrier.
template <int T, int MAXE>
MSG_DEV void f64_rfft(double2* buf, const Real64Plan& rp, double2* scr = nullptr) {
    const int n = rp.n;
    if (!rp.even) {
        f64_real_to_complex<T, MAXE>(buf, n, scr);
        f64_cfft<false, T, MAXE>(buf, rp.c, scr);
        return;
    }
    f64_cfft<false, T, MAXE>(buf, rp.c, scr);   // packed z_j = x_2j + i x_2j+1, m = n/2
    const int m = n / 2;
    for (int k = threadIdx.x; k <= m / 2; k += T) {
        if (k == 0) {
            const double2 z = buf[0];
            buf[0] = d2(z.x + z.y, 0.0);
            buf[m] = d2(z.x - z.y, 0.0);
            continue;
        }
        const int k2 = m - k;
        const double2 A = buf[k], Bv = buf[k2];
        // X[k] = E + W^k O, E = (Z_k + conj Z_{m-k}) / 2, O = (Z_k - conj Z_{m-k}) / 2i
        auto post = [&](double2 a, double2 b, int kk) {
            const double2 c = dconj(b);
            const double2 e = dscale(dadd(a, c), 0.5);
            const double2 df = dsub(a, c);
            const double2 o = d2(0.5 * df.y, -0.5 * df.x);
            return dadd(e, dmul(rp.rt[kk], o));
        };
        const double2 Xk = post(A, Bv, k);
        const double2 Xk2 = post(Bv, A, k2);
        buf[k] = Xk;
        if (k2 != k) buf[k2] = Xk2;
    }
    __syncthreads();
}

// np.fft.irfft(X, n): X[0..n/2] in buf -> real d[0..n).  The imaginary parts
// of X[0] (and X[n/2] for even n) are ignored, as pocketfft's c2r does.
template <int T, int MAXE>
MSG_DEV void f64_irfft(double2* buf, const Real64Plan& rp, double2* scr = nullptr) {
    const int n = rp.n;
    __syncthreads();
    if (!rp.even) {
        const int K = (n + 1) / 2;
        for (int k = threadIdx.x; k < K; k += T) {
            if (k == 0) buf[0].y = 0.0;
            else buf[n - k] = dconj(buf[k]);
        }
        f64_cfft<true, T, MAXE>(buf, rp.c, scr);
        f64_complex_to_real<T, MAXE>(buf, n, 1.0 / (double)n, scr);
        return;
    }
    const int m = n / 2;
    for (int k = threadIdx.x; k <= m / 2; k += T) {
        if (k == 0) {
            const double a = buf[0].x, b = buf[m].x;
            buf[0] = d2(0.5 * (a + b), 0.5 * (a - b));
            continue;
        }
        const int k2 = m - k;
        const double2 A = buf[k], Bv = buf[k2];
        // Z_k = E_k + i O_k, E = (X_k + conj X_{m-k}) / 2, O = (X_k - conj X_{m-k}) conj(W^k) / 2
        auto pre = [&](double2 a, double2 b, int kk) {
            const double2 c = dconj(b);
            const double2 e = dscale(dadd(a, c), 0.5);
            const double2 o = dscale(dmul(dsub(a, c), dconj(rp.rt[kk])), 0.5);
            return d2(e.x - o.y, e.y + o.x);
        };
        const double2 Zk = pre(A, Bv, k);
        const double2 Zk2 = pre(Bv, A, k2);
        buf[k] = Zk;
        if (k2 != k) buf[k2] = Zk2;
    }
    f64_cfft<true, T, MAXE>(buf, rp.c, scr);
    const double s = 1.0 / (double)m;
    double* d = reinterpret_cast<double*>(buf);
    for (int j = threadIdx.x; j < n; j += T) d[j] *= s;
    __syncthreads();
}
#endif  // __HIPCC__

// ---------------------------------------------------------------------------
// Host-side plan tables (float64, long-double built).
// ---------------------------------------------------------------------------
#include <cmath>
#include <vector>

namespace fft64plan {

// Radices 16, 8, 4, 2 first, then 3, 5, 7, 11, 13; false if another prime divides m.
inline bool factor(int m, std::vector<int>& rad) {
    rad.clear();
    int r = m;
    for (int p : {16, 8, 4, 2, 3, 5, 7, 11, 13})
        while (r % p == 0) { rad.push_back(p); r /= p; }
    return r == 1;
}

inline int next_pow2(int v) { int p = 1; while (p < v) p <<= 1; return p; }

inline void twiddles(int N, std::vector<double>& out) {
    out.resize(2 * (size_t)N);
    for (int j = 0; j < N; ++j) {
        const long double a = -2.0L * 3.14159265358979323846264338327950288L * (long double)j / (long double)N;
        out[2 * j] = (double)cosl(a);
        out[2 * j + 1] = (double)sinl(a);
    }
}

inline void chirp(int m, std::vector<double>& out) {
    out.resize(2 * (size_t)m);
    for (int j = 0; j < m; ++j) {
        const long long q = ((long long)j * j) % (2LL * m);
        const long double a = -3.14159265358979323846264338327950288L * (long double)q / (long double)m;
        out[2 * j] = (double)cosl(a);
        out[2 * j + 1] = (double)sinl(a);
    }
}

// B = FFT_M(b) / M with b_l = conj(w_l) for |l| < m wrapped mod M (direct
// long-double DFT through a radix-2 recursion on the host).
inline void bluestein_spec(int m, int M, const std::vector<double>& w, std::vector<double>& out) {
    std::vector<long double> re(M, 0.0L), im(M, 0.0L);
    for (int l = 0; l < m; ++l) {
        re[l] = w[2 * l]; im[l] = -w[2 * l + 1];
        if (l > 0) { re[M - l] = w[2 * l]; im[M - l] = -w[2 * l + 1]; }
    }
    // iterative radix-2 DIT FFT in long double
    int lg = 0; while ((1 << lg) < M) ++lg;
    for (int i = 0; i < M; ++i) {
        int r = 0;
        for (int b = 0; b < lg; ++b) if (i & (1 << b)) r |= 1 << (lg - 1 - b);
        if (r > i) { std::swap(re[i], re[r]); std::swap(im[i], im[r]); }
    }
    const long double PI = 3.14159265358979323846264338327950288L;
    for (int len = 2; len <= M; len <<= 1) {
        for (int i = 0; i < M; i += len)
            for (int k = 0; k < len / 2; ++k) {
                const long double a = -2.0L * PI * k / len;
                const long double wr = cosl(a), wi = sinl(a);
                const long double xr = re[i + k + len / 2] * wr - im[i + k + len / 2] * wi;
                const long double xi = re[i + k + len / 2] * wi + im[i + k + len / 2] * wr;
                re[i + k + len / 2] = re[i + k] - xr; im[i + k + len / 2] = im[i + k] - xi;
                re[i + k] += xr; im[i + k] += xi;
            }
    }
    out.resize(2 * (size_t)M);
    for (int k = 0; k < M; ++k) { out[2 * k] = (double)(re[k] / M); out[2 * k + 1] = (double)(im[k] / M); }
}

}  // namespace fft64plan
