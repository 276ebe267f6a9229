// fft_lds.h — LDS-resident mixed-radix (2,3,4,5,7,8) Stockham FFT + Bluestein,
// one workgroup per transform, for gfx950.
//
// The reference calls NumPy's pocketfft rfft/irfft at arbitrary lengths
// (MS:46, 66, 106, 122, 135, 153-163, 226-233, 432-435, 573-581).  A grain of
// up to ~40 k samples fits the 160 KiB LDS of one CU as n/2 packed complex
// float32, so the whole spectral chain of one grain runs without touching HBM
// between passes.  Each pass: every thread loads all operands of its
// butterflies into registers, barrier, twiddle + radix-R DFT, store in the
// Stockham autosort position, barrier (in-place, no ping-pong buffer).
// Twiddles come from a per-size float32 table (L2-resident) computed in
// float64 on the host.
#pragma once
#include "msg_common.h"

struct FftDesc {
    int32_t m;            // complex transform length handled by the caller
    int32_t nrad;         // Stockham passes over `size`
    int32_t size;         // = m, or the power-of-two Bluestein length
    int32_t blue;         // 1 -> Bluestein (chirp-z) through `size`
    int32_t rad[24];
    const float2* tw;     // tw[j] = exp(-2*pi*i*j/size), j < size
    const float2* chirp;  // Bluestein: exp(-pi*i*(j*j mod 2m)/m), j < m
    const float2* bspec;  // Bluestein: FFT_size of conj(chirp) wrapped
};

// Real-FFT plan: n real samples.  even n: m = n/2 packed complex + post-twiddles;
// odd n: m = n complex with zero imaginary parts.
struct RealPlan {
    int32_t n;
    int32_t even;
    int32_t lds_c;        // complex slots of LDS the transform needs
    int32_t pad;
    FftDesc c;
    const float2* rtw;    // even: rtw[k] = exp(-2*pi*i*k/n), k <= n/2
};

MSG_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
MSG_DEV float2 cmulc(float2 a, float2 b) { return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y); } // a*conj(b)
MSG_DEV float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
MSG_DEV float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
MSG_DEV float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
MSG_DEV float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// multiply by -i (forward) or +i (inverse)
template <bool INV> MSG_DEV float2 mul_mi(float2 a) { return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x); }

// ---- radix-R DFT kernels (sign -1 forward, +1 inverse) ----
template <int R, bool INV> struct Dft;

template <bool INV> struct Dft<2, INV> {
    static MSG_DEV void run(float2* v) { float2 a = v[0], b = v[1]; v[0] = cadd(a, b); v[1] = csub(a, b); }
};
template <bool INV> struct Dft<4, INV> {
    static MSG_DEV void run(float2* v) {
        float2 a0 = cadd(v[0], v[2]), a1 = csub(v[0], v[2]);
        float2 b0 = cadd(v[1], v[3]), b1 = mul_mi<INV>(csub(v[1], v[3]));
        v[0] = cadd(a0, b0); v[2] = csub(a0, b0);
        v[1] = cadd(a1, b1); v[3] = csub(a1, b1);
    }
};
template <bool INV> struct Dft<8, INV> {
    static MSG_DEV void run(float2* v) {
        const float r = 0.70710678118654752440f;
        float2 e[4] = {v[0], v[2], v[4], v[6]};
        float2 o[4] = {v[1], v[3], v[5], v[7]};
        Dft<4, INV>::run(e);
        Dft<4, INV>::run(o);
        // o[k] *= w8^k, w8 = exp(-+ i pi/4)
        float2 o1 = INV ? make_float2(r * (o[1].x - o[1].y), r * (o[1].x + o[1].y))
                        : make_float2(r * (o[1].x + o[1].y), r * (o[1].y - o[1].x));
        float2 o2 = mul_mi<INV>(o[2]);
        float2 o3 = INV ? make_float2(-r * (o[3].x + o[3].y), r * (o[3].x - o[3].y))
                        : make_float2(r * (o[3].y - o[3].x), -r * (o[3].x + o[3].y));
        v[0] = cadd(e[0], o[0]); v[4] = csub(e[0], o[0]);
        v[1] = cadd(e[1], o1);   v[5] = csub(e[1], o1);
        v[2] = cadd(e[2], o2);   v[6] = csub(e[2], o2);
        v[3] = cadd(e[3], o3);   v[7] = csub(e[3], o3);
    }
};
// odd prime radices via the symmetric-pair form
template <int R, bool INV> struct DftOdd {
    static MSG_DEV void run(float2* v) {
        constexpr int H = (R - 1) / 2;
        float2 a[H], b[H];
        float2 x0 = v[0];
        float2 s0 = x0;
#pragma unroll
        for (int j = 1; j <= H; ++j) {
            a[j - 1] = cadd(v[j], v[R - j]);
            b[j - 1] = csub(v[j], v[R - j]);
            s0 = cadd(s0, a[j - 1]);
        }
        float2 out[R];
        out[0] = s0;
#pragma unroll
        for (int k = 1; k <= H; ++k) {
            float2 re = x0;
            float2 im = make_float2(0.f, 0.f);
#pragma unroll
            for (int j = 1; j <= H; ++j) {
                const int jk = (j * k) % R;
                const float c = (float)__builtin_cos(2.0 * 3.14159265358979323846 * jk / R);
                const float s = (float)__builtin_sin(2.0 * 3.14159265358979323846 * jk / R);
                re = make_float2(re.x + a[j - 1].x * c, re.y + a[j - 1].y * c);
                im = make_float2(im.x + b[j - 1].x * s, im.y + b[j - 1].y * s);
            }
            // X[k] = re - i*sgn*im ; X[R-k] = re + i*sgn*im   (sgn = +1 forward)
            const float2 t = INV ? make_float2(-im.y, im.x) : make_float2(im.y, -im.x);
            out[k] = cadd(re, t);
            out[R - k] = csub(re, t);
        }
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = out[k];
    }
};
template <bool INV> struct Dft<3, INV> { static MSG_DEV void run(float2* v) { DftOdd<3, INV>::run(v); } };
template <bool INV> struct Dft<5, INV> { static MSG_DEV void run(float2* v) { DftOdd<5, INV>::run(v); } };
template <bool INV> struct Dft<7, INV> { static MSG_DEV void run(float2* v) { DftOdd<7, INV>::run(v); } };

// One Stockham pass of radix R over buf[0..size), Ns = product of earlier radices.
template <int R, int T, int MAXC, bool INV>
MSG_DEV void stockham_pass(float2* buf, int size, int Ns, const float2* __restrict__ tw) {
    constexpr int BMAX = (MAXC + R * T - 1) / (R * T);
    const int nb = size / R;
    const int stride = size / (Ns * R);
    float2 v[BMAX][R];
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
        const int j = (int)threadIdx.x + b * T;
        if (j < nb) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = buf[j + r * nb];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
        const int j = (int)threadIdx.x + b * T;
        if (j < nb) {
            const int q = j / Ns;
            const int k = j - q * Ns;
            if (Ns > 1) {
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    const float2 w = tw[r * k * stride];
                    v[b][r] = INV ? cmulc(v[b][r], w) : cmul(v[b][r], w);
                }
            }
            Dft<R, INV>::run(v[b]);
            const int base = q * Ns * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) buf[base + r * Ns] = v[b][r];
        }
    }
    __syncthreads();
}

// Unnormalised complex DFT of buf[0..size) by the plan's radix sequence.
template <int T, int MAXC, bool INV>
MSG_DEV void stockham(float2* buf, int size, const int32_t* rad, int nrad, const float2* tw) {
    int Ns = 1;
    for (int p = 0; p < nrad; ++p) {
        const int R = rad[p];
        switch (R) {
            case 2: stockham_pass<2, T, MAXC, INV>(buf, size, Ns, tw); break;
            case 3: stockham_pass<3, T, MAXC, INV>(buf, size, Ns, tw); break;
            case 4: stockham_pass<4, T, MAXC, INV>(buf, size, Ns, tw); break;
            case 5: stockham_pass<5, T, MAXC, INV>(buf, size, Ns, tw); break;
            case 7: stockham_pass<7, T, MAXC, INV>(buf, size, Ns, tw); break;
            default: stockham_pass<8, T, MAXC, INV>(buf, size, Ns, tw); break;
        }
        Ns *= R;
    }
}

// Complex DFT of length d.m in buf (Bluestein-aware).  Forward uses exp(-2*pi*i jk/m).
template <int T, int MAXC, bool INV>
MSG_DEV void cfft(float2* buf, const FftDesc& d) {
    if (!d.blue) {
        stockham<T, MAXC, INV>(buf, d.size, d.rad, d.nrad, d.tw);
        return;
    }
    // Bluestein: X = chirp . IFFT_M( FFT_M(x . chirp) . B ) / M ; inverse via conjugation.
    const int m = d.m, M = d.size;
    for (int j = (int)threadIdx.x; j < M; j += T) {
        float2 x = j < m ? buf[j] : make_float2(0.f, 0.f);
        if (INV) x = cconj(x);
        buf[j] = j < m ? cmul(x, d.chirp[j]) : x;
    }
    __syncthreads();
    stockham<T, MAXC, false>(buf, M, d.rad, d.nrad, d.tw);
    for (int j = (int)threadIdx.x; j < M; j += T) buf[j] = cmul(buf[j], d.bspec[j]);
    __syncthreads();
    stockham<T, MAXC, true>(buf, M, d.rad, d.nrad, d.tw);
    const float s = 1.0f / (float)M;
    for (int j = (int)threadIdx.x; j < m; j += T) {
        float2 y = cscale(cmul(buf[j], d.chirp[j]), s);
        buf[j] = INV ? cconj(y) : y;
    }
    __syncthreads();
}

// ---- real transforms over the LDS buffer ----
// Layout after rfft: spectrum X[k] at buf[k], k = 0 .. n/2 (n even) or (n-1)/2 (n odd).
// Input of rfft / output of irfft: real x[t] at ((float*)buf)[t] for even n,
// at buf[t].x for odd n.
MSG_DEV int rspec_bins(const RealPlan& rp) { return rp.n / 2 + 1; }
MSG_DEV float rx_get(const float2* buf, const RealPlan& rp, int t) {
    return rp.even ? reinterpret_cast<const float*>(buf)[t] : buf[t].x;
}
MSG_DEV void rx_set(float2* buf, const RealPlan& rp, int t, float v) {
    if (rp.even) reinterpret_cast<float*>(buf)[t] = v;
    else buf[t] = make_float2(v, 0.f);
}

template <int T, int MAXC>
MSG_DEV void rfft_lds(float2* buf, const RealPlan& rp) {
    cfft<T, MAXC, false>(buf, rp.c);
    if (!rp.even) return;
    const int m = rp.n / 2;
    // X[k] = E + W^k O, E = (Z[k] + conj Z[m-k])/2, O = -i (Z[k] - conj Z[m-k])/2
    for (int k = (int)threadIdx.x; k <= m / 2; k += T) {
        if (k == 0) {
            const float2 z0 = buf[0];
            buf[0] = make_float2(z0.x + z0.y, 0.f);
            buf[m] = make_float2(z0.x - z0.y, 0.f);
            continue;
        }
        const float2 zk = buf[k], zm = buf[m - k];
        const float2 e1 = cscale(cadd(zk, cconj(zm)), 0.5f);
        const float2 d1 = csub(zk, cconj(zm));
        const float2 o1 = make_float2(0.5f * d1.y, -0.5f * d1.x);       // -i*d/2
        const float2 xk = cadd(e1, cmul(rp.rtw[k], o1));
        // partner bin m-k: E' = conj(e1), O' = conj(o1)*(-1)?  compute directly
        const float2 e2 = cscale(cadd(zm, cconj(zk)), 0.5f);
        const float2 d2 = csub(zm, cconj(zk));
        const float2 o2 = make_float2(0.5f * d2.y, -0.5f * d2.x);
        const float2 xm = cadd(e2, cmul(rp.rtw[m - k], o2));
        buf[k] = xk;
        buf[m - k] = xm;
    }
    __syncthreads();
}

// Inverse of rfft_lds, normalised like numpy.fft.irfft (imaginary parts of the
// DC and Nyquist bins are ignored, as irfft does).
template <int T, int MAXC>
MSG_DEV void irfft_lds(float2* buf, const RealPlan& rp) {
    const int n = rp.n;
    if (rp.even) {
        const int m = n / 2;
        for (int k = (int)threadIdx.x; k <= m / 2; k += T) {
            if (k == 0) {
                const float y0 = buf[0].x, ym = buf[m].x;
                // E0 = (y0+ym)/2, O0 = (y0-ym)/2 -> Z0 = E0 + i O0
                buf[0] = make_float2(0.5f * (y0 + ym), 0.5f * (y0 - ym));
                continue;
            }
            const float2 yk = buf[k], ym = buf[m - k];
            // E = (Y[k] + conj Y[m-k])/2 ; O = conj(W^k) (Y[k] - conj Y[m-k])/2 ; Z = E + i O
            const float2 e1 = cscale(cadd(yk, cconj(ym)), 0.5f);
            const float2 o1 = cscale(cmulc(csub(yk, cconj(ym)), rp.rtw[k]), 0.5f);
            const float2 zk = make_float2(e1.x - o1.y, e1.y + o1.x);
            const float2 e2 = cscale(cadd(ym, cconj(yk)), 0.5f);
            const float2 o2 = cscale(cmulc(csub(ym, cconj(yk)), rp.rtw[m - k]), 0.5f);
            const float2 zm = make_float2(e2.x - o2.y, e2.y + o2.x);
            buf[k] = zk;
            buf[m - k] = zm;
        }
        __syncthreads();
        cfft<T, MAXC, true>(buf, rp.c);
        const float s = 1.0f / (float)m;
        for (int j = (int)threadIdx.x; j < m; j += T) buf[j] = cscale(buf[j], s);
        __syncthreads();
    } else {
        const int K = (n + 1) / 2;
        for (int k = (int)threadIdx.x; k < K; k += T) {
            if (k == 0) { buf[0].y = 0.f; continue; }
            buf[n - k] = cconj(buf[k]);
        }
        __syncthreads();
        cfft<T, MAXC, true>(buf, rp.c);
        const float s = 1.0f / (float)n;
        for (int j = (int)threadIdx.x; j < n; j += T) buf[j] = make_float2(buf[j].x * s, 0.f);
        __syncthreads();
    }
}
