// fft_lds.h — LDS-resident mixed-radix Stockham FFT (+ Bluestein) for gfx950,
// one workgroup per transform.
//
// The reference calls NumPy's pocketfft rfft/irfft at arbitrary lengths
// (MS:46, 66, 106, 122, 135, 153-163, 226-233, 432-435, 573-581).  A grain of
// up to ~40 k samples fits the 160 KiB LDS of one CU as n/2 packed complex
// float32, so a whole spectral chain runs with one HBM read and one HBM write.
//
// Each pass with radix R: every thread loads the R operands of its
// butterflies from LDS into registers, barrier, applies twiddles and a
// register-resident radix-R DFT (R in 2..25; composite radices are
// Cooley-Tukey in registers with compile-time constants), and stores to the
// Stockham autosort position, barrier — in place, no ping-pong buffer.
// Twiddle w^(k*stride) comes from a two-level table staged in LDS
// (tw(i) = T1[i>>7] * T0[i&127], float64-built); its powers w^r by a balanced
// product tree (depth <= 4).  Passes per length (host factorisation): 16384 ->
// 16,16,16,4; 18750 -> 25,25,5,6; 1200 -> 25,3,16.
#pragma once
#include "msg_common.h"

constexpr int FFT_MAXRAD = 16;
constexpr int TW_LO = 128;            // entries of the low-level twiddle table

struct FftDesc {
    int32_t m;            // complex transform length handled by the caller
    int32_t nrad;         // Stockham passes over `size`
    int32_t size;         // = m, or the power-of-two Bluestein length
    int32_t blue;         // 1 -> Bluestein (chirp-z) through `size`
    int32_t rad[FFT_MAXRAD];
    int32_t tw_hi_n;      // entries of the high-level table = ceil(size / 128)
    int32_t pad;
    const float2* tw0;    // exp(-2 pi i j / size), j < 128
    const float2* tw1;    // exp(-2 pi i 128 j / size), j < tw_hi_n
    const float2* chirp;  // Bluestein: exp(-pi i (j*j mod 2m) / m), j < m
    const float2* bspec;  // Bluestein: FFT_size of conj(chirp) wrapped
};

// Real-FFT plan for n samples.  even n: m = n/2 packed complex + post-twiddles;
// odd n: m = n complex with zero imaginary parts.
struct RealPlan {
    int32_t n;
    int32_t even;
    int32_t lds_c;        // complex slots of LDS for data
    int32_t lds_bytes;    // data + staged twiddle tables
    FftDesc c;
    const float2* rtw;    // even: exp(-2 pi i k / n), k <= n/2
};

MSG_DEV float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
MSG_DEV float2 cmulc(float2 a, float2 b) { return make_float2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y); } // a*conj(b)
MSG_DEV float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
MSG_DEV float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
MSG_DEV float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
MSG_DEV float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
template <bool INV> MSG_DEV float2 mul_mi(float2 a) { return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x); }

// ---- register-resident DFT kernels (forward sign -1, inverse +1), in place ----
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
template <int R, bool INV> struct DftOdd {   // odd prime radices, symmetric-pair form
    static MSG_DEV void run(float2* v) {
        constexpr int H = (R - 1) / 2;
        float2 a[H], b[H];
        const float2 x0 = v[0];
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
            float2 re = x0, im = make_float2(0.f, 0.f);
#pragma unroll
            for (int j = 1; j <= H; ++j) {
                const int jk = (j * k) % R;
                const float c = (float)__builtin_cos(2.0 * 3.14159265358979323846 * jk / R);
                const float s = (float)__builtin_sin(2.0 * 3.14159265358979323846 * jk / R);
                re = make_float2(fmaf(a[j - 1].x, c, re.x), fmaf(a[j - 1].y, c, re.y));
                im = make_float2(fmaf(b[j - 1].x, s, im.x), fmaf(b[j - 1].y, s, im.y));
            }
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

// Composite radix R1*R2 by Cooley-Tukey in registers: input n = R2*n1 + n2,
// output k = k1 + R1*k2.
template <int R1, int R2, bool INV> struct DftComp {
    static MSG_DEV void run(float2* v) {
        constexpr int N = R1 * R2;
        float2 a[R2][R1];
#pragma unroll
        for (int n2 = 0; n2 < R2; ++n2) {
#pragma unroll
            for (int n1 = 0; n1 < R1; ++n1) a[n2][n1] = v[R2 * n1 + n2];
            Dft<R1, INV>::run(a[n2]);
#pragma unroll
            for (int k1 = 1; k1 < R1; ++k1) {
                if (n2 == 0) continue;
                const int e = (n2 * k1) % N;
                const float c = (float)__builtin_cos(2.0 * 3.14159265358979323846 * e / N);
                const float s = (float)__builtin_sin(2.0 * 3.14159265358979323846 * e / N);
                a[n2][k1] = cmul(a[n2][k1], make_float2(c, INV ? s : -s));
            }
        }
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) {
            float2 b[R2];
#pragma unroll
            for (int n2 = 0; n2 < R2; ++n2) b[n2] = a[n2][k1];
            Dft<R2, INV>::run(b);
#pragma unroll
            for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = b[k2];
        }
    }
};
template <bool INV> struct Dft<6, INV> { static MSG_DEV void run(float2* v) { DftComp<2, 3, INV>::run(v); } };
template <bool INV> struct Dft<8, INV> { static MSG_DEV void run(float2* v) { DftComp<2, 4, INV>::run(v); } };
template <bool INV> struct Dft<9, INV> { static MSG_DEV void run(float2* v) { DftComp<3, 3, INV>::run(v); } };
template <bool INV> struct Dft<10, INV> { static MSG_DEV void run(float2* v) { DftComp<2, 5, INV>::run(v); } };
template <bool INV> struct Dft<12, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 3, INV>::run(v); } };
template <bool INV> struct Dft<15, INV> { static MSG_DEV void run(float2* v) { DftComp<3, 5, INV>::run(v); } };
template <bool INV> struct Dft<16, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 4, INV>::run(v); } };
template <bool INV> struct Dft<20, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 5, INV>::run(v); } };
template <bool INV> struct Dft<25, INV> { static MSG_DEV void run(float2* v) { DftComp<5, 5, INV>::run(v); } };

// Staged twiddle tables in LDS.
struct TwLds { const float2* t0; const float2* t1; };
MSG_DEV float2 tw_at(const TwLds& tw, int i) { return cmul(tw.t1[i >> 7], tw.t0[i & (TW_LO - 1)]); }

// floor(j / d) for 0 <= j < 2^24 via a float reciprocal plus one correction.
MSG_DEV int fdiv(int j, int d, float inv_d) {
    int q = (int)((float)j * inv_d);
    const int r = j - q * d;
    if (r < 0) --q; else if (r >= d) ++q;
    return q;
}

template <int R, int T, int MAXM, bool INV>
MSG_DEV void stockham_pass(float2* buf, int size, int Ns, const TwLds& tw) {
    constexpr int BMAX = (MAXM + R * T - 1) / (R * T);
    const int nb = size / R;
    const int stride = size / (Ns * R);
    const float inv_ns = 1.0f / (float)Ns;
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
            const int q = fdiv(j, Ns, inv_ns);
            const int k = j - q * Ns;
            if (k != 0) {
                float2 p[R];
                p[1] = tw_at(tw, k * stride);
#pragma unroll
                for (int r = 2; r < R; ++r) p[r] = cmul(p[r >> 1], p[r - (r >> 1)]);
#pragma unroll
                for (int r = 1; r < R; ++r) v[b][r] = INV ? cmulc(v[b][r], p[r]) : cmul(v[b][r], p[r]);
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
// Not inlined: one copy per (T, MAXM, INV) keeps code size and build time sane.
template <int T, int MAXM, bool INV>
MSG_NOINL void stockham(float2* buf, int size, const int32_t* rad, int nrad, const TwLds& tw) {
    int Ns = 1;
    for (int p = 0; p < nrad; ++p) {
        const int R = rad[p];
        switch (R) {
            case 2: stockham_pass<2, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 3: stockham_pass<3, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 4: stockham_pass<4, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 5: stockham_pass<5, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 6: stockham_pass<6, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 7: stockham_pass<7, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 8: stockham_pass<8, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 9: stockham_pass<9, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 10: stockham_pass<10, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 12: stockham_pass<12, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 15: stockham_pass<15, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 16: stockham_pass<16, T, MAXM, INV>(buf, size, Ns, tw); break;
            case 20: stockham_pass<20, T, MAXM, INV>(buf, size, Ns, tw); break;
            default: stockham_pass<25, T, MAXM, INV>(buf, size, Ns, tw); break;
        }
        Ns *= R;
    }
}

// Copy the plan's twiddle tables into LDS at `dst` (after the data region).
template <int T>
MSG_DEV TwLds stage_twiddles(float2* dst, const FftDesc& d) {
    for (int i = threadIdx.x; i < TW_LO; i += T) dst[i] = d.tw0[i];
    for (int i = threadIdx.x; i < d.tw_hi_n; i += T) dst[TW_LO + i] = d.tw1[i];
    __syncthreads();
    return TwLds{dst, dst + TW_LO};
}

// Complex DFT of length d.m in buf (Bluestein-aware).  Forward: exp(-2 pi i jk/m).
template <int T, int MAXM, bool INV>
MSG_DEV void cfft(float2* buf, const FftDesc& d, const TwLds& tw) {
    if (!d.blue) {
        stockham<T, MAXM, INV>(buf, d.size, d.rad, d.nrad, tw);
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
    stockham<T, MAXM, false>(buf, M, d.rad, d.nrad, tw);
    for (int j = (int)threadIdx.x; j < M; j += T) buf[j] = cmul(buf[j], d.bspec[j]);
    __syncthreads();
    stockham<T, MAXM, true>(buf, M, d.rad, d.nrad, tw);
    const float s = 1.0f / (float)M;
    for (int j = (int)threadIdx.x; j < m; j += T) {
        const float2 y = cscale(cmul(buf[j], d.chirp[j]), s);
        buf[j] = INV ? cconj(y) : y;
    }
    __syncthreads();
}

// ---- real transforms over the LDS buffer ----
// After rfft: X[k] at buf[k], k = 0 .. n/2 (even n) or (n-1)/2 (odd n).
// Real samples x[t]: ((float*)buf)[t] for even n, buf[t].x for odd n.
MSG_DEV float rx_get(const float2* buf, const RealPlan& rp, int t) {
    return rp.even ? reinterpret_cast<const float*>(buf)[t] : buf[t].x;
}
MSG_DEV void rx_set(float2* buf, const RealPlan& rp, int t, float v) {
    if (rp.even) reinterpret_cast<float*>(buf)[t] = v;
    else buf[t] = make_float2(v, 0.f);
}

template <int T, int MAXM>
MSG_DEV void rfft_lds(float2* buf, const RealPlan& rp, const TwLds& tw) {
    cfft<T, MAXM, false>(buf, rp.c, tw);
    if (!rp.even) return;
    const int m = rp.n / 2;
    // X[k] = E + W^k O ; E = (Z[k] + conj Z[m-k])/2 ; O = -i (Z[k] - conj Z[m-k])/2
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
        const float2 o1 = make_float2(0.5f * d1.y, -0.5f * d1.x);
        const float2 e2 = cscale(cadd(zm, cconj(zk)), 0.5f);
        const float2 d2 = csub(zm, cconj(zk));
        const float2 o2 = make_float2(0.5f * d2.y, -0.5f * d2.x);
        buf[k] = cadd(e1, cmul(rp.rtw[k], o1));
        buf[m - k] = cadd(e2, cmul(rp.rtw[m - k], o2));
    }
    __syncthreads();
}

// Inverse of rfft_lds with numpy.fft.irfft normalisation; the imaginary parts of
// the DC and (even n) Nyquist bins are ignored, as irfft does.
template <int T, int MAXM>
MSG_DEV void irfft_lds(float2* buf, const RealPlan& rp, const TwLds& tw) {
    const int n = rp.n;
    if (rp.even) {
        const int m = n / 2;
        for (int k = (int)threadIdx.x; k <= m / 2; k += T) {
            if (k == 0) {
                const float y0 = buf[0].x, ym = buf[m].x;
                buf[0] = make_float2(0.5f * (y0 + ym), 0.5f * (y0 - ym));
                continue;
            }
            const float2 yk = buf[k], ym = buf[m - k];
            // E = (Y[k] + conj Y[m-k])/2 ; O = conj(W^k) (Y[k] - conj Y[m-k])/2 ; Z = E + i O
            const float2 e1 = cscale(cadd(yk, cconj(ym)), 0.5f);
            const float2 o1 = cscale(cmulc(csub(yk, cconj(ym)), rp.rtw[k]), 0.5f);
            const float2 e2 = cscale(cadd(ym, cconj(yk)), 0.5f);
            const float2 o2 = cscale(cmulc(csub(ym, cconj(yk)), rp.rtw[m - k]), 0.5f);
            buf[k] = make_float2(e1.x - o1.y, e1.y + o1.x);
            buf[m - k] = make_float2(e2.x - o2.y, e2.y + o2.x);
        }
        __syncthreads();
        cfft<T, MAXM, true>(buf, rp.c, tw);
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
        cfft<T, MAXM, true>(buf, rp.c, tw);
        const float s = 1.0f / (float)n;
        for (int j = (int)threadIdx.x; j < n; j += T) buf[j] = make_float2(buf[j].x * s, 0.f);
        __syncthreads();
    }
}
