// kernels_stereo_odd.h — spectral stereo rotation of an odd-length output
// (TU: k_stereo_odd.hip).
//
// spectral_diffusion_stereo (MS:423-436) rotates the phase of the full-length
// rfft of R = roll(x, -dr) by exp(i 0.9w sin(2 pi k / K)), K = n // 2.  For even
// n that is exactly a 25-tap circular FIR (kernels_core.h).  For odd n the
// rotation is a fractional-shift operator, so the transform is done: an
// n-point DFT by Bluestein through a power-of-two length M >= 2n - 1, each
// M-point FFT in four steps (M = M1 x M2, M1 <= 2048 column transforms of
// strided data, M2 <= 4096 row transforms of contiguous data) with the chirp
// convolution's pointwise product fused between the forward and inverse row
// transforms, and no transposes (the kernel spectrum is kept in the same
// permuted order).  Above M = 2^23 (odd outputs longer than 4 194 304 frames,
// e.g. 95 s at 44.1 kHz) one more column level splits M = M0 x L, L = M1 x M2:
// column transforms of length M0 over stride L with the W_M twiddle, then the
// four-step FFT_L inside each of the M0 contiguous chunks (k_so_cols with a
// chunk index in blockIdx.y).  float64 data, twiddles and chirps: the rotation
// reads the whole output's energy through three transforms, and float32 (even a
// correctly rounded float32 FFT, pocketfft) leaves ~1e-5 RMS after the tanh
// clip when the filtered output is large (a 192 kHz ER + IR preset with
// max|y| ~ 600), against the north star's 1e-5.
#pragma once
#include "rt.h"

constexpr int SO_T = 512;
constexpr int SO_ROW_MAX = 4096;          // M2
constexpr int SO_COL_MAX = 2048;          // M1
constexpr int SO_COL_ELEMS = 8192;        // columns per block x M1 (128 KiB of LDS, double2)

#if defined(__HIPCC__)
MSG_DEV double2 so_cmul(double2 a, double2 b) { return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x)); }
// exp(-2 pi i e / N) for 0 <= e < N, float64-evaluated
MSG_DEV double2 so_w(int64_t e, int64_t N) {
    double s, c;
    sincospi(-2.0 * (double)e / (double)N, &s, &c);
    return make_double2(c, s);
}

// In-place Stockham FFT (radix 4, final radix 2) of C independent length-N
// sequences s[c N + i] in LDS; tw[j] = exp(-2 pi i j / N).  MAXE >= C N / T.
template <int R, bool INV, int MAXE>
MSG_DEV void so_pass(double2* s, int C, int N, int Ns, const double2* tw) {
    constexpr int B = MAXE / R;
    const int nb = N / R;
    const int total = C * nb;
    const int mul = N / (Ns * R);
    double2 v[B][R];
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int g = threadIdx.x + b * SO_T;
        if (g < total) {
            const int c = g / nb, idx = g - c * nb;
            const int j = idx % Ns;
            double2* sc = s + c * N;
#pragma unroll
            for (int q = 0; q < R; ++q) {
                double2 x = sc[idx + q * nb];
                if (q > 0 && Ns > 1) {
                    double2 w = tw[j * q * mul];
                    if (INV) w.y = -w.y;
                    x = so_cmul(x, w);
                }
                v[b][q] = x;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < B; ++b) {
        const int g = threadIdx.x + b * SO_T;
        if (g < total) {
            const int c = g / nb, idx = g - c * nb;
            const int j = idx % Ns;
            double2* sc = s + c * N;
            double2 o[R];
            if constexpr (R == 2) {
                o[0] = make_double2(v[b][0].x + v[b][1].x, v[b][0].y + v[b][1].y);
                o[1] = make_double2(v[b][0].x - v[b][1].x, v[b][0].y - v[b][1].y);
            } else {
                const double2 a0 = make_double2(v[b][0].x + v[b][2].x, v[b][0].y + v[b][2].y);
                const double2 a1 = make_double2(v[b][0].x - v[b][2].x, v[b][0].y - v[b][2].y);
                const double2 b0 = make_double2(v[b][1].x + v[b][3].x, v[b][1].y + v[b][3].y);
                const double2 d = make_double2(v[b][1].x - v[b][3].x, v[b][1].y - v[b][3].y);
                const double2 b1 = INV ? make_double2(-d.y, d.x) : make_double2(d.y, -d.x);
                o[0] = make_double2(a0.x + b0.x, a0.y + b0.y);
                o[2] = make_double2(a0.x - b0.x, a0.y - b0.y);
                o[1] = make_double2(a1.x + b1.x, a1.y + b1.y);
                o[3] = make_double2(a1.x - b1.x, a1.y - b1.y);
            }
            const int base = (idx - j) * R + j;
#pragma unroll
            for (int q = 0; q < R; ++q) sc[base + q * Ns] = o[q];
        }
    }
    __syncthreads();
}

template <bool INV, int MAXE>
MSG_DEV void so_fft(double2* s, int C, int N, const double2* tw) {
    __syncthreads();
    int Ns = 1;
    while (Ns < N) {
        if (N / Ns >= 4) { so_pass<4, INV, MAXE>(s, C, N, Ns, tw); Ns *= 4; }
        else { so_pass<2, INV, MAXE>(s, C, N, Ns, tw); Ns *= 2; }
    }
}

MSG_DEV void so_stage_tw(double2* tw, int N) {
    for (int j = threadIdx.x; j < N; j += SO_T) tw[j] = so_w(j, N);
}

// Column step over A (M1 rows x M2 columns, row-major), C columns per block.
// forward: FFT_M1 down each column, then x W_M^(j2 k1);  inverse: x conj(W_M^(j2 k1)),
// then inverse FFT_M1.
// blockIdx.y: chunk of A (stride `chunk` elements) for the inner level of a
// three-level transform.
template <bool INV>
__global__ void __launch_bounds__(SO_T)
k_so_cols(double2* __restrict__ A, int M1, int M2, int C, int64_t chunk) {
    extern __shared__ __attribute__((aligned(16))) double2 so_lds[];
    double2* tw = so_lds;                   // M1 entries
    double2* s = so_lds + M1;               // C x M1
    A += (int64_t)blockIdx.y * chunk;
    so_stage_tw(tw, M1);
    const int j20 = blockIdx.x * C;
    const int64_t M = (int64_t)M1 * M2;
    const int tot = C * M1;
    for (int e = threadIdx.x; e < tot; e += SO_T) {
        const int c = e % C, j1 = e / C;
        double2 x = A[(int64_t)j1 * M2 + j20 + c];
        if (INV) {
            double2 w = so_w(((int64_t)(j20 + c) * j1) % M, M);
            w.y = -w.y;
            x = so_cmul(x, w);
        }
        s[c * M1 + j1] = x;
    }
    so_fft<INV, SO_COL_ELEMS / SO_T>(s, C, M1, tw);
    for (int e = threadIdx.x; e < tot; e += SO_T) {
        const int c = e % C, k1 = e / C;
        double2 x = s[c * M1 + k1];
        if (!INV) x = so_cmul(x, so_w(((int64_t)(j20 + c) * k1) % M, M));
        A[(int64_t)k1 * M2 + j20 + c] = x;
    }
}

// Row step: FFT_M2 of each row; with Bp: x Bp (the chirp kernel spectrum in the
// same permuted order, pre-scaled by 1/M), then inverse FFT_M2.
__global__ void __launch_bounds__(SO_T)
k_so_rows(double2* __restrict__ A, int M2, const double2* __restrict__ Bp) {
    extern __shared__ __attribute__((aligned(16))) double2 so_lds[];
    double2* tw = so_lds;
    double2* s = so_lds + M2;
    so_stage_tw(tw, M2);
    double2* row = A + (int64_t)blockIdx.x * M2;
    for (int j = threadIdx.x; j < M2; j += SO_T) s[j] = row[j];
    so_fft<false, SO_ROW_MAX / SO_T>(s, 1, M2, tw);
    if (Bp) {
        const double2* brow = Bp + (int64_t)blockIdx.x * M2;
        for (int k = threadIdx.x; k < M2; k += SO_T) s[k] = so_cmul(s[k], brow[k]);
        so_fft<true, SO_ROW_MAX / SO_T>(s, 1, M2, tw);
    }
    __syncthreads();
    for (int j = threadIdx.x; j < M2; j += SO_T) row[j] = s[j];
}

// Bluestein chirp w_j = exp(-pi i (j^2 mod 2n) / n)
MSG_DEV double2 so_chirp(int64_t j, int64_t n) {
    const int64_t q = (j * j) % (2 * n);
    double s, c;
    sincospi(-(double)q / (double)n, &s, &c);
    return make_double2(c, s);
}

// b_l = conj(w_l) for |l| < n, wrapped mod M, scaled by 1/M (kernel of the chirp convolution)
__global__ void k_so_bfill(double2* __restrict__ A, int64_t n, int64_t M) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    double2 v = make_double2(0.f, 0.f);
    const int64_t l = j < n ? j : (M - j < n ? M - j : -1);
    if (l >= 0) {
        const double2 w = so_chirp(l, n);
        v = make_double2(w.x / (double)M, -w.y / (double)M);
    }
    A[j] = v;
}

// a_j = R_j w_j, R = roll(y, -dr) (MS:432), zero padded to M
__global__ void k_so_pre(double2* __restrict__ A, const float* __restrict__ y, int64_t n, int dr, int64_t M) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    double2 v = make_double2(0.f, 0.f);
    if (j < n) {
        int64_t i = (j + dr) % n;
        if (i < 0) i += n;
        const double r = (double)y[i];
        const double2 w = so_chirp(j, n);
        v = make_double2(r * w.x, r * w.y);
    }
    A[j] = v;
}

// X_j = w_j c_j (= rfft(R) on the full circle); Y = X exp(i a sin(2 pi k / K))
// (conjugate on the negative-frequency half, as irfft's Hermitian extension);
// then a_j = conj(Y_j) w_j for the inverse DFT (conj trick).
__global__ void k_so_mid(double2* __restrict__ A, int64_t n, double a, int64_t K, int64_t M) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= M) return;
    double2 v = make_double2(0.f, 0.f);
    if (j < n) {
        const double2 w = so_chirp(j, n);
        const double2 X = so_cmul(w, A[j]);
        const int64_t k = j <= K ? j : n - j;
        const double ph = a * sinpi(2.0 * (double)k / (double)(K > 0 ? K : 1));
        double sn, cs;
        sincos(ph, &sn, &cs);
        double2 h = make_double2(cs, j <= K ? sn : -sn);
        if (j == 0) h = make_double2(1.f, 0.f);
        double2 Y = so_cmul(X, h);
        if (j == 0) Y.y = 0.f;                    // irfft ignores Im Y[0]
        Y.y = -Y.y;
        v = so_cmul(Y, w);
    }
    A[j] = v;
}

// R2_t = Re(conj(w_t c_t)) / n = Re(w_t c_t) / n
__global__ void k_so_post(const double2* __restrict__ A, float* __restrict__ r2, int64_t n) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const double2 w = so_chirp(t, n);
    const double2 c = A[t];
    r2[t] = (float)((w.x * c.x - w.y * c.y) / (double)n);
}
#endif
