// fftplan.h — host-side construction of FFT plans (factorisation, float64
// twiddles rounded once to float32, Bluestein chirps) for fft_lds.h.
#pragma once
#include <cmath>
#include <complex>
#include <vector>
#include <stdint.h>

namespace fftplan {

// Radix sequence for a Stockham FFT of length m using {8,4,2,5,3,7}; returns
// false when m has another prime factor (-> Bluestein).
inline bool factor(int m, std::vector<int>& rad) {
    rad.clear();
    int r = m;
    while (r % 8 == 0 && r >= 8) { rad.push_back(8); r /= 8; }
    if (r % 4 == 0) { rad.push_back(4); r /= 4; }
    if (r % 2 == 0) { rad.push_back(2); r /= 2; }
    for (int p : {5, 3, 7}) {
        while (r % p == 0) { rad.push_back(p); r /= p; }
    }
    return r == 1;
}

inline int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }

inline std::vector<float> twiddles(int size) {   // interleaved re,im of exp(-2 pi i j / size)
    std::vector<float> t(2 * (size_t)size);
    for (int j = 0; j < size; ++j) {
        // exact octant symmetry keeps the float64 values symmetric
        const long double a = -2.0L * 3.14159265358979323846264338327950288L * (long double)j / (long double)size;
        t[2 * j] = (float)std::cos(a);
        t[2 * j + 1] = (float)std::sin(a);
    }
    return t;
}

// Bluestein tables for length m through power-of-two M >= 2m-1.
inline void bluestein(int m, int M, std::vector<float>& chirp, std::vector<float>& bspec) {
    typedef std::complex<long double> cld;
    const long double PI = 3.14159265358979323846264338327950288L;
    std::vector<cld> c(m);
    for (int j = 0; j < m; ++j) {
        const long long jj = ((long long)j * (long long)j) % (2LL * m);
        const long double a = -PI * (long double)jj / (long double)m;
        c[j] = cld(std::cos(a), std::sin(a));
    }
    chirp.resize(2 * (size_t)m);
    for (int j = 0; j < m; ++j) { chirp[2 * j] = (float)c[j].real(); chirp[2 * j + 1] = (float)c[j].imag(); }
    // b_l = conj(c_|l|) for |l| < m, wrapped into [0, M); B = FFT_M(b) in long double (O(M log M)).
    std::vector<cld> b(M, cld(0, 0));
    for (int j = 0; j < m; ++j) {
        b[j] = std::conj(c[j]);
        if (j) b[M - j] = std::conj(c[j]);
    }
    // iterative radix-2 FFT, long double
    int lg = 0; while ((1 << lg) < M) ++lg;
    for (int i = 0; i < M; ++i) {
        int r = 0; for (int k = 0; k < lg; ++k) if (i & (1 << k)) r |= 1 << (lg - 1 - k);
        if (r > i) std::swap(b[i], b[r]);
    }
    for (int len = 2; len <= M; len <<= 1) {
        for (int i = 0; i < M; i += len) {
            for (int k = 0; k < len / 2; ++k) {
                const long double a = -2.0L * PI * (long double)k / (long double)len;
                const cld w(std::cos(a), std::sin(a));
                const cld u = b[i + k], v = b[i + k + len / 2] * w;
                b[i + k] = u + v;
                b[i + k + len / 2] = u - v;
            }
        }
    }
    bspec.resize(2 * (size_t)M);
    for (int j = 0; j < M; ++j) { bspec[2 * j] = (float)b[j].real(); bspec[2 * j + 1] = (float)b[j].imag(); }
}

}  // namespace fftplan
