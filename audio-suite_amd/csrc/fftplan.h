// fftplan.h — host-side construction of FFT plans (factorisation, float64
// twiddles rounded once to float32, Bluestein chirps) for fft_lds.h.
#pragma once
#include <cmath>
#include <complex>
#include <vector>
#include <algorithm>
#include <stdint.h>

namespace fftplan {

// Radix sequence for a Stockham FFT of length m over the register DFTs of
// fft_lds.h {2,3,4,5,6,7,8,9,10,12,15,16,20,25}; false when m has a prime
// factor > 7 (-> Bluestein).  Few passes = few LDS round trips.
inline bool factor(int m, std::vector<int>& rad) {
    rad.clear();
    int r = m, a2 = 0, a3 = 0, a5 = 0, a7 = 0;
    while (r % 2 == 0) { r /= 2; ++a2; }
    while (r % 3 == 0) { r /= 3; ++a3; }
    while (r % 5 == 0) { r /= 5; ++a5; }
    while (r % 7 == 0) { r /= 7; ++a7; }
    if (r != 1) return false;
    for (; a5 >= 2; a5 -= 2) rad.push_back(25);
    if (a5) rad.push_back(5);
    for (; a3 >= 2; a3 -= 2) rad.push_back(9);
    if (a3) rad.push_back(3);
    for (; a7; --a7) rad.push_back(7);
    for (; a2 >= 4; a2 -= 4) rad.push_back(16);
    if (a2 == 3) rad.push_back(8);
    else if (a2 == 2) rad.push_back(4);
    else if (a2 == 1) rad.push_back(2);
    auto ok = [](int x) {
        for (int v : {2, 3, 4, 5, 6, 7, 8, 9, 10, 12, 15, 16, 20, 25}) if (v == x) return true;
        return false;
    };
    for (bool merged = true; merged;) {   // merge the smallest mergeable pair
        merged = false;
        std::sort(rad.begin(), rad.end());
        for (size_t i = 0; i < rad.size() && !merged; ++i)
            for (size_t j = i + 1; j < rad.size() && !merged; ++j)
                if (ok(rad[i] * rad[j])) {
                    rad[i] *= rad[j];
                    rad.erase(rad.begin() + j);
                    merged = true;
                }
    }
    return true;
}

inline int next_pow2(int x) { int p = 1; while (p < x) p <<= 1; return p; }

// interleaved re,im of exp(-2 pi i j * step / size), j < count
inline std::vector<float> twiddles(int size, int count, int step) {
    std::vector<float> t(2 * (size_t)count);
    for (int j = 0; j < count; ++j) {
        const long long e = ((long long)j * step) % size;
        const long double a = -2.0L * 3.14159265358979323846264338327950288L * (long double)e / (long double)size;
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
