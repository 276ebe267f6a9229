// digest.h — per-render summary and digest (msg_digest / msg_digest_host): the
// definition, shared by the device kernels (kernels_digest.h) and the host
// reference below (built into libmsgpu and into the host sanitizer build).
//
// a multi-GPU batch returns per-preset checksums, not audio
// (C5's 1024 presets per GPU are 68.7 GB of output).  The reference's own batch
// path writes one render at a time (main_v2.py:1585-1589); here each render is
// reduced where it lies in HBM and only 48 B per preset cross PCIe.
//
// For one render, the 2 out_n float32 words of its interleaved (out_n, 2)
// buffer, word j holding bit pattern w_j:
//   ss    = sum of x^2 over both channels     (float64)
//   peak  = max |x|                            (exact)
//   sum_l, sum_r = sums of each channel        (float64)
//   h0 = sum_j fmix64(k_j ^ DG_S0) mod 2^64,   h1 = the same with DG_S1,
//        k_j = j << 32 | w_j,  fmix64 = MurmurHash3's 64-bit finaliser
// The digest depends on every bit and on each word's position (fmix64 is a
// bijection, so two words differ in k_j unless they are the same word at the
// same place) and, being a sum, does not depend on the reduction order.  The
// float64 sums are formed in a fixed order (kernels_digest.h; digest_host below
// follows it step for step), so a render gives the same bits on any device and
// on the host.
//
// Tiles of DG_TILE frames; thread i of the 256 takes frames i, i + 256, ... of
// its tile (float2 loads: a preset's frames start 8 B-aligned, not 16 B), sums
// in that order, then the wave folds by xor-butterfly and the four waves add in
// wave order.  The preset pass folds its tiles the same way: thread i takes
// tiles i, i + 256, ... in order.
#pragma once
#include <stdint.h>
#include <cmath>
#include <cstring>
#include <vector>
#include "msg_common.h"

constexpr int DG_T = 256;                 // threads per workgroup (4 waves)
constexpr int DG_PER = 8;                 // frames per thread per tile
constexpr int DG_TILE = DG_T * DG_PER;    // 2048 frames = 16 KB per tile
constexpr uint64_t DG_S0 = 0x9E3779B97F4A7C15ull, DG_S1 = 0xD1B54A32D192ED03ull;

struct DigestPart {                       // one tile's (or one preset's) partial; layout of msg_digest_rec
    double ss, peak, sl, sr;
    uint64_t h0, h1;
};

MSG_HD uint64_t dg_fmix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

MSG_HD void dg_add(DigestPart& a, const DigestPart& b) {
    a.ss += b.ss; a.sl += b.sl; a.sr += b.sr;
    a.peak = a.peak > b.peak ? a.peak : b.peak;
    a.h0 += b.h0; a.h1 += b.h1;
}

MSG_HD DigestPart dg_zero() { DigestPart p; p.ss = p.sl = p.sr = p.peak = 0.0; p.h0 = p.h1 = 0; return p; }

// one frame (L, R) at word index 2 f of its render (float products are exact in
// float64, so contraction could not change the sums either)
MSG_HD void dg_frame(DigestPart& a, float l, float r, uint32_t wl, uint32_t wr, int64_t f) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
    const double dl = (double)l, dr = (double)r;
    a.ss += dl * dl + dr * dr;
    a.sl += dl;
    a.sr += dr;
    const double m = fabs(dl) > fabs(dr) ? fabs(dl) : fabs(dr);
    a.peak = a.peak > m ? a.peak : m;
    const uint64_t kl = ((uint64_t)(2 * f) << 32) | wl, kr = ((uint64_t)(2 * f + 1) << 32) | wr;
    a.h0 += dg_fmix64(kl ^ DG_S0) + dg_fmix64(kr ^ DG_S0);
    a.h1 += dg_fmix64(kl ^ DG_S1) + dg_fmix64(kr ^ DG_S1);
}

// The host reference: the workgroup fold on the host (256 per-thread partials,
// xor-butterfly inside each wave of 64, then the waves in order), tiles in order.
inline DigestPart dg_host_fold(std::vector<DigestPart>& th) {
    for (int o = 32; o >= 1; o >>= 1) {
        std::vector<DigestPart> nx(th);
        for (int i = 0; i < DG_T; ++i) {
            DigestPart a = th[i];
            dg_add(a, th[i ^ o]);
            nx[i] = a;
        }
        th.swap(nx);
    }
    DigestPart r = th[0];
    for (int w = 1; w < DG_T / 64; ++w) dg_add(r, th[w * 64]);
    return r;
}
inline int64_t dg_tiles(int64_t frames) { return (frames + DG_TILE - 1) / DG_TILE; }
inline void dg_host(const float* x, int64_t frames, DigestPart* rec) {
    const int64_t tiles = dg_tiles(frames);
    std::vector<DigestPart> part((size_t)tiles), th(DG_T);
    for (int64_t t = 0; t < tiles; ++t) {
        for (int i = 0; i < DG_T; ++i) {
            DigestPart a = dg_zero();
            for (int k = 0; k < DG_PER; ++k) {
                const int64_t f = t * DG_TILE + k * DG_T + i;
                if (f >= frames) continue;
                uint32_t wl, wr;
                std::memcpy(&wl, x + 2 * f, 4);
                std::memcpy(&wr, x + 2 * f + 1, 4);
                dg_frame(a, x[2 * f], x[2 * f + 1], wl, wr, f);
            }
            th[i] = a;
        }
        part[(size_t)t] = dg_host_fold(th);
    }
    for (int i = 0; i < DG_T; ++i) {
        DigestPart a = dg_zero();
        for (int64_t t = i; t < tiles; t += DG_T) dg_add(a, part[(size_t)t]);
        th[i] = a;
    }
    *rec = dg_host_fold(th);
}
