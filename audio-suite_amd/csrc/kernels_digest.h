// kernels_digest.h — per-render summary and digest on the device (msg_digest).
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
// float64 sums are formed in a fixed order (below; the host reference
// digest_host in k_digest.hip follows it step for step), so a render gives the
// same bits on any device and on the host.
//
// Tiles of DG_TILE frames; thread i of the 256 takes frames i, i + 256, ... of
// its tile (float2 loads: a preset's frames start 8 B-aligned, not 16 B), sums
// in that order, then the wave folds by xor-butterfly and the four waves add in
// wave order.  The preset pass folds its tiles the same way: thread i takes
// tiles i, i + 256, ... in order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
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
#pragma clang fp contract(off)
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

MSG_DEV double dg_shfl(double v, int o) { return __shfl_xor(v, o, 64); }
MSG_DEV uint64_t dg_shfl(uint64_t v, int o) {
    const uint32_t lo = __shfl_xor((uint32_t)v, o, 64), hi = __shfl_xor((uint32_t)(v >> 32), o, 64);
    return ((uint64_t)hi << 32) | lo;
}

// the workgroup's fold: xor-butterfly in each wave (every lane ends with the
// same value: each pair adds the same two operands), then waves 0..3 in order
MSG_DEV DigestPart dg_block_fold(DigestPart a, DigestPart* lds) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        a.ss += dg_shfl(a.ss, o);
        a.sl += dg_shfl(a.sl, o);
        a.sr += dg_shfl(a.sr, o);
        const double pk = dg_shfl(a.peak, o);
        a.peak = a.peak > pk ? a.peak : pk;
        a.h0 += dg_shfl(a.h0, o);
        a.h1 += dg_shfl(a.h1, o);
    }
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) lds[wave] = a;
    __syncthreads();
    DigestPart r = lds[0];
    for (int w = 1; w < DG_T / 64; ++w) dg_add(r, lds[w]);
    return r;
}

// pass 1: one workgroup per tile; tile_base[i] = first tile of render i (n + 1 entries)
__global__ void __launch_bounds__(DG_T)
k_digest_tiles(const float* __restrict__ out, const int64_t* __restrict__ frame_off, const int64_t* __restrict__ frames,
               const int32_t* __restrict__ tile_base, int n, DigestPart* __restrict__ part) {
    __shared__ DigestPart lds[DG_T / 64];
    const int tile = blockIdx.x;
    int lo = 0, hi = n;                              // the render holding this tile: last i with tile_base[i] <= tile
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (tile_base[mid] <= tile) lo = mid; else hi = mid;
    }
    const int p = __builtin_amdgcn_readfirstlane(lo);
    const int64_t n_fr = frames[p];
    const int64_t f0 = (int64_t)(tile - tile_base[p]) * DG_TILE;
    typedef float v2f __attribute__((ext_vector_type(2)));
    const v2f* x = reinterpret_cast<const v2f*>(out) + frame_off[p];
    DigestPart a = dg_zero();
    v2f v[DG_PER];
#pragma unroll
    for (int k = 0; k < DG_PER; ++k) {               // all loads in flight first (read once: nontemporal)
        const int64_t f = f0 + k * DG_T + threadIdx.x;
        v[k] = f < n_fr ? __builtin_nontemporal_load(x + f) : v2f{0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < DG_PER; ++k) {
        const int64_t f = f0 + k * DG_T + threadIdx.x;
        if (f < n_fr) dg_frame(a, v[k].x, v[k].y, __float_as_uint(v[k].x), __float_as_uint(v[k].y), f);
    }
    const DigestPart r = dg_block_fold(a, lds);
    if (threadIdx.x == 0) part[tile] = r;
}

// pass 2: one workgroup per render folds its tiles; res[i] = the render's summary
__global__ void __launch_bounds__(DG_T)
k_digest_presets(const DigestPart* __restrict__ part, const int32_t* __restrict__ tile_base, DigestPart* __restrict__ res) {
    __shared__ DigestPart lds[DG_T / 64];
    const int p = blockIdx.x;
    const int t0 = tile_base[p], t1 = tile_base[p + 1];
    DigestPart a = dg_zero();
    for (int t = t0 + (int)threadIdx.x; t < t1; t += DG_T) dg_add(a, part[t]);
    const DigestPart r = dg_block_fold(a, lds);
    if (threadIdx.x == 0) res[p] = r;
}
