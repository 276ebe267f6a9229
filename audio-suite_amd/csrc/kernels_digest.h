// kernels_digest.h — the device side of msg_digest (TU k_digest.hip): tiles
// of DG_TILE frames, one workgroup each, then one workgroup per render folding
// its tiles.  The definition and the host reference are in digest.h.
#pragma once
#include <hip/hip_runtime.h>
#include "digest.h"

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
