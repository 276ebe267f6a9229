// hbuild.h — one tile of the space filter h = (delta + ER taps) * IR in the time
// domain (MS:409-445), shared by k_h_build (kernels_fir.h) and k_h64
// (kernels_fir64.h).
#pragma once
#include "rt.h"

constexpr int H_T = 256, H_PER = 4, H_TILE = H_T * H_PER, H_IRMAX = 8192;
// One tile h[t0, t0 + H_TILE) of a preset's h (hl taps) into h (shared arrays
// passed in: irp, s_off, s_g).
MSG_DEV void h_build_tile(const PresetRt& r, int hl, int t0, const int32_t* __restrict__ er_off,
                          const double* __restrict__ er_gain, const double* __restrict__ ir_bank, float* irp,
                          int32_t* s_off, double* s_g, float* __restrict__ h) {
    const int irl = r.ir_len > 0 ? r.ir_len : 1;
    const int tid = threadIdx.x;
    const double* src = ir_bank + r.ir_off;
    for (int i = tid; i < irl + 2 * H_TILE; i += H_T) {
        const int d = i - H_TILE;
        irp[i] = (d >= 0 && d < irl) ? (r.ir_len > 0 ? (float)src[d] : 1.0f) : 0.0f;
    }
    // taps whose shifted IR reaches [t0, t0 + H_TILE): o in (t0 - irl, t0 + H_TILE)
    const int32_t* off = er_off + r.er_base;
    const double* gain = er_gain + r.er_base;
    int lo = 0, hi = r.n_taps;          // first o > t0 - irl
    while (lo < hi) { const int m = (lo + hi) >> 1; if (off[m] > t0 - irl) hi = m; else lo = m + 1; }
    const int klo = lo;
    hi = r.n_taps;                      // first o >= t0 + H_TILE
    while (lo < hi) { const int m = (lo + hi) >> 1; if (off[m] >= t0 + H_TILE) hi = m; else lo = m + 1; }
    const int khi = lo;
    __syncthreads();
    double acc[H_PER];
#pragma unroll
    for (int i = 0; i < H_PER; ++i) {                          // delta * IR
        const int t = t0 + tid + i * H_T;
        acc[i] = t < irl ? (double)irp[H_TILE + t] : 0.0;
    }
    for (int k0 = klo; k0 < khi; k0 += H_T) {
        const int kn = khi - k0 < H_T ? khi - k0 : H_T;
        __syncthreads();                                        // previous chunk's reads done
        if (tid < kn) { s_off[tid] = off[k0 + tid]; s_g[tid] = gain[k0 + tid]; }
        __syncthreads();
        for (int k = 0; k < kn; ++k) {
            const float* base = irp + (H_TILE + t0 - s_off[k]) + tid;   // in [0, irl + H_TILE]
            const double g = s_g[k];
#pragma unroll
            for (int i = 0; i < H_PER; ++i) acc[i] = fma(g, (double)base[i * H_T], acc[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < H_PER; ++i) {
        const int t = t0 + tid + i * H_T;
        if (t < hl) h[t] = (float)acc[i];
    }
}

