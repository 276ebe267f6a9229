// kernels_fir.h — space FIR kernels (TU: k_fir.hip).
#pragma once
#include "rt.h"

// ---------------------------------------------------------------------------
// Space FIR (MS:409-445): h = (delta + ER taps) * IR, folded into one kernel
// so ER and IR become a single partitioned FFT overlap-save convolution.
// ---------------------------------------------------------------------------
// IR spectra at the FIR size of each (IR, N) pair of the batch.
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_ir_spec(const int64_t* __restrict__ jobs /* [ir_off, ir_len, plan, out_off] */, int n_jobs,
          const RealPlan* __restrict__ fir_plans, const double* __restrict__ ir_bank,
          float2* __restrict__ ir_spec) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    if (b >= n_jobs) return;
    const int64_t* j = jobs + 4 * b;
    const RealPlan& rp = fir_plans[j[2]];
    const bool evn = rp.even != 0;
    const double* ir = ir_bank + j[0];
    const int64_t irl = j[1];
    for (int u = threadIdx.x; u < rp.n; u += T) rx_set(lds, evn, u, u < irl ? (float)ir[u] : 0.f);
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, false);
    float2* dst = ir_spec + j[3];
    for (int k = threadIdx.x; k <= rp.n / 2; k += T) dst[k] = cx(lds, k);
}

// The space filter h = (delta + ER taps) * IR (MS:409-445) in the time domain:
// h[t] = ir[t] + sum_k g_k ir[t - o_k] over the preset's merged, offset-sorted
// taps (o_k in (0, out_n), msg_render_batch), ir = delta without an IR, summed
// in float64.  One workgroup per tile of H_TILE taps of h.  The IR sits in LDS
// zero-padded by H_TILE on both sides, so every (tap, output) pair is one LDS
// read at a tap-uniform base plus the thread's fixed offsets (no bounds tests),
// and only the taps whose shifted IR overlaps the tile are walked, staged
// through LDS H_T at a time.  Any length: the ER span is not limited by a
// transform size (192 kHz x 150 ms + 8192 IR taps = 36 992 taps).  Output:
// h_len floats at hs_off, cut into partitions by k_fir_h / k_fir4_hpart / k_fir8_hpart.
constexpr int H_T = 256, H_PER = 4, H_TILE = H_T * H_PER, H_IRMAX = 8192;
__global__ void __launch_bounds__(H_T)
k_h_build(const PresetRt* __restrict__ rt, const int32_t* __restrict__ tile_begin, int n_presets,
          const int32_t* __restrict__ er_off, const double* __restrict__ er_gain,
          const double* __restrict__ ir_bank, float* __restrict__ hs) {
    __shared__ float irp[H_IRMAX + 2 * H_TILE];          // irp[H_TILE + d] = ir[d], zero outside [0, irl)
    __shared__ int32_t s_off[H_T];
    __shared__ double s_g[H_T];
    const int b = blockIdx.x;
    const int p = find_preset(tile_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int hl = r.h_len;
    const int irl = r.ir_len > 0 ? r.ir_len : 1;
    const int t0 = (b - tile_begin[p]) * H_TILE;
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
    float* h = hs + r.hs_off;
#pragma unroll
    for (int i = 0; i < H_PER; ++i) {
        const int t = t0 + tid + i * H_T;
        if (t < hl) h[t] = (float)acc[i];
    }
}

// One workgroup per (preset, partition q) of the presets whose spectra are not
// on the k_fir4 engine: H_q = rfft_N(h[qP, qP + P) zero-padded to N), h from
// k_h_build's scratch.
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_fir_h(const PresetRt* __restrict__ rt, const int32_t* __restrict__ hblk_begin, int n_presets,
        const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
        const float* __restrict__ hs, float2* __restrict__ hspec) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int p = find_preset(hblk_begin, n_presets, b);
    const PresetRt& r = rt[p];
    if (r.h_fir4) return;   // built by k_fir4_hpart (fir4_fft.h)
    const int q = b - r.h_block_begin;
    const RealPlan& rp = fir_plans[fir_plan_of[p]];
    const bool evn = rp.even != 0;
    const int N = r.fir_N, P = r.fir_P;
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    const float* hsrc = hs + r.hs_off;
    const int64_t s0 = (int64_t)q * P;
    for (int u = threadIdx.x; u < N; u += T)
        rx_set(lds, evn, u, (u < P && s0 + u < r.h_len) ? hsrc[s0 + u] : 0.f);
    __syncthreads();
    rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, false);
    const int K = N / 2 + 1;
    float2* dst = hspec + r.h_off + (int64_t)q * K;
    for (int k = threadIdx.x; k < K; k += T) dst[k] = cx(lds, k);
}
