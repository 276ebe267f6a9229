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

// The space filter h = (delta + ER taps) * IR (MS:409-445) in the time domain,
// float64: h[t] = ir[t] + sum_k g_k ir[t - o_k] over the preset's merged,
// offset-sorted taps (o_k in (0, out_n), msg_render_batch), with ir = delta
// when the preset has no IR.  One workgroup per tile of H_TILE taps; the IR is
// staged in LDS as float64 and each tile walks only the taps whose shifted IR
// overlaps it (the offsets are sorted).  Any length: the ER span is not limited
// by a transform size (192 kHz x 150 ms + 8192 IR taps = 36 992 taps).  Output:
// h_len floats at hs_off, cut into partitions by k_fir_h / k_fir4_hpart.
constexpr int H_T = 256, H_PER = 4, H_TILE = H_T * H_PER, H_IRMAX = 8192;
__global__ void __launch_bounds__(H_T)
k_h_build(const PresetRt* __restrict__ rt, const int32_t* __restrict__ tile_begin, int n_presets,
          const int32_t* __restrict__ er_off, const double* __restrict__ er_gain,
          const double* __restrict__ ir_bank, float* __restrict__ hs) {
    __shared__ double ir[H_IRMAX];
    const int b = blockIdx.x;
    const int p = find_preset(tile_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int hl = r.h_len;
    const int irl = r.ir_len > 0 ? r.ir_len : 1;
    const int t0 = (b - tile_begin[p]) * H_TILE;
    if (r.ir_len > 0) {
        const double* src = ir_bank + r.ir_off;
        for (int i = threadIdx.x; i < irl; i += H_T) ir[i] = src[i];
    } else if (threadIdx.x == 0) {
        ir[0] = 1.0;
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
    for (int i = 0; i < H_PER; ++i) {
        const int t = t0 + (int)threadIdx.x + i * H_T;
        acc[i] = t < irl ? ir[t] : 0.0;                       // the direct path (delta * IR)
    }
    for (int k = klo; k < khi; ++k) {
        const int o = off[k];
        const double g = gain[k];
#pragma unroll
        for (int i = 0; i < H_PER; ++i) {
            const int d = t0 + (int)threadIdx.x + i * H_T - o;
            if ((unsigned)d < (unsigned)irl) acc[i] = fma(g, ir[d], acc[i]);
        }
    }
    float* h = hs + r.hs_off;
#pragma unroll
    for (int i = 0; i < H_PER; ++i) {
        const int t = t0 + (int)threadIdx.x + i * H_T;
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
