// kernels_fir.h — space FIR kernels (TU: k_fir.hip).
#pragma once
#include "rt.h"
#include "hbuild.h"

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
    h_build_tile(r, r.h_len, (b - tile_begin[p]) * H_TILE, er_off, er_gain, ir_bank, irp, s_off, s_g, hs + r.hs_off);
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
