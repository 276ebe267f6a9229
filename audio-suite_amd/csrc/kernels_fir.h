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
    const double* ir = ir_bank + j[0];
    const int64_t irl = j[1];
    for (int u = threadIdx.x; u < rp.n; u += T) rx_set(lds, rp, u, u < irl ? (float)ir[u] : 0.f);
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp.c);
    rfft_lds<T, MAXM>(lds, rp, tw);
    float2* dst = ir_spec + j[3];
    for (int k = threadIdx.x; k <= rp.n / 2; k += T) dst[k] = lds[k];
}

// One workgroup per (preset, partition q): build h in LDS (ER taps scattered,
// convolved with the IR through its spectrum when both are on), cut
// h[qP, qP+P), zero-pad to N, and store its spectrum H_q.
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_fir_h(const PresetRt* __restrict__ rt, const int32_t* __restrict__ hblk_begin, int n_presets,
        const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
        const int32_t* __restrict__ er_off, const double* __restrict__ er_gain,
        const double* __restrict__ ir_bank, const float2* __restrict__ ir_spec,
        float2* __restrict__ hspec) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int p = find_preset(hblk_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const int q = b - r.h_block_begin;
    const RealPlan& rp = fir_plans[fir_plan_of[p]];
    const int N = r.fir_N, P = r.fir_P;
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp.c);
    float* h = reinterpret_cast<float*>(lds);   // N real samples (N even)
    const int irl = r.ir_len;
    if (r.n_taps > 0) {
        for (int u = threadIdx.x; u < N; u += T) h[u] = u == 0 ? 1.f : 0.f;
        __syncthreads();
        for (int k = threadIdx.x; k < r.n_taps; k += T) {
            const int64_t o = er_off[r.er_base + k];
            if (o <= 0 || o >= r.out_n || o >= N) continue;   // MS:418-420
            atomicAdd(h + o, (float)er_gain[r.er_base + k]);
        }
        __syncthreads();
        if (irl > 0) {   // h = e * ir via the IR spectrum (linear: M <= N checked on the host)
            rfft_lds<T, MAXM>(lds, rp, tw);
            const float2* S = ir_spec + r.irs_off;
            for (int k = threadIdx.x; k <= N / 2; k += T) lds[k] = cmul(lds[k], S[k]);
            __syncthreads();
            irfft_lds<T, MAXM>(lds, rp, tw);
        }
    } else {
        const double* ir = ir_bank + r.ir_off;
        for (int u = threadIdx.x; u < N; u += T) h[u] = u < irl ? (float)ir[u] : 0.f;
        __syncthreads();
    }
    // cut partition q into place
    constexpr int PER = (2 * MAXM + T - 1) / T;
    float v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int u = (int)threadIdx.x + i * T;
        const int src = q * P + u;
        v[i] = (u < P && src < N) ? h[src] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int u = (int)threadIdx.x + i * T;
        if (u < N) h[u] = v[i];
    }
    __syncthreads();
    rfft_lds<T, MAXM>(lds, rp, tw);
    const int K = N / 2 + 1;
    float2* dst = hspec + r.h_off + (int64_t)q * K;
    for (int k = threadIdx.x; k < K; k += T) dst[k] = lds[k];
}

// Partitioned FFT overlap-save: a block outputs B samples; Q forward FFTs
// accumulate X_q * H_q in registers, then one inverse FFT.
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_fir(const PresetRt* __restrict__ rt, const int32_t* __restrict__ fblk_begin, int n_presets,
      const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
      const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int p = find_preset(fblk_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const RealPlan& rp = fir_plans[fir_plan_of[p]];
    const int N = r.fir_N, P = r.fir_P, Q = r.fir_Q, B = r.fir_B;
    const int64_t n = r.out_n;
    const int64_t t0 = (int64_t)(b - r.fir_block_begin) * B;
    const float* x = x_in + r.y_off;
    const int K = N / 2 + 1;
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp.c);
    constexpr int PER = (MAXM + 1 + T - 1) / T;
    float2 acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = make_float2(0.f, 0.f);
    for (int q = 0; q < Q; ++q) {
        const int64_t s0 = t0 - (int64_t)q * P - (P - 1);
        for (int u = threadIdx.x; u < N; u += T) {
            const int64_t s = s0 + u;
            rx_set(lds, rp, u, (s >= 0 && s < n) ? x[s] : 0.f);
        }
        __syncthreads();
        rfft_lds<T, MAXM>(lds, rp, tw);
        const float2* H = hspec + r.h_off + (int64_t)q * K;
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int k = (int)threadIdx.x + u * T;
            if (k < K) acc[u] = cadd(acc[u], cmul(lds[k], H[k]));
        }
        __syncthreads();
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int k = (int)threadIdx.x + u * T;
        if (k < K) lds[k] = acc[u];
    }
    __syncthreads();
    irfft_lds<T, MAXM>(lds, rp, tw);
    float* y = y_out + r.y_off;
    for (int u = threadIdx.x + (P - 1); u < N; u += T) {
        const int64_t t = t0 + (u - (P - 1));
        if (t < n) y[t] = rx_get(lds, rp, u);
    }
}

