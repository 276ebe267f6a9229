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

// One workgroup per preset with both early reflections and an IR: h =
// (delta + ER taps) * IR through the IR spectrum (forward, product, inverse),
// written once to a float scratch of N samples, so the Q partition transforms
// of k_fir_h read it instead of each rebuilding h (2 + Q transforms, not 3 Q).
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_fir_hconv(const PresetRt* __restrict__ rt, const int32_t* __restrict__ conv_list,
            const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
            const int32_t* __restrict__ er_off, const double* __restrict__ er_gain,
            const float2* __restrict__ ir_spec, float* __restrict__ hs) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int p = conv_list[blockIdx.x];
    const PresetRt& r = rt[p];
    const RealPlan& rp = fir_plans[fir_plan_of[p]];
    const bool evn = rp.even != 0;
    const int N = r.fir_N;
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    for (int u = threadIdx.x; u < N; u += T) rx_set(lds, evn, u, u == 0 ? 1.f : 0.f);
    __syncthreads();
    for (int k = threadIdx.x; k < r.n_taps; k += T) {
        const int64_t o = er_off[r.er_base + k];
        if (o <= 0 || o >= r.out_n || o >= N) continue;   // MS:418-420
        float* h = reinterpret_cast<float*>(lds);
        atomicAdd(h + 2 * lp((int)o >> 1) + ((int)o & 1), (float)er_gain[r.er_base + k]);
    }
    __syncthreads();
    for (int step = 0; step < 2; ++step) {   // [F, I], one rtransform call site
        const int tid = otid();
        rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, step == 1);
        if (step == 0) {
            const float2* S = ir_spec + r.irs_off;
            for (int k = tid; k <= N / 2; k += T) cx(lds, k) = cmul(cx(lds, k), S[k]);
            __syncthreads();
        }
    }
    float* dst = hs + r.hs_off;
    for (int u = threadIdx.x; u < N; u += T) dst[u] = rx_get(lds, evn, u);
}

// One workgroup per (preset, partition q): h[qP, qP+P) zero-padded to N (from
// k_fir_hconv's scratch, or built in LDS from the ER taps or the IR alone),
// and its spectrum H_q.
template <int T, int MAXM>
__global__ void __launch_bounds__(T)
k_fir_h(const PresetRt* __restrict__ rt, const int32_t* __restrict__ hblk_begin, int n_presets,
        const RealPlan* __restrict__ fir_plans, const int32_t* __restrict__ fir_plan_of,
        const int32_t* __restrict__ er_off, const double* __restrict__ er_gain,
        const double* __restrict__ ir_bank, const float* __restrict__ hs,
        float2* __restrict__ hspec) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const int b = blockIdx.x;
    const int p = find_preset(hblk_begin, n_presets, b);
    const PresetRt& r = rt[p];
    if (r.h_fir4) return;   // built by k_fir4_hconv / k_fir4_hpart (fir4_fft.h)
    const int q = b - r.h_block_begin;
    const RealPlan& rp = fir_plans[fir_plan_of[p]];
    const bool evn = rp.even != 0;
    const int N = r.fir_N, P = r.fir_P;
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    const int irl = r.ir_len;
    const bool conv = r.n_taps > 0 && irl > 0;   // h = e * ir, built by k_fir_hconv
    if (conv) {
        const float* hsrc = hs + r.hs_off;
        const int64_t s0 = (int64_t)q * P;
        for (int u = threadIdx.x; u < N; u += T)
            rx_set(lds, evn, u, (u < P && s0 + u < N) ? hsrc[s0 + u] : 0.f);
    } else if (r.n_taps > 0) {
        for (int u = threadIdx.x; u < N; u += T) rx_set(lds, evn, u, u == 0 ? 1.f : 0.f);
        __syncthreads();
        for (int k = threadIdx.x; k < r.n_taps; k += T) {
            const int64_t o = er_off[r.er_base + k];
            if (o <= 0 || o >= r.out_n || o >= N) continue;   // MS:418-420
            float* h = reinterpret_cast<float*>(lds);
            atomicAdd(h + 2 * lp((int)o >> 1) + ((int)o & 1), (float)er_gain[r.er_base + k]);
        }
    } else {
        const double* ir = ir_bank + r.ir_off;
        for (int u = threadIdx.x; u < N; u += T) rx_set(lds, evn, u, u < irl ? (float)ir[u] : 0.f);
    }
    __syncthreads();
    {
        const int Nn = opaque(N);
        const int tid = otid();
        if (!conv) {   // cut partition q of h into place, zero-padded to N
            constexpr int PER = (2 * MAXM + T - 1) / T;
            float v[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int u = tid + i * T;
                const int src = q * P + u;
                v[i] = (u < P && src < Nn) ? rx_get(lds, evn, src) : 0.f;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int u = tid + i * T;
                if (u < Nn) rx_set(lds, evn, u, v[i]);
            }
            __syncthreads();
        }
        rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, false);
    }
    const int K = N / 2 + 1;
    float2* dst = hspec + r.h_off + (int64_t)q * K;
    for (int k = threadIdx.x; k < K; k += T) dst[k] = cx(lds, k);
}
