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
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, false);
    float2* dst = ir_spec + j[3];
    for (int k = threadIdx.x; k <= rp.n / 2; k += T) dst[k] = cx(lds, k);
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
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    const int irl = r.ir_len;
    const bool conv = r.n_taps > 0 && irl > 0;   // h = e * ir through the IR spectrum
    if (r.n_taps > 0) {
        for (int u = threadIdx.x; u < N; u += T) rx_set(lds, rp, u, u == 0 ? 1.f : 0.f);
        __syncthreads();
        for (int k = threadIdx.x; k < r.n_taps; k += T) {
            const int64_t o = er_off[r.er_base + k];
            if (o <= 0 || o >= r.out_n || o >= N) continue;   // MS:418-420
            float* h = reinterpret_cast<float*>(lds);
            atomicAdd(h + 2 * lp((int)o >> 1) + ((int)o & 1), (float)er_gain[r.er_base + k]);
        }
    } else {
        const double* ir = ir_bank + r.ir_off;
        for (int u = threadIdx.x; u < N; u += T) rx_set(lds, rp, u, u < irl ? (float)ir[u] : 0.f);
    }
    __syncthreads();
    // transform sequence: conv ? [F, I, F] : [F]; one rtransform call site
    const int nsteps = conv ? 3 : 1;
    for (int step = 0; step < nsteps; ++step) {
        const int Nn = opaque(N);
        const int tid = otid();
        if (step == nsteps - 1) {   // cut partition q of h into place, zero-padded to N
            constexpr int PER = (2 * MAXM + T - 1) / T;
            float v[PER];
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int u = tid + i * T;
                const int src = q * P + u;
                v[i] = (u < P && src < Nn) ? rx_get(lds, rp, src) : 0.f;
            }
            __syncthreads();
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int u = tid + i * T;
                if (u < Nn) rx_set(lds, rp, u, v[i]);
            }
            __syncthreads();
        }
        rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, step == 1);
        if (step == 0 && conv) {
            const float2* S = ir_spec + r.irs_off;
            for (int k = tid; k <= N / 2; k += T) cx(lds, k) = cmul(cx(lds, k), S[k]);
            __syncthreads();
        }
    }
    const int K = N / 2 + 1;
    float2* dst = hspec + r.h_off + (int64_t)q * K;
    for (int k = threadIdx.x; k < K; k += T) dst[k] = cx(lds, k);
}

// x[s0 + u] for u < N (zero outside [0, n)) into the LDS real view, read as
// 16-byte aligned float4 quads (x is 16-byte aligned: y_off % 4 == 0).
template <int T>
MSG_DEV void load_segment(float2* lds, const RealPlan& rp, const float* __restrict__ x, int64_t n, int64_t s0,
                          int N, int tid) {
    const int64_t a0 = (s0 >> 2) << 2;
    const int shift = (int)(s0 - a0);
    const int nq = (N + shift + 3) >> 2;
    const float4* xq = reinterpret_cast<const float4*>(x);
    for (int v0 = 0; v0 < nq; v0 += 8 * T) {
        float4 q[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int v = v0 + i * T + tid;
            const int64_t a = a0 + 4 * (int64_t)v;
            if (v < nq && a >= 0 && a + 3 < n) {
                q[i] = xq[a >> 2];
            } else {
                q[i].x = (v < nq && a >= 0 && a < n) ? x[a] : 0.f;
                q[i].y = (v < nq && a + 1 >= 0 && a + 1 < n) ? x[a + 1] : 0.f;
                q[i].z = (v < nq && a + 2 >= 0 && a + 2 < n) ? x[a + 2] : 0.f;
                q[i].w = (v < nq && a + 3 >= 0 && a + 3 < n) ? x[a + 3] : 0.f;
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int v = v0 + i * T + tid;
            if (v >= nq) continue;
            const int u = 4 * v - shift;
            const float e[4] = {q[i].x, q[i].y, q[i].z, q[i].w};
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (u + c >= 0 && u + c < N) rx_set(lds, rp, u + c, e[c]);
        }
    }
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
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    constexpr int PER = (MAXM + 1 + T - 1) / T;
    float2 acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = make_float2(0.f, 0.f);
    for (int step = 0; step <= Q; ++step) {   // Q forward transforms, then the inverse
        const int Nn = opaque(N);
        const int tid = otid();
        if (step < Q) {
            const int64_t s0 = t0 - (int64_t)step * P - (P - 1);
            load_segment<T>(lds, rp, x, n, s0, Nn, tid);
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int k = tid + u * T;
                if (k < K) cx(lds, k) = acc[u];
            }
        }
        __syncthreads();
        rtransform<T, MAXM, RSET_PO2>(lds, rp, tw, step == Q);
        if (step < Q) {
            const float2* H = hspec + r.h_off + (int64_t)step * K;
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int k = tid + u * T;
                if (k < K) acc[u] = cadd(acc[u], cmul(cx(lds, k), H[k]));
            }
            __syncthreads();
        }
    }
    float* y = y_out + r.y_off;
    for (int u = threadIdx.x + (P - 1); u < N; u += T) {
        const int64_t t = t0 + (u - (P - 1));
        if (t < n) y[t] = rx_get(lds, rp, u);
    }
}

