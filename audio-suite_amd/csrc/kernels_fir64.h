// kernels_fir64.h — the float64 space FIR for heavily saturated renders (TU:
// k_fir64.hip).
//
// The float32 FFT overlap-save FIR (k_fir8 / k_fir4 / k_fir2) leaves an error
// of ~eps32 x the block's rms in every output sample.  Where the render's
// tanh clip (MS:31-34, 780) saturates -- large early-reflection + IR gains, the
// 192 kHz er_max_ms = 150 filters of VERDICT r03 -- the loud samples are
// compressed and the quiet ones carry that error up to the output: the float32
// floor of an exact-twiddle FFT is 5-7e-6 RMS there (tools/fir_error_model.py),
// next to the 1e-5 tolerance.  Such presets get the FIR again in float64:
//
//   k_stereo_fused / k_stereo_max (first pass, kernels_stereo.h) adds per
//     preset sum y^2 and sum (1 + (d y)^2)^-2 (the share of samples the clip
//     leaves in its linear range) over the float32 y, in tile order, predicts
//     the float32 error from them (fir64_pred, rt.h: eps32 rms(y) x
//     sqrt(share) x the clip's slope and the peak scale, within 2-3x of the
//     exact-twiddle float32 error, tools/fir_error_model.py) and flags every
//     preset above FIR64_PRED (flag64);
//   k_fir64_flag gives every flagged preset a slot, in batch order, and resets
//     its stereo peak;
//   then, per window of `cap` slots (all of them at once unless their buffers
//   would pass FIR64_WINDOW_BYTES):
//   k_h64      h = (delta + ER) * IR in the time domain (k_h_build's tiles);
//   k_hspec64  H_q = rfft_N(h[q P, q P + P)) in float64, N = 16384, P = N/2;
//   k_fir64    one output block of B = N - P + 1 frames: sum_q rfft(seg_q) H_q
//              (Q + 1 float64 transforms on the LDS engine of the grain chain)
//              -> irfft -> y as float32 (its rounding: ~1e-8 RMS);
// then the odd-length stereo rotation and the peak pass run again for the
// slots (kernels_stereo_odd.h, k_stereo_remax) and k_stereo_out_list writes
// their output (k_stereo_fused deferred it).  A preset's route depends only on
// its own render, never on the batch it shares (at most 128 slots
// had been served, in batch order).
// Every kernel of the chain walks a virtual (slot, unit) space in a grid-stride
// loop and skips units of empty slots, so a batch without flagged presets (C3,
// C4, C5, the shipped presets but wavelet_mist) pays a few microseconds.
#pragma once
#include "rt.h"
#include "fft64.h"
#include "hbuild.h"

constexpr int FIR64_T = 512, FIR64_E = 16;          // the float64 LDS engine (G64_T, G64_MAXE)

// Slot kernel: one wave walks the presets 64 at a time, slots in batch order
// (a 64-thread workgroup finds a CU at once beside other streams' kernels,
// where a 1024-thread one waited ~80 us for a free CU).
__global__ void __launch_bounds__(64)
k_fir64_flag(int n_presets, const int32_t* __restrict__ flag64, unsigned* __restrict__ maxbits,
             int32_t* __restrict__ slot_preset, int32_t* __restrict__ n_slots) {
    const int lane = (int)threadIdx.x;
    int base = 0;
    for (int p0 = 0; p0 < n_presets; p0 += 64) {
        const int p = p0 + lane;
        const bool f = p < n_presets && flag64[p] != 0;
        const uint64_t bal = __ballot(f);
        if (f) {
            slot_preset[base + __popcll(bal & ((1ULL << lane) - 1))] = p;
            maxbits[p] = 0u;                               // k_stereo_remax takes the float64 y's peak
        }
        base += __popcll(bal);
    }
    if (lane == 0) *n_slots = base;
}

// slots of the window [w0, w0 + cap)
MSG_DEV int fir64_window(const int32_t* __restrict__ n_slots, int w0, int cap) {
    const int ns = *n_slots - w0;
    return ns < cap ? ns : cap;
}

// h of the slots' presets (k_h_build's tile, float64 sums, float32 taps).
__global__ void __launch_bounds__(H_T)
k_h64(const PresetRt* __restrict__ rt, const Fir64Rt* __restrict__ fr, const int32_t* __restrict__ slot_preset,
      const int32_t* __restrict__ n_slots, int w0, int cap, int tmax, const int32_t* __restrict__ er_off,
      const double* __restrict__ er_gain, const double* __restrict__ ir_bank, float* __restrict__ h64,
      int64_t h_stride) {
    __shared__ float irp[H_IRMAX + 2 * H_TILE];
    __shared__ int32_t s_off[H_T];
    __shared__ double s_g[H_T];
    const int ns = fir64_window(n_slots, w0, cap);
    for (int64_t j = blockIdx.x; j < (int64_t)ns * tmax; j += gridDim.x) {
        const int sl = (int)(j / tmax), t = (int)(j - (int64_t)sl * tmax);
        const int p = slot_preset[w0 + sl];
        if (t * H_TILE >= fr[p].h_len) continue;               // uniform
        __syncthreads();
        h_build_tile(rt[p], fr[p].h_len, t * H_TILE, er_off, er_gain, ir_bank, irp, s_off, s_g,
                     h64 + (int64_t)sl * h_stride);
    }
}

// H_q = rfft_N(h[q P, q P + P) zero-padded) in float64, one (slot, q) per pass.
__global__ void __launch_bounds__(FIR64_T)
k_hspec64(const Fir64Rt* __restrict__ fr, const Real64Plan* __restrict__ plans, int plan,
          const int32_t* __restrict__ slot_preset, const int32_t* __restrict__ n_slots, int w0, int cap, int qmax,
          const float* __restrict__ h64, int64_t h_stride, double2* __restrict__ hs64, int64_t hs_stride) {
    extern __shared__ __attribute__((aligned(16))) double2 buf[];
    const Real64Plan& rp = plans[plan];
    double* d = reinterpret_cast<double*>(buf);
    const int ns = fir64_window(n_slots, w0, cap);
    for (int64_t j = blockIdx.x; j < (int64_t)ns * qmax; j += gridDim.x) {
        const int sl = (int)(j / qmax), q = (int)(j - (int64_t)sl * qmax);
        const int p = slot_preset[w0 + sl];
        const int hl = fr[p].h_len;
        if (q >= fr[p].q) continue;
        const float* h = h64 + (int64_t)sl * h_stride + (int64_t)q * FIR64_P;
        const int len = hl - q * FIR64_P < FIR64_P ? hl - q * FIR64_P : FIR64_P;
        __syncthreads();
        for (int u = threadIdx.x; u < FIR64_N; u += FIR64_T) d[u] = u < len ? (double)h[u] : 0.0;
        __syncthreads();
        f64_rfft<FIR64_T, FIR64_E>(buf, rp);
        double2* H = hs64 + (int64_t)sl * hs_stride + (int64_t)q * FIR64_K;
        for (int k = threadIdx.x; k < FIR64_K; k += FIR64_T) H[k] = buf[k];
    }
}

// One output block y[t0, t0 + B) of a slot's preset: overlap-save over the Q
// partitions, the spectrum sum held per thread in registers (bins tid + i T).
__global__ void __launch_bounds__(FIR64_T)
k_fir64(const PresetRt* __restrict__ rt, const Fir64Rt* __restrict__ fr, const Real64Plan* __restrict__ plans,
        int plan, const int32_t* __restrict__ slot_preset, const int32_t* __restrict__ n_slots, int w0, int cap, int bmax,
        const double2* __restrict__ hs64, int64_t hs_stride, const float* __restrict__ x_in,
        float* __restrict__ y_out) {
    extern __shared__ __attribute__((aligned(16))) double2 buf[];
    const Real64Plan& rp = plans[plan];
    double* d = reinterpret_cast<double*>(buf);
    const int ns = fir64_window(n_slots, w0, cap);
    constexpr int NE = (FIR64_K + FIR64_T - 1) / FIR64_T;
    static_assert(NE <= FIR64_E + 1, "bins per thread");
    for (int64_t j = blockIdx.x; j < (int64_t)ns * bmax; j += gridDim.x) {
        const int sl = (int)(j / bmax), b = (int)(j - (int64_t)sl * bmax);
        const int p = slot_preset[w0 + sl];
        const Fir64Rt f = fr[p];
        if (b >= f.blocks) continue;
        const PresetRt& r = rt[p];
        const int64_t n = r.out_n;
        const int64_t t0 = (int64_t)b * FIR64_B;
        const float* x = x_in + r.y_off;
        double2 acc[NE];
#pragma unroll
        for (int i = 0; i < NE; ++i) acc[i] = d2(0.0, 0.0);
        for (int q = 0; q < f.q; ++q) {
            // segment x[s0, s0 + N), s0 = t0 - q P - (P - 1): y[t0 + i] = its circular
            // convolution with h_q at P - 1 + i
            const int64_t s0 = t0 - (int64_t)q * FIR64_P - (FIR64_P - 1);
            __syncthreads();
            for (int u = threadIdx.x; u < FIR64_N; u += FIR64_T) {
                const int64_t i = s0 + u;
                d[u] = (i >= 0 && i < n) ? (double)x[i] : 0.0;
            }
            __syncthreads();
            f64_rfft<FIR64_T, FIR64_E>(buf, rp);
            const double2* H = hs64 + (int64_t)sl * hs_stride + (int64_t)q * FIR64_K;
#pragma unroll
            for (int i = 0; i < NE; ++i) {
                const int k = threadIdx.x + i * FIR64_T;
                if (k < FIR64_K) acc[i] = dadd(acc[i], dmul(buf[k], H[k]));
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < NE; ++i) {
            const int k = threadIdx.x + i * FIR64_T;
            if (k < FIR64_K) buf[k] = acc[i];
        }
        __syncthreads();
        f64_irfft<FIR64_T, FIR64_E>(buf, rp);
        float* y = y_out + r.y_off;
        for (int i = threadIdx.x; i < FIR64_B; i += FIR64_T)
            if (t0 + i < n) y[t0 + i] = (float)d[FIR64_P - 1 + i];
    }
}
