// fir_fft.h — register-resident partitioned FFT overlap-save FIR (TU: k_fir.hip).
//
// The space FIR (ER taps + IR as one filter h, MS:409-445, 766-773) on an
// output block of B = N - P + 1 frames:
//     y_block = last B samples of IFFT_N( sum_q FFT_N(x segment q) . H_q ).
// N = 2M real samples go through an M-point complex FFT (even/odd packing).
// Everything about the transform is compile-time for each M in {1024 ..
// 16384}: three Stockham passes of radices (R1, R2, R3), T = M / (2 R3)
// threads, every LDS offset an immediate.
//
// Data movement per forward transform:
//   pass 1  global x -> registers (packed pairs, coalesced) -> DFT_R1 -> LDS (A)
//   pass 2  LDS (A) -> twiddle (exact table) -> DFT_R2 -> LDS (B)
//   pass 3  LDS (B) -> twiddle (power tree) -> DFT_R3 -> stays in registers
// Pass 3 gives each thread the butterflies j and NB3 - j, so bins k and M - k
// of the packed spectrum are in the same thread: the real-FFT split
// (X[k], X[M-k] from Z[k], Z[M-k]), the multiply-accumulate with H_q and the
// inverse's pre-step all run in registers.  The inverse runs the same engine
// on conj(Z') with radices (R3, R2, R1): its first pass reads the registers,
// its last pass writes the output block straight to HBM.  Two LDS exchanges
// per transform instead of one per pass plus staging.
//
// LDS exchanges use "one pad slot per S" layouts, phys(x) = x + x / S, chosen
// per exchange so the strided Stockham stores hit distinct banks
// (ds_write_b64: 16-lane groups over 32 banks) while the unit-stride reads
// stay conflict-free; twiddle tables sit below the data at LDS offset 0.
#pragma once
#include <cmath>
#include <vector>
#include "rt.h"

template <int M> struct FirCfg;
template <> struct FirCfg<16384> { static constexpr int R1 = 32, R2 = 32, R3 = 16; };
template <> struct FirCfg<8192> { static constexpr int R1 = 32, R2 = 16, R3 = 16; };
template <> struct FirCfg<4096> { static constexpr int R1 = 16, R2 = 16, R3 = 16; };
template <> struct FirCfg<2048> { static constexpr int R1 = 16, R2 = 16, R3 = 8; };
template <> struct FirCfg<1024> { static constexpr int R1 = 16, R2 = 8, R3 = 8; };

constexpr int fir_ilog2(int x) { return x <= 1 ? 0 : 1 + fir_ilog2(x / 2); }

template <int M> struct FirGeo {
    static constexpr int R1 = FirCfg<M>::R1, R2 = FirCfg<M>::R2, R3 = FirCfg<M>::R3;
    static constexpr int T = M / (2 * R3);
    static constexpr int NB1 = M / R1, NB2 = M / R2, NB3 = M / R3;
    static constexpr int BP1 = NB1 / T, BP2 = NB2 / T;        // butterflies per thread
    static_assert(NB1 % T == 0 && NB2 % T == 0 && NB3 == 2 * T, "FIR FFT plan");
    // twiddle tables (float2 entries) at LDS offset 0.  The radix-R2 passes
    // read w_{NS R2}^{k r} at [r][k] (k = butterfly index mod NS): the lanes of a
    // wave read consecutive entries, so the table reads are conflict-free
    // (a k*r-strided single table conflicted up to 16-way at r = 16).
    static constexpr int OFF_T2A = 0;                           // pass 2:  NS = R1, [R2][R1]
    static constexpr int OFF_T2B = R2 * R1;                     // pass 2': NS = R3, [R2][R3]
    static constexpr int OFF_MLO = OFF_T2B + R2 * R3;           // w_M^x, x < 128
    static constexpr int OFF_MHI = OFF_MLO + 128;               // w_M^(128 x), x < M/128
    static constexpr int OFF_PLO = OFF_MHI + M / 128;           // w_2M^x, x < 128
    static constexpr int OFF_PHI = OFF_PLO + 128;               // w_2M^(128 x), 128 x <= NB3
    static constexpr int TAB_USED = OFF_PHI + NB3 / 128 + 1;
    static constexpr int TAB = (TAB_USED + 15) & ~15;
    // exchange layouts: A (pass 1 -> 2), B (2 -> 3), C (1' -> 2'), D (2' -> 3')
    static constexpr int SA = R1, SB = 32, SC = R3, SD = 32;
    static constexpr int SMIN = SA < SC ? SA : SC;
    static constexpr int BUF = M + M / SMIN;
    static constexpr int LDS_BYTES = (TAB + BUF) * 8;
    static_assert(LDS_BYTES <= 163840, "FIR LDS budget");
};

// phys(x) = x + x / S (S a power of two)
template <int S> MSG_HD constexpr int padx(int x) { return x + (x >> fir_ilog2(S)); }

// One radix-R Stockham pass LDS -> LDS: read layout SI with NB = M/R
// butterflies, twiddles w_{NS R}^{k r} from the exact [r][k] table, write layout SO.
template <int M, int R, int NS, int BP, int SI, int SO>
MSG_DEV void fir_pass_lds(float2* buf, const float2* tab, int t) {
    using G = FirGeo<M>;
    constexpr int NB = M / R, T = G::T;
    constexpr int OFF_T = NS == G::R1 ? G::OFF_T2A : G::OFF_T2B;
    static_assert(NS == G::R1 || NS == G::R3, "radix-R2 pass after R1 or R3");
    float2 v[BP][R];
#pragma unroll
    for (int b = 0; b < BP; ++b) {
        const int base = padx<SI>(t + b * T);
#pragma unroll
        for (int r = 0; r < R; ++r) v[b][r] = buf[base + padx<SI>(r * NB)];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BP; ++b) {
        const int j = t + b * T;
        const int k = j & (NS - 1), q = j / NS;
#pragma unroll
        for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tab[OFF_T + r * NS + k]);
        Dft<R, false>::run(v[b]);
        const int obase = padx<SO>(q * NS * R + k);
#pragma unroll
        for (int r = 0; r < R; ++r) buf[obase + r * NS + (r * NS) / SO] = v[b][r];
    }
}

MSG_DEV float2 fir_wM(const float2* tab, int lo, int hi, int j) {   // two-level table
    return cmul(tab[hi + (j >> 7)], tab[lo + (j & 127)]);
}

// Real-FFT split of bins k, M-k of the packed spectrum Z:
//     X[k] = E + W o,  X[M-k] = conj(E - W o),  E = (Zk + conj Zm)/2,
//     o = (Zk - conj Zm)/2i.
// With S = Zk + conj Zm, P = W (Zk - conj Zm) and t = (P.y, -P.x)/2 = W o:
//     X[k] = S/2 + t,  X[M-k] = (S.x/2 - t.x, t.y - S.y/2)
// -- seven packed instructions, the halvings folded into the FMAs.
MSG_DEV void fir_split(float2 zk, float2 zm, float2 wk, float2& xk, float2& xm) {
    const f2v S = add_conj(vv(zk), vv(zm));
    const f2v P = vv(cmul(wk, ff(sub_conj(vv(zk), vv(zm)))));
#if MSG_ASM_CMUL
    f2v t, a, b;
    asm("v_pk_mul_f32 %2, %4, 0.5 op_sel:[1,0] op_sel_hi:[0,0] neg_hi:[1,0]\n\t"
        "v_pk_fma_f32 %0, %3, 0.5, %2 op_sel_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %1, %3, 0.5, %2 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[1,0,0]"
        : "=&v"(a), "=v"(b), "=&v"(t) : "v"(S), "v"(P));
    xk = ff(a); xm = ff(b);
#else
    const f2v t = f2v{0.5f * P.y, -0.5f * P.x};
    xk = ff(0.5f * S + t);
    xm = make_float2(0.5f * S.x - t.x, t.y - 0.5f * S.y);
#endif
}

// forward real-FFT split of bins k, M-k and the multiply-accumulate with H
MSG_DEV void fir_pair_mac(float2 zk, float2 zm, float2 wk, float2 hk, float2 hm, float2& ak, float2& am) {
    float2 xk, xm;
    fir_split(zk, zm, wk, xk, xm);
    ak = cfma(ak, xk, hk);
    am = cfma(am, xm, hm);
}

// inverse pre-step: Y[k], Y[M-k] -> conj Z'[k], conj Z'[M-k] (irfft packing):
//     e = (Yk + conj Ym)/2, o = (Yk - conj Ym) conj(W)/2,
//     Z'k* = (e.x - o.y, -(e.y + o.x)),  Z'm* = (e.x + o.y, e.y - o.x).
// With S = Yk + conj Ym, t = (Pc.y, Pc.x)/2, Pc = (Yk - conj Ym) conj(W):
//     Z'k* = (S.x/2 - t.x, -S.y/2 - t.y),  Z'm* = (S.x/2 + t.x, S.y/2 - t.y).
MSG_DEV void fir_pair_pre(float2& yk, float2& ym, float2 wk) {
    const f2v S = add_conj(vv(yk), vv(ym));
    const f2v Pc = vv(cmulc(ff(sub_conj(vv(yk), vv(ym))), wk));
#if MSG_ASM_CMUL
    f2v t, a, b;
    asm("v_pk_mul_f32 %2, %4, 0.5 op_sel:[1,0] op_sel_hi:[0,0]\n\t"
        "v_pk_fma_f32 %0, %3, 0.5, %2 op_sel_hi:[1,0,1] neg_lo:[0,0,1] neg_hi:[1,0,1]\n\t"
        "v_pk_fma_f32 %1, %3, 0.5, %2 op_sel_hi:[1,0,1] neg_hi:[0,0,1]"
        : "=&v"(a), "=v"(b), "=&v"(t) : "v"(S), "v"(Pc));
    yk = ff(a); ym = ff(b);
#else
    const f2v t = f2v{0.5f * Pc.y, 0.5f * Pc.x};
    yk = make_float2(0.5f * S.x - t.x, -0.5f * S.y - t.y);
    ym = make_float2(0.5f * S.x + t.x, 0.5f * S.y - t.y);
#endif
}

// exp(-pi i r / R3): the post-twiddle step between the butterflies' bins
template <int R3> MSG_DEV float2 fir_cr(int r) {
    return make_float2((float)__builtin_cos(3.14159265358979323846 * r / R3),
                       (float)-__builtin_sin(3.14159265358979323846 * r / R3));
}

// Thread 0 holds the two self-paired butterflies j = 0 and j = NB3/2.  Its
// bins are permuted into the general slot pairing (A'[r] <-> B'[R3-1-r], bins
// k and M-k) so every thread runs the same branch-free split; the one slot
// left over (A'[R3-1] = DC/Nyquist, B'[0] = bin M/2) is fixed up by select.
//   A'[r]: r < R3/2 -> (B, r); r < R3-1 -> (A, r - R3/2 + 1); r = R3-1 -> (A, 0)
//   B'[u]: u >= R3/2 -> (B, u); u >= 1 -> (A, R3/2 + u); u = 0 -> (A, R3/2)
template <int R3> MSG_HD constexpr int slotA_h(int r) { return r < R3 / 2 ? 1 : 0; }
template <int R3> MSG_HD constexpr int slotA_r(int r) { return r < R3 / 2 ? r : (r < R3 - 1 ? r - R3 / 2 + 1 : 0); }
template <int R3> MSG_HD constexpr int slotB_h(int u) { return u >= R3 / 2 ? 1 : 0; }
template <int R3> MSG_HD constexpr int slotB_r(int u) { return u >= R3 / 2 ? u : (u >= 1 ? R3 / 2 + u : R3 / 2); }
// bin k of slot A'[r] in thread 0, and w_2M^k
template <int M, int R3> MSG_HD constexpr int fir_k0(int r) {
    return r < R3 / 2 ? M / R3 / 2 + (M / R3) * r : (r < R3 - 1 ? (M / R3) * (r - R3 / 2 + 1) : 0);
}
template <int M, int R3> MSG_DEV float2 fir_w0(int r) {
    const double a = 3.14159265358979323846 * (double)fir_k0<M, R3>(r) / (double)M;
    return make_float2((float)__builtin_cos(a), (float)-__builtin_sin(a));
}

template <int R3>
MSG_DEV void fir_slots(const float2 (&v)[2][R3], float2 (&a)[R3], float2 (&b)[R3], bool t0z) {
#pragma unroll
    for (int r = 0; r < R3; ++r) {
        a[r] = t0z ? v[slotA_h<R3>(r)][slotA_r<R3>(r)] : v[0][r];
        b[r] = t0z ? v[slotB_h<R3>(r)][slotB_r<R3>(r)] : v[1][r];
    }
}

template <int R3>
MSG_DEV void fir_unslots(float2 (&acc)[2][R3], bool t0z) {
    float2 v[2][R3];
#pragma unroll
    for (int r = 0; r < R3; ++r) {
        v[slotA_h<R3>(r)][slotA_r<R3>(r)] = acc[0][r];
        v[slotB_h<R3>(r)][slotB_r<R3>(r)] = acc[1][r];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R3; ++r) acc[h][r] = t0z ? v[h][r] : acc[h][r];
}

template <int M>
__global__ void __launch_bounds__(FirGeo<M>::T)
k_fir2(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
       const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out) {
    using G = FirGeo<M>;
    constexpr int T = G::T, R1 = G::R1, R2 = G::R2, R3 = G::R3;
    constexpr int NB1 = G::NB1, NB3 = G::NB3, BP1 = G::BP1, BP2 = G::BP2;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int2 job = jobs[xcd_block(blockIdx.x, gridDim.x)];
    const PresetRt& pr = rt[job.x];
    const int P = pr.fir_P, Q = pr.fir_Q;
    const int64_t n = pr.out_n;
    const int64_t t0 = (int64_t)job.y * pr.fir_B;
    const float* x = x_in + pr.y_off;
    const int t = threadIdx.x;
    for (int i = t; i < G::TAB_USED; i += T) tab[i] = tables[i];   // visible after the first exchange

    float2 acc[2][R3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R3; ++r) acc[h][r] = make_float2(0.f, 0.f);

    for (int q = 0; q < Q; ++q) {
        // per-iteration opaque copy of the thread index: nothing derived from it
        // is hoisted out of the segment loop (register pressure)
        const int t = otid();
        const bool t0z = (t == 0);
        const int js[2] = {t, t0z ? NB3 / 2 : NB3 - t};
        // ---- pass 1: x segment (zero outside [0, n)) -> DFT_R1 -> LDS A
        const int64_t s0 = t0 - (int64_t)q * P - (P - 1);
        const bool fast = s0 >= 0 && s0 + 2 * M <= n && (((uintptr_t)(x + s0)) & 7) == 0;
#pragma unroll
        for (int b = 0; b < BP1; ++b) {
            const int j = t + b * T;
            float2 v[R1];
            if (fast) {
                const float2* z = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
                for (int r = 0; r < R1; ++r) v[r] = z[(uint32_t)(j + r * NB1)];   // 32-bit offsets: saddr
            } else {
#pragma unroll
                for (int r = 0; r < R1; ++r) {
                    const int64_t a = s0 + 2 * (int64_t)(j + r * NB1);
                    const bool in0 = a >= 0 && a < n, in1 = a + 1 >= 0 && a + 1 < n;   // branch-free
                    const float x0 = x[(uint32_t)(in0 ? a : 0)], x1 = x[(uint32_t)(in1 ? a + 1 : 0)];
                    v[r] = make_float2(in0 ? x0 : 0.f, in1 ? x1 : 0.f);
                }
            }
            Dft<R1, false>::run(v);
            const int base = padx<G::SA>(j * R1);
#pragma unroll
            for (int r = 0; r < R1; ++r) buf[base + r] = v[r];
        }
        __syncthreads();
        // ---- pass 2: LDS A -> LDS B
        fir_pass_lds<M, R2, R1, BP2, G::SA, G::SB>(buf, tab, t);
        __syncthreads();
        // ---- pass 3: LDS B -> registers
        float2 v[2][R3];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int base = padx<G::SB>(js[h]);
#pragma unroll
            for (int r = 0; r < R3; ++r) v[h][r] = buf[base + padx<G::SB>(r * NB3)];
        }
        __syncthreads();   // LDS free for the next segment / the inverse
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            twiddle_pow_ab<R3, tw_base<R3>()>(v[h], fir_wM(tab, G::OFF_MLO, G::OFF_MHI, js[h]),
                                              fir_wM(tab, G::OFF_MLO, G::OFF_MHI, (js[h] * tw_base<R3>()) & (M - 1)));
            Dft<R3, false>::run(v[h]);
        }
        // ---- real split, X . H_q accumulated in registers.  Every thread but 0
        // pairs bins k (butterfly j, slot r) and M - k (butterfly NB3 - j, slot
        // R3-1-r); thread 0 holds the self-paired butterflies (DC/Nyquist and bin
        // M/2) and runs its own branch (slot layout, fir_slots) instead of every
        // thread paying selects for it.
        const float2* H = hspec + pr.h_off + (int64_t)q * (M + 1);
        if (!t0z) {
            const float2 wA = fir_wM(tab, G::OFF_PLO, G::OFF_PHI, js[0]);
#pragma unroll
            for (int r = 0; r < R3; ++r) {
                const int kA = js[0] + r * NB3;
                const float2 hk = H[(uint32_t)kA], hm = H[(uint32_t)(M - kA)];
                fir_pair_mac(v[0][r], v[1][R3 - 1 - r], cmul_k(wA, fir_cr<R3>(r)), hk, hm, acc[0][r],
                             acc[1][R3 - 1 - r]);
            }
        } else {
            float2 a[R3], bb[R3];
            fir_slots<R3>(v, a, bb, true);
            const float2 hmid = H[M / 2];
#pragma unroll
            for (int r = 0; r < R3; ++r) {
                const int kA = fir_k0<M, R3>(r);
                const float2 hk = H[(uint32_t)kA], hm = H[(uint32_t)(M - kA)];
                if (r < R3 - 1) {
                    fir_pair_mac(a[r], bb[R3 - 1 - r], fir_w0<M, R3>(r), hk, hm, acc[0][r], acc[1][R3 - 1 - r]);
                } else {   // DC/Nyquist packed as (Y[0], Y[M]) and bin M/2
                    const float2 z0 = a[r];
                    acc[0][r] = cadd(acc[0][r], make_float2((z0.x + z0.y) * hk.x, (z0.x - z0.y) * hm.x));
                    acc[1][0] = cfma(acc[1][0], cconj(bb[0]), hmid);
                }
            }
        }
    }

    // ---- inverse: conj Z' from Y in registers, back to the natural butterflies
    {
        const int t = otid();
        if (t != 0) {
            const float2 wA = fir_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
            for (int r = 0; r < R3; ++r) fir_pair_pre(acc[0][r], acc[1][R3 - 1 - r], cmul_k(wA, fir_cr<R3>(r)));
        } else {
#pragma unroll
            for (int r = 0; r < R3 - 1; ++r) fir_pair_pre(acc[0][r], acc[1][R3 - 1 - r], fir_w0<M, R3>(r));
            const float y0 = acc[0][R3 - 1].x, yN = acc[0][R3 - 1].y;
            acc[0][R3 - 1] = make_float2(0.5f * (y0 + yN), -0.5f * (y0 - yN));   // bin M/2: conj Z' = Y
            fir_unslots<R3>(acc, true);
        }
    }
    // ---- pass 1': registers -> DFT_R3 -> LDS C
    const int js[2] = {t, t == 0 ? NB3 / 2 : NB3 - t};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Dft<R3, false>::run(acc[h]);
        const int base = padx<G::SC>(js[h] * R3);
#pragma unroll
        for (int r = 0; r < R3; ++r) buf[base + r] = acc[h][r];
    }
    __syncthreads();
    // ---- pass 2': LDS C -> LDS D
    fir_pass_lds<M, R2, R3, BP2, G::SC, G::SD>(buf, tab, t);
    __syncthreads();
    // ---- pass 3': LDS D -> DFT_R1 -> output block (samples u >= P-1 of the segment)
    float* y = y_out + pr.y_off;
    const float s = 1.0f / (float)M;
#pragma unroll
    for (int b = 0; b < BP1; ++b) {
        const int j = t + b * T;
        float2 v[R1];
        const int base = padx<G::SD>(j);
#pragma unroll
        for (int r = 0; r < R1; ++r) v[r] = buf[base + padx<G::SD>(r * NB1)];
        twiddle_pow_ab<R1, tw_base<R1>()>(v, fir_wM(tab, G::OFF_MLO, G::OFF_MHI, j),
                                          fir_wM(tab, G::OFF_MLO, G::OFF_MHI, (j * tw_base<R1>()) & (M - 1)));
        Dft<R1, false>::run(v);
#pragma unroll
        for (int r = 0; r < R1; ++r) {
            const int u = 2 * (j + r * NB1);                 // z[u/2] = x[u] + i x[u+1]
            const int64_t o = t0 + u - (P - 1);
            if (u >= P - 1 && o < n) y[(uint32_t)o] = v[r].x * s;
            if (u + 1 >= P - 1 && o + 1 < n) y[(uint32_t)(o + 1)] = -v[r].y * s;
        }
    }
}

// ---------------------------------------------------------------------------
// Frequency-domain delay line (standalone FIR with many partitions, msg_fir).
// Partitions and blocks are both P = M samples (N = 2M): segment b is
// x[bM - M, bM + M), its spectrum X_b is computed once (k_fdl_fwd) and reused
// by the Q blocks b .. b+Q-1, so a block costs two transforms instead of Q+1:
//     y[bM, bM + M) = samples [M, 2M) of IFFT_N( sum_q X_{b-q} . H_q ).
// Spectra are stored at natural bins (M+1 float2 per segment, H's layout);
// PresetRt.fir_block_begin is the signal's first segment index.
// ---------------------------------------------------------------------------
// real-FFT split of bins k, M-k from the packed Z (the first half of fir_pair_mac)
MSG_DEV void fir_pair_split(float2 zk, float2 zm, float2 wk, float2& xk, float2& xm) {
    fir_split(zk, zm, wk, xk, xm);
}

template <int M>
__global__ void __launch_bounds__(FirGeo<M>::T)
k_fdl_fwd(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
          const float* __restrict__ x_in, float2* __restrict__ xspec) {
    using G = FirGeo<M>;
    constexpr int T = G::T, R1 = G::R1, R2 = G::R2, R3 = G::R3;
    constexpr int NB1 = G::NB1, NB3 = G::NB3, BP1 = G::BP1, BP2 = G::BP2;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int2 job = jobs[xcd_block(blockIdx.x, gridDim.x)];
    const PresetRt& pr = rt[job.x];
    const int64_t n = pr.out_n;
    const float* x = x_in + pr.y_off;
    const int t = threadIdx.x;
    for (int i = t; i < G::TAB_USED; i += T) tab[i] = tables[i];
    const bool t0z = (t == 0);
    const int js[2] = {t, t0z ? NB3 / 2 : NB3 - t};
    const int64_t s0 = (int64_t)job.y * M - M;
    const bool fast = s0 >= 0 && s0 + 2 * M <= n && (((uintptr_t)(x + s0)) & 7) == 0;
#pragma unroll
    for (int b = 0; b < BP1; ++b) {
        const int j = t + b * T;
        float2 v[R1];
        if (fast) {
            const float2* z = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
            for (int r = 0; r < R1; ++r) v[r] = z[(uint32_t)(j + r * NB1)];
        } else {
#pragma unroll
            for (int r = 0; r < R1; ++r) {
                const int64_t a = s0 + 2 * (int64_t)(j + r * NB1);
                const bool in0 = a >= 0 && a < n, in1 = a + 1 >= 0 && a + 1 < n;
                const float x0 = x[(uint32_t)(in0 ? a : 0)], x1 = x[(uint32_t)(in1 ? a + 1 : 0)];
                v[r] = make_float2(in0 ? x0 : 0.f, in1 ? x1 : 0.f);
            }
        }
        Dft<R1, false>::run(v);
        const int base = padx<G::SA>(j * R1);
#pragma unroll
        for (int r = 0; r < R1; ++r) buf[base + r] = v[r];
    }
    __syncthreads();
    fir_pass_lds<M, R2, R1, BP2, G::SA, G::SB>(buf, tab, t);
    __syncthreads();
    float2 v[2][R3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int base = padx<G::SB>(js[h]);
#pragma unroll
        for (int r = 0; r < R3; ++r) v[h][r] = buf[base + padx<G::SB>(r * NB3)];
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        twiddle_pow_ab<R3, tw_base<R3>()>(v[h], fir_wM(tab, G::OFF_MLO, G::OFF_MHI, js[h]),
                                          fir_wM(tab, G::OFF_MLO, G::OFF_MHI, (js[h] * tw_base<R3>()) & (M - 1)));
        Dft<R3, false>::run(v[h]);
    }
    float2 a[R3], bb[R3];
    fir_slots<R3>(v, a, bb, t0z);
    const float2 wA = fir_wM(tab, G::OFF_PLO, G::OFF_PHI, js[0]);
    float2* X = xspec + (int64_t)(pr.fir_block_begin + job.y) * (M + 1);
#pragma unroll
    for (int r = 0; r < R3; ++r) {
        const int kA = t0z ? fir_k0<M, R3>(r) : js[0] + r * NB3;
        const float2 wk = t0z ? fir_w0<M, R3>(r) : cmul_v(wA, fir_cr<R3>(r));
        if (t0z && r == R3 - 1) {          // DC and Nyquist (packed in z0), bin M/2
            const float2 z0 = a[r];
            X[0] = make_float2(z0.x + z0.y, 0.f);
            X[M] = make_float2(z0.x - z0.y, 0.f);
            X[M / 2] = cconj(bb[0]);
        } else {
            float2 xk, xm;
            fir_pair_split(a[r], bb[R3 - 1 - r], wk, xk, xm);
            X[(uint32_t)kA] = xk;
            X[(uint32_t)(M - kA)] = xm;
        }
    }
}

template <int M>
__global__ void __launch_bounds__(FirGeo<M>::T)
k_fdl_mac(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
          const float2* __restrict__ hspec, const float2* __restrict__ xspec, float* __restrict__ y_out) {
    using G = FirGeo<M>;
    constexpr int T = G::T, R1 = G::R1, R2 = G::R2, R3 = G::R3;
    constexpr int NB1 = G::NB1, NB3 = G::NB3, BP1 = G::BP1, BP2 = G::BP2;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int2 job = jobs[xcd_block(blockIdx.x, gridDim.x)];
    const PresetRt& pr = rt[job.x];
    const int Q = pr.fir_Q;
    const int64_t n = pr.out_n;
    const int t = threadIdx.x;
    for (int i = t; i < G::TAB_USED; i += T) tab[i] = tables[i];
    float2 acc[2][R3];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R3; ++r) acc[h][r] = make_float2(0.f, 0.f);
    {
        const bool t0z = (t == 0);
        const int j0 = t;
        const int nq = Q < job.y + 1 ? Q : job.y + 1;   // X_{b-q} of segments before the signal are zero
        for (int q = 0; q < nq; ++q) {
            const float2* X = xspec + (int64_t)(pr.fir_block_begin + job.y - q) * (M + 1);
            const float2* H = hspec + pr.h_off + (int64_t)q * (M + 1);
#pragma unroll
            for (int r = 0; r < R3; ++r) {
                const int kA = t0z ? fir_k0<M, R3>(r) : j0 + r * NB3;
                if (t0z && r == R3 - 1) {
                    const float2 x0 = X[0], xM = X[M], h0 = H[0], hM = H[M];
                    acc[0][r] = cadd(acc[0][r], make_float2(x0.x * h0.x, xM.x * hM.x));   // (Y[0], Y[M]) packed
                    acc[1][0] = cfma(acc[1][0], X[M / 2], H[M / 2]);
                } else {
                    acc[0][r] = cfma(acc[0][r], X[(uint32_t)kA], H[(uint32_t)kA]);
                    acc[1][R3 - 1 - r] = cfma(acc[1][R3 - 1 - r], X[(uint32_t)(M - kA)], H[(uint32_t)(M - kA)]);
                }
            }
        }
    }
    __syncthreads();   // twiddle table visible
    // ---- inverse: as k_fir2
    {
        const int tt = otid();
        const bool t0z = (tt == 0);
        const float2 wA = fir_wM(tab, G::OFF_PLO, G::OFF_PHI, tt);
#pragma unroll
        for (int r = 0; r < R3; ++r) {
            const float2 wk = t0z ? fir_w0<M, R3>(r) : cmul_v(wA, fir_cr<R3>(r));
            if (r < R3 - 1) {
                fir_pair_pre(acc[0][r], acc[1][R3 - 1 - r], wk);
            } else {
                float2 yk = acc[0][r], ym = acc[1][0];
                fir_pair_pre(yk, ym, wk);
                const float y0 = acc[0][r].x, yN = acc[0][r].y;
                const float2 dc = make_float2(0.5f * (y0 + yN), -0.5f * (y0 - yN));
                acc[0][r] = t0z ? dc : yk;
                acc[1][0] = t0z ? acc[1][0] : ym;
            }
        }
        fir_unslots<R3>(acc, t0z);
    }
    const int js[2] = {t, t == 0 ? NB3 / 2 : NB3 - t};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Dft<R3, false>::run(acc[h]);
        const int base = padx<G::SC>(js[h] * R3);
#pragma unroll
        for (int r = 0; r < R3; ++r) buf[base + r] = acc[h][r];
    }
    __syncthreads();
    fir_pass_lds<M, R2, R3, BP2, G::SC, G::SD>(buf, tab, t);
    __syncthreads();
    float* y = y_out + pr.y_off;
    const float s = 1.0f / (float)M;
    const int64_t t0 = (int64_t)job.y * M - M;       // segment start
#pragma unroll
    for (int b = 0; b < BP1; ++b) {
        const int j = t + b * T;
        float2 v[R1];
        const int base = padx<G::SD>(j);
#pragma unroll
        for (int r = 0; r < R1; ++r) v[r] = buf[base + padx<G::SD>(r * NB1)];
        twiddle_pow<R1>(v, fir_wM(tab, G::OFF_MLO, G::OFF_MHI, j));
        Dft<R1, false>::run(v);
#pragma unroll
        for (int r = 0; r < R1; ++r) {
            const int u = 2 * (j + r * NB1);
            const int64_t o = t0 + u;
            if (u >= M && o < n) y[(uint32_t)o] = v[r].x * s;
            if (u + 1 >= M && o + 1 < n) y[(uint32_t)(o + 1)] = -v[r].y * s;
        }
    }
}

// Host: the twiddle tables of FirGeo<M> (float64-built, rounded once).
template <int M>
inline void fir2_tables(std::vector<float>& out) {
    using G = FirGeo<M>;
    out.assign(2 * (size_t)G::TAB_USED, 0.f);
    const long double PI = 3.14159265358979323846264338327950288L;
    auto put = [&](int at, long double num, long double den) {
        const long double a = -2.0L * PI * num / den;
        out[2 * at] = (float)cosl(a);
        out[2 * at + 1] = (float)sinl(a);
    };
    for (int r = 0; r < G::R2; ++r)
        for (int k = 0; k < G::R1; ++k) put(G::OFF_T2A + r * G::R1 + k, (long double)k * r, (long double)G::R1 * G::R2);
    for (int r = 0; r < G::R2; ++r)
        for (int k = 0; k < G::R3; ++k) put(G::OFF_T2B + r * G::R3 + k, (long double)k * r, (long double)G::R3 * G::R2);
    for (int x = 0; x < 128; ++x) put(G::OFF_MLO + x, x, M);
    for (int x = 0; x < M / 128; ++x) put(G::OFF_MHI + x, 128.0L * x, M);
    for (int x = 0; x < 128; ++x) put(G::OFF_PLO + x, x, 2.0L * M);
    for (int x = 0; x <= G::NB3 / 128; ++x) put(G::OFF_PHI + x, 128.0L * x, 2.0L * M);
}
