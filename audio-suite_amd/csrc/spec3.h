// spec3.h — band-pruned, register-resident spectral chain for the hot grain
// length of the 30 MHz configurations (n = 37500: C3, C4), TU k_spec3.hip.
//
// The chain of one event (MS:690-702, 719-721; lowpass_fft MS:39-59 and
// fft_partial_stretch MS:117-128, with irfft's dropped imaginary parts between
// the fused stages) is
//     grain = irfft( S( W . rfft(micro) ) )
// with W the band-limit weights (zero from bin kz up) and S the stretch
// interpolation (Y[k] = interp(k / f, X) restricted to sources below kz).
// At the design rate of C3/C4 the band keeps ~9 % of the bins and the
// stretched spectrum ~19 % (f = 2) to ~38 % (f = 4), so:
//
//   forward  M = n/2 = 18750-point complex FFT of the packed grain in three
//            Stockham passes (radices 25, 30, 25), registers between passes,
//            two LDS exchanges.  Pass 1 reads the grain straight from HBM
//            (coalesced float2), pass 3 leaves Z in registers.
//   band     only the bins the chain keeps move through LDS: Z[k], Z[M-k] for
//            k < kz (the real-FFT split), X[k] = split * W[k] in place.
//   inverse  the stretch gather and the irfft packing are evaluated on the fly
//            as inverse pass 1's inputs (zero outside the stretched band, no
//            zero fill), then the same two exchanges, and pass 3 writes the
//            grain straight to HBM with the 1/M scale.
//
// LDS traffic per event is four full exchanges plus the band (the LDS Stockham
// kernel of spec_ct.h moves the grain through LDS ~15 times).  Exchange A
// (pass 1 -> 2) uses the identity layout, exchange B (pass 2 -> 3) one pad slot
// every 750 entries: both are bank-conflict-free for their strided writes and
// unit-stride reads (ds_write_b64 16-lane groups / ds_read_b64 32-lane groups;
// checked exhaustively by tools/lds_banks.py).
//
// Eligibility (host, spec3_eligible): grain length 37500, chain = band limit
// [+ stretch] with no tilt or power warp.  A stretched band no wider than M/2
// (C3) has Y[M - k] = 0 wherever Y[k] is used: the packed inverse inputs are
// built once per kept bin.  A wider one (C4's x4 stretch, ky ~ 0.96 M) builds
// each inverse input from Y[i] and Y[M - i] inside inverse pass 1, gathering
// from X in LDS.  Other events keep k_spectral_ct.
#pragma once
#include <cmath>
#include <vector>
#include "kernels_spectral.h"

template <int M_, int T_, int R1_, int R2_, int R3_, int PADB_>
struct Spec3Plan {
    static constexpr int M = M_, T = T_, R1 = R1_, R2 = R2_, R3 = R3_, PADB = PADB_;
    static constexpr int NB1 = M / R1, NB2 = M / R2, NB3 = M / R3;
    static constexpr int NS2 = R1, NS3 = R1 * R2;
    static_assert(R1 * R2 * R3 == M && NS3 == NB3, "three passes");
    static_assert(NB1 <= T && NB2 <= T && NB3 <= T, "one butterfly per thread and pass");
    static constexpr int K = M + 1;                            // rfft bins
    // LDS: twiddle tables at offset 0, then the exchange buffer
    static constexpr int OFF_T2 = 0;                           // w_{NS2 R2}^{k r} at [r][k]
    static constexpr int HI_M = (M + 127) / 128;
    static constexpr int HI_P = (M / 2) / 128 + 2;
    static constexpr int OFF_MLO = OFF_T2 + R2 * NS2;          // w_M^x two-level
    static constexpr int OFF_MHI = OFF_MLO + 128;
    static constexpr int OFF_PLO = OFF_MHI + HI_M;             // w_2M^x two-level
    static constexpr int OFF_PHI = OFF_PLO + 128;
    static constexpr int TAB_USED = OFF_PHI + HI_P;
    static constexpr int TAB = (TAB_USED + 15) & ~15;
    static constexpr int BUF = (M - 1) + ((M - 1) / NB3) * PADB + 1;
    static constexpr int LDS_BYTES = (TAB + BUF) * 8;
    static_assert(LDS_BYTES <= 163840, "LDS budget");
    static MSG_HD constexpr int phB(int x) { return x + (x / NB3) * PADB; }
};

// MSG_S3_WIDE_TW: the wide band's inverse pass 1 takes w_i as w_j times a
// compile-time constant per r instead of a two-level table product per input
#ifndef MSG_S3_WIDE_TW
#define MSG_S3_WIDE_TW 1
#endif
// MSG_S3_PLAN (tuning builds): radices R1, R2, R3 and the exchange-B pad
#ifndef MSG_S3_PLAN
#define MSG_S3_PLAN 25, 30, 25, 11
#endif
using Spec3P18750 = Spec3Plan<18750, 768, MSG_S3_PLAN>;

template <class P> MSG_DEV float2 s3_wM(const float2* tab, int x) {    // exp(-2 pi i x / M)
    return cmul(tab[P::OFF_MHI + (x >> 7)], tab[P::OFF_MLO + (x & 127)]);
}
template <class P> MSG_DEV float2 s3_w2M(const float2* tab, int x) {   // exp(-2 pi i x / 2M)
    return cmul(tab[P::OFF_PHI + (x >> 7)], tab[P::OFF_PLO + (x & 127)]);
}

// Pass 1 of a transform: v = DFT_R1 of the inputs in(j + r NB1) (registers;
// the caller writes exchange A after its barrier).
template <class P, class In>
MSG_DEV void s3_pass1(float2 (&v)[P::R1], int j, In&& in) {
#pragma unroll
    for (int r = 0; r < P::R1; ++r) v[r] = in(j + r * P::NB1);
    Dft<P::R1, false>::run(v);
}
// The stretch interpolation Y[k] = interp(k / f, X) over X[0, kz) (zero
// outside; MS:117-128), branch-free: both loads issue at clamped indices and
// the range tests select (a divergent early return cost ~25 scalar and
// exec-mask instructions per bin).  EXACT32: k / f is exact in float32
// (1 / f dyadic, spec3_eligible's exact32), with the same j0 and fraction as
// the float64 form.
template <bool EXACT32>
MSG_DEV float2 s3_interp(const float2* buf, int k, int kz, int K, float inv_f32, double inv_f) {
    int j0;
    float fr;
    bool in;
    if (EXACT32) {
        const float xs = (float)k * inv_f32;
        in = xs <= (float)(K - 1) && xs < (float)kz;
        j0 = in ? (int)xs : 0;
        fr = xs - (float)j0;
    } else {
        const double xs = (double)k * inv_f;
        in = xs <= (double)(K - 1) && xs < (double)kz;
        j0 = in ? (int)xs : 0;
        fr = (float)(xs - (double)j0);
    }
    const bool has1 = j0 + 1 < kz;
    const float2 a = buf[j0];
    const float2 b1 = buf[has1 ? j0 + 1 : j0];
    const float2 b = has1 ? b1 : make_float2(0.f, 0.f);
    const float2 y = make_float2((b.x - a.x) * fr + a.x, (b.y - a.y) * fr + a.y);
    return in ? y : make_float2(0.f, 0.f);
}

// (a.x / 2 - o.y, a.y / 2 + o.x) as one packed FMA (a / 2 - i o for the wide
// band's inverse inputs; halving is exact, so each half is fma(0.5, a, +-o))
MSG_DEV f2v s3_half_mi(float2 a, float2 o) {
    f2v r;
    asm("v_pk_fma_f32 %0, 0.5, %1, %2 op_sel:[0,0,1] op_sel_hi:[0,1,0] neg_lo:[0,0,1]"
        : "=v"(r) : "v"(vv(a)), "v"(vv(o)));
    return r;
}
// (a.x + b.x, a.y - b.y)
MSG_DEV f2v s3_add_neghi(f2v a, f2v b) {
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <class P> MSG_DEV void s3_store_a(float2* buf, const float2 (&v)[P::R1], int j) {
#pragma unroll
    for (int r = 0; r < P::R1; ++r) buf[j * P::R1 + r] = v[r];   // exchange A, identity layout
}

// Pass 2: exchange A -> twiddle [r][k] -> DFT_R2 -> exchange B (in place).
template <class P> MSG_DEV void s3_pass2(float2* buf, const float2* tab) {
    constexpr int R = P::R2, NS = P::NS2, NB = P::NB2;
    const int j = otid();
    float2 v[R];
    if (j < NB) {
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = buf[j + r * NB];
    }
    __syncthreads();
    if (j < NB) {
        const int k = j % NS, q = j / NS;
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tab[P::OFF_T2 + r * NS + k]);
        Dft<R, false>::run(v);
        // phB(q NS R + k + r NS) = q (NS R + PADB) + k + r NS, as k + r NS < NS R = NB3:
        // one base address, immediate offsets
        const int o = q * (NS * R + P::PADB) + k;
        static_assert(NS * R == P::NB3, "pass 2 writes whole exchange-B rows");
#pragma unroll
        for (int r = 0; r < R; ++r) buf[o + r * NS] = v[r];
    }
    __syncthreads();
}

// Pass 3: exchange B -> twiddle w_M^{j r} (power tree) -> DFT_R3; v[r] = Z[j + r NB3].
template <class P> MSG_DEV void s3_pass3(const float2* buf, const float2* tab, float2 (&v)[P::R3], int j) {
#pragma unroll
    for (int r = 0; r < P::R3; ++r) v[r] = buf[j + r * (P::NB3 + P::PADB)];
    constexpr int B = tw_base<P::R3>();
    static_assert(B * (P::NB3 - 1) < P::M, "w^(B j) index within the table");
    twiddle_pow_ab<P::R3, B>(v, s3_wM<P>(tab, j), s3_wM<P>(tab, B * j));
    Dft<P::R3, false>::run(v);
}

// Band of one event: bins [0, kz) survive the band limit; Y = S(X) is zero from ky up.
struct Spec3Band {
    int kb, kz, ky;
    double inv_f;
    bool stretch;
};
// Host and device: the same float64 threshold arithmetic as Lowpass (rfftfreq, MS:46-58).
MSG_HD int s3_first_bin(double val, double x, int K, bool strict) {
    double g = floor(x / val);
    int k = g < 0.0 ? 0 : (g > (double)K ? K : (int)g);
    if (strict) {
        while (k > 0 && (double)(k - 1) * val > x) --k;
        while (k < K && (double)k * val <= x) ++k;
    } else {
        while (k > 0 && (double)(k - 1) * val >= x) --k;
        while (k < K && (double)k * val < x) ++k;
    }
    return k;
}
MSG_HD Spec3Band s3_band(int n, int sr, double cutoff, double roll, bool stretch, double factor) {
    const int K = n / 2 + 1;
    const double nyq = 0.5 * (double)sr;
    const double c = fmin(fmax(cutoff, 1.0), nyq);
    const double r = fmax(0.0, roll);
    const double val = 1.0 / ((double)n * (1.0 / (double)sr));
    const double f1 = fmin(nyq, c + r);
    const double lim = r <= 0 ? c : f1;
    Spec3Band b;
    b.kb = s3_first_bin(val, c, K, false);
    b.kz = s3_first_bin(val, lim, K, true);
    b.stretch = stretch;
    const double f = fmax(1e-12, factor);
    b.inv_f = 1.0 / f;
    if (stretch) {
        const double e = ceil((double)b.kz * f) + 2.0;
        b.ky = e < (double)K ? (int)e : K;
    } else {
        b.ky = b.kz;
    }
    return b;
}

// LDS of the band phase: Z[k] and Z[M-k] (k < kz), then Z'[i] and Z'[M-i] (i < ky) and a zero slot
template <class P> MSG_HD constexpr bool s3_band_fits(int kz, int ky) {
    return ((kz + 15) & ~15) + 2 * ((ky + 15) & ~15) + 16 <= P::BUF && 2 * ((kz + 15) & ~15) <= P::BUF;
}

// Everything of one event after forward pass 1 (exchange A written, barrier
// passed): pass 2, the band, the inverse and the grain store.
template <class P>
MSG_DEV void s3_rest(float2* buf, const float2* tab, const EventRt* __restrict__ ert, int ei, int64_t off,
                     float* __restrict__ grain_pool) {
    constexpr int M = P::M, T = P::T, K = P::K;
    (void)K;
    SPEC_STAMP_INIT;
    int j = otid();
    SPEC_STAMP(0);
    s3_pass2<P>(buf, tab);
    SPEC_STAMP(1);

    // ---- band (host-computed, spec3_eligible)
    const EventRt& ex = ert[ei];
    const int kb = ex.s3_kb, kz = ex.s3_kz, ky = ex.s3_ky;
    const int zh = (kz + 15) & ~15;                 // Z[M - m], m < kz, at buf[zh + m]
    const int pl = zh;                              // Z'[i], i < ky (after the split frees Z[M - m])
    const int ph = pl + ((ky + 15) & ~15);          // Z'[M - m], 1 <= m < ky
    const int zs = ph + ((ky + 15) & ~15);          // one zero slot

    // ---- forward pass 3 -> Z in registers -> band to LDS
    j = otid();
    {
        float2 v[P::R3];
        if (j < P::NB3) s3_pass3<P>(buf, tab, v, j);
        __syncthreads();                            // exchange B fully read
        // a thread keeps v[r] only for r in two uniform ranges (i < kz needs
        // r <= (kz - 1) / NB3, M - i < kz needs r >= R3 - 2 - (kz - 1) / NB3): scalar
        // tests skip the per-lane tests and exec-mask writes of the other r
        const int rlo = __builtin_amdgcn_readfirstlane((kz - 1) / P::NB3);
        const int rhi = __builtin_amdgcn_readfirstlane(P::R3 - 2 - (kz - 1) / P::NB3);
        if (j < P::NB3) {
#pragma unroll
            for (int r = 0; r < P::R3; ++r) {
                const int i = j + r * P::NB3;
                if (r <= rlo && i < kz) buf[i] = v[r];
                if (r >= rhi && M - i < kz && i > 0) buf[zh + (M - i)] = v[r];
            }
        }
    }
    __syncthreads();
    SPEC_STAMP(2);
    // ---- real split X[k] (k < kz) and band-limit weights (MS:48-58), in place
    {
        const Lowpass lpw(2 * M, ex.gen_sr, ex.cutoff_gen, ex.roll);
        for (int k = otid(); k < kz; k += T) {
            float2 x;
            if (k == 0) {
                const float2 z0 = buf[0];
                x = make_float2(z0.x + z0.y, 0.f);   // DC (imag dropped: drop_edge_imag)
            } else {
                const float2 zk = buf[k], zm = buf[zh + k];
                const float2 w = s3_w2M<P>(tab, k);
                const float2 ee = make_float2(0.5f * (zk.x + zm.x), 0.5f * (zk.y - zm.y));
                const float2 d = make_float2(zk.x - zm.x, zk.y + zm.y);
                const float2 wo = cmul(w, make_float2(0.5f * d.y, -0.5f * d.x));
                x = cadd(ee, wo);
            }
            if (k >= kb) {
                const float wk = lpw.w(k);
                if (wk != 1.f) x = cscale(x, wk);
            }
            buf[k] = x;
        }
    }
    __syncthreads();
    SPEC_STAMP(3);
    const bool stretch = (ex.ops & SPEC_STRETCH) != 0;
    const double inv_f = ex.s3_inv_f;
    if (ky > M / 2) {
        // ---- wide band (C4's x4 stretch: Y reaches past M/2, so both Y[i] and
        // Y[M - i] feed inverse input i).  Y = S(X) is gathered once per bin into
        // LDS over X itself: bins [kz, ky) first (they read X below kz and write
        // above it), then bins [0, kz) chunk by chunk from the top (a wide band
        // has f > 1, so S reads X only below the bin it writes).
        {
            // k / f in float when that is exact for every k (ex.s3_pad: 1 / f a dyadic
            // fraction, e.g. the x4 stretch), else in float64 as the narrow path does.
            // The loops are instantiated per case (uniform): tested inside the loop,
            // the flags cost exec-mask instructions per bin.
            const bool exact32 = ex.s3_pad != 0;
            const float inv_f32 = (float)inv_f;
            // [0, kz) in T-bin chunks from the top down: chunk [a, a + T) reads X
            // at or below its own bins (f > 1), so one barrier between a chunk's
            // reads and its writes orders it against every lower chunk's reads
            // (a register array over all of [0, kz) spilled to scratch).  No
            // read of this loop reaches past (kz - 1) / f + 1, so the chunks
            // above it need no barrier (C4: 2 of 6 chunks take one).
            const int rmax = stretch ? (int)((double)(kz - 1) * inv_f) + 2 : kz;   // one bin of margin
            auto gather = [&](auto Y) {
                for (int k = kz + otid(); k < ky; k += T) buf[k] = Y(k);
                __syncthreads();                        // those reads reach up to ~kz
                for (int a = ((kz - 1) / T) * T; a >= 0; a -= T) {
                    const int k = a + otid();
                    const float2 v = k < kz ? Y(k) : make_float2(0.f, 0.f);
                    if (a <= rmax) __syncthreads();     // uniform
                    if (k < kz) buf[k] = v;
                }
            };
            if (!stretch)
                gather([&](int k) { return k < kz ? buf[k] : make_float2(0.f, 0.f); });
            else if (exact32)
                gather([&](int k) { return s3_interp<true>(buf, k, kz, K, inv_f32, inv_f); });
            else
                gather([&](int k) { return s3_interp<false>(buf, k, kz, K, inv_f32, inv_f); });
        }
        __syncthreads();
        SPEC_STAMP(7);                                  // (stamps build) the wide band's Y gather
        // ---- inverse pass 1 from Y in LDS: conj Z'[i] = PL(Y[i], w_i) + PH(Y[M - i],
        // w_{M-i}), the narrow band's two per-bin terms (w_x = exp(-i pi x / M);
        // w_{M-x} = -conj w_x)
        j = otid();
        {
            const float2 z0 = make_float2(0.f, 0.f);
            float2 v[P::R1];
#if MSG_S3_WIDE_TW
            // inputs i = j + r NB1: w_i = w_j . exp(-i pi r NB1 / M), one table twiddle
            // per thread and a compile-time constant per r (no table reads per input)
            // the 1/2 of both terms folded into the twiddle (w / 2 is exact, so every
            // product below is exactly half the unscaled one: the same bits)
            const float2 wjh = cscale(s3_w2M<P>(tab, j < P::NB1 ? j : 0), 0.5f);
            if (j < P::NB1)
                s3_pass1<P>(v, j, [&](int i) {
                    const float2 a = i < ky ? buf[i] : z0, b = M - i < ky ? buf[M - i] : z0;
                    if (i == 0) return make_float2(0.5f * (a.x + b.x), -0.5f * (a.x - b.x));   // DC, Nyquist (irfft)
                    const int r = (i - j) / P::NB1;
                    const float2 wr = make_float2((float)__builtin_cos(3.14159265358979323846 * r * P::NB1 / M),
                                                  (float)-__builtin_sin(3.14159265358979323846 * r * P::NB1 / M));
                    // wr in an SGPR pair (cmul_k: the same two packed instructions): as a
                    // VGPR operand the 24 constant pairs are hoisted out of k_spec3p's
                    // event loop and spilled
                    const float2 wh = r == 0 ? wjh : cmul_k(wjh, wr);       // w_i / 2
                    const float2 o1 = cmulc(a, wh);                          // a conj(w_i) / 2
                    // mirror term with w_{M-i} = -conj(w_i): -(b . w_i) / 2
                    const float2 p2 = cmul(b, wh);
                    const f2v t1 = s3_half_mi(a, o1), t2 = s3_half_mi(b, p2);
                    return ff(s3_add_neghi(t2, t1));     // (t1.x + t2.x, -t1.y + t2.y)
                });
#else
            if (j < P::NB1)
                s3_pass1<P>(v, j, [&](int i) {
                    const float2 a = i < ky ? buf[i] : z0, b = M - i < ky ? buf[M - i] : z0;
                    if (i == 0) return make_float2(0.5f * (a.x + b.x), -0.5f * (a.x - b.x));   // DC, Nyquist (irfft)
                    const bool lo = i <= M / 2;
                    const float2 wk = s3_w2M<P>(tab, lo ? i : M - i);
                    const float2 wi = lo ? wk : make_float2(-wk.x, wk.y);      // w_i
                    const float2 e1 = cscale(a, 0.5f), o1 = cscale(cmulc(a, wi), 0.5f);
                    // mirror term with w_{M-i} = -conj(w_i): o1' = -(b . w_i) / 2
                    const float2 e2 = cscale(b, 0.5f), o2 = cscale(cmul(b, wi), -0.5f);
                    return make_float2((e1.x - o1.y) + (e2.x + o2.y), -(e1.y + o1.x) + (e2.y - o2.x));
                });
#endif
            __syncthreads();                            // Y fully read
            if (j < P::NB1) s3_store_a<P>(buf, v, j);
        }
        __syncthreads();
    } else {
    const bool exact32 = ex.s3_pad != 0;
    const float inv_f32 = (float)inv_f;
    // ---- stretch gather Y = S(X) (MS:117-128) and the irfft packing of bins k
    // and M - k (Y[M - k] = 0 in the band), conjugated for the forward engine
    // (inverse = conj . F . conj): inverse pass 1's nonzero inputs
    {
        auto pack = [&](auto Y) {                   // instantiated per case, as the wide gather
            for (int k = otid(); k < ky; k += T) {
                const float2 y = Y(k);
                if (k == 0) {
                    buf[pl] = make_float2(0.5f * y.x, -0.5f * y.x);   // imag of Y[0] ignored; Y[M] = 0
                    buf[zs] = make_float2(0.f, 0.f);
                } else {
                    const float2 w = s3_w2M<P>(tab, k);
                    const float2 e1 = cscale(y, 0.5f);
                    const float2 o1 = cscale(cmulc(y, w), 0.5f);
                    buf[pl + k] = make_float2(e1.x - o1.y, -(e1.y + o1.x));
                    buf[ph + k] = make_float2(e1.x + o1.y, e1.y - o1.x);
                }
            }
        };
        if (!stretch)
            pack([&](int k) { return buf[k]; });
        else if (exact32)
            pack([&](int k) { return s3_interp<true>(buf, k, kz, K, inv_f32, inv_f); });
        else
            pack([&](int k) { return s3_interp<false>(buf, k, kz, K, inv_f32, inv_f); });
    }
    __syncthreads();
    // ---- inverse pass 1 (inputs zero outside the stretched band)
    j = otid();
    {
        const int qlo = __builtin_amdgcn_readfirstlane((ky - 1) / P::NB1);
        const int qhi = __builtin_amdgcn_readfirstlane(P::R1 - 2 - (ky - 1) / P::NB1);
        float2 v[P::R1];
        if (j < P::NB1)
            s3_pass1<P>(v, j, [&](int i) {
                // inputs i = j + r NB1 outside the band for every thread: r between
                // the uniform bounds (as forward pass 3's band write), no LDS read
                const int r = (i - j) / P::NB1;
                if (r > qlo && r < qhi) return make_float2(0.f, 0.f);
                const int at = i < ky ? pl + i : (M - i < ky ? ph + (M - i) : zs);
                return buf[at];
            });
        __syncthreads();                            // band fully read
        if (j < P::NB1) s3_store_a<P>(buf, v, j);
    }
    __syncthreads();
    }
    SPEC_STAMP(4);
    s3_pass2<P>(buf, tab);
    SPEC_STAMP(5);
    // ---- inverse pass 3 -> grain (x[2i] = Re z / M, x[2i+1] = -Im z / M) to HBM
    j = otid();
    if (j < P::NB3) {
        float2 v[P::R3];
        s3_pass3<P>(buf, tab, v, j);
        float2* g = reinterpret_cast<float2*>(grain_pool + off);
        const float s = 1.0f / (float)M;
#pragma unroll
        for (int r = 0; r < P::R3; ++r) g[j + r * P::NB3] = make_float2(v[r].x * s, -v[r].y * s);
    }
    SPEC_STAMP(6);
}

// Forward pass 1 of an event from its packed grain in registers (exchange A).
template <class P> MSG_DEV void s3_first(float2* buf, float2 (&v)[P::R1]) {
    const int j = otid();
    if (j < P::NB1) {
        Dft<P::R1, false>::run(v);
        s3_store_a<P>(buf, v, j);
    }
}
template <class P>
MSG_DEV void s3_load(const msg_event* __restrict__ events, const PresetRt* __restrict__ rt, const int32_t* __restrict__ ev_list,
                     int li, const float* __restrict__ micro_pool, float2 (&v)[P::R1]) {
    const msg_event& e = events[ev_list[li]];
    const float2* z = reinterpret_cast<const float2*>(micro_pool + rt[e.preset].pool_base + e.pool_off);
    const int j = otid();
    if (j < P::NB1) {
#pragma unroll
        for (int r = 0; r < P::R1; ++r) v[r] = z[j + r * P::NB1];
    }
}

// Events li, li + G, li + 2G, ... (G = gridDim.x), MSG_S3_EVENTS of them, run
// one after another in one workgroup: each next event's grain is loaded into
// registers right after the current one's pass 1, so its HBM latency hides
// behind the current event (one 158 KB workgroup per CU leaves nothing else to
// cover it), and the twiddle tables are staged once.  Written as an inlined
// template chain rather than a loop: an event loop lets LLVM hoist every DFT
// and band constant out of the loop (100 VGPRs of spills).
#ifndef MSG_S3_EVENTS
#define MSG_S3_EVENTS 2
#endif
template <class P, int KE>
MSG_DEV void s3_chain(float2* buf, const float2* tab, const msg_event* __restrict__ events,
                      const EventRt* __restrict__ ert, const PresetRt* __restrict__ rt,
                      const int32_t* __restrict__ ev_list, int n_list, const float* __restrict__ micro_pool,
                      float* __restrict__ grain_pool, int li, float2 (&cur)[P::R1]) {
    s3_first<P>(buf, cur);
    __syncthreads();
    const msg_event& e = events[ev_list[li]];
    const int64_t off = rt[e.preset].pool_base + e.pool_off;   // even (n even, 16-B aligned preset regions)
    if constexpr (KE > 1) {
        const int l2 = li + (int)gridDim.x;
        float2 pre[P::R1];
        if (l2 < n_list) s3_load<P>(events, rt, ev_list, l2, micro_pool, pre);   // in flight through event li
        s3_rest<P>(buf, tab, ert, ev_list[li], off, grain_pool);
        if (l2 >= n_list) return;
        __syncthreads();                            // exchange B read before the next pass 1 writes
        s3_chain<P, KE - 1>(buf, tab, events, ert, rt, ev_list, n_list, micro_pool, grain_pool, l2, pre);
    } else {
        s3_rest<P>(buf, tab, ert, ev_list[li], off, grain_pool);
    }
}
template <class P>
__global__ void __launch_bounds__(P::T)
k_spec3(const msg_event* __restrict__ events, const EventRt* __restrict__ ert, const PresetRt* __restrict__ rt,
        const float2* __restrict__ tables, const int32_t* __restrict__ ev_list, int n_list,
        const float* __restrict__ micro_pool, float* __restrict__ grain_pool) {
    constexpr int T = P::T;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + P::TAB;
    const int li = blockIdx.x;
    if (li >= n_list) return;
    float2 v[P::R1];
    // table loads, then the grain's, all in flight; the table stores wait for the tables only
    TabCopy<P::TAB_USED, T> tc;
    tc.fetch(tables);
    s3_load<P>(events, rt, ev_list, li, micro_pool, v);
    tc.put(tab);
    s3_chain<P, MSG_S3_EVENTS>(buf, tab, events, ert, rt, ev_list, n_list, micro_pool, grain_pool, li, v);
}

// Persistent form (MSGPU_SPEC3P=1; VERDICT r05 item 2a, the k_fir8p recipe):
// one workgroup per CU for the whole launch stages the tables once and loops
// over events taken from per-XCD counters (XCD x takes events x, x + 8, ...,
// then helps the other XCDs); every event's grain is loaded into registers
// while the previous event runs (the two-event chain above leaves each
// workgroup's first load exposed).  Events are independent, so which
// workgroup runs which one does not change a bit of the output.
// ctr: (MSG_XCDS + 1) x S3P_CTR int32, zero before the launch; the last
// workgroup to finish zeroes it again.
template <class P>
__global__ void __launch_bounds__(P::T)
k_spec3p(const msg_event* __restrict__ events, const EventRt* __restrict__ ert, const PresetRt* __restrict__ rt,
         const float2* __restrict__ tables, const int32_t* __restrict__ ev_list, int n_list,
         const float* __restrict__ micro_pool, float* __restrict__ grain_pool, int32_t* __restrict__ ctr) {
    constexpr int T = P::T;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ int s_take[2];
    float2* tab = lds;
    float2* buf = lds + P::TAB;
    const int x0 = (int)(blockIdx.x % MSG_XCDS);
    int k = 0;                                      // thread 0: counters exhausted so far
    auto take = [&]() -> int {                      // thread 0 only; -1 when every counter is done
        while (k < MSG_XCDS) {
            const int x = (x0 + k) % MSG_XCDS;
            const int li = atomicAdd(ctr + x * S3P_CTR, 1) * MSG_XCDS + x;
            if (li < n_list) return li;
            ++k;
        }
        return -1;
    };
    TabCopy<P::TAB_USED, T> tc;
    tc.fetch(tables);
    if (threadIdx.x == 0) s_take[0] = take();
    __syncthreads();
    int cur = s_take[0];
    float2 v[P::R1];
    if (cur >= 0) s3_load<P>(events, rt, ev_list, cur, micro_pool, v);
    tc.put(tab);
    if (threadIdx.x == 0 && cur >= 0) s_take[1] = take();   // read after the first pass 1's barrier
    int par = 1;
    while (cur >= 0) {                              // uniform
        s3_first<P>(buf, v);
        __syncthreads();
        const int nxt = s_take[par];
        float2 pre[P::R1];
        if (nxt >= 0) {
            s3_load<P>(events, rt, ev_list, nxt, micro_pool, pre);   // in flight through event cur
            // the event after next: s_take[par ^ 1] was last read before this
            // iteration's barriers, and is read again after the next pass 1's
            if (threadIdx.x == 0) s_take[par ^ 1] = take();
        }
        const msg_event& e = events[ev_list[cur]];
        const int64_t off = rt[e.preset].pool_base + e.pool_off;
        s3_rest<P>(buf, tab, ert, ev_list[cur], off, grain_pool);
        if (nxt < 0) break;
        __syncthreads();                            // exchange B read before the next pass 1 writes
        cur = nxt;
#pragma unroll
        for (int r = 0; r < P::R1; ++r) v[r] = pre[r];
        par ^= 1;
    }
    // every take of this workgroup has returned (thread 0 made them in order)
    if (threadIdx.x == 0 && atomicAdd(ctr + MSG_XCDS * S3P_CTR, 1) == (int)gridDim.x - 1) {
        for (int x = 0; x < MSG_XCDS; ++x) ctr[x * S3P_CTR] = 0;
        ctr[MSG_XCDS * S3P_CTR] = 0;
    }
}

// Host: twiddle tables (float64-built, rounded once).
template <class P>
inline void spec3_tables(std::vector<float>& out) {
    out.assign(2 * (size_t)P::TAB_USED, 0.f);
    const long double PI = 3.14159265358979323846264338327950288L;
    auto put = [&](int at, long double num, long double den) {
        const long double a = -2.0L * PI * num / den;
        out[2 * at] = (float)cosl(a);
        out[2 * at + 1] = (float)sinl(a);
    };
    for (int r = 0; r < P::R2; ++r)
        for (int k = 0; k < P::NS2; ++k) put(P::OFF_T2 + r * P::NS2 + k, (long double)k * r, (long double)P::NS2 * P::R2);
    for (int x = 0; x < 128; ++x) put(P::OFF_MLO + x, x, P::M);
    for (int x = 0; x < P::HI_M; ++x) put(P::OFF_MHI + x, 128.0L * x, P::M);
    for (int x = 0; x < 128; ++x) put(P::OFF_PLO + x, x, 2.0L * P::M);
    for (int x = 0; x < P::HI_P; ++x) put(P::OFF_PHI + x, 128.0L * x, 2.0L * P::M);
}
