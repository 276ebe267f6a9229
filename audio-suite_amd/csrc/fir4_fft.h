// fir4_fft.h — four-pass variant of the overlap-save FIR kernel (TU: k_fir.hip).
//
// k_fir2<16384> runs its 16384-point transforms as three radix (32, 32, 16)
// passes on 512 threads: 224 VGPRs, 8 waves per CU (2 per SIMD) and, per the
// r02q SQ counters, ~50 % VALU-busy -- the rest is barrier / LDS / HBM latency
// that two waves per SIMD cannot cover.  k_fir4<16384> runs the same
// algorithm (same blocks, partitions, real split and multiply-accumulate) as
// four radix (16, 16, 8, 8) passes on 1024 threads: at most 128 VGPRs, 16
// waves per CU (4 per SIMD), for one more LDS exchange per transform.
//
// Stockham pass p (radix R, NS = product of the earlier radices, NB = M/R):
// butterfly j reads logical j + r NB, multiplies by w_{NS R}^{(j mod NS) r},
// runs DFT_R and writes logical (j / NS) NS R + (j mod NS) + r NS.
// Forward (16, 16, 8, 8): pass 1 reads HBM, pass 4 leaves butterflies j and
// NB4 - j in registers (bins k and M - k of the packed spectrum, as in
// k_fir2).  Inverse: the same engine on conj Z' with radices (8, 8, 16, 16),
// pass 1' from registers, pass 4' to HBM.
//
// Exchange layouts phys(x) = x + x / S (S = 0: identity), chosen per exchange
// with the LDS bank model of MI355X_MICROARCH.md (ds_write_b64: 16-lane groups
// over 32 banks; ds_read_b64: 32-lane groups over 64 banks), extra cycles per
// transform (write, read): E1 S=16 (0, 512), E2 S=0 (0, 0), E3 S=0 (0, 0),
// E1' S=8 (0, 512), E2' S=8 (0, 512), E3' S=0 (0, 0).
#pragma once
#include "fir_fft.h"

template <int M> struct Fir4Cfg;
template <> struct Fir4Cfg<16384> { static constexpr int R1 = 16, R2 = 16, R3 = 8, R4 = 8; };

// Exchange-buffer layouts.  S > 0: one pad slot per S elements.  S < 0: XOR
// swizzles that keep the buffer unpadded and every access of the k_fir4 engine
// bank-conflict-free in the MI355X_MICROARCH.md LDS model (tools/lds_banks_fir8.py):
//   -16  x ^ ((x >> 4) & 15)        pass-1 writes of 16 consecutive, reads of consecutive
//    -8  x ^ ((x >> 4) & 7)         pass-1' writes of 8 consecutive, reads of consecutive
//    -1  x ^ (((x >> 6) & 1) << 3)  pass-2' writes of 8-runs at stride 8 (NS R = 64), consecutive reads
// (additive pads cannot serve both sides of E1 / E1': the reads of 32 consecutive
// elements wrap the 64 banks when a pad falls inside them).  The swizzles move
// bits below 8 only, so lay(x + r NB) = lay(x) + r NB for the 1024-multiples NB.
template <int S> MSG_HD constexpr int pads(int x) {
    if constexpr (S > 0) return x + x / S;
    else if constexpr (S == -16) return x ^ ((x >> 4) & 15);
    else if constexpr (S == -8) return x ^ ((x >> 4) & 7);
    else if constexpr (S == -1) return x ^ (((x >> 6) & 1) << 3);
    else return x;
}
// Block epilogue of the overlap-save kernels: segment samples (u, u + 1) go to
// frames t0 + d, d = u - (P - 1), kept for d in [0, span), span = min(n - t0,
// B).  32-bit offsets from the block's (uniform) first frame, one unsigned
// compare per value (d < 0 wraps), and the pair as one 8-byte store when P is
// odd (d even) and the mono region is 8-byte aligned.
struct SegOut {
    float* yt;
    uint32_t span;
    bool pairs;
    MSG_DEV void put(uint32_t d, float2 val) const {
        if (pairs) {
            if (d + 1 < span) *reinterpret_cast<float2*>(reinterpret_cast<char*>(yt) + d * 4u) = val;
            else if (d < span) at32(yt, d) = val.x;
        } else {
            if (d < span) at32(yt, d) = val.x;
            if (d + 1 < span) at32(yt, d + 1) = val.y;
        }
    }
};
MSG_DEV SegOut seg_out(float* y_out, int64_t y_off, int64_t t0, int64_t n, int B, int P) {
    SegOut so;
    so.yt = y_out + y_off + t0;
    so.span = (uint32_t)(n - t0 < (int64_t)B ? n - t0 : (int64_t)B);
    so.pairs = (P & 1) && ((y_off & 1) == 0);
    return so;
}

// Pass-1 style writes of R consecutive elements from R j: element r at base + r
// (pads) or base ^ r (swizzles, whose source bits lie above log2 R).
template <int S, int R> MSG_DEV void put_run(float2* buf, int j, const float2 (&v)[R]) {
    const int b = pads<S>(R * j);
    if constexpr (S < 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) buf[b ^ r] = v[r];
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) buf[b + r] = v[r];
    }
}

// Two-level twiddle table of Fir4Geo: w_M^j = hi[j >> 7] * lo[j & 127].  The lo
// table is stored padded, lo[x] at x + (x >> 5): the radix-16 table passes and
// the radix-8 power passes read lo at (e r) & 127 for power-of-two multiples e,
// which the unpadded layout put on 2 - 8 banks of a 32-lane read group
// (tools/lds_banks_fir8.py: 2240 -> 704 extra LDS cycles per forward + inverse
// transform pair of k_fir8).
constexpr int FIR4_LO = 132;                       // padded lo entries (127 + 3 + 1, rounded)
MSG_HD constexpr int fir4_lo(int x) { return x + (x >> 5); }
MSG_DEV float2 fir4_wM(const float2* tab, int lo, int hi, int j) {
    return cmul(tab[hi + (j >> 7)], tab[lo + fir4_lo(j & 127)]);
}

// v[r] *= W_M^(e r), r = 1 .. R-1, W_M from the two-level table at (lo, hi).
// Table twiddles: each is one product of two correctly rounded entries (~1 ulp,
// two LDS reads and a complex multiply); power twiddles (twiddle_pow_ab): from
// two table values by up to ~6 roundings at R = 16 (R = 8: ~3).
// MSG_FIR_TWTAB = 1: table twiddles in every pass, 2: for the radix-16 passes
// (the inverse's passes 3' and 4'; the forward's radix-16 pass 2 reads exact
// [r][k] tables), powers for radix 8, 0: powers everywhere.
#ifndef MSG_FIR_TWTAB
#define MSG_FIR_TWTAB 2
#endif
template <int M, int R>
MSG_DEV void fir_twiddle(float2 (&v)[R], const float2* tab, int lo, int hi, int e) {
    if constexpr (MSG_FIR_TWTAB == 1 || (MSG_FIR_TWTAB == 2 && R >= 16)) {
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], fir4_wM(tab, lo, hi, (e * r) & (M - 1)));
    } else {
        constexpr int B = tw_base<R>();
        twiddle_pow_ab<R, B>(v, fir4_wM(tab, lo, hi, e), fir4_wM(tab, lo, hi, (e * B) & (M - 1)));
    }
}

// v[r] *= w_M^(e r), r = 1 .. R-1, e = 64 a + b < 64 NA, from the split tables at
// (oa, ob): w_M^(64 a r) at oa + r NA + a, w_M^(b r) at ob + r 64 + b.
template <int R, int NA>
MSG_DEV void fir_twiddle_t(float2 (&v)[R], const float2* tab, int oa, int ob, int e) {
    const float2* ta = tab + oa + (e >> 6);
    const float2* tb = tab + ob + (e & 63);
#pragma unroll
    for (int r = 1; r < R; ++r) v[r] = cmul(v[r], cmul(ta[r * NA], tb[r * 64]));
}

// Forward pass 4's twiddles (radix R4, exponent j < NB4): split tables (1, one
// product of two correctly rounded entries) or powers of two two-level table
// values (0, twiddle_pow_ab: up to ~3 roundings at R = 8).  Tuning macro.
#ifndef MSG_FIR_P4TAB
#define MSG_FIR_P4TAB 1
#endif

template <int M> struct Fir4Geo {
    static constexpr int R1 = Fir4Cfg<M>::R1, R2 = Fir4Cfg<M>::R2, R3 = Fir4Cfg<M>::R3, R4 = Fir4Cfg<M>::R4;
    static_assert(R1 * R2 * R3 * R4 == M, "four passes");
    static constexpr int T = M / (2 * R4);
    static constexpr int NB1 = M / R1, NB2 = M / R2, NB3 = M / R3, NB4 = M / R4;
    static constexpr int BP1 = NB1 / T, BP2 = NB2 / T, BP3 = NB3 / T;
    static_assert(NB1 % T == 0 && NB2 % T == 0 && NB3 % T == 0 && NB4 == 2 * T, "FIR4 plan");
    // exchange pads: forward E1..E3, inverse E1'..E3'
#ifndef MSG_FIR4_PADS   // tuning builds: exchange layouts S1, S2, S3, S1I, S2I, S3I (pads()); round 2: 16, 0, 0, 8, 8, 0
#define MSG_FIR4_PADS -16, 0, 0, -8, -1, 0
#endif
    static constexpr int PADS_[6] = {MSG_FIR4_PADS};
    static constexpr int S1 = PADS_[0], S2 = PADS_[1], S3 = PADS_[2], S1I = PADS_[3], S2I = PADS_[4], S3I = PADS_[5];
    static_assert((S1 == R1 || S1 == -16) && (S1I == R4 || S1I == -8), "pass-1 writes of R consecutive elements");
    static_assert(S2I != -1 || R3 * R4 == 64, "swizzle -1: pass-2' writes of 8-runs at stride 8");
    // twiddle tables at LDS offset 0 (float2 entries): exact [r][k] tables for the
    // two passes with small NS, two-level w_M and w_2M tables for the rest
    static constexpr int OFF_TA = 0;                    // forward pass 2: radix R2, NS = R1, [R2][R1]
    static constexpr int OFF_TB = OFF_TA + R2 * R1;     // inverse pass 2': radix R3, NS = R4, [R3][R4]
    static constexpr int OFF_MLO = OFF_TB + R3 * R4;    // w_M^x, x < 128 (at fir4_lo(x))
    static constexpr int OFF_MHI = OFF_MLO + FIR4_LO;   // w_M^(128 x), x < M / 128
    static constexpr int OFF_PLO = OFF_MHI + M / 128;   // w_2M^x, x < 128 (at fir4_lo(x))
    static constexpr int OFF_PHI = OFF_PLO + FIR4_LO;   // w_2M^(128 x), 128 x <= NB4
    static constexpr int OFF_TC = OFF_PHI + NB4 / 128 + 1;   // inverse pass 3': radix R2, NS = R4 R3, [R2][R4 R3]
    // inverse pass 4' (radix R1, twiddle w_M^(t r), t < T): w_M^(64 a r) [R1][T/64] times w_M^(b r) [R1][64],
    // t = 64 a + b -- one product of two table entries at fixed offsets, no index arithmetic
    static constexpr int OFF_T4A = OFF_TC + R2 * R4 * R3;
    static constexpr int OFF_T4B = OFF_T4A + R1 * (T / 64);
    // forward pass 4 (radix R4, w_M^(j r), j < NB4): the same split, [R4][NB4/64] and [R4][64]
    static constexpr int OFF_T5A = OFF_T4B + R1 * 64;
    static constexpr int OFF_T5B = OFF_T5A + R4 * (NB4 / 64);
    static constexpr int TAB_USED = OFF_T5B + R4 * 64;
    static constexpr int TAB = (TAB_USED + 15) & ~15;
    static constexpr int BUF = M + ((S1 > 0 || S2 > 0 || S3 > 0 || S1I > 0 || S2I > 0 || S3I > 0) ? M / 8 : 0);
    static constexpr int LDS_BYTES = (TAB + BUF) * 8;
    static_assert(LDS_BYTES <= 163840, "FIR4 LDS budget");
};

template <int M, int R4>
MSG_DEV void fir_twiddle_p4(float2 (&v)[R4], const float2* tab, int j) {
    using G = Fir4Geo<M>;
#if MSG_FIR_P4TAB
    fir_twiddle_t<R4, G::NB4 / 64>(v, tab, G::OFF_T5A, G::OFF_T5B, j);
#else
    fir_twiddle<M, R4>(v, tab, G::OFF_MLO, G::OFF_MHI, j);
#endif
}

// One radix-R Stockham pass LDS -> LDS on the 1024-thread grid.  TW: the
// twiddles w_{NS R}^{k r} from the exact [r][k] table at OFF_T (TAB = true) or
// as powers of w_M^{k M/(NS R)} from the two-level w_M table.
template <int M, int R, int NS, int BP, int SI, int SO, bool TAB, int OFF_T>
MSG_DEV void fir4_pass_lds(float2* buf, const float2* tab, int t) {
    using G = Fir4Geo<M>;
    constexpr int NB = M / R, T = G::T, STEP = M / (NS * R);
    static_assert(SI == 0 || NB % SI == 0, "additive read addresses");
    float2 v[BP][R];
#pragma unroll
    for (int b = 0; b < BP; ++b) {
        const int base = pads<SI>(t + b * T);
#pragma unroll
        for (int r = 0; r < R; ++r) v[b][r] = buf[base + pads<SI>(r * NB)];
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BP; ++b) {
        const int j = t + b * T;
        const int k = j & (NS - 1), q = j / NS;
        if constexpr (TAB) {
#pragma unroll
            for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tab[OFF_T + r * NS + k]);
        } else {
            fir_twiddle<M, R>(v[b], tab, G::OFF_MLO, G::OFF_MHI, k * STEP);
        }
        Dft<R, false>::run(v[b]);
        const int lo = q * NS * R + k;
        if constexpr (SO == -1) {                   // lo + r NS = lo | r NS (NS R = 64): base ^ r NS
            const int bb = lo | (((lo >> 6) & 1) << 3);
#pragma unroll
            for (int r = 0; r < R; ++r) buf[bb ^ (r * NS)] = v[b][r];
        } else {
#pragma unroll
            for (int r = 0; r < R; ++r) buf[pads<SO>(lo + r * NS)] = v[b][r];
        }
    }
}

template <int M>
__global__ void __launch_bounds__(Fir4Geo<M>::T)
k_fir4(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
       const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out) {
    using G = Fir4Geo<M>;
    constexpr int T = G::T, R1 = G::R1, R2 = G::R2, R3 = G::R3, R4 = G::R4;
    constexpr int NB1 = G::NB1, NB4 = G::NB4;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int2 job = jobs[xcd_block(blockIdx.x, gridDim.x)];
    const PresetRt& pr = rt[job.x];
    const int P = pr.fir_P, Q = pr.fir_Q;
    const int64_t n = pr.out_n;
    const int64_t t0 = (int64_t)job.y * pr.fir_B;
    const float* x = x_in + pr.y_off;
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }   // one memory latency, not one per T entries

    float2 acc[2][R4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R4; ++r) acc[h][r] = make_float2(0.f, 0.f);

    for (int q = 0; q < Q; ++q) {
        const int t = otid();
        const bool t0z = (t == 0);
        const int js[2] = {t, t0z ? NB4 / 2 : NB4 - t};
        // ---- pass 1: x segment (zero outside [0, n)) -> DFT_R1 -> LDS (E1)
        const int64_t s0 = t0 - (int64_t)q * P - (P - 1);
        const bool fast = s0 >= 0 && s0 + 2 * M <= n && (((uintptr_t)(x + s0)) & 7) == 0;
        {
            float2 v[R1];
            if (fast) {
                const float2* z = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
                for (int r = 0; r < R1; ++r) v[r] = z[(uint32_t)(t + r * NB1)];
            } else {
#pragma unroll
                for (int r = 0; r < R1; ++r) {
                    const int64_t a = s0 + 2 * (int64_t)(t + r * NB1);
                    const bool in0 = a >= 0 && a < n, in1 = a + 1 >= 0 && a + 1 < n;
                    const float x0 = x[(uint32_t)(in0 ? a : 0)], x1 = x[(uint32_t)(in1 ? a + 1 : 0)];
                    v[r] = make_float2(in0 ? x0 : 0.f, in1 ? x1 : 0.f);
                }
            }
            Dft<R1, false>::run(v);
            put_run<G::S1, R1>(buf, t, v);
        }
        __syncthreads();
        // ---- passes 2, 3: LDS -> LDS (E1 -> E2 -> E3)
        fir4_pass_lds<M, R2, R1, G::BP2, G::S1, G::S2, true, G::OFF_TA>(buf, tab, t);
        __syncthreads();
        fir4_pass_lds<M, R3, R1 * R2, G::BP3, G::S2, G::S3, false, 0>(buf, tab, t);
        __syncthreads();
        // ---- pass 4: LDS (E3) -> registers, butterflies j and NB4 - j
        float2 v[2][R4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int r = 0; r < R4; ++r) v[h][r] = buf[pads<G::S3>(js[h] + r * NB4)];
        }
        __syncthreads();   // LDS free for the next segment / the inverse
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            fir_twiddle_p4<M, R4>(v[h], tab, js[h]);
            Dft<R4, false>::run(v[h]);
        }
        // ---- real split, X . H_q accumulated in registers (k_fir2's pairing)
        const float2* H = hspec + pr.h_off + (int64_t)q * (M + 1);
        if (!t0z) {
            const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, js[0]);
#pragma unroll
            for (int r = 0; r < R4; ++r) {
                const int kA = js[0] + r * NB4;
                const float2 hk = at32(H, kA), hm = at32(H, M - kA);
                fir_pair_mac(v[0][r], v[1][R4 - 1 - r], cmul_k(wA, fir_cr<R4>(r)), hk, hm, acc[0][r],
                             acc[1][R4 - 1 - r]);
            }
        } else {
            float2 a[R4], bb[R4];
            fir_slots<R4>(v, a, bb, true);
            const float2 hmid = H[M / 2];
#pragma unroll
            for (int r = 0; r < R4; ++r) {
                const int kA = fir_k0<M, R4>(r);
                const float2 hk = at32(H, kA), hm = at32(H, M - kA);
                if (r < R4 - 1) {
                    fir_pair_mac(a[r], bb[R4 - 1 - r], fir_w0<M, R4>(r), hk, hm, acc[0][r], acc[1][R4 - 1 - r]);
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
            const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
            for (int r = 0; r < R4; ++r) fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], cmul_k(wA, fir_cr<R4>(r)));
        } else {
#pragma unroll
            for (int r = 0; r < R4 - 1; ++r) fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], fir_w0<M, R4>(r));
            const float y0 = acc[0][R4 - 1].x, yN = acc[0][R4 - 1].y;
            acc[0][R4 - 1] = make_float2(0.5f * (y0 + yN), -0.5f * (y0 - yN));   // bin M/2: conj Z' = Y
            fir_unslots<R4>(acc, true);
        }
    }
    const int t = otid();
    const int js[2] = {t, t == 0 ? NB4 / 2 : NB4 - t};
    // ---- pass 1': registers -> DFT_R4 -> LDS (E1')
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Dft<R4, false>::run(acc[h]);
        put_run<G::S1I, R4>(buf, js[h], acc[h]);
    }
    __syncthreads();
    // ---- passes 2', 3': LDS -> LDS (E1' -> E2' -> E3')
    fir4_pass_lds<M, R3, R4, G::BP3, G::S1I, G::S2I, true, G::OFF_TB>(buf, tab, t);
    __syncthreads();
    fir4_pass_lds<M, R2, R4 * R3, G::BP2, G::S2I, G::S3I, true, G::OFF_TC>(buf, tab, t);
    __syncthreads();
    // ---- pass 4': LDS (E3') -> DFT_R1 -> output block (samples u >= P-1 of the segment)
    const float s = 1.0f / (float)M;
    {
        float2 v[R1];
#pragma unroll
        for (int r = 0; r < R1; ++r) v[r] = buf[pads<G::S3I>(t + r * NB1)];
        fir_twiddle_t<R1, T / 64>(v, tab, G::OFF_T4A, G::OFF_T4B, t);
        Dft<R1, false>::run(v);
        const SegOut so = seg_out(y_out, pr.y_off, t0, n, 2 * M - P + 1, P);
#pragma unroll
        for (int r = 0; r < R1; ++r)                         // z[u/2] = x[u] + i x[u+1], u = 2 (t + r NB1)
            so.put((uint32_t)(2 * (t + r * NB1) - (P - 1)), make_float2(v[r].x * s, -v[r].y * s));
    }
}

// ---------------------------------------------------------------------------
// Streaming variant: uniformly partitioned overlap-save with the one pending
// partition product held in registers across a workgroup's consecutive blocks.
//
// With the block hop equal to the partition size (B = P = M, N = 2M), the
// segment of partition q of block b is the segment of partition 0 of block
// b - q, so X_{b,q} = X_{b-q}.  For Q <= 2 a workgroup walking blocks b0 ..
// b0+K-1 of one preset keeps A = X_{b-1} . H_1 in the accumulator registers:
//     Y_b = X_b . H_0 + A,   then A <- X_b . H_1 once Y_b has left for LDS,
// so a block costs one forward and one inverse transform (plus one forward
// for X_{b0-1} per workgroup) instead of Q + 1 = 3.  The transforms, the real
// split and the MAC are k_fir4's, so the result equals k_fir4 run with B = P.
// Register pressure: A is live through the inverse passes 2'..4' exactly as
// the accumulator is live through the forward passes of k_fir4's segment loop.
// Jobs: (preset, first block); the workgroup runs min(K, blocks - b0) blocks.
//
// Measured on MI355X (C3, 512 presets per launch, profiles/r02t_*): 17 % fewer
// transforms and VALU instructions than k_fir4, but every block re-reads H_0
// and H_1 (256 KB), and with a C3 preset's 24 blocks cut into runs of K the 32
// workgroups of an XCD touch 32/(24/K) presets at once: their spectra do not
// stay in the 4 MB L2 beside the x/y streams.  HBM traffic 1.82 -> 3.40 GB
// (K = 6) / 4.20 GB (K = 12) per launch; isolated kernel time 2.59 ms (k_fir4)
// vs 2.55-2.67 ms, whole step unchanged.  Hence opt-in (MSGPU_FIR4S=1).
// ---------------------------------------------------------------------------
// The x segments and y blocks stream through L2 once (x twice, one block apart,
// from the same workgroup) while H_0 and H_1 are re-read by every block.
// MSG_FIR4S_NT=1 (tuning builds) sends the streams with the nontemporal policy:
// measured on C3 it cut reads 2.6 -> 2.0 GB per 512 presets but split the
// interleaved y stores into partial lines (writes 0.81 -> 1.24 GB), net slower.
#ifndef MSG_FIR4S_NT
#define MSG_FIR4S_NT 0
#endif
MSG_DEV float fir4s_ld(const float* p) {
#if MSG_FIR4S_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}
MSG_DEV float2 fir4s_ld(const float2* p) {
#if MSG_FIR4S_NT
    return ff(__builtin_nontemporal_load(reinterpret_cast<const f2v*>(p)));
#else
    return *p;
#endif
}
MSG_DEV void fir4s_st(float* p, float v) {
#if MSG_FIR4S_NT
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}

// Forward transform of x[s0, s0 + 2M) (zero outside [0, n)), passes 1-4 and the
// real split: v holds X at bins (js[0] + r NB4, M - that) in k_fir4's slot pairing
// (thread 0: the slot layout of fir_slots, a[R4-1] = (X[0], X[M]), b[0] = X[M/2]).
// LDS_IN: the packed input z[m] = x[2m] + i x[2m+1], m < M, is already in buf
// (natural order) instead of being read from x.
template <int M, bool LDS_IN = false>
MSG_DEV void fir4s_forward(float2* buf, const float2* tab, const float* x, int64_t n, int64_t s0,
                           float2 (&v)[2][Fir4Geo<M>::R4]) {
    using G = Fir4Geo<M>;
    constexpr int R1 = G::R1, R2 = G::R2, R3 = G::R3, R4 = G::R4, NB1 = G::NB1, NB4 = G::NB4;
    const int t = otid();
    const bool t0z = (t == 0);
    const int js[2] = {t, t0z ? NB4 / 2 : NB4 - t};
    const bool fast = !LDS_IN && s0 >= 0 && s0 + 2 * M <= n && (((uintptr_t)(x + s0)) & 7) == 0;
    {
        float2 u[R1];
        if (LDS_IN) {
#pragma unroll
            for (int r = 0; r < R1; ++r) u[r] = buf[t + r * NB1];
            __syncthreads();   // every input read before pass 1 overwrites buf
        } else if (fast) {
            const float2* z = reinterpret_cast<const float2*>(x + s0);
#pragma unroll
            for (int r = 0; r < R1; ++r) u[r] = fir4s_ld(z + (uint32_t)(t + r * NB1));
        } else {
#pragma unroll
            for (int r = 0; r < R1; ++r) {
                const int64_t a = s0 + 2 * (int64_t)(t + r * NB1);
                const bool in0 = a >= 0 && a < n, in1 = a + 1 >= 0 && a + 1 < n;
                const float x0 = fir4s_ld(x + (uint32_t)(in0 ? a : 0)), x1 = fir4s_ld(x + (uint32_t)(in1 ? a + 1 : 0));
                u[r] = make_float2(in0 ? x0 : 0.f, in1 ? x1 : 0.f);
            }
        }
        Dft<R1, false>::run(u);
        put_run<G::S1, R1>(buf, t, u);
    }
    __syncthreads();
    fir4_pass_lds<M, R2, R1, G::BP2, G::S1, G::S2, true, G::OFF_TA>(buf, tab, t);
    __syncthreads();
    fir4_pass_lds<M, R3, R1 * R2, G::BP3, G::S2, G::S3, false, 0>(buf, tab, t);
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int r = 0; r < R4; ++r) v[h][r] = buf[pads<G::S3>(js[h] + r * NB4)];
    }
    __syncthreads();   // LDS free for the inverse
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        fir_twiddle_p4<M, R4>(v[h], tab, js[h]);
        Dft<R4, false>::run(v[h]);
    }
    if (!t0z) {
        const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, js[0]);
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            float2 xk, xm;
            fir_split(v[0][r], v[1][R4 - 1 - r], cmul_k(wA, fir_cr<R4>(r)), xk, xm);
            v[0][r] = xk;
            v[1][R4 - 1 - r] = xm;
        }
    } else {
        float2 a[R4], bb[R4];
        fir_slots<R4>(v, a, bb, true);
#pragma unroll
        for (int r = 0; r < R4 - 1; ++r) fir_split(a[r], bb[R4 - 1 - r], fir_w0<M, R4>(r), a[r], bb[R4 - 1 - r]);
        const float2 z0 = a[R4 - 1];
        a[R4 - 1] = make_float2(z0.x + z0.y, z0.x - z0.y);   // (X[0], X[M]), both real
        bb[0] = cconj(bb[0]);                                 // X[M/2]
#pragma unroll
        for (int r = 0; r < R4; ++r) { v[0][r] = a[r]; v[1][r] = bb[r]; }
    }
}

// acc += X . H (bins as fir4s_forward leaves them)
template <int M>
MSG_DEV void fir4s_mac(float2 (&acc)[2][Fir4Geo<M>::R4], const float2 (&v)[2][Fir4Geo<M>::R4],
                       const float2* __restrict__ H) {
    constexpr int R4 = Fir4Geo<M>::R4, NB4 = Fir4Geo<M>::NB4;
    const int t = otid();
    if (t != 0) {
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            const int kA = t + r * NB4;
            acc[0][r] = cfma(acc[0][r], v[0][r], at32(H, kA));
            acc[1][R4 - 1 - r] = cfma(acc[1][R4 - 1 - r], v[1][R4 - 1 - r], at32(H, M - kA));
        }
    } else {
#pragma unroll
        for (int r = 0; r < R4 - 1; ++r) {
            const int kA = fir_k0<M, R4>(r);
            acc[0][r] = cfma(acc[0][r], v[0][r], H[kA]);
            acc[1][R4 - 1 - r] = cfma(acc[1][R4 - 1 - r], v[1][R4 - 1 - r], H[M - kA]);
        }
        const float2 x0 = v[0][R4 - 1];
        acc[0][R4 - 1] = cadd(acc[0][R4 - 1], make_float2(x0.x * H[0].x, x0.y * H[M].x));
        acc[1][0] = cfma(acc[1][0], v[1][0], H[M / 2]);
    }
}

template <int M>
__global__ void __launch_bounds__(Fir4Geo<M>::T)
k_fir4s(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
        const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out, int kblk) {
    using G = Fir4Geo<M>;
    constexpr int T = G::T, R1 = G::R1, R4 = G::R4, NB1 = G::NB1, NB4 = G::NB4;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int2 job = jobs[xcd_block(blockIdx.x, gridDim.x)];
    const PresetRt& pr = rt[job.x];
    const int P = pr.fir_P, Q = pr.fir_Q;   // P == M (B == P), Q <= 2
    const int64_t n = pr.out_n;
    const int nblk = (int)((n + P - 1) / P);
    const int b0 = job.y, b1 = b0 + kblk < nblk ? b0 + kblk : nblk;
    const float* x = x_in + pr.y_off;
    float* y = y_out + pr.y_off;
    const float2* H0 = hspec + pr.h_off;
    const float2* H1 = H0 + (M + 1);
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }   // one memory latency, not one per T entries

    float2 acc[2][R4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R4; ++r) acc[h][r] = make_float2(0.f, 0.f);
    // Q == 2: the walk starts one block early, where it only forms A = X_{b0-1} . H_1
    for (int b = Q == 2 ? b0 - 1 : b0; b < b1; ++b) {
        const int64_t t0 = (int64_t)b * P;
        float2 v[2][R4];
        fir4s_forward<M>(buf, tab, x, n, t0 - (P - 1), v);
        fir4s_mac<M>(acc, v, b < b0 ? H1 : H0);
        if (b < b0) continue;
        // ---- inverse pre-step and pass 1' (registers -> LDS E1'), as k_fir4
        {
            const int t = otid();
            if (t != 0) {
                const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
                for (int r = 0; r < R4; ++r) fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], cmul_k(wA, fir_cr<R4>(r)));
            } else {
#pragma unroll
                for (int r = 0; r < R4 - 1; ++r) fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], fir_w0<M, R4>(r));
                const float y0 = acc[0][R4 - 1].x, yN = acc[0][R4 - 1].y;
                acc[0][R4 - 1] = make_float2(0.5f * (y0 + yN), -0.5f * (y0 - yN));
                fir_unslots<R4>(acc, true);
            }
            const int js[2] = {t, t == 0 ? NB4 / 2 : NB4 - t};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                Dft<R4, false>::run(acc[h]);
                put_run<G::S1I, R4>(buf, js[h], acc[h]);
            }
        }
        // ---- A <- X_b . H_1 (Y_b is in LDS; X_b dies here)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < R4; ++r) acc[h][r] = make_float2(0.f, 0.f);
        if (Q == 2) fir4s_mac<M>(acc, v, H1);
        __syncthreads();
        const int t = otid();
        fir4_pass_lds<M, G::R3, R4, G::BP3, G::S1I, G::S2I, true, G::OFF_TB>(buf, tab, t);
        __syncthreads();
        fir4_pass_lds<M, G::R2, R4 * G::R3, G::BP2, G::S2I, G::S3I, true, G::OFF_TC>(buf, tab, t);
        __syncthreads();
        // ---- pass 4': LDS (E3') -> DFT_R1 -> outputs [t0, t0 + P) (segment samples u >= P-1)
        {
            const float s = 1.0f / (float)M;
            float2 u[R1];
#pragma unroll
            for (int r = 0; r < R1; ++r) u[r] = buf[pads<G::S3I>(t + r * NB1)];
            fir_twiddle_t<R1, T / 64>(u, tab, G::OFF_T4A, G::OFF_T4B, t);
            Dft<R1, false>::run(u);
#pragma unroll
            for (int r = 0; r < R1; ++r) {
                const int w = 2 * (t + r * NB1) - (P - 1);   // output offset in the block
                const int64_t o = t0 + w;
                if (w >= 0 && w < P && o < n) fir4s_st(y + (uint32_t)o, u[r].x * s);
                if (w + 1 >= 0 && w + 1 < P && o + 1 < n) fir4s_st(y + (uint32_t)(o + 1), -u[r].y * s);
            }
        }
        __syncthreads();   // pass 4' reads done before the next forward's pass 1 writes
    }
}

// ---------------------------------------------------------------------------
// FIR partition spectra on the k_fir4 engine (N = 2M = 32768), the C3/C4 path:
// one workgroup per (preset, q), H_q = rfft(h[qP, qP + P)) zero-padded to N,
// from k_h_build's time-domain h (kernels_fir.h), written in natural bin order
// (k_fir4 / k_fir2's hspec layout).  The general-size k_fir_h runs the same
// transform on the 512-thread runtime-plan engine at ~3x k_fir4's time.
// ---------------------------------------------------------------------------
template <int M>
__global__ void __launch_bounds__(Fir4Geo<M>::T)
k_fir4_hpart(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
             const float* __restrict__ hs, float2* __restrict__ hspec) {
    using G = Fir4Geo<M>;
    constexpr int T = G::T, R4 = G::R4, NB4 = G::NB4;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int2 job = jobs[blockIdx.x];
    const PresetRt& r = rt[job.x];
    const int q = job.y, P = r.fir_P;
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }   // one memory latency, not one per T entries
    const int64_t s0 = (int64_t)q * P;
    const int64_t len = P < r.h_len - s0 ? P : r.h_len - s0;               // h[qP, qP + P), zero-padded to N
    float2 v[2][R4];
    fir4s_forward<M>(buf, tab, hs + r.hs_off + s0, len, 0, v);
    float2* H = hspec + r.h_off + (int64_t)q * (M + 1);
    const int t = otid();
    if (t != 0) {
#pragma unroll
        for (int k = 0; k < R4; ++k) {
            const int kA = t + k * NB4;
            at32(H, kA) = v[0][k];
            at32(H, M - kA) = v[1][R4 - 1 - k];
        }
    } else {   // thread 0's slot layout (fir4s_forward): (X[0], X[M]) packed, X[M/2]
#pragma unroll
        for (int k = 0; k < R4 - 1; ++k) {
            const int kA = fir_k0<M, R4>(k);
            H[kA] = v[0][k];
            H[M - kA] = v[1][R4 - 1 - k];
        }
        H[0] = make_float2(v[0][R4 - 1].x, 0.f);
        H[M] = make_float2(v[0][R4 - 1].y, 0.f);
        H[M / 2] = v[1][0];
    }
}

// One-partition spectra at N = 2M straight from the taps, the k_fir8_hconv
// recipe on the k_fir4 engine (round 5; H48's 48 kHz filters: k_h_build's
// float64 time-domain h was 0.21 of the h stage's 0.26 ms per 1024 presets):
//   k_fir4_irspec  S = rfft_N(IR) of each IR of the batch (float64 bank, the
//                  8192-tap cap), jobs (src offset, length, spectrum offset, -);
//   k_fir4_hconv   H = rfft_N(delta + ER taps) . S for a preset whose h =
//                  (delta + ER) * IR fits the transform (h_len <= N: the circular
//                  product is the linear convolution), one workgroup per preset;
//                  the taps are scattered into LDS as the packed input.
// Spectra in natural bin order, M + 1 float2 (k_fir4's hspec layout).
template <int M>
MSG_DEV void fir4_store_spec(const float2 (&v)[2][Fir4Geo<M>::R4], const float2* __restrict__ S, float2* __restrict__ H) {
    constexpr int R4 = Fir4Geo<M>::R4, NB4 = Fir4Geo<M>::NB4;
    const int t = otid();
    auto put = [&](int k, float2 x) { at32(H, (uint32_t)k) = S ? cmul(x, at32(S, (uint32_t)k)) : x; };
    if (t != 0) {
#pragma unroll
        for (int k = 0; k < R4; ++k) {
            const int kA = t + k * NB4;
            put(kA, v[0][k]);
            put(M - kA, v[1][R4 - 1 - k]);
        }
    } else {   // thread 0's slot layout (fir4s_forward): (X[0], X[M]) packed, X[M/2]
#pragma unroll
        for (int k = 0; k < R4 - 1; ++k) {
            const int kA = fir_k0<M, R4>(k);
            put(kA, v[0][k]);
            put(M - kA, v[1][R4 - 1 - k]);
        }
        put(0, make_float2(v[0][R4 - 1].x, 0.f));
        put(M, make_float2(v[0][R4 - 1].y, 0.f));
        put(M / 2, v[1][0]);
    }
}

template <int M>
__global__ void __launch_bounds__(Fir4Geo<M>::T)
k_fir4_irspec(const int64_t* __restrict__ jobs, const float2* __restrict__ tables, const double* __restrict__ src,
              float2* __restrict__ hspec) {
    using G = Fir4Geo<M>;
    constexpr int T = G::T;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int64_t* j = jobs + 4 * blockIdx.x;
    const double* x = src + j[0];
    const int64_t len = j[1];
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }
    for (int m = threadIdx.x; m < M; m += T) {                 // packed z[m] = x[2m] + i x[2m + 1], zero-padded
        const int64_t i = 2 * (int64_t)m;
        buf[m] = make_float2(i < len ? (float)x[i] : 0.f, i + 1 < len ? (float)x[i + 1] : 0.f);
    }
    __syncthreads();
    float2 v[2][G::R4];
    fir4s_forward<M, true>(buf, tab, nullptr, 0, 0, v);
    fir4_store_spec<M>(v, nullptr, hspec + j[2]);
}

template <int M>
__global__ void __launch_bounds__(Fir4Geo<M>::T)
k_fir4_hconv(const PresetRt* __restrict__ rt, const int32_t* __restrict__ list, const float2* __restrict__ tables,
             const int32_t* __restrict__ er_off, const double* __restrict__ er_gain, float2* __restrict__ hspec) {
    using G = Fir4Geo<M>;
    constexpr int T = G::T;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const PresetRt& r = rt[list[blockIdx.x]];
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }
    for (int m = threadIdx.x; m < M; m += T) buf[m] = make_float2(0.f, 0.f);
    __syncthreads();
    // e = delta + taps at real index o (the host merged equal offsets: a slot holds the
    // delta and at most one tap, and two float adds give the same sum in either order)
    float* e = reinterpret_cast<float*>(buf);
    if (threadIdx.x == 0) atomicAdd(e, 1.0f);
    for (int k = threadIdx.x; k < r.n_taps; k += T)
        atomicAdd(e + er_off[r.er_base + k], (float)er_gain[r.er_base + k]);
    __syncthreads();
    float2 v[2][G::R4];
    fir4s_forward<M, true>(buf, tab, nullptr, 0, 0, v);
    fir4_store_spec<M>(v, r.ir_len > 0 ? hspec + r.irs_off : nullptr, hspec + r.h_off);
}

// Host: the twiddle tables of Fir4Geo<M> (float64-built, rounded once).
template <int M>
inline void fir4_tables(std::vector<float>& out) {
    using G = Fir4Geo<M>;
    out.assign(2 * (size_t)G::TAB_USED, 0.f);
    const long double PI = 3.14159265358979323846264338327950288L;
    auto put = [&](int at, long double num, long double den) {
        const long double a = -2.0L * PI * num / den;
        out[2 * at] = (float)cosl(a);
        out[2 * at + 1] = (float)sinl(a);
    };
    for (int r = 0; r < G::R2; ++r)
        for (int k = 0; k < G::R1; ++k) put(G::OFF_TA + r * G::R1 + k, (long double)k * r, (long double)G::R1 * G::R2);
    for (int r = 0; r < G::R3; ++r)
        for (int k = 0; k < G::R4; ++k) put(G::OFF_TB + r * G::R4 + k, (long double)k * r, (long double)G::R4 * G::R3);
    for (int x = 0; x < 128; ++x) put(G::OFF_MLO + fir4_lo(x), x, M);
    for (int x = 0; x < M / 128; ++x) put(G::OFF_MHI + x, 128.0L * x, M);
    for (int x = 0; x < 128; ++x) put(G::OFF_PLO + fir4_lo(x), x, 2.0L * M);
    for (int x = 0; x <= G::NB4 / 128; ++x) put(G::OFF_PHI + x, 128.0L * x, 2.0L * M);
    for (int r = 0; r < G::R2; ++r)
        for (int k = 0; k < G::R4 * G::R3; ++k)
            put(G::OFF_TC + r * G::R4 * G::R3 + k, (long double)k * r, (long double)G::R4 * G::R3 * G::R2);
    for (int r = 0; r < G::R1; ++r) {
        for (int a = 0; a < G::T / 64; ++a) put(G::OFF_T4A + r * (G::T / 64) + a, (long double)((64 * a * r) % M), M);
        for (int b = 0; b < 64; ++b) put(G::OFF_T4B + r * 64 + b, (long double)b * r, M);
    }
    for (int r = 0; r < G::R4; ++r) {
        for (int a = 0; a < G::NB4 / 64; ++a) put(G::OFF_T5A + r * (G::NB4 / 64) + a, (long double)((64 * a * r) % M), M);
        for (int b = 0; b < 64; ++b) put(G::OFF_T5B + r * 64 + b, (long double)b * r, M);
    }
}
