// fft_lds.h — LDS-resident mixed-radix Stockham FFT (+ Bluestein) for gfx950,
// one workgroup per transform.
//
// The reference calls NumPy's pocketfft rfft/irfft at arbitrary lengths
// (MS:46, 66, 106, 122, 135, 153-163, 226-233, 432-435, 573-581).  A grain of
// up to ~40 k samples fits the 160 KiB LDS of one CU as n/2 packed complex
// float32, so a whole spectral chain runs with one HBM read and one HBM write.
//
// Each pass with radix R: every thread loads the R operands of its
// butterflies from LDS into registers, barrier, applies twiddles and a
// register-resident radix-R DFT (R in 2..25; composite radices are
// Cooley-Tukey in registers with compile-time constants), and stores to the
// Stockham autosort position, barrier — in place, no ping-pong buffer.
// Twiddle w^(k*stride) comes from a two-level table staged in LDS
// (tw(i) = T1[i>>7] * T0[i&127], float64-built); its powers w^r by a balanced
// product tree (depth <= 4).  Passes per length (host factorisation): 16384 ->
// 16,16,16,4; 18750 -> 25,25,5,6; 1200 -> 25,3,16.
#pragma once
#include "msg_common.h"

constexpr int FFT_MAXRAD = 16;
constexpr int TW_LO = 128;            // entries of the low-level twiddle table

struct FftDesc {
    int32_t m;            // complex transform length handled by the caller
    int32_t nrad;         // Stockham passes over `size`
    int32_t size;         // = m, or the power-of-two Bluestein length
    int32_t blue;         // 1 -> Bluestein (chirp-z) through `size`
    int32_t rad[FFT_MAXRAD];
    int32_t tw_hi_n;      // entries of the high-level table = ceil(size / 128)
    int32_t pad;
    const float2* tw0;    // exp(-2 pi i j / size), j < 128
    const float2* tw1;    // exp(-2 pi i 128 j / size), j < tw_hi_n
    const float2* chirp;  // Bluestein: exp(-pi i (j*j mod 2m) / m), j < m
    const float2* bspec;  // Bluestein: FFT_size of conj(chirp) wrapped
};

// Real-FFT plan for n samples.  even n: m = n/2 packed complex + post-twiddles;
// odd n: m = n complex with zero imaginary parts.
struct RealPlan {
    int32_t n;
    int32_t even;
    int32_t lds_c;        // physical complex slots of LDS for data (padded, lds_phys)
    int32_t lds_bytes;    // data + staged twiddle tables
    FftDesc c;
    int32_t rt_hi_n;      // even: entries of rt1 = ceil((n/2+1) / 128)
    int32_t pad2;
    const float2* rt0;    // even: exp(-2 pi i j / n), j < 128
    const float2* rt1;    // even: exp(-2 pi i 128 j / n), j < rt_hi_n
};

// Complex arithmetic in the two-lane vector form the gfx950 packed FP32 ALU
// executes directly (v_pk_mul/fma/add_f32 with op_sel/neg modifiers): a complex
// multiply is one v_pk_mul + one v_pk_fma, where the scalar-component form
// compiled to three packed ops and a v_mov per product (static VALU count of
// a radix-5 DFT 25 -> 19, of the k_spec3 kernel 4561 -> 3033).
typedef float f2v __attribute__((ext_vector_type(2)));
MSG_DEV f2v vv(float2 a) { return f2v{a.x, a.y}; }
MSG_DEV float2 ff(f2v a) { return make_float2(a.x, a.y); }
// Products of two register values are written as the two packed instructions
// directly: from the vector form the compiler often materialises (-a.y, a.y)
// with a v_xor + v_mov per product instead of folding the negation and the
// broadcast into neg_lo/op_sel (k_fir2: 451 v_xor + 836 v_mov of 4952 VALU).
// Products with compile-time constants (twc) keep the vector form, whose
// constants the compiler places in SGPRs.
#ifndef MSG_ASM_CMUL
#define MSG_ASM_CMUL 1
#endif
MSG_DEV float2 cmul_v(float2 a, float2 b) {
    return ff(f2v{a.x, a.x} * f2v{b.x, b.y} + f2v{-a.y, a.y} * f2v{b.y, b.x});
}
MSG_DEV float2 cmul(float2 a, float2 b) {
#if MSG_ASM_CMUL
    const f2v x = vv(a), y = vv(b);
    f2v r, t;
    // t = (a.x b.x, a.x b.y);  r = (-a.y b.y + t.x, a.y b.x + t.y)
    asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
        : "=v"(r), "=&v"(t) : "v"(x), "v"(y));
    return ff(r);
#else
    return cmul_v(a, b);
#endif
}
// a * b for a wave-uniform (compile-time) b, held in an SGPR pair
MSG_DEV float2 cmul_k(float2 a, float2 b) {
#if MSG_ASM_CMUL
    const f2v x = vv(a), y = vv(b);
    f2v r, t;
    asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
        : "=v"(r), "=&v"(t) : "v"(x), "s"(y));
    return ff(r);
#else
    return cmul_v(a, b);
#endif
}
// a + (-+i) d and a - (-+i) d (forward sign -1, inverse +1) as single packed adds
template <bool INV> MSG_DEV f2v add_mi(f2v a, f2v d) {
#if MSG_ASM_CMUL
    f2v r;
    if (INV) asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(d));
    else asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(d));
    return r;
#else
    return a + f2v{d.y, d.x} * (INV ? f2v{-1.f, 1.f} : f2v{1.f, -1.f});
#endif
}
template <bool INV> MSG_DEV f2v sub_mi(f2v a, f2v d) { return add_mi<!INV>(a, d); }
// acc + (b.y, b.x) * (s, -s): the odd-radix sine term, s wave-uniform
MSG_DEV f2v fma_swap_k(f2v b, f2v sv, f2v acc) {
#if MSG_ASM_CMUL
    f2v r;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,1,1]" : "=v"(r) : "v"(b), "s"(sv), "v"(acc));
    return r;
#else
    return acc + f2v{b.y, b.x} * sv;
#endif
}
// acc + a * b (complex multiply-accumulate in two packed FMAs)
MSG_DEV float2 cfma(float2 acc, float2 a, float2 b) {
#if MSG_ASM_CMUL
    const f2v x = vv(a), y = vv(b), c = vv(acc);
    f2v r, t;
    asm("v_pk_fma_f32 %1, %2, %3, %4 op_sel_hi:[0,1,1]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
        : "=v"(r), "=&v"(t) : "v"(x), "v"(y), "v"(c));
    return ff(r);
#else
    return ff(vv(acc) + vv(cmul_v(a, b)));
#endif
}
// (a.x + b.x, a.y - b.y) and (a.x - b.x, a.y + b.y): a + conj(b), a - conj(b)
MSG_DEV f2v add_conj(f2v a, f2v b) {
#if MSG_ASM_CMUL
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return f2v{a.x + b.x, a.y - b.y};
#endif
}
MSG_DEV f2v sub_conj(f2v a, f2v b) {
#if MSG_ASM_CMUL
    f2v r;
    asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return f2v{a.x - b.x, a.y + b.y};
#endif
}
MSG_DEV float2 cmulc(float2 a, float2 b) {   // a * conj(b)
#if MSG_ASM_CMUL
    const f2v x = vv(a), y = vv(b);
    f2v r, t;
    // t = (a.x b.x, a.y b.x);  r = (a.y b.y + t.x, -a.x b.y + t.y)
    asm("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %0, %2, %3, %1 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]"
        : "=v"(r), "=&v"(t) : "v"(x), "v"(y));
    return ff(r);
#else
    return ff(f2v{a.x, a.y} * f2v{b.x, b.x} + f2v{a.y, -a.x} * f2v{b.y, b.y});
#endif
}
MSG_DEV float2 cadd(float2 a, float2 b) { return ff(vv(a) + vv(b)); }
MSG_DEV float2 csub(float2 a, float2 b) { return ff(vv(a) - vv(b)); }
MSG_DEV float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
MSG_DEV float2 cscale(float2 a, float s) { return ff(vv(a) * s); }
template <bool INV> MSG_DEV float2 mul_mi(float2 a) { return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x); }

// ---- register-resident DFT kernels (forward sign -1, inverse +1), in place ----
template <int R, bool INV> struct Dft;

template <bool INV> struct Dft<2, INV> {
    static MSG_DEV void run(float2* v) { const f2v a = vv(v[0]), b = vv(v[1]); v[0] = ff(a + b); v[1] = ff(a - b); }
};
template <bool INV> struct Dft<4, INV> {
    static MSG_DEV void run(float2* v) {
        const f2v a0 = vv(v[0]) + vv(v[2]), a1 = vv(v[0]) - vv(v[2]);
        const f2v b0 = vv(v[1]) + vv(v[3]), d = vv(v[1]) - vv(v[3]);
        // v1 = a1 + (-+i) d, v3 = a1 - (-+i) d
        v[0] = ff(a0 + b0); v[2] = ff(a0 - b0);
        v[1] = ff(add_mi<INV>(a1, d)); v[3] = ff(sub_mi<INV>(a1, d));
    }
};
template <int R, bool INV> struct DftOdd {   // odd prime radices, symmetric-pair form
    static MSG_DEV void run(float2* v) {
        constexpr int H = (R - 1) / 2;
        f2v a[H], b[H];
        const f2v x0 = vv(v[0]);
        f2v s0 = x0;
#pragma unroll
        for (int j = 1; j <= H; ++j) {
            a[j - 1] = vv(v[j]) + vv(v[R - j]);
            b[j - 1] = vv(v[j]) - vv(v[R - j]);
            s0 += a[j - 1];
        }
        float2 out[R];
        out[0] = ff(s0);
#pragma unroll
        for (int k = 1; k <= H; ++k) {
            f2v re = x0, im = f2v{0.f, 0.f};
#pragma unroll
            for (int j = 1; j <= H; ++j) {
                const int jk = (j * k) % R;
                const float c = (float)__builtin_cos(2.0 * 3.14159265358979323846 * jk / R);
                const float sn = (float)__builtin_sin(2.0 * 3.14159265358979323846 * jk / R);
                re += a[j - 1] * c;
                // -+i sn b: (b.y sn, -b.x sn) forward, (-b.y sn, b.x sn) inverse
                im = fma_swap_k(b[j - 1], INV ? f2v{-sn, sn} : f2v{sn, -sn}, im);
            }
            out[k] = ff(re + im);
            out[R - k] = ff(re - im);
        }
#pragma unroll
        for (int k = 0; k < R; ++k) v[k] = out[k];
    }
};
template <bool INV> struct Dft<3, INV> { static MSG_DEV void run(float2* v) { DftOdd<3, INV>::run(v); } };
template <bool INV> struct Dft<5, INV> { static MSG_DEV void run(float2* v) { DftOdd<5, INV>::run(v); } };
template <bool INV> struct Dft<7, INV> { static MSG_DEV void run(float2* v) { DftOdd<7, INV>::run(v); } };

// a * exp(-+2 pi i e / N) for a compile-time e (after unrolling): the
// quarter turns are swaps/negations (x * 0.f is not folded without fast-math).
template <bool INV> MSG_DEV float2 twc(float2 a, int e, int N) {
    if (e == 0) return a;
    if (4 * e == N) return mul_mi<INV>(a);
    if (2 * e == N) return make_float2(-a.x, -a.y);
    if (4 * e == 3 * N) return mul_mi<!INV>(a);
    const float c = (float)__builtin_cos(2.0 * 3.14159265358979323846 * e / N);
    const float s = (float)__builtin_sin(2.0 * 3.14159265358979323846 * e / N);
    return cmul_k(a, make_float2(c, INV ? s : -s));
}

// Composite radix R1*R2 by Cooley-Tukey in registers: input n = R2*n1 + n2,
// output k = k1 + R1*k2.
template <int R1, int R2, bool INV> struct DftComp {
    static MSG_DEV void run(float2* v) {
        constexpr int N = R1 * R2;
        float2 a[R2][R1];
#pragma unroll
        for (int n2 = 0; n2 < R2; ++n2) {
#pragma unroll
            for (int n1 = 0; n1 < R1; ++n1) a[n2][n1] = v[R2 * n1 + n2];
            Dft<R1, INV>::run(a[n2]);
#pragma unroll
            for (int k1 = 1; k1 < R1; ++k1) {
                if (n2 == 0) continue;
                a[n2][k1] = twc<INV>(a[n2][k1], (n2 * k1) % N, N);
            }
        }
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) {
            float2 b[R2];
#pragma unroll
            for (int n2 = 0; n2 < R2; ++n2) b[n2] = a[n2][k1];
            Dft<R2, INV>::run(b);
#pragma unroll
            for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = b[k2];
        }
    }
};
template <bool INV> struct Dft<6, INV> { static MSG_DEV void run(float2* v) { DftComp<2, 3, INV>::run(v); } };
template <bool INV> struct Dft<8, INV> { static MSG_DEV void run(float2* v) { DftComp<2, 4, INV>::run(v); } };
template <bool INV> struct Dft<9, INV> { static MSG_DEV void run(float2* v) { DftComp<3, 3, INV>::run(v); } };
template <bool INV> struct Dft<10, INV> { static MSG_DEV void run(float2* v) { DftComp<2, 5, INV>::run(v); } };
template <bool INV> struct Dft<12, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 3, INV>::run(v); } };
template <bool INV> struct Dft<15, INV> { static MSG_DEV void run(float2* v) { DftComp<3, 5, INV>::run(v); } };
template <bool INV> struct Dft<16, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 4, INV>::run(v); } };
template <bool INV> struct Dft<20, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 5, INV>::run(v); } };
template <bool INV> struct Dft<25, INV> { static MSG_DEV void run(float2* v) { DftComp<5, 5, INV>::run(v); } };
template <bool INV> struct Dft<24, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 6, INV>::run(v); } };
template <bool INV> struct Dft<30, INV> { static MSG_DEV void run(float2* v) { DftComp<5, 6, INV>::run(v); } };
template <bool INV> struct Dft<32, INV> { static MSG_DEV void run(float2* v) { DftComp<4, 8, INV>::run(v); } };

// LDS data layout: logical complex element i lives at lp(i) = i ^ ((i>>4)&15),
// an XOR swizzle inside each aligned 16-element (128-byte) block.  Contiguous
// runs stay conflict-free (each block is permuted in place) and the strided
// Stockham stores of the early passes (element stride R*8 bytes) spread over
// all banks of a ds_write_b64 16-lane group.
MSG_DEV int lp(int i) { return i ^ ((i >> 4) & 15); }
MSG_HD constexpr int lds_phys(int logical) { return (logical + 15) & ~15; }

// Staged twiddle tables in LDS.
// t0/t1: FFT twiddles exp(-2 pi i j/size); r0/r1: real-FFT post-twiddles
// exp(-2 pi i k/n), both as two-level tables: w(i) = hi[i>>7] * lo[i&127].
struct TwLds { const float2* t0; const float2* t1; const float2* r0; const float2* r1; };
MSG_DEV float2 tw_at(const TwLds& tw, int i) { return cmul(tw.t1[i >> 7], tw.t0[i & (TW_LO - 1)]); }
MSG_DEV float2 rtw_at(const TwLds& tw, int k) { return cmul(tw.r1[k >> 7], tw.r0[k & (TW_LO - 1)]); }

// floor(j / d) for 0 <= j < 2^24 via a float reciprocal plus one correction.
MSG_DEV int fdiv(int j, int d, float inv_d) {
    int q = (int)((float)j * inv_d);
    const int r = j - q * d;
    if (r < 0) --q; else if (r >= d) ++q;
    return q;
}

// Opaque copy of a wave-uniform int: values derived from it are not hoisted
// out of the enclosing loop by LICM (register-pressure guard).
MSG_DEV int opaque(int v) {
    int o = __builtin_amdgcn_readfirstlane(v);
    asm volatile("" : "+s"(o));
    return o;
}

// Opaque copy of a wave-uniform pointer: loads through it are re-issued
// (scalar loads) where they are used instead of being hoisted and kept live.
template <class P> MSG_DEV P* opaque_ptr(P* p) {
    const uint64_t v = (uint64_t)p;
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return (P*)(((uint64_t)hi << 32) | lo);
}

// Opaque thread index: per-thread LDS addresses derived from it are rebuilt
// inside each pass/step instead of being hoisted (and spilled) by LICM.
MSG_DEV int otid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// One forward Stockham pass of radix R over buf[0..size), Ns = product of the
// earlier radices.  Twiddles w^r for r < R come from w, w^2, w^3, w^4 (w and
// w^4 from the table) and a running power of w^4 (five live values, product
// depth <= R/4 + 2).
template <int R, int T, int MAXM>
MSG_DEV void stockham_pass(float2* buf, int size, int Ns, const TwLds& tw) {
    constexpr int BMAX = (MAXM + R * T - 1) / (R * T);
    const int nb = size / R;
    const int stride = size / (Ns * R);
    const float inv_ns = 1.0f / (float)Ns;
    const int tid = otid();
    float2 v[BMAX][R];
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
        const int j = tid + b * T;
        if (j < nb) {
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = buf[lp(j + r * nb)];
        }
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
        const int j = tid + b * T;
        if (j < nb) {
            const int q = fdiv(j, Ns, inv_ns);
            const int k = j - q * Ns;
            if (k != 0) {
                // w^4 read from the table, not squared twice: a power carries its
                // base's rounding error times the exponent (see twiddle_pow_ab)
                const float2 w1 = tw_at(tw, k * stride);
                const float2 w2 = cmul(w1, w1);
                const float2 w3 = cmul(w2, w1);
                const float2 w4 = R > 4 ? tw_at(tw, 4 * k * stride) : cmul(w2, w2);
                float2 pw = make_float2(1.f, 0.f);   // w^(4a)
#pragma unroll
                for (int r = 1; r < R; ++r) {
                    if (r % 4 == 0) pw = (r == 4) ? w4 : cmul(pw, w4);
                    const int e = r % 4;
                    const float2 wr = e == 0 ? pw : (r < 4 ? (e == 1 ? w1 : e == 2 ? w2 : w3)
                                                           : cmul(pw, e == 1 ? w1 : e == 2 ? w2 : w3));
                    v[b][r] = cmul(v[b][r], wr);
                }
            }
            Dft<R, false>::run(v[b]);
            const int base = q * Ns * R + k;
#pragma unroll
            for (int r = 0; r < R; ++r) buf[lp(base + r * Ns)] = v[b][r];
        }
    }
    __syncthreads();
}

// Radix sets compiled into a kernel: all (arbitrary grain lengths) or powers
// of two only (FIR transforms).
enum { RSET_ALL = 0, RSET_PO2 = 1 };

// Unnormalised forward complex DFT of buf[0..size) by the plan's radix sequence.
template <int T, int MAXM, int RSET>
MSG_DEV void stockham_fwd(float2* buf, int size, const int32_t* rad, int nrad, const TwLds& tw) {
    int Ns = 1;
    for (int p = 0; p < nrad; ++p) {
        const int R = rad[p];
        // Opaque per-pass copy of the length: stops LICM from hoisting the
        // address arithmetic of every switch case out of the pass loop (which
        // kept hundreds of values live and spilled them to scratch).
        size = opaque(size);
        if (RSET == RSET_PO2) {
            switch (R) {
                case 2: stockham_pass<2, T, MAXM>(buf, size, Ns, tw); break;
                case 4: stockham_pass<4, T, MAXM>(buf, size, Ns, tw); break;
                case 8: stockham_pass<8, T, MAXM>(buf, size, Ns, tw); break;
                default: stockham_pass<16, T, MAXM>(buf, size, Ns, tw); break;
            }
        } else {
            switch (R) {
                case 2: stockham_pass<2, T, MAXM>(buf, size, Ns, tw); break;
                case 3: stockham_pass<3, T, MAXM>(buf, size, Ns, tw); break;
                case 4: stockham_pass<4, T, MAXM>(buf, size, Ns, tw); break;
                case 5: stockham_pass<5, T, MAXM>(buf, size, Ns, tw); break;
                case 6: stockham_pass<6, T, MAXM>(buf, size, Ns, tw); break;
                case 7: stockham_pass<7, T, MAXM>(buf, size, Ns, tw); break;
                case 8: stockham_pass<8, T, MAXM>(buf, size, Ns, tw); break;
                case 9: stockham_pass<9, T, MAXM>(buf, size, Ns, tw); break;
                case 10: stockham_pass<10, T, MAXM>(buf, size, Ns, tw); break;
                case 12: stockham_pass<12, T, MAXM>(buf, size, Ns, tw); break;
                case 15: stockham_pass<15, T, MAXM>(buf, size, Ns, tw); break;
                case 16: stockham_pass<16, T, MAXM>(buf, size, Ns, tw); break;
                case 20: stockham_pass<20, T, MAXM>(buf, size, Ns, tw); break;
                default: stockham_pass<25, T, MAXM>(buf, size, Ns, tw); break;
            }
        }
        Ns *= R;
    }
}

// A fixed-size float2 table copied from global memory into LDS with every load
// of the block issued before the first LDS store: fetch() puts the thread's
// entries in registers, put() stores them.  The plain `for (i = tid; i < N;
// i += T) dst[i] = src[i]` loop compiles to load / s_waitcnt vmcnt(0) /
// ds_write per iteration -- one full memory latency per iteration, before the
// kernel's data loads even issue (k_fir8: 4 iterations, k_spec3: 2).  Kernels
// issue their data loads between fetch() and put(); put() then waits for the
// table loads only (vmcnt counts in order), and the data loads' latency runs
// under the stores and the barrier.  MSG_TAB_PRELOAD=0 (tuning A/B): the loop.
#ifndef MSG_TAB_PRELOAD
#define MSG_TAB_PRELOAD 1
#endif
template <int N, int T>
struct TabCopy {
    static constexpr int PER = (N + T - 1) / T;
#if MSG_TAB_PRELOAD
    float2 v[PER];
    MSG_DEV void fetch(const float2* __restrict__ src) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int k = (int)threadIdx.x + i * T;
            if (i < PER - 1 || k < N) v[i] = src[k];
        }
    }
    MSG_DEV void put(float2* dst) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int k = (int)threadIdx.x + i * T;
            if (i < PER - 1 || k < N) dst[k] = v[i];
        }
    }
#else
    const float2* s = nullptr;
    MSG_DEV void fetch(const float2* __restrict__ src) { s = src; }
    MSG_DEV void put(float2* dst) const {
        for (int k = threadIdx.x; k < N; k += T) dst[k] = s[k];
    }
#endif
};

// Copy the plan's twiddle tables into LDS at `dst` (after the data region).
template <int T>
MSG_DEV TwLds stage_twiddles(float2* dst, const RealPlan& rp) {
    const FftDesc& d = rp.c;
    float2* r0 = dst + TW_LO + d.tw_hi_n;
    for (int i = threadIdx.x; i < TW_LO; i += T) dst[i] = d.tw0[i];
    for (int i = threadIdx.x; i < d.tw_hi_n; i += T) dst[TW_LO + i] = d.tw1[i];
    if (rp.even) {
        for (int i = threadIdx.x; i < TW_LO; i += T) r0[i] = rp.rt0[i];
        for (int i = threadIdx.x; i < rp.rt_hi_n; i += T) r0[TW_LO + i] = rp.rt1[i];
    }
    __syncthreads();
    return TwLds{dst, dst + TW_LO, r0, r0 + TW_LO};
}

// Forward complex DFT of length d.m in buf (Bluestein-aware, exp(-2 pi i jk/m)).
// Bluestein: X = chirp . IFFT_M( FFT_M(x . chirp) . B ) / M, the inner inverse
// as conj(FFT_M(conj(.))).  One call site of the Stockham engine.
template <int T, int MAXM, int RSET>
MSG_DEV void cfft_fwd(float2* buf, const FftDesc& d, const TwLds& tw) {
    const int m = d.m, M = d.size;
    const int rounds = d.blue ? 2 : 1;
    const int tid = otid();
    for (int round = 0; round < rounds; ++round) {
        if (d.blue) {
            for (int j = tid; j < M; j += T) {
                float2 x;
                if (round == 0) x = j < m ? cmul(buf[lp(j)], d.chirp[j]) : make_float2(0.f, 0.f);
                else x = cconj(cmul(buf[lp(j)], d.bspec[j]));
                buf[lp(j)] = x;
            }
            __syncthreads();
        }
        stockham_fwd<T, MAXM, RSET>(buf, d.size, d.rad, d.nrad, tw);
    }
    if (d.blue) {
        const float s = 1.0f / (float)M;
        for (int j = tid; j < m; j += T) buf[lp(j)] = cscale(cmul(cconj(buf[lp(j)]), d.chirp[j]), s);
        __syncthreads();
    }
}

// ---- real transforms over the LDS buffer ----
// Spectrum bin / complex element k lives at cx(buf, k) (swizzled).  Real
// samples x[t] are the packed pairs of element t/2 (even n) or element t's
// real part (odd n): rx_get / rx_set.
// `even` is the plan's parity, passed by value (a uniform bit, not re-read
// from the plan in global memory on every access).
MSG_DEV int rx_idx(bool even, int t) { return even ? 2 * lp(t >> 1) + (t & 1) : 2 * lp(t); }
MSG_DEV float rx_get(const float2* buf, bool even, int t) { return reinterpret_cast<const float*>(buf)[rx_idx(even, t)]; }
MSG_DEV void rx_set(float2* buf, bool even, int t, float v) {
    if (even) reinterpret_cast<float*>(buf)[rx_idx(true, t)] = v;
    else buf[lp(t)] = make_float2(v, 0.f);
}
MSG_DEV float2& cx(float2* buf, int k) { return buf[lp(k)]; }

// Real transform in place: forward (rfft: x -> X[0..n/2]) or inverse
// (irfft, numpy normalisation; imaginary parts of the DC and even-n Nyquist
// bins ignored as irfft does).  The inverse runs the forward engine on the
// conjugated half-spectrum, so each kernel inlines the engine once.
template <int T, int MAXM, int RSET>
MSG_DEV void rtransform(float2* buf, const RealPlan& rp, const TwLds& tw, bool inverse) {
    const int n = rp.n;
    const int m = n / 2;
    const int tid = otid();
    if (inverse) {   // pre: Z = E + i O from Y, stored conjugated
        if (rp.even) {
            for (int k = tid; k <= m / 2; k += T) {
                if (k == 0) {
                    const float y0 = cx(buf, 0).x, ym = cx(buf, m).x;
                    cx(buf, 0) = make_float2(0.5f * (y0 + ym), -0.5f * (y0 - ym));
                    continue;
                }
                const float2 yk = cx(buf, k), ym = cx(buf, m - k);
                const float2 e1 = cscale(cadd(yk, cconj(ym)), 0.5f);
                const float2 o1 = cscale(cmulc(csub(yk, cconj(ym)), rtw_at(tw, k)), 0.5f);
                const float2 e2 = cscale(cadd(ym, cconj(yk)), 0.5f);
                const float2 o2 = cscale(cmulc(csub(ym, cconj(yk)), rtw_at(tw, m - k)), 0.5f);
                cx(buf, k) = make_float2(e1.x - o1.y, -(e1.y + o1.x));
                cx(buf, m - k) = make_float2(e2.x - o2.y, -(e2.y + o2.x));
            }
        } else {
            const int K = (n + 1) / 2;
            for (int k = tid; k < K; k += T) {
                const float2 y = cx(buf, k);
                if (k == 0) { cx(buf, 0) = make_float2(y.x, 0.f); continue; }
                cx(buf, n - k) = y;          // conj of the mirrored conj(Y[k])
                cx(buf, k) = cconj(y);
            }
        }
        __syncthreads();
    }
    cfft_fwd<T, MAXM, RSET>(buf, rp.c, tw);
    if (!inverse) {
        if (!rp.even) return;
        // X[k] = E + W^k O ; E = (Z[k] + conj Z[m-k])/2 ; O = -i (Z[k] - conj Z[m-k])/2
        for (int k = tid; k <= m / 2; k += T) {
            if (k == 0) {
                const float2 z0 = cx(buf, 0);
                cx(buf, 0) = make_float2(z0.x + z0.y, 0.f);
                cx(buf, m) = make_float2(z0.x - z0.y, 0.f);
                continue;
            }
            const float2 zk = cx(buf, k), zm = cx(buf, m - k);
            const float2 e1 = cscale(cadd(zk, cconj(zm)), 0.5f);
            const float2 d1 = csub(zk, cconj(zm));
            const float2 o1 = make_float2(0.5f * d1.y, -0.5f * d1.x);
            const float2 e2 = cscale(cadd(zm, cconj(zk)), 0.5f);
            const float2 d2 = csub(zm, cconj(zk));
            const float2 o2 = make_float2(0.5f * d2.y, -0.5f * d2.x);
            cx(buf, k) = cfma(e1, rtw_at(tw, k), o1);
            cx(buf, m - k) = cfma(e2, rtw_at(tw, m - k), o2);
        }
        __syncthreads();
    } else {
        // post: x = conj(result) / (m or n)
        if (rp.even) {
            const float s = 1.0f / (float)m;
            for (int j = tid; j < m; j += T) { const float2 z = cx(buf, j); cx(buf, j) = make_float2(z.x * s, -z.y * s); }
        } else {
            const float s = 1.0f / (float)n;
            for (int j = tid; j < n; j += T) cx(buf, j) = make_float2(cx(buf, j).x * s, 0.f);
        }
        __syncthreads();
    }
}

// v[r] *= w^r for r < R, powers by a balanced product tree (depth <= 2 log2 R)
// v[r] *= w^r for r < R from two table values w1 = w and wB = w^B (B ~ sqrt R):
// w^r = wB^(r / B) * w1^(r % B).  A power of a rounded twiddle carries r times
// its rounding error (twiddle_pow below: up to 31x for R = 32); here no factor
// is raised beyond ~sqrt R, which keeps the FIR and spectral transforms within
// ~2x of a float32 FFT with exact twiddles (pocketfft) instead of ~3.5x.
template <int R, int B>
MSG_DEV void twiddle_pow_ab(float2 (&v)[R], float2 w1, float2 wB) {
    constexpr int A = (R + B - 1) / B;
    float2 p1[B], pb[A];
    p1[0] = make_float2(1.f, 0.f);
    p1[1 % B] = w1;
#pragma unroll
    for (int b = 2; b < B; ++b) p1[b] = (b % 2 == 0) ? cmul(p1[b / 2], p1[b / 2]) : cmul(p1[b - 1], w1);
    pb[0] = make_float2(1.f, 0.f);
    if (A > 1) pb[1] = wB;
#pragma unroll
    for (int a = 2; a < A; ++a) pb[a] = (a % 2 == 0) ? cmul(pb[a / 2], pb[a / 2]) : cmul(pb[a - 1], wB);
#pragma unroll
    for (int r = 1; r < R; ++r) {
        const int a = r / B, b = r % B;
        if (a == 0) v[r] = cmul(v[r], p1[b]);
        else if (b == 0) v[r] = cmul(v[r], pb[a]);
        else v[r] = cmul(v[r], cmul(pb[a], p1[b]));
    }
}
template <int R> constexpr int tw_base() { return R <= 4 ? R : (R <= 9 ? 3 : (R <= 16 ? 4 : (R <= 25 ? 5 : 6))); }

template <int R>
MSG_DEV void twiddle_pow(float2 (&v)[R], float2 w) {
    float2 p[R];
    p[1] = w;
    v[1] = cmul(v[1], w);
#pragma unroll
    for (int r = 2; r < R; ++r) {   // each power applied as soon as it exists (short live ranges)
        const int hb = 1 << (31 - __builtin_clz(r));
        p[r] = (r == hb) ? cmul(p[hb / 2], p[hb / 2]) : cmul(p[hb], p[r - hb]);
        v[r] = cmul(v[r], p[r]);
    }
}
