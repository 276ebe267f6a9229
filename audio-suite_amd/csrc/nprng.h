// nprng.h — NumPy Generator(PCG64) streams, bit-exact, for host and gfx950 device code.
//
// The reference draws every random number through np.random.default_rng(seed)
// (microsound_0.2.1/main_v2.py: MS:220, 272, 284, 304, 318, 334, 351, 370, 387,
// 410, 509, 620).  Reproducing its output therefore needs NumPy's exact streams:
//   SeedSequence(seed).generate_state(4, uint64)   numpy/random/bit_generator.pyx
//   PCG64 (XSL-RR 128/64, pcg_setseq_128_srandom_r) numpy/random/src/pcg64
//   next_double / buffered next_uint32              numpy/random/_pcg64.pyx
//   ziggurat standard_normal / standard_exponential numpy/random/src/distributions
//   Lemire bounded integers (32- and 64-bit)        numpy/random/src/distributions
// (NumPy 2.2.6, BSD-3-Clause).  tests/test_rng_host.py pins every function here
// against NumPy itself.
#pragma once
#include <stdint.h>
#include <math.h>
#include "msg_common.h"

namespace nprng {

typedef unsigned __int128 u128;

MSG_HD constexpr u128 mk128(uint64_t hi, uint64_t lo) { return ((u128)hi << 64) | lo; }
// PCG_DEFAULT_MULTIPLIER_128
#define NPRNG_MULT (((unsigned __int128)0x2360ED051FC65DA4ULL << 64) | 0x4385DF649FCCF645ULL)

struct Pcg64 {
    u128 state;
    u128 inc;
    uint32_t has_u32;
    uint32_t u32;
};

// Ziggurat tables, passed by pointer so host and device code share one implementation.
struct Zig {
    const uint64_t* ki;
    const double* wi;
    const double* fi;
    const uint64_t* ke;
    const double* we;
    const double* fe;
};

constexpr double ZIG_NOR_R = 3.6541528853610087963519472518;
constexpr double ZIG_NOR_INV_R = 0.27366123732975827203338247596;
constexpr double ZIG_EXP_R = 7.6971174701310497140446280481;

MSG_HD uint64_t rotr64(uint64_t v, unsigned r) { return (v >> r) | (v << ((64u - r) & 63u)); }
MSG_HD uint64_t xsl_rr(u128 s) {
    const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
    return rotr64(hi ^ lo, (unsigned)(hi >> 58));
}
MSG_HD void step(Pcg64& g) { g.state = g.state * NPRNG_MULT + g.inc; }
MSG_HD uint64_t next_u64(Pcg64& g) { step(g); return xsl_rr(g.state); }
MSG_HD uint32_t next_u32(Pcg64& g) {
    if (g.has_u32) { g.has_u32 = 0; return g.u32; }
    const uint64_t v = next_u64(g);
    g.has_u32 = 1;
    g.u32 = (uint32_t)(v >> 32);
    return (uint32_t)v;
}
MSG_HD double u64_to_unit(uint64_t r) { return (double)(r >> 11) * (1.0 / 9007199254740992.0); }
MSG_HD double next_double(Pcg64& g) { return u64_to_unit(next_u64(g)); }

// ---- SeedSequence(entropy=seed).generate_state(4, uint64) -> PCG64 state ----
MSG_HD uint32_t ss_hashmix(uint32_t v, uint32_t& hc) {
    v ^= hc;
    hc *= 0x931e8875u;          // MULT_A
    v *= hc;
    v ^= v >> 16;
    return v;
}
MSG_HD uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;   // MIX_MULT_L, MIX_MULT_R
    r ^= r >> 16;
    return r;
}
MSG_HD void seed_sequence_u64x4(uint64_t seed, uint64_t out[4]) {
    uint32_t ent[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    const int nent = (seed >> 32) ? 2 : 1;   // _int_to_uint32_array; 0 -> [0]
    uint32_t pool[4];
    uint32_t hc = 0x43b0d7e5u;               // INIT_A
    for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < nent ? ent[i] : 0u, hc);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
    uint32_t hb = 0x8b51f9ddu;               // INIT_B
    uint32_t w[8];
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= 0x58f38dedu;                   // MULT_B
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    for (int k = 0; k < 4; ++k) out[k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
}
// np.random.default_rng(seed) for an int seed >= 0.
MSG_HD Pcg64 default_rng(uint64_t seed) {
    uint64_t v[4];
    seed_sequence_u64x4(seed, v);
    Pcg64 g;
    const u128 initstate = mk128(v[0], v[1]);
    const u128 initseq = mk128(v[2], v[3]);
    g.state = 0;
    g.inc = (initseq << 1) | 1u;
    step(g);
    g.state += initstate;
    step(g);
    g.has_u32 = 0;
    g.u32 = 0;
    return g;
}

// ---- jump-ahead: state after k steps = A_k * s + inc * S_k (mod 2^128) ----
struct Jump { u128 a; u128 s; };
MSG_HD Jump jump_of(uint64_t k) {
    // (a, s) for one step = (MULT, 1); compose by doubling.
    u128 acc_a = 1, acc_s = 0;
    u128 cur_a = NPRNG_MULT, cur_s = 1;
    while (k) {
        if (k & 1) { acc_s = acc_s * cur_a + cur_s; acc_a = acc_a * cur_a; }
        cur_s = cur_s * (cur_a + 1);
        cur_a = cur_a * cur_a;
        k >>= 1;
    }
    return Jump{acc_a, acc_s};
}
MSG_HD u128 apply_jump(const Jump& j, u128 state, u128 inc) { return j.a * state + inc * j.s; }

// ---- distributions ----
MSG_HD double standard_normal(Pcg64& g, const Zig& z) {
    for (;;) {
        uint64_t r = next_u64(g);
        const int idx = (int)(r & 0xff);
        r >>= 8;
        const int sign = (int)(r & 1);
        const uint64_t rabs = (r >> 1) & 0x000fffffffffffffULL;
        double x = (double)rabs * z.wi[idx];
        if (sign) x = -x;
        if (rabs < z.ki[idx]) return x;
        if (idx == 0) {
            for (;;) {
                const double xx = -ZIG_NOR_INV_R * log1p(-next_double(g));
                const double yy = -log1p(-next_double(g));
                if (yy + yy > xx * xx)
                    return ((rabs >> 8) & 1) ? -(ZIG_NOR_R + xx) : ZIG_NOR_R + xx;
            }
        } else {
            if (((z.fi[idx - 1] - z.fi[idx]) * next_double(g) + z.fi[idx]) < exp(-0.5 * x * x))
                return x;
        }
    }
}

MSG_HD double standard_exponential(Pcg64& g, const Zig& z) {
    for (;;) {
        uint64_t ri = next_u64(g);
        ri >>= 3;
        const int idx = (int)(ri & 0xff);
        ri >>= 8;
        const double x = (double)ri * z.we[idx];
        if (ri < z.ke[idx]) return x;
        if (idx == 0) return ZIG_EXP_R - log1p(-next_double(g));
        if ((z.fe[idx - 1] - z.fe[idx]) * next_double(g) + z.fe[idx] < exp(-x)) return x;
        // else: draw again (tail recursion in NumPy)
    }
}

MSG_HD double uniform(Pcg64& g, double lo, double hi) { return lo + (hi - lo) * next_double(g); }
MSG_HD double normal(Pcg64& g, const Zig& z, double loc, double scale) {
    return loc + scale * standard_normal(g, z);
}
MSG_HD double exponential(Pcg64& g, const Zig& z, double scale) {
    return scale * standard_exponential(g, z);
}
MSG_HD double pareto(Pcg64& g, const Zig& z, double a) {
    return expm1(standard_exponential(g, z) / a);
}

// Generator.integers(low, high) (int64, endpoint=False): random_bounded_uint64_fill.
MSG_HD int64_t integers(Pcg64& g, int64_t low, int64_t high) {
    const uint64_t rng = (uint64_t)(high - low - 1);
    const uint64_t off = (uint64_t)low;
    if (rng == 0) return low;
    if (rng <= 0xFFFFFFFFULL) {
        if (rng == 0xFFFFFFFFULL) return (int64_t)(off + next_u32(g));
        const uint32_t rng_excl = (uint32_t)rng + 1u;
        uint64_t m = (uint64_t)next_u32(g) * rng_excl;
        uint32_t left = (uint32_t)m;
        if (left < rng_excl) {
            const uint32_t thr = (uint32_t)((0xFFFFFFFFu - (uint32_t)rng) % rng_excl);
            while (left < thr) {
                m = (uint64_t)next_u32(g) * rng_excl;
                left = (uint32_t)m;
            }
        }
        return (int64_t)(off + (m >> 32));
    }
    if (rng == 0xFFFFFFFFFFFFFFFFULL) return (int64_t)(off + next_u64(g));
    const uint64_t rng_excl = rng + 1;
    u128 m = (u128)next_u64(g) * rng_excl;
    uint64_t left = (uint64_t)m;
    if (left < rng_excl) {
        const uint64_t thr = (0xFFFFFFFFFFFFFFFFULL - rng) % rng_excl;
        while (left < thr) {
            m = (u128)next_u64(g) * rng_excl;
            left = (uint64_t)m;
        }
    }
    return (int64_t)(off + (uint64_t)(m >> 64));
}

}  // namespace nprng
