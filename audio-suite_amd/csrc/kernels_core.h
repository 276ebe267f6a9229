// kernels_core.h — planner, generator, overlap-add and stereo kernels (TU: msgpu.hip).
#pragma once
#include "rt.h"
#include "ola.h"
#include <type_traits>

// ---------------------------------------------------------------------------
// Planner (one thread per preset).
// ---------------------------------------------------------------------------
__global__ void k_plan_sizes(const msg_preset* __restrict__ presets, int n_presets,
                             const double* __restrict__ bp, const int64_t* __restrict__ frag_len, nprng::Zig z,
                             msg_plan_info* __restrict__ info) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_presets) return;
    msg_plan_info inf;
    msgplan::plan_sizes(presets[p], bp, z, frag_len[p], inf);
    info[p] = inf;
}

__global__ void k_plan_events(const msg_preset* __restrict__ presets, int n_presets,
                              const double* __restrict__ bp, const int64_t* __restrict__ frag_len, nprng::Zig z,
                              const int32_t* __restrict__ slot_base, const int32_t* __restrict__ tap_base,
                              msg_event* __restrict__ events, int32_t* __restrict__ er_off,
                              double* __restrict__ er_gain, msg_plan_info* __restrict__ info) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n_presets) return;
    msg_plan_info inf;
    const msg_preset& pr = presets[p];
    const bool er = (pr.flags & MSG_F_ER_CLOUD) != 0;
    msgplan::plan_events(pr, bp, z, frag_len[p], p, inf, events + slot_base[p],
                         er ? er_off + tap_base[p] : nullptr, er ? er_gain + tap_base[p] : nullptr);
    info[p] = inf;
}

// ---------------------------------------------------------------------------
// Generators driven by standard_normal(n): parallel ziggurat walk.
//
// The stream of raw PCG64 draws is consumed 64 at a time: lane l holds the
// state of draw base+l (jump-ahead), classifies it as a fast ziggurat accept,
// and a wave ballot locates the rare draws that start a slow (rejection)
// normal.  Those lanes finish their slow normal from their own state and
// report how many draws it consumed, which moves the parse position.  The
// emitted sequence is exactly NumPy's standard_normal(n).
// ---------------------------------------------------------------------------
#ifndef MSG_GEN_G
#define MSG_GEN_G 8
#endif
constexpr int GEN_G = MSG_GEN_G;   // chunks of 64 draws classified per pass
// Waves per event (MSG_GEN_K): wave w of an event's workgroup takes groups
// w, w + K, w + 2K, ... of its draw stream.  Classification (the fast test and
// the slow normals) does not depend on where the parse stands, only the walk
// does; each wave walks its group as if no earlier slow normal reached into it,
// and after one barrier per round every wave scans the K (count, overhang)
// pairs; a group whose predecessor's last slow normal does reach into it walks
// again from that overhang (rare: the last draws of a group must be slow).
#ifndef MSG_GEN_K
#define MSG_GEN_K 1
#endif
constexpr int GEN_K = MSG_GEN_K;
// MSG_GEN_LDS=0 (tuning builds): the ziggurat tables are read through L1 and the
// resonant rotation by cross-lane reads, so k_gen_normal allocates no LDS and its
// waves can sit beside k_spec3's 162 KB workgroups.
#ifndef MSG_GEN_LDS
#define MSG_GEN_LDS 1
#endif
// Emission of a chunk (tuning macro): 3 = the resonant value from bases at
// multiples of 64 samples, evaluated 64 at a time (one per lane, once per 64
// chunks) into LDS, rotated by a 128-entry offset table; 2 = the round-3 form
// (bases at each group's chunk starts, evaluated by lanes g < G once per group
// of 8 chunks); rank by v_mbcnt and the valid lanes as the exec mask in both;
// 1 = the round-2 form (the chunk's base evaluated per chunk, rank by
// popcount); 0 = cost experiment only (raw normals, wrong output).
#ifndef MSG_GEN_NOSLOW
#define MSG_GEN_NOSLOW 0
#endif
#ifndef MSG_GEN_EMIT
#define MSG_GEN_EMIT 3
#endif
#if MSG_GEN_EMIT != 1 && !MSG_GEN_LDS
#error "MSG_GEN_EMIT 0/2/3 need MSG_GEN_LDS"
#endif
#if MSG_GEN_EMIT == 3 && MSG_GEN_K != 1
#error "MSG_GEN_EMIT 3 evaluates its bases with one wave per event"
#endif
// Jump-ahead constants and the ziggurat fast-path table (ki >> 20, wi * 2^20 as
// float32 bits).
struct JumpTab {
    nprng::u128 a[GEN_T]; nprng::u128 s[GEN_T]; nprng::u128 a64, s64, aG, sG;
    nprng::u128 aW[GEN_K], sW[GEN_K];   // jump by w groups (wave w's first group)
    nprng::u128 aR, sR;                 // jump by K groups (one round)
    uint2 kw[256]; float fif[256];
};

// The walk over one group's G chunks: from the first lane not consumed by an
// earlier slow normal (local, >= 64 skips whole chunks), mark the draws each
// slow normal consumed; bit g of a lane's vb = the lane's draw of chunk g starts
// a normal (a VGPR, not 2 G SGPRs of masks), cnt = their number.  Returns the
// overhang into the next group.  Wave-uniform apart from vb.
template <int G>
MSG_DEV int gen_walk(const uint64_t (&F)[G], const int (&consumed)[G], int local, uint32_t& vb, int& cnt) {
    cnt = 0;
    vb = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        if (local >= 64) { local -= 64; continue; }   // chunk consumed by an earlier slow normal
        uint64_t valid = ~0ULL << local;
        uint64_t S = ~F[g] & valid;
        int pos = 64;
        while (S) {
            const int q = __builtin_ctzll(S);
            const int end = q + __builtin_amdgcn_readlane(consumed[g], q);
            const uint64_t after_q = ~((2ULL << q) - 1);                  // lanes q+1..63
            const uint64_t before_end = end >= 64 ? ~0ULL : ((1ULL << end) - 1);
            valid &= ~(after_q & before_end);
            if (end >= 64) { pos = end; break; }
            S &= ~0ULL << end;
        }
        if (__builtin_amdgcn_inverse_ballot_w64(valid)) vb |= 1u << g;
        cnt += __popcll(valid);
        local = pos - 64;
    }
    return local;
}

// The slow part of NumPy's ziggurat normal (legacy_gauss / random_standard_normal,
// the same walk as nprng::standard_normal) from a draw that missed the fast test.
// ki / wi / fif are the LDS copies of the tables (fif: fi as float32); the global
// float64 fi is read only when the wedge test is too close to call in float32.
MSG_DEV double slow_normal(nprng::u128 st, nprng::u128 inc, uint64_t rabs, int idx, double x,
                           const nprng::Zig& z, const uint64_t* ki, const double* wi, const float* fif,
                           int& consumed) {
    nprng::Pcg64 g;
    g.state = st; g.inc = inc; g.has_u32 = 0; g.u32 = 0;
    int c = 1;
    for (;;) {
        if (idx == 0) {
            for (;;) {
                const double xx = -nprng::ZIG_NOR_INV_R * log1p(-nprng::next_double(g));
                const double yy = -log1p(-nprng::next_double(g));
                c += 2;
                if (yy + yy > xx * xx) {
                    consumed = c;
                    return ((rabs >> 8) & 1) ? -(nprng::ZIG_NOR_R + xx) : nprng::ZIG_NOR_R + xx;
                }
            }
        }
        const double u = nprng::next_double(g);
        c += 1;
        // the wedge test lhs < exp(-x^2/2), decided in float32 (lhs from the float32
        // table: relative error <~ 3e-7; the hardware exp2: ~1e-6) unless the two
        // sides are within 2e-5, then in float64 from the float64 table
        const float lhf = fmaf(fif[idx - 1] - fif[idx], (float)u, fif[idx]);
        const float ef = __builtin_amdgcn_exp2f((float)(-0.72134752044448170 * x * x));
        const float dd = lhf - ef;
        bool accept;
        if (fabsf(dd) > 2e-5f * ef) {
            accept = dd < 0.f;
        } else {
            const double lhs = (z.fi[idx - 1] - z.fi[idx]) * u + z.fi[idx];
            accept = lhs < exp(-0.5 * x * x);
        }
        if (accept) { consumed = c; return x; }
        uint64_t r = nprng::next_u64(g);
        c += 1;
        idx = (int)(r & 0xff);
        r >>= 8;
        const int sign = (int)(r & 1);
        rabs = (r >> 1) & 0x000fffffffffffffULL;
        x = (double)rabs * wi[idx];
        if (sign) x = -x;
        if (rabs < ki[idx]) { consumed = c; return x; }
    }
}

// Closed-form part of gen_basic for sample j given its normal N_j (MS:235-268).
// The ring phase frac(j f / sr) is reduced exactly in float32 from a two-term
// split of f / sr (j * fa with its fma rounding error, plus j * fb), so the
// hardware sine (v_sin_f32 takes revolutions: one transcendental instead of a
// software sinpi) only ever sees [0, 1); the decays are the hardware exp2 of j
// times a float64-built coefficient (arguments >= -126: no denormal path).
struct GenBasicConst {
    int mode;            // MSG_GEN_*
    int n, fade;
    float inv_fade;
    float fa, fb;        // resonant: cycles per sample, fa + fb = f / sr
    float k_ring, k_exc; // resonant: log2 decay per sample
    float inv_sigma;     // gaussian click
};
MSG_DEV float ring_phase(float jf, float fa, float fb) {
#pragma clang fp contract(off)
    const float p = jf * fa;
    const float e = fmaf(jf, fa, -p);                 // exact: j * fa = p + e
    float ph = (p - floorf(p)) + (e + jf * fb);
    return ph - floorf(ph);
}
// (sin, cos)(2 pi frac(j f / sr)) to float32 accuracy for the chunk bases and
// the rotation table of the resonant strike: the phase as a float pair (hi +
// lo, lo the rounding of hi) and sinpi / cospi of hi corrected to first order
// in lo.  The hardware sine of the rounded phase left a ~5e-7 relative error
// coherent at the ring frequency, which the band limit passes and a saturating
// space filter + tanh clip (MS:31-34) amplified to ~6e-6 RMS at 48 kHz
// (tools/diag_fir64.py).  Contraction is off: fused into p - floor(p), the
// product j fa would enter f0 unrounded and its tail e a second time (a phase
// error of up to ulp(j f / sr) / 2: 7e-4 rad at j = 40000, f / sr = 0.0875,
// tools/probe/ring_probe.hip).
MSG_DEV float2 ring_sincos(float jf, float fa, float fb) {
#pragma clang fp contract(off)
    const float p = jf * fa;
    const float e = fmaf(jf, fa, -p);
    const float f0 = p - floorf(p), f1 = e + jf * fb;
    float hi = f0 + f1;
    float lo = (f0 - hi) + f1;                        // |f0| >= |f1|: exact two-sum tail
    const float fl = -floorf(hi);
    const float h2 = hi + fl;                         // two-sum: the wrap's rounding joins lo
    const float bv = h2 - hi;
    lo += (hi - (h2 - bv)) + (fl - bv);
    hi = h2;
    const float a = 2.0f * hi;
    const float sn = sinpif(a), cs = cospif(a);
    const float d = 6.2831853071795865f * lo;         // 2 pi lo, |d| ~ 1e-7
    return make_float2(fmaf(d, cs, sn), fmaf(-d, sn, cs));
}
MSG_DEV float gen_basic_sample(const GenBasicConst& c, int j, float nrm) {
    float x;
    const float jf = (float)j;
    if (c.mode == MSG_GEN_RESONANT) {
        const float ph = ring_phase(jf, c.fa, c.fb);
        x = 0.9f * __builtin_amdgcn_sinf(ph) * __builtin_amdgcn_exp2f(fmaxf(jf * c.k_ring, -126.f)) +
            0.25f * nrm * __builtin_amdgcn_exp2f(fmaxf(jf * c.k_exc, -126.f));
    } else if (c.mode == MSG_GEN_GAUSSIAN_CLICK) {
        const float u = jf * c.inv_sigma;
        x = expf(-0.5f * (u * u)) * (nrm * 0.12f + 1.0f);
    } else if (c.mode == MSG_GEN_NOISE_BURST || c.mode == MSG_GEN_SKEWED) {
        return nrm;                                           // raw normals; tilt/env in k_spectral
    } else {
        x = nrm * 0.1f;                                       // gen_basic's last branch (MS:263)
    }
    if (j < c.fade) x *= jf * c.inv_fade;
    if (j >= c.n - c.fade) x *= (float)(j - (c.n - c.fade)) * -c.inv_fade + 1.0f;
    return x;
}
MSG_DEV float gen_fade(const GenBasicConst& c, int j, float x) {
    if (j < c.fade) x *= (float)j * c.inv_fade;
    if (j >= c.n - c.fade) x *= (float)(j - (c.n - c.fade)) * -c.inv_fade + 1.0f;
    return x;
}

// RAW64: raw float64 normals for the float64 chain; else the float32 grain.
// The float32 path forms the fast-path normal in float32 from the top 32 bits
// of its 52-bit ziggurat integer (|error| <= 1 ulp of float32); slow draws and
// RAW64 use the exact float64 product.
#ifndef MSG_GEN_WAVES
#define MSG_GEN_WAVES 1
#endif
#ifndef MSG_GEN_VGPRS
#define MSG_GEN_VGPRS 0
#endif
template <bool RAW64>
__global__ void __launch_bounds__(GEN_T * GEN_K, MSG_GEN_WAVES)
#if MSG_GEN_VGPRS
__attribute__((amdgpu_num_vgpr(MSG_GEN_VGPRS)))
#endif
k_gen_normal(const msg_preset* __restrict__ presets, const msg_event* __restrict__ events,
             const PresetRt* __restrict__ rt, const int32_t* __restrict__ ev_list, int n_list,
             nprng::Zig z, const JumpTab* __restrict__ jt, float* __restrict__ pool,
             double* __restrict__ pool64, const int64_t* __restrict__ off64) {
#if MSG_GEN_LDS
    __shared__ uint64_t s_ki[256];
    __shared__ double s_wi[256];
    __shared__ uint2 s_kw[256];          // (ki >> 20, wi * 2^20 as float32 bits): the fast path's one read
    __shared__ float s_fif[256];         // fi as float32: the slow path's wedge test
#if MSG_GEN_EMIT == 3
    __shared__ float4 s_rot[128];        // resonant: (cos, sin)(2 pi r f/sr), 0.9 * 2^(r k_ring), 0.25 * 2^(r k_exc), r = i
    __shared__ float4 s_base[64];        // resonant: (sin, cos, 2^(j k_ring), 2^(j k_exc)) at j = 64 (q0 + i)
#elif MSG_GEN_EMIT == 2
    __shared__ float4 s_rot[128];        // resonant: (cos, sin)(2 pi r f/sr), 0.9 * 2^(r k_ring), 0.25 * 2^(r k_exc), r = i - 64
    __shared__ float4 s_grp[GEN_K][GEN_G];   // resonant, per wave: (sin, cos, 2^(j k_ring), 2^(j k_exc)) at j = group start + 64 g
#else
    __shared__ float4 s_rot[64];         // resonant: (cos, sin)(2 pi r f/sr), 2^(r k_ring), 2^(r k_exc), r < 64
#endif
#else
    const uint64_t* __restrict__ s_ki = z.ki;
    const double* __restrict__ s_wi = z.wi;
    const uint2* __restrict__ s_kw = jt->kw;
    const float* __restrict__ s_fif = jt->fif;
#endif
    const int li = blockIdx.x;
    if (li >= n_list) return;
    const int lane = (int)(threadIdx.x & (GEN_T - 1));
    const int wv = GEN_K == 1 ? 0 : __builtin_amdgcn_readfirstlane((int)(threadIdx.x / GEN_T));
    __shared__ int2 s_carry[2][GEN_K];   // GEN_K > 1, per round (parity) and wave: (normals, overhang)
#if MSG_GEN_LDS
    for (int i = (int)threadIdx.x; i < 256; i += GEN_T * GEN_K) {
        s_ki[i] = z.ki[i];
        s_wi[i] = z.wi[i];
        s_kw[i] = jt->kw[i];
        s_fif[i] = jt->fif[i];
    }
#endif
    const msg_event& e = events[ev_list[li]];
    const msg_preset& pr = presets[e.preset];
    const PresetRt& r = rt[e.preset];
    const int n = e.n;
    float* out = pool + r.pool_base + e.pool_off;
    // float64 grain chain (kernels_grain64.h): raw normals into its pool
    double* out64 = RAW64 ? pool64 + off64[li] : nullptr;

    GenBasicConst c;
    c.mode = pr.gen_mode == MSG_GEN_FALLBACK ? MSG_GEN_NOISE_BURST : pr.gen_mode;   // MS:686
    c.n = n;
    c.fade = (int)(0.01 * n) > 8 ? (int)(0.01 * n) : 8;
    c.inv_fade = (float)(1.0 / (double)c.fade);
    const double inv_sr = 1.0 / (double)e.gen_sr;
    const double f_over_sr = fmax(10.0, pr.ring_hz) * inv_sr;
    c.fa = (float)f_over_sr;
    c.fb = (float)(f_over_sr - (double)c.fa);
    const double log2e = 1.4426950408889634;
    c.k_ring = (float)(-inv_sr / fmax(1e-6, pr.ring_decay_ms / 1000.0) * log2e);
    c.k_exc = (float)(-inv_sr / fmax(1e-6, (pr.micro_ms / 1000.0) * 0.15) * log2e);
    const int sigma = (int)(0.0025 * n) > 1 ? (int)(0.0025 * n) : 1;
    c.inv_sigma = (float)(1.0 / (double)sigma);
    // Resonant strike: sample j = j0 + r of a chunk (j0 = samples already
    // emitted, r = the lane's rank) from the chunk's uniform sin/cos and decay
    // at j0 and the per-rank rotation/decay table (angle addition, one ds_read
    // per sample instead of the phase reduction, a sine and two exponentials).
#if MSG_GEN_EMIT == 3
    // The value at j = B + t (B = 64 floor(j0 / 64) for the chunk starting at j0,
    // t in [0, 127)) is the rotation of the base's (sin, cos, decays) by the
    // offset table entry t, with the 0.9 and 0.25 gains folded into the table.
    int q0 = -64;                         // s_base holds the bases 64 (q0 + i), i < 64
    if (!RAW64 && c.mode == MSG_GEN_RESONANT) {
        for (int i = (int)threadIdx.x; i < 128; i += GEN_T * GEN_K) {
            const float rf = (float)i;
            const float2 sc = ring_sincos(rf, c.fa, c.fb);
            s_rot[i] = make_float4(sc.y, sc.x, 0.9f * __builtin_amdgcn_exp2f(rf * c.k_ring),
                                   0.25f * __builtin_amdgcn_exp2f(rf * c.k_exc));
        }
    }
#elif MSG_GEN_EMIT == 2
    // Two-level form: the value at j = B + t (B = a group's chunk base, |t| < 64
    // or t in [-64, 0) after slow draws shifted the chunk) is the rotation of the
    // base's (sin, cos, decays) by the offset table entry t, with the 0.9 and
    // 0.25 gains folded into the table.
    if (!RAW64 && c.mode == MSG_GEN_RESONANT) {
        for (int i = (int)threadIdx.x; i < 128; i += GEN_T * GEN_K) {
            const float rf = (float)(i - 64);
            const float2 sc = ring_sincos(rf, c.fa, c.fb);
            s_rot[i] = make_float4(sc.y, sc.x, 0.9f * __builtin_amdgcn_exp2f(rf * c.k_ring),
                                   0.25f * __builtin_amdgcn_exp2f(rf * c.k_exc));
        }
    }
#else
    float4 rot = make_float4(0.f, 0.f, 0.f, 0.f);
    if (!RAW64 && c.mode == MSG_GEN_RESONANT) {
        const float rf = (float)lane;
        const float ph = ring_phase(rf, c.fa, c.fb);
        rot = make_float4(__builtin_amdgcn_cosf(ph), __builtin_amdgcn_sinf(ph),
                          __builtin_amdgcn_exp2f(rf * c.k_ring), __builtin_amdgcn_exp2f(rf * c.k_exc));
#if MSG_GEN_LDS
        s_rot[lane] = rot;
#endif
    }
#endif

    // default_rng(seed + i): every lane computes the (uniform) seed state.
    const nprng::Pcg64 g0 = nprng::default_rng((uint64_t)(pr.seed + e.index));
    const nprng::u128 inc = g0.inc;
    const nprng::u128 a64 = jt->a64;
    const nprng::u128 c64 = inc * jt->s64;

    // Per group of GEN_G chunks of 64 draws: every lane classifies its GEN_G
    // draws, then finishes its (rare) slow ziggurat draws in one divergent loop
    // -- the wave runs that loop max-over-lanes times (usually once) instead of
    // once per chunk that holds a slow draw.  A wave-uniform walk per chunk then
    // marks the draws each slow normal consumed and all surviving lanes emit
    // their sample at once (rank = popcount of the valid lanes below).
    constexpr int G = GEN_G;
    nprng::u128 st[G];
    st[0] = jt->a[lane] * g0.state + inc * jt->s[lane];   // state after lane+1 steps
    if (GEN_K > 1) st[0] = jt->aW[wv] * st[0] + inc * jt->sW[wv];   // + wv groups
#pragma unroll
    for (int g = 1; g < G; ++g) st[g] = a64 * st[g - 1] + c64;
    const nprng::u128 aG = GEN_K > 1 ? jt->aR : jt->aG;   // the next group of this wave
    const nprng::u128 cG = inc * (GEN_K > 1 ? jt->sR : jt->sG);
#if MSG_GEN_LDS
    __syncthreads();
#endif

    int produced = 0;   // normals of all groups walked so far (workgroup-uniform)
    int local = 0;      // first lane of the next group not consumed by an earlier slow normal
    int rpar = 0;       // s_carry buffer of this round
    (void)rpar;
    while (produced < n) {
        using XT = typename std::conditional<RAW64, double, float>::type;
        uint64_t rabs[G], F[G];
        int idx[G], consumed[G];
        (void)rabs; (void)idx;
        XT x[G];
        unsigned slow = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            consumed[g] = 1;
            bool fast;
            if constexpr (RAW64) {
                const uint64_t raw = nprng::xsl_rr(st[g]);
                const int id = (int)(raw & 0xff);
                const uint64_t rr = raw >> 8;
                rabs[g] = (rr >> 1) & 0x000fffffffffffffULL;
                idx[g] = id | (int)((rr & 1) << 8);               // sign in bit 8
                x[g] = (double)rabs[g] * s_wi[id];
                if (rr & 1) x[g] = -x[g];
                fast = rabs[g] < s_ki[id];
            } else {
                // XSL-RR output in 32-bit halves: rotr64(hi ^ lo, hi >> 58) by
                // two alignbits.  The fast test compares bits 29..60 of the draw
                // (rabs >> 20) with ki >> 20; a tie is left to the slow pass,
                // which repeats the exact 52-bit test.
                const uint64_t hi = (uint64_t)(st[g] >> 64), lo = (uint64_t)st[g];
                const uint32_t rot = (uint32_t)(hi >> 58);
                uint32_t xl = (uint32_t)(hi ^ lo), xh = (uint32_t)((hi ^ lo) >> 32);
                if (rot & 32) { const uint32_t tmp = xl; xl = xh; xh = tmp; }
                const uint32_t olo = __builtin_amdgcn_alignbit(xh, xl, rot);
                const uint32_t ohi = __builtin_amdgcn_alignbit(xl, xh, rot);
                const uint32_t r32 = __builtin_amdgcn_alignbit(ohi, olo, 29);
                const int id = (int)(olo & 0xff);
                const uint2 kw = s_kw[id];
                const float xf = (float)r32 * __uint_as_float(kw.y);
                x[g] = (olo & 0x100) ? -xf : xf;
                fast = r32 < kw.x;
            }
            F[g] = __ballot(fast);
            if (!fast) slow |= 1u << g;
        }
#if MSG_GEN_NOSLOW                                // cost experiment only: slow draws left as classified
        slow = 0;
#endif
        while (slow) {                            // divergent: each lane walks its own slow draws
            const int gs = __builtin_ctz(slow);
            slow &= slow - 1;
            nprng::u128 s0 = st[0];
#pragma unroll
            for (int g = 1; g < G; ++g)
                if (gs == g) s0 = st[g];
            const uint64_t raw = nprng::xsl_rr(s0);
            const int id = (int)(raw & 0xff);
            const uint64_t ra = (raw >> 9) & 0x000fffffffffffffULL;
            if (!RAW64 && ra < s_ki[id]) continue;   // a tie of the 32-bit test: fast after all
            double xv = (double)ra * s_wi[id];
            if ((raw >> 8) & 1) xv = -xv;
            int cn = 1;
            const double v = slow_normal(s0, inc, ra, id, xv, z, s_ki, s_wi, s_fif, cn);
#pragma unroll
            for (int g = 0; g < G; ++g)
                if (gs == g) { x[g] = (XT)v; consumed[g] = cn; }
        }
        // the walk: which lanes of each chunk start a normal (vb), and this wave's
        // first output index pw
        uint32_t vb;
        int cnt, pw;
        if constexpr (GEN_K == 1) {
            local = gen_walk<G>(F, consumed, local, vb, cnt);
            pw = produced;
            produced += cnt;
        } else {
            int lout = gen_walk<G>(F, consumed, 0, vb, cnt);   // as if nothing reaches into the group
            if (lane == 0) s_carry[rpar][wv] = make_int2(cnt, lout);
            __syncthreads();
            pw = produced;
            int lin = local;
#pragma unroll 1
            for (int j = 0; j < GEN_K; ++j) {
                if (lin != 0) {                   // workgroup-uniform: group j starts inside a slow normal
                    if (wv == j) {
                        lout = gen_walk<G>(F, consumed, lin, vb, cnt);
                        if (lane == 0) s_carry[rpar][j] = make_int2(cnt, lout);
                    }
                    __syncthreads();
                }
                const int2 cj = s_carry[rpar][j];
                if (wv == j) pw = produced;
                produced += cj.x;
                lin = cj.y;
            }
            local = lin;
            rpar ^= 1;
        }
#if MSG_GEN_EMIT == 3
        const bool reson = !RAW64 && c.mode == MSG_GEN_RESONANT;
#elif MSG_GEN_EMIT == 2
        // resonant: lanes g < G evaluate the group's chunk bases p0 + 64 g (one set
        // of transcendentals per group instead of per chunk)
        const bool reson = !RAW64 && c.mode == MSG_GEN_RESONANT;
        const int p0 = pw;
        if (reson) {
            if (lane < G) {
                const float jb = (float)(p0 + 64 * lane);
                const float2 sc = ring_sincos(jb, c.fa, c.fb);
                s_grp[wv][lane] = make_float4(sc.x, sc.y, __builtin_amdgcn_exp2f(fmaxf(jb * c.k_ring, -126.f)),
                                              __builtin_amdgcn_exp2f(fmaxf(jb * c.k_exc, -126.f)));
            }
            __syncthreads();                      // orders the LDS writes before the reads
        }
#endif
        int pc = pw;                              // output index of the chunk's first normal
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const uint64_t valid = __ballot((vb >> g) & 1u);
            if (pc >= n || !valid) continue;
            if constexpr (RAW64) {
                if ((valid >> lane) & 1) {
                    const int j = pc + __popcll(valid & ((1ULL << lane) - 1));
                    if (j < n) out64[j] = x[g];
                }
            }
#if MSG_GEN_EMIT == 3
            else {
                // rank among the valid lanes (v_mbcnt), the valid mask as the exec mask
                const int rk = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(valid >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)valid, 0u));
                const bool vl = __builtin_amdgcn_inverse_ballot_w64(valid);
                const int room = n - pc;          // uniform
                float* __restrict__ ob = out + pc;
                if (reson) {
                    // j = pc + rk = 64 q + (d + rk), d = pc - 64 q in [0, 64)
                    const int q = pc >> 6, d = pc & 63;
                    if (q - q0 >= 64) {           // uniform, once per 64 chunks: the next 64 bases
                        q0 = q;
                        const float jb = (float)(64 * (q0 + lane));
                        const float2 sc = ring_sincos(jb, c.fa, c.fb);
                        __syncthreads();          // the previous bases are read
                        s_base[lane] = make_float4(sc.x, sc.y, __builtin_amdgcn_exp2f(fmaxf(jb * c.k_ring, -126.f)),
                                                   __builtin_amdgcn_exp2f(fmaxf(jb * c.k_exc, -126.f)));
                        __syncthreads();
                    }
                    const float4 u = s_base[q - q0];
                    const bool edge = pc < c.fade || pc + 64 > c.n - c.fade;
                    if (vl && rk < room) {
                        const float4 tb = s_rot[rk + d];
                        float v = fmaf(u.x, tb.x, u.y * tb.y) * (u.z * tb.z) + x[g] * (u.w * tb.w);
                        if (edge) v = gen_fade(c, pc + rk, v);
                        ob[rk] = v;
                    }
                } else if (vl && rk < room) {
                    ob[rk] = gen_basic_sample(c, pc + rk, (float)x[g]);
                }
            }
#elif MSG_GEN_EMIT == 2
            else {
                // rank among the valid lanes (v_mbcnt), the valid mask as the exec mask
                const int rk = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(valid >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)valid, 0u));
                const bool vl = __builtin_amdgcn_inverse_ballot_w64(valid);
                const int room = n - pc;          // uniform
                float* __restrict__ ob = out + pc;
                if (reson) {
                    // j = pc + rk = B_g + (d + rk), d = pc - B_g in [-64, 0]
                    const int d = pc - (p0 + 64 * g);
                    float4 u;
                    int off;
                    if (d >= -64) {
                        u = s_grp[wv][g];
                        off = d + 64;
                    } else {                          // a slow normal spanned > 64 draws: exact base
                        const float j0 = (float)pc;
                        const float2 sc = ring_sincos(j0, c.fa, c.fb);
                        u = make_float4(sc.x, sc.y, __builtin_amdgcn_exp2f(fmaxf(j0 * c.k_ring, -126.f)),
                                        __builtin_amdgcn_exp2f(fmaxf(j0 * c.k_exc, -126.f)));
                        off = 64;
                    }
                    const bool edge = pc < c.fade || pc + 64 > c.n - c.fade;
                    if (vl && rk < room) {
                        const float4 tb = s_rot[rk + off];
                        float v = fmaf(u.x, tb.x, u.y * tb.y) * (u.z * tb.z) + x[g] * (u.w * tb.w);
                        if (edge) v = gen_fade(c, pc + rk, v);
                        ob[rk] = v;
                    }
                } else if (vl && rk < room) {
                    ob[rk] = gen_basic_sample(c, pc + rk, (float)x[g]);
                }
            }
#elif MSG_GEN_EMIT == 0
            else {                                // cost experiment only: raw normals, no generator formula
                const int rk = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(valid >> 32),
                                                              __builtin_amdgcn_mbcnt_lo((uint32_t)valid, 0u));
                if (__builtin_amdgcn_inverse_ballot_w64(valid) && rk < n - pc) out[pc + rk] = (float)x[g];
            }
#else
            else if (c.mode == MSG_GEN_RESONANT) {
                // chunk-uniform phase and decays at j0 = pc
                const float j0 = (float)pc;
                const float ph0 = ring_phase(j0, c.fa, c.fb);
                const float s0 = __builtin_amdgcn_sinf(ph0), c0 = __builtin_amdgcn_cosf(ph0);
                const float dA = __builtin_amdgcn_exp2f(fmaxf(j0 * c.k_ring, -126.f));
                const float dE = __builtin_amdgcn_exp2f(fmaxf(j0 * c.k_exc, -126.f));
                const bool edge = pc < c.fade || pc + 64 > c.n - c.fade;
                const int rk = __popcll(valid & ((1ULL << lane) - 1));
#if MSG_GEN_LDS
                const float4 tb = s_rot[rk];
#else
                const float4 tb = make_float4(__shfl(rot.x, rk), __shfl(rot.y, rk), __shfl(rot.z, rk),
                                              __shfl(rot.w, rk));   // every lane: lane rk holds rank rk's rotation
#endif
                if ((valid >> lane) & 1) {
                    const int j = pc + rk;
                    if (j < n) {
                        float v = 0.9f * fmaf(s0, tb.x, c0 * tb.y) * (dA * tb.z) + 0.25f * x[g] * (dE * tb.w);
                        if (edge) v = gen_fade(c, j, v);
                        out[j] = v;
                    }
                }
            } else {
                if ((valid >> lane) & 1) {
                    const int j = pc + __popcll(valid & ((1ULL << lane) - 1));
                    if (j < n) out[j] = gen_basic_sample(c, j, (float)x[g]);
                }
            }
#endif
            pc += __popcll(valid);
        }
#pragma unroll
        for (int g = 0; g < G; ++g) st[g] = aG * st[g] + cG;   // next group of G chunks
    }
}

// ---------------------------------------------------------------------------
// Early-reflection gains of the host batch path (MS:410-417).  The host planned
// the offsets (draws j of default_rng(seed + 202)) and merged equal ones; tap
// j's gain is draw ntap + j of the same stream times exp(-42 d_j), and the taps
// of one merged slot add in tap order.  One workgroup per preset: each thread
// jumps to its run of taps in both halves of the stream and steps through it,
// writing the per-tap gains to g_tap; then threads over the live slots add
// them up.  Products and sums are rounded one by one (no contraction), as the
// host's plan.h does them.
// ---------------------------------------------------------------------------
constexpr int ER_T = 256;

MSG_DEV double er_uniform(nprng::Pcg64& g, double lo, double hi) {
    return __dadd_rn(lo, __dmul_rn(hi - lo, nprng::next_double(g)));
}

__global__ void __launch_bounds__(ER_T)
k_er_gains(const msg_preset* __restrict__ presets, const PresetRt* __restrict__ rt, int n_presets,
           const int32_t* __restrict__ er_key, const int32_t* __restrict__ er_first,
           const int32_t* __restrict__ er_cnt, double* __restrict__ g_tap, double* __restrict__ er_gain) {
    const int p = blockIdx.x;
    if (p >= n_presets) return;
    const msg_preset& pr = presets[p];
    if (!(pr.flags & MSG_F_ER_CLOUD)) return;                // uniform: before any barrier
    const PresetRt& r = rt[p];
    const int ntap = pr.er_taps > 1 ? pr.er_taps : 1;
    const int b = r.er_base;
    const int per = (ntap + ER_T - 1) / ER_T;
    const int j0 = (int)threadIdx.x * per, j1 = min(j0 + per, ntap);
    if (j0 < j1) {
        const nprng::Pcg64 g0 = nprng::default_rng((uint64_t)(pr.seed + 202));
        nprng::Pcg64 gd = g0, gu = g0;                        // draws j0 .. and ntap + j0 ..
        gd.state = nprng::apply_jump(nprng::jump_of((uint64_t)j0), g0.state, g0.inc);
        gu.state = nprng::apply_jump(nprng::jump_of((uint64_t)(ntap + j0)), g0.state, g0.inc);
        for (int j = j0; j < j1; ++j) {
            const double d = er_uniform(gd, 0.3, pr.er_max_ms) / 1000.0;
            const double u = er_uniform(gu, -1.0, 1.0);
            g_tap[b + j] = __dmul_rn(u, exp(__dmul_rn(-d, 42.0)));
        }
    }
    __syncthreads();                                          // the preset's per-tap gains, workgroup-visible
    for (int sl = (int)threadIdx.x; sl < r.n_taps; sl += ER_T) {
        const int f = er_first[b + sl], c = er_cnt[b + sl];
        double acc = g_tap[b + er_key[b + f]];
        for (int i = 1; i < c; ++i) acc = __dadd_rn(acc, g_tap[b + er_key[b + f + i]]);
        er_gain[b + sl] = acc;
    }
}

// ---------------------------------------------------------------------------
// Overlap-add of placed grains (event order) x ADSR -> mono a[t].
// ---------------------------------------------------------------------------
// Traversal order against the Infinity Cache (tuning A/B): MSG_OLA_REV = 1
// walks each XCD's job range backwards, so overlap-add starts on the most
// recently written end of the spectral kernel's grains (measured neutral,
// profiles/r03ak_traversal_ab.txt).
#ifndef MSG_OLA_REV
#define MSG_OLA_REV 0
#endif
MSG_DEV int job_order(int rev) {
    const int b = xcd_block(blockIdx.x, gridDim.x);
    return rev ? (int)gridDim.x - 1 - b : b;
}

// One OLA_TILE tile [t0, t0 + OLA_TILE) of preset r: the placed grains in event
// order times the ADSR (MS:742-764), into its mono buffer.
MSG_DEV void ola_tile(const msg_event* __restrict__ events, const PresetRt& r, int64_t t0,
                      const float* __restrict__ grain_pool, float* __restrict__ mono) {
    const int64_t t1 = t0 + OLA_TILE < r.out_n ? t0 + OLA_TILE : r.out_n;
    constexpr int PER = OLA_TILE / OLA_T;
    const int lane = threadIdx.x & 63;
    float acc[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) acc[u] = 0.f;
    // events are sorted by start: the first one that can reach t0 starts after t0 - max_n
    const msg_event* ev = events + r.ev_begin;
    const int lo = events_starting_by(ev, r.n_events, t0 - (int64_t)r.max_n);
    // 64 events per round: lane k fetches event lo+k, then the wave walks them
    // from registers (readlane) so all their grain reads are in flight together
    for (int k0 = lo; k0 < r.n_events; k0 += 64) {
        const int k = k0 + lane;
        int s = INT32_MAX, L = 0;
        float amp = 0.f;
        int64_t goff = 0;
        if (k < r.n_events) {
            const msg_event& e = ev[k];
            s = e.start; L = e.len; amp = (float)e.amp;
            goff = r.pool_base + e.pool_off + e.offset;
        }
        const uint64_t live = __ballot(s < t1);           // sorted: a prefix of the lanes
        const int cnt = __popcll(live);
        // two events per iteration: both grains' loads are in flight before the
        // first multiply-add (accumulation stays in event order)
        for (int i = 0; i < cnt; i += 2) {
            float gv[2][PER];
            bool take[2][PER];
            float av[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ii = i + h < cnt ? i + h : i;
                const int si = __builtin_amdgcn_readlane(s, ii);
                const int Li = (i + h < cnt) ? __builtin_amdgcn_readlane(L, ii) : 0;
                av[h] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(amp), ii));
                const int64_t gi = ((int64_t)__builtin_amdgcn_readlane((int)(goff >> 32), ii) << 32) |
                                   (uint32_t)__builtin_amdgcn_readlane((int)goff, ii);
                const float* g = grain_pool + gi;
                const bool ev_on = Li > 0 && (int64_t)si + Li > t0;
                const int q0 = (int)t0 - si + (int)threadIdx.x;
#pragma unroll
                for (int u = 0; u < PER; ++u) {
                    const int q = q0 + u * OLA_T;
                    take[h][u] = ev_on && u * OLA_T + (int)threadIdx.x < (int)(t1 - t0) && q >= 0 && q < Li;
                    gv[h][u] = take[h][u] ? g[q] : 0.f;
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int u = 0; u < PER; ++u)
                    if (take[h][u]) acc[u] = fmaf(av[h], gv[h][u], acc[u]);
        }
        if (cnt < 64) break;
    }
    float* y = mono + r.y_off;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int t = (int)t0 + (int)threadIdx.x + u * OLA_T;
        if (t < t1) y[t] = acc[u] * adsr_at(r, t);
    }
}

__global__ void __launch_bounds__(OLA_T)
k_ola_env(const msg_event* __restrict__ events, const PresetRt* __restrict__ rt,
          const int32_t* __restrict__ tile_begin, int n_presets,
          const float* __restrict__ grain_pool, float* __restrict__ mono) {
    const int b = job_order(MSG_OLA_REV);
    const int p = find_preset(tile_begin, n_presets, b);
    const PresetRt& r = rt[p];
    ola_tile(events, r, (int64_t)(b - r.tile_begin) * OLA_TILE, grain_pool, mono);
}

// The overlap-add of the float64 FIR's slots (kernels_fir64.h) among the presets
// whose overlap-add runs inside k_fir8p (ola_fir): the float64 FIR reads their
// mono a, which k_fir8p never writes.  A grid-stride walk over (slot, tile).
__global__ void __launch_bounds__(OLA_T)
k_ola_slots(const msg_event* __restrict__ events, const PresetRt* __restrict__ rt,
            const int32_t* __restrict__ slot_preset, const int32_t* __restrict__ n_slots, int tmax,
            const float* __restrict__ grain_pool, float* __restrict__ mono) {
    const int ns = *n_slots;
    for (int64_t j = blockIdx.x; j < (int64_t)ns * tmax; j += gridDim.x) {   // 64-bit: ns * tmax can pass 2^31
        const int sl = (int)(j / tmax), t = (int)(j - (int64_t)sl * tmax);
        const PresetRt& r = rt[__builtin_amdgcn_readfirstlane(slot_preset[sl])];
        if (!r.ola_fir || (int64_t)t * OLA_TILE >= r.out_n) continue;   // uniform
        ola_tile(events, r, (int64_t)t * OLA_TILE, grain_pool, mono);
    }
}
