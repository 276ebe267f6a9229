// fir8_fft.h — overlap-save FIR with a 65 536-point transform (TU: k_fir.hip).
//
// One output block of B = N - P + 1 frames per workgroup, N = 65 536 real
// samples, one partition (Q = 1, P <= ~45 000 taps): the C3/C4 space filter
// (25 473 taps) takes 2 transforms of N per ~40 000 outputs instead of k_fir4's
// 3 transforms of 32 768 per ~20 000 (a third fewer transform passes per output,
// and each output goes through two transforms instead of three).
//
// The packed complex sequence z[m] = x[2m] + i x[2m+1] has M = 32 768 points,
// twice what LDS holds.  It is split once, in registers, by a radix-2
// decimation-in-frequency step:
//     a[m] = z[m] + z[m + MH],  b[m] = (z[m] - z[m + MH]) W_M^m,   m < MH = M/2
//     Z[2k] = FFT_MH(a)[k],     Z[2k+1] = FFT_MH(b)[k]
// and each half runs on the k_fir4 engine (Fir4Geo<16384>: 1024 threads,
// radices 16 16 8 8, LDS exchanges, last pass into registers).  Real-FFT pairs
// (k, M - k) stay inside a half: even bins pair kappa <-> MH - kappa (k_fir4's
// pairing: butterflies j, NB4 - j, thread 0 self-paired), odd bins kappa <->
// MH - 1 - kappa (butterflies j, NB4 - 1 - j, no self-paired bins).  The
// product with H and the inverse pre-step run per half in registers; the
// inverse of each half is the k_fir4 inverse engine (forward FFT of conj Z'),
// and the two halves are joined by the decimation-in-time step
//     F[m] = A[m] + W_M^m B[m],  F[m + MH] = A[m] - W_M^m B[m]
// before the outputs go to HBM.  Register live set at every point: one half
// (32 VGPRs: b while the even half transforms, A while the odd half does)
// beside the working set -- k_fir4's accumulator profile.
//
// H layout (k_fir8_hpart): He[kappa] = H[2 kappa] (kappa <= MH), then
// Ho[kappa] = H[2 kappa + 1] (kappa < MH): M + 1 float2 per preset, contiguous
// per half so the MAC reads are unit-stride.
//
// k_fir8p<true> (round 5) also serves presets whose overlap-add runs in its
// load phase (PresetRt::ola_fir, ola_split below): the segment is summed from
// the placed grains instead of read from the mono buffer k_ola_env writes.
#pragma once
#include "fir4_fft.h"
#include "ola.h"

// Phase timing (debug builds with -DMSG_STAMPS, tools/fir8_stamps.py): block-summed
// wall-clock deltas per phase of k_fir8, read back with msg_debug_stamps_fir.
#ifdef MSG_STAMPS
__device__ unsigned long long g_fir_stamps[16];
#define FIR_STAMP(i)                                                             \
    do {                                                                         \
        __syncthreads();                                                         \
        if (threadIdx.x == 0) {                                                  \
            const long long now_ = wall_clock64();                               \
            atomicAdd(&g_fir_stamps[i], (unsigned long long)(now_ - stamp_));    \
            stamp_ = now_;                                                       \
        }                                                                        \
    } while (0)
#define FIR_STAMP_INIT long long stamp_ = wall_clock64()
#else
#define FIR_STAMP(i) do {} while (0)
#define FIR_STAMP_INIT do {} while (0)
#endif

namespace fir8 {
using G = Fir4Geo<16384>;
constexpr int MH = 16384, M = 2 * MH, N = 2 * M;
// Ho follows He (MH + 1 bins) at a 128-byte-aligned offset: at MH + 1 every
// wave-wide Ho load straddled one more cache line; a spectrum takes HSTRIDE float2
constexpr int HO = MH + 16, HSTRIDE = HO + MH;
constexpr int T = G::T, R1 = G::R1, R2 = G::R2, R3 = G::R3, R4 = G::R4;
constexpr int NB1 = G::NB1, NB4 = G::NB4;
static_assert(NB1 == T && NB4 == 2 * T, "fir8 geometry");

// W_M^(1024 r) = W_32^r and exp(-2 pi i / N)
template <int R> MSG_DEV float2 w32(int r) {
    return make_float2((float)__builtin_cos(2.0 * 3.14159265358979323846 * r / 32),
                       (float)-__builtin_sin(2.0 * 3.14159265358979323846 * r / 32));
}
MSG_DEV float2 wN1() {
    return make_float2((float)__builtin_cos(2.0 * 3.14159265358979323846 / N),
                       (float)-__builtin_sin(2.0 * 3.14159265358979323846 / N));
}

// butterflies of the last forward pass held by thread t
template <bool ODD> MSG_DEV void js_of(int t, int (&js)[2]) {
    js[0] = t;
    js[1] = ODD ? NB4 - 1 - t : (t == 0 ? NB4 / 2 : NB4 - t);
}

// Forward FFT_MH of one half from registers (in[r] = element t + r NB1) to the
// last pass's butterflies js in v (k_fir4's passes 1-4).
template <bool ODD>
MSG_DEV void fwd_half(float2* buf, const float2* tab, float2 (&in)[R1], float2 (&v)[2][R4]) {
    const int t = otid();
    Dft<R1, false>::run(in);
    {
        put_run<G::S1, R1>(buf, t, in);
    }
    __syncthreads();
    fir4_pass_lds<MH, R2, R1, G::BP2, G::S1, G::S2, true, G::OFF_TA>(buf, tab, t);
    __syncthreads();
    fir4_pass_lds<MH, R3, R1 * R2, G::BP3, G::S2, G::S3, false, 0>(buf, tab, t);
    __syncthreads();
    int js[2];
    js_of<ODD>(t, js);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R4; ++r) v[h][r] = buf[pads<G::S3>(js[h] + r * NB4)];
    __syncthreads();   // LDS free for the inverse
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        fir_twiddle_p4<MH, R4>(v[h], tab, js[h]);
        Dft<R4, false>::run(v[h]);
    }
}

// Inverse of one half: the pre-stepped pairs acc (butterflies js) through the
// k_fir4 inverse engine; u[r] = FFT_MH(conj Z'_half)[t + r NB1].
template <bool ODD>
MSG_DEV void inv_half(float2* buf, const float2* tab, float2 (&acc)[2][R4], float2 (&u)[R1]) {
    const int t = otid();
    int js[2];
    js_of<ODD>(t, js);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        Dft<R4, false>::run(acc[h]);
        put_run<G::S1I, R4>(buf, js[h], acc[h]);
    }
    __syncthreads();
    fir4_pass_lds<MH, R3, R4, G::BP3, G::S1I, G::S2I, true, G::OFF_TB>(buf, tab, t);
    __syncthreads();
    fir4_pass_lds<MH, R2, R4 * R3, G::BP2, G::S2I, G::S3I, true, G::OFF_TC>(buf, tab, t);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R1; ++r) u[r] = buf[pads<G::S3I>(t + r * NB1)];
    __syncthreads();   // LDS free for the next half
    fir_twiddle_t<R1, T / 64>(u, tab, G::OFF_T4A, G::OFF_T4B, t);
    Dft<R1, false>::run(u);
}

// Even half: X[2 kappa] . He (k_fir4's split and MAC, thread 0's self-paired
// slots included), then the inverse pre-step; acc leaves as conj Z' pairs.
MSG_DEV void even_mac_pre(const float2* tab, const float2 (&v)[2][R4], const float2* __restrict__ He,
                          float2 (&acc)[2][R4]) {
    const int t = otid();
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < R4; ++r) acc[h][r] = make_float2(0.f, 0.f);
    if (t != 0) {
        const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            const int kA = t + r * NB4;
            const float2 wk = cmul_k(wA, fir_cr<R4>(r));
            fir_pair_mac(v[0][r], v[1][R4 - 1 - r], wk, at32(He, kA), at32(He, MH - kA), acc[0][r],
                         acc[1][R4 - 1 - r]);
            fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], wk);
        }
    } else {
        float2 a[R4], bb[R4];
        fir_slots<R4>(v, a, bb, true);
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            const int kA = fir_k0<MH, R4>(r);
            if (r < R4 - 1) {
                fir_pair_mac(a[r], bb[R4 - 1 - r], fir_w0<MH, R4>(r), He[kA], He[MH - kA], acc[0][r],
                             acc[1][R4 - 1 - r]);
            } else {   // DC/Nyquist packed as (Y[0], Y[M]) and bin M/2
                const float2 z0 = a[r];
                acc[0][r] = make_float2((z0.x + z0.y) * He[0].x, (z0.x - z0.y) * He[MH].x);
                acc[1][0] = cmul(cconj(bb[0]), He[MH / 2]);
            }
        }
#pragma unroll
        for (int r = 0; r < R4 - 1; ++r) fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], fir_w0<MH, R4>(r));
        const float y0 = acc[0][R4 - 1].x, yN = acc[0][R4 - 1].y;
        acc[0][R4 - 1] = make_float2(0.5f * (y0 + yN), -0.5f * (y0 - yN));   // bin M/2: conj Z' = Y
        fir_unslots<R4>(acc, true);
    }
}

// Odd half: X[2 kappa + 1] . Ho and the inverse pre-step (pairs kappa, MH-1-kappa).
MSG_DEV void odd_mac_pre(const float2* tab, const float2 (&v)[2][R4], const float2* __restrict__ Ho,
                         float2 (&acc)[2][R4]) {
    const int t = otid();
    const float2 wA = cmul_k(fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t), wN1());   // W_N^(2t+1)
#pragma unroll
    for (int r = 0; r < R4; ++r) {
        const int kA = t + r * NB4;
        const float2 wk = cmul_k(wA, fir_cr<R4>(r));
        float2 xk, xm;
        fir_split(v[0][r], v[1][R4 - 1 - r], wk, xk, xm);
        acc[0][r] = cmul(xk, at32(Ho, kA));
        acc[1][R4 - 1 - r] = cmul(xm, at32(Ho, MH - 1 - kA));
        fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], wk);
    }
}

// Load z[t + r NB1] and z[t + r NB1 + MH] of the segment x[s0, s0 + N) (zero
// outside [0, n)) into a and (z0 - z1) into b (twiddled after the tables are in LDS).
MSG_DEV void load_halves(const float* __restrict__ x, int64_t n, int64_t s0, float2 (&a)[R1], float2 (&b)[R1]) {
    const int t = otid();
    // segment samples u in [ulo, ulo + cnt) lie inside [0, n); 32-bit offsets from
    // xs = x + s0 (uniform), so every load takes its base in SGPRs
    const int64_t hi = n - s0 < (int64_t)N ? n - s0 : (int64_t)N;
    const uint32_t ulo = s0 < 0 ? (uint32_t)(-s0) : 0u;
    const uint32_t cnt = hi > (int64_t)ulo ? (uint32_t)(hi - ulo) : 0u;
    const float* xs = x + s0;
    if (ulo == 0 && cnt == (uint32_t)N && (((uintptr_t)xs) & 7) == 0) {
        const float2* z = reinterpret_cast<const float2*>(xs);
#pragma unroll
        for (int r = 0; r < R1; ++r) {
            a[r] = at32(z, t + r * NB1);
            b[r] = at32(z, t + r * NB1 + MH);
        }
    } else {                                          // the first and last blocks of a signal
#pragma unroll
        for (int r = 0; r < R1; ++r) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t u = 2u * (uint32_t)(t + r * NB1 + h * MH);
                const bool in0 = u - ulo < cnt, in1 = u + 1 - ulo < cnt;
                const float x0 = at32(xs, in0 ? u : ulo), x1 = at32(xs, in1 ? u + 1 : ulo);
                (h ? b : a)[r] = make_float2(in0 ? x0 : 0.f, in1 ? x1 : 0.f);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The overlap-add fused into the segment load (PresetRt::ola_fir): x[s0, s0 + N)
// is summed from the placed grains (MS:742-764) instead of read from a mono
// buffer k_ola_env wrote.  The arithmetic is ola_tile's (kernels_core.h): per
// frame, fmaf over the events in event order from 0.f, times the ADSR, so the
// FIR's input is the same bits.  Wave w owns frames [w OLA_CHUNK, (w + 1)
// OLA_CHUNK) of each half, lane l the frames l + 64 j: a grain's reads are
// coalesced over the wave, and one event puts up to OLA_J loads per lane in
// flight.  The DIF split is folded in: half 0 goes to LDS, each lane combines
// its half-1 frames with its own half-0 frames (x0 + x1 in place, x0 - x1 kept),
// and the sums, then the differences, leave LDS in the a / b layout -- so no
// half is held in registers while the other is gathered (the first form held
// a[] there: 128 VGPRs and scratch spills inside the transform passes).
// ---------------------------------------------------------------------------
constexpr int OLA_J = M / T;                  // frames per lane per half (32)
constexpr int OLA_CHUNK = 64 * OLA_J;         // frames per wave per half

// lane k's event of a 64-event round (start INT32_MAX past the preset's last)
struct OlaEv {
    int s, L;
    float amp;
    int64_t goff;
};
MSG_DEV OlaEv ola_ev(const msg_event* __restrict__ ev, const PresetRt& pr, int k) {
    OlaEv o{INT32_MAX, 0, 0.f, 0};
    if (k < pr.n_events) {
        const msg_event& e = ev[k];
        o.s = e.start; o.L = e.len; o.amp = (float)e.amp;
        o.goff = pr.pool_base + e.pool_off + e.offset;
    }
    return o;
}

// this lane's frames c0 + w OLA_CHUNK + lane + 64 j of the half starting at c0
// (absolute), times the ADSR, zero outside [0, n).  first: the lanes' events
// lo + lane (fetched once per segment, for both halves).  (Two events per
// iteration, both grains' loads in flight before the first FMA, ran slower:
// 146 SGPR spills, C5's FIR 5.84 -> 6.10 ms per sub-batch.)
MSG_DEV void ola_sum(const msg_event* __restrict__ ev, const PresetRt& pr, const float* __restrict__ grain_pool,
                     int lo, const OlaEv& first, int64_t c0, float (&acc)[OLA_J]) {
    const int t = otid();
    const int lane = t & 63, w = t >> 6;
    const int64_t w0 = c0 + (int64_t)w * OLA_CHUNK, w1 = w0 + OLA_CHUNK;
#pragma unroll
    for (int j = 0; j < OLA_J; ++j) acc[j] = 0.f;
    OlaEv e = first;
    for (int k0 = lo;;) {
        const uint64_t before = __ballot(e.s < w1);         // sorted: a prefix of the lanes
        uint64_t live = before & __ballot(e.L > 0 && (int64_t)e.s + e.L > w0);
        while (live) {                                      // in event order
            const int i = __builtin_ctzll(live);
            live &= live - 1;
            const int si = __builtin_amdgcn_readlane(e.s, i);
            const uint32_t Li = (uint32_t)__builtin_amdgcn_readlane(e.L, i);
            const float av = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(e.amp), i));
            const int64_t gi = ((int64_t)__builtin_amdgcn_readlane((int)(e.goff >> 32), i) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)e.goff, i);
            const float* g = grain_pool + gi;
            const int q0 = (int)(w0 - si) + lane;           // in (-OLA_CHUNK, L): the event meets the chunk
            float gv[OLA_J];
#pragma unroll
            for (int j = 0; j < OLA_J; ++j) {
                const int q = q0 + 64 * j;
                gv[j] = (uint32_t)q < Li ? g[q] : 0.f;
            }
#pragma unroll
            for (int j = 0; j < OLA_J; ++j)
                if ((uint32_t)(q0 + 64 * j) < Li) acc[j] = fmaf(av, gv[j], acc[j]);
        }
        if (before != ~0ull) break;
        k0 += 64;
        if (k0 >= pr.n_events) break;
        e = ola_ev(ev, pr, k0 + lane);
    }
    const int64_t n = pr.out_n;
#pragma unroll
    for (int j = 0; j < OLA_J; ++j) {
        const int64_t f = w0 + lane + 64 * j;
        acc[j] = (f >= 0 && f < n) ? acc[j] * adsr_at(pr, (int)f) : 0.f;
    }
}

// load_halves + dif_split for an ola_fir preset: (a, b) = (z0 + z1, (z0 - z1) W)
// of the segment x[s0, s0 + N) summed from its grains (the same float adds and
// products as dif_split on the loaded halves)
// lo: the first event that can reach s0 (its start after s0 - max_n; the host
// computes it per block, fir_lo)
MSG_DEV void ola_split(const msg_event* __restrict__ ev, const PresetRt& pr, const float* __restrict__ grain_pool,
                       int64_t s0, int lo, float2* buf, const float2* tab, float2 (&a)[R1], float2 (&b)[R1]) {
    const int t = otid();
    const int lane = t & 63, w = t >> 6;
    const OlaEv first = ola_ev(ev, pr, lo + lane);
    float* xf = reinterpret_cast<float*>(buf) + w * OLA_CHUNK + lane;   // buf is free: inv_half ends on a barrier
    {
        float x0[OLA_J];
        ola_sum(ev, pr, grain_pool, lo, first, s0, x0);
#pragma unroll
        for (int j = 0; j < OLA_J; ++j) xf[64 * j] = x0[j];             // read back by this lane only
    }
    float d[OLA_J];
    {
        float x1[OLA_J];
        ola_sum(ev, pr, grain_pool, lo, first, s0 + M, x1);
#pragma unroll
        for (int j = 0; j < OLA_J; ++j) {
            const float x0 = xf[64 * j];
            d[j] = x0 - x1[j];
            xf[64 * j] = x0 + x1[j];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R1; ++r) a[r] = buf[t + r * NB1];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < OLA_J; ++j) xf[64 * j] = d[j];
    __syncthreads();
    const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
    for (int r = 0; r < R1; ++r) {
        const float2 dd = buf[t + r * NB1];
        b[r] = r == 0 ? cmul(dd, wt) : cmul(dd, cmul_k(wt, w32<R1>(r)));
    }
}

// (a, b) <- (a + b, (a - b) W_M^(t + r NB1))
MSG_DEV void dif_split(const float2* tab, float2 (&a)[R1], float2 (&b)[R1]) {
    const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, otid());   // W_M^t (PLO/PHI: W_{2 MH} = W_M)
#pragma unroll
    for (int r = 0; r < R1; ++r) {
        const float2 z0 = a[r], z1 = b[r];
        a[r] = ff(vv(z0) + vv(z1));
        const float2 d = ff(vv(z0) - vv(z1));
        b[r] = r == 0 ? cmul(d, wt) : cmul(d, cmul_k(wt, w32<R1>(r)));
    }
}
}  // namespace fir8

template <int UNUSED = 0>
__global__ void __launch_bounds__(fir8::T)
k_fir8(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, const float2* __restrict__ tables,
       const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out) {
    using namespace fir8;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    FIR_STAMP_INIT;
    const int2 job = jobs[xcd_block(blockIdx.x, gridDim.x)];
    const PresetRt& pr = rt[job.x];
    const int P = pr.fir_P;                       // Q == 1
    const int64_t n = pr.out_n;
    const int64_t t0 = (int64_t)job.y * pr.fir_B;
    TabCopy<G::TAB_USED, T> tc;
    tc.fetch(tables);                             // table loads, then the segment's, all in flight
    float2 a[R1], b[R1];
    load_halves(x_in + pr.y_off, n, t0 - (P - 1), a, b);
    tc.put(tab);
    __syncthreads();                              // tables visible
    dif_split(tab, a, b);
    FIR_STAMP(0);
    const float2* He = hspec + pr.h_off;
    const float2* Ho = He + HO;
    float2 v[2][R4], acc[2][R4], A[R1];
    fwd_half<false>(buf, tab, a, v);
    FIR_STAMP(1);
    even_mac_pre(tab, v, He, acc);
    FIR_STAMP(2);
    inv_half<false>(buf, tab, acc, A);
    FIR_STAMP(3);
    fwd_half<true>(buf, tab, b, v);
    FIR_STAMP(4);
    odd_mac_pre(tab, v, Ho, acc);
    FIR_STAMP(5);
    float2 (&B)[R1] = a;                          // a is dead: its registers take B
    inv_half<true>(buf, tab, acc, B);
    FIR_STAMP(6);
    // F[m] = A + W_M^m B, F[m + MH] = A - W_M^m B; z'[m] = conj(F[m]) / M
    const int t = otid();
    const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
    const SegOut so = seg_out(y_out, pr.y_off, t0, n, N - P + 1, P);
    const int d0 = 2 * t - (P - 1);
    const float s = 1.0f / (float)M;
#pragma unroll
    for (int r = 0; r < R1; ++r) {
        const float2 wb = r == 0 ? cmul(B[r], wt) : cmul(B[r], cmul_k(wt, w32<R1>(r)));
        const float2 f[2] = {ff(vv(A[r]) + vv(wb)), ff(vv(A[r]) - vv(wb))};
#pragma unroll
        for (int h = 0; h < 2; ++h)                   // segment sample u = 2 (t + r NB1 + h MH)
            so.put((uint32_t)(d0 + 2 * (r * NB1 + h * MH)), make_float2(f[h].x * s, -f[h].y * s));
    }
    FIR_STAMP(7);
}

// ---------------------------------------------------------------------------
// Persistent k_fir8 (MSGPU_FIR8P, default 1): one workgroup per CU loops over
// blocks.  Phase stamps of k_fir8 (tools/fir8_stamps.py,
// profiles/r04p_fir_stamps.txt) put 28 % of a block's 53 us in its opening
// phase -- the job header, the 30 KB of twiddle tables and the 256 KB segment
// arriving while all 16 waves wait.  A resident workgroup stages the tables
// once and takes the next block from its XCD's counter while the current one
// runs.  Each XCD's workgroups take that XCD's contiguous range of blocks
// first (the segments of one preset overlap by P - 1 samples and share the
// filter spectrum), then help the other XCDs' ranges.  A workgroup stays on
// its CU for the launch, so the blocks no longer queue for CUs freed by other
// streams' kernels (the FIR window per 341-preset launch in the timed region:
// 2.69 -> 0.69 ms).  Two ways of hiding the segment load behind the previous
// block were measured and dropped (profiles/r04r_ab.json, r04t_*): streaming
// it through L2 during the epilogue with LDS-DMA loads into a never-read slot
// (the blocks of a launch run in step, so the prefetch joins the same HBM
// burst: isolated FIR 2.05 - 2.10 ms against 1.86), and loading it into the
// registers the epilogue frees (328 B of spills per lane: 2.64 - 2.70 ms).
// ---------------------------------------------------------------------------
namespace fir8 {
// this XCD's share [lo, lo + cnt) of n jobs (the xcd_block partition)
MSG_DEV void xcd_range(int n, int x, int& lo, int& cnt) {
    const int per = n / MSG_XCDS, rem = n % MSG_XCDS;
    lo = x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per;
    cnt = per + (x < rem ? 1 : 0);
}
}  // namespace fir8

// OLA: the instantiation with the fused overlap-add (PresetRt::ola_fir) -- its
// extra live state pushed the plain path to 128 VGPRs with spills in the
// transform passes (C3 isolated FIR 1.94 -> 2.11 ms), so batches without an
// ola_fir preset run the plain instantiation.
template <bool OLA>
__global__ void __launch_bounds__(fir8::T)
k_fir8p(const PresetRt* __restrict__ rt, const int2* __restrict__ jobs, int n_jobs, const float2* __restrict__ tables,
        const float2* __restrict__ hspec, const float* __restrict__ x_in, float* __restrict__ y_out,
        int32_t* __restrict__ ctr, int stagger, const msg_event* __restrict__ events,
        const float* __restrict__ grain_pool, const int32_t* __restrict__ ev_lo) {
    using namespace fir8;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ int s_take[2];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int t = otid();
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }
    // Stagger (MSGPU_FIR8P_STAGGER wall-clock ticks of 10 ns): every other
    // workgroup of an XCD starts its first block that much later, so the two
    // halves of the chip load their 256 KB segments and store their outputs
    // out of phase instead of all together.
    if (stagger > 0 && ((blockIdx.x / MSG_XCDS) & 1)) {
        const long long t_end = wall_clock64() + stagger;
        while (wall_clock64() < t_end) __builtin_amdgcn_s_sleep(16);
    }
    // ctr[x * FIR8P_CTR]: XCD x's next block; ctr[MSG_XCDS * FIR8P_CTR]: workgroups
    // done.  The last workgroup to finish zeroes them for the next launch (no
    // memset kernel: one would queue for a CU behind the other streams' work).
    // ranges in order: this workgroup's XCD first, then the others'
    const int x0 = (int)(blockIdx.x % MSG_XCDS);
    int k = 0, lo, cnt;
    xcd_range(n_jobs, x0, lo, cnt);
    if (t == 0) s_take[0] = atomicAdd(ctr + x0 * FIR8P_CTR, 1);
    __syncthreads();                              // tables visible, first take
    int cur = s_take[0], par = 1;
    for (;;) {
        while (cur >= cnt) {                      // range done: the next XCD's (uniform)
            if (++k == MSG_XCDS) break;
            const int x = (x0 + k) % MSG_XCDS;
            xcd_range(n_jobs, x, lo, cnt);
            __syncthreads();                      // every wave has read s_take[par] of the last block
            if (t == 0) s_take[par] = atomicAdd(ctr + x * FIR8P_CTR, 1);
            __syncthreads();
            cur = s_take[par];
            par ^= 1;
        }
        if (k == MSG_XCDS) break;
        const int xr = (x0 + k) % MSG_XCDS;
        FIR_STAMP_INIT;
        const int2 job = jobs[lo + cur];
        const PresetRt& pr = rt[job.x];
        const int P = pr.fir_P;                   // Q == 1
        const int64_t n = pr.out_n;
        const int64_t t0 = (int64_t)job.y * pr.fir_B;
        float2 a[R1], b[R1];
        const bool ola = OLA && __builtin_amdgcn_readfirstlane(pr.ola_fir);
        if (ola)
            ola_split(events + pr.ev_begin, pr, grain_pool, t0 - (P - 1), ev_lo[lo + cur], buf, tab, a, b);
        else
            load_halves(x_in + pr.y_off, n, t0 - (P - 1), a, b);
        if (t == 0) s_take[par] = atomicAdd(ctr + xr * FIR8P_CTR, 1);   // the block after this one
        if (!ola) dif_split(tab, a, b);
        FIR_STAMP(0);
        const float2* He = hspec + pr.h_off;
        const float2* Ho = He + HO;
        float2 v[2][R4], acc[2][R4], A[R1];
        fwd_half<false>(buf, tab, a, v);
        FIR_STAMP(1);
        even_mac_pre(tab, v, He, acc);
        FIR_STAMP(2);
        inv_half<false>(buf, tab, acc, A);
        FIR_STAMP(3);
        fwd_half<true>(buf, tab, b, v);
        FIR_STAMP(4);
        odd_mac_pre(tab, v, Ho, acc);
        FIR_STAMP(5);
        float2 (&B)[R1] = a;                      // a is dead: its registers take B
        inv_half<true>(buf, tab, acc, B);
        FIR_STAMP(6);
        const int nxt = s_take[par];              // written before this block's first barrier
        // F[m] = A + W_M^m B, F[m + MH] = A - W_M^m B; z'[m] = conj(F[m]) / M
        const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
        const SegOut so = seg_out(y_out, pr.y_off, t0, n, N - P + 1, P);
        const int d0 = 2 * t - (P - 1);
        const float s = 1.0f / (float)M;
#pragma unroll
        for (int r = 0; r < R1; ++r) {
            const float2 wb = r == 0 ? cmul(B[r], wt) : cmul(B[r], cmul_k(wt, w32<R1>(r)));
            const float2 f[2] = {ff(vv(A[r]) + vv(wb)), ff(vv(A[r]) - vv(wb))};
#pragma unroll
            for (int h = 0; h < 2; ++h)
                so.put((uint32_t)(d0 + 2 * (r * NB1 + h * MH)), make_float2(f[h].x * s, -f[h].y * s));
        }
        FIR_STAMP(7);
        cur = nxt;
        par ^= 1;
    }
    // every take of this workgroup has returned (thread 0 made them in order)
    if (t == 0 && atomicAdd(ctr + MSG_XCDS * FIR8P_CTR, 1) == (int)gridDim.x - 1) {
        for (int x = 0; x < MSG_XCDS; ++x) ctr[x * FIR8P_CTR] = 0;
        ctr[MSG_XCDS * FIR8P_CTR] = 0;
    }
}

// ---------------------------------------------------------------------------
// k_fir8q: two partitions on the 65 536-point engine (the standalone FIR of
// SURVEY §8 at 64 k taps; round 5 ran it on k_fir4 with
// five partitions of 13 108 taps at N = 32 768).  Uniformly partitioned
// overlap-save: P = B = N / 2 = 32 768, H_q = FFT_N(h[q P, (q + 1) P)), q < 2,
// and block j (outputs [j P, (j + 1) P)) is the last half of
//     IFFT(X_j H_0 + X_{j-1} H_1),   X_j = FFT_N(x[(j - 1) P, (j + 1) P)),
// one forward and one inverse transform per block, as k_fir8p's one-partition
// blocks but with B = P instead of N - P + 1 (2 transforms per 32 768 outputs
// instead of 6 of 32 768 points per 19 661 on k_fir4).  A workgroup takes a run
// of consecutive blocks of one signal (one atomic per run) and keeps X_{j-1}
// for the next block in a per-workgroup scratch slot (the even and odd halves'
// last-pass registers v, 2 x 2 R4 float2 per thread, 256 KB per workgroup) --
// as the carry C_{j+1} = X_j H_1 (the product formed while X_j's bins are
// split for X_j H_0, so X_{j-1} is never split again): block j adds C_j to
// X_j H_0 before the inverse pre-step.  Each thread reads back only what it
// wrote, pair by pair just before overwriting it, so no extra registers stay
// live.  A run that starts past a signal's first block opens with one forward
// transform of X_{j0-1} for its carry; a run's last block emits none.
// ---------------------------------------------------------------------------
namespace fir8 {
constexpr int Q2_SLOT = 2 * 2 * R4 * T;          // float2 per workgroup: halves x (2 R4) x threads

// the slot of one half: 2 R4 carries per thread, element e of thread t at e T + t
MSG_DEV float2* q2_slot(float2* scratch, int half) { return scratch + half * 2 * R4 * T; }

// One pair (k, M - k) of a half: the split X of this block's bins, acc = X H0
// (+ the carry C_j = X_{j-1} H1 that the previous block left in the slot, read
// into ck / cm at the start of the half: all of the half's carry loads are in
// flight before the first product), and the new carry X H1 into the slot (each
// thread overwrites only what it read).
MSG_DEV void q2_pair(float2 xk, float2 xm, float2 h0k, float2 h0m, float2 h1k, float2 h1m, float2& ak, float2& am,
                     float2 ck, float2 cm, float2& sk, float2& sm, bool prev, bool emit) {
    ak = cmul(xk, h0k);
    am = cmul(xm, h0m);
    if (prev) {
        ak = ff(vv(ak) + vv(ck));
        am = ff(vv(am) + vv(cm));
    }
    if (emit) {
        sk = cmul(xk, h1k);
        sm = cmul(xm, h1m);
    }
}
// this thread's carries of pair r of one half (elements r and R4 + r at e T + t),
// loaded MSG_Q2_AHEAD pairs ahead of their use; the empty asm statements (memory
// clobbers) keep the compiler from hoisting every load to the top of the half
// (sixteen carries beside v, b and the accumulators: scratch spills).  Measured
// at 64 k taps per 1024 x 384 000 (profiles/r06h_fir8q_prefetch_ab.txt): 0 pairs
// ahead 2.89 / 2.90 ms, 2 ahead 2.96 / 2.94, 4 ahead 3.14 / 3.10 (each pair
// ahead costs 16 B of scratch spills per lane); 1 ahead 2.92 vs 2.88 – 2.90
// (profiles/r06a1_fir8q_ahead1_ab.txt)
#ifndef MSG_Q2_AHEAD
#define MSG_Q2_AHEAD 0
#endif
constexpr int Q2_AHEAD = MSG_Q2_AHEAD;
MSG_DEV void q2_carry_load(const float2* sl, bool prev, int r, float2 (&c)[2][R4]) {
    if (r >= R4) return;
    const uint32_t tu = (uint32_t)otid();
    asm volatile("" ::: "memory");
    c[0][r] = prev ? at32(sl, tu + (uint32_t)(r * T)) : make_float2(0.f, 0.f);
    c[1][r] = prev ? at32(sl, tu + (uint32_t)((R4 + r) * T)) : make_float2(0.f, 0.f);
    asm volatile("" ::: "memory");
}
MSG_DEV void q2_carry_first(const float2* sl, bool prev, float2 (&c)[2][R4]) {
#pragma unroll
    for (int r = 0; r < Q2_AHEAD; ++r) q2_carry_load(sl, prev, r, c);
}

// Even half of a block on the carry form (k_fir8's even_mac_pre with H0, plus
// the carry in / out); leaves acc as conj Z' pairs for inv_half.
MSG_DEV void even_q2(const float2* tab, const float2 (&v)[2][R4], const float2* __restrict__ H0,
                     const float2* __restrict__ H1, float2* sl, bool prev, bool emit, float2 (&acc)[2][R4]) {
    const int t = otid();
    const uint32_t tu = (uint32_t)t;
    float2 c[2][R4];
    q2_carry_first(sl, prev, c);
    if (t != 0) {
        const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            const int kA = t + r * NB4;
            const float2 wk = cmul_k(wA, fir_cr<R4>(r));
            float2 xk, xm;
            q2_carry_load(sl, prev, r + Q2_AHEAD, c);
            fir_split(v[0][r], v[1][R4 - 1 - r], wk, xk, xm);
            q2_pair(xk, xm, at32(H0, kA), at32(H0, MH - kA), at32(H1, kA), at32(H1, MH - kA), acc[0][r],
                    acc[1][R4 - 1 - r], c[0][r], c[1][r], at32(sl, tu + (uint32_t)(r * T)),
                    at32(sl, tu + (uint32_t)((R4 + r) * T)), prev, emit);
            fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], wk);
        }
    } else {
        float2 a[R4], bb[R4];
        fir_slots<R4>(v, a, bb, true);
#pragma unroll
        for (int r = 0; r < R4; ++r) {
            const int kA = fir_k0<MH, R4>(r);
            q2_carry_load(sl, prev, r + Q2_AHEAD, c);
            if (r < R4 - 1) {
                float2 xk, xm;
                fir_split(a[r], bb[R4 - 1 - r], fir_w0<MH, R4>(r), xk, xm);
                q2_pair(xk, xm, H0[kA], H0[MH - kA], H1[kA], H1[MH - kA], acc[0][r], acc[1][R4 - 1 - r],
                        c[0][r], c[1][r], sl[r * T], sl[(R4 + r) * T], prev, emit);
            } else {   // DC/Nyquist packed as (Y[0], Y[M]) and bin M/2
                const float2 z0 = a[r];
                const float2 xd = make_float2(z0.x + z0.y, z0.x - z0.y), xh = cconj(bb[0]);
                acc[0][r] = make_float2(xd.x * H0[0].x, xd.y * H0[MH].x);
                acc[1][0] = cmul(xh, H0[MH / 2]);
                float2& s0 = sl[r * T];
                float2& s1 = sl[(2 * R4 - 1) * T];
                if (prev) {
                    acc[0][r] = ff(vv(acc[0][r]) + vv(c[0][r]));
                    acc[1][0] = ff(vv(acc[1][0]) + vv(c[1][R4 - 1]));
                }
                if (emit) {
                    s0 = make_float2(xd.x * H1[0].x, xd.y * H1[MH].x);
                    s1 = cmul(xh, H1[MH / 2]);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R4 - 1; ++r) fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], fir_w0<MH, R4>(r));
        const float y0 = acc[0][R4 - 1].x, yN = acc[0][R4 - 1].y;
        acc[0][R4 - 1] = make_float2(0.5f * (y0 + yN), -0.5f * (y0 - yN));   // bin M/2: conj Z' = Y
        fir_unslots<R4>(acc, true);
    }
    asm volatile("" ::: "memory");
}

// Odd half (pairs kappa, MH-1-kappa), the same carry form
MSG_DEV void odd_q2(const float2* tab, const float2 (&v)[2][R4], const float2* __restrict__ H0,
                    const float2* __restrict__ H1, float2* sl, bool prev, bool emit, float2 (&acc)[2][R4]) {
    const int t = otid();
    const uint32_t tu = (uint32_t)t;
    float2 c[2][R4];
    q2_carry_first(sl, prev, c);
    const float2 wA = cmul_k(fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t), wN1());   // W_N^(2t+1)
#pragma unroll
    for (int r = 0; r < R4; ++r) {
        const int kA = t + r * NB4;
        const float2 wk = cmul_k(wA, fir_cr<R4>(r));
        float2 xk, xm;
        q2_carry_load(sl, prev, r + Q2_AHEAD, c);
        fir_split(v[0][r], v[1][R4 - 1 - r], wk, xk, xm);
        q2_pair(xk, xm, at32(H0, kA), at32(H0, MH - 1 - kA), at32(H1, kA), at32(H1, MH - 1 - kA), acc[0][r],
                acc[1][R4 - 1 - r], c[0][r], c[1][r], at32(sl, tu + (uint32_t)(r * T)),
                at32(sl, tu + (uint32_t)((R4 + r) * T)), prev, emit);
        fir_pair_pre(acc[0][r], acc[1][R4 - 1 - r], wk);
    }
    asm volatile("" ::: "memory");
}
}  // namespace fir8

// jobs: runs (signal, first block); every run has run_len blocks but the
// signal's last, which stops at its end (rt[signal].fir_Q holds the signal's
// block count).  ctr: the launch's run counter at ctr[0] and the done count at
// ctr[MSG_XCDS * FIR8P_CTR] (k_fir8p's counter block; zero before, left zero).
__global__ void __launch_bounds__(fir8::T)
k_fir8q(const PresetRt* __restrict__ rt, const int2* __restrict__ runs, int n_runs, int run_len,
        const float2* __restrict__ tables, const float2* __restrict__ hspec, const float* __restrict__ x_in,
        float* __restrict__ y_out, float2* __restrict__ scratch_all, int32_t* __restrict__ ctr, int mode) {
    using namespace fir8;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    __shared__ int s_take;
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    float2* scratch = scratch_all + (int64_t)blockIdx.x * Q2_SLOT;
    const int t = otid();
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }
    constexpr int P = MH * 2;                      // partition length = block length = N / 2
    const float2* He0 = hspec;
    const float2* Ho0 = He0 + HO;
    const float2* He1 = hspec + HSTRIDE;
    const float2* Ho1 = He1 + HO;
    for (;;) {
        __syncthreads();                          // tables visible; the last run's s_take read
        if (t == 0) s_take = atomicAdd(ctr, 1);
        __syncthreads();
        const int run = s_take;
        if (run >= n_runs) break;
        const int2 job = runs[run];
        const PresetRt& pr = rt[job.x];
        const int64_t n = pr.out_n;
        const int nb = pr.fir_Q;
        const int j0 = job.y, j1 = j0 + run_len < nb ? j0 + run_len : nb;
        const float* x = x_in + pr.y_off;
        float2 a[R1], b[R1];
        float2 v[2][R4];
        if (j0 > 0) {                             // the carry X_{j0-1} H1 into the slot
            float2 acc[2][R4];
            load_halves(x, n, (int64_t)(j0 - 2) * P, a, b);
            dif_split(tab, a, b);
            fwd_half<false>(buf, tab, a, v);
            even_q2(tab, v, He0, He1, q2_slot(scratch, 0), false, true, acc);
            fwd_half<true>(buf, tab, b, v);
            odd_q2(tab, v, Ho0, Ho1, q2_slot(scratch, 1), false, true, acc);
        }
        for (int j = j0; j < j1; ++j) {
            const int64_t t0 = (int64_t)j * P;
            load_halves(x, n, t0 - P, a, b);
            dif_split(tab, a, b);
            float2 acc[2][R4], A[R1];
            fwd_half<false>(buf, tab, a, v);
            even_q2(tab, v, He0, He1, q2_slot(scratch, 0), j > 0 && !(mode & 1), j + 1 < j1 && !(mode & 2), acc);
            inv_half<false>(buf, tab, acc, A);
            fwd_half<true>(buf, tab, b, v);
            odd_q2(tab, v, Ho0, Ho1, q2_slot(scratch, 1), j > 0 && !(mode & 1), j + 1 < j1 && !(mode & 2), acc);
            float2 (&B)[R1] = a;                  // a is dead: its registers take B
            inv_half<true>(buf, tab, acc, B);
            const int tt = otid();                // per block: loop-invariant twiddles would be hoisted
            const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, tt);
            const SegOut so = seg_out(y_out, pr.y_off, t0, n, P, P + 1);
            const int d0 = 2 * tt - P;
            const float s = 1.0f / (float)M;
#pragma unroll
            for (int r = 0; r < R1; ++r) {
                const float2 wb = r == 0 ? cmul(B[r], wt) : cmul(B[r], cmul_k(wt, w32<R1>(r)));
                const float2 f[2] = {ff(vv(A[r]) + vv(wb)), ff(vv(A[r]) - vv(wb))};
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
                    so.put((uint32_t)(d0 + 2 * (r * NB1 + hh * MH)), make_float2(f[hh].x * s, -f[hh].y * s));
            }
        }
    }
    if (t == 0 && atomicAdd(ctr + MSG_XCDS * FIR8P_CTR, 1) == (int)gridDim.x - 1) {
        ctr[0] = 0;
        ctr[MSG_XCDS * FIR8P_CTR] = 0;
    }
}

// ---------------------------------------------------------------------------
// Filter spectra in the even/odd layout, one workgroup per (filter, half): the
// even half needs a = z0 + z1 and the odd half b = (z0 - z1) W only, so each
// half is its own workgroup (twice the workgroups of a per-filter kernel, each
// half as long: the h stage had 1.3 rounds of 256 long workgroups per launch).
//   k_fir8_hconv   ER (+ IR) presets: H = rfft(delta + ER taps) . S_IR.  The
//                  linear convolution fits the transform (h_len < N for one
//                  partition), so h never exists in the time domain: the taps
//                  are scattered into LDS as a (or z0 - z1) directly, and the
//                  IR's spectrum S_IR (k_fir8_spec, once per IR of the batch)
//                  multiplies the result.  IR-only presets use S_IR itself.
//   k_fir8_spec    H = rfft of float64 (IR bank) or float32 (msg_fir taps)
//                  samples: jobs (source offset, length, spectrum offset).
// ---------------------------------------------------------------------------
namespace fir8 {
// X of one half, from the last forward pass (v, butterflies js), times S (if
// non-null, same layout) into Hh (He or Ho).
template <bool ODD>
MSG_DEV void store_half(const float2* tab, const float2 (&v)[2][R4], const float2* __restrict__ S,
                        float2* __restrict__ Hh) {
    const int t = otid();
    auto put = [&](int k, float2 x) { Hh[(uint32_t)k] = S ? cmul(x, S[(uint32_t)k]) : x; };
    if (ODD) {
        const float2 wA = cmul_k(fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t), wN1());
#pragma unroll
        for (int q = 0; q < R4; ++q) {
            const int kA = t + q * NB4;
            float2 xk, xm;
            fir_split(v[0][q], v[1][R4 - 1 - q], cmul_k(wA, fir_cr<R4>(q)), xk, xm);
            put(kA, xk);
            put(MH - 1 - kA, xm);
        }
    } else if (t != 0) {
        const float2 wA = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
        for (int q = 0; q < R4; ++q) {
            const int kA = t + q * NB4;
            float2 xk, xm;
            fir_split(v[0][q], v[1][R4 - 1 - q], cmul_k(wA, fir_cr<R4>(q)), xk, xm);
            put(kA, xk);
            put(MH - kA, xm);
        }
    } else {
        float2 aa[R4], bb[R4];
        fir_slots<R4>(v, aa, bb, true);
#pragma unroll
        for (int q = 0; q < R4 - 1; ++q) {
            const int kA = fir_k0<MH, R4>(q);
            float2 xk, xm;
            fir_split(aa[q], bb[R4 - 1 - q], fir_w0<MH, R4>(q), xk, xm);
            put(kA, xk);
            put(MH - kA, xm);
        }
        const float2 z0 = aa[R4 - 1];
        put(0, make_float2(z0.x + z0.y, 0.f));
        put(MH, make_float2(z0.x - z0.y, 0.f));
        put(MH / 2, cconj(bb[0]));
    }
}

// one half of the input: a = z0 + z1 (ODD = false) or (z0 - z1) W_M^m, from x[0, n) of type T
template <bool ODD, class T>
MSG_DEV void load_half(const float2* tab, const T* __restrict__ x, int64_t n, float2 (&in)[R1]) {
    const int t = otid();
#pragma unroll
    for (int r = 0; r < R1; ++r) {
        float2 z[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int64_t i = 2 * (int64_t)(t + r * NB1 + h * MH);
            z[h] = make_float2(i < n ? (float)x[i] : 0.f, i + 1 < n ? (float)x[i + 1] : 0.f);
        }
        in[r] = ODD ? ff(vv(z[0]) - vv(z[1])) : ff(vv(z[0]) + vv(z[1]));
    }
    if (ODD) {
        const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
        for (int r = 0; r < R1; ++r) in[r] = r == 0 ? cmul(in[r], wt) : cmul(in[r], cmul_k(wt, w32<R1>(r)));
    }
}
}  // namespace fir8

// jobs[4 i ..]: source offset (elements of T), length, spectrum offset (float2), unused
template <class SRC>
__global__ void __launch_bounds__(fir8::T)
k_fir8_spec(const int64_t* __restrict__ jobs, const float2* __restrict__ tables, const SRC* __restrict__ src,
            float2* __restrict__ hspec) {
    using namespace fir8;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const int64_t* j = jobs + 4 * (blockIdx.x >> 1);
    const bool odd = blockIdx.x & 1;
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }   // one memory latency, not one per T entries
    __syncthreads();
    float2 in[R1], v[2][R4];
    float2* He = hspec + j[2];
    if (!odd) {
        load_half<false>(tab, src + j[0], j[1], in);
        fwd_half<false>(buf, tab, in, v);
        store_half<false>(tab, v, nullptr, He);
    } else {
        load_half<true>(tab, src + j[0], j[1], in);
        fwd_half<true>(buf, tab, in, v);
        store_half<true>(tab, v, nullptr, He + HO);
    }
}

template <int UNUSED = 0>
__global__ void __launch_bounds__(fir8::T)
k_fir8_hconv(const PresetRt* __restrict__ rt, const int32_t* __restrict__ list, const float2* __restrict__ tables,
             const int32_t* __restrict__ er_off, const double* __restrict__ er_gain, float2* __restrict__ hspec) {
    using namespace fir8;
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    float2* tab = lds;
    float2* buf = lds + G::TAB;
    const PresetRt& r = rt[list[blockIdx.x >> 1]];
    const bool odd = blockIdx.x & 1;
    { TabCopy<G::TAB_USED, T> tc; tc.fetch(tables); tc.put(tab); }   // one memory latency, not one per T entries
    for (int m = threadIdx.x; m < MH; m += T) buf[m] = make_float2(0.f, 0.f);
    __syncthreads();
    // e = delta + taps as the half's input: slot m & (MH-1), minus for m >= MH in the odd half
    // (the host merged equal offsets, so a slot takes at most one tap from each half, and
    // the LDS float adds of at most two values in either order give the same sum)
    float* e = reinterpret_cast<float*>(buf);
    if (threadIdx.x == 0) atomicAdd(e, 1.0f);
    for (int k = threadIdx.x; k < r.n_taps; k += T) {
        const int o = er_off[r.er_base + k];
        const int m = o >> 1;
        const float g = (float)er_gain[r.er_base + k];
        atomicAdd(e + 2 * (m & (MH - 1)) + (o & 1), (odd && m >= MH) ? -g : g);
    }
    __syncthreads();
    float2 in[R1], v[2][R4];
    const int t = otid();
#pragma unroll
    for (int q = 0; q < R1; ++q) in[q] = buf[t + q * NB1];
    if (odd) {
        const float2 wt = fir4_wM(tab, G::OFF_PLO, G::OFF_PHI, t);
#pragma unroll
        for (int q = 0; q < R1; ++q) in[q] = q == 0 ? cmul(in[q], wt) : cmul(in[q], cmul_k(wt, w32<R1>(q)));
    }
    __syncthreads();                                  // every read done before pass 1 writes buf
    const float2* S = r.ir_len > 0 ? hspec + r.irs_off : nullptr;
    float2* He = hspec + r.h_off;
    if (!odd) {
        fwd_half<false>(buf, tab, in, v);
        store_half<false>(tab, v, S, He);
    } else {
        fwd_half<true>(buf, tab, in, v);
        store_half<true>(tab, v, S ? S + HO : nullptr, He + HO);
    }
}
