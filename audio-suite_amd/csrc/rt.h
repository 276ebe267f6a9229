// rt.h — runtime records and helpers shared by the libmsgpu kernels.
//
//   k_plan_sizes / k_plan_events   per-preset planner (one thread per preset)      MS:589-646, 409-417
//   k_gen_normal                   grain generator, one wave per event              MS:219-269
//   k_spectral<T>                  LDS-resident spectral chain, one WG per event    MS:39-128, 224-233, 690-702
//   k_ola_env                      grain overlap-add x ADSR, one WG per tile        MS:742-764
//   k_h_build / k_fir_h            h = (delta + ER) * IR, its partition spectra      MS:409-445
//   k_fir2<M>                      register-resident FFT overlap-save FIR           MS:766-773
//   k_stereo_max / k_stereo_out    25-tap Bessel stereo, tanh, peak normalise       MS:423-436, 775-781
//   k_fir8p (ola_fir)              overlap-add x ADSR fused into the FIR's loads    MS:742-773
#pragma once
#include "msg_common.h"
#include "nprng.h"
#include "plan.h"
#include "fft_lds.h"

#if defined(__HIPCC__)
// x[i] of a uniform base with the byte offset formed in 32 bits, so the load or
// store takes the base in SGPRs (a 64-bit index costs two VALU per access).
template <class T> MSG_DEV T& at32(T* base, uint32_t i) {
    return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + i * (uint32_t)sizeof(T));
}
template <class T> MSG_DEV const T& at32(const T* base, uint32_t i) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + i * (uint32_t)sizeof(T));
}
#endif

// Per-preset runtime record, built on the host after planning.
struct PresetRt {
    int64_t out_n;
    int64_t out_off;       // first output frame of this preset
    int64_t pool_base;     // grain pool offset (floats)
    int64_t y_off;         // mono buffers offset (floats)
    int32_t ev_begin;      // first event slot
    int32_t n_events;
    int32_t er_base;       // first ER tap
    int32_t n_taps;        // ER taps (0 when ER off)
    int32_t tile_begin;    // first overlap-add tile
    int32_t max_n;
    // ADSR (MS:172-195), in samples
    int32_t envA, envD, envR;
    float envS, envC;
    int32_t envJ, envS1;           // decay end, release start (MS:185-190)
    float envInvA, envInvD, envInvR;
    // FIR (combined ER + IR), 0 = identity
    int32_t fir_on, fir_N, fir_P, fir_Q, fir_B;
    int32_t fir_block_begin;
    int32_t h_block_begin;
    int32_t ir_len;        // taps of the IR (0 -> delta)
    int64_t ir_off;        // offset of the IR in the device IR bank (float64)
    int64_t h_off;         // offset of the Q partition spectra (float2)
    int32_t h_len;         // taps of h = (delta + ER) * IR (k_h_build), <= out_n
    int32_t ola_fir;       // 1: the overlap-add runs inside k_fir8p's segment loads (fir8_fft.h), no mono a
    // stereo / saturation / normalisation
    int32_t stereo_fir;    // 1: 25-tap Bessel FIR (even n), 2: precomputed R (odd n), 0: L = R = y
    int32_t dl, dr;
    float bess[25];        // J_m(0.9 w), m = -12..12
    float drive, peak;
    int32_t h_fir4;        // spectra: 1 k_fir4_hpart, 2 k_fir8_hconv / IR spectrum, 3 k_fir4_hconv / IR spectrum
    // generator sources: IR fragment (float64 IR bank) and image (uint8 bank)
    int64_t frag_off, frag_len;
    int64_t img_off;
    int32_t img_h, img_w;
    int64_t r2_off;        // stereo_fir == 2: rotated right channel in the odd-stereo buffer
    int64_t hs_off;        // h in the FIR scratch (h_len floats, k_h_build)
    int64_t irs_off;       // k_fir8 ER + IR presets: the IR's spectrum in hspec (k_fir8_spec)
};

// Per-event spectral work descriptor (host-built after planning).
struct EventRt {
    int32_t plan;          // RealPlan index for n
    int32_t ops;           // bit mask of SPEC_* below
    int32_t n, gen_sr;
    double cutoff_gen, roll;
    double stretch;
    double tilt_alpha;     // log2 of the per-octave gain (MS:229-230)
    double env_tau;        // noise/skewed envelope time constant (s)
    double warp_power;     // fft_warp_power exponent (MS:103-115)
    // band of the band-pruned spectral kernel (spec3.h, host-computed by s3_band)
    int32_t s3_kb, s3_kz, s3_ky, s3_pad;   // s3_pad: k / f exact in float32 (wide band's gather)
    double s3_inv_f;
};
enum : int32_t {
    SPEC_TILT_NOISE = 1, SPEC_TILT_SKEW = 2, SPEC_LOWPASS = 4, SPEC_STRETCH = 8, SPEC_WARP = 16,
};

// float64 grain chain (kernels_grain64.h): per-event and per-preset records
struct Ev64 {
    int32_t plan;          // Real64Plan index for n
    int32_t ops;           // G64_* stages
    int32_t n;             // grain length through the chain
    int32_t n0;            // generator's own length (crackle: grain is max(n0, kernel))
    int32_t gen_sr;
    int32_t preset;        // batch index
    int32_t index;         // event i (generator seed = seed + i)
    int32_t ei;            // global event slot
    int64_t off64;         // offset in the float64 micro/grain pools (doubles)
    int64_t save_off;      // cepstral warp: saved spectrum (double2 slots)
    int64_t grain_off;     // float grain pool offset (pool_base + pool_off)
    double cutoff_gen;     // band-limit cutoff at the design rate (MS:691)
    double stretch;        // stretch lane value (MS:637)
};
enum : int32_t {
    G64_LOWPASS = 1, G64_WARP = 2, G64_CEP = 4, G64_LOCK = 8, G64_STRETCH = 16,
    G64_RES = 32, G64_WG = 64, G64_MB = 128, G64_CHAIN = 256,
    G64_SPEC = G64_LOWPASS | G64_WARP | G64_CEP | G64_LOCK | G64_STRETCH,
};

struct Chain64 {
    int32_t preset;
    int32_t ev_begin, n_events;   // Ev64 indices [ev_begin, ev_begin + n_events)
    int32_t pad;
    int64_t prev_off;             // previous grain (doubles, max_n)
    int64_t mem_off;              // imprint memory (doubles, max_n/2 + 1)
};

// The float64 space FIR of heavily saturated renders (kernels_fir64.h): one
// record per FIR preset, the shape of its float64 overlap-save.
constexpr int FIR64_N = 16384, FIR64_P = FIR64_N / 2, FIR64_B = FIR64_N - FIR64_P + 1, FIR64_K = FIR64_N / 2 + 1;
// float64 slots buffered per window of the chain (h and H_q of every slot of a
// window are resident at once): all flagged presets of a batch are processed,
// in windows of this many slots when the slots' buffers would exceed
// FIR64_WINDOW_BYTES
constexpr int FIR64_CAP = 1024;
constexpr int64_t FIR64_WINDOW_BYTES = (int64_t)1 << 30;
constexpr double FIR64_PRED = 5e-7;   // predicted float32 error above which a preset takes float64
struct Fir64Rt {
    int32_t h_len;                 // taps of h (<= out_n)
    int32_t q;                     // partitions of FIR64_P taps
    int32_t blocks;                // output blocks of FIR64_B frames
    int32_t st_tiles;              // stereo tiles (k_stereo_remax)
};

// Cross-workgroup state of the max pass (per context, reused launch to launch).
struct StereoSync {
    int32_t* done;       // per preset: max-pass tiles finished (the preset's last tile resets it to 0)
    uint32_t* ready;     // per preset: (epoch << 1) | deferred once every max-pass tile is done
    int32_t* flag64;     // per preset: 1 = takes the float64 FIR (null when the route is off)
    double* part;        // per stereo tile: the tile's sum y^2, sum q^2 (null when the route is off)
    double* stats;       // per preset: the same sums over the preset, added in tile order
    uint32_t epoch;      // this launch's tag, 1 .. 2^30
    int f64mode;         // 0 route off, 1 predicted, 2 every FIR preset (MSGPU_FIR64)
};
constexpr int ST_CTR_A = 0, ST_CTR_E = 32, ST_CTR_N = 64;   // k_stereo_fused counters, 128 B apart
// the fused stereo launch takes batches whose presets have at most this many
// stereo tiles (kernels_stereo.h: its deadlock-freedom bound); longer ones run
// k_stereo_max + k_stereo_out
constexpr int ST_FUSED_MAX_TILES = 2048;

constexpr int GEN_T = 64;          // one wave per event
constexpr int OLA_T = 256;
constexpr int OLA_TILE = 4096;
constexpr int ST_T = 256;
#ifndef MSG_ST_TILE
#define MSG_ST_TILE 4096           // tuning builds override (build.py --exp)
#endif
constexpr int ST_TILE = MSG_ST_TILE;

// shared helpers
//
// XCD-aware block order.  Workgroups are dispatched round-robin over the 8
// XCDs (block b -> XCD b % 8), and each XCD has its own L2.  Kernels whose
// neighbouring jobs share input (FIR blocks of one preset re-read the same
// partition spectra and overlapping input segments; overlap-add tiles read the
// same grains; stereo tiles overlap by their halo) remap b so that each XCD
// takes one contiguous range of jobs: the shared lines then stay in one L2.
constexpr int MSG_XCDS = 8;
constexpr int FIR8P_CTR = 32;   // int32 stride of k_fir8p's per-XCD block counters (128 B apart)
constexpr int S3P_CTR = 32;     // int32 stride of k_spec3p's per-XCD event counters (128 B apart)
__device__ __forceinline__ int xcd_block(int b, int grid) {
    const int x = b % MSG_XCDS, i = b / MSG_XCDS;
    const int per = grid / MSG_XCDS, rem = grid % MSG_XCDS;
    return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}

// Largest p with begin[p] <= b (begin non-decreasing, begin[0] = 0): a 64-ary
// search, one candidate per lane and a ballot per level, so a block finds its
// preset in ceil(log64 n) dependent loads (2 for 1024 presets) instead of
// log2 n.  Short-lived blocks (a 4096-frame tile) were latency-bound on the
// binary search.  Call from every lane of a wave (uniform control flow).
__device__ __forceinline__ int find_preset(const int32_t* __restrict__ begin, int n_presets, int b) {
    const int lane = (int)(threadIdx.x & 63);
    int lo = 0, len = n_presets;
    while (len > 1) {
        const int step = (len + 63) >> 6;
        const int off = lane * step;
        const bool ok = off < len && begin[lo + off] <= b;
        const unsigned long long m = __ballot(ok);
        const int c = 63 - __clzll(m);      // lane 0 always holds (begin[lo] <= b)
        lo += c * step;
        len = min(step, len - c * step);
    }
    return lo;
}

#if defined(__HIPCC__)
// The float64 FIR's error predictor (kernels_fir64.h): eps32 rms(y) x sqrt(the
// clip's linear share) x the clip's slope at 0 x the peak scale (MS:26-34),
// from sum y^2 (sy2), sum (1 + (d y)^2)^-2 (sq) and the float32 peak bits.
MSG_DEV double fir64_pred(const PresetRt& r, double sy2, double sq, unsigned peak_bits) {
    const double n = (double)r.out_n;
    const double d = (double)r.drive;
    const double rms = sqrt(sy2 / n), share = sq / n;
    const double M = (double)__uint_as_float(peak_bits);
    double slope = 1.0, mc = M;
    if (d > 0.0) { slope = d / tanh(d); mc = tanh(M * d) / tanh(d); }
    const double scale = mc > 0.0 ? (double)r.peak / mc : 1.0;
    return 5.9604644775390625e-8 * rms * sqrt(share) * slope * scale;
}
#endif

MSG_DEV float fade_w(int j, int n, int fade) {
    double w = 1.0;
    if (j < fade) w *= (double)j * (1.0 / (double)fade);
    if (j >= n - fade) w *= (double)(j - (n - fade)) * (-1.0 / (double)fade) + 1.0;
    return (float)w;
}
