// launch.h — host-side launchers of the kernels compiled in their own
// translation units (k_spectral.hip, k_fir.hip), so the FFT-heavy kernels
// build in parallel.
#pragma once
#include <hip/hip_runtime.h>
#include <vector>
#include "rt.h"
#include "fft64.h"

constexpr int LDS_MAX = 163840;                              // 160 KiB per CU
constexpr int SPEC_T_BIG = 512, SPEC_M_BIG = 20480;           // up to 160 KiB LDS
constexpr int SPEC_T_SMALL = 256, SPEC_M_SMALL = 8192;        // up to 64 KiB LDS
constexpr int SPEC_SMALL_BYTES = 65536;
constexpr int FIR_T = 512, FIR_M = 16384;                     // N <= 32768 real
constexpr int FIR_NMAX = 32768;

void spectral_init_attrs();
hipError_t launch_spectral(bool big, unsigned grid, int lds_bytes, hipStream_t s,
                           const msg_preset* presets, const msg_event* events, const EventRt* ert,
                           const PresetRt* rt, const RealPlan* plans, const int32_t* ev_list, int n_list,
                           float* micro_pool, float* grain_pool);

// compile-time-plan spectral kernels for hot grain lengths (spec_ct.h)
constexpr int SPEC_CT_PLANS = 6;
void spectral_ct_init_attrs();
int spectral_ct_plan(int n);
bool spectral_ct_tables(int plan, std::vector<float>& out);
hipError_t launch_spectral_ct(int plan, unsigned grid, hipStream_t s, const msg_event* events, const EventRt* ert,
                              const PresetRt* rt, const float2* tables, const int32_t* ev_list, int n_list,
                              float* micro_pool, float* grain_pool);

// band-pruned register-resident spectral kernel for the 30 MHz hot length (spec3.h)
void spec3_init_attrs();
bool spec3_tables(std::vector<float>& out);
bool spec3_eligible(int n, int ops, int gen_sr, double cutoff_gen, double roll, double stretch, int64_t float_off,
                    int32_t* kb, int32_t* kz, int32_t* ky, double* inv_f, int32_t* exact32);
// persist > 0: k_spec3p on that many workgroups (one per CU) with the per-XCD
// event counters ctr ((MSG_XCDS + 1) x S3P_CTR int32, zero; left zero)
hipError_t launch_spec3(unsigned grid, hipStream_t s, const msg_event* events, const EventRt* ert, const PresetRt* rt,
                        const float2* tables, const int32_t* ev_list, int n_list, const float* micro_pool,
                        float* grain_pool, int persist = 0, int32_t* ctr = nullptr);

void fir_init_attrs();
// the float64 space FIR of heavily saturated renders (kernels_fir64.h): flag, h, H_q, blocks
struct Fir64Launch {
    const PresetRt* rt; int n_presets; const int32_t* flag64; unsigned* maxbits;
    int32_t* slot_preset; int32_t* n_slots;
    int n_cand;   // FIR presets of the batch (the most slots there can be)
    int cap;      // slots per window (their h and H_q buffers)
    const Fir64Rt* fr; int tmax, qmax, bmax;
    const int32_t* er_off; const double* er_gain; const double* irbank;
    float* h64; int64_t h_stride; double2* hs64; int64_t hs_stride;
    const Real64Plan* plans; int plan; int lds_bytes;
    const float* x; float* y;
};
void fir64_init_attrs();
// k_fir64_flag: the flagged presets into slot_preset / n_slots; then the windows
hipError_t launch_fir64_flag(const Fir64Launch& a, hipStream_t s);
hipError_t launch_fir64(const Fir64Launch& a, hipStream_t s);
hipError_t launch_ir_spec(unsigned grid, int lds_bytes, hipStream_t s, const int64_t* jobs, int n_jobs,
                          const RealPlan* fir_plans, const double* ir_bank, float2* ir_spec);
// h = (delta + ER) * IR in the time domain, one workgroup per H_TILE taps of a preset
// (tile_begin: first tile per preset, non-decreasing)
hipError_t launch_h_build(unsigned grid, hipStream_t s, const PresetRt* rt, const int32_t* tile_begin, int n_presets,
                          const int32_t* er_off, const double* er_gain, const double* ir_bank, float* hs);
constexpr int H_BUILD_TILE = 1024;   // kernels_fir.h H_TILE
hipError_t launch_fir_h(unsigned grid, int lds_bytes, hipStream_t s, const PresetRt* rt, const int32_t* hblk_begin,
                        int n_presets, const RealPlan* fir_plans, const int32_t* fir_plan_of, const float* hs,
                        float2* hspec);
// register-resident FIR with compile-time transform size M = N/2 in {1024..16384}
bool fir2_tables_host(int M, std::vector<float>& out);
// frequency-domain delay line (msg_fir with many partitions): segment spectra, then MAC + inverse
hipError_t launch_fdl(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs, const float2* tables,
                      const float2* hspec, float2* xspec, const float* x_in, float* y_out);
hipError_t launch_fir2(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                       const float2* tables, const float2* hspec, const float* x_in, float* y_out);
// four-pass variant on 1024 threads (M = 16384 only; fir4_fft.h), same jobs and spectra as k_fir2
bool fir4_tables_host(int M, std::vector<float>& out);
hipError_t launch_fir4(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                       const float2* tables, const float2* hspec, const float* x_in, float* y_out);
// streaming variant (B = P = 16384, Q <= 2): jobs (preset, first block), kblk blocks per workgroup
constexpr int FIR4S_P = 16384;
// partition spectra on the k_fir4 engine (fir4_fft.h): k_fir4_hpart over the (preset, q) jobs
hipError_t launch_fir4_hpart(int M, unsigned n_parts, hipStream_t s, const PresetRt* rt, const int2* part_jobs,
                             const float2* tables, const float* hs, float2* hspec);
// one-partition spectra at N = 32768 from the taps (fir4_fft.h): S = rfft(IR) per job
// [src off, len, spec off, 0] of the float64 bank; H = rfft(delta + ER taps) . S per listed preset
hipError_t launch_fir4_hconv(unsigned n_presets, hipStream_t s, const PresetRt* rt, const int32_t* list,
                             const float2* tables, const int32_t* er_off, const double* er_gain, float2* hspec);
hipError_t launch_fir4_irspec(unsigned n_jobs, hipStream_t s, const int64_t* jobs, const float2* tables,
                              const double* src, float2* hspec);
// N = 65536 overlap-save, one partition (fir8_fft.h): blocks on the k_fir4 engine in
// two halves.  Spectra (even/odd bin layout, N/2 + 1 float2): k_fir8_hconv per listed
// ER preset (rfft(delta + taps) . S_IR), k_fir8_spec per job [src off, len, spec off, 0]
// of float64 (IR bank) or float32 samples.
constexpr int FIR8_N = 65536;
// float2 per filter spectrum on the N = 65536 engine: He (N / 4 + 1 bins) then Ho
// (N / 4) from a 128-byte-aligned offset (fir8::HO), a multiple of 16 float2
constexpr int FIR8_HSTRIDE = FIR8_N / 4 + 16 + FIR8_N / 4;
hipError_t launch_fir8(unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs, const float2* tables,
                       const float2* hspec, const float* x_in, float* y_out);
hipError_t launch_fir8p(unsigned n_jobs, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                        const float2* tables, const float2* hspec, const float* x_in, float* y_out, int32_t* ctr,
                        int stagger, const msg_event* events, const float* grain_pool,
                        const int32_t* ev_lo);   // events: null if no ola_fir preset; ev_lo: per job, the
                                                 // first event reaching its segment
// two partitions of N / 2 taps on the N = 65536 engine (fir8_fft.h k_fir8q): B = P = 32768,
// runs (signal, first block) of run_len blocks; the signal's PresetRt::fir_Q holds its block count
constexpr int FIR8Q_P = FIR8_N / 2;
hipError_t launch_fir8q(unsigned n_runs, int run_len, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* runs,
                        const float2* tables, const float2* hspec, const float* x_in, float* y_out, float2* scratch,
                        int32_t* ctr, int mode = 0);   // mode: timing experiments only (MSGPU_FIR8Q_MODE)
int64_t fir8q_scratch_per_wg();
hipError_t launch_fir8_hconv(unsigned n_presets, hipStream_t s, const PresetRt* rt, const int32_t* list,
                             const float2* tables, const int32_t* er_off, const double* er_gain, float2* hspec);
hipError_t launch_fir8_spec64(unsigned n_jobs, hipStream_t s, const int64_t* jobs, const float2* tables,
                              const double* src, float2* hspec);
hipError_t launch_fir8_spec32(unsigned n_jobs, hipStream_t s, const int64_t* jobs, const float2* tables,
                              const float* src, float2* hspec);
hipError_t launch_fir4s(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                        const float2* tables, const float2* hspec, const float* x_in, float* y_out, int kblk);

void fft_bench_init_attrs();
hipError_t launch_fft_bench(bool po2, unsigned grid, int lds_bytes, hipStream_t s, const RealPlan* plans, int plan,
                            int reps, float* sink);

// float64 grain chain (kernels_grain64.h): one workgroup per event / per chained preset
constexpr int G64_THREADS = 512, G64_SLOTS = 8192, G64_MAXPAR_HOST = 256;   // must match kernels_grain64.h
// global-memory slots for grains beyond the LDS engine (persistent workgroups)
struct G64Global {
    double2* A;           // grain buffers, slot_cap double2 per workgroup
    double2* B;           // FFT ping-pong scratch, same size
    uint32_t* mask;       // partial-lock selection bits, mask_words per workgroup
    int64_t slot_cap, mask_words;
};
void grain64_init_attrs();
// the two k_grain64 instantiations live in their own TUs (k_grain64_lds.hip,
// k_grain64_glb.hip) so they compile in parallel; launch_grain64 picks one
void grain64_lds_init_attr();
hipError_t launch_grain64_lds(unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets,
                              const Ev64* ev64, const PresetRt* rt, const Real64Plan* plans, const int32_t* list,
                              int n_list, const double* irbank, const uint8_t* imgbank, nprng::Zig z,
                              double* micro64, double* grain64, double2* save, float* grain_pool);
hipError_t launch_grain64_glb(const G64Global& g, unsigned grid, hipStream_t s, const msg_preset* presets,
                              const Ev64* ev64, const PresetRt* rt, const Real64Plan* plans, const int32_t* list,
                              int n_list, const double* irbank, const uint8_t* imgbank, nprng::Zig z,
                              double* micro64, double* grain64, double2* save, float* grain_pool);
hipError_t launch_grain64(const G64Global* g, unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets,
                          const Ev64* ev64, const PresetRt* rt, const Real64Plan* plans, const int32_t* list,
                          int n_list, const double* irbank, const uint8_t* imgbank, nprng::Zig z, double* micro64,
                          double* grain64, double2* save, float* grain_pool);
hipError_t launch_chain64(const G64Global* g, unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets,
                          const Ev64* ev64, const Chain64* chains, int n_chains, const Real64Plan* plans,
                          const double* grain64, double* state, float* grain_pool);
hipError_t launch_fft64_one(int lds_bytes, hipStream_t s, const Real64Plan* plans, int plan, int inverse,
                            double* io, double2* gA, double2* gB);

// stereo, tanh clip and peak normalisation (kernels_stereo.h)
hipError_t launch_stereo_max(unsigned n_tiles, hipStream_t s, const PresetRt* rt, const int32_t* st_begin, int n_presets,
                             const float* y, unsigned* maxbits, const StereoSync& sy);
// after k_stereo_max, with the float64 FIR on: per preset the predictor's sums (tile order) and flag64
hipError_t launch_stereo_pred(unsigned n_presets, hipStream_t s, const PresetRt* rt, const int32_t* st_begin,
                              int n_tiles, const unsigned* maxbits, const StereoSync& sy);
hipError_t launch_stereo_fused(unsigned grid, unsigned n_tiles, hipStream_t s, const PresetRt* rt,
                               const int32_t* st_begin, int n_presets, const float* y, unsigned* maxbits,
                               const StereoSync& sy, int32_t* ctr, float* out);
hipError_t launch_stereo_out(unsigned n_tiles, hipStream_t s, const PresetRt* rt, const int32_t* st_begin, int n_presets,
                             const float* y, const float* r2, const unsigned* maxbits, float* out);
hipError_t launch_stereo_remax(unsigned grid, hipStream_t s, const PresetRt* rt, const int32_t* st_count,
                               const int32_t* list, const int32_t* n_list, int tmax, const float* y, const float* r2,
                               unsigned* maxbits);
hipError_t launch_stereo_out_list(unsigned grid, hipStream_t s, const PresetRt* rt, const int32_t* st_count,
                                  const int32_t* list, const int32_t* n_list, int tmax, const float* y, const float* r2,
                                  const unsigned* maxbits, float* out);

// odd-length stereo rotation (kernels_stereo_odd.h): Bluestein through M = pow2 >= 2n-1
void stereo_odd_init_attrs();
// row_max / col_max: transform-split limits (0: the defaults 4096 / 2048)
int64_t stereo_odd_len(int64_t n, int row_max, int col_max);   // M, or -1 when n is too long
hipError_t launch_stereo_odd_kernel(int64_t n, int row_max, int col_max, double2* Bp, double2* A, hipStream_t s);
hipError_t launch_stereo_odd(int64_t n, int row_max, int col_max, int dr, double width, const float* y,
                             const double2* Bp, double2* A, float* r2, hipStream_t s);
// the app's spectrogram (stft_mag_db, MS:197-212) on the float64 engine
hipError_t launch_stft64(unsigned frames, int lds_bytes, hipStream_t s, const Real64Plan* plans, int plan,
                         const void* x, int elem_bytes, int64_t n, int channels, int win, int hop, double* S);

// per-render summary and digest (kernels_digest.h): tiles of 2048 frames, then
// one fold per render into res (msg_digest_rec records); part holds one
// 48-byte partial per tile.  digest_host: the same fold on the host.
hipError_t launch_digest(int n, int n_tiles, hipStream_t s, const float* out, const int64_t* frame_off,
                         const int64_t* frames, const int32_t* tile_base, void* part, void* res);
int64_t digest_tiles(int64_t frames);
void digest_host(const float* x, int64_t frames, void* rec);
