// k_fir.hip — translation unit of the space FIR kernels.
#include "kernels_fir.h"
#include "fir_fft.h"
#include "fir4_fft.h"
#include "fir8_fft.h"
#include "launch.h"
static_assert(fir8::HSTRIDE == FIR8_HSTRIDE, "fir8 spectrum stride: fir8_fft.h and launch.h");

template <int M> static void fir2_attr() {
    (void)hipFuncSetAttribute((const void*)k_fir2<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              FirGeo<M>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fdl_fwd<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              FirGeo<M>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fdl_mac<M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              FirGeo<M>::LDS_BYTES);
}

static_assert(H_TILE == H_BUILD_TILE, "k_h_build tile");

void fir_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_fir4<16384>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir4s<16384>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir4_hconv<16384>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir4_irspec<16384>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir4_hpart<16384>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8p<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8q, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8p<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8_hconv<0>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8_spec<double>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_fir8_spec<float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Fir4Geo<16384>::LDS_BYTES);
    fir2_attr<1024>(); fir2_attr<2048>(); fir2_attr<4096>(); fir2_attr<8192>(); fir2_attr<16384>();
    (void)hipFuncSetAttribute((const void*)k_fir_h<FIR_T, FIR_M>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_ir_spec<FIR_T, FIR_M>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_MAX);
}

hipError_t launch_ir_spec(unsigned grid, int lds_bytes, hipStream_t s, const int64_t* jobs, int n_jobs,
                          const RealPlan* fir_plans, const double* ir_bank, float2* ir_spec) {
    hipLaunchKernelGGL((k_ir_spec<FIR_T, FIR_M>), dim3(grid), dim3(FIR_T), lds_bytes, s, jobs, n_jobs, fir_plans,
                       ir_bank, ir_spec);
    return hipGetLastError();
}

hipError_t launch_h_build(unsigned grid, hipStream_t s, const PresetRt* rt, const int32_t* tile_begin, int n_presets,
                          const int32_t* er_off, const double* er_gain, const double* ir_bank, float* hs) {
    hipLaunchKernelGGL(k_h_build, dim3(grid), dim3(H_T), 0, s, rt, tile_begin, n_presets, er_off, er_gain, ir_bank, hs);
    return hipGetLastError();
}

hipError_t launch_fir_h(unsigned grid, int lds_bytes, hipStream_t s, const PresetRt* rt, const int32_t* hblk_begin,
                        int n_presets, const RealPlan* fir_plans, const int32_t* fir_plan_of, const float* hs,
                        float2* hspec) {
    hipLaunchKernelGGL((k_fir_h<FIR_T, FIR_M>), dim3(grid), dim3(FIR_T), lds_bytes, s, rt, hblk_begin, n_presets,
                       fir_plans, fir_plan_of, hs, hspec);
    return hipGetLastError();
}

bool fir2_tables_host(int M, std::vector<float>& out) {
    switch (M) {
        case 1024: fir2_tables<1024>(out); return true;
        case 2048: fir2_tables<2048>(out); return true;
        case 4096: fir2_tables<4096>(out); return true;
        case 8192: fir2_tables<8192>(out); return true;
        case 16384: fir2_tables<16384>(out); return true;
        default: return false;
    }
}

template <int M>
static hipError_t fir2_go(unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs, const float2* tables,
                          const float2* hspec, const float* x_in, float* y_out) {
    hipLaunchKernelGGL((k_fir2<M>), dim3(grid), dim3(FirGeo<M>::T), FirGeo<M>::LDS_BYTES, s, rt, jobs, tables, hspec,
                       x_in, y_out);
    return hipGetLastError();
}

hipError_t launch_fir2(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                       const float2* tables, const float2* hspec, const float* x_in, float* y_out) {
    switch (M) {
        case 1024: return fir2_go<1024>(grid, s, rt, jobs, tables, hspec, x_in, y_out);
        case 2048: return fir2_go<2048>(grid, s, rt, jobs, tables, hspec, x_in, y_out);
        case 4096: return fir2_go<4096>(grid, s, rt, jobs, tables, hspec, x_in, y_out);
        case 8192: return fir2_go<8192>(grid, s, rt, jobs, tables, hspec, x_in, y_out);
        case 16384: return fir2_go<16384>(grid, s, rt, jobs, tables, hspec, x_in, y_out);
        default: return hipErrorInvalidValue;
    }
}

bool fir4_tables_host(int M, std::vector<float>& out) {
    if (M != 16384) return false;
    fir4_tables<16384>(out);
    return true;
}

hipError_t launch_fir4(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                       const float2* tables, const float2* hspec, const float* x_in, float* y_out) {
    if (M != 16384) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_fir4<16384>), dim3(grid), dim3(Fir4Geo<16384>::T), Fir4Geo<16384>::LDS_BYTES, s, rt, jobs,
                       tables, hspec, x_in, y_out);
    return hipGetLastError();
}

hipError_t launch_fir4s(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                        const float2* tables, const float2* hspec, const float* x_in, float* y_out, int kblk) {
    static_assert(FIR4S_P == 16384, "k_fir4s<16384>: P = M");
    if (M != 16384 || kblk < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_fir4s<16384>), dim3(grid), dim3(Fir4Geo<16384>::T), Fir4Geo<16384>::LDS_BYTES, s, rt, jobs,
                       tables, hspec, x_in, y_out, kblk);
    return hipGetLastError();
}

hipError_t launch_fir4_hpart(int M, unsigned n_parts, hipStream_t s, const PresetRt* rt, const int2* part_jobs,
                             const float2* tables, const float* hs, float2* hspec) {
    if (M != 16384) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_fir4_hpart<16384>), dim3(n_parts), dim3(Fir4Geo<16384>::T), Fir4Geo<16384>::LDS_BYTES, s,
                       rt, part_jobs, tables, hs, hspec);
    return hipGetLastError();
}

hipError_t launch_fir4_hconv(unsigned n_presets, hipStream_t s, const PresetRt* rt, const int32_t* list,
                             const float2* tables, const int32_t* er_off, const double* er_gain, float2* hspec) {
    hipLaunchKernelGGL((k_fir4_hconv<16384>), dim3(n_presets), dim3(Fir4Geo<16384>::T), Fir4Geo<16384>::LDS_BYTES, s,
                       rt, list, tables, er_off, er_gain, hspec);
    return hipGetLastError();
}

hipError_t launch_fir4_irspec(unsigned n_jobs, hipStream_t s, const int64_t* jobs, const float2* tables,
                              const double* src, float2* hspec) {
    hipLaunchKernelGGL((k_fir4_irspec<16384>), dim3(n_jobs), dim3(Fir4Geo<16384>::T), Fir4Geo<16384>::LDS_BYTES, s,
                       jobs, tables, src, hspec);
    return hipGetLastError();
}

hipError_t launch_fir8(unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs, const float2* tables,
                       const float2* hspec, const float* x_in, float* y_out) {
    hipLaunchKernelGGL((k_fir8<0>), dim3(grid), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, rt, jobs, tables, hspec,
                       x_in, y_out);
    return hipGetLastError();
}

// persistent k_fir8 (fir8_fft.h): one resident workgroup per CU, blocks from
// per-XCD counters (ctr: (MSG_XCDS + 1) x FIR8P_CTR int32, zero before the first
// launch; each launch leaves them zero)
hipError_t launch_fir8p(unsigned n_jobs, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs,
                        const float2* tables, const float2* hspec, const float* x_in, float* y_out, int32_t* ctr,
                        int stagger, const msg_event* events, const float* grain_pool, const int32_t* ev_lo) {
    if (events)
        hipLaunchKernelGGL((k_fir8p<true>), dim3(grid), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, rt, jobs,
                           (int)n_jobs, tables, hspec, x_in, y_out, ctr, stagger, events, grain_pool, ev_lo);
    else
        hipLaunchKernelGGL((k_fir8p<false>), dim3(grid), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, rt, jobs,
                           (int)n_jobs, tables, hspec, x_in, y_out, ctr, stagger, events, grain_pool, ev_lo);
    return hipGetLastError();
}

// two-partition k_fir8q (fir8_fft.h): runs of run_len blocks, scratch: grid x fir8q_scratch_per_wg() float2
hipError_t launch_fir8q(unsigned n_runs, int run_len, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* runs,
                        const float2* tables, const float2* hspec, const float* x_in, float* y_out, float2* scratch,
                        int32_t* ctr, int mode) {
    hipLaunchKernelGGL(k_fir8q, dim3(grid), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, rt, runs, (int)n_runs, run_len,
                       tables, hspec, x_in, y_out, scratch, ctr, mode);
    return hipGetLastError();
}
int64_t fir8q_scratch_per_wg() { return fir8::Q2_SLOT; }

hipError_t launch_fir8_hconv(unsigned n_presets, hipStream_t s, const PresetRt* rt, const int32_t* list,
                             const float2* tables, const int32_t* er_off, const double* er_gain, float2* hspec) {
    hipLaunchKernelGGL((k_fir8_hconv<0>), dim3(2 * n_presets), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, rt, list,
                       tables, er_off, er_gain, hspec);
    return hipGetLastError();
}

hipError_t launch_fir8_spec64(unsigned n_jobs, hipStream_t s, const int64_t* jobs, const float2* tables,
                              const double* src, float2* hspec) {
    hipLaunchKernelGGL((k_fir8_spec<double>), dim3(2 * n_jobs), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, jobs,
                       tables, src, hspec);
    return hipGetLastError();
}

hipError_t launch_fir8_spec32(unsigned n_jobs, hipStream_t s, const int64_t* jobs, const float2* tables,
                              const float* src, float2* hspec) {
    hipLaunchKernelGGL((k_fir8_spec<float>), dim3(2 * n_jobs), dim3(fir8::T), Fir4Geo<16384>::LDS_BYTES, s, jobs,
                       tables, src, hspec);
    return hipGetLastError();
}

template <int M>
static hipError_t fdl_go(unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs, const float2* tables,
                         const float2* hspec, float2* xspec, const float* x_in, float* y_out) {
    hipLaunchKernelGGL((k_fdl_fwd<M>), dim3(grid), dim3(FirGeo<M>::T), FirGeo<M>::LDS_BYTES, s, rt, jobs, tables,
                       x_in, xspec);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_fdl_mac<M>), dim3(grid), dim3(FirGeo<M>::T), FirGeo<M>::LDS_BYTES, s, rt, jobs, tables,
                       hspec, (const float2*)xspec, y_out);
    return hipGetLastError();
}

hipError_t launch_fdl(int M, unsigned grid, hipStream_t s, const PresetRt* rt, const int2* jobs, const float2* tables,
                      const float2* hspec, float2* xspec, const float* x_in, float* y_out) {
    switch (M) {
        case 8192: return fdl_go<8192>(grid, s, rt, jobs, tables, hspec, xspec, x_in, y_out);
        case 16384: return fdl_go<16384>(grid, s, rt, jobs, tables, hspec, xspec, x_in, y_out);
        default: return hipErrorInvalidValue;
    }
}

// ---- FFT engine micro-benchmark (msg_bench_fft): reps x (forward + inverse)
// real transforms of length n per block, LDS-resident, no HBM traffic.
template <int T, int MAXM, int RSET>
__global__ void __launch_bounds__(T) k_fft_bench(const RealPlan* __restrict__ plans, int plan, int reps,
                                                  float* __restrict__ sink) {
    extern __shared__ __attribute__((aligned(16))) float2 lds[];
    const RealPlan& rp = plans[plan];
    const bool evn = rp.even != 0;
    for (int u = threadIdx.x; u < rp.n; u += T) rx_set(lds, evn, u, (float)((u * 7919) % 113) * 1e-2f);
    const TwLds tw = stage_twiddles<T>(lds + rp.lds_c, rp);
    for (int r = 0; r < 2 * reps; ++r) rtransform<T, MAXM, RSET>(lds, rp, tw, (r & 1) != 0);
    if (threadIdx.x == 0) sink[blockIdx.x] = rx_get(lds, evn, 1);
}

void fft_bench_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_fft_bench<FIR_T, FIR_M, RSET_PO2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_fft_bench<SPEC_T_BIG, SPEC_M_BIG, RSET_ALL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

hipError_t launch_fft_bench(bool po2, unsigned grid, int lds_bytes, hipStream_t s, const RealPlan* plans, int plan,
                            int reps, float* sink) {
    if (po2)
        hipLaunchKernelGGL((k_fft_bench<FIR_T, FIR_M, RSET_PO2>), dim3(grid), dim3(FIR_T), lds_bytes, s, plans, plan,
                           reps, sink);
    else
        hipLaunchKernelGGL((k_fft_bench<SPEC_T_BIG, SPEC_M_BIG, RSET_ALL>), dim3(grid), dim3(SPEC_T_BIG), lds_bytes,
                           s, plans, plan, reps, sink);
    return hipGetLastError();
}

#ifdef MSG_STAMPS
// phase stamps of k_fir8 (debug builds): read and reset
extern "C" int msg_debug_stamps_fir(unsigned long long* out, int n) {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fir_stamps), sizeof(h)) != hipSuccess) return 3;
    for (int i = 0; i < n && i < 16; ++i) out[i] = h[i];
    const unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_fir_stamps), z, sizeof(z)) == hipSuccess ? 0 : 3;
}
#endif
