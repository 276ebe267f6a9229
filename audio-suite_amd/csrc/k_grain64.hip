// k_grain64.hip — translation unit of the float64 chain's smaller kernels
// (kernels_grain64.h): k_chain64, k_fft64_one, k_stft64.  The two k_grain64
// instantiations compile in k_grain64_lds.hip and k_grain64_glb.hip.
#include "kernels_grain64.h"
#include "launch.h"

// launch.h keeps host copies of the float64 engine's shape for the planner
static_assert(G64_THREADS == G64_T, "launch.h G64_THREADS must match kernels_grain64.h G64_T");
static_assert(G64_SLOTS == G64_CAP, "launch.h G64_SLOTS must match kernels_grain64.h G64_CAP");
static_assert(G64_MAXPAR_HOST == G64_MAXPAR, "launch.h G64_MAXPAR_HOST must match kernels_grain64.h G64_MAXPAR");

// Single float64 real transform (tests / precision probes): inverse = 0 ->
// io[0..n) real in, io[0..2K) = X[0..K) out; inverse = 1 -> X in, real out.
__global__ void __launch_bounds__(G64_T)
k_fft64_one(const Real64Plan* __restrict__ plans, int plan, int inverse, double* __restrict__ io,
            double2* gA, double2* gB) {
    extern __shared__ __attribute__((aligned(16))) double2 lds_buf[];
    double2* buf = gA ? gA : lds_buf;      // global buffers: the engine's ping-pong mode
    double2* scr = gA ? gB : nullptr;
    const Real64Plan& rp = plans[plan];
    const int n = rp.n, K = n / 2 + 1;
    double* d = reinterpret_cast<double*>(buf);
    const int cnt = inverse ? 2 * K : n;
    for (int j = threadIdx.x; j < cnt; j += G64_T) d[j] = io[j];
    __syncthreads();
    if (inverse) f64_irfft<G64_T, G64_MAXE>(buf, rp, scr);
    else f64_rfft<G64_T, G64_MAXE>(buf, rp, scr);
    __syncthreads();
    const int cnt2 = inverse ? n : 2 * K;
    for (int j = threadIdx.x; j < cnt2; j += G64_T) io[j] = d[j];
}

void grain64_init_attrs() {
    grain64_lds_init_attr();
    (void)hipFuncSetAttribute((const void*)k_chain64<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              G64_CAP * 16);
    (void)hipFuncSetAttribute((const void*)k_fft64_one, hipFuncAttributeMaxDynamicSharedMemorySize, G64_CAP * 16);
}

hipError_t launch_grain64(const G64Global* g, unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets,
                          const Ev64* ev64, const PresetRt* rt, const Real64Plan* plans, const int32_t* list,
                          int n_list, const double* irbank, const uint8_t* imgbank, nprng::Zig z, double* micro64,
                          double* grain64, double2* save, float* grain_pool) {
    if (g)
        return launch_grain64_glb(*g, grid, s, presets, ev64, rt, plans, list, n_list, irbank, imgbank, z, micro64,
                                  grain64, save, grain_pool);
    return launch_grain64_lds(grid, lds_bytes, s, presets, ev64, rt, plans, list, n_list, irbank, imgbank, z,
                              micro64, grain64, save, grain_pool);
}

hipError_t launch_chain64(const G64Global* g, unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets,
                          const Ev64* ev64, const Chain64* chains, int n_chains, const Real64Plan* plans,
                          const double* grain64, double* state, float* grain_pool) {
    if (g)
        hipLaunchKernelGGL(k_chain64<true>, dim3(grid), dim3(G64_T), 0, s, presets, ev64, chains, n_chains, plans,
                           grain64, state, grain_pool, g->A, g->B, g->slot_cap);
    else
        hipLaunchKernelGGL(k_chain64<false>, dim3(grid), dim3(G64_T), lds_bytes, s, presets, ev64, chains, n_chains,
                           plans, grain64, state, grain_pool, (double2*)nullptr, (double2*)nullptr, (int64_t)0);
    return hipGetLastError();
}

hipError_t launch_fft64_one(int lds_bytes, hipStream_t s, const Real64Plan* plans, int plan, int inverse,
                            double* io, double2* gA, double2* gB) {
    hipLaunchKernelGGL(k_fft64_one, dim3(1), dim3(G64_T), gA ? 0 : lds_bytes, s, plans, plan, inverse, io, gA, gB);
    return hipGetLastError();
}

hipError_t launch_stft64(unsigned frames, int lds_bytes, hipStream_t s, const Real64Plan* plans, int plan,
                         const void* x, int elem_bytes, int64_t n, int channels, int win, int hop, double* S) {
    if (elem_bytes == 8) {
        (void)hipFuncSetAttribute((const void*)k_stft64<double>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  G64_CAP * 16);
        hipLaunchKernelGGL(k_stft64<double>, dim3(frames), dim3(G64_T), lds_bytes, s, plans, plan,
                           (const double*)x, n, channels, win, hop, S);
    } else {
        (void)hipFuncSetAttribute((const void*)k_stft64<float>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  G64_CAP * 16);
        hipLaunchKernelGGL(k_stft64<float>, dim3(frames), dim3(G64_T), lds_bytes, s, plans, plan,
                           (const float*)x, n, channels, win, hop, S);
    }
    return hipGetLastError();
}
