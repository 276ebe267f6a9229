// k_grain64.hip — translation unit of the float64 grain chain (kernels_grain64.h).
#include "kernels_grain64.h"
#include "launch.h"

void grain64_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_grain64, hipFuncAttributeMaxDynamicSharedMemorySize, G64_CAP * 16);
    (void)hipFuncSetAttribute((const void*)k_chain64, hipFuncAttributeMaxDynamicSharedMemorySize, G64_CAP * 16);
}

hipError_t launch_grain64(unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets, const Ev64* ev64,
                          const PresetRt* rt, const Real64Plan* plans, const int32_t* list, int n_list,
                          const double* irbank, const uint8_t* imgbank, nprng::Zig z, double* micro64,
                          double* grain64, double2* save, float* grain_pool) {
    hipLaunchKernelGGL(k_grain64, dim3(grid), dim3(G64_T), lds_bytes, s, presets, ev64, rt, plans, list, n_list,
                       irbank, imgbank, z, micro64, grain64, save, grain_pool);
    return hipGetLastError();
}

hipError_t launch_chain64(unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets, const Ev64* ev64,
                          const Chain64* chains, int n_chains, const Real64Plan* plans, const double* grain64,
                          double* state, float* grain_pool) {
    hipLaunchKernelGGL(k_chain64, dim3(grid), dim3(G64_T), lds_bytes, s, presets, ev64, chains, n_chains, plans,
                       grain64, state, grain_pool);
    return hipGetLastError();
}

hipError_t launch_fft64_one(int lds_bytes, hipStream_t s, const Real64Plan* plans, int plan, int inverse,
                            double* io) {
    (void)hipFuncSetAttribute((const void*)k_fft64_one, hipFuncAttributeMaxDynamicSharedMemorySize, G64_CAP * 16);
    hipLaunchKernelGGL(k_fft64_one, dim3(1), dim3(G64_T), lds_bytes, s, plans, plan, inverse, io);
    return hipGetLastError();
}
