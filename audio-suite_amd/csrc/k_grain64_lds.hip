// k_grain64_lds.hip — k_grain64<false>: the float64 grain chain with the grain
// resident in LDS (kernels_grain64.h).  Its own TU so that it compiles in
// parallel with the global-memory instantiation (k_grain64_glb.hip).
#include "kernels_grain64.h"
#include "launch.h"

void grain64_lds_init_attr() {
    (void)hipFuncSetAttribute((const void*)k_grain64<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              G64_CAP * 16);
}

hipError_t launch_grain64_lds(unsigned grid, int lds_bytes, hipStream_t s, const msg_preset* presets,
                              const Ev64* ev64, const PresetRt* rt, const Real64Plan* plans, const int32_t* list,
                              int n_list, const double* irbank, const uint8_t* imgbank, nprng::Zig z,
                              double* micro64, double* grain64, double2* save, float* grain_pool) {
    hipLaunchKernelGGL(k_grain64<false>, dim3(grid), dim3(G64_T), lds_bytes, s, presets, ev64, rt, plans, list,
                       n_list, irbank, imgbank, z, micro64, grain64, save, grain_pool, (double2*)nullptr,
                       (double2*)nullptr, (uint32_t*)nullptr, (int64_t)0, (int64_t)0);
    return hipGetLastError();
}
