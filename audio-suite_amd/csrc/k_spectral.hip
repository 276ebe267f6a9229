// k_spectral.hip — translation unit of the per-event spectral chain kernels.
#include "kernels_spectral.h"
#include "launch.h"

void spectral_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_spectral<SPEC_T_BIG, SPEC_M_BIG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_spectral<SPEC_T_SMALL, SPEC_M_SMALL>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, SPEC_SMALL_BYTES);
}

hipError_t launch_spectral(bool big, unsigned grid, int lds_bytes, hipStream_t s,
                           const msg_preset* presets, const msg_event* events, const EventRt* ert,
                           const PresetRt* rt, const RealPlan* plans, const int32_t* ev_list, int n_list,
                           float* micro_pool, float* grain_pool) {
    if (big)
        hipLaunchKernelGGL((k_spectral<SPEC_T_BIG, SPEC_M_BIG>), dim3(grid), dim3(SPEC_T_BIG), lds_bytes, s,
                           presets, events, ert, rt, plans, ev_list, n_list, micro_pool, grain_pool);
    else
        hipLaunchKernelGGL((k_spectral<SPEC_T_SMALL, SPEC_M_SMALL>), dim3(grid), dim3(SPEC_T_SMALL), lds_bytes, s,
                           presets, events, ert, rt, plans, ev_list, n_list, micro_pool, grain_pool);
    return hipGetLastError();
}

#ifdef MSG_STAMPS
extern "C" int msg_debug_skip(int flags) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_spec_skip), &flags, sizeof(int)) == hipSuccess ? 0 : 3;
}

extern "C" int msg_debug_stamps(unsigned long long* out, int n) {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_spec_stamps), sizeof(h)) != hipSuccess) return 3;
    for (int i = 0; i < n && i < 16; ++i) out[i] = h[i];
    const unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_spec_stamps), z, sizeof(z)) == hipSuccess ? 0 : 3;
}
#endif
