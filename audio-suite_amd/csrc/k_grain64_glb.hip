// k_grain64_glb.hip — k_grain64<true>: the float64 grain chain for grains beyond
// the LDS engine, in global-memory slots (kernels_grain64.h).  Its own TU so
// that it compiles in parallel with the LDS instantiation (k_grain64_lds.hip).
#include "kernels_grain64.h"
#include "launch.h"

hipError_t launch_grain64_glb(const G64Global& g, unsigned grid, hipStream_t s, const msg_preset* presets,
                              const Ev64* ev64, const PresetRt* rt, const Real64Plan* plans, const int32_t* list,
                              int n_list, const double* irbank, const uint8_t* imgbank, nprng::Zig z,
                              double* micro64, double* grain64, double2* save, float* grain_pool) {
    hipLaunchKernelGGL(k_grain64<true>, dim3(grid), dim3(G64_T), 0, s, presets, ev64, rt, plans, list, n_list,
                       irbank, imgbank, z, micro64, grain64, save, grain_pool, g.A, g.B, g.mask, g.slot_cap,
                       g.mask_words);
    return hipGetLastError();
}
