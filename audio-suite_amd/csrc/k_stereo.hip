// k_stereo.hip — translation unit of the stereo / tanh / normalise kernels (kernels_stereo.h).
#include "kernels_stereo.h"
#include "launch.h"

hipError_t launch_stereo_max(unsigned n_tiles, hipStream_t s, const PresetRt* rt, const int32_t* st_begin, int n_presets,
                             const float* y, unsigned* maxbits, const StereoSync& sy) {
    hipLaunchKernelGGL(k_stereo_max, dim3(n_tiles), dim3(ST_T), 0, s, rt, st_begin, n_presets, (int)n_tiles, y, maxbits,
                       sy);
    return hipGetLastError();
}

hipError_t launch_stereo_pred(unsigned n_presets, hipStream_t s, const PresetRt* rt, const int32_t* st_begin,
                              int n_tiles, const unsigned* maxbits, const StereoSync& sy) {
    hipLaunchKernelGGL(k_stereo_pred, dim3(n_presets), dim3(ST_T), 0, s, rt, st_begin, (int)n_presets, n_tiles, maxbits,
                       sy);
    return hipGetLastError();
}

hipError_t launch_stereo_fused(unsigned grid, unsigned n_tiles, hipStream_t s, const PresetRt* rt,
                               const int32_t* st_begin, int n_presets, const float* y, unsigned* maxbits,
                               const StereoSync& sy, int32_t* ctr, float* out) {
    hipLaunchKernelGGL(k_stereo_fused, dim3(grid), dim3(ST_T), 0, s, rt, st_begin, n_presets, (int)n_tiles, y, maxbits,
                       sy, ctr, out);
    return hipGetLastError();
}

hipError_t launch_stereo_out(unsigned n_tiles, hipStream_t s, const PresetRt* rt, const int32_t* st_begin, int n_presets,
                             const float* y, const float* r2, const unsigned* maxbits, float* out) {
    hipLaunchKernelGGL(k_stereo_out, dim3(n_tiles), dim3(ST_T), 0, s, rt, st_begin, n_presets, y, r2, maxbits, out);
    return hipGetLastError();
}

hipError_t launch_stereo_remax(unsigned grid, hipStream_t s, const PresetRt* rt, const int32_t* st_count,
                               const int32_t* list, const int32_t* n_list, int tmax, const float* y, const float* r2,
                               unsigned* maxbits) {
    hipLaunchKernelGGL(k_stereo_remax, dim3(grid), dim3(ST_T), 0, s, rt, st_count, list, n_list, tmax, y, r2, maxbits);
    return hipGetLastError();
}

hipError_t launch_stereo_out_list(unsigned grid, hipStream_t s, const PresetRt* rt, const int32_t* st_count,
                                  const int32_t* list, const int32_t* n_list, int tmax, const float* y, const float* r2,
                                  const unsigned* maxbits, float* out) {
    hipLaunchKernelGGL(k_stereo_out_list, dim3(grid), dim3(ST_T), 0, s, rt, st_count, list, n_list, tmax, y, r2,
                       maxbits, out);
    return hipGetLastError();
}
