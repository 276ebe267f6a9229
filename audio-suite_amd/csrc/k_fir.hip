// k_fir.hip — translation unit of the space FIR kernels.
#include "kernels_fir.h"
#include "launch.h"

void fir_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_fir<FIR_T, FIR_M>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
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

hipError_t launch_fir_h(unsigned grid, int lds_bytes, hipStream_t s, const PresetRt* rt, const int32_t* hblk_begin,
                        int n_presets, const RealPlan* fir_plans, const int32_t* fir_plan_of,
                        const int32_t* er_off, const double* er_gain, const double* ir_bank,
                        const float2* ir_spec, float2* hspec) {
    hipLaunchKernelGGL((k_fir_h<FIR_T, FIR_M>), dim3(grid), dim3(FIR_T), lds_bytes, s, rt, hblk_begin, n_presets,
                       fir_plans, fir_plan_of, er_off, er_gain, ir_bank, ir_spec, hspec);
    return hipGetLastError();
}

hipError_t launch_fir(unsigned grid, int lds_bytes, hipStream_t s, const PresetRt* rt, const int32_t* fblk_begin,
                      int n_presets, const RealPlan* fir_plans, const int32_t* fir_plan_of,
                      const float2* hspec, const float* x_in, float* y_out) {
    hipLaunchKernelGGL((k_fir<FIR_T, FIR_M>), dim3(grid), dim3(FIR_T), lds_bytes, s, rt, fblk_begin, n_presets,
                       fir_plans, fir_plan_of, hspec, x_in, y_out);
    return hipGetLastError();
}
