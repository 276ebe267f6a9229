// k_fir64.hip — translation unit of the float64 space FIR (kernels_fir64.h).
#include "kernels_fir64.h"
#include "launch.h"

void fir64_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_hspec64, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    (void)hipFuncSetAttribute((const void*)k_fir64, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
}

hipError_t launch_fir64_flag(const Fir64Launch& a, hipStream_t s) {
    hipLaunchKernelGGL(k_fir64_flag, dim3(1), dim3(64), 0, s, a.n_presets, a.flag64, a.maxbits, a.slot_preset,
                       a.n_slots);
    return hipGetLastError();
}

hipError_t launch_fir64(const Fir64Launch& a, hipStream_t s) {
    // small persistent grids: with no flagged preset every workgroup exits at once,
    // and one waiting for a CU held by another stream's kernel delays little
    for (int w0 = 0; w0 < a.n_cand; w0 += a.cap) {
        hipLaunchKernelGGL(k_h64, dim3((unsigned)std::min<int64_t>((int64_t)a.cap * a.tmax, 256)), dim3(H_T), 0, s, a.rt, a.fr,
                           a.slot_preset, a.n_slots, w0, a.cap, a.tmax, a.er_off, a.er_gain, a.irbank, a.h64,
                           a.h_stride);
        hipLaunchKernelGGL(k_hspec64, dim3((unsigned)std::min<int64_t>((int64_t)a.cap * a.qmax, 128)), dim3(FIR64_T), a.lds_bytes, s,
                           a.fr, a.plans, a.plan, a.slot_preset, a.n_slots, w0, a.cap, a.qmax, a.h64, a.h_stride,
                           a.hs64, a.hs_stride);
        hipLaunchKernelGGL(k_fir64, dim3((unsigned)std::min<int64_t>((int64_t)a.cap * a.bmax, 256)), dim3(FIR64_T), a.lds_bytes, s,
                           a.rt, a.fr, a.plans, a.plan, a.slot_preset, a.n_slots, w0, a.cap, a.bmax, a.hs64,
                           a.hs_stride, a.x, a.y);
    }
    return hipGetLastError();
}
