// k_spec3.hip — translation unit of the band-pruned register-resident spectral
// kernel (spec3.h) for the 30 MHz hot length.
#include "spec3.h"
#include "launch.h"
#include <algorithm>
#include <cstdlib>
#include <cmath>

void spec3_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_spec3<Spec3P18750>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Spec3P18750::LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)k_spec3p<Spec3P18750>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              Spec3P18750::LDS_BYTES);
}

bool spec3_tables(std::vector<float>& out) {
    spec3_tables<Spec3P18750>(out);
    return true;
}

// The event runs on k_spec3 (see spec3.h "Eligibility"): returns true and its band.
bool spec3_eligible(int n, int ops, int gen_sr, double cutoff_gen, double roll, double stretch, int64_t float_off,
                    int32_t* kb, int32_t* kz, int32_t* ky, double* inv_f, int32_t* exact32) {
    using P = Spec3P18750;
    if (n != 2 * P::M || (float_off & 1)) return false;
    if (ops & (SPEC_TILT_NOISE | SPEC_TILT_SKEW | SPEC_WARP)) return false;
    if (!(ops & SPEC_LOWPASS)) return false;
    const Spec3Band b = s3_band(n, gen_sr, cutoff_gen, roll, (ops & SPEC_STRETCH) != 0, stretch);
    if (b.kz > b.ky) return false;
    if (b.ky <= P::M / 2 ? !s3_band_fits<P>(b.kz, b.ky)                       // narrow: X, Z' halves in LDS
                         : (2 * ((b.kz + 15) & ~15) > P::BUF || b.ky > P::BUF ||  // wide: Z[k], Z[M-k]; Y over X,
                            ((ops & SPEC_STRETCH) && stretch <= 1.0))) return false;   // which needs f > 1
    static const bool wide_on = !(getenv("MSGPU_S3_WIDE") && getenv("MSGPU_S3_WIDE")[0] == '0');   // A/B switch
    if (b.ky > P::M / 2 && !wide_on) return false;
    *kb = b.kb; *kz = b.kz; *ky = b.ky; *inv_f = b.inv_f;
    // k / f exact in float32 for every bin k < 2^15 (the wide path's gather):
    // 1 / f = q 2^-12 with q's odd part below 2^24 / 2^15
    double sc = b.inv_f * 4096.0;
    bool ok = sc == std::floor(sc) && sc > 0.0 && sc < 4096.0 * 4096.0;
    if (ok)
        while (std::fmod(sc, 2.0) == 0.0) sc *= 0.5;
    *exact32 = (ok && sc < 512.0) ? 1 : 0;
    return true;
}

hipError_t launch_spec3(unsigned grid, hipStream_t s, const msg_event* events, const EventRt* ert, const PresetRt* rt,
                        const float2* tables, const int32_t* ev_list, int n_list, const float* micro_pool,
                        float* grain_pool, int persist, int32_t* ctr) {
    using P = Spec3P18750;
    if (persist > 0 && ctr) {
        grid = (unsigned)std::max(1, std::min(persist, n_list));
        hipLaunchKernelGGL((k_spec3p<P>), dim3(grid), dim3(P::T), P::LDS_BYTES, s, events, ert, rt, tables, ev_list,
                           n_list, micro_pool, grain_pool, ctr);
        return hipGetLastError();
    }
    grid = (unsigned)((n_list + MSG_S3_EVENTS - 1) / MSG_S3_EVENTS);   // MSG_S3_EVENTS per workgroup (spec3.h)
    hipLaunchKernelGGL((k_spec3<P>), dim3(grid), dim3(P::T), P::LDS_BYTES, s, events, ert, rt, tables, ev_list,
                       n_list, micro_pool, grain_pool);
    return hipGetLastError();
}

#ifdef MSG_STAMPS
// per-TU phase stamps of k_spec3 (debug builds): read and reset
extern "C" int msg_debug_stamps_s3(unsigned long long* out, int n) {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_spec_stamps), sizeof(h)) != hipSuccess) return 3;
    for (int i = 0; i < n && i < 16; ++i) out[i] = h[i];
    const unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_spec_stamps), z, sizeof(z)) == hipSuccess ? 0 : 3;
}
#endif
