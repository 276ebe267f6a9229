// k_spectral_ct.hip — translation unit of the compile-time-plan spectral kernels.
#include "spec_ct.h"
#include "launch.h"

template <class P> static void ct_attr() {
    (void)hipFuncSetAttribute((const void*)k_spectral_ct<P>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              P::LDS_BYTES);
}

void spectral_ct_init_attrs() {
    ct_attr<SpecP18750>(); ct_attr<SpecP15000>(); ct_attr<SpecP1200>(); ct_attr<SpecP960>(); ct_attr<SpecP750>();
    ct_attr<SpecP240>();
}

// index of the compile-time plan for grain length n, -1 if none
int spectral_ct_plan(int n) {
    switch (n) {
        case 2 * SpecP18750::M: return 0;
        case 2 * SpecP15000::M: return 1;
        case 2 * SpecP1200::M: return 2;
        case 2 * SpecP960::M: return 3;
        case 2 * SpecP750::M: return 4;
        case 2 * SpecP240::M: return 5;
        default: return -1;
    }
}

bool spectral_ct_tables(int plan, std::vector<float>& out) {
    switch (plan) {
        case 0: spec_ct_tables<SpecP18750>(out); return true;
        case 1: spec_ct_tables<SpecP15000>(out); return true;
        case 2: spec_ct_tables<SpecP1200>(out); return true;
        case 3: spec_ct_tables<SpecP960>(out); return true;
        case 4: spec_ct_tables<SpecP750>(out); return true;
        case 5: spec_ct_tables<SpecP240>(out); return true;
        default: return false;
    }
}

template <class P>
static hipError_t ct_go(unsigned grid, hipStream_t s, const msg_event* events, const EventRt* ert,
                        const PresetRt* rt, const float2* tables, const int32_t* ev_list, int n_list,
                        float* micro_pool, float* grain_pool) {
    hipLaunchKernelGGL((k_spectral_ct<P>), dim3(grid), dim3(P::T), P::LDS_BYTES, s, events, ert, rt, tables,
                       ev_list, n_list, micro_pool, grain_pool);
    return hipGetLastError();
}

hipError_t launch_spectral_ct(int plan, unsigned grid, hipStream_t s, const msg_event* events, const EventRt* ert,
                              const PresetRt* rt, const float2* tables, const int32_t* ev_list, int n_list,
                              float* micro_pool, float* grain_pool) {
    switch (plan) {
        case 0: return ct_go<SpecP18750>(grid, s, events, ert, rt, tables, ev_list, n_list, micro_pool, grain_pool);
        case 1: return ct_go<SpecP15000>(grid, s, events, ert, rt, tables, ev_list, n_list, micro_pool, grain_pool);
        case 2: return ct_go<SpecP1200>(grid, s, events, ert, rt, tables, ev_list, n_list, micro_pool, grain_pool);
        case 3: return ct_go<SpecP960>(grid, s, events, ert, rt, tables, ev_list, n_list, micro_pool, grain_pool);
        case 4: return ct_go<SpecP750>(grid, s, events, ert, rt, tables, ev_list, n_list, micro_pool, grain_pool);
        case 5: return ct_go<SpecP240>(grid, s, events, ert, rt, tables, ev_list, n_list, micro_pool, grain_pool);
        default: return hipErrorInvalidValue;
    }
}

#ifdef MSG_STAMPS
// per-TU copy of the phase stamps (no relocatable device code): the
// compile-time-plan kernels' own counters
extern "C" int msg_debug_stamps_ct(unsigned long long* out, int n) {
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_spec_stamps), sizeof(h)) != hipSuccess) return 3;
    for (int i = 0; i < n && i < 16; ++i) out[i] = h[i];
    const unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_spec_stamps), z, sizeof(z)) == hipSuccess ? 0 : 3;
}
#endif
