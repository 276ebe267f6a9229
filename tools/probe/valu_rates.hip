// Issue-rate probe for the integer ops of the PCG64 step (v_mad_u64_u32,
// v_mul_lo_u32, v_mul_hi_u32) against v_fma_f32: 8 independent chains per lane,
// 4 waves per SIMD; prints cycles per wave-instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
constexpr int ITER = 4096;
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
    uint32_t a[8]; uint64_t w[8];
    for (int i = 0; i < 8; ++i) { a[i] = threadIdx.x * 7 + i + seed; w[i] = a[i]; }
    float f[8];
    for (int i = 0; i < 8; ++i) f[i] = (float)a[i];
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (OP == 0) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[i]) : "v"(a[i]), "s"(seed) : "vcc");
            if (OP == 1) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(seed));
            if (OP == 2) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(seed));
            if (OP == 3) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[i]) : "s"(seed));
            if (OP == 4) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(w[i]) : "v"(a[i]));
            if (OP == 5) asm volatile("v_alignbit_b32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(a[(i + 1) & 7]));
            if (OP == 6) asm volatile("v_exp_f32 %0, %0" : "+v"(f[i]));
            if (OP == 7) asm volatile("v_pk_fma_f32 %0, %0, %0, %0" : "+v"(w[i]));
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)w[i] + __float_as_uint(f[i]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
    int dev; hipGetDevice(&dev); hipDeviceProp_t pr; hipGetDeviceProperties(&pr, dev);
    const int cus = pr.multiProcessorCount;
    const int blocks = cus * 4;          // 4 x 256 threads per CU = 4 waves per SIMD
    uint32_t* out; hipMalloc(&out, sizeof(uint32_t) * blocks * 256);
    const char* names[] = {"v_mad_u64_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_fma_f32", "v_lshlrev_b64", "v_alignbit_b32", "v_exp_f32", "v_pk_fma_f32"};
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int clk = 0; hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
    for (int op = 0; op < 8; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0);
            switch (op) {
                case 0: k<0><<<blocks, 256>>>(out, 3); break; case 1: k<1><<<blocks, 256>>>(out, 3); break;
                case 2: k<2><<<blocks, 256>>>(out, 3); break; case 3: k<3><<<blocks, 256>>>(out, 3); break;
                case 4: k<4><<<blocks, 256>>>(out, 3); break; case 5: k<5><<<blocks, 256>>>(out, 3); break;
                case 6: k<6><<<blocks, 256>>>(out, 3); break; case 7: k<7><<<blocks, 256>>>(out, 3); break;
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            // wave-instructions per SIMD: 4 waves x ITER x 8
            const double per_simd = 4.0 * ITER * 8;
            if (rep) printf("%-16s %.3f ms  %.2f ns per wave-instr per SIMD  (%.1f cycles at %d MHz)\n", names[op], ms,
                            ms * 1e6 / per_simd, ms * 1e-3 / per_simd * clk * 1e3, clk / 1000);
        }
    }
    return 0;
}
