// k_stereo_odd.hip — translation unit of the odd-length stereo rotation (kernels_stereo_odd.h).
#include "kernels_stereo_odd.h"
#include "launch.h"

void stereo_odd_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_so_cols<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_so_cols<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_so_rows, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

static bool so_shape(int64_t n, int64_t& M, int& M1, int& M2, int& C) {
    M = 1;
    while (M < 2 * n - 1) M <<= 1;
    M2 = (int)std::min<int64_t>(M, SO_ROW_MAX);
    M1 = (int)(M / M2);
    if (M1 > SO_COL_MAX) return false;
    C = std::min(M2, SO_COL_ELEMS / std::max(M1, 1));
    return true;
}

int64_t stereo_odd_len(int64_t n) {
    int64_t M; int M1, M2, C;
    return so_shape(n, M, M1, M2, C) ? M : -1;
}

// A <- F(A) . Bp -> inverse (natural order, unscaled but Bp carries 1/M)
static hipError_t so_conv(float2* A, const float2* Bp, int64_t M, int M1, int M2, int C, hipStream_t s) {
    const size_t lc = (size_t)(M1 + C * M1) * sizeof(float2), lr = (size_t)2 * M2 * sizeof(float2);
    if (M1 > 1) hipLaunchKernelGGL(k_so_cols<false>, dim3(M2 / C), dim3(SO_T), lc, s, A, M1, M2, C);
    hipLaunchKernelGGL(k_so_rows, dim3(M1), dim3(SO_T), lr, s, A, M2, Bp);
    if (M1 > 1) hipLaunchKernelGGL(k_so_cols<true>, dim3(M2 / C), dim3(SO_T), lc, s, A, M1, M2, C);
    (void)M;
    return hipGetLastError();
}

hipError_t launch_stereo_odd_kernel(int64_t n, float2* Bp, float2* A, hipStream_t s) {
    int64_t M; int M1, M2, C;
    if (!so_shape(n, M, M1, M2, C)) return hipErrorInvalidValue;
    const unsigned g = (unsigned)((M + 255) / 256);
    hipLaunchKernelGGL(k_so_bfill, dim3(g), dim3(256), 0, s, Bp, n, M);
    const size_t lc = (size_t)(M1 + C * M1) * sizeof(float2), lr = (size_t)2 * M2 * sizeof(float2);
    if (M1 > 1) hipLaunchKernelGGL(k_so_cols<false>, dim3(M2 / C), dim3(SO_T), lc, s, Bp, M1, M2, C);
    hipLaunchKernelGGL(k_so_rows, dim3(M1), dim3(SO_T), lr, s, Bp, M2, (const float2*)nullptr);
    (void)A;
    return hipGetLastError();
}

hipError_t launch_stereo_odd(int64_t n, int dr, double width, const float* y, const float2* Bp, float2* A,
                             float* r2, hipStream_t s) {
    int64_t M; int M1, M2, C;
    if (!so_shape(n, M, M1, M2, C)) return hipErrorInvalidValue;
    const unsigned g = (unsigned)((M + 255) / 256);
    hipLaunchKernelGGL(k_so_pre, dim3(g), dim3(256), 0, s, A, y, n, dr, M);
    hipError_t e = so_conv(A, Bp, M, M1, M2, C, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_so_mid, dim3(g), dim3(256), 0, s, A, n, 0.9 * width, n / 2, M);
    e = so_conv(A, Bp, M, M1, M2, C, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_so_post, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, r2, n);
    return hipGetLastError();
}
