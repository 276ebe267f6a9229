// k_stereo_odd.hip — translation unit of the odd-length stereo rotation (kernels_stereo_odd.h).
#include "kernels_stereo_odd.h"
#include "launch.h"

void stereo_odd_init_attrs() {
    (void)hipFuncSetAttribute((const void*)k_so_cols<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_so_cols<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)k_so_rows, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
}

// M = M0 x M1 x M2 (M0 = 1 up to 2^23): row transforms of M2 <= 4096
// contiguous elements, column transforms of M1 <= 2048, and above that a top
// column level of M0 <= 2048 over stride M1 M2.  row_max / col_max lower the
// row and column limits (MSGPU_SO_ROW / MSGPU_SO_COL at msg_create, tests
// only) so the three-level path runs at small n.
struct SoShape { int64_t M; int M0, M1, M2, C0, C; };
static bool so_shape(int64_t n, int row_max, int col_max, SoShape& g) {
    if (row_max < 4 || row_max > SO_ROW_MAX || (row_max & (row_max - 1))) row_max = SO_ROW_MAX;
    if (col_max < 2 || col_max > SO_COL_MAX || (col_max & (col_max - 1))) col_max = SO_COL_MAX;
    g.M = 1;
    while (g.M < 2 * n - 1) g.M <<= 1;
    g.M2 = (int)std::min<int64_t>(g.M, row_max);
    const int64_t rest = g.M / g.M2;
    g.M1 = (int)std::min<int64_t>(rest, col_max);
    const int64_t top = rest / g.M1;
    if (top > SO_COL_MAX) return false;
    g.M0 = (int)top;
    g.C = std::min(g.M2, SO_COL_ELEMS / std::max(g.M1, 1));
    const int64_t L = (int64_t)g.M1 * g.M2;
    g.C0 = (int)std::min<int64_t>(L, SO_COL_ELEMS / std::max(g.M0, 1));
    return true;
}

int64_t stereo_odd_len(int64_t n, int row_max, int col_max) {
    SoShape g;
    return so_shape(n, row_max, col_max, g) ? g.M : -1;
}

static size_t so_col_lds(int Mc, int C) { return (size_t)(Mc + C * Mc) * sizeof(double2); }

// forward FFT_M of A up to (not including) the row transforms
static void so_fwd_cols(double2* A, const SoShape& g, hipStream_t s) {
    const int64_t L = (int64_t)g.M1 * g.M2;
    if (g.M0 > 1)
        hipLaunchKernelGGL(k_so_cols<false>, dim3((unsigned)(L / g.C0), 1), dim3(SO_T), so_col_lds(g.M0, g.C0), s, A,
                           g.M0, (int)L, g.C0, (int64_t)0);
    if (g.M1 > 1)
        hipLaunchKernelGGL(k_so_cols<false>, dim3((unsigned)(g.M2 / g.C), (unsigned)g.M0), dim3(SO_T),
                           so_col_lds(g.M1, g.C), s, A, g.M1, g.M2, g.C, L);
}
static void so_inv_cols(double2* A, const SoShape& g, hipStream_t s) {
    const int64_t L = (int64_t)g.M1 * g.M2;
    if (g.M1 > 1)
        hipLaunchKernelGGL(k_so_cols<true>, dim3((unsigned)(g.M2 / g.C), (unsigned)g.M0), dim3(SO_T),
                           so_col_lds(g.M1, g.C), s, A, g.M1, g.M2, g.C, L);
    if (g.M0 > 1)
        hipLaunchKernelGGL(k_so_cols<true>, dim3((unsigned)(L / g.C0), 1), dim3(SO_T), so_col_lds(g.M0, g.C0), s, A,
                           g.M0, (int)L, g.C0, (int64_t)0);
}

// A <- F(A) . Bp -> inverse (natural order, unscaled but Bp carries 1/M)
static hipError_t so_conv(double2* A, const double2* Bp, const SoShape& g, hipStream_t s) {
    so_fwd_cols(A, g, s);
    hipLaunchKernelGGL(k_so_rows, dim3((unsigned)(g.M / g.M2)), dim3(SO_T), (size_t)2 * g.M2 * sizeof(double2), s, A,
                       g.M2, Bp);
    so_inv_cols(A, g, s);
    return hipGetLastError();
}

hipError_t launch_stereo_odd_kernel(int64_t n, int row_max, int col_max, double2* Bp, double2* A, hipStream_t s) {
    SoShape g;
    if (!so_shape(n, row_max, col_max, g)) return hipErrorInvalidValue;
    const unsigned grid = (unsigned)((g.M + 255) / 256);
    hipLaunchKernelGGL(k_so_bfill, dim3(grid), dim3(256), 0, s, Bp, n, g.M);
    so_fwd_cols(Bp, g, s);
    hipLaunchKernelGGL(k_so_rows, dim3((unsigned)(g.M / g.M2)), dim3(SO_T), (size_t)2 * g.M2 * sizeof(double2), s, Bp,
                       g.M2, (const double2*)nullptr);
    (void)A;
    return hipGetLastError();
}

hipError_t launch_stereo_odd(int64_t n, int row_max, int col_max, int dr, double width, const float* y,
                             const double2* Bp, double2* A, float* r2, hipStream_t s) {
    SoShape sh;
    if (!so_shape(n, row_max, col_max, sh)) return hipErrorInvalidValue;
    const int64_t M = sh.M;
    const unsigned g = (unsigned)((M + 255) / 256);
    hipLaunchKernelGGL(k_so_pre, dim3(g), dim3(256), 0, s, A, y, n, dr, M);
    hipError_t e = so_conv(A, Bp, sh, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_so_mid, dim3(g), dim3(256), 0, s, A, n, 0.9 * width, n / 2, M);
    e = so_conv(A, Bp, sh, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_so_post, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, r2, n);
    return hipGetLastError();
}
