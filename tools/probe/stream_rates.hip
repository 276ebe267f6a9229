// Streaming-rate probe: what HBM rate a pass with the stereo pair's access
// pattern can reach on one MI355X, as the practical ceiling its roofline
// fraction is read against.
// Buffers of C3's size (393 M frames: y 1.57 GB, stereo out 3.15 GB):
//   read       sum of y                                   4 B / frame
//   write      out = const                                8 B / frame
//   copy       out[f] = (y[f], y[f])                      4 + 8 B / frame
//   copy2      out[f] = (y[f - dl], y[f + dr])            4 + 8 B / frame (second read from L2)
// float4 accesses, grid-stride over 8 workgroups of 256 threads per CU; the
// best of 10 timed repetitions after 2 warm-up runs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int T = 256;

__global__ void __launch_bounds__(T) k_read(const float4* __restrict__ y, int64_t n4, float* __restrict__ sink) {
    float acc = 0.f;
    for (int64_t i = blockIdx.x * (int64_t)T + threadIdx.x; i < n4; i += (int64_t)gridDim.x * T) {
        const float4 v = y[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 1234.5f) sink[threadIdx.x] = acc;   // keeps the loads, never true for the data used
}

__global__ void __launch_bounds__(T) k_write(float4* __restrict__ out, int64_t n4) {
    for (int64_t i = blockIdx.x * (int64_t)T + threadIdx.x; i < n4; i += (int64_t)gridDim.x * T)
        out[i] = make_float4(0.5f, -0.5f, 0.25f, -0.25f);
}

// frame f of y -> (L, R) pair of out; 4 frames per thread-iteration: one float4
// load, two float4 stores
__global__ void __launch_bounds__(T) k_copy(const float4* __restrict__ y, int64_t n4, float4* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)T + threadIdx.x; i < n4; i += (int64_t)gridDim.x * T) {
        const float4 v = y[i];
        out[2 * i] = make_float4(v.x, v.x, v.y, v.y);
        out[2 * i + 1] = make_float4(v.z, v.z, v.w, v.w);
    }
}

// L from y shifted back by dl4 float4s, R shifted forward by dr4 (wrapped)
__global__ void __launch_bounds__(T) k_copy2(const float4* __restrict__ y, int64_t n4, int dl4, int dr4,
                                             float4* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)T + threadIdx.x; i < n4; i += (int64_t)gridDim.x * T) {
        int64_t il = i - dl4, ir = i + dr4;
        if (il < 0) il += n4;
        if (ir >= n4) ir -= n4;
        const float4 l = y[il], r = y[ir];
        out[2 * i] = make_float4(l.x, r.x, l.y, r.y);
        out[2 * i + 1] = make_float4(l.z, r.z, l.w, r.w);
    }
}

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const int64_t frames = 393216000, n4 = frames / 4;
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const unsigned grid = (unsigned)cus * 8;
    float4 *y, *out;
    float* sink;
    CHK(hipMalloc(&y, sizeof(float4) * n4));
    CHK(hipMalloc(&out, 2 * sizeof(float4) * n4));
    CHK(hipMalloc(&sink, sizeof(float) * T));
    CHK(hipMemset(y, 0, sizeof(float4) * n4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto run = [&](const char* name, double bytes, auto launch) -> int {
        float best = 1e30f;
        for (int it = 0; it < 12; ++it) {
            CHK(hipEventRecord(a, nullptr));
            launch();
            CHK(hipGetLastError());
            CHK(hipEventRecord(b, nullptr));
            CHK(hipEventSynchronize(b));
            float ms = 0.f;
            CHK(hipEventElapsedTime(&ms, a, b));
            if (it >= 2 && ms < best) best = ms;
        }
        printf("%-8s %8.3f ms  %7.1f GB/s  (%.2f GB)\n", name, best, bytes / (best * 1e-3) / 1e9, bytes / 1e9);
        return 0;
    };
    if (run("read", 4.0 * frames, [&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(T), 0, nullptr, y, n4, sink); })) return 1;
    if (run("write", 8.0 * frames, [&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(T), 0, nullptr, out, 2 * n4); })) return 1;
    if (run("copy", 12.0 * frames, [&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(T), 0, nullptr, y, n4, out); })) return 1;
    if (run("copy2", 12.0 * frames,
            [&] { hipLaunchKernelGGL(k_copy2, dim3(grid), dim3(T), 0, nullptr, y, n4, 96, 128, out); })) return 1;
    CHK(hipFree(y));
    CHK(hipFree(out));
    CHK(hipFree(sink));
    return 0;
}
