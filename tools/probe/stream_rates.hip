// Streaming-rate probe: what HBM rate a pass with the stereo pair's access
// pattern can reach on one MI355X, as the practical ceiling its roofline
// fraction is read against.
// Buffers of C3's size (393 M frames: y 1.57 GB, stereo out 3.15 GB):
//   read       sum of y                                   4 B / frame
//   write      out = const                                8 B / frame
//   copy       out[f] = (y[f], y[f])                      4 + 8 B / frame
//   copy2      out[f] = (y[f - dl], y[f + dr])            4 + 8 B / frame (second read from L2)
// Variants (the round-5 probe kept one float4 load per thread in
// flight, grid-stride, default-policy stores, and reached 4.52 TB/s copy
// against the guide's 6.29):
//   U   float4 loads in flight per thread per iteration (1, 4, 8)
//   NT  nontemporal stores (and, for NT = 2, nontemporal loads too)
//   W   workgroups per CU (T threads each); 8 = the round-5 grid
//   C   traversal: 0 grid-stride, 1 one contiguous chunk per workgroup
// The best of 10 timed repetitions after 2 warm-up runs, per variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef float v4f __attribute__((ext_vector_type(4)));
template <int NT> __device__ __forceinline__ float4 ld(const float4* p) {
    if constexpr (NT >= 2) {
        const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f*>(p));
        return make_float4(v.x, v.y, v.z, v.w);
    } else {
        return *p;
    }
}
template <int NT> __device__ __forceinline__ void st(float4* p, float4 v) {
    if constexpr (NT >= 1) __builtin_nontemporal_store(v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<v4f*>(p));
    else *p = v;
}

// the index walk: element k of iteration `it` of this thread
template <int T, int U, int C> struct Walk {
    int64_t base, step, end;
    __device__ Walk(int64_t n) {
        if (C == 0) {
            base = ((int64_t)blockIdx.x * T + threadIdx.x);
            step = (int64_t)gridDim.x * T;
            end = n;
        } else {
            const int64_t per = (n + gridDim.x - 1) / gridDim.x;
            const int64_t lo = per * blockIdx.x;
            base = lo + threadIdx.x;
            step = T;
            end = lo + per < n ? lo + per : n;
        }
    }
};

template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_read(const float4* __restrict__ y, int64_t n4, float* __restrict__ sink) {
    Walk<T, U, C> w(n4);
    float acc = 0.f;
    for (int64_t i = w.base; i < w.end; i += U * w.step) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            v[u] = j < w.end ? ld<NT>(y + j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
    }
    if (acc == 1234.5f) sink[threadIdx.x] = acc;   // keeps the loads, never true for the data used
}

template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_write(float4* __restrict__ out, int64_t n4) {
    Walk<T, U, C> w(n4);
    for (int64_t i = w.base; i < w.end; i += U * w.step)
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            if (j < w.end) st<NT>(out + j, make_float4(0.5f, -0.5f, 0.25f, -0.25f));
        }
}

// frame f of y -> (L, R) pair of out; per float4 of y two float4 stores
template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_copy(const float4* __restrict__ y, int64_t n4, float4* __restrict__ out) {
    Walk<T, U, C> w(n4);
    for (int64_t i = w.base; i < w.end; i += U * w.step) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            v[u] = j < w.end ? ld<NT>(y + j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            if (j < w.end) {
                st<NT>(out + 2 * j, make_float4(v[u].x, v[u].x, v[u].y, v[u].y));
                st<NT>(out + 2 * j + 1, make_float4(v[u].z, v[u].z, v[u].w, v[u].w));
            }
        }
    }
}

// L from y shifted back by dl4 float4s, R shifted forward by dr4 (wrapped)
template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_copy2(const float4* __restrict__ y, int64_t n4, int dl4, int dr4,
                                             float4* __restrict__ out) {
    Walk<T, U, C> w(n4);
    for (int64_t i = w.base; i < w.end; i += U * w.step) {
        float4 l[U], r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            int64_t j = i + u * w.step;
            if (j >= w.end) j = i;
            int64_t il = j - dl4, ir = j + dr4;
            if (il < 0) il += n4;
            if (ir >= n4) ir -= n4;
            l[u] = ld<NT>(y + il);
            r[u] = ld<0>(y + ir);                  // the second read of a line: keep it cacheable
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            if (j < w.end) {
                st<NT>(out + 2 * j, make_float4(l[u].x, r[u].x, l[u].y, r[u].y));
                st<NT>(out + 2 * j + 1, make_float4(l[u].z, r[u].z, l[u].w, r[u].w));
            }
        }
    }
}

// copy with contiguous stores: each lane loads two frames (8 B, 512 B per wave
// instruction) and stores their (L, R) pairs as one float4 (1 KB per wave
// instruction) -- k_copy's two float4 stores per lane each cover every other
// 16 B of 2 KB, so every store instruction leaves half-written lines
template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_copyb(const float2* __restrict__ y, int64_t n2, float4* __restrict__ out) {
    Walk<T, U, C> w(n2);
    for (int64_t i = w.base; i < w.end; i += U * w.step) {
        float2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            v[u] = j < w.end ? y[j] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            if (j < w.end) st<NT>(out + j, make_float4(v[u].x, v[u].x, v[u].y, v[u].y));
        }
    }
}

// k_copy's ownership (four frames per lane) with the two stores made
// contiguous per instruction by a cross-lane exchange (ds_bpermute): store s
// of lane l writes pair-chunk 64 s + l, frames 2 (64 s + l) .. + 1, which lane
// (64 s + l) / 2 of the wave holds
template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_copys(const float4* __restrict__ y, int64_t n4, float4* __restrict__ out) {
    Walk<T, U, C> w(n4);
    const int lane = (int)(threadIdx.x & 63);
    for (int64_t i = w.base; i < w.end; i += U * w.step) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            v[u] = j < w.end ? ld<NT>(y + j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j0 = i + u * w.step - lane;          // the wave's first float4 of y
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int src = (64 * s + lane) >> 1;
                const bool hi = lane & 1;                        // frames 2, 3 of the source lane's four
                const float a1 = __shfl(v[u].x, src, 64), b1 = __shfl(v[u].y, src, 64);
                const float a2 = __shfl(v[u].z, src, 64), b2 = __shfl(v[u].w, src, 64);
                const float p = hi ? a2 : a1, q = hi ? b2 : b1;
                const int64_t chunk = 2 * j0 + 64 * s + lane;
                if (j0 + src < w.end) st<NT>(out + chunk, make_float4(p, p, q, q));
            }
        }
    }
}

// 1:1 copy (the guide's float4 copy: 16 B read, 16 B written per lane)
template <int T, int U, int NT, int C>
__global__ void __launch_bounds__(T) k_copy1(const float4* __restrict__ y, int64_t n4, float4* __restrict__ out) {
    Walk<T, U, C> w(n4);
    for (int64_t i = w.base; i < w.end; i += U * w.step) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            v[u] = j < w.end ? ld<NT>(y + j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + u * w.step;
            if (j < w.end) st<NT>(out + j, v[u]);
        }
    }
}

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Bufs { float4* y; float4* out; float* sink; int64_t frames, n4; int cus; hipEvent_t a, b; };

template <class L> static int timeit(Bufs& B, const char* name, double bytes, L launch) {
    float best = 1e30f;
    for (int it = 0; it < 12; ++it) {
        CHK(hipEventRecord(B.a, nullptr));
        launch();
        CHK(hipGetLastError());
        CHK(hipEventRecord(B.b, nullptr));
        CHK(hipEventSynchronize(B.b));
        float ms = 0.f;
        CHK(hipEventElapsedTime(&ms, B.a, B.b));
        if (it >= 2 && ms < best) best = ms;
    }
    printf("%-44s %8.3f ms  %7.1f GB/s\n", name, best, bytes / (best * 1e-3) / 1e9);
    return 0;
}

template <int T, int U, int NT, int C> static int variant(Bufs& B, int wpc) {
    const unsigned grid = (unsigned)(B.cus * wpc);
    char tag[64];
    const double fr = (double)B.frames;
    snprintf(tag, sizeof tag, "T=%d U=%d NT=%d W=%d C=%d", T, U, NT, wpc, C);
    char nm[96];
    snprintf(nm, sizeof nm, "read   %s", tag);
    if (timeit(B, nm, 4.0 * fr, [&] { hipLaunchKernelGGL((k_read<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr, B.y, B.n4, B.sink); })) return 1;
    snprintf(nm, sizeof nm, "write  %s", tag);
    if (timeit(B, nm, 8.0 * fr, [&] { hipLaunchKernelGGL((k_write<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr, B.out, 2 * B.n4); })) return 1;
    snprintf(nm, sizeof nm, "copy   %s", tag);
    if (timeit(B, nm, 12.0 * fr, [&] { hipLaunchKernelGGL((k_copy<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr, B.y, B.n4, B.out); })) return 1;
    snprintf(nm, sizeof nm, "copy2  %s", tag);
    if (timeit(B, nm, 12.0 * fr, [&] { hipLaunchKernelGGL((k_copy2<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr, B.y, B.n4, 96, 128, B.out); })) return 1;
    return 0;
}

// the contiguous-store copies and the 1:1 copy
template <int T, int U, int NT, int C> static int variant2(Bufs& B, int wpc) {
    const unsigned grid = (unsigned)(B.cus * wpc);
    char tag[64];
    const double fr = (double)B.frames;
    snprintf(tag, sizeof tag, "T=%d U=%d NT=%d W=%d C=%d", T, U, NT, wpc, C);
    char nm[96];
    snprintf(nm, sizeof nm, "copyb  %s", tag);
    if (timeit(B, nm, 12.0 * fr, [&] { hipLaunchKernelGGL((k_copyb<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr,
                                                         reinterpret_cast<const float2*>(B.y), 2 * B.n4, B.out); })) return 1;
    snprintf(nm, sizeof nm, "copys  %s", tag);
    if (timeit(B, nm, 12.0 * fr, [&] { hipLaunchKernelGGL((k_copys<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr, B.y, B.n4, B.out); })) return 1;
    snprintf(nm, sizeof nm, "copy1  %s", tag);
    if (timeit(B, nm, 8.0 * fr, [&] { hipLaunchKernelGGL((k_copy1<T, U, NT, C>), dim3(grid), dim3(T), 0, nullptr, B.y, B.n4, B.out); })) return 1;
    return 0;
}

int main() {
    Bufs B;
    B.frames = 393216000;
    B.n4 = B.frames / 4;
    CHK(hipDeviceGetAttribute(&B.cus, hipDeviceAttributeMultiprocessorCount, 0));
    CHK(hipMalloc(&B.y, sizeof(float4) * B.n4));
    CHK(hipMalloc(&B.out, 2 * sizeof(float4) * B.n4));
    CHK(hipMalloc(&B.sink, sizeof(float) * 1024));
    CHK(hipMemset(B.y, 0, sizeof(float4) * B.n4));
    CHK(hipEventCreate(&B.a));
    CHK(hipEventCreate(&B.b));
    int rc = 0;
    rc |= variant2<256, 1, 0, 0>(B, 8);
    rc |= variant2<256, 4, 0, 0>(B, 8);
    rc |= variant2<256, 4, 1, 0>(B, 8);
    rc |= variant2<256, 4, 0, 1>(B, 8);
    rc |= variant2<1024, 4, 0, 0>(B, 2);
    rc |= variant2<1024, 4, 1, 0>(B, 1);
    rc |= variant<256, 1, 0, 0>(B, 8);     // the round-5 probe
    rc |= variant<256, 4, 0, 0>(B, 8);
    rc |= variant<256, 4, 1, 0>(B, 8);
    rc |= variant<256, 4, 2, 0>(B, 8);
    rc |= variant<256, 8, 1, 0>(B, 8);
    rc |= variant<256, 4, 1, 0>(B, 4);
    rc |= variant<512, 4, 1, 0>(B, 2);
    rc |= variant<1024, 4, 1, 0>(B, 1);
    rc |= variant<1024, 4, 1, 0>(B, 2);
    rc |= variant<256, 4, 1, 1>(B, 8);
    rc |= variant<1024, 4, 1, 1>(B, 2);
    rc |= variant<256, 4, 0, 1>(B, 8);
    CHK(hipFree(B.y));
    CHK(hipFree(B.out));
    CHK(hipFree(B.sink));
    return rc;
}
