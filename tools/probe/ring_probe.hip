// Probe: ring_sincos (kernels_core.h) and the two-level rotation of the
// resonant strike against float64, j in [0, n) at f / sr = 4200 / sr.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../audio-suite_amd/csrc/kernels_core.h"

__global__ void k_probe(int n, float fa, float fb, float* out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const float2 sc = ring_sincos((float)j, fa, fb);
    const int B = j & ~63, t = j - B;
    const float2 sb = ring_sincos((float)B, fa, fb), st = ring_sincos((float)t, fa, fb);
    out[4 * j] = sc.x;
    out[4 * j + 1] = sc.y;
    out[4 * j + 2] = fmaf(sb.x, st.y, sb.y * st.x);
    out[4 * j + 3] = sinpif(2.0f * ring_phase((float)j, fa, fb));
}

int main() {
    const int n = 40000;
    float* d;
    if (hipMalloc(&d, sizeof(float) * 4 * n) != hipSuccess) return 1;
    std::vector<float> h(4 * n);
    for (double sr : {1.2e6, 3.0e7, 48000.0}) {
        const double fos = 4200.0 / sr;
        const float fa = (float)fos, fb = (float)(fos - (double)fa);
        k_probe<<<(n + 255) / 256, 256>>>(n, fa, fb, d);
        if (hipMemcpy(h.data(), d, sizeof(float) * 4 * n, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        double e[4] = {0, 0, 0, 0}, m[4] = {0, 0, 0, 0};
        for (int j = 0; j < n; ++j) {
            const double ph = 2.0 * M_PI * fmod((double)j * fos, 1.0);
            const double ref[4] = {sin(ph), cos(ph), sin(ph), sin(ph)};
            for (int k = 0; k < 4; ++k) {
                const double x = fabs((double)h[4 * j + k] - ref[k]);
                e[k] += x * x;
                if (x > m[k]) m[k] = x;
            }
        }
        printf("sr %.0f: rms/max err  sin %.2e/%.2e  cos %.2e/%.2e  rot %.2e/%.2e  phase+sinpi %.2e/%.2e\n", sr,
               sqrt(e[0] / n), m[0], sqrt(e[1] / n), m[1], sqrt(e[2] / n), m[2], sqrt(e[3] / n), m[3]);
    }
    (void)hipFree(d);
    return 0;
}
