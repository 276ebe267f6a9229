// k_digest.hip — translation unit of the per-render summary / digest (kernels_digest.h)
// and its host reference, which folds in the device's order (bit-identical results).
#include <cmath>
#include <cstring>
#include <vector>
#include "kernels_digest.h"
#include "launch.h"

static_assert(sizeof(DigestPart) == 48, "DigestPart is msg_digest_rec");

hipError_t launch_digest(int n, int n_tiles, hipStream_t s, const float* out, const int64_t* frame_off,
                         const int64_t* frames, const int32_t* tile_base, void* part, void* res) {
    if (n_tiles > 0) {
        hipLaunchKernelGGL(k_digest_tiles, dim3((unsigned)n_tiles), dim3(DG_T), 0, s, out, frame_off, frames, tile_base,
                           n, static_cast<DigestPart*>(part));
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_digest_presets, dim3((unsigned)n), dim3(DG_T), 0, s, static_cast<const DigestPart*>(part),
                       tile_base, static_cast<DigestPart*>(res));
    return hipGetLastError();
}

int64_t digest_tiles(int64_t frames) { return (frames + DG_TILE - 1) / DG_TILE; }

// the workgroup fold of kernels_digest.h on the host: 256 per-thread partials,
// xor-butterfly inside each wave of 64, then the waves in order
static DigestPart host_fold(std::vector<DigestPart>& th) {
    for (int o = 32; o >= 1; o >>= 1) {
        std::vector<DigestPart> nx(th);
        for (int i = 0; i < DG_T; ++i) {
            DigestPart a = th[i];
            dg_add(a, th[i ^ o]);
            nx[i] = a;
        }
        th.swap(nx);
    }
    DigestPart r = th[0];
    for (int w = 1; w < DG_T / 64; ++w) dg_add(r, th[w * 64]);
    return r;
}

void digest_host(const float* x, int64_t frames, void* rec) {
    const int64_t tiles = digest_tiles(frames);
    std::vector<DigestPart> part((size_t)tiles), th(DG_T);
    for (int64_t t = 0; t < tiles; ++t) {
        for (int i = 0; i < DG_T; ++i) {
            DigestPart a = dg_zero();
            for (int k = 0; k < DG_PER; ++k) {
                const int64_t f = t * DG_TILE + k * DG_T + i;
                if (f >= frames) continue;
                uint32_t wl, wr;
                std::memcpy(&wl, x + 2 * f, 4);
                std::memcpy(&wr, x + 2 * f + 1, 4);
                dg_frame(a, x[2 * f], x[2 * f + 1], wl, wr, f);
            }
            th[i] = a;
        }
        part[(size_t)t] = host_fold(th);
    }
    for (int i = 0; i < DG_T; ++i) {
        DigestPart a = dg_zero();
        for (int64_t t = i; t < tiles; t += DG_T) dg_add(a, part[(size_t)t]);
        th[i] = a;
    }
    const DigestPart r = host_fold(th);
    std::memcpy(rec, &r, sizeof(r));
}
