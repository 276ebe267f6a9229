// k_digest.hip — translation unit of the per-render summary / digest (kernels_digest.h)
// and the entry to its host reference (digest.h), which folds in the device's
// order (bit-identical results).
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

int64_t digest_tiles(int64_t frames) { return dg_tiles(frames); }

void digest_host(const float* x, int64_t frames, void* rec) {
    DigestPart r;
    dg_host(x, frames, &r);
    std::memcpy(rec, &r, sizeof(r));
}
