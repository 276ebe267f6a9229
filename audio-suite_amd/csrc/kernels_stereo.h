// kernels_stereo.h — stereo diffusion (MS:423-436), tanh saturation and peak
// normalisation (MS:26-34, 775-781) of the mono FIR output (TU: k_stereo.hip).
//
// Two passes over y per preset: the peak max(|L|, |R|) over every frame, then
// the clipped, normalised (L, R) pairs: k_stereo_max + k_stereo_out, two
// launches (the render path).  k_stereo_fused (MSGPU_STEREO_FUSED=1, an option)
// runs both in one persistent launch: workgroups take max-pass tiles in batch
// order from one counter and later run the output pass of the same tiles, once
// the tile's preset is complete (the last of its tiles to finish publishes the
// peak), so the output pass can re-read y from the XCD's L2 or the Infinity
// Cache -- 4 + 8 B of HBM per frame instead of 4 + 4 + 8.  Measured slower
// (C3 isolated stereo 1.79 vs 1.60 ms, C5 7.35 vs 5.59 ms per sub-batch, DESIGN
// §4): the chunk claims and the waits for a preset's last tile cost more than
// the re-read saves.
//
// The float64 FIR's error predictor (kernels_fir64.h) needs per preset sum y^2
// and sum (1 + (d y)^2)^-2: each tile stores its two partial sums, and the
// preset's last tile adds them in tile order (so the sums and the route decision
// do not depend on which tile finished last), decides the route (flag64) and
// marks flagged and odd-length presets deferred: their output tiles are written
// after the float64 FIR / the odd rotation by k_stereo_out_list.
#pragma once
#include "rt.h"

// ---------------------------------------------------------------------------
// Tiles
// ---------------------------------------------------------------------------
// A block handles ST_TILE frames [t0, t0+ST_TILE) of one preset; each thread
// owns runs of 4 consecutive frames.  The right-channel window
// y[(t0 + dr - 24 + u) mod n], u < ST_TILE + 48, is staged in LDS with
// coalesced loads; a run's 25-tap outputs then need 13 ds_read_b128 of the
// window instead of 100 scalar reads (the kernels were LDS-issue bound).
// L[t] = y[(t - dl) mod n] is staged the same way in k_stereo_out.
constexpr int ST_RUNS = ST_TILE / (4 * ST_T);     // runs of 4 frames per thread
static_assert(ST_TILE >= 4 * ST_T && ST_TILE % (4 * ST_T) == 0,
              "MSG_ST_TILE must be a multiple of 4 * ST_T (every frame of a tile has a run)");
static_assert((2 * ST_TILE + 48) * 4 <= 160 * 1024, "MSG_ST_TILE: stereo tile window exceeds the 160 KiB LDS of a CU");
constexpr int ST_WIN = ST_TILE + 48;

struct StereoTile {
    int t0, cnt;             // first frame, frames in this tile
    int lbase;               // (t0 - dl) mod n
};

MSG_DEV int mod_n(int64_t i, int64_t n) {
    i %= n;
    return (int)(i < 0 ? i + n : i);
}

// threadIdx.x behind an empty asm: the kernels that loop over tiles
// (k_stereo_fused, the list kernels) would otherwise keep every tile-invariant
// per-thread address (33 window slots, the runs' LDS and output offsets) live
// across the loop -- 175-188 VGPRs, or spills at 128; recomputed per tile they
// cost a few VALU and the loops fit k_stereo_out's register budget.
MSG_DEV int st_tid() {
    int t = (int)threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

MSG_DEV int st_rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Stage len floats y[(b0 + u) mod n] into w[0 .. len) with 16-byte loads
// (round 5 staged them with dword loads, 256 B per wave
// instruction): the aligned float4s covering y[b0, b0 + len)
// are loaded (all of them in flight before the first LDS store), then stored
// to LDS shifted back by the misalignment sh (uniform: the window's address
// mod 16).  Reads past either end stay inside the aligned 16-byte blocks
// holding the window's first and last samples (no other page).  A window that
// wraps past n (at most one per preset and pass) takes dword loads in the same
// register layout with sh = 0.
constexpr int ST_PER4 = (ST_WIN + 3 + 3) / 4 / ST_T + 1;   // float4s per thread, any shift
struct Win4 {
    float4 q[ST_PER4];
    int sh;
};
MSG_DEV void stereo_load4(const float* __restrict__ y, int n, int b0, int len, Win4& W) {
    const int tid = st_tid();
    if (b0 + len <= n) {
        const float* a = y + b0;
        W.sh = (int)((reinterpret_cast<uintptr_t>(a) >> 2) & 3);
        const float4* a4 = reinterpret_cast<const float4*>(a - W.sh);
        const int c4 = (len + W.sh + 3) >> 2;
#pragma unroll
        for (int i = 0; i < ST_PER4; ++i) {
            const int j = tid + i * ST_T;
            W.q[i] = j < c4 ? at32(a4, (uint32_t)j) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
        return;
    }
    W.sh = 0;
#pragma unroll
    for (int i = 0; i < ST_PER4; ++i) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int u = 4 * (tid + i * ST_T) + k;
            int j = b0 + u;
            if (n >= len) { if (j >= n) j -= n; }
            else j = (int)(((int64_t)b0 + u) % n);
            v[k] = u < len ? y[j] : 0.f;                  // j up to n: 64-bit addressing (n may pass 2^30)
        }
        W.q[i] = make_float4(v[0], v[1], v[2], v[3]);
    }
}
MSG_DEV void stereo_store4(int len, const Win4& W, float* w) {
    const int tid = st_tid();
    const int sh = st_rfl(W.sh);
#pragma unroll
    for (int i = 0; i < ST_PER4; ++i) {
        const int u0 = 4 * (tid + i * ST_T) - sh;
        if (sh == 0 && u0 + 4 <= len) {
            *reinterpret_cast<float4*>(w + u0) = W.q[i];
            continue;
        }
        const float v[4] = {W.q[i].x, W.q[i].y, W.q[i].z, W.q[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int u = u0 + k;
            if (u >= 0 && u < len) w[u] = v[k];
        }
    }
}

MSG_DEV StereoTile stereo_tile(const PresetRt& r, int64_t t0) {
    const int n = (int)r.out_n;
    StereoTile st;
    st.t0 = (int)t0;
    st.cnt = (int)(t0 + ST_TILE < n ? ST_TILE : n - t0);
    st.lbase = mod_n(t0 - r.dl, n);
    return st;
}

// R[u + k] = sum_m J_m w[u + k + 2m], k < 4, u a multiple of 4 (same fma order as the
// reference-checked scalar form: m = 0 .. 24); x receives w[u .. u + 52).
MSG_DEV void stereo_r4(const PresetRt& r, const float* w, int u, float (&R)[4], float (&x)[52]) {
    const float4* w4 = reinterpret_cast<const float4*>(w + u);
#pragma unroll
    for (int i = 0; i < 13; ++i) {
        const float4 q = w4[i];
        x[4 * i] = q.x; x[4 * i + 1] = q.y; x[4 * i + 2] = q.z; x[4 * i + 3] = q.w;
    }
    // outputs (u, u+1) and (u+2, u+3) as packed pairs: the pair (x[k+2m], x[k+1+2m])
    // is one aligned register pair, so each tap is one v_pk_fma per pair
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 a01 = f2{0.f, 0.f}, a23 = f2{0.f, 0.f};
#pragma unroll
    for (int m = 0; m < 25; ++m) {
        const f2 b = f2{r.bess[m], r.bess[m]};
        a01 = __builtin_elementwise_fma(b, f2{x[2 * m], x[2 * m + 1]}, a01);
        a23 = __builtin_elementwise_fma(b, f2{x[2 * m + 2], x[2 * m + 3]}, a23);
    }
    R[0] = a01.x; R[1] = a01.y; R[2] = a23.x; R[3] = a23.y;
}

// tanh from the hardware exp2 and reciprocal (two transcendentals instead of the
// library tanhf's ~30 instructions; k_stereo_out runs two per frame):
// 1 - 2 / (e^{2|x|} + 1), |error| <= ~2 float32 ulp of 1, and an odd Taylor
// polynomial below |x| = 0.05 where the subtraction would lose relative digits.
// MSG_TANH_TAYLOR = 0 (tuning only) drops the polynomial: the subtraction's
// ~1e-7 absolute error becomes a large relative one once the peak normalisation
// scales a quiet render (drive x peak << 1) back up, and test_feedback_imprint_chain
// fails (profiles/r03ab_stereo_ab.json).
#ifndef MSG_TANH_TAYLOR
#define MSG_TANH_TAYLOR 1
#endif
MSG_DEV float tanh_fast(float x) {
    const float ax = fabsf(x);
    const float e = __builtin_amdgcn_exp2f(fminf(2.8853900817779268f * ax, 126.f));   // e^{2|x|}
    float t = 1.0f - 2.0f * __builtin_amdgcn_rcpf(e + 1.0f);
#if MSG_TANH_TAYLOR
    const float x2 = ax * ax;
    if (ax < 0.05f) t = ax * fmaf(x2, fmaf(x2, 0.13333333f, -0.33333333f), 1.0f);
#endif
    return copysignf(t, x);
}
MSG_DEV float sat(float v, float d, float inv_td) { return d > 0.f ? tanh_fast(v * d) * inv_td : v; }
// tanh_fast of an (L, R) pair in the packed form: the arithmetic runs as
// v_pk_* pairs, the four transcendentals stay scalar (same operations and
// rounding as tanh_fast on each lane).
typedef float f2p __attribute__((ext_vector_type(2)));
MSG_DEV f2p tanh_fast2(f2p x) {
    const f2p ax = __builtin_elementwise_abs(x);
    const f2p a = __builtin_elementwise_min(2.8853900817779268f * ax, f2p{126.f, 126.f});
    const f2p e1 = f2p{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)} + 1.0f;
    const f2p r = f2p{__builtin_amdgcn_rcpf(e1.x), __builtin_amdgcn_rcpf(e1.y)};
    f2p t = 1.0f - 2.0f * r;
#if MSG_TANH_TAYLOR
    const f2p x2 = ax * ax;
    const f2p tp = ax * __builtin_elementwise_fma(x2, __builtin_elementwise_fma(x2, f2p{0.13333333f, 0.13333333f},
                                                                                f2p{-0.33333333f, -0.33333333f}),
                                                  f2p{1.0f, 1.0f});
    t.x = ax.x < 0.05f ? tp.x : t.x;
    t.y = ax.y < 0.05f ? tp.y : t.y;
#endif
    return __builtin_elementwise_copysign(t, x);
}

MSG_DEV int job_order_st() { return xcd_block(blockIdx.x, gridDim.x); }

constexpr int ST_EXIT = INT32_MIN;


// Cross-workgroup hand-off without agent-scope fences.  Every value another
// workgroup reads in this launch (tile peaks, partial sums, counters, the ready
// word) is written and read with agent-scope atomics, which gfx950 performs at
// the coherence point past the XCDs' L2s; what orders a producer's writes
// before its hand-off is this drain -- all of the wave's memory operations
// acknowledged (s_waitcnt 0; the signal fences keep the compiler from moving
// the atomics across it).  An agent-scope release / acquire fence would write
// back / invalidate the whole XCD L2 per tile (buffer_wbl2 / buffer_inv): the
// first build did so and ran C3's stereo pass in 486 ms instead of ~1.5.
MSG_DEV void st_drain() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// max|L|, |R| of one tile, returned to thread 0; with part, also the tile's
// sum y^2 and sum (1 + (d y)^2)^-2 into part[0], part[1] (the float64 FIR's
// error predictor, kernels_fir64.h).  Consecutive calls need no barrier
// between them (every read of w precedes the barrier before wm is read).
MSG_DEV float stereo_max_vals(const PresetRt& r, int tile, const float* __restrict__ ybuf,
                              const float* __restrict__ rbuf, double* __restrict__ part, bool with_r2, float* w,
                              float* wm) {
    const float* y = ybuf + r.y_off;
    const int n = (int)r.out_n;
    const StereoTile st = stereo_tile(r, (int64_t)tile * ST_TILE);
    const int tid = st_tid();
    // max|L| over all frames equals max|y| (L is a rotation of y).  With the
    // Bessel FIR, the centre tap of output u + k is y[(t0 + u + k + dr) mod n]:
    // over all tiles those cover every sample once, so max|y| comes from the
    // staged window; otherwise read y directly (16-byte aligned regions, t0 a
    // multiple of ST_TILE).
    const bool fir = r.stereo_fir == 1;
    float4 yv[ST_RUNS];
    if (fir) {
        Win4 wv;
        stereo_load4(y, n, mod_n((int64_t)st.t0 + r.dr - 24, n), ST_WIN, wv);
        stereo_store4(ST_WIN, wv, w);
    } else {
#pragma unroll
        for (int i = 0; i < ST_RUNS; ++i) {
            const int u = 4 * (tid + i * ST_T);
            if (u + 4 <= st.cnt) {
                yv[i] = *reinterpret_cast<const float4*>(y + st.t0 + u);
            } else {
                yv[i].x = u < st.cnt ? y[st.t0 + u] : 0.f;
                yv[i].y = u + 1 < st.cnt ? y[st.t0 + u + 1] : 0.f;
                yv[i].z = u + 2 < st.cnt ? y[st.t0 + u + 2] : 0.f;
                yv[i].w = 0.f;
            }
        }
    }
    __syncthreads();
    const float d = r.drive > 0.f ? r.drive : 0.f;
    float m = 0.f, s2 = 0.f, sq = 0.f;
    auto stat = [&](float v) {
        const float u = d * v;
        const float q = __builtin_amdgcn_rcpf(fmaf(u, u, 1.f));
        s2 = fmaf(v, v, s2);
        sq = fmaf(q, q, sq);
    };
#pragma unroll
    for (int i = 0; i < ST_RUNS; ++i) {
        const int u = 4 * (tid + i * ST_T);
        if (fir) {
            if (u < st.cnt) {
                float R[4], x[52];
                stereo_r4(r, w, u, R, x);
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (u + k < st.cnt) {
                        m = fmaxf(m, fmaxf(fabsf(R[k]), fabsf(x[k + 24])));
                        if (part) stat(x[k + 24]);
                    }
            }
            continue;
        }
        m = fmaxf(m, fmaxf(fmaxf(fabsf(yv[i].x), fabsf(yv[i].y)), fmaxf(fabsf(yv[i].z), fabsf(yv[i].w))));
        if (part) {
            if (u < st.cnt) stat(yv[i].x);
            if (u + 1 < st.cnt) stat(yv[i].y);
            if (u + 2 < st.cnt) stat(yv[i].z);
            if (u + 3 < st.cnt) stat(yv[i].w);
        }
        if (r.stereo_fir == 2 && with_r2) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (u + k < st.cnt) m = fmaxf(m, fabsf(rbuf[r.r2_off + st.t0 + u + k]));
        }
    }
    for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
    if (part)
        for (int off = 32; off > 0; off >>= 1) { s2 += __shfl_xor(s2, off); sq += __shfl_xor(sq, off); }
    if ((threadIdx.x & 63) == 0) {
        wm[threadIdx.x >> 6] = m;
        wm[ST_T / 64 + (threadIdx.x >> 6)] = s2;
        wm[2 * (ST_T / 64) + (threadIdx.x >> 6)] = sq;
    }
    __syncthreads();
    float v = 0.f;
    if (threadIdx.x == 0) {
        v = wm[0];
        for (int k = 1; k < ST_T / 64; ++k) v = fmaxf(v, wm[k]);
        if (part) {
            double a = 0.0, b = 0.0;
            for (int k = 0; k < ST_T / 64; ++k) { a += (double)wm[ST_T / 64 + k]; b += (double)wm[2 * (ST_T / 64) + k]; }
            __hip_atomic_store(part, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(part + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    return v;
}

// max|L|, |R| of one tile of preset p into maxbits[p] (and part as above)
MSG_DEV void stereo_max_tile(const PresetRt& r, int p, int tile, const float* __restrict__ ybuf,
                             const float* __restrict__ rbuf, unsigned* __restrict__ maxbits, double* __restrict__ part,
                             bool with_r2, float* w, float* wm) {
    const float v = stereo_max_vals(r, tile, ybuf, rbuf, part, with_r2, w, wm);
    if (threadIdx.x == 0) atomicMax(maxbits + p, __float_as_uint(v));
}

// After the max pass of `add` tiles of preset p (every thread; thread 0 holds
// their peak run_max and stored their partials): the peak into maxbits[p],
// then the tiles are counted; the workgroup that counts the preset's last tile
// adds the partial sums of tiles [tile0, tile0 + cnt) in tile order, decides the
// float64 route, resets the count and publishes the preset as ready.
// s_last / s_red: LDS.
MSG_DEV void stereo_run_done(const PresetRt& r, int p, int tile0, int cnt, int add, float run_max,
                             unsigned* __restrict__ maxbits, const StereoSync& sy, int* s_last, double* s_red) {
    if (threadIdx.x == 0) {
        atomicMax(maxbits + p, __float_as_uint(run_max));
        st_drain();                                        // the peak and partials before the count
        *s_last = atomicAdd(sy.done + p, add) + add == cnt;
    }
    __syncthreads();
    if (!*s_last) return;                                  // uniform
    const bool st = sy.part != nullptr && r.fir_on;
    double a = 0.0, b = 0.0;
    if (st) {
        for (int i = threadIdx.x; i < cnt; i += ST_T) {    // fixed order: tile i, i + ST_T, ...
            a += __hip_atomic_load(sy.part + 2 * (tile0 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b += __hip_atomic_load(sy.part + 2 * (tile0 + i) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        for (int off = 32; off > 0; off >>= 1) { a += __shfl_xor(a, off); b += __shfl_xor(b, off); }
        if ((threadIdx.x & 63) == 0) {
            s_red[threadIdx.x >> 6] = a;
            s_red[ST_T / 64 + (threadIdx.x >> 6)] = b;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        int f = 0;
        if (st) {
            a = s_red[0];
            b = s_red[ST_T / 64];
            for (int k = 1; k < ST_T / 64; ++k) { a += s_red[k]; b += s_red[ST_T / 64 + k]; }
            sy.stats[2 * p] = a;
            sy.stats[2 * p + 1] = b;
            const unsigned mb = __hip_atomic_load(maxbits + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            f = (sy.f64mode >= 2 || fir64_pred(r, a, b, mb) > FIR64_PRED) ? 1 : 0;
        }
        if (sy.flag64) sy.flag64[p] = f;
        __hip_atomic_store(sy.done + p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t defer = (f || r.stereo_fir == 2) ? 1u : 0u;
        st_drain();                                        // stats, flag64 and the reset first
        __hip_atomic_store(sy.ready + p, (sy.epoch << 1) | defer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

MSG_DEV int st_tiles_of(const int32_t* __restrict__ st_begin, int n_presets, int n_tiles, int p) {
    return (p + 1 < n_presets ? st_begin[p + 1] : n_tiles) - st_begin[p];
}

// The max pass of the two-launch path: each tile's peak into maxbits[p] (a
// non-returning atomic) and, for the float64 FIR's predictor, its two partial
// sums into part[2 b] -- no count of finished tiles: round 5 ended every tile
// with stereo_run_done's drain and returning atomic (the last tile of a preset
// summed the partials), a memory round trip per 4096 frames the workgroup
// waited out; k_stereo_pred now does that per preset after the launch.
__global__ void __launch_bounds__(ST_T)
k_stereo_max(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_begin, int n_presets, int n_tiles,
             const float* __restrict__ ybuf, unsigned* __restrict__ maxbits, StereoSync sy) {
    __shared__ __attribute__((aligned(16))) float w[ST_WIN];
    __shared__ float wm[3 * (ST_T / 64)];
    const int b = job_order_st();
    const int p = find_preset(st_begin, n_presets, b);
    const PresetRt& r = rt[p];
    const float m = stereo_max_vals(r, b - st_begin[p], ybuf, nullptr,
                                    (sy.part && r.fir_on) ? sy.part + 2 * b : nullptr, false, w, wm);
    if (threadIdx.x == 0) atomicMax(maxbits + p, __float_as_uint(m));
    (void)n_tiles;
}

// Per preset, after k_stereo_max (sy.part set: the float64 FIR is on): the
// tiles' partial sums added in tile order -- thread i takes tiles i, i + ST_T,
// ..., then the waves' butterflies and the waves in order, the arithmetic of
// stereo_run_done's last tile, so the sums and the route are the same bits --
// then the predictor and flag64 (0 for a preset without a filter).
__global__ void __launch_bounds__(ST_T)
k_stereo_pred(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_begin, int n_presets, int n_tiles,
              const unsigned* __restrict__ maxbits, StereoSync sy) {
    __shared__ double s_red[2 * (ST_T / 64)];
    const int p = blockIdx.x;
    const PresetRt& r = rt[p];
    if (!r.fir_on) {
        if (threadIdx.x == 0) sy.flag64[p] = 0;
        return;
    }
    const int tile0 = st_begin[p], cnt = st_tiles_of(st_begin, n_presets, n_tiles, p);
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < cnt; i += ST_T) {
        a += __hip_atomic_load(sy.part + 2 * (tile0 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        b += __hip_atomic_load(sy.part + 2 * (tile0 + i) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int off = 32; off > 0; off >>= 1) { a += __shfl_xor(a, off); b += __shfl_xor(b, off); }
    if ((threadIdx.x & 63) == 0) {
        s_red[threadIdx.x >> 6] = a;
        s_red[ST_T / 64 + (threadIdx.x >> 6)] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = s_red[0];
        b = s_red[ST_T / 64];
        for (int k = 1; k < ST_T / 64; ++k) { a += s_red[k]; b += s_red[ST_T / 64 + k]; }
        sy.stats[2 * p] = a;
        sy.stats[2 * p + 1] = b;
        sy.flag64[p] = (sy.f64mode >= 2 || fir64_pred(r, a, b, maxbits[p]) > FIR64_PRED) ? 1 : 0;
    }
}

// The float64 FIR's presets again (kernels_fir64.h) and the odd-length presets
// (R from the rotation): their peak from the final y and R.
__global__ void __launch_bounds__(ST_T) __attribute__((amdgpu_waves_per_eu(4)))
k_stereo_remax(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_count,
               const int32_t* __restrict__ slot_preset, const int32_t* __restrict__ n_slots, int tmax,
               const float* __restrict__ ybuf, const float* __restrict__ rbuf, unsigned* __restrict__ maxbits) {
    __shared__ __attribute__((aligned(16))) float w[ST_WIN];
    __shared__ float wm[3 * (ST_T / 64)];
    const int ns = *n_slots;
    for (int64_t j = blockIdx.x; j < (int64_t)ns * tmax; j += gridDim.x) {   // 64-bit: ns * tmax can pass 2^31
        const int sl = (int)(j / tmax), t = (int)(j - (int64_t)sl * tmax);
        const int p = st_rfl(slot_preset[sl]);
        if (t >= st_count[p]) continue;                          // uniform
        __syncthreads();
        stereo_max_tile(rt[p], p, t, ybuf, rbuf, maxbits, nullptr, true, w, wm);
    }
}

// The clipped, normalised (L, R) of one tile of preset p, peak M = the float
// bits peak_bits (sm: LDS of ST_SM floats -- the L window, then the R window;
// after the arithmetic, the tile's (L, R) pairs).  (L straight into registers
// -- 16.6 KB of LDS per workgroup instead of 33 -- measured 1.64 vs 1.60 ms
// isolated on C3: the pass is not limited by its workgroups per CU.)
// Round 6: the windows come in with 16-byte loads (stereo_load4), and the
// output leaves through LDS so that every store instruction writes 1 KB of
// consecutive frames (two frames per lane); a thread's own runs of four frames
// would store 32 B per lane at a 32-byte stride, leaving every line
// half-written by each instruction (the streaming probe: 4.8 TB/s for that
// shape against 5.2 - 5.3 for contiguous stores, profiles/r06c_stream_rates.txt).
constexpr int ST_SM = ST_TILE + ST_WIN;
static_assert(ST_SM >= 2 * ST_TILE, "the (L, R) staging reuses both windows");
#ifndef MSG_ST_NT
#define MSG_ST_NT 0                 // nontemporal output stores (tuning builds)
#endif
MSG_DEV void stereo_out_tile(const PresetRt& r, int tile, const float* __restrict__ ybuf, const float* __restrict__ rbuf,
                             unsigned peak_bits, float* __restrict__ out, float* sm) {
    float* lw = sm;
    float* w = sm + ST_TILE;
    const float* y = ybuf + r.y_off;
    const int n = (int)r.out_n;
    const StereoTile st = stereo_tile(r, (int64_t)tile * ST_TILE);
    const int tid = st_tid();
    {
        Win4 lv, wv;
        stereo_load4(y, n, r.stereo_fir ? st.lbase : st.t0, st.cnt, lv);
        if (r.stereo_fir == 1) stereo_load4(y, n, mod_n((int64_t)st.t0 + r.dr - 24, n), ST_WIN, wv);
        stereo_store4(st.cnt, lv, lw);
        if (r.stereo_fir == 1) stereo_store4(ST_WIN, wv, w);
    }
    const float d = r.drive;
    const float inv_td = d > 0.f ? 1.0f / tanh_fast(d) : 1.f;
    const float M = __uint_as_float(peak_bits);
    const float mc = sat(M, d, inv_td);
    const float scale = mc > 0.f ? r.peak / mc : 1.f;
    const float k_out = inv_td * scale;                     // one multiply per channel after the tanh
    __syncthreads();
    float4 res[ST_RUNS][2];                                 // (L, R) of frames u .. u + 3 per run
#pragma unroll
    for (int i = 0; i < ST_RUNS; ++i) {
        const int u = 4 * (tid + i * ST_T);
        if (u >= st.cnt) continue;
        const float4 l4 = *reinterpret_cast<const float4*>(lw + u);
        const float L[4] = {l4.x, l4.y, l4.z, l4.w};
        float R[4];
        if (r.stereo_fir == 1) {
            float x[52];
            stereo_r4(r, w, u, R, x);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                R[k] = r.stereo_fir == 2 ? (u + k < st.cnt ? rbuf[r.r2_off + st.t0 + u + k] : 0.f) : L[k];
        }
        float2 v[4];
        if (d > 0.f) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const f2p t = tanh_fast2(f2p{L[k], R[k]} * d) * k_out;
                v[k] = make_float2(t.x, t.y);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = make_float2(L[k] * scale, R[k] * scale);
        }
        res[i][0] = make_float4(v[0].x, v[0].y, v[1].x, v[1].y);
        res[i][1] = make_float4(v[2].x, v[2].y, v[3].x, v[3].y);
    }
    __syncthreads();                                        // every window read done: sm takes the pairs
#pragma unroll
    for (int i = 0; i < ST_RUNS; ++i) {
        const int u = 4 * (tid + i * ST_T);
        if (u >= st.cnt) continue;
        float4* o = reinterpret_cast<float4*>(sm + 2 * u);
        o[0] = res[i][0];
        o[1] = res[i][1];
    }
    __syncthreads();
    // frame pairs aligned to the output: pair j holds local frames 2 j - a, 2 j - a + 1
    const int a = (int)((r.out_off + st.t0) & 1);
    float* ob = out + 2 * (r.out_off + st.t0 - a);          // 16-byte aligned
    const int pairs = (st.cnt + a + 1) >> 1;
#pragma unroll
    for (int i = 0; i < (ST_TILE / 2 + 1 + ST_T - 1) / ST_T; ++i) {
        const int j = tid + i * ST_T;
        if (j >= pairs) break;
        const int f0 = 2 * j - a;
        if (f0 >= 0 && f0 + 1 < st.cnt) {
            // a == 0 (even output offsets: every C3 / C4 / C5 preset): the pair is one
            // aligned 16-byte read (two 8-byte reads at a 16-byte lane stride hit each
            // bank twice per 32-lane group)
            float4 pp;
            if (a == 0) {
                pp = *reinterpret_cast<const float4*>(sm + 2 * f0);
            } else {
                const float2 p0 = *reinterpret_cast<const float2*>(sm + 2 * f0);
                const float2 p1 = *reinterpret_cast<const float2*>(sm + 2 * f0 + 2);
                pp = make_float4(p0.x, p0.y, p1.x, p1.y);
            }
            float* dst = ob + 4 * (uint32_t)j;
#if MSG_ST_NT
            typedef float v4f __attribute__((ext_vector_type(4)));
            __builtin_nontemporal_store(v4f{pp.x, pp.y, pp.z, pp.w}, reinterpret_cast<v4f*>(dst));
#else
            *reinterpret_cast<float4*>(dst) = pp;
#endif
        } else {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int f = f0 + k;
                if (f >= 0 && f < st.cnt)
                    *reinterpret_cast<float2*>(ob + 4 * (uint32_t)j + 2 * k) = *reinterpret_cast<const float2*>(sm + 2 * f);
            }
        }
    }
}

__global__ void __launch_bounds__(ST_T)
k_stereo_out(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_begin, int n_presets,
             const float* __restrict__ ybuf, const float* __restrict__ rbuf, const unsigned* __restrict__ maxbits,
             float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float sm[ST_SM];
    const int b = job_order_st();
    const int p = find_preset(st_begin, n_presets, b);
    stereo_out_tile(rt[p], b - st_begin[p], ybuf, rbuf, maxbits[p], out, sm);
}

// The output tiles of the listed presets (the deferred ones of k_stereo_fused:
// float64 FIR slots, odd lengths), a grid-stride walk over (entry, tile).
__global__ void __launch_bounds__(ST_T) __attribute__((amdgpu_waves_per_eu(4)))
k_stereo_out_list(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_count,
                  const int32_t* __restrict__ list, const int32_t* __restrict__ n_list, int tmax,
                  const float* __restrict__ ybuf, const float* __restrict__ rbuf, const unsigned* __restrict__ maxbits,
                  float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float sm[ST_SM];
    const int nl = *n_list;
    for (int64_t j = blockIdx.x; j < (int64_t)nl * tmax; j += gridDim.x) {
        const int sl = (int)(j / tmax), t = (int)(j - (int64_t)sl * tmax);
        const int p = st_rfl(list[sl]);
        if (t >= st_count[p]) continue;                          // uniform
        __syncthreads();                                         // the previous tile's LDS reads are done
        stereo_out_tile(rt[p], t, ybuf, rbuf, maxbits[p], out, sm);
    }
}

// Both passes in one persistent launch (see the header).  Jobs are chunks of
// ST_CHUNK consecutive tiles of the batch (a chunk may span short presets): one
// claim, one preset lookup and one count per preset run amortised over the
// chunk (each returning atomic costs ~1 us while the chip streams,
// MI355X_MICROARCH.md "dequeue"; per-tile jobs ran C3's pass at 3.4 ms).  A
// workgroup owns the output pass of the chunks whose max pass it ran: wave 0
// keeps them in a ring in LDS and picks the next job -- the oldest owned chunk
// if the presets of its first and last tiles are ready, else the next chunk
// from the launch's one counter, else (every chunk taken, or the ring full)
// the oldest owned chunk, waiting for its presets.  The output pass then
// re-reads y on the CU that just read it (its XCD's L2, else the Infinity
// Cache).
// Waiting cannot deadlock once every chunk is taken: each is held by a running
// workgroup that finishes its max pass without waiting.  With the ring full,
// all W resident workgroups could only wait together if the preset at the front
// had 32 W ST_CHUNK claimed tiles; the host takes this launch only for presets
// of at most ST_FUSED_MAX_TILES = 2048 tiles (C5's 8.4 M frames), so even eight
// contexts' fused launches sharing the CUs (W >= 1024 / 8 each) cannot all
// stall.  The last workgroup to leave resets the counters.
constexpr int ST_RING = 32;
#ifndef MSG_ST_CHUNK
#define MSG_ST_CHUNK 4
#endif
constexpr int ST_CHUNK = MSG_ST_CHUNK;
constexpr int ST_LDS_PRESETS = 1024;    // st_begin staged in LDS up to this many presets

MSG_DEV uint32_t st_poll(const uint32_t* ready, int p) {
    return __hip_atomic_load(ready + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(ST_T) __attribute__((amdgpu_waves_per_eu(4)))
k_stereo_fused(const PresetRt* __restrict__ rt, const int32_t* __restrict__ st_begin, int n_presets, int n_tiles,
               const float* __restrict__ ybuf, unsigned* __restrict__ maxbits, StereoSync sy,
               int32_t* __restrict__ ctr, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float sm[ST_SM];
    float* w = sm + ST_TILE;                                    // the max pass's window
    __shared__ float wm[3 * (ST_T / 64)];
    __shared__ double s_red[2 * (ST_T / 64)];
    __shared__ int32_t s_begin[ST_LDS_PRESETS];
    __shared__ int s_ring[ST_RING];
    __shared__ int s_job, s_last, s_skip;
    __shared__ unsigned s_peak;
    const int lane = (int)(threadIdx.x & 63);
    const bool lds_begin = n_presets <= ST_LDS_PRESETS;
    if (lds_begin)
        for (int i = threadIdx.x; i < n_presets; i += ST_T) s_begin[i] = st_begin[i];
    const int32_t* beg = lds_begin ? s_begin : st_begin;
    const int n_chunks = (n_tiles + ST_CHUNK - 1) / ST_CHUNK;
    int head = 0, cnt = 0;                                          // wave 0's ring state (uniform)
    bool a_done = false;
    __syncthreads();
    for (;;) {
        if (threadIdx.x < 64) {
            int job = ST_EXIT;
            bool out_now = false;
            if (cnt > 0) {
                const int c = s_ring[head];
                const int p0 = find_preset(beg, n_presets, c * ST_CHUNK);
                const int p1 = find_preset(beg, n_presets, min(n_tiles, c * ST_CHUNK + ST_CHUNK) - 1);
                uint32_t r0 = 0, r1 = 0;
                if (lane == 0) {
                    r0 = st_poll(sy.ready, p0);
                    r1 = p1 == p0 ? r0 : st_poll(sy.ready, p1);
                }
                out_now = ((uint32_t)st_rfl((int)r0) >> 1) == sy.epoch && ((uint32_t)st_rfl((int)r1) >> 1) == sy.epoch;
                out_now = out_now || cnt == ST_RING;
            }
            if (!out_now && !a_done) {
                const int c = st_rfl(lane == 0 ? atomicAdd(ctr + ST_CTR_A, 1) : 0);
                if (c < n_chunks) {
                    job = c;
                    if (lane == 0) s_ring[(head + cnt) & (ST_RING - 1)] = c;
                    ++cnt;
                } else {
                    a_done = true;
                }
            }
            if (job == ST_EXIT && cnt > 0) {                        // output pass of the oldest owned chunk
                job = -2 - s_ring[head];
                head = (head + 1) & (ST_RING - 1);
                --cnt;
            }
            if (lane == 0) s_job = job;
        }
        __syncthreads();
        const int job = st_rfl(s_job);                              // uniform: scalar registers
        if (job == ST_EXIT) break;
        const int c = job >= 0 ? job : -2 - job;
        const int c1 = min(n_tiles, c * ST_CHUNK + ST_CHUNK);
        for (int t = c * ST_CHUNK; t < c1;) {                       // one run per preset the chunk touches
            const int p = st_rfl(find_preset(beg, n_presets, t));
            const PresetRt& r = rt[p];
            const int tb = beg[p];
            const int tcnt = st_tiles_of(beg, n_presets, n_tiles, p);
            const int te = min(c1, tb + tcnt);
            if (job >= 0) {                                         // max pass
                float m = 0.f;
                for (int u = t; u < te; ++u)
                    m = fmaxf(m, stereo_max_vals(r, u - tb, ybuf, nullptr,
                                                 (sy.part && r.fir_on) ? sy.part + 2 * u : nullptr, false, w, wm));
                stereo_run_done(r, p, tb, tcnt, te - t, m, maxbits, sy, &s_last, s_red);
            } else {                                                // output pass
                if (threadIdx.x == 0) {
                    uint32_t rd;
                    while (((rd = st_poll(sy.ready, p)) >> 1) != sy.epoch) __builtin_amdgcn_s_sleep(4);
                    s_skip = (int)(rd & 1u);
                    s_peak = __hip_atomic_load(maxbits + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __syncthreads();
                if (!st_rfl(s_skip)) {
                    const unsigned peak = (unsigned)st_rfl((int)s_peak);
                    for (int u = t; u < te; ++u) {
                        stereo_out_tile(r, u - tb, ybuf, nullptr, peak, out, sm);
                        __syncthreads();                            // LDS windows free for the next tile
                    }
                }
            }
            __syncthreads();                                        // s_last / s_skip / s_peak free
            t = te;
        }
    }
    if (threadIdx.x == 0 && atomicAdd(ctr + ST_CTR_E, 1) == (int)gridDim.x - 1) {
        __hip_atomic_store(ctr + ST_CTR_A, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctr + ST_CTR_E, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
