// host_san.cpp — host-only build of libmsgpu's host entry points for the
// sanitizers (SURVEY §5 "race detection / sanitizers"): the render plan
// (plan.h, msg_plan_host), the NumPy stream primitives (nprng.h, msg_rng_*) and
// the render digest's host reference (digest.h, msg_digest_host)
// compiled by g++ with -fsanitize=address,undefined into
// msgpu/libmsgpu_hostsan.so.  The device entry points are stubs that fail with
// MSG_E_DEVICE, so the ctypes binding (_lib.py) loads this library unchanged
// and tests/test_plan_host.py / tests/test_rng_host.py run against it
// (tests/test_host_sanitizers.py).  Never the product library.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>

#include "msg_common.h"
#include "ziggurat_tables.h"
#include "nprng.h"
#include "plan.h"
#include "host_pool.h"
#include "digest.h"
#include "../../include/msgpu.h"

namespace {
const nprng::Zig kHostZig = {zig_ki_double, zig_wi_double, zig_fi_double,
                             zig_ke_double, zig_we_double, zig_fe_double};
thread_local std::string g_err;
int fail(msg_ctx*, int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int no_device() { return fail(nullptr, MSG_E_DEVICE, "host sanitizer build: no device entry points"); }
}  // namespace

extern "C" {
int msg_abi_version(void) { return MSG_ABI_VERSION; }
int msg_host_threads(void) { return HostPool::get().threads(); }
int64_t msg_sizeof(int32_t which) {
    switch (which) {
        case 0: return (int64_t)sizeof(msg_preset);
        case 1: return (int64_t)sizeof(msg_event);
        case 2: return (int64_t)sizeof(msg_plan_info);
        case 3: return (int64_t)sizeof(msg_digest_rec);
        default: return -1;
    }
}
const char* msg_last_error(msg_ctx*) { return g_err.c_str(); }
msg_ctx* msg_create(int) { no_device(); return nullptr; }
void msg_destroy(msg_ctx*) {}
int msg_render_batch(msg_ctx*, const msg_preset*, int32_t, const double*, int64_t, const double* const*,
                     const int64_t*, int32_t,
                     const uint8_t* const*, const int32_t*, const int32_t*, int32_t, float*, const int64_t*, void*) {
    return no_device();
}
int msg_last_plan(msg_ctx*, msg_plan_info*, int32_t) { return no_device(); }
int msg_last_events(msg_ctx*, int32_t, msg_event*, int32_t, int32_t*) { return no_device(); }
int msg_last_meta(msg_ctx*, int32_t, double*, double*, int64_t, int64_t*) { return no_device(); }
int msg_last_grain64(msg_ctx*, int32_t, int32_t, double*, int64_t, int64_t*) { return no_device(); }
int msg_set_profiling(msg_ctx*, int32_t) { return no_device(); }
int msg_stage_times(msg_ctx*, float*, int32_t) { return no_device(); }
int msg_gate(msg_ctx*, msg_ctx*, int32_t, int32_t) { return no_device(); }
int msg_bench_fft(msg_ctx*, int32_t, int32_t, int32_t, float*) { return no_device(); }
int msg_fft64(msg_ctx*, int32_t, int32_t, const double*, double*) { return no_device(); }
int msg_fir(msg_ctx*, const float*, float*, int64_t, int32_t, const double*, int64_t, int32_t*, void*) {
    return no_device();
}
int msg_stft_mag_db(msg_ctx*, const void*, int32_t, int64_t, int32_t, int32_t, int32_t, int32_t, double*, int32_t*,
                    void*) {
    return no_device();
}
int msg_digest(msg_ctx*, const float*, const int64_t*, const int64_t*, int32_t, msg_digest_rec*, void*) {
    return no_device();
}
// the digest's host reference (digest.h), the same code the product library runs
int msg_digest_host(const float* x, int64_t out_n, msg_digest_rec* rec) {
    if (!rec || out_n < 0 || (out_n > 0 && !x)) return fail(nullptr, MSG_E_ARG, "bad arguments");
    static_assert(sizeof(DigestPart) == sizeof(msg_digest_rec), "DigestPart is msg_digest_rec");
    DigestPart r;
    dg_host(x, out_n, &r);
    std::memcpy(rec, &r, sizeof(r));
    return MSG_OK;
}
#include "host_abi.inc"
}  // extern "C"
