// msgpu.hip — libmsgpu: host orchestration and the C ABI (include/msgpu.h).
//
// One msg_render_batch call renders N independent presets (each one call of
// the reference's render(), microsound_0.2.1/main_v2.py:588-792) on one
// MI355X: device planner -> generator -> LDS spectral chain -> overlap-add x
// ADSR -> partitioned FFT FIR (ER + IR) -> stereo/tanh/normalise.  All work is
// batched across presets so every launch has thousands of workgroups.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <sched.h>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "msg_common.h"
#include "ziggurat_tables.h"
#include "nprng.h"
#include "plan.h"
#include "fftplan.h"
#include "fft_lds.h"
#include "kernels_core.h"
#include "launch.h"
#include "host_pool.h"
#include "tap_sort.h"
#ifndef MSG_TAP_RADIX
#define MSG_TAP_RADIX 1   // tuning A/B: 0 = std::sort of the tap keys
#endif
#include "../../include/msgpu.h"

namespace {

const nprng::Zig kHostZig = {zig_ki_double, zig_wi_double, zig_fi_double,
                             zig_ke_double, zig_we_double, zig_fe_double};


thread_local std::string g_err;   // errors before a context exists
std::mutex g_gate_mu;              // msg_gate links between contexts

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;   // elements
    hipError_t ensure(size_t n) {
        if (n <= cap && p) return hipSuccess;
        if (p) { hipFree(p); p = nullptr; cap = 0; }
        size_t want = std::max<size_t>(n, 1);
        want = want + want / 4;
        hipError_t e = hipMalloc(&p, want * sizeof(T));
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() { if (p) hipFree(p); p = nullptr; cap = 0; }
};

// ensure() that leaves a new allocation zeroed (counters and flags the kernels reset themselves)
template <class T>
static hipError_t ensure_zeroed(DevBuf<T>& b, size_t n, hipStream_t s) {
    if (n <= b.cap && b.p) return hipSuccess;
    hipError_t e = b.ensure(n);
    if (e != hipSuccess) return e;
    return hipMemsetAsync(b.p, 0, b.cap * sizeof(T), s);
}

// Pinned staging for a batch's host -> device uploads.  Every per-batch input
// (presets, events, runtime records, job lists, IR bank ...) is packed into one
// pinned slot and moved by ONE copy into a device arena; each input's device
// pointer is then set to its place in the arena.  (One copy per input cost ~35
// copy-engine blits per batch, ~2 ms of GPU time per C3 sub-batch.)  Two pinned
// slots alternate between batches; a slot is refilled only after the copy that
// read it (two batches back) has run, so msg_render_batch never waits on the
// render stream.  The arena itself is reused in stream order.
struct Staging {
    struct Item { void** slot; const void* src; size_t bytes; };
    struct Slot { char* host = nullptr; size_t cap = 0; hipEvent_t done = nullptr; bool armed = false; };
    Slot slot[2];
    int cur = 0;
    char* arena = nullptr;
    size_t arena_cap = 0;
    std::vector<Item> items;
    template <class T> void add(T** dst, const T* src, size_t bytes) {
        items.push_back(Item{reinterpret_cast<void**>(dst), src, bytes});
    }
    hipError_t flush(hipStream_t s) {
        Slot& sl = slot[cur];
        hipError_t e = hipSuccess;
        if (!sl.done) e = hipEventCreateWithFlags(&sl.done, hipEventDisableTiming);
        if (e == hipSuccess && sl.armed) e = hipEventSynchronize(sl.done);
        std::vector<size_t> at(items.size());
        size_t total = 0;
        for (size_t i = 0; i < items.size(); ++i) {
            at[i] = total;
            total += (items[i].bytes + 255) & ~size_t(255);
        }
        total = std::max<size_t>(total, 256);
        if (e == hipSuccess && total > sl.cap) {
            if (sl.host) hipHostFree(sl.host);
            sl.host = nullptr;
            sl.cap = 0;
            const size_t want = total + total / 4 + 4096;
            e = hipHostMalloc((void**)&sl.host, want, hipHostMallocDefault);
            if (e == hipSuccess) sl.cap = want;
        }
        if (e == hipSuccess && total > arena_cap) {     // growth frees the old arena (hipFree waits)
            if (arena) hipFree(arena);
            arena = nullptr;
            arena_cap = 0;
            const size_t want = total + total / 4 + 4096;
            e = hipMalloc((void**)&arena, want);
            if (e == hipSuccess) arena_cap = want;
        }
        if (e == hipSuccess) {   // pack in 1 MiB pieces on the host pool (C5: ~100 MB per sub-batch)
            constexpr size_t PIECE = size_t(1) << 20;
            std::vector<std::pair<size_t, size_t>> pieces;   // (item, byte offset in item)
            for (size_t i = 0; i < items.size(); ++i)
                for (size_t b = 0; b < items[i].bytes; b += PIECE) pieces.emplace_back(i, b);
            HostPool::get().run((int)pieces.size(), [&](int k) {
                const Item& it = items[pieces[k].first];
                const size_t b = pieces[k].second;
                std::memcpy(sl.host + at[pieces[k].first] + b, (const char*)it.src + b, std::min(PIECE, it.bytes - b));
            });
            size_t used = 0;
            for (size_t i = 0; i < items.size(); ++i) used = at[i] + items[i].bytes;
            if (used) e = hipMemcpyAsync(arena, sl.host, used, hipMemcpyHostToDevice, s);
        }
        for (size_t i = 0; i < items.size(); ++i) *items[i].slot = e == hipSuccess ? arena + at[i] : nullptr;
        if (e == hipSuccess) e = hipEventRecord(sl.done, s);
        sl.armed = e == hipSuccess;
        items.clear();
        cur ^= 1;
        return e;
    }
    void release() {
        for (Slot& sl : slot) {
            if (sl.done) { hipEventSynchronize(sl.done); hipEventDestroy(sl.done); }
            if (sl.host) hipHostFree(sl.host);
            sl = Slot();
        }
        if (arena) hipFree(arena);
        arena = nullptr;
        arena_cap = 0;
    }
};

// A per-batch input living in the Staging arena (set at each flush).
template <class T> struct Slice { T* p = nullptr; };

template <class P>
struct PlanStoreT {
    std::vector<P> host;                 // descriptors (device pointers inside)
    std::vector<void*> allocs;
    std::map<int, int> by_n;
    bool dirty = false;
    DevBuf<P> dev;
};
using PlanStore = PlanStoreT<RealPlan>;
using Plan64Store = PlanStoreT<Real64Plan>;

}  // namespace

struct msg_ctx {
    int device = 0;
    std::string err;
    bool profiling = false;
    // msg_gate: this context's stream waits, before stage gate_wait, for the
    // peer's gate event, and records its own after stage gate_rec begins
    // (gate_peer / gated_by change under g_gate_mu: msg_gate, msg_destroy)
    msg_ctx* gate_peer = nullptr;
    std::vector<msg_ctx*> gated_by;   // contexts whose gate_peer is this one (cleared at msg_destroy)
    int gate_wait = -1, gate_rec = -1;
    hipEvent_t gate_ev = nullptr;
    std::atomic<bool> gate_armed{false};   // gate_ev recorded at least once (read by the gated context)
    // the stream of the last batch and an event at its end: a batch enqueued on
    // another stream first waits for it (the staging arena and the per-batch
    // buffers are reused in stream order only)
    hipStream_t last_stream = nullptr;
    hipEvent_t done_ev = nullptr;
    bool done_armed = false;
    // stage events: two sets alternate between batches; a set is read (folded
    // into the sums) when it comes round again, two batches later, or at
    // msg_stage_times -- profiling never makes the host wait for the last batch
    bool pending[2] = {false, false};
    bool pending_fir[2] = {false, false};
    bool pending_h_early[2] = {false, false};
    int ev_cur = 0;
    // msg_set_profiling(ctx, k): batches 0, k, 2k, ... of the context record the
    // stage events and host clocks (k = 1: every batch).  Each profiled batch
    // adds 12 timed events to its stream and a host read of the set two batches
    // back (bench.py samples every 4th batch)
    int prof_every = 1;
    int64_t prof_n = 0;
    bool prof_batch = false;      // this batch records (profiling && its turn)
    double stage_sum[10] = {0};   // accumulated stage times since msg_set_profiling(ctx, 1)
    int64_t stage_cnt = 0;
    // host wall clock per batch: plan, records, pinned upload, then the splits
    // plan sizes, plan events + tap merge, preset records, event records, lists + buffers
    double host_sum[8] = {0};
    double ola_fir_sum = 0.0;    // presets whose overlap-add ran inside k_fir8p, summed over profiled batches
    int64_t host_cnt = 0;
    hipEvent_t ev[2][12] = {};
    bool device_plan = false;     // MSGPU_DEVICE_PLAN=1: plan on the device (k_plan_*), read back
    Staging staging;              // pinned uploads of a batch
    // constant tables
    uint64_t* d_ki = nullptr; double* d_wi = nullptr; double* d_fi = nullptr;
    uint64_t* d_ke = nullptr; double* d_we = nullptr; double* d_fe = nullptr;
    JumpTab* d_jump = nullptr;
    float2* d_fir2tab[5] = {};   // k_fir2 twiddle tables, M = 1024 << i
    float2* d_fir4tab = nullptr; // k_fir4 twiddle tables (M = 16384)
    bool fir4 = true;            // M = 16384 blocks on k_fir4 (MSGPU_FIR4=0: k_fir2, A/B and tests)
    // one-partition k_fir4 spectra from the taps (k_fir4_hconv; MSGPU_FIR4C=0: k_h_build + k_fir4_hpart)
    bool fir4c = true;
    bool fir8 = true;            // N = 65536 one-partition filters on k_fir8 (MSGPU_FIR8=0: off, A/B and tests)
    int fir64 = 1;               // float64 FIR of saturated renders: 0 off, 1 predicted, 2 every FIR preset (MSGPU_FIR64)
    int fir64_cap = FIR64_CAP;   // float64 FIR slots per window (MSGPU_FIR64_CAP: tests force several windows)
    // k_fir8 blocks (MSGPU_FIR8P): 0 one workgroup per block, 1 persistent workgroups
    // (one per CU, per-XCD block counters; C3 isolated FIR 2.03 -> 1.86 ms, C5 131.6
    // -> 125.9 ms per step, profiles/r04r_ab.json)
    int fir8p = 1;
    bool fir8q = true;           // msg_fir: 32 k < M <= 64 k taps as two partitions on k_fir8q (MSGPU_FIR8Q=0: off)
    int n_cu = 256;              // compute units (persistent grids)
    int fir8p_cus = 0;           // persistent FIR workgroups (MSGPU_FIR8P_CUS, A/B; 0: one per CU)
    int fir8p_stagger = 0;       // k_fir8p: every other workgroup starts this many 10-ns ticks later (MSGPU_FIR8P_STAGGER)
    // k_spec3 events (MSGPU_SPEC3P): 0 two per workgroup (the chain), 1 persistent
    // workgroups, one per CU, events from per-XCD counters (k_spec3p); > 1: that
    // many persistent workgroups (A/B)
    int spec3p = 0;
    // overlap-add inside k_fir8p's loads (PresetRt::ola_fir) for batches whose k_fir8p
    // presets' grains total at most ola_fir_density x their frames (MSGPU_OLA_FIR=0: never)
    bool ola_fir = true;
    // filter spectra before the generator (MSGPU_H_EARLY): 0 at the FIR stage, 1 always,
    // 2 (default) for batches with an output of at least 2^22 frames, whose FIR
    // holds every CU for milliseconds (C5 -2.5 %); shorter ones lose by it (C3 +2 %)
    int h_early = 2;
    bool er_dev = true;          // ER gains drawn on the device (k_er_gains; MSGPU_ER_DEV=0: on the host plan)
    double ola_fir_density = 1.25;
    // Q <= 2 presets on the streaming k_fir4s (MSGPU_FIR4S=1; off by default: at
    // C3's 24 blocks per preset its H re-reads miss L2 and cancel the saved transforms)
    bool fir4s = false;
    int fir4s_wgs = 1024;        // k_fir4s workgroups a batch aims for (MSGPU_FIR4S_WGS)
    // at most this many blocks per k_fir4s workgroup (MSGPU_FIR4S_K): every block
    // re-reads H_0 and H_1 (2 x 128 KB), so the workgroups running at once on an
    // XCD must share presets for those reads to hit its 4 MB L2
    int fir4s_kmax = 6;
    float2* d_spec_ct_tab[SPEC_CT_PLANS] = {};   // compile-time spectral plans (spec_ct.h)
    float2* d_spec3_tab = nullptr;               // band-pruned spectral kernel (spec3.h)
    Slice<int32_t> spec3_list;
    nprng::Zig dzig{};
    PlanStore grain_plans, fir_plans;
    // per-batch buffers
    // device planner (MSGPU_DEVICE_PLAN=1)
    DevBuf<msg_preset> dp_presets;
    DevBuf<double> dp_bp;                                 // breakpoint bank (device planner)
    DevBuf<int64_t> frag_len;
    DevBuf<msg_plan_info> info;
    DevBuf<int32_t> slot_base, tap_base;
    DevBuf<msg_event> dp_events;
    DevBuf<int32_t> dp_er_off;
    DevBuf<double> dp_er_gain;
    // per-batch inputs, uploaded in one copy (Staging arena)
    Slice<msg_preset> presets;
    Slice<msg_event> events;
    Slice<int32_t> er_off;
    Slice<double> er_gain;
    Slice<int32_t> er_key, er_first, er_cnt;
    DevBuf<double> er_gain_d;           // k_er_gains' output (host batch path)
    DevBuf<double> er_tap_d;            // k_er_gains' per-tap gains
    Slice<EventRt> ert;
    Slice<PresetRt> prt;
    Slice<int32_t> gen_list, spec_small, spec_big, tile_begin, fir_begin, h_begin, st_begin, fir_plan_of;
    DevBuf<float> micro, grain, mono_a, mono_y;
    DevBuf<float2> hspec;
    DevBuf<float> hscratch;                     // h of every FIR preset (k_h_build -> k_fir_h / k_fir4_hpart)
    Slice<int32_t> h_tile_begin, fir8_list, fir_lo;
    Slice<int64_t> ir8_jobs;
    Slice<int32_t> fir4c_list;                  // k_fir4_hconv presets (one partition at N = 32768)
    Slice<int64_t> ir4_jobs;                    // k_fir4_irspec jobs
    Slice<int2> hpart_jobs;
    Slice<int2> fir_jobs;
    Slice<int32_t> spec_ct_list;
    Slice<double> irbank;
    Slice<unsigned> maxbits;            // per preset: k_stereo_max's peak bits, zeroed by the batch's upload
    std::vector<unsigned> maxbits_zero;
    // float64 space FIR of saturated renders (kernels_fir64.h)
    Slice<Fir64Rt> f64rt;
    Slice<int32_t> st_count, odd_list, odd_cnt;
    DevBuf<double> f64_stats;                   // per preset: sum y^2, sum (1 + (d y)^2)^-2
    DevBuf<int32_t> f64_flag, f64_slot_preset, f64_nslots;
    // stereo pass (kernels_stereo.h): the fused persistent launch (MSGPU_STEREO_FUSED=1;
    // off by default) and its per-preset sync state, per-tile partial sums, counters
    bool stereo_fused = false;          // measured slower than the two launches
    int st_wgs = 4;                     // k_stereo_fused workgroups per CU (MSGPU_STEREO_WGS)
    uint32_t st_epoch = 0;
    DevBuf<int32_t> st_done, st_ctr;
    DevBuf<uint32_t> st_ready;
    DevBuf<double> st_part;
    DevBuf<int32_t> fir8_ctr;           // k_fir8p's per-XCD block counters
    DevBuf<int32_t> spec3_ctr;          // k_spec3p's per-XCD event counters
    DevBuf<float> f64_h;
    DevBuf<double2> f64_hs;
    // float64 grain chain (kernels_grain64.h)
    Plan64Store plans64;
    Slice<Ev64> ev64;
    Slice<int32_t> g64_list, gen64_list;
    Slice<int64_t> gen64_off;
    DevBuf<double> micro64, grain64, state64;
    DevBuf<double2> save64;
    Slice<Chain64> chains;
    Slice<uint8_t> imgbank;
    DevBuf<double2> g64A, g64B;                 // global-class float64 grains (G64Global)
    DevBuf<uint32_t> g64mask;
    // standalone FIR (msg_fir): its own buffers, so it never touches a render batch's
    DevBuf<PresetRt> sf_prt;
    DevBuf<int2> sf_jobs;
    DevBuf<int64_t> sf_irjobs;
    DevBuf<double> sf_h;
    DevBuf<float2> sf_hspec, sf_xspec;
    DevBuf<float> sf_hf;                        // float taps of a k_fir8 filter
    // msg_digest: render extents + tile bases, per-tile partials
    DevBuf<int64_t> dg_meta;
    DevBuf<char> dg_part;
    // odd-length stereo rotation (kernels_stereo_odd.h)
    std::map<int64_t, DevBuf<double2>> so_bp;  // chirp kernel spectra by n (float64), LRU-bounded
    std::map<int64_t, uint64_t> so_bp_use;     // batch serial of each entry's last use
    uint64_t batch_serial = 0;
    int so_row = 0, so_col = 0;                // transform-split limits (MSGPU_SO_ROW / _COL, tests; 0 = default)
    DevBuf<double2> so_A;
    DevBuf<float> so_r2;
    // host mirrors of the last batch
    std::vector<msg_plan_info> h_info;
    std::vector<msg_event> h_events;
    std::unique_ptr<EventRt[]> h_ert;   // host EventRt records (grow-only, msg_render_batch)
    size_t h_ert_cap = 0;
    std::vector<int32_t> h_er_off;
    std::vector<double> h_er_gain;
    // the host batch path's merged ER taps: per live slot its first key and
    // key count, the keys' tap indices (k_er_gains draws the gains on the device)
    std::vector<int32_t> h_er_key, h_er_first, h_er_cnt;
    std::vector<PresetRt> h_prt;
    std::vector<int32_t> h_slot_base;
    std::vector<Ev64> h_ev64;
    std::vector<int32_t> h_last64;      // per preset: Ev64 index of its last event, -1 = float32 chain
    int32_t last_n = 0;
};

// the longest output a preset may have: every kernel indexes a preset's frames
// with 32-bit integers (round 4 stopped at 2^29, where a 32-bit byte offset of
// the float2 output from the preset's own base ran out; the offsets are now
// formed from each tile's or block's base)
constexpr int64_t MSG_MAX_FRAMES = ((int64_t)1 << 31) - ((int64_t)1 << 20);

#define HIPCHK(ctx, expr)                                                        \
    do {                                                                         \
        hipError_t _e = (expr);                                                  \
        if (_e != hipSuccess) {                                                  \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);      \
            return MSG_E_DEVICE;                                                 \
        }                                                                        \
    } while (0)

static int fail(msg_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg; else g_err = msg;
    return code;
}

// ---------------------------------------------------------------------------
// FFT plan creation
// ---------------------------------------------------------------------------
static hipError_t upload(PlanStore& ps, const std::vector<float>& v, const float2** out) {
    void* d = nullptr;
    hipError_t e = hipMalloc(&d, v.size() * sizeof(float));
    if (e != hipSuccess) return e;
    e = hipMemcpy(d, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice);
    ps.allocs.push_back(d);
    *out = reinterpret_cast<const float2*>(d);
    return e;
}

static bool make_fftdesc(PlanStore& ps, int m, FftDesc& d, std::string& why) {
    std::vector<int> rad;
    memset(&d, 0, sizeof(d));
    d.m = m;
    if (fftplan::factor(m, rad)) {
        d.blue = 0;
        d.size = m;
    } else {
        d.blue = 1;
        d.size = fftplan::next_pow2(2 * m - 1);
        fftplan::factor(d.size, rad);
        std::vector<float> chirp, bspec;
        fftplan::bluestein(m, d.size, chirp, bspec);
        if (upload(ps, chirp, &d.chirp) != hipSuccess || upload(ps, bspec, &d.bspec) != hipSuccess) {
            why = "hip upload failed";
            return false;
        }
    }
    if ((int)rad.size() > FFT_MAXRAD) { why = "too many radix passes"; return false; }
    d.nrad = (int)rad.size();
    for (size_t i = 0; i < rad.size(); ++i) d.rad[i] = rad[i];
    d.tw_hi_n = (d.size + TW_LO - 1) / TW_LO;
    if (upload(ps, fftplan::twiddles(d.size, TW_LO, 1), &d.tw0) != hipSuccess ||
        upload(ps, fftplan::twiddles(d.size, d.tw_hi_n, TW_LO), &d.tw1) != hipSuccess) {
        why = "hip upload failed";
        return false;
    }
    return true;
}

// Real-FFT plan for n samples; returns index or -1.
static int real_plan(PlanStore& ps, int n, std::string& why) {
    auto it = ps.by_n.find(n);
    if (it != ps.by_n.end()) return it->second;
    RealPlan rp;
    memset(&rp, 0, sizeof(rp));
    rp.n = n;
    rp.even = (n % 2 == 0);
    const int m = rp.even ? n / 2 : n;
    if (!make_fftdesc(ps, m, rp.c, why)) return -1;
    rp.lds_c = lds_phys(std::max(rp.even ? m + 1 : m, rp.c.size));
    if (rp.even) {
        rp.rt_hi_n = (m + 1 + TW_LO - 1) / TW_LO;
        if (upload(ps, fftplan::twiddles(n, TW_LO, 1), &rp.rt0) != hipSuccess ||
            upload(ps, fftplan::twiddles(n, rp.rt_hi_n, TW_LO), &rp.rt1) != hipSuccess) {
            why = "hip upload failed";
            return -1;
        }
    }
    rp.lds_bytes = (rp.lds_c + TW_LO + rp.c.tw_hi_n + (rp.even ? TW_LO + rp.rt_hi_n : 0)) * 8;
    const int idx = (int)ps.host.size();
    ps.host.push_back(rp);
    ps.by_n[n] = idx;
    ps.dirty = true;
    return idx;
}

static hipError_t upload64(Plan64Store& ps, const std::vector<double>& v, const double2** out) {
    void* d = nullptr;
    hipError_t e = hipMalloc(&d, v.size() * sizeof(double));
    if (e != hipSuccess) return e;
    e = hipMemcpy(d, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice);
    ps.allocs.push_back(d);
    *out = reinterpret_cast<const double2*>(d);
    return e;
}

// float64 real-FFT plan for n samples (fft64.h); returns index or -1.
static int real64_plan(Plan64Store& ps, int n, std::string& why) {
    auto it = ps.by_n.find(n);
    if (it != ps.by_n.end()) return it->second;
    Real64Plan rp;
    memset(&rp, 0, sizeof(rp));
    rp.n = n;
    rp.even = (n % 2 == 0);
    const int m = rp.even ? n / 2 : n;
    Fft64& c = rp.c;
    c.m = m;
    std::vector<int> rad;
    std::vector<double> tab;
    if (fft64plan::factor(m, rad)) {
        c.blue = 0;
        c.size = m;
    } else {
        c.blue = 1;
        c.size = fft64plan::next_pow2(2 * m - 1);
        fft64plan::factor(c.size, rad);
        std::vector<double> bs;
        fft64plan::chirp(m, tab);
        fft64plan::bluestein_spec(m, c.size, tab, bs);
        if (upload64(ps, tab, &c.chirp) != hipSuccess || upload64(ps, bs, &c.bspec) != hipSuccess) {
            why = "hip upload failed";
            return -1;
        }
    }
    if ((int)rad.size() > F64_MAXRAD) { why = "too many radix passes"; return -1; }
    c.nrad = (int)rad.size();
    for (size_t i = 0; i < rad.size(); ++i) c.rad[i] = rad[i];
    fft64plan::twiddles(c.size, tab);
    if (upload64(ps, tab, &c.tw) != hipSuccess) { why = "hip upload failed"; return -1; }
    if (rp.even) {
        std::vector<double> rt(2 * (size_t)(m + 1));
        for (int k = 0; k <= m; ++k) {
            const long double a = -2.0L * 3.14159265358979323846264338327950288L * (long double)k / (long double)n;
            rt[2 * k] = (double)cosl(a);
            rt[2 * k + 1] = (double)sinl(a);
        }
        if (upload64(ps, rt, &rp.rt) != hipSuccess) { why = "hip upload failed"; return -1; }
    }
    rp.cap = std::max(std::max(c.size, rp.even ? m + 1 : n), n);
    const int idx = (int)ps.host.size();
    ps.host.push_back(rp);
    ps.by_n[n] = idx;
    ps.dirty = true;
    return idx;
}

template <class P>
static hipError_t sync_plans(PlanStoreT<P>& ps, hipStream_t s) {
    if (!ps.dirty) return hipSuccess;
    hipError_t e = ps.dev.ensure(ps.host.size());
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(ps.dev.p, ps.host.data(), ps.host.size() * sizeof(P), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    ps.dirty = false;
    return e;
}

// Bessel J_m(x), m >= 0, power series (x <= 0.9 here).
static double bessel_j(int m, double x) {
    double term = 1.0;
    for (int k = 1; k <= m; ++k) term *= (x / 2.0) / k;
    double sum = term;
    for (int k = 1; k < 60; ++k) {
        term *= -(x / 2.0) * (x / 2.0) / ((double)k * (double)(k + m));
        sum += term;
        if (std::fabs(term) < 1e-30) break;
    }
    return sum;
}

// Choose (N, P, Q) minimising FFT work for an M-tap FIR over n outputs (h is
// built in the time domain by k_h_build, so any N with P < N qualifies).
// fir8: also consider N = 65536 with one partition (k_fir8: two half-size
// transforms per transform of N, P = M).
// stream: when non-null, also consider k_fir4s (N = 32768, P = B = 16384, Q <= 2:
// one forward and one inverse transform per block plus, for Q = 2, one forward
// per workgroup of kblk blocks) and report whether it won.
// M8: the length of the filter k_fir8 would apply (its spectrum holds every
// in-range ER tap and the whole IR, so it can be longer than an M capped at
// out_n); the 65536-point candidate needs M8 + B - 1 <= N or it wraps.
static void choose_fir(int64_t M, int64_t n, int& N, int& P, int& Q, bool fir8, bool* stream = nullptr,
                       int kblk = 1, int64_t M8 = -1) {
    if (M8 < M) M8 = M;
    double best = 1e300;
    N = FIR_NMAX; P = (int)std::min<int64_t>(M, FIR_NMAX / 2); Q = (int)((M + P - 1) / P);
    for (int lg = 11; lg <= 15; ++lg) {   // k_fir2 / k_fir4 sizes: M = N/2 in 1024..16384
        const int NN = 1 << lg;
        for (int q = 1; q <= 64; ++q) {
            const int64_t pp = (M + q - 1) / q;
            if (pp >= NN) continue;
            const int64_t B = NN - pp + 1;
            const int64_t blocks = (n + B - 1) / B;
            const double cost = (double)blocks * (q + 1) * NN * lg + (double)blocks * NN * 4.0;
            if (cost < best) { best = cost; N = NN; P = (int)pp; Q = q; }
        }
    }
    if (fir8 && M8 < FIR8_N / 2 + FIR8_N / 4) {   // B >= N/4
        const int64_t B = FIR8_N - M8 + 1;
        const int64_t blocks = (n + B - 1) / B;
        const double cost = (double)blocks * 2 * FIR8_N * 16 + (double)blocks * FIR8_N * 4.0;
        if (cost < best) { best = cost; N = FIR8_N; P = (int)M8; Q = 1; }
    }
    if (stream) {
        *stream = false;
        const int NN = 2 * FIR4S_P, lg = 15;
        const int64_t q = (M + FIR4S_P - 1) / FIR4S_P;
        if (q <= 2) {
            const int64_t blocks = (n + FIR4S_P - 1) / FIR4S_P;
            const double cost = (double)blocks * (2.0 + (q - 1) / (double)kblk) * NN * lg + (double)blocks * NN * 4.0;
            if (cost < best) { best = cost; N = NN; P = FIR4S_P; Q = (int)q; *stream = true; }
        }
    }
}

static int spec_ops(const msg_preset& p, const msg_event& e) {
    int ops = 0;
    if (p.gen_mode == MSG_GEN_NOISE_BURST || p.gen_mode == MSG_GEN_FALLBACK) ops |= SPEC_TILT_NOISE;
    if (p.gen_mode == MSG_GEN_SKEWED) ops |= SPEC_TILT_SKEW;
    if ((p.flags & MSG_F_BANDLIMIT) && e.n >= 8) ops |= SPEC_LOWPASS;
    if ((p.flags & MSG_F_NL_WARP) && e.n >= 16) ops |= SPEC_WARP;
    if (!(p.flags & MSG_F_PARTIAL_LOCK) && e.n >= 16 && std::fabs(e.stretch - 1.0) >= 1e-9) ops |= SPEC_STRETCH;
    return ops;
}

// Presets whose grains run the float64 chain (kernels_grain64.h): the
// generators outside the normal-driven closed forms, and every stage whose
// reference result hinges on float64 magnitudes or noise floors.
static bool is_precise(const msg_preset& p) {
    const uint32_t f64_stages = MSG_F_PARTIAL_LOCK | MSG_F_CEP_WARP | MSG_F_RES_BANK | MSG_F_WAVEGUIDE |
                                MSG_F_EVENT_FEEDBACK | MSG_F_IMPRINT | MSG_F_MULTIBAND;
    if (p.flags & f64_stages) return true;
    switch (p.gen_mode) {
        case MSG_GEN_GAUSSIAN_CLICK: case MSG_GEN_NOISE_BURST: case MSG_GEN_SKEWED:
        case MSG_GEN_RESONANT: case MSG_GEN_FALLBACK: return false;
        default: return true;
    }
}
static bool normal_driven(int gen_mode) {
    return gen_mode == MSG_GEN_GAUSSIAN_CLICK || gen_mode == MSG_GEN_NOISE_BURST || gen_mode == MSG_GEN_SKEWED ||
           gen_mode == MSG_GEN_RESONANT || gen_mode == MSG_GEN_FALLBACK;
}

// Stages of the float64 chain one event runs, with the reference's own
// length / identity guards (MS:42, 105, 119-121, 132-134, 152, 372, 389).
static int g64_ops(const msg_preset& p, const msg_event& e) {
    int ops = 0;
    const int n = e.n;
    const bool stretch_id = std::fabs(e.stretch - 1.0) < 1e-9;
    if ((p.flags & MSG_F_BANDLIMIT) && n >= 8) ops |= G64_LOWPASS;
    if ((p.flags & MSG_F_NL_WARP) && n >= 16) ops |= G64_WARP;
    if ((p.flags & MSG_F_CEP_WARP) && n >= 64) ops |= G64_CEP;
    if (p.flags & MSG_F_PARTIAL_LOCK) {
        if (n >= 64 && !stretch_id) ops |= G64_LOCK;
    } else if (n >= 16 && !stretch_id) {
        ops |= G64_STRETCH;
    }
    if ((p.flags & MSG_F_RES_BANK) && n >= 32) ops |= G64_RES;
    if ((p.flags & MSG_F_WAVEGUIDE) && n >= 64) ops |= G64_WG;
    if (p.flags & MSG_F_MULTIBAND) ops |= G64_MB;
    if (p.flags & (MSG_F_EVENT_FEEDBACK | MSG_F_IMPRINT)) ops |= G64_CHAIN;
    return ops;
}

static void stage_mark(msg_ctx* ctx, int i, hipStream_t s) {
    if (ctx->gate_wait >= 0 || ctx->gate_rec >= 0) {
        std::lock_guard<std::mutex> lk(g_gate_mu);   // the peer may be unlinked by msg_destroy
        if (ctx->gate_peer) {
            // the gate's wait comes before the stage's profiling event, so a stage's
            // time is its kernels' span on the stream, not the time it was held
            if (i == ctx->gate_wait && ctx->gate_peer->gate_armed.load())
                hipStreamWaitEvent(s, ctx->gate_peer->gate_ev, 0);
            if (i == ctx->gate_rec) {
                hipEventRecord(ctx->gate_ev, s);
                ctx->gate_armed.store(true);
            }
        }
    }
    if (ctx->prof_batch) hipEventRecord(ctx->ev[ctx->ev_cur][i], s);
}

// A batch on a different stream than the context's last one waits for that
// batch's end (the staging arena and buffers are stream-ordered).
static hipError_t stream_handover(msg_ctx* ctx, hipStream_t s) {
    if (ctx->done_armed && s != ctx->last_stream) return hipStreamWaitEvent(s, ctx->done_ev, 0);
    return hipSuccess;
}
static hipError_t stream_done(msg_ctx* ctx, hipStream_t s) {
    if (!ctx->done_ev) {
        const hipError_t e = hipEventCreateWithFlags(&ctx->done_ev, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    ctx->last_stream = s;
    ctx->done_armed = true;
    return hipEventRecord(ctx->done_ev, s);
}

// Records done_ev on every exit of a call that may have enqueued work, the
// early fail() returns included: a later batch on another stream
// then still waits for this one before it reuses the staging arena and buffers.
struct DoneGuard {
    msg_ctx* ctx;
    hipStream_t s;
    bool armed = true;
    DoneGuard(msg_ctx* c, hipStream_t st) : ctx(c), s(st) {}
    hipError_t finish() { armed = false; return stream_done(ctx, s); }
    ~DoneGuard() { if (armed) stream_done(ctx, s); }
};

// k_fir8p's per-XCD block counters: zeroed once; every launch leaves them zero
static hipError_t fir8_counters(msg_ctx* ctx, hipStream_t s) {
    if (ctx->fir8_ctr.p) return hipSuccess;
    const hipError_t e = ctx->fir8_ctr.ensure((size_t)(MSG_XCDS + 1) * FIR8P_CTR);
    if (e != hipSuccess) return e;
    return hipMemsetAsync(ctx->fir8_ctr.p, 0, sizeof(int32_t) * ctx->fir8_ctr.cap, s);
}

// k_spec3p's per-XCD event counters: zeroed once; every launch leaves them zero
static hipError_t spec3_counters(msg_ctx* ctx, hipStream_t s) {
    if (ctx->spec3_ctr.p) return hipSuccess;
    const hipError_t e = ctx->spec3_ctr.ensure((size_t)(MSG_XCDS + 1) * S3P_CTR);
    if (e != hipSuccess) return e;
    return hipMemsetAsync(ctx->spec3_ctr.p, 0, sizeof(int32_t) * ctx->spec3_ctr.cap, s);
}

// Wait for the context's last batch (not the whole device: other contexts'
// streams keep running).
static hipError_t wait_last(msg_ctx* ctx) {
    return ctx->done_armed ? hipEventSynchronize(ctx->done_ev) : hipSuccess;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
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

const char* msg_last_error(msg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

msg_ctx* msg_create(int device_ordinal) {
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) { g_err = "no HIP device available"; return nullptr; }
    if (device_ordinal < 0 || device_ordinal >= ndev) { g_err = "bad device ordinal"; return nullptr; }
    if (hipSetDevice(device_ordinal) != hipSuccess) { g_err = "hipSetDevice failed"; return nullptr; }
    std::unique_ptr<msg_ctx> ctx(new msg_ctx());
    ctx->device = device_ordinal;
    auto up = [&](auto*& dst, const auto* src, size_t n) {
        using T = std::remove_pointer_t<std::remove_reference_t<decltype(dst)>>;
        if (hipMalloc(&dst, n * sizeof(T)) != hipSuccess) return false;
        return hipMemcpy(dst, src, n * sizeof(T), hipMemcpyHostToDevice) == hipSuccess;
    };
    if (!up(ctx->d_ki, zig_ki_double, 256) || !up(ctx->d_wi, zig_wi_double, 256) ||
        !up(ctx->d_fi, zig_fi_double, 256) || !up(ctx->d_ke, zig_ke_double, 256) ||
        !up(ctx->d_we, zig_we_double, 256) || !up(ctx->d_fe, zig_fe_double, 256)) {
        g_err = "uploading ziggurat tables failed";
        return nullptr;
    }
    ctx->dzig = nprng::Zig{ctx->d_ki, ctx->d_wi, ctx->d_fi, ctx->d_ke, ctx->d_we, ctx->d_fe};
    JumpTab jt;
    for (int l = 0; l < GEN_T; ++l) {
        const nprng::Jump j = nprng::jump_of((uint64_t)l + 1);
        jt.a[l] = j.a; jt.s[l] = j.s;
    }
    const nprng::Jump j64 = nprng::jump_of(GEN_T);
    jt.a64 = j64.a; jt.s64 = j64.s;
    const nprng::Jump jG = nprng::jump_of((uint64_t)GEN_T * GEN_G);
    jt.aG = jG.a; jt.sG = jG.s;
    for (int w = 0; w < GEN_K; ++w) {
        const nprng::Jump jw = nprng::jump_of((uint64_t)GEN_T * GEN_G * w);
        jt.aW[w] = jw.a; jt.sW[w] = jw.s;
    }
    const nprng::Jump jR = nprng::jump_of((uint64_t)GEN_T * GEN_G * GEN_K);
    jt.aR = jR.a; jt.sR = jR.s;
    for (int i = 0; i < 256; ++i) {
        const float w = (float)(zig_wi_double[i] * 1048576.0);
        uint32_t wb;
        memcpy(&wb, &w, 4);
        jt.kw[i] = make_uint2((uint32_t)(zig_ki_double[i] >> 20), wb);
        jt.fif[i] = (float)zig_fi_double[i];
    }
    if (!up(ctx->d_jump, &jt, 1)) { g_err = "uploading jump table failed"; return nullptr; }
    for (int i = 0; i < 5; ++i) {
        std::vector<float> tab;
        if (!fir2_tables_host(1024 << i, tab) || !up(ctx->d_fir2tab[i], reinterpret_cast<float2*>(tab.data()),
                                                     tab.size() / 2)) {
            g_err = "uploading FIR twiddle tables failed";
            return nullptr;
        }
    }
    {
        std::vector<float> tab;
        if (!fir4_tables_host(16384, tab) || !up(ctx->d_fir4tab, reinterpret_cast<float2*>(tab.data()), tab.size() / 2)) {
            g_err = "uploading FIR4 twiddle tables failed";
            return nullptr;
        }
    }
    if (const char* e = getenv("MSGPU_FIR4")) ctx->fir4 = e[0] != '0';
    if (const char* e = getenv("MSGPU_FIR4C")) ctx->fir4c = e[0] != '0';
    if (const char* e = getenv("MSGPU_FIR8")) ctx->fir8 = e[0] != '0';
    if (const char* e = getenv("MSGPU_FIR64")) ctx->fir64 = atoi(e);
    if (const char* e = getenv("MSGPU_FIR64_CAP")) ctx->fir64_cap = std::max(1, std::min(FIR64_CAP, atoi(e)));
    if (const char* e = getenv("MSGPU_FIR8P")) ctx->fir8p = atoi(e);
    if (const char* e = getenv("MSGPU_FIR8Q")) ctx->fir8q = e[0] != '0';
    if (const char* e = getenv("MSGPU_FIR8P_CUS")) ctx->fir8p_cus = std::max(0, atoi(e));
    if (const char* e = getenv("MSGPU_FIR8P_STAGGER")) ctx->fir8p_stagger = std::max(0, atoi(e));
    if (const char* e = getenv("MSGPU_SPEC3P")) ctx->spec3p = atoi(e);
    if (const char* e = getenv("MSGPU_OLA_FIR")) ctx->ola_fir = e[0] != '0';
    if (const char* e = getenv("MSGPU_H_EARLY")) ctx->h_early = atoi(e);
    if (const char* e = getenv("MSGPU_ER_DEV")) ctx->er_dev = e[0] != '0';
    if (const char* e = getenv("MSGPU_OLA_FIR_DENSITY")) ctx->ola_fir_density = atof(e);
    if (const char* e = getenv("MSGPU_STEREO_FUSED")) ctx->stereo_fused = e[0] != '0';
    if (const char* e = getenv("MSGPU_STEREO_WGS")) ctx->st_wgs = std::max(1, std::min(16, atoi(e)));
    {
        int cu = 0;
        if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device_ordinal) == hipSuccess && cu >= MSG_XCDS)
            ctx->n_cu = cu;
    }
    if (const char* e = getenv("MSGPU_FIR4S")) ctx->fir4s = e[0] == '1';
    if (const char* e = getenv("MSGPU_FIR4S_WGS")) ctx->fir4s_wgs = std::max(1, atoi(e));
    if (const char* e = getenv("MSGPU_FIR4S_K")) ctx->fir4s_kmax = std::max(2, std::min(64, atoi(e)));
    for (int i = 0; i < SPEC_CT_PLANS; ++i) {
        std::vector<float> tab;
        if (!spectral_ct_tables(i, tab) || !up(ctx->d_spec_ct_tab[i], reinterpret_cast<float2*>(tab.data()),
                                               tab.size() / 2)) {
            g_err = "uploading spectral twiddle tables failed";
            return nullptr;
        }
    }
    {
        std::vector<float> tab;
        if (!spec3_tables(tab) || !up(ctx->d_spec3_tab, reinterpret_cast<float2*>(tab.data()), tab.size() / 2)) {
            g_err = "uploading spectral twiddle tables failed";
            return nullptr;
        }
    }
    for (auto& set : ctx->ev)
        for (auto& ev : set) hipEventCreate(&ev);
    if (const char* e = getenv("MSGPU_DEVICE_PLAN")) ctx->device_plan = e[0] == '1';
    if (const char* e = getenv("MSGPU_SO_ROW")) ctx->so_row = atoi(e);
    if (const char* e = getenv("MSGPU_SO_COL")) ctx->so_col = atoi(e);
    spectral_ct_init_attrs();
    spec3_init_attrs();
    spectral_init_attrs();
    fir_init_attrs();
    fft_bench_init_attrs();
    grain64_init_attrs();
    stereo_odd_init_attrs();
    fir64_init_attrs();
    return ctx.release();
}

void msg_destroy(msg_ctx* ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    hipDeviceSynchronize();
    for (PlanStore* ps : {&ctx->grain_plans, &ctx->fir_plans}) {
        for (void* p : ps->allocs) hipFree(p);
        ps->dev.release();
    }
    hipFree(ctx->d_ki); hipFree(ctx->d_wi); hipFree(ctx->d_fi);
    hipFree(ctx->d_ke); hipFree(ctx->d_we); hipFree(ctx->d_fe); hipFree(ctx->d_jump);
    for (float2* t : ctx->d_fir2tab) hipFree(t);
    hipFree(ctx->d_fir4tab);
    for (float2* t : ctx->d_spec_ct_tab) hipFree(t);
    hipFree(ctx->d_spec3_tab);
    ctx->sf_prt.release(); ctx->sf_jobs.release(); ctx->sf_irjobs.release(); ctx->sf_h.release();
    ctx->sf_hspec.release(); ctx->sf_xspec.release(); ctx->sf_hf.release();
    ctx->dg_meta.release(); ctx->dg_part.release();
    for (auto& set : ctx->ev)
        for (auto& ev : set) hipEventDestroy(ev);
    {
        std::lock_guard<std::mutex> lk(g_gate_mu);
        for (msg_ctx* c : ctx->gated_by) { c->gate_peer = nullptr; c->gate_wait = c->gate_rec = -1; }
        if (ctx->gate_peer) {
            auto& v = ctx->gate_peer->gated_by;
            v.erase(std::remove(v.begin(), v.end(), ctx), v.end());
        }
    }
    if (ctx->gate_ev) hipEventDestroy(ctx->gate_ev);
    if (ctx->done_ev) hipEventDestroy(ctx->done_ev);
    ctx->staging.release();
    ctx->dp_presets.release(); ctx->dp_bp.release(); ctx->frag_len.release(); ctx->info.release(); ctx->slot_base.release();
    ctx->tap_base.release(); ctx->dp_events.release(); ctx->dp_er_off.release(); ctx->dp_er_gain.release();
    ctx->micro.release(); ctx->grain.release();
    ctx->mono_a.release(); ctx->mono_y.release(); ctx->hspec.release();
    ctx->hscratch.release();
    ctx->f64_stats.release(); ctx->f64_flag.release(); ctx->st_done.release(); ctx->st_ctr.release();
    ctx->fir8_ctr.release(); ctx->spec3_ctr.release();
    ctx->st_ready.release(); ctx->st_part.release(); ctx->f64_slot_preset.release(); ctx->f64_nslots.release();
    ctx->f64_h.release(); ctx->f64_hs.release();
    for (void* p : ctx->plans64.allocs) hipFree(p);
    ctx->plans64.dev.release();
    ctx->micro64.release(); ctx->grain64.release(); ctx->state64.release(); ctx->save64.release();
    ctx->g64A.release(); ctx->g64B.release(); ctx->g64mask.release();
    for (auto& kv : ctx->so_bp) kv.second.release();
    ctx->so_A.release(); ctx->so_r2.release();
    delete ctx;
}

// Fold the event times of the last profiled batch into the running sums.
// The events are read lazily (here, at the next batch of the same context or
// at msg_stage_times) so profiling never blocks the host between batches.
static void collect_stage_set(msg_ctx* ctx, int k) {
    if (!ctx->pending[k]) return;
    hipEvent_t* ev = ctx->ev[k];
    hipEventSynchronize(ev[7]);
    float ms[10] = {0};
    for (int i = 0; i < 7; ++i) hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]);
    hipEventElapsedTime(&ms[7], ev[0], ev[7]);
    if (ctx->pending_fir[k]) {   // the FIR kernel alone, and the filter spectra
        hipEventElapsedTime(&ms[8], ev[8], ev[9]);
        if (ctx->pending_h_early[k]) {   // launched before the generator: out of host_prep
            hipEventElapsedTime(&ms[9], ev[10], ev[11]);
            hipEventElapsedTime(&ms[1], ev[1], ev[10]);
        } else {
            hipEventElapsedTime(&ms[9], ev[5], ev[8]);
        }
    }
    for (int i = 0; i < 10; ++i) ctx->stage_sum[i] += ms[i];
    ++ctx->stage_cnt;
    ctx->pending[k] = false;
}
// all sets (msg_stage_times / msg_set_profiling): waits for the profiled batches
static void collect_stage_times(msg_ctx* ctx) {
    collect_stage_set(ctx, ctx->ev_cur ^ 1);
    collect_stage_set(ctx, ctx->ev_cur);
}

int msg_set_profiling(msg_ctx* ctx, int32_t on) {
    if (!ctx) return MSG_E_ARG;
    collect_stage_times(ctx);
    ctx->profiling = on != 0;
    ctx->prof_every = on > 1 ? on : 1;
    ctx->prof_n = 0;
    if (ctx->profiling) {
        for (double& v : ctx->stage_sum) v = 0.0;
        for (double& v : ctx->host_sum) v = 0.0;
        ctx->ola_fir_sum = 0.0;
        ctx->stage_cnt = 0;
        ctx->host_cnt = 0;
    }
    return MSG_OK;
}

int msg_gate(msg_ctx* ctx, msg_ctx* peer, int32_t wait_stage, int32_t record_stage) {
    if (!ctx || peer == ctx || wait_stage < -1 || wait_stage > 9 || record_stage < -1 || record_stage > 9)
        return MSG_E_ARG;
    if (peer && peer->device != ctx->device) return MSG_E_ARG;
    if (peer && !ctx->gate_ev && hipEventCreateWithFlags(&ctx->gate_ev, hipEventDisableTiming) != hipSuccess)
        return fail(ctx, MSG_E_DEVICE, "hipEventCreate failed");
    std::lock_guard<std::mutex> lk(g_gate_mu);
    if (ctx->gate_peer) {
        auto& v = ctx->gate_peer->gated_by;
        v.erase(std::remove(v.begin(), v.end(), ctx), v.end());
    }
    ctx->gate_peer = peer;
    if (peer) peer->gated_by.push_back(ctx);
    ctx->gate_wait = peer ? wait_stage : -1;
    ctx->gate_rec = peer ? record_stage : -1;
    ctx->gate_armed.store(false);
    return MSG_OK;
}

int msg_stage_times(msg_ctx* ctx, float* ms, int32_t n) {
    if (!ctx || !ms) return MSG_E_ARG;
    collect_stage_times(ctx);
    for (int i = 0; i < n && i < 10; ++i)
        ms[i] = ctx->stage_cnt ? (float)(ctx->stage_sum[i] / (double)ctx->stage_cnt) : 0.f;
    for (int i = 10; i < n && i < 13; ++i)
        ms[i] = ctx->host_cnt ? (float)(ctx->host_sum[i - 10] / (double)ctx->host_cnt) : 0.f;
    for (int i = 13; i < n && i < 18; ++i)
        ms[i] = ctx->host_cnt ? (float)(ctx->host_sum[i - 10] / (double)ctx->host_cnt) : 0.f;
    if (n > 18) ms[18] = ctx->host_cnt ? (float)(ctx->ola_fir_sum / (double)ctx->host_cnt) : 0.f;
    return MSG_OK;
}

#include "host_abi.inc"

int msg_bench_fft(msg_ctx* ctx, int32_t n, int32_t reps, int32_t blocks, float* ms_out) {
    if (!ctx || !ms_out || n < 2 || reps < 1 || blocks < 1) return MSG_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    std::string why;
    const bool po2 = (n & (n - 1)) == 0;
    PlanStore& ps = po2 ? ctx->fir_plans : ctx->grain_plans;
    const int pi = real_plan(ps, n, why);
    if (pi < 0) return fail(ctx, MSG_E_DEVICE, why);
    HIPCHK(ctx, sync_plans(ps, nullptr));
    const RealPlan& rp = ps.host[pi];
    if (rp.lds_bytes > LDS_MAX) return fail(ctx, MSG_E_UNSUPPORTED, "too large for LDS");
    float* sink = nullptr;
    HIPCHK(ctx, hipMalloc(&sink, sizeof(float) * blocks));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    HIPCHK(ctx, launch_fft_bench(po2, blocks, rp.lds_bytes, nullptr, ps.dev.p, pi, 1, sink));   // warm-up
    hipEventRecord(a, nullptr);
    HIPCHK(ctx, launch_fft_bench(po2, blocks, rp.lds_bytes, nullptr, ps.dev.p, pi, reps, sink));
    hipEventRecord(b, nullptr);
    HIPCHK(ctx, hipEventSynchronize(b));
    hipEventElapsedTime(ms_out, a, b);
    hipEventDestroy(a); hipEventDestroy(b);
    hipFree(sink);
    return MSG_OK;
}

int msg_fft64(msg_ctx* ctx, int32_t n, int32_t inverse, const double* in, double* out) {
    if (!ctx || !in || !out || n < 2) return MSG_E_ARG;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    std::string why;
    const int pi = real64_plan(ctx->plans64, n, why);
    if (pi < 0) return fail(ctx, MSG_E_DEVICE, why);
    const Real64Plan rp = ctx->plans64.host[pi];
    HIPCHK(ctx, sync_plans(ctx->plans64, nullptr));
    const int K = n / 2 + 1;
    const size_t cnt = (size_t)std::max(n, 2 * K);
    double* io = nullptr;
    HIPCHK(ctx, hipMalloc(&io, cnt * sizeof(double)));
    hipError_t e = hipMemcpy(io, in, (inverse ? 2 * K : n) * sizeof(double), hipMemcpyHostToDevice);
    double2* gA = nullptr;
    double2* gB = nullptr;
    if (e == hipSuccess && rp.cap > G64_SLOTS) {     // beyond LDS: the engine's global ping-pong mode
        e = hipMalloc(&gA, (size_t)rp.cap * sizeof(double2));
        if (e == hipSuccess) e = hipMalloc(&gB, (size_t)rp.cap * sizeof(double2));
    }
    if (e == hipSuccess) e = launch_fft64_one(rp.cap * 16, nullptr, ctx->plans64.dev.p, pi, inverse ? 1 : 0, io, gA, gB);
    if (e == hipSuccess) e = hipMemcpy(out, io, (inverse ? n : 2 * K) * sizeof(double), hipMemcpyDeviceToHost);
    hipFree(io);
    if (gA) hipFree(gA);
    if (gB) hipFree(gB);
    HIPCHK(ctx, e);
    return MSG_OK;
}

int msg_stft_mag_db(msg_ctx* ctx, const void* x_dev, int32_t elem_bytes, int64_t n, int32_t channels, int32_t win,
                    int32_t hop, int32_t max_frames, double* S_dev, int32_t* frames, void* stream) {
    if (!ctx || !frames || n < 1 || win < 2 || hop < 1 || (channels != 1 && channels != 2) ||
        (elem_bytes != 4 && elem_bytes != 8))
        return fail(ctx, MSG_E_ARG, "bad arguments");
    const int64_t fr = n < win ? 1 : std::min<int64_t>(1 + (n - win) / hop, std::max(max_frames, 0));
    *frames = (int32_t)fr;
    if (!S_dev || fr <= 0) return MSG_OK;                 // size query
    if (!x_dev) return fail(ctx, MSG_E_ARG, "null input");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    std::string why;
    const int pi = real64_plan(ctx->plans64, win, why);
    if (pi < 0) return fail(ctx, MSG_E_DEVICE, why);
    const int cap = ctx->plans64.host[pi].cap;
    if (cap > G64_SLOTS) return fail(ctx, MSG_E_UNSUPPORTED, "STFT window beyond the LDS float64 engine");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(ctx, sync_plans(ctx->plans64, s));
    HIPCHK(ctx, launch_stft64((unsigned)fr, cap * 16, s, ctx->plans64.dev.p, pi, x_dev, elem_bytes, n, channels, win,
                                     hop, S_dev));
    return MSG_OK;
}

int msg_fir(msg_ctx* ctx, const float* x_dev, float* y_dev, int64_t n, int32_t n_signals, const double* h,
            int64_t M, int32_t* fir_shape, void* stream) {
    if (!ctx || !x_dev || !y_dev || !h || n < 1 || n_signals < 1 || M < 1)
        return fail(ctx, MSG_E_ARG, "bad arguments");
    if ((const void*)x_dev == (const void*)y_dev) return fail(ctx, MSG_E_ARG, "x and y must not alias");
    if (M > (int64_t)64 * (FIR_NMAX - 1)) return fail(ctx, MSG_E_UNSUPPORTED, "FIR longer than 64 partitions");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(ctx, stream_handover(ctx, s));
    DoneGuard done(ctx, s);
    int N = 0, Pp = 0, Q = 0;
    choose_fir(M, n, N, Pp, Q, ctx->fir8);
    // Many partitions: a frequency-domain delay line (fir_fft.h) computes each
    // input segment's spectrum once and reuses it for Q blocks -- two transforms
    // per block of N/2 outputs instead of Q + 1 per block of N - P + 1, for
    // 8 B/output of spectrum writes and 8 Q B/output of reads.  Measured on
    // MI355X: slower at 64 k taps (classic Q = 5: 7.1 ms vs 7.7 ms per 1024
    // signals), so it takes over only from Q = 8 (>= ~115 k taps).
    // Two partitions of 32 768 taps on the 65 536-point engine (k_fir8q, 32 768
    // < M <= 65 536 beyond the one-partition limit): one forward and one inverse
    // per 32 768 outputs (MSGPU_FIR8Q=0: the choice above, k_fir4 at 64 k taps).
    // Above 35 748 taps the two partitions' 32 768-frame blocks beat one
    // partition's 65 537 - M (a k_fir8q block costs ~1.1 k_fir8p blocks).
    if (ctx->fir8 && ctx->fir8q && ctx->fir8p > 0 && M <= 2 * (int64_t)FIR8Q_P &&
        (double)(FIR8_N + 1 - M) * 1.1 < (double)FIR8Q_P) {
        const int64_t nb = (n + FIR8Q_P - 1) / FIR8Q_P;
        if (nb * n_signals > INT32_MAX) return fail(ctx, MSG_E_UNSUPPORTED, "too many output blocks");
        if (fir_shape) { fir_shape[0] = FIR8_N; fir_shape[1] = FIR8Q_P; fir_shape[2] = 2; }
        // runs of consecutive blocks: about four per CU over the call, whole signals when they suffice
        const int64_t want = 4 * (int64_t)ctx->n_cu;
        const int run_len = (int)std::max<int64_t>(1, std::min<int64_t>(nb, (nb * n_signals + want - 1) / want));
        std::vector<PresetRt> prt((size_t)n_signals);
        std::vector<int2> runs;
        for (int i = 0; i < n_signals; ++i) {
            PresetRt& r = prt[i];
            memset(&r, 0, sizeof(r));
            r.out_n = n;
            r.y_off = (int64_t)i * n;
            r.fir_on = 1; r.fir_N = FIR8_N; r.fir_P = FIR8Q_P; r.fir_Q = (int32_t)nb; r.fir_B = FIR8Q_P;
            for (int64_t j = 0; j < nb; j += run_len) runs.push_back(make_int2(i, (int)j));
        }
        std::vector<float> hf((size_t)M);
        for (int64_t i = 0; i < M; ++i) hf[i] = (float)h[i];
        const int64_t K8 = FIR8_HSTRIDE;          // float2 per spectrum (fir8_fft.h layout)
        const int64_t job[8] = {0, FIR8Q_P, 0, 0, FIR8Q_P, M - FIR8Q_P, K8, 0};   // H_0, H_1 from the float taps
        const unsigned grid = (unsigned)std::min<int64_t>((int64_t)runs.size(), ctx->n_cu);
        HIPCHK(ctx, ctx->sf_prt.ensure(prt.size()));
        HIPCHK(ctx, ctx->sf_jobs.ensure(runs.size()));
        HIPCHK(ctx, ctx->sf_hf.ensure((size_t)M));
        HIPCHK(ctx, ctx->sf_irjobs.ensure(8));
        HIPCHK(ctx, ctx->sf_hspec.ensure((size_t)(2 * K8)));
        HIPCHK(ctx, ctx->sf_xspec.ensure((size_t)grid * (size_t)fir8q_scratch_per_wg()));
        HIPCHK(ctx, fir8_counters(ctx, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_prt.p, prt.data(), sizeof(PresetRt) * prt.size(), hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_jobs.p, runs.data(), sizeof(int2) * runs.size(), hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_hf.p, hf.data(), sizeof(float) * (size_t)M, hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_irjobs.p, job, sizeof(job), hipMemcpyHostToDevice, s));
        HIPCHK(ctx, launch_fir8_spec32(2, s, ctx->sf_irjobs.p, ctx->d_fir4tab, ctx->sf_hf.p, ctx->sf_hspec.p));
        HIPCHK(ctx, launch_fir8q((unsigned)runs.size(), run_len, grid, s, ctx->sf_prt.p, ctx->sf_jobs.p, ctx->d_fir4tab,
                                 ctx->sf_hspec.p, x_dev, y_dev, ctx->sf_xspec.p, ctx->fir8_ctr.p,
                                 getenv("MSGPU_FIR8Q_MODE") ? atoi(getenv("MSGPU_FIR8Q_MODE")) : 0));
        HIPCHK(ctx, done.finish());
        return MSG_OK;
    }
    const bool fdl = Q >= 8;
    if (fdl) {
        N = FIR_NMAX;
        Pp = N / 2;
        Q = (int)((M + Pp - 1) / Pp);
    }
    const int64_t B = fdl ? Pp : N - Pp + 1;
    const int64_t blocks = (n + B - 1) / B;
    if (blocks * n_signals > INT32_MAX) return fail(ctx, MSG_E_UNSUPPORTED, "too many output blocks");
    if (fir_shape) { fir_shape[0] = N; fir_shape[1] = Pp; fir_shape[2] = Q; }
    if (N == FIR8_N) {   // one partition on k_fir8: H from the float taps by k_fir8_hpart
        std::vector<PresetRt> prt((size_t)n_signals);
        std::vector<int2> fj;
        fj.reserve((size_t)(blocks * n_signals));
        for (int i = 0; i < n_signals; ++i) {
            PresetRt& r = prt[i];
            memset(&r, 0, sizeof(r));
            r.out_n = n;
            r.y_off = (int64_t)i * n;
            r.fir_on = 1; r.fir_N = N; r.fir_P = Pp; r.fir_Q = 1; r.fir_B = (int32_t)B;
            r.h_off = 0; r.hs_off = 0; r.h_len = (int32_t)M;
            for (int64_t b = 0; b < blocks; ++b) fj.push_back(make_int2(i, (int)b));
        }
        std::vector<float> hf((size_t)M);
        for (int64_t i = 0; i < M; ++i) hf[i] = (float)h[i];
        const int64_t job[4] = {0, M, 0, 0};      // k_fir8_spec: taps [0, M) -> spectrum at 0
        HIPCHK(ctx, ctx->sf_prt.ensure(prt.size()));
        HIPCHK(ctx, ctx->sf_jobs.ensure(fj.size()));
        HIPCHK(ctx, ctx->sf_hf.ensure((size_t)M));
        HIPCHK(ctx, ctx->sf_irjobs.ensure(4));
        HIPCHK(ctx, ctx->sf_hspec.ensure((size_t)FIR8_HSTRIDE));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_prt.p, prt.data(), sizeof(PresetRt) * prt.size(), hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_jobs.p, fj.data(), sizeof(int2) * fj.size(), hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_hf.p, hf.data(), sizeof(float) * (size_t)M, hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->sf_irjobs.p, job, sizeof(job), hipMemcpyHostToDevice, s));
        HIPCHK(ctx, launch_fir8_spec32(1, s, ctx->sf_irjobs.p, ctx->d_fir4tab, ctx->sf_hf.p, ctx->sf_hspec.p));
        if (ctx->fir8p > 0) {   // persistent, as in the render (one workgroup per CU, per-XCD block counters)
            const int nj = (int)fj.size();
            const unsigned grid = (unsigned)std::max(MSG_XCDS, (std::min(nj, ctx->n_cu) / MSG_XCDS) * MSG_XCDS);
            HIPCHK(ctx, fir8_counters(ctx, s));
            HIPCHK(ctx, launch_fir8p((unsigned)nj, grid, s, ctx->sf_prt.p, ctx->sf_jobs.p, ctx->d_fir4tab,
                                     ctx->sf_hspec.p, x_dev, y_dev, ctx->fir8_ctr.p, 0, nullptr, nullptr, nullptr));
        } else {
            HIPCHK(ctx, launch_fir8((unsigned)fj.size(), s, ctx->sf_prt.p, ctx->sf_jobs.p, ctx->d_fir4tab,
                                    ctx->sf_hspec.p, x_dev, y_dev));
        }
        HIPCHK(ctx, done.finish());
        return MSG_OK;
    }
    std::string why;
    const int fp = real_plan(ctx->fir_plans, N, why);
    if (fp < 0) return fail(ctx, MSG_E_DEVICE, "FIR plan: " + why);
    HIPCHK(ctx, sync_plans(ctx->fir_plans, s));
    const int K = N / 2 + 1;
    // partition spectra H_q = FFT_N(h[qP, qP + P)) by the IR-spectrum kernel
    std::vector<int64_t> jobs;
    for (int q = 0; q < Q; ++q)
        jobs.insert(jobs.end(), {(int64_t)q * Pp, std::min<int64_t>(Pp, M - (int64_t)q * Pp), (int64_t)fp,
                                 (int64_t)q * K});
    std::vector<PresetRt> prt((size_t)n_signals);
    std::vector<int2> fj;
    fj.reserve((size_t)(blocks * n_signals));
    for (int i = 0; i < n_signals; ++i) {
        PresetRt& r = prt[i];
        memset(&r, 0, sizeof(r));
        r.out_n = n;
        r.y_off = (int64_t)i * n;
        r.fir_on = 1; r.fir_N = N; r.fir_P = Pp; r.fir_Q = Q; r.fir_B = (int32_t)B;
        r.h_off = 0;
        r.fir_block_begin = (int32_t)(i * blocks);     // FDL: first segment spectrum of this signal
        for (int64_t b = 0; b < blocks; ++b) fj.push_back(make_int2(i, (int)b));
    }
    HIPCHK(ctx, ctx->sf_prt.ensure(prt.size()));
    HIPCHK(ctx, ctx->sf_jobs.ensure(fj.size()));
    HIPCHK(ctx, ctx->sf_irjobs.ensure(jobs.size()));
    HIPCHK(ctx, ctx->sf_h.ensure((size_t)M));
    HIPCHK(ctx, ctx->sf_hspec.ensure((size_t)Q * K));
    if (fdl) HIPCHK(ctx, ctx->sf_xspec.ensure((size_t)fj.size() * K));
    HIPCHK(ctx, hipMemcpyAsync(ctx->sf_prt.p, prt.data(), sizeof(PresetRt) * prt.size(), hipMemcpyHostToDevice, s));
    HIPCHK(ctx, hipMemcpyAsync(ctx->sf_jobs.p, fj.data(), sizeof(int2) * fj.size(), hipMemcpyHostToDevice, s));
    HIPCHK(ctx, hipMemcpyAsync(ctx->sf_irjobs.p, jobs.data(), sizeof(int64_t) * jobs.size(), hipMemcpyHostToDevice,
                               s));
    HIPCHK(ctx, hipMemcpyAsync(ctx->sf_h.p, h, sizeof(double) * (size_t)M, hipMemcpyHostToDevice, s));
    HIPCHK(ctx, launch_ir_spec((unsigned)Q, ctx->fir_plans.host[fp].lds_bytes, s, ctx->sf_irjobs.p, Q,
                               ctx->fir_plans.dev.p, ctx->sf_h.p, ctx->sf_hspec.p));
    int ti = 0;
    while ((1024 << ti) != N / 2) ++ti;
    if (fdl)
        HIPCHK(ctx, launch_fdl(N / 2, (unsigned)fj.size(), s, ctx->sf_prt.p, ctx->sf_jobs.p, ctx->d_fir2tab[ti],
                               ctx->sf_hspec.p, ctx->sf_xspec.p, x_dev, y_dev));
    else if (N / 2 == 16384 && ctx->fir4)
        HIPCHK(ctx, launch_fir4(N / 2, (unsigned)fj.size(), s, ctx->sf_prt.p, ctx->sf_jobs.p, ctx->d_fir4tab,
                                ctx->sf_hspec.p, x_dev, y_dev));
    else
        HIPCHK(ctx, launch_fir2(N / 2, (unsigned)fj.size(), s, ctx->sf_prt.p, ctx->sf_jobs.p, ctx->d_fir2tab[ti],
                                ctx->sf_hspec.p, x_dev, y_dev));
    // pageable-host H2D copies are staged before hipMemcpyAsync returns (as in
    // msg_render_batch), so the host vectors may go; the FIR runs asynchronously.
    HIPCHK(ctx, done.finish());
    return MSG_OK;
}

int msg_digest(msg_ctx* ctx, const float* out_dev, const int64_t* out_offsets, const int64_t* out_n,
               int32_t n_renders, msg_digest_rec* rec_dev, void* stream) {
    if (!ctx || !out_offsets || !out_n || !rec_dev || n_renders < 0) return fail(ctx, MSG_E_ARG, "bad arguments");
    if (n_renders == 0) return MSG_OK;
    // rows: [0, n) frame offsets, [n, 2n) frames, then n + 1 tile bases (int32) in the same upload
    std::vector<int64_t> meta((size_t)2 * n_renders + (n_renders + 2) / 2 + 1, 0);
    int32_t* tb = reinterpret_cast<int32_t*>(meta.data() + 2 * (size_t)n_renders);
    int64_t tiles = 0;
    for (int i = 0; i < n_renders; ++i) {
        if (out_n[i] < 0 || out_n[i] > MSG_MAX_FRAMES || out_offsets[i] < 0)
            return fail(ctx, MSG_E_ARG, "bad render extent");
        meta[i] = out_offsets[i];
        meta[(size_t)n_renders + i] = out_n[i];
        tb[i] = (int32_t)tiles;
        tiles += digest_tiles(out_n[i]);
        if (tiles > INT32_MAX) return fail(ctx, MSG_E_UNSUPPORTED, "too many digest tiles");
    }
    tb[n_renders] = (int32_t)tiles;
    if (tiles > 0 && !out_dev) return fail(ctx, MSG_E_ARG, "null output buffer");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(ctx, stream_handover(ctx, s));
    DoneGuard done(ctx, s);
    HIPCHK(ctx, ctx->dg_meta.ensure(meta.size()));
    HIPCHK(ctx, ctx->dg_part.ensure((size_t)std::max<int64_t>(1, tiles) * sizeof(msg_digest_rec)));
    // a pageable source is staged before hipMemcpyAsync returns (as msg_fir's uploads)
    HIPCHK(ctx, hipMemcpyAsync(ctx->dg_meta.p, meta.data(), sizeof(int64_t) * meta.size(), hipMemcpyHostToDevice, s));
    const int64_t* dm = ctx->dg_meta.p;
    HIPCHK(ctx, launch_digest(n_renders, (int)tiles, s, out_dev, dm, dm + n_renders,
                              reinterpret_cast<const int32_t*>(dm + 2 * (size_t)n_renders), ctx->dg_part.p, rec_dev));
    HIPCHK(ctx, done.finish());
    return MSG_OK;
}

int msg_digest_host(const float* x, int64_t out_n, msg_digest_rec* rec) {
    if (!rec || out_n < 0 || (out_n > 0 && !x)) return fail(nullptr, MSG_E_ARG, "bad arguments");
    digest_host(x, out_n, rec);
    return MSG_OK;
}

int msg_last_plan(msg_ctx* ctx, msg_plan_info* info, int32_t n_presets) {
    if (!ctx || !info) return MSG_E_ARG;
    if (n_presets > ctx->last_n) return fail(ctx, MSG_E_ARG, "n_presets exceeds last batch");
    std::memcpy(info, ctx->h_info.data(), sizeof(msg_plan_info) * n_presets);
    return MSG_OK;
}

int msg_last_events(msg_ctx* ctx, int32_t preset, msg_event* events, int32_t cap, int32_t* n) {
    if (!ctx || !n) return MSG_E_ARG;
    if (preset < 0 || preset >= ctx->last_n) return fail(ctx, MSG_E_ARG, "bad preset index");
    const int32_t k = ctx->h_info[preset].n_events;
    *n = k;
    if (!events) return MSG_OK;
    if (k > cap) return fail(ctx, MSG_E_ARG, "event buffer too small");
    std::memcpy(events, ctx->h_events.data() + ctx->h_slot_base[preset], sizeof(msg_event) * k);
    return MSG_OK;
}

int msg_last_meta(msg_ctx* ctx, int32_t preset, double* micro, double* grain, int64_t cap, int64_t* n) {
    if (!ctx || !n) return MSG_E_ARG;
    if (preset < 0 || preset >= ctx->last_n) return fail(ctx, MSG_E_ARG, "bad preset index");
    hipSetDevice(ctx->device);
    const msg_plan_info& inf = ctx->h_info[preset];
    *n = 0;
    if (inf.n_events <= 0) return MSG_OK;
    const msg_event& e = ctx->h_events[ctx->h_slot_base[preset] + inf.n_events - 1];
    if (e.n > cap) return fail(ctx, MSG_E_ARG, "meta buffer too small");
    std::vector<float> tmp(e.n);
    const int64_t off = ctx->h_prt[preset].pool_base + e.pool_off;
    HIPCHK(ctx, wait_last(ctx));
    const int32_t l64 = ctx->h_last64.empty() ? -1 : ctx->h_last64[preset];
    if (l64 >= 0) {   // float64 chain: micro_last / grain_last kept in float64
        const int64_t o64 = ctx->h_ev64[l64].off64;
        if (micro) HIPCHK(ctx, hipMemcpy(micro, ctx->micro64.p + o64, e.n * sizeof(double), hipMemcpyDeviceToHost));
        if (grain) HIPCHK(ctx, hipMemcpy(grain, ctx->grain64.p + o64, e.n * sizeof(double), hipMemcpyDeviceToHost));
        *n = e.n;
        return MSG_OK;
    }
    if (micro) {
        HIPCHK(ctx, hipMemcpy(tmp.data(), ctx->micro.p + off, e.n * sizeof(float), hipMemcpyDeviceToHost));
        for (int i = 0; i < e.n; ++i) micro[i] = tmp[i];
    }
    if (grain) {
        HIPCHK(ctx, hipMemcpy(tmp.data(), ctx->grain.p + off, e.n * sizeof(float), hipMemcpyDeviceToHost));
        for (int i = 0; i < e.n; ++i) grain[i] = tmp[i];
    }
    *n = e.n;
    return MSG_OK;
}

int msg_last_grain64(msg_ctx* ctx, int32_t preset, int32_t k, double* grain, int64_t cap, int64_t* n) {
    if (!ctx || !n) return MSG_E_ARG;
    if (preset < 0 || preset >= ctx->last_n) return fail(ctx, MSG_E_ARG, "bad preset index");
    const int32_t l64 = ctx->h_last64.empty() ? -1 : ctx->h_last64[preset];
    const int32_t ne = ctx->h_info[preset].n_events;
    if (l64 < 0) return fail(ctx, MSG_E_ARG, "preset is not on the float64 chain");
    if (k < 0 || k >= ne) return fail(ctx, MSG_E_ARG, "bad event index");
    const int64_t at = (int64_t)l64 - (ne - 1) + k;   // the preset's events end at its last float64 record
    if (at < 0 || at >= (int64_t)ctx->h_ev64.size()) return fail(ctx, MSG_E_ARG, "event not on the float64 chain");
    const Ev64& v = ctx->h_ev64[at];
    *n = v.n;
    if (!grain) return MSG_OK;
    if (v.n > cap) return fail(ctx, MSG_E_ARG, "grain buffer too small");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, wait_last(ctx));
    HIPCHK(ctx, hipMemcpy(grain, ctx->grain64.p + v.off64, v.n * sizeof(double), hipMemcpyDeviceToHost));
    return MSG_OK;
}

int msg_render_batch(msg_ctx* ctx, const msg_preset* presets, int32_t P,
                     const double* bp_bank, int64_t bp_pairs, const double* const* irs, const int64_t* ir_lens, int32_t n_irs,
                     const uint8_t* const* images, const int32_t* img_h, const int32_t* img_w,
                     int32_t n_images, float* out_dev, const int64_t* out_offsets, void* stream) {
    if (!ctx || !presets || P <= 0 || !out_dev || !out_offsets) return fail(ctx, MSG_E_ARG, "bad arguments");
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, stream_handover(ctx, s));
    DoneGuard done(ctx, s);
    collect_stage_set(ctx, ctx->ev_cur);   // this batch's event set: from two batches back
    for (int p = 0; p < P; ++p) {
        for (int l = 0; l < 4; ++l) {   // lanes inside the breakpoint bank
            const int32_t nb = presets[p].n_bp[l], ob = presets[p].bp_off[l];
            if (nb < 0 || (nb > 0 && (!bp_bank || ob < 0 || (int64_t)ob + nb > bp_pairs)))
                return fail(ctx, MSG_E_ARG, "preset " + std::to_string(p) + ": breakpoint lane outside the bank");
        }
        const int ic = presets[p].ir_conv;
        if (ic >= n_irs || (ic >= 0 && !irs)) return fail(ctx, MSG_E_ARG, "bad IR index");
    }
    ctx->prof_batch = ctx->profiling && (ctx->prof_n++ % ctx->prof_every) == 0;
    stage_mark(ctx, 0, s);
    using hclock = std::chrono::steady_clock;
    const auto h0 = hclock::now();
    auto hA = h0;
    std::vector<int64_t> flen(P, 0);
    for (int p = 0; p < P; ++p) {
        const int f = presets[p].ir_frag;
        flen[p] = (f >= 0 && f < n_irs) ? ir_lens[f] : 0;
    }
    std::vector<msg_plan_info> info(P);
    std::vector<int32_t> slot_base(P), tap_base(P);
    int64_t nslots = 0, ntaps = 0;
    auto bases = [&]() -> int {
        nslots = ntaps = 0;
        int64_t frames = 0;
        for (int p = 0; p < P; ++p) {
            slot_base[p] = (int32_t)nslots;
            tap_base[p] = (int32_t)ntaps;
            nslots += info[p].n_slots;
            if (presets[p].flags & MSG_F_ER_CLOUD) ntaps += std::max(1, presets[p].er_taps);
            // kernels index a preset's frames with 32-bit integers (byte offsets
            // from a tile's or block's own base; the tile counters of a batch in 32 bits)
            if (info[p].out_n > MSG_MAX_FRAMES) return fail(ctx, MSG_E_UNSUPPORTED, "output longer than 2^31 - 2^20 frames");
            frames += info[p].out_n;
        }
        if (nslots > INT32_MAX / 2) return fail(ctx, MSG_E_UNSUPPORTED, "too many events in one batch");
        if (frames > ((int64_t)1 << 40)) return fail(ctx, MSG_E_UNSUPPORTED, "more than 2^40 frames in one batch");
        return MSG_OK;
    };
    if (!ctx->device_plan) {
        // ---- host plan (plan.h, the device planner's code) on the host pool:
        // no device round trip, so the call returns once the batch is enqueued
        HostPool& pool = HostPool::get();
        pool.run(P, [&](int p) { msgplan::plan_sizes(presets[p], bp_bank, kHostZig, flen[p], info[p]); });
        hA = hclock::now();
        if (int st = bases()) return st;
        ctx->h_events.resize(nslots);
        ctx->h_er_off.resize(ntaps);
        if (ctx->er_dev) {
            ctx->h_er_key.resize(ntaps);
            ctx->h_er_first.resize(ntaps);
            ctx->h_er_cnt.resize(ntaps);
        } else {
            ctx->h_er_gain.resize(ntaps);
        }
        // offsets only: the gains (two thirds of the host plan of a 320-tap preset,
        // a float64 exp each) are drawn on the device by k_er_gains
        pool.run(P, [&](int p) {
            const bool er = (presets[p].flags & MSG_F_ER_CLOUD) != 0;
            msgplan::plan_events(presets[p], bp_bank, kHostZig, flen[p], p, info[p], ctx->h_events.data() + slot_base[p],
                                 er ? ctx->h_er_off.data() + tap_base[p] : nullptr,
                                 (er && !ctx->er_dev) ? ctx->h_er_gain.data() + tap_base[p] : nullptr, true);
        });

    } else {
        // ---- device plan, phase 1: sizes ----
        HIPCHK(ctx, ctx->frag_len.ensure(P));
        HIPCHK(ctx, ctx->info.ensure(P));
        HIPCHK(ctx, ctx->dp_presets.ensure(P));
        HIPCHK(ctx, hipMemcpyAsync(ctx->dp_presets.p, presets, sizeof(msg_preset) * P, hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->frag_len.p, flen.data(), sizeof(int64_t) * P, hipMemcpyHostToDevice, s));
        HIPCHK(ctx, ctx->dp_bp.ensure((size_t)std::max<int64_t>(1, 2 * bp_pairs)));
        if (bp_pairs > 0)
            HIPCHK(ctx, hipMemcpyAsync(ctx->dp_bp.p, bp_bank, sizeof(double) * 2 * bp_pairs, hipMemcpyHostToDevice, s));
        const int pb = 64;
        hipLaunchKernelGGL(k_plan_sizes, dim3((P + pb - 1) / pb), dim3(pb), 0, s,
                           ctx->dp_presets.p, P, ctx->dp_bp.p, ctx->frag_len.p, ctx->dzig, ctx->info.p);
        HIPCHK(ctx, hipGetLastError());
        HIPCHK(ctx, hipMemcpyAsync(info.data(), ctx->info.p, sizeof(msg_plan_info) * P, hipMemcpyDeviceToHost, s));
        HIPCHK(ctx, hipStreamSynchronize(s));
        // ---- phase 2: events + ER taps ----
        if (int st = bases()) return st;
        HIPCHK(ctx, ctx->slot_base.ensure(P));
        HIPCHK(ctx, ctx->tap_base.ensure(P));
        HIPCHK(ctx, ctx->dp_events.ensure(nslots));
        HIPCHK(ctx, ctx->dp_er_off.ensure(ntaps));
        HIPCHK(ctx, ctx->dp_er_gain.ensure(ntaps));
        HIPCHK(ctx, hipMemcpyAsync(ctx->slot_base.p, slot_base.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, s));
        HIPCHK(ctx, hipMemcpyAsync(ctx->tap_base.p, tap_base.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_plan_events, dim3((P + pb - 1) / pb), dim3(pb), 0, s,
                           ctx->dp_presets.p, P, ctx->dp_bp.p, ctx->frag_len.p, ctx->dzig, ctx->slot_base.p,
                           ctx->tap_base.p,
                           ctx->dp_events.p, ctx->dp_er_off.p, ctx->dp_er_gain.p, ctx->info.p);
        HIPCHK(ctx, hipGetLastError());
        ctx->h_events.resize(nslots);
        HIPCHK(ctx, hipMemcpyAsync(info.data(), ctx->info.p, sizeof(msg_plan_info) * P, hipMemcpyDeviceToHost, s));
        if (nslots)
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_events.data(), ctx->dp_events.p, sizeof(msg_event) * nslots,
                                       hipMemcpyDeviceToHost, s));
        ctx->h_er_off.resize(ntaps);
        ctx->h_er_gain.resize(ntaps);
        if (ntaps) {
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_er_off.data(), ctx->dp_er_off.p, sizeof(int32_t) * ntaps,
                                       hipMemcpyDeviceToHost, s));
            HIPCHK(ctx, hipMemcpyAsync(ctx->h_er_gain.data(), ctx->dp_er_gain.p, sizeof(double) * ntaps,
                                       hipMemcpyDeviceToHost, s));
        }
        HIPCHK(ctx, hipStreamSynchronize(s));
    }
    // Early-reflection taps whose rounded delays coincide are merged here, in tap
    // order and in float64 (the order MS:416-420 adds them), and the taps that
    // act on the output (0 < offset < out_n, MS:418-420) are compacted to the
    // front of the preset's tap range sorted by offset: k_h_build walks only the
    // taps whose shifted IR overlaps its tile.  n_taps_live[p]: their count,
    // tap_max[p]: the largest offset (0 without taps).
    std::vector<int32_t> n_taps_live(P, 0), tap_max(P, 0);
    {
        auto merge = [&](int p) {
            if (!(presets[p].flags & MSG_F_ER_CLOUD)) return;
            const int nt = std::max(1, presets[p].er_taps);
            int32_t* off = ctx->h_er_off.data() + tap_base[p];
            const bool dev_gain = !ctx->device_plan && ctx->er_dev;
            double* g = dev_gain ? nullptr : ctx->h_er_gain.data() + tap_base[p];
            // (offset, tap index) packed in one key, sorted stably by offset (tap_sort.h)
            thread_local std::vector<uint64_t> keybuf, tmpbuf;
            thread_local std::vector<double> g0;
            keybuf.resize(nt);
            tmpbuf.resize(nt);
            if (!dev_gain) g0.assign(g, g + nt);
            const int64_t n = info[p].out_n;
            int m = 0;
            uint32_t omax = 0;
            for (int k = 0; k < nt; ++k)
                if (off[k] > 0 && off[k] < n) {
                    keybuf[m++] = ((uint64_t)(uint32_t)off[k] << 32) | (uint32_t)k;
                    omax = std::max(omax, (uint32_t)off[k]);
                }
#if MSG_TAP_RADIX
            const uint64_t* key = sort_taps_by_offset(keybuf.data(), tmpbuf.data(), m, omax);
#else                                                    // tuning A/B: the comparison sort
            std::sort(keybuf.begin(), keybuf.begin() + m);
            const uint64_t* key = keybuf.data();
#endif
            int live = 0;
            if (dev_gain) {                              // slots -> key ranges, summed by k_er_gains
                int32_t* kx = ctx->h_er_key.data() + tap_base[p];
                int32_t* first = ctx->h_er_first.data() + tap_base[p];
                int32_t* cnt = ctx->h_er_cnt.data() + tap_base[p];
                for (int i = 0; i < m; ++i) kx[i] = (int32_t)(uint32_t)key[i];
                for (int i = 0; i < m;) {
                    const uint32_t o = (uint32_t)(key[i] >> 32);
                    int j = i + 1;
                    while (j < m && (uint32_t)(key[j] >> 32) == o) ++j;
                    off[live] = (int32_t)o;
                    first[live] = i;
                    cnt[live] = j - i;
                    ++live;
                    i = j;
                }
            } else {
                for (int i = 0; i < m;) {
                    const uint32_t o = (uint32_t)(key[i] >> 32);
                    double acc = g0[(uint32_t)key[i]];
                    int j = i + 1;
                    for (; j < m && (uint32_t)(key[j] >> 32) == o; ++j) acc += g0[(uint32_t)key[j]];
                    off[live] = (int32_t)o;
                    g[live] = acc;
                    ++live;
                    i = j;
                }
            }
            n_taps_live[p] = live;
            tap_max[p] = live ? off[live - 1] : 0;
        };
        if (ctx->device_plan) for (int p = 0; p < P; ++p) merge(p);
        else HostPool::get().run(P, merge);
    }
    stage_mark(ctx, 1, s);
    const auto h1 = hclock::now();
    ctx->staging.add(&ctx->presets.p, presets, sizeof(msg_preset) * P);
    ctx->staging.add(&ctx->events.p, ctx->h_events.data(), sizeof(msg_event) * nslots);
    ctx->staging.add(&ctx->er_off.p, ctx->h_er_off.data(), sizeof(int32_t) * ntaps);
    const bool er_dev = !ctx->device_plan && ctx->er_dev;
    if (!er_dev) {
        ctx->staging.add(&ctx->er_gain.p, ctx->h_er_gain.data(), sizeof(double) * ntaps);
    } else {
        ctx->staging.add(&ctx->er_key.p, ctx->h_er_key.data(), sizeof(int32_t) * ntaps);
        ctx->staging.add(&ctx->er_first.p, ctx->h_er_first.data(), sizeof(int32_t) * ntaps);
        ctx->staging.add(&ctx->er_cnt.p, ctx->h_er_cnt.data(), sizeof(int32_t) * ntaps);
    }

    // ---- host: runtime records ----
    std::vector<PresetRt> prt(P);
    // host EventRt records: a grow-only buffer reused across batches (a C5 sub-batch
    // holds 512 k events; a fresh zero-filled vector cost ~8 ms of page faults and
    // memset per batch).  Every slot an event list references is written below.
    if ((size_t)nslots > ctx->h_ert_cap) {
        ctx->h_ert.reset(new EventRt[(size_t)nslots + nslots / 4]);
        ctx->h_ert_cap = (size_t)nslots + nslots / 4;
    }
    EventRt* const ert = ctx->h_ert.get();
    // slots a preset reserves beyond its events are never written below: zero them
    // so the whole uploaded range is defined
    for (int p = 0; p < P; ++p)
        if (info[p].n_slots > info[p].n_events)
            memset(ert + slot_base[p] + info[p].n_events, 0,
                   sizeof(EventRt) * (size_t)(info[p].n_slots - info[p].n_events));
    std::vector<Fir64Rt> f64rt(P);
    std::vector<int32_t> st_count(P);
    int f64_cand = 0, f64_qmax = 0, f64_bmax = 0, f64_stmax = 0;
    int64_t f64_hmax = 0;
    std::vector<int32_t> gen_list, spec_small, spec_big, tile_begin(P), fir_begin(P), h_begin(P), st_begin(P),
        fir_plan_of(P, 0);
    std::vector<double> irbank;
    std::vector<int64_t> ir_off(std::max(n_irs, 1), 0);
    for (int i = 0; i < n_irs; ++i) {
        ir_off[i] = (int64_t)irbank.size();
        irbank.insert(irbank.end(), irs[i], irs[i] + ir_lens[i]);
    }
    int64_t pool = 0, ysum = 0, hsum = 0;
    int32_t tiles = 0, fblocks = 0, hblocks = 0, stiles = 0;
    int n_ola_fir = 0;                               // presets with PresetRt::ola_fir
    int64_t ola_fir_nmax = 0;                        // their longest output
    std::vector<int2> hpart_jobs;                  // (preset, q) of the presets on the k_fir4 engine
    std::vector<int32_t> h_tile_begin(P, 0);       // k_h_build tiles per preset (prefix)
    int32_t htiles = 0;
    int32_t hblocks_gen = 0;                       // k_fir_h blocks of presets not on the k_fir4 engine
    int64_t hs_sum = 0;
    int spec_small_lds = 0, spec_big_lds = 0, fir_lds = 0;
    std::vector<int32_t> spec_ct[SPEC_CT_PLANS];           // events of the compile-time spectral plans
    const char* ct_env = getenv("MSGPU_SPEC_CT");         // "0": runtime-plan kernels only (tests)
    const bool use_ct = !(ct_env && ct_env[0] == '0');
    const char* s3_env = getenv("MSGPU_SPEC3");          // "0": no band-pruned kernel (A/B, tests)
    const bool use_s3 = use_ct && !(s3_env && s3_env[0] == '0');
    // MSGPU_G64_STOP=cep (tests only): float64-chain grains stop before the cepstral
    // warp (MS:696-697), so meta grain_last is that stage's input (stage-pin tests)
    const char* stop_env = getenv("MSGPU_G64_STOP");
    const bool stop_cep = stop_env && std::strcmp(stop_env, "cep") == 0;
    std::vector<int32_t> spec3;                           // events of the band-pruned kernel
    std::vector<int32_t> f32_presets;                     // presets on the float32 chain
    std::vector<int2> fjobs_by[7];                        // FIR output blocks per transform size; [5]: k_fir4s, [6]: k_fir8
    std::vector<int32_t> fir8_list;                       // ER presets on k_fir8 (N = 65536): k_fir8_hconv
    std::vector<int32_t> ir_only8;                        // IR-only presets on k_fir8: H = the IR's spectrum
    std::map<int, int64_t> ir8_spec_of;                   // IR index -> spectrum offset (before relocation)
    std::vector<int64_t> ir8_jobs;                        // k_fir8_spec jobs: [ir_off, len, spec_off, 0]
    int64_t ir8_sum = 0;
    // the same at N = 32768 on the k_fir4 engine (k_fir4_hconv / k_fir4_irspec, MSGPU_FIR4C)
    std::vector<int32_t> fir4c_list, ir_only4;
    std::map<int, int64_t> ir4_spec_of;
    std::vector<int64_t> ir4_jobs;
    int64_t ir4_sum = 0;
    std::vector<int2> fir4s_presets;                      // (preset, blocks) on the streaming FIR
    // float64 grain chain records
    std::vector<Ev64> ev64;
    std::vector<int32_t> gen64_list;                      // normal-driven float64 events (event slots)
    std::vector<int64_t> gen64_off;                       // their raw-normal offsets in micro64
    std::vector<Chain64> chains;
    std::vector<int32_t> last64(P, -1);
    std::vector<uint8_t> imgbank;
    std::vector<int64_t> img_off(std::max(n_images, 1), 0);
    for (int i = 0; i < n_images; ++i) {
        img_off[i] = (int64_t)imgbank.size();
        imgbank.insert(imgbank.end(), images[i], images[i] + (int64_t)img_h[i] * img_w[i]);
    }
    int64_t sum64 = 0, save_sum = 0, state_sum = 0;
    int64_t r2_sum = 0, so_M = 0;
    std::vector<int32_t> odd_presets;
    int g64_cap = 0;                                      // LDS slots of the LDS-class float64 grains
    int64_t g64_big_cap = 0;                              // slot size of the global-class grains
    std::vector<int32_t> g64_lds, g64_glb;                // Ev64 indices by class
    std::vector<Chain64> chains_glb;
    // Taps of the space filter h = (delta + ER) * IR of preset p (MS:409-445), 0
    // without a FIR: the largest ER offset (planned span or actual) plus the IR
    // length, at most out_n (later taps never reach y[:out_n]).
    // full8: instead the length of the filter k_fir8's spectrum holds (every
    // in-range tap, offset < out_n, and the whole IR), not capped at out_n.
    auto h_taps = [&](int p, bool full8 = false) -> int64_t {
        const msg_preset& pr = presets[p];
        const bool er = (pr.flags & MSG_F_ER_CLOUD) != 0;
        const int ic = pr.ir_conv;
        const bool ir = (pr.flags & MSG_F_SPACE_IR) && ic >= 0 && ir_lens[ic] > 0;
        if (!er && !ir) return 0;
        const int64_t irl = ir ? std::min<int64_t>(ir_lens[ic], 8192) : 1;
        const int64_t span = er ? std::max<int64_t>((int64_t)std::nearbyint(pr.er_max_ms / 1000.0 * (double)pr.base_sr),
                                                    tap_max[p]) : 0;
        if (full8) return std::min<int64_t>(span, std::max<int64_t>(0, info[p].out_n - 1)) + irl;
        return std::max<int64_t>(1, std::min<int64_t>(span + irl, info[p].out_n));
    };
    // k_fir4s pays one extra forward transform per workgroup: it is offered only
    // when the batch's streaming-eligible blocks give >= 2 blocks per workgroup
    bool fir4s_ok = false;
    int fir4s_k = 1;                                      // blocks per k_fir4s workgroup
    if (ctx->fir4 && ctx->fir4s) {
        int64_t total = 0;
        for (int p = 0; p < P; ++p) {
            const int64_t M = h_taps(p);
            if (M > 0 && M <= 2 * FIR4S_P)
                total += (info[p].out_n + FIR4S_P - 1) / FIR4S_P;
        }
        fir4s_k = (int)std::min<int64_t>(ctx->fir4s_kmax, total / std::max(1, ctx->fir4s_wgs));
        fir4s_ok = fir4s_k >= 2;
    }
    // the per-preset pure functions of the records (FIR partitioning, stereo
    // Bessel taps) in parallel; the loop below does the prefix bookkeeping
    struct FirPick { int64_t M; int N, P, Q; bool stream; float bess[25]; };
    std::vector<FirPick> pick(P);
    HostPool::get().run(P, [&](int p) {
        FirPick& f = pick[p];
        f.M = h_taps(p);
        f.N = f.P = f.Q = 0;
        f.stream = false;
        if (f.M > 0)
            choose_fir(f.M, info[p].out_n, f.N, f.P, f.Q, ctx->fir8, fir4s_ok ? &f.stream : nullptr, fir4s_k,
                       h_taps(p, true));
        const double w = std::min(std::max(presets[p].stereo_width, 0.0), 1.0);
        for (int m = 0; m <= 12; ++m) {                // J_{-m} = (-1)^m J_m: one series per |m|
            const double j = bessel_j(m, w * 0.9);
            f.bess[m + 12] = (float)j;
            f.bess[12 - m] = (float)((m & 1) ? -j : j);
        }
    });
    // The overlap-add inside k_fir8p, decided for the batch as a whole: all of its
    // k_fir8p presets or none, by their grains against their outputs.  A batch
    // with any ola_fir preset runs the fused instantiation for all of its blocks,
    // and that kernel's extra live state costs the plain blocks ~10 % (C3: a few
    // sparse seeds had put every C3 batch on it, isolated FIR 1.88 -> 2.13 ms).
    bool batch_ola = false;
    if (ctx->ola_fir && ctx->fir8p > 0) {
        double grains = 0.0, frames = 0.0;
        for (int p = 0; p < P; ++p)
            if (pick[p].M > 0 && pick[p].N == FIR8_N && !pick[p].stream) {
                grains += (double)info[p].pool_len;
                frames += (double)info[p].out_n;
            }
        batch_ola = frames > 0.0 && grains <= ctx->ola_fir_density * frames;
    }
    for (int p = 0; p < P; ++p) {
        const msg_preset& pr = presets[p];
        const msg_plan_info& inf = info[p];
        PresetRt& r = prt[p];
        memset(&r, 0, sizeof(r));
        r.out_n = inf.out_n;
        r.out_off = out_offsets[p];
        r.pool_base = pool;
        r.y_off = ysum;
        r.ev_begin = slot_base[p];
        r.n_events = inf.n_events;
        r.er_base = tap_base[p];
        r.n_taps = n_taps_live[p];          // merged, in-range, offset-sorted taps
        r.tile_begin = tiles;
        r.max_n = inf.max_n;
        // generator sources (MS:333-362)
        r.frag_len = flen[p];
        r.frag_off = (pr.ir_frag >= 0 && pr.ir_frag < n_irs) ? ir_off[pr.ir_frag] : 0;
        if (pr.gen_mode == MSG_GEN_IMAGE && pr.image >= 0) {
            if (pr.image >= n_images || !images) return fail(ctx, MSG_E_ARG, "bad image index");
            r.img_off = img_off[pr.image];
            r.img_h = img_h[pr.image];
            r.img_w = img_w[pr.image];
            if (r.img_h <= 0 || r.img_w <= 0) return fail(ctx, MSG_E_ARG, "empty image");
        }
        // ADSR (MS:173-177); A > n raises ValueError in the reference (MS:182)
        const double sr = (double)pr.base_sr;
        const int64_t A = std::max<int64_t>(0, (int64_t)std::nearbyint(sr * pr.env_a / 1000.0));
        const int64_t D = std::max<int64_t>(0, (int64_t)std::nearbyint(sr * pr.env_d / 1000.0));
        const int64_t R = std::max<int64_t>(0, (int64_t)std::nearbyint(sr * pr.env_r / 1000.0));
        if (A > inf.out_n)
            return fail(ctx, MSG_E_VALUE, "could not broadcast input array from shape (" + std::to_string(A) +
                                              ",) into shape (" + std::to_string(inf.out_n) + ",)");
        r.envA = (int32_t)A; r.envD = (int32_t)std::min<int64_t>(D, INT32_MAX);
        r.envR = (int32_t)std::min<int64_t>(R, INT32_MAX);
        r.envS = (float)std::min(std::max(pr.env_s, 0.0), 1.0);
        r.envC = (float)std::max(1e-6, pr.env_curve);
        {
            const int64_t n = inf.out_n;
            const int64_t j = std::min<int64_t>(n, A + D);
            const int64_t s1 = std::max<int64_t>(j, n - R);
            r.envJ = (int32_t)j;
            r.envS1 = (int32_t)s1;
            r.envInvA = A > 0 ? (float)(1.0 / (double)A) : 0.f;
            r.envInvD = j > A ? (float)(1.0 / (double)(j - A)) : 0.f;
            r.envInvR = n - s1 > 1 ? (float)(1.0 / (double)(n - s1 - 1)) : 0.f;
        }
        // space FIR
        const bool er = (pr.flags & MSG_F_ER_CLOUD) != 0;
        const int ic = pr.ir_conv;
        const bool ir = (pr.flags & MSG_F_SPACE_IR) && ic >= 0 && ir_lens[ic] > 0;   // size<8 check: caller
        r.ir_len = ir ? (int32_t)std::min<int64_t>(ir_lens[ic], 8192) : 0;
        r.ir_off = ir ? ir_off[ic] : 0;
        r.fir_on = (er || ir) ? 1 : 0;
        r.fir_block_begin = fblocks;   // prefix arrays must stay monotone for find_preset
        r.h_block_begin = hblocks;
        r.h_fir4 = 0;
        if (r.fir_on) {
            const int64_t M = pick[p].M;
            const int N = pick[p].N, Pp = pick[p].P, Q = pick[p].Q;
            const bool stream = pick[p].stream;
            if (N != FIR8_N) {                     // runtime plan for k_fir_h (k_fir8 has its own engine)
                std::string why;
                const int fp = real_plan(ctx->fir_plans, N, why);
                if (fp < 0) return fail(ctx, MSG_E_DEVICE, "FIR plan: " + why);
                fir_plan_of[p] = fp;
                fir_lds = std::max(fir_lds, ctx->fir_plans.host[fp].lds_bytes);
            }
            r.fir_N = N; r.fir_P = Pp; r.fir_Q = Q; r.fir_B = stream ? Pp : N - Pp + 1;
            r.h_off = hsum;
            r.h_len = (int32_t)M;
            h_tile_begin[p] = htiles;
            if (N == FIR8_N) {
                // one partition: H = rfft(delta + ER taps) . S_IR straight into the spectrum
                // (k_fir8_hconv), or the IR's spectrum itself for an IR-only preset
                r.h_fir4 = 2;
                const bool er = (pr.flags & MSG_F_ER_CLOUD) != 0;
                int64_t irs = -1;
                if (r.ir_len > 0) {
                    auto it = ir8_spec_of.find(pr.ir_conv);
                    if (it == ir8_spec_of.end()) {
                        it = ir8_spec_of.emplace(pr.ir_conv, ir8_sum).first;
                        ir8_jobs.insert(ir8_jobs.end(), {r.ir_off, (int64_t)r.ir_len, ir8_sum, 0});
                        ir8_sum += (N / 2 + 1 + 15) & ~15;
                    }
                    irs = it->second;
                }
                if (er) {
                    r.irs_off = irs;
                    fir8_list.push_back(p);
                } else {
                    r.h_off = irs;                 // relocated past the per-preset spectra below
                    ir_only8.push_back(p);
                }
            } else if (N == 2 * 16384 && ctx->fir4 && ctx->fir4c && Q == 1 && M <= N) {
                // one partition on k_fir4: the k_fir8_hconv recipe at N = 32768 (fir4_fft.h),
                // H = rfft(delta + ER taps) . S_IR, or S_IR itself for an IR-only preset
                r.h_fir4 = 3;
                const bool er = (pr.flags & MSG_F_ER_CLOUD) != 0;
                int64_t irs = -1;
                if (r.ir_len > 0) {
                    auto it = ir4_spec_of.find(pr.ir_conv);
                    if (it == ir4_spec_of.end()) {
                        it = ir4_spec_of.emplace(pr.ir_conv, ir4_sum).first;
                        ir4_jobs.insert(ir4_jobs.end(), {r.ir_off, (int64_t)r.ir_len, ir4_sum, 0});
                        ir4_sum += (N / 2 + 1 + 15) & ~15;
                    }
                    irs = it->second;
                }
                if (er) {
                    r.irs_off = irs;
                    fir4c_list.push_back(p);
                } else {
                    r.h_off = irs;                 // relocated past the per-preset spectra below
                    ir_only4.push_back(p);
                }
            } else {                               // h in the time domain (k_h_build), cut into partitions
                r.hs_off = hs_sum;
                hs_sum += (M + 3) & ~int64_t(3);    // 16-byte aligned h regions
                htiles += (int32_t)((M + H_BUILD_TILE - 1) / H_BUILD_TILE);
                if (N == 2 * 16384 && ctx->fir4) {   // k_fir4_hpart
                    r.h_fir4 = 1;
                    for (int q = 0; q < Q; ++q) hpart_jobs.push_back(make_int2(p, q));
                }
            }
            const int32_t nblk = (int32_t)((inf.out_n + r.fir_B - 1) / r.fir_B);
            // the overlap-add in k_fir8p's segment loads: each segment sums its grains
            // again (N / B ~ 1.6 times per frame), worth it while the grains are sparse
            if (N == FIR8_N && !stream && batch_ola) {
                r.ola_fir = 1;
                n_ola_fir++;
                ola_fir_nmax = std::max<int64_t>(ola_fir_nmax, inf.out_n);
            }
            if (stream) {
                fir4s_presets.push_back(make_int2(p, nblk));   // jobs cut once the batch's total is known
            } else {
                std::vector<int2>& fj = fjobs_by[N == FIR8_N ? 6 : __builtin_ctz(N) - 11];
                for (int32_t b = 0; b < nblk; ++b) fj.push_back(make_int2(p, b));
            }
            fblocks += nblk;
            hblocks += Q;
            if (!r.h_fir4) hblocks_gen += Q;
            // each preset's spectra start on a 128-byte boundary (N / 2 + 1 float2 per
            // partition is odd: unpadded, every other preset's He straddled one more
            // cache line per wave-wide load)
            // (N = 65536: one spectrum of FIR8_HSTRIDE float2, Ho 128-byte aligned inside it)
            static_assert(((FIR8_N / 2 + 1 + 15) & ~15) == FIR8_HSTRIDE, "fir8 spectrum stride");
            if (!((N == FIR8_N || r.h_fir4 == 3) && r.ir_len > 0 && !(pr.flags & MSG_F_ER_CLOUD)))
                hsum += ((int64_t)Q * (N / 2 + 1) + 15) & ~int64_t(15);
        } else {
            h_tile_begin[p] = htiles;
        }
        fir_begin[p] = r.fir_block_begin;
        h_begin[p] = r.h_block_begin;
        // stereo (MS:423-436)
        const double w = std::min(std::max(pr.stereo_width, 0.0), 1.0);
        const bool stereo = (pr.flags & MSG_F_STEREO) && inf.out_n >= 64;
        r.stereo_fir = stereo ? 1 : 0;
        if (stereo && (inf.out_n % 2)) {      // full-length rotation through Bluestein (kernels_stereo_odd.h)
            const int64_t M = stereo_odd_len(inf.out_n, ctx->so_row, ctx->so_col);
            if (M < 0)
                return fail(ctx, MSG_E_UNSUPPORTED, "stereo diffusion of an odd output beyond the 2^34-point transform");
            r.stereo_fir = 2;
            r.r2_off = r2_sum;
            r2_sum += (inf.out_n + 3) & ~int64_t(3);
            so_M = std::max(so_M, M);
            odd_presets.push_back(p);
        }
        r.dl = (int32_t)std::nearbyint((1 + 7 * w) * 0.0005 * sr);
        r.dr = (int32_t)std::nearbyint((1 + 9 * w) * 0.0007 * sr);
        std::memcpy(r.bess, pick[p].bess, sizeof(r.bess));
        r.drive = (float)pr.sat_drive;
        r.peak = (float)pr.peak;
        st_begin[p] = stiles;
        st_count[p] = (int32_t)((inf.out_n + ST_TILE - 1) / ST_TILE);
        stiles += st_count[p];
        {   // the float64 FIR's shape (kernels_fir64.h), for every FIR preset
            Fir64Rt& f = f64rt[p];
            f.h_len = r.fir_on ? (int32_t)pick[p].M : 0;
            f.q = (f.h_len + FIR64_P - 1) / FIR64_P;
            f.blocks = (int32_t)((inf.out_n + FIR64_B - 1) / FIR64_B);
            f.st_tiles = st_count[p];
            if (r.fir_on) {
                f64_cand++;
                f64_hmax = std::max<int64_t>(f64_hmax, f.h_len);
                f64_qmax = std::max(f64_qmax, f.q);
                f64_bmax = std::max(f64_bmax, f.blocks);
                f64_stmax = std::max(f64_stmax, f.st_tiles);
            }
        }
        if (!r.ola_fir) tiles += (int32_t)((inf.out_n + OLA_TILE - 1) / OLA_TILE);
        pool += (inf.pool_len + 3) & ~int64_t(3);   // 16-byte aligned grain regions (float4 loads)
        ysum += (inf.out_n + 3) & ~int64_t(3);   // keep every mono region 16-byte aligned
        // events
        bool precise = is_precise(pr);
        if (!precise) {
            // grains beyond the LDS-resident float32 spectral kernels run the float64
            // chain in global memory (micro_ms up to 80 ms at 30 MHz: 2.4 M samples)
            int last_n = -1;
            for (int k = 0; k < inf.n_events && !precise; ++k) {
                const msg_event& e = ctx->h_events[slot_base[p] + k];
                if (!spec_ops(pr, e) || e.n == last_n) continue;   // each spectral grain length once
                last_n = e.n;
                if (use_ct && spectral_ct_plan(e.n) >= 0) continue;
                std::string why;
                const int pi = real_plan(ctx->grain_plans, e.n, why);
                if (pi < 0) return fail(ctx, MSG_E_DEVICE, "grain plan: " + why);
                const RealPlan& gp = ctx->grain_plans.host[pi];
                if (gp.lds_bytes > LDS_MAX || gp.c.size > SPEC_M_BIG) precise = true;
            }
        }
        if (precise && inf.n_events > 0) {
            const bool chained = (pr.flags & (MSG_F_EVENT_FEEDBACK | MSG_F_IMPRINT)) != 0;
            bool chain_global = false;
            if (chained) {
                Chain64 c;
                memset(&c, 0, sizeof(c));
                c.preset = p;
                c.ev_begin = (int32_t)ev64.size();
                c.n_events = inf.n_events;
                c.prev_off = state_sum;
                c.mem_off = state_sum + ((inf.max_n + 1) & ~1);
                state_sum += ((inf.max_n + 1) & ~1) + ((inf.max_n / 2 + 2) & ~1);
                chains.push_back(c);
            }
            const size_t ev_first = ev64.size();
            for (int k = 0; k < inf.n_events; ++k) {
                const int ei = slot_base[p] + k;
                const msg_event& e = ctx->h_events[ei];
                memset(&ert[ei], 0, sizeof(EventRt));
                Ev64 v;
                memset(&v, 0, sizeof(v));
                std::string why;
                v.plan = real64_plan(ctx->plans64, e.n, why);
                if (v.plan < 0) return fail(ctx, MSG_E_DEVICE, "float64 grain plan: " + why);
                const Real64Plan& gp = ctx->plans64.host[v.plan];
                if (gp.cap > G64_SLOTS) {        // beyond the LDS engine: a global-memory slot
                    g64_big_cap = std::max<int64_t>(g64_big_cap, gp.cap);
                    g64_glb.push_back((int32_t)ev64.size());
                    chain_global = true;
                } else {
                    g64_cap = std::max(g64_cap, gp.cap);
                    g64_lds.push_back((int32_t)ev64.size());
                }
                v.ops = g64_ops(pr, e);
                if (stop_cep && (v.ops & G64_CEP))   // debug: the grain as cepstral_warp receives it
                    v.ops &= G64_LOWPASS | G64_WARP | G64_CHAIN;
                v.n = e.n;
                v.n0 = msgplan::grain_len(e.gen_sr, pr.micro_ms, 16);
                v.gen_sr = e.gen_sr;
                v.preset = p;
                v.index = e.index;
                v.ei = ei;
                v.off64 = sum64;
                v.grain_off = r.pool_base + e.pool_off;
                v.cutoff_gen = e.cutoff_out * e.ufac;
                v.stretch = e.stretch;
                if (v.ops & G64_CEP) { v.save_off = save_sum; save_sum += e.n / 2 + 1; }
                if (pr.gen_mode == MSG_GEN_WAVELET) {
                    // morlet_atom is max(16, round(..)) long, the grain max(128, ..): shorter
                    // atoms do not broadcast into the grain (MS:319, 166, 329)
                    const int na = msgplan::grain_len(e.gen_sr, pr.micro_ms, 16);
                    if (na < e.n)
                        return fail(ctx, MSG_E_VALUE, "operands could not be broadcast together with shapes (" +
                                                          std::to_string(e.n) + ",) (" + std::to_string(na) +
                                                          ",) (" + std::to_string(e.n) + ",)");
                }
                if (normal_driven(pr.gen_mode)) {
                    gen64_list.push_back(ei);
                    gen64_off.push_back(sum64);
                }
                sum64 += (e.n + 1) & ~1;
                last64[p] = (int32_t)ev64.size();
                ev64.push_back(v);
            }
            (void)ev_first;
            if (chained && chain_global) {                  // the chain walks big grains too
                chains_glb.push_back(chains.back());
                chains.pop_back();
            }
            continue;
        }
        f32_presets.push_back(p);
    }
    const auto hB = hclock::now();
    // ---- float32-chain event records (EventRt), presets in parallel on the host
    // pool; the per-kernel event lists are concatenated in preset order.  Events
    // that need a runtime FFT plan (no compile-time plan for their length) are
    // planned afterwards on this thread (the plan cache is not shared).
    struct F32Lists { std::vector<int32_t> gen, s3, ct[SPEC_CT_PLANS], small, pending; };
    std::vector<F32Lists> f32l(f32_presets.size());
    HostPool::get().run((int)f32_presets.size(), [&](int i) {
        const int p = f32_presets[i];
        const msg_preset& pr = presets[p];
        const PresetRt& r = prt[p];
        F32Lists& L = f32l[i];
        const double tilt = pr.gen_mode == MSG_GEN_FALLBACK ? -3.0 : pr.noise_tilt;
        const double tilt_alpha = std::log(std::pow(10.0, tilt / 20.0)) / std::log(2.0);
        const double env_tau = std::max(1e-6, (pr.micro_ms / 1000.0) * (pr.gen_mode == MSG_GEN_SKEWED ? 0.2 : 0.25));
        const int ne = info[p].n_events;
        L.gen.reserve(ne);
        for (int k = 0; k < ne; ++k) {
            const int ei = slot_base[p] + k;
            const msg_event& e = ctx->h_events[ei];
            EventRt& x = ert[ei];
            memset(&x, 0, sizeof(x));
            x.n = e.n;
            x.gen_sr = e.gen_sr;
            x.ops = spec_ops(pr, e);
            x.cutoff_gen = e.cutoff_out * e.ufac;
            x.roll = pr.bandlimit_roll_hz;
            x.stretch = e.stretch;
            x.tilt_alpha = tilt_alpha;
            x.env_tau = env_tau;
            x.warp_power = pr.nl_warp_power;
            L.gen.push_back(ei);
            const int ctp = (x.ops && use_ct) ? spectral_ct_plan(e.n) : -1;
            if (use_s3 && x.ops &&
                spec3_eligible(e.n, x.ops, x.gen_sr, x.cutoff_gen, x.roll, x.stretch, r.pool_base + e.pool_off,
                               &x.s3_kb, &x.s3_kz, &x.s3_ky, &x.s3_inv_f, &x.s3_pad))
                L.s3.push_back(ei);
            else if (ctp >= 0)
                L.ct[ctp].push_back(ei);
            else if (x.ops)
                L.pending.push_back(ei);
            else
                L.small.push_back(ei);
        }
    });
    for (F32Lists& L : f32l) {
        gen_list.insert(gen_list.end(), L.gen.begin(), L.gen.end());
        spec3.insert(spec3.end(), L.s3.begin(), L.s3.end());
        for (int c = 0; c < SPEC_CT_PLANS; ++c) spec_ct[c].insert(spec_ct[c].end(), L.ct[c].begin(), L.ct[c].end());
        spec_small.insert(spec_small.end(), L.small.begin(), L.small.end());
        for (int ei : L.pending) {
            EventRt& x = ert[ei];
            std::string why;
            const int pi = real_plan(ctx->grain_plans, x.n, why);
            if (pi < 0) return fail(ctx, MSG_E_DEVICE, "grain plan: " + why);
            x.plan = pi;
            const RealPlan& gp = ctx->grain_plans.host[pi];
            if (gp.lds_bytes <= SPEC_SMALL_BYTES && gp.c.size <= SPEC_M_SMALL) {
                spec_small.push_back(ei);
                spec_small_lds = std::max(spec_small_lds, gp.lds_bytes);
            } else if (gp.lds_bytes <= LDS_MAX && gp.c.size <= SPEC_M_BIG) {
                spec_big.push_back(ei);
                spec_big_lds = std::max(spec_big_lds, gp.lds_bytes);
            } else {
                return fail(ctx, MSG_E_UNSUPPORTED, "grain of " + std::to_string(x.n) +
                            " samples exceeds the LDS-resident FFT (even n <= ~39900)");
            }
        }
    }
    const auto hC = hclock::now();
    int f64_plan = -1;                                   // the float64 FIR's transform (kernels_fir64.h)
    if (ctx->fir64 > 0 && f64_cand > 0) {
        std::string why;
        f64_plan = real64_plan(ctx->plans64, FIR64_N, why);
        if (f64_plan < 0) return fail(ctx, MSG_E_DEVICE, "float64 FIR plan: " + why);
    }
    HIPCHK(ctx, sync_plans(ctx->grain_plans, s));
    HIPCHK(ctx, sync_plans(ctx->fir_plans, s));
    HIPCHK(ctx, sync_plans(ctx->plans64, s));
    std::vector<int32_t> g64_list(g64_lds);
    g64_list.insert(g64_list.end(), g64_glb.begin(), g64_glb.end());
    const size_t n_lds_chains = chains.size();
    chains.insert(chains.end(), chains_glb.begin(), chains_glb.end());
    // global slots: persistent workgroups, at most ~8 GB of grain + scratch buffers
    G64Global gg{};
    unsigned g_grid = 0, c_grid = 0;
    if (!g64_glb.empty() || !chains_glb.empty()) {
        int64_t cap = g64_big_cap;
        for (const Chain64& c : chains_glb)
            for (int q = 0; q < c.n_events; ++q)
                cap = std::max<int64_t>(cap, ctx->plans64.host[ev64[c.ev_begin + q].plan].cap);
        gg.slot_cap = (cap + 1) & ~int64_t(1);
        gg.mask_words = gg.slot_cap / 32 + 2;
        const int64_t per_slot = 2 * gg.slot_cap * 16 + gg.mask_words * 4;
        const int64_t lim = std::max<int64_t>(1, std::min<int64_t>(1024, (int64_t(8) << 30) / per_slot));
        g_grid = (unsigned)std::min<int64_t>((int64_t)g64_glb.size(), lim);
        c_grid = (unsigned)std::min<int64_t>((int64_t)chains_glb.size(), lim);
        const int64_t slots = std::max<int64_t>(std::max(g_grid, c_grid), 1);
        HIPCHK(ctx, ctx->g64A.ensure(slots * gg.slot_cap));
        HIPCHK(ctx, ctx->g64B.ensure(slots * gg.slot_cap));
        HIPCHK(ctx, ctx->g64mask.ensure(slots * gg.mask_words));
        gg.A = ctx->g64A.p;
        gg.B = ctx->g64B.p;
        gg.mask = ctx->g64mask.p;
    }
    HIPCHK(ctx, ctx->micro64.ensure(sum64));
    HIPCHK(ctx, ctx->grain64.ensure(sum64));
    HIPCHK(ctx, ctx->save64.ensure(save_sum));
    HIPCHK(ctx, ctx->state64.ensure(state_sum));
    HIPCHK(ctx, ctx->so_r2.ensure(r2_sum));
    HIPCHK(ctx, ctx->so_A.ensure(so_M));
    // k_fir4s: each workgroup walks fir4s_k consecutive blocks of one preset
    for (const int2& pb : fir4s_presets)
        for (int32_t b = 0; b < pb.y; b += fir4s_k) fjobs_by[5].push_back(make_int2(pb.x, b));
    std::vector<int2> fir_jobs;
    int32_t fjob_off[8] = {0};
    for (int i = 0; i < 7; ++i) {
        fjob_off[i] = (int32_t)fir_jobs.size();
        fir_jobs.insert(fir_jobs.end(), fjobs_by[i].begin(), fjobs_by[i].end());
    }
    fjob_off[7] = (int32_t)fir_jobs.size();
    // the fused overlap-add's first event per k_fir8p block: the events of a
    // preset are sorted by start, so one moving index per preset finds, block by
    // block, the first event starting after the segment's start - max_n
    std::vector<int32_t> fir_lo;
    if (n_ola_fir > 0) {
        const std::vector<int2>& fj = fjobs_by[6];
        fir_lo.resize(fj.size());
        int cur_p = -1, k = 0;
        for (size_t j = 0; j < fj.size(); ++j) {
            const int p = fj[j].x;
            if (p != cur_p) { cur_p = p; k = 0; }
            const PresetRt& r = prt[p];
            const int64_t lim = (int64_t)fj[j].y * r.fir_B - (r.fir_P - 1) - (int64_t)r.max_n;
            const msg_event* ev = ctx->h_events.data() + r.ev_begin;
            if (fj[j].y == 0) k = 0;
            while (k < r.n_events && (int64_t)ev[k].start <= lim) ++k;
            fir_lo[j] = k;
        }
    }
    HIPCHK(ctx, ctx->micro.ensure(pool));
    HIPCHK(ctx, ctx->grain.ensure(pool));
    HIPCHK(ctx, ctx->mono_a.ensure(ysum));
    HIPCHK(ctx, ctx->mono_y.ensure(ysum));
    // the IR spectra of the k_fir8 presets follow the per-preset spectra in hspec
    for (int p : fir8_list)
        if (prt[p].ir_len > 0) prt[p].irs_off += hsum;
    for (int p : ir_only8) prt[p].h_off += hsum;
    for (size_t j = 0; j < ir8_jobs.size(); j += 4) ir8_jobs[j + 2] += hsum;
    // then the k_fir4_hconv presets' IR spectra
    for (int p : fir4c_list)
        if (prt[p].ir_len > 0) prt[p].irs_off += hsum + ir8_sum;
    for (int p : ir_only4) prt[p].h_off += hsum + ir8_sum;
    for (size_t j = 0; j < ir4_jobs.size(); j += 4) ir4_jobs[j + 2] += hsum + ir8_sum;
    HIPCHK(ctx, ctx->hspec.ensure(hsum + ir8_sum + ir4_sum));
    HIPCHK(ctx, ctx->hscratch.ensure(hs_sum));
    auto h2d = [&](auto** dst, const auto* src, size_t bytes) -> hipError_t {
        ctx->staging.add(dst, src, bytes);    // copied at the flush below, one copy for all
        return hipSuccess;
    };
    for (int p = 0; p < P; ++p) tile_begin[p] = prt[p].tile_begin;
    HIPCHK(ctx, h2d(&ctx->ert.p, ert, sizeof(EventRt) * nslots));
    HIPCHK(ctx, h2d(&ctx->prt.p, prt.data(), sizeof(PresetRt) * P));
    HIPCHK(ctx, h2d(&ctx->gen_list.p, gen_list.data(), sizeof(int32_t) * gen_list.size()));
    HIPCHK(ctx, h2d(&ctx->spec_small.p, spec_small.data(), sizeof(int32_t) * spec_small.size()));
    HIPCHK(ctx, h2d(&ctx->spec_big.p, spec_big.data(), sizeof(int32_t) * spec_big.size()));
    std::vector<int32_t> ct_list;
    int32_t ct_off[SPEC_CT_PLANS + 1] = {0};
    for (int i = 0; i < SPEC_CT_PLANS; ++i) {
        ct_off[i] = (int32_t)ct_list.size();
        ct_list.insert(ct_list.end(), spec_ct[i].begin(), spec_ct[i].end());
    }
    ct_off[SPEC_CT_PLANS] = (int32_t)ct_list.size();
    HIPCHK(ctx, h2d(&ctx->spec3_list.p, spec3.data(), sizeof(int32_t) * spec3.size()));
    HIPCHK(ctx, h2d(&ctx->spec_ct_list.p, ct_list.data(), sizeof(int32_t) * ct_list.size()));
    HIPCHK(ctx, h2d(&ctx->tile_begin.p, tile_begin.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->fir_begin.p, fir_begin.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->fir_jobs.p, fir_jobs.data(), sizeof(int2) * fir_jobs.size()));
    HIPCHK(ctx, h2d(&ctx->fir_lo.p, fir_lo.data(), sizeof(int32_t) * fir_lo.size()));
    HIPCHK(ctx, h2d(&ctx->h_begin.p, h_begin.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->st_begin.p, st_begin.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->fir_plan_of.p, fir_plan_of.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->irbank.p, irbank.data(), sizeof(double) * irbank.size()));
    HIPCHK(ctx, h2d(&ctx->h_tile_begin.p, h_tile_begin.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->fir8_list.p, fir8_list.data(), sizeof(int32_t) * fir8_list.size()));
    HIPCHK(ctx, h2d(&ctx->ir8_jobs.p, ir8_jobs.data(), sizeof(int64_t) * ir8_jobs.size()));
    HIPCHK(ctx, h2d(&ctx->fir4c_list.p, fir4c_list.data(), sizeof(int32_t) * fir4c_list.size()));
    HIPCHK(ctx, h2d(&ctx->ir4_jobs.p, ir4_jobs.data(), sizeof(int64_t) * ir4_jobs.size()));
    HIPCHK(ctx, h2d(&ctx->hpart_jobs.p, hpart_jobs.data(), sizeof(int2) * hpart_jobs.size()));
    if (ctx->maxbits_zero.size() < (size_t)P) ctx->maxbits_zero.assign((size_t)P, 0u);
    HIPCHK(ctx, h2d(&ctx->maxbits.p, ctx->maxbits_zero.data(), sizeof(unsigned) * P));   // zeros in the one upload, no fill launch
    // the float64 FIR chain: slots for up to FIR64_CAP flagged presets of the batch
    const bool f64_on = ctx->fir64 > 0 && f64_cand > 0;
    const int64_t f64_hstride = (f64_hmax + 3) & ~int64_t(3);
    const int64_t f64_hsstride = (int64_t)f64_qmax * FIR64_K;
    // slots per window: every flagged preset is served, FIR64_WINDOW_BYTES of h and H_q at a time
    const int64_t f64_slot_bytes = f64_hstride * (int64_t)sizeof(float) + f64_hsstride * (int64_t)sizeof(double2);
    const int f64_cap = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(f64_cand, ctx->fir64_cap),
                                                                     FIR64_WINDOW_BYTES / std::max<int64_t>(1, f64_slot_bytes)));
    if (f64_on) {
        HIPCHK(ctx, ctx->f64_stats.ensure(2 * (size_t)P));
        HIPCHK(ctx, ctx->f64_flag.ensure(P));
        HIPCHK(ctx, ctx->st_part.ensure(2 * (size_t)stiles));
        HIPCHK(ctx, ctx->f64_slot_preset.ensure(f64_cand));
        HIPCHK(ctx, ctx->f64_nslots.ensure(1));
        HIPCHK(ctx, ctx->f64_h.ensure((size_t)(f64_cap * f64_hstride)));
        HIPCHK(ctx, ctx->f64_hs.ensure((size_t)(f64_cap * f64_hsstride)));
        HIPCHK(ctx, h2d(&ctx->f64rt.p, f64rt.data(), sizeof(Fir64Rt) * P));
    }
    const int32_t n_odd = (int32_t)odd_presets.size();
    HIPCHK(ctx, h2d(&ctx->st_count.p, st_count.data(), sizeof(int32_t) * P));
    HIPCHK(ctx, h2d(&ctx->odd_list.p, odd_presets.data(), sizeof(int32_t) * odd_presets.size()));
    HIPCHK(ctx, h2d(&ctx->odd_cnt.p, &n_odd, sizeof(int32_t)));
    HIPCHK(ctx, h2d(&ctx->ev64.p, ev64.data(), sizeof(Ev64) * ev64.size()));
    HIPCHK(ctx, h2d(&ctx->g64_list.p, g64_list.data(), sizeof(int32_t) * g64_list.size()));
    HIPCHK(ctx, h2d(&ctx->gen64_list.p, gen64_list.data(), sizeof(int32_t) * gen64_list.size()));
    HIPCHK(ctx, h2d(&ctx->gen64_off.p, gen64_off.data(), sizeof(int64_t) * gen64_off.size()));
    HIPCHK(ctx, h2d(&ctx->chains.p, chains.data(), sizeof(Chain64) * chains.size()));
    HIPCHK(ctx, h2d(&ctx->imgbank.p, imgbank.data(), imgbank.size()));
    const auto h2 = hclock::now();
    HIPCHK(ctx, ctx->staging.flush(s));
    // the merged ER gains (host batch path): k_er_gains runs first in
    // launch_h_spectra, before every filter kernel that reads them (the float64
    // FIR's k_h64 comes later still), so it does not hold up the generator
    const double* erg = ctx->er_gain.p;
    if (er_dev) {
        HIPCHK(ctx, ctx->er_gain_d.ensure((size_t)std::max<int64_t>(1, ntaps)));
        HIPCHK(ctx, ctx->er_tap_d.ensure((size_t)std::max<int64_t>(1, ntaps)));
        erg = ctx->er_gain_d.p;
    }
    if (ctx->prof_batch) {
        const auto h3 = hclock::now();
        ctx->host_sum[0] += std::chrono::duration<double, std::milli>(h1 - h0).count();
        ctx->host_sum[1] += std::chrono::duration<double, std::milli>(h2 - h1).count();
        ctx->host_sum[2] += std::chrono::duration<double, std::milli>(h3 - h2).count();
        ctx->host_sum[3] += std::chrono::duration<double, std::milli>(hA - h0).count();
        ctx->host_sum[4] += std::chrono::duration<double, std::milli>(h1 - hA).count();
        ctx->host_sum[5] += std::chrono::duration<double, std::milli>(hB - h1).count();
        ctx->host_sum[6] += std::chrono::duration<double, std::milli>(hC - hB).count();
        ctx->host_sum[7] += std::chrono::duration<double, std::milli>(h2 - hC).count();
        ctx->ola_fir_sum += n_ola_fir;
        ++ctx->host_cnt;
    }

    // The filter spectra depend on the presets' taps and IRs only, not on the
    // audio: launched before the generator (h_early), they run while
    // the GPU holds the other streams' earlier stages, instead of queueing
    // behind a persistent k_fir8p of another stream that holds every CU
    // (C5's fir_h window had been ~100x its isolated time).
    auto launch_h_spectra = [&]() -> int {
        if (er_dev && ntaps > 0) {
            hipLaunchKernelGGL(k_er_gains, dim3((unsigned)P), dim3(ER_T), 0, s, ctx->presets.p, ctx->prt.p, P,
                               ctx->er_key.p, ctx->er_first.p, ctx->er_cnt.p, ctx->er_tap_d.p, ctx->er_gain_d.p);
            HIPCHK(ctx, hipGetLastError());
        }
        if (htiles > 0)
            HIPCHK(ctx, launch_h_build((unsigned)htiles, s, ctx->prt.p, ctx->h_tile_begin.p, P, ctx->er_off.p,
                                       erg, ctx->irbank.p, ctx->hscratch.p));
        if (!ir8_jobs.empty())
            HIPCHK(ctx, launch_fir8_spec64((unsigned)(ir8_jobs.size() / 4), s, ctx->ir8_jobs.p, ctx->d_fir4tab,
                                           ctx->irbank.p, ctx->hspec.p));
        if (!hpart_jobs.empty())
            HIPCHK(ctx, launch_fir4_hpart(16384, (unsigned)hpart_jobs.size(), s, ctx->prt.p, ctx->hpart_jobs.p,
                                          ctx->d_fir4tab, ctx->hscratch.p, ctx->hspec.p));
        if (!fir8_list.empty())
            HIPCHK(ctx, launch_fir8_hconv((unsigned)fir8_list.size(), s, ctx->prt.p, ctx->fir8_list.p, ctx->d_fir4tab,
                                          ctx->er_off.p, erg, ctx->hspec.p));
        if (!ir4_jobs.empty())
            HIPCHK(ctx, launch_fir4_irspec((unsigned)(ir4_jobs.size() / 4), s, ctx->ir4_jobs.p, ctx->d_fir4tab,
                                           ctx->irbank.p, ctx->hspec.p));
        if (!fir4c_list.empty())
            HIPCHK(ctx, launch_fir4_hconv((unsigned)fir4c_list.size(), s, ctx->prt.p, ctx->fir4c_list.p, ctx->d_fir4tab,
                                          ctx->er_off.p, erg, ctx->hspec.p));
        if (hblocks_gen > 0)   // blocks of k_fir4/k_fir8-engine presets return at once
            HIPCHK(ctx, launch_fir_h((unsigned)hblocks, fir_lds, s, ctx->prt.p, ctx->h_begin.p, P,
                                     ctx->fir_plans.dev.p, ctx->fir_plan_of.p, ctx->hscratch.p, ctx->hspec.p));
        return MSG_OK;
    };
    int64_t fir_nmax = 0;
    for (int p = 0; p < P; ++p)
        if (prt[p].fir_on) fir_nmax = std::max<int64_t>(fir_nmax, prt[p].out_n);
    const bool h_early = hblocks > 0 && (ctx->h_early == 1 || (ctx->h_early == 2 && fir_nmax >= ((int64_t)1 << 22)));
    if (h_early) {
        stage_mark(ctx, 10, s);
        if (const int rc = launch_h_spectra()) return rc;
        stage_mark(ctx, 11, s);
    }
    // ---- generate ----
    stage_mark(ctx, 2, s);
    if (!gen_list.empty())
        hipLaunchKernelGGL(k_gen_normal<false>, dim3((unsigned)gen_list.size()), dim3(GEN_T * GEN_K), 0, s,
                           ctx->presets.p, ctx->events.p, ctx->prt.p, ctx->gen_list.p, (int)gen_list.size(),
                           ctx->dzig, ctx->d_jump, ctx->micro.p, (double*)nullptr, (const int64_t*)nullptr);
    HIPCHK(ctx, hipGetLastError());
    if (!gen64_list.empty())   // raw normals of the float64 chain's normal-driven generators
        hipLaunchKernelGGL(k_gen_normal<true>, dim3((unsigned)gen64_list.size()), dim3(GEN_T * GEN_K), 0, s,
                           ctx->presets.p, ctx->events.p, ctx->prt.p, ctx->gen64_list.p, (int)gen64_list.size(),
                           ctx->dzig, ctx->d_jump, ctx->micro.p, ctx->micro64.p, (const int64_t*)ctx->gen64_off.p);
    HIPCHK(ctx, hipGetLastError());
    // ---- spectral chain ----
    stage_mark(ctx, 3, s);
    if (!spec3.empty()) {
        if (ctx->spec3p > 0) HIPCHK(ctx, spec3_counters(ctx, s));
        HIPCHK(ctx, launch_spec3((unsigned)spec3.size(), s, ctx->events.p, ctx->ert.p, ctx->prt.p, ctx->d_spec3_tab,
                                 ctx->spec3_list.p, (int)spec3.size(), ctx->micro.p, ctx->grain.p,
                                 ctx->spec3p > 1 ? ctx->spec3p : (ctx->spec3p > 0 ? ctx->n_cu : 0),
                                 ctx->spec3_ctr.p));
    }
    for (int i = 0; i < SPEC_CT_PLANS; ++i)
        if (ct_off[i + 1] > ct_off[i])
            HIPCHK(ctx, launch_spectral_ct(i, (unsigned)(ct_off[i + 1] - ct_off[i]), s, ctx->events.p, ctx->ert.p,
                                           ctx->prt.p, ctx->d_spec_ct_tab[i], ctx->spec_ct_list.p + ct_off[i],
                                           ct_off[i + 1] - ct_off[i], ctx->micro.p, ctx->grain.p));
    if (!spec_small.empty())
        HIPCHK(ctx, launch_spectral(false, (unsigned)spec_small.size(), spec_small_lds, s, ctx->presets.p,
                                    ctx->events.p, ctx->ert.p, ctx->prt.p, ctx->grain_plans.dev.p, ctx->spec_small.p,
                                    (int)spec_small.size(), ctx->micro.p, ctx->grain.p));
    if (!spec_big.empty())
        HIPCHK(ctx, launch_spectral(true, (unsigned)spec_big.size(), spec_big_lds, s, ctx->presets.p,
                                    ctx->events.p, ctx->ert.p, ctx->prt.p, ctx->grain_plans.dev.p, ctx->spec_big.p,
                                    (int)spec_big.size(), ctx->micro.p, ctx->grain.p));
    if (!g64_lds.empty())
        HIPCHK(ctx, launch_grain64(nullptr, (unsigned)g64_lds.size(), g64_cap * 16, s, ctx->presets.p, ctx->ev64.p,
                                   ctx->prt.p, ctx->plans64.dev.p, ctx->g64_list.p, (int)g64_lds.size(),
                                   ctx->irbank.p, ctx->imgbank.p, ctx->dzig, ctx->micro64.p, ctx->grain64.p,
                                   ctx->save64.p, ctx->grain.p));
    if (!g64_glb.empty())
        HIPCHK(ctx, launch_grain64(&gg, g_grid, 0, s, ctx->presets.p, ctx->ev64.p, ctx->prt.p, ctx->plans64.dev.p,
                                   ctx->g64_list.p + g64_lds.size(), (int)g64_glb.size(), ctx->irbank.p,
                                   ctx->imgbank.p, ctx->dzig, ctx->micro64.p, ctx->grain64.p, ctx->save64.p,
                                   ctx->grain.p));
    if (n_lds_chains > 0)
        HIPCHK(ctx, launch_chain64(nullptr, (unsigned)n_lds_chains, g64_cap * 16, s, ctx->presets.p, ctx->ev64.p,
                                   ctx->chains.p, (int)n_lds_chains, ctx->plans64.dev.p, ctx->grain64.p,
                                   ctx->state64.p, ctx->grain.p));
    if (!chains_glb.empty())
        HIPCHK(ctx, launch_chain64(&gg, c_grid, 0, s, ctx->presets.p, ctx->ev64.p, ctx->chains.p + n_lds_chains,
                                   (int)chains_glb.size(), ctx->plans64.dev.p, ctx->grain64.p, ctx->state64.p,
                                   ctx->grain.p));
    // ---- overlap-add x ADSR ----
    stage_mark(ctx, 4, s);
    if (tiles > 0) {
        hipLaunchKernelGGL(k_ola_env, dim3((unsigned)tiles), dim3(OLA_T), 0, s, ctx->events.p, ctx->prt.p,
                           ctx->tile_begin.p, P, ctx->grain.p, ctx->mono_a.p);
        HIPCHK(ctx, hipGetLastError());
    }
    // ---- FIR (presets without ER/IR pass a through) ----
    stage_mark(ctx, 5, s);
    float* yb = ctx->mono_a.p;
    if (hblocks > 0) {
        if (!h_early)
            if (const int rc = launch_h_spectra()) return rc;
        stage_mark(ctx, 8, s);
        for (int i = 0; i < 7; ++i) {
            if (fjob_off[i + 1] <= fjob_off[i]) continue;
            const unsigned nj = (unsigned)(fjob_off[i + 1] - fjob_off[i]);
            if (i == 6 && ctx->fir8p > 0) {
                // persistent: one workgroup per CU (at most one per block), a multiple of the XCD
                // count.  Long outputs (h_early: milliseconds per launch) leave one CU in eight
                // to the other streams' small kernels, which cannot start beside a k_fir8p
                // workgroup (its VGPRs fill the CU): C5 118.4 - 119.4 ms with 224 of 256 CUs
                // against 118.8 - 124.0 with all of them; C3 keeps every CU
                const int cus = ctx->fir8p_cus > 0 ? std::min(ctx->fir8p_cus, ctx->n_cu)
                                                   : (h_early ? ctx->n_cu - ctx->n_cu / 8 : ctx->n_cu);
                const unsigned grid = (unsigned)std::max(MSG_XCDS, (std::min((int)nj, cus) / MSG_XCDS) * MSG_XCDS);
                HIPCHK(ctx, fir8_counters(ctx, s));
                HIPCHK(ctx, launch_fir8p(nj, grid, s, ctx->prt.p, ctx->fir_jobs.p + fjob_off[i],
                                         ctx->d_fir4tab, ctx->hspec.p, ctx->mono_a.p, ctx->mono_y.p, ctx->fir8_ctr.p,
                                         ctx->fir8p_stagger,
                                         n_ola_fir > 0 ? ctx->events.p : nullptr, ctx->grain.p, ctx->fir_lo.p));
            } else if (i == 6)
                HIPCHK(ctx, launch_fir8(nj, s, ctx->prt.p, ctx->fir_jobs.p + fjob_off[i], ctx->d_fir4tab, ctx->hspec.p,
                                        ctx->mono_a.p, ctx->mono_y.p));
            else if (i == 5)
                HIPCHK(ctx, launch_fir4s(16384, nj, s, ctx->prt.p, ctx->fir_jobs.p + fjob_off[i], ctx->d_fir4tab,
                                         ctx->hspec.p, ctx->mono_a.p, ctx->mono_y.p, fir4s_k));
            else if (i == 4 && ctx->fir4)
                HIPCHK(ctx, launch_fir4(16384, nj, s, ctx->prt.p, ctx->fir_jobs.p + fjob_off[i], ctx->d_fir4tab,
                                        ctx->hspec.p, ctx->mono_a.p, ctx->mono_y.p));
            else
                HIPCHK(ctx, launch_fir2(1024 << i, nj, s, ctx->prt.p, ctx->fir_jobs.p + fjob_off[i],
                                        ctx->d_fir2tab[i], ctx->hspec.p, ctx->mono_a.p, ctx->mono_y.p));
        }
        stage_mark(ctx, 9, s);
        // presets with fir_on == 0 in a mixed batch: copy a -> y
        for (int p = 0; p < P; ++p)
            if (!prt[p].fir_on)
                HIPCHK(ctx, hipMemcpyAsync(ctx->mono_y.p + prt[p].y_off, ctx->mono_a.p + prt[p].y_off,
                                           sizeof(float) * prt[p].out_n, hipMemcpyDeviceToDevice, s));
        yb = ctx->mono_y.p;
    }
    // ---- stereo, tanh, normalise ----
    stage_mark(ctx, 6, s);
    // peak of L (and the float64 FIR's error predictor) over the float32 y; the
    // fused launch also writes the output of every preset it does not defer
    // (float64 FIR slots, odd lengths: k_stereo_out_list below)
    StereoSync sy{};
    HIPCHK(ctx, ensure_zeroed(ctx->st_done, P, s));
    HIPCHK(ctx, ensure_zeroed(ctx->st_ready, P, s));
    sy.done = ctx->st_done.p;
    sy.ready = ctx->st_ready.p;
    sy.flag64 = f64_on ? ctx->f64_flag.p : nullptr;
    sy.part = f64_on ? ctx->st_part.p : nullptr;
    sy.stats = f64_on ? ctx->f64_stats.p : nullptr;
    ctx->st_epoch = ctx->st_epoch % ((1u << 30) - 1) + 1;
    sy.epoch = ctx->st_epoch;
    sy.f64mode = f64_on ? ctx->fir64 : 0;
    int st_tmax = 0;
    for (int p = 0; p < P; ++p) st_tmax = std::max(st_tmax, st_count[p]);
    const bool st_fused = ctx->stereo_fused && st_tmax <= ST_FUSED_MAX_TILES;
    if (st_fused) {
        if (!ctx->st_ctr.p) HIPCHK(ctx, ensure_zeroed(ctx->st_ctr, ST_CTR_N, s));   // every launch leaves them zero
        const unsigned grid = (unsigned)std::max(1, std::min(stiles, ctx->n_cu * ctx->st_wgs));
        HIPCHK(ctx, launch_stereo_fused(grid, (unsigned)stiles, s, ctx->prt.p, ctx->st_begin.p, P, yb, ctx->maxbits.p,
                                        sy, ctx->st_ctr.p, out_dev));
    } else {
        HIPCHK(ctx, launch_stereo_max((unsigned)stiles, s, ctx->prt.p, ctx->st_begin.p, P, yb, ctx->maxbits.p, sy));
        if (f64_on)   // the float64 FIR's predictor per preset, from the tiles' partial sums
            HIPCHK(ctx, launch_stereo_pred((unsigned)P, s, ctx->prt.p, ctx->st_begin.p, stiles, ctx->maxbits.p, sy));
    }
    if (f64_on) {   // flagged presets: the FIR again in float64, y overwritten (kernels_fir64.h)
        Fir64Launch a;
        a.rt = ctx->prt.p; a.n_presets = P; a.flag64 = ctx->f64_flag.p; a.maxbits = ctx->maxbits.p;
        a.slot_preset = ctx->f64_slot_preset.p; a.n_slots = ctx->f64_nslots.p;
        a.n_cand = f64_cand; a.cap = f64_cap;
        a.fr = ctx->f64rt.p; a.tmax = (int)((f64_hmax + H_BUILD_TILE - 1) / H_BUILD_TILE); a.qmax = f64_qmax;
        a.bmax = f64_bmax;
        a.er_off = ctx->er_off.p; a.er_gain = erg; a.irbank = ctx->irbank.p;
        a.h64 = ctx->f64_h.p; a.h_stride = f64_hstride; a.hs64 = ctx->f64_hs.p; a.hs_stride = f64_hsstride;
        a.plans = ctx->plans64.dev.p; a.plan = f64_plan;
        a.lds_bytes = FIR64_K * (int)sizeof(double2);   // the packed transform and its Nyquist slot
        a.x = ctx->mono_a.p; a.y = yb;
        HIPCHK(ctx, launch_fir64_flag(a, s));
        if (n_ola_fir > 0) {   // the flagged ola_fir presets' mono a, which k_fir8p never wrote
            const int tmax = (int)((ola_fir_nmax + OLA_TILE - 1) / OLA_TILE);
            hipLaunchKernelGGL(k_ola_slots, dim3((unsigned)std::min<int64_t>((int64_t)f64_cand * tmax, 1024)),
                               dim3(OLA_T), 0, s, ctx->events.p, ctx->prt.p, ctx->f64_slot_preset.p,
                               ctx->f64_nslots.p, tmax, ctx->grain.p, ctx->mono_a.p);
            HIPCHK(ctx, hipGetLastError());
        }
        HIPCHK(ctx, launch_fir64(a, s));
    }
    ++ctx->batch_serial;
    for (int p : odd_presets) {           // odd out_n: R = irfft(rfft(roll(y, -dr)) . rot) (MS:432-435)
        const int64_t n = info[p].out_n;
        auto it = ctx->so_bp.find(n);
        if (it == ctx->so_bp.end()) {
            // bound the cache (one entry per distinct odd length, for the
            // life of the process): drop least-recently-used spectra of earlier
            // batches while the cache holds more than 1 GiB (hipFree waits for them)
            auto bytes = [&]() {
                size_t b = 0;
                for (auto& kv : ctx->so_bp) b += kv.second.cap * sizeof(double2);
                return b;
            };
            while (bytes() > ((size_t)1 << 30)) {
                int64_t victim = -1;
                uint64_t oldest = ctx->batch_serial;
                for (auto& kv : ctx->so_bp_use)
                    if (kv.second < oldest) { oldest = kv.second; victim = kv.first; }
                if (victim < 0) break;
                ctx->so_bp[victim].release();
                ctx->so_bp.erase(victim);
                ctx->so_bp_use.erase(victim);
            }
            it = ctx->so_bp.emplace(n, DevBuf<double2>()).first;
            HIPCHK(ctx, it->second.ensure(stereo_odd_len(n, ctx->so_row, ctx->so_col)));
            HIPCHK(ctx, launch_stereo_odd_kernel(n, ctx->so_row, ctx->so_col, it->second.p, ctx->so_A.p, s));
        }
        ctx->so_bp_use[n] = ctx->batch_serial;
        const double w = std::min(std::max(presets[p].stereo_width, 0.0), 1.0);
        HIPCHK(ctx, launch_stereo_odd(n, ctx->so_row, ctx->so_col, prt[p].dr, w, yb + prt[p].y_off, it->second.p, ctx->so_A.p,
                                      ctx->so_r2.p + prt[p].r2_off, s));
    }
    int odd_tmax = 0;
    for (int p : odd_presets) odd_tmax = std::max(odd_tmax, st_count[p]);
    if (f64_on)   // the float64 presets' peak from their new y (and R)
        HIPCHK(ctx, launch_stereo_remax((unsigned)std::min<int64_t>((int64_t)f64_cand * f64_stmax, 256), s, ctx->prt.p, ctx->st_count.p,
                                        ctx->f64_slot_preset.p, ctx->f64_nslots.p, f64_stmax, yb, ctx->so_r2.p,
                                        ctx->maxbits.p));
    if (n_odd > 0)   // odd lengths: the peak of the rotated R
        HIPCHK(ctx, launch_stereo_remax((unsigned)std::min<int64_t>((int64_t)n_odd * odd_tmax, 4096), s, ctx->prt.p,
                                        ctx->st_count.p, ctx->odd_list.p, ctx->odd_cnt.p, odd_tmax, yb, ctx->so_r2.p,
                                        ctx->maxbits.p));
    if (st_fused) {   // the deferred presets' output
        if (f64_on)
            HIPCHK(ctx, launch_stereo_out_list((unsigned)std::min<int64_t>((int64_t)f64_cand * f64_stmax, 1024), s, ctx->prt.p,
                                               ctx->st_count.p, ctx->f64_slot_preset.p, ctx->f64_nslots.p, f64_stmax,
                                               yb, ctx->so_r2.p, ctx->maxbits.p, out_dev));
        if (n_odd > 0)
            HIPCHK(ctx, launch_stereo_out_list((unsigned)std::min<int64_t>((int64_t)n_odd * odd_tmax, 4096), s,
                                               ctx->prt.p, ctx->st_count.p, ctx->odd_list.p, ctx->odd_cnt.p, odd_tmax,
                                               yb, ctx->so_r2.p, ctx->maxbits.p, out_dev));
    } else {
        HIPCHK(ctx, launch_stereo_out((unsigned)stiles, s, ctx->prt.p, ctx->st_begin.p, P, yb, ctx->so_r2.p,
                                      ctx->maxbits.p, out_dev));
    }
    stage_mark(ctx, 7, s);
    HIPCHK(ctx, done.finish());
    ctx->h_info = info;
    ctx->h_prt = prt;
    ctx->h_slot_base = slot_base;
    ctx->h_ev64 = ev64;
    ctx->h_last64 = last64;
    ctx->last_n = P;
    if (ctx->prof_batch) {
        ctx->pending[ctx->ev_cur] = true;
        ctx->pending_fir[ctx->ev_cur] = hblocks > 0;
        ctx->pending_h_early[ctx->ev_cur] = h_early;
        ctx->ev_cur ^= 1;
    }
    return MSG_OK;
}

}  // extern "C"
