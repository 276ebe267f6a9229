// plan.h — the render plan: every scalar and random decision of render() that
// precedes synthesis, shared by the host (msg_plan_host, tests) and the device
// planner kernels.  Follows microsound_0.2.1/main_v2.py ("MS"):
//   out_n / design SR                 MS:589-597
//   breakpoint lanes                  MS:452-482, 602-605, 634-637
//   event fields                      MS:507-558, 609-618
//   per-render stream seed+123456     MS:620, 639-642, 742-751
//   grain lengths per generator       MS:221, 273, 285, 305, 319, 337, 352
//   early-reflection taps seed+202    MS:409-417
#pragma once
#include "msg_common.h"
#include "nprng.h"
#include "../../include/msgpu.h"

namespace msgplan {
using nprng::Pcg64;
using nprng::Zig;

constexpr int32_t GEN_SR_CAP = 30000000;

// eval_breakpoints (MS:469-482): piecewise linear, held at the ends.  The lane's
// points are (t, v) pairs in the batch's breakpoint bank, sorted by t on the host
// exactly as parse_breakpoints sorts them (MS:452-467); any number of points.
MSG_HD double eval_bp(const msg_preset& p, const double* bank, int lane, double t, double def) {
    const int n = p.n_bp[lane];
    if (n <= 0) return def;
    const double* B = bank + 2 * (int64_t)p.bp_off[lane];   // B[2i] = t_i, B[2i + 1] = v_i
    if (t <= B[0]) return B[1];
    if (t >= B[2 * (n - 1)]) return B[2 * (n - 1) + 1];
    for (int i = 0; i + 1 < n; ++i) {
        const double t0 = B[2 * i], t1 = B[2 * i + 2];
        if (t0 <= t && t <= t1) {
            const double a = (t - t0) / fmax(1e-12, (t1 - t0));
            return (1 - a) * B[2 * i + 1] + a * B[2 * i + 3];
        }
    }
    return def;
}

// int(np.clip(int(round(base_sr*u)), base_sr, 30e6)) — Python round = half-even = rint.
MSG_HD int32_t design_sr(int32_t base_sr, double u) {
    double r = rint((double)base_sr * u);
    if (r < (double)base_sr) r = (double)base_sr;
    if (r > (double)GEN_SR_CAP) r = (double)GEN_SR_CAP;
    return (int32_t)r;
}

MSG_HD int32_t grain_len(int32_t gen_sr, double micro_ms, int32_t floor_n) {
    const double r = rint((double)gen_sr * micro_ms / 1000.0);
    return r > (double)floor_n ? (int32_t)r : floor_n;
}

// Grain length by generator mode; unchanged through the whole chain (MS:650-727).
MSG_HD int32_t event_grain_len(const msg_preset& p, int32_t gen_sr, int64_t ir_frag_len) {
    switch (p.gen_mode) {
        case MSG_GEN_STICK_SLIP: case MSG_GEN_MICRO_CHAOS: case MSG_GEN_IMAGE:
            return grain_len(gen_sr, p.micro_ms, 64);
        case MSG_GEN_WAVELET:
            return grain_len(gen_sr, p.micro_ms, 128);
        case MSG_GEN_IR_FRAGMENT:
            return grain_len(gen_sr, p.micro_ms, ir_frag_len < 32 ? 16 : 64);
        case MSG_GEN_CRACKLE: {
            // np.convolve(x, ker, "same") returns max(len(x), len(ker)) samples (MS:280-281)
            const int32_t n0 = grain_len(gen_sr, p.micro_ms, 16);
            const int32_t K = p.crackle_kernel > 8 ? p.crackle_kernel : 8;
            return n0 > K ? n0 : K;
        }
        default:
            return grain_len(gen_sr, p.micro_ms, 16);
    }
}

MSG_HD int64_t out_frames(const msg_preset& p) {
    const double r = rint(p.out_dur_s * (double)p.base_sr);
    return r > 1.0 ? (int64_t)r : 1;
}

// Event onsets (MS:507-558).  emit(t) is called in generation order and returns
// false to stop early (only legal where generation order == output order).
// Clustered children are emitted unsorted; the caller sorts (MS:541).
template <class Emit>
MSG_HD void event_times(const msg_preset& p, const Zig& z, Emit&& emit) {
    Pcg64 g = nprng::default_rng((uint64_t)(p.seed + 9999));
    const double rate = p.grains_per_sec;
    const double dur = p.out_dur_s;
    if (p.process == MSG_PROC_SINGLE || rate <= 0) { emit(0.0); return; }
    if (p.process == MSG_PROC_POISSON) {
        double t = 0.0;
        while (t < dur) {
            t += nprng::exponential(g, z, 1.0 / rate);
            if (t < dur && !emit(t)) return;
        }
        return;
    }
    if (p.process == MSG_PROC_CLUSTERED) {
        // Parents are drawn first, then children per parent (MS:527-540). The
        // parent list is regenerated from a stream copy instead of stored.
        const double prate = fmax(0.1, rate / (double)(p.cluster_size > 1 ? p.cluster_size : 1));
        Pcg64 gp = g;
        int64_t nparents = 0;
        double t = 0.0;
        while (t < dur) {
            t += nprng::exponential(gp, z, 1.0 / prate);
            if (t < dur) ++nparents;
        }
        // gp is now positioned after all parent draws: children stream continues there.
        Pcg64 gc = gp;
        const double spread = p.cluster_spread_ms / 1000.0;
        t = 0.0;
        for (int64_t k = 0; k < nparents;) {
            t += nprng::exponential(g, z, 1.0 / prate);
            if (!(t < dur)) continue;   // cannot happen before nparents are seen
            ++k;
            const double u = nprng::uniform(gc, 0.6, 1.4);
            const double kr = rint(u * (double)p.cluster_size);
            const int64_t nk = kr > 1.0 ? (int64_t)kr : 1;
            for (int64_t c = 0; c < nk; ++c) {
                const double tt = t + nprng::normal(gc, z, 0.0, spread);
                if (0.0 <= tt && tt < dur) emit(tt);
            }
        }
        return;
    }
    if (p.process == MSG_PROC_HAWKES) {
        const double dt = 0.002;
        const int64_t nstep = (int64_t)ceil(dur / dt);
        const double decay = exp(-dt / fmax(1e-6, p.hawkes_decay_s));
        double act = 0.0;
        for (int64_t i = 0; i < nstep; ++i) {
            const double t = (double)i * dt;
            act *= decay;
            const double lam = rate + p.hawkes_gain * act * rate;
            const double pr = fmin(0.95, lam * dt);
            if (nprng::next_double(g) < pr) {
                if (!emit(t + nprng::uniform(g, 0.0, dt))) return;
                act += 1.0;
            }
        }
        return;
    }
    // unknown process: no events (MS:558)
}

MSG_HD bool time_order_is_generation_order(const msg_preset& p) {
    return p.process != MSG_PROC_CLUSTERED;
}

// Phase 1: sizes only.  n_slots counts the events that must be materialised
// before truncation (all children for Clustered); pool_len/max_n are bounds
// over those slots.
MSG_HD void plan_sizes(const msg_preset& p, const double* bp, const Zig& z, int64_t ir_frag_len,
                       msg_plan_info& info) {
    info.out_n = out_frames(p);
    const double unfold0 = fmax(1.0, p.time_unfold);
    info.design_sr = design_sr(p.base_sr, unfold0);
    int32_t slots = 0, max_n = 0;
    int64_t pool = 0;
    const bool ordered = time_order_is_generation_order(p);
    const int32_t cap = p.max_grains;
    event_times(p, z, [&](double t) -> bool {
        if (ordered && slots >= cap) return false;
        double uf = eval_bp(p, bp, 1, t, unfold0);
        uf = fmax(1.0, uf);
        const int32_t n = event_grain_len(p, design_sr(p.base_sr, uf), ir_frag_len);
        ++slots;
        pool += n;
        if (n > max_n) max_n = n;
        return !(ordered && slots >= cap);
    });
    info.n_slots = slots;
    info.n_events = slots < cap ? slots : (cap > 0 ? cap : 0);
    info.max_n = max_n;
    info.pool_len = pool;
}

// Insertion sort of ev[0..n) by t0 (Clustered, MS:541); stable like list.sort.
MSG_HD void sort_by_time(msg_event* ev, int32_t n) {
    for (int32_t i = 1; i < n; ++i) {
        const double t = ev[i].t0;
        int32_t j = i - 1;
        while (j >= 0 && ev[j].t0 > t) { ev[j + 1].t0 = ev[j].t0; --j; }
        ev[j + 1].t0 = t;
    }
}

// Phase 2: fill ev[0..n_slots) (times, then per-event fields for the first
// n_events), exact pool offsets, and the ER taps.  sizes_known: info already
// holds this preset's plan_sizes (the host batch path runs phase 1 for every
// preset first); otherwise phase 1 runs here.
MSG_HD void plan_events(const msg_preset& p, const double* bp, const Zig& z, int64_t ir_frag_len, int32_t preset_index,
                        msg_plan_info& info, msg_event* ev, int32_t* er_off, double* er_gain,
                        bool sizes_known = false) {
    if (!sizes_known) plan_sizes(p, bp, z, ir_frag_len, info);
    int32_t k = 0;
    const bool ordered = time_order_is_generation_order(p);
    const int32_t cap = p.max_grains;
    const int32_t slots = info.n_slots;
    event_times(p, z, [&](double t) -> bool {
        if (k >= slots) return false;
        ev[k].t0 = t;
        ++k;
        return !(ordered && k >= cap);
    });
    if (!ordered) sort_by_time(ev, k);
    const int32_t nev = info.n_events;
    const double rate = p.grains_per_sec;
    const double unfold0 = fmax(1.0, p.time_unfold);
    const double ar = p.grain_amp_rand;
    const int64_t out_n = info.out_n;
    const double max_off_d = rint((p.grain_offset_max_ms / 1000.0) * (double)p.base_sr);
    const int64_t max_off = (int64_t)max_off_d;
    Pcg64 g = nprng::default_rng((uint64_t)(p.seed + 123456));
    int64_t pool = 0;
    int32_t max_n = 0;
    for (int32_t i = 0; i < nev; ++i) {
        msg_event& e = ev[i];
        const double t0 = e.t0;
        const double dens = eval_bp(p, bp, 0, t0, rate);
        double uf = eval_bp(p, bp, 1, t0, unfold0);
        const double cut = eval_bp(p, bp, 2, t0, p.bandlimit_out_hz);
        const double st = eval_bp(p, bp, 3, t0, p.partial_stretch);
        double amp = 1.0;
        if (rate > 0) amp *= fmin(fmax(dens / fmax(1e-6, rate), 0.15), 4.0);
        amp *= nprng::uniform(g, 1.0 - ar, 1.0 + ar);
        uf = fmax(1.0, uf);
        const int32_t gsr = design_sr(p.base_sr, uf);
        const int32_t n = event_grain_len(p, gsr, ir_frag_len);
        const double sd = rint(t0 * (double)p.base_sr);
        const int64_t start = (int64_t)sd;
        e.amp = amp;
        e.ufac = uf;
        e.cutoff_out = cut;
        e.stretch = st;
        e.pool_off = pool;
        e.index = i;
        e.preset = preset_index;
        e.gen_sr = gsr;
        e.n = n;
        e.start = (int32_t)(start < out_n ? start : out_n);
        e.offset = 0;
        e.len = 0;
        e.pad = 0;
        pool += n;
        if (n > max_n) max_n = n;
        if (start >= out_n) continue;                 // MS:743-744, before the offset draw
        int64_t off = 0;
        if ((p.flags & MSG_F_GRAIN_OFFSET) && max_off > 0) {
            const int64_t hi = max_off < (int64_t)n ? max_off : (int64_t)n;
            off = nprng::integers(g, 0, hi > 1 ? hi : 1);
        }
        e.offset = (int32_t)off;
        const int64_t avail = (int64_t)n - off;
        const int64_t L = (out_n - start) < avail ? (out_n - start) : avail;
        e.len = L > 0 ? (int32_t)L : 0;
    }
    info.pool_len = pool;
    info.max_n = max_n;
    // early reflections (MS:410-417): uniform delays, then uniform gains, same stream.
    // er_gain null: the offsets only (the host batch path; k_er_gains draws the
    // gains on the device from the same stream positions)
    if (er_off && !er_gain) {
        Pcg64 ge = nprng::default_rng((uint64_t)(p.seed + 202));
        const int32_t ntap = p.er_taps > 1 ? p.er_taps : 1;
        for (int32_t j = 0; j < ntap; ++j) {
            const double d = nprng::uniform(ge, 0.3, p.er_max_ms) / 1000.0;
            er_off[j] = (int32_t)rint(d * (double)p.base_sr);
        }
    }
    if (er_off && er_gain) {
        Pcg64 ge = nprng::default_rng((uint64_t)(p.seed + 202));
        const int32_t ntap = p.er_taps > 1 ? p.er_taps : 1;
        for (int32_t j = 0; j < ntap; ++j) er_gain[j] = nprng::uniform(ge, 0.3, p.er_max_ms) / 1000.0;
        for (int32_t j = 0; j < ntap; ++j) {
            const double d = er_gain[j];
            const double gn = nprng::uniform(ge, -1.0, 1.0) * exp(-d * 42.0);
            er_off[j] = (int32_t)rint(d * (double)p.base_sr);
            er_gain[j] = gn;
        }
    }
}

}  // namespace msgplan
