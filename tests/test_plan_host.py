"""The render plan (csrc/plan.h, host build) vs the oracle's plan_render / er_taps.

Event times, amplitudes, design SRs, grain lengths, start samples, offsets and
the ER tap table must match the NumPy restatement exactly (they are the
reference's scalar RNG decisions, MS:589-646, 742-751, 409-417).
"""
import ctypes as C

import numpy as np
import pytest

from msgpu import _lib as L
from msgpu.pack import Banks, pack_preset, fragment_source
from msgpu.params import config_params, merged
from oracle import msound_oracle as O


def host_plan(p):
    lib = L.lib()
    banks = Banks()
    s = pack_preset(p, banks)
    bp = banks.bp_array()
    frag = fragment_source(merged(p)) if merged(p)["gen_mode"] == "IR fragment" else None
    flen = 0 if frag is None else frag.size
    info = L.MsgPlanInfo()
    assert lib.msg_plan_host(C.byref(s), bp, None, flen, C.byref(info), None, 0, None, None) == 0
    ev = (L.MsgEvent * max(1, info.n_slots))()
    ntap = max(1, s.er_taps)
    off = np.zeros(ntap, dtype=np.int32)
    gain = np.zeros(ntap, dtype=np.float64)
    st = lib.msg_plan_host(C.byref(s), bp, None, flen, C.byref(info), ev, info.n_slots,
                           off.ctypes.data_as(C.POINTER(C.c_int32)), gain.ctypes.data_as(C.POINTER(C.c_double)))
    assert st == 0
    return info, list(ev)[:info.n_events], off, gain


def check_plan(p):
    info, ev, off, gain = host_plan(p)
    ref = O.plan_render(p)
    assert info.out_n == ref.out_n
    assert info.design_sr == ref.gen_sr
    assert info.n_events == len(ref.events)
    for e, r in zip(ev, ref.events):
        assert e.index == r.index
        assert e.t0 == r.t0
        assert e.amp == r.amp
        assert e.ufac == r.ufac
        assert e.gen_sr == r.gen_sr and e.n == r.n
        assert e.cutoff_out == r.cutoff_out and e.stretch == r.stretch
        if r.placed:
            assert e.start == r.start and e.offset == r.offset
            assert e.len == max(0, min(ref.out_n - r.start, r.n - r.offset))
        else:
            assert e.len == 0
    pm = merged(p)
    if pm["er_cloud_on"]:
        ro, rg = O.er_taps(int(pm["base_sr"]), int(pm["er_taps"]), float(pm["er_max_ms"]), int(pm["seed"]))
        assert np.array_equal(off, ro.astype(np.int32))
        # numpy's SIMD exp (MS:415) and libm exp differ by <= 1 ulp
        np.testing.assert_allclose(gain, rg, rtol=4e-16, atol=0)
    return info


@pytest.mark.parametrize("cfg", ["C1", "C2", "C3", "C4", "C5"])
@pytest.mark.parametrize("seed", [1000, 1001, 12345])
def test_configs(irs, cfg, seed):
    info = check_plan(config_params(cfg, seed=seed, irs=irs))
    if cfg == "C5":
        assert info.n_events == 4000   # max_grains cap (MS:617-618)


def test_presets(irs, golden_info):
    for name in golden_info["presets"]:
        for dur in (0.5, 3.0):
            p = merged(golden_info["preset_params"][name])
            p["out_dur_s"] = dur
            p["_ir_audio"] = irs["tiny_room_ir"]
            check_plan(p)


@pytest.mark.parametrize("proc", ["Single", "Poisson", "Clustered", "Hawkes", "bogus"])
def test_processes_and_lanes(proc):
    for seed in (1, 77, 4242):
        p = merged(event_process=proc, seed=seed, out_dur_s=2.5, base_sr=44100,
                   bp_unfold="0:5, 1:40, 2.2:3", bp_cutoff="0:9000, 2:15000",
                   bp_stretch="0.5:0.8, 2:1.6", bp_density="0:4, 1:30", max_grains=25,
                   gen_mode="Noise burst", grain_offset_max_ms=3.0)
        check_plan(p)


def test_grain_lengths_by_mode(irs):
    for mode in ["Gaussian click", "Crackle / corona", "Stick–slip friction", "Micro-chaos",
                 "Wavelet atoms", "IR fragment", "Image scanline", "unknown mode"]:
        for ir in (None, irs["tiny_room_ir"], irs["tiny_room_ir"][:20]):
            p = merged(gen_mode=mode, event_process="Poisson", out_dur_s=0.7, micro_ms=0.05,
                       _ir_audio=ir)
            check_plan(p)


def _lane(n, seed, t_max, v_lo, v_hi, shuffle=True):
    """A lane string of n 't:v' points (unsorted, with repeated times)."""
    rng = np.random.default_rng(seed)
    t = np.round(rng.uniform(0, t_max, n), 3)
    t[n // 3] = t[n // 2]                      # a repeated time: stable sort keeps input order
    v = np.round(rng.uniform(v_lo, v_hi, n), 2)
    order = rng.permutation(n) if shuffle else np.arange(n)
    return ", ".join(f"{t[i]}:{v[i]}" for i in order)


@pytest.mark.parametrize("npts", [33, 40, 200])
def test_long_breakpoint_lanes(npts):
    """Lanes beyond the 32 points of the round-3 ABI (the UI's QLineEdits take any
    number, MS:1070-1073): every lane of every event evaluated as MS:469-482."""
    for seed in (3, 11):
        p = merged(event_process="Poisson", seed=seed, out_dur_s=2.0, base_sr=48000, grains_per_sec=40.0,
                   bp_density=_lane(npts, seed, 2.2, 2, 60), bp_unfold=_lane(npts, seed + 1, 2.2, 1, 60),
                   bp_cutoff=_lane(npts, seed + 2, 2.2, 500, 20000), bp_stretch=_lane(npts, seed + 3, 2.2, 0.4, 3.5))
        assert len(O.parse_breakpoints(p["bp_unfold"])) == npts
        check_plan(p)
