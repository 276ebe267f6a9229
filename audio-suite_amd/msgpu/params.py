"""Render parameter dictionary: factory defaults, preset merge, bench configs.

The reference's ``render(params)`` (microsound_0.2.1/main_v2.py:588, "MS" below)
indexes an 83-key dict built by ``MicrosoundV2.get_params`` (MS:1166-1266).  The
factory defaults are the widget initial values (MS:893-1137); partial presets are
merged over them (MS:1288-1290).  ``DEFAULTS`` reproduces that snapshot; the
drop-in :func:`msgpu.render` raises ``KeyError`` for a key the reference would
index and not find (:func:`first_missing_key`), and :func:`merged` builds a full
dict from a partial one the way the UI's preset loader does.
"""
from __future__ import annotations

import copy

# MS:893-1137 widget initial values, in get_params order (MS:1166-1266).
DEFAULTS: dict = {
    "base_sr": 48000,                # MS:896
    "out_dur_s": 8.0,                # MS:899
    "time_unfold": 25.0,             # MS:902
    "peak": 0.98,                    # MS:905
    "sat_drive": 1.0,                # MS:908
    "stereo_on": True,               # MS:910
    "stereo_width": 0.65,            # MS:913
    "gen_mode": "Gaussian click",    # MS:919 (combo index 0)
    "micro_ms": 1.25,                # MS:926
    "seed": 12345,                   # MS:928
    "dust_density": 0.02,            # MS:931
    "noise_tilt": -3.0,              # MS:934
    "ring_hz": 4200.0,               # MS:937
    "ring_decay_ms": 12.0,           # MS:940
    "crackle_alpha": 1.4,            # MS:944
    "crackle_density": 180.0,        # MS:947
    "crackle_kernel": 64,            # MS:950
    "ss_threshold": 0.9,             # MS:954
    "ss_build": 0.06,                # MS:957
    "ss_decay": 0.75,                # MS:960
    "ss_noise": 0.08,                # MS:963
    "chaos_r": 3.92,                 # MS:967
    "chaos_gate": 0.35,              # MS:970
    "wav_base_hz": 2400.0,           # MS:974
    "wav_count": 8,                  # MS:976
    "wav_spread": 0.6,               # MS:979
    "unfold_mode": "Classic reinterpret",  # MS:988
    "partial_stretch": 1.0,          # MS:991
    "partial_lock_on": False,        # MS:994
    "pl_top_n": 24,                  # MS:995
    "pl_neigh": 4,                   # MS:997
    "nl_warp_on": False,             # MS:999
    "nl_warp_power": 1.25,           # MS:1002
    "cep_warp_on": False,            # MS:1004
    "cep_factor": 1.2,               # MS:1007
    "mb_b1": 2000.0,                 # MS:1011
    "mb_b2": 8000.0,
    "mb_b3": 20000.0,
    "mb_u1": 35.0,                   # MS:1017
    "mb_u2": 20.0,
    "mb_u3": 12.0,
    "mb_roll": 2000.0,               # MS:1023
    "bandlimit_on": True,            # MS:1028
    "bandlimit_out_hz": 18000.0,     # MS:1031
    "bandlimit_roll_hz": 2500.0,     # MS:1034
    "event_process": "Single",       # MS:1039 (combo index 0)
    "grains_per_sec": 18.0,          # MS:1042
    "max_grains": 4000,              # MS:1044
    "grain_amp_rand": 0.35,          # MS:1047
    "grain_offset_on": True,         # MS:1049
    "grain_offset_max_ms": 60.0,     # MS:1052
    "cluster_size": 6,               # MS:1054
    "cluster_spread_ms": 25.0,       # MS:1057
    "hawkes_gain": 0.6,              # MS:1060
    "hawkes_decay_s": 0.25,          # MS:1063
    "bp_density": "0:18, 4:40, 8:14",  # MS:1070
    "bp_unfold": "",                 # MS:1071
    "bp_cutoff": "",                 # MS:1072
    "bp_stretch": "",                # MS:1073
    "res_bank_on": False,            # MS:1077
    "res_modes": 24,                 # MS:1079
    "res_fmin": 120.0,               # MS:1081
    "res_fmax": 12000.0,             # MS:1083
    "res_decay_ms": 80.0,            # MS:1085
    "wg_on": False,                  # MS:1087
    "wg_lines": 8,                   # MS:1089
    "wg_max_ms": 8.0,                # MS:1091
    "wg_fb": 0.7,                    # MS:1093
    "event_feedback_on": False,      # MS:1098
    "event_feedback_amt": 0.35,      # MS:1101
    "spectral_imprint_on": False,    # MS:1103
    "spectral_imprint_amt": 0.35,    # MS:1106
    "spectral_imprint_smooth": 0.92,  # MS:1109
    "er_cloud_on": True,             # MS:1114
    "er_taps": 320,                  # MS:1116
    "er_max_ms": 45.0,               # MS:1118
    "space_ir_on": False,            # MS:1120
    "space_ir_max_samps": 12000,     # MS:1122
    "env_a": 20.0,                   # MS:1127
    "env_d": 250.0,                  # MS:1129
    "env_s": 0.65,                   # MS:1131
    "env_r": 1800.0,                 # MS:1133
    "env_curve": 1.8,                # MS:1135
}

GEN_MODES = ("Gaussian click", "Dust impulses", "Noise burst", "Skewed transient",
             "Resonant strike", "Crackle / corona", "Stick–slip friction",
             "Micro-chaos", "Wavelet atoms", "IR fragment", "Image scanline")  # MS:919-923
EVENT_PROCESSES = ("Single", "Poisson", "Clustered", "Hawkes")              # MS:1039
UNFOLD_MODES = ("Classic reinterpret", "Multi-band unfold")                 # MS:988


def merged(params: dict | None = None, **overrides) -> dict:
    """Factory defaults with ``params`` then ``overrides`` merged on top (MS:1288-1290).

    Unknown keys (e.g. the dead ``harm_*`` keys some presets carry) are kept and
    ignored by ``render`` exactly as the reference ignores them.
    """
    out = copy.copy(DEFAULTS)
    if params:
        out.update(params)
    out.update(overrides)
    return out


# ---------------------------------------------------------------------------
# Benchmark / parity configurations (SURVEY.md section 8, table "Configs").
# IR names refer to microsound_0.2.1/irs/*.wav; the arrays are committed as data
# in tests/golden/irs.npz (int16/32768 -> mono -> normalize(0.9), MS:1405-1409).
# ---------------------------------------------------------------------------
CONFIGS: dict = {
    # C1: 48 kHz, 1 s, resonant transient, no band-limit, unfold x1, stretch x1.
    "C1": dict(base_sr=48000, out_dur_s=1.0, gen_mode="Resonant strike",
               bandlimit_on=False, time_unfold=1.0, partial_stretch=1.0,
               event_process="Single"),
    # C2: 192 kHz, 4096-tap IR, unfold x10, stretch x1, Poisson.
    "C2": dict(base_sr=192000, out_dur_s=1.0, gen_mode="Resonant strike",
               time_unfold=10.0, partial_stretch=1.0, event_process="Poisson",
               space_ir_on=True, space_ir_max_samps=4096, _ir_name="ir_metallic_ping_180ms"),
    # H48: the metric label's "384 kHz -> 48 kHz" read literally:
    # design SR 384 kHz (unfold x8) rendered to a 48 kHz output, C2's IR.
    "H48": dict(base_sr=48000, out_dur_s=1.0, gen_mode="Resonant strike",
                time_unfold=8.0, partial_stretch=1.0, event_process="Poisson",
                space_ir_on=True, space_ir_max_samps=4096, _ir_name="ir_metallic_ping_180ms"),
    # C3: 384 kHz, unfold x100 (design SR clamps to 30 MHz, MS:597), stretch x2,
    # IR request 16384 taps (capped to 8192 by MS:443).
    "C3": dict(base_sr=384000, out_dur_s=1.0, gen_mode="Resonant strike",
               time_unfold=100.0, partial_stretch=2.0, event_process="Poisson",
               space_ir_on=True, space_ir_max_samps=16384, _ir_name="ir_tiny_room_250ms"),
    # C4: as C3 with unfold x200, stretch x4, IR request 65536 taps.
    "C4": dict(base_sr=384000, out_dur_s=1.0, gen_mode="Resonant strike",
               time_unfold=200.0, partial_stretch=4.0, event_process="Poisson",
               space_ir_on=True, space_ir_max_samps=65536, _ir_name="ir_tiny_room_250ms"),
    # C5 (reading A): 3072 Hz x500 = 1.536 MHz design SR, 8 M-sample outputs.
    "C5": dict(base_sr=3072, out_dur_s=8388608 / 3072, gen_mode="Resonant strike",
               time_unfold=500.0, partial_stretch=4.0, event_process="Poisson",
               space_ir_on=True, space_ir_max_samps=65536, _ir_name="ir_tiny_room_250ms"),
}


def config_params(name: str, seed: int = 1000, irs: dict | None = None, **overrides) -> dict:
    """Full params dict for bench/parity config ``name`` with ``seed``.

    ``irs`` maps IR name -> float64 mono array; when the config names an IR it is
    attached as ``_ir_audio`` (MS:1438).
    """
    cfg = dict(CONFIGS[name])
    ir_name = cfg.pop("_ir_name", None)
    p = merged(cfg, seed=int(seed), **overrides)
    p["_ir_audio"] = None
    p["_img_gray"] = None
    if ir_name is not None:
        if irs is None or ir_name not in irs:
            raise KeyError(f"config {name} needs IR {ir_name!r}")
        p["_ir_audio"] = irs[ir_name]
    return p


_BASIC_MODES = ("Gaussian click", "Dust impulses", "Noise burst", "Skewed transient", "Resonant strike")
_MODE_KEYS = {
    "Crackle / corona": ("crackle_alpha", "crackle_density", "crackle_kernel"),
    "Stick–slip friction": ("ss_threshold", "ss_build", "ss_decay", "ss_noise"),
    "Micro-chaos": ("chaos_r", "chaos_gate"),
    "Wavelet atoms": ("wav_base_hz", "wav_count", "wav_spread"),
}


def accessed_keys(params: dict, has_events: bool = True):
    """The keys ``render`` indexes (MS:589-784), in the order it indexes them, for
    the branches ``params`` selects.  The event loop's keys are included when the
    render has events (the reference reads them at its first event, MS:633-758)."""
    get = params.get
    yield from ("base_sr", "out_dur_s", "time_unfold", "bp_density", "bp_unfold", "bp_cutoff",
                "bp_stretch", "event_process", "grains_per_sec", "seed", "cluster_size",
                "cluster_spread_ms", "hawkes_gain", "hawkes_decay_s", "max_grains",
                "spectral_imprint_on")                                           # MS:589-625
    if has_events:
        yield from ("bandlimit_out_hz", "partial_stretch", "grain_amp_rand", "micro_ms", "gen_mode")  # MS:634-648
        mode = get("gen_mode")
        if mode in _BASIC_MODES:
            yield from ("seed", "dust_density", "noise_tilt", "ring_hz", "ring_decay_ms")   # MS:650-660
        else:
            yield "seed"
            yield from _MODE_KEYS.get(mode, ())
        yield "bandlimit_on"                                                     # MS:690
        if get("bandlimit_on"):
            yield "bandlimit_roll_hz"
        for flag, keys in (("nl_warp_on", ("nl_warp_power",)), ("cep_warp_on", ("cep_factor",)),
                           ("partial_lock_on", ("pl_top_n", "pl_neigh"))):       # MS:694-702
            yield flag
            if get(flag):
                yield from keys
        for flag, keys in (("res_bank_on", ("res_modes", "res_fmin", "res_fmax", "res_decay_ms", "seed")),
                           ("wg_on", ("wg_lines", "wg_max_ms", "wg_fb", "seed"))):   # MS:704-717
            yield flag
            if get(flag):
                yield from keys
        yield "unfold_mode"                                                      # MS:719
        if get("unfold_mode", "Classic reinterpret") != "Classic reinterpret":
            yield from ("mb_b1", "mb_b2", "mb_b3", "mb_u1", "mb_u2", "mb_u3", "mb_roll")
        yield "event_feedback_on"                                                # MS:731 (1st event: no prev)
        if get("spectral_imprint_on"):
            yield from ("spectral_imprint_amt", "spectral_imprint_smooth")       # MS:736-738
        yield "grain_offset_on"                                                  # MS:746
        if get("grain_offset_on"):
            yield "grain_offset_max_ms"
    yield from ("env_a", "env_d", "env_s", "env_r", "env_curve", "er_cloud_on")  # MS:760-766
    if get("er_cloud_on"):
        yield from ("er_taps", "er_max_ms", "seed")
    yield "space_ir_on"                                                          # MS:772
    if get("space_ir_on") and get("_ir_audio") is not None:
        yield "space_ir_max_samps"
    yield "stereo_on"                                                            # MS:775
    if get("stereo_on"):
        yield "stereo_width"
    yield from ("sat_drive", "peak")                                             # MS:780-781


def first_missing_key(params: dict):
    """The key whose absence makes the reference's ``render`` raise KeyError, or None.
    Whether the event loop runs is decided by the host planner (msg_plan_host, the
    event process of MS:507-558 and the max_grains cut of MS:617-618)."""
    keys = list(accessed_keys(params, has_events=False))
    for k in keys:
        if k not in params:
            return k
    if _n_events(params) > 0:
        for k in accessed_keys(params, has_events=True):
            if k not in params:
                return k
    return None


def _n_events(params: dict) -> int:
    import ctypes as C
    from . import _lib as L
    from .pack import Banks, pack_preset
    banks = Banks()
    s = pack_preset(merged(params), banks)
    info = L.MsgPlanInfo()
    L.check(L.lib().msg_plan_host(C.byref(s), banks.bp_array(), None, 0, C.byref(info), None, 0, None, None), None)
    return int(info.n_events)

