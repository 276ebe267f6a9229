"""Flatten reference params dicts into ``msg_preset`` structs (include/msgpu.h).

Follows how ``render`` reads its dict (microsound_0.2.1/main_v2.py, "MS"):
conversions ``int(...)`` / ``float(...)`` at the point of use (MS:589-773),
truthiness of the boolean switches, breakpoint strings parsed as in MS:452-467,
and the two uses of ``_ir_audio`` — the space FIR (MS:772-773, 438-445) and the
"IR fragment" generator source (MS:333-341).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .params import DEFAULTS, merged

_LANES = ("bp_density", "bp_unfold", "bp_cutoff", "bp_stretch")   # MS:602-605


def parse_breakpoints(s):
    """'t:v, t:v' -> sorted [(t, v)] (MS:452-467).

    Parts without ':' are skipped, unparsable numbers are skipped, and a part
    with two ':' raises ValueError like the reference's tuple unpacking.
    """
    out = []
    s = (s or "").strip()
    if not s:
        return out
    for part in s.split(","):
        part = part.strip()
        if not part or ":" not in part:
            continue
        a, b = part.split(":")
        try:
            out.append((float(a.strip()), float(b.strip())))
        except Exception:
            pass
    out.sort(key=lambda q: q[0])
    return out


def space_ir_taps(p: dict):
    """FIR taps the reference convolves with, or None (MS:772-773, 438-443)."""
    if not (p["space_ir_on"] and p.get("_ir_audio") is not None):
        return None
    ir = p["_ir_audio"][:int(p["space_ir_max_samps"])]
    if ir is None or ir.size < 8:
        return None
    ir = np.asarray(ir).astype(np.float64)
    if ir.ndim > 1:
        ir = ir.mean(axis=1)
    return np.ascontiguousarray(ir[:min(ir.size, 8192)], dtype=np.float64)


def fragment_source(p: dict):
    """Mono float64 source of the 'IR fragment' generator, or None (MS:335-340)."""
    ir = p.get("_ir_audio")
    if ir is None or ir.size < 32:
        return None
    src = np.asarray(ir).astype(np.float64)
    if src.ndim > 1:
        src = src.mean(axis=1)
    return np.ascontiguousarray(src, dtype=np.float64)


@dataclass
class Banks:
    """Per-batch IR / image banks, de-duplicated by array identity, and the
    breakpoint bank: every distinct lane string parsed once (MS:452-467), its
    sorted (t, v) pairs appended to ``bp`` (include/msgpu.h)."""
    irs: list = field(default_factory=list)
    _ir_keys: dict = field(default_factory=dict)
    images: list = field(default_factory=list)
    _img_keys: dict = field(default_factory=dict)
    bp: list = field(default_factory=list)
    _lane_keys: dict = field(default_factory=dict)

    def ir(self, key, make):
        if key not in self._ir_keys:
            arr = make()
            if arr is None:
                self._ir_keys[key] = -1
            else:
                self._ir_keys[key] = len(self.irs)
                self.irs.append(arr)
        return self._ir_keys[key]

    def image(self, img):
        if img is None:
            return -1
        k = id(img)
        if k not in self._img_keys:
            self._img_keys[k] = len(self.images)
            self.images.append(np.ascontiguousarray(img, dtype=np.uint8))
        return self._img_keys[k]

    def lane(self, s):
        """(first pair, pair count) of lane string ``s`` in the bank."""
        try:
            hit = self._lane_keys.get(s)
        except TypeError:                      # unhashable: parse (and fail) as the reference does
            hit = None
        if hit is not None:
            return hit
        pts = parse_breakpoints(s)
        if len(self.bp) // 2 + len(pts) > 2 ** 31 - 1:
            raise NotImplementedError("breakpoint bank beyond 2^31 points")
        hit = (len(self.bp) // 2, len(pts))
        for t, v in pts:
            self.bp.append(t)
            self.bp.append(v)
        try:
            self._lane_keys[s] = hit
        except TypeError:
            pass
        return hit

    def bp_array(self):
        """The breakpoint bank as a ctypes double array (None when empty)."""
        return (C.c_double * len(self.bp))(*self.bp) if self.bp else None


def pack_preset(params: dict, banks: Banks) -> L.MsgPreset:
    """One params dict -> msg_preset (the Python statement of what the native
    packer ``_mspack.pack`` does; tests hold the two byte-identical)."""
    p = merged(params)
    s = L.MsgPreset()
    s.seed = int(p["seed"])
    s.base_sr = int(p["base_sr"])
    s.gen_mode = L.GEN_MODE.get(p["gen_mode"], L.GEN_FALLBACK)
    s.process = L.PROCESS.get(p["event_process"], L.PROC_NONE)
    s.max_grains = int(p["max_grains"])
    s.cluster_size = int(p["cluster_size"])
    s.crackle_kernel = int(p["crackle_kernel"])
    s.wav_count = int(p["wav_count"])
    s.pl_top_n = int(p["pl_top_n"])
    s.pl_neigh = int(p["pl_neigh"])
    s.res_modes = int(p["res_modes"])
    s.wg_lines = int(p["wg_lines"])
    s.er_taps = int(p["er_taps"])
    flags = 0
    for key, bit in FLAG_KEYS:
        if p[key]:
            flags |= bit
    if p["unfold_mode"] != "Classic reinterpret":          # MS:720-727
        flags |= L.F_MULTIBAND
    s.ir_conv, fl, s.ir_frag, s.image = sources(p, banks)
    s.flags = flags | fl
    for lane, key in enumerate(_LANES):
        s.bp_off[lane], s.n_bp[lane] = banks.lane(p[key])
    for name in FLOAT_KEYS:
        setattr(s, name, float(p[name]))
    for i, k in enumerate(("mb_b1", "mb_b2", "mb_b3")):
        s.mb_b[i] = float(p[k])
    for i, k in enumerate(("mb_u1", "mb_u2", "mb_u3")):
        s.mb_u[i] = float(p[k])
    return s


FLAG_KEYS = (("stereo_on", L.F_STEREO), ("bandlimit_on", L.F_BANDLIMIT),
             ("partial_lock_on", L.F_PARTIAL_LOCK), ("nl_warp_on", L.F_NL_WARP),
             ("cep_warp_on", L.F_CEP_WARP), ("grain_offset_on", L.F_GRAIN_OFFSET),
             ("res_bank_on", L.F_RES_BANK), ("wg_on", L.F_WAVEGUIDE),
             ("event_feedback_on", L.F_EVENT_FEEDBACK), ("spectral_imprint_on", L.F_IMPRINT),
             ("er_cloud_on", L.F_ER_CLOUD))
FLOAT_KEYS = ("out_dur_s", "time_unfold", "peak", "sat_drive", "stereo_width", "micro_ms",
              "dust_density", "noise_tilt", "ring_hz", "ring_decay_ms", "crackle_alpha",
              "crackle_density", "ss_threshold", "ss_build", "ss_decay", "ss_noise", "chaos_r",
              "chaos_gate", "wav_base_hz", "wav_spread", "partial_stretch", "nl_warp_power",
              "cep_factor", "mb_roll", "bandlimit_out_hz", "bandlimit_roll_hz", "grains_per_sec",
              "grain_amp_rand", "grain_offset_max_ms", "cluster_spread_ms", "hawkes_gain",
              "hawkes_decay_s", "res_fmin", "res_fmax", "res_decay_ms", "wg_max_ms", "wg_fb",
              "event_feedback_amt", "spectral_imprint_amt", "spectral_imprint_smooth", "er_max_ms",
              "env_a", "env_d", "env_s", "env_r", "env_curve")


def sources(p: dict, banks: Banks):
    """(ir_conv, F_SPACE_IR or 0, ir_frag, image) of a full params dict: the space
    FIR's taps (MS:772-773) and the IR-fragment / image generator sources."""
    ir_obj = p.get("_ir_audio")
    taps_key = ("conv", id(ir_obj), int(p["space_ir_max_samps"]), bool(p["space_ir_on"]))
    ic = banks.ir(taps_key, lambda: space_ir_taps(p))
    frag = banks.ir(("frag", id(ir_obj)), lambda: fragment_source(p)) if p["gen_mode"] == "IR fragment" else -1
    img = banks.image(p.get("_img_gray")) if p["gen_mode"] == "Image scanline" else -1
    return (ic, L.F_SPACE_IR if ic >= 0 else 0, frag, img)


def out_frames(params: dict) -> int:
    """out_n = int(max(1, round(out_dur_s * base_sr))) (MS:589-591)."""
    p = merged(params)
    return int(max(1, round(float(p["out_dur_s"]) * int(p["base_sr"]))))


def design_sr(params: dict) -> int:
    """meta['design_sr_base'] (MS:593-597)."""
    p = merged(params)
    base_sr = int(p["base_sr"])
    g = int(round(base_sr * max(1.0, float(p["time_unfold"]))))
    return int(np.clip(g, base_sr, 30_000_000))


def _native():
    try:
        from . import _mspack
    except ImportError as e:
        raise RuntimeError("msgpu/_mspack not built (run `python -c 'import __graft_entry__ as g; g.build()'`)") from e
    return _mspack


class PackedBatch:
    """ctypes arrays for one msg_render_batch call; build once, render many times.

    The dicts are flattened by the native packer (``_mspack``, csrc/mspack.c: one
    pass over each dict in C, defaults for absent keys as :func:`merged` gives
    them); ``python=True`` uses :func:`pack_preset` instead (tests hold the two
    byte-identical)."""

    def __init__(self, params_list, python: bool = False):
        params_list = params_list if isinstance(params_list, list) else list(params_list)
        self.n = len(params_list)
        if self.n == 0:
            raise ValueError("empty batch")
        banks = Banks()
        self.presets = (L.MsgPreset * self.n)()
        self.out_n = np.empty(self.n, dtype=np.int64)
        if python:
            for i, prm in enumerate(params_list):
                self.presets[i] = pack_preset(prm, banks)
                self.out_n[i] = out_frames(prm)
        else:
            _native().pack(params_list, self.presets, self.out_n, DEFAULTS, L.GEN_MODE, L.PROCESS,
                           banks.lane, lambda p: sources(merged(p), banks))
        self._finish(banks)

    @classmethod
    def variants(cls, template: dict, keys):
        """The batch of ``template`` with (seed, time_unfold, partial_stretch) set to
        each of ``keys`` (the on_batch loop's dicts, MS:1578-1584): the template is
        packed once and copied, and only the three fields differ (held equal to
        packing every variant dict by tests/test_batch_host.py)."""
        keys = list(keys)
        self = cls.__new__(cls)
        self.n = len(keys)
        if self.n == 0:
            raise ValueError("empty batch")
        banks = Banks()
        one = (L.MsgPreset * 1)()
        n1 = np.empty(1, dtype=np.int64)
        _native().pack([template], one, n1, DEFAULTS, L.GEN_MODE, L.PROCESS, banks.lane,
                       lambda p: sources(merged(p), banks))
        self.presets = (L.MsgPreset * self.n)()
        rec = np.frombuffer(self.presets, dtype=np.dtype(L.MsgPreset))
        rec[:] = np.frombuffer(one, dtype=np.dtype(L.MsgPreset))[0]
        rec["seed"] = [((int(sd) + 2 ** 63) % 2 ** 64) - 2 ** 63 for sd, _, _ in keys]   # ctypes' int64 wrap
        rec["time_unfold"] = [float(u) for _, u, _ in keys]
        rec["partial_stretch"] = [float(st) for _, _, st in keys]
        self.out_n = np.full(self.n, n1[0], dtype=np.int64)   # out_dur_s and base_sr are the template's
        self._finish(banks)
        return self

    def _finish(self, banks):
        self.offsets = np.zeros(self.n, dtype=np.int64)
        self.offsets[1:] = np.cumsum(self.out_n)[:-1]
        self.total_frames = int(self.out_n.sum())
        self._offsets_c = self.offsets.ctypes.data_as(C.POINTER(C.c_int64))
        self._bp = banks.bp_array()
        self.bp_pairs = len(banks.bp) // 2
        self.bp_ptr = C.cast(self._bp, C.POINTER(C.c_double)) if self._bp is not None else None
        self._irs = banks.irs
        nir = len(self._irs)
        self.n_irs = nir
        self.ir_ptrs = (C.POINTER(C.c_double) * max(nir, 1))()
        self.ir_lens = (C.c_int64 * max(nir, 1))()
        for i, a in enumerate(self._irs):
            self.ir_ptrs[i] = a.ctypes.data_as(C.POINTER(C.c_double))
            self.ir_lens[i] = a.size
        self._imgs = banks.images
        nim = len(self._imgs)
        self.n_images = nim
        self.img_ptrs = (C.POINTER(C.c_uint8) * max(nim, 1))()
        self.img_h = (C.c_int32 * max(nim, 1))()
        self.img_w = (C.c_int32 * max(nim, 1))()
        for i, a in enumerate(self._imgs):
            self.img_ptrs[i] = a.ctypes.data_as(C.POINTER(C.c_uint8))
            self.img_h[i], self.img_w[i] = a.shape
