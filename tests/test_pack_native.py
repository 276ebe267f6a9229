"""The native dict packer (csrc/mspack.c, ``_mspack``) against its Python
statement ``msgpu.pack.pack_preset`` (MS:589-773's reads of the params dict).

Both must give byte-identical msg_preset arrays, identical output lengths and the
same breakpoint bank for: the 27 shipped presets, the bench configs, partial
dicts (defaults for absent keys, as ``merged``), values the reference converts
with int() / float() (strings, bools, numpy scalars), lanes of any length, IR /
image sources; and the same exception types for bad values.
"""
import ctypes as C
import time

import numpy as np
import pytest

import msgpu
from msgpu import _lib as L
from msgpu.pack import PackedBatch
from msgpu.params import merged


def _same(params):
    a = PackedBatch(params)
    b = PackedBatch(params, python=True)
    raw = lambda pk: bytes(C.string_at(C.addressof(pk.presets), C.sizeof(pk.presets)))  # noqa: E731
    assert raw(a) == raw(b)
    assert np.array_equal(a.out_n, b.out_n)
    assert a.bp_pairs == b.bp_pairs
    if a.bp_pairs:
        assert list(a._bp) == list(b._bp)
    assert a.n_irs == b.n_irs and a.n_images == b.n_images
    for x, y in zip(a._irs, b._irs):
        assert np.array_equal(x, y)
    return a


def test_presets_and_configs(irs, golden_info):
    params = []
    for name in golden_info["presets"]:
        p = merged(golden_info["preset_params"][name])
        p["_ir_audio"] = irs["tiny_room_ir"]
        params.append(p)
    for cfg in ("C1", "C2", "H48", "C3", "C4", "C5"):
        params += [msgpu.config_params(cfg, seed=s, irs=irs) for s in (1000, 1001)]
    _same(params)


def test_partial_dicts_and_conversions(irs):
    img = (np.arange(12 * 40) % 251).astype(np.uint8).reshape(12, 40)
    params = [
        {},                                                     # all defaults
        {"seed": "77", "base_sr": 44100.9, "out_dur_s": "0.5", "stereo_on": 0, "er_cloud_on": "",
         "time_unfold": np.float32(3.5), "max_grains": np.int64(9), "bandlimit_on": [1]},
        {"gen_mode": "Image scanline", "_img_gray": img, "seed": True},
        {"gen_mode": "IR fragment", "_ir_audio": irs["tiny_room_ir"], "space_ir_on": True,
         "space_ir_max_samps": 5000},
        {"gen_mode": "no such mode", "event_process": "bogus", "unfold_mode": "Multi-band unfold"},
        {"_ir_audio": irs["tiny_room_ir"], "space_ir_on": True, "space_ir_max_samps": 4},    # < 8 taps: no FIR
        {"out_dur_s": 1e-9},                                    # out_n floors at 1
        {"out_dur_s": 2.5 / 48000},                             # round half to even
        {"bp_unfold": "0:5, junk, 1:x, 2:40, , 0.5:7", "bp_cutoff": None},
        {"seed": 2 ** 64 + 5},                                  # ctypes wraps int64
    ]
    a = _same(params)
    assert a.presets[2].image == 0 and a.presets[3].ir_frag >= 0
    assert a.out_n[6] == 1 and a.out_n[7] == 2


@pytest.mark.parametrize("npts", [1, 32, 33, 200, 1000])
def test_lanes_any_length(npts):
    rng = np.random.default_rng(npts)
    lane = ", ".join(f"{t:.4f}:{v:.3f}" for t, v in zip(rng.uniform(0, 5, npts), rng.uniform(1, 50, npts)))
    params = [merged(bp_unfold=lane, bp_density=lane, seed=i) for i in range(3)]
    a = _same(params)
    assert a.presets[0].n_bp[1] == npts and a.bp_pairs == npts   # one bank entry per distinct string
    t = np.array(a._bp)[0::2][:npts]
    assert np.all(np.diff(t) >= 0)


@pytest.mark.parametrize("bad, exc", [({"seed": "x"}, ValueError), ({"out_dur_s": float("nan")}, ValueError),
                                      ({"peak": "high"}, ValueError), ({"bp_unfold": "1:2:3"}, ValueError),
                                      ({"gen_mode": ["list"]}, TypeError), ({"out_dur_s": float("inf")}, OverflowError)])
def test_errors_match(bad, exc):
    with pytest.raises(exc):
        PackedBatch([bad], python=True)
    with pytest.raises(exc):
        PackedBatch([bad])


def test_native_pack_speed(irs):
    """1024 C3 dicts: the packing of one bench step (VERDICT r03 weak #6 asks
    <= 2 ms on the GPU box's host; this container's CPU is slower and shared,
    so the bound here is loose and the figure is printed)."""
    params = [msgpu.config_params("C3", seed=1000 + b, irs=irs) for b in range(1024)]
    PackedBatch(params)
    best = min(_timed(lambda: PackedBatch(params)) for _ in range(5))
    py = _timed(lambda: PackedBatch(params, python=True))
    print(f"pack 1024 C3 dicts: native {best * 1e3:.2f} ms, python {py * 1e3:.1f} ms")
    assert best < py / 5


def _timed(f):
    t = time.perf_counter()
    f()
    return time.perf_counter() - t
