"""Host side of the batch driver (on_batch, MS:1524-1596): list parsing, loop order, names, WAV files."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-suite_amd"))

from msgpu import batch as B  # noqa: E402


def test_parse_list_skips_bad_entries():
    assert B.parse_list("1001, 1002,,x,1003", int) == [1001, 1002, 1003]
    assert B.parse_list("15,2.5e1, ,40", float) == [15.0, 25.0, 40.0]
    assert B.parse_list("", float) == []


def test_variant_order_and_params():
    v = B.variants({"seed": 1, "gen_mode": "Noise"}, [7, 8], [15.0], [0.9, 1.0])
    assert [k for k, _ in v] == [(7, 15.0, 0.9), (7, 15.0, 1.0), (8, 15.0, 0.9), (8, 15.0, 1.0)]
    assert v[3][1] == {"seed": 8, "gen_mode": "Noise", "time_unfold": 15.0, "partial_stretch": 1.0}


def test_names():
    # the reference's exact string (MS:1587): every '.' becomes 'p', the suffix included
    assert B.variant_name(1001, 15.0, 0.9, 48000, "reference") == "ms_seed1001_unf15_st0p9_48000Hzpwav"
    assert B.variant_name(1001, 2.5, 1.0, 192000, "wav") == "ms_seed1001_unf2p5_st1_192000Hz.wav"


def test_wav_float32_round_trip(tmp_path):
    from scipy.io import wavfile
    rng = np.random.default_rng(3)
    a = rng.standard_normal((1001, 2)).astype(np.float32)
    path = os.path.join(tmp_path, "x.wav")
    B.write_wav_float32(path, a, 192000)
    sr, b = wavfile.read(path)           # an independent reader of IEEE-float WAV
    assert sr == 192000 and b.dtype == np.float32
    np.testing.assert_array_equal(b, a)
    c, sr2 = B.read_wav_float32(path)
    assert sr2 == 192000
    np.testing.assert_array_equal(c, a)


def test_chunks_bound_presets_and_frames(monkeypatch):
    monkeypatch.setattr(B, "MAX_BATCH_PRESETS", 3)
    monkeypatch.setattr(B, "MAX_BATCH_FRAMES", 10)
    ch = list(B._chunks(list(range(8)), lambda i: 4))
    assert ch == [[0, 1], [2, 3], [4, 5], [6, 7]]
    ch = list(B._chunks(list(range(7)), lambda i: 1))
    assert ch == [[0, 1, 2], [3, 4, 5], [6]]


def test_template_variants_pack_like_each_dict():
    """PackedBatch.variants (template packed once, three fields patched) equals
    packing every variant dict of the on_batch loop (MS:1578-1584)."""
    import ctypes as C
    from msgpu.pack import PackedBatch
    from msgpu.params import merged
    base = merged(gen_mode="Noise burst", event_process="Poisson", bp_unfold="0:5, 1:9", out_dur_s=0.3)
    v = B.variants(base, "1001, 1002, 99", "15, 2.5", "0.9,1,1.75")
    a = PackedBatch.variants(base, [k for k, _ in v])
    b = PackedBatch([p for _, p in v])
    raw = lambda pk: bytes(C.string_at(C.addressof(pk.presets), C.sizeof(pk.presets)))  # noqa: E731
    assert a.n == 18 and raw(a) == raw(b)
    assert np.array_equal(a.out_n, b.out_n) and list(a._bp) == list(b._bp)
