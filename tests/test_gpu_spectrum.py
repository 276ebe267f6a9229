"""Device spectrogram (k_stft64, msg_stft_mag_db) and the batch driver (on_batch).

stft_mag_db (MS:197-212) is checked against the reference's own outputs
(tests/golden/stft.npz, from tools/gen_golden_stft.py) and against the oracle
in float64.  Bins whose magnitude lies near the float64 rounding floor of the
frame (|X| < 1e-9 max|X|, i.e. below -180 dB relative) carry no significant
digits in either implementation and are compared only for being that small.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ("c2", "defaults", "capped", "short", "odd")
DB_TOL = 1e-6          # dB, for bins above the floor (float64 vs float64)
FLOOR_REL_DB = 180.0


def _golden():
    return np.load(os.path.join(HERE, "golden", "stft.npz"))


def _cmp(S, R, tol):
    assert S.shape == R.shape
    top = R.max(axis=0, keepdims=True)
    sig = R > top - FLOOR_REL_DB
    err = np.abs(S - R)
    assert np.max(err[sig]) <= tol, float(np.max(err[sig]))
    # floor bins: the device's are as far below the frame's peak
    lim = np.broadcast_to(top - FLOOR_REL_DB + 40.0, R.shape)
    assert np.all(S[~sig] <= lim[~sig])


@pytest.mark.parametrize("name", CASES)
def test_stft_vs_reference_golden(name):
    import msgpu
    z = _golden()
    sr, win, hop, mf = (int(v) for v in z[f"{name}_cfg"])
    S = msgpu.stft_mag_db(z[f"{name}_x"], sr, win=win, hop=hop, max_frames=mf)
    _cmp(S.astype(np.float32).astype(np.float64), z[f"{name}_S"].astype(np.float64), 1e-3)


@pytest.mark.parametrize("name", CASES)
def test_stft_vs_oracle_float64(name):
    import msgpu
    from oracle import msound_oracle as O
    z = _golden()
    sr, win, hop, mf = (int(v) for v in z[f"{name}_cfg"])
    x = z[f"{name}_x"]
    S = msgpu.stft_mag_db(x, sr, win=win, hop=hop, max_frames=mf)
    _cmp(S, O.stft_mag_db(x, sr, win=win, hop=hop, max_frames=mf), DB_TOL)


def test_stft_of_device_render_stereo():
    """The UI's view of a render (MS:1498-1500): L/R mean of the device output, float32 input."""
    import torch
    import msgpu
    from msgpu.engine import default_engine
    from msgpu.pack import PackedBatch
    from msgpu.spectrum import display_stft_params
    from oracle import msound_oracle as O
    p = msgpu.merged({"out_dur_s": 0.5, "base_sr": 96000})
    eng = default_engine(0)
    out = eng.render_packed(PackedBatch([p]))
    win, hop = display_stft_params(96000)
    S = msgpu.stft_mag_db(out, 96000, win=win, hop=hop)
    assert isinstance(S, torch.Tensor) and S.shape[0] == win // 2 + 1
    y = out.cpu().numpy().astype(np.float64)
    _cmp(S.cpu().numpy(), O.stft_mag_db(y.mean(axis=1), 96000, win=win, hop=hop), DB_TOL)


def test_stft_errors():
    import msgpu
    with pytest.raises(RuntimeError):
        msgpu.stft_mag_db(np.zeros(100), 48000, win=2048, hop=0)
    with pytest.raises(NotImplementedError):
        msgpu.stft_mag_db(np.zeros(1 << 16), 48000, win=1 << 15, hop=256)


def test_batch_variations_match_single_renders(tmp_path):
    """on_batch (MS:1524-1596): every variant equals render() of the same params, files round-trip."""
    import msgpu
    from msgpu.batch import read_wav_float32
    base = {"out_dur_s": 0.25, "base_sr": 48000}
    res = msgpu.render_variations(base, "1001, 1002", "15", "0.9,1.2", folder=str(tmp_path))
    assert [r[0] for r in res] == ["ms_seed1001_unf15_st0p9_48000Hz.wav", "ms_seed1001_unf15_st1p2_48000Hz.wav",
                                   "ms_seed1002_unf15_st0p9_48000Hz.wav", "ms_seed1002_unf15_st1p2_48000Hz.wav"]
    for (name, audio, sr), (sd, st) in zip(res, [(1001, 0.9), (1001, 1.2), (1002, 0.9), (1002, 1.2)]):
        p = msgpu.merged(base, seed=sd, time_unfold=15.0, partial_stretch=st)   # full dict, as get_params
        ref, meta = msgpu.render(p)
        assert sr == meta["out_sr"] == 48000
        # same engine; the FIR transform size is chosen per batch, so float32 rounding
        # may differ from a one-preset batch (parity bar: 1e-5 RMS)
        np.testing.assert_allclose(audio, ref, rtol=0, atol=1e-6)
        back, sr2 = read_wav_float32(os.path.join(tmp_path, name))
        assert sr2 == 48000
        np.testing.assert_array_equal(back, audio)
