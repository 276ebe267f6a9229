"""Standalone FIR (msg_fir): y = np.convolve(x, h)[:n] at 16 k / 64 k taps (SURVEY §8 config
remarks and §8(d)), on the render path's partitioned FFT kernels (k_ir_spec, k_fir2).

The oracle is oracle.fir_causal (np.convolve, MS:444 without the 8192 cap).  At
these sizes np.convolve takes minutes, so the float64 reference is
scipy.signal.fftconvolve, itself checked against fir_causal on a short case here.
The bar is float32 FFT convolution accuracy relative to the output RMS: 1e-5.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REL = 1e-5


def _ref(x, h):
    from scipy.signal import fftconvolve
    return fftconvolve(np.asarray(x, np.float64), h)[:len(x)]


def _rel_rms(y, r):
    return float(np.sqrt(np.mean((y - r) ** 2)) / max(np.sqrt(np.mean(r ** 2)), 1e-30))


def test_fftconvolve_matches_oracle():
    from oracle import msound_oracle as O
    rng = np.random.default_rng(1)
    x, h = rng.standard_normal(5000), O.synthetic_fir_taps(3000)
    np.testing.assert_allclose(_ref(x, h), O.fir_causal(x, h), rtol=0, atol=1e-9)


@pytest.mark.parametrize("M,n,S", [(16384, 60000, 3), (65536, 200000, 2), (8192, 384000, 1),
                                   (262144, 300000, 2)])   # the last: frequency-domain delay line
def test_fir_long_taps(M, n, S):
    import torch
    from msgpu.engine import default_engine
    from oracle import msound_oracle as O
    h = O.synthetic_fir_taps(M)
    x = np.stack([np.random.default_rng(b).standard_normal(n).astype(np.float32) for b in range(S)])
    eng = default_engine(0)
    y, (N, P, Q) = eng.fir(torch.from_numpy(x).cuda(), h)
    torch.cuda.synchronize()
    assert P * Q >= M and N <= 65536
    if M >= 200000:
        assert P == N // 2            # the frequency-domain delay line path
    y = y.cpu().numpy()
    for b in range(S):
        assert _rel_rms(y[b], _ref(x[b], h)) <= REL, (b, N, P, Q)


@pytest.mark.parametrize("M,n", [(1, 1000), (5, 1), (300, 7), (20000, 9000), (70000, 30000), (4097, 4096)])
def test_fir_edges(M, n):
    import msgpu
    from oracle import msound_oracle as O
    rng = np.random.default_rng(M + n)
    h = rng.standard_normal(M)
    x = rng.standard_normal(n).astype(np.float32)
    y = msgpu.fir(x, h)
    r = O.fir_causal(x, h)
    assert y.shape == (n,)
    assert _rel_rms(y, r) <= REL


def test_fir_errors():
    import torch
    from msgpu.engine import default_engine
    eng = default_engine(0)
    x = torch.zeros(1000, device="cuda")
    with pytest.raises(RuntimeError):
        eng.fir(x, np.ones(10), out=x)
    with pytest.raises(NotImplementedError):
        eng.fir(x, np.ones(64 * 32768))


@pytest.mark.parametrize("M", [16383, 16384, 25473, 35000])
def test_fir8_block_edges_and_alignment(M):
    """k_fir8's block epilogue and edge-block loads: odd and even tap counts (the
    output pairs are written as 8-byte stores only for odd P and an 8-byte-aligned
    row), an odd signal length so that every other row of the batch starts at an
    odd float offset (misaligned loads and single stores), and a length that is
    not a multiple of the block."""
    import torch
    from msgpu.engine import default_engine
    from oracle import msound_oracle as O
    n, S = 100001, 3
    h = O.synthetic_fir_taps(M)
    x = np.stack([np.random.default_rng(7 + b).standard_normal(n).astype(np.float32) for b in range(S)])
    y, (N, P, Q) = default_engine(0).fir(torch.from_numpy(x).cuda(), h)
    torch.cuda.synchronize()
    assert (N, Q) == (65536, 1) and P == M        # one partition on k_fir8
    y = y.cpu().numpy()
    for b in range(S):
        e = _rel_rms(y[b], _ref(x[b], h))
        print(f"M={M} row {b}: rel rms {e:.3e}")
        assert e <= REL, (M, b)
        assert np.all(np.isfinite(y[b]))


@pytest.mark.parametrize("M,n,S", [(65536, 384000, 4), (40000, 100001, 3), (36000, 1_000_000, 3), (65536, 20000, 2)])
def test_fir8q_two_partitions(M, n, S):
    """k_fir8q: 35 749 <= M <= 64 k taps as two 32 768-tap
    partitions on the 65 536-point engine, B = P = 32 768 (below, one partition
    on k_fir8 has the longer block).  Whole-signal runs
    (C3-like batch), runs of single blocks that open with X_{j0-1} (few signals,
    many blocks: every run past block 0 takes the pre-block path), an odd length
    with odd row offsets, and a signal shorter than one block; MSGPU_FIR8Q=0
    (k_fir4, five partitions) agrees too."""
    import os
    import torch
    from msgpu.engine import Engine
    from oracle import msound_oracle as O
    h = O.synthetic_fir_taps(M)
    x = np.stack([np.random.default_rng(11 + b).standard_normal(n).astype(np.float32) for b in range(S)])
    outs = {}
    for flag in ("1", "0"):
        os.environ["MSGPU_FIR8Q"] = flag
        try:
            eng = Engine(0)
        finally:
            os.environ.pop("MSGPU_FIR8Q", None)
        y, shape = eng.fir(torch.from_numpy(x).cuda(), h)
        torch.cuda.synchronize()
        outs[flag] = (y.cpu().numpy(), shape)
    assert outs["1"][1] == (65536, 32768, 2) and outs["0"][1] != (65536, 32768, 2)
    for b in range(S):
        r = _ref(x[b], h)
        for flag, (y, shape) in outs.items():
            e = _rel_rms(y[b], r)
            print(f"M={M} n={n} row {b} FIR8Q={flag} {shape}: rel rms {e:.3e}")
            assert e <= REL and np.all(np.isfinite(y[b])), (flag, b)
