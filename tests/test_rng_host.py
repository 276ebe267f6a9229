"""libmsgpu's NumPy-stream primitives (csrc/nprng.h), host build, vs NumPy itself.

The device kernels run the same header, so bit-exact host results pin the
algorithms (SeedSequence, PCG64, ziggurat normal/exponential, Lemire integers)
and the chunked parallel walk used by k_gen_normal.
"""
import ctypes as C

import numpy as np
import pytest

from msgpu import _lib as L


@pytest.fixture(scope="module")
def lib():
    return L.lib()


def _call(fn, seed, n, dtype, ctype):
    out = np.zeros(n, dtype=dtype)
    assert fn(seed, out.ctypes.data_as(C.POINTER(ctype)), n) == 0
    return out


@pytest.mark.parametrize("seed", [0, 1, 12345, 12345 + 123456, 2**32 - 1, 2**32 + 5, 2_000_000_000 + 9999])
def test_raw_stream(lib, seed):
    got = _call(lib.msg_rng_raw, seed, 1000, np.uint64, C.c_uint64)
    ref = np.random.default_rng(seed).bit_generator.random_raw(1000)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("seed", [0, 7, 1000, 12345, 9999 + 1000])
def test_standard_normal(lib, seed):
    n = 200_000   # ~1% of draws take the slow rejection paths
    got = _call(lib.msg_rng_normal, seed, n, np.float64, C.c_double)
    ref = np.random.default_rng(seed).standard_normal(n)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("seed", [3, 1000, 31337])
def test_chunked_walk_matches_sequential(lib, seed):
    # the wave-parallel walk must emit exactly standard_normal(n) for any n
    for n in (1, 63, 64, 65, 1920, 37500, 100_003):
        got = _call(lib.msg_rng_normal_chunked, seed, n, np.float64, C.c_double)
        ref = np.random.default_rng(seed).standard_normal(n)
        assert np.array_equal(got, ref), n


@pytest.mark.parametrize("seed", [0, 5, 10000 + 9999])
def test_standard_exponential(lib, seed):
    n = 200_000
    got = _call(lib.msg_rng_exponential, seed, n, np.float64, C.c_double)
    ref = np.random.default_rng(seed).standard_exponential(n)
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("low,high", [(0, 1), (0, 2), (0, 17), (0, 2880), (-300, 300),
                                      (0, 2**32 - 1), (0, 2**32), (0, 2**32 + 1), (5, 2**40)])
def test_integers(lib, low, high):
    for seed in (1, 12345 + 123456):
        out = np.zeros(2000, dtype=np.int64)
        assert lib.msg_rng_integers(seed, low, high, out.ctypes.data_as(C.POINTER(C.c_int64)), 2000) == 0
        ref = np.random.default_rng(seed).integers(low, high, size=2000)
        assert np.array_equal(out, ref), (low, high, seed)


def test_integers_scalar_interleaved_with_doubles(lib):
    # render() interleaves rng.uniform and scalar rng.integers on one stream
    # (MS:642, 750); the buffered 32-bit half must carry across calls.  The
    # host planner test (test_plan_host.py) checks that interleaving; here the
    # scalar path alone must equal the vector path.
    g = np.random.default_rng(99)
    ref = [int(g.integers(0, 2880)) for _ in range(50)]
    out = np.zeros(50, dtype=np.int64)
    lib.msg_rng_integers(99, 0, 2880, out.ctypes.data_as(C.POINTER(C.c_int64)), 50)
    assert out.tolist() == ref
