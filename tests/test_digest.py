"""Per-render summary and digest (msg_digest / msg_digest_host, kernels_digest.h).

VERDICT r05 "what's missing" 1: the multi-GPU library's stats mode copied every
render to the host for a SHA-1 (68.7 GB per GPU for 1024 C5 presets).  The
summary is now reduced on the device; these tests pin its definition:

* CPU: msg_digest_host (the library's host reference) equals a NumPy restatement
  of the definition in include/msgpu.h -- the digest words exactly, and the
  float64 sums bit for bit when NumPy folds in the kernels' tile / wave order --
  at awkward lengths (empty, one frame, tile edges, several tiles per thread);
  the digest sees a flipped bit, a swap of two words and -0.0 vs 0.0.
* GPU: msg_digest of a rendered batch equals msg_digest_host of the same bytes,
  record for record, and its rms / sums match the reference's summaries.
"""
import numpy as np
import pytest

from msgpu import multi

S0, S1 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xD1B54A32D192ED03)
DG_T, DG_PER = 256, 8
DG_TILE = DG_T * DG_PER


def fmix64(x):
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xff51afd7ed558ccd)
    x = x ^ (x >> np.uint64(33))
    x = x * np.uint64(0xc4ceb9fe1a85ec53)
    return x ^ (x >> np.uint64(33))


def fold(arr, op=np.add):
    """The workgroup fold over axis -1 (256 thread partials): xor-butterfly in
    each wave of 64, then the four waves in order."""
    idx = np.arange(DG_T)
    for o in (32, 16, 8, 4, 2, 1):
        arr = op(arr, arr[..., idx ^ o])
    r = arr[..., 0]
    for w in (1, 2, 3):
        r = op(r, arr[..., 64 * w])
    return r


def np_digest(a):
    """include/msgpu.h's definition, in the kernels' order (NumPy)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    n = a.shape[0]
    with np.errstate(over="ignore"):
        w = a.reshape(-1).view(np.uint32).astype(np.uint64)
        k = (np.arange(2 * n, dtype=np.uint64) << np.uint64(32)) | w
        h0 = int(fmix64(k ^ S0).sum(dtype=np.uint64))
        h1 = int(fmix64(k ^ S1).sum(dtype=np.uint64))
    tiles = -(-n // DG_TILE)
    d = np.zeros((tiles * DG_TILE, 2), np.float64)
    d[:n] = a
    d = d.reshape(tiles, DG_PER, DG_T, 2)
    vals = {"ss": d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1], "sl": d[..., 0], "sr": d[..., 1],
            "peak": np.maximum(np.abs(d[..., 0]), np.abs(d[..., 1]))}
    out = {}
    for key, v in vals.items():
        op = np.maximum if key == "peak" else np.add
        acc = np.zeros((tiles, DG_T))
        for kk in range(DG_PER):                     # each thread in frame order
            acc = op(acc, v[:, kk, :])
        part = fold(acc, op) if tiles else np.zeros(0)
        rows = max(1, -(-tiles // DG_T))
        pp = np.zeros(rows * DG_T)
        pp[:tiles] = part
        acc2 = np.zeros(DG_T)
        for r in range(rows):                        # thread i: tiles i, i + 256, ... in order
            acc2 = op(acc2, pp[r * DG_T:(r + 1) * DG_T])
        out[key] = float(fold(acc2, op))
    return {"sum_sq": out["ss"], "peak": out["peak"], "sum_l": out["sl"], "sum_r": out["sr"], "h0": h0, "h1": h1}


def as_dict(rec):
    return {k: (int(rec[k]) if k in ("h0", "h1") else float(rec[k])) for k in rec.dtype.names}


@pytest.mark.parametrize("n", [0, 1, 255, 2047, 2048, 2049, 600_001])
def test_host_digest_matches_definition(n):
    rng = np.random.default_rng(n + 3)
    a = (rng.standard_normal((n, 2)) * 0.4).astype(np.float32)
    got = as_dict(multi.digest_host(a))
    want = np_digest(a)
    assert got == want, (got, want)                  # every field bit for bit
    d = a.astype(np.float64)
    if n:
        assert abs(got["sum_sq"] - float((d * d).sum())) <= 1e-12 * float((d * d).sum())
        assert got["peak"] == float(np.abs(d).max())
    st = multi.audio_stats(a)
    assert st["out_n"] == n and st["digest"] == f"{want['h0']:016x}{want['h1']:016x}"


def test_digest_sees_bits_and_positions():
    rng = np.random.default_rng(5)
    a = rng.standard_normal((5000, 2)).astype(np.float32)
    base = multi.audio_stats(a)["digest"]
    b = a.copy()
    b.view(np.uint32)[1234, 1] ^= 1                  # one mantissa bit
    assert multi.audio_stats(b)["digest"] != base
    c = a.copy()
    c[[10, 4000]] = c[[4000, 10]]                   # two frames swapped: same sums, other digest
    sc = multi.audio_stats(c)
    assert sc["digest"] != base and sc["peak"] == multi.audio_stats(a)["peak"]
    z = np.zeros((100, 2), np.float32)
    nz = z.copy()
    nz[7, 0] = -0.0
    assert multi.audio_stats(z)["digest"] != multi.audio_stats(nz)["digest"]
    assert multi.audio_stats(a, sha1=True)["sha1"]


def test_stats_sha1_opt_in(irs):
    """The stub pool's stats carry the digest; sha1=True adds the SHA-1."""
    from msgpu import DevicePool, config_params
    from msgpu.pack import PackedBatch
    params = [config_params("C2", seed=1000 + i, irs=irs, out_dur_s=0.01 * (i + 1)) for i in range(3)]
    p = DevicePool([0, 1], stub=True)
    try:
        plain = p.render_batch(params, results="stats")
        with_sha = p.render_batch(params, results="stats", sha1=True)
    finally:
        p.close()
    out_n = PackedBatch(params).out_n
    assert all("sha1" not in s and len(s["digest"]) == 32 for s in plain)
    assert all(len(s["sha1"]) == 40 for s in with_sha)
    assert [{k: v for k, v in s.items() if k != "sha1"} for s in with_sha] == plain
    assert [s["out_n"] for s in plain] == [int(v) for v in out_n]


def test_failed_device_job_drops_kept_renders():
    """a device-mode job that fails on one worker must not leave the
    renders kept for it in HBM.  Worker protocol: a job whose second preset
    cannot be made keeps the first; ("drop", seq, job) frees it."""
    from msgpu import DevicePool
    p = DevicePool([0], stub=True)
    try:
        c = p._conns[0]
        c.send(("job", 900, "device", None, [0, 1], [{}, {}], [0, 0], [16, -1]))
        reply = c.recv()
        assert reply[0] == "done" and reply[7]               # the error of preset 1
        c.send(("fetch", 901, (900, 0)))
        assert c.recv()[4] is None                           # preset 0 was kept
        c.send(("drop", 902, 900))
        assert c.recv() == ("released", 902)
        c.send(("fetch", 903, (900, 0)))
        assert c.recv()[4] is not None                       # and is gone
    finally:
        p.close()


@pytest.mark.gpu
def test_device_digest_equals_host(irs, golden_info):
    """msg_digest over a batch in HBM equals msg_digest_host of the same bytes
    (every field, bit for bit), for the batch's renders at their offsets, and
    the summaries match the reference's (golden_info.json) within 1e-5."""
    import msgpu
    import torch
    from msgpu.engine import default_engine
    from msgpu.pack import PackedBatch
    params = [msgpu.config_params("C3", seed=1000 + s, irs=irs) for s in range(3)]
    params += [msgpu.config_params("C2", seed=1000, irs=irs), msgpu.merged(out_dur_s=0.2000208, seed=6, base_sr=48000)]
    eng = default_engine(0)
    packed = PackedBatch(params)
    out = eng.render_packed(packed)
    torch.cuda.synchronize(0)
    recs = eng.digest(out, packed.offsets, packed.out_n)
    host = out.cpu().numpy()
    for i, (o, n) in enumerate(zip(packed.offsets, packed.out_n)):
        a = host[int(o):int(o) + int(n)]
        assert as_dict(recs[i]) == as_dict(multi.digest_host(a)), i
    st = msgpu.render_batch(params, results="stats")
    for s, cfg in zip(st[:3], ("C3_1000", "C3_1001", "C3_1002")):
        ref = golden_info["summaries"].get(cfg)
        if ref is None:
            continue
        assert abs(s["rms"] - ref["rms"]) <= 1e-5
        assert abs(s["sum_l"] - ref["sum_l"]) <= 1e-5 * s["out_n"]
    # a C5-length render: 4097 tiles, several per thread in the preset fold
    p5 = msgpu.config_params("C5", seed=1000, irs=irs)
    pk = PackedBatch([p5])
    o5 = eng.render_packed(pk)
    torch.cuda.synchronize(0)
    r5 = eng.digest(o5, pk.offsets, pk.out_n)
    assert as_dict(r5[0]) == as_dict(multi.digest_host(o5.cpu().numpy()))
