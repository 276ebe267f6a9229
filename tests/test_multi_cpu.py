"""Multi-GPU rendering as a library call (msgpu.multi),
on the CPU with the device work stubbed: one spawned worker per device, the
batch cut into contiguous ranges of equal predicted cost (shard.balance over
the host plans), outputs back in the caller's order through shared memory.

The stub worker fills each preset's frames with (its index in the call, its
device), so the test sees which worker rendered which preset."""
import numpy as np
import pytest

import msgpu
from msgpu.multi import DevicePool
from msgpu.pack import PackedBatch
from msgpu.shard import balance, plan_costs


@pytest.fixture(scope="module")
def pool2():
    p = DevicePool([0, 1], stub=True)
    yield p
    p.close()


def mixed(irs):
    cfgs = ["C2", "H48", "C3", "C2", "C5", "H48", "C3", "C2", "C3", "H48", "C2", "C3"]
    return [msgpu.config_params(c, seed=2000 + i, irs=irs, out_dur_s=0.05 if c != "C5" else 0.5)
            for i, c in enumerate(cfgs)]


def test_order_disjoint_and_balanced(pool2, irs):
    params = mixed(irs)
    outs = pool2.render_batch(params)
    out_n = PackedBatch(params).out_n
    assert len(outs) == len(params)
    seen = {}
    for i, (a, n) in enumerate(zip(outs, out_n)):
        assert a.shape == (n, 2) and a.dtype == np.float32
        assert np.all(a[:, 0] == i)                       # the caller's order
        devs = np.unique(a[:, 1])
        assert devs.size == 1                             # one worker per preset
        seen[i] = int(devs[0])
    split = pool2.last_split
    assert [s["device"] for s in split] == [0, 1]
    assert len({s["pid"] for s in split}) == 2            # two processes
    lo0, hi0 = split[0]["presets"]
    lo1, hi1 = split[1]["presets"]
    assert (lo0, hi1) == (0, len(params)) and hi0 == lo1  # contiguous, disjoint, complete
    assert all(seen[i] == (0 if i < hi0 else 1) for i in range(len(params)))
    costs = plan_costs(params)
    cuts = balance(costs, 2)
    assert [lo0, hi0, hi1] == cuts
    # the cut is the best contiguous one: moving it by one preset does not reduce the max
    best = max(sum(costs[:hi0]), sum(costs[hi0:]))
    for c in (hi0 - 1, hi0 + 1):
        if 0 < c < len(params):
            assert best <= max(sum(costs[:c]), sum(costs[c:])) + 1e-9


def test_more_workers_than_heavy_presets(irs):
    p = DevicePool([0, 1, 2], stub=True)
    try:
        params = mixed(irs)[:2]
        outs = p.render_batch(params)
        assert [int(a[0, 0]) for a in outs] == [0, 1]
        assert sum(s["presets"][1] - s["presets"][0] for s in p.last_split) == 2
    finally:
        p.close()


def test_worker_pins_its_own_cpus(pool2):
    assert [w["device"] for w in pool2.workers] == [0, 1]
    assert all(w["host_threads"] >= 1 for w in pool2.workers)


def test_variations_across_devices(monkeypatch, irs):
    """render_variations(devices=...) shards the on_batch product and keeps the
    reference's loop order and names (MS:1580-1587)."""
    from msgpu import batch as B
    from msgpu import multi
    p = DevicePool([0, 1], stub=True)
    monkeypatch.setitem(multi._POOLS, (0, 1), p)
    try:
        base = msgpu.merged(gen_mode="Noise burst", out_dur_s=0.02, event_process="Poisson")
        res = B.render_variations(base, "7, 8", "5, 9", "1, 1.5", devices=[0, 1])
        keys = [k for k, _ in B.variants(base, [7, 8], [5.0, 9.0], [1.0, 1.5])]
        assert [r[0] for r in res] == [B.variant_name(*k, 48000) for k in keys]
        assert [int(r[1][0, 0]) for r in res] == list(range(8))
        assert {int(r[1][0, 1]) for r in res} == {0, 1}
    finally:
        p.close()


def test_pool_refuses_after_gpu_use(monkeypatch):
    from msgpu import engine, multi
    monkeypatch.setitem(engine._engines, 0, object())
    with pytest.raises(RuntimeError, match="before this process"):
        multi.DevicePool([0, 1])


def test_shared_device_rehearsal(irs):
    """Two workers on one device only with share_devices=True (the one-GPU
    rehearsal, tools/multi_rehearsal.py); the split is the same cost cut."""
    with pytest.raises(ValueError, match="distinct"):
        DevicePool([0, 0], stub=True)
    p = DevicePool([0, 0], stub=True, share_devices=True)
    try:
        params = mixed(irs)
        outs = p.render_batch(params)
        assert [int(a[0, 0]) for a in outs] == list(range(len(params)))
        split = p.last_split
        assert [s["device"] for s in split] == [0, 0] and len({s["pid"] for s in split}) == 2
        assert [split[0]["presets"][0], split[0]["presets"][1], split[1]["presets"][1]] == balance(plan_costs(params), 2)
    finally:
        p.close()


def test_stats_mode(pool2, irs):
    """results="stats": one summary per preset in the caller's order, equal to a
    host computation on the worker's fill (the stub writes (index, device))."""
    from msgpu.multi import audio_stats
    params = mixed(irs)
    stats = pool2.render_batch(params, results="stats")
    out_n = PackedBatch(params).out_n
    cut = pool2.last_split[0]["presets"][1]
    assert len(stats) == len(params)
    for i, (s, n) in enumerate(zip(stats, out_n)):
        a = np.empty((n, 2), np.float32)
        a[:, 0] = i
        a[:, 1] = 0 if i < cut else 1
        assert s == audio_stats(a)
        assert s["out_n"] == n and s["sum_l"] == i * n


def test_device_mode_fetch_and_release(pool2, irs):
    """results="device": handles in the caller's order; fetch copies one render
    back, release frees it (a fetch after that raises)."""
    params = mixed(irs)[:5]
    hs = pool2.render_batch(params, results="device")
    out_n = PackedBatch(params).out_n
    assert [h.index for h in hs] == list(range(5))
    for h, n in zip(hs, out_n):
        a = pool2.fetch(h)
        assert a.shape == (n, 2) and np.all(a[:, 0] == h.index) and np.all(a[:, 1] == h.device)
    pool2.release(hs[:2])
    with pytest.raises(KeyError):
        pool2.fetch(hs[0])
    assert np.all(pool2.fetch(hs[2])[:, 0] == 2)
    pool2.release(hs[2:])


def test_interrupted_call_closes_the_pool(monkeypatch, irs):
    """an interrupted call must not leave replies in the pipes for
    the next one.  The interrupted pool is closed and dropped from pool_for's
    cache; a new pool renders the next call correctly."""
    from msgpu import multi
    p = DevicePool([0, 1], stub=True)
    monkeypatch.setitem(multi._POOLS, (7, 8), p)
    params = mixed(irs)[:6]
    real = p._recv_checked
    calls = {"n": 0}

    def flaky(*a):
        calls["n"] += 1
        if calls["n"] == 1:
            raise KeyboardInterrupt
        return real(*a)
    monkeypatch.setattr(p, "_recv_checked", flaky)
    with pytest.raises(KeyboardInterrupt):
        p.render_batch(params)
    assert p._closed and (7, 8) not in multi._POOLS
    with pytest.raises(RuntimeError, match="closed"):
        p.render_batch(params)
    q = DevicePool([0, 1], stub=True)
    try:
        outs = q.render_batch(params)
        assert [int(a[0, 0]) for a in outs] == list(range(6))
    finally:
        q.close()


def test_stale_reply_is_detected(irs):
    """A reply that belongs to another job (sequence number, shared block or
    preset range) is refused and closes the pool instead of being paired with
    the current job."""
    p = DevicePool([0, 1], stub=True)
    try:
        params = mixed(irs)[:4]
        # a stray job whose reply will sit in worker 0's pipe ahead of the real one
        p._conns[0].send(("job", 10_000, "stats", None, [0], params[:1], [0], [int(PackedBatch(params[:1]).out_n[0])]))
        with pytest.raises(RuntimeError, match="out of step"):
            p.render_batch(params, results="stats")
        assert p._closed
    finally:
        p.close()
