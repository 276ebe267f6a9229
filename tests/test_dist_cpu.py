"""Multi-rank path of bench.py on CPU (gloo, world size 2).

The render shards by preset with no data-path collective:
each rank packs its own seeds, and only the timing barrier, the MAX of the
elapsed times and the per-rank record cross ranks, on a host gloo group.
These tests run that logic in two processes -- through bench.py's own
``--gpus 2`` launcher with the device work stubbed (``--dry-run``), and through
the rank helpers directly; the device render itself is covered by -m gpu.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, batch, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import msgpu
        from msgpu.pack import PackedBatch
        seeds = bench.rank_seeds(rank, batch)
        irs = bench.load_irs()
        packed = PackedBatch([msgpu.config_params("C2", seed=s, irs=irs) for s in seeds])
        elapsed = 0.25 * (rank + 1)            # rank 1 is the slow one
        dist.barrier()
        t = bench.max_over_ranks(elapsed, world, "cpu")
        q.put((rank, seeds, int(packed.total_frames), t))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharding_gloo():
    world, batch = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = [s for _, ss, _, _ in res for s in ss]
    assert seeds == list(range(1000, 1000 + world * batch))      # disjoint, contiguous
    assert all(t == pytest.approx(0.5) for *_, t in res)          # max over ranks
    assert res[0][2] == res[1][2] == batch * 192000               # C2: 1 s at 192 kHz


def _run_bench(*args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    # stdout is the one JSON line: gloo's "[Gloo] Rank r is connected to ..." goes to stderr
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    return json.loads(lines[0])


def test_launcher_two_ranks_dry_run():
    """bench.py --gpus 2 starts two rank processes itself (no torchrun): disjoint
    contiguous seeds, two child PIDs (neither the parent's), devices 0 and 1, and
    the job time is the slow rank's."""
    d = _run_bench("--gpus", "2", "--steps", "4", "--warmup", "1", "--batch", "3", "--config", "C2",
                   "--dry-run", "50")
    assert d["dry_run"] is True and d["n_gpus"] == 2
    ranks = sorted(d["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == [0, 1]
    assert [r["device"] for r in ranks] == [0, 1]
    pids = {r["pid"] for r in ranks}
    assert len(pids) == 2 and os.getpid() not in pids
    seeds = [s for r in ranks for s in r["seeds"]]
    assert seeds == list(range(1000, 1006))
    # rank 1 sleeps 100 ms per step, rank 0 50 ms: the max-reduced time is rank 1's
    assert d["elapsed_max_s"] >= 0.4
    assert d["elapsed_max_s"] == pytest.approx(max(r["elapsed_s"] for r in ranks), rel=0.05)
    assert ranks[0]["elapsed_s"] < d["elapsed_max_s"] + 1e-9
    assert d["value"] == pytest.approx(2 * 4 * 3 * 192000 / d["elapsed_max_s"] / 1e6)
    _check_rank_cpus(ranks)


def _check_rank_cpus(ranks):
    """Each rank runs on its own slice of the CPUs with a host pool sized to it."""
    have = len(os.sched_getaffinity(0))
    sets = [set(r["cpus"]) for r in ranks]
    if have >= len(ranks):
        assert not set.intersection(*sets), sets                        # disjoint
        assert all(len(c) == have // len(ranks) for c in sets), sets
    for r in ranks:
        assert 1 <= r["host_threads"] <= min(16, max(1, len(r["cpus"]))), r


def test_torchrun_two_ranks_dry_run():
    """The driver's N > 1 launch: ``python -m torch.distributed.run --nproc-per-node 2
    ... bench.py --gpus 2``.  Each process is one rank (RANK / LOCAL_RANK from the
    launcher, no second spawn), rank 0 prints the one line: two ranks on devices 0
    and 1 with disjoint contiguous seeds and the slow rank's time."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "2", "--config", "C2", "--dry-run", "40"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert all(x.startswith("{") for x in r.stdout.splitlines() if x.strip()), r.stdout   # nothing but the line
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout                       # rank 0 only
    d = lines[0]
    assert d["dry_run"] is True and d["n_gpus"] == 2
    ranks = sorted(d["ranks"], key=lambda q: q["rank"])
    assert [q["device"] for q in ranks] == [0, 1]
    assert len({q["pid"] for q in ranks}) == 2
    assert [s for q in ranks for s in q["seeds"]] == list(range(1000, 1004))
    assert d["elapsed_max_s"] == pytest.approx(max(q["elapsed_s"] for q in ranks), rel=0.05)
    _check_rank_cpus(ranks)


def test_launcher_one_rank_dry_run():
    """--gpus 1 stays in-process (no child)."""
    d = _run_bench("--gpus", "1", "--steps", "2", "--warmup", "0", "--batch", "2", "--config", "C2",
                   "--dry-run", "10")
    assert d["n_gpus"] == 1 and len(d["ranks"]) == 1
    assert d["ranks"][0]["seeds"] == [1000, 1001]


def test_launcher_propagates_rank_failure():
    """A failing rank stops the job with its exit code (the other rank is not left
    waiting in the barrier)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run", "10",
                        "--config", "NOPE", "--batch", "1"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=REPO)
    assert r.returncode != 0


def test_balance_contiguous_and_even():
    rng = np.random.default_rng(0)
    costs = rng.uniform(1, 10, size=1000)
    for world in (1, 2, 3, 8):
        cuts = bench.balance(costs, world)
        assert cuts[0] == 0 and cuts[-1] == costs.size and len(cuts) == world + 1
        assert all(a <= b for a, b in zip(cuts, cuts[1:]))
        loads = [costs[a:b].sum() for a, b in zip(cuts, cuts[1:])]
        assert max(loads) - min(loads) <= 2 * costs.max()
    # one expensive preset among cheap ones goes to a rank of its own
    cuts = bench.balance([1, 1, 1, 100, 1, 1, 1], 2)
    assert cuts == [0, 3, 7] or cuts == [0, 4, 7]


def test_plan_costs_track_config_size():
    """The host planner's cost estimate orders configs by their device work."""
    import msgpu
    irs = bench.load_irs()
    c2 = bench.plan_costs([msgpu.config_params("C2", seed=1000, irs=irs)])[0]
    c3 = bench.plan_costs([msgpu.config_params("C3", seed=1000, irs=irs)])[0]
    c5 = bench.plan_costs([msgpu.config_params("C5", seed=1000, irs=irs)])[0]
    assert 0 < c2 < c3 < c5


def test_single_rank_reduce_is_identity():
    assert bench.max_over_ranks(1.5, 1, "cpu") == 1.5
    assert np.array_equal(bench.rank_seeds(0, 4), [1000, 1001, 1002, 1003])


def test_stage_bytes_follow_the_fused_overlap_add():
    """bench.stage_bytes: with the overlap-add inside the FIR (fused share f),
    the grain reads move from the overlap-add to the FIR kernel and the mono
    write + read between them disappear; f = 0 is the two-kernel accounting,
    and fir_rfft sums the spectral and FIR bytes over the three stage windows."""
    class Info:
        def __init__(self, pool_len, out_n):
            self.pool_len, self.out_n = pool_len, out_n
    infos = [Info(1000, 400), Info(3000, 600)]
    sum_n, out_n = 4000, 1000
    plain = bench.stage_bytes(infos)
    assert plain["overlap_add"] == 4 * sum_n + 4 * out_n
    assert plain["fir_kernel"] == plain["fir"] == 8 * out_n
    assert plain["spectral"] == 8 * sum_n and plain["stereo"] == 16 * out_n
    fused = bench.stage_bytes(infos, fused=1.0)
    assert fused["overlap_add"] == 0
    assert fused["fir_kernel"] == 4 * sum_n + 4 * out_n
    half = bench.stage_bytes(infos, fused=0.5)
    assert half["overlap_add"] == 0.5 * plain["overlap_add"]
    assert half["fir_kernel"] == 0.5 * plain["fir_kernel"] + 0.5 * fused["fir_kernel"]
    assert bench.stage_bytes(infos, fused=7.0) == fused          # clamped to [0, 1]
    st = {"spectral": 2.0, "fir_h": 0.5, "fir_kernel": 1.5}
    r = bench.fir_rfft(plain, st, "test")
    assert r["ms"] == 4.0
    assert r["algorithmic_bytes"] == plain["spectral"] + plain["fir_kernel"]
    assert abs(r["achieved"] - r["algorithmic_bytes"] / 4e-3 / 1e9) < 0.1
