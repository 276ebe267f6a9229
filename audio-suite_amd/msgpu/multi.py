"""Multi-GPU rendering: one worker process per GPU.

A batch of presets is cut into contiguous ranges of equal predicted cost
(shard.balance over shard.plan_costs, the host plans) and each range renders on
its own GPU in its own process; the outputs come back through one shared-memory
block in the caller's order.  Nothing crosses GPUs, so there is no collective
(no RCCL): presets are independent renders (MS:588-792).

The workers are started with the ``spawn`` method before the calling process
touches the GPU -- a process that has initialised HIP must not start programs
(its children would inherit the device state), so :class:`DevicePool` refuses
to start after the first GPU call in this process.  Create it early::

    import msgpu
    pool = msgpu.DevicePool([0, 1, 2, 3, 4, 5, 6, 7])
    outs = pool.render_batch(params_list)          # list of (out_n, 2) float32
    # or: msgpu.render_batch(params_list, devices=range(8))

``stub=True`` replaces the device render with a host fill (column 0 = the
preset's index in the call, column 1 = the worker's device) so the sharding and
plumbing are testable without a GPU (tests/test_multi_cpu.py).
"""
from __future__ import annotations

import atexit
import os
import time
import uuid

import numpy as np


def _gpu_touched() -> bool:
    import sys
    if "torch" in sys.modules:
        try:
            if sys.modules["torch"].cuda.is_initialized():
                return True
        except Exception:
            pass
    from . import engine
    return bool(engine._engines)


def _worker(slot, device, nworkers, stub, conn):
    """Per-GPU worker: pin host CPUs, then render jobs until told to stop."""
    from multiprocessing import shared_memory
    from .shard import pin_worker_cpus
    cpus = pin_worker_cpus(slot, nworkers)
    eng = None
    if not stub:
        from .engine import Engine
        eng = Engine(device)
    conn.send(("ready", os.getpid(), device, len(cpus)))
    while True:
        msg = conn.recv()
        if msg[0] == "stop":
            break
        _, shm_name, idx, params, frame_off, out_n = msg
        t0 = time.perf_counter()
        err = None
        try:
            shm = shared_memory.SharedMemory(name=shm_name)
            try:
                _fill(shm, stub, eng, device, idx, params, frame_off, out_n)
            finally:
                shm.close()
        except Exception as e:       # reported to the caller, which raises
            err = repr(e)
        conn.send(("done", os.getpid(), device, list(idx), time.perf_counter() - t0, err))


def _fill(shm, stub, eng, device, idx, params, frame_off, out_n):
    buf = np.ndarray((shm.size // 8, 2), dtype=np.float32, buffer=shm.buf)
    if stub:
        for i, (o, n) in enumerate(zip(frame_off, out_n)):
            buf[o:o + n, 0] = float(idx[i])
            buf[o:o + n, 1] = float(device)
    elif params:
        _render_into(eng, params, buf, frame_off, out_n)


def _render_into(eng, params, buf, frame_off, out_n):
    """Render ``params`` on this worker's GPU in device batches, copying each
    batch's output into its frames of the shared block."""
    from .batch import _chunks
    from .pack import PackedBatch
    order = list(range(len(params)))
    for chunk in _chunks(order, lambda i: int(out_n[i])):
        packed = PackedBatch([params[i] for i in chunk])
        out = eng.render_packed(packed)
        eng.torch.cuda.synchronize(eng.device)
        host = out.cpu().numpy()
        for i, o, n in zip(chunk, packed.offsets, packed.out_n):
            buf[frame_off[i]:frame_off[i] + n] = host[o:o + n]


class DevicePool:
    """One worker process per device; ``render_batch`` shards by predicted cost."""

    def __init__(self, devices, stub: bool = False, share_devices: bool = False):
        """``share_devices=True`` lets several workers use one device (a rehearsal
        of the multi-process path on a one-GPU box, tools/multi_rehearsal.py)."""
        import multiprocessing as mp
        self.devices = [int(d) for d in devices]
        if not self.devices:
            raise ValueError("no devices")
        if not share_devices and len(set(self.devices)) != len(self.devices):
            raise ValueError("devices must be distinct")
        if not stub and _gpu_touched():
            raise RuntimeError("DevicePool must be created before this process makes its first GPU call "
                               "(its workers would inherit the initialised device)")
        self.stub = stub
        ctx = mp.get_context("spawn")
        self._conns, self._procs = [], []
        for slot, dev in enumerate(self.devices):
            a, b = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(slot, dev, len(self.devices), stub, b), daemon=True)
            p.start()
            self._conns.append(a)
            self._procs.append(p)
        self.workers = []
        for c in self._conns:
            tag, pid, dev, ncpu = c.recv()
            assert tag == "ready"
            self.workers.append({"pid": pid, "device": dev, "host_threads": ncpu})
        self.last_split = None
        atexit.register(self.close)

    def render_batch(self, params_list, costs=None):
        """Render ``params_list`` across the pool's GPUs; returns the (out_n, 2)
        float32 outputs in the caller's order.  ``last_split`` records each
        worker's preset range, predicted cost, pid and time."""
        from multiprocessing import shared_memory
        from .pack import PackedBatch
        from .shard import balance, plan_costs
        params_list = list(params_list)
        n = len(params_list)
        if n == 0:
            return []
        out_n = PackedBatch(params_list).out_n           # native pack: lengths (and early errors)
        costs = plan_costs(params_list) if costs is None else list(costs)
        cuts = balance(costs, len(self.devices))
        frames = int(out_n.sum())
        off = np.zeros(n, dtype=np.int64)
        off[1:] = np.cumsum(out_n)[:-1]
        shm = shared_memory.SharedMemory(create=True, size=max(8, frames * 8), name="msgpu_" + uuid.uuid4().hex[:16])
        try:
            live = []
            for w, c in enumerate(self._conns):
                lo, hi = cuts[w], cuts[w + 1]
                c.send(("job", shm.name, list(range(lo, hi)), params_list[lo:hi], off[lo:hi].tolist(),
                        out_n[lo:hi].tolist()))
                live.append((w, lo, hi))
            split, errors = [], []
            for w, lo, hi in live:
                tag, pid, dev, idx, dt, err = self._conns[w].recv()
                split.append({"device": dev, "pid": pid, "presets": [lo, hi], "cost": float(sum(costs[lo:hi])),
                              "seconds": dt})
                if err:
                    errors.append(f"device {dev}: {err}")
            self.last_split = split
            if errors:
                raise RuntimeError("; ".join(errors))
            return _copy_out(shm, frames, off, out_n)
        finally:
            shm.close()
            shm.unlink()

    def close(self):
        for c in getattr(self, "_conns", []):
            try:
                c.send(("stop",))
            except Exception:
                pass
        for p in getattr(self, "_procs", []):
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self._conns, self._procs = [], []


def _copy_out(shm, frames, off, out_n):
    all_frames = np.ndarray((frames, 2), dtype=np.float32, buffer=shm.buf)
    return [all_frames[o:o + k].copy() for o, k in zip(off, out_n)]


_POOLS: dict = {}


def pool_for(devices) -> DevicePool:
    key = tuple(int(d) for d in devices)
    if key not in _POOLS:
        _POOLS[key] = DevicePool(key)
    return _POOLS[key]
