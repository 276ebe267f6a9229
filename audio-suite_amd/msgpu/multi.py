"""Multi-GPU rendering: one worker process per GPU.

A batch of presets is cut into contiguous ranges of equal predicted cost
(shard.balance over shard.plan_costs, the host plans) and each range renders on
its own GPU in its own process.  Nothing crosses GPUs, so there is no
collective (no RCCL): presets are independent renders (MS:588-792).

Three result modes (``render_batch(..., results=...)``):

* ``"audio"`` (default): the (out_n, 2) float32 outputs come back through one
  shared-memory block, in the caller's order -- what ``render`` returns, for
  batches whose outputs fit in host memory.
* ``"stats"``: per preset only a summary -- out_n, rms over both channels, peak
  |x|, the sum of each channel and a 128-bit digest of the float32 interleaved
  bit patterns, all reduced on the device where the render lies (msg_digest,
  kernels_digest.h): 48 bytes per preset cross PCIe, no audio.  For C4/C5-scale
  batches (C5's ~550 GB of outputs cannot come back to one
  host); the reference's own batch path writes each render out one at a time
  (MS:1585-1589).  ``sha1=True`` adds the SHA-1 of each render's bytes (each
  preset then copied to the host alone and hashed).
* ``"device"``: the outputs stay in the workers' HBM; the call returns one
  :class:`DeviceResult` handle per preset.  ``pool.fetch(handle)`` copies one
  back, ``pool.release(handles)`` frees them.

Each worker renders its range in device batches (batch._chunks) and overlaps
the host side of the next batch (packing, the library's host plan, the enqueue)
with the device render of the current one; the previous batch's results are
drained on a second stream meanwhile.

The workers are started with the ``spawn`` method before the calling process
touches the GPU -- a process that has initialised HIP must not start programs
(its children would inherit the device state), so :class:`DevicePool` refuses
to start after the first GPU call in this process.  Create it early::

    import msgpu
    pool = msgpu.DevicePool([0, 1, 2, 3, 4, 5, 6, 7])
    outs = pool.render_batch(params_list)          # list of (out_n, 2) float32
    # or: msgpu.render_batch(params_list, devices=range(8))

Every job carries a sequence number and its shared-memory name, and every
reply is checked against both and against the job's preset range; a call that
is interrupted (or whose worker dies) closes the pool rather than leaving
replies in the pipes for the next call.

``stub=True`` replaces the device render with a host fill (column 0 = the
preset's index in the call, column 1 = the worker's device) so the sharding and
plumbing are testable without a GPU (tests/test_multi_cpu.py).
"""
from __future__ import annotations

import atexit
import hashlib
import os
import time
import uuid

import numpy as np

MODES = ("audio", "stats", "device")


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


def rec_stats(rec, out_n) -> dict:
    """The summary dict of one msg_digest record (rms over both channels)."""
    n = int(out_n)
    return {"out_n": n, "rms": float(np.sqrt(rec["sum_sq"] / (2 * n))) if n else 0.0,
            "peak": float(rec["peak"]), "sum_l": float(rec["sum_l"]), "sum_r": float(rec["sum_r"]),
            "digest": f"{int(rec['h0']):016x}{int(rec['h1']):016x}"}


def digest_host(a):
    """msg_digest_host of one (out_n, 2) float32 render in host memory: the record
    the device computes, bit for bit (numpy structured scalar)."""
    import ctypes as C
    from . import _lib as L
    from .engine import DIGEST_DTYPE
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != 2:
        raise ValueError("a must be (out_n, 2)")
    r = L.MsgDigestRec()
    L.check(L.lib().msg_digest_host(a.ctypes.data_as(C.c_void_p), int(a.shape[0]), C.byref(r)), None)
    return np.array([(r.sum_sq, r.peak, r.sum_l, r.sum_r, r.h0, r.h1)], dtype=DIGEST_DTYPE)[0]


def audio_stats(a, sha1: bool = False) -> dict:
    """Summary of one (out_n, 2) float32 render on the host: the same record
    msg_digest forms on the device (msg_digest_host), and the SHA-1 of its bytes
    when asked."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    st = rec_stats(digest_host(a), a.shape[0])
    if sha1:
        st["sha1"] = hashlib.sha1(a.tobytes()).hexdigest()
    return st


def device_stats(eng, out, offsets, out_n, stream=None, sha1: bool = False) -> list:
    """Summaries of the renders in a device output tensor, reduced on the device
    (Engine.digest); with sha1, each render is also copied to the host alone and
    hashed."""
    recs = eng.digest(out, offsets, out_n, stream=stream)
    res = [rec_stats(r, n) for r, n in zip(recs, out_n)]
    if sha1:
        for st, o, n in zip(res, offsets, out_n):
            st["sha1"] = hashlib.sha1(np.ascontiguousarray(out[int(o):int(o) + int(n)].cpu().numpy()).tobytes()).hexdigest()
    return res


def _stub_audio(i, device, n):
    a = np.empty((n, 2), dtype=np.float32)
    a[:, 0] = float(i)
    a[:, 1] = float(device)
    return a


def _worker(slot, device, nworkers, stub, conn):
    """Per-GPU worker: pin host CPUs, then render jobs until told to stop."""
    from .shard import pin_worker_cpus
    cpus = pin_worker_cpus(slot, nworkers)
    eng = None
    if not stub:
        from .engine import Engine
        eng = Engine(device)
    kept = {}                      # device mode: key -> device tensor (or host array in the stub)
    conn.send(("ready", os.getpid(), device, len(cpus)))
    while True:
        msg = conn.recv()
        if msg[0] == "stop":
            break
        if msg[0] == "fetch":
            _, seq, key = msg
            try:
                v = kept[key]
                arr = v if isinstance(v, np.ndarray) else v.cpu().numpy()
                conn.send(("fetched", seq, key, arr, None))
            except Exception as e:  # noqa: BLE001
                conn.send(("fetched", seq, key, None, repr(e)))
            continue
        if msg[0] == "release":
            for key in msg[2]:
                kept.pop(key, None)
            conn.send(("released", msg[1]))
            continue
        if msg[0] == "drop":          # a failed device-mode job: everything kept for it
            for key in [k for k in kept if k[0] == msg[2]]:
                del kept[key]
            conn.send(("released", msg[1]))
            continue
        _, seq, mode, shm_name, idx, params, frame_off, out_n = msg
        t0 = time.perf_counter()
        err, payload = None, None
        try:
            payload = _run_job(eng, stub, device, seq, mode, shm_name, idx, params, frame_off, out_n, kept)
        except Exception as e:  # noqa: BLE001  reported to the caller, which raises
            err = repr(e)
        conn.send(("done", seq, shm_name, os.getpid(), device, list(idx), time.perf_counter() - t0, err, payload))


def _run_job(eng, stub, device, seq, mode, shm_name, idx, params, frame_off, out_n, kept):
    """One job on this worker; the shared block (audio mode) is opened and
    closed here, and no view of it outlives the call (a live view would make
    close() raise BufferError and hide the job's own error)."""
    if mode == "audio":
        from multiprocessing import shared_memory
        shm = shared_memory.SharedMemory(name=shm_name)
        err = None
        try:
            _fill_audio(shm, stub, eng, device, idx, params, frame_off, out_n)
        except Exception as e:  # noqa: BLE001
            err = e
        finally:
            e2 = None
            try:
                shm.close()
            except BufferError as e:
                e2 = e
        if err is not None:
            raise err
        if e2 is not None:
            raise e2
        return None
    sha1 = mode == "stats_sha1"
    if sha1:
        mode = "stats"
    if stub:
        out = []
        for i, n in zip(idx, out_n):
            a = _stub_audio(i, device, int(n))
            if mode == "stats":
                out.append(audio_stats(a, sha1=sha1))
            else:
                key = (seq, int(i))
                kept[key] = a
                out.append(key)
        return out
    sink = _StatsSink(eng, sha1) if mode == "stats" else _KeepSink(kept, seq, idx)
    _render_chunks(eng, params, out_n, sink)
    return sink.result()


def _fill_audio(shm, stub, eng, device, idx, params, frame_off, out_n):
    buf = np.ndarray((shm.size // 8, 2), dtype=np.float32, buffer=shm.buf)
    try:
        if stub:
            for i, (o, n) in enumerate(zip(frame_off, out_n)):
                buf[o:o + n, 0] = float(idx[i])
                buf[o:o + n, 1] = float(device)
        elif params:
            _render_chunks(eng, params, out_n, _ShmSink(buf, frame_off))
    finally:
        del buf


class _ShmSink:
    """Audio mode: each preset's frames into its place in the shared block."""

    def __init__(self, buf, frame_off):
        self.buf, self.frame_off = buf, frame_off

    def take(self, chunk, packed, out):
        host = out.cpu().numpy()
        for i, o, n in zip(chunk, packed.offsets, packed.out_n):
            self.buf[self.frame_off[i]:self.frame_off[i] + n] = host[o:o + n]

    def result(self):
        return None


class _StatsSink:
    """Stats mode: per-preset summaries reduced on the device (one msg_digest per
    device batch, on the drain stream); with sha1, one preset's bytes at a time
    on the host."""

    def __init__(self, eng, sha1=False):
        self.eng, self.sha1 = eng, sha1
        self.stats = {}

    def take(self, chunk, packed, out):
        import torch
        res = device_stats(self.eng, out, packed.offsets, packed.out_n, stream=torch.cuda.current_stream(out.device),
                           sha1=self.sha1)
        for i, st in zip(chunk, res):
            self.stats[i] = st

    def result(self):
        return [self.stats[i] for i in sorted(self.stats)]


class _KeepSink:
    """Device mode: each preset's slice of its batch's output stays in HBM."""

    def __init__(self, kept, seq, idx):
        self.kept, self.seq, self.idx = kept, seq, list(idx)
        self.keys = {}

    def take(self, chunk, packed, out):
        for i, o, n in zip(chunk, packed.offsets, packed.out_n):
            key = (self.seq, int(self.idx[i]))
            self.kept[key] = out[int(o):int(o) + int(n)]
            self.keys[i] = key

    def result(self):
        return [self.keys[i] for i in sorted(self.keys)]


def _render_chunks(eng, params, lens, sink):
    """Render ``params`` (out_n ``lens``, from the job) in device batches on a
    render stream; while batch k renders, the host packs and plans batch k + 1
    and drains batch k - 1 (its output handed to ``sink.take(chunk, packed,
    out)`` on a second stream)."""
    from .batch import _chunks
    from .pack import PackedBatch
    torch = eng.torch
    dev = eng.device
    rs = torch.cuda.Stream(device=dev)
    cs = torch.cuda.Stream(device=dev)
    prev = None

    def drain(item):
        chunk, packed, out, ev = item
        with torch.cuda.stream(cs):
            cs.wait_event(ev)
            sink.take(chunk, packed, out)
        cs.synchronize()

    for chunk in _chunks(list(range(len(params))), lambda i: int(lens[i])):
        packed = PackedBatch([params[i] for i in chunk])
        out = eng.render_packed(packed, stream=rs)
        ev = torch.cuda.Event()
        ev.record(rs)
        if prev is not None:
            drain(prev)
        prev = (chunk, packed, out, ev)
    if prev is not None:
        drain(prev)
    rs.synchronize()


class DeviceResult:
    """A render kept in a worker's HBM (``results="device"``)."""

    __slots__ = ("pool_id", "worker", "key", "device", "index")

    def __init__(self, pool_id, worker, key, device, index):
        self.pool_id, self.worker, self.key, self.device, self.index = pool_id, worker, key, device, index

    def __repr__(self):
        return f"DeviceResult(preset {self.index} on device {self.device})"


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
        self._id = uuid.uuid4().hex[:12]
        self._seq = 0
        self._closed = False
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

    # ------------------------------------------------------------------
    def _next_seq(self):
        if self._closed:
            raise RuntimeError("DevicePool is closed (an earlier call failed or close() was called)")
        self._seq += 1
        return self._seq

    def _recv_checked(self, w, seq, shm_name, lo, hi):
        msg = self._conns[w].recv()
        if msg[0] != "done" or msg[1] != seq or msg[2] != shm_name or list(msg[5]) != list(range(lo, hi)):
            raise RuntimeError(f"worker {w} answered {msg[:3]} for job {seq} presets [{lo}, {hi}): "
                               "out of step, pool closed")
        return msg

    def render_batch(self, params_list, costs=None, results: str = "audio", sha1: bool = False):
        """Render ``params_list`` across the pool's GPUs.  Returns, in the caller's
        order, the (out_n, 2) float32 outputs (``results="audio"``), a summary dict
        per preset (``"stats"``: reduced on the device, see :func:`rec_stats`;
        ``sha1=True`` adds each render's SHA-1, which copies it to the host) or a
        :class:`DeviceResult` per preset (``"device"``).  ``last_split`` records
        each worker's preset range, predicted cost, pid and time."""
        from multiprocessing import shared_memory
        from .pack import PackedBatch
        from .shard import balance, plan_costs
        if results not in MODES:
            raise ValueError(f"results must be one of {MODES}")
        params_list = list(params_list)
        n = len(params_list)
        if n == 0:
            return []
        out_n = PackedBatch(params_list).out_n           # native pack: lengths (and early errors)
        costs = plan_costs(params_list) if costs is None else list(costs)
        cuts = balance(costs, len(self.devices))
        seq = self._next_seq()
        frames = int(out_n.sum())
        off = np.zeros(n, dtype=np.int64)
        off[1:] = np.cumsum(out_n)[:-1]
        shm = None
        if results == "audio":
            shm = shared_memory.SharedMemory(create=True, size=max(8, frames * 8),
                                             name="msgpu_" + uuid.uuid4().hex[:16])
        shm_name = shm.name if shm is not None else None
        try:
            try:
                live = []
                for w, c in enumerate(self._conns):
                    lo, hi = cuts[w], cuts[w + 1]
                    c.send(("job", seq, "stats_sha1" if (results == "stats" and sha1) else results, shm_name,
                            list(range(lo, hi)), params_list[lo:hi],
                            (off[lo:hi] if results == "audio" else np.zeros(hi - lo, np.int64)).tolist(),
                            out_n[lo:hi].tolist()))
                    live.append((w, lo, hi))
                split, errors, payloads = [], [], {}
                for w, lo, hi in live:
                    _, _, _, pid, dev, idx, dt, err, payload = self._recv_checked(w, seq, shm_name, lo, hi)
                    split.append({"device": dev, "pid": pid, "presets": [lo, hi],
                                  "cost": float(sum(costs[lo:hi])), "seconds": dt})
                    if err:
                        errors.append(f"device {dev}: {err}")
                    payloads[w] = payload
            except BaseException:
                self._fail()
                raise
            self.last_split = split
            if errors:
                if results == "device":     # drop what every worker kept for this job (a leak)
                    self._drop_job(seq, [w for w, _, _ in live])
                raise RuntimeError("; ".join(errors))
            if results == "audio":
                return _copy_out(shm, frames, off, out_n)
            out = []
            for w, lo, hi in live:
                got = payloads[w] or []
                if len(got) != hi - lo:
                    self._fail()
                    raise RuntimeError(f"worker {w} returned {len(got)} results for {hi - lo} presets")
                if results == "stats":
                    out.extend(got)
                else:
                    out.extend(DeviceResult(self._id, w, key, self.devices[w], lo + k) for k, key in enumerate(got))
            return out
        finally:
            if shm is not None:
                shm.close()
                shm.unlink()

    def fetch(self, handle: DeviceResult):
        """Copy one kept render back: (out_n, 2) float32."""
        if handle.pool_id != self._id:
            raise ValueError("handle belongs to another pool")
        seq = self._next_seq()
        try:
            self._conns[handle.worker].send(("fetch", seq, handle.key))
            tag, s, key, arr, err = self._conns[handle.worker].recv()
        except BaseException:
            self._fail()
            raise
        if tag != "fetched" or s != seq or key != handle.key:
            self._fail()
            raise RuntimeError("fetch reply out of step, pool closed")
        if err:
            raise KeyError(f"{handle}: {err}")
        return arr

    def release(self, handles):
        """Free kept renders (device mode)."""
        by_w = {}
        for h in handles:
            if h.pool_id != self._id:
                raise ValueError("handle belongs to another pool")
            by_w.setdefault(h.worker, []).append(h.key)
        self._release_keys(by_w)

    def _drop_job(self, job_seq, workers):
        """Device mode, failed job: each worker frees every render it kept for it
        (the successful workers' and a failed worker's partial ones)."""
        for w in workers:
            seq = self._next_seq()
            try:
                self._conns[w].send(("drop", seq, job_seq))
                tag, s = self._conns[w].recv()
            except BaseException:
                self._fail()
                raise
            if tag != "released" or s != seq:
                self._fail()
                raise RuntimeError("drop reply out of step, pool closed")

    def _release_keys(self, by_w):
        for w, keys in by_w.items():
            seq = self._next_seq()
            try:
                self._conns[w].send(("release", seq, keys))
                tag, s = self._conns[w].recv()
            except BaseException:
                self._fail()
                raise
            if tag != "released" or s != seq:
                self._fail()
                raise RuntimeError("release reply out of step, pool closed")

    def _fail(self):
        """A call was interrupted or a worker answered out of step: its pipes may
        hold stale replies, so the pool is closed and dropped from the cache."""
        for k, v in list(_POOLS.items()):
            if v is self:
                del _POOLS[k]
        self._closed = True
        for p in getattr(self, "_procs", []):
            if p.is_alive():
                p.terminate()
        for p in getattr(self, "_procs", []):
            p.join(timeout=10)
        self._conns, self._procs = [], []

    def close(self):
        self._closed = True
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
    try:
        return [all_frames[o:o + k].copy() for o, k in zip(off, out_n)]
    finally:
        del all_frames


_POOLS: dict = {}


def pool_for(devices) -> DevicePool:
    key = tuple(int(d) for d in devices)
    p = _POOLS.get(key)
    if p is None or p._closed:
        p = _POOLS[key] = DevicePool(key)
    return p
