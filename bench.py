#!/usr/bin/env python3
"""Benchmark: Msamples/s rendered by the MI355X Microsound render path.

Headline workload (BASELINE.json configs[2], SURVEY.md section 8 "C3"): 384 kHz
output, unfold x100 (design SR clamps to 30 MHz), spectral stretch x2, resonant
transient, Poisson events, 16 k-tap IR request (8192-tap cap, MS:443), early
reflections, stereo diffusion -- 1024 presets per GPU, seeds 1000 + rank*batch + b.
One step = one full render of the batch (device plan -> generate -> spectral ->
overlap-add -> FIR -> stereo/normalise) with the packed presets and IRs resident
and the output left in HBM.  Weak scaling: every rank renders its own batch.

    python bench.py [--gpus N --steps K --warmup W --config C3 --batch 1024 --points C4,C5]

Multi-GPU (presets are independent, no data-path
collective), two launch modes with the same per-rank code:
  * under torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK in the env): this
    process is one rank on device LOCAL_RANK;
  * ``--gpus N`` without a launcher: this process starts N rank processes itself
    (before it touches the GPU), one per device, and relays rank 0's line.
Ranks meet on a gloo group (127.0.0.1) for the timing barrier, the MAX of the
elapsed times and the per-rank record -- host-side only, no RCCL.

``--dry-run`` replaces the device render by a host sleep (for the CPU launcher
tests); it never prints a bench line the driver could take for a measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
# Per-launch HBM bytes of each kernel from rocprofv3 PMC passes (FETCH_SIZE x2
# per the gfx950 correction + WRITE_SIZE), written by tools/pmc_traffic.py:
# profiles/traffic_<config>.json, else the newest profiles/r*_traffic_<config>.json
# of the same launch size, else profiles/traffic.json (C3, round 1).
PROFILES = os.path.join(REPO, "profiles")
# bench stage -> the kernels it times (rocprofv3 kernel-name prefixes)
STAGE_KERNEL = {"generate": ("k_gen_normal",), "spectral": ("k_spec3", "k_spectral"), "overlap_add": ("k_ola_env",),
                "fir_kernel": ("k_fir8p<", "k_fir8<", "k_fir4<", "k_fir2<"),
                # the stereo window also holds the float64 FIR route (flag, h, spectra,
                # blocks, peak again) and the odd-length rotation
                "stereo": ("k_stereo_max", "k_stereo_out", "k_stereo_remax", "k_fir64", "k_h64", "k_hspec64", "k_so_"),
                "fir_h": ("k_er_gains", "k_fir8_hconv", "k_fir8_spec", "k_h_build", "k_fir4_hpart", "k_fir4_hconv",
                          "k_fir4_irspec", "k_fir_h", "k_ir_spec")}
STAGE_NAMES = ["plan", "host_prep", "generate", "spectral", "overlap_add", "fir", "stereo", "total",
               "fir_kernel", "fir_h", "host_plan_wall", "host_records_wall", "host_upload_wall",
               "host_plan_sizes", "host_plan_events", "host_preset_records", "host_event_records", "host_lists",
               "ola_fir_presets"]
KERNEL_STAGES = ["generate", "spectral", "overlap_add", "fir_kernel", "stereo"]
# the line's roofline kernel per config: the stage of the config's rocprof-dominant
# kernel (largest share of GPU time in profiles/r04h_*kernel_stats.csv: k_spec3 for
# C3 and C4, k_fir8p for C5), fixed so that roofline.frac is one kernel's series
# across rounds; other configs: the longest window of the run
DOMINANT_STAGE = {"C3": "spectral", "C4": "spectral", "C5": "fir_kernel"}
# the north star's "FIR + rFFT stage": the band-pruned / compile-time spectral
# kernels (rFFT -> band limit -> stretch -> irFFT), the filter spectra and the
# overlap-save FIR
FIR_RFFT_STAGES = ("spectral", "fir_h", "fir_kernel")
# host cores one GPU's rank uses at most (the GPU box's CPU share per GPU; nproc
# shows the whole machine).  The rank's actual set is its slice of the process
# affinity (pin_rank_cpus).
CORES_PER_GPU = 16

# Per-GPU batch of each config (BASELINE.json configs: C2 batch 1; C3 1024 on one
# GPU; C4 4096 and C5 8192 across 8 GPUs = 512 and 1024 per GPU) and the presets
# per in-flight sub-batch.  A C5 preset (8.4 M frames, 4000 events) needs ~0.2 GB
# of working buffers besides its 67 MB output, so C5 renders in sub-batches of 171
# (~35 GB of working buffers per context, three contexts, all outputs resident).
CONFIG_BATCH = {"C1": 1, "C2": 1, "C3": 1024, "C4": 512, "C5": 1024, "H48": 1024}
CONFIG_SUB = {"C5": 171}   # six sub-batches, two per stream (C5 ungated: 126.8 ms vs 130.6-132.2 at 128)
# host-bound short-step points: at ~2 ms per step, 10 steps (20 ms) swung by +-40 % between
# back-to-back runs on a shared-host box (profiles/r03an_h48_sweep.txt); time at least 50
POINT_STEPS_MIN = {"H48": 50, "C4": 30}
# stage events (msg_set_profiling) on every PROFILE_EVERY-th batch of a context
# inside the timed region, so that most batches run without the 12 timed events
# and the host read of the set: on H48's short step, in one session a run with
# every batch profiled took 1.02 - 1.18 ms against 0.81 - 0.87 for three
# unprofiled runs after it, but alternating A/Bs on other boxes stayed inside
# their +-30 % noise (profiles/r06pe_profile_sampling.txt)
PROFILE_EVERY = int(os.environ.get("MSGPU_BENCH_PROFILE_EVERY", "4"))   # the env: A/B only (0: no events)
# configs that run ungated under the default gate (measured slower with 2,4): C5, and
# H48, whose step is a per-stream chain of small kernels the gate serialises across
# the streams (1.06-1.24 vs 1.26-1.60 ms per step in five alternating pairs,
# profiles/r06g2_gate_points.txt; C4 within noise either way, so it keeps the gate)
GATE_OFF = {"C5", "H48"}
DEFAULT_GATE = "2,4"
WORKLOAD = {
    "C1": "C1: 48 kHz out, no band limit, unfold x1, stretch x1, Single event, 1 s, ER 320 taps, stereo",
    "C2": "C2: 192 kHz out, unfold x10 (1.92 MHz design SR), stretch x1, Poisson 18/s, 1 s, 4096-tap IR, "
          "ER 320 taps, stereo",
    "C3": "C3: 384 kHz out, unfold x100 (30 MHz design SR), stretch x2, Poisson 18/s, 1 s, "
          "16k-tap IR request (8192 cap), ER 320 taps, stereo",
    "C4": "C4: 384 kHz out, unfold x200 (30 MHz design SR), stretch x4, Poisson 18/s, 1 s, "
          "64k-tap IR request (8192 cap), ER 320 taps, stereo",
    "C5": "C5: 3072 Hz out x unfold 500 (1.536 MHz design SR), stretch x4, 8388608 frames, Poisson capped "
          "at 4000 events, 64k-tap IR request (8192 cap), ER 320 taps, stereo",
    "H48": "H48: 48 kHz out, unfold x8 (384 kHz design SR), Poisson 18/s, 1 s, 4096-tap IR, ER 320 taps, "
           "stereo",
}


def load_irs():
    z = np.load(os.path.join(REPO, "tests", "golden", "irs.npz"))
    return {k: z[k] for k in z.files}


def stage_bytes(infos, fused=0.0):
    """Algorithmic (compulsory) HBM bytes per stage for the presets in ``infos``
    (DESIGN.md section 4).  ``fused``: the share of them whose overlap-add ran
    inside the FIR kernel (stage time "ola_fir_presets" over the presets per
    batch): their grain reads move from the overlap-add to the FIR, and the
    mono buffer between the two is neither written nor read."""
    sum_n = sum(int(i.pool_len) for i in infos)
    out_n = sum(int(i.out_n) for i in infos)
    f = min(max(float(fused), 0.0), 1.0)
    ola = 4 * sum_n + 4 * out_n                # placed grains read + mono written (upper bound)
    fir = 8 * out_n                            # mono read + y written
    fir_fused = 4 * sum_n + 4 * out_n          # placed grains read + y written
    return {
        "generate": 4 * sum_n,                 # grain samples written once
        "spectral": 8 * sum_n,                 # grain read + grain written (one LDS round trip)
        "overlap_add": (1 - f) * ola,
        "fir": (1 - f) * fir + f * fir_fused,
        "fir_kernel": (1 - f) * fir + f * fir_fused,   # k_fir alone: same compulsory bytes
        "stereo": 16 * out_n,                  # max pass reads y; output pass reads y, writes L/R
    }


def measured_traffic(prefixes, cfg, batch):
    """HBM bytes per launch of the stage's kernels (name prefixes) from the
    committed PMC summary of this workload, or None when there is none (bench
    cannot read PMC itself)."""
    import glob
    import re

    def tag_order(path):                # r03z < r03aa < r03ae: round, then tag length, then tag
        m = re.match(r"r(\d+)([a-z]*)_", os.path.basename(path))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, "")
    newest = sorted(glob.glob(os.path.join(PROFILES, f"r*_traffic_{cfg}.json")), key=tag_order, reverse=True)
    for path in (os.path.join(PROFILES, f"traffic_{cfg}.json"), *newest, os.path.join(PROFILES, "traffic.json")):
        try:
            with open(path) as f:
                t = json.load(f)
        except (OSError, ValueError):
            continue
        if t.get("config") != cfg or int(t.get("batch", -1)) != batch:
            continue
        tot = [rec.get("hbm_bytes_per_launch") for name, rec in t.get("kernels", {}).items()
               if name.startswith(tuple(prefixes))]
        if tot and all(v is not None for v in tot):
            return sum(tot)
    return None


def kernel_label(stage):
    if stage == "fir_kernel":           # one of them per preset, by FIR size (C3/C4/C5: k_fir8p)
        return " / ".join(k.rstrip("<") for k in STAGE_KERNEL[stage])
    if stage == "stereo":               # the window also holds the float64 route's flag / slot kernels
        return "k_stereo_max+k_stereo_out (window incl. the float64 FIR route's flag)"
    return "+".join(k.rstrip("<") for k in STAGE_KERNEL[stage])


# ---------------------------------------------------------------------------
# CPU baseline (rank 0 at N = 1 only, before the GPU is touched)
def _cpu_worker(job):
    """Render presets seed0, seed0 + stride, ... with the oracle for budget_s seconds."""
    cfg, seed0, stride, budget_s = job
    from oracle import msound_oracle as O   # CPU baseline only
    import msgpu
    irs = load_irs()
    done = frames = 0
    t0 = time.perf_counter()
    while True:
        p = msgpu.config_params(cfg, seed=seed0 + done * stride, irs=irs)
        a, _ = O.render(p)
        frames += a.shape[0]
        done += 1
        if time.perf_counter() - t0 >= budget_s or done >= 256:
            break
    return done, frames, time.perf_counter() - t0


def cpu_baseline(cfg, budget_s):
    """The NumPy restatement of render() on the host: one core,
    then one process per core of the box's share.  Runs before the GPU is touched
    (the pool forks)."""
    import multiprocessing as mp
    done, frames, dt = _cpu_worker((cfg, 1000, 1, budget_s))
    single = frames / dt / 1e6
    procs = max(1, min(CORES_PER_GPU, len(os.sched_getaffinity(0))))
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(cfg, 1000 + i, procs, budget_s) for i in range(procs)])
    wall = time.perf_counter() - t0
    pdone = sum(r[0] for r in res)
    pframes = sum(r[1] for r in res)
    # one C2 preset on one core: the per-render time the drop-in is compared with
    from oracle import msound_oracle as O
    p2 = msgpu_config("C2")
    c2 = []
    for _ in range(3):
        t1 = time.perf_counter()
        O.render(p2)
        c2.append(time.perf_counter() - t1)
    return {"value": pframes / wall / 1e6, "unit": "Msamples/s", "cores": procs, "kind": "port",
            "cores_note": f"one process per core of this rank's CPU share: min({CORES_PER_GPU}, affinity "
                          f"{len(os.sched_getaffinity(0))}); the GPU box gives one GPU a 16-core share of a "
                          "host whose affinity lists all of its cores (nproc shows the whole machine)",
            "single_core": round(single, 4),
            "per_render_ms_1core": {"C2": round(1e3 * float(np.median(c2)), 2), cfg: round(1e3 * dt / done, 2)},
            "sample": f"{cfg} presets rendered by oracle/msound_oracle.py (NumPy restatement of "
                      f"main_v2.render): {done} presets on 1 core in {dt:.1f} s "
                      f"({single:.3f} Msamples/s), then {pdone} presets on {procs} processes in "
                      f"{wall:.1f} s"}


# ---------------------------------------------------------------------------
# sharding
def msgpu_config(cfg, seed=1000):
    import msgpu
    return msgpu.config_params(cfg, seed=seed, irs=load_irs())


def dropin_latency(cpu, reps=5):
    """msgpu.render() of one preset, end to end as the unchanged UI calls it
    (MS:811): dict checks and packing, host plan, enqueue, device render, D2H copy
    of the (out_n, 2) float32 buffer and meta -- beside the CPU per-render time."""
    import msgpu
    out = {}
    for cfg in ("C2", "C3"):
        p = msgpu_config(cfg)
        msgpu.render(p)                                    # warm (plans, buffers)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            msgpu.render(p)
            ts.append(time.perf_counter() - t0)
        rec = {"gpu_ms": round(1e3 * float(np.median(ts)), 3), "reps": reps}
        c = (cpu or {}).get("per_render_ms_1core", {}).get(cfg)
        if c:
            rec["cpu_ms_1core"] = c
            rec["speedup"] = round(c / rec["gpu_ms"], 1)
        out[cfg] = rec
    return out


def pin_rank_cpus(local, local_world):
    """Before the first GPU call: this rank's slice of the process affinity and
    host pool size (msgpu.shard.pin_worker_cpus, shared with msgpu.DevicePool)."""
    from msgpu.shard import pin_worker_cpus
    return pin_worker_cpus(local, local_world)


def host_threads():
    from msgpu import _lib as L
    return int(L.lib().msg_host_threads())


def rank_seeds(rank, batch):
    """Preset seeds of one rank: contiguous, disjoint across ranks (weak scaling)."""
    return [1000 + rank * batch + b for b in range(batch)]


from msgpu.shard import balance, plan_costs, preset_cost  # noqa: E402,F401  (the library's sharding)


class Comm:
    """Host-side rank group (gloo over 127.0.0.1): barrier, MAX, gather.  No RCCL:
    nothing on the data path crosses GPUs."""

    def __init__(self, rank, world):
        self.rank, self.world = rank, world
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=rank, world_size=world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if not self.dist:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def max_over_ranks(elapsed, world, _device=None):
    """The job's time is the slowest rank's (all-reduce MAX on the host group)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---------------------------------------------------------------------------
# one GPU's work
class Workload:
    """One config's presets on this rank, packed into in-flight sub-batches."""

    def __init__(self, cfg, seeds, sub, irs, n_engines):
        import msgpu
        from msgpu.pack import PackedBatch
        self.cfg = cfg
        self.seeds = seeds
        self.params = [msgpu.config_params(cfg, seed=s, irs=irs) for s in seeds]
        sub = max(1, min(sub, len(seeds)))
        nsub = max(n_engines, -(-len(seeds) // sub)) if len(seeds) >= n_engines else len(seeds)
        self.cut = [len(seeds) * i // nsub for i in range(nsub + 1)]
        self.subs = [PackedBatch(self.params[self.cut[i]:self.cut[i + 1]]) for i in range(nsub)]
        self.frames = sum(p.total_frames for p in self.subs)
        self.outs = None


class GpuRunner:
    """S contexts + HIP streams on one device (one in-flight render per stream,
    SURVEY section 8(e)); sub-batch i renders on context i mod S, so the host
    plans one sub-batch while the device runs another and their kernels share
    the CUs."""

    def __init__(self, dev, streams, gate=None, threaded=True):
        import torch
        from msgpu.engine import Engine
        self.torch = torch
        self.dev = dev
        torch.cuda.set_device(dev)
        self.engs = [Engine(dev) for _ in range(streams)]
        self.streams = [torch.cuda.Stream(device=dev) for _ in range(streams)]
        self.set_gate(gate)
        # one enqueueing host thread per context: the host plans / records / uploads
        # of the contexts' sub-batches overlap (ctypes drops the GIL in the library,
        # whose host pool runs the callers' jobs side by side)
        self.pool = None
        if threaded and streams > 1:
            from concurrent.futures import ThreadPoolExecutor
            self.pool = ThreadPoolExecutor(max_workers=streams, thread_name_prefix="msgpu-enqueue")

    def set_gate(self, gate):
        """msg_gate between the contexts: each waits for the previous one's stage
        gate[1] before its stage gate[0]; None clears."""
        if len(self.engs) < 2:
            return
        for i, e in enumerate(self.engs):
            if gate:
                e.gate(self.engs[i - 1], gate[0], gate[1])
            else:
                e.gate(None)

    def prepare(self, w: Workload):
        S = len(self.engs)
        w.outs = [self.engs[i % S].alloc_output(p) for i, p in enumerate(w.subs)]

    def step(self, w: Workload, from_dicts: bool = False):
        """One render of the workload; from_dicts: each sub-batch's param dicts are
        packed again inside the step (what msgpu.render_batch's caller pays)."""
        S = len(self.engs)

        def sub(i):
            if not from_dicts:
                return w.subs[i]
            from msgpu.pack import PackedBatch
            return PackedBatch(w.params[w.cut[i]:w.cut[i + 1]])
        if self.pool is None:
            for i, o in enumerate(w.outs):
                self.engs[i % S].render_packed(sub(i), o, self.streams[i % S])
            return

        def run(e):
            for i in range(e, len(w.subs), S):
                self.engs[e].render_packed(sub(i), w.outs[i], self.streams[e])
        for f in [self.pool.submit(run, e) for e in range(min(S, len(w.subs)))]:
            f.result()

    def sync(self):
        self.torch.cuda.synchronize(self.dev)

    def profiling(self, on):
        for e in self.engs:
            e.set_profiling(on)

    def stage_ms(self):
        return np.mean([np.array(e.stage_times()) for e in self.engs], axis=0)

    def infos(self, w: Workload):
        """Plan summaries of every preset of ``w``.  Each context keeps the plan of
        the last sub-batch it rendered; earlier sub-batches are planned again."""
        S = len(self.engs)
        nsub = len(w.subs)
        self.sync()
        per = {i: self.engs[i % S].last_plan() for i in range(max(0, nsub - S), nsub)}
        for i in range(max(0, nsub - S)):
            e = self.engs[i % S]
            e.render_packed(w.subs[i], w.outs[i], self.streams[i % S])
            self.sync()
            per[i] = e.last_plan()
        return [x for i in range(nsub) for x in per[i]]

    def check(self, w: Workload, golden, k=4):
        """Summaries of the first k presets of sub-batch 0 against the reference's
        (tests/golden/golden_info.json, golden_extra.json): |rms - ref| <= 1e-5,
        |sum - ref| <= 1e-5 n."""
        res = {}
        host = None
        for j, seed in enumerate(w.seeds[:min(k, w.subs[0].n)]):
            ref = golden.get(f"{w.cfg}_{seed}")
            if ref is None:
                continue
            if host is None:
                self.sync()
                host = w.outs[0].cpu().numpy()
            o, n = int(w.subs[0].offsets[j]), int(w.subs[0].out_n[j])
            a = host[o:o + n].astype(np.float64)
            d = {"rms": abs(float(np.sqrt(np.mean(a ** 2))) - ref["rms"]),
                 "sum_l": abs(float(a[:, 0].sum()) - ref["sum_l"]) / n,
                 "sum_r": abs(float(a[:, 1].sum()) - ref["sum_r"]) / n}
            res[str(seed)] = {k2: float(f"{v:.3g}") for k2, v in d.items()}
            res[str(seed)]["ok"] = bool(max(d.values()) <= 1e-5 and list(a.shape) == ref["shape"])
        return {"presets": res, "all_ok": bool(res) and all(v["ok"] for v in res.values()),
                "tolerance": "|rms - ref| <= 1e-5 and |sum_ch - ref| <= 1e-5 * out_n against the "
                             "reference render's summaries (golden_info.json)"} if res else None

    def free(self, w: Workload):
        w.outs = None
        self.torch.cuda.empty_cache()

    def free_cache(self):
        self.torch.cuda.empty_cache()


class DryRunner:
    """Stand-in for GpuRunner in the CPU launcher tests: a step sleeps
    dry_ms * (rank + 1) ms, so the slowest rank is known."""

    def __init__(self, rank, dry_ms):
        self.delay = dry_ms * (rank + 1) / 1e3
        self.dev = rank

    def prepare(self, w):
        pass

    def step(self, w, **kw):
        time.sleep(self.delay)

    def sync(self):
        pass


def timed(runner, w, steps, warmup, comm, **kw):
    """W untimed steps, then K steps bracketed by barrier + device sync; returns
    (this rank's seconds, max over ranks)."""
    for _ in range(warmup):
        runner.step(w, **kw)
    runner.sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.step(w, **kw)
    runner.sync()
    comm.barrier()
    mine = time.perf_counter() - t0
    return mine, comm.max(mine)


def measure(runner, cfg, seeds, sub, steps, warmup, comm, irs, golden, iso_steps=0, from_dicts_steps=0):
    """Time one config on this rank; returns the point record (rank 0 fills it)."""
    world = comm.world
    w = Workload(cfg, seeds, sub, irs, len(runner.engs))
    runner.prepare(w)
    for _ in range(max(1, warmup)):
        runner.step(w)
    runner.sync()
    runner.profiling(PROFILE_EVERY)
    mine, elapsed = timed(runner, w, steps, 0, comm)
    runner.profiling(False)
    stages = {n: round(float(v), 4) for n, v in zip(STAGE_NAMES, runner.stage_ms())}
    check = runner.check(w, golden) if comm.rank == 0 else None
    infos = runner.infos(w)
    nsub = len(w.subs)
    sb = stage_bytes(infos, stages.get("ola_fir_presets", 0.0) * nsub / max(1, len(seeds)))
    sb_launch = {k: v / nsub for k, v in sb.items()}
    longest = max(KERNEL_STAGES, key=lambda k: stages[k])
    dom = DOMINANT_STAGE.get(cfg, longest)
    achieved = sb_launch[dom] / (stages[dom] * 1e-3) / 1e9 if stages[dom] > 0 else 0.0
    launch_batch = len(seeds) // nsub
    sum_n = sum(int(i.pool_len) for i in infos)
    n_ev = sum(int(i.n_events) for i in infos)
    rec = {
        "value": round(w.frames * world * steps / elapsed / 1e6, 3), "unit": "Msamples/s",
        "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps,
        "workload": WORKLOAD.get(cfg, cfg), "presets_per_gpu": len(seeds), "sub_batches": nsub,
        "frames_per_gpu_step": w.frames, "events_per_gpu_step": n_ev, "design_samples_per_gpu_step": sum_n,
        "design_msamples_per_s": round(sum_n * world * steps / elapsed / 1e6, 1),
        "roofline": {"bound": "hbm", "kernel": kernel_label(dom),
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": measured_traffic(STAGE_KERNEL[dom], cfg, launch_batch),
                     "algorithmic_bytes": sb_launch[dom], "kernel_ms": stages[dom],
                     "kernel_choice": "the config's rocprof-dominant kernel (DOMINANT_STAGE)" if cfg in DOMINANT_STAGE
                                      else "the longest window of this run",
                     "longest_window_stage": longest,
                     "fir_rfft_stage": {"timed": fir_rfft(sb_launch, stages, "per launch in the timed region")},
                     "note": f"per launch in the timed region ({nsub} sub-batches of ~{launch_batch} presets "
                             f"on {len(runner.engs)} streams sharing the GPU)"},
        "stage_ms": stages,
        "stage_algorithmic_GBs": {k: round(sb_launch[k] / (stages[k] * 1e-3) / 1e9, 1)
                                  for k in sb if stages.get(k, 0) > 0},
        "check": check, "_rank_s": mine,
    }
    if from_dicts_steps > 0:
        # the same steps with the dict -> msg_preset packing inside each step
        # (native packer, msgpu/_mspack): what a caller of msgpu.render_batch pays
        _, el2 = timed(runner, w, from_dicts_steps, 1, comm, from_dicts=True)
        rec["from_dicts"] = {"value": round(w.frames * world * from_dicts_steps / el2 / 1e6, 3),
                             "ms_per_step": round(el2 / from_dicts_steps * 1e3, 3), "steps": from_dicts_steps,
                             "pack_ms_per_step": round(pack_ms(w), 3),
                             "note": "packing of every sub-batch's param dicts inside the timed step"}
    if iso_steps > 0:
        rec["roofline_isolated"] = isolated(runner, w, iso_steps, sb, cfg)
        rec["roofline"]["fir_rfft_stage"]["isolated"] = rec["roofline_isolated"]["fir_rfft_stage"]
    runner.free(w)
    return rec


def fir_rfft(sbytes, st_ms, where):
    """The north star's FIR + rFFT stage (FIR_RFFT_STAGES): the spectral and FIR
    kernels' algorithmic bytes (grain read + write, mono read + write; the filter
    spectra's own writes, 8 B x 32 769 per preset, are not counted) over the sum
    of the three stages' windows (h spectra included)."""
    b = sbytes["spectral"] + sbytes["fir_kernel"]
    ms = sum(st_ms.get(k, 0.0) for k in FIR_RFFT_STAGES)
    ach = b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    return {"kernels": "k_spec3 / k_spectral_ct + k_fir8_hconv / k_fir8_spec + k_fir8p",
            "algorithmic_bytes": b, "ms": round(ms, 4), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "stage_ms": {k: st_ms.get(k) for k in FIR_RFFT_STAGES}, "note": where}


# ---------------------------------------------------------------------------
# standalone FIR points (SURVEY section 8 config remarks, 8(d)): the 16 k / 64 k-tap
# filters BASELINE configs[2] / [3] request, which render() caps at 8192 taps (MS:443)
FIR_SIGNALS, FIR_N = 1024, 384000     # C3's batch and output length


def fir_taps(M, seed=7):
    """SURVEY section 8(d)'s synthetic IR: default_rng(7).standard_normal(M) exp(-6t/M), peak 0.9."""
    h = np.random.default_rng(seed).standard_normal(M) * np.exp(-6.0 * np.arange(M) / M)
    return h * (0.9 / float(np.max(np.abs(h))))


def fir_signals(seeds, n):
    """x_b = default_rng(b).standard_normal(n) as float32, drawn on host threads."""
    from concurrent.futures import ThreadPoolExecutor
    x = np.empty((len(seeds), n), np.float32)

    def fill(i):
        x[i] = np.random.default_rng(seeds[i]).standard_normal(n, dtype=np.float32)
    with ThreadPoolExecutor(max_workers=CORES_PER_GPU) as ex:
        list(ex.map(fill, range(len(seeds))))
    return x


def np_fir_window(x, h, lo, hi):
    """y[lo:hi] of np.convolve(x, h)[:n] (MS:444's arithmetic, float64), from the
    inputs that reach it only: x[max(0, lo - M + 1):hi]."""
    M = len(h)
    a = max(0, lo - M + 1)
    y = np.convolve(np.asarray(x[a:hi], np.float64), h)
    return y[lo - a:hi - a]


class FirRunner:
    """One msg_fir call over the batch of signals = one step (same timing protocol)."""

    def __init__(self, eng, x, y, h, stream):
        self.eng, self.x, self.y, self.h, self.stream = eng, x, y, h, stream
        self.shape = None
        self.torch = eng.torch

    def step(self, w=None, **kw):
        _, self.shape = self.eng.fir(self.x, self.h, out=self.y, stream=self.stream)

    def sync(self):
        self.torch.cuda.synchronize(self.eng.device)


def measure_fir(runner, M, steps, comm, rank, cpu=False):
    """The standalone FIR point: FIR_SIGNALS signals of FIR_N samples through
    msg_fir with an M-tap filter.  value = output samples / s over all ranks;
    roofline = algorithmic bytes S (8 n + 4 M) over the device time per call
    (HIP events on the call's stream); check = |y - np.convolve(x, h)[:n]| RMS
    relative to the output RMS <= 1e-5 on the first and last signal, over a head
    and a tail window (edges of the first and last blocks)."""
    import torch
    seeds = [rank * FIR_SIGNALS + b for b in range(FIR_SIGNALS)]
    xh = fir_signals(seeds, FIR_N)
    h = fir_taps(M)
    eng = runner.engs[0]
    stream = runner.streams[0]
    x = torch.from_numpy(xh).to(f"cuda:{runner.dev}")
    y = torch.empty_like(x)
    fr = FirRunner(eng, x, y, h, stream)
    for _ in range(3):
        fr.step()
    fr.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    comm.barrier()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fr.step()
    e1.record(stream)
    fr.sync()
    comm.barrier()
    mine = time.perf_counter() - t0
    elapsed = comm.max(mine)
    dev_ms = e0.elapsed_time(e1) / steps
    N, P, Q = fr.shape
    engine = {(65536, 1): "k_fir8p", (65536, 2): "k_fir8p (two partitions)"}.get(
        (N, Q), "k_fdl" if P == N // 2 and Q >= 8 else ("k_fir4" if N == 32768 else "k_fir2"))
    S, n = FIR_SIGNALS, FIR_N
    alg = S * (8.0 * n + 4.0 * M)
    rec = {"value": round(S * n * comm.world * steps / elapsed / 1e6, 3), "unit": "Msamples/s",
           "ms_per_step": round(elapsed / steps * 1e3, 4), "steps": steps,
           "workload": f"standalone FIR: {S} signals x {n} samples, {M}-tap synthetic IR (SURVEY 8(d)), "
                       "y = np.convolve(x, h)[:n] (MS:444 without the MS:443 cap)",
           "fir_shape": {"N": fr.shape[0], "P": fr.shape[1], "Q": fr.shape[2]},
           "roofline": {"bound": "hbm", "kernel": f"msg_fir: filter spectra + {engine}", "achieved": round(alg / (dev_ms * 1e-3) / 1e9, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(alg / (dev_ms * 1e-3) / 8e12, 4),
                        "algorithmic_bytes": alg, "kernel_ms": round(dev_ms, 4),
                        "note": "device time per call (HIP events on its stream), filter spectra included"},
           "_rank_s": mine}
    if rank == 0:
        yh = y.cpu().numpy()
        res, ok = {}, True
        for b in (0, S - 1):
            for lo, hi in ((0, 40000), (n - 20000, n)):
                r = np_fir_window(xh[b], h, lo, hi)
                e = float(np.sqrt(np.mean((yh[b, lo:hi] - r) ** 2)) / max(np.sqrt(np.mean(r ** 2)), 1e-30))
                res[f"{b}:{lo}-{hi}"] = float(f"{e:.3g}")
                ok &= e <= 1e-5
        rec["check"] = {"windows": res, "all_ok": bool(ok),
                        "tolerance": "RMS(y - np.convolve(x, h)[:n]) / RMS <= 1e-5 (float64 reference) on the "
                                     "first and last signal, head and tail windows"}
        if cpu:
            t0 = time.perf_counter()
            np_fir_window(xh[0], h, 0, 40000)
            dt = time.perf_counter() - t0
            rec["cpu_baseline"] = {"value": round(40000 / dt / 1e6, 4), "unit": "Msamples/s", "cores": 1,
                                   "kind": "reference",
                                   "sample": "np.convolve (the reference's own call, MS:444) of a 40000-sample "
                                             "window on one host core"}
    del x, y
    runner.free_cache()
    return rec


def pack_ms(w, reps=5):
    """Host time to pack the workload's param dicts (all sub-batches), best of reps."""
    from msgpu.pack import PackedBatch
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        for i in range(len(w.subs)):
            PackedBatch(w.params[w.cut[i]:w.cut[i + 1]])
        best = min(best, time.perf_counter() - t0)
    return best * 1e3


def isolated(runner, w, iso_steps, sb, cfg):
    """The whole batch on one stream, kernels not sharing the GPU."""
    from msgpu.pack import PackedBatch
    whole = len(w.subs) == len(runner.engs)
    # sub-batched configs (C5): the whole batch does not fit one launch, so the
    # isolated figure is one sub-batch alone on one stream, with its own bytes
    packed = PackedBatch(w.params) if whole else w.subs[0]
    e = runner.engs[0]
    o = e.alloc_output(packed)
    e.render_packed(packed, o, runner.streams[0])
    runner.sync()
    e.set_profiling(True)
    for _ in range(iso_steps):
        e.render_packed(packed, o, runner.streams[0])
    runner.sync()
    e.set_profiling(False)
    iso = {n: round(float(v), 4) for n, v in zip(STAGE_NAMES, e.stage_times())}
    infos = e.last_plan()
    sb = stage_bytes(infos, iso.get("ola_fir_presets", 0.0) / max(1, len(infos)))
    dom = DOMINANT_STAGE.get(cfg, max(KERNEL_STAGES, key=lambda k: iso[k]))
    ach = sb[dom] / (iso[dom] * 1e-3) / 1e9
    kern = [k for k in KERNEL_STAGES if iso.get(k, 0) > 0]
    tot_bytes = sum(sb[k] for k in kern)
    tot_ms = sum(iso[k] for k in kern)
    del o
    return {"kernel": kernel_label(dom), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "algorithmic_bytes": sb[dom],
            "kernel_ms": iso[dom], "traffic": measured_traffic(STAGE_KERNEL[dom], cfg, packed.n),
            "stage_ms": iso,
            "stage_frac": {k: round(sb[k] / (iso[k] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) for k in kern},
            "kernels_frac": round(tot_bytes / (tot_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "fir_rfft_stage": fir_rfft(sb, iso, "whole batch (or one sub-batch) alone on one stream"),
            "presets": packed.n,
            "note": (f"whole batch on one stream, {iso_steps} renders after the timed region" if whole else
                     f"one sub-batch of {packed.n} presets alone on one stream, {iso_steps} renders after the "
                     "timed region")}


# ---------------------------------------------------------------------------
def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100,
                    help="timed steps (100 C3 steps keep the GPU busy for ~1 s, long enough for an outside sampler)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batch", type=int, default=0, help="presets per GPU (0: the config's default)")
    ap.add_argument("--sub", type=int, default=0, help="presets per in-flight sub-batch (0: config default)")
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--streams", type=int, default=3,
                    help="in-flight sub-batches (contexts/streams) per GPU (C3 with the 2,4 gate: 3 streams "
                         "9.35-9.38 ms vs 2 streams 9.45 ms per step, profiles/r02zh_streams.txt)")
    ap.add_argument("--gate", default=DEFAULT_GATE,
                    help="WAIT,RECORD stages of msg_gate between the streams' contexts, or none.  Default 2,4: a "
                         "sub-batch's generator waits until the previous sub-batch's overlap-add begins, so it "
                         "runs beside that sub-batch's FIR and stereo passes rather than its spectral kernel "
                         "(C3: 9.43-9.45 vs 9.52-9.54 ms per step ungated, profiles/r02ze_gate.txt)")
    ap.add_argument("--iso-steps", type=int, default=3, help="single-stream renders for roofline_isolated")
    ap.add_argument("--from-dicts-steps", type=int, default=20,
                    help="steps timed again with the param-dict packing inside the step (0 = skip)")
    ap.add_argument("--enqueue", choices=["threads", "serial"], default="threads",
                    help="enqueue the contexts' sub-batches from one host thread each (threads) or in turn")
    ap.add_argument("--points", default="H48,C4,C5",
                    help="secondary configs timed after the headline (comma list, '' = none)")
    ap.add_argument("--point-steps", type=int, default=10)
    ap.add_argument("--fir-points", default="16384,65536",
                    help="standalone FIR tap counts timed after the points (comma list, '' = none)")
    ap.add_argument("--dry-run", type=float, default=0.0, metavar="MS",
                    help="CPU launcher test: a step sleeps MS*(rank+1) ms instead of rendering")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="every rank renders on device 0 (a rehearsal of the multi-rank path on a "
                         "one-GPU box; the ranks share the GPU, so the line is not a scaling point)")
    return ap.parse_args()


def default_batch(cfg, args):
    return args.batch if (args.batch > 0 and cfg == args.config) else CONFIG_BATCH.get(cfg, 1024)


def default_sub(cfg, args, batch):
    if args.sub > 0 and cfg == args.config:
        return args.sub
    return CONFIG_SUB.get(cfg, -(-batch // max(1, args.streams)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(args):
    """--gpus N without torch.distributed.run: one rank process per GPU, started
    before this process touches the GPU; rank 0 prints the line.  Returns the
    exit code (the first failing rank's, after stopping the others)."""
    n = args.gpus
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, MSGPU_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    code = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0 and code == 0:
                code = rc
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    return code


def line_stream():
    """The bench line's own stream: fd 1 as it was, while fd 1 itself is pointed
    at stderr for everything else in this process (gloo prints its "[Gloo] Rank
    r is connected to ..." lines to fd 1 from C++), so stdout carries the one
    JSON line and nothing else."""
    sys.stdout.flush()
    out = os.fdopen(os.dup(1), "w", buffering=1)
    os.dup2(2, 1)
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and args.gpus > 1:
        sys.exit(launch(args))
    out = line_stream()
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    cpus = pin_rank_cpus(local, local_world)
    cfg = args.config
    batch = default_batch(cfg, args)
    seeds = rank_seeds(rank, batch)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and not args.dry_run:
        cpu = cpu_baseline(cfg, args.cpu_budget)
    comm = Comm(rank, world)
    try:
        if args.dry_run:
            return dry_main(args, comm, cfg, seeds, local, cpus, out)
        irs = load_irs()
        with open(os.path.join(REPO, "tests", "golden", "golden_info.json")) as f:
            golden = json.load(f)["summaries"]
        with open(os.path.join(REPO, "tests", "golden", "golden_extra.json")) as f:
            golden.update(json.load(f)["summaries"])          # H48_1000..1003 (tools/gen_golden_r3.py)
        gate = None if args.gate in ("", "none") else tuple(int(v) for v in args.gate.split(","))
        head_gate = None if (cfg in GATE_OFF and args.gate == DEFAULT_GATE) else gate
        device = 0 if args.rehearse_one_gpu else local
        runner = GpuRunner(device, max(1, args.streams), head_gate, threaded=args.enqueue == "threads")
        head = measure(runner, cfg, seeds, default_sub(cfg, args, batch), args.steps, args.warmup, comm, irs,
                       golden, iso_steps=args.iso_steps, from_dicts_steps=args.from_dicts_steps)
        points = {}
        for pc in [c for c in args.points.split(",") if c and c != cfg]:
            pb = default_batch(pc, args)
            # C5's 8 sub-batches of 128 ran 3 % slower gated (135.2 vs 139.5 ms per step)
            runner.set_gate(None if pc in GATE_OFF else gate)
            psteps = max(args.point_steps, POINT_STEPS_MIN.get(pc, 0))
            points[pc] = measure(runner, pc, rank_seeds(rank, pb), default_sub(pc, args, pb), psteps, 3, comm,
                                 irs, golden, iso_steps=args.iso_steps,
                                 from_dicts_steps=psteps if (pc == "H48" and args.from_dicts_steps) else 0)
            if points[pc] is not None:
                points[pc]["stream_gate"] = "none" if (pc in GATE_OFF or gate is None) else ",".join(map(str, gate))
        for M in [int(t) for t in args.fir_points.split(",") if t]:
            points[f"FIR{M // 1024}K"] = measure_fir(runner, M, max(args.point_steps, 20), comm, rank,
                                                     cpu=(rank == 0 and not args.no_cpu))
        lat = dropin_latency(cpu) if (rank == 0 and world == 1 and not args.no_cpu) else None
        ranks = comm.gather({"rank": rank, "pid": os.getpid(), "device": device,
                             "cpus": [cpus[0], cpus[-1], len(cpus)], "host_threads": host_threads(),
                             "seeds": [seeds[0], seeds[-1]], "elapsed_s": round(head["_rank_s"], 6),
                             "frames": head["frames_per_gpu_step"] * args.steps})
        if rank == 0:
            for r in [head, *points.values()]:
                r.pop("_rank_s", None)
            line = {
                "metric": "Msamples/sec rendered (microsound full pipe, 384 kHz->48 kHz) at 1/2/4/8 GPUs",
                "value": head["value"], "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
                "data": "synthetic presets (reference param dicts, seeds per rank), IRs from irs/",
                "config": {"workload": head["workload"], "presets_per_gpu": batch,
                           "frames_per_gpu_step": head["frames_per_gpu_step"],
                           "events_per_gpu_step": head["events_per_gpu_step"],
                           "design_samples_per_gpu_step": head["design_samples_per_gpu_step"],
                           "sub_batches_per_gpu": head["sub_batches"],
                           "parallelism": f"preset-sharded x{world}" + (
                               " (rehearsal: every rank on device 0)" if args.rehearse_one_gpu else ""),
                           "streams_per_gpu": len(runner.engs),
                           "stream_gate": ",".join(map(str, head_gate)) if head_gate else "none", "enqueue": args.enqueue},
                "roofline": head["roofline"], "roofline_isolated": head.get("roofline_isolated"),
                "stage_ms": head["stage_ms"], "stage_algorithmic_GBs": head["stage_algorithmic_GBs"],
                "design_msamples_per_s": head["design_msamples_per_s"],
                "stage_sampling": f"stage events on batches 0, {PROFILE_EVERY}, {2 * PROFILE_EVERY}, ... of each context",
                "checked": head["check"],
                "from_dicts": head.get("from_dicts"),
                "cpu_baseline": cpu,
                "dropin_latency": lat,
                "points": points,
                "ranks": ranks,
            }
            if args.rehearse_one_gpu:
                line["rehearsal"] = "all ranks shared device 0: checks the multi-rank path, not a scaling point"
            # last, so that a reader keeping only the line's tail sees every point and its check
            line["points_summary"] = points_summary(head, points)
            print(json.dumps(line), file=out, flush=True)
    finally:
        comm.close()


def points_summary(head, points):
    """{config: [ms_per_step, value, check.all_ok, roofline frac]} for the headline
    and every point: the FIR + rFFT stage's isolated frac for render configs, the
    standalone FIR's frac for the FIR points."""
    def row(r):
        rf = r.get("roofline") or {}
        frac = ((rf.get("fir_rfft_stage") or {}).get("isolated") or {}).get("frac", rf.get("frac"))
        return [r.get("ms_per_step"), round(float(r.get("value", 0.0)), 1), bool((r.get("check") or {}).get("all_ok")),
                frac]
    out = {"fields": "ms_per_step, Msamples/s, check.all_ok, frac (FIR+rFFT isolated | FIR)", "head": row(head)}
    out.update({k: row(v) for k, v in points.items()})
    return out


def dry_main(args, comm, cfg, seeds, local, cpus, out):
    """The launcher path with the device work stubbed (CPU tests): same seeds,
    same timing protocol, per-rank record; prints a 'dry_run' line, no metric."""
    from msgpu.pack import PackedBatch
    import msgpu
    irs = load_irs()
    runner = DryRunner(comm.rank, args.dry_run)
    w = type("W", (), {})()
    frames = PackedBatch([msgpu.config_params(cfg, seed=s, irs=irs) for s in seeds]).total_frames
    mine, elapsed = timed(runner, w, args.steps, args.warmup, comm)
    ranks = comm.gather({"rank": comm.rank, "pid": os.getpid(), "device": local, "seeds": seeds,
                         "cpus": sorted(os.sched_getaffinity(0)), "host_threads": host_threads(),
                         "elapsed_s": mine, "frames": frames * args.steps})
    if comm.rank == 0:
        total = sum(r["frames"] for r in ranks)
        print(json.dumps({"dry_run": True, "n_gpus": comm.world, "elapsed_max_s": elapsed,
                          "value": total / elapsed / 1e6, "ranks": ranks}), file=out, flush=True)


if __name__ == "__main__":
    main()
