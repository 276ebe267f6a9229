#!/usr/bin/env python3
"""Benchmark: Msamples/s rendered by the MI355X Microsound render path.

Workload (BASELINE.json configs[2], SURVEY.md section 8 "C3"): 384 kHz output,
unfold x100 (design SR clamps to 30 MHz), spectral stretch x2, resonant
transient, Poisson events, 16 k-tap IR request (8192-tap cap, MS:443),
early reflections, stereo diffusion — a batch of 1024 presets per GPU, seeds
1000 + rank*batch + b.  One step = one full render of the batch (device plan ->
generate -> spectral -> overlap-add -> FIR -> stereo/normalise) with inputs
(packed presets + IR) resident.  Weak scaling: every rank renders its own batch.

    python bench.py [--gpus N --steps K --warmup W --config C3 --batch 1024]

Multi-GPU: launched by torch.distributed.run, one process per GPU, no
data-path collective (presets are independent); barrier + max-over-ranks timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
# Per-launch HBM bytes of each kernel from rocprofv3 PMC passes (FETCH_SIZE x2
# per the gfx950 correction + WRITE_SIZE), written by tools/pmc_traffic.py.
TRAFFIC_JSON = os.path.join(REPO, "profiles", "traffic.json")
# bench stage -> the kernel it times (rocprofv3 kernel-name prefix)
STAGE_KERNEL = {"generate": "k_gen_normal", "spectral": "k_spectral", "overlap_add": "k_ola_env",
                "fir_kernel": "k_fir2<", "stereo": "k_stereo_out"}
# host cores of the GPU box available to one job (its CPU share; nproc shows the machine)
BOX_CORES = 16


def load_irs():
    z = np.load(os.path.join(REPO, "tests", "golden", "irs.npz"))
    return {k: z[k] for k in z.files}


def stage_bytes(infos, _packed, params):
    """Algorithmic (compulsory) HBM bytes per stage for one step."""
    sum_n = sum(int(i.pool_len) for i in infos)
    out_n = sum(int(i.out_n) for i in infos)
    return {
        "generate": 4 * sum_n,                 # grain samples written once
        "spectral": 8 * sum_n,                 # grain read + grain written (one LDS round trip)
        "overlap_add": 4 * sum_n + 4 * out_n,  # placed grains read + mono written (upper bound)
        "fir": 8 * out_n,                      # mono read + mono written
        "fir_kernel": 8 * out_n,               # k_fir alone: same compulsory bytes
        "stereo": 16 * out_n,                  # max pass reads y; output pass reads y, writes L/R
    }


def measured_traffic(kernel, cfg, batch):
    """HBM bytes per launch of `kernel` from the committed PMC summary, or None
    when no summary for this workload exists (bench cannot read PMC itself)."""
    try:
        with open(TRAFFIC_JSON) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("config") != cfg or int(t.get("batch", -1)) != batch:
        return None
    for name, rec in t.get("kernels", {}).items():
        if name.startswith(kernel):
            return rec.get("hbm_bytes_per_launch")
    return None


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
    procs = max(1, min(BOX_CORES, len(os.sched_getaffinity(0))))
    ctx = mp.get_context("fork")
    t0 = time.perf_counter()
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(cfg, 1000 + i, procs, budget_s) for i in range(procs)])
    wall = time.perf_counter() - t0
    pdone = sum(r[0] for r in res)
    pframes = sum(r[1] for r in res)
    return {"value": pframes / wall / 1e6, "unit": "Msamples/s", "cores": procs, "kind": "port",
            "single_core": round(single, 4),
            "sample": f"{cfg} presets rendered by oracle/msound_oracle.py (NumPy restatement of "
                      f"main_v2.render): {done} presets on 1 core in {dt:.1f} s "
                      f"({single:.3f} Msamples/s), then {pdone} presets on {procs} processes in "
                      f"{wall:.1f} s"}


def rank_seeds(rank, batch):
    """Preset seeds of one rank: contiguous, disjoint across ranks (weak scaling)."""
    return [1000 + rank * batch + b for b in range(batch)]


def max_over_ranks(elapsed, world, device):
    """The job's time is the slowest rank's (all-reduce MAX; no data-path collective)."""
    if world <= 1:
        return elapsed
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--cpu-budget", type=float, default=12.0, help="seconds of CPU-baseline work")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--streams", type=int, default=2, help="in-flight sub-batches (contexts/streams) per GPU")
    ap.add_argument("--iso-steps", type=int, default=3, help="single-stream renders for roofline_isolated")
    ap.add_argument("--h48-steps", type=int, default=5,
                    help="steps of the 384 kHz -> 48 kHz point (config H48, same batch), 0 = skip")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.config, args.cpu_budget)

    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = local if world > 1 else 0

    import msgpu
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch

    irs = load_irs()
    seeds = rank_seeds(rank, args.batch)
    params = [msgpu.config_params(args.config, seed=s, irs=irs) for s in seeds]
    S = max(1, min(args.streams, args.batch))
    # S in-flight renders per GPU, one context + one HIP stream each (SURVEY
    # section 8e: "one HIP stream per render"): the host plans one sub-batch
    # while the device runs the other, and their kernels share the CUs.
    cut = [len(params) * i // S for i in range(S + 1)]
    subs = [PackedBatch(params[cut[i]:cut[i + 1]]) for i in range(S)]
    engs = [Engine(dev) for _ in range(S)]
    outs = [e.alloc_output(p) for e, p in zip(engs, subs)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(S)]

    def barrier():
        if world > 1:
            dist.barrier()

    def step():
        for e, p, o, st in zip(engs, subs, outs, streams):
            e.render_packed(p, o, st)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    infos = [i for e in engs for i in e.last_plan()]

    for e in engs:
        e.set_profiling(True)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    for e in engs:
        e.set_profiling(False)
    elapsed = max_over_ranks(elapsed, world, f"cuda:{dev}")
    names = ["plan", "host_prep", "generate", "spectral", "overlap_add", "fir", "stereo", "total",
             "fir_kernel", "fir_h"]
    # per-launch stage times in the timed region (each sub-batch on its own stream)
    stage_ms = np.mean([np.array(e.stage_times()) for e in engs], axis=0)
    stages = {n: round(float(v), 4) for n, v in zip(names, stage_ms)}

    # isolated pass: the whole batch on one stream, kernels not sharing the GPU
    iso = {}
    if args.iso_steps > 0:
        packed = PackedBatch(params)
        e1 = engs[0]
        o1 = e1.alloc_output(packed)
        e1.render_packed(packed, o1, streams[0])
        torch.cuda.synchronize(dev)
        e1.set_profiling(True)
        for _ in range(args.iso_steps):
            e1.render_packed(packed, o1, streams[0])
        torch.cuda.synchronize(dev)
        e1.set_profiling(False)
        iso = {n: round(float(v), 4) for n, v in zip(names, e1.stage_times())}
        del o1

    frames_rank = sum(p.total_frames for p in subs)
    total_frames = frames_rank * world * args.steps
    value = total_frames / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3
    sb = stage_bytes(infos, None, params)
    sb_launch = {k: v / S for k, v in sb.items()}
    stage_gbs = {k: round(sb_launch[k] / (stages[k] * 1e-3) / 1e9, 1) for k in sb if stages.get(k, 0) > 0}
    # dominant single kernel (the FIR stage is timed without its h build)
    kernel_stages = ["generate", "spectral", "overlap_add", "fir_kernel", "stereo"]
    dom = max(kernel_stages, key=lambda k: stages[k])
    achieved = sb_launch[dom] / (stages[dom] * 1e-3) / 1e9
    traffic = measured_traffic(STAGE_KERNEL[dom], args.config, args.batch // S)
    sum_n = sum(int(i.pool_len) for i in infos)
    n_ev = sum(int(i.n_events) for i in infos)
    roof_iso = None
    if iso:
        dom_i = max(kernel_stages, key=lambda k: iso[k])
        ach_i = sb[dom_i] / (iso[dom_i] * 1e-3) / 1e9
        roof_iso = {"kernel": STAGE_KERNEL[dom_i].rstrip("<"), "achieved": round(ach_i, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach_i / HBM_PEAK_GBS, 4),
                    "algorithmic_bytes": sb[dom_i], "kernel_ms": iso[dom_i],
                    "traffic": measured_traffic(STAGE_KERNEL[dom_i], args.config, args.batch),
                    "stage_ms": iso, "note": f"whole batch on one stream, {args.iso_steps} renders after the "
                                             f"timed region"}

    # the metric label's "384 kHz -> 48 kHz" read literally: H48 presets, same batch
    h48 = None
    if args.h48_steps > 0 and args.config != "H48":
        hp = [msgpu.config_params("H48", seed=s, irs=irs) for s in seeds]
        hsubs = [PackedBatch(hp[cut[i]:cut[i + 1]]) for i in range(S)]
        houts = [e.alloc_output(p) for e, p in zip(engs, hsubs)]

        def hstep():
            for e, p, o, st in zip(engs, hsubs, houts, streams):
                e.render_packed(p, o, st)

        hstep()
        torch.cuda.synchronize(dev)
        barrier()
        t1 = time.perf_counter()
        for _ in range(args.h48_steps):
            hstep()
        torch.cuda.synchronize(dev)
        barrier()
        he = max_over_ranks(time.perf_counter() - t1, world, f"cuda:{dev}")
        hframes = sum(p.total_frames for p in hsubs)
        h48 = {"config": "H48: 48 kHz out, unfold x8 (384 kHz design SR), Poisson 18/s, 1 s, 4096-tap IR, "
                         "ER 320 taps, stereo",
               "value": round(hframes * world * args.h48_steps / he / 1e6, 3), "unit": "Msamples/s",
               "ms_per_step": round(he / args.h48_steps * 1e3, 3), "steps": args.h48_steps,
               "presets_per_gpu": args.batch, "streams_per_gpu": S}
        del houts

    if rank == 0:
        line = {
            "metric": "Msamples/sec rendered (microsound full pipe, 384 kHz->48 kHz) at 1/2/4/8 GPUs",
            "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic presets (reference param dicts, seeds per rank), IR ir_tiny_room_250ms",
            "config": {"workload": f"{args.config}: 384 kHz out, unfold x100 (30 MHz design SR), stretch x2, "
                                   f"Poisson 18/s, 1 s, 16k-tap IR request (8192 cap), ER 320 taps, stereo",
                       "presets_per_gpu": args.batch, "frames_per_gpu_step": frames_rank,
                       "events_per_gpu_step": n_ev, "design_samples_per_gpu_step": sum_n,
                       "parallelism": f"preset-sharded x{world}", "streams_per_gpu": S},
            "roofline": {"bound": "hbm", "kernel": STAGE_KERNEL[dom].rstrip("<"),
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "algorithmic_bytes": sb_launch[dom], "kernel_ms": stages[dom],
                         "note": f"per launch in the timed region ({S} sub-batches of {args.batch // S} presets "
                                 f"on {S} streams sharing the GPU)"},
            "roofline_isolated": roof_iso,
            "stage_ms": stages, "stage_algorithmic_GBs": stage_gbs,
            "design_msamples_per_s": round(sum_n * world * args.steps / elapsed / 1e6, 1),
            "cpu_baseline": cpu,
            "point_384k_to_48k": h48,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
