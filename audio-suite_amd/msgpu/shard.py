"""Preset sharding across GPUs.

Presets are independent renders (MS:588-792 holds no state across calls), so a
batch shards by preset with no collective: contiguous ranges of equal predicted
cost, one range per GPU.  The cost of a preset comes from its host plan
(msg_plan_host, the same code the device planner runs): sum n log2 n over its
grains plus out_n (log2 L + taps / L) for the FIR and stereo passes.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

# host cores one GPU's worker uses at most (the GPU box's CPU share per GPU;
# nproc shows the whole machine)
CORES_PER_GPU = 16


def preset_cost(info, taps=8192):
    """Predicted device cost of one preset from its plan summary."""
    n_ev = max(int(info.n_events), 0)
    if n_ev == 0:
        grain = 0.0
    else:
        n = max(float(info.pool_len) / n_ev, 2.0)
        grain = float(info.pool_len) * np.log2(n)
    L = 16384.0
    return grain + float(info.out_n) * (np.log2(L) + taps / L)


def balance(costs, world):
    """Contiguous partition of presets into ``world`` chunks of near-equal total
    cost (greedy on the prefix sum: chunk r ends where the running cost crosses
    (r + 1) / world of the total).  Returns world + 1 cut indices."""
    c = np.asarray(costs, dtype=np.float64)
    n = c.size
    pref = np.concatenate([[0.0], np.cumsum(c)])
    total = pref[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        k = int(np.searchsorted(pref, target, side="left"))
        # pick the closer of the two prefix points around the target
        if k > 0 and abs(pref[k - 1] - target) <= abs(pref[min(k, n)] - target):
            k -= 1
        cuts.append(min(max(k, cuts[-1]), n))
    cuts.append(n)
    return cuts


def plan_costs(params_list):
    """Host plans (msg_plan_host) -> predicted costs, one per preset."""
    from . import _lib as L
    from .pack import Banks, fragment_source, pack_preset, space_ir_taps
    from .params import merged
    lib = L.lib()
    out = []
    for prm in params_list:
        p = merged(prm)
        banks = Banks()
        s = pack_preset(p, banks)
        info = L.MsgPlanInfo()
        frag = fragment_source(p) if p["gen_mode"] == "IR fragment" else None
        fp = frag.ctypes.data_as(C.POINTER(C.c_double)) if frag is not None else None
        L.check(lib.msg_plan_host(C.byref(s), banks.bp_array(), fp, 0 if frag is None else frag.size,
                                  C.byref(info), None, 0, None, None), None)
        ir = space_ir_taps(p)
        out.append(preset_cost(info, 0 if ir is None else ir.size))
    return out


def pin_worker_cpus(local, local_world):
    """Before the first GPU call of a per-GPU worker: pin it to its own contiguous
    slice of the process's CPU affinity (one host pool per GPU) and
    size the library's host pool to it (MSGPU_HOST_THREADS, at most
    CORES_PER_GPU).  Returns the slice."""
    cpus = sorted(os.sched_getaffinity(0))
    if local_world > 1 and len(cpus) >= local_world:
        per = len(cpus) // local_world
        cpus = cpus[local * per:(local + 1) * per]
        os.sched_setaffinity(0, cpus)
    cpus = cpus[:max(1, min(len(cpus), CORES_PER_GPU))] if local_world > 1 else cpus
    os.environ.setdefault("MSGPU_HOST_THREADS", str(max(1, min(len(cpus), CORES_PER_GPU))))
    return cpus
