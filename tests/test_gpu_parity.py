"""GPU parity: libmsgpu on an MI355X vs the reference's golden outputs and the oracle.

Tolerance (north star): RMS of (gpu - reference) <= 1e-5 over the whole
(out_n, 2) buffer, float32 compute.  Everything goes through the C ABI via the
drop-in ``msgpu.render`` / ``render_batch``.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5
FIR_TOL = 5e-6   # long / ER + IR space filters: half the budget (kernels_fir64.h)


def rms(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.fixture(scope="module")
def msgpu():
    import msgpu as m
    from msgpu import _lib
    import ctypes
    lib = _lib.lib()
    m.render(m.merged(out_dur_s=0.05, er_cloud_on=False))   # initialise the engine
    # the product path must have loaded the in-tree HIP library
    maps = open("/proc/self/maps").read()
    assert "libmsgpu" in maps          # the HIP library (or a tuning build of it, MSGPU_LIB)
    assert isinstance(lib, ctypes.CDLL)
    return m


CASES = [
    ("C1", "C1", {}), ("C2", "C2", {}), ("C3", "C3", {}),
    ("C2odd", "C2", dict(seed=1002, out_dur_s=0.5 + 1 / 192000)),   # odd out_n: full-length rotation
    ("C3s1001", "C3", dict(seed=1001, out_dur_s=0.25)),
    ("C4s1000short", "C4", dict(out_dur_s=0.25)),
]


@pytest.mark.parametrize("name,cfg,kw", CASES)
def test_config_renders_match_golden(msgpu, full_renders, irs, name, cfg, kw):
    kw = dict(kw)
    seed = kw.pop("seed", 1000)
    p = msgpu.config_params(cfg, seed=seed, irs=irs, **kw)
    audio, meta = msgpu.render(p)
    ref = full_renders[f"{name}_audio"]
    assert audio.dtype == np.float32 and audio.flags["C_CONTIGUOUS"]
    err = rms(audio, ref)
    print(f"{name}: rms err {err:.3e}  max {np.max(np.abs(audio - ref)):.3e}")
    assert err <= RMS_TOL
    assert meta["out_sr"] == p["base_sr"]
    assert meta["design_sr_base"] == int(full_renders[f"{name}_design_sr"])
    for k in ("micro_last", "grain_last"):
        rk = f"{name}_{k}"
        if rk in full_renders.files:
            r = full_renders[rk]
            assert meta[k].shape == r.shape
            assert rms(meta[k], r) <= 1e-5 * max(1.0, float(np.sqrt(np.mean(r ** 2))))


def test_defaults_gaussian_click(msgpu, full_renders):
    p = msgpu.merged(out_dur_s=0.5)
    audio, _ = msgpu.render(p)
    assert rms(audio, full_renders["defaults_short_audio"]) <= RMS_TOL


def test_all_shipped_presets(msgpu, full_renders, irs, golden_info):
    """All 27 shipped presets (0.5 s, tiny-room IR, the golden image) against the
    reference's renders — every generator, spectral stage, physics model,
    multi-band unfold and feedback/imprint chain on the device path."""
    import json
    import os
    spread = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "render_spread.json")))["spread"]
    errs, lims = {}, {}
    for name in golden_info["presets"]:
        p = msgpu.merged(golden_info["preset_params"][name])
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        p["_img_gray"] = full_renders["image_gray"]
        audio, _ = msgpu.render(p)
        errs[name] = rms(audio, full_renders[f"preset_{name}_audio"])
        # ill-conditioned presets (cepstral warp, imprint under a cutoff lane): the
        # reference's own output moves by `spread` under
        # float64 rounding changes (AVX2 vs AVX-512 NumPy, FFT rounding); hold the
        # device to that band (tools/gen_spread.py)
        lims[name] = max(RMS_TOL, 1.5 * spread[name]) if name in spread else RMS_TOL
        print(f"preset {name}: rms err {errs[name]:.3e} (limit {lims[name]:.3e})")
    assert len(errs) == 27
    bad = {k: v for k, v in errs.items() if not v <= lims[k]}
    assert not bad, bad


def test_all_presets_one_batch(msgpu, full_renders, irs, golden_info):
    """The 27 presets as one device batch give the single-render results."""
    params = []
    for name in golden_info["presets"]:
        p = msgpu.merged(golden_info["preset_params"][name])
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        p["_img_gray"] = full_renders["image_gray"]
        params.append(p)
    import json
    import os
    spread = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "render_spread.json")))["spread"]
    outs = msgpu.render_batch(params)
    for name, a in zip(golden_info["presets"], outs):
        lim = max(RMS_TOL, 1.5 * spread[name]) if name in spread else RMS_TOL
        assert rms(a, full_renders[f"preset_{name}_audio"]) <= lim, name


def test_batch_equals_single_and_oracle(msgpu, irs):
    from oracle import msound_oracle as O
    params = [msgpu.config_params("C3", seed=s, irs=irs) for s in (1000, 1001, 1002, 1003)]
    outs = msgpu.render_batch(params)
    for p, a in zip(params, outs):
        ref, _ = O.render(p)
        assert rms(a, ref) <= RMS_TOL
    single, _ = msgpu.render(params[2])
    assert np.array_equal(single, outs[2])      # batching does not change results


def test_mixed_batch(msgpu, irs):
    from oracle import msound_oracle as O
    params = [msgpu.config_params("C2", seed=7, irs=irs, out_dur_s=0.3),
              msgpu.merged(out_dur_s=0.2, gen_mode="Noise burst", event_process="Poisson", seed=3),
              msgpu.merged(out_dur_s=0.25, gen_mode="Skewed transient", event_process="Poisson",
                           er_cloud_on=False, stereo_on=False, seed=4),
              msgpu.config_params("C1", seed=11, irs=irs)]
    outs = msgpu.render_batch(params)
    for p, a in zip(params, outs):
        ref, _ = O.render(p)
        assert rms(a, ref) <= RMS_TOL


def test_error_behaviour(msgpu):
    with pytest.raises(ValueError):                 # attack longer than the buffer (MS:182)
        msgpu.render(msgpu.merged(out_dur_s=0.01, env_a=100.0))
    with pytest.raises(ValueError):                 # "a:b:c" breakpoint (MS:461)
        msgpu.render(msgpu.merged(out_dur_s=0.1, bp_density="1:2:3"))


def test_fir_transform_sizes(msgpu, irs):
    """Every compile-time FIR transform size (N = 2048 .. 32768, one and two
    partitions), odd and even block alignments, ER-only / IR-only / both."""
    from oracle import msound_oracle as O
    base = dict(base_sr=48000, out_dur_s=0.3, gen_mode="Resonant strike", event_process="Poisson",
                space_ir_on=True, seed=21)
    params = []
    for taps in (100, 300, 700, 1500, 8192):                  # N = 2048, 4096, 8192, 16384, 32768
        params.append(msgpu.merged(base, er_cloud_on=False, space_ir_max_samps=taps,
                                   _ir_audio=irs["tiny_room_ir"]))
    params.append(msgpu.merged(base, er_cloud_on=True, space_ir_max_samps=8192,
                               _ir_audio=irs["tiny_room_ir"]))          # ER + IR
    params.append(msgpu.merged(base, er_cloud_on=True, space_ir_on=False, seed=5))   # ER only
    params.append(msgpu.merged(base, base_sr=192000, out_dur_s=0.21, er_cloud_on=True,
                               space_ir_max_samps=8192, _ir_audio=irs["tiny_room_ir"]))   # Q = 2
    outs = msgpu.render_batch(params)
    errs = []
    for i, (p, a) in enumerate(zip(params, outs)):
        ref, _ = O.render(p)
        errs.append(rms(a, ref))
        print(f"fir case {i}: rms err {errs[-1]:.3e}")
    # ER + IR filters (cases 5 and 7) saturate the clip; the float64 FIR keeps them
    # at half the budget (<= 5e-6), the others at the tolerance
    assert all(e <= (FIR_TOL if i in (5, 7) else RMS_TOL) for i, e in enumerate(errs)), errs


def test_fir_16384_kernels_agree(msgpu, irs, monkeypatch):
    """Blocks with M = 16384 (N = 32768, the 192 kHz two-partition case and C3)
    run on k_fir4 (four passes, 1024 threads) by default and on k_fir2 (three
    passes, 512 threads) with MSGPU_FIR4=0: both match the oracle, and each
    other to float32 rounding."""
    import torch
    from oracle import msound_oracle as O
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    base = dict(base_sr=48000, out_dur_s=0.3, gen_mode="Resonant strike", event_process="Poisson",
                space_ir_on=True, seed=21, _ir_audio=irs["tiny_room_ir"])
    params = [msgpu.merged(base, er_cloud_on=False, space_ir_max_samps=8192),       # IR only, one partition
              msgpu.merged(base, er_cloud_on=True, space_ir_max_samps=8192),        # ER + IR
              msgpu.merged(base, base_sr=192000, out_dur_s=0.21, er_cloud_on=True,
                           space_ir_max_samps=8192)]                                  # Q = 2
    packed = PackedBatch(params)
    outs = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("MSGPU_FIR4", flag)
        eng = Engine(0)
        outs[flag] = eng.render_packed(packed)
        torch.cuda.synchronize(0)
        outs[flag] = outs[flag].cpu().numpy()
    errs = []
    for i, p in enumerate(params):
        ref, _ = O.render(p)
        off, n = int(packed.offsets[i]), int(packed.out_n[i])
        assert ref.shape[0] == n
        d = np.abs(outs["0"][off:off + n] - outs["1"][off:off + n])
        print(f"case {i}: k_fir2 vs k_fir4 max {float(d.max()):.3e} at frame {int(d.max(axis=1).argmax())}")
        for flag in ("0", "1"):
            errs.append(rms(outs[flag][off:off + n], ref))
            print(f"case {i} MSGPU_FIR4={flag}: rms err {errs[-1]:.3e}")
    assert all(e <= RMS_TOL for e in errs), errs
    # two float32 transforms of different radix orders: their rounding noise
    # differs pointwise (up to ~7e-5 at a peak frame), not in rms
    assert rms(outs["0"], outs["1"]) <= RMS_TOL


def test_fir_streaming_kernel(msgpu, irs, full_renders, monkeypatch):
    """Two-partition presets at N = 32768 (C3's ER + IR filter) run on the
    streaming k_fir4s (opt-in, MSGPU_FIR4S=1) when the batch gives >= 2 blocks
    per workgroup: B = P =
    16384, the pending X_{b-1} . H_1 kept in registers across a workgroup's
    blocks.  MSGPU_FIR4S_WGS=1 puts whole presets (6, 12 and 8 blocks) on one
    workgroup, =8 cuts them into runs of 3 blocks (workgroup boundaries inside
    every preset);
    both match the reference renders, the oracle and the recomputing kernel
    (MSGPU_FIR4S=0) to float32 rounding."""
    import torch
    from oracle import msound_oracle as O
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    params = [msgpu.config_params("C3", seed=1001, irs=irs, out_dur_s=0.25),
              msgpu.config_params("C3", seed=1002, irs=irs, out_dur_s=0.5),
              msgpu.merged(base_sr=192000, out_dur_s=0.6826, gen_mode="Resonant strike", event_process="Poisson",
                           space_ir_on=True, seed=21, er_cloud_on=True, space_ir_max_samps=8192,
                           _ir_audio=irs["tiny_room_ir"])]
    packed = PackedBatch(params)
    outs = {}
    for key, env in (("off", {"MSGPU_FIR4S": "0"}), ("w1", {"MSGPU_FIR4S": "1", "MSGPU_FIR4S_WGS": "1"}),
                     ("w8", {"MSGPU_FIR4S": "1", "MSGPU_FIR4S_WGS": "8"})):
        monkeypatch.delenv("MSGPU_FIR4S", raising=False)
        monkeypatch.delenv("MSGPU_FIR4S_WGS", raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        eng = Engine(0)
        outs[key] = eng.render_packed(packed)
        torch.cuda.synchronize(0)
        outs[key] = outs[key].cpu().numpy()
    off0, n0 = int(packed.offsets[0]), int(packed.out_n[0])
    for key in outs:
        e = rms(outs[key][off0:off0 + n0], full_renders["C3s1001_audio"])
        print(f"C3 seed 1001 0.25 s [{key}]: rms err vs reference {e:.3e}")
        assert e <= RMS_TOL, key
    for i, p in enumerate(params):
        ref, _ = O.render(p)
        off, n = int(packed.offsets[i]), int(packed.out_n[i])
        for key in outs:
            e = rms(outs[key][off:off + n], ref)
            print(f"case {i} [{key}]: rms err vs oracle {e:.3e}")
            assert e <= RMS_TOL, (i, key)
    # the streaming runs agree with each other exactly (same transforms, same
    # order of the two partition products), and with the recomputing kernel at
    # float32 rounding (different block length B)
    assert np.array_equal(outs["w1"], outs["w8"])
    assert rms(outs["off"], outs["w1"]) <= RMS_TOL


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_full_size_configs(msgpu, irs, large_renders, golden_info, name):
    """C4 (384 kHz, 30 MHz design rate) and C5 (8.4 M frames, 4000 events) at full
    size: every step-th frame, the first/last 8192 frames and the whole-buffer
    rms / channel sums against the reference's render (seed 1000)."""
    p = msgpu.config_params(name, seed=1000, irs=irs)
    audio, _ = msgpu.render(p)
    info = golden_info["summaries"][f"{name}_1000"]
    assert list(audio.shape) == info["shape"]
    step = int(large_renders[f"{name}_step"])
    for part, ref in ((audio[::step], large_renders[f"{name}_dec"]),
                      (audio[:8192], large_renders[f"{name}_head"]),
                      (audio[-8192:], large_renders[f"{name}_tail"])):
        assert rms(part, ref) <= RMS_TOL
    a64 = audio.astype(np.float64)
    assert abs(float(np.sqrt(np.mean(a64 ** 2))) - info["rms"]) <= RMS_TOL
    n = audio.shape[0]
    assert abs(float(a64[:, 0].sum()) - info["sum_l"]) <= RMS_TOL * n
    assert abs(float(a64[:, 1].sum()) - info["sum_r"]) <= RMS_TOL * n


@pytest.mark.parametrize("ct", ["0", "1"])
def test_spectral_runtime_and_compile_time_plans(msgpu, irs, full_renders, monkeypatch, ct):
    """Hot grain lengths run compile-time plans (spec_ct.h); MSGPU_SPEC_CT=0 forces
    the runtime-plan engine.  Both must match the reference."""
    monkeypatch.setenv("MSGPU_SPEC_CT", ct)
    for name, cfg, kw in (("C2", "C2", {}), ("C3s1001", "C3", dict(seed=1001, out_dur_s=0.25))):
        kw = dict(kw)
        seed = kw.pop("seed", 1000)
        audio, _ = msgpu.render(msgpu.config_params(cfg, seed=seed, irs=irs, **kw))
        assert rms(audio, full_renders[f"{name}_audio"]) <= RMS_TOL, (name, ct)
    audio, _ = msgpu.render(msgpu.merged(out_dur_s=0.5))      # factory default: n = 1500
    assert rms(audio, full_renders["defaults_short_audio"]) <= RMS_TOL


@pytest.mark.parametrize("frames", [65, 127, 4097, 48001, 240001])
def test_odd_length_stereo(msgpu, irs, frames):
    """Odd out_n: the stereo rotation as a full-length transform (Bluestein,
    four-step M = 256 .. 2^20), against the oracle; mixed with an even preset
    in one batch."""
    from oracle import msound_oracle as O
    sr = 48000
    proc = "Single" if frames < 5000 else "Poisson"     # short outputs: one event at t = 0
    params = [msgpu.merged(base_sr=sr, out_dur_s=frames / sr, gen_mode="Resonant strike", event_process=proc,
                           grains_per_sec=30.0, env_a=0.0, env_r=1.0, seed=frames, stereo_width=w)
              for w in (0.65, 1.0)]
    params.append(msgpu.merged(base_sr=sr, out_dur_s=(frames + 1) / sr, env_a=0.0, env_r=1.0, seed=3))
    outs = msgpu.render_batch(params)
    for p, a in zip(params, outs):
        assert a.shape[0] % 2 == (1 if p is not params[-1] else 0)
        ref, _ = O.render(p)
        err = rms(a, ref)
        print(f"odd stereo n={a.shape[0]} w={p['stereo_width']}: rms {err:.3e}")
        assert err <= RMS_TOL
        assert np.max(np.abs(a)) > 0.5                 # a real signal, normalised to the peak


def test_gated_engines_equal_single(msgpu, irs):
    """msg_gate between the two contexts (bench.py --gate 2,6: a batch's
    generator waits for the other batch's stereo pass) reorders work only:
    three rounds of gated renders equal single-engine renders exactly, and
    clearing the gate restores ungated rendering."""
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    params = [msgpu.config_params("C2", seed=s, irs=irs) for s in range(2000, 2006)]
    halves = [PackedBatch(params[:3]), PackedBatch(params[3:])]
    engs = [Engine(0), Engine(0)]
    engs[0].gate(engs[1], 2, 6)
    engs[1].gate(engs[0], 2, 6)
    streams = [torch.cuda.Stream(device=0) for _ in range(2)]
    outs = [e.alloc_output(p) for e, p in zip(engs, halves)]
    for _ in range(3):
        for e, p, o, st in zip(engs, halves, outs, streams):
            e.render_packed(p, o, st)
    torch.cuda.synchronize(0)
    gated = [o.cpu().numpy() for o in outs]
    single = Engine(0)
    for h, p in enumerate(halves):
        ref = single.render_packed(p)
        torch.cuda.synchronize(0)
        assert np.array_equal(gated[h], ref.cpu().numpy()), h
    for e in engs:
        e.gate(None)
    engs[0].render_packed(halves[0], outs[0], streams[0])
    torch.cuda.synchronize(0)
    assert np.array_equal(outs[0].cpu().numpy(), gated[0])


def test_two_engines_two_streams_concurrent(msgpu, irs, golden_info):
    """The bench's in-flight mode: two contexts rendering on two HIP streams at
    once (sub-batches enqueued back to back, one sync at the end) give exactly
    the single-engine renders; the C3 seeds 1000-1003 also match the reference
    summaries."""
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    seeds = list(range(1000, 1008))
    params = [msgpu.config_params("C3", seed=s, irs=irs) for s in seeds]
    halves = [PackedBatch(params[:4]), PackedBatch(params[4:])]
    engs = [Engine(0), Engine(0)]
    streams = [torch.cuda.Stream(device=0) for _ in range(2)]
    outs = [e.alloc_output(p) for e, p in zip(engs, halves)]
    for _ in range(2):                      # twice: the second pass reuses every buffer
        for e, p, o, st in zip(engs, halves, outs, streams):
            e.render_packed(p, o, st)
    torch.cuda.synchronize(0)
    conc = [o.cpu().numpy() for o in outs]
    single = Engine(0)
    for h, p in enumerate(halves):
        ref = single.render_packed(p)
        torch.cuda.synchronize(0)
        assert np.array_equal(conc[h], ref.cpu().numpy()), h
    for j, s in enumerate(seeds[:4]):
        g = golden_info["summaries"][f"C3_{s}"]
        o, n = int(halves[0].offsets[j]), int(halves[0].out_n[j])
        a = conc[0][o:o + n].astype(np.float64)
        assert abs(float(np.sqrt(np.mean(a ** 2))) - g["rms"]) <= RMS_TOL
        assert abs(float(a[:, 0].sum()) - g["sum_l"]) <= RMS_TOL * n
        assert abs(float(a[:, 1].sum()) - g["sum_r"]) <= RMS_TOL * n


def test_host_plan_equals_device_plan(msgpu, irs, golden_info, monkeypatch):
    """msg_render_batch plans on the host pool (no device round trip); the device
    planner (k_plan_sizes / k_plan_events, MSGPU_DEVICE_PLAN=1) runs the same
    plan.h code.  Both give the same events and the same audio, on a batch that
    mixes every event process and several generators."""
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    params = [msgpu.config_params("C3", seed=1000, irs=irs, out_dur_s=0.3),
              msgpu.config_params("C2", seed=1001, irs=irs)]
    for name in ("wavelet_mist", "02_friction_lattice", "chaotic_dustfield", "micro_carillon"):
        p = msgpu.merged(golden_info["preset_params"][name])
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        params.append(p)
    for proc in ("Clustered", "Hawkes", "Single"):
        params.append(msgpu.config_params("C2", seed=1002, irs=irs, event_process=proc, out_dur_s=0.5))
    packed = PackedBatch(params)
    host_eng = Engine(0)
    monkeypatch.setenv("MSGPU_DEVICE_PLAN", "1")
    dev_eng = Engine(0)
    a = host_eng.render_packed(packed)
    b = dev_eng.render_packed(packed)
    torch.cuda.synchronize(0)
    for i in range(packed.n):
        eh, ed = host_eng.last_events(i), dev_eng.last_events(i)
        assert len(eh) == len(ed) > 0
        for x, y in zip(eh, ed):
            assert (x.n, x.start, x.offset, x.len, x.gen_sr) == (y.n, y.start, y.offset, y.len, y.gen_sr), i
            # float64 event times / amplitudes: the host's libm and the device's
            # log1p/exp (ziggurat slow paths) may differ in the last ulp
            assert abs(x.t0 - y.t0) <= 4e-16 * max(1.0, abs(y.t0)), (i, x.t0, y.t0)
            assert abs(x.amp - y.amp) <= 4e-16 * abs(y.amp), (i, x.amp, y.amp)
    assert float(np.max(np.abs(a.cpu().numpy() - b.cpu().numpy()))) <= 1e-6


def test_progress_messages_match_reference(msgpu, irs, full_renders):
    """msgpu.render's progress callback gets the reference's messages, per-event
    generator notes included (Image line y=<row> of event i, MS:362, 758)."""
    import json
    import os
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "progress.json")))
    for name, case in cases.items():
        p = msgpu.merged(case["params"])
        p["_img_gray"] = full_renders["image_gray"] if case["image"] else None
        p["_ir_audio"] = irs["tiny_room_ir"] if case["ir"] else None
        msgs = []
        msgpu.render(p, progress=lambda v, m: msgs.append([int(v), str(m)]))
        assert msgs == case["messages"], (name, msgs[:4], case["messages"][:4])


@pytest.mark.parametrize("cfg,stretch,roll,cut", [("C3", 0.5, None, None), ("C3", 2.0, 0.0, None),
                                                  ("C3", 4.0, None, 36000.0), ("C3", 4.0, 0.0, 37400.0),
                                                  ("C3", 1.0, None, None), ("C3", 4.0, None, None),
                                                  ("C4", 4.0, None, None), ("C4", 4.0, 0.0, None),
                                                  ("C4", 3.3, None, 14000.0), ("C4", 2.6, 4000.0, 23000.0),
                                                  ("C5", 4.0, None, None), ("C5", 2.0, None, 600.0),
                                                  ("C5", 0.5, None, None), ("C5", 1.0, 0.0, 300.0)])
def test_spec3_band_pruned_vs_general(msgpu, irs, monkeypatch, cfg, stretch, roll, cut):
    """The band-pruned 37 500-sample spectral kernel (k_spec3, default) against
    the general compile-time-plan kernel (MSGPU_SPEC3=0): stretch below 1, at 1
    and above, no roll-off, stretched bands whose top bin ky stays below M/2
    (C3 x4 at 18 kHz) and wide ones past it (C4's x4 stretch at x200 unfold:
    ky ~ 0.96 M, and a 36 kHz or 37.4 kHz cutoff at x100), which build each
    inverse input from Y[i] and Y[M - i].  Both match the oracle at 1e-5 RMS and
    each other, audio and meta grain_last.  C5's 1920-sample grains (a band limit
    above the design Nyquist, stretches 4, 2, 0.5, 1) run k_spectral_ct either
    way: a 960-point k_spec3 plan matched them (1.1e-6 RMS) but was no faster
    (C5 spectral 4.12 vs 4.09 ms isolated, profiles/r04v_c5_spec3.json)."""
    from oracle import msound_oracle as O
    kw = dict(seed=31, out_dur_s=2.0 if cfg == "C5" else 0.1, partial_stretch=stretch)
    if roll is not None:
        kw["bandlimit_roll_hz"] = roll
    if cut is not None:
        kw["bandlimit_out_hz"] = cut
    p = msgpu.config_params(cfg, irs=irs, **kw)
    got = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("MSGPU_SPEC3", flag)
        got[flag] = msgpu.render(p)
    ref, ref_meta = O.render(p)
    for flag, (audio, meta) in got.items():
        err = rms(audio, ref)
        g = np.asarray(meta["grain_last"], np.float64)
        gref = np.asarray(ref_meta["grain_last"], np.float64)
        gerr = float(np.sqrt(np.mean((g - gref) ** 2)) / max(1e-30, np.sqrt(np.mean(gref ** 2))))
        print(f"stretch {stretch} roll {roll} cut {cut} MSGPU_SPEC3={flag}: audio rms {err:.3e}, grain rel {gerr:.3e}")
        assert err <= RMS_TOL and gerr <= 1e-5
    assert rms(got["0"][0], got["1"][0]) <= RMS_TOL


@pytest.mark.parametrize("sr,unfold", [(48000, 25.0), (192000, 25.0), (384000, 100.0), (44100, 7.3)])
def test_resonant_generator_accuracy(msgpu, sr, unfold):
    """The resonant strike's float32 samples (meta micro_last, MS:253-258)
    against the oracle: float32 rounding only (the chunk bases and rotation
    table from an exact-wrap phase pair and sinpi / cospi, FP contraction off
    in the phase split: contracted, j fa's rounding entered the phase twice,
    5e-7 relative and growing with j, 7e-8 without; profiles/r04k_gpu_tests.txt)."""
    from oracle import msound_oracle as O
    p = msgpu.merged(gen_mode="Resonant strike", event_process="Single", base_sr=sr, time_unfold=unfold,
                     out_dur_s=0.05, seed=7, er_cloud_on=False, space_ir_on=False, ring_hz=5300.0)
    _, m = msgpu.render(p)
    _, rm = O.render(p)
    g, r = np.asarray(m["micro_last"], np.float64), rm["micro_last"]
    rel = float(np.sqrt(np.mean((g - r) ** 2) / np.mean(r ** 2)))
    print(f"{sr} Hz x{unfold}: micro rel err {rel:.2e}")
    assert rel <= 1.5e-7
