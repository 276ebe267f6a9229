"""Inputs the UI reaches beyond one transform (round 3), against the reference.

* Space filters longer than one 32 768-point transform: early reflections up to
  er_max_ms = 150 (MS:1118) at 176.4 / 192 kHz followed by an 8192-tap IR
  (MS:409-421, MS:438-445), and early reflections alone at a preset-JSON rate of
  384 kHz (57 601-sample span).  h = (delta + ER) * IR is built in the time
  domain (k_h_build) and partitioned like any other filter.
* Odd-length stereo rotations above 2^22 frames (MS:423-436): 95.25 s at
  44.1 kHz (4 200 525 frames, M = 2^24) and 60 s + 1 frame at 192 kHz
  (11 520 001 frames, M = 2^25) run the three-level Bluestein transform.
* The metric label's 384 kHz -> 48 kHz point (config H48), seeds 1000..1003.

Goldens: tests/golden/render_extra.npz + golden_extra.json (tools/gen_golden_r3.py,
rendered by the reference itself).  Tolerance: 1e-5 RMS (north star).
"""
import numpy as np
import pytest

from conftest import extra_params

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5
FIR_TOL = 5e-6    # long and ER + IR space filters: half the budget (kernels_fir64.h)


def rms(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.fixture(scope="module")
def msgpu():
    import msgpu as m
    m.render(m.merged(out_dur_s=0.05, er_cloud_on=False))
    assert "libmsgpu" in open("/proc/self/maps").read()   # the HIP library (or a tuning build of it)
    return m


LONG = ["ERIR192", "ERIR192t2000", "ERIR176", "ER384"]


def test_long_space_filters(msgpu, irs, extra_renders, golden_extra):
    params = [extra_params(golden_extra, irs, n) for n in LONG]
    outs = msgpu.render_batch(params)
    for name, p, a in zip(LONG, params, outs):
        err = rms(a, extra_renders[f"{name}_audio"])
        print(f"{name}: rms err {err:.3e}")
        assert err <= FIR_TOL, name
    single, _ = msgpu.render(params[0])
    assert np.array_equal(single, outs[0])          # batching does not change results


def test_long_space_filter_partitions(msgpu, irs):
    """The 36 992-tap filter of ERIR192 against the oracle over a longer output
    (several output blocks of each partition) and on the runtime-plan FIR
    (MSGPU_FIR4=0 moves the N = 32 768 blocks to k_fir2 / k_fir_h)."""
    import torch
    from oracle import msound_oracle as O
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    p = msgpu.merged(base_sr=192000, out_dur_s=0.9, gen_mode="Resonant strike", event_process="Poisson", seed=77,
                     er_cloud_on=True, er_max_ms=150.0, er_taps=700, space_ir_on=True, space_ir_max_samps=8192,
                     _ir_audio=irs["tiny_room_ir"])
    ref, _ = O.render(p)
    packed = PackedBatch([p])
    outs = {}
    for flag in ("1", "0"):
        import os
        os.environ["MSGPU_FIR4"] = flag
        try:
            eng = Engine(0)
            outs[flag] = eng.render_packed(packed)
            torch.cuda.synchronize(0)
            outs[flag] = outs[flag].cpu().numpy()
        finally:
            os.environ.pop("MSGPU_FIR4", None)
        err = rms(outs[flag][: ref.shape[0]], ref)
        print(f"MSGPU_FIR4={flag}: rms err vs oracle {err:.3e}")
        assert err <= FIR_TOL


@pytest.mark.parametrize("name", ["ODD44", "ODD192L"])
def test_odd_stereo_beyond_2_22(msgpu, irs, extra_renders, golden_extra, name):
    p = extra_params(golden_extra, irs, name)
    audio, _ = msgpu.render(p)
    info = golden_extra["summaries"][name]
    assert list(audio.shape) == info["shape"] and audio.shape[0] % 2 == 1
    step = int(golden_extra["decimation"])
    errs = {}
    for part, key in ((audio[::step], "dec"), (audio[:8192], "head"), (audio[-8192:], "tail")):
        errs[key] = rms(part, extra_renders[f"{name}_{key}"])
    print(f"{name} n={audio.shape[0]}: " + ", ".join(f"{k} {v:.3e}" for k, v in errs.items()))
    assert all(v <= RMS_TOL for v in errs.values()), errs
    a64 = audio.astype(np.float64)
    n = audio.shape[0]
    assert abs(float(np.sqrt(np.mean(a64 ** 2))) - info["rms"]) <= RMS_TOL
    assert abs(float(a64[:, 0].sum()) - info["sum_l"]) <= RMS_TOL * n
    assert abs(float(a64[:, 1].sum()) - info["sum_r"]) <= RMS_TOL * n


@pytest.mark.parametrize("frames", [4097, 240001])
def test_odd_stereo_three_level_split(msgpu, frames):
    """The three-level split (top column level over chunks of M1 x M2) at small
    n: MSGPU_SO_ROW=64 / MSGPU_SO_COL=16 make every M > 1024 take it; the render
    matches the oracle and the default two-level split to float32 rounding."""
    import os
    import torch
    from oracle import msound_oracle as O
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    sr = 48000
    p = msgpu.merged(base_sr=sr, out_dur_s=frames / sr, gen_mode="Resonant strike", event_process="Poisson",
                     grains_per_sec=30.0, env_a=0.0, env_r=1.0, seed=frames + 5, stereo_width=0.9)
    packed = PackedBatch([p])
    ref, _ = O.render(p)
    outs = {}
    for key, env in (("split", {"MSGPU_SO_ROW": "64", "MSGPU_SO_COL": "16"}), ("default", {})):
        os.environ.update(env)
        try:
            eng = Engine(0)
        finally:
            for k in env:
                os.environ.pop(k, None)
        o = eng.render_packed(packed)
        torch.cuda.synchronize(0)
        outs[key] = o.cpu().numpy()[:frames]
        err = rms(outs[key], ref)
        print(f"odd stereo n={frames} [{key}]: rms err {err:.3e}")
        assert err <= RMS_TOL
    assert rms(outs["split"], outs["default"]) <= RMS_TOL


def test_h48_metric_point(msgpu, irs, extra_renders, golden_extra):
    """H48 (design 384 kHz, 48 kHz out: the metric label's point) seeds 1000..1003
    as one batch: seed 1000 whole-buffer, all four by summary."""
    names = [f"H48_{s}" for s in (1000, 1001, 1002, 1003)]
    outs = msgpu.render_batch([extra_params(golden_extra, irs, n) for n in names])
    assert rms(outs[0], extra_renders["H48_1000_audio"]) <= RMS_TOL
    for name, a in zip(names, outs):
        g = golden_extra["summaries"][name]
        a64 = a.astype(np.float64)
        n = a.shape[0]
        assert list(a.shape) == g["shape"]
        assert abs(float(np.sqrt(np.mean(a64 ** 2))) - g["rms"]) <= RMS_TOL, name
        assert abs(float(a64[:, 0].sum()) - g["sum_l"]) <= RMS_TOL * n, name
        assert abs(float(a64[:, 1].sum()) - g["sum_r"]) <= RMS_TOL * n, name


@pytest.mark.parametrize("ct", ["0", "1"])
def test_h48_grain_plans(msgpu, irs, extra_renders, golden_extra, monkeypatch, ct):
    """H48's 480-sample grains on the compile-time plan (SpecPlan<240>: radices
    5, 6, 8, one wave per grain) and on the runtime-plan kernel
    (MSGPU_SPEC_CT=0): both match the reference's seed-1000 buffer."""
    monkeypatch.setenv("MSGPU_SPEC_CT", ct)
    a, _ = msgpu.render(extra_params(golden_extra, irs, "H48_1000"))
    err = rms(a, extra_renders["H48_1000_audio"])
    print(f"H48 MSGPU_SPEC_CT={ct}: rms err {err:.3e}")
    assert err <= RMS_TOL


def test_fir8_kernel_agrees(msgpu, irs, full_renders):
    """One-partition filters of 12 k .. 45 k taps run on k_fir8 (N = 65 536, two
    half-size transforms on the k_fir4 engine); MSGPU_FIR8=0 puts them back on
    k_fir4 (N = 32 768, two partitions).  Both match the reference / oracle, and
    each other to float32 rounding: C3 (25 473 taps), the 192 kHz ER + IR case,
    an IR-only and an ER-only filter, and two ER + IR filters longer than the
    output (the block must fit the unclipped filter)."""
    import os
    import torch
    from oracle import msound_oracle as O
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    params = [msgpu.config_params("C3", seed=1001, irs=irs, out_dur_s=0.25),
              msgpu.merged(base, base_sr=192000, out_dur_s=0.6826, space_ir_on=True, seed=21, er_cloud_on=True,
                           space_ir_max_samps=8192),
              msgpu.merged(base, base_sr=384000, out_dur_s=0.2, space_ir_on=True, seed=5, er_cloud_on=True,
                           er_max_ms=90.0, space_ir_max_samps=8192),
              msgpu.merged(base, base_sr=384000, out_dur_s=0.3, space_ir_on=False, seed=6, er_cloud_on=True,
                           er_max_ms=60.0),
              # taps + IR longer than the output (28 800 + 8192 > 32 640 frames): k_fir8's
              # spectrum holds the whole filter, so its block must leave room for all of it
              msgpu.merged(base, base_sr=192000, out_dur_s=0.17, space_ir_on=True, seed=8, er_cloud_on=True,
                           er_max_ms=150.0, er_taps=600, space_ir_max_samps=8192),
              msgpu.merged(base, base_sr=176400, out_dur_s=0.19, space_ir_on=True, seed=9, er_cloud_on=True,
                           er_max_ms=140.0, space_ir_max_samps=8192)]
    packed = PackedBatch(params)
    outs = {}
    for flag in ("1", "0"):
        os.environ["MSGPU_FIR8"] = flag
        try:
            eng = Engine(0)
        finally:
            os.environ.pop("MSGPU_FIR8", None)
        o = eng.render_packed(packed)
        torch.cuda.synchronize(0)
        outs[flag] = o.cpu().numpy()
    off0, n0 = int(packed.offsets[0]), int(packed.out_n[0])
    for flag in outs:
        e = rms(outs[flag][off0:off0 + n0], full_renders["C3s1001_audio"])
        print(f"C3 seed 1001 [MSGPU_FIR8={flag}]: rms err vs reference {e:.3e}")
        assert e <= RMS_TOL
    for i, p in enumerate(params):
        ref, _ = O.render(p)
        off, n = int(packed.offsets[i]), int(packed.out_n[i])
        for flag in outs:
            e = rms(outs[flag][off:off + n], ref)
            print(f"case {i} [MSGPU_FIR8={flag}]: rms err vs oracle {e:.3e}")
            assert e <= (RMS_TOL if i in (0, 3) else FIR_TOL), (i, flag)
    assert rms(outs["0"], outs["1"]) <= RMS_TOL


def _render_env(params, env):
    import os
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    packed = PackedBatch(params)
    os.environ.update(env)
    try:
        eng = Engine(0)
    finally:
        for k in env:
            os.environ.pop(k, None)
    o = eng.render_packed(packed)
    torch.cuda.synchronize(0)
    return packed, o.cpu().numpy()


def test_fir64_route(msgpu, irs, extra_renders, golden_extra):
    """The float64 FIR (kernels_fir64.h): MSGPU_FIR64=2 puts every FIR preset on
    it, =0 none.  Forced, C3 and the saturated ER + IR filters all match the
    reference / oracle; the predictor (default) leaves C3 on the float32 kernels
    (bit-identical to MSGPU_FIR64=0) and moves the saturated ones (errors printed
    for all three routes)."""
    from oracle import msound_oracle as O
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    params = [msgpu.config_params("C3", seed=1001, irs=irs, out_dur_s=0.25),
              extra_params(golden_extra, irs, "ERIR192t2000"),
              msgpu.merged(base, base_sr=192000, out_dur_s=0.6826, space_ir_on=True, seed=21, er_cloud_on=True,
                           space_ir_max_samps=8192),
              msgpu.merged(base, base_sr=48000, out_dur_s=0.7, space_ir_on=True, seed=22, er_cloud_on=True,
                           space_ir_max_samps=8192, stereo_width=0.3)]
    refs = [None, extra_renders["ERIR192t2000_audio"], O.render(params[2])[0], O.render(params[3])[0]]
    outs = {m: _render_env(params, {"MSGPU_FIR64": m}) for m in ("0", "1", "2")}
    for i in range(len(params)):
        for m, (packed, o) in outs.items():
            off, n = int(packed.offsets[i]), int(packed.out_n[i])
            ref = refs[i] if refs[i] is not None else O.render(params[i])[0]
            e = rms(o[off:off + n], ref)
            print(f"case {i} [MSGPU_FIR64={m}]: rms err {e:.3e}")
            if m != "0":
                assert e <= FIR_TOL, (i, m)
    p0, o0 = outs["0"]
    p1, o1 = outs["1"]
    n0 = int(p0.out_n[0])
    assert np.array_equal(o0[:n0], o1[:n0])               # C3 stays on the float32 FIR



def test_fir8_persistent_bit_identical(msgpu, irs, full_renders):
    """k_fir8's persistent form (MSGPU_FIR8P=1, the default: one workgroup per
    CU taking blocks from per-XCD counters) computes every block with the same
    arithmetic as one workgroup per block (=0): the outputs are bit-identical,
    for a batch
    whose block count is not a multiple of the XCD count (edge blocks, short
    presets, a preset without a filter among them) and for C3."""
    params = [msgpu.config_params("C3", seed=1000 + s, irs=irs) for s in range(3)]
    params += [msgpu.config_params("C3", seed=2000, irs=irs, out_dur_s=0.06),
               msgpu.config_params("C3", seed=2001, irs=irs, out_dur_s=0.035),   # C3's attack: 7680 frames
               msgpu.merged(out_dur_s=0.2, seed=5)]
    outs = {m: _render_env(params, {"MSGPU_FIR8P": m})[1] for m in ("0", "1")}
    assert np.array_equal(outs["0"], outs["1"])
    packed, _ = _render_env(params[:1], {})
    assert rms(outs["1"][:int(packed.out_n[0])], full_renders["C3_audio"]) <= RMS_TOL


def test_spec3_persistent_bit_identical(msgpu, irs, full_renders):
    """k_spec3's persistent form (MSGPU_SPEC3P=1: one workgroup per CU taking
    events from per-XCD counters, each next grain loaded during the current
    event) runs every event with the two-event chain's arithmetic (=0): the
    outputs are bit-identical on C3 (narrow band), C4 (wide band), a batch of
    fewer events than CUs and one whose event count is not a multiple of the
    XCD count; C3 still matches the reference render."""
    params = [msgpu.config_params("C3", seed=1000 + s, irs=irs) for s in range(3)]
    params += [msgpu.config_params("C4", seed=1000, irs=irs), msgpu.merged(out_dur_s=0.2, seed=5)]
    outs = {m: _render_env(params, {"MSGPU_SPEC3P": m})[1] for m in ("0", "1")}
    assert np.array_equal(outs["0"], outs["1"])
    few = [msgpu.config_params("C3", seed=3000, irs=irs, out_dur_s=0.2)]      # a handful of events
    fo = {m: _render_env(few, {"MSGPU_SPEC3P": m})[1] for m in ("0", "1")}
    assert np.array_equal(fo["0"], fo["1"])
    packed, _ = _render_env(params[:1], {})
    assert rms(outs["1"][:int(packed.out_n[0])], full_renders["C3_audio"]) <= RMS_TOL


def test_fir64_serves_every_flagged_preset(msgpu, irs):
    """the float64 FIR had 128 slots per batch and left flagged
    presets beyond them on float32, so a preset's output depended on the batch
    it shared.  Every flagged preset is now served (in windows of slots): 140
    copies of one saturated ER + IR preset in one batch all match the preset
    rendered alone, bit for bit, and the oracle within FIR_TOL."""
    from oracle import msound_oracle as O
    p = msgpu.merged(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"],
                     base_sr=48000, out_dur_s=0.3, space_ir_on=True, seed=22, er_cloud_on=True,
                     space_ir_max_samps=8192, stereo_width=0.3)
    packed1, one = _render_env([p], {})
    packedN, many = _render_env([p] * 140, {})
    n = int(packed1.out_n[0])
    for i in (0, 127, 128, 139):
        off = int(packedN.offsets[i])
        assert np.array_equal(many[off:off + n], one[:n]), i
    e = rms(one[:n], O.render(p)[0])
    _, f32 = _render_env([p], {"MSGPU_FIR64": "0"})
    e32 = rms(f32[:n], O.render(p)[0])
    print(f"saturated preset: rms err {e:.3e} (float32 FIR alone: {e32:.3e})")
    assert e <= FIR_TOL and not np.array_equal(one[:n], f32[:n])   # the float64 route did run


def test_fir64_windows_bit_identical(msgpu, irs):
    """with the default cap (1024 slots, 1 GiB) the batch above fits
    one window, so the w0 > 0 path never ran.  MSGPU_FIR64_CAP=48 cuts 140
    flagged copies into three windows (48 + 48 + 44 slots: slot_preset[w0 + sl],
    h / H_q buffers reused between windows, fir64_window clamping the last one),
    and a mixed batch interleaves unflagged presets between the flagged ones;
    every copy matches the preset rendered alone, bit for bit."""
    p = msgpu.merged(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"],
                     base_sr=48000, out_dur_s=0.3, space_ir_on=True, seed=22, er_cloud_on=True,
                     space_ir_max_samps=8192, stereo_width=0.3)
    q = msgpu.config_params("C3", seed=1001, irs=irs, out_dur_s=0.05)      # float32 FIR, not flagged
    packed1, one = _render_env([p], {})
    packedq, oneq = _render_env([q], {})
    batch = [p] * 100 + [q, p, q] + [p] * 39
    packedN, many = _render_env(batch, {"MSGPU_FIR64_CAP": "48"})
    n, nq = int(packed1.out_n[0]), int(packedq.out_n[0])
    for i, pp in enumerate(batch):
        off = int(packedN.offsets[i])
        if pp is p:
            assert np.array_equal(many[off:off + n], one[:n]), i
        else:
            assert np.array_equal(many[off:off + nq], oneq[:nq]), i


def test_stereo_fused_matches_two_launches(msgpu, irs):
    """k_stereo_fused (MSGPU_STEREO_FUSED=1: max and output passes in one
    persistent launch, deferred float64-FIR and odd-length presets) writes the
    same bits as k_stereo_max + k_stereo_out, and the float64 FIR's per-preset
    sums are added in tile order, so two renders are identical."""
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    params = [msgpu.config_params("C3", seed=1000 + s, irs=irs, out_dur_s=0.3) for s in range(3)]
    params += [msgpu.merged(base, base_sr=48000, out_dur_s=0.3, space_ir_on=True, seed=22, er_cloud_on=True,
                            space_ir_max_samps=8192, stereo_width=0.3),          # float64 FIR (deferred)
               msgpu.merged(out_dur_s=0.2, seed=5),                             # no filter
               msgpu.merged(out_dur_s=0.2000208, seed=6, base_sr=48000),        # odd length (deferred)
               msgpu.config_params("C2", seed=1000, irs=irs, out_dur_s=0.25)]
    _, two = _render_env(params, {"MSGPU_STEREO_FUSED": "0"})
    _, two_again = _render_env(params, {"MSGPU_STEREO_FUSED": "0"})
    packed, fused = _render_env(params, {"MSGPU_STEREO_FUSED": "1"})
    assert int(packed.out_n[5]) % 2 == 1
    assert np.array_equal(two, two_again)
    assert np.array_equal(two, fused)


def test_fir4_spectra_from_taps(msgpu, irs):
    """One-partition filters at N = 32 768 (H48's 48 kHz ER + 4096-tap IR, an
    IR-only one, an ER-only one): the spectra straight from the taps
    (k_fir4_hconv / k_fir4_irspec, MSGPU_FIR4C=1, the default) against the
    time-domain float64 h cut into one partition (k_h_build + k_fir4_hpart,
    MSGPU_FIR4C=0): both match the oracle within the tolerance."""
    from oracle import msound_oracle as O
    params = [msgpu.config_params("H48", seed=1000 + s, irs=irs, out_dur_s=0.5) for s in range(2)]
    params += [msgpu.merged(msgpu.config_params("H48", seed=1010, irs=irs, out_dur_s=0.5), er_cloud_on=False),
               msgpu.merged(msgpu.config_params("H48", seed=1011, irs=irs, out_dur_s=0.5), space_ir_on=False)]
    outs = {m: _render_env(params, {"MSGPU_FIR4C": m}) for m in ("0", "1")}
    for i, p in enumerate(params):
        ref, _ = O.render(p)
        for m, (packed, o) in outs.items():
            off, n = int(packed.offsets[i]), int(packed.out_n[i])
            e = rms(o[off:off + n], ref)
            print(f"case {i} [MSGPU_FIR4C={m}]: rms err vs oracle {e:.3e}")
            assert e <= RMS_TOL, (i, m)


def test_ola_fused_matches_ola_kernel(msgpu, irs):
    """The overlap-add inside k_fir8p's segment loads (PresetRt::ola_fir) sums
    the same events in the same order as k_ola_env, so the renders are the same
    bits: C3 / C5 presets forced onto the fused path (MSGPU_OLA_FIR_DENSITY
    raised past their grain density), short outputs (one block, first and last
    blocks partial), and a float64-FIR preset whose mono a k_ola_slots writes."""
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    params = [msgpu.config_params("C3", seed=1200 + s, irs=irs, out_dur_s=d) for s, d in enumerate((1.3, 0.2))]
    params += [msgpu.config_params("C5", seed=1300 + s, irs=irs, out_dur_s=d) for s, d in enumerate((200.0, 9.0))]
    params += [msgpu.merged(base, base_sr=48000, out_dur_s=0.9, space_ir_on=True, seed=22, er_cloud_on=True,
                            space_ir_max_samps=8192, stereo_width=0.3, sat_drive=6.0)]
    fused_env = {"MSGPU_OLA_FIR": "1", "MSGPU_OLA_FIR_DENSITY": "1e9"}
    _, ref = _render_env(params, {"MSGPU_OLA_FIR": "0"})
    _, fused = _render_env(params, fused_env)
    _, default = _render_env(params, {})
    assert np.array_equal(ref, fused)
    assert np.array_equal(ref, default)
    # every FIR preset on the float64 FIR: k_ola_slots writes the fused presets' mono a
    _, ref64 = _render_env(params, {"MSGPU_OLA_FIR": "0", "MSGPU_FIR64": "2"})
    _, fused64 = _render_env(params, dict(fused_env, MSGPU_FIR64="2"))
    assert np.array_equal(ref64, fused64)


def test_filter_spectra_early_same_bits(msgpu, irs):
    """The filter spectra launched before the generator (MSGPU_H_EARLY=1; the
    default, 2, does so only for batches with an output of at least 2^22 frames)
    or at the FIR stage (=0): the same kernels on the same inputs, so the same
    bits, for the k_fir8 / k_fir4 one-partition and the partitioned paths."""
    params = [msgpu.config_params("C3", seed=1400, irs=irs, out_dur_s=0.4),
              msgpu.config_params("H48", seed=1401, irs=irs, out_dur_s=0.5),
              msgpu.config_params("C2", seed=1402, irs=irs, out_dur_s=0.25)]
    _, late = _render_env(params, {"MSGPU_H_EARLY": "0"})
    _, early = _render_env(params, {"MSGPU_H_EARLY": "1"})
    assert np.array_equal(late, early)


def test_er_gains_on_device(msgpu, irs):
    """The host batch path plans the ER offsets and k_er_gains draws the gains on
    the device (MSGPU_ER_DEV=1, the default) from the same stream positions,
    merged taps summed in tap order; against the host-drawn gains (=0) the
    renders agree to the last float64 ulp of exp: a preset with many merged
    offsets (2000 taps within 5 ms at 48 kHz), C3, H48 and a 192 kHz ER + IR."""
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    params = [msgpu.merged(base, base_sr=48000, out_dur_s=0.4, er_cloud_on=True, er_taps=2000, er_max_ms=5.0,
                           space_ir_on=False, seed=31),
              msgpu.config_params("C3", seed=1500, irs=irs, out_dur_s=0.3),
              msgpu.config_params("H48", seed=1501, irs=irs, out_dur_s=0.5),
              msgpu.merged(base, base_sr=192000, out_dur_s=0.3, er_cloud_on=True, er_taps=640, er_max_ms=120.0,
                           space_ir_on=True, space_ir_max_samps=8192, seed=32)]
    _, host = _render_env(params, {"MSGPU_ER_DEV": "0"})
    _, dev = _render_env(params, {"MSGPU_ER_DEV": "1"})
    d = float(np.max(np.abs(host - dev)))
    print(f"max |host-drawn - device-drawn| = {d:.3e}, identical samples {np.mean(host == dev):.4f}")
    assert d <= 1e-6
