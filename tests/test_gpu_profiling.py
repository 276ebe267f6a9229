"""Stage profiling (msg_set_profiling / msg_stage_times, include/msgpu.h): every
batch, or every k-th batch of a context (bench.py samples every 4th inside its
timed region).  Profiling never changes a bit of the output."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def msgpu():
    import msgpu as m
    m.render(m.merged(out_dur_s=0.05, er_cloud_on=False))
    assert "libmsgpu" in open("/proc/self/maps").read()   # the HIP library
    return m


def _batch(msgpu, irs):
    return [msgpu.config_params("C3", seed=1000 + s, irs=irs, out_dur_s=0.2) for s in range(4)]


def test_sampled_profiling(msgpu, irs):
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    packed = PackedBatch(_batch(msgpu, irs))
    eng = Engine(0)
    out = eng.alloc_output(packed)
    eng.render_packed(packed, out)                     # plans and buffers in place
    torch.cuda.synchronize(0)
    ref = out.cpu().numpy().copy()
    times = {}
    for k in (1, 4):
        eng.set_profiling(k)
        for _ in range(8):
            eng.render_packed(packed, out)
        torch.cuda.synchronize(0)
        times[k] = eng.stage_times()
        eng.set_profiling(False)
        assert np.array_equal(out.cpu().numpy(), ref)  # the events do not touch the render
    for k, t in times.items():
        # [2] generate .. [7] total are device windows, [10] the host plan wall clock
        assert all(v > 0.0 for v in (t[2], t[3], t[6], t[7], t[10])), (k, t)
        assert t[7] >= t[2], (k, t)
    # batches 0 and 4 of 8 were profiled with k = 4: the same stages, averaged over fewer batches
    assert times[4][7] < 20.0 * times[1][7] and times[1][7] < 20.0 * times[4][7]
