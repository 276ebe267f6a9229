"""The drop-in's error contract for missing keys (CPU, no device work).

The reference ``render`` indexes its params dict directly, so a dict missing a
key it reads raises ``KeyError(key)`` (MS:589-784).  tests/golden/keyerrors.json
holds, for four full dicts, the key of the KeyError the reference raised with
each single key deleted (tools/gen_keyerrors.py).  msgpu.render raises the same
KeyError before it touches the device.
"""
import json
import os

import numpy as np
import pytest

import msgpu
from msgpu.params import first_missing_key

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _cases():
    with open(os.path.join(GOLDEN, "keyerrors.json")) as f:
        return json.load(f)


def _full(rec, irs):
    d = dict(rec["params"])
    if rec["ir"]:
        d["_ir_audio"] = irs[rec["ir"]]
    return d


@pytest.fixture(scope="module")
def irs():
    z = np.load(os.path.join(GOLDEN, "irs.npz"))
    return {k: z[k] for k in z.files}


@pytest.mark.parametrize("base", ["C2", "defaults", "everything_on", "all_off"])
def test_missing_key_matches_reference(base, irs):
    rec = _cases()[base]
    full = _full(rec, irs)
    assert first_missing_key(full) is None
    bad = {}
    for k, want in rec["missing_key_raises"].items():
        d = dict(full)
        del d[k]
        got = first_missing_key(d)
        if got != want:
            bad[k] = (got, want)
    assert not bad, bad


def test_render_raises_keyerror_before_device(irs):
    rec = _cases()["defaults"]
    d = _full(rec, irs)
    del d["base_sr"]
    with pytest.raises(KeyError) as ei:
        msgpu.render(d)          # raises before any HIP call (no GPU in the CPU suite)
    assert ei.value.args[0] == "base_sr"
    d = msgpu.merged(out_dur_s=0.1)
    del d["peak"]
    with pytest.raises(KeyError):
        msgpu.render(d)
