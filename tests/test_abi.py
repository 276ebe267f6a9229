"""C-ABI library: loads without a GPU and exports every symbol include/msgpu.h declares."""
import ctypes as C
import os
import re

from msgpu import _lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "msgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b(msg_[a-z0-9_]+)\s*\(", src)
    return sorted(set(names))


def test_header_symbols_exported():
    lib = L.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(L.EXPORTS), set(names) ^ set(L.EXPORTS)


def test_struct_layout_and_version():
    lib = L.lib()
    assert lib.msg_abi_version() == L.ABI_VERSION
    assert lib.msg_sizeof(0) == C.sizeof(L.MsgPreset)
    assert lib.msg_sizeof(1) == C.sizeof(L.MsgEvent) == 80
    assert lib.msg_sizeof(2) == C.sizeof(L.MsgPlanInfo) == 32


def test_create_without_gpu_fails_cleanly():
    # In the build container there is no GPU: msg_create must return NULL with
    # a message, never crash (the product path then raises; no CPU fallback).
    lib = L.lib()
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    ctx = lib.msg_create(0)
    assert not ctx
    assert b"device" in lib.msg_last_error(None).lower()
