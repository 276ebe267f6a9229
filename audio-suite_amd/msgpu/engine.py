"""Device engine: one libmsgpu context per (process, device).

``Engine.render_packed`` enqueues one batched render on the current torch
stream and returns the device output tensor (frames x 2, float32,
interleaved L/R).  PyTorch-ROCm is used only as the device-buffer container
and for its stream handle.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np

from . import _lib as L
from .pack import PackedBatch


# msg_digest_rec as a numpy record
DIGEST_DTYPE = np.dtype([("sum_sq", "<f8"), ("peak", "<f8"), ("sum_l", "<f8"), ("sum_r", "<f8"),
                         ("h0", "<u8"), ("h1", "<u8")])


class Engine:
    def __init__(self, device: int = 0):
        import torch  # device buffers only

        if not torch.cuda.is_available():
            raise RuntimeError("msgpu needs a HIP device (torch.cuda.is_available() is False)")
        self.torch = torch
        self.device = int(device)
        lib = L.lib()
        with torch.cuda.device(self.device):
            torch.cuda.current_stream()  # initialise the runtime on this device first
            ctx = lib.msg_create(self.device)
        if not ctx:
            raise RuntimeError("msg_create failed: " + lib.msg_last_error(None).decode())
        self._ctx = C.c_void_p(ctx)
        self._lock = threading.Lock()
        self._last_n = 0

    def close(self):
        if getattr(self, "_ctx", None):
            L.lib().msg_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------
    def set_profiling(self, on):
        """False / 0 off, True / 1 every batch, k > 1 every k-th batch of this context."""
        k = 0 if not on else max(1, int(on))
        L.check(L.lib().msg_set_profiling(self._ctx, k), self._ctx)

    def gate(self, peer, wait_stage: int = 2, record_stage: int = 6):
        """Order this context's batches against ``peer``'s (msg_gate): stage
        ``wait_stage`` of each batch waits for the stage ``record_stage`` of the
        peer's latest batch to begin.  ``peer=None`` clears the gate."""
        L.check(L.lib().msg_gate(self._ctx, peer._ctx if peer is not None else None, int(wait_stage),
                                 int(record_stage)), self._ctx)
        self._gate_peer = peer      # the peer context stays alive while this one gates on it

    def stage_times(self):
        arr = (C.c_float * 19)()
        L.check(L.lib().msg_stage_times(self._ctx, arr, 19), self._ctx)
        return list(arr)

    def alloc_output(self, packed: PackedBatch):
        return self.torch.empty((packed.total_frames, 2), dtype=self.torch.float32,
                                device=f"cuda:{self.device}")

    def render_packed(self, packed: PackedBatch, out=None, stream=None):
        """Enqueue the batch; returns the output tensor (not yet synchronised)."""
        torch = self.torch
        if out is None:
            out = self.alloc_output(packed)
        if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < 2 * packed.total_frames:
            raise ValueError("output tensor must be contiguous float32 with 2*frames elements")
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        with self._lock:
            st = L.lib().msg_render_batch(
                self._ctx, packed.presets, packed.n, packed.bp_ptr, packed.bp_pairs,
                packed.ir_ptrs, packed.ir_lens, packed.n_irs,
                packed.img_ptrs, packed.img_h, packed.img_w, packed.n_images,
                C.c_void_p(out.data_ptr()), packed._offsets_c, C.c_void_p(stream.cuda_stream))
            L.check(st, self._ctx)
            self._last_n = packed.n
        return out

    def render_batch(self, params_list, out=None):
        packed = PackedBatch(params_list)
        return self.render_packed(packed, out), packed

    def stft_mag_db(self, x, win=2048, hop=256, max_frames=3000, stream=None):
        """Spectrogram of a device float32/float64 tensor (n,) mono or (n, 2) stereo (L/R
        mean): returns a device float64 tensor (frames, win//2 + 1), enqueued on ``stream``."""
        torch = self.torch
        if x.dtype not in (torch.float32, torch.float64) or not x.is_contiguous() or x.device.type != "cuda":
            raise ValueError("x must be a contiguous float32 or float64 device tensor")
        eb = x.element_size()
        channels = 1 if x.dim() == 1 else int(x.shape[1])
        if x.dim() > 2 or channels not in (1, 2):
            raise ValueError("x must be (n,) or (n, 2)")
        n = int(x.shape[0])
        frames = C.c_int32(0)
        lib = L.lib()
        L.check(lib.msg_stft_mag_db(self._ctx, None, eb, n, channels, int(win), int(hop), int(max_frames),
                                    None, C.byref(frames), None), self._ctx)
        S = torch.empty((frames.value, int(win) // 2 + 1), dtype=torch.float64, device=x.device)
        if frames.value == 0:
            return S
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        with self._lock:
            L.check(lib.msg_stft_mag_db(self._ctx, C.c_void_p(x.data_ptr()), eb, n, channels, int(win), int(hop),
                                        int(max_frames), C.c_void_p(S.data_ptr()), C.byref(frames),
                                        C.c_void_p(stream.cuda_stream)), self._ctx)
        return S

    def fir(self, x, h, out=None, stream=None):
        """Causal FIR y = np.convolve(x, h)[:n] of each row of a device float32 tensor
        (S, n) or (n,), h float64 taps (host); returns (y, (N, P, Q)) enqueued on ``stream``."""
        torch = self.torch
        if x.dtype != torch.float32 or not x.is_contiguous() or x.device.type != "cuda" or x.dim() > 2:
            raise ValueError("x must be a contiguous float32 device tensor (n,) or (S, n)")
        S, n = (1, int(x.shape[0])) if x.dim() == 1 else (int(x.shape[0]), int(x.shape[1]))
        hh = np.ascontiguousarray(h, dtype=np.float64)
        if hh.ndim != 1 or hh.size < 1:
            raise ValueError("h must be a non-empty 1-D array")
        if out is None:
            out = torch.empty_like(x)
        if out.shape != x.shape or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("out must match x")
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        shape = (C.c_int32 * 3)()
        with self._lock:
            L.check(L.lib().msg_fir(self._ctx, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), n, S,
                                    hh.ctypes.data_as(C.c_void_p), int(hh.size), shape,
                                    C.c_void_p(stream.cuda_stream)), self._ctx)
        return out, tuple(shape)

    def digest(self, out, offsets, out_n, stream=None):
        """msg_digest of renders lying in a device output tensor ((frames, 2)
        float32, render i at frame offsets[i], out_n[i] frames): one record per
        render reduced on the device (float64 sums, peak, the 128-bit digest);
        only the records (48 B each) are copied back.  Returns a numpy structured
        array with fields sum_sq, peak, sum_l, sum_r, h0, h1."""
        torch = self.torch
        if out.dtype != torch.float32 or not out.is_contiguous() or out.device.type != "cuda":
            raise ValueError("out must be a contiguous float32 device tensor")
        off = np.ascontiguousarray(offsets, dtype=np.int64)
        cnt = np.ascontiguousarray(out_n, dtype=np.int64)
        if off.shape != cnt.shape or off.ndim != 1:
            raise ValueError("offsets and out_n must be 1-D of one length")
        if off.size and int((off + cnt).max()) * 2 > out.numel():
            raise ValueError("a render extends past the output tensor")
        n = int(off.size)
        rec = torch.empty((max(n, 1), 6), dtype=torch.float64, device=out.device)
        if stream is None:
            stream = torch.cuda.current_stream(out.device)
        with self._lock:
            L.check(L.lib().msg_digest(self._ctx, C.c_void_p(out.data_ptr()),
                                       off.ctypes.data_as(C.POINTER(C.c_int64)),
                                       cnt.ctypes.data_as(C.POINTER(C.c_int64)), n, C.c_void_p(rec.data_ptr()),
                                       C.c_void_p(stream.cuda_stream)), self._ctx)
        with torch.cuda.stream(stream):
            host = rec.cpu().numpy()       # ordered after the digest on its stream
        return host[:n].copy().view(DIGEST_DTYPE).reshape(n)

    # ---- last-batch inspection -----------------------------------------
    def last_plan(self):
        arr = (L.MsgPlanInfo * self._last_n)()
        L.check(L.lib().msg_last_plan(self._ctx, arr, self._last_n), self._ctx)
        return list(arr)

    def last_events(self, preset: int):
        n = C.c_int32(0)
        L.check(L.lib().msg_last_events(self._ctx, preset, None, 0, C.byref(n)), self._ctx)
        arr = (L.MsgEvent * max(n.value, 1))()
        L.check(L.lib().msg_last_events(self._ctx, preset, arr, n.value, C.byref(n)), self._ctx)
        return list(arr)[:n.value]

    def last_grain64(self, preset: int, k: int):
        """Float64 grain of event k of a float64-chain preset of the last batch."""
        n = C.c_int64(0)
        L.check(L.lib().msg_last_grain64(self._ctx, preset, k, None, 0, C.byref(n)), self._ctx)
        g = np.zeros(max(n.value, 1), dtype=np.float64)
        L.check(L.lib().msg_last_grain64(self._ctx, preset, k, g.ctypes.data_as(C.POINTER(C.c_double)), n.value,
                                         C.byref(n)), self._ctx)
        return g[:n.value].copy()

    def last_meta(self, preset: int, cap: int):
        micro = np.zeros(max(cap, 1), dtype=np.float64)
        grain = np.zeros(max(cap, 1), dtype=np.float64)
        n = C.c_int64(0)
        L.check(L.lib().msg_last_meta(self._ctx, preset, micro.ctypes.data_as(C.POINTER(C.c_double)),
                                      grain.ctypes.data_as(C.POINTER(C.c_double)), cap, C.byref(n)),
                self._ctx)
        if n.value == 0:
            return None, None
        return micro[:n.value].copy(), grain[:n.value].copy()


_engines: dict = {}
_engines_lock = threading.Lock()


def default_engine(device: int = 0) -> Engine:
    with _engines_lock:
        eng = _engines.get(device)
        if eng is None:
            eng = Engine(device)
            _engines[device] = eng
        return eng
