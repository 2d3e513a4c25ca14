"""ctypes binding of the gfx950 C-ABI (include/pis_capi.h).

This is the only door to the kernels: there is no CPU or eager-PyTorch
fallback. If ``_lib/libpis.so`` is missing (not built) or no GPU is visible,
every call raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_double, c_float, c_int, c_int64, c_size_t, c_void_p
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libpis.so")

PIS_RELU, PIS_SCALE, PIS_MASK, PIS_ACCUMULATE, PIS_WINO_PREPARED, PIS_W_UNFLIPPED = 1, 2, 4, 8, 16, 32
PIS_FILTER_READY = 64
PIS_LOSS_ALL_TERMS, PIS_LOSS_CHAIN_SIGMOID, PIS_LOSS_NO_REACTION = 1, 2, 4
PIS_TUNE_LAST_WGRAD_MAIN = 42  # include/pis_capi.h: host schedule knob (unet.py)
LOSS_NTERMS = 8
TERM_TOTAL, TERM_DICE, TERM_BCE, TERM_RD, TERM_PF, TERM_I, TERM_P, TERM_T = range(8)


class FilterJob(ctypes.Structure):
    """pis_filter_job (include/pis_capi.h): one layer's filter transform in pis_conv3x3_filters."""
    _fields_ = [("w", c_void_p), ("out", c_void_p), ("out_bytes", c_size_t), ("B", c_int), ("H", c_int),
                ("W", c_int), ("Cin", c_int), ("Cout", c_int), ("dgrad", c_int)]


class LossParams(ctypes.Structure):
    _fields_ = [("dice_w", c_float), ("bce_w", c_float), ("rd_w", c_float), ("pf_w", c_float),
                ("smooth", c_float), ("D", c_float), ("a", c_float), ("eps", c_float),
                ("thr", c_float), ("flags", c_int)]


P, I, L, Z, Dbl = c_void_p, c_int, c_int64, c_size_t, c_double
# void hook(const char* kernel, int phase, void* stream, double flop, void* user)
LAUNCH_HOOK_T = ctypes.CFUNCTYPE(None, ctypes.c_char_p, c_int, c_void_p, ctypes.c_double, c_void_p)

_SIGNATURES = {
    "pis_set_launch_hook": ([LAUNCH_HOOK_T, P], None),
    "pis_arm_gemm_event": ([P], c_int),
    "pis_stream_create": ([I, ctypes.POINTER(c_void_p)], c_int),
    "pis_stream_destroy": ([P], c_int),
    "pis_stream_capture_status": ([P], c_int),
    "pis_version": ([], c_int),
    "pis_last_error": ([], ctypes.c_char_p),
    "pis_tune": ([I, I], c_int),
    "pis_debug_gemm_nt": ([P, P, P, I, I, I, I, I, P], c_int),
    "pis_debug_stream_probe": ([P, P, P, L, P, I, P], c_int),
    "pis_debug_band_probe": ([P, L, I, P, I, P], c_int),
    "pis_conv3x3_dgrad_direct": ([I, I, I, I, I, I, Z], c_int),
    "pis_conv3x3_bwd_prep": ([P, I, I, I, I, I, I, P, Z, P, Z, P], c_int),
    "pis_conv3x3_filter_bytes": ([I, I, I, I, I, I], c_size_t),
    "pis_conv3x3_filter_format": ([I, I, I, I, I, I], c_int),
    "pis_conv3x3_filter": ([P, I, I, I, I, I, I, P, Z, P], c_int),
    "pis_conv3x3_filters": ([P, I, P], c_int),
    "pis_conv3x3_fwd_pool": ([P, I, P, P, P, P, I, I, I, I, I, I, I, P, Z, P, P, P], c_int),
    "pis_conv3x3_fwd": ([P, I, P, P, P, P, I, I, I, I, I, I, I, P], c_int),
    "pis_conv3x3_flip": ([P, P, I, I, P], c_int),
    "pis_conv3x3_dgrad": ([P, I, P, P, I, P, P, I, I, I, I, I, I, I, P], c_int),
    "pis_conv3x3_ex_ws": ([I, I, I, I, I], c_size_t),
    "pis_conv3x3_fwd_ex": ([P, I, P, P, P, P, I, I, I, I, I, I, I, P, Z, P], c_int),
    "pis_conv3x3_dgrad_ex": ([P, I, P, P, I, P, P, I, I, I, I, I, I, I, P, Z, P], c_int),
    "pis_conv3x3_wgrad_ws": ([I, I, I, I, I], c_size_t),
    "pis_conv3x3_keep_bytes": ([I, I, I, I, I], c_size_t),
    "pis_conv3x3_fwd_keep": ([P, I, P, P, P, P, I, I, I, I, I, I, I, P, Z, P, P], c_int),
    "pis_conv3x3_wgrad_keep": ([P, I, P, I, P, P, I, I, I, I, I, I, P, Z, P, P], c_int),
    "pis_conv3x3_wgrad": ([P, I, P, I, P, P, I, I, I, I, I, I, P, Z, P], c_int),
    "pis_convt2x2_fwd": ([P, I, P, P, P, I, I, I, I, I, I, P], c_int),
    "pis_convt2x2_prep": ([P, P, I, I, P], c_int),
    "pis_convt2x2_dgrad": ([P, I, P, P, I, P, I, I, I, I, I, I, I, P], c_int),
    "pis_convt2x2_wgrad_ws": ([I, I, I, I, I], c_size_t),
    "pis_convt2x2_wgrad": ([P, I, P, I, P, P, I, I, I, I, I, I, P, Z, P], c_int),
    "pis_maxpool2x2_fwd": ([P, I, P, I, I, I, I, P], c_int),
    "pis_maxpool2x2_bwd": ([P, I, P, P, I, P, I, I, I, I, I, P], c_int),
    "pis_head_fwd": ([P, I, P, P, P, P, L, I, P], c_int),
    "pis_head_bwd_ws": ([L, I], c_size_t),
    "pis_head_bwd": ([P, I, P, P, P, P, I, P, P, L, I, I, P, Z, P], c_int),
    "pis_loss_ws": ([I, I, I], c_size_t),
    "pis_loss_fwd": ([P, P, I, I, I, ctypes.POINTER(LossParams), P, P, P, P, Z, P], c_int),
    "pis_loss_bwd": ([P, P, I, I, I, ctypes.POINTER(LossParams), P, P, P, I, P], c_int),
    "pis_head_loss_fwd_ws": ([I, I, I], c_size_t),
    "pis_head_loss_fwd_ok": ([I, I, I, I], c_int),
    "pis_head_loss_fwd": ([P, I, P, P, P, P, P, I, I, I, I, ctypes.POINTER(LossParams), P, P, P, P, Z, P], c_int),
    "pis_head_loss_bwd_ws": ([I, I, I, I], c_size_t),
    "pis_head_loss_bwd": ([P, I, P, P, P, P, I, I, I, I, ctypes.POINTER(LossParams), P, P, P, I, P, P, I, P, Z,
                           P], c_int),
    "pis_adamw_step": ([P, P, P, P, L, Dbl, Dbl, Dbl, Dbl, Dbl, Dbl, Dbl, Dbl, P], c_int),
    "pis_colsum_ws": ([L, I], c_size_t),
    "pis_colsum": ([P, I, L, I, P, I, P, Z, P], c_int),
    "pis_pde_fields": ([P, I, I, I, c_float, c_float, P, P, P, P], c_int),
    "pis_pde_fields_bwd": ([P, P, P, P, I, I, I, c_float, c_float, P, P], c_int),
    "pis_synth_ws": ([I, I, I], c_size_t),
    "pis_synth_discs": ([P, P, I, ctypes.c_uint64, P, P, P, I, I, I, P, Z, P], c_int),
}

_lib: Optional[ctypes.CDLL] = None


class HipError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    """Load (once) and return the kernel library. Raises if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise HipError(f"HIP extension not built: {LIB_PATH} is missing "
                           "(run __graft_entry__.build() or `python -m physics_informed_image_segmentation_amd.build`)")
        import torch  # noqa: F401  (torch's libamdhip64.so.7 must be the runtime we bind to)
        so = ctypes.CDLL(LIB_PATH)
        for name, (argtypes, restype) in _SIGNATURES.items():
            fn = getattr(so, name)
            fn.argtypes = argtypes
            fn.restype = restype
        _lib = so
    return _lib


def exported_symbols():
    return list(_SIGNATURES)


def ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


def stream_handle(device: Optional[torch.device] = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().pis_last_error()
        raise HipError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


_tracer = None


_hook_ref = None


def set_launch_hook(fn) -> None:
    """Install fn(kernel: str, phase: int, stream: int, flop: float) around the heavy kernel
    launches of the C-ABI (pis_set_launch_hook); None removes it."""
    global _hook_ref
    if fn is None:
        lib().pis_set_launch_hook(LAUNCH_HOOK_T(), None)
        _hook_ref = None
        return
    _hook_ref = LAUNCH_HOOK_T(lambda k, ph, st, fl, user: fn(k.decode(), ph, st or 0, fl))
    lib().pis_set_launch_hook(_hook_ref, None)


def set_tracer(tracer) -> None:
    """Install an object with begin(name, args) -> token / end(token) around every
    C-ABI call (bench.py uses it to time launches with HIP events); None removes it."""
    global _tracer
    _tracer = tracer


def call(name: str, *args) -> None:
    tr = _tracer
    if tr is None:
        check(getattr(lib(), name)(*args), name)
        return
    tok = tr.begin(name, args)
    check(getattr(lib(), name)(*args), name)
    tr.end(tok)


# owned streams no longer in use, keyed by (device index, priority): handed to the next OwnedStream
# of the same device and priority, never destroyed
_free_streams = {}
# streams closed while a graph capture was running: they join the free list only once no capture
# runs and their queued work has drained (_reclaim), so the next owner never receives a stream
# with captured work still pending
_closing_streams = []


def _device_index(device) -> int:
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device) if not isinstance(device, torch.device) else device
    if d.type != "cuda":
        raise HipError(f"OwnedStream: a cuda device is needed, got {d}")
    return torch.cuda.current_device() if d.index is None else d.index


def _reclaim() -> None:
    if not _closing_streams:
        return
    try:
        if torch.cuda.is_current_stream_capturing():
            return
    except Exception:
        return
    while _closing_streams:
        h, dev, prio, ext = _closing_streams.pop()
        ext.synchronize()
        _free_streams.setdefault((dev, prio), []).append(h)


class OwnedStream:
    """A HIP stream this process owns (pis_stream_create), usable as a torch stream
    (``.stream`` is a torch.cuda.ExternalStream). torch's ``torch.cuda.Stream()`` hands out a
    fixed round-robin pool, so a stream that took part in a graph capture would later be given to
    unrelated code; an owned stream is recycled only into other OwnedStreams of the same device
    (``close()`` returns it to a free list after its work drains). It is never destroyed
    (``pis_stream_destroy`` stays in the C-ABI for other hosts; this one does not call it):
    PyTorch keeps raw stream handles beyond the objects that used them — autograd's
    AccumulateGrad nodes record the stream of the forward that created them and sync with it in
    every later backward, and the caching allocator tags blocks with their allocation stream — so
    a destroyed stream would leave those handles dangling
    (tests/test_graph_gpu.py::test_graph_dropped_without_close reproduced exactly that: a segfault
    in the next eager backward of the graphed model).

    The HIP stream is created ON ``device`` (hipStreamCreate uses the calling thread's current
    device, so the call runs inside ``torch.cuda.device(device)``): a model on cuda:1 gets its
    weight-gradient stream on cuda:1 even when cuda:0 is current."""

    def __init__(self, device=None, priority: int = 0):
        _reclaim()
        self.device_index = _device_index(device)
        self.priority = priority
        free = _free_streams.get((self.device_index, priority))
        self.handle = free.pop() if free else None
        if self.handle is None:
            raw = c_void_p()
            with torch.cuda.device(self.device_index):
                check(lib().pis_stream_create(priority, ctypes.byref(raw)), "pis_stream_create")
            self.handle = raw.value
        self.stream = torch.cuda.ExternalStream(self.handle, device=torch.device("cuda", self.device_index))

    def capture_status(self) -> int:
        return lib().pis_stream_capture_status(self.handle)

    def close(self) -> None:
        """Return the stream to the free list once its queued work is done. Inside a capture no
        sync is possible: the stream waits on a closing list until the capture has ended and its
        work has drained (the next OwnedStream() reclaims it)."""
        h, self.handle = self.handle, None
        if not h:
            return
        try:
            capturing = torch.cuda.is_current_stream_capturing()
        except Exception:
            capturing = False
        if capturing:
            _closing_streams.append((h, self.device_index, self.priority, self.stream))
            return
        self.stream.synchronize()
        _free_streams.setdefault((self.device_index, self.priority), []).append(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown: the runtime may already be gone
            pass


def require_cuda(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise HipError(f"{what}: the MI355X path needs a GPU tensor (got {t.device}); "
                       "this build has no CPU fallback")
