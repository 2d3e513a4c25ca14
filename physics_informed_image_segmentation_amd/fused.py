"""Autograd wrapper of the fused Dice + BCE + reaction-diffusion + phase-field
kernel (pis_loss_fwd / pis_loss_bwd). One forward launch pair computes every
loss term, the whole-batch Dice sums and the per-sample thresholded metric
counters; the backward is one elementwise launch — or, when the prediction is
the U-Net's own output, part of the head backward kernel (pis_head_loss_bwd).

Used by src-compatible ``loss`` (src/loss.py:7-162), ``pde``
(src/pde.py:124-212) and ``metrics`` (src/metrics.py:4-73) modules.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Dict, Tuple

import torch

from . import _hip
from ._hip import LossParams, PIS_LOSS_ALL_TERMS, PIS_LOSS_NO_REACTION, call


@dataclass(frozen=True)
class LossConfig:
    dice_w: float = 0.5
    bce_w: float = 0.5
    rd_w: float = 0.0
    pf_w: float = 0.0
    smooth: float = 1e-6
    D: float = 1.0
    a: float = 0.5
    eps: float = 0.05
    thr: float = 0.5
    all_terms: bool = False
    reaction: bool = True  # False: diffusion-only residual (src/ablation.py:53-86)

    def params(self) -> LossParams:
        flags = (PIS_LOSS_ALL_TERMS if self.all_terms else 0) | (0 if self.reaction else PIS_LOSS_NO_REACTION)
        return LossParams(self.dice_w, self.bce_w, self.rd_w, self.pf_w, self.smooth, self.D, self.a,
                          self.eps, self.thr, flags)


_WS: Dict[Tuple, torch.Tensor] = {}


def _workspace(B: int, H: int, W: int, dev: torch.device) -> torch.Tensor:
    key = (B, H, W, dev)
    ws = _WS.get(key)
    if ws is None:
        n = _hip.lib().pis_loss_ws(B, H, W)
        ws = torch.zeros((n + 3) // 4, dtype=torch.float32, device=dev)  # zeroed once (pis_capi.h)
        _WS[key] = ws
    return ws


def _bhw(u: torch.Tensor) -> Tuple[int, int, int]:
    if u.dim() < 2:
        raise ValueError("expected (B, 1, H, W) or (B, H, W) tensors")
    B, H, W = u.shape[0], u.shape[-2], u.shape[-1]
    if u.numel() != B * H * W:
        raise ValueError(f"single-channel maps expected, got {tuple(u.shape)}")
    return B, H, W


def _prep(u: torch.Tensor, t: torch.Tensor, what: str):
    _hip.require_cuda(u, what)
    if t.shape != u.shape and t.numel() != u.numel():
        raise ValueError(f"{what}: target shape {tuple(t.shape)} does not match prediction {tuple(u.shape)}")
    if u.dtype != torch.float32:
        raise TypeError(f"{what}: float32 predictions expected")
    u = u.detach().contiguous()
    t = t.to(device=u.device, dtype=torch.float32).contiguous()
    return u, t


def loss_forward(u: torch.Tensor, t: torch.Tensor, cfg: LossConfig):
    """-> (terms[8], counts (B,3) int32, scores (B,2)); all on the device, no sync."""
    u, t = _prep(u, t, "fused loss")
    B, H, W = _bhw(u)
    dev = u.device
    terms = torch.empty(_hip.LOSS_NTERMS, dtype=torch.float32, device=dev)
    counts = torch.empty(B, 3, dtype=torch.int32, device=dev)
    scores = torch.empty(B, 2, dtype=torch.float32, device=dev)
    ws = _workspace(B, H, W, dev)
    prm = cfg.params()
    call("pis_loss_fwd", u.data_ptr(), t.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(),
         counts.data_ptr(), scores.data_ptr(), ws.data_ptr(), ws.numel() * 4, _hip.stream_handle())
    return terms, counts, scores


class _FusedLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, u, t, cfg: LossConfig, sink: dict, precomputed: bool = False):
        if precomputed:  # the U-Net's head + loss forward already filled the sink (pis_head_loss_fwd)
            terms = sink["terms"]
        else:
            terms, counts, scores = loss_forward(u, t, cfg)
            sink["terms"], sink["counts"], sink["scores"] = terms, counts, scores
        ctx.cfg = cfg
        ctx.shape = u.shape
        # produced directly by the U-Net engine? then the backward runs fused with its head
        ctx.eng = getattr(u.grad_fn, "eng", None)
        ctx.gen = getattr(u.grad_fn, "gen", None)
        ctx.save_for_backward(u.detach().contiguous(), t.to(device=u.device, dtype=torch.float32).contiguous(),
                              terms)
        # a view of the terms buffer (allocated per call, never written again): no copy launch
        return terms[0]

    @staticmethod
    def backward(ctx, g):
        u, t, terms = ctx.saved_tensors
        B, H, W = _bhw(u)
        g = g.to(torch.float32).contiguous()
        prm = ctx.cfg.params()
        eng = ctx.eng
        if eng is not None and hasattr(eng, "can_fuse_loss") and eng.can_fuse_loss(u, ctx.gen):
            du = eng.fuse_loss_backward(t, ctypes.byref(prm), terms, g)
            return du.view(ctx.shape), None, None, None, None
        du = torch.empty_like(u)
        call("pis_loss_bwd", u.data_ptr(), t.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(),
             g.data_ptr(), du.data_ptr(), 0, _hip.stream_handle())
        return du.view(ctx.shape), None, None, None, None


def fused_loss(u: torch.Tensor, t: torch.Tensor, cfg: LossConfig, sink: dict = None) -> torch.Tensor:
    """Differentiable total loss (0-dim); per-term values land in ``sink``.

    In grad mode the returned loss is a view of ``sink["terms"]`` (no copy launch in the step):
    modifying it in place (``loss /= k``) raises autograd's custom-Function view error; write
    ``loss = loss / k`` instead. In no-grad mode it is a copy, so in-place updates never reach the
    logged terms."""
    if sink is None:
        sink = {}
    if not (torch.is_grad_enabled() and u.requires_grad):
        terms, counts, scores = loss_forward(u, t, cfg)
        sink["terms"], sink["counts"], sink["scores"] = terms, counts, scores
        return terms[0].clone()
    return _FusedLoss.apply(u, t, cfg, sink)


def loss_from_forward(u: torch.Tensor, t: torch.Tensor, cfg: LossConfig, sink: dict) -> torch.Tensor:
    """The differentiable total loss of terms the U-Net's fused head + loss forward already wrote
    into ``sink`` (UNet.forward_with_loss): an autograd node with no forward launch of its own.
    Same aliasing rule as ``fused_loss``: a view of the terms in grad mode, a copy otherwise."""
    if not (torch.is_grad_enabled() and u.requires_grad):
        return sink["terms"][0].clone()
    return _FusedLoss.apply(u, t, cfg, sink, True)
