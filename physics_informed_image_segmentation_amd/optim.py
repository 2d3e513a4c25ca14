"""Decoupled AdamW of src/train.py:658-662 (``optim.AdamW(params, lr,
weight_decay=1e-5)``) as ONE HIP kernel launch over the U-Net's flat
parameter arena.

Semantics are torch.optim.AdamW's single-tensor path (torch/optim/adam.py):
p *= 1 - lr*wd; m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps), scalars rounded to fp32 as torch
rounds its Python floats. ``grad_scale`` multiplies the gradient inside the
kernel (data-parallel averaging without an extra pass).
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Tuple

import torch

from . import _hip


class AdamW(torch.optim.Optimizer):
    def __init__(self, params: Iterable[torch.Tensor], lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 1e-2, grad_scale: float = 1.0):
        if lr < 0 or eps < 0 or weight_decay < 0:
            raise ValueError("invalid AdamW hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.grad_scale = grad_scale
        self._flat = {}  # group index -> (arena tensor, m, v, offsets) when every param views one arena

    # ---- arena discovery ------------------------------------------------------
    @staticmethod
    def _storage(t: torch.Tensor) -> Tuple[int, int]:
        s = t.untyped_storage()
        return s.data_ptr(), s.nbytes()

    def _flat_state(self, gi: int, group):
        params: List[torch.Tensor] = group["params"]
        key = (gi, params[0].untyped_storage().data_ptr())
        st = self._flat.get(gi)
        if st is not None and st["key"] == key:
            return st
        base, nbytes = self._storage(params[0])
        if any(self._storage(p) != (base, nbytes) for p in params):
            return None
        arena = torch.empty(0, dtype=torch.float32, device=params[0].device).set_(
            params[0].untyped_storage(), 0, (nbytes // 4,), (1,))
        offs = [(p.data_ptr() - base) // 4 for p in params]
        # adopt moments a previous (per-tensor or older) state may hold
        m = torch.zeros_like(arena)
        v = torch.zeros_like(arena)
        step = 0
        for p, o in zip(params, offs):
            s = self.state.get(p)
            if s and "exp_avg" in s and s["exp_avg"].data_ptr() != m.data_ptr() + 4 * o:
                m.narrow(0, o, p.numel()).copy_(s["exp_avg"].reshape(-1))
                v.narrow(0, o, p.numel()).copy_(s["exp_avg_sq"].reshape(-1))
                step = int(s.get("step", 0))
        for p, o in zip(params, offs):
            self.state[p] = {"step": torch.tensor(float(step)),
                             "exp_avg": m.narrow(0, o, p.numel()).view(p.shape) if p.is_contiguous()
                             else m.narrow(0, o, p.numel()),
                             "exp_avg_sq": v.narrow(0, o, p.numel()).view(p.shape) if p.is_contiguous()
                             else v.narrow(0, o, p.numel())}
        st = {"key": key, "arena": arena, "m": m, "v": v, "offs": offs, "step": step}
        self._flat[gi] = st
        return st

    # ---- step -----------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            params = [p for p in group["params"]]
            if not params:
                continue
            _hip.require_cuda(params[0], "AdamW.step")
            st = self._flat_state(gi, group)
            if st is None:
                raise NotImplementedError("AdamW (MI355X) expects the parameters of one UNet (a single arena)")
            with_grad = [p.grad is not None for p in params]
            if not any(with_grad):
                continue
            st["step"] += 1
            step = st["step"]
            for p in params:
                self.state[p]["step"].fill_(float(step))
            lr, (b1, b2), eps, wd = group["lr"], group["betas"], group["eps"], group["weight_decay"]
            bc1 = 1.0 - b1 ** step
            bc2 = 1.0 - b2 ** step
            step_size, bc2_sqrt = lr / bc1, bc2 ** 0.5
            arena, m, v, offs = st["arena"], st["m"], st["v"], st["offs"]
            g_flat = self._grad_arena(params, offs, arena)
            stream = _hip.stream_handle()
            if g_flat is not None and all(with_grad):
                _hip.call("pis_adamw_step", arena.data_ptr(), g_flat.data_ptr(), m.data_ptr(), v.data_ptr(),
                          arena.numel(), lr, b1, b2, eps, wd, step_size, bc2_sqrt, self.grad_scale, stream)
                continue
            for p, o in zip(params, offs):  # per-tensor launches (params without grad are skipped, as torch)
                if p.grad is None:
                    continue
                g = p.grad
                if g.stride() != p.stride():
                    g = torch.empty_strided(p.shape, p.stride(), device=p.device).copy_(g)
                _hip.call("pis_adamw_step", p.data_ptr(), g.data_ptr(), m.data_ptr() + 4 * o, v.data_ptr() + 4 * o,
                          p.numel(), lr, b1, b2, eps, wd, step_size, bc2_sqrt, self.grad_scale, stream)
        return loss

    @staticmethod
    def _grad_arena(params, offs, arena) -> Optional[torch.Tensor]:
        """The flat gradient arena when every .grad views one storage at its parameter's offset."""
        g0 = params[0].grad
        if g0 is None:
            return None
        gs = g0.untyped_storage()
        if gs.nbytes() != arena.numel() * 4:
            return None
        gbase = gs.data_ptr()
        for p, o in zip(params, offs):
            if p.grad is None or p.grad.untyped_storage().data_ptr() != gbase or \
                    p.grad.data_ptr() != gbase + 4 * o or p.grad.stride() != p.stride():
                return None
        return torch.empty(0, dtype=torch.float32, device=arena.device).set_(gs, 0, (arena.numel(),), (1,))
