"""PDE regularisation of src/pde.py on the MI355X kernel path.

``PDERegularization`` keeps the reference's constructor checks, buffers and
method names (src/pde.py:6-212). The two losses the training step uses,
``compute_loss`` (reaction-diffusion residual, :124-145) and
``compute_phase_field_loss`` (:180-212), are the fused HIP kernel. The
per-pixel field helpers (``compute_laplacian``, ``reaction_term``,
``compute_residual``, ``compute_gradient_magnitude``, :49-178) are one HIP
stencil kernel each way (``pis_pde_fields`` / ``pis_pde_fields_bwd``) and are
differentiable, like the reference's F.pad + F.conv2d compositions.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _hip
from .fused import LossConfig, fused_loss

_LAP, _RES, _GM = 0, 1, 2


class _PDEField(torch.autograd.Function):
    """One reflect-padded stencil field of u and its exact adjoint."""

    @staticmethod
    def forward(ctx, u, which: int, D: float, a: float):
        _hip.require_cuda(u, "PDERegularization")
        if u.dtype != torch.float32:
            raise TypeError("PDERegularization: float32 input expected")
        uc = u.detach().contiguous()
        B, H, W = uc.shape[0], uc.shape[-2], uc.shape[-1]
        if uc.numel() != B * H * W:
            raise ValueError(f"single-channel maps expected, got {tuple(u.shape)}")
        out = torch.empty_like(uc)
        ptrs = [0, 0, 0]
        ptrs[which] = out.data_ptr()
        _hip.call("pis_pde_fields", uc.data_ptr(), B, H, W, float(D), float(a), *ptrs, _hip.stream_handle())
        ctx.save_for_backward(uc)
        ctx.which, ctx.D, ctx.a = which, float(D), float(a)
        return out

    @staticmethod
    def backward(ctx, g):
        (u,) = ctx.saved_tensors
        B, H, W = u.shape[0], u.shape[-2], u.shape[-1]
        g = g.to(torch.float32).contiguous()
        ptrs = [0, 0, 0]
        ptrs[ctx.which] = g.data_ptr()
        du = torch.empty_like(u)
        _hip.call("pis_pde_fields_bwd", u.data_ptr(), *ptrs, B, H, W, ctx.D, ctx.a, du.data_ptr(),
                  _hip.stream_handle())
        return du, None, None, None


class PDERegularization(nn.Module):
    def __init__(self, diffusion_coeff: float = 1.0, reaction_threshold: float = 0.5):
        super().__init__()
        if diffusion_coeff <= 0:
            raise ValueError("diffusion_coeff must be positive")
        if not (0 < reaction_threshold < 1):
            raise ValueError("reaction_threshold must be in (0,1)")
        self.diffusion_coeff = diffusion_coeff
        self.reaction_threshold = reaction_threshold
        # stencil coefficients kept as buffers for state_dict compatibility (src/pde.py:24-47);
        # the kernels hard-code the same 5-point / central-difference taps
        lap = torch.tensor([[0.0, 1.0, 0.0], [1.0, -4.0, 1.0], [0.0, 1.0, 0.0]])
        gx = torch.tensor([[0.0, 0.0, 0.0], [-0.5, 0.0, 0.5], [0.0, 0.0, 0.0]])
        self.register_buffer("laplacian_kernel", lap[None, None].clone())
        self.register_buffer("grad_x_kernel", gx[None, None].clone())
        self.register_buffer("grad_y_kernel", gx.t()[None, None].contiguous())

    # ---- per-pixel fields (differentiable) ----------------------------------------
    def compute_laplacian(self, u: torch.Tensor) -> torch.Tensor:
        """5-point Laplacian with reflect padding (src/pde.py:49-79)."""
        return _PDEField.apply(u, _LAP, 0.0, 0.0)

    def reaction_term(self, u: torch.Tensor) -> torch.Tensor:
        """u (1 - u) (u - a) (src/pde.py:81-99): the residual with D = 0."""
        return _PDEField.apply(u, _RES, 0.0, self.reaction_threshold)

    def compute_residual(self, u: torch.Tensor) -> torch.Tensor:
        """D Lap(u) + u (1 - u) (u - a) (src/pde.py:101-122)."""
        return _PDEField.apply(u, _RES, self.diffusion_coeff, self.reaction_threshold)

    def compute_gradient_magnitude(self, u: torch.Tensor) -> torch.Tensor:
        """gx^2 + gy^2 of the reflect-padded central differences (src/pde.py:147-178)."""
        return _PDEField.apply(u, _GM, 0.0, 0.0)

    # ---- losses (fused kernel, differentiable) ----------------------------------
    def compute_loss(self, u: torch.Tensor) -> torch.Tensor:
        cfg = LossConfig(dice_w=0.0, bce_w=0.0, rd_w=1.0, pf_w=0.0, D=self.diffusion_coeff,
                         a=self.reaction_threshold)
        return fused_loss(u, u.detach(), cfg)

    def compute_phase_field_loss(self, u: torch.Tensor, epsilon: float = 0.05) -> torch.Tensor:
        if epsilon <= 0:
            raise ValueError("epsilon must be positive")
        cfg = LossConfig(dice_w=0.0, bce_w=0.0, rd_w=0.0, pf_w=1.0, eps=epsilon, D=self.diffusion_coeff,
                         a=self.reaction_threshold)
        return fused_loss(u, u.detach(), cfg)


def create_pde_regularization(diffusion_coeff: float = 1.0, reaction_threshold: float = 0.5) -> PDERegularization:
    """src/pde.py:215-232."""
    return PDERegularization(diffusion_coeff=diffusion_coeff, reaction_threshold=reaction_threshold)
