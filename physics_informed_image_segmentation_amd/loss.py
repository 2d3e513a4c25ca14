"""Segmentation losses of src/loss.py on the fused MI355X kernel.

``DiceBCELoss`` (src/loss.py:7-68) and ``DiceBCEPDELoss`` (src/loss.py:71-162)
keep the reference's constructor arguments, defaults, attributes read by the
training loop (``smooth``, ``bce``, ``pde_weight``, ``phase_field_weight``,
``epsilon``, ``pde_regularization``) and term gating (a PDE term enters the
total only when its weight is > 0). The forward is ONE fused kernel pass that
also leaves every per-term value and the per-sample Dice/IoU counters in
``criterion.last`` for the step loop, so nothing is recomputed for logging
(the reference recomputes every term, src/train.py:120-150).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .fused import LossConfig, fused_loss
from .pde import PDERegularization


class BCELoss(nn.Module):
    """``nn.BCELoss()`` (mean, log clamped at -100) on the fused kernel."""

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        return fused_loss(predictions, targets, LossConfig(dice_w=0.0, bce_w=1.0))


class DiceBCELoss(nn.Module):
    def __init__(self, dice_weight: float = 0.5, bce_weight: float = 0.5, smooth: float = 1e-6):
        super().__init__()
        self.dice_weight = dice_weight
        self.bce_weight = bce_weight
        self.smooth = smooth
        self.bce = BCELoss()
        self.last: dict = {}

    def config(self, all_terms: bool = False) -> LossConfig:
        return LossConfig(dice_w=self.dice_weight, bce_w=self.bce_weight, smooth=self.smooth, all_terms=all_terms)

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        self.last = {}
        return fused_loss(predictions, targets, self.config(), self.last)


class DiceBCEPDELoss(nn.Module):
    def __init__(self, dice_weight: float = 0.5, bce_weight: float = 0.5, pde_weight: float = 1e-3,
                 phase_field_weight: float = 0.0, smooth: float = 1e-6, diffusion_coeff: float = 1.0,
                 reaction_threshold: float = 0.5, epsilon: float = 0.05):
        super().__init__()
        self.dice_weight = dice_weight
        self.bce_weight = bce_weight
        self.pde_weight = pde_weight
        self.phase_field_weight = phase_field_weight
        self.smooth = smooth
        self.epsilon = epsilon
        self.pde_regularization = PDERegularization(diffusion_coeff=diffusion_coeff,
                                                    reaction_threshold=reaction_threshold)
        self.bce = BCELoss()
        self.last: dict = {}

    def config(self, all_terms: bool = False) -> LossConfig:
        if self.phase_field_weight > 0 and self.epsilon <= 0:
            raise ValueError("epsilon must be positive")
        pr = self.pde_regularization
        return LossConfig(dice_w=self.dice_weight, bce_w=self.bce_weight, rd_w=max(self.pde_weight, 0.0),
                          pf_w=max(self.phase_field_weight, 0.0), smooth=self.smooth, D=pr.diffusion_coeff,
                          a=pr.reaction_threshold, eps=self.epsilon, all_terms=all_terms)

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        self.last = {}
        return fused_loss(predictions, targets, self.config(), self.last)
