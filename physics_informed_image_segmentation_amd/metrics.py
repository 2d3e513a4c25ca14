"""Thresholded Dice of src/metrics.py:4-73 from the fused kernel's exact
per-sample counters (one launch pair, no Python loop over the batch)."""
from __future__ import annotations

import torch

from .fused import LossConfig, loss_forward


def sample_counts(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                  smooth: float = 1e-6):
    """(B, 3) int32 counts (I_hat, P_hat, T) and (B, 2) (Dice, IoU) scores, on the device."""
    _, counts, scores = loss_forward(predictions, targets,
                                     LossConfig(dice_w=0.0, bce_w=0.0, smooth=smooth, thr=threshold))
    return counts, scores


def compute_dice_score(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                       smooth: float = 1e-6) -> torch.Tensor:
    counts, _ = sample_counts(predictions, targets, threshold, smooth)
    tot = counts.sum(dim=0).to(torch.float32)
    return (2.0 * tot[0] + smooth) / (tot[1] + tot[2] + smooth)


def compute_dice_score_batch(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                             smooth: float = 1e-6) -> torch.Tensor:
    return sample_counts(predictions, targets, threshold, smooth)[1][:, 0].contiguous()
