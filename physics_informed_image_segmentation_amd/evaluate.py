"""IoU of src/evaluate.py:26-97 on the fused counters, plus the boundary
metrics the step loop logs (src/evaluate.py:102-275).

IoU is on the hot path (computed every step, src/train.py:155) and comes from
the same per-sample counters as Dice. Boundary-F1 / Hausdorff are host-side
OpenCV routines in the reference (cv2 is not installed here); they are
out of this round's scope and raise a clear error.
"""
from __future__ import annotations

import torch

from .metrics import sample_counts


def compute_iou(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                smooth: float = 1e-6) -> torch.Tensor:
    counts, _ = sample_counts(predictions, targets, threshold, smooth)
    tot = counts.sum(dim=0).to(torch.float32)
    return (tot[0] + smooth) / (tot[1] + tot[2] - tot[0] + smooth)


def compute_iou_batch(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                      smooth: float = 1e-6) -> torch.Tensor:
    return sample_counts(predictions, targets, threshold, smooth)[1][:, 1].contiguous()


def _boundary_unavailable(*_a, **_k):
    raise NotImplementedError("boundary-F1 / Hausdorff (OpenCV contours, src/evaluate.py:102-275) are not "
                              "part of this build's hot path; train_epoch reports boundary_f1_score=0.0")


compute_boundary_f1 = _boundary_unavailable
compute_boundary_f1_batch = _boundary_unavailable
compute_hausdorff_distance = _boundary_unavailable
