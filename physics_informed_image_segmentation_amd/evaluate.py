"""Evaluation metrics of src/evaluate.py on this build.

* IoU (src/evaluate.py:26-97) is on the hot path (every step, src/train.py:155) and comes
  from the fused loss kernel's exact per-sample counters, like Dice.
* Boundary-F1 and Hausdorff (src/evaluate.py:102-275) are host-side in the reference
  (OpenCV contours + distance transform, scipy Hausdorff). OpenCV is not installed here, so
  they are restated with scipy.ndimage:
    - ``extract_boundaries`` (src/evaluate.py:102-120: cv2.findContours(RETR_EXTERNAL,
      CHAIN_APPROX_NONE) + drawContours(thickness 1)) = the foreground pixels 4-adjacent to
      the OUTER background, i.e. the background component (4-connected, the dual of
      OpenCV's 8-connected foreground) that touches a zero frame around the image. Borders
      of holes and components nested inside holes are not outer contours, as with
      RETR_EXTERNAL.
    - the tolerance test ``distanceTransform(DIST_L2, 5) <= 2`` (:150-175) equals a
      Euclidean-disk test for radius 2 (the 5x5 chamfer gives 1, 1.4, 2 at offsets (1,0),
      (1,1), (2,0) and 2.1969 > 2 at (2,1), exactly where dx^2 + dy^2 <= 4 holds).
    - Hausdorff = scipy's directed_hausdorff both ways on the boundary coordinates (:232-275).
  Parity for these two is unpinned against OpenCV itself (absent); tests/test_host.py pins
  them on hand-drawn shapes with known contours.
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
from scipy import ndimage
from scipy.spatial.distance import directed_hausdorff

from .metrics import compute_dice_score_batch, sample_counts

_FOUR = ndimage.generate_binary_structure(2, 1)
_DISK2 = np.array([[dy * dy + dx * dx <= 4 for dx in range(-2, 3)] for dy in range(-2, 3)])


def compute_iou(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                smooth: float = 1e-6) -> torch.Tensor:
    counts, _ = sample_counts(predictions, targets, threshold, smooth)
    tot = counts.sum(dim=0).to(torch.float32)
    return (tot[0] + smooth) / (tot[1] + tot[2] - tot[0] + smooth)


def compute_iou_batch(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                      smooth: float = 1e-6) -> torch.Tensor:
    return sample_counts(predictions, targets, threshold, smooth)[1][:, 1].contiguous()


def _dilate4(x: np.ndarray, iterations: int = 1) -> np.ndarray:
    """Binary dilation by the 4-neighbour cross (= ndimage.binary_dilation(x, _FOUR)), as
    shifted ORs; two iterations give the Euclidean disk of radius 2 (|dx| + |dy| <= 2 and
    dx^2 + dy^2 <= 4 select the same 13 offsets)."""
    for _ in range(iterations):
        y = x.copy()
        y[1:] |= x[:-1]
        y[:-1] |= x[1:]
        y[:, 1:] |= x[:, :-1]
        y[:, :-1] |= x[:, 1:]
        x = y
    return x


def extract_boundaries(mask: np.ndarray) -> np.ndarray:
    """Outer-contour pixels of a binary (H, W) mask as float32 {0, 1} (src/evaluate.py:102-120)."""
    fg = np.asarray(mask) > 0
    if not fg.any():
        return np.zeros(fg.shape, np.float32)
    pad = np.pad(fg, 1, constant_values=False)
    lab, _ = ndimage.label(~pad, structure=_FOUR)
    outer = lab == lab[0, 0]  # the frame is background and connected to itself
    return (pad & _dilate4(outer))[1:-1, 1:-1].astype(np.float32)


def _near(b: np.ndarray, tolerance: int) -> np.ndarray:
    """Pixels within Euclidean distance ``tolerance`` of a boundary pixel."""
    if tolerance <= 2:
        return _dilate4(b, tolerance)
    disk = np.array([[dy * dy + dx * dx <= tolerance * tolerance for dx in range(-tolerance, tolerance + 1)]
                     for dy in range(-tolerance, tolerance + 1)])
    return ndimage.binary_dilation(b, structure=disk)


def _binary_np(x: torch.Tensor, threshold: float = None) -> np.ndarray:
    a = x.detach().reshape(x.shape[-2], x.shape[-1])
    if threshold is not None:
        a = a > threshold
    return a.cpu().numpy().astype(np.float32)


def _boundary_f1_np(pred_b: np.ndarray, target_b: np.ndarray, tolerance: int, smooth: float) -> float:
    if tolerance > 0:
        near_t = _near(target_b > 0, tolerance)
        near_p = _near(pred_b > 0, tolerance)
        precision = ((near_t * pred_b).sum() + smooth) / (pred_b.sum() + smooth)
        recall = ((near_p * target_b).sum() + smooth) / (target_b.sum() + smooth)
        return float((2.0 * precision * recall + smooth) / (precision + recall + smooth))
    inter = (pred_b * target_b).sum()
    return float((2.0 * inter + smooth) / (pred_b.sum() + target_b.sum() + smooth))


def compute_boundary_f1(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                        tolerance: int = 2, smooth: float = 1e-6) -> torch.Tensor:
    """Boundary F1 of the first sample within ``tolerance`` pixels (src/evaluate.py:123-182)."""
    pb = extract_boundaries(_binary_np(predictions[0, 0], threshold))
    tb = extract_boundaries(_binary_np(targets[0, 0]))
    return torch.tensor(_boundary_f1_np(pb, tb, tolerance, smooth), dtype=torch.float32)


def compute_boundary_f1_batch(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5,
                              tolerance: int = 2, smooth: float = 1e-6) -> torch.Tensor:
    """Per-sample boundary F1 (src/evaluate.py:185-215); one device->host copy per batch."""
    p = (predictions.detach() > threshold).reshape(predictions.shape[0], *predictions.shape[-2:]).cpu().numpy()
    t = targets.detach().reshape(targets.shape[0], *targets.shape[-2:]).cpu().numpy()
    return torch.tensor([_boundary_f1_np(extract_boundaries(p[i]), extract_boundaries(t[i]), tolerance, smooth)
                         for i in range(p.shape[0])], dtype=torch.float32)


def compute_hausdorff_distance(predictions: torch.Tensor, targets: torch.Tensor, threshold: float = 0.5) -> float:
    """Symmetric Hausdorff distance of the first sample's boundaries; inf when one is
    empty (src/evaluate.py:218-275)."""
    pc = np.column_stack(np.where(extract_boundaries(_binary_np(predictions[0, 0], threshold)) > 0))
    tc = np.column_stack(np.where(extract_boundaries(_binary_np(targets[0, 0])) > 0))
    if len(pc) == 0 or len(tc) == 0:
        return float("inf")
    return float(max(directed_hausdorff(pc, tc)[0], directed_hausdorff(tc, pc)[0]))


@torch.no_grad()
def evaluate_model(model, dataloader, device, threshold: float = 0.5,
                   boundary_metrics: bool = True) -> Dict[str, np.ndarray]:
    """Per-image Dice / IoU (fused counters on the GPU) and boundary F1 / Hausdorff (host)
    over a loader (src/evaluate.py:279-350)."""
    model.eval()
    dice, iou, bf1, hd = [], [], [], []
    for images, masks in dataloader:
        images, masks = images.to(device, non_blocking=True), masks.to(device, non_blocking=True)
        outputs = model(images)
        _, scores = sample_counts(outputs, masks, threshold)
        s = scores.cpu().numpy()
        dice.extend(s[:, 0].tolist())
        iou.extend(s[:, 1].tolist())
        if boundary_metrics:
            bf1.extend(compute_boundary_f1_batch(outputs, masks, threshold=threshold, tolerance=2).tolist())
            for i in range(outputs.shape[0]):
                h = compute_hausdorff_distance(outputs[i:i + 1], masks[i:i + 1], threshold=threshold)
                hd.append(h if np.isfinite(h) else np.nan)
    out = {"dice_scores": np.array(dice), "iou_scores": np.array(iou)}
    if boundary_metrics:
        out["boundary_f1_scores"] = np.array(bf1)
        out["hausdorff_distances"] = np.array(hd)
    return out


# ----------------------------------------------------------------------------
# Statistics and test-set evaluation (src/evaluate.py:349-523) — host-side, after training
# ----------------------------------------------------------------------------

def compute_statistics(metric_array: np.ndarray) -> Dict[str, float]:
    """Mean, sample std (ddof=1) and count over the non-NaN entries (src/evaluate.py:349-369)."""
    a = np.asarray(metric_array, dtype=np.float64)
    a = a[~np.isnan(a)]
    if a.size == 0:
        return {"mean": np.nan, "std": np.nan, "count": 0}
    return {"mean": float(a.mean()), "std": float(a.std(ddof=1)), "count": int(a.size)}


_NO_TEST = {"t_statistic": np.nan, "t_pvalue": np.nan, "wilcoxon_statistic": np.nan,
            "wilcoxon_pvalue": np.nan, "significant": False}


def compare_models_statistically(metrics_baseline: Dict[str, np.ndarray], metrics_pde: Dict[str, np.ndarray],
                                 alpha: float = 0.05) -> Dict[str, Dict[str, float]]:
    """Paired t-test + two-sided Wilcoxon signed-rank per metric over the images where both
    models have a value; significant if either p < alpha (src/evaluate.py:372-438)."""
    from scipy import stats
    out = {}
    for name, base in metrics_baseline.items():
        b = np.asarray(base, dtype=np.float64)
        p = np.asarray(metrics_pde[name], dtype=np.float64)
        keep = ~(np.isnan(b) | np.isnan(p))
        b, p = b[keep], p[keep]
        if b.size < 2:
            out[name] = dict(_NO_TEST)
            continue
        t_stat, t_p = stats.ttest_rel(b, p)
        w_stat, w_p = stats.wilcoxon(b, p, alternative="two-sided")
        sb, sp = compute_statistics(b), compute_statistics(p)
        out[name] = {"t_statistic": float(t_stat), "t_pvalue": float(t_p), "wilcoxon_statistic": float(w_stat),
                     "wilcoxon_pvalue": float(w_p), "significant": bool(t_p < alpha or w_p < alpha),
                     "baseline_mean": sb["mean"], "baseline_std": sb["std"], "pde_mean": sp["mean"],
                     "pde_std": sp["std"], "improvement": float(p.mean() - b.mean())}
    return out


def format_metric_report(metrics: Dict[str, np.ndarray], model_name: str = "Model") -> str:
    """'<Metric Title>: mean ± std (n=count)' lines (src/evaluate.py:441-472)."""
    lines = [f"\n{model_name} Performance:", "=" * 60]
    for name, arr in metrics.items():
        st = compute_statistics(arr)
        title = name.replace("_", " ").title()
        lines.append(f"{title}: {st['mean']:.4f} ± {st['std']:.4f} (n={st['count']})" if st["count"] > 0
                     else f"{title}: N/A")
    return "\n".join(lines)


def evaluate_on_test_set(model, test_dir, test_json, device, batch_size: int = 8, threshold: float = 0.5,
                         model_name: str = "Model") -> Dict[str, np.ndarray]:
    """Per-image metrics of ``model`` on a COCO-annotated test folder (src/evaluate.py:476-522)."""
    from torch.utils.data import DataLoader

    from .dataset import CellSegmentationDataset
    print(f"\nEvaluating {model_name} on test set...")
    print("=" * 70)
    ds = CellSegmentationDataset(test_dir, test_json)
    loader = DataLoader(ds, batch_size=batch_size, shuffle=False, num_workers=2,
                        pin_memory=torch.cuda.is_available())
    print(f"Test samples: {len(ds)}")
    metrics = evaluate_model(model, loader, device, threshold=threshold)
    print(format_metric_report(metrics, model_name=model_name))
    return metrics


__all__ = ["compute_iou", "compute_iou_batch", "extract_boundaries", "compute_boundary_f1",
           "compute_boundary_f1_batch", "compute_hausdorff_distance", "evaluate_model",
           "compute_dice_score_batch", "compute_statistics", "compare_models_statistically",
           "format_metric_report", "evaluate_on_test_set"]
