"""Two-stage training of src/train.py on the MI355X path.

Public surface kept for drop-in: ``EarlyStopping`` (src/train.py:32-81),
``train_epoch`` (:84-185), ``validate`` (:188-286), ``train_stage``
(:289-391), ``save_metrics_to_csv`` (:394-433), ``save_test_metrics``
(:436-508), ``create_subset_dataset`` (:511-528) and ``train`` (:531-915),
with the same result keys, CSV columns and defaults.

What changes underneath:
  * the step is UNet engine fwd -> fused loss -> engine bwd -> flat AdamW,
    all HIP kernels; per-term losses and per-sample Dice/IoU counters come out
    of the one fused loss launch instead of a second logging recompute;
  * accumulators stay on the device; the host synchronises once per epoch
    (the reference calls ``.item()``/``.cpu()`` several times per step);
  * optional data-parallel training (torchrun, RCCL), see ``distributed``.
Boundary-F1 needs OpenCV (absent here) and is outside this path: it is
reported as 0.0, the value the reference reports when it has no scores.
"""
from __future__ import annotations

import csv
import json
import os
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Subset

from . import _hip
from .dataset import CellSegmentationDataset, DeviceDiscLoader, SyntheticDiscDataset
from .distributed import GradBucketer, allreduce_scalars, broadcast_parameters, init_from_env
from .fused import LossConfig, loss_forward
from .loss import DiceBCELoss, DiceBCEPDELoss
from .optim import AdamW
from .unet import UNet

CSV_FIELDS = ["epoch", "train_loss", "train_dice_loss", "train_bce_loss", "train_pde_loss",
              "train_phase_field_loss", "train_dice_score", "train_iou_score", "train_boundary_f1_score",
              "val_loss", "val_dice_score", "val_dice_loss", "val_bce_loss", "val_pde_loss",
              "val_phase_field_loss", "val_iou_score", "val_boundary_f1_score"]


class EarlyStopping:
    """Stop after ``patience`` epochs without a > min_delta improvement."""

    def __init__(self, patience: int = 10, min_delta: float = 1e-4, mode: str = "max"):
        self.patience, self.min_delta, self.mode = patience, min_delta, mode
        self.counter = 0
        self.best_score = None
        self.best_epoch = 0
        self.early_stop = False

    def _better(self, score: float) -> bool:
        if self.mode == "max":
            return score > self.best_score + self.min_delta
        return score < self.best_score - self.min_delta

    def __call__(self, score: float, epoch: int) -> bool:
        if self.best_score is None:
            self.best_score, self.best_epoch = score, epoch
            return False
        if self._better(score):
            self.best_score, self.best_epoch, self.counter = score, epoch, 0
        else:
            self.counter += 1
            if self.counter >= self.patience:
                self.early_stop = True
        return self.early_stop


# ----------------------------------------------------------------------------
# step-loop accounting (device side)
# ----------------------------------------------------------------------------

def _criterion_terms(criterion, outputs, masks):
    """Per-term values of the last criterion call: from the fused launch when the
    criterion is ours, otherwise one extra fused forward on its attributes."""
    last = getattr(criterion, "last", None)
    if last and "terms" in last:
        return last["terms"], last["scores"]
    is_pde = isinstance(criterion, DiceBCEPDELoss)
    cfg = LossConfig(dice_w=getattr(criterion, "dice_weight", 0.5), bce_w=getattr(criterion, "bce_weight", 0.5),
                     rd_w=criterion.pde_weight if is_pde else 0.0,
                     pf_w=criterion.phase_field_weight if is_pde else 0.0,
                     smooth=getattr(criterion, "smooth", 1e-6),
                     D=criterion.pde_regularization.diffusion_coeff if is_pde else 1.0,
                     a=criterion.pde_regularization.reaction_threshold if is_pde else 0.5,
                     eps=criterion.epsilon if is_pde else 0.05)
    terms, _, scores = loss_forward(outputs.detach(), masks, cfg)
    return terms, scores


class _Meter:
    """Device accumulators: sums of (loss, dice, bce, rd, pf) per batch, of
    per-sample (dice, iou), of whole-batch thresholded dice; counts."""

    def __init__(self, device):
        self.terms = torch.zeros(5, dtype=torch.float64, device=device)
        self.scores = torch.zeros(2, dtype=torch.float64, device=device)
        self.batch_dice = torch.zeros(1, dtype=torch.float64, device=device)
        self.bf1 = torch.zeros(1, dtype=torch.float64, device=device)  # host-computed boundary F1 sums
        self.batches = 0
        self.samples = 0

    def add(self, terms, scores, batch_dice=None):
        self.terms += terms[:5].double()
        if scores is not None:
            self.scores += scores.double().sum(dim=0)
            self.samples += scores.shape[0]
        if batch_dice is not None:
            self.batch_dice += batch_dice.double()
        self.batches += 1

    def reduce(self) -> Tuple[List[float], List[float], float, int, int]:
        packed = torch.cat([self.terms, self.scores, self.batch_dice, self.bf1,
                            torch.tensor([self.batches, self.samples], dtype=torch.float64,
                                         device=self.terms.device)])
        packed = allreduce_scalars(packed)
        vals = packed.tolist()  # the epoch's single host synchronisation
        self.bf1_total = vals[8]
        return vals[0:5], vals[5:7], vals[7], int(vals[9]), int(vals[10])


def _results(meter: _Meter, criterion, return_components: bool, compute_metrics: bool, val: bool):
    terms, scores, batch_dice, nb, ns = meter.reduce()
    nb = max(nb, 1)
    out: Dict[str, float] = {"loss": terms[0] / nb}
    if val:
        out["dice_score"] = batch_dice / nb
    if return_components:
        out["dice_loss"] = terms[1] / nb
        out["bce_loss"] = terms[2] / nb
        if isinstance(criterion, DiceBCEPDELoss):
            if criterion.pde_weight > 0:
                out["pde_loss"] = terms[3] / nb
            if criterion.phase_field_weight > 0:
                out["phase_field_loss"] = terms[4] / nb
    if compute_metrics:
        if not val:
            out["dice_score"] = scores[0] / ns if ns else 0.0
        out["iou_score"] = scores[1] / ns if ns else 0.0
        # 0.0 unless boundary_metrics=True (host-side, off the hot path): the reference's value
        # without scores
        out["boundary_f1_score"] = meter.bf1_total / ns if ns else 0.0
    return out


def _boundary_sum(outputs, masks) -> float:
    from .evaluate import compute_boundary_f1_batch
    return float(compute_boundary_f1_batch(outputs, masks, threshold=0.5, tolerance=2).sum())


def train_epoch(model, dataloader, criterion, optimizer, device, return_components: bool = False,
                compute_metrics: bool = True, boundary_metrics: bool = False) -> Dict[str, float]:
    """One pass over ``dataloader`` (src/train.py:84-185); same result keys. The reference
    computes boundary F1 on the host every step (src/train.py:152-160); here that is opt-in
    (``boundary_metrics``, cv2-free, evaluate.py) so the step stays device-only."""
    model.train()
    meter = _Meter(device)
    for images, masks in dataloader:
        images = images.to(device, non_blocking=True)
        masks = masks.to(device, non_blocking=True)
        optimizer.zero_grad()
        outputs = model(images)
        loss = criterion(outputs, masks)
        terms, scores = _criterion_terms(criterion, outputs, masks)
        meter.add(terms, scores if compute_metrics else None)
        if compute_metrics and boundary_metrics:
            meter.bf1 += _boundary_sum(outputs, masks)
        loss.backward()
        optimizer.step()
    return _results(meter, criterion, return_components, compute_metrics, val=False)


@torch.no_grad()
def validate(model, dataloader, criterion, device, return_components: bool = False,
             compute_metrics: bool = True, boundary_metrics: bool = False) -> Dict[str, float]:
    """Eval-mode pass (src/train.py:188-286); ``dice_score`` is the mean of
    whole-batch thresholded Dice, as in the reference."""
    model.eval()
    meter = _Meter(device)
    for images, masks in dataloader:
        images = images.to(device, non_blocking=True)
        masks = masks.to(device, non_blocking=True)
        outputs = model(images)
        criterion(outputs, masks)
        terms, scores = _criterion_terms(criterion, outputs, masks)
        last = getattr(criterion, "last", {})
        counts = last.get("counts")
        if counts is None:
            _, counts, _ = loss_forward(outputs, masks, LossConfig(dice_w=0.0, bce_w=0.0))
        tot = counts.sum(dim=0).to(torch.float32)
        s = criterion.smooth if hasattr(criterion, "smooth") else 1e-6
        batch_dice = (2.0 * tot[0] + 1e-6) / (tot[1] + tot[2] + 1e-6)
        meter.add(terms, scores if compute_metrics else None, batch_dice)
        if compute_metrics and boundary_metrics:
            meter.bf1 += _boundary_sum(outputs, masks)
    return _results(meter, criterion, return_components, compute_metrics, val=True)


def train_stage(model, train_loader, val_loader, criterion, optimizer, device, num_epochs: int,
                stage_name: str, early_stopping: Optional[EarlyStopping] = None, verbose: bool = True,
                csv_path: Optional[Path] = None) -> Tuple[Dict, int, List[Dict]]:
    """Epoch loop with best-val-Dice tracking, CSV and early stopping (src/train.py:289-391)."""
    best_dice, best_epoch, best = 0.0, 0, {}
    history: List[Dict] = []
    is_main = not (torch.distributed.is_available() and torch.distributed.is_initialized()) or \
        torch.distributed.get_rank() == 0
    for epoch in range(1, num_epochs + 1):
        sampler = getattr(train_loader, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        tr = train_epoch(model, train_loader, criterion, optimizer, device, return_components=True,
                         compute_metrics=True)
        va = validate(model, val_loader, criterion, device, return_components=True, compute_metrics=True)
        if va["dice_score"] > best_dice:
            best_dice, best_epoch, best = va["dice_score"], epoch, {"train": tr, "val": va}
        row = {"epoch": epoch}
        for k in CSV_FIELDS[1:]:
            side, key = k.split("_", 1)
            src = tr if side == "train" else va
            row[k] = src[key] if key in ("loss", "dice_score") and key in src else src.get(key, 0.0)
        history.append(row)
        if csv_path is not None and is_main:
            save_metrics_to_csv(history, csv_path)
        if verbose and is_main:
            print(f"\n{stage_name} - Epoch {epoch}/{num_epochs}")
            print(f"  Train Loss: {tr['loss']:.6f}")
            for key, label in (("dice_loss", "Dice Loss"), ("bce_loss", "BCE Loss"), ("pde_loss", "PDE Loss")):
                if key in tr:
                    print(f"    - {label}: {tr[key]:.6f}")
            print(f"  Val Loss: {va['loss']:.6f}")
            print(f"  Val Dice Score: {va['dice_score']:.6f}")
            for key, label in (("dice_loss", "Dice Loss"), ("bce_loss", "BCE Loss"), ("pde_loss", "PDE Loss")):
                if key in va:
                    print(f"    - {label}: {va[key]:.6f}")
        if early_stopping is not None and early_stopping(va["dice_score"], epoch):
            if verbose and is_main:
                print(f"\nEarly stopping triggered at epoch {epoch}")
                print(f"Best validation Dice score: {best_dice:.6f} at epoch {best_epoch}")
            break
    return best, best_epoch, history


def save_metrics_to_csv(metrics: List[Dict], csv_path: Path):
    if not metrics:
        return
    csv_path = Path(csv_path)
    csv_path.parent.mkdir(parents=True, exist_ok=True)
    with open(csv_path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=CSV_FIELDS)
        w.writeheader()
        w.writerows(metrics)


def save_test_metrics(test_metrics: Dict[str, np.ndarray], output_path: Path, model_name: str = "Model"):
    """Per-image metrics -> JSON (with mean/std/count) + CSV (src/train.py:436-508)."""
    output_path = Path(output_path)
    output_path.parent.mkdir(parents=True, exist_ok=True)
    stats = {}
    for k, arr in test_metrics.items():
        a = np.asarray(arr, dtype=np.float64)
        fin = a[np.isfinite(a)]
        stats[k] = {"mean": float(fin.mean()) if fin.size else float("nan"),
                    "std": float(fin.std(ddof=1)) if fin.size > 1 else 0.0, "count": int(fin.size)}
    with open(output_path.with_suffix(".json"), "w") as f:
        json.dump({"model_name": model_name, "statistics": stats,
                   "per_image_metrics": {k: np.asarray(v).tolist() for k, v in test_metrics.items()}}, f, indent=2)
    n = max(len(v) for v in test_metrics.values())
    with open(output_path.with_suffix(".csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(test_metrics))
        w.writeheader()
        for i in range(n):
            row = {}
            for k, v in test_metrics.items():
                val = float(v[i]) if i < len(v) else float("nan")
                row[k] = val if np.isfinite(val) else ""
            w.writerow(row)
    print("Test metrics saved to:")
    print(f"  CSV: {output_path.with_suffix('.csv')}")
    print(f"  JSON: {output_path.with_suffix('.json')}")


def create_subset_dataset(dataset, fraction: float) -> Subset:
    """Random ``fraction`` of the dataset drawn with numpy's global RNG (src/train.py:511-528)."""
    total = len(dataset)
    idx = np.random.choice(total, int(total * fraction), replace=False)
    return Subset(dataset, idx)


def _loaders(train_ds, val_ds, batch_size: int, world: int, rank: int, workers: int):
    pin = torch.cuda.is_available()
    if world > 1:
        from torch.utils.data.distributed import DistributedSampler
        ts = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True)
        vs = DistributedSampler(val_ds, num_replicas=world, rank=rank, shuffle=False)
        return (DataLoader(train_ds, batch_size=batch_size, sampler=ts, num_workers=workers, pin_memory=pin),
                DataLoader(val_ds, batch_size=batch_size, sampler=vs, num_workers=workers, pin_memory=pin))
    return (DataLoader(train_ds, batch_size=batch_size, shuffle=True, num_workers=workers, pin_memory=pin),
            DataLoader(val_ds, batch_size=batch_size, shuffle=False, num_workers=workers, pin_memory=pin))


def train(use_two_stage: bool = True, pde_weight: float = 1e-4, diffusion_coeff: float = 5.0,
          reaction_threshold: float = 0.5, phase_field_weight: float = 1e-4, epsilon: float = 0.05,
          batch_size: int = 8, learning_rate: float = 1e-4, stage1_epochs: int = 50, stage2_epochs: int = 50,
          early_stopping_patience: int = 10, train_fraction: Optional[float] = None, seed: int = 42,
          base_dir: Optional[str] = None, synthetic: Optional[Tuple[int, int, int, int]] = None,
          num_workers: int = 2, device_data: bool = True):
    """Two-stage training (src/train.py:531-915). Extra, build-only arguments:
    ``base_dir`` (where images/, output/, models/ live; default: cwd) and
    ``synthetic=(n_train, n_val, H, W)`` to train on the SURVEY §8(c) disc
    generator when the cell dataset is not present — rasterised on the GPU
    (``DeviceDiscLoader``, sharded like DistributedSampler) unless ``device_data=False``."""
    rank, local_rank, world = init_from_env()
    if not torch.cuda.is_available():
        raise _hip.HipError("train(): the MI355X path needs a GPU (no CPU fallback in this build)")
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    torch.manual_seed(seed)
    np.random.seed(seed)
    torch.cuda.manual_seed(seed)
    is_main = rank == 0

    base = Path(base_dir) if base_dir else Path.cwd()
    img_dir, out_dir = base / "images", base / "output"
    ann_dir = img_dir / "annotation"
    out_dir.mkdir(exist_ok=True)
    stamp = datetime.now().strftime("%Y%m%d_%H%M%S")
    say = print if is_main else (lambda *a, **k: None)
    say("=" * 70)
    say("PDE-CONSTRAINED CELL SEGMENTATION TRAINING (MI355X)")
    say("=" * 70)
    say(f"Device: {device} x {world}")
    say(f"Training strategy: {'Two-stage' if use_two_stage else 'Single-stage (PDE from start)'}")

    if synthetic is not None:
        n_tr, n_va, H, W = synthetic
        train_ds = SyntheticDiscDataset(n_tr, (H, W), seed=seed)
        val_ds = SyntheticDiscDataset(n_va, (H, W), seed=seed + 1)
    else:
        train_ds = CellSegmentationDataset(img_dir / "training", ann_dir / "training_annotation.json")
        val_ds = CellSegmentationDataset(img_dir / "validation", ann_dir / "validation_annotation.json")
    if train_fraction is not None:
        say(f"Using {train_fraction * 100:.1f}% of training data ({int(len(train_ds) * train_fraction)} samples)")
        train_ds = create_subset_dataset(train_ds, train_fraction)
    frac = f"_frac{train_fraction:.2f}" if train_fraction is not None else ""
    if synthetic is not None and device_data:
        subset = train_ds.indices if isinstance(train_ds, Subset) else None
        train_loader = DeviceDiscLoader(n_tr, batch_size, (H, W), seed=seed, shuffle=True, rank=rank, world=world,
                                        device=device, subset=subset)
        val_loader = DeviceDiscLoader(n_va, batch_size, (H, W), seed=seed + 1, shuffle=False, rank=rank,
                                      world=world, device=device)
    else:
        train_loader, val_loader = _loaders(train_ds, val_ds, batch_size, world, rank, num_workers)
    say(f"Training samples: {len(train_ds)}")
    say(f"Validation samples: {len(val_ds)}")
    say(f"Batch size: {batch_size} per GPU")

    model = UNet(in_channels=1, out_channels=1, base_channels=64).to(device)
    broadcast_parameters(model)
    if world > 1:
        GradBucketer(model)
    grad_scale = 1.0 / world

    def run(criterion, lr, epochs, name, csv_path):
        opt = AdamW(model.parameters(), lr=lr, weight_decay=1e-5, grad_scale=grad_scale)
        stopper = EarlyStopping(patience=early_stopping_patience, min_delta=1e-4, mode="max")
        return train_stage(model, train_loader, val_loader, criterion, opt, device, num_epochs=epochs,
                           stage_name=name, early_stopping=stopper, verbose=True, csv_path=csv_path)

    def pde_loss():
        return DiceBCEPDELoss(dice_weight=0.5, bce_weight=0.5, pde_weight=pde_weight,
                              phase_field_weight=phase_field_weight, diffusion_coeff=diffusion_coeff,
                              reaction_threshold=reaction_threshold, epsilon=epsilon).to(device)

    models_dir = base / "models"
    result = {}
    if use_two_stage:
        say("\n" + "=" * 70 + "\nSTAGE I: BASELINE TRAINING (Unconstrained)\n" + "=" * 70)
        csv1 = out_dir / f"metrics_stage1_{stamp}{frac}.csv"
        best1, ep1, hist1 = run(DiceBCELoss(0.5, 0.5).to(device), learning_rate, stage1_epochs, "Stage I", csv1)
        result["stage1"] = (best1, ep1, hist1)
        if is_main:
            models_dir.mkdir(exist_ok=True)
            torch.save(model.state_dict(), models_dir / "unet_baseline.pth")
        say("\n" + "=" * 70 + "\nSTAGE II: PDE-CONSTRAINED FINE-TUNING\n" + "=" * 70)
        lr2 = learning_rate * 0.1  # src/train.py:720
        say(f"  Learning rate for Stage II: {lr2:.2e} (reduced from {learning_rate:.2e})")
        csv2 = out_dir / f"metrics_stage2_{stamp}{frac}.csv"
        best2, ep2, hist2 = run(pde_loss(), lr2, stage2_epochs, "Stage II", csv2)
        result["stage2"] = (best2, ep2, hist2)
        if best2 and "val" in best2:
            say("\nStability checks:")
            for key in ("pde_loss", "dice_loss", "bce_loss"):
                if key in best2["val"]:
                    say(f"  Final {key}: {best2['val'][key]:.6f}")
            if best1 and "val" in best1:
                say(f"  Dice score improvement: {best2['val']['dice_score'] - best1['val']['dice_score']:+.6f}")
        if is_main:
            torch.save(model.state_dict(), models_dir / "unet_pde_regularized.pth")
    else:
        say("\n" + "=" * 70 + "\nSINGLE-STAGE TRAINING (PDE from start)\n" + "=" * 70)
        csv1 = out_dir / f"metrics_single_stage_{stamp}{frac}.csv"
        best, ep, hist = run(pde_loss(), learning_rate, stage1_epochs, "Training", csv1)
        result["single"] = (best, ep, hist)
        if is_main:
            models_dir.mkdir(exist_ok=True)
            torch.save(model.state_dict(), models_dir / "unet_pde_regularized.pth")
    say("\n" + "=" * 70 + "\nTRAINING COMPLETE\n" + "=" * 70)
    return model, result
