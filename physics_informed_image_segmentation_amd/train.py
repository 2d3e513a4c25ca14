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
  * optional data-parallel training (torchrun, RCCL), see ``distributed``;
  * boundary F1 (OpenCV in the reference, a cv2-free restatement here) is
    scored on host threads beside the GPU, not inside the step.
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

def _forward_loss(model, images, masks, criterion):
    """``outputs = model(images); loss = criterion(outputs, masks)`` (src/train.py:108-110,
    :216-218): this package's U-Net runs its head fused with the loss forward
    (UNet.forward_with_loss); any other model takes the two calls."""
    fwd = getattr(model, "forward_with_loss", None)
    if fwd is not None:
        return fwd(images, masks, criterion)
    outputs = model(images)
    return outputs, criterion(outputs, masks)


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
        # host threads beside the GPU (_BoundaryF1Async); 0.0 with boundary_metrics=False
        out["boundary_f1_score"] = meter.bf1_total / ns if ns else 0.0
    return out


class _BoundaryF1Async:
    """Per-sample boundary F1 of every step (src/train.py:156,259), off the critical path: the
    step's probabilities and masks are copied to pinned host memory on a copy stream (ordered
    after the forward by an event) and scored by host threads (cv2-free ``evaluate``
    restatement, scipy releases the GIL) while the GPU runs the backward and the next steps.
    The only GPU-side cost is one stream wait before the next forward, so the engine's
    probability buffer is not overwritten before its copy has landed."""

    def __init__(self, device, workers: Optional[int] = None):
        from concurrent.futures import ThreadPoolExecutor
        n = workers or max(1, min(8, len(os.sched_getaffinity(0)) - 1))
        self.pool = ThreadPoolExecutor(max_workers=n)
        # backpressure: at most this many steps in flight; beyond it the oldest is waited for and
        # folded into the running sum (bounded pinned memory when scoring is slower than the GPU)
        self.max_inflight = 2 * n
        self.total = 0.0
        self.cuda = torch.device(device).type == "cuda"  # host tensors (tests): no streams
        self.copy = torch.cuda.Stream(device=device) if self.cuda else None
        self.fence: Optional[torch.cuda.Event] = None
        self.futures = []
        self.free = []  # pinned host buffers ready for reuse

    def before_forward(self):
        if self.cuda and self.fence is not None:
            torch.cuda.current_stream().wait_event(self.fence)
            self.fence = None

    def _pinned(self, shape):
        for i, (p, t) in enumerate(self.free):
            if p.shape == shape:
                return self.free.pop(i)
        return (torch.empty(shape, dtype=torch.float32, pin_memory=True),
                torch.empty(shape, dtype=torch.float32, pin_memory=True))

    def _drain(self, keep: int) -> None:
        while len(self.futures) > keep:
            self.total += self.futures.pop(0).result()[0]

    def submit(self, outputs: torch.Tensor, masks: torch.Tensor):
        self._drain(self.max_inflight - 1)
        B, H, W = outputs.shape[0], outputs.shape[-2], outputs.shape[-1]
        if not self.cuda:
            hp = outputs.detach().reshape(B, H, W).float().clone()
            ht = masks.detach().reshape(B, H, W).float().clone()
            self.futures.append(self.pool.submit(self._score, None, hp, ht))
            return
        hp, ht = self._pinned((B, H, W))
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream())
        self.copy.wait_event(ready)
        with torch.cuda.stream(self.copy):
            hp.copy_(outputs.detach().reshape(B, H, W), non_blocking=True)
            ht.copy_(masks.detach().reshape(B, H, W), non_blocking=True)
            masks.record_stream(self.copy)
            done = torch.cuda.Event()
            done.record(self.copy)
        self.fence = done
        self.futures.append(self.pool.submit(self._score, done, hp, ht))

    def _score(self, done, hp, ht) -> Tuple[float, int]:
        from .evaluate import _boundary_f1_np, extract_boundaries
        if done is not None:
            done.synchronize()
        p, t = hp.numpy() > 0.5, ht.numpy()
        tot = sum(_boundary_f1_np(extract_boundaries(p[i]), extract_boundaries(t[i]), 2, 1e-6)
                  for i in range(p.shape[0]))
        if done is not None:
            self.free.append((hp, ht))
        return tot, p.shape[0]

    def collect(self) -> float:
        """Sum of the per-sample scores submitted so far (waits for the host threads)."""
        self._drain(0)
        tot, self.total = self.total, 0.0
        return tot

    def close(self):
        self.pool.shutdown(wait=True)


def train_epoch(model, dataloader, criterion, optimizer, device, return_components: bool = False,
                compute_metrics: bool = True, boundary_metrics: bool = True) -> Dict[str, float]:
    """One pass over ``dataloader`` (src/train.py:84-185); same result keys and averaging:
    loss terms averaged over batches, Dice / IoU / boundary F1 over samples. Boundary F1
    (src/train.py:156) is scored on host threads beside the GPU (``_BoundaryF1Async``);
    ``boundary_metrics=False`` reports 0.0 instead."""
    model.train()
    meter = _Meter(device)
    bf1 = _BoundaryF1Async(device) if compute_metrics and boundary_metrics else None
    try:
        for images, masks in dataloader:
            images = images.to(device, non_blocking=True)
            masks = masks.to(device, non_blocking=True)
            optimizer.zero_grad()
            if bf1 is not None:
                bf1.before_forward()
            outputs, loss = _forward_loss(model, images, masks, criterion)
            terms, scores = _criterion_terms(criterion, outputs, masks)
            meter.add(terms, scores if compute_metrics else None)
            if bf1 is not None:
                bf1.submit(outputs, masks)
            loss.backward()
            optimizer.step()
        if bf1 is not None:
            meter.bf1 += bf1.collect()
    finally:
        if bf1 is not None:
            bf1.close()
    return _results(meter, criterion, return_components, compute_metrics, val=False)


@torch.no_grad()
def validate(model, dataloader, criterion, device, return_components: bool = False,
             compute_metrics: bool = True, boundary_metrics: bool = True) -> Dict[str, float]:
    """Eval-mode pass (src/train.py:188-286); ``dice_score`` is the mean of
    whole-batch thresholded Dice, as in the reference."""
    model.eval()
    meter = _Meter(device)
    bf1 = _BoundaryF1Async(device) if compute_metrics and boundary_metrics else None
    try:
        for images, masks in dataloader:
            images = images.to(device, non_blocking=True)
            masks = masks.to(device, non_blocking=True)
            if bf1 is not None:
                bf1.before_forward()
            outputs, _ = _forward_loss(model, images, masks, criterion)
            terms, scores = _criterion_terms(criterion, outputs, masks)
            last = getattr(criterion, "last", {})
            counts = last.get("counts")
            if counts is None:
                _, counts, _ = loss_forward(outputs, masks, LossConfig(dice_w=0.0, bce_w=0.0))
            tot = counts.sum(dim=0).to(torch.float32)
            batch_dice = (2.0 * tot[0] + 1e-6) / (tot[1] + tot[2] + 1e-6)  # src/metrics.py:4-35
            meter.add(terms, scores if compute_metrics else None, batch_dice)
            if bf1 is not None:
                bf1.submit(outputs, masks)
        if bf1 is not None:
            meter.bf1 += bf1.collect()
    finally:
        if bf1 is not None:
            bf1.close()
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
        # reshuffle per epoch like DataLoader(shuffle=True): DistributedSampler or DeviceDiscLoader
        for obj in (train_loader, getattr(train_loader, "sampler", None)):
            if hasattr(obj, "set_epoch"):
                obj.set_epoch(epoch)
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


_REPO_ROOT = Path(__file__).resolve().parent.parent


def train(use_two_stage: bool = True, pde_weight: float = 1e-4, diffusion_coeff: float = 5.0,
          reaction_threshold: float = 0.5, phase_field_weight: float = 1e-4, epsilon: float = 0.05,
          batch_size: int = 8, learning_rate: float = 1e-4, stage1_epochs: int = 50, stage2_epochs: int = 50,
          early_stopping_patience: int = 10, train_fraction: Optional[float] = None, seed: int = 42,
          base_dir: Optional[str] = None, synthetic: Optional[Tuple[int, int, int, int]] = None,
          num_workers: int = 2, device_data: bool = True):
    """Two-stage training (src/train.py:531-915), same control flow: Stage I (Dice+BCE) always
    runs and saves models/unet_baseline.pth; then either Stage II (PDE loss at lr x 0.1) ->
    unet_pde_regularized.pth, or, with ``use_two_stage=False``, a PDE-loss run at the full lr for
    ``stage1_epochs`` on top of the Stage-I weights (src/train.py:777-832); finally the test-set
    evaluation when images/testing and its annotation exist (src/train.py:848-911), writing
    test_metrics_stage{1,2}_* / test_metrics_single_stage_* (JSON + CSV). The training plots
    (src/plot.py) are not produced (out of scope).

    Extra, build-only arguments: ``base_dir`` (where images/, output/, models/ live; default:
    the repository root, like the reference's ``Path(__file__).parent.parent``),
    ``synthetic=(n_train, n_val, H, W)`` to train on the SURVEY §8(c) disc generator when the
    cell dataset is not present — rasterised on the GPU (``DeviceDiscLoader``, sharded like
    DistributedSampler) unless ``device_data=False``."""
    rank, local_rank, world = init_from_env()
    if not torch.cuda.is_available():
        raise _hip.HipError("train(): the MI355X path needs a GPU (no CPU fallback in this build)")
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    torch.manual_seed(seed)
    np.random.seed(seed)
    torch.cuda.manual_seed(seed)
    is_main = rank == 0

    base = Path(base_dir) if base_dir else _REPO_ROOT
    img_dir, out_dir = base / "images", base / "output"
    ann_dir = img_dir / "annotation"
    test_dir, test_json = img_dir / "testing", ann_dir / "testing_annotation.json"
    out_dir.mkdir(parents=True, exist_ok=True)
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
        # every replica starts from rank 0's weights; Dropout2d masks (the device RNG) differ per
        # rank, as its data shard does (rank 0 keeps the reference's seed)
        torch.cuda.manual_seed(seed + rank)
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

    def describe_pde():
        say("Objective: L = L_Dice + L_BCE + λ_RD * L_RD + λ_PF * L_PF")
        say(f"  λ_RD (reaction-diffusion): {pde_weight}")
        say(f"  λ_PF (phase-field): {phase_field_weight}")
        say(f"  Diffusion coefficient (D): {diffusion_coeff}")
        say(f"  Reaction threshold (a): {reaction_threshold}")
        if phase_field_weight > 0:
            say(f"  Phase-field epsilon (ε): {epsilon}")

    models_dir = base / "models"
    result = {}
    # ---- Stage I: always (src/train.py:651-691) ----
    say("\n" + "=" * 70 + "\nSTAGE I: BASELINE TRAINING (Unconstrained)\n" + "=" * 70)
    say("Objective: L = L_Dice + L_BCE")
    csv1 = out_dir / f"metrics_stage1_{stamp}{frac}.csv"
    best1, ep1, hist1 = run(DiceBCELoss(0.5, 0.5).to(device), learning_rate, stage1_epochs, "Stage I", csv1)
    result["stage1"] = (best1, ep1, hist1)
    if best1:
        say(f"\nStage I complete. Best validation Dice: {best1['val']['dice_score']:.6f} at epoch {ep1}")
    say(f"Stage I metrics saved to: {csv1}")
    stage1_path = models_dir / "unet_baseline.pth"
    if is_main:
        models_dir.mkdir(parents=True, exist_ok=True)
        torch.save(model.state_dict(), stage1_path)
    say(f"Stage I model saved to: {stage1_path}")
    if use_two_stage:
        say("\n" + "=" * 70 + "\nSTAGE II: PDE-CONSTRAINED FINE-TUNING\n" + "=" * 70)
        describe_pde()
        lr2 = learning_rate * 0.1  # src/train.py:720
        say(f"  Learning rate for Stage II: {lr2:.2e} (reduced from {learning_rate:.2e})")
        csv2 = out_dir / f"metrics_stage2_{stamp}{frac}.csv"
        best2, ep2, hist2 = run(pde_loss(), lr2, stage2_epochs, "Stage II", csv2)
        result["stage2"] = (best2, ep2, hist2)
        if best2 and "val" in best2:
            say(f"\nStage II complete. Best validation Dice: {best2['val']['dice_score']:.6f} at epoch {ep2}")
            say("\nStability checks:")
            for key, label in (("pde_loss", "PDE"), ("dice_loss", "Dice"), ("bce_loss", "BCE")):
                if key in best2["val"]:  # the reference raises KeyError when lambda_RD = 0
                    say(f"  Final {label} loss: {best2['val'][key]:.6f}")
            if best1 and "val" in best1:
                say("\nPDE regularization effect:")
                say(f"  Dice score improvement: {best2['val']['dice_score'] - best1['val']['dice_score']:+.6f}")
        say(f"Stage II metrics saved to: {csv2}")
        final_path = models_dir / "unet_pde_regularized.pth"
    else:
        say("\n" + "=" * 70 + "\nSINGLE-STAGE TRAINING (PDE from start)\n" + "=" * 70)
        describe_pde()
        csv1s = out_dir / f"metrics_single_stage_{stamp}{frac}.csv"
        best, ep, hist = run(pde_loss(), learning_rate, stage1_epochs, "Training", csv1s)
        result["single"] = (best, ep, hist)
        say(f"Single-stage metrics saved to: {csv1s}")
        final_path = models_dir / "unet_pde_regularized.pth"
    if is_main:
        torch.save(model.state_dict(), final_path)
    say(f"Model saved to: {final_path}")

    # ---- test-set evaluation (src/train.py:848-911), rank 0 ----
    say("\n" + "=" * 70 + "\nTEST SET EVALUATION\n" + "=" * 70)
    if is_main and test_json.exists() and test_dir.exists():
        from .evaluate import evaluate_on_test_set
        name = "PDE-Constrained (Stage II)" if use_two_stage else "Single-Stage PDE-Constrained"
        m = evaluate_on_test_set(model, test_dir, test_json, device, batch_size=batch_size, threshold=0.5,
                                 model_name=name)
        tag = "stage2" if use_two_stage else "single_stage"
        save_test_metrics(m, out_dir / f"test_metrics_{tag}_{stamp}{frac}", model_name=name)
        result["test"] = m
        if use_two_stage:
            say("\n" + "=" * 70 + "\nEVALUATING STAGE I MODEL ON TEST SET\n" + "=" * 70)
            stage1 = UNet(in_channels=1, out_channels=1, base_channels=64)
            stage1.load_state_dict(torch.load(stage1_path, map_location="cpu", weights_only=True))
            stage1 = stage1.to(device)
            m1 = evaluate_on_test_set(stage1, test_dir, test_json, device, batch_size=batch_size, threshold=0.5,
                                      model_name="Baseline (Stage I)")
            save_test_metrics(m1, out_dir / f"test_metrics_stage1_{stamp}{frac}", model_name="Baseline (Stage I)")
            result["test_stage1"] = m1
    elif is_main:
        say(f"Warning: Test set not found at {test_dir} or {test_json}")
        say("Skipping test set evaluation.")
    say("\n" + "=" * 70 + "\nTRAINING COMPLETE\n" + "=" * 70)
    return model, result
