"""Ablation studies of src/ablation.py + run_ablation.py on the MI355X path.

Kept for drop-in: ``AblationConfig`` (src/ablation.py:20-50, same fields and defaults),
``create_ablation_loss`` (:89-154; the diffusion-only variant is the fused kernel with
``PIS_LOSS_NO_REACTION``), the six study definitions R1-R3 / S1-S3 (run_ablation.py:23-294),
``run_ablation_variant`` (:157-1237: Stage I DiceBCE when two-stage with PDE, then the
variant's loss at the same learning rate, both with early stopping on val Dice, per-image
test metrics after each stage) and ``run_ablation_study`` (:1240-1474: one run per variant,
``results.json`` + ``summary.csv`` under ``output/ablation/{name}_{timestamp}``).

What is not rebuilt: the plots and the paired statistical tests of the reference's study
report (matplotlib/seaborn reporting, outside the hot path). The BASELINE configs C4 (R1
sweep) and C5 (S2 D-sweep) run through ``run_ablation.py --ablation R1|S2`` on this path;
``--synthetic N_TRAIN N_VAL H W`` trains on the SURVEY §8(c) disc generator when the cell
dataset is absent.
"""
from __future__ import annotations

import csv
import json
from dataclasses import asdict, dataclass
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from .dataset import CellSegmentationDataset, SyntheticDiscDataset
from .evaluate import evaluate_model
from .fused import LossConfig, fused_loss
from .loss import BCELoss, DiceBCELoss, DiceBCEPDELoss
from .optim import AdamW
from .pde import PDERegularization
from .train import EarlyStopping, create_subset_dataset, train_stage
from .unet import UNet


@dataclass
class AblationConfig:
    """One ablation variant (src/ablation.py:20-50)."""
    name: str
    description: str
    use_pde: bool = False
    pde_weight: float = 1e-4
    phase_field_weight: float = 1e-4
    epsilon: float = 0.05
    diffusion_coeff: float = 5.0
    reaction_threshold: float = 0.5
    use_reaction_term: bool = True
    use_two_stage: bool = True
    use_three_stage: bool = False
    train_fraction: Optional[float] = None
    stage1_epochs: Optional[int] = None
    stage2_epochs: Optional[int] = None
    stage3_epochs: Optional[int] = None
    output_activation: str = "sigmoid"
    intermediate_activation: str = "relu"
    seed: int = 42

    def to_dict(self) -> Dict:
        return asdict(self)


class PDERegularizationAblation:
    """RD residual loss with the reaction term optional (src/ablation.py:53-86)."""

    def __init__(self, diffusion_coeff: float = 1.0, reaction_threshold: float = 0.5,
                 use_reaction_term: bool = True):
        self.pde_reg = PDERegularization(diffusion_coeff=diffusion_coeff, reaction_threshold=reaction_threshold)
        self.use_reaction_term = use_reaction_term

    def compute_loss(self, u: torch.Tensor) -> torch.Tensor:
        cfg = LossConfig(dice_w=0.0, bce_w=0.0, rd_w=1.0, D=self.pde_reg.diffusion_coeff,
                         a=self.pde_reg.reaction_threshold, reaction=self.use_reaction_term)
        return fused_loss(u, torch.zeros_like(u), cfg)


class DiffusionOnlyLoss(nn.Module):
    """0.5 Dice + 0.5 BCE + pde_weight * mean((D Lap u)^2) — the reference's local class
    (src/ablation.py:107-151), one fused launch (reaction term off in the kernel). Like the
    reference's, it is not a DiceBCEPDELoss, so the step loop logs no pde_loss for it."""

    def __init__(self, config: AblationConfig):
        super().__init__()
        self.dice_weight = 0.5
        self.bce_weight = 0.5
        self.pde_weight = config.pde_weight
        self.smooth = 1e-6
        self.pde_reg = PDERegularizationAblation(config.diffusion_coeff, config.reaction_threshold,
                                                 use_reaction_term=False)
        self.bce = BCELoss()
        self.last: dict = {}

    def config(self) -> LossConfig:
        return LossConfig(dice_w=self.dice_weight, bce_w=self.bce_weight, rd_w=self.pde_weight, smooth=self.smooth,
                          D=self.pde_reg.pde_reg.diffusion_coeff, a=self.pde_reg.pde_reg.reaction_threshold,
                          reaction=False)

    def forward(self, predictions: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        self.last = {}
        return fused_loss(predictions, targets, self.config(), self.last)


def create_ablation_loss(config: AblationConfig) -> nn.Module:
    """src/ablation.py:89-154."""
    if not config.use_pde:
        return DiceBCELoss(dice_weight=0.5, bce_weight=0.5)
    if not config.use_reaction_term:
        return DiffusionOnlyLoss(config)
    return DiceBCEPDELoss(dice_weight=0.5, bce_weight=0.5, pde_weight=config.pde_weight,
                          phase_field_weight=config.phase_field_weight, diffusion_coeff=config.diffusion_coeff,
                          reaction_threshold=config.reaction_threshold, epsilon=config.epsilon)


# ---- the six studies (run_ablation.py:23-294) -------------------------------------------

_FULL = dict(use_pde=True, pde_weight=1e-4, phase_field_weight=1e-4, diffusion_coeff=5.0, reaction_threshold=0.5,
             epsilon=0.05, use_two_stage=True)


def _component_ablation(prefix: str, fraction: Optional[float]) -> List[AblationConfig]:
    tag = " with 10% data" if fraction else ""
    return [
        AblationConfig(name=f"{prefix}.0 Baseline", description=f"Baseline UNet (Dice + BCE only, no PDE constraints){tag}",
                       use_pde=False, pde_weight=0.0, phase_field_weight=0.0, train_fraction=fraction,
                       use_two_stage=False),
        AblationConfig(name=f"{prefix}.1 RD Only", description=f"Reaction-Diffusion PDE only (λ_RD=1e-4, λ_PF=0.0){tag}",
                       use_pde=True, pde_weight=1e-4, phase_field_weight=0.0, diffusion_coeff=5.0,
                       reaction_threshold=0.5, train_fraction=fraction, use_two_stage=True),
        AblationConfig(name=f"{prefix}.2 Phase-Field Only",
                       description=f"Phase-field energy only (λ_RD=0.0, λ_PF=1e-4){tag}", use_pde=True,
                       pde_weight=0.0, phase_field_weight=1e-4, epsilon=0.05, diffusion_coeff=5.0,
                       reaction_threshold=0.5, train_fraction=fraction, use_two_stage=True),
        AblationConfig(name=f"{prefix}.3 RD + Phase-Field",
                       description=f"Reaction-Diffusion + Phase-Field (λ_RD=1e-4, λ_PF=1e-4){tag}",
                       train_fraction=fraction, **_FULL),
    ]


def define_ablation_r1() -> List[AblationConfig]:
    """R1: PDE components at 100 % data (run_ablation.py:23-83)."""
    return _component_ablation("R1", None)


def define_ablation_r2() -> List[AblationConfig]:
    """R2: full model at 10/25/50/75/100 % data (run_ablation.py:86-117)."""
    return [AblationConfig(name=f"R2.{i} {int(f * 100)}% Data",
                           description=f"Full model (RD + Phase-Field) with {int(f * 100)}% training data",
                           train_fraction=f, **_FULL)
            for i, f in enumerate([0.1, 0.25, 0.5, 0.75, 1.0])]


def define_ablation_r3() -> List[AblationConfig]:
    """R3: PDE components at 10 % data (run_ablation.py:230-294)."""
    return _component_ablation("R3", 0.1)


def define_ablation_s1() -> List[AblationConfig]:
    """S1: reaction threshold a in {0.3 .. 0.7}, 10 % data (run_ablation.py:120-155)."""
    kw = dict(_FULL)
    kw.pop("reaction_threshold")
    return [AblationConfig(name=f"S1.{i} a={a:.1f}",
                           description=f"Full model (RD + Phase-Field) with reaction threshold a={a}",
                           reaction_threshold=a, train_fraction=0.1, **kw)
            for i, a in enumerate([0.3, 0.4, 0.5, 0.6, 0.7])]


def define_ablation_s2() -> List[AblationConfig]:
    """S2: diffusion coefficient D in {0.5 .. 100}, RD only at lambda 1e-3, 10 % data
    (run_ablation.py:158-188) — BASELINE config C5."""
    return [AblationConfig(name=f"S2.{i} D={d:.1f}" if d < 10 else f"S2.{i} D={d:.0f}",
                           description=f"Reaction-diffusion with diffusion coefficient D={d}", use_pde=True,
                           pde_weight=1e-3, diffusion_coeff=d, phase_field_weight=0.0, train_fraction=0.1,
                           use_two_stage=True)
            for i, d in enumerate([0.5, 1.0, 2.0, 5.0, 10.0, 100.0])]


def define_ablation_s3() -> List[AblationConfig]:
    """S3: interface width eps in {0.001 .. 0.2}, 10 % data (run_ablation.py:191-227)."""
    kw = dict(_FULL)
    kw.pop("epsilon")
    return [AblationConfig(name=f"S3.{i} ε={e:.3f}" if e < 0.01 else f"S3.{i} ε={e:.2f}",
                           description=f"Reaction-diffusion + phase-field (ε={e}, λ_RD=1e-4, λ_PF=1e-4, D=5.0)",
                           epsilon=e, train_fraction=0.1, **kw)
            for i, e in enumerate([0.001, 0.01, 0.05, 0.1, 0.2])]


ABLATIONS = {"R1": define_ablation_r1, "R2": define_ablation_r2, "R3": define_ablation_r3,
             "S1": define_ablation_s1, "S2": define_ablation_s2, "S3": define_ablation_s3}


# ---- running a variant --------------------------------------------------------------------

@dataclass
class DataSpec:
    """Where a variant's data comes from: the reference's directory/JSON pairs, or the disc
    generator (``synthetic=(n_train, n_val, n_test, H, W)``)."""
    train_dir: Optional[Path] = None
    train_json: Optional[Path] = None
    val_dir: Optional[Path] = None
    val_json: Optional[Path] = None
    in_dist_test_dir: Optional[Path] = None
    in_dist_test_json: Optional[Path] = None
    out_dist_test_dir: Optional[Path] = None
    out_dist_test_json: Optional[Path] = None
    synthetic: Optional[Tuple[int, int, int, int, int]] = None

    def datasets(self, seed: int):
        if self.synthetic is not None:
            ntr, nva, nte, H, W = self.synthetic
            return (SyntheticDiscDataset(ntr, (H, W), seed=seed), SyntheticDiscDataset(nva, (H, W), seed=seed + 1),
                    SyntheticDiscDataset(nte, (H, W), seed=seed + 2), SyntheticDiscDataset(nte, (H, W), seed=seed + 3))
        return (CellSegmentationDataset(self.train_dir, self.train_json),
                CellSegmentationDataset(self.val_dir, self.val_json),
                CellSegmentationDataset(self.in_dist_test_dir, self.in_dist_test_json),
                CellSegmentationDataset(self.out_dist_test_dir, self.out_dist_test_json))


def _slug(name: str) -> str:
    return name.replace(" ", "_").lower()


def _summary(metrics: Dict[str, np.ndarray]) -> Dict[str, Dict[str, float]]:
    out = {}
    for k, v in metrics.items():
        a = np.asarray(v, dtype=np.float64)
        fin = a[np.isfinite(a)]
        out[k] = {"mean": float(fin.mean()) if fin.size else float("nan"),
                  "std": float(fin.std(ddof=1)) if fin.size > 1 else 0.0, "count": int(fin.size)}
    return out


_PATH_ARGS = ("train_dir", "train_json", "val_dir", "val_json", "in_dist_test_dir", "in_dist_test_json",
              "out_dist_test_dir", "out_dist_test_json")
_DEFAULT_OUT = Path(__file__).resolve().parent.parent / "output" / "ablation"


def _data_spec(first, paths) -> DataSpec:
    """The reference passes eight directory/JSON paths (src/ablation.py:157-175); this build
    also accepts one ``DataSpec`` (e.g. the synthetic generator) in the first path's place."""
    if isinstance(first, DataSpec):
        return first
    return DataSpec(*(Path(p) if p is not None else None for p in (first,) + tuple(paths)))


def run_ablation_variant(config: AblationConfig, train_dir, train_json=None, val_dir=None, val_json=None,
                         in_dist_test_dir=None, in_dist_test_json=None, out_dist_test_dir=None,
                         out_dist_test_json=None, device: Optional[torch.device] = None, batch_size: int = 8,
                         learning_rate: float = 1e-4, stage1_epochs: int = 50, stage2_epochs: int = 50,
                         early_stopping_patience: int = 10, output_dir: Optional[Path] = None,
                         ablation_folder: Optional[Path] = None, num_workers: int = 2, boundary_metrics: bool = True,
                         verbose: bool = False) -> Dict:
    """Train one variant and evaluate it on both test sets (src/ablation.py:157-1237); same
    positional signature as the reference (``train_dir`` may be a ``DataSpec`` instead)."""
    data = _data_spec(train_dir, (train_json, val_dir, val_json, in_dist_test_dir, in_dist_test_json,
                                  out_dist_test_dir, out_dist_test_json))
    if device is None:
        device = torch.device("cuda")
    if config.output_activation != "sigmoid" or config.intermediate_activation != "relu":
        raise ValueError("this build runs the reference configuration: sigmoid output, ReLU activations")
    folder = Path(ablation_folder) if ablation_folder else (Path(output_dir) if output_dir else _DEFAULT_OUT)
    folder.mkdir(parents=True, exist_ok=True)
    torch.manual_seed(config.seed)
    np.random.seed(config.seed)
    torch.cuda.manual_seed(config.seed)
    train_ds, val_ds, in_ds, out_ds = data.datasets(config.seed)
    if config.train_fraction is not None:
        train_ds = create_subset_dataset(train_ds, config.train_fraction)
    pin = torch.cuda.is_available()
    mk = lambda ds, sh: DataLoader(ds, batch_size=batch_size, shuffle=sh, num_workers=num_workers, pin_memory=pin)
    train_loader, val_loader = mk(train_ds, True), mk(val_ds, False)
    in_loader, out_loader = mk(in_ds, False), mk(out_ds, False)
    model = UNet(1, 1, 64).to(device)

    def evaluate():
        return {"in_dist": evaluate_model(model, in_loader, device, 0.5, boundary_metrics),
                "out_dist": evaluate_model(model, out_loader, device, 0.5, boundary_metrics)}

    def stage(criterion, epochs, name, csv_name):
        opt = AdamW(model.parameters(), lr=learning_rate, weight_decay=1e-5)
        stop = EarlyStopping(patience=early_stopping_patience, min_delta=1e-4, mode="max")
        return train_stage(model, train_loader, val_loader, criterion.to(device), opt, device, num_epochs=epochs,
                           stage_name=name, early_stopping=stop, verbose=verbose,
                           csv_path=folder / f"{_slug(config.name)}_{csv_name}_metrics.csv")

    result: Dict = {"config": config.to_dict()}
    three = config.use_three_stage
    if (config.use_two_stage and config.use_pde) or three:
        ep1 = config.stage1_epochs if config.stage1_epochs is not None else (50 if three else stage1_epochs)
        best1, bep1, _ = stage(DiceBCELoss(0.5, 0.5), ep1, "Stage I", "stage1")
        path = folder / f"{_slug(config.name)}_baseline_after_stage1.pth"
        torch.save(model.state_dict(), path)
        result["baseline_model_path"] = str(path)
        result["stage1_best_epoch"] = bep1
        base = evaluate()
        result["baseline_in_dist_metrics"] = {k: v.tolist() for k, v in base["in_dist"].items()}
        result["baseline_out_dist_metrics"] = {k: v.tolist() for k, v in base["out_dist"].items()}
    if config.use_pde or not config.use_two_stage or three:
        if config.use_two_stage:
            ep2 = config.stage2_epochs if config.stage2_epochs is not None else stage2_epochs
        else:
            ep2 = config.stage1_epochs if config.stage1_epochs is not None else stage1_epochs
        best2, bep2, _ = stage(create_ablation_loss(config), ep2,
                               "Stage II (PDE)" if config.use_two_stage else "Training", "stage2")
        result["stage2_best_epoch"] = bep2
    if three:
        ep3 = config.stage3_epochs if config.stage3_epochs is not None else (config.stage2_epochs or stage2_epochs)
        stage(DiceBCELoss(0.5, 0.5), ep3, "Stage III", "stage3")
    path = folder / f"{_slug(config.name)}_final.pth"
    torch.save(model.state_dict(), path)
    result["model_path"] = str(path)
    final = evaluate()
    result["in_dist_metrics"] = {k: v.tolist() for k, v in final["in_dist"].items()}
    result["out_dist_metrics"] = {k: v.tolist() for k, v in final["out_dist"].items()}
    result["in_dist_summary"] = _summary(final["in_dist"])
    result["out_dist_summary"] = _summary(final["out_dist"])
    return result


def run_ablation_study(ablation_name: str, variants: List[AblationConfig], train_dir, train_json=None, val_dir=None,
                       val_json=None, in_dist_test_dir=None, in_dist_test_json=None, out_dist_test_dir=None,
                       out_dist_test_json=None, device: Optional[torch.device] = None, batch_size: int = 8,
                       learning_rate: float = 1e-4, stage1_epochs: int = 50, stage2_epochs: int = 50,
                       early_stopping_patience: int = 10, output_dir: Optional[Path] = None, **kw) -> Dict:
    """One run per variant; results JSON + summary CSV (src/ablation.py:1240-1474); same
    positional signature as the reference (``train_dir`` may be a ``DataSpec`` instead)."""
    data = _data_spec(train_dir, (train_json, val_dir, val_json, in_dist_test_dir, in_dist_test_json,
                                  out_dist_test_dir, out_dist_test_json))
    root = Path(output_dir) if output_dir else _DEFAULT_OUT
    folder = root / f"{ablation_name}_{datetime.now().strftime('%Y%m%d_%H%M%S')}"
    folder.mkdir(parents=True, exist_ok=True)
    results = []
    for v in variants:
        print(f"\n{'=' * 70}\nAblation {ablation_name}: {v.name}\n  {v.description}\n{'=' * 70}", flush=True)
        results.append(run_ablation_variant(v, data, device=device, batch_size=batch_size, learning_rate=learning_rate,
                                            stage1_epochs=stage1_epochs, stage2_epochs=stage2_epochs,
                                            early_stopping_patience=early_stopping_patience, ablation_folder=folder,
                                            **kw))
    results_json = folder / "results.json"
    with open(results_json, "w") as f:
        json.dump({"ablation": ablation_name, "variants": results}, f, indent=2)
    summary_csv = folder / "summary.csv"
    metrics = ["dice_scores", "iou_scores", "boundary_f1_scores", "hausdorff_distances"]
    with open(summary_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["variant", "test_set"] + [f"{m}_{s}" for m in metrics for s in ("mean", "std")])
        for r in results:
            for side in ("in_dist", "out_dist"):
                summ = r[f"{side}_summary"]
                row = [r["config"]["name"], side]
                for m in metrics:
                    row += [summ[m]["mean"], summ[m]["std"]] if m in summ else ["", ""]
                w.writerow(row)
    return {"results": results, "results_json": str(results_json), "summary_csv": str(summary_csv),
            "folder": str(folder)}
