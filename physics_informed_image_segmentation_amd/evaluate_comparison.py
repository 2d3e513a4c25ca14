"""Offline checkpoint comparison of src/evaluate_comparison.py on this build.

The two reference checkpoints (``unet_baseline.pth``, ``unet_pde_regularized.pth``) are loaded
into the HIP ``UNet`` with ``torch.load(..., weights_only=True)`` (state_dict keys and shapes are
the reference's), evaluated on the test folder (per-image Dice / IoU from the fused
kernel's counters, boundary F1 / Hausdorff on the host) and compared with paired tests. Output
files and their columns are the reference's:
  * ``evaluate_and_compare`` (src/evaluate_comparison.py:79-227): evaluation_results_<ts>.csv
    (per image), evaluation_summary_<ts>.csv (per metric), statistical_comparison_<ts>.json;
  * ``run_repeated_evaluations`` (:230-396): aggregated_results_<ts>.csv.
"""
from __future__ import annotations

import json
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .evaluate import compare_models_statistically, compute_statistics, evaluate_on_test_set, format_metric_report
from .unet import UNet

METRIC_KEYS = ("dice_scores", "iou_scores", "boundary_f1_scores", "hausdorff_distances")
_DEFAULT_OUT = Path(__file__).resolve().parent.parent / "output"


def make_json_serializable(obj: Any) -> Any:
    """numpy scalars/arrays -> Python natives, recursively; anything else unknown -> str
    (src/evaluate_comparison.py:32-58)."""
    if isinstance(obj, np.bool_):
        return bool(obj)
    if isinstance(obj, np.integer):
        return int(obj)
    if isinstance(obj, np.floating):
        return float(obj)
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    if isinstance(obj, dict):
        return {k: make_json_serializable(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [make_json_serializable(v) for v in obj]
    if obj is None or isinstance(obj, (bool, int, float, str)):
        return obj
    return str(obj)


def load_model(model_path: Path, device: torch.device) -> UNet:
    """A reference-format checkpoint in the HIP UNet, eval mode (src/evaluate_comparison.py:61-76).
    The file is read with weights_only=True: a checkpoint never executes code here."""
    model = UNet(in_channels=1, out_channels=1, base_channels=64)
    model.load_state_dict(torch.load(model_path, map_location="cpu", weights_only=True))
    return model.to(device).eval()


def _print_comparison(results: Dict[str, Dict[str, float]]):
    print("\nStatistical Test Results (α = 0.05):")
    print("-" * 70)
    for name, r in results.items():
        print(f"\n{name.replace('_', ' ').title()}:")
        if "baseline_mean" not in r:
            print("  fewer than two paired values: no test")
            continue
        print(f"  Baseline Mean: {r['baseline_mean']:.4f}")
        print(f"  PDE Mean:      {r['pde_mean']:.4f}")
        print(f"  Improvement:   {r['improvement']:+.4f}")
        print(f"  Paired t-test:\n    t-statistic: {r['t_statistic']:.4f}\n    p-value:     {r['t_pvalue']:.4f}")
        print(f"  Wilcoxon signed-rank test:\n    statistic:   {r['wilcoxon_statistic']:.4f}\n"
              f"    p-value:     {r['wilcoxon_pvalue']:.4f}")
        print(f"  Significant:  {'Yes' if r['significant'] else 'No'}")


def evaluate_and_compare(baseline_model_path: Path, pde_model_path: Path, test_dir: Path, test_json: Path,
                         device: torch.device, batch_size: int = 8, threshold: float = 0.5,
                         output_dir: Optional[Path] = None) -> Dict:
    import pandas as pd
    out_dir = Path(output_dir) if output_dir is not None else _DEFAULT_OUT
    out_dir.mkdir(parents=True, exist_ok=True)
    print("=" * 70 + "\nMODEL EVALUATION AND STATISTICAL COMPARISON\n" + "=" * 70)
    print("\nLoading models...")
    base = evaluate_on_test_set(load_model(baseline_model_path, device), test_dir, test_json, device,
                                batch_size=batch_size, threshold=threshold, model_name="Baseline (Unconstrained)")
    pde = evaluate_on_test_set(load_model(pde_model_path, device), test_dir, test_json, device,
                               batch_size=batch_size, threshold=threshold, model_name="PDE-Constrained")
    print("\n" + "=" * 70 + "\nSTATISTICAL COMPARISON\n" + "=" * 70)
    cmp = compare_models_statistically(base, pde, alpha=0.05)
    _print_comparison(cmp)

    ts = datetime.now().strftime("%Y%m%d_%H%M%S")
    per_image = {"image_id": range(len(base["dice_scores"]))}
    for key, col in (("dice_scores", "dice"), ("iou_scores", "iou"), ("boundary_f1_scores", "boundary_f1"),
                     ("hausdorff_distances", "hausdorff")):
        per_image[f"baseline_{col}"] = base[key]
        per_image[f"pde_{col}"] = pde[key]
    results_csv = out_dir / f"evaluation_results_{ts}.csv"
    pd.DataFrame(per_image).to_csv(results_csv, index=False)
    print(f"\nPer-image metrics saved to: {results_csv}")

    summary = {}
    for name in base:
        sb, sp, c = compute_statistics(base[name]), compute_statistics(pde[name]), cmp[name]
        summary[name] = {"baseline_mean": sb["mean"], "baseline_std": sb["std"], "pde_mean": sp["mean"],
                         "pde_std": sp["std"], "improvement": c.get("improvement", np.nan),
                         "t_pvalue": c["t_pvalue"], "wilcoxon_pvalue": c["wilcoxon_pvalue"],
                         "significant": c["significant"]}
    summary_csv = out_dir / f"evaluation_summary_{ts}.csv"
    pd.DataFrame(summary).T.to_csv(summary_csv)
    print(f"Summary statistics saved to: {summary_csv}")
    comparison_json = out_dir / f"statistical_comparison_{ts}.json"
    with open(comparison_json, "w") as f:
        json.dump(make_json_serializable(cmp), f, indent=2)
    print(f"Statistical comparison saved to: {comparison_json}")
    return {"baseline_metrics": base, "pde_metrics": pde, "comparison_results": cmp, "results_csv": results_csv,
            "summary_csv": summary_csv, "comparison_json": comparison_json}


def run_repeated_evaluations(baseline_model_paths: List[Path], pde_model_paths: List[Path], test_dir: Path,
                             test_json: Path, device: torch.device, batch_size: int = 8, threshold: float = 0.5,
                             output_dir: Optional[Path] = None) -> Dict:
    import pandas as pd
    out_dir = Path(output_dir) if output_dir is not None else _DEFAULT_OUT
    out_dir.mkdir(parents=True, exist_ok=True)
    print("=" * 70 + "\nREPEATED EXPERIMENTS EVALUATION\n" + "=" * 70)
    print(f"Number of runs: {len(baseline_model_paths)}")
    pooled = {"baseline": {k: [] for k in METRIC_KEYS}, "pde": {k: [] for k in METRIC_KEYS}}
    for i, (bp, pp) in enumerate(zip(baseline_model_paths, pde_model_paths)):
        print(f"\n{'=' * 70}\nRun {i + 1}/{len(baseline_model_paths)}\n{'=' * 70}")
        for tag, path, label in (("baseline", bp, f"Baseline Run {i + 1}"), ("pde", pp, f"PDE-Constrained Run {i + 1}")):
            m = evaluate_on_test_set(load_model(path, device), test_dir, test_json, device, batch_size=batch_size,
                                     threshold=threshold, model_name=label)
            for k in METRIC_KEYS:
                pooled[tag][k].extend(m[k])
    base = {k: np.array(v) for k, v in pooled["baseline"].items()}
    pde = {k: np.array(v) for k, v in pooled["pde"].items()}
    print("\n" + "=" * 70 + "\nAGGREGATED RESULTS (All Runs Combined)\n" + "=" * 70)
    print(format_metric_report(base, model_name="Baseline (All Runs)"))
    print(format_metric_report(pde, model_name="PDE-Constrained (All Runs)"))
    cmp = compare_models_statistically(base, pde, alpha=0.05)
    print("\n" + "=" * 70 + "\nSTATISTICAL COMPARISON (Aggregated)\n" + "=" * 70)
    for name, r in cmp.items():
        print(f"\n{name.replace('_', ' ').title()}:")
        if "baseline_mean" in r:
            print(f"  Baseline: {r['baseline_mean']:.4f} ± {r.get('baseline_std', 0):.4f}")
            print(f"  PDE:      {r['pde_mean']:.4f} ± {r.get('pde_std', 0):.4f}")
            print(f"  Improvement: {r['improvement']:+.4f}")
        print(f"  Significant: {'Yes' if r['significant'] else 'No'} (p={r['t_pvalue']:.4f})")
    rows = []
    for name in METRIC_KEYS:
        for tag, arrs in (("baseline", base), ("pde", pde)):
            st = compute_statistics(arrs[name])
            rows.append({"metric": name, "model": tag, "mean": st["mean"], "std": st["std"], "count": st["count"]})
    aggregated_csv = out_dir / f"aggregated_results_{datetime.now().strftime('%Y%m%d_%H%M%S')}.csv"
    pd.DataFrame(rows, columns=["metric", "model", "mean", "std", "count"]).to_csv(aggregated_csv, index=False)
    print(f"\nAggregated results saved to: {aggregated_csv}")
    return {"baseline_metrics": base, "pde_metrics": pde, "comparison_results": cmp, "aggregated_csv": aggregated_csv}


__all__ = ["make_json_serializable", "load_model", "evaluate_and_compare", "run_repeated_evaluations"]
