"""Evaluate and compare a baseline and a PDE-constrained checkpoint on the test set — the
reference's eval CLI (evaluate.py:17-146) on the MI355X build: same flags and defaults.

    python evaluate.py --baseline models/unet_baseline.pth --pde models/unet_pde_regularized.pth
    python evaluate.py --baseline 'runs/*/unet_baseline.pth' --pde 'runs/*/unet_pde_regularized.pth' --repeated
"""
import argparse
import os
import sys
from glob import glob
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="Evaluate and compare segmentation models")
    ap.add_argument("--baseline", type=str, required=True,
                    help="Path to baseline model checkpoint (or pattern for repeated experiments)")
    ap.add_argument("--pde", type=str, required=True,
                    help="Path to PDE-constrained model checkpoint (or pattern for repeated experiments)")
    ap.add_argument("--test-dir", type=str, default="images/testing",
                    help="Directory containing test images (default: images/testing)")
    ap.add_argument("--test-json", type=str, default="images/annotation/testing_annotation.json",
                    help="Path to test annotations JSON (default: images/annotation/testing_annotation.json)")
    ap.add_argument("--batch-size", type=int, default=8, help="Batch size for evaluation (default: 8)")
    ap.add_argument("--threshold", type=float, default=0.5,
                    help="Threshold for binarizing predictions (default: 0.5)")
    ap.add_argument("--output-dir", type=str, default="output",
                    help="Directory to save evaluation results (default: output)")
    ap.add_argument("--repeated", action="store_true",
                    help="Run repeated experiments evaluation (baseline and pde should be glob patterns)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    import torch

    from physics_informed_image_segmentation_amd.evaluate_comparison import (evaluate_and_compare,
                                                                             run_repeated_evaluations)
    # the HIP UNet has no CPU path: evaluation needs the GPU (it raises otherwise)
    device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    print(f"Using device: {device}")
    common = dict(test_dir=Path(args.test_dir), test_json=Path(args.test_json), device=device,
                  batch_size=args.batch_size, threshold=args.threshold, output_dir=Path(args.output_dir))
    if args.repeated:
        base = sorted(glob(args.baseline))
        pde = sorted(glob(args.pde))
        if not base:
            print(f"Error: No baseline models found matching pattern: {args.baseline}")
            return None
        if not pde:
            print(f"Error: No PDE models found matching pattern: {args.pde}")
            return None
        if len(base) != len(pde):
            print(f"Warning: Number of baseline models ({len(base)}) != number of PDE models ({len(pde)})")
        print(f"\nFound {len(base)} baseline models")
        print(f"Found {len(pde)} PDE-constrained models")
        results = run_repeated_evaluations([Path(p) for p in base], [Path(p) for p in pde], **common)
    else:
        bp, pp = Path(args.baseline), Path(args.pde)
        for label, p in (("Baseline", bp), ("PDE", pp)):
            if not p.exists():
                print(f"Error: {label} model not found: {p}")
                return None
        results = evaluate_and_compare(bp, pp, **common)
    print("\n" + "=" * 70 + "\nEVALUATION COMPLETE\n" + "=" * 70)
    return results


if __name__ == "__main__":
    main()
