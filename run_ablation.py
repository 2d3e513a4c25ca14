"""Ablation studies on the MI355X path — the CLI of the reference's run_ablation.py
(run_ablation.py:297-470: same flags and defaults), plus ``--synthetic`` to train on the
disc generator when the cell dataset is absent and ``--no-boundary-metrics`` to skip the
host-side boundary F1 / Hausdorff.

    python run_ablation.py --ablation R1                       # BASELINE config C4
    python run_ablation.py --ablation S2 --synthetic 64 16 16 1024 1024   # C5 shape, synthetic
"""
import argparse
from pathlib import Path

import torch

from physics_informed_image_segmentation_amd.ablation import ABLATIONS, DataSpec, run_ablation_study


def main(argv=None):
    ap = argparse.ArgumentParser(description="Run ablation studies for PDE-constrained cell segmentation")
    ap.add_argument("--ablation", type=str, required=True, choices=["R1", "R2", "R3", "S1", "S2", "S3", "all"])
    ap.add_argument("--train-dir", default="images/training")
    ap.add_argument("--train-json", default="images/annotation/training_annotation.json")
    ap.add_argument("--val-dir", default="images/validation")
    ap.add_argument("--val-json", default="images/annotation/validation_annotation.json")
    ap.add_argument("--test-dir", default="images/testing", help="[DEPRECATED] use --in-dist-test-dir")
    ap.add_argument("--test-json", default="images/annotation/testing_annotation.json",
                    help="[DEPRECATED] use --in-dist-test-json")
    ap.add_argument("--in-dist-test-dir", default="images/in_dist_testing")
    ap.add_argument("--in-dist-test-json", default="images/annotation/in_dist_testing_annotation.json")
    ap.add_argument("--out-dist-test-dir", default="images/out_dist_testing")
    ap.add_argument("--out-dist-test-json", default="images/annotation/out_dist_testing_annotation.json")
    ap.add_argument("--batch-size", type=int, default=8)
    ap.add_argument("--learning-rate", type=float, default=1e-4)
    ap.add_argument("--stage1-epochs", type=int, default=50)
    ap.add_argument("--stage2-epochs", type=int, default=50)
    ap.add_argument("--early-stopping-patience", type=int, default=10)
    ap.add_argument("--output-dir", type=str, default=None)
    ap.add_argument("--synthetic", type=int, nargs=5, default=None, metavar=("N_TRAIN", "N_VAL", "N_TEST", "H", "W"),
                    help="train/evaluate on the seeded disc generator instead of the image folders")
    ap.add_argument("--no-boundary-metrics", action="store_true")
    ap.add_argument("--num-workers", type=int, default=2)
    args = ap.parse_args(argv)
    if not torch.cuda.is_available():
        raise SystemExit("run_ablation.py: the MI355X path needs a GPU (no CPU fallback in this build)")
    device = torch.device("cuda")
    R = lambda p: Path(p).resolve()
    in_dir, in_json = R(args.in_dist_test_dir), R(args.in_dist_test_json)
    if args.test_dir != "images/testing" or args.test_json != "images/annotation/testing_annotation.json":
        print("Warning: --test-dir and --test-json are deprecated. Using them as in-distribution test set.")
        in_dir, in_json = R(args.test_dir), R(args.test_json)
    data = DataSpec(R(args.train_dir), R(args.train_json), R(args.val_dir), R(args.val_json), in_dir, in_json,
                    R(args.out_dist_test_dir), R(args.out_dist_test_json),
                    synthetic=tuple(args.synthetic) if args.synthetic else None)
    names = list(ABLATIONS) if args.ablation == "all" else [args.ablation]
    out = {}
    for name in names:
        print(f"\n{'=' * 70}\nStarting Ablation Study: {name}\n{'=' * 70}")
        res = run_ablation_study(name, ABLATIONS[name](), data, device=device, batch_size=args.batch_size,
                                 learning_rate=args.learning_rate, stage1_epochs=args.stage1_epochs,
                                 stage2_epochs=args.stage2_epochs,
                                 early_stopping_patience=args.early_stopping_patience,
                                 output_dir=Path(args.output_dir) if args.output_dir else None,
                                 num_workers=args.num_workers, boundary_metrics=not args.no_boundary_metrics)
        print(f"\nAblation {name} complete!\nResults: {res['results_json']}\nSummary: {res['summary_csv']}")
        out[name] = res
    print("\n" + "=" * 70 + "\nALL ABLATION STUDIES COMPLETE\n" + "=" * 70)
    return out


if __name__ == "__main__":
    main()
