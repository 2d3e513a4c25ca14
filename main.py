"""CLI of the reference (main.py:5-102): same flags and defaults, training on
the MI355X path. Build-only flags: --synthetic N_TRAIN N_VAL H W, --base-dir."""
import argparse

from physics_informed_image_segmentation_amd.train import train


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Train PDE-constrained cell segmentation model")
    p.add_argument("--single-stage", action="store_true",
                   help="Use single-stage training (PDE from start) instead of two-stage")
    p.add_argument("--pde-weight", type=float, default=1e-4, help="Weight for PDE regularization λ_RD")
    p.add_argument("--diffusion-coeff", type=float, default=5.0, help="Diffusion coefficient D for PDE")
    p.add_argument("--reaction-threshold", type=float, default=0.5, help="Reaction term threshold a for PDE")
    p.add_argument("--phase-field-weight", type=float, default=1e-4, help="Weight for phase-field energy λ_PF")
    p.add_argument("--epsilon", type=float, default=0.05, help="Interface width parameter ε")
    p.add_argument("--batch-size", type=int, default=8, help="Batch size per GPU")
    p.add_argument("--learning-rate", type=float, default=1e-4, help="Learning rate for AdamW")
    p.add_argument("--stage1-epochs", type=int, default=50, help="Maximum epochs for Stage I")
    p.add_argument("--stage2-epochs", type=int, default=50, help="Maximum epochs for Stage II")
    p.add_argument("--early-stopping-patience", type=int, default=5, help="Patience for early stopping")
    p.add_argument("--train-fraction", type=float, default=None, help="Fraction of training data to use")
    p.add_argument("--seed", type=int, default=42, help="Random seed")
    p.add_argument("--synthetic", type=int, nargs=4, metavar=("N_TRAIN", "N_VAL", "H", "W"), default=None,
                   help="train on the synthetic disc generator instead of images/")
    p.add_argument("--base-dir", type=str, default=None, help="directory holding images/, output/, models/")
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    return train(use_two_stage=not a.single_stage, pde_weight=a.pde_weight, diffusion_coeff=a.diffusion_coeff,
                 reaction_threshold=a.reaction_threshold, phase_field_weight=a.phase_field_weight,
                 epsilon=a.epsilon, batch_size=a.batch_size, learning_rate=a.learning_rate,
                 stage1_epochs=a.stage1_epochs, stage2_epochs=a.stage2_epochs,
                 early_stopping_patience=a.early_stopping_patience, train_fraction=a.train_fraction,
                 seed=a.seed, base_dir=a.base_dir,
                 synthetic=tuple(a.synthetic) if a.synthetic else None)


if __name__ == "__main__":
    main()
