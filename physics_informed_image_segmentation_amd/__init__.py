"""MI355X-native (gfx950) PDE-constrained U-Net segmentation training step.

Drop-in for the hot path of seemapoudel58/Physics_informed_image_segmentation
(src/unet.py, src/pde.py, src/loss.py, src/metrics.py, src/train.py): the
same Python surface, computed by hand-written HIP kernels behind the C-ABI in
include/pis_capi.h. There is no CPU fallback.

Exports the reference package's names (src/__init__.py:35-67) except the four
matplotlib plotting helpers of src/plot.py (out of scope).
"""
__version__ = "0.2.0"

from .dataset import CellSegmentationDataset, SyntheticDiscDataset  # noqa: E402
from .evaluate import (compare_models_statistically, compute_boundary_f1, compute_boundary_f1_batch,  # noqa: E402
                       compute_hausdorff_distance, compute_iou, compute_iou_batch, compute_statistics,
                       evaluate_model, evaluate_on_test_set, format_metric_report)
from .loss import DiceBCELoss, DiceBCEPDELoss  # noqa: E402
from .metrics import compute_dice_score, compute_dice_score_batch  # noqa: E402
from .optim import AdamW  # noqa: E402
from .pde import PDERegularization, create_pde_regularization  # noqa: E402
from .train import EarlyStopping, train, train_epoch, train_stage, validate  # noqa: E402
from .unet import UNet, count_parameters  # noqa: E402
from .evaluate_comparison import evaluate_and_compare, run_repeated_evaluations  # noqa: E402
from .ablation import AblationConfig, run_ablation_study, run_ablation_variant  # noqa: E402

__all__ = ["CellSegmentationDataset", "UNet", "DiceBCELoss", "DiceBCEPDELoss", "PDERegularization",
           "create_pde_regularization", "compute_dice_score", "compute_dice_score_batch", "EarlyStopping",
           "train_stage", "validate", "train", "compute_iou", "compute_iou_batch", "compute_boundary_f1",
           "compute_boundary_f1_batch", "compute_hausdorff_distance", "evaluate_model", "evaluate_on_test_set",
           "compare_models_statistically", "format_metric_report", "compute_statistics", "evaluate_and_compare",
           "run_repeated_evaluations", "AblationConfig", "run_ablation_variant", "run_ablation_study",
           # build additions
           "SyntheticDiscDataset", "count_parameters", "train_epoch", "AdamW"]
