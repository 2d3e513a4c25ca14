"""MI355X-native (gfx950) PDE-constrained U-Net segmentation training step.

Drop-in for the hot path of seemapoudel58/Physics_informed_image_segmentation
(src/unet.py, src/pde.py, src/loss.py, src/metrics.py, src/train.py): the
same Python surface, computed by hand-written HIP kernels behind the C-ABI in
include/pis_capi.h. There is no CPU fallback.
"""
__version__ = "0.1.0"

from .dataset import CellSegmentationDataset, SyntheticDiscDataset  # noqa: E402
from .evaluate import compute_iou, compute_iou_batch  # noqa: E402
from .loss import DiceBCELoss, DiceBCEPDELoss  # noqa: E402
from .metrics import compute_dice_score, compute_dice_score_batch  # noqa: E402
from .optim import AdamW  # noqa: E402
from .pde import PDERegularization, create_pde_regularization  # noqa: E402
from .train import EarlyStopping, train, train_epoch, train_stage, validate  # noqa: E402
from .unet import UNet, count_parameters  # noqa: E402

__all__ = ["CellSegmentationDataset", "SyntheticDiscDataset", "UNet", "count_parameters", "DiceBCELoss",
           "DiceBCEPDELoss", "PDERegularization", "create_pde_regularization", "compute_dice_score",
           "compute_dice_score_batch", "compute_iou", "compute_iou_batch", "EarlyStopping", "train_epoch",
           "train_stage", "validate", "train", "AdamW"]
