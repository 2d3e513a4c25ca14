"""MI355X-native (gfx950) PDE-constrained U-Net segmentation training step.

Drop-in for the hot path of seemapoudel58/Physics_informed_image_segmentation
(src/unet.py, src/pde.py, src/loss.py, src/metrics.py, src/train.py): the
same Python surface, computed by hand-written HIP kernels behind the C-ABI in
include/pis_capi.h. There is no CPU fallback.
"""
__version__ = "0.1.0"
