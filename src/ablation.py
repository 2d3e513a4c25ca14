"""Alias of physics_informed_image_segmentation_amd.ablation (reference module src/ablation.py)."""
import importlib as _importlib
import sys as _sys

_sys.modules[__name__] = _importlib.import_module("physics_informed_image_segmentation_amd.ablation")
