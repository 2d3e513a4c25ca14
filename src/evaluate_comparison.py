"""Alias of physics_informed_image_segmentation_amd.evaluate_comparison (reference module src/evaluate_comparison.py)."""
import importlib as _importlib
import sys as _sys

_sys.modules[__name__] = _importlib.import_module("physics_informed_image_segmentation_amd.evaluate_comparison")
