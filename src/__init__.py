"""Drop-in alias: ``import src`` / ``from src.train import train`` resolve to the
MI355X implementation (physics_informed_image_segmentation_amd), with the
module names of the reference's ``src`` package. Importing it does not need
OpenCV (the reference's src/__init__.py:13 does)."""
from physics_informed_image_segmentation_amd import *  # noqa: F401,F403
from physics_informed_image_segmentation_amd import __all__  # noqa: F401
