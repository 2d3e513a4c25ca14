"""ORACLE — test infrastructure only.

This package is the CPU restatement of the reference's hot path
(seemapoudel58/Physics_informed_image_segmentation: src/unet.py, src/pde.py,
src/loss.py, src/metrics.py, src/evaluate.py IoU, src/train.py step loop).
It exists to CHECK the MI355X product path, never to run it:

  * only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import it;
  * the product package ``physics_informed_image_segmentation_amd`` never
    imports it and has no CPU fallback.

Pinning: the reference cannot be imported or run in this pipeline (permission
denial recorded in SURVEY.md §8(c)). The restatement is pinned by
  1. the one-shot observation of the real reference recorded in SURVEY.md
     §8(c) (seed-42 synthetic batch, UNet init, every loss term) — reproduced
     to fp32 rounding by ``tests/test_oracle.py::test_pinned_reference_observation``;
  2. the analytic known-answer tests of SURVEY.md §4;
  3. float64 autograd vs. the hand-derived backward in ``loss_numpy``.
"""
