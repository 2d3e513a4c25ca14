"""Known-answer tests of CellSegmentationDataset (src/dataset.py:9-118) on a COCO file the test
writes itself: one image with a square polygon and a triangle, one image without annotations
and one annotated image missing on disk. The expected mask is derived by hand from PIL's
documented semantics (polygon fill includes the outline; NEAREST samples the source pixel under
each target pixel centre, i.e. source index floor((i + 0.5) * scale))."""
import json

import numpy as np
import pytest
import torch
from PIL import Image

from physics_informed_image_segmentation_amd.dataset import CellSegmentationDataset


def _write(tmp_path):
    img_dir = tmp_path / "images"
    img_dir.mkdir()
    H, W = 40, 60
    yy, xx = np.mgrid[0:H, 0:W]
    Image.fromarray((50 + 2 * xx + yy).astype(np.uint8), mode="L").save(img_dir / "a.png")
    Image.fromarray(np.full((H, W), 7, np.uint8), mode="L").save(img_dir / "b.png")
    coco = {
        "images": [{"id": 1, "file_name": "a.png", "height": H, "width": W},
                   {"id": 2, "file_name": "b.png", "height": H, "width": W},
                   {"id": 3, "file_name": "missing.png", "height": H, "width": W}],
        "annotations": [
            {"id": 10, "image_id": 1, "segmentation": [[10, 8, 29, 8, 29, 23, 10, 23]]},  # x 10..29, y 8..23
            {"id": 11, "image_id": 1, "segmentation": [[40, 30, 44, 30]]},               # < 3 points: ignored
            {"id": 12, "image_id": 3, "segmentation": [[0, 0, 5, 0, 5, 5]]},
        ],
    }
    ann = tmp_path / "ann.json"
    ann.write_text(json.dumps(coco))
    return img_dir, ann


def test_coco_square_mask_after_nearest_resize(tmp_path, capsys):
    img_dir, ann = _write(tmp_path)
    ds = CellSegmentationDataset(img_dir, ann, image_size=(30, 20))  # PIL size = (W, H)
    out = capsys.readouterr().out
    assert "1 image(s) referenced in annotations but not found on disk" in out and "missing.png" in out
    assert len(ds) == 1  # image 2 has no annotation, image 3 is missing
    image, mask = ds[0]
    assert image.shape == (1, 20, 30) and mask.shape == (1, 20, 30)
    assert image.dtype == torch.float32 and mask.dtype == torch.float32
    expect = np.zeros((20, 30), np.float32)
    # target (i, j) samples source (2 i + 1, 2 j + 1): inside for 8 <= 2i+1 <= 23, 10 <= 2j+1 <= 29
    expect[4:12, 5:15] = 1.0
    np.testing.assert_array_equal(mask[0].numpy(), expect)
    # per-image min-max of the bilinear-resized image (src/dataset.py:82)
    a = image[0].numpy()
    assert a.min() == pytest.approx(0.0, abs=1e-6) and a.max() == pytest.approx(1.0, abs=1e-6)
    ref = np.asarray(Image.open(img_dir / "a.png").convert("L").resize((30, 20), resample=Image.BILINEAR),
                     np.float32)
    np.testing.assert_allclose(a, (ref - ref.min()) / (ref.max() - ref.min() + 1e-8), rtol=0, atol=1e-7)


def test_coco_full_resolution_mask_is_the_filled_polygon(tmp_path):
    img_dir, ann = _write(tmp_path)
    ds = CellSegmentationDataset(img_dir, ann, image_size=(60, 40))  # no resize
    _, mask = ds[0]
    expect = np.zeros((40, 60), np.float32)
    expect[8:24, 10:30] = 1.0  # fill and outline, both ends inclusive
    np.testing.assert_array_equal(mask[0].numpy(), expect)


def test_coco_transform_applies_to_both(tmp_path):
    img_dir, ann = _write(tmp_path)
    ds = CellSegmentationDataset(img_dir, ann, image_size=(30, 20), transform=lambda x: x.flip(-1))
    _, mask = ds[0]
    expect = np.zeros((20, 30), np.float32)
    expect[4:12, 30 - 15:30 - 5] = 1.0
    np.testing.assert_array_equal(mask[0].numpy(), expect)
