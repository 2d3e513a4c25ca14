"""Data feeding the step (src/dataset.py:9-118).

``CellSegmentationDataset`` restates the reference loader's behaviour (COCO
polygons filled with PIL, NEAREST mask resize, bilinear image resize,
per-image min-max) — host-side, outside the kernel path.
``SyntheticDiscDataset`` is the benchmark/parity generator of SURVEY.md
§8(c)-(d): per-sample union of random discs, noisy image, min-max.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Tuple

import numpy as np
import torch
from torch.utils.data import Dataset


class CellSegmentationDataset(Dataset):
    def __init__(self, image_dir, annotation_file, image_size=(128, 128), transform=None):
        self.image_dir = Path(image_dir).resolve()
        self.image_size = tuple(image_size)
        self.transform = transform
        with open(Path(annotation_file).resolve(), "r") as f:
            coco = json.load(f)
        self.images_dict = {img["id"]: img for img in coco["images"]}
        self.anns_by_image = {}
        for ann in coco["annotations"]:
            self.anns_by_image.setdefault(ann["image_id"], []).append(ann)
        self.image_ids, missing = [], []
        for img_id, info in self.images_dict.items():
            if img_id not in self.anns_by_image:
                continue
            if (self.image_dir / info["file_name"]).exists():
                self.image_ids.append(img_id)
            else:
                missing.append(info["file_name"])
        if missing:
            print(f"Warning: {len(missing)} image(s) referenced in annotations but not found on disk:")
            for name in missing[:10]:
                print(f"  - {name}")
            if len(missing) > 10:
                print(f"  ... and {len(missing) - 10} more")
            print(f"These images will be skipped. Dataset size: {len(self.image_ids)}")

    def __len__(self):
        return len(self.image_ids)

    def _mask(self, anns, hw, size):
        from PIL import Image, ImageDraw
        H, W = hw
        canvas = Image.new("L", (W, H), 0)
        draw = ImageDraw.Draw(canvas)
        for ann in anns:
            seg = ann.get("segmentation", [])
            if isinstance(seg, list):
                for poly in seg:
                    if len(poly) >= 6:
                        draw.polygon(np.asarray(poly).reshape(-1, 2).flatten().tolist(), outline=1, fill=1)
        canvas = canvas.resize(size, resample=Image.NEAREST)
        return (np.asarray(canvas, dtype=np.float32) > 0).astype(np.float32)

    def __getitem__(self, idx):
        from PIL import Image
        image_id = self.image_ids[idx]
        info = self.images_dict[image_id]
        img = Image.open(self.image_dir / info["file_name"]).convert("L")
        img = np.asarray(img.resize(self.image_size, resample=Image.BILINEAR), dtype=np.float32)
        mask = self._mask(self.anns_by_image[image_id], (info["height"], info["width"]), self.image_size)
        img = (img - img.min()) / (img.max() - img.min() + 1e-8)
        image = torch.from_numpy(img).unsqueeze(0)
        mask_t = torch.from_numpy(mask).unsqueeze(0)
        if self.transform is not None:
            image, mask_t = self.transform(image), self.transform(mask_t)
        return image, mask_t


def disc_sample(H: int, W: int, g: torch.Generator) -> Tuple[torch.Tensor, torch.Tensor]:
    """One (image, mask) pair of the SURVEY.md §8(c) generator."""
    rows, cols = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    n = int(torch.randint(5, 15, (1,), generator=g))
    cx = torch.rand(n, generator=g) * W
    cy = torch.rand(n, generator=g) * H
    rad = (0.03 + 0.07 * torch.rand(n, generator=g)) * min(H, W)
    inside = torch.zeros(H, W, dtype=torch.bool)
    for k in range(n):
        inside |= (cols - cx[k]) ** 2 + (rows - cy[k]) ** 2 <= rad[k] ** 2
    mask = inside.float()[None]
    img = 0.2 + 0.6 * mask + 0.1 * torch.randn(1, H, W, generator=g)
    img = (img - img.min()) / (img.max() - img.min() + 1e-8)
    return img, mask


class SyntheticDiscDataset(Dataset):
    """Deterministic synthetic cell-like masks: sample i is drawn from its own
    generator seeded ``seed * 1_000_003 + i`` (shard-independent)."""

    def __init__(self, n: int, image_size=(512, 512), seed: int = 42):
        self.n, self.size, self.seed = n, tuple(image_size), seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        return disc_sample(self.size[0], self.size[1], g)
