"""Data feeding the step (src/dataset.py:9-118).

``CellSegmentationDataset`` restates the reference loader's behaviour (COCO
polygons filled with PIL, NEAREST mask resize, bilinear image resize,
per-image min-max) — host-side, outside the kernel path.
``SyntheticDiscDataset`` is the benchmark/parity generator of SURVEY.md
§8(c)-(d): per-sample union of random discs, noisy image, min-max;
``DeviceDiscLoader`` rasterises the same samples on the GPU (§8(f) row 1).
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


def disc_params(H: int, W: int, g: torch.Generator) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """The disc centres and radii of one sample, drawn in the generator's order."""
    n = int(torch.randint(5, 15, (1,), generator=g))
    cx = torch.rand(n, generator=g) * W
    cy = torch.rand(n, generator=g) * H
    rad = (0.03 + 0.07 * torch.rand(n, generator=g)) * min(H, W)
    return cx, cy, rad


def disc_sample(H: int, W: int, g: torch.Generator) -> Tuple[torch.Tensor, torch.Tensor]:
    """One (image, mask) pair of the SURVEY.md §8(c) generator."""
    rows, cols = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    cx, cy, rad = disc_params(H, W, g)
    inside = torch.zeros(H, W, dtype=torch.bool)
    for k in range(cx.numel()):
        inside |= (cols - cx[k]) ** 2 + (rows - cy[k]) ** 2 <= rad[k] ** 2
    mask = inside.float()[None]
    img = 0.2 + 0.6 * mask + 0.1 * torch.randn(1, H, W, generator=g)
    img = (img - img.min()) / (img.max() - img.min() + 1e-8)
    return img, mask


def _sample_generator(seed: int, idx: int) -> torch.Generator:
    return torch.Generator().manual_seed(seed * 1_000_003 + idx)


class DeviceDiscLoader:
    """Batches of the disc generator rasterised ON THE GPU (``pis_synth_discs``,
    SURVEY §8(f) row 1): only the disc parameters (<= 14 x 3 floats per sample) cross
    PCIe. Sample ``i`` uses the same generator as ``SyntheticDiscDataset`` item ``i``, so
    its mask is bit-identical to the host generator's; the image noise comes from a device
    hash of (seed, i, pixel) instead of torch.randn.

    Sharding follows ``DistributedSampler``: per epoch (``set_epoch``) a seeded
    permutation when ``shuffle``, padded to a multiple of ``world`` by repeating its head,
    rank ``r`` taking every ``world``-th index from ``r``. Iterating yields
    ``(images, masks)`` of shape (b, 1, H, W) on ``device``, already resident."""

    MAX_DISCS = 16

    def __init__(self, n: int, batch_size: int, image_size=(512, 512), seed: int = 42, shuffle: bool = True,
                 rank: int = 0, world: int = 1, device=None, drop_last: bool = False, subset=None):
        from . import _hip  # noqa: F401  (fail early when the library is missing)
        self.n, self.batch_size, self.size, self.seed = n, batch_size, tuple(image_size), seed
        self.shuffle, self.rank, self.world, self.drop_last = shuffle, rank, world, drop_last
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.epoch = 0
        self.dataset = SyntheticDiscDataset(n, image_size, seed)  # host twin (parity, len())
        self.ids = [int(i) for i in subset] if subset is not None else list(range(n))  # e.g. a train_fraction
        self._params = {}

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self):
        m = len(self.ids)
        perm = (torch.randperm(m, generator=torch.Generator().manual_seed(self.seed + self.epoch)).tolist()
                if self.shuffle else list(range(m)))
        idx = [self.ids[k] for k in perm]
        total = -(-m // self.world) * self.world
        idx += idx[:total - len(idx)]
        return idx[self.rank:total:self.world]

    def __len__(self):
        m = len(self.indices())
        return m // self.batch_size if self.drop_last else -(-m // self.batch_size)

    def _disc(self, i: int):
        p = self._params.get(i)
        if p is None:
            H, W = self.size
            cx, cy, rad = disc_params(H, W, _sample_generator(self.seed, i))
            p = torch.stack([cx, cy, rad], 1)
            self._params[i] = p
        return p

    def batch(self, ids):
        from . import _hip
        H, W = self.size
        b = len(ids)
        discs = torch.zeros(b, self.MAX_DISCS, 3)
        nd = torch.empty(b, dtype=torch.int32)
        for j, i in enumerate(ids):
            p = self._disc(i)
            discs[j, :p.shape[0]] = p
            nd[j] = p.shape[0]
        dev = self.device
        discs_d = discs.to(dev, non_blocking=True)
        nd_d = nd.to(dev, non_blocking=True)
        sid = torch.tensor(ids, dtype=torch.int64).to(dev, non_blocking=True)
        img = torch.empty(b, 1, H, W, device=dev)
        mask = torch.empty(b, 1, H, W, device=dev)
        nws = _hip.lib().pis_synth_ws(b, H, W)
        ws = torch.empty((nws + 3) // 4, device=dev)
        _hip.call("pis_synth_discs", discs_d.data_ptr(), nd_d.data_ptr(), self.MAX_DISCS, self.seed, sid.data_ptr(),
                  img.data_ptr(), mask.data_ptr(), b, H, W, ws.data_ptr(), nws, _hip.stream_handle())
        return img, mask

    def __iter__(self):
        idx = self.indices()
        bs = self.batch_size
        stop = len(idx) - (len(idx) % bs if self.drop_last else 0)
        for k in range(0, stop, bs):
            yield self.batch(idx[k:k + bs])


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
