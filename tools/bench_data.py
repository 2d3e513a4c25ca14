"""Input-pipeline rate at C2 (B = 8, 512^2): the on-device disc generator
(DeviceDiscLoader / pis_synth_discs) against the host generator (SyntheticDiscDataset,
one process), images per second.

    python tools/bench_data.py [--batches 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd.dataset import DeviceDiscLoader  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--size", type=int, default=512)
    args = ap.parse_args()
    B, S = 8, args.size
    ld = DeviceDiscLoader(B * args.batches, B, (S, S), seed=42, shuffle=False, device="cuda")
    it = iter(ld)
    next(it)  # warm-up (library load, first allocation)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for img, mask in it:
        n += img.shape[0]
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    for i in range(B):
        ld.dataset[i]
    dth = time.perf_counter() - t1
    print(f"device generator: {n / dt:.1f} images/s ({dt / (n / B) * 1e3:.2f} ms per batch of {B} at {S}^2); "
          f"host generator: {B / dth:.1f} images/s (one process)")


if __name__ == "__main__":
    main()
