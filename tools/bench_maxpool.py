"""Time pis_maxpool2x2_bwd at the C2 encoder shapes (B = 8, 512^2 / 64 ch down to 64^2 / 512 ch):
median of 50 launches, the algorithmic bytes (x, dskip, dx at full resolution + dy) and the HBM
fraction of 8 TB/s. (Round 4 timed a two-lanes-per-pooled-pixel form beside it with this tool,
profiles/r4_ad_maxpool_bwd_pairs.txt: equal, not kept.)

    python tools/bench_maxpool.py
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402


def main():
    argparse.ArgumentParser(description=__doc__).parse_args()
    lib = _hip.lib()
    s = torch.cuda.current_stream().cuda_stream
    for H, C in ((512, 64), (256, 128), (128, 256), (64, 512)):
        B, W = 8, H
        x = torch.relu(torch.randn(B, H, W, C, device="cuda"))
        dy = torch.randn(B, H // 2, W // 2, C, device="cuda")
        dsk = torch.randn(B, H, W, C, device="cuda")
        dx = torch.empty(B, H, W, C, device="cuda")
        nbytes = 4 * (3 * x.numel() + dy.numel())
        ts = []
        for _ in range(60):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            rc = lib.pis_maxpool2x2_bwd(x.data_ptr(), C, dy.data_ptr(), dsk.data_ptr(), C, dx.data_ptr(), C,
                                        B, H, W, C, s)
            b.record()
            assert rc == 0
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ms = sorted(ts[10:])[len(ts[10:]) // 2]
        print(f"{H:4d}^2 x {C:3d} ch: {ms * 1e3:7.1f} us {nbytes / ms / 1e9:6.2f} TB/s ({nbytes / ms / 1e9 / 8:.2f})",
              flush=True)


if __name__ == "__main__":
    main()
