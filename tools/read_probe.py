"""Probe (analysis tooling): the box's streaming rate for a pure-read stream (two 256 MiB arrays,
partial sums only) and for the 2:1 read:write stream bench.py reports (hbm_probe), best over grid
sizes — the ceiling a read-dominated kernel such as the fused head + loss forward can reach."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402


def main():
    lib = _hip.lib()
    dev = torch.device("cuda")
    n = 64 << 20
    a, b, c = torch.ones(n, device=dev), torch.ones(n, device=dev), torch.empty(n, device=dev)
    part = torch.empty(1 << 16, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for name, dst, pt, nbytes in (("read-only", 0, part.data_ptr(), 8.0 * n), ("read2+write1", c.data_ptr(), 0, 12.0 * n)):
        best = None
        for grid in (256, 512, 1024, 2048, 4096, 8192, 16384):
            evs = []
            for _ in range(11):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert lib.pis_debug_stream_probe(a.data_ptr(), b.data_ptr(), dst, n, pt, grid, st) == 0
                e1.record()
                evs.append((e0, e1))
            torch.cuda.synchronize()
            ms = statistics.median(x.elapsed_time(y) for x, y in evs[1:])
            if best is None or ms < best[0]:
                best = (ms, grid)
        print(f"{name:14s} grid {best[1]:6d}  {best[0] * 1e3:7.1f} us  {nbytes / best[0] / 1e9:7.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
