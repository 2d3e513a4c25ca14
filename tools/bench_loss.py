"""Fused PDE-loss kernel micro-benchmark (C2: B=8, 512x512, Stage-II weights).

Times pis_loss_fwd (one launch: whole-row bands, the last block reduces) and pis_loss_bwd with HIP events and
prints algorithmic HBM GB/s: forward reads p and t (8 B/px), backward reads p, t
and writes dL/dz (12 B/px).

    python tools/bench_loss.py [--B 8] [--H 512] [--W 512] [--reps 50]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--W", type=int, default=512)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rd", type=float, default=1e-4)
    ap.add_argument("--pf", type=float, default=1e-4)
    ap.add_argument("--modes", default="", help="comma list of PIS_TUNE_LOSS_ROWS[:ROWMUL] values to time")
    args = ap.parse_args()
    lib = _hip.lib()
    for mode in [m for m in args.modes.split(",") if m] or [None]:
        if mode is not None:
            rows, _, mul = mode.partition(":")
            lib.pis_tune(18, int(rows))
            lib.pis_tune(19, int(mul or 1))
            print(f"-- PIS_TUNE_LOSS_ROWS = {rows}, ROWMUL = {mul or 1}", flush=True)
        run(lib, args, fwd_only=mode is not None)


def run(lib, args, fwd_only=False):
    B, H, W = args.B, args.H, args.W
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device="cuda").manual_seed(0)
    p = torch.sigmoid(torch.randn(B, H, W, device="cuda", generator=g))
    t = (torch.rand(B, H, W, device="cuda", generator=g) > 0.9).float()
    prm = _hip.LossParams(0.5, 0.5, args.rd, args.pf, 1e-6, 5.0, 0.5, 0.05, 0.5, 0)
    terms = torch.empty(8, device="cuda")
    counts = torch.empty(B, 3, dtype=torch.int32, device="cuda")
    scores = torch.empty(B, 2, device="cuda")
    nws = lib.pis_loss_ws(B, H, W)
    ws = torch.zeros(nws // 4 + 1, device="cuda")
    dst = torch.empty(B, H, W, device="cuda")
    # 1 GiB READ between reps: evicts L2 + Infinity Cache with clean lines (a write-flush leaves
    # ~256 MB of dirty lines whose write-back then competes with the timed kernel)
    flush = torch.ones(256 << 20, device="cuda")
    sink = torch.empty((), device="cuda")

    def fwd():
        lib.pis_loss_fwd(p.data_ptr(), t.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(),
                         counts.data_ptr(), scores.data_ptr(), ws.data_ptr(), nws, s)

    def bwd():
        lib.pis_loss_bwd(p.data_ptr(), t.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(), 0,
                         dst.data_ptr(), 2, s)

    npx = B * H * W
    for name, fn, nbytes in (("loss_fwd", fwd, 8 * npx), ("loss_bwd", bwd, 12 * npx))[:1 if fwd_only else 2]:
        for cold in (False, True):
            fn()
            ms = []
            for _ in range(args.reps):
                if cold:
                    torch.sum(flush, dim=0, out=sink)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                ms.append((e0, e1))
            torch.cuda.synchronize()
            t_ms = sorted(a.elapsed_time(b) for a, b in ms)[len(ms) // 2]
            print(f"{name:18s} {'cold' if cold else 'warm'}: {t_ms * 1e3:7.1f} us  "
                  f"{nbytes / t_ms / 1e6:7.1f} GB/s ({nbytes / t_ms / 1e6 / 8000 * 100:.0f}% of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
