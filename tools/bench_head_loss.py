"""Fused head + loss forward (pis_head_loss_fwd) micro-benchmark at C2 (B=8, 512x512, 64-channel head
input, Stage-II weights): per variant (pis_tune key 38, key 36 rows) the call (HIP events around the
C-ABI call: kernel + any finalize launch) and the kernel alone (launch hook), each after a 1 GiB read
so the head input comes from HBM as in the step; algorithmic bytes 4 C + 12 B/px.

    python tools/bench_head_loss.py [--B 8] [--H 512] [--W 512] [--reps 20] [--variants 1,3,3:16]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402
from physics_informed_image_segmentation_amd._hip import LossParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=8)
    ap.add_argument("--H", type=int, default=512)
    ap.add_argument("--W", type=int, default=512)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="1,2,1,2", help="key38[:key36] list")
    ap.add_argument("--probe", action="store_true", help="also time pis_debug_band_probe: sweep vs band order")
    args = ap.parse_args()
    lib = _hip.lib()
    if args.probe:
        probe(lib, args.reps)
    B, H, W, C = args.B, args.H, args.W, 64
    g = torch.Generator().manual_seed(3)
    x = torch.relu(torch.randn(B, H, W, C, generator=g)).cuda()
    w = (torch.randn(C, generator=g) * 0.15).cuda()
    bias = torch.tensor([-0.3]).cuda()
    t = (torch.rand(B, H, W, generator=g) > 0.8).float().cuda()
    z, u = torch.empty(B, H, W, device="cuda"), torch.empty(B, H, W, device="cuda")
    terms = torch.empty(8, device="cuda")
    counts = torch.empty(B, 3, dtype=torch.int32, device="cuda")
    scores = torch.empty(B, 2, device="cuda")
    nws = lib.pis_head_loss_fwd_ws(B, H, W)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    prm = LossParams(0.5, 0.5, 1e-4, 1e-4, 1e-6, 5.0, 0.5, 0.05, 0.5, 0)
    flush = torch.ones(256 << 20, device="cuda")
    sink = torch.empty((), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    nbytes = B * H * W * (4.0 * C + 12.0)
    kev = []

    def hook(kernel, phase, stream, flop):
        if kernel == "head_loss_fwd":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            kev.append(ev)

    _hip.set_launch_hook(hook)
    for var in args.variants.split(","):
        k38, _, k36 = var.partition(":")
        p38 = lib.pis_tune(38, int(k38))
        p36 = lib.pis_tune(36, int(k36 or 0))
        try:
            call, kern = [], []
            for rep in range(args.reps + 2):
                torch.sum(flush, dim=0, out=sink)
                kev.clear()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.pis_head_loss_fwd(x.data_ptr(), C, w.data_ptr(), bias.data_ptr(), t.data_ptr(), z.data_ptr(),
                                           u.data_ptr(), B, H, W, C, ctypes.byref(prm), terms.data_ptr(),
                                           counts.data_ptr(), scores.data_ptr(), ws.data_ptr(), nws, st)
                e1.record()
                if rc != 0:
                    raise RuntimeError(lib.pis_last_error().decode())
                torch.cuda.synchronize()
                if rep >= 2:
                    call.append(e0.elapsed_time(e1))
                    kern.append(kev[0].elapsed_time(kev[1]))
            mc, mk = statistics.median(call), statistics.median(kern)
            print(f"key38={k38} key36={k36 or 0}: call {mc * 1e3:7.1f} us ({nbytes / mc / 1e9 / 8:.3f} of 8 TB/s)  "
                  f"kernel {mk * 1e3:7.1f} us ({nbytes / mk / 1e9 / 8:.3f})  loss {terms[0].item():.7f}", flush=True)
        finally:
            lib.pis_tune(38, p38)
            lib.pis_tune(36, p36)
    _hip.set_launch_hook(None)


def probe(lib, reps):
    """The head input's bytes (537 MB at C2) read in sweep order vs one contiguous run per block."""
    n = 8 * 512 * 512 * 64
    a = torch.ones(n, device="cuda")
    flush = torch.ones(256 << 20, device="cuda")
    sink = torch.empty((), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for grid in (256, 512):
        part = torch.empty(grid * 16, device="cuda")
        for mode in (0, 1, 0, 1):
            ts = []
            for _ in range(reps):
                torch.sum(flush, dim=0, out=sink)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if lib.pis_debug_band_probe(a.data_ptr(), n, mode, part.data_ptr(), grid, st) != 0:
                    raise RuntimeError(lib.pis_last_error().decode())
                e1.record()
                ts.append((e0, e1))
            torch.cuda.synchronize()
            ms = statistics.median(x.elapsed_time(y) for x, y in ts)
            print(f"band probe grid {grid} mode {'sweep' if mode == 0 else 'band '}: {ms * 1e3:7.1f} us "
                  f"{4.0 * n / ms / 1e6:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
