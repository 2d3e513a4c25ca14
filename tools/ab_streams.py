"""A/B of the step's stream arrangement on one GPU (C2 shape), interleaved rounds in one process
(cdna_hip_programming.md §5.4 rule 24):
  default   : main = torch's current stream, weight gradients on a side stream (priority 0)
  main_hi   : the whole step inside a high-priority stream, side stream at normal priority
  side_hi   : the weight-gradient side stream at high priority (its blocks dispatch first whenever a
              CU frees up: the fused contraction kernels fill every CU's registers and LDS)
  serial    : weight gradients serialised on the main stream (no side stream)
  sync_gemm : a prepared layer's weight gradient waits for the input gradient's contractions
  sync_dgrad: ... waits for the whole input gradient (PIS_SIDE_SYNC, unet.py conv_bwd)

    python tools/ab_streams.py [--rounds 4] [--steps 10]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import AdamW, DiceBCEPDELoss, UNet  # noqa: E402
from physics_informed_image_segmentation_amd.dataset import disc_sample  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE")
    ap.add_argument("--variants", default="default,side_hi,main_hi,serial,sync_gemm,sync_dgrad")
    args = ap.parse_args()
    from physics_informed_image_segmentation_amd import _hip
    for kv in args.tune:
        k, v = (int(z) for z in kv.split("="))
        _hip.lib().pis_tune(k, v)
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(42)
    imgs, masks = zip(*[disc_sample(512, 512, g) for _ in range(8)])
    x, t = torch.stack(imgs).to(dev), torch.stack(masks).to(dev)
    torch.manual_seed(42)
    model = UNet(1, 1, 64).to(dev).train()
    crit = DiceBCEPDELoss(pde_weight=1e-4, phase_field_weight=1e-4, diffusion_coeff=5.0, epsilon=0.05)
    opt = AdamW(model.parameters(), lr=1e-5, weight_decay=1e-5)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    hi_stream = torch.cuda.Stream(priority=hi)
    side_hi = torch.cuda.Stream(priority=hi)
    print(f"stream priority range (low, high) = ({lo}, {hi})", flush=True)

    def step():
        opt.zero_grad()
        model.forward_with_loss(x, t, crit)[1].backward()  # the step as bench.py runs it
        opt.step()

    step()  # plans the engine (buffers, side stream)
    torch.cuda.synchronize()

    def run(variant):
        eng = model.engine()
        side, sync = eng.side, eng.side_sync
        if variant.startswith("sync_"):
            eng.side_sync = variant[5:]
        if variant == "serial":
            eng.side = None
        if variant == "side_hi":
            eng.side = side_hi
        ctx = torch.cuda.stream(hi_stream) if variant == "main_hi" else torch.cuda.stream(torch.cuda.current_stream())
        with ctx:
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        eng.side, eng.side_sync = side, sync
        return dt / args.steps * 1e3

    res = {}
    for _ in range(args.rounds):
        for v in args.variants.split(","):
            res.setdefault(v, []).append(run(v))
    for v, ms in res.items():
        ms.sort()
        print(f"{v:10s} ms/step median {ms[len(ms) // 2]:.2f}  min {ms[0]:.2f}  -> {8e3 / ms[len(ms) // 2]:.1f} img/s",
              flush=True)


if __name__ == "__main__":
    main()
