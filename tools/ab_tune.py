"""A/B of pis_tune settings on the C2 training step, interleaved rounds in one process on one
GPU (box-to-box variance is ~3 %; same-process interleaving is not).

    python tools/ab_tune.py --variants "base;20=0;15=0,17=4" [--rounds 4] [--steps 10] [--shared]

Each variant is a comma list of KEY=VALUE (include/pis_capi.h PIS_TUNE_*); "base" = defaults;
"fa=0..5" plans that variant's engine with PIS_FILTER_AHEAD = that value, "dwm=0|1" runs the direct
layers' weight gradients on the main stream (PIS_DIRECT_WGRAD_MAIN; unet.py).
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import AdamW, DiceBCEPDELoss, UNet, _hip  # noqa: E402
from physics_informed_image_segmentation_amd.dataset import disc_sample  # noqa: E402


def parse(v):
    if v.strip() in ("", "base"):
        return {}
    return {(k if k in HOST else int(k)): (x if k in HOST else int(x)) for k, x in (kv.split("=") for kv in v.split(","))}


# host-side engine attributes a variant may set (unet.UNetEngine): fa = filter_ahead, dwm =
# direct_wgrad_main, ss = side_sync (prep / gemm / dgrad)
HOST = {"fa": "filter_ahead", "dwm": "direct_wgrad_main", "ss": "side_sync", "fwm": "fused_wgrad_main",
        "cwm": "convt_wgrad_main"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--shared", action="store_true",
                    help="one model (planned with the defaults) for every variant: for knobs that do not change "
                         "the engine's plan; removes the 2-3 %% placement effect of separately allocated models")
    args = ap.parse_args()
    lib = _hip.lib()
    variants = [(v.strip(), parse(v)) for v in args.variants.split(";")]
    keys = sorted({k for _, kv in variants for k in kv if k not in HOST})
    defaults = {k: lib.pis_tune(k, -1) for k in keys}
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(42)
    imgs, masks = zip(*[disc_sample(512, 512, g) for _ in range(8)])
    x, t = torch.stack(imgs).to(dev), torch.stack(masks).to(dev)
    crit = DiceBCEPDELoss(pde_weight=1e-4, phase_field_weight=1e-4, diffusion_coeff=5.0, epsilon=0.05)

    def setv(kv):
        for k in keys:
            lib.pis_tune(k, kv.get(k, defaults[k]))

    # one model (and engine plan: workspaces depend on the knobs) per variant, same seed
    models = {}
    for name, kv in variants:
        if args.shared and models:
            models[name] = next(iter(models.values()))
            continue
        setv({} if args.shared else kv)
        torch.manual_seed(42)
        m = UNet(1, 1, 64).to(dev).train()
        models[name] = (m, AdamW(m.parameters(), lr=1e-5, weight_decay=1e-5))

    from physics_informed_image_segmentation_amd.unet import UNetEngine
    host_default = {k: getattr(UNetEngine, a) for k, a in HOST.items()}

    def step(name):
        model, opt = models[name]
        for k, a in HOST.items():
            setattr(UNetEngine, a, str(dict(variants)[name].get(k, host_default[k])))
        opt.zero_grad()
        model.forward_with_loss(x, t, crit)[1].backward()  # the step as bench.py / train_epoch run it
        opt.step()

    def run(name, kv):
        setv(kv)
        step(name)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(name)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3

    res = {}
    for _ in range(args.rounds):
        for name, kv in variants:
            res.setdefault(name, []).append(run(name, kv))
    for k in keys:
        lib.pis_tune(k, defaults[k])
    for name, ms in res.items():
        ms.sort()
        med = ms[len(ms) // 2]
        print(f"{name:16s} ms/step median {med:.2f}  min {ms[0]:.2f}  -> {8e3 / med:.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
