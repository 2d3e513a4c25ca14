"""Generate the committed golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_golden.py``). Test infrastructure only.

* reference_observation.json — the one observation of the REAL reference made before
  importing it was refused; copied from there, not regenerated.
* loss_cases.npz — float64 oracle (oracle/loss_numpy.py) loss terms, dL/dp and exact
  per-sample metric counters for seeded (p, t) pairs: ragged widths, tiny reflect-padded
  images, all four R1 ablation gatings (src/loss.py:144-160, run_ablation.py:42-83).
* unet_small.npz — seed-42 UNet(1,1,64) (oracle/reference_torch.py, the reference's
  parameter creation order) on the seed-42 disc batch at B=2, 32x32, eval mode: the
  probabilities, the Stage-II loss terms, and per-parameter gradient norms/sums (float64
  oracle on its own ReLU/pool decisions).
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import loss_numpy as ln  # noqa: E402
from oracle import reference_torch as rt  # noqa: E402

LOSS_SHAPES = [(1, 1, 2, 3), (2, 1, 9, 11), (3, 1, 33, 70), (1, 1, 16, 130)]
LOSS_CONFIGS = {  # name -> kwargs of ln.loss_forward
    "baseline": dict(),
    "rd_only": dict(rd_w=1e-4, D=5.0, a=0.5),
    "pf_only": dict(pf_w=1e-4, eps=0.05),
    "rd_pf": dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05),
    "strong": dict(rd_w=0.3, pf_w=0.2, D=0.5, a=0.3, eps=0.1),
}
STAGE2 = dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05)


def loss_cases():
    out = {}
    for si, shape in enumerate(LOSS_SHAPES):
        g = torch.Generator().manual_seed(100 + si)
        p = (0.02 + 0.96 * torch.rand(shape, generator=g)).numpy().astype(np.float32)
        t = (torch.rand(shape, generator=g) > 0.7).numpy().astype(np.float32)
        out[f"s{si}_p"], out[f"s{si}_t"] = p, t
        i, ph, ts = ln.sample_counts(p, t)
        out[f"s{si}_counts"] = np.stack([i, ph, ts], 1).astype(np.int64)
        for name, kw in LOSS_CONFIGS.items():
            f = ln.loss_forward(p, t, **kw)
            out[f"s{si}_{name}_terms"] = np.array([f["loss"], f["dice_loss"], f["bce_loss"], f["rd"], f["pf"]])
            out[f"s{si}_{name}_dp"] = ln.loss_backward(p, t, **kw).astype(np.float64)
    return out


def unet_small():
    img, mask = rt.synthetic_batch(2, 32, 32, seed=42)
    torch.manual_seed(42)
    net = rt.UNetRef(1, 1, 64).double().eval()
    u = net(img.double())
    terms = rt.loss_terms(u, mask.double(), **STAGE2)
    terms["loss"].backward()
    names = [n for n, _ in net.named_parameters()]
    return {
        "img": img.numpy(), "mask": mask.numpy(), "u": u.detach().numpy(),
        "terms": np.array([terms[k].item() for k in ("loss", "dice_loss", "bce_loss", "pde_loss", "phase_field_loss")]),
        "param_names": np.array(names),
        "grad_norm": np.array([p.grad.norm().item() for p in net.parameters()]),
        "grad_sum": np.array([p.grad.sum().item() for p in net.parameters()]),
    }


def main():
    np.savez_compressed(os.path.join(HERE, "loss_cases.npz"), **loss_cases())
    np.savez_compressed(os.path.join(HERE, "unet_small.npz"), **unet_small())
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
