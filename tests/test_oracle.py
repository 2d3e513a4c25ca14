"""Oracle pinning (CPU): the restatement reproduces the one-shot observation of
the real reference and the analytic KATs;
the hand-derived loss backward matches float64 autograd."""
import math

import numpy as np
import pytest
import torch

from oracle import loss_numpy as ln
from oracle import reference_torch as rt

PDE_KW = dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05)


def test_pinned_reference_observation():
    # torch 2.10 CPU, B=2 256x256 seed-42 discs, UNet(1,1,64).eval() after manual_seed(42)
    img, mask = rt.synthetic_batch(2, 256, 256, seed=42)
    assert mask.mean().item() == 0.10665130615234375
    torch.manual_seed(42)
    net = rt.UNetRef(1, 1, 64).eval()
    assert rt.count_parameters(net) == 20_543_809
    with torch.no_grad():
        u = net(img)
    assert u.min().item() == pytest.approx(0.5088648, rel=1e-6)
    assert u.max().item() == pytest.approx(0.5125621, rel=1e-6)
    assert u.mean().item() == pytest.approx(0.5106269, rel=1e-6)
    assert rt.loss_terms(u, mask)["loss"].item() == pytest.approx(0.7670366764, rel=1e-7)
    t2 = rt.loss_terms(u, mask, **PDE_KW)
    assert t2["loss"].item() == pytest.approx(0.7671615481, rel=1e-7)
    assert t2["pde_loss"].item() == pytest.approx(2.58888e-05, rel=1e-5)
    assert t2["phase_field_loss"].item() == pytest.approx(1.24887013, rel=1e-7)
    assert rt.dice_score(u, mask).item() == pytest.approx(0.19274600, rel=1e-6)
    assert rt.rd_loss(mask, 5.0, 0.5).item() == pytest.approx(1.025390625, rel=1e-7)
    assert rt.pf_loss(mask, 0.05).item() == pytest.approx(1.6098024e-04, rel=1e-6)


def test_state_dict_keys_match_reference_layout():
    net = rt.UNetRef()
    sd = net.state_dict()
    assert "enc1.conv.0.weight" in sd and "enc1.conv.2.weight" in sd
    assert "enc2.conv.3.weight" in sd and "bottleneck.conv.3.bias" in sd
    assert "dec1.conv.2.weight" in sd
    assert tuple(sd["up4.weight"].shape) == (512, 512, 2, 2)
    assert tuple(sd["out_conv.weight"].shape) == (1, 64, 1, 1)


# --- analytic known-answer tests, SURVEY.md §4 ---------------------------------

def test_kat_constant_field():
    for c, a, eps, rd, pf in ((0.5, 0.5, 0.05, 0.0, 1.25), (0.25, 0.5, 0.05, 0.002197265625, 0.703125)):
        u = torch.full((2, 1, 9, 11), c, dtype=torch.float64)
        assert torch.all(rt.laplacian(u) == 0)
        assert torch.all(rt.grad_mag_sq(u) == 0)
        assert rt.rd_loss(u, 3.0, a).item() == pytest.approx(rd, rel=1e-12, abs=1e-15)
        assert rt.pf_loss(u, eps).item() == pytest.approx(pf, rel=1e-12)


def test_kat_quadratic_along_width():
    W = 11
    j = torch.arange(W, dtype=torch.float64)
    u = (j ** 2).expand(1, 1, 7, W).clone()
    lap = rt.laplacian(u)[0, 0]
    assert torch.all(lap[:, :-1] == 2.0)
    assert torch.all(lap[:, -1] == -4 * W + 6)
    np.testing.assert_allclose(ln.stencil(u[:, 0].numpy(), ln._LAP), lap[None].numpy())


def test_kat_ramp_gradient():
    H, W, h, eps = 6, 10, 0.05, 0.05
    u = (h * torch.arange(W, dtype=torch.float64)).expand(1, 1, H, W).clone()
    gx = rt._stencil(u, rt._GX)[0, 0]
    assert torch.allclose(gx[:, 1:-1], torch.full_like(gx[:, 1:-1], h))
    assert torch.all(gx[:, 0] == 0) and torch.all(gx[:, -1] == 0)
    assert torch.all(rt._stencil(u, rt._GY) == 0)
    expect = (eps / 2) * h * h * (W - 2) / W + (1 / eps) * torch.mean(u ** 2 * (1 - u) ** 2).item()
    assert rt.pf_loss(u, eps).item() == pytest.approx(expect, rel=1e-12)


def test_kat_bce_dice():
    p = torch.full((1, 1, 4, 4), 0.5)
    t = (torch.arange(16).reshape(1, 1, 4, 4) % 2).float()
    assert rt.bce_loss(p, t).item() == pytest.approx(math.log(2), rel=1e-6)
    assert rt.bce_loss(t, t).item() == 0.0
    assert rt.dice_loss(t, t).item() == pytest.approx(0.0, abs=1e-6)


# --- numpy restatement vs torch (forward) and vs float64 autograd (backward) ----

@pytest.mark.parametrize("shape", [(2, 1, 9, 11), (1, 1, 2, 3), (3, 1, 16, 5)])
@pytest.mark.parametrize("kw", [dict(), PDE_KW, dict(rd_w=1e-3, D=0.5, a=0.3), dict(pf_w=0.3, eps=0.2)])
def test_numpy_loss_matches_torch_autograd(shape, kw):
    g = torch.Generator().manual_seed(7)
    p = (0.02 + 0.96 * torch.rand(shape, generator=g, dtype=torch.float64)).requires_grad_(True)
    t = (torch.rand(shape, generator=g, dtype=torch.float64) > 0.6).double()
    terms = rt.loss_terms(p, t, **kw)
    terms["loss"].backward()
    f = ln.loss_forward(p.detach().numpy(), t.numpy(), **kw)
    for k in ("loss", "dice_loss", "bce_loss"):
        assert f[k] == pytest.approx(terms[k].item(), rel=1e-12)
    for k in ("pde_loss", "phase_field_loss"):
        if k in terms:
            assert f[k] == pytest.approx(terms[k].item(), rel=1e-12)
    gb = ln.loss_backward(p.detach().numpy(), t.numpy(), **kw)
    np.testing.assert_allclose(gb, p.grad.numpy(), rtol=1e-10, atol=1e-14)


def test_numpy_chain_sigmoid():
    g = torch.Generator().manual_seed(3)
    z = torch.randn(2, 1, 7, 6, generator=g, dtype=torch.float64, requires_grad=True)
    t = (torch.rand(2, 1, 7, 6, generator=g, dtype=torch.float64) > 0.5).double()
    p = torch.sigmoid(z)
    rt.loss_terms(p, t, **PDE_KW)["loss"].backward()
    gz = ln.loss_backward(p.detach().numpy(), t.numpy(), chain_sigmoid=True, **PDE_KW)
    np.testing.assert_allclose(gz, z.grad.numpy(), rtol=1e-10, atol=1e-14)


def test_counts_match_metric_restatement():
    img, mask = rt.synthetic_batch(3, 32, 48, seed=5)
    p = torch.sigmoid(4 * (img - 0.5))
    inter, phat, tsum = ln.sample_counts(p.numpy(), mask.numpy())
    dice, iou = ln.dice_iou_from_counts(inter, phat, tsum)
    np.testing.assert_allclose(dice, rt.dice_score_batch(p, mask).numpy(), rtol=1e-6)
    np.testing.assert_allclose(iou, rt.iou_batch(p, mask).numpy(), rtol=1e-6)


def test_decision_conditioned_forward_matches_free_forward():
    # pinning ReLU masks / pool argmaxes to the oracle's own decisions is the identity,
    # and decision_flips() reports none (the mechanism the GPU gradient test relies on)
    torch.manual_seed(3)
    m = rt.UNetRef(1, 1, 8).double().eval()
    x = torch.rand(2, 1, 32, 32, dtype=torch.float64)
    rec = {}
    p_free = rt.unet_forward(m, x, record=rec)
    dec = {}
    for k, v in rec.items():
        if k.startswith("pool"):
            B, C, H, W = v.shape
            win = v.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
            dec[k] = win.argmax(-1)
        else:
            dec[k] = v > 0
    assert len(dec) == 22
    rec2 = {}
    p_pin = rt.unet_forward(m, x, decisions=dec, record=rec2)
    assert torch.equal(p_free, p_pin)
    assert all(n == 0 for n, _ in rt.decision_flips(dec, rec2).values())
    flipped = dict(dec)
    flipped["enc2.0"] = dec["enc2.0"].clone()
    flipped["enc2.0"].view(-1)[0] ^= True
    n, margin = rt.decision_flips(flipped, rec2)["enc2.0"]
    assert n == 1 and margin > 0


def test_chunked_truth_equals_whole_truth():
    """rt.chunked_truth (the C5 B = 8 float64 truth: per-chunk forward / backward, whole-batch loss
    and dL/dp) equals rt.whole_truth on a batch both fit: probabilities, logits, every term and
    every parameter gradient, and the same decision-flip / near-tie counts. Decisions are the fp32
    oracle's own (a stand-in for a HIP run's), so some sites differ from float64's."""
    B, H, W = 3, 32, 32
    img, mask = rt.synthetic_batch(B, H, W, seed=3)
    torch.manual_seed(3)
    ref = rt.UNetRef(1, 1, 64).train()
    scales = rt.make_drop_scales(ref, B, torch.Generator().manual_seed(3))
    rec32 = {}
    with torch.no_grad():
        rt.unet_forward(ref, img, scales, record=rec32)
    decisions = {}
    for k, v in rec32.items():
        if k.startswith("pool"):
            b, c, h, w = v.shape
            win = v.reshape(b, c, h // 2, 2, w // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(b, c, h // 2, w // 2, 4)
            decisions[k] = win.argmax(-1)
        else:
            decisions[k] = v > 0
    kws = [dict(rd_w=1e-2, pf_w=1e-2, D=5.0, a=0.5, eps=0.05), dict(rd_w=1e-3, D=100.0, a=0.5)]
    p_w, z_w, f_w, t_w = rt.whole_truth(ref, img, mask, scales, decisions, kws)
    p_c, z_c, f_c, t_c = rt.chunked_truth(ref, img, mask, scales, decisions, kws, chunk=2)
    assert torch.allclose(p_w, p_c, rtol=0, atol=1e-15) and torch.allclose(z_w, z_c, rtol=0, atol=1e-13)
    assert {k: (v[0], v[2]) for k, v in f_w.items()} == {k: (v[0], v[2]) for k, v in f_c.items()}
    for (tw, gw), (tc, gc) in zip(t_w, t_c):
        for k in tw:
            assert abs(tw[k] - tc[k]) <= 1e-12 * max(abs(tw[k]), 1e-30), k
        for n in gw:
            assert ((gc[n] - gw[n]).norm() / gw[n].norm().clamp_min(1e-300)).item() < 1e-10, n
