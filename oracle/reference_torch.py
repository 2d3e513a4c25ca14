"""ORACLE (test infrastructure only) — stock-PyTorch CPU restatement of the
reference training step. Never imported by the product package.

Every function cites the reference file:line whose behaviour it restates.
Arithmetic is stock ATen on CPU (the same ops the reference calls), in the
dtype of the inputs (fp32 for parity, fp64 for gradchecks). The one exception is
the float64 truth of the full-size GPU tests (whole_truth / chunked_truth with
device="cuda"): the same float64 ops evaluated by the GPU's ATen, pinned to the
CPU evaluation by tests/test_fullsize_gpu.py::test_float64_truth_device_independent.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

# ---------------------------------------------------------------------------
# Synthetic data — SURVEY.md §8(c) generator (the one the pinned observation
# was taken on): per-sample union of random discs + noisy image, min-max.
# ---------------------------------------------------------------------------


def synthetic_batch(B: int, H: int, W: int, seed: int = 42) -> Tuple[torch.Tensor, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    rows, cols = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    masks = torch.zeros(B, 1, H, W)
    for b in range(B):
        n_discs = int(torch.randint(5, 15, (1,), generator=g))
        cx = torch.rand(n_discs, generator=g) * W
        cy = torch.rand(n_discs, generator=g) * H
        rad = (0.03 + 0.07 * torch.rand(n_discs, generator=g)) * min(H, W)
        inside = torch.zeros(H, W, dtype=torch.bool)
        for k in range(n_discs):
            inside |= (cols - cx[k]) ** 2 + (rows - cy[k]) ** 2 <= rad[k] ** 2
        masks[b, 0] = inside.float()
    img = 0.2 + 0.6 * masks + 0.1 * torch.randn(B, 1, H, W, generator=g)
    lo = img.amin(dim=(1, 2, 3), keepdim=True)
    hi = img.amax(dim=(1, 2, 3), keepdim=True)
    # src/dataset.py:82 per-image min-max normalisation
    img = (img - lo) / (hi - lo + 1e-8)
    return img, masks


# ---------------------------------------------------------------------------
# U-Net — src/unet.py:19-216. Module tree, parameter names and creation order
# match the reference exactly so torch.manual_seed(s) yields identical weights
# and state_dict keys.
# ---------------------------------------------------------------------------

# (name, cin_mult, cout_mult, dropout_mult) in creation order, src/unet.py:120-154
_BLOCKS = (
    ("enc1", None, 1, 0.0),
    ("enc2", 1, 2, 0.5),
    ("enc3", 2, 4, 1.0),
    ("enc4", 4, 8, 1.0),
    ("bottleneck", 8, 8, 1.0),
    ("dec4", 16, 8, 1.0),
    ("dec3", 8, 4, 0.5),
    ("dec2", 4, 2, 0.5),
    ("dec1", 2, 1, 0.0),
)


class _Block(nn.Module):
    """conv3x3 -> ReLU -> [Dropout2d] -> conv3x3 -> ReLU (src/unet.py:28-42)."""

    def __init__(self, cin: int, cout: int, p: float):
        super().__init__()
        act = nn.ReLU(inplace=True)
        seq: List[nn.Module] = [nn.Conv2d(cin, cout, 3, padding=1), act]
        if p > 0:
            seq.append(nn.Dropout2d(p))
        seq += [nn.Conv2d(cout, cout, 3, padding=1), act]
        self.conv = nn.Sequential(*seq)
        self.p = p

    @property
    def conv0(self) -> nn.Conv2d:
        return self.conv[0]

    @property
    def conv1(self) -> nn.Conv2d:
        return self.conv[3] if self.p > 0 else self.conv[2]


class UNetRef(nn.Module):
    """Restatement of ``UNet(in,out,base,dropout)`` (src/unet.py:108-167)."""

    def __init__(self, in_channels: int = 1, out_channels: int = 1, base_channels: int = 64,
                 dropout: float = 0.2):
        super().__init__()
        c = base_channels
        specs = {name: (cm, om, dm) for name, cm, om, dm in _BLOCKS}
        # creation order (RNG order) = enc1, enc2, enc3, enc4, bottleneck,
        # up4, dec4, up3, dec3, up2, dec2, up1, dec1, out_conv
        def blk(name):
            cm, om, dm = specs[name]
            cin = in_channels if cm is None else cm * c
            return _Block(cin, om * c, dropout * dm)
        self.enc1 = blk("enc1")
        self.enc2 = blk("enc2")
        self.enc3 = blk("enc3")
        self.enc4 = blk("enc4")
        self.pool = nn.MaxPool2d(2, 2)
        self.bottleneck = blk("bottleneck")
        self.up4 = nn.ConvTranspose2d(8 * c, 8 * c, 2, stride=2)
        self.dec4 = blk("dec4")
        self.up3 = nn.ConvTranspose2d(8 * c, 4 * c, 2, stride=2)
        self.dec3 = blk("dec3")
        self.up2 = nn.ConvTranspose2d(4 * c, 2 * c, 2, stride=2)
        self.dec2 = blk("dec2")
        self.up1 = nn.ConvTranspose2d(2 * c, c, 2, stride=2)
        self.dec1 = blk("dec1")
        self.out_conv = nn.Conv2d(c, out_channels, 1)

    def block_names(self) -> Sequence[str]:
        return [b[0] for b in _BLOCKS]

    def forward(self, x: torch.Tensor, drop_scales: Optional[Dict[str, torch.Tensor]] = None,
                return_logits: bool = False):
        return unet_forward(self, x, drop_scales, return_logits)


def _relu(pre: torch.Tensor, name: str, decisions, record) -> torch.Tensor:
    """ReLU, or — when ``decisions`` holds a mask for this site — the linear map
    pre * mask, i.e. the same network evaluated on another run's activation
    pattern (gradient parity conditioned on identical ReLU decisions)."""
    if record is not None:
        record[name] = pre.detach()
    if decisions is not None and name in decisions:
        return pre * decisions[name].to(pre.dtype)
    return F.relu(pre)


def _pool(x: torch.Tensor, name: str, decisions, record) -> torch.Tensor:
    """2x2/2 max-pool (src/unet.py:181-187), or the gather of given window argmaxes
    (index dy * 2 + dx per window) when ``decisions`` holds them for this site."""
    if record is not None:
        record[name] = x.detach()
    if decisions is not None and name in decisions:
        B, C, H, W = x.shape
        win = x.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
        return win.gather(-1, decisions[name].long().unsqueeze(-1)).squeeze(-1)
    return F.max_pool2d(x, 2, 2)


def _block_forward(blk: _Block, x: torch.Tensor, scale: Optional[torch.Tensor], training: bool,
                   name: str = "", decisions=None, record=None):
    y = _relu(F.conv2d(x, blk.conv0.weight, blk.conv0.bias, padding=1), f"{name}.0", decisions, record)
    if blk.p > 0:
        if scale is not None:  # injected Dropout2d keep-scale (B, C): 0 or 1/(1-p)
            y = y * scale[:, :, None, None].to(y.dtype)
        elif training:
            y = F.dropout2d(y, blk.p, True)
    return _relu(F.conv2d(y, blk.conv1.weight, blk.conv1.bias, padding=1), f"{name}.1", decisions, record)


def unet_forward(m: UNetRef, x: torch.Tensor, drop_scales=None, return_logits=False, decisions=None,
                 record=None):
    """src/unet.py:169-216; concat order is [upsampled, skip] (:190-202).

    ``decisions`` ({"enc1.0": relu mask, ..., "pool1": window argmax, ...}, NCHW)
    pins every ReLU / max-pool decision to another run's; ``record`` collects the
    pre-activations and pool inputs under the same keys."""
    s = drop_scales or {}
    tr = m.training
    kw = dict(decisions=decisions, record=record)
    e1 = _block_forward(m.enc1, x, s.get("enc1"), tr, "enc1", **kw)
    e2 = _block_forward(m.enc2, _pool(e1, "pool1", **kw), s.get("enc2"), tr, "enc2", **kw)
    e3 = _block_forward(m.enc3, _pool(e2, "pool2", **kw), s.get("enc3"), tr, "enc3", **kw)
    e4 = _block_forward(m.enc4, _pool(e3, "pool3", **kw), s.get("enc4"), tr, "enc4", **kw)
    bn = _block_forward(m.bottleneck, _pool(e4, "pool4", **kw), s.get("bottleneck"), tr, "bottleneck", **kw)
    d = bn
    for up, dec, skip, name in ((m.up4, m.dec4, e4, "dec4"), (m.up3, m.dec3, e3, "dec3"),
                                (m.up2, m.dec2, e2, "dec2"), (m.up1, m.dec1, e1, "dec1")):
        u = F.conv_transpose2d(d, up.weight, up.bias, stride=2)
        d = _block_forward(dec, torch.cat([u, skip], dim=1), s.get(name), tr, name, **kw)
    z = F.conv2d(d, m.out_conv.weight, m.out_conv.bias)
    p = torch.sigmoid(z)
    return (p, z) if return_logits else p


def site_maxima(record) -> Dict[str, float]:
    """max |value| per decision site of a record (the scale decision_flips / near_ties measure
    margins in); a batch evaluated in chunks takes the max over its chunks' maxima."""
    return {k: float(v.abs().max()) for k, v in record.items()}


def decision_flips(decisions, record, drop_scales=None, site_scale=None) -> Dict[str, Tuple[int, float]]:
    """Where a run's ReLU / max-pool decisions differ from the ones this oracle makes
    on ``record`` (its own pre-activations): per site (count, worst margin), the
    margin being |pre-activation| for a ReLU and the gap between the window max and
    the chosen element for a pool, relative to the site's max |value| (``site_scale``
    overrides it: a chunk of a batch measured in the whole batch's scale). Channels a
    Dropout2d keep-scale zeroes (``drop_scales``) carry no decision and are skipped."""
    out = {}
    drop_scales = drop_scales or {}
    for name, dec in decisions.items():
        ref = record[name]
        scale = ref.abs().max().clamp_min(1e-30) if site_scale is None else max(site_scale[name], 1e-30)
        if name.startswith("pool"):
            B, C, H, W = ref.shape
            win = ref.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
            chosen = win.gather(-1, dec.long().unsqueeze(-1)).squeeze(-1)
            gap = win.amax(-1) - chosen
            bad = gap > 0
            margin = gap[bad]
        else:
            bad = dec.bool() != (ref > 0)
            blk = name.rsplit(".", 1)[0]
            if name.endswith(".0") and blk in drop_scales:
                bad &= (drop_scales[blk] != 0)[:, :, None, None]
            margin = ref[bad].abs()
        out[name] = (int(bad.sum()), float(margin.max() / scale) if margin.numel() else 0.0)
    return out


def near_ties(record, tol: float = 1e-5, drop_scales=None, site_scale=None) -> Dict[str, int]:
    """Per decision site, how many decisions of THIS oracle's record are near-ties: ReLU
    pre-activations with |value| <= tol * the site's max |value| (or ``site_scale``'s), and 2x2
    pool windows whose two largest elements are within tol * that max (channels a Dropout2d
    keep-scale zeroes carry no decision). The decisions a run with fp32-class rounding may take
    differently are among them."""
    out = {}
    drop_scales = drop_scales or {}
    for name, ref in record.items():
        scale = ref.abs().max().clamp_min(1e-30) if site_scale is None else max(site_scale[name], 1e-30)
        if name.startswith("pool"):
            B, C, H, W = ref.shape
            win = ref.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
            top2 = win.topk(2, dim=-1).values
            near = (top2[..., 0] - top2[..., 1]) <= tol * scale
        else:
            near = ref.abs() <= tol * scale
            blk = name.rsplit(".", 1)[0]
            if name.endswith(".0") and blk in drop_scales:
                near &= (drop_scales[blk] != 0)[:, :, None, None]
        out[name] = int(near.sum())
    return out


def _on(device, img, mask, scales, decisions):
    """The truth's inputs on ``device`` (None: where they are)."""
    if device is None:
        return img, mask, scales, decisions
    mv = lambda d: {k: v.to(device) for k, v in d.items()}  # noqa: E731
    return img.to(device), mask.to(device), mv(scales), mv(decisions)


def whole_truth(ref: "UNetRef", img, mask, scales, decisions, loss_kws, log=None, device=None):
    """The float64 truth of one training step per loss config on given ReLU / max-pool decisions:
    (p64, z64, flips {site: (n, worst margin, near-ties)}, [(terms, {param: grad})] per config).
    ``device``: where the float64 arithmetic runs (None: the inputs' device, the CPU in the CPU
    suite). The full-size GPU tests evaluate it on the GPU's float64 ATen — the same ops in the
    same dtype, pinned to the CPU evaluation by tests/test_fullsize_gpu.py — and get the results
    back on the CPU."""
    log = log or (lambda msg: None)
    img, mask, scales, decisions = _on(device, img, mask, scales, decisions)
    ref64 = UNetRef().double().train().to(img.device)
    ref64.load_state_dict(ref.state_dict())
    record = {}
    log("float64 oracle forward")
    p64, z64 = unet_forward(ref64, img.double(), {k: v.double() for k, v in scales.items()},
                            decisions=decisions, record=record, return_logits=True)
    near = near_ties(record, 1e-5, scales)
    flips = {k: (n, m, near[k]) for k, (n, m) in decision_flips(decisions, record, scales).items()}
    del record
    truth = []
    for kw in loss_kws:
        log(f"float64 oracle backward {kw}")
        ref64.zero_grad(set_to_none=True)
        t64 = loss_terms(p64, mask.double(), **kw)
        t64["loss"].backward(retain_graph=True)
        truth.append(({k: float(torch.as_tensor(v).detach()) for k, v in t64.items()},
                      {n: q.grad.detach().cpu().clone() for n, q in ref64.named_parameters()}))
    return p64.detach().cpu(), z64.detach().cpu(), flips, truth


def chunked_truth(ref: "UNetRef", img, mask, scales, decisions, loss_kws, chunk: int, log=None, device=None):
    """whole_truth for a batch whose float64 graph does not fit host memory (C5: B = 8 at 1024^2
    would need ~220 GB). The U-Net has no cross-sample coupling (no normalisation layer,
    src/unet.py:19-67; Dropout2d masks injected per sample), and the loss couples the samples only
    through its whole-batch sums (Dice's I, P, T and the 1/N of the means, src/loss.py:130-160). So:
      1. per chunk of ``chunk`` images, the float64 forward on the decisions without a graph: the
         probabilities, the logits and each decision site's max |value| over the batch;
      2. the loss terms and dL/dp on the WHOLE batch's float64 probabilities (loss_terms);
      3. per chunk again, the forward with a graph and one backward per loss config seeded with
         that chunk's slice of dL/dp; parameter gradients summed over the chunks; the chunk's
         decision flips / near-ties measured in the whole batch's site scales.
    Equal to whole_truth up to float64 summation order (tests/test_oracle.py). ``device`` as for
    whole_truth."""
    log = log or (lambda msg: None)
    img, mask, scales, decisions = _on(device, img, mask, scales, decisions)
    B = img.shape[0]
    ref64 = UNetRef().double().train().to(img.device)
    ref64.load_state_dict(ref.state_dict())
    s64 = {k: v.double() for k, v in scales.items()}

    def sl(d, c0):
        return {k: v[c0:c0 + chunk] for k, v in d.items()}

    ps, zs, smax = [], [], {}
    with torch.no_grad():
        for c0 in range(0, B, chunk):
            log(f"float64 oracle forward, images {c0}..{min(B, c0 + chunk) - 1}")
            rec = {}
            p, z = unet_forward(ref64, img[c0:c0 + chunk].double(), sl(s64, c0), decisions=sl(decisions, c0),
                                record=rec, return_logits=True)
            for k, v in site_maxima(rec).items():
                smax[k] = max(smax.get(k, 0.0), v)
            ps.append(p)
            zs.append(z)
            del rec
    p64, z64 = torch.cat(ps), torch.cat(zs)
    del ps, zs
    terms, seeds = [], []
    for kw in loss_kws:
        pl = p64.clone().requires_grad_(True)
        t64 = loss_terms(pl, mask.double(), **kw)
        t64["loss"].backward()
        terms.append({k: float(torch.as_tensor(v).detach()) for k, v in t64.items()})
        seeds.append(pl.grad.detach())
    grads = [dict() for _ in loss_kws]
    flips, near = {}, {}
    for c0 in range(0, B, chunk):
        log(f"float64 oracle forward + {len(loss_kws)} backward(s), images {c0}..{min(B, c0 + chunk) - 1}")
        rec = {}
        dec = sl(decisions, c0)
        p = unet_forward(ref64, img[c0:c0 + chunk].double(), sl(s64, c0), decisions=dec, record=rec)
        for k, v in near_ties(rec, 1e-5, sl(scales, c0), site_scale=smax).items():
            near[k] = near.get(k, 0) + v
        for k, (n, m) in decision_flips(dec, rec, sl(scales, c0), site_scale=smax).items():
            n0, m0 = flips.get(k, (0, 0.0))
            flips[k] = (n0 + n, max(m0, m))
        del rec
        for i in range(len(loss_kws)):
            ref64.zero_grad(set_to_none=True)
            p.backward(seeds[i][c0:c0 + chunk], retain_graph=i + 1 < len(loss_kws))
            for n, q in ref64.named_parameters():
                grads[i][n] = grads[i][n] + q.grad if n in grads[i] else q.grad.detach().clone()
        del p
    flips = {k: (n, m, near[k]) for k, (n, m) in flips.items()}
    grads = [{n: g.cpu() for n, g in gi.items()} for gi in grads]
    return p64.cpu(), z64.cpu(), flips, list(zip(terms, grads))


def make_drop_scales(m: UNetRef, B: int, generator: torch.Generator) -> Dict[str, torch.Tensor]:
    """Dropout2d keep-scales per block: bernoulli(1-p)/(1-p) of shape (B, C)
    (same draw ATen's feature_dropout makes: noise (B,C,1,1).bernoulli_(1-p).div_(1-p))."""
    out = {}
    for name in m.block_names():
        blk = getattr(m, name)
        if blk.p > 0:
            C = blk.conv0.out_channels
            keep = torch.bernoulli(torch.full((B, C), 1.0 - blk.p), generator=generator)
            out[name] = keep / (1.0 - blk.p)
    return out


def count_parameters(m: nn.Module) -> int:
    return sum(p.numel() for p in m.parameters() if p.requires_grad)


# ---------------------------------------------------------------------------
# PDE terms — src/pde.py:24-212 (reflect pad + cross-correlation stencils)
# ---------------------------------------------------------------------------

_LAP = torch.tensor([[0.0, 1.0, 0.0], [1.0, -4.0, 1.0], [0.0, 1.0, 0.0]])
_GX = torch.tensor([[0.0, 0.0, 0.0], [-0.5, 0.0, 0.5], [0.0, 0.0, 0.0]])
_GY = torch.tensor([[0.0, -0.5, 0.0], [0.0, 0.0, 0.0], [0.0, 0.5, 0.0]])


def _stencil(u: torch.Tensor, k: torch.Tensor) -> torch.Tensor:
    up = F.pad(u, (1, 1, 1, 1), mode="reflect")  # src/pde.py:67,164
    return F.conv2d(up, k.to(u.device, u.dtype)[None, None], padding=0)


def laplacian(u):  # src/pde.py:49-79
    return _stencil(u, _LAP)


def reaction(u, a):  # src/pde.py:81-99
    return u * (1.0 - u) * (u - a)


def rd_residual(u, D, a):  # src/pde.py:101-122
    return D * laplacian(u) + reaction(u, a)


def rd_loss(u, D, a):  # src/pde.py:124-145
    return torch.mean(rd_residual(u, D, a) ** 2)


def grad_mag_sq(u):  # src/pde.py:147-178
    return _stencil(u, _GX) ** 2 + _stencil(u, _GY) ** 2


def pf_loss(u, eps):  # src/pde.py:180-212
    return torch.mean((eps / 2.0) * grad_mag_sq(u) + (1.0 / eps) * (u ** 2) * ((1.0 - u) ** 2))


# ---------------------------------------------------------------------------
# Losses — src/loss.py:36-68 (DiceBCELoss) and :114-162 (DiceBCEPDELoss)
# ---------------------------------------------------------------------------


def dice_loss(p, t, smooth=1e-6):  # src/loss.py:51-60 (whole-batch ratio)
    pf, tf = p.reshape(-1), t.reshape(-1)
    return 1 - (2.0 * (pf * tf).sum() + smooth) / (pf.sum() + tf.sum() + smooth)


def bce_loss(p, t):  # nn.BCELoss() mean, log clamped at -100
    return F.binary_cross_entropy(p, t)


def loss_terms(p, t, dice_w=0.5, bce_w=0.5, rd_w=0.0, pf_w=0.0, smooth=1e-6, D=1.0, a=0.5, eps=0.05):
    """Per-term dict + total, gating identical to src/loss.py:144-160."""
    ld = dice_loss(p, t, smooth)
    lb = bce_loss(p, t)
    total = dice_w * ld + bce_w * lb
    out = {"dice_loss": ld, "bce_loss": lb}
    if rd_w > 0:
        out["pde_loss"] = rd_loss(p, D, a)
        total = total + rd_w * out["pde_loss"]
    if pf_w > 0:
        out["phase_field_loss"] = pf_loss(p, eps)
        total = total + pf_w * out["phase_field_loss"]
    out["loss"] = total
    return out


# ---------------------------------------------------------------------------
# Metrics — src/metrics.py:4-73 (Dice), src/evaluate.py:26-97 (IoU)
# ---------------------------------------------------------------------------


def dice_score(p, t, thr=0.5, smooth=1e-6):
    pb = (p > thr).float().reshape(-1)
    tf = t.reshape(-1)
    return (2.0 * (pb * tf).sum() + smooth) / (pb.sum() + tf.sum() + smooth)


def dice_score_batch(p, t, thr=0.5, smooth=1e-6):
    return torch.stack([dice_score(p[i], t[i], thr, smooth) for i in range(p.shape[0])])


def iou(p, t, thr=0.5, smooth=1e-6):
    pb = (p > thr).float().reshape(-1)
    tf = t.reshape(-1)
    inter = (pb * tf).sum()
    return (inter + smooth) / (pb.sum() + tf.sum() - inter + smooth)


def iou_batch(p, t, thr=0.5, smooth=1e-6):
    return torch.stack([iou(p[i], t[i], thr, smooth) for i in range(p.shape[0])])


# ---------------------------------------------------------------------------
# One training step — src/train.py:108-167 (zero_grad, fwd, loss, bwd, AdamW)
# ---------------------------------------------------------------------------


def make_adamw(m: nn.Module, lr: float, weight_decay: float = 1e-5):
    """src/train.py:658-662 / :722-726."""
    return torch.optim.AdamW(m.parameters(), lr=lr, weight_decay=weight_decay)


def train_step(m: UNetRef, opt, x, t, loss_kw: dict, drop_scales=None):
    m.train()
    opt.zero_grad()
    p = m(x, drop_scales)
    terms = loss_terms(p, t, **loss_kw)
    terms["loss"].backward()
    opt.step()
    return p.detach(), {k: float(v.detach()) for k, v in terms.items()}


# ---------------------------------------------------------------------------
# Epoch loops — src/train.py:84-185 (train_epoch) and :188-286 (validate): loss terms
# averaged over batches (via .item() per batch), Dice / IoU / boundary F1 averaged over
# samples; validate's dice_score is the batch mean of the whole-batch thresholded Dice.
# ``boundary_f1_batch`` is passed in (OpenCV, which the reference uses, is absent here).
# ---------------------------------------------------------------------------


def _components(p, t, loss_kw):
    out = loss_terms(p, t, **loss_kw)
    return {k: float(v) for k, v in out.items()}


def train_epoch_ref(m: UNetRef, batches, opt, loss_kw: dict, drop_scales=None, boundary_f1_batch=None):
    """src/train.py:84-185 with return_components=True, compute_metrics=True."""
    m.train()
    tot = {"loss": 0.0, "dice_loss": 0.0, "bce_loss": 0.0, "pde_loss": 0.0, "phase_field_loss": 0.0}
    dice, iou, bf1 = [], [], []
    for k, (x, t) in enumerate(batches):
        opt.zero_grad()
        p = m(x, None if drop_scales is None else drop_scales[k])
        terms = loss_terms(p, t, **loss_kw)
        with torch.no_grad():
            c = {kk: float(v) for kk, v in terms.items()}
            tot["dice_loss"] += c["dice_loss"]
            tot["bce_loss"] += c["bce_loss"]
            tot["pde_loss"] += c.get("pde_loss", 0.0)
            tot["phase_field_loss"] += c.get("phase_field_loss", 0.0)
            dice += dice_score_batch(p, t).tolist()
            iou += iou_batch(p, t).tolist()
            if boundary_f1_batch is not None:
                bf1 += boundary_f1_batch(p.detach(), t).tolist()
        terms["loss"].backward()
        opt.step()
        tot["loss"] += float(terms["loss"].detach())
    n = len(batches)
    res = {"loss": tot["loss"] / n, "dice_loss": tot["dice_loss"] / n, "bce_loss": tot["bce_loss"] / n}
    if loss_kw.get("rd_w", 0.0) > 0:
        res["pde_loss"] = tot["pde_loss"] / n
    if loss_kw.get("pf_w", 0.0) > 0:
        res["phase_field_loss"] = tot["phase_field_loss"] / n
    res["dice_score"] = float(sum(dice) / len(dice))
    res["iou_score"] = float(sum(iou) / len(iou))
    res["boundary_f1_score"] = float(sum(bf1) / len(bf1)) if bf1 else 0.0
    return res


@torch.no_grad()
def validate_ref(m: UNetRef, batches, loss_kw: dict, boundary_f1_batch=None):
    """src/train.py:188-286 with return_components=True, compute_metrics=True."""
    m.eval()
    tot = {"loss": 0.0, "dice_score": 0.0, "dice_loss": 0.0, "bce_loss": 0.0, "pde_loss": 0.0,
           "phase_field_loss": 0.0}
    iou, bf1 = [], []
    for x, t in batches:
        p = m(x)
        c = _components(p, t, loss_kw)
        tot["dice_score"] += float(dice_score(p, t))  # src/metrics.py:4-35, whole batch
        for key in ("loss", "dice_loss", "bce_loss"):
            tot[key] += c[key]
        tot["pde_loss"] += c.get("pde_loss", 0.0)
        tot["phase_field_loss"] += c.get("phase_field_loss", 0.0)
        iou += iou_batch(p, t).tolist()
        if boundary_f1_batch is not None:
            bf1 += boundary_f1_batch(p, t).tolist()
    n = len(batches)
    res = {"loss": tot["loss"] / n, "dice_score": tot["dice_score"] / n, "dice_loss": tot["dice_loss"] / n,
           "bce_loss": tot["bce_loss"] / n}
    if loss_kw.get("rd_w", 0.0) > 0:
        res["pde_loss"] = tot["pde_loss"] / n
    if loss_kw.get("pf_w", 0.0) > 0:
        res["phase_field_loss"] = tot["phase_field_loss"] / n
    res["iou_score"] = float(sum(iou) / len(iou))
    res["boundary_f1_score"] = float(sum(bf1) / len(bf1)) if bf1 else 0.0
    return res
