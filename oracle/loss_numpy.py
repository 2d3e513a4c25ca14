"""ORACLE (test infrastructure only) — float64 numpy restatement of the fused
loss the HIP kernel computes: Dice + BCE (src/loss.py:51-66), reaction-
diffusion residual (src/pde.py:49-145) and phase-field energy
(src/pde.py:147-212), forward AND hand-derived backward, plus the per-sample
thresholded counters behind Dice/IoU (src/metrics.py:57-71,
src/evaluate.py:81-95).

The backward is written out explicitly (adjoint of "reflect-pad then
stencil" by folding the ghost rows/columns back onto rows 1 and n-2), not
taken from autograd, so the tests can check it against torch autograd in
float64 and the HIP kernel against it independently.
"""
from __future__ import annotations

import numpy as np

LOG_CLAMP = -100.0   # nn.BCELoss log clamp (torch/_decomp/decompositions.py:631-633)
BCE_EPS = 1e-12      # binary_cross_entropy_backward clamp (decompositions.py:649-654)


def _pad_reflect(u):
    return np.pad(u, ((0, 0), (1, 1), (1, 1)), mode="reflect")


def _pad_reflect_adjoint(g):
    """Adjoint of reflect padding on the last two axes: ghost row -1 is a copy
    of row 1 and ghost row n is a copy of row n-2 (same for columns)."""
    g = g.copy()
    g[:, 2, :] += g[:, 0, :]
    g[:, -3, :] += g[:, -1, :]
    g = g[:, 1:-1, :]
    g[:, :, 2] += g[:, :, 0]
    g[:, :, -3] += g[:, :, -1]
    return g[:, :, 1:-1]


_LAP = np.array([[0.0, 1.0, 0.0], [1.0, -4.0, 1.0], [0.0, 1.0, 0.0]])
_GX = np.array([[0.0, 0.0, 0.0], [-0.5, 0.0, 0.5], [0.0, 0.0, 0.0]])
_GY = np.array([[0.0, -0.5, 0.0], [0.0, 0.0, 0.0], [0.0, 0.5, 0.0]])


def _correlate(up, k):
    """Valid cross-correlation of (N, H+2, W+2) with a 3x3 kernel (F.conv2d)."""
    H, W = up.shape[1] - 2, up.shape[2] - 2
    out = np.zeros((up.shape[0], H, W))
    for i in range(3):
        for j in range(3):
            if k[i, j] != 0.0:
                out += k[i, j] * up[:, i:i + H, j:j + W]
    return out


def _correlate_adjoint(g, k):
    """Adjoint of _correlate: scatter g back onto the padded grid."""
    N, H, W = g.shape
    out = np.zeros((N, H + 2, W + 2))
    for i in range(3):
        for j in range(3):
            if k[i, j] != 0.0:
                out[:, i:i + H, j:j + W] += k[i, j] * g
    return out


def stencil(u, k):
    return _correlate(_pad_reflect(u), k)


def stencil_adjoint(g, k):
    return _pad_reflect_adjoint(_correlate_adjoint(g, k))


def loss_forward(p, t, dice_w=0.5, bce_w=0.5, rd_w=0.0, pf_w=0.0, smooth=1e-6, D=1.0, a=0.5, eps=0.05,
                 reaction=True):
    """p, t: arrays (B, H, W) or (B, 1, H, W). Returns dict of float64 terms and sums."""
    p = np.asarray(p, dtype=np.float64).reshape(p.shape[0], p.shape[-2], p.shape[-1])
    t = np.asarray(t, dtype=np.float64).reshape(p.shape)
    n = p.size
    I, P, T = float((p * t).sum()), float(p.sum()), float(t.sum())
    dice = 1.0 - (2.0 * I + smooth) / (P + T + smooth)
    bce = float(np.mean((t - 1.0) * np.maximum(np.log1p(-p), LOG_CLAMP)
                        - t * np.maximum(np.log(p), LOG_CLAMP)))
    out = {"I": I, "P": P, "T": T, "dice_loss": dice, "bce_loss": bce}
    total = dice_w * dice + bce_w * bce
    rx = 1.0 if reaction else 0.0  # src/ablation.py:75-86 (use_reaction_term=False: f(u) = 0)
    r = D * stencil(p, _LAP) + rx * p * (1.0 - p) * (p - a)
    out["rd"] = float(np.mean(r * r))
    gx, gy = stencil(p, _GX), stencil(p, _GY)
    out["pf"] = float(np.mean(0.5 * eps * (gx * gx + gy * gy) + (p * p) * (1.0 - p) ** 2 / eps))
    if rd_w > 0:
        out["pde_loss"] = out["rd"]
        total += rd_w * out["rd"]
    if pf_w > 0:
        out["phase_field_loss"] = out["pf"]
        total += pf_w * out["pf"]
    out["loss"] = total
    return out


def loss_backward(p, t, dice_w=0.5, bce_w=0.5, rd_w=0.0, pf_w=0.0, smooth=1e-6, D=1.0, a=0.5, eps=0.05,
                  grad_out=1.0, chain_sigmoid=False, reaction=True):
    """dL/dp (or dL/dz through the sigmoid when chain_sigmoid) — SURVEY §8(a) A6-A8."""
    shape = p.shape
    p = np.asarray(p, dtype=np.float64).reshape(p.shape[0], p.shape[-2], p.shape[-1])
    t = np.asarray(t, dtype=np.float64).reshape(p.shape)
    n = p.size
    I, P, T = (p * t).sum(), p.sum(), t.sum()
    S = P + T + smooth
    g = dice_w * (-(2.0 * t * S - (2.0 * I + smooth)) / (S * S))
    g += bce_w * (p - t) / np.maximum(p * (1.0 - p), BCE_EPS) / n
    if rd_w > 0:
        rx = 1.0 if reaction else 0.0
        r = D * stencil(p, _LAP) + rx * p * (1.0 - p) * (p - a)
        fprime = rx * (-3.0 * p * p + 2.0 * (1.0 + a) * p - a)
        g += rd_w * (2.0 / n) * (D * stencil_adjoint(r, _LAP) + r * fprime)
    if pf_w > 0:
        gx, gy = stencil(p, _GX), stencil(p, _GY)
        g += pf_w * (1.0 / n) * (eps * (stencil_adjoint(gx, _GX) + stencil_adjoint(gy, _GY))
                                 + 2.0 * p * (1.0 - p) * (1.0 - 2.0 * p) / eps)
    g *= grad_out
    if chain_sigmoid:
        g = g * p * (1.0 - p)
    return g.reshape(shape)


def sample_counts(p, t, thr=0.5):
    """Per-sample exact integers (I, P_hat, T) of the thresholded prediction."""
    B = p.shape[0]
    pb = (np.asarray(p).reshape(B, -1) > thr)
    tb = np.asarray(t).reshape(B, -1)
    inter = (pb * tb).sum(axis=1).astype(np.int64)
    return inter, pb.sum(axis=1).astype(np.int64), tb.sum(axis=1).astype(np.int64)


def dice_iou_from_counts(inter, phat, tsum, smooth=1e-6):
    inter, phat, tsum = (np.asarray(v, dtype=np.float64) for v in (inter, phat, tsum))
    dice = (2.0 * inter + smooth) / (phat + tsum + smooth)
    iou = (inter + smooth) / (phat + tsum - inter + smooth)
    return dice, iou
