"""Host-side step-loop plumbing of train.py on CPU stand-ins (no kernels run): per-epoch
reshuffling through set_epoch (loader or sampler), result keys and the reference's averaging
(src/train.py:84-286), and boundary F1 computed on the host threads for every step."""
import numpy as np
import torch
import torch.nn as nn

from oracle import reference_torch as rt
import importlib
from physics_informed_image_segmentation_amd.evaluate import compute_boundary_f1_batch

tr = importlib.import_module("physics_informed_image_segmentation_amd.train")  # the module, not train()


class _Loader:
    """DeviceDiscLoader stand-in: a seeded permutation per epoch, set only by set_epoch."""

    def __init__(self, n=6, bs=2, H=16, W=16):
        self.n, self.bs, self.epoch, self.seen = n, bs, 0, []
        self.img, self.mask = rt.synthetic_batch(n, H, W, seed=3)

    def set_epoch(self, e):
        self.epoch = e

    def __iter__(self):
        order = torch.randperm(self.n, generator=torch.Generator().manual_seed(100 + self.epoch)).tolist()
        self.seen.append(order)
        for k in range(0, self.n, self.bs):
            idx = order[k:k + self.bs]
            yield self.img[idx], self.mask[idx]


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.w = nn.Parameter(torch.tensor(3.0))

    def forward(self, x):
        return torch.sigmoid(self.w * (x - 0.5))


class _Crit(nn.Module):
    """Criterion stand-in leaving the fused kernel's outputs in .last (terms, counts, scores)."""
    smooth = 1e-6

    def forward(self, p, t):
        terms = rt.loss_terms(p, t)
        B = p.shape[0]
        pb = (p.detach() > 0.5).float().reshape(B, -1)
        tf = t.reshape(B, -1)
        counts = torch.stack([(pb * tf).sum(1), pb.sum(1), tf.sum(1)], 1).to(torch.int32)
        scores = torch.stack([rt.dice_score_batch(p.detach(), t), rt.iou_batch(p.detach(), t)], 1)
        self.last = {"terms": torch.stack([terms["loss"].detach(), terms["dice_loss"].detach(),
                                           terms["bce_loss"].detach(), torch.tensor(0.0), torch.tensor(0.0),
                                           torch.tensor(0.0), torch.tensor(0.0), torch.tensor(0.0)]),
                     "counts": counts, "scores": scores}
        return terms["loss"]


def test_train_stage_reshuffles_every_epoch(tmp_path):
    net, crit, loader = _Net(), _Crit(), _Loader()
    opt = torch.optim.SGD(net.parameters(), lr=0.0)
    best, ep, hist = tr.train_stage(net, loader, _Loader(), crit, opt, torch.device("cpu"), num_epochs=3,
                                    stage_name="t", verbose=False, csv_path=tmp_path / "m.csv")
    assert len(hist) == 3 and len(loader.seen) == 3
    assert loader.seen[0] != loader.seen[1] != loader.seen[2]  # set_epoch reached the loader
    assert set(hist[0]) == set(tr.CSV_FIELDS)
    assert (tmp_path / "m.csv").read_text().splitlines()[0].split(",") == tr.CSV_FIELDS


def test_train_epoch_averages_like_the_reference():
    net, crit, loader = _Net(), _Crit(), _Loader()
    opt = torch.optim.SGD(net.parameters(), lr=0.0)  # lr 0: every batch sees the same weights
    res = tr.train_epoch(net, loader, crit, opt, torch.device("cpu"), return_components=True)
    order = loader.seen[0]
    losses, dl, bl, dice, iou, bf1 = [], [], [], [], [], []
    with torch.no_grad():
        for k in range(0, 6, 2):
            x, t = loader.img[order[k:k + 2]], loader.mask[order[k:k + 2]]
            p = net(x)
            terms = rt.loss_terms(p, t)
            losses.append(terms["loss"].item())
            dl.append(terms["dice_loss"].item())
            bl.append(terms["bce_loss"].item())
            dice += rt.dice_score_batch(p, t).tolist()
            iou += rt.iou_batch(p, t).tolist()
            bf1 += compute_boundary_f1_batch(p, t).tolist()
    assert set(res) == {"loss", "dice_loss", "bce_loss", "dice_score", "iou_score", "boundary_f1_score"}
    np.testing.assert_allclose(res["loss"], np.mean(losses), rtol=1e-6)  # per batch
    np.testing.assert_allclose(res["dice_loss"], np.mean(dl), rtol=1e-6)
    np.testing.assert_allclose(res["bce_loss"], np.mean(bl), rtol=1e-6)
    np.testing.assert_allclose(res["dice_score"], np.mean(dice), rtol=1e-6)  # per sample
    np.testing.assert_allclose(res["iou_score"], np.mean(iou), rtol=1e-6)
    np.testing.assert_allclose(res["boundary_f1_score"], np.mean(bf1), rtol=1e-6)
    assert res["boundary_f1_score"] > 0


def test_boundary_f1_scorer_backpressure():
    """_BoundaryF1Async keeps at most 2 x workers steps in flight (the oldest is folded into a
    running sum first), so pinned buffers cannot pile up over an epoch; the sum is unchanged."""
    import torch
    import importlib
    trm = importlib.import_module("physics_informed_image_segmentation_amd.train")
    from physics_informed_image_segmentation_amd.evaluate import compute_boundary_f1_batch
    g = torch.Generator().manual_seed(4)
    sc = trm._BoundaryF1Async("cpu", workers=1)
    want, peak = 0.0, 0
    try:
        for _ in range(9):
            p = torch.rand(2, 1, 32, 32, generator=g)
            t = (torch.rand(2, 1, 32, 32, generator=g) > 0.5).float()
            want += float(compute_boundary_f1_batch(p, t).sum())
            sc.submit(p, t)
            peak = max(peak, len(sc.futures))
        got = sc.collect()
    finally:
        sc.close()
    assert peak <= sc.max_inflight == 2
    assert abs(got - want) < 1e-5  # float32 per-batch sums
