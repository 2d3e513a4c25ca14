"""The direct 3x3 convolution in fp16x3 (csrc/direct.hip, pis_tune key 29): the forward of
src/unet.py:29,38's nn.Conv2d (bias, ReLU, Dropout2d keep-scale, the encoder's fused 2x2 max
pool) and its input gradient (ReLU mask of the conv's input, keep-scale, accumulate; flipped or
original weights) against float64, as accurate as the native fp32 MFMA direct kernel (key 8 = 0)
for unit, gradient-sized and large operands and for a region spanning 2^-60 .. 1."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from oracle import reference_torch as rt

pytestmark = pytest.mark.gpu

RELU, SCALE, MASK, ACC, UNFLIPPED = 1, 2, 4, 8, 32


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def krsc(w):
    return w.permute(0, 2, 3, 1).contiguous()


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-300)).item()


def s():
    return torch.cuda.current_stream().cuda_stream


class Knobs:
    def __init__(self, hip, **kv):
        self.hip, self.kv, self.prev = hip, kv, {}

    def __enter__(self):
        for k, v in self.kv.items():
            self.prev[k] = self.hip.pis_tune(int(k[1:]), v)

    def __exit__(self, *a):
        for k, v in self.prev.items():
            self.hip.pis_tune(int(k[1:]), v)


DIRECT = dict(k29=2)
NATIVE = dict(k29=0, k8=0)  # the fp32-MFMA direct halo kernel


def _fwd(hip, x, w, b, scale, flags, pool=False, ldx_extra=0):
    B, Cin, H, W = x.shape
    Cout = w.shape[0]
    ldx = Cin + ldx_extra
    xb = torch.zeros(B, H, W, ldx, device="cuda")
    xb[..., :Cin] = nhwc(x.float()).cuda()
    nws = max(hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout), 4)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    y = torch.empty(B, H, W, Cout, device="cuda")
    wd = krsc(w.float()).cuda()
    bd = b.float().cuda() if b is not None else None
    sd = scale.float().cuda() if scale is not None else None
    if pool:
        pl = torch.empty(B, H // 2, W // 2, Cout, device="cuda")
        rc = hip.pis_conv3x3_fwd_pool(xb.data_ptr(), ldx, wd.data_ptr(), bd.data_ptr() if bd is not None else 0,
                                      sd.data_ptr() if sd is not None else 0, y.data_ptr(), Cout, B, H, W, Cin, Cout,
                                      flags, ws.data_ptr(), nws, 0, pl.data_ptr(), s())
    else:
        rc = hip.pis_conv3x3_fwd_ex(xb.data_ptr(), ldx, wd.data_ptr(), bd.data_ptr() if bd is not None else 0,
                                    sd.data_ptr() if sd is not None else 0, y.data_ptr(), Cout, B, H, W, Cin, Cout,
                                    flags, ws.data_ptr(), nws, s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    return (nchw(y.cpu()), nchw(pl.cpu())) if pool else nchw(y.cpu())


# kernel variants behind pis_tune: key 32 the input gradient's mask prefetch (default on)
FWD_VARIANTS = [dict(), dict(k32=0)]
# weight gradient: key 43 = 1 (default) each block walks a contiguous run of tiles down the image
# columns, 0 the strided round-3 tile order; key 49 = 2 (default): 2-row tiles, two blocks per CU, 4:
# the 4-row kernel
WG_VARIANTS = [dict(), dict(k43=0), dict(k49=4), dict(k49=4, k43=0)]


@pytest.mark.parametrize("variant", FWD_VARIANTS)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 64, 64, 64), (1, 8, 32, 128, 64), (2, 16, 32, 64, 128),
                                           (1, 16, 32, 256, 128)])
def test_direct_fwd_is_fp32_accurate(hip, B, H, W, Cin, Cout, variant):
    g = torch.Generator().manual_seed(61)
    x0 = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64))
    x0[0, :, :8, :8] *= torch.pow(2.0, -60 * torch.rand(Cin, 8, 8, generator=g, dtype=torch.float64))
    w = (torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)).float().double()
    b = torch.randn(Cout, generator=g, dtype=torch.float64).float().double()
    scale = ((torch.rand(B, Cout, generator=g) > 0.2).double() / 0.8).float().double()
    errs = {}
    for sc in (1.0, 1e-12, 1e6):
        x = (x0 * sc).float().double()
        ref = F.relu(F.conv2d(x, w, b * sc, padding=1)) * scale[:, :, None, None]
        for name, knobs in (("direct", {**DIRECT, **variant}), ("native", NATIVE)):
            with Knobs(hip, **knobs):
                y = _fwd(hip, x, w, b * sc, scale, RELU | SCALE)
            errs[name, sc] = rel(y, ref)
    for sc in (1.0, 1e-12, 1e6):
        assert errs["direct", sc] <= 1.25 * errs["native", sc] + 1e-9, errs
        assert errs["direct", sc] < 2e-6, errs


def test_direct_fwd_pool_and_row_pitch(hip):
    """Encoder conv1 + MaxPool2d(2, 2) in one call (pooled in the epilogue), the input read from a
    channel slice of a wider buffer (the concat layout), against float64."""
    B, H, W, Cin, Cout = 2, 16, 64, 64, 128
    g = torch.Generator().manual_seed(62)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)).float().double()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)).float().double()
    b = torch.randn(Cout, generator=g, dtype=torch.float64).float().double()
    with Knobs(hip, **DIRECT):
        y, pl = _fwd(hip, x, w, b, None, RELU, pool=True, ldx_extra=64)
    ref = F.relu(F.conv2d(x, w, b, padding=1))
    assert rel(y, ref) < 2e-6
    assert torch.equal(pl, F.max_pool2d(y, 2))  # the pool of exactly the values written


@pytest.mark.parametrize("variant", FWD_VARIANTS)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 64, 64, 64), (1, 8, 32, 128, 64), (2, 16, 32, 64, 128)])
@pytest.mark.parametrize("unflipped", [False, True])
def test_direct_dgrad_is_fp32_accurate(hip, B, H, W, Cin, Cout, unflipped, variant):
    """dx = conv_input(dz, w) * (x > 0) * keep-scale (+ dx), from a flipped copy of the weights or
    from the original ones (PIS_W_UNFLIPPED), for gradient-sized and unit dz."""
    g = torch.Generator().manual_seed(63)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)).float().double()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)).float().double()
    scale = ((torch.rand(B, Cin, generator=g) > 0.2).double() / 0.8).float().double()
    dz0 = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
    xd = nhwc(x.float()).cuda()
    wd = krsc(w.float()).cuda()
    wf = torch.empty(Cin * 9 * Cout, device="cuda")
    assert hip.pis_conv3x3_flip(wd.data_ptr(), wf.data_ptr(), Cin, Cout, s()) == 0
    sd = scale.float().cuda()
    errs = {}
    for sc in (1.0, 1e-9):
        dz = (dz0 * sc).float().double()
        base = 0.5 * sc  # the accumulated-into gradient, of the same magnitude
        ref = torch.nn.grad.conv2d_input(x.shape, w, dz, padding=1) * (x > 0) * scale[:, :, None, None] + base
        for name, knobs in (("direct", {**DIRECT, **variant}), ("native", NATIVE)):
            with Knobs(hip, **knobs):
                nws = max(hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout), 4)
                ws = torch.empty(nws // 4 + 1, device="cuda")
                direct = hip.pis_conv3x3_dgrad_direct(B, H, W, Cin, Cout, Cout, nws)
                assert direct == (name == "direct")
                use_orig = unflipped and name == "direct"
                dx = torch.full((B, H, W, Cin), base, device="cuda")
                rc = hip.pis_conv3x3_dgrad_ex(nhwc(dz.float()).cuda().data_ptr(), Cout,
                                              (wd if use_orig else wf).data_ptr(), xd.data_ptr(), Cin, sd.data_ptr(),
                                              dx.data_ptr(), Cin, B, H, W, Cin, Cout,
                                              MASK | SCALE | ACC | (UNFLIPPED if use_orig else 0), ws.data_ptr(), nws,
                                              s())
                assert rc == 0, hip.pis_last_error()
                torch.cuda.synchronize()
            errs[name, sc] = rel(nchw(dx.cpu()).double() - torch.tensor(base, dtype=torch.float32).double(),
                                 ref - torch.tensor(base, dtype=torch.float32).double())
    for sc in (1.0, 1e-9):
        assert errs["direct", sc] <= 1.25 * errs["native", sc] + 1e-9, errs
        assert errs["direct", sc] < 2e-6, errs


def test_direct_mixed_magnitude_chunks(hip):
    """The input's scale is chosen per block and 16-channel chunk: channels 0-15 ~1, 16-31 ~1e-30,
    32-47 ~1e20 — the partial sums are re-expressed at each chunk (rises capped, common.h
    h3_keep) without overflow, and the result is as accurate as the fp32 MFMA kernel's."""
    B, H, W, Cin, Cout = 1, 8, 32, 64, 64
    g = torch.Generator().manual_seed(64)
    x = torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)
    x[:, 16:32] *= 1e-30
    x[:, 32:48] *= 1e20
    x = x.float().double()
    w = (torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / 24).float().double()
    ref = F.conv2d(x, w, padding=1)
    out = {}
    for name, knobs in (("direct", DIRECT), ("native", NATIVE)):
        with Knobs(hip, **knobs):
            out[name] = _fwd(hip, x, w, None, None, 0)
    assert torch.isfinite(out["direct"]).all()
    assert rel(out["direct"], ref) <= 1.25 * rel(out["native"], ref) + 1e-9


@pytest.mark.parametrize("variant", WG_VARIANTS)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 64, 64, 64), (1, 8, 32, 128, 64), (2, 16, 32, 64, 128),
                                           (1, 16, 32, 128, 128), (3, 24, 64, 64, 64)])
def test_direct_wgrad_is_fp32_accurate(hip, B, H, W, Cin, Cout, variant):
    """dW = sum_p dz[p] x[p + tap] and db = sum_p dz[p] (direct fp16x3 weight gradient, split-K slabs
    reduced in fixed order) against float64: as accurate as the fp32 MFMA weight gradient
    (keys 29 = 0, 14 = 0), for unit and gradient-sized dz, a batch whose second sample's dz is
    1e-30 of the first's (the per-tile scale jumps), and accumulation into existing gradients."""
    g = torch.Generator().manual_seed(65)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)).float().double()
    dz0 = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
    cases = {"unit": dz0, "tiny": dz0 * 1e-9}
    if B > 1:
        mixed = dz0.clone()
        mixed[1] *= 1e-30
        cases["mixed"] = mixed
    xd = nhwc(x.float()).cuda()
    for case, dz in cases.items():
        dz = dz.float().double()
        dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1)
        db_ref = dz.sum(dim=(0, 2, 3))
        errs = {}
        for name, knobs in (("direct", {**DIRECT, **variant}), ("native", dict(k29=0, k14=0))):
            with Knobs(hip, **knobs):
                nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
                ws = torch.empty(nws // 4 + 1, device="cuda")
                dw = torch.full((Cout, 3, 3, Cin), 0.25, device="cuda")
                db = torch.full((Cout,), 0.25, device="cuda")
                rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, nhwc(dz.float()).cuda().data_ptr(), Cout, dw.data_ptr(),
                                           db.data_ptr(), B, H, W, Cin, Cout, ACC, ws.data_ptr(), nws, s())
                assert rc == 0, hip.pis_last_error()
                torch.cuda.synchronize()
            dwc = dw.cpu().double().permute(0, 3, 1, 2) - 0.25
            assert torch.isfinite(dwc).all(), (case, name)
            errs[name] = (rel(dwc, dw_ref), rel(db.cpu().double() - 0.25, db_ref))
        if case == "unit":  # accumulation onto 0.25 is exact to fp32 only at unit scale
            assert errs["direct"][0] <= 1.25 * errs["native"][0] + 1e-9, (case, errs)
            assert errs["direct"][0] < 5e-6 and errs["direct"][1] < 1e-5, (case, errs)


@pytest.mark.parametrize("variant", WG_VARIANTS)
@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 64, 64, 64), (2, 16, 32, 128, 128)])
def test_direct_wgrad_scales_any_magnitude(hip, B, H, W, Cin, Cout, variant):
    """Without accumulation: gradient-sized (1e-9), tiny (1e-30) and large (1e6) dz and a batch
    mixing 1 and 1e-30 per sample — finite and within 1.25x of the fp32 MFMA path's error."""
    g = torch.Generator().manual_seed(66)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)).float().double()
    dz0 = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
    xd = nhwc(x.float()).cuda()
    mixed = dz0.clone()
    mixed[1] *= 1e-30
    for case, dz in {"1e-9": dz0 * 1e-9, "1e-30": dz0 * 1e-30, "1e6": dz0 * 1e6, "mixed": mixed}.items():
        dz = dz.float().double()
        dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1)
        errs = {}
        for name, knobs in (("direct", {**DIRECT, **variant}), ("native", dict(k29=0, k14=0))):
            with Knobs(hip, **knobs):
                nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
                ws = torch.empty(nws // 4 + 1, device="cuda")
                dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
                rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, nhwc(dz.float()).cuda().data_ptr(), Cout, dw.data_ptr(),
                                           0, B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s())
                assert rc == 0, hip.pis_last_error()
                torch.cuda.synchronize()
            dwc = dw.cpu().double().permute(0, 3, 1, 2)
            assert torch.isfinite(dwc).all(), (case, name)
            errs[name] = rel(dwc, dw_ref)
        assert errs["direct"] <= 1.25 * errs["native"] + 1e-9, (case, errs)
        assert errs["direct"] < 5e-6, (case, errs)


@pytest.mark.parametrize("variant", WG_VARIANTS)
def test_direct_wgrad_x_magnitude_down_the_strip(hip, variant):
    """x whose magnitude changes down the image (rows 0-7 ~1, 8-15 ~1e-12, 16-23 ~1e9): a block's
    tiles walk down a column (key 43 = 1), so the x scale is re-chosen inside one accumulation chain
    — finite and within 1.25x of the fp32 MFMA path's error against float64."""
    B, H, W, Cin, Cout = 2, 24, 64, 64, 128
    g = torch.Generator().manual_seed(67)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64))
    x[:, :, 8:16] *= 1e-12
    x[:, :, 16:] *= 1e9
    x = x.float().double()
    dz = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64).float().double()
    dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1)
    xd = nhwc(x.float()).cuda()
    errs = {}
    for name, knobs in (("direct", {**DIRECT, **variant}), ("native", dict(k29=0, k14=0))):
        with Knobs(hip, **knobs):
            nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
            ws = torch.empty(nws // 4 + 1, device="cuda")
            dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
            rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, nhwc(dz.float()).cuda().data_ptr(), Cout, dw.data_ptr(),
                                       0, B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s())
            assert rc == 0, hip.pis_last_error()
            torch.cuda.synchronize()
        dwc = dw.cpu().double().permute(0, 3, 1, 2)
        assert torch.isfinite(dwc).all(), name
        errs[name] = rel(dwc, dw_ref)
    assert errs["direct"] <= 1.25 * errs["native"] + 1e-9, errs
    assert errs["direct"] < 5e-6, errs


@pytest.mark.parametrize("knobs", [dict(k29=2), dict(k29=2, k43=0), dict(k29=2, k49=4)])
@pytest.mark.parametrize("loss_kw", [dict(), dict(rd_w=1e-2, pf_w=1e-2, D=5.0, a=0.5, eps=0.05)])
def test_train_step_with_direct_convs(hip, loss_kw, knobs):
    """The whole training step with every eligible conv on the direct kernels (key 29 = 2: forward
    with the fused pool, input gradients from the original weights, weight gradients; with either
    weight-gradient tile order, key 43): outputs, loss terms and every parameter gradient against
    the float64 oracle on the HIP decisions at the north-star 1e-4 (tests/test_unet_gpu.py's check)."""
    import importlib
    tu = importlib.import_module("test_unet_gpu")
    with Knobs(hip, **knobs):
        net, ref, u, crit, p_ref, terms, ref64 = tu._step_pair(2, 64, 64, loss_kw)
    assert tu.rel(u, p_ref) < 1e-4
    got = crit.last["terms"].cpu()
    for i, k in enumerate(("loss", "dice_loss", "bce_loss", "pde_loss", "phase_field_loss")):
        if k in terms:
            assert got[i].item() == pytest.approx(terms[k].item(), rel=1e-4), k
    flips = {k: v for k, v in ref64.flips.items() if v[0]}
    assert sum(n for n, _ in flips.values()) <= 8 and all(m <= 1e-5 for _, m in flips.values()), flips
    worst = sorted(((tu.rel(p.grad, q.grad), n) for (n, p), q in zip(net.named_parameters(), ref64.parameters())),
                   reverse=True)
    assert worst[0][0] < 1e-4, worst[:5]


@pytest.mark.parametrize("cin,cout", [(64, 64), (64, 128), (128, 64)])
def test_direct_split_ready_bitwise(hip, cin, cout):
    """The direct kernel's weight split computed ahead (pis_conv3x3_filter / pis_conv3x3_filters, format 3)
    and passed with PIS_FILTER_READY gives bitwise the forward (plain and with the fused pool) and the
    input gradient from the original weights that the calls compute with their own split."""
    from physics_informed_image_segmentation_amd import _hip
    B, H, W = 1, 256, 64  # H >= 256, <= 128 channels: the direct layers of the default policy
    g = torch.Generator().manual_seed(71)
    x = F.relu(torch.randn(B, H, W, cin, generator=g)).cuda()
    dz = torch.randn(B, H, W, cout, generator=g).cuda()
    w = (torch.randn(cout, 3, 3, cin, generator=g) * 0.05).cuda()
    bias = torch.randn(cout, generator=g).cuda()
    nws = hip.pis_conv3x3_ex_ws(B, H, W, cin, cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    splits = {}
    for dg in (0, 1):
        nb = hip.pis_conv3x3_filter_bytes(B, H, W, cin, cout, dg)
        assert nb > 0
        one = torch.empty(nb // 4 + 1, device="cuda")
        assert hip.pis_conv3x3_filter(w.data_ptr(), B, H, W, cin, cout, dg, one.data_ptr(), nb, s()) == 0
        splits[dg] = (one, nb)
    # the batched form writes the same bytes
    jobs = (_hip.FilterJob * 2)()
    bat = {}
    for dg in (0, 1):
        nb = splits[dg][1]
        bat[dg] = torch.empty(nb // 4 + 1, device="cuda")
        jobs[dg] = _hip.FilterJob(w.data_ptr(), bat[dg].data_ptr(), nb, B, H, W, cin, cout, dg)
    assert hip.pis_conv3x3_filters(ctypes.addressof(jobs), 2, s()) == 0
    outs = {}
    for ready in (False, True):
        wptr, fl = (splits[0][0].data_ptr(), 64) if ready else (w.data_ptr(), 0)
        y = torch.empty(B, H, W, cout, device="cuda")
        assert hip.pis_conv3x3_fwd_ex(x.data_ptr(), cin, wptr, bias.data_ptr(), 0, y.data_ptr(), cout, B, H, W,
                                      cin, cout, RELU | fl, ws.data_ptr(), nws, s()) == 0, hip.pis_last_error()
        yp = torch.empty(B, H, W, cout, device="cuda")
        pl = torch.empty(B, H // 2, W // 2, cout, device="cuda")
        assert hip.pis_conv3x3_fwd_pool(x.data_ptr(), cin, wptr, bias.data_ptr(), 0, yp.data_ptr(), cout, B, H, W,
                                        cin, cout, RELU | fl, ws.data_ptr(), nws, 0, pl.data_ptr(), s()) == 0
        dwp, dfl = (splits[1][0].data_ptr(), 64) if ready else (w.data_ptr(), UNFLIPPED)
        dx = torch.empty(B, H, W, cin, device="cuda")
        assert hip.pis_conv3x3_dgrad_ex(dz.data_ptr(), cout, dwp, x.data_ptr(), cin, 0, dx.data_ptr(), cin, B, H, W,
                                        cin, cout, MASK | dfl, ws.data_ptr(), nws, s()) == 0, hip.pis_last_error()
        outs[ready] = (y, yp, pl, dx)
    torch.cuda.synchronize()
    for dg in (0, 1):
        C, N = (cout, cin) if dg else (cin, cout)  # contraction, outputs
        nw = 9 * C * N + N  # floats written: the hi / lo fp16 planes, then 1 / t_n (the rest is padding)
        assert torch.equal(splits[dg][0][:nw], bat[dg][:nw])
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)


def _hip_step(B, H, W, seed=11):
    """One HIP training step (Stage-II loss, injected Dropout2d masks) -> u, every gradient, and the
    C-ABI calls in order (the call tracer)."""
    from physics_informed_image_segmentation_amd import DiceBCEPDELoss, UNet, _hip
    img, mask = rt.synthetic_batch(B, H, W, seed=seed)
    torch.manual_seed(seed)
    net = UNet(1, 1, 64).cuda().train()
    net.set_dropout_scales(rt.make_drop_scales(rt.UNetRef(1, 1, 64), B, torch.Generator().manual_seed(seed)))
    crit = DiceBCEPDELoss(pde_weight=1e-2, phase_field_weight=1e-2, diffusion_coeff=5.0, epsilon=0.05)
    calls = []

    class Tr:
        def begin(self, name, args):
            calls.append(name)

        def end(self, tok):
            pass
    _hip.set_tracer(Tr())
    try:
        u = net(img.cuda())
        loss = crit(u, mask.cuda())
        calls.append("<backward>")
        loss.backward()
        torch.cuda.synchronize()
    finally:
        _hip.set_tracer(None)
    return u.detach().clone(), [p.grad.detach().clone() for p in net.parameters()], calls


def test_engine_filters_ahead_default_policy_bitwise(hip):
    """PIS_FILTER_AHEAD modes 2-5 against mode 0 at the DEFAULT layer policy (pis_tune
    key 29 as shipped) on a grid where both filter tables are non-empty — B = 1 at 256 x 256: the
    direct layers (<= 128 channels at 256^2) and the Winograd ones (128^2 and below) — bitwise the
    same u and gradients; in modes 4 / 5 (every filter operand and the transposed convs' input-
    gradient weights at the forward's start) the backward issues no pis_convt2x2_prep of its own."""
    from physics_informed_image_segmentation_amd import unet as U
    lib = hip
    assert lib.pis_conv3x3_filter_format(1, 256, 256, 64, 64, 0) == 3  # a direct layer (weight split)
    assert lib.pis_conv3x3_filter_format(1, 128, 128, 256, 256, 0) in (1, 2)  # a Winograd layer
    res = {}
    prev = U.UNetEngine.filter_ahead
    try:
        for mode in ("0", "2", "3", "4", "5"):
            U.UNetEngine.filter_ahead = mode
            u, grads, calls = _hip_step(1, 256, 256)
            res[mode] = (u, grads)
            bwd = calls[calls.index("<backward>"):]
            n_prep = sum(c == "pis_convt2x2_prep" for c in bwd)
            assert n_prep == (0 if mode in ("4", "5") else 4), (mode, n_prep)
    finally:
        U.UNetEngine.filter_ahead = prev
    for mode in ("2", "3", "4", "5"):
        assert torch.equal(res["0"][0], res[mode][0]), mode
        for a, b in zip(res["0"][1], res[mode][1]):
            assert torch.equal(a, b), mode


def test_engine_direct_splits_ahead_bitwise(hip):
    """PIS_FILTER_AHEAD 2 / 3 / 4 / 5 (the engine computes the Winograd layers' filter transforms
    (2), the direct layers' weight splits (3) or both (4: two launches on the main stream; 5: on the
    side stream behind events), both directions, at the forward's start and passes
    PIS_FILTER_READY): one training step gives bitwise the outputs and gradients of the default
    engine."""
    import importlib
    from physics_informed_image_segmentation_amd import unet as U
    tu = importlib.import_module("test_unet_gpu")
    res = {}
    prev = U.UNetEngine.filter_ahead
    try:
        for mode in ("0", "2", "3", "4", "5"):
            U.UNetEngine.filter_ahead = mode
            with Knobs(hip, k29=2):
                net, ref, u, crit, p_ref, terms, ref64 = tu._step_pair(1, 64, 64, dict())
            res[mode] = (u.detach().clone(), [p.grad.detach().clone() for p in net.parameters()])
            del net, ref, ref64
    finally:
        U.UNetEngine.filter_ahead = prev
    for mode in ("2", "3", "4", "5"):
        assert torch.equal(res["0"][0], res[mode][0]), mode
        for a, b in zip(res["0"][1], res[mode][1]):
            assert torch.equal(a, b), mode


def test_engine_schedule_knobs_bitwise(hip):
    """The backward's stream placements (unet.UNetEngine): the direct layers' weight gradients
    (PIS_DIRECT_WGRAD_MAIN), the fused-input-gradient layer's weight gradient (PIS_FUSED_WGRAD_MAIN)
    and the transposed convs' weight gradients (PIS_CONVT_WGRAD_MAIN levels) on the main stream or
    the weight-gradient stream run the same kernels on the same splits, so one training step is
    bitwise the same either way — B = 1 at 256 x 256 engages all three (direct 256^2 layers, the
    fused dec2.conv0 input gradient at 128^2, four transposed convs)."""
    from physics_informed_image_segmentation_amd import unet as U
    assert hip.pis_conv3x3_filter_format(1, 256, 256, 64, 64, 0) == 3  # direct
    assert hip.pis_conv3x3_filter_format(1, 128, 128, 256, 128, 1) == 2  # fused input gradient
    knobs = (("direct_wgrad_main", "0"), ("fused_wgrad_main", "0"), ("convt_wgrad_main", "1234"))
    prev = {a: getattr(U.UNetEngine, a) for a, _ in knobs}
    res = {}
    try:
        u, grads, _ = _hip_step(1, 256, 256)
        res["default"] = (u, grads)
        for a, v in knobs:
            setattr(U.UNetEngine, a, v)
            u, grads, _ = _hip_step(1, 256, 256)
            res[a] = (u, grads)
            setattr(U.UNetEngine, a, prev[a])
    finally:
        for a, v in prev.items():
            setattr(U.UNetEngine, a, v)
    for a, _ in knobs:
        assert torch.equal(res["default"][0], res[a][0]), a
        for g0, g1 in zip(res["default"][1], res[a][1]):
            assert torch.equal(g0, g1), a
