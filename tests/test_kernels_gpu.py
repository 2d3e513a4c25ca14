"""Per-kernel parity through the C-ABI on the GPU, against stock fp32 PyTorch on
the CPU (the ATen ops the reference calls) and the float64 numpy loss oracle."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import loss_numpy as ln
from oracle import reference_torch as rt

pytestmark = pytest.mark.gpu

RELU, SCALE, MASK, ACC = 1, 2, 4, 8


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()


def krsc(w):  # (O, I, 3, 3) -> [O][3][3][I]
    return w.permute(0, 2, 3, 1).contiguous()


def s():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("B,H,W,Cin,Cout,ld_extra", [(2, 16, 24, 64, 64, 0), (1, 8, 8, 128, 256, 64),
                                                      (3, 5, 7, 64, 128, 0), (2, 16, 16, 1, 64, 0), (2, 8, 128, 1, 64, 64), (1, 5, 64, 1, 64, 0),
                                                      (2, 16, 32, 64, 128, 64), (1, 8, 16, 132, 64, 0),
                                                      (2, 24, 48, 256, 192, 0)])
def test_conv3x3_fwd(hip, B, H, W, Cin, Cout, ld_extra):
    """H % 8 == 0 and W % 16 == 0 shapes take the halo kernel, the others the generic one."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(B, Cin, H, W, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g)
    scale = (torch.rand(B, Cout, generator=g) > 0.2).float() / 0.8
    ref = F.relu(F.conv2d(x, w, b, padding=1)) * scale[:, :, None, None]
    ldx = Cin + (ld_extra if Cin > 1 else 0)
    xbuf = torch.zeros(B, H, W, ldx)
    xbuf[..., :Cin] = nhwc(x)
    xd = xbuf.cuda()
    ldy = Cout + ld_extra
    y = torch.full((B, H, W, ldy), 7.0, device="cuda")
    wd, bd, sd = krsc(w).cuda(), b.cuda(), scale.cuda()
    rc = hip.pis_conv3x3_fwd(xd.data_ptr(), ldx, wd.data_ptr(), bd.data_ptr(), sd.data_ptr(), y.data_ptr(), ldy,
                             B, H, W, Cin, Cout, RELU | SCALE, s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    out = nchw(y[..., :Cout].cpu())
    assert rel_err(out, ref) < 1e-5
    if ld_extra:
        assert torch.all(y[..., Cout:] == 7.0)  # untouched channel slice


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 16, 24, 64, 64), (1, 8, 8, 256, 128), (2, 6, 10, 128, 64),
                                           (2, 16, 32, 64, 128), (1, 32, 16, 128, 64), (3, 5, 48, 192, 64)])
def test_conv3x3_dgrad_wgrad(hip, B, H, W, Cin, Cout):
    """W % 16 == 0 shapes take the 9-tap halo wgrad kernel, the others the generic one."""
    g = torch.Generator().manual_seed(1)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g))
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    dz = torch.randn(B, Cout, H, W, generator=g)
    scale = (torch.rand(B, Cin, generator=g) > 0.2).float() / 0.8
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dz, padding=1) * (x > 0) * scale[:, :, None, None]
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dz, padding=1)
    db_ref = dz.sum(dim=(0, 2, 3))
    xd, dzd, wd, sd = nhwc(x).cuda(), nhwc(dz).cuda(), krsc(w).cuda(), scale.cuda()
    wf = torch.empty(Cin * 9 * Cout, device="cuda")
    assert hip.pis_conv3x3_flip(wd.data_ptr(), wf.data_ptr(), Cin, Cout, s()) == 0
    dx = torch.empty(B, H, W, Cin, device="cuda")
    rc = hip.pis_conv3x3_dgrad(dzd.data_ptr(), Cout, wf.data_ptr(), xd.data_ptr(), Cin, sd.data_ptr(),
                               dx.data_ptr(), Cin, B, H, W, Cin, Cout, MASK | SCALE, s())
    assert rc == 0, hip.pis_last_error()
    nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
    db = torch.empty(Cout, device="cuda")
    rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                               B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    assert rel_err(nchw(dx.cpu()), dx_ref) < 1e-5
    assert rel_err(dw.cpu().permute(0, 3, 1, 2), dw_ref) < 1e-5
    assert rel_err(db.cpu(), db_ref) < 1e-5
    # accumulate mode adds on top
    rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                               B, H, W, Cin, Cout, ACC, ws.data_ptr(), nws, s())
    torch.cuda.synchronize()
    assert rel_err(dw.cpu().permute(0, 3, 1, 2), 2 * dw_ref) < 1e-5


# every non-default kernel variant behind pis_tune (include/pis_capi.h) stays exact too
TUNE_VARIANTS = [(4, 1), (4, 2), (4, 3), (5, 0), (6, 2048), (3, 0), (7, 1), (8, 0), (8, 2), (10, 0), (10, 1),
                 (11, 0), (13, 0), (13, 1), (13, 2), (13, 3), (10, 2), (10, 3), (14, 0), (14, 1), (14, 2), (15, 0), (16, 0), (17, 4), (22, 0), (25, 1), (26, 0), (26, 1), (27, 0), (31, 0), (46, 0)]


@pytest.mark.parametrize("key,value", TUNE_VARIANTS)
def test_conv3x3_tuned_variants(hip, key, value):
    prev = hip.pis_tune(key, value)
    try:
        for shape in [(2, 16, 32, 64, 64, 0), (2, 16, 32, 128, 256, 64), (1, 8, 16, 256, 64, 0)]:
            test_conv3x3_fwd(hip, *shape)
        for shape in [(2, 16, 32, 64, 128), (1, 32, 16, 128, 64), (2, 16, 48, 256, 256)]:
            test_conv3x3_dgrad_wgrad(hip, *shape)
        test_conv3x3_c1_wgrad(hip)
        for shape in [(2, 8, 12, 128, 64), (1, 16, 32, 256, 128)]:
            test_convt2x2(hip, *shape)
        for shape in [(2, 8, 8, 256, 256, 2), (1, 6, 10, 132, 64, 2), (2, 32, 64, 64, 128, 1),
                      (2, 32, 64, 128, 64, 1), (2, 32, 64, 128, 128, 1)]:
            test_conv3x3_ex_winograd(hip, *shape)
    finally:
        hip.pis_tune(key, prev)


@pytest.mark.parametrize("B,H,W,Cin,Cout,mode", [(2, 8, 8, 256, 256, 1), (1, 4, 6, 512, 256, 1),
                                                 (2, 8, 12, 128, 64, 1), (1, 12, 8, 64, 128, 1), (1, 8, 8, 64, 64, 1),
                                                 (2, 16, 32, 64, 128, 2), (1, 6, 10, 132, 64, 2),
                                                 (1, 5, 8, 256, 256, 2), (2, 8, 16, 256, 512, 0),
                                                 (3, 10, 6, 128, 64, 2),
                                                 # 64 -> 64 runs the fused contraction + output
                                                 # transform (key 15); the others the 3-pass path
                                                 (2, 32, 64, 64, 64, 1), (2, 32, 64, 128, 64, 1),
                                                 (2, 32, 64, 64, 128, 1), (2, 64, 64, 256, 128, 1),
                                                 (2, 32, 64, 128, 128, 1), (2, 64, 64, 128, 256, 1)])
def test_conv3x3_ex_winograd(hip, B, H, W, Cin, Cout, mode):
    """pis_conv3x3_fwd_ex / dgrad_ex with a workspace, and pis_conv3x3_wgrad: Winograd where the
    policy (pis_tune key 8: 1 = auto, 2 = whenever H, W are even) picks it, direct otherwise."""
    prev = hip.pis_tune(8, mode)
    try:
        g = torch.Generator().manual_seed(12)
        x = F.relu(torch.randn(B, Cin, H, W, generator=g))
        w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
        b = torch.randn(Cout, generator=g)
        scale = (torch.rand(B, Cout, generator=g) > 0.2).float() / 0.8
        dz = torch.randn(B, Cout, H, W, generator=g)
        sc_in = (torch.rand(B, Cin, generator=g) > 0.2).float() / 0.8
        y_ref = F.relu(F.conv2d(x, w, b, padding=1)) * scale[:, :, None, None]
        dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dz, padding=1) * (x > 0) * sc_in[:, :, None, None]
        nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
        f4 = hip.pis_tune(11, -1) != 0 and H % 4 == 0 and W % 4 == 0
        if f4:  # F(4x4,3x3) policy
            wino_fwd = wino_dgrad = max(Cin, Cout) >= 128 or (hip.pis_tune(10, -1) >= 3 and min(Cin, Cout) >= 64)
        else:  # F(2x2,3x3) policy
            wino_fwd = Cin >= 256 and Cout >= 128
            wino_dgrad = Cout >= 256 and Cin >= 128
        # a training forward that keeps its transform for the F(3x3,4x4) weight gradient runs
        # Winograd regardless, so the workspace covers it
        keepable = mode != 0 and f4 and Cin % 64 == 0 and Cout % 64 == 0
        assert (nws > 0) == (mode == 2 and H % 2 == 0 and W % 2 == 0 or mode == 1 and (wino_fwd or wino_dgrad)
                             or keepable)
        ws = torch.empty(max(nws, 4) // 4 + 1, device="cuda")
        xd, wd, bd, sd, dzd, sid = (nhwc(x).cuda(), krsc(w).cuda(), b.cuda(), scale.cuda(), nhwc(dz).cuda(),
                                    sc_in.cuda())
        y = torch.empty(B, H, W, Cout, device="cuda")
        rc = hip.pis_conv3x3_fwd_ex(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), sd.data_ptr(), y.data_ptr(),
                                    Cout, B, H, W, Cin, Cout, RELU | SCALE, ws.data_ptr(), nws, s())
        assert rc == 0, hip.pis_last_error()
        wf = torch.empty(Cin * 9 * Cout, device="cuda")
        assert hip.pis_conv3x3_flip(wd.data_ptr(), wf.data_ptr(), Cin, Cout, s()) == 0
        dx = torch.full((B, H, W, Cin), 0.5, device="cuda")
        rc = hip.pis_conv3x3_dgrad_ex(dzd.data_ptr(), Cout, wf.data_ptr(), xd.data_ptr(), Cin, sid.data_ptr(),
                                      dx.data_ptr(), Cin, B, H, W, Cin, Cout, MASK | SCALE | ACC, ws.data_ptr(), nws,
                                      s())
        assert rc == 0, hip.pis_last_error()
        torch.cuda.synchronize()
        assert rel_err(nchw(y.cpu()), y_ref) < 1e-5
        assert rel_err(nchw(dx.cpu()) - 0.5, dx_ref) < 1e-5
        if Cin % 64 or Cout % 64:
            return  # the weight-gradient API takes multiples of 64 channels
        # weight gradient (Winograd F(3x3,2x2) under the same policy)
        dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dz, padding=1)
        nwg = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
        wsg = torch.empty(nwg // 4 + 1, device="cuda")
        dw = torch.full((Cout, 3, 3, Cin), 0.25, device="cuda")
        db = torch.full((Cout,), 0.25, device="cuda")
        rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(), B, H, W,
                                   Cin, Cout, ACC, wsg.data_ptr(), nwg, s())
        assert rc == 0, hip.pis_last_error()
        torch.cuda.synchronize()
        assert rel_err(dw.cpu().permute(0, 3, 1, 2) - 0.25, dw_ref) < 1e-5
        assert rel_err(db.cpu() - 0.25, dz.sum(dim=(0, 2, 3))) < 1e-5
    finally:
        hip.pis_tune(8, prev)


def test_conv3x3_c1_wgrad(hip):
    _check_c1_wgrad(hip, 2, 32, 16)


@pytest.mark.parametrize("B,H,W", [(2, 24, 128), (1, 3, 64)])
def test_conv3x3_c1_wgrad_rows(hip, B, H, W):
    """W % 64 == 0: the row-segment Cin == 1 weight-gradient kernel."""
    _check_c1_wgrad(hip, B, H, W)


def _check_c1_wgrad(hip, B, H, W):
    Cout = 64
    g = torch.Generator().manual_seed(2)
    x = torch.rand(B, 1, H, W, generator=g)
    dz = torch.randn(B, Cout, H, W, generator=g)
    w = torch.zeros(Cout, 1, 3, 3)
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dz, padding=1)
    xd, dzd = nhwc(x).cuda(), nhwc(dz).cuda()
    nws = hip.pis_conv3x3_wgrad_ws(B, H, W, 1, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    dw = torch.empty(Cout, 3, 3, 1, device="cuda")
    db = torch.empty(Cout, device="cuda")
    assert hip.pis_conv3x3_wgrad(xd.data_ptr(), 1, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                                 B, H, W, 1, Cout, 0, ws.data_ptr(), nws, s()) == 0
    torch.cuda.synchronize()
    assert rel_err(dw.cpu().permute(0, 3, 1, 2), dw_ref) < 1e-5
    assert rel_err(db.cpu(), dz.sum(dim=(0, 2, 3))) < 1e-5


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 8, 12, 128, 64), (1, 4, 4, 512, 512), (2, 3, 5, 256, 128),
                                           (2, 8, 16, 128, 64), (1, 16, 32, 256, 128)])
def test_convt2x2(hip, B, H, W, Cin, Cout):
    """H % 8 == 0 and W % 16 == 0 inputs use 8x16-pixel tiles (shift-only pixel indexing)."""
    g = torch.Generator().manual_seed(3)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g)).requires_grad_(True)
    w = (torch.randn(Cin, Cout, 2, 2, generator=g) / Cin ** 0.5).requires_grad_(True)
    b = torch.randn(Cout, generator=g).requires_grad_(True)
    y = F.conv_transpose2d(x, w, b, stride=2)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    w_ijoc = w.detach().permute(2, 3, 1, 0).contiguous().cuda()  # [i][j][o][c]
    xd, bd = nhwc(x.detach()).cuda(), b.detach().cuda()
    ld = 2 * Cout  # write into the first half of a concat buffer
    yb = torch.zeros(B, 2 * H, 2 * W, ld, device="cuda")
    assert hip.pis_convt2x2_fwd(xd.data_ptr(), Cin, w_ijoc.data_ptr(), bd.data_ptr(), yb.data_ptr(), ld,
                                B, H, W, Cin, Cout, s()) == 0
    dyb = torch.zeros(B, 2 * H, 2 * W, ld, device="cuda")
    dyb[..., :Cout] = nhwc(dy).cuda()
    wc = torch.empty(Cin * 4 * Cout, device="cuda")
    assert hip.pis_convt2x2_prep(w_ijoc.data_ptr(), wc.data_ptr(), Cin, Cout, s()) == 0
    dx = torch.empty(B, H, W, Cin, device="cuda")
    assert hip.pis_convt2x2_dgrad(dyb.data_ptr(), ld, wc.data_ptr(), xd.data_ptr(), Cin, dx.data_ptr(), Cin,
                                  B, H, W, Cin, Cout, MASK, s()) == 0
    nws = hip.pis_convt2x2_wgrad_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    dw = torch.empty(2, 2, Cout, Cin, device="cuda")
    db = torch.empty(Cout, device="cuda")
    assert hip.pis_convt2x2_wgrad(xd.data_ptr(), Cin, dyb.data_ptr(), ld, dw.data_ptr(), db.data_ptr(),
                                  B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s()) == 0
    torch.cuda.synchronize()
    assert rel_err(nchw(yb[..., :Cout].cpu()), y.detach()) < 1e-5
    assert torch.all(yb[..., Cout:] == 0)
    assert rel_err(nchw(dx.cpu()), x.grad * (x.detach() > 0)) < 1e-5
    assert rel_err(dw.cpu().permute(3, 2, 0, 1), w.grad) < 1e-5
    assert rel_err(db.cpu(), b.grad) < 1e-5


@pytest.mark.parametrize("B,H,W,Cin,Cout,ld_extra", [(2, 16, 32, 128, 64, 64), (1, 8, 64, 256, 128, 0),
                                                    (1, 8, 32, 512, 256, 0), (2, 4, 32, 1024, 512, 0)])
def test_convt2x2_k32(hip, B, H, W, Cin, Cout, ld_extra):
    """The K-step-32 transposed-conv kernel (pis_tune key 13 = 4): forward into a concat slice (+bias),
    input gradient gathered from a strided dy with the ReLU mask and accumulate, vs fp32 ATen."""
    prev = hip.pis_tune(13, 4)
    try:
        g = torch.Generator().manual_seed(33)
        x = F.relu(torch.randn(B, Cin, H, W, generator=g))
        w = torch.randn(Cin, Cout, 2, 2, generator=g) / Cin ** 0.5
        b = torch.randn(Cout, generator=g)
        y_ref = F.conv_transpose2d(x, w, b, stride=2)
        dy = torch.randn(y_ref.shape, generator=g)
        xr, wr, br = x.clone().requires_grad_(True), w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        F.conv_transpose2d(xr, wr, br, stride=2).backward(dy)
        dx_ref = xr.grad * (x > 0)
        ld = Cout + ld_extra
        w_ijoc = w.permute(2, 3, 1, 0).contiguous().cuda()
        xd, bd = nhwc(x).cuda(), b.cuda()
        yb = torch.zeros(B, 2 * H, 2 * W, ld, device="cuda")
        assert hip.pis_convt2x2_fwd(xd.data_ptr(), Cin, w_ijoc.data_ptr(), bd.data_ptr(), yb.data_ptr(), ld,
                                    B, H, W, Cin, Cout, s()) == 0, hip.pis_last_error()
        dyb = torch.zeros(B, 2 * H, 2 * W, ld, device="cuda")
        dyb[..., :Cout] = nhwc(dy).cuda()
        wc = torch.empty(Cin * 4 * Cout, device="cuda")
        assert hip.pis_convt2x2_prep(w_ijoc.data_ptr(), wc.data_ptr(), Cin, Cout, s()) == 0
        dx = torch.full((B, H, W, Cin), 0.5, device="cuda")
        assert hip.pis_convt2x2_dgrad(dyb.data_ptr(), ld, wc.data_ptr(), xd.data_ptr(), Cin, dx.data_ptr(), Cin,
                                      B, H, W, Cin, Cout, MASK | ACC, s()) == 0, hip.pis_last_error()
        # weight + bias gradient (the row-staged split-K kernel with the up-sampled A gather), accumulating
        nws = hip.pis_convt2x2_wgrad_ws(B, H, W, Cin, Cout)
        ws = torch.empty(nws // 4 + 1, device="cuda")
        dw = torch.full((2, 2, Cout, Cin), 0.25, device="cuda")
        db = torch.full((Cout,), 0.25, device="cuda")
        assert hip.pis_convt2x2_wgrad(xd.data_ptr(), Cin, dyb.data_ptr(), ld, dw.data_ptr(), db.data_ptr(),
                                      B, H, W, Cin, Cout, ACC, ws.data_ptr(), nws, s()) == 0, hip.pis_last_error()
        torch.cuda.synchronize()
        assert rel_err(nchw(yb[..., :Cout].cpu()), y_ref) < 1e-5
        assert torch.all(yb[..., Cout:] == 0)
        assert rel_err(nchw(dx.cpu()) - 0.5, dx_ref) < 1e-5
        assert rel_err(dw.cpu().permute(3, 2, 0, 1) - 0.25, wr.grad) < 1e-5
        assert rel_err(db.cpu() - 0.25, br.grad) < 1e-5
    finally:
        hip.pis_tune(13, prev)


def test_maxpool(hip):
    B, H, W, C = 2, 8, 12, 64
    g = torch.Generator().manual_seed(4)
    x = F.relu(torch.randn(B, C, H, W, generator=g))
    x[0, :, 0:2, 0:2] = 0.5  # ties -> first occurrence, as ATen
    x.requires_grad_(True)
    y = F.max_pool2d(x, 2, 2)
    dy = torch.randn(y.shape, generator=g)
    y.backward(dy)
    dskip = torch.randn(B, C, H, W, generator=g)
    ld = 2 * C
    xb = torch.zeros(B, H, W, ld)
    xb[..., C:] = nhwc(x.detach())
    xb = xb.cuda()
    xs = xb[..., C:]
    yd = torch.empty(B, H // 2, W // 2, C, device="cuda")
    assert hip.pis_maxpool2x2_fwd(xs.data_ptr(), ld, yd.data_ptr(), B, H, W, C, s()) == 0
    dsk = nhwc(dskip).cuda()
    dx = torch.empty(B, H, W, C, device="cuda")
    assert hip.pis_maxpool2x2_bwd(xs.data_ptr(), ld, nhwc(dy).cuda().data_ptr(), dsk.data_ptr(), C,
                                  dx.data_ptr(), C, B, H, W, C, s()) == 0
    torch.cuda.synchronize()
    assert torch.equal(nchw(yd.cpu()), y.detach())
    ref = (x.grad + dskip) * (x.detach() > 0)
    assert rel_err(nchw(dx.cpu()), ref) < 1e-6


def test_head(hip):
    B, H, W, C = 2, 16, 8, 64
    g = torch.Generator().manual_seed(5)
    x = F.relu(torch.randn(B, C, H, W, generator=g)).requires_grad_(True)
    w = torch.randn(1, C, 1, 1, generator=g).requires_grad_(True)
    b = torch.randn(1, generator=g).requires_grad_(True)
    z = F.conv2d(x, w, b)
    z.retain_grad()
    u = torch.sigmoid(z)
    du = torch.randn(u.shape, generator=g)
    u.backward(du)
    xd = nhwc(x.detach()).cuda()
    wd, bd = w.detach().reshape(C).cuda(), b.detach().cuda()
    zd = torch.empty(B * H * W, device="cuda")
    ud = torch.empty(B * H * W, device="cuda")
    assert hip.pis_head_fwd(xd.data_ptr(), C, wd.data_ptr(), bd.data_ptr(), zd.data_ptr(), ud.data_ptr(),
                            B * H * W, C, s()) == 0
    dz = z.grad.reshape(-1).cuda()
    dx = torch.empty(B, H, W, C, device="cuda")
    dw = torch.empty(C, device="cuda")
    db = torch.empty(1, device="cuda")
    nws = hip.pis_head_bwd_ws(B * H * W, C)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    assert hip.pis_head_bwd(xd.data_ptr(), C, wd.data_ptr(), dz.data_ptr(), 0, dx.data_ptr(), C, dw.data_ptr(),
                            db.data_ptr(), B * H * W, C, 0, ws.data_ptr(), nws, s()) == 0
    # sigmoid-chained form: feed dL/du and u
    dx2 = torch.empty_like(dx)
    dw2 = torch.empty_like(dw)
    db2 = torch.empty_like(db)
    dud = du.reshape(-1).cuda()
    assert hip.pis_head_bwd(xd.data_ptr(), C, wd.data_ptr(), dud.data_ptr(), ud.data_ptr(), dx2.data_ptr(), C,
                            dw2.data_ptr(), db2.data_ptr(), B * H * W, C, 0, ws.data_ptr(), nws, s()) == 0
    torch.cuda.synchronize()
    assert rel_err(nchw(dx2.cpu()), x.grad * (x.detach() > 0)) < 1e-5
    assert rel_err(dw2.cpu(), w.grad.reshape(C)) < 1e-5
    assert rel_err(db2.cpu(), b.grad) < 1e-5
    assert rel_err(ud.cpu(), u.detach().reshape(-1)) < 1e-6
    assert rel_err(zd.cpu(), z.detach().reshape(-1)) < 1e-6
    assert rel_err(nchw(dx.cpu()), x.grad * (x.detach() > 0)) < 1e-6
    assert rel_err(dw.cpu(), w.grad.reshape(C)) < 1e-5
    assert rel_err(db.cpu(), b.grad) < 1e-5


@pytest.mark.parametrize("B,H,W,ldx", [(2, 64, 64, 64), (1, 48, 80, 128), (3, 2, 3 * 4, 64), (1, 40, 1024, 64)])
@pytest.mark.parametrize("kw", [dict(), dict(rd_w=0.3, pf_w=0.2, D=5.0, a=0.5, eps=0.05), dict(rd_w=0.3, D=0.5),
                                dict(pf_w=0.2, eps=0.1)])
def test_head_loss_bwd_fused(hip, B, H, W, ldx, kw):
    """pis_head_loss_bwd == pis_loss_bwd (dL/du) followed by pis_head_bwd (sigmoid chain)."""
    from physics_informed_image_segmentation_amd._hip import LossParams
    import ctypes
    C = 64
    g = torch.Generator().manual_seed(9)
    x = F.relu(torch.randn(B, H, W, ldx, generator=g)).cuda()
    w = torch.randn(C, generator=g).cuda() * 0.1
    u = (0.02 + 0.96 * torch.rand(B, H, W, generator=g)).cuda()
    t = (torch.rand(B, H, W, generator=g) > 0.7).float().cuda()
    prm = LossParams(0.5, 0.5, kw.get("rd_w", 0.0), kw.get("pf_w", 0.0), 1e-6, kw.get("D", 1.0), kw.get("a", 0.5),
                     kw.get("eps", 0.05), 0.5, 0)
    terms = torch.empty(8, device="cuda")
    lws = torch.zeros(hip.pis_loss_ws(B, H, W) // 4 + 1, device="cuda")
    assert hip.pis_loss_fwd(u.data_ptr(), t.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(), 0, 0,
                            lws.data_ptr(), lws.numel() * 4, s()) == 0
    go = torch.tensor([0.75], device="cuda")
    # reference composition
    du_ref = torch.empty(B, H, W, device="cuda")
    assert hip.pis_loss_bwd(u.data_ptr(), t.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(), go.data_ptr(),
                            du_ref.data_ptr(), 0, s()) == 0
    npix = B * H * W
    hws = torch.empty(hip.pis_head_bwd_ws(npix, C) // 4 + 1, device="cuda")
    dx_ref = torch.empty(B, H, W, C, device="cuda")
    dw_ref, db_ref = torch.empty(C, device="cuda"), torch.empty(1, device="cuda")
    assert hip.pis_head_bwd(x.data_ptr(), ldx, w.data_ptr(), du_ref.data_ptr(), u.data_ptr(), dx_ref.data_ptr(), C,
                            dw_ref.data_ptr(), db_ref.data_ptr(), npix, C, 0, hws.data_ptr(), hws.numel() * 4,
                            s()) == 0
    # fused, accumulating onto 1.0 to check the flag
    fws = torch.empty(hip.pis_head_loss_bwd_ws(B, H, W, C) // 4 + 1, device="cuda")
    du = torch.empty(B, H, W, device="cuda")
    dx = torch.full((B, H, W, C), 3.0, device="cuda")
    dw, db = torch.ones(C, device="cuda"), torch.ones(1, device="cuda")
    rc = hip.pis_head_loss_bwd(x.data_ptr(), ldx, w.data_ptr(), u.data_ptr(), t.data_ptr(), du.data_ptr(), B, H, W,
                               C, ctypes.byref(prm), terms.data_ptr(), go.data_ptr(), dx.data_ptr(), C,
                               dw.data_ptr(), db.data_ptr(), ACC, fws.data_ptr(), fws.numel() * 4, s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    assert rel_err(du.cpu(), du_ref.cpu()) < 1e-6
    assert rel_err(dx.cpu(), dx_ref.cpu()) < 1e-6
    assert rel_err(dw.cpu(), (dw_ref + 1).cpu()) < 1e-6  # accumulated onto the 1.0 already there
    assert rel_err(db.cpu(), (db_ref + 1).cpu()) < 1e-6


def _loss_call(hip, p, t, kw, chain=False, grad_out=None, ws=None, all_terms=True):
    from physics_informed_image_segmentation_amd._hip import LossParams
    import ctypes
    B, H, W = p.shape[0], p.shape[-2], p.shape[-1]
    prm = LossParams(kw.get("dice_w", 0.5), kw.get("bce_w", 0.5), kw.get("rd_w", 0.0), kw.get("pf_w", 0.0),
                     kw.get("smooth", 1e-6), kw.get("D", 1.0), kw.get("a", 0.5), kw.get("eps", 0.05), 0.5,
                     1 if all_terms else 0)
    pd, td = p.contiguous().cuda(), t.contiguous().cuda()
    terms = torch.empty(8, device="cuda")
    counts = torch.empty(B, 3, dtype=torch.int32, device="cuda")
    scores = torch.empty(B, 2, device="cuda")
    nws = hip.pis_loss_ws(B, H, W)
    if ws is None:
        ws = torch.zeros(nws // 4 + 1, device="cuda")
    assert hip.pis_loss_fwd(pd.data_ptr(), td.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(),
                            counts.data_ptr(), scores.data_ptr(), ws.data_ptr(), nws, s()) == 0
    dst = torch.empty(B, H, W, device="cuda")
    go = None if grad_out is None else torch.tensor([grad_out], device="cuda")
    assert hip.pis_loss_bwd(pd.data_ptr(), td.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(),
                            0 if go is None else go.data_ptr(), dst.data_ptr(), 2 if chain else 0, s()) == 0
    torch.cuda.synchronize()
    return terms.cpu(), counts.cpu(), scores.cpu(), dst.cpu()


# shapes cover ragged widths (W % 4 != 0), partial 16x128 tiles, full vector tiles and
# tiny reflect-padded images
@pytest.mark.parametrize("shape", [(2, 9, 11), (8, 64, 64), (1, 2, 3), (3, 130, 70), (2, 40, 260), (1, 33, 256)])
@pytest.mark.parametrize("kw", [dict(), dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05),
                                dict(rd_w=0.3, D=0.5, a=0.3), dict(pf_w=0.2, eps=0.1)])
def test_fused_loss_vs_oracle(hip, shape, kw):
    g = torch.Generator().manual_seed(6)
    p = 0.02 + 0.96 * torch.rand(shape, generator=g)
    t = (torch.rand(shape, generator=g) > 0.7).float()
    terms, counts, scores, dp = _loss_call(hip, p, t, kw, grad_out=0.75)
    f = ln.loss_forward(p.numpy(), t.numpy(), **kw)
    assert terms[0].item() == pytest.approx(f["loss"], rel=1e-5)
    assert terms[1].item() == pytest.approx(f["dice_loss"], rel=1e-5)
    assert terms[2].item() == pytest.approx(f["bce_loss"], rel=1e-5)
    assert terms[3].item() == pytest.approx(f["rd"], rel=1e-4, abs=1e-12)
    assert terms[4].item() == pytest.approx(f["pf"], rel=1e-4, abs=1e-12)
    gref = ln.loss_backward(p.numpy(), t.numpy(), grad_out=0.75, **kw)
    err = np.linalg.norm(dp.numpy() - gref) / np.linalg.norm(gref)
    assert err < 1e-5
    assert np.abs(dp.numpy() - gref).max() <= 1e-5 * np.abs(gref).max()  # every pixel, boundaries included
    i, ph, ts = ln.sample_counts(p.numpy(), t.numpy())
    assert np.array_equal(counts.numpy(), np.stack([i, ph, ts], 1))
    d, u = ln.dice_iou_from_counts(i, ph, ts)
    np.testing.assert_allclose(scores.numpy(), np.stack([d, u], 1), rtol=1e-6)


def _c4_prediction(B, H, W, seed):
    """A prediction-like probability map for the disc masks of rt.synthetic_batch: the mask blurred
    with noise and squashed into (0, 1), so the stencils see real edges and BCE / Dice real errors."""
    _, mask = rt.synthetic_batch(B, H, W, seed=42)
    g = torch.Generator().manual_seed(seed)
    z = 6.0 * (mask - 0.5) + 2.0 * torch.randn(B, 1, H, W, generator=g)
    z = F.avg_pool2d(F.pad(z, (2, 2, 2, 2), mode="reflect"), 5, stride=1)
    return torch.sigmoid(z)[:, 0].float(), mask[:, 0].float()


# BASELINE C4 = run_ablation.py:42-83 R1 (Baseline / RD-only / PF-only / RD+PF) at lambda 1e-4, D = 5,
# a = 0.5, eps = 0.05
C4_GATINGS = [(0.0, 0.0), (1e-4, 0.0), (0.0, 1e-4), (1e-4, 1e-4)]


@pytest.mark.parametrize("rd_w,pf_w", C4_GATINGS)
def test_fused_loss_c4_grid_vs_oracle(hip, rd_w, pf_w):
    """C4 at its stated size, (8, 512, 512), through the production gating (no PIS_LOSS_ALL_TERMS: the
    kernels specialise on the weights, the lambda = 0 instantiation included) on the whole-row band
    grid the C2 step runs, against the float64 oracle (oracle/loss_numpy.py, src/loss.py:144-160):
    every term in the total, every pixel of dL/dp (boundaries included), exact per-sample counters."""
    p, t = _c4_prediction(8, 512, 512, seed=14)
    kw = dict(rd_w=rd_w, pf_w=pf_w, D=5.0, a=0.5, eps=0.05)
    terms, counts, scores, dp = _loss_call(hip, p, t, kw, grad_out=0.75, all_terms=False)
    f = ln.loss_forward(p.numpy(), t.numpy(), **kw)
    assert terms[0].item() == pytest.approx(f["loss"], rel=1e-5)
    assert terms[1].item() == pytest.approx(f["dice_loss"], rel=1e-5)
    assert terms[2].item() == pytest.approx(f["bce_loss"], rel=1e-5)
    if rd_w > 0:
        assert terms[3].item() == pytest.approx(f["rd"], rel=1e-4)
    if pf_w > 0:
        assert terms[4].item() == pytest.approx(f["pf"], rel=1e-4)
    gref = ln.loss_backward(p.numpy(), t.numpy(), grad_out=0.75, **kw)
    assert np.linalg.norm(dp.numpy() - gref) / np.linalg.norm(gref) < 1e-5
    assert np.abs(dp.numpy() - gref).max() <= 1e-5 * np.abs(gref).max()
    i, ph, ts = ln.sample_counts(p.numpy(), t.numpy())
    assert np.array_equal(counts.numpy(), np.stack([i, ph, ts], 1))
    d, u = ln.dice_iou_from_counts(i, ph, ts)
    np.testing.assert_allclose(scores.numpy(), np.stack([d, u], 1), rtol=1e-6)


@pytest.mark.parametrize("rd_w,pf_w", C4_GATINGS)
def test_head_loss_bwd_c4_grid_vs_oracle(hip, rd_w, pf_w):
    """The C2 step's loss backward is head_loss_bwd_kernel<RD, PF> (the loss adjoint fused into the
    head backward), not loss_bwd_kernel: here it runs at the C2 grid (8, 512, 512) under the four R1
    gatings (BASELINE C4, run_ablation.py:42-83) through the production gating, against float64:
    oracle/loss_numpy.py:loss_backward (src/loss.py:114-162, src/pde.py:124-212) -> dL/du at every
    pixel, the sigmoid chain (src/unet.py:206-210) -> dL/dz, and the 64-channel 1x1 head's
    gradients dx = dz w [x > 0], dw = sum dz x, db = sum dz (src/unet.py:157) at every pixel and
    channel."""
    from physics_informed_image_segmentation_amd._hip import LossParams
    B, H, W, C = 8, 512, 512, 64
    u, t = _c4_prediction(B, H, W, seed=15)
    g = torch.Generator().manual_seed(16)
    x = F.relu(torch.randn(B, H, W, C, generator=g))
    w = torch.randn(C, generator=g) * 0.1
    kw = dict(rd_w=rd_w, pf_w=pf_w, D=5.0, a=0.5, eps=0.05)
    prm = LossParams(0.5, 0.5, rd_w, pf_w, 1e-6, 5.0, 0.5, 0.05, 0.5, 0)
    ud, td, xd, wd = u.cuda(), t.cuda(), x.cuda(), w.cuda()
    terms = torch.empty(8, device="cuda")
    lws = torch.zeros(hip.pis_loss_ws(B, H, W) // 4 + 1, device="cuda")
    assert hip.pis_loss_fwd(ud.data_ptr(), td.data_ptr(), B, H, W, ctypes.byref(prm), terms.data_ptr(), 0, 0,
                            lws.data_ptr(), lws.numel() * 4, s()) == 0
    fws = torch.empty(hip.pis_head_loss_bwd_ws(B, H, W, C) // 4 + 1, device="cuda")
    du = torch.empty(B, H, W, device="cuda")
    dx = torch.empty(B, H, W, C, device="cuda")
    dw, db = torch.empty(C, device="cuda"), torch.empty(1, device="cuda")
    rc = hip.pis_head_loss_bwd(xd.data_ptr(), C, wd.data_ptr(), ud.data_ptr(), td.data_ptr(), du.data_ptr(), B, H, W,
                               C, ctypes.byref(prm), terms.data_ptr(), 0, dx.data_ptr(), C, dw.data_ptr(),
                               db.data_ptr(), 0, fws.data_ptr(), fws.numel() * 4, s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    del xd
    gref = ln.loss_backward(u.numpy(), t.numpy(), **kw)  # float64 dL/du
    du_h = du.cpu().numpy()
    assert np.linalg.norm(du_h - gref) / np.linalg.norm(gref) < 1e-5
    assert np.abs(du_h - gref).max() <= 1e-5 * np.abs(gref).max()  # every pixel, boundaries included
    u64 = u.double()
    dz64 = torch.from_numpy(gref) * u64 * (1.0 - u64)  # sigmoid chain
    x64 = x.reshape(-1, C).double()
    dw64 = x64.t() @ dz64.reshape(-1)
    db64 = dz64.sum()
    assert rel_err(dw.cpu().double(), dw64) < 1e-5
    assert abs(db.item() - db64.item()) <= 1e-5 * dz64.abs().sum().item()  # fp32 summation bound
    dx_h = dx.cpu().reshape(-1, C)
    scale = (dz64.abs().max() * w.double().abs().max()).item()
    for i0 in range(0, x64.shape[0], 1 << 19):  # every pixel and channel, in chunks
        sl = slice(i0, i0 + (1 << 19))
        dx64 = dz64.reshape(-1)[sl, None] * w.double()[None, :] * (x64[sl] > 0)
        assert (dx_h[sl].double() - dx64).abs().max().item() <= 1e-5 * scale


def _head_loss_fwd_call(hip, x, ldx, w, b, t, kw, all_terms=False):
    """pis_head_loss_fwd on x ([B,H,W,ldx], the first 64 channels the head input) -> (z, u, terms,
    counts, scores) on the host."""
    from physics_informed_image_segmentation_amd._hip import LossParams
    B, H, W = t.shape
    prm = LossParams(0.5, 0.5, kw.get("rd_w", 0.0), kw.get("pf_w", 0.0), 1e-6, kw.get("D", 1.0), kw.get("a", 0.5),
                     kw.get("eps", 0.05), 0.5, 1 if all_terms else 0)
    z, u = torch.empty(B, H, W, device="cuda"), torch.empty(B, H, W, device="cuda")
    terms = torch.empty(8, device="cuda")
    counts = torch.empty(B, 3, dtype=torch.int32, device="cuda")
    scores = torch.empty(B, 2, device="cuda")
    nws = hip.pis_head_loss_fwd_ws(B, H, W)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    assert hip.pis_head_loss_fwd_ok(B, H, W, 64) == 1
    rc = hip.pis_head_loss_fwd(x.data_ptr(), ldx, w.data_ptr(), b.data_ptr(), t.data_ptr(), z.data_ptr(), u.data_ptr(),
                               B, H, W, 64, ctypes.byref(prm), terms.data_ptr(), counts.data_ptr(), scores.data_ptr(),
                               ws.data_ptr(), nws, s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    return z.cpu(), u.cpu(), terms.cpu(), counts.cpu(), scores.cpu()


@pytest.mark.parametrize("B,H,W,ldx", [(2, 64, 64, 64), (1, 48, 128, 128), (3, 2, 64, 64), (1, 40, 1024, 64),
                                       (2, 37, 512, 64), (8, 512, 512, 64), (1, 11, 1280, 64), (2, 9, 2048, 64)])
@pytest.mark.parametrize("rd_w,pf_w", C4_GATINGS)
def test_head_loss_fwd_fused(hip, B, H, W, ldx, rd_w, pf_w):
    """pis_head_loss_fwd (the head's 1x1 conv + sigmoid fused with the loss forward, the C2 step's
    path) == pis_head_fwd then pis_loss_fwd: z and u bitwise, the counters exactly, the terms to fp32
    summation order; and against the float64 oracle (oracle/loss_numpy.py on the same u): every
    term in the total, the counters and scores. Shapes: band heights that do not divide H (37),
    H = 2 (every row a reflect ghost), 1024-wide rows (8 rows per band), the C2 grid (8, 512, 512)
    under the four R1 gatings (BASELINE C4), a wider row pitch (concat-style ldx), and rows wider
    than 4 x 256 threads (1280: 256-thread blocks walk 320 column items; 2048) so a thread's loss
    pass covers several column items."""
    g = torch.Generator().manual_seed(31)
    x = F.relu(torch.randn(B, H, W, ldx, generator=g)).cuda()
    w = (torch.randn(64, generator=g) * 0.15).cuda()
    b = torch.tensor([-0.3]).cuda()
    _, mask = rt.synthetic_batch(B, H, W, seed=42)
    t = mask[:, 0].contiguous().cuda()
    kw = dict(rd_w=rd_w, pf_w=pf_w, D=5.0, a=0.5, eps=0.05)
    z, u, terms, counts, scores = _head_loss_fwd_call(hip, x, ldx, w, b, t, kw)
    # the unfused pair on the same input
    z2, u2 = torch.empty(B, H, W, device="cuda"), torch.empty(B, H, W, device="cuda")
    assert hip.pis_head_fwd(x.data_ptr(), ldx, w.data_ptr(), b.data_ptr(), z2.data_ptr(), u2.data_ptr(), B * H * W, 64,
                            s()) == 0
    torch.cuda.synchronize()
    assert torch.equal(z, z2.cpu()) and torch.equal(u, u2.cpu())
    ref = _loss_call(hip, u2, t, kw, all_terms=False)
    np.testing.assert_allclose(terms.numpy(), ref[0].numpy(), rtol=2e-6, atol=1e-12)
    assert torch.equal(counts, ref[1]) and torch.equal(scores, ref[2])
    # float64 oracle on the same probabilities
    f = ln.loss_forward(u.numpy(), t.cpu().numpy(), **kw)
    assert terms[0].item() == pytest.approx(f["loss"], rel=1e-5)
    assert terms[1].item() == pytest.approx(f["dice_loss"], rel=1e-5)
    assert terms[2].item() == pytest.approx(f["bce_loss"], rel=1e-5)
    if rd_w > 0:
        assert terms[3].item() == pytest.approx(f["rd"], rel=1e-4)
    if pf_w > 0:
        assert terms[4].item() == pytest.approx(f["pf"], rel=1e-4)
    i, ph, ts = ln.sample_counts(u.numpy(), t.cpu().numpy())
    assert np.array_equal(counts.numpy(), np.stack([i, ph, ts], 1))
    # z against fp64 of the same fp32 inputs
    z64 = (x[..., :64].double() @ w.double() + b.double()).cpu()
    assert ((z.double() - z64).abs().max() / z64.abs().max()).item() < 1e-6


@pytest.mark.parametrize("B,H,W", [(2, 37, 512), (8, 512, 512), (1, 40, 1024), (1, 13, 2048), (3, 2, 512),
                                   (16, 512, 512)])
def test_head_loss_fwd_variants(hip, B, H, W):
    """pis_tune(38): the 256-thread bands (0), the 1024-thread bands (1) and the same with three
    register sets in flight (2) give bitwise the same z, u and counters, and the same terms to fp32
    summation order; repeated calls are bitwise the same. Shapes: ragged bands (37), H = 2 (every
    staged row a reflect ghost), 1024 / 2048-wide rows (2 / 4 chunks per row), C2, and 2x C2's
    batch."""
    g = torch.Generator().manual_seed(37)
    x = F.relu(torch.randn(B, H, W, 64, generator=g)).cuda()
    w = (torch.randn(64, generator=g) * 0.15).cuda()
    b = torch.tensor([-0.3]).cuda()
    _, mask = rt.synthetic_batch(B, H, W, seed=43)
    t = mask[:, 0].contiguous().cuda()
    kw = dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05)
    outs = {}
    for v in (0, 1, 2):
        prev = hip.pis_tune(38, v)
        try:
            outs[v] = _head_loss_fwd_call(hip, x, 64, w, b, t, kw)
            if v == 1:
                for _ in range(2):
                    again = _head_loss_fwd_call(hip, x, 64, w, b, t, kw)
                    assert all(torch.equal(a_, b_) for a_, b_ in zip(again, outs[v]))
        finally:
            hip.pis_tune(38, prev)
    for v in (1, 2):
        for k in (0, 1, 3, 4):  # z, u, counts, scores
            assert torch.equal(outs[v][k], outs[0][k]), (v, k)
        np.testing.assert_allclose(outs[v][2].numpy(), outs[0][2].numpy(), rtol=2e-6, atol=1e-12)


@pytest.mark.parametrize("shape", [(16, 512, 512), (3, 130, 68), (2, 2, 8), (1, 37, 1024), (5, 64, 4096), (4, 5, 20), (64, 512, 512)])
@pytest.mark.parametrize("terms", [(1e-4, 1e-4), (0.0, 0.0), (1e-4, 0.0), (0.0, 1e-4)])
def test_loss_fwd_row_bands_match_tile_path(hip, shape, terms):
    """The whole-row forward (PIS_TUNE_LOSS_ROWS = 1) and the 16x128-tile forward give the same
    terms and exactly the same counters; repeated launches on one workspace are bitwise identical
    (fixed-order reductions)."""
    g = torch.Generator().manual_seed(12)
    p = 0.02 + 0.96 * torch.rand(shape, generator=g)
    t = (torch.rand(shape, generator=g) > 0.8).float()
    kw = dict(rd_w=terms[0], pf_w=terms[1], D=5.0, a=0.5, eps=0.05)
    prev = hip.pis_tune(18, 0)
    try:
        ref = _loss_call(hip, p, t, kw)
    finally:
        hip.pis_tune(18, prev)
    assert hip.pis_tune(18, -1) == 1
    ws = torch.zeros(hip.pis_loss_ws(*shape) // 4 + 1, device="cuda")
    first = None
    for _ in range(3):  # one workspace, reused
        got = _loss_call(hip, p, t, kw, ws=ws)
        np.testing.assert_allclose(got[0].numpy(), ref[0].numpy(), rtol=2e-6, atol=1e-12)
        assert torch.equal(got[1], ref[1])
        assert torch.equal(got[2], ref[2])
        np.testing.assert_allclose(got[3].numpy(), ref[3].numpy(), rtol=1e-5, atol=1e-12)
        if first is not None:
            assert torch.equal(got[0], first)  # deterministic: fixed-order reduction
        first = got[0]


def test_fused_loss_chain_sigmoid(hip):
    g = torch.Generator().manual_seed(8)
    p = torch.sigmoid(torch.randn(2, 33, 17, generator=g))
    t = (torch.rand(2, 33, 17, generator=g) > 0.5).float()
    kw = dict(rd_w=1e-2, pf_w=1e-2, D=5.0, a=0.5, eps=0.05)
    _, _, _, dz = _loss_call(hip, p, t, kw, chain=True)
    gref = ln.loss_backward(p.numpy(), t.numpy(), chain_sigmoid=True, **kw)
    assert np.linalg.norm(dz.numpy() - gref) / np.linalg.norm(gref) < 1e-5


def test_pinned_observation_loss_terms(hip):
    # the reference's own loss values on its own seed-42 batch via the fused kernel
    img, mask = rt.synthetic_batch(2, 256, 256, seed=42)
    torch.manual_seed(42)
    net = rt.UNetRef(1, 1, 64).eval()
    with torch.no_grad():
        u = net(img)
    kw = dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05)
    terms, counts, scores, _ = _loss_call(hip, u[:, 0], mask[:, 0], kw)
    assert terms[0].item() == pytest.approx(0.7671615481, rel=1e-5)
    assert terms[3].item() == pytest.approx(2.58888e-05, rel=1e-4)
    assert terms[4].item() == pytest.approx(1.24887013, rel=1e-5)


def test_adamw_matches_torch(hip):
    g = torch.Generator().manual_seed(9)
    n = 1000 + 3
    p0 = torch.randn(n, generator=g)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-5)
    pd = p0.clone().cuda()
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    for step in range(1, 4):
        grad = torch.randn(n, generator=g)
        ref.grad = grad.clone()
        opt.step()
        gd = grad.cuda()
        bc1 = 1 - 0.9 ** step
        bc2 = 1 - 0.999 ** step
        assert hip.pis_adamw_step(pd.data_ptr(), gd.data_ptr(), m.data_ptr(), v.data_ptr(), n, 1e-3, 0.9, 0.999,
                                  1e-8, 1e-5, 1e-3 / bc1, bc2 ** 0.5, 1.0, s()) == 0
    torch.cuda.synchronize()
    assert rel_err(pd.cpu(), ref.detach()) < 1e-6


@pytest.mark.parametrize("B,H,W,Cin,Cout,small_ws", [(2, 8, 8, 128, 128, False), (1, 8, 12, 64, 128, False),
                                                     (2, 12, 8, 128, 64, False), (1, 8, 8, 256, 128, True),
                                                     (2, 16, 8, 64, 64, False), (1, 8, 16, 64, 64, True)])
def test_conv3x3_kept_transform(hip, B, H, W, Cin, Cout, small_ws):
    """pis_conv3x3_fwd_keep leaves the F(4x4,3x3) input transform for pis_conv3x3_wgrad_keep:
    same outputs as the plain calls, also when the forward falls back to the direct kernel
    (workspace too small) and has to write the transform separately."""
    g = torch.Generator().manual_seed(21)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g))
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g)
    dz = torch.randn(B, Cout, H, W, generator=g)
    nk = hip.pis_conv3x3_keep_bytes(B, H, W, Cin, Cout)
    assert nk > 0
    keep = torch.full((nk // 4,), float("nan"), device="cuda")
    nws = 0 if small_ws else hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
    ws = torch.empty(max(nws, 4) // 4 + 1, device="cuda")
    xd, wd, bd, dzd = nhwc(x).cuda(), krsc(w).cuda(), b.cuda(), nhwc(dz).cuda()
    y = torch.empty(B, H, W, Cout, device="cuda")
    rc = hip.pis_conv3x3_fwd_keep(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), 0, y.data_ptr(), Cout, B, H, W,
                                  Cin, Cout, RELU, ws.data_ptr(), nws, keep.data_ptr(), s())
    assert rc == 0, hip.pis_last_error()
    nwg = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
    wsg = torch.empty(nwg // 4 + 1, device="cuda")
    dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
    db = torch.empty(Cout, device="cuda")
    rc = hip.pis_conv3x3_wgrad_keep(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(), B, H, W,
                                    Cin, Cout, 0, wsg.data_ptr(), nwg, keep.data_ptr(), s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    assert torch.isfinite(keep).all()
    assert rel_err(nchw(y.cpu()), F.relu(F.conv2d(x, w, b, padding=1))) < 1e-5
    assert rel_err(dw.cpu().permute(0, 3, 1, 2), torch.nn.grad.conv2d_weight(x, w.shape, dz, padding=1)) < 1e-5
    assert rel_err(db.cpu(), dz.sum(dim=(0, 2, 3))) < 1e-5


@pytest.mark.parametrize("Cin,Cout", [(256, 256), (512, 128), (128, 64)])
def test_winograd_gemm_bf16x6_is_fp32_accurate(hip, Cin, Cout):
    """The bf16x6 Winograd GEMM (pis_tune(10, 3): each fp32 operand split exactly into three
    bf16, the six partial products above 2^-24 on bf16 MFMA, fp32 accumulation) and the fp16x3
    one (pis_tune(10, 4): each K-step's operand tiles scaled by a power of two into fp16 range and
    split into hi + lo fp16, three products on fp16 MFMA) must be as accurate as the native fp32
    MFMA GEMM (pis_tune(10, 2)): same conv against a float64 reference, error no larger than
    fp32's (+25 % slack for rounding-order luck)."""
    B, H, W = 2, 16, 32
    g = torch.Generator().manual_seed(31)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64))
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, b, padding=1)
    xd, wd, bd = nhwc(x.float()).cuda(), krsc(w.float()).cuda(), b.float().cuda()
    prev8 = hip.pis_tune(8, 2)
    errs = {}
    try:
        for v in (2, 3, 4):
            prev = hip.pis_tune(10, v)
            nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
            ws = torch.empty(nws // 4 + 1, device="cuda")
            y = torch.empty(B, H, W, Cout, device="cuda")
            assert hip.pis_conv3x3_fwd_ex(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), 0, y.data_ptr(), Cout,
                                          B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s()) == 0
            torch.cuda.synchronize()
            hip.pis_tune(10, prev)
            errs[v] = ((nchw(y.cpu()).double() - ref).norm() / ref.norm()).item()
    finally:
        hip.pis_tune(8, prev8)
    for v in (3, 4):
        assert errs[v] <= 1.25 * errs[2] + 1e-9, errs
        assert errs[v] < 5e-6, errs


def test_winograd_gemm_fp16x3_scales_any_magnitude(hip):
    """fp16x3's per-K-step power-of-two scales keep gradient-sized (1e-12) and large (1e6)
    operands exactly as accurate as unit ones (the scales are powers of two: the same fp16
    digits, no underflow or overflow), and every one as accurate as the native fp32 MFMA GEMM."""
    B, H, W, Cin, Cout = 2, 16, 32, 256, 128
    g = torch.Generator().manual_seed(32)
    x0 = torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)
    wd = krsc(w.float()).cuda()
    prev8 = hip.pis_tune(8, 2)
    errs = {}
    try:
        for v in (2, 4):
            prev10 = hip.pis_tune(10, v)
            for scale in (1.0, 1e-12, 1e-6, 1e6):
                x = x0 * scale
                ref = F.conv2d(x, w, padding=1)
                nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
                ws = torch.empty(nws // 4 + 1, device="cuda")
                y = torch.empty(B, H, W, Cout, device="cuda")
                assert hip.pis_conv3x3_fwd_ex(nhwc(x.float()).cuda().data_ptr(), Cin, wd.data_ptr(), 0, 0,
                                              y.data_ptr(), Cout, B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s()) == 0
                torch.cuda.synchronize()
                errs[v, scale] = ((nchw(y.cpu()).double() - ref).norm() / ref.norm()).item()
            hip.pis_tune(10, prev10)
    finally:
        hip.pis_tune(8, prev8)
    for scale in (1e-12, 1e-6, 1e6):
        assert errs[4, scale] <= 1.05 * errs[4, 1.0] + 1e-9, errs
        assert errs[4, scale] <= 1.25 * errs[2, scale] + 1e-9, errs


@pytest.mark.parametrize("Cin,Cout", [(256, 256), (512, 128), (64, 128), (128, 64)])
def test_winograd_wgrad_bf16x6_is_fp32_accurate(hip, Cin, Cout):
    """The bf16x6 (pis_tune(14, 1)) and fp16x3 (pis_tune(14, 2)) weight-gradient GEMMs against
    the fp32 MFMA one (pis_tune(14, 0)): dW and db of the same conv against a float64 reference,
    error no larger than fp32's (+25 % slack); fp16x3 again with dz scaled to gradient size."""
    B, H, W = 2, 16, 32
    g = torch.Generator().manual_seed(37)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64))
    dz = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
    dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1)
    db_ref = dz.sum(dim=(0, 2, 3))
    xd, dzd = nhwc(x.float()).cuda(), nhwc(dz.float()).cuda()
    errs = {}
    for v in (0, 1, 2, "2tiny"):
        sc = 1e-9 if v == "2tiny" else 1.0
        dzd = nhwc((dz * sc).float()).cuda()
        prev = hip.pis_tune(14, 2 if v == "2tiny" else v)
        try:
            nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
            ws = torch.empty(nws // 4 + 1, device="cuda")
            dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
            db = torch.empty(Cout, device="cuda")
            rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                                       B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s())
            assert rc == 0, hip.pis_last_error()
            torch.cuda.synchronize()
        finally:
            hip.pis_tune(14, prev)
        dwc = dw.cpu().permute(0, 3, 1, 2).double() / sc
        errs[v] = ((dwc - dw_ref).norm() / dw_ref.norm()).item()
        assert rel_err(db.cpu().double() / sc, db_ref) < 1e-5
    for v in (1, 2, "2tiny"):
        assert errs[v] <= 1.25 * errs[0] + 1e-9, errs
        assert errs[v] < 5e-6, errs


@pytest.mark.parametrize("Cin,Cout", [(64, 64), (256, 128)])
def test_wgrad_fp16x3_mixed_magnitude_samples(hip, Cin, Cout):
    """fp16x3 weight-gradient GEMM (pis_tune(14, 2)) over a batch whose first sample's dz is ~1
    and whose second sample's is ~1e-30 (then the reverse): the contraction runs over pixels, so
    one wave's scale jumps by ~2^100 between K-steps. The rise is capped at 2^32 above the largest
    operands already accumulated (common.h h3_keep), so the partial sums are re-expressed without
    overflow: dW and db finite and as accurate as the native fp32 MFMA path against float64."""
    B, H, W = 2, 16, 32
    g = torch.Generator().manual_seed(59)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64))
    for order in ((1.0, 1e-30), (1e-30, 1.0)):
        dz = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
        dz[0] *= order[0]
        dz[1] *= order[1]
        dz = dz.float().double()  # the exact fp32 inputs
        dw_ref = torch.nn.grad.conv2d_weight(x.float().double(), (Cout, Cin, 3, 3), dz, padding=1)
        db_ref = dz.sum(dim=(0, 2, 3))
        xd, dzd = nhwc(x.float()).cuda(), nhwc(dz.float()).cuda()
        errs = {}
        for v in (0, 2):
            prev = hip.pis_tune(14, v)
            try:
                nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
                ws = torch.empty(nws // 4 + 1, device="cuda")
                dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
                db = torch.empty(Cout, device="cuda")
                rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                                           B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s())
                assert rc == 0, hip.pis_last_error()
                torch.cuda.synchronize()
            finally:
                hip.pis_tune(14, prev)
            dwc = dw.cpu().permute(0, 3, 1, 2).double()
            assert torch.isfinite(dwc).all() and torch.isfinite(db.cpu()).all(), (order, v)
            errs[v] = ((dwc - dw_ref).norm() / dw_ref.norm()).item()
            assert rel_err(db.cpu().double(), db_ref) < 1e-5, (order, v)
        assert errs[2] <= 1.25 * errs[0] + 1e-9, (order, errs)
        assert errs[2] < 5e-6, (order, errs)


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 64, 64, 256, 256), (2, 36, 36, 512, 128), (1, 12, 20, 128, 256)])
@pytest.mark.parametrize("mags", [(1.0, 1.0), (1.0, 1e-30), (1e-30, 1.0), (1e-9, 1e-9), (1e-30, 1e-30, 1e-2)])
def test_wgrad_rowstaged_fp16x3(hip, B, H, W, Cin, Cout, mags):
    """The row-staged fp16x3 Winograd weight-gradient GEMM (pis_tune(31, 1): float4 row loads,
    transposed LDS reads, 32-pixel K-steps, block-wide scales, two register sets in flight) against
    float64, next to the column-staged fp16x3 kernel (31 = 0) and the fp32 MFMA path (14 = 0):
    K-step counts from 1 to 16 per split with ragged tails (T = 162, 15), per-sample dz
    magnitudes 1e30 apart in both orders (the scale jumps inside one accumulation chain), and
    BOTH operands small (dz ~ 1e-30, x ~ 1e-2: the two power-of-two scales multiply to more than
    fp32's range, so the accumulator units must stay two factors — ADVICE r3)."""
    g = torch.Generator().manual_seed(71)
    xm = mags[2] if len(mags) > 2 else 1.0
    x = (F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)) * xm).float().double()
    dz = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
    for i in range(B):
        dz[i] *= mags[i % 2]
    dz = dz.float().double()
    dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1)
    db_ref = dz.sum(dim=(0, 2, 3))
    xd, dzd = nhwc(x.float()).cuda(), nhwc(dz.float()).cuda()
    errs, outs = {}, {}
    for name, knobs in (("f32", {14: 0}), ("h3col", {14: 2, 31: 0}), ("h3row", {14: 2, 31: 1}),
                        ("h3row_d3", {14: 2, 31: 1, 39: 3})):
        prev = {k: hip.pis_tune(k, v) for k, v in knobs.items()}
        try:
            nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
            ws = torch.empty(nws // 4 + 1, device="cuda")
            dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
            db = torch.empty(Cout, device="cuda")
            rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                                       B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s())
            assert rc == 0, hip.pis_last_error()
            torch.cuda.synchronize()
        finally:
            for k, v in prev.items():
                hip.pis_tune(k, v)
        dwc = dw.cpu().permute(0, 3, 1, 2).double()
        assert torch.isfinite(dwc).all(), name
        errs[name] = ((dwc - dw_ref).norm() / dw_ref.norm()).item()
        outs[name] = dwc
        assert rel_err(db.cpu().double(), db_ref) < 1e-5, name
    # three register sets in flight (key 39 = 3) change only when the loads are issued
    assert torch.equal(outs["h3row"], outs["h3row_d3"])
    assert errs["h3row"] <= 1.25 * errs["f32"] + 1e-9, errs
    assert errs["h3row"] < 5e-6, errs


def test_wino_wgrad_split_slabs(hip):
    """The F(3x3,4x4) weight gradient with split-K slabs summed inside the block-tiled output
    transform (wino4_wgrad_out_tiled_kernel: T = 1024 tiles -> 2 slabs per output) against float64,
    plain and accumulating into an existing gradient."""
    B, H, W, Cin, Cout = 4, 64, 64, 256, 256
    g = torch.Generator().manual_seed(73)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)).float().double()
    dz = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64).float().double()
    dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1)
    xd, dzd = nhwc(x.float()).cuda(), nhwc(dz.float()).cuda()
    nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    dw0 = torch.randn(Cout, 3, 3, Cin, generator=g).cuda()
    for flags in (0, 8):  # PIS_ACCUMULATE
        dw = dw0.clone()
        rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), 0, B, H, W, Cin, Cout,
                                   flags, ws.data_ptr(), nws, s())
        assert rc == 0, hip.pis_last_error()
        ref = dw_ref.permute(0, 2, 3, 1) + (dw0.cpu().double() if flags else 0)
        assert rel_err(dw.cpu().double(), ref) < 5e-6


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(4, 64, 64, 256, 256), (2, 32, 32, 512, 512), (2, 64, 64, 128, 64),
                                             (1, 48, 40, 128, 256), (8, 128, 128, 256, 256)])
def test_wino_wgrad_out_float4_bitwise(hip, B, H, W, Cin, Cout):
    """The float4 slab sum + output transform (pis_tune(48, 1), 64 / 128 / 256 entries per block by
    layer size) writes the weight and folded bias gradients bitwise as the scalar tiled form
    (48 = 0), plain and accumulating, and both sit at the F(3x3,4x4) accuracy against float64."""
    g = torch.Generator().manual_seed(B + H + Cin)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g)).double()
    dz = torch.randn(B, Cout, H, W, generator=g).double()
    dw_ref = torch.nn.grad.conv2d_weight(x, (Cout, Cin, 3, 3), dz, padding=1).permute(0, 2, 3, 1)
    xd, dzd = nhwc(x.float()).cuda(), nhwc(dz.float()).cuda()
    nws = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    dw0, db0 = torch.randn(Cout, 3, 3, Cin, generator=g).cuda(), torch.randn(Cout, generator=g).cuda()
    outs = {}
    for key in (0, 1):
        prev = hip.pis_tune(48, key)
        try:
            for flags in (0, 8):  # PIS_ACCUMULATE
                dw, db = dw0.clone(), db0.clone()
                rc = hip.pis_conv3x3_wgrad(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(), B,
                                           H, W, Cin, Cout, flags, ws.data_ptr(), nws, s())
                assert rc == 0, hip.pis_last_error()
                torch.cuda.synchronize()
                outs[key, flags] = (dw.cpu(), db.cpu())
        finally:
            hip.pis_tune(48, prev)
    for flags in (0, 8):
        assert torch.equal(outs[0, flags][0], outs[1, flags][0]), flags
        assert torch.equal(outs[0, flags][1], outs[1, flags][1]), flags
    assert rel_err(outs[1, 0][0].double(), dw_ref) < 5e-6
    assert rel_err(outs[1, 0][1].double(), dz.sum(dim=(0, 2, 3))) < 1e-5


@pytest.mark.parametrize("Cin,Cout", [(128, 64), (512, 256)])
def test_convt_bf16x6_is_fp32_accurate(hip, Cin, Cout):
    """Transposed conv forward / input gradient (key 13: 1 bf16x6, 3 fp16x3 vs 2 fp32 MFMA) and
    weight gradient (key 14: 1 bf16x6, 2 fp16x3 vs 0) against float64: the bf16x6 and fp16x3 errors
    no larger than fp32's (+25 %)."""
    B, H, W = 2, 16, 32
    g = torch.Generator().manual_seed(41)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64)).requires_grad_(True)
    w = (torch.randn(Cin, Cout, 2, 2, generator=g, dtype=torch.float64) / Cin ** 0.5).requires_grad_(True)
    b = torch.randn(Cout, generator=g, dtype=torch.float64).requires_grad_(True)
    y = F.conv_transpose2d(x, w, b, stride=2)
    dy = torch.randn(y.shape, generator=g, dtype=torch.float64)
    y.backward(dy)
    w_ijoc = w.detach().float().permute(2, 3, 1, 0).contiguous().cuda()
    xd, bd, dyd = nhwc(x.detach().float()).cuda(), b.detach().float().cuda(), nhwc(dy.float()).cuda()
    wc = torch.empty(Cin * 4 * Cout, device="cuda")
    assert hip.pis_convt2x2_prep(w_ijoc.data_ptr(), wc.data_ptr(), Cin, Cout, s()) == 0
    errs = {}
    for name, (v13, v14) in {"x6": (1, 1), "h3": (3, 2), "h3k32": (4, 2), "f32": (2, 0)}.items():
        p13, p14 = hip.pis_tune(13, v13), hip.pis_tune(14, v14)
        try:
            yd = torch.empty(B, 2 * H, 2 * W, Cout, device="cuda")
            assert hip.pis_convt2x2_fwd(xd.data_ptr(), Cin, w_ijoc.data_ptr(), bd.data_ptr(), yd.data_ptr(), Cout,
                                        B, H, W, Cin, Cout, s()) == 0
            dx = torch.empty(B, H, W, Cin, device="cuda")
            assert hip.pis_convt2x2_dgrad(dyd.data_ptr(), Cout, wc.data_ptr(), xd.data_ptr(), Cin, dx.data_ptr(),
                                          Cin, B, H, W, Cin, Cout, 0, s()) == 0
            nws = hip.pis_convt2x2_wgrad_ws(B, H, W, Cin, Cout)
            ws = torch.empty(nws // 4 + 1, device="cuda")
            dw = torch.empty(2, 2, Cout, Cin, device="cuda")
            db = torch.empty(Cout, device="cuda")
            assert hip.pis_convt2x2_wgrad(xd.data_ptr(), Cin, dyd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(),
                                          B, H, W, Cin, Cout, 0, ws.data_ptr(), nws, s()) == 0
            torch.cuda.synchronize()
        finally:
            hip.pis_tune(13, p13)
            hip.pis_tune(14, p14)
        errs[name] = [rel_err(nchw(yd.cpu()), y.detach()), rel_err(nchw(dx.cpu()), x.grad),
                      rel_err(dw.cpu().permute(3, 2, 0, 1), w.grad), rel_err(db.cpu(), b.grad)]
    for v in ("x6", "h3", "h3k32"):
        for e6, e32 in zip(errs[v], errs["f32"]):
            assert e6 <= 1.25 * e32 + 1e-9, errs
            assert e6 < 5e-6, errs


@pytest.mark.parametrize("B,H,W", [(2, 32, 64), (1, 16, 128), (3, 32, 32)])
def test_fused_64_groups_per_block_bitwise(hip, B, H, W):
    """The fused 64->64 contraction + output transform takes G groups of 32 tiles per block
    (pis_tune key 15: 1 -> G = 4 where the group count divides, 2 -> 1, 3 -> 2, 4 -> 8), with and
    without the staggered fold (key 25): every variant gives bit-for-bit the same forward (ReLU,
    keep-scale, fused max pool) and input gradient (ReLU mask, keep-scale, accumulate), and G = 1
    matches the float64 reference."""
    Cin = Cout = 64
    g = torch.Generator().manual_seed(31)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g))
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g)
    scale = (torch.rand(B, Cout, generator=g) > 0.2).float() / 0.8
    dz = torch.randn(B, Cout, H, W, generator=g)
    xd, wd, bd, sd, dzd = nhwc(x).cuda(), krsc(w).cuda(), b.cuda(), scale.cuda(), nhwc(dz).cuda()
    nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    wf = torch.empty(Cin * 9 * Cout, device="cuda")
    assert hip.pis_conv3x3_flip(wd.data_ptr(), wf.data_ptr(), Cin, Cout, s()) == 0
    prev, prev25 = hip.pis_tune(15, -1), hip.pis_tune(25, -1)
    out = {}
    try:
        for v in (2, 1, 3, 4, "stagger"):
            hip.pis_tune(15, 1 if v == "stagger" else v)
            hip.pis_tune(25, 1 if v == "stagger" else 0)
            y = torch.empty(B, H, W, Cout, device="cuda")
            pool = torch.empty(B, H // 2, W // 2, Cout, device="cuda")
            rc = hip.pis_conv3x3_fwd_pool(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), sd.data_ptr(),
                                          y.data_ptr(), Cout, B, H, W, Cin, Cout, RELU | SCALE, ws.data_ptr(), nws,
                                          0, pool.data_ptr(), s())
            assert rc == 0, hip.pis_last_error()
            dx = torch.full((B, H, W, Cin), 0.5, device="cuda")
            rc = hip.pis_conv3x3_dgrad_ex(dzd.data_ptr(), Cout, wf.data_ptr(), xd.data_ptr(), Cin, sd.data_ptr(),
                                          dx.data_ptr(), Cin, B, H, W, Cin, Cout, MASK | SCALE | ACC, ws.data_ptr(),
                                          nws, s())
            assert rc == 0, hip.pis_last_error()
            torch.cuda.synchronize()
            out[v] = (y.cpu(), pool.cpu(), dx.cpu())
    finally:
        hip.pis_tune(15, prev)
        hip.pis_tune(25, prev25)
    for v in (1, 3, 4, "stagger"):
        for a, c in zip(out[2], out[v]):
            assert torch.equal(a, c), v
    y_ref = F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1)) * scale[:, :, None, None]
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w.double(), dz.double(), padding=1) * (x > 0) * scale[:, :, None, None]
    assert rel_err(nchw(out[2][0]), y_ref) < 1e-6
    assert rel_err(nchw(out[2][1]), F.max_pool2d(y_ref, 2)) < 1e-6
    assert rel_err(nchw(out[2][2]) - 0.5, dx_ref) < 1e-6


@pytest.mark.parametrize("C", [64, 128])
def test_fused_64_fp16x3_is_fp32_accurate(hip, C):
    """The fused kernel (C -> C channels: 64-channel contractions, and 128-channel ones with two
    64-channel output blocks, keys 26 / 27) in fp16x3 (pis_tune(22, 1): per-tile and per-channel power-of-two
    scales, hi + lo fp16, three fp16 products) against float64: forward and input gradient as
    accurate (+25 % slack) as the same Winograd pipeline with the native fp32 MFMA GEMM, as the
    bf16x6 fused kernel (22, 0) and as the 3-pass fp16x3 GEMM path (15, 0), for unit,
    gradient-sized (1e-9, 1e-12) and large (1e6) operands, and with one region whose values span
    2^-60 .. 1 (the tile scale's worst case)."""
    B, H, W = 2, 32, 64
    g = torch.Generator().manual_seed(53)
    x0 = F.relu(torch.randn(B, C, H, W, generator=g, dtype=torch.float64))
    x0[0, :, :8, :8] *= torch.pow(2.0, -60 * torch.rand(C, 8, 8, generator=g, dtype=torch.float64))
    w = torch.randn(C, C, 3, 3, generator=g, dtype=torch.float64) / (3 * C ** 0.5)
    dz0 = torch.randn(B, C, H, W, generator=g, dtype=torch.float64)
    wd = krsc(w.float()).cuda()
    wf = torch.empty(C * 9 * C, device="cuda")
    assert hip.pis_conv3x3_flip(wd.data_ptr(), wf.data_ptr(), C, C, s()) == 0
    nws = hip.pis_conv3x3_ex_ws(B, H, W, C, C)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    # f32: the same F(4x4,3x3) pipeline with the native fp32 MFMA GEMM (key 8 = 2 keeps Winograd;
    # key 10 = 2 alone would route 64 -> 64 to the direct conv, whose error has no transforms in it)
    variants = {"h3": ((22, 1),), "x6": ((22, 0),), "f32": ((8, 2), (15, 0), (10, 2)), "h3gemm": ((15, 0), (10, 4))}
    errs = {}
    for name, knobs in variants.items():
        prev = [(k, hip.pis_tune(k, v)) for k, v in knobs]
        try:
            for sc in (1.0, 1e-12, 1e-9, 1e6):
                x, dz = x0 * sc, dz0 * sc
                y = torch.empty(B, H, W, C, device="cuda")
                assert hip.pis_conv3x3_fwd_ex(nhwc(x.float()).cuda().data_ptr(), C, wd.data_ptr(), 0, 0,
                                              y.data_ptr(), C, B, H, W, C, C, 0, ws.data_ptr(), nws, s()) == 0
                dx = torch.empty(B, H, W, C, device="cuda")
                assert hip.pis_conv3x3_dgrad_ex(nhwc(dz.float()).cuda().data_ptr(), C, wf.data_ptr(), 0, 0, 0,
                                                dx.data_ptr(), C, B, H, W, C, C, 0, ws.data_ptr(), nws, s()) == 0
                torch.cuda.synchronize()
                y_ref = F.conv2d(x.float().double(), w.float().double(), padding=1)
                dx_ref = torch.nn.grad.conv2d_input(x.shape, w.float().double(), dz.float().double(), padding=1)
                errs[name, sc] = (((nchw(y.cpu()).double() - y_ref).norm() / y_ref.norm()).item(),
                                  ((nchw(dx.cpu()).double() - dx_ref).norm() / dx_ref.norm()).item())
        finally:
            for k, v in prev:
                hip.pis_tune(k, v)
    for sc in (1.0, 1e-12, 1e-9, 1e6):
        for i in range(2):
            e = errs["h3", sc][i]
            for ref in ("f32", "x6", "h3gemm"):
                assert e <= 1.25 * errs[ref, sc][i] + 1e-9, (ref, errs)
            assert e < 2e-6, errs


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 32, 64, 64, 64), (2, 16, 32, 128, 128), (1, 32, 32, 128, 64),
                                           (2, 16, 16, 256, 256), (2, 32, 64, 128, 64), (2, 32, 64, 128, 128)])
def test_conv3x3_bwd_prep(hip, B, H, W, Cin, Cout):
    """pis_conv3x3_bwd_prep: one pass over dz writes both backward transforms; the dgrad_ex and
    wgrad_keep calls that then pass PIS_WINO_PREPARED give the same results as without it (and
    as the float64 reference), bias gradient included. With PIS_W_UNFLIPPED the input gradient
    reads the original weights (the rotating filter transform) and matches the flipped-copy path
    bit for bit."""
    PREP, UNFLIPPED = 16, 32
    g = torch.Generator().manual_seed(23)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g))
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    dz = torch.randn(B, Cout, H, W, generator=g)
    xd, wd, dzd = nhwc(x).cuda(), krsc(w).cuda(), nhwc(dz).cuda()
    mask = xd.clone()
    nk = hip.pis_conv3x3_keep_bytes(B, H, W, Cin, Cout)
    keep = torch.empty(nk // 4 + 1, device="cuda")
    nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    y = torch.empty(B, H, W, Cout, device="cuda")
    assert hip.pis_conv3x3_fwd_keep(xd.data_ptr(), Cin, wd.data_ptr(), 0, 0, y.data_ptr(), Cout, B, H, W, Cin,
                                    Cout, 0, ws.data_ptr(), nws, keep.data_ptr(), s()) == 0
    wf = torch.empty(Cin * 9 * Cout, device="cuda")
    assert hip.pis_conv3x3_flip(wd.data_ptr(), wf.data_ptr(), Cin, Cout, s()) == 0
    nwg = hip.pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout)
    out = {}
    for prep in (False, True, "unflipped"):
        wsg = torch.full((nwg // 4 + 1,), float("nan"), device="cuda")
        wsd = torch.full((nws // 4 + 1,), float("nan"), device="cuda")
        flag, wdg = 0, wf
        if prep:
            rc = hip.pis_conv3x3_bwd_prep(dzd.data_ptr(), Cout, B, H, W, Cin, Cout, wsd.data_ptr(), nws,
                                          wsg.data_ptr(), nwg, s())
            assert rc == 1, hip.pis_last_error()
            flag = PREP
        if prep == "unflipped":  # the dgrad reads the original weights and rotates them itself
            wdg = wd
        dw = torch.empty(Cout, 3, 3, Cin, device="cuda")
        db = torch.empty(Cout, device="cuda")
        assert hip.pis_conv3x3_wgrad_keep(xd.data_ptr(), Cin, dzd.data_ptr(), Cout, dw.data_ptr(), db.data_ptr(), B,
                                          H, W, Cin, Cout, flag, wsg.data_ptr(), nwg, keep.data_ptr(), s()) == 0
        dx = torch.empty(B, H, W, Cin, device="cuda")
        dflag = MASK | flag | (UNFLIPPED if prep == "unflipped" else 0)
        assert hip.pis_conv3x3_dgrad_ex(dzd.data_ptr(), Cout, wdg.data_ptr(), mask.data_ptr(), Cin, 0, dx.data_ptr(),
                                        Cin, B, H, W, Cin, Cout, dflag, wsd.data_ptr(), nws, s()) == 0, \
            hip.pis_last_error()
        torch.cuda.synchronize()
        out[prep] = (dw.cpu(), db.cpu(), dx.cpu())
    for variant in (True, "unflipped"):
        for a, b in zip(out[False], out[variant]):
            assert torch.equal(a, b)  # the same arithmetic, only one read of dz (or one weight flip) fewer
    # unflipped weights are only understood on the prepared F(4x4) path
    assert hip.pis_conv3x3_dgrad_ex(dzd.data_ptr(), Cout, wd.data_ptr(), 0, 0, 0, dx.data_ptr(), Cin, B, H, W,
                                    Cin, Cout, UNFLIPPED, wsd.data_ptr(), nws, s()) != 0
    dw_ref = torch.nn.grad.conv2d_weight(x.double(), w.shape, dz.double(), padding=1)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w.double(), dz.double(), padding=1) * (x > 0)
    assert rel_err(out[True][0].permute(0, 3, 1, 2), dw_ref) < 1e-5
    assert rel_err(out[True][1], dz.sum(dim=(0, 2, 3))) < 1e-5
    assert rel_err(nchw(out[True][2]), dx_ref) < 1e-5


def test_conv3x3_bwd_prep_not_applicable(hip):
    """Layers off the F(4x4) path (odd grid) return 0 and leave the calls to transform dz."""
    B, H, W, Cin, Cout = 1, 6, 10, 64, 64
    dz = torch.zeros(B, H, W, Cout, device="cuda")
    ws = torch.empty(1 << 20, device="cuda")
    assert hip.pis_conv3x3_bwd_prep(dz.data_ptr(), Cout, B, H, W, Cin, Cout, ws.data_ptr(), 4 << 20,
                                    ws.data_ptr(), 4 << 20, s()) == 0
    # nor channel counts the weight-gradient call rejects (Cin % 64 != 0)
    dz = torch.zeros(1, 16, 16, 128, device="cuda")
    assert hip.pis_conv3x3_bwd_prep(dz.data_ptr(), 128, 1, 16, 16, 144, 128, ws.data_ptr(), 4 << 20,
                                    ws.data_ptr(), 4 << 20, s()) == 0


@pytest.mark.parametrize("B,H,W,Cin,Cout,keep", [(2, 32, 64, 64, 64, True), (2, 16, 32, 128, 128, True),
                                                (2, 16, 32, 128, 128, False), (1, 6, 10, 64, 64, False),
                                                (2, 16, 16, 1, 64, False), (1, 8, 8, 512, 256, True)])
def test_conv3x3_fwd_pool(hip, B, H, W, Cin, Cout, keep):
    """pis_conv3x3_fwd_pool = conv (bias, ReLU, keep-scale) + MaxPool2d(2,2) of its output: pooled in
    the F(4x4) output epilogues (fused 64->64 kernel and the output-transform kernel), by the
    pooling kernel on every other path; y lands in a concat slice (ldy = 2 Cout)."""
    g = torch.Generator().manual_seed(29)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g))
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g)
    scale = (torch.rand(B, Cout, generator=g) > 0.2).float() / 0.8
    y_ref = F.relu(F.conv2d(x, w, b, padding=1)) * scale[:, :, None, None]
    p_ref = F.max_pool2d(y_ref, 2)
    xd, wd, bd, sd = nhwc(x).cuda(), krsc(w).cuda(), b.cuda(), scale.cuda()
    nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
    ws = torch.empty(max(nws, 4) // 4 + 1, device="cuda")
    nk = hip.pis_conv3x3_keep_bytes(B, H, W, Cin, Cout)
    kp = torch.empty(max(nk, 4) // 4 + 1, device="cuda") if keep and nk else None
    y = torch.full((B, H, W, 2 * Cout), 7.0, device="cuda")
    pool = torch.empty(B, H // 2, W // 2, Cout, device="cuda")
    rc = hip.pis_conv3x3_fwd_pool(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), sd.data_ptr(), y.data_ptr(),
                                  2 * Cout, B, H, W, Cin, Cout, RELU | SCALE, ws.data_ptr(), nws,
                                  kp.data_ptr() if kp is not None else 0, pool.data_ptr(), s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    assert rel_err(nchw(y[..., :Cout].cpu()), y_ref) < 1e-5
    assert torch.all(y[..., Cout:] == 7.0)
    assert rel_err(nchw(pool.cpu()), p_ref) < 1e-5


@pytest.mark.parametrize("shape", [(2, 1, 9, 11), (1, 1, 2, 3), (3, 1, 64, 48)])
def test_pde_fields_and_their_gradients(hip, shape):
    """PDERegularization's per-pixel fields (pis_pde_fields) equal the oracle's reflect-pad +
    conv2d stencils (src/pde.py:49-178), and their gradients (pis_pde_fields_bwd) equal float64
    autograd through the oracle for an arbitrary upstream gradient — odd sizes and the 2-pixel
    minimum exercise every reflect fold."""
    from physics_informed_image_segmentation_amd.pde import PDERegularization
    g = torch.Generator().manual_seed(14)
    u = torch.rand(shape, generator=g) * 0.9 + 0.05
    up = torch.randn(shape, generator=g)
    reg = PDERegularization(diffusion_coeff=5.0, reaction_threshold=0.3)
    u64 = u.double().requires_grad_(True)
    refs = {"compute_laplacian": rt.laplacian(u64), "reaction_term": rt.reaction(u64, 0.3),
            "compute_residual": rt.rd_residual(u64, 5.0, 0.3), "compute_gradient_magnitude": rt.grad_mag_sq(u64)}
    for name, ref in refs.items():
        ud = u.cuda().requires_grad_(True)
        f = getattr(reg, name)(ud)
        assert f.shape == u.shape
        (f * up.cuda()).sum().backward()
        (gref,) = torch.autograd.grad((ref * up.double()).sum(), u64)
        fa = f.detach().cpu().double()
        assert (fa - ref.detach()).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item()), name
        ga = ud.grad.cpu().double()
        assert ((ga - gref).norm() / gref.norm()).item() < 1e-6, name
        assert (ga - gref).abs().max().item() <= 1e-5 * gref.abs().max().item(), name


@pytest.mark.parametrize("H,cin,cout", [(64, 64, 64), (32, 128, 128), (32, 256, 128), (16, 512, 256)])
def test_filter_ready_matches_inline_transform(hip, H, cin, cout):
    """pis_conv3x3_filter + PIS_FILTER_READY (the engine's filter transforms computed ahead on the
    side stream) gives bitwise the conv the call computes with its own filter transform: forward
    with a kept input transform, and the prepared input gradient from the original weights."""
    B = 2
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(21)
    x = torch.randn(B, H, H, cin, generator=g).cuda()
    dz = torch.randn(B, H, H, cout, generator=g).cuda()
    w = (torch.randn(cout, 3, 3, cin, generator=g) * 0.05).cuda()
    bias = torch.randn(cout, generator=g).cuda()
    nws = hip.pis_conv3x3_ex_ws(B, H, H, cin, cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    nk = hip.pis_conv3x3_keep_bytes(B, H, H, cin, cout)
    assert nk > 0
    ys, keeps = [], []
    for ready in (False, True):
        wptr, flags = w.data_ptr(), 1  # PIS_RELU
        if ready:
            nb = hip.pis_conv3x3_filter_bytes(B, H, H, cin, cout, 0)
            assert nb > 0
            U = torch.empty(nb // 4 + 1, device="cuda")
            assert hip.pis_conv3x3_filter(w.data_ptr(), B, H, H, cin, cout, 0, U.data_ptr(), nb, s) == 0
            wptr, flags = U.data_ptr(), flags | 64  # PIS_FILTER_READY
        y = torch.empty(B, H, H, cout, device="cuda")
        keep = torch.empty(nk // 4 + 1, device="cuda")
        assert hip.pis_conv3x3_fwd_keep(x.data_ptr(), cin, wptr, bias.data_ptr(), 0, y.data_ptr(), cout, B, H, H,
                                        cin, cout, flags, ws.data_ptr(), nws, keep.data_ptr(), s) == 0
        ys.append(y)
        keeps.append(keep)
    torch.cuda.synchronize()
    assert torch.equal(ys[0], ys[1])
    assert torch.equal(keeps[0][:nk // 4], keeps[1][:nk // 4])  # (the +1 float is padding)
    nw3 = hip.pis_conv3x3_wgrad_ws(B, H, H, cin, cout)
    ws3 = torch.empty(nw3 // 4 + 1, device="cuda")
    dxs = []
    for ready in (False, True):
        assert hip.pis_conv3x3_bwd_prep(dz.data_ptr(), cout, B, H, H, cin, cout, ws.data_ptr(), nws,
                                        ws3.data_ptr(), nw3, s) == 1
        wptr, flags = w.data_ptr(), 16 | 32  # PIS_WINO_PREPARED | PIS_W_UNFLIPPED
        if ready:
            nb = hip.pis_conv3x3_filter_bytes(B, H, H, cin, cout, 1)
            assert nb > 0
            Ub = torch.empty(nb // 4 + 1, device="cuda")
            assert hip.pis_conv3x3_filter(w.data_ptr(), B, H, H, cin, cout, 1, Ub.data_ptr(), nb, s) == 0
            wptr, flags = Ub.data_ptr(), flags | 64
        dx = torch.empty(B, H, H, cin, device="cuda")
        assert hip.pis_conv3x3_dgrad_ex(dz.data_ptr(), cout, wptr, 0, 0, 0, dx.data_ptr(), cin, B, H, H, cin, cout,
                                        flags, ws.data_ptr(), nws, s) == 0
        dxs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(dxs[0], dxs[1])


def test_filter_ready_refused_off_the_winograd_path(hip):
    """A conv that would not take the F(4x4,3x3) GEMM path reports 0 filter bytes and refuses
    PIS_FILTER_READY loudly."""
    assert hip.pis_conv3x3_filter_bytes(2, 16, 16, 1, 64, 0) == 0  # Cin = 1: direct kernels
    x = torch.randn(1, 16, 16, 1, device="cuda")
    y = torch.empty(1, 16, 16, 64, device="cuda")
    w = torch.randn(64 * 9, device="cuda")
    rc = hip.pis_conv3x3_fwd_ex(x.data_ptr(), 1, w.data_ptr(), 0, 0, y.data_ptr(), 64, 1, 16, 16, 1, 64, 64, 0, 0,
                                torch.cuda.current_stream().cuda_stream)
    assert rc != 0


def test_batched_filter_transforms_match_single(hip):
    """pis_conv3x3_filters (every layer's filter transform in one launch) writes bitwise what
    pis_conv3x3_filter writes per layer, both directions and both formats."""
    from physics_informed_image_segmentation_amd import _hip
    s = torch.cuda.current_stream().cuda_stream
    g = torch.Generator().manual_seed(4)
    shapes = [(2, 64, 64, 64, 64, 0), (2, 64, 64, 64, 64, 1), (2, 32, 32, 128, 128, 0), (2, 32, 32, 256, 128, 1),
              (2, 16, 16, 512, 256, 0), (2, 16, 16, 512, 256, 1)]
    jobs = (_hip.FilterJob * len(shapes))()
    keep = []
    for k, (B, H, W, ci, co, dg) in enumerate(shapes):
        w = (torch.randn(co, 3, 3, ci, generator=g) * 0.1).cuda()
        nb = hip.pis_conv3x3_filter_bytes(B, H, W, ci, co, dg)
        assert nb > 0
        one = torch.empty(nb // 4 + 1, device="cuda")
        bat = torch.empty(nb // 4 + 1, device="cuda")
        assert hip.pis_conv3x3_filter(w.data_ptr(), B, H, W, ci, co, dg, one.data_ptr(), nb, s) == 0
        jobs[k] = _hip.FilterJob(w.data_ptr(), bat.data_ptr(), nb, B, H, W, ci, co, dg)
        keep.append((w, one, bat, nb))
    assert hip.pis_conv3x3_filters(ctypes.addressof(jobs), len(shapes), s) == 0
    torch.cuda.synchronize()
    for w, one, bat, nb in keep:
        assert torch.equal(one[:nb // 4], bat[:nb // 4])


@pytest.mark.parametrize("npix,C", [(35, 64), (1, 64), (4099, 64), (35, 32)])
def test_head_fwd_ragged(hip, npix, C):
    """pis_head_fwd on pixel counts that are not a multiple of the 4 pixels per lane group of the
    C == 64 kernel (and the generic path, C == 32): z = x . w + b and u = sigmoid(z)."""
    g = torch.Generator().manual_seed(9)
    x = torch.randn(npix, C, generator=g)
    w = torch.randn(C, generator=g)
    b = torch.randn(1, generator=g)
    zd = torch.empty(npix, device="cuda")
    ud = torch.empty(npix, device="cuda")
    xd, wd, bd = x.cuda(), w.cuda(), b.cuda()
    assert hip.pis_head_fwd(xd.data_ptr(), C, wd.data_ptr(), bd.data_ptr(), zd.data_ptr(), ud.data_ptr(),
                            npix, C, s()) == 0
    torch.cuda.synchronize()
    z = x.double() @ w.double() + b.double()
    assert rel_err(zd.cpu().double(), z) < 1e-6
    assert rel_err(ud.cpu().double(), torch.sigmoid(z)) < 1e-6
