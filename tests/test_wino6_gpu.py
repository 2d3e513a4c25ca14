"""Winograd F(6x6,3x3) (csrc/winograd.hip launch_wino6, pis_tune key 47): the forward and input
gradient of the deep 3x3 layers of src/unet.py:28-42 (nn.Conv2d(k=3, padding=1) + ReLU, Dropout2d
keep-scales) on 8 x 8 input tiles. Every output against float64 (the conv evaluated in double on the
host), with the error bounded absolutely (fp32-class: <= 3e-5 relative, per element <= 1e-4 of the
output scale) and against the F(4x4,3x3) pipeline the same call takes with key 47 = 0 (F(6x6)'s
transform rounding is ~3x F(4x4)'s: DESIGN.md §4 round 6). Shapes: the C2 levels (128^2, 64^2 at
reduced batch), a ragged tile grid (48 x 40: 8 x 7 tiles of 6, the last ones partly outside), the
pooled encoder forward, the masked / accumulating input gradient from the ORIGINAL weights with the
transform computed ahead (PIS_W_UNFLIPPED | PIS_FILTER_READY, as the engine runs it), and the filter
batch (pis_conv3x3_filters) writing the same operand as the single call."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

RELU, SCALE, MASK, ACC = 1, 2, 4, 8
W_UNFLIPPED, FILTER_READY = 32, 64


def nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def krsc(w):
    return w.permute(0, 2, 3, 1).contiguous()


def s():
    return torch.cuda.current_stream().cuda_stream


@pytest.fixture(autouse=True)
def f6_on(hip):
    """F(6x6) is opt-in (pis_tune(47) = 0 by default: measured slower on the C2 step); these tests
    exercise it with key 47 = 1 unless they set another value themselves."""
    prev = hip.pis_tune(47, 1)
    yield
    hip.pis_tune(47, prev)


def errs(got, ref):
    got, ref = got.double().cpu(), ref.double().cpu()
    rel = ((got - ref).norm() / ref.norm()).item()
    elem = ((got - ref).abs().max() / ref.abs().max()).item()
    return rel, elem


SHAPES = [(2, 128, 128, 512, 256), (2, 64, 64, 256, 512), (1, 64, 64, 512, 256), (1, 48, 40, 128, 256),
          (2, 128, 128, 256, 256)]


@pytest.mark.parametrize("B,H,W,Cin,Cout", SHAPES)
def test_wino6_forward_and_input_gradient_vs_float64(hip, B, H, W, Cin, Cout):
    assert hip.pis_conv3x3_filter_format(B, H, W, Cin, Cout, 0) == 4
    assert hip.pis_conv3x3_filter_format(B, H, W, Cin, Cout, 1) == 4
    assert hip.pis_conv3x3_keep_bytes(B, H, W, Cin, Cout) == 0  # no kept F(4x4) transform
    g = torch.Generator().manual_seed(60 + H + Cin)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g, dtype=torch.float64))
    w = torch.randn(Cout, Cin, 3, 3, generator=g, dtype=torch.float64) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g, dtype=torch.float64) * 0.1
    scale = (torch.rand(B, Cout, generator=g) > 0.2).double() / 0.8
    dz = torch.randn(B, Cout, H, W, generator=g, dtype=torch.float64)
    sc_in = (torch.rand(B, Cin, generator=g) > 0.2).double() / 0.8
    xf, wf32, dzf = x.float(), w.float(), dz.float()
    # float64 truth of the fp32 inputs
    y64 = F.relu(F.conv2d(xf.double(), wf32.double(), b.float().double(), padding=1)) * scale[:, :, None, None]
    pre = F.conv2d(xf.double(), wf32.double(), b.float().double(), padding=1)
    dx64 = (torch.nn.grad.conv2d_input(x.shape, wf32.double(), dzf.double(), padding=1) * (xf.double() > 0)
            * sc_in[:, :, None, None])
    nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    xd, wd, bd, sd, dzd, sid = (nhwc(xf).cuda(), krsc(wf32).cuda(), b.float().cuda(), scale.float().cuda(),
                                nhwc(dzf).cuda(), sc_in.float().cuda())
    out = {}
    for key in (1, 2, 3, 0):  # F(6x6): 1 / 2 channels per thread, the runtime-looped forms; then F(4x4)
        prev = hip.pis_tune(47, key)
        try:
            y = torch.empty(B, H, W, Cout, device="cuda")
            rc = hip.pis_conv3x3_fwd_ex(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), sd.data_ptr(), y.data_ptr(),
                                        Cout, B, H, W, Cin, Cout, RELU | SCALE, ws.data_ptr(), nws, s())
            assert rc == 0, hip.pis_last_error()
            dx = torch.full((B, H, W, Cin), 0.5, device="cuda")
            if key:
                # the engine's input gradient: the ORIGINAL weights' transform computed ahead
                nb = hip.pis_conv3x3_filter_bytes(B, H, W, Cin, Cout, 1)
                assert nb == 64 * Cin * Cout * 4
                U = torch.empty(nb // 4, device="cuda")
                assert hip.pis_conv3x3_filter(wd.data_ptr(), B, H, W, Cin, Cout, 1, U.data_ptr(), nb, s()) == 0
                rc = hip.pis_conv3x3_dgrad_ex(dzd.data_ptr(), Cout, U.data_ptr(), xd.data_ptr(), Cin, sid.data_ptr(),
                                              dx.data_ptr(), Cin, B, H, W, Cin, Cout,
                                              MASK | SCALE | ACC | W_UNFLIPPED | FILTER_READY, ws.data_ptr(), nws, s())
            else:
                wfl = torch.empty(Cin * 9 * Cout, device="cuda")
                assert hip.pis_conv3x3_flip(wd.data_ptr(), wfl.data_ptr(), Cin, Cout, s()) == 0
                rc = hip.pis_conv3x3_dgrad_ex(dzd.data_ptr(), Cout, wfl.data_ptr(), xd.data_ptr(), Cin, sid.data_ptr(),
                                              dx.data_ptr(), Cin, B, H, W, Cin, Cout, MASK | SCALE | ACC,
                                              ws.data_ptr(), nws, s())
            assert rc == 0, hip.pis_last_error()
            torch.cuda.synchronize()
            out[key] = (errs(nchw(y.cpu()), y64), errs(nchw(dx.cpu()) - 0.5, dx64))
        finally:
            hip.pis_tune(47, prev)
    print(f"F6 vs F4 (rel, elem): fwd {out[1][0]} / {out[0][0]}, dgrad {out[1][1]} / {out[0][1]}")
    for key in (1, 2, 3):
        for (rel, elem), (rel4, _) in zip(out[key], out[0]):
            assert rel <= 3e-5 and elem <= 1e-4, (key, rel, elem)
            assert rel <= max(6.0 * rel4, 5e-6), (key, rel, rel4)  # ~3x F(4x4)'s rounding
    assert pre.abs().max() > 0


@pytest.mark.parametrize("B,H,W,Cin,Cout", [(2, 128, 128, 256, 256), (1, 48, 40, 128, 256)])
def test_wino6_pooled_forward(hip, B, H, W, Cin, Cout):
    """pis_conv3x3_fwd_pool on an F(6x6) layer: the 2x2 max pool of the tile's 6 x 6 outputs in the
    output transform (3 x 3 pooled outputs per tile; at 48 x 40 the last tile column holds 4 of 6
    columns), bitwise the max of the written outputs."""
    g = torch.Generator().manual_seed(7)
    x = F.relu(torch.randn(B, Cin, H, W, generator=g))
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (3 * Cin ** 0.5)
    b = torch.randn(Cout, generator=g) * 0.1
    nws = hip.pis_conv3x3_ex_ws(B, H, W, Cin, Cout)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    y = torch.empty(B, H, W, Cout, device="cuda")
    pool = torch.empty(B, H // 2, W // 2, Cout, device="cuda")
    xd, wd, bd = nhwc(x).cuda(), krsc(w).cuda(), b.cuda()  # held: a freed temporary's block can be reused
    rc = hip.pis_conv3x3_fwd_pool(xd.data_ptr(), Cin, wd.data_ptr(), bd.data_ptr(), 0, y.data_ptr(), Cout, B, H, W,
                                  Cin, Cout, RELU, ws.data_ptr(), nws, 0, pool.data_ptr(), s())
    assert rc == 0, hip.pis_last_error()
    torch.cuda.synchronize()
    y64 = F.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1))
    rel, elem = errs(nchw(y.cpu()), y64)
    assert rel <= 3e-5 and elem <= 1e-4, (rel, elem)
    yc = nchw(y.cpu())
    assert torch.equal(nchw(pool.cpu()), F.max_pool2d(yc, 2))


def test_wino6_filter_batch_equals_single(hip):
    """pis_conv3x3_filters (the engine's batched filter launch) writes the F(6x6) operands (forward
    and rotated input-gradient transforms) bitwise as pis_conv3x3_filter does."""
    from physics_informed_image_segmentation_amd._hip import FilterJob
    B, H, W, Cin, Cout = 8, 64, 64, 256, 512
    g = torch.Generator().manual_seed(9)
    w = krsc(torch.randn(Cout, Cin, 3, 3, generator=g)).cuda()
    outs = []
    for dg in (0, 1):
        nb = hip.pis_conv3x3_filter_bytes(B, H, W, Cin, Cout, dg)
        a, b_ = torch.empty(nb // 4, device="cuda"), torch.empty(nb // 4, device="cuda")
        assert hip.pis_conv3x3_filter(w.data_ptr(), B, H, W, Cin, Cout, dg, a.data_ptr(), nb, s()) == 0
        outs.append((a, b_, nb, dg))
    jobs = (FilterJob * 2)()
    for k, (_, b_, nb, dg) in enumerate(outs):
        jobs[k] = FilterJob(w.data_ptr(), b_.data_ptr(), nb, B, H, W, Cin, Cout, dg)
    assert hip.pis_conv3x3_filters(ctypes.addressof(jobs), 2, s()) == 0
    torch.cuda.synchronize()
    for a, b_, _, _ in outs:
        assert torch.equal(a, b_)


def test_wino6_policy_at_c2(hip):
    """Which C2 layers take F(6x6): the 128^2 and 64^2 layers whose contractions run the batched
    GEMM both ways; not the bottleneck (32^2: no fewer products), not the fused 128-channel
    contractions (enc3.conv0), not the direct layers (<= 128 channels at >= 256^2)."""
    B = 8
    f6 = lambda H, ci, co: hip.pis_conv3x3_filter_format(B, H, H, ci, co, 0) == 4  # noqa: E731
    assert f6(128, 256, 256) and f6(128, 512, 256) and f6(64, 256, 512) and f6(64, 512, 512) and f6(64, 1024, 512)
    assert not f6(32, 512, 1024) and not f6(32, 1024, 1024)
    assert not f6(128, 128, 256)  # enc3.conv0: its forward is the fused 128-channel contraction
    assert not f6(512, 64, 64) and not f6(256, 128, 128)
    hip.pis_tune(47, 0)  # the default: no F(6x6) layer (the fixture restores the key)
    assert not f6(128, 256, 256)
