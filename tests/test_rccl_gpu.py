"""The data-parallel gradient path over RCCL itself (torch.distributed backend "nccl" = RCCL on
ROCm) on the one GPU of the test box: a world-size-1 process group, so RCCL is initialised on
cuda:0 and every bucket of ``GradBucketer`` goes through ``dist.all_reduce(async_op=True)`` issued
while the HIP backward is still running on both streams, and ``finish()`` waits on RCCL's work
objects. RCCL refuses two ranks on one device, so the exchange between ranks is covered by the
gloo tests (``test_distributed_gpu.py``) and measured by the driver's 8-GPU run; this test pins
that the RCCL path runs on hardware and leaves the gradients (sum over one rank = the rank's own)
and the AdamW step bitwise equal to the single-process step. The reference has no distributed
code."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import reference_torch as rt

pytestmark = pytest.mark.gpu

B, H, W = 2, 64, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(bucketed):
    """Two eval-mode steps (loss, backward, AdamW) on a fixed batch; returns grads and weights."""
    from physics_informed_image_segmentation_amd import AdamW, UNet, DiceBCEPDELoss
    torch.manual_seed(5)
    net = UNet(1, 1, 64).cuda().eval()
    nb = 0
    if bucketed:
        from physics_informed_image_segmentation_amd.distributed import GradBucketer, broadcast_parameters
        broadcast_parameters(net)
        bk = GradBucketer(net, bucket_bytes=4 << 20)
        nb = len(bk.buckets)
    opt = AdamW(net.parameters(), lr=1e-3, weight_decay=1e-5, grad_scale=1.0)
    crit = DiceBCEPDELoss(pde_weight=1e-2, phase_field_weight=1e-2, diffusion_coeff=5.0, epsilon=0.05)
    img, mask = rt.synthetic_batch(B, H, W, seed=21)
    x, t = img.cuda(), mask.cuda()
    losses = []
    for _ in range(2):
        opt.zero_grad(set_to_none=True)
        loss = crit(net(x), t)
        loss.backward()
        opt.step()
        losses.append(loss.detach())
    torch.cuda.synchronize()
    return (net.grad_arena().cpu().numpy().copy(), net.arena.detach().cpu().numpy().copy(),
            torch.stack(losses).cpu().numpy().copy(), nb)


def _worker(port, q, k29):
    import torch.distributed as dist
    from physics_informed_image_segmentation_amd import _hip
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if k29 is not None:
        _hip.lib().pis_tune(29, k29)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        plain = _run(False)
        rccl = _run(True)
        q.put((plain, rccl))
    finally:
        dist.destroy_process_group()


# k29 = 2: every 3x3 conv the direct fp16x3 kernels can take runs them (at 64 x 64 the default
# picks none), so the direct weight gradients — on the MAIN stream, the side stream ordered after
# them before a bucket's all-reduce starts — feed the RCCL buckets
@pytest.mark.parametrize("k29", [None, 2], ids=["default", "direct"])
def test_rccl_bucketed_step_equals_single_process(hip, k29):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q, k29))
    p.start()
    plain, rccl = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert rccl[3] > 2  # several buckets went through RCCL during the backward
    for a, b, name in zip(plain[:3], rccl[:3], ("grads", "weights", "losses")):
        assert (a == b).all(), name
