"""Data-parallel step on the GPU: two ranks (gloo over CUDA tensors, both on cuda:0 —
RCCL needs one GPU per rank, the 8-GPU RCCL run is the driver's) each run the real
U-Net step on their shard; the bucketed all-reduce that GradBucketer overlaps with
the HIP backward must leave every rank with the sum of the per-shard gradients.
The reference has no distributed code; the expectation is
computed in this process, one shard at a time."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import reference_torch as rt

pytestmark = pytest.mark.gpu

B_PER_RANK, H, W = 2, 64, 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shard(rank):
    img, mask = rt.synthetic_batch(2 * B_PER_RANK, H, W, seed=21)
    sl = slice(rank * B_PER_RANK, (rank + 1) * B_PER_RANK)
    return img[sl].cuda(), mask[sl].cuda()


def _model():
    from physics_informed_image_segmentation_amd import UNet
    torch.manual_seed(5)
    return UNet(1, 1, 64).cuda().eval()  # eval: no dropout draw, the shards are deterministic


def _loss():
    from physics_informed_image_segmentation_amd import DiceBCEPDELoss
    return DiceBCEPDELoss(pde_weight=1e-2, phase_field_weight=1e-2, diffusion_coeff=5.0, epsilon=0.05)


def _worker(rank, world, port, q, k29=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    if k29 is not None:
        from physics_informed_image_segmentation_amd import _hip
        _hip.lib().pis_tune(29, k29)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from physics_informed_image_segmentation_amd.distributed import GradBucketer, broadcast_parameters
        net = _model()
        if rank == 1:
            with torch.no_grad():
                net.arena.mul_(3.0)  # broadcast must restore rank 0's weights
        broadcast_parameters(net)
        bk = GradBucketer(net, bucket_bytes=4 << 20)
        x, t = _shard(rank)
        crit = _loss()
        for _ in range(2):  # second step exercises the re-armed bucketer
            net.zero_grad(set_to_none=True)
            crit(net(x), t).backward()
        torch.cuda.synchronize()
        q.put((rank, net.grad_arena().cpu().numpy().copy(), len(bk.buckets)))  # plain bytes, no fd sharing
    finally:
        dist.destroy_process_group()


# k29 = 2 engages the direct fp16x3 layers at 64 x 64 (the default picks none there): their weight
# gradients run on the MAIN stream and the weight-gradient stream is ordered after them before a
# bucket's all-reduce is issued from it; a missing order would all-reduce stale bytes
@pytest.mark.parametrize("k29", [None, 2], ids=["default", "direct"])
def test_two_rank_bucketed_allreduce_on_gpu(hip, k29):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, k29)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, nb)) for r, g, nb in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    # expectation: per-shard gradients from the same kernels, summed
    from physics_informed_image_segmentation_amd import _hip
    prev = _hip.lib().pis_tune(29, k29) if k29 is not None else None
    try:
        net = _model()
        crit = _loss()
        total = torch.zeros_like(net.arena)
        for r in range(2):
            net.zero_grad(set_to_none=True)
            x, t = _shard(r)
            crit(net(x), t).backward()
            total += net.grad_arena()
        total = total.cpu()
    finally:
        if prev is not None:
            _hip.lib().pis_tune(29, prev)
    for r in range(2):
        g, nb = res[r]
        g = torch.from_numpy(g)
        assert nb > 2
        err = ((g - total).norm() / total.norm()).item()
        assert err < 1e-6, (r, err)


# ---------------------------------------------------------------------------------------------
# Train-mode equivalence against the oracle (north_star config C3): each rank
# draws different Dropout2d masks for its own shard; the all-reduced gradients must equal the sum
# of the per-shard float64 oracle gradients (on each rank's own ReLU / max-pool decisions), and
# the weights after each AdamW step (1/world folded into the kernel) must equal torch.optim.AdamW
# fed the oracle's mean gradient — two steps, for the default bucketing and for tiny buckets (every
# parameter its own bucket, so out_conv's bucket is all-reduced from the MAIN stream, unet.py's
# head, while the others go from the weight-gradient stream).
# ---------------------------------------------------------------------------------------------

LR = 1e-3
PDE = dict(rd_w=1e-2, pf_w=1e-2, D=5.0, a=0.5, eps=0.05)


def _scales(rank, step, B):
    ref = rt.UNetRef(1, 1, 64)
    return rt.make_drop_scales(ref, B, torch.Generator().manual_seed(1000 + 17 * rank + step))


def _worker_train(rank, world, port, q, bucket_bytes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from physics_informed_image_segmentation_amd import AdamW, UNet
        from physics_informed_image_segmentation_amd.distributed import GradBucketer, broadcast_parameters
        torch.manual_seed(5)
        net = UNet(1, 1, 64).cuda().train()
        if rank == 1:
            with torch.no_grad():
                net.arena.mul_(3.0)
        broadcast_parameters(net)
        bk = GradBucketer(net, bucket_bytes=bucket_bytes)
        opt = AdamW(net.parameters(), lr=LR, weight_decay=1e-5, grad_scale=1.0 / world)
        x, t = _shard(rank)
        crit = _loss()
        steps = []
        for step in range(2):
            net.set_dropout_scales(_scales(rank, step, B_PER_RANK))
            w_before = net.arena.cpu().numpy().copy()
            opt.zero_grad(set_to_none=True)
            crit(net(x), t).backward()
            torch.cuda.synchronize()
            dec = {k: v.numpy() for k, v in net.activation_decisions().items()}
            g = net.grad_arena().cpu().numpy().copy()
            opt.step()
            torch.cuda.synchronize()
            steps.append((w_before, g, dec))
        q.put((rank, steps, net.arena.cpu().numpy().copy(), len(bk.buckets)))
    finally:
        dist.destroy_process_group()


def _oracle_grads(w_arena, rank, step, dec):
    """float64 oracle gradients of one rank's shard at the given weights, on that rank's decisions,
    in arena layout (a CPU UNet maps arena <-> reference parameters)."""
    from physics_informed_image_segmentation_amd import UNet
    holder = UNet(1, 1, 64)
    holder.arena.copy_(torch.from_numpy(w_arena))
    ref64 = rt.UNetRef().double().train()
    ref64.load_state_dict({k: v.double() for k, v in holder.state_dict().items()})
    x, t = rt.synthetic_batch(2 * B_PER_RANK, H, W, seed=21)
    sl = slice(rank * B_PER_RANK, (rank + 1) * B_PER_RANK)
    scales = {k: v.double() for k, v in _scales(rank, step, B_PER_RANK).items()}
    decisions = {k: torch.from_numpy(v) for k, v in dec.items()}
    record = {}
    p = rt.unet_forward(ref64, x[sl].double(), scales, decisions=decisions, record=record)
    flips = {k: v for k, v in rt.decision_flips(decisions, record, scales).items() if v[0]}
    assert sum(n for n, _ in flips.values()) <= 8 and all(m <= 1e-5 for _, m in flips.values()), flips
    rt.loss_terms(p, t[sl].double(), **PDE)["loss"].backward()
    g = torch.zeros_like(holder.arena, dtype=torch.float64)
    ref_grads = {n: q.grad for n, q in ref64.named_parameters()}
    for n, view in _per_param(holder, g).items():
        view.copy_(ref_grads[n])
    return g, holder


def _per_param(holder, flat):
    from physics_informed_image_segmentation_amd.unet import _phys_view
    names = [n for n, _ in holder.named_parameters()]
    return {nm: _phys_view(flat[o:o + n], shape, kind)
            for nm, (_, _, shape, kind, o, n) in zip(names, holder._entries)}


@pytest.mark.parametrize("bucket_bytes", [16 << 20, 4])
def test_two_rank_train_mode_matches_oracle(hip, bucket_bytes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_train, args=(r, 2, port, q, bucket_bytes)) for r in range(2)]
    for p in procs:
        p.start()
    res = {r: (steps, w, nb) for r, steps, w, nb in (q.get(timeout=300) for _ in procs)}
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    if bucket_bytes == 4:
        assert res[0][2] == 46  # one bucket per parameter tensor: out_conv's closes on the main stream
    for step in range(2):
        w = res[0][0][step][0]
        assert (w == res[1][0][step][0]).all(), "replicas diverged"  # bitwise-identical replicas
        g_sum = None
        for r in range(2):
            g, holder = _oracle_grads(w, r, step, res[r][0][step][2])
            g_sum = g if g_sum is None else g_sum + g
        for r in range(2):
            got = _per_param(holder, torch.from_numpy(res[r][0][step][1]).double())
            want = _per_param(holder, g_sum)
            worst = max(((got[n] - want[n]).norm() / want[n].norm()).item() for n in want)
            assert worst < 1e-4, (step, r, worst)
        # AdamW with 1/world folded in == torch.optim.AdamW on the oracle's mean gradient; the
        # state carries over, so the second step checks the moments too
        if step == 0:
            cpu = rt.UNetRef(1, 1, 64)
            cpu.load_state_dict({k: v.float() for k, v in holder.state_dict().items()})
            opt = rt.make_adamw(cpu, lr=LR, weight_decay=1e-5)
        else:  # continue the oracle trajectory from the HIP weights the step-2 gradients were taken at
            sd = holder.state_dict()
            with torch.no_grad():
                for n, qq in cpu.named_parameters():
                    qq.copy_(sd[n])
        mean = _per_param(holder, g_sum / 2)
        for n, qq in cpu.named_parameters():
            qq.grad = mean[n].float().clone()
        opt.step()
        w_next = res[0][0][step + 1][0] if step == 0 else res[0][1]
        got_w = UNet_state(w_next)
        worst = max((((got_w[n] - qq.detach()).norm() / qq.detach().norm()).item(), n)
                    for n, qq in cpu.named_parameters())
        assert worst[0] < 1e-4, (step, worst)


def UNet_state(w_arena):
    from physics_informed_image_segmentation_amd import UNet
    holder = UNet(1, 1, 64)
    holder.arena.copy_(torch.from_numpy(w_arena))
    return {k: v.clone() for k, v in holder.state_dict().items()}
