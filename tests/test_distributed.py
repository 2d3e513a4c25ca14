"""Data-parallel path on CPU (gloo, world_size 2 and 8 — C3's rank count): bucket planning over
the gradient arena, the backward-order launch protocol of GradBucketer, the summed result, the
metric all-reduce and the parameter broadcast."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from physics_informed_image_segmentation_amd.distributed import (GradBucketer, allreduce_scalars,
                                                                 broadcast_parameters, plan_buckets)


class FakeModel:
    """Stand-in for UNet's arena interface (arena, grad_arena, arena_entries)."""

    def __init__(self, sizes, align=64):
        self.entries = []
        off = 0
        for i, n in enumerate(sizes):
            self.entries.append((f"p{i}", off, n))
            off += (n + align - 1) // align * align
        self.arena = torch.zeros(off)
        self._g = torch.zeros(off)
        self.grad_ready_hook = None

    def arena_entries(self):
        return self.entries

    def grad_arena(self):
        return self._g


SIZES = [576, 64, 36864, 64, 73728, 128, 147456, 128, 4096, 256, 1000, 1]


def test_plan_buckets_cover_arena_contiguously():
    m = FakeModel(SIZES)
    for cap in (1024, 64 * 1024, 1 << 30):
        b = plan_buckets(m.arena_entries(), m.arena.numel(), cap)
        assert b[0][1] == m.arena.numel() and b[-1][0] == 0
        for (lo, hi), (lo2, hi2) in zip(b, b[1:]):
            assert hi2 == lo  # back-to-front, no gaps
        starts = {o for _, o, _ in m.entries}
        assert all(lo in starts for lo, _ in b)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = FakeModel(SIZES)
        # broadcast: every replica starts from rank 0's arena
        m.arena.copy_(torch.arange(m.arena.numel(), dtype=torch.float32) * (rank + 1))
        broadcast_parameters(m)
        ok_bcast = torch.equal(m.arena, torch.arange(m.arena.numel(), dtype=torch.float32))
        bk = GradBucketer(m, bucket_bytes=64 * 1024 * 4)
        assert m.grad_ready_hook is bk
        launched_trace = []
        for step in range(2):
            g = m.grad_arena()
            g.fill_(0)
            # backward order: last parameter first, gradient = (rank+1) * (index+1) * (step+1)
            for i in reversed(range(len(m.entries))):
                _, o, n = m.entries[i]
                g[o:o + n] = float((rank + 1) * (i + 1) * (step + 1))
                bk.on_ready(o, o + n)
                launched_trace.append(bk.next_bucket)
            bk.finish()
            expect = torch.zeros_like(g)
            for i, (_, o, n) in enumerate(m.entries):
                expect[o:o + n] = float(sum(r + 1 for r in range(world)) * (i + 1) * (step + 1))
            ok = torch.equal(g, expect)
            if not ok:
                break
        # buckets were launched progressively during "backward", not all at the end
        progressive = 0 < launched_trace[len(m.entries) // 2] < len(bk.buckets)
        t = torch.tensor([1.0 * rank, 2.0, 3.0], dtype=torch.float64)
        allreduce_scalars(t)
        ok_metrics = t.tolist() == [float(sum(range(world))), 2.0 * world, 3.0 * world]
        q.put((rank, ok and ok_bcast and ok_metrics, progressive, len(bk.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_bucketed_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(ok for _, ok, _, _ in res), res
    assert all(prog for _, _, prog, _ in res), res
    assert all(nb > 2 for _, _, _, nb in res)
