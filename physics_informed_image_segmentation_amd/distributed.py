"""Data-parallel training over RCCL (torch.distributed backend "nccl" = RCCL on
ROCm), one process per GPU.

The reference has no distributed code; this is the one
strategy the north star adds: every rank holds a full replica, runs the step
on its own shard of the batch (Dice is over the local batch, standard DDP
semantics) and the 20.5 M fp32 gradients (82 MB) are summed
across ranks while the backward is still running:

  * the gradient arena is laid out in parameter-creation order and the
    backward produces it back to front (out_conv ... enc1), so buckets are
    contiguous arena ranges cut from the END;
  * the engine reports each finished layer range (``on_ready``); when a
    bucket is fully written it is all-reduced with ``async_op=True`` — RCCL
    runs on its own stream, ordered after the kernels already enqueued on the
    compute stream, concurrently with the rest of the backward;
  * at the end of backward ``finish`` makes the compute stream wait for the
    outstanding buckets (no host synchronisation); the 1/world averaging is
    folded into the AdamW kernel (``grad_scale``).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist


def env_world() -> Tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1 process = 1 GPU)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init_from_env(backend: Optional[str] = None) -> Tuple[int, int, int]:
    rank, local_rank, world = env_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group(backend, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
    return rank, local_rank, world


def plan_buckets(entries: List[Tuple[str, int, int]], arena_numel: int, bucket_bytes: int) -> List[Tuple[int, int]]:
    """Contiguous [lo, hi) arena ranges, cut from the end at parameter
    boundaries, each about ``bucket_bytes`` (the last one may be larger or
    smaller). Returned in backward (completion) order."""
    bounds = sorted({o for _, o, _ in entries})
    cap = max(1, bucket_bytes // 4)
    buckets = []
    hi = arena_numel
    lo = hi
    for o in reversed(bounds):
        lo = o
        if hi - lo >= cap:
            buckets.append((lo, hi))
            hi = lo
    if hi > 0:
        buckets.append((0, hi))
    return buckets


class GradBucketer:
    """Overlaps the gradient all-reduce with the U-Net backward (see module doc)."""

    def __init__(self, model, bucket_bytes: int = 16 << 20, process_group=None):
        self.model = model
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.bucket_bytes = bucket_bytes
        self.buckets = plan_buckets(model.arena_entries(), model.arena.numel(), bucket_bytes)
        # timing (bench.py): per step, HIP events at the end of the backward's compute on both
        # streams and after the all-reduces have been waited for -> the exposed all-reduce time
        self.timing = False
        self._marks = None
        self._events: List = []
        self._reset()
        model.grad_ready_hook = self

    def _reset(self):
        self.low_water = [hi for _, hi in self.buckets]  # lowest written offset inside each bucket
        self.launched = [False] * len(self.buckets)
        self.works: List = []
        self.next_bucket = 0

    def on_ready(self, lo: int, hi: int) -> None:
        """Engine callback: gradient range [lo, hi) is enqueued (backward order)."""
        for i in range(self.next_bucket, len(self.buckets)):
            blo, bhi = self.buckets[i]
            if hi <= blo or lo >= bhi:
                continue
            self.low_water[i] = min(self.low_water[i], max(lo, blo))
        # launch every leading bucket that is now complete, in order
        while self.next_bucket < len(self.buckets):
            i = self.next_bucket
            blo, bhi = self.buckets[i]
            if self.low_water[i] > self._first_param_start(blo, bhi):
                break
            self._launch(i)
            self.next_bucket += 1

    def _first_param_start(self, blo: int, bhi: int) -> int:
        starts = [o for _, o, _ in self.model.arena_entries() if blo <= o < bhi]
        return min(starts) if starts else blo

    def _launch(self, i: int) -> None:
        blo, bhi = self.buckets[i]
        g = self.model.grad_arena()
        self.works.append(dist.all_reduce(g[blo:bhi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
        self.launched[i] = True

    def mark_backward_done(self, main, side) -> None:
        """Engine callback right before ``finish``: every gradient kernel is enqueued on ``main`` /
        ``side``. With ``timing`` set, an event on each marks where the compute ends."""
        if not self.timing:
            return
        e_main, e_side = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e_main.record(main)
        e_side.record(side)
        self._marks = (e_main, e_side)

    def finish(self) -> None:
        """After backward: launch anything left, make the compute stream wait."""
        while self.next_bucket < len(self.buckets):
            self._launch(self.next_bucket)
            self.next_bucket += 1
        for w in self.works:
            w.wait()
        if self._marks is not None:  # the current stream now waits for every all-reduce
            e_after = torch.cuda.Event(enable_timing=True)
            e_after.record()
            self._events.append((*self._marks, e_after))
            self._marks = None
        self._reset()

    def exposed_ms(self) -> List[float]:
        """Per timed step (``timing`` set), the all-reduce time NOT hidden behind the backward: from
        the later of the two streams' last gradient kernel to the point where the gradients are
        summed on every rank. Synchronises the device; clears the record."""
        torch.cuda.synchronize()
        out = [max(0.0, min(em.elapsed_time(ea), es.elapsed_time(ea))) for em, es, ea in self._events]
        self._events = []
        return out


def allreduce_scalars(t: torch.Tensor, op=None) -> torch.Tensor:
    """Sum (default) a small metrics tensor across ranks; no-op when single-process."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return t


def broadcast_parameters(model, src: int = 0) -> None:
    """Start every replica from rank 0's weights (one broadcast of the arena)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(model.arena, src)
