"""The training step of src/train.py:84-176 (Dropout2d draws, U-Net forward, fused loss,
backward, AdamW) with its forward + backward captured ONCE in a HIP graph and replayed.

The engine enqueues ~250 kernels per step from Python over two HIP streams; replaying them as
one graph removes the host from the step (no per-kernel launch latency, no gaps while Python
catches up). Two pieces stay outside the graph, launched eagerly around each replay:

* the Dropout2d keep-scales: drawn with exactly the eager forward's calls (per block in
  ``BLOCK_ORDER``, ``bernoulli_(1 - p).div_(1 - p)``) into persistent buffers the captured
  kernels read (RNG ops inside a capture make torch-ROCm's ``capture_end`` crash), so graph and
  eager steps consume the generator identically;
* ``AdamW.step``: one launch whose bias corrections change every step (kernel arguments are
  frozen in a graph).

Gradients: the capture runs with every ``.grad`` None, so the engine writes the gradient arena in
overwrite mode and every replay overwrites it (no ``zero_grad`` between replays).
"""
from __future__ import annotations

from typing import Optional

import torch

from .unet import BLOCK_ORDER, UNet


class StepGraph:
    """``StepGraph(model, criterion, optimizer, x, target)``: runs ``warmup`` eager steps (they
    are real training steps), captures the next step's forward + backward, and then each
    ``step()`` is one full training step; ``step(x, target)`` copies a new batch of the same
    shape into the captured input buffers first. Returns the loss tensor (device)."""

    def __init__(self, model: UNet, criterion, optimizer, x: torch.Tensor, target: torch.Tensor, warmup: int = 2):
        if not x.is_cuda:
            raise RuntimeError("StepGraph needs the model and batch on the GPU")
        self.model, self.criterion, self.opt = model, criterion, optimizer
        self.x, self.t = x, target
        B = x.shape[0]
        self.blocks = [(n, model.block(n).p, model.block(n).conv0.out_channels) for n in BLOCK_ORDER
                       if model.training and model.block(n).p > 0]
        self.scales = {n: torch.empty(B, c, device=x.device) for n, _, c in self.blocks}
        if self.blocks:
            if any(p >= 1.0 for _, p, _ in self.blocks):
                raise ValueError("StepGraph: dropout p >= 1")
            model.set_dropout_scales(self.scales)
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):  # plans the engine, allocates every persistent buffer
                self._eager()
        cur.wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)
        # captured on the warm-up stream: autograd's AccumulateGrad nodes remember the stream they
        # were created on, and one created on another stream syncs with it mid-capture (a model
        # that already ran eager steps on the default stream crashes torch-ROCm's capture_end)
        with torch.cuda.graph(self.graph, stream=side):
            self.loss = criterion(model(self.x), self.t)
            self.loss.backward()

    def _refill(self):
        for n, p, _ in self.blocks:
            self.scales[n].bernoulli_(1.0 - p).div_(1.0 - p)

    def _eager(self):
        self._refill()
        self.opt.zero_grad(set_to_none=True)
        loss = self.criterion(self.model(self.x), self.t)
        loss.backward()
        self.opt.step()
        return loss

    def step(self, x: Optional[torch.Tensor] = None, target: Optional[torch.Tensor] = None) -> torch.Tensor:
        if x is not None:
            self.x.copy_(x)
        if target is not None:
            self.t.copy_(target)
        self._refill()
        self.graph.replay()
        self.opt.step()
        return self.loss

    def close(self):
        """Back to the model's own dropout draws (the graph and its buffers are released).
        Synchronises first and releases the graph at once, so its executable (and the events and
        streams its capture referenced) are never torn down by a later garbage collection while
        other work is in flight."""
        torch.cuda.synchronize()
        if self.blocks:
            self.model.set_dropout_scales(None)
        graph, self.graph = self.graph, None
        del graph
        torch.cuda.synchronize()
