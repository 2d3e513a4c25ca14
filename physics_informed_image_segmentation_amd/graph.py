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
import torch.distributed as dist

from . import _hip
from .unet import BLOCK_ORDER, UNet


class StepGraph:
    """``StepGraph(model, criterion, optimizer, x, target)``: runs ``warmup`` eager steps (they
    are real training steps), captures the next step's forward + backward, and then each
    ``step()`` is one full training step; ``step(x, target)`` copies a new batch of the same
    shape into the captured input buffers first. Returns the loss of that step (a fresh device
    tensor: the captured one is overwritten by the next replay).

    Lifetime. A captured graph references everything its capture touched: the engine's
    activation / workspace buffers, its weight-gradient stream, the capture stream and the HIP
    events through which the two streams' edges were recorded; the captured loss's autograd graph
    holds the parameters' AccumulateGrad nodes, which recorded the capture stream and sync with it
    in every later backward of the model while they live. The StepGraph owns all of them — the
    engine, the events (``UNetEngine.capture_events``), the loss (``step()`` hands out detached
    copies, so no caller keeps that autograd graph alive) and the capture stream
    (``_hip.OwnedStream``, recycled only into other owned streams, never destroyed) — and releases
    them in ``close()`` only after the device is idle: the graph, the loss and its autograd graph,
    the events, the engine, then the stream. ``close()`` also runs when the StepGraph is garbage
    collected without it."""

    def __init__(self, model: UNet, criterion, optimizer, x: torch.Tensor, target: torch.Tensor, warmup: int = 2,
                 fused_loss: bool = False, before_capture=None):
        """``fused_loss``: the step runs ``model.forward_with_loss`` (the head + loss forward in one
        kernel, as bench.py and train_epoch do) instead of ``criterion(model(x), target)``.
        ``before_capture``: called once after the eager warm-up steps, right before the capture
        (bench.py clears its launch-hook timers there, so the events the hooks record during the
        capture — graph nodes, re-recorded by every replay — are the only ones they hold)."""
        if not x.is_cuda:
            raise RuntimeError("StepGraph needs the model and batch on the GPU")
        if model.grad_ready_hook is not None or (dist.is_available() and dist.is_initialized()
                                                 and dist.get_world_size() > 1):
            raise RuntimeError("StepGraph captures a single-process step: data-parallel all-reduces "
                               "(GradBucketer) cannot be replayed from a graph")
        self.graph = None
        self.fused_loss = fused_loss
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
        self._stream = _hip.OwnedStream(device=x.device)
        side = self._stream.stream
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):  # plans the engine, allocates every persistent buffer
                self._eager()
        cur.wait_stream(side)
        torch.cuda.synchronize()
        self.engine = model.engine()
        self.engine.capture_events = []
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)
        # captured on the warm-up stream: autograd's AccumulateGrad nodes remember the stream they
        # were created on, and one created on another stream syncs with it mid-capture (a model
        # that already ran eager steps on the default stream crashes torch-ROCm's capture_end)
        if before_capture is not None:
            before_capture()
        with torch.cuda.graph(self.graph, stream=side):
            self.loss = self._forward_loss()
            self.loss.backward()
        # the events the capture recorded through, including the engine's workspace fences
        self._events = list(self.engine.capture_events) + [e for e in self.engine.ws3_free if e is not None]
        self.engine.capture_events = []
        self.engine.ws3_free = [None, None]
        # the gradient buffers the replays write: AdamW must see exactly these
        self._grads = [(p, p.grad.data_ptr()) for p in model.parameters() if p.grad is not None]

    def _refill(self):
        for n, p, _ in self.blocks:
            self.scales[n].bernoulli_(1.0 - p).div_(1.0 - p)

    def _forward_loss(self):
        if self.fused_loss:
            return self.model.forward_with_loss(self.x, self.t, self.criterion)[1]
        return self.criterion(self.model(self.x), self.t)

    def _eager(self):
        self._refill()
        self.opt.zero_grad(set_to_none=True)
        loss = self._forward_loss()
        loss.backward()
        self.opt.step()
        return loss

    def step(self, x: Optional[torch.Tensor] = None, target: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.graph is None:
            raise RuntimeError("StepGraph.step after close()")
        if x is not None:
            self.x.copy_(x)
        if target is not None:
            self.t.copy_(target)
        for p, ptr in self._grads:  # e.g. zero_grad(set_to_none=True) between steps would detach them
            if p.grad is None or p.grad.data_ptr() != ptr:
                raise RuntimeError("StepGraph: a parameter's .grad no longer views the captured gradient "
                                   "buffer (do not zero_grad / replace grads between graph steps)")
        self._refill()
        self.graph.replay()
        self.opt.step()
        return self.loss.detach().clone()

    def close(self):
        """Back to the model's own dropout draws; the graph, then the events, the engine reference
        and the owned capture stream are released, each only once the device is idle."""
        if self.graph is None and getattr(self, "_stream", None) is None:
            return
        torch.cuda.synchronize()
        if self.blocks:
            self.model.set_dropout_scales(None)
        graph, self.graph = self.graph, None
        del graph
        self.loss = None  # its autograd graph (AccumulateGrad nodes on the capture stream) with it
        torch.cuda.synchronize()
        self._events = []
        self.engine = None
        stream, self._stream = getattr(self, "_stream", None), None
        if stream is not None:
            stream.close()

    def __del__(self):
        try:
            if getattr(self, "graph", None) is not None or getattr(self, "_stream", None) is not None:
                self.close()
        except Exception:  # interpreter shutdown
            pass
