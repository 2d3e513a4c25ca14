"""U-Net of src/unet.py on the MI355X kernel path.

``UNet`` keeps the reference's constructor, module tree, parameter creation
order (so ``torch.manual_seed`` gives identical weights), state_dict keys and
shapes (src/unet.py:108-167). Its forward returns sigmoid probabilities
(src/unet.py:169-216) but never runs an ATen convolution: the whole network
is one autograd node whose forward/backward are sequences of HIP kernels
(``UNetEngine``) over NHWC activations.

Memory layout (MI355X-first):
  * every parameter is a view into ONE flat fp32 arena; conv weights are
    physically KRSC ([Cout][3][3][Cin] = OIHW channels_last) and ConvTranspose
    weights [2][2][Cout][Cin], so the kernels read them directly and AdamW /
    the RCCL all-reduce see one contiguous buffer;
  * gradients land in a second arena with the same layout, in reverse
    creation order during backward (out_conv first), which is what lets
    data-parallel buckets be contiguous ranges all-reduced while backward runs;
  * skip concatenation is free: the encoder block writes its output straight
    into the second channel half of the decoder's concat buffer and the
    transposed conv writes the first half (src/unet.py:190-202).
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import _hip
from ._hip import (PIS_ACCUMULATE, PIS_FILTER_READY, PIS_MASK, PIS_RELU, PIS_SCALE, PIS_W_UNFLIPPED, PIS_WINO_PREPARED,
                   call, ptr)

# block name -> dropout multiplier of UNet(dropout=d), src/unet.py:120-154
_DROP_MULT = {"enc1": 0.0, "enc2": 0.5, "enc3": 1.0, "enc4": 1.0, "bottleneck": 1.0,
              "dec4": 1.0, "dec3": 0.5, "dec2": 0.5, "dec1": 0.0}
BLOCK_ORDER = ("enc1", "enc2", "enc3", "enc4", "bottleneck", "dec4", "dec3", "dec2", "dec1")
_ALIGN = 64  # floats: every parameter starts on a 256-byte boundary of the arena


class DoubleConv(nn.Module):
    """Parameter container with the reference's layout (src/unet.py:19-42):
    ``conv = Sequential(Conv2d, ReLU, [Dropout2d], Conv2d, ReLU)``. Its compute
    only exists inside the fused ``UNet`` engine."""

    def __init__(self, in_channels: int, out_channels: int, dropout: float = 0.0, activation: str = "relu"):
        super().__init__()
        if activation.lower() != "relu":
            raise NotImplementedError(
                f"intermediate_activation={activation!r}: only 'relu' is on the MI355X path "
                "(the reference's configs never select another, src/ablation.py:44-45)")
        act = nn.ReLU(inplace=True)
        layers: List[nn.Module] = [nn.Conv2d(in_channels, out_channels, kernel_size=3, padding=1), act]
        if dropout > 0:
            layers.append(nn.Dropout2d(dropout))
        layers += [nn.Conv2d(out_channels, out_channels, kernel_size=3, padding=1), act]
        self.conv = nn.Sequential(*layers)
        self.p = float(dropout)

    @property
    def conv0(self) -> nn.Conv2d:
        return self.conv[0]

    @property
    def conv1(self) -> nn.Conv2d:
        return self.conv[3] if self.p > 0 else self.conv[2]

    def forward(self, x):  # pragma: no cover - guard against silent ATen fallbacks
        raise RuntimeError("DoubleConv is evaluated only inside UNet.forward (HIP engine)")


def count_parameters(model: nn.Module) -> int:
    """src/unet.py:220-230."""
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def _phys_view(flat: torch.Tensor, logical: torch.Size, kind: str) -> torch.Tensor:
    """View of the arena slice with the logical (reference) shape."""
    if kind == "conv":  # logical (O, I, kh, kw) stored [O][kh][kw][I]
        O, I_, kh, kw = logical
        return flat.view(O, kh, kw, I_).permute(0, 3, 1, 2)
    if kind == "convt":  # logical (Cin, Cout, 2, 2) stored [i][j][o][c]
        Ci, Co, kh, kw = logical
        return flat.view(kh, kw, Co, Ci).permute(3, 2, 0, 1)
    return flat.view(logical)


class UNet(nn.Module):
    """Drop-in for ``src.unet.UNet`` (src/unet.py:79-216) on the HIP path."""

    def __init__(self, in_channels: int = 1, out_channels: int = 1, base_channels: int = 64,
                 dropout: float = 0.2, output_activation: str = "sigmoid",
                 intermediate_activation: str = "relu"):
        super().__init__()
        if output_activation.lower() not in ("sigmoid", "tanh"):
            raise ValueError(f"Unsupported output_activation: {output_activation}. Must be 'sigmoid' or 'tanh'")
        if output_activation.lower() != "sigmoid":
            raise NotImplementedError("output_activation='tanh' is not on the MI355X path (sigmoid only)")
        if out_channels != 1:
            raise NotImplementedError("out_channels must be 1 (single probability map, src/unet.py:157)")
        if not (in_channels == 1 or in_channels % 4 == 0):
            raise NotImplementedError("in_channels must be 1 or a multiple of 4")
        if base_channels % 64 != 0:
            raise NotImplementedError("base_channels must be a multiple of 64 on the MI355X path")
        c = base_channels
        self.in_channels, self.base_channels, self.dropout_rate = in_channels, c, float(dropout)
        act = intermediate_activation
        # creation order == RNG order == reference parameter order
        self.enc1 = DoubleConv(in_channels, c, dropout=0.0, activation=act)
        self.enc2 = DoubleConv(c, 2 * c, dropout=dropout * 0.5, activation=act)
        self.enc3 = DoubleConv(2 * c, 4 * c, dropout=dropout, activation=act)
        self.enc4 = DoubleConv(4 * c, 8 * c, dropout=dropout, activation=act)
        self.pool = nn.MaxPool2d(kernel_size=2, stride=2)
        self.bottleneck = DoubleConv(8 * c, 8 * c, dropout=dropout, activation=act)
        self.up4 = nn.ConvTranspose2d(8 * c, 8 * c, kernel_size=2, stride=2)
        self.dec4 = DoubleConv(16 * c, 8 * c, dropout=dropout, activation=act)
        self.up3 = nn.ConvTranspose2d(8 * c, 4 * c, kernel_size=2, stride=2)
        self.dec3 = DoubleConv(8 * c, 4 * c, dropout=dropout * 0.5, activation=act)
        self.up2 = nn.ConvTranspose2d(4 * c, 2 * c, kernel_size=2, stride=2)
        self.dec2 = DoubleConv(4 * c, 2 * c, dropout=dropout * 0.5, activation=act)
        self.up1 = nn.ConvTranspose2d(2 * c, c, kernel_size=2, stride=2)
        self.dec1 = DoubleConv(2 * c, c, dropout=0.0, activation=act)
        self.out_conv = nn.Conv2d(c, out_channels, kernel_size=1)
        self.output_activation = nn.Sigmoid()
        self.activation_name = "sigmoid"
        self._pack_arena()
        self._engine: Optional[UNetEngine] = None
        self._drop_override: Optional[Dict[str, torch.Tensor]] = None
        self.grad_ready_hook = None  # object with on_ready(lo, hi) / finish(): DDP bucketer
        self.last_logits: Optional[torch.Tensor] = None

    # ---- arena -------------------------------------------------------------
    def _param_kinds(self):
        kinds = {}
        for name, mod in self.named_modules():
            if isinstance(mod, nn.ConvTranspose2d):
                kinds[id(mod.weight)] = "convt"
            elif isinstance(mod, nn.Conv2d) and mod.kernel_size == (3, 3):
                kinds[id(mod.weight)] = "conv"
        return kinds

    def _pack_arena(self):
        kinds = self._param_kinds()
        entries = []  # (module, name, shape, kind, offset, numel)
        off = 0
        for mname, mod in self.named_modules():
            for pname, p in list(mod._parameters.items()):
                if p is None:
                    continue
                n = p.numel()
                entries.append((mod, pname, p.shape, kinds.get(id(p), "plain"), off, n))
                off += (n + _ALIGN - 1) // _ALIGN * _ALIGN
        arena = torch.zeros(off, dtype=torch.float32)
        for mod, pname, shape, kind, o, n in entries:
            old = mod._parameters[pname]
            view = _phys_view(arena[o:o + n], shape, kind)
            view.copy_(old.detach())
            mod._parameters[pname] = nn.Parameter(view, requires_grad=old.requires_grad)
        self._arena = arena
        self._entries = [(mod, pname, shape, kind, o, n) for mod, pname, shape, kind, o, n in entries]
        self._grad_arena: Optional[torch.Tensor] = None

    @property
    def arena(self) -> torch.Tensor:
        return self._arena

    def grad_arena(self) -> torch.Tensor:
        if self._grad_arena is None or self._grad_arena.device != self._arena.device:
            self._grad_arena = torch.zeros_like(self._arena)
        return self._grad_arena

    def param_offset(self, p: torch.Tensor) -> int:
        for mod, pname, shape, kind, o, n in self._entries:
            if mod._parameters[pname] is p:
                return o
        raise KeyError("parameter does not belong to this UNet")

    def arena_entries(self):
        """[(qualified_name, offset, numel)] in arena order."""
        names = {id(p): n for n, p in self.named_parameters()}
        return [(names[id(mod._parameters[pn])], o, n) for mod, pn, _, _, o, n in self._entries]

    def grad_views(self) -> List[torch.Tensor]:
        g = self.grad_arena()
        return [_phys_view(g[o:o + n], shape, kind) for _, _, shape, kind, o, n in self._entries]

    def _rebind(self):
        for mod, pname, shape, kind, o, n in self._entries:
            mod._parameters[pname].data = _phys_view(self._arena[o:o + n], shape, kind)

    def _apply(self, fn, recurse=True):
        new = fn(self._arena)
        if new.dtype != torch.float32:
            raise NotImplementedError("the MI355X path is fp32 (reference parity); dtype casts are unsupported")
        self._arena = new
        self._rebind()
        if self._grad_arena is not None:
            self._grad_arena = fn(self._grad_arena)
        for mod, pname, shape, kind, o, n in self._entries:
            mod._parameters[pname].grad = None
        for name, buf in self._buffers.items():
            if buf is not None:
                self._buffers[name] = fn(buf)
        self._engine = None
        return self

    # ---- dropout control -----------------------------------------------------
    def set_dropout_scales(self, scales: Optional[Dict[str, torch.Tensor]]):
        """Inject Dropout2d keep-scales {block: (B, C) tensor of 0 or 1/(1-p)} for
        the next training forward (parity runs); None restores the RNG draw."""
        self._drop_override = scales

    def block(self, name: str) -> DoubleConv:
        return getattr(self, name)

    @torch.no_grad()
    def activation_decisions(self) -> Dict[str, torch.Tensor]:
        """The ReLU masks and 2x2 max-pool window argmaxes (dy * 2 + dx, first max)
        of the last forward, NCHW on the host, keyed like the oracle's sites
        ("enc1.0", "enc1.1", "pool1", ..., "dec1.1"). Introspection for parity
        tests: fp32 rounding decides ReLU pre-activations within ~1e-7 of zero, so
        gradients are compared with float64 evaluated on the same decisions."""
        eng = self._engine
        if eng is None or not eng.bufs:
            raise RuntimeError("activation_decisions: no forward has run")
        bf, c = eng.bufs, self.base_channels
        nchw = lambda t: t.permute(0, 3, 1, 2).contiguous()
        out = {}
        for l in range(1, 5):
            Cl = c << (l - 1)
            skip = nchw(bf[f"cat{l}"][..., Cl:])
            out[f"enc{l}.0"] = nchw(bf[f"a{l}"]) > 0
            out[f"enc{l}.1"] = skip > 0
            B, C, H, W = skip.shape
            win = skip.reshape(B, C, H // 2, 2, W // 2, 2).permute(0, 1, 2, 4, 3, 5).reshape(B, C, H // 2, W // 2, 4)
            out[f"pool{l}"] = win.argmax(-1)
            out[f"dec{l}.0"] = nchw(bf[f"d0_{l}"]) > 0
            out[f"dec{l}.1"] = nchw(bf[f"d1_{l}"]) > 0
        out["bottleneck.0"] = nchw(bf["b0"]) > 0
        out["bottleneck.1"] = nchw(bf["b1"]) > 0
        return {k: v.cpu() for k, v in out.items()}

    # ---- forward -------------------------------------------------------------
    def engine(self) -> "UNetEngine":
        if self._engine is None:
            self._engine = UNetEngine(self)
        return self._engine

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _hip.require_cuda(x, "UNet.forward")
        if x.dim() != 4 or x.shape[1] != self.in_channels:
            raise ValueError(f"expected input (B, {self.in_channels}, H, W), got {tuple(x.shape)}")
        if x.dtype != torch.float32:
            raise TypeError("UNet expects float32 input")
        if x.shape[2] % 16 or x.shape[3] % 16:
            raise ValueError("H and W must be divisible by 16 (four 2x2 max-pools, src/unet.py:180-186)")
        if self._arena.device != x.device:
            raise RuntimeError(f"model is on {self._arena.device}, input on {x.device}")
        params = [mod._parameters[pn] for mod, pn, *_ in self._entries]
        needs_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        eng = self.engine()
        scales = eng.dropout_scales(x.shape[0], self.training, self._drop_override)
        if not needs_grad:
            return eng.forward(x, scales, keep=False)
        return _UNetFunction.apply(x, eng, scales, *params)

    def forward_with_loss(self, x: torch.Tensor, targets: torch.Tensor, criterion) -> Tuple[torch.Tensor, torch.Tensor]:
        """``u = model(x); loss = criterion(u, targets)`` (src/train.py:108-110) with the head's 1x1 conv +
        sigmoid and the whole loss forward in ONE kernel (pis_head_loss_fwd: the 64-channel head input
        is read once, the loss's own pass over u and the targets disappears). Same outputs as the two
        calls: u, the differentiable loss, and ``criterion.last`` (terms, per-sample counters, scores);
        the backward is the usual fused head + loss backward. Criteria other than this package's
        losses, or shapes the fused kernel does not cover, take the two calls."""
        from .fused import loss_from_forward
        config = getattr(criterion, "config", None)
        if not callable(config):
            u = self(x)
            return u, criterion(u, targets)
        cfg = config()
        t = targets.to(device=x.device, dtype=torch.float32).contiguous()
        if t.numel() != x.shape[0] * x.shape[2] * x.shape[3]:
            raise ValueError(f"target shape {tuple(targets.shape)} does not match the input {tuple(x.shape)}")
        sink: Dict[str, torch.Tensor] = {}
        eng = self.engine()
        eng.loss_request = (t, cfg.params(), sink)
        try:
            u = self(x)
        finally:
            eng.loss_request = None
        if "terms" not in sink:  # not fusable here: the two calls
            return u, criterion(u, targets)
        criterion.last = sink
        return u, loss_from_forward(u, t, cfg, sink)


class _UNetFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eng, scales, *params):
        u = eng.forward(x, scales, keep=True)
        ctx.eng = eng
        ctx.gen = eng.generation
        ctx.n_params = len(params)
        return u

    @staticmethod
    def backward(ctx, du):
        eng: UNetEngine = ctx.eng
        if eng.generation != ctx.gen:
            raise RuntimeError("UNet.backward: another forward ran since this graph was built "
                               "(activations are kept in one set of engine buffers)")
        grads = eng.backward(du)
        return (None, None, None) + tuple(grads)


# =============================================================================
#  Engine
# =============================================================================

class _Buf:
    """NHWC activation: tensor + channel stride + channel offset."""
    __slots__ = ("t", "ld", "off")

    def __init__(self, t: torch.Tensor, ld: int, off: int = 0):
        self.t, self.ld, self.off = t, ld, off

    @property
    def p(self) -> int:
        return self.t.data_ptr() + 4 * self.off

    def slice(self, off: int) -> "_Buf":
        return _Buf(self.t, self.ld, self.off + off)


class UNetEngine:
    """Explicit forward/backward schedule of the U-Net over HIP kernels.

    Forward keeps every activation the backward needs (no recomputation);
    backward walks out_conv -> dec1 -> up1 -> ... -> enc1, writing each
    layer's weight gradient into the gradient arena as soon as it is known and
    reporting the finished arena range to ``model.grad_ready_hook`` (the DDP
    bucket trigger)."""

    # weight gradients on a second HIP stream: they depend only on (x, dz) and write their own
    # arena slice, so they overlap the input-gradient chain (the critical path), whose
    # transforms are HBM-bound while the weight-gradient GEMMs are MFMA-bound
    # (PIS_SIDE_STREAM=0 serialises them on the caller's stream, for A/B measurements)
    side_stream = os.environ.get("PIS_SIDE_STREAM", "1") != "0"
    # where a prepared layer's weight gradient joins the side stream (tools/ab_streams.py): "prep"
    # right after dz's transforms, "gemm" after the input gradient's contractions, "dgrad" after
    # the whole input gradient
    side_sync = os.environ.get("PIS_SIDE_SYNC", "prep")
    # PIS_FILTER_AHEAD=1: the F(4x4,3x3) filter transforms of a step (forward: the layers' weights;
    # backward: their rotated input-gradient form) run on the side stream, idle during the forward,
    # at its start, and the main stream's convs wait on one event each instead of transforming
    # their own. Measured 1.5 % SLOWER at C2 in round 2 (tools/ab_tune.py: 31.48 vs 31.01 ms, and
    # 31.39 vs 30.95 with the backward's transforms at the start of the backward).
    # PIS_FILTER_AHEAD=2: every filter transform of the step (both directions) in ONE launch on the
    # main stream at the start of the training forward (pis_conv3x3_filters) instead of 34 small,
    # latency-bound launches: measured neutral at C2 in round 2 (31.29 vs 31.27 ms). 0: each conv
    # transforms its own filter.
    # PIS_FILTER_AHEAD=3: only the direct fp16x3 layers' weight splits (both directions) in ONE launch
    # at the forward's start: 12 small main-stream launches fewer, six of them in the backward.
    # Measured neutral on the C2 step (344.2 vs 344.0 img/s, profiles/r3_q25_ab_env.txt).
    # PIS_FILTER_AHEAD=4: 2 and 3 together (the direct splits, then the Winograd transforms: two
    # launches on the main stream at the forward's start); 5 (default since round 5): the same two
    # launches on the side stream (idle during the forward), the first consumer of each waiting on
    # its event. With the direct layers' weight gradients on the main stream (below), the main
    # stream is the step's critical path and its ~34 small latency-bound transform launches show:
    # 5 vs 0 is 21.47-21.55 vs 21.85-22.48 ms over four same-process A/B runs, 2 at 21.46-21.91,
    # 3 at 21.68-21.96 (profiles/r5_j_ab_filter_ahead.txt).
    filter_ahead = os.environ.get("PIS_FILTER_AHEAD", "5")
    # "1" (default): every direct-kernel layer's weight gradient on the main stream right after its
    # input gradient (see the backward); "0": on the weight-gradient stream; "dec": the decoder's on
    # the main stream, the encoder's on the weight-gradient stream
    direct_wgrad_main = os.environ.get("PIS_DIRECT_WGRAD_MAIN", "1")
    # a prepared layer whose input gradient runs the fused contraction + output transform (one
    # 139-KB block per CU: it cannot share a CU, so beside the side stream's weight gradient it
    # waits for whole CUs — dec2.conv0 at C2: 1.13 ms live, 0.45 ms alone): "1" (default) runs that
    # layer's weight gradient on the main stream right after its input gradient. Step-neutral
    # (21.68 / 21.62 / 22.03 vs 21.71 / 21.61 / 22.03 ms, interleaved, profiles/r6_ab2_fused_wgrad_main.txt),
    # but the fused kernel runs at its own rate: 0.667 -> 0.459 ms per launch live
    fused_wgrad_main = os.environ.get("PIS_FUSED_WGRAD_MAIN", "1")
    # the U-Net levels (digits 1-4) whose transposed conv's weight gradient runs on the main stream
    # right after its input gradient, in the main workspace, instead of on the weight-gradient stream
    convt_wgrad_main = os.environ.get("PIS_CONVT_WGRAD_MAIN", "")

    def __init__(self, model: UNet):
        self.m = model
        self.c = model.base_channels
        self.plan_key = None
        self.generation = 0
        self.bufs: Dict[str, torch.Tensor] = {}
        self._offsets = {id(mod._parameters[pn]): (o, n) for mod, pn, _, _, o, n in model._entries}
        self.last_grad_mode = None
        self.pending_head = None  # dL/du tensor whose head backward already ran fused with the loss
        self.convt_ready = False  # the transposed convs' input-gradient weights prepared by the forward
        # (targets, LossParams, sink) set by UNet.forward_with_loss for the next forward: its head runs
        # fused with the loss forward (pis_head_loss_fwd) and the loss outputs land in the sink
        self.loss_request = None
        # HIP events created while a graph capture runs: the captured graph's cross-stream edges
        # were recorded through them, so they are kept (and handed to the StepGraph that owns the
        # graph) instead of being destroyed mid-capture when the local reference goes
        self.capture_events: List[torch.cuda.Event] = []

    # ---- planning -----------------------------------------------------------
    def _plan(self, B: int, H: int, W: int, dev: torch.device):
        key = (B, H, W, dev)
        if key == self.plan_key:
            return
        c = self.c
        f = lambda *shape: torch.empty(*shape, dtype=torch.float32, device=dev)
        b = {}
        for l in range(1, 5):
            Hl, Wl, Cl = H >> (l - 1), W >> (l - 1), c << (l - 1)
            b[f"a{l}"] = f(B, Hl, Wl, Cl)            # conv0 output of enc_l
            b[f"cat{l}"] = f(B, Hl, Wl, 2 * Cl)      # [up_l | enc_l]
            b[f"pool{l}"] = f(B, Hl // 2, Wl // 2, Cl)
            b[f"d0_{l}"] = f(B, Hl, Wl, Cl)          # dec_l conv0 output
            b[f"d1_{l}"] = f(B, Hl, Wl, Cl)          # dec_l conv1 output
        H5, W5 = H >> 4, W >> 4
        b["b0"] = f(B, H5, W5, 8 * c)
        b["b1"] = f(B, H5, W5, 8 * c)
        b["u"] = f(B, 1, H, W)
        b["z"] = f(B, 1, H, W)  # pre-sigmoid logits of the last forward (out_conv output)
        self.bufs = b
        self.gbufs: Dict[str, torch.Tensor] = {}
        self.plan_key = key
        self.B, self.H, self.W = B, H, W
        lib = _hip.lib()
        # the fused head + loss forward's partials (per-block sums, overwritten every call)
        self.hl_ws = torch.empty((lib.pis_head_loss_fwd_ws(B, H, W) + 15) // 4, dtype=torch.float32, device=dev)
        ws = lib.pis_head_bwd_ws(B * H * W, c)
        if W <= 1024:
            ws = max(ws, lib.pis_head_loss_bwd_ws(B, H, W, c))
        for l in range(1, 5):
            Hl, Wl, Cl = H >> (l - 1), W >> (l - 1), c << (l - 1)
            cin0 = self.m.in_channels if l == 1 else Cl // 2
            ws = max(ws, lib.pis_conv3x3_wgrad_ws(B, Hl, Wl, cin0, Cl), lib.pis_conv3x3_wgrad_ws(B, Hl, Wl, Cl, Cl),
                     lib.pis_conv3x3_wgrad_ws(B, Hl, Wl, 2 * Cl, Cl), lib.pis_conv3x3_ex_ws(B, Hl, Wl, cin0, Cl),
                     lib.pis_conv3x3_ex_ws(B, Hl, Wl, Cl, Cl), lib.pis_conv3x3_ex_ws(B, Hl, Wl, 2 * Cl, Cl))
            cup = 8 * c if l == 4 else 2 * Cl
            ws = max(ws, lib.pis_convt2x2_wgrad_ws(B, Hl // 2, Wl // 2, cup, Cl))
        ws = max(ws, lib.pis_conv3x3_wgrad_ws(B, H5, W5, 8 * c, 8 * c), lib.pis_conv3x3_ex_ws(B, H5, W5, 8 * c, 8 * c))
        self.ws = torch.empty((ws + 15) // 4, dtype=torch.float32, device=dev)
        self.ws_bytes = self.ws.numel() * 4
        # weight gradients run on a second stream beside the input-gradient chain (backward)
        self.ws2 = torch.empty_like(self.ws) if self.side_stream else self.ws
        # an owned stream, not one of torch's pooled ones: it takes part in any graph capture of
        # the step (graph.StepGraph); created on the model's device and, when the engine goes,
        # recycled only into other owned streams of that device (never destroyed: _hip.OwnedStream)
        # (confining this stream to 64 or 128 CUs with a CU mask measured 16 % slower on the step,
        # profiles/r3_q25_ab_env.txt: the two streams time-share the whole chip)
        self._side_owner = _hip.OwnedStream(device=dev) if self.side_stream else None
        self.side = self._side_owner.stream if self.side_stream else None
        # pis_conv3x3_bwd_prep writes a layer's weight-gradient dz transform from the MAIN stream
        # while the side stream may still read the previous layer's: two alternating workspaces
        # for those weight gradients, each reused only after the side stream has finished with it
        ws3 = 0
        for l in range(1, 6):
            Hl, Wl, Cl = (H >> (l - 1), W >> (l - 1), c << (l - 1)) if l < 5 else (H5, W5, 8 * c)
            for cin in (Cl // 2, Cl, 2 * Cl):
                ws3 = max(ws3, lib.pis_conv3x3_wgrad_ws(B, Hl, Wl, cin, Cl))
        self.ws3 = [torch.empty((ws3 + 15) // 4, dtype=torch.float32, device=dev) for _ in range(2)]
        self.ws3_bytes = self.ws3[0].numel() * 4
        self.ws3_free: List[Optional[torch.cuda.Event]] = [None, None]
        # per-layer kept Winograd input transforms (training forward -> weight gradient);
        # ~2.25x each layer's input activation, ~12 GB at B=8 512^2
        self.keep: Dict[int, torch.Tensor] = {}
        for name in BLOCK_ORDER:
            blk = self.m.block(name)
            lvl = 5 if name == "bottleneck" else int(name[-1])
            Hl, Wl = H >> (lvl - 1), W >> (lvl - 1)
            for conv in (blk.conv0, blk.conv1):
                nb = lib.pis_conv3x3_keep_bytes(B, Hl, Wl, conv.in_channels, conv.out_channels)
                if nb:
                    self.keep[id(conv)] = torch.empty((nb + 3) // 4, dtype=torch.float32, device=dev)
        # per-layer filter transforms computed ahead (forward order; the backward walks them in
        # reverse): {id(conv): (conv, H, W, buffer)}
        self.ffilt: Dict[int, tuple] = {}
        self.bfilt: Dict[int, tuple] = {}
        self.fev: Dict[int, Optional[torch.cuda.Event]] = {}  # filters computed for this forward
        self.bev: Dict[int, Optional[torch.cuda.Event]] = {}  # ... for its backward (None: same stream)
        self.filter_jobs = None
        self.filter_jobs_d = None  # modes 4 / 5: the direct layers' splits (the Winograd ones in filter_jobs)
        mode = str(self.filter_ahead)
        if mode == "5" and self.side is None:
            mode = "4"
        self._fa_mode = mode
        if (mode == "1" and self.side is not None) or mode in ("2", "3", "4", "5"):
            for name in BLOCK_ORDER:
                blk = self.m.block(name)
                lvl = 5 if name == "bottleneck" else int(name[-1])
                Hl, Wl = H >> (lvl - 1), W >> (lvl - 1)
                for conv in (blk.conv0, blk.conv1):
                    if conv.in_channels == 1:
                        continue
                    # modes 1/2: the layers whose transform is kept for the weight gradient (the
                    # Winograd ones); mode 3: the others, i.e. the direct kernel's layers
                    if mode in ("1", "2", "3") and (id(conv) in self.keep) != (mode != "3"):
                        continue
                    ci, co = conv.in_channels, conv.out_channels
                    nb = lib.pis_conv3x3_filter_bytes(B, Hl, Wl, ci, co, 0)
                    if nb:
                        self.ffilt[id(conv)] = (conv, Hl, Wl, torch.empty((nb + 3) // 4, dtype=torch.float32,
                                                                          device=dev))
                    nb = lib.pis_conv3x3_filter_bytes(B, Hl, Wl, ci, co, 1)
                    if nb and not (name == "enc1" and conv is blk.conv0):  # the first conv has no dgrad
                        self.bfilt[id(conv)] = (conv, Hl, Wl, torch.empty((nb + 3) // 4, dtype=torch.float32,
                                                                          device=dev))
        if mode in ("2", "3", "4", "5") and (self.ffilt or self.bfilt):
            jobs = [(t, 0) for t in self.ffilt.values()] + [(t, 1) for t in self.bfilt.values()]

            def table(sel):
                arr = (_hip.FilterJob * len(sel))()
                for k, ((conv, Hl, Wl, buf), dg) in enumerate(sel):
                    arr[k] = _hip.FilterJob(conv.weight.data_ptr(), buf.data_ptr(), buf.numel() * 4, B, Hl, Wl,
                                            conv.in_channels, conv.out_channels, dg)
                return arr
            if mode in ("4", "5"):  # two tables: the direct splits first (enc1.conv1 needs its split next)
                def direct(j):
                    (conv, Hl, Wl, _), dg = j
                    return lib.pis_conv3x3_filter_format(B, Hl, Wl, conv.in_channels, conv.out_channels, dg) == 3
                self.filter_jobs_d = table([j for j in jobs if direct(j)])
                self.filter_jobs = table([j for j in jobs if not direct(j)])
            else:
                self.filter_jobs = table(jobs)

    def _filters_ahead(self, table, dgrad: int, order):
        """Launch the filter transforms of `table` on the side stream (after everything the main
        stream has enqueued: the weights are final), one event per layer."""
        main, side = torch.cuda.current_stream(), self.side
        side.wait_stream(main)
        events = {}
        with torch.cuda.stream(side):
            for cid in order:
                conv, Hl, Wl, buf = table[cid]
                call("pis_conv3x3_filter", conv.weight.data_ptr(), self.B, Hl, Wl, conv.in_channels,
                     conv.out_channels, dgrad, buf.data_ptr(), buf.numel() * 4, side.cuda_stream)
                ev = self._event()
                ev.record(side)
                events[cid] = ev
        return events

    def _filters_batched(self):
        """PIS_FILTER_AHEAD 4 / 5: every filter operand of the step — the direct layers' weight splits
        (one launch), then the Winograd layers' transforms, both directions (a second) — at the
        training forward's start. Mode 4 on the main stream (no events); mode 5 on the side stream,
        idle during the forward, with one event per launch that the first consumer of each kind
        waits for (every later consumer, forward or backward, follows it on the main stream)."""
        main = torch.cuda.current_stream()
        tables = [t for t in (self.filter_jobs_d, self.filter_jobs) if t is not None and len(t)]
        self.fev = dict.fromkeys(self.ffilt)
        self.bev = dict.fromkeys(self.bfilt)
        if self._fa_mode == "4" or self.side is None:  # (side None: the serialised A/B step)
            for t in tables:
                call("pis_conv3x3_filters", ctypes.addressof(t), len(t), main.cuda_stream)
            self._convt_prep(main.cuda_stream)
            return
        side = self.side
        side.wait_stream(main)  # the weights are final (the previous step's optimizer)
        with torch.cuda.stream(side):
            for i, t in enumerate(tables):
                call("pis_conv3x3_filters", ctypes.addressof(t), len(t), side.cuda_stream)
                if i + 1 == len(tables):  # ... and the transposed convs' input-gradient weights
                    self._convt_prep(side.cuda_stream)
                ev = self._event()
                ev.record(side)
                first = next((cid for cid in self.ffilt if any(j.w == self.ffilt[cid][0].weight.data_ptr() and
                                                                 j.dgrad == 0 for j in t)), None)
                if first is None:  # no forward consumer in this table: order the main stream now
                    main.wait_event(ev)
                else:
                    self.fev[first] = ev

    def _convt_prep(self, stream):
        """The four transposed convs' input-gradient weight layouts (pis_convt2x2_prep) for the
        coming backward, which then skips them (``convt_ready``)."""
        for l in (1, 2, 3, 4):
            up = getattr(self.m, f"up{l}")
            t = self._gbuf(f"prep_up{l}", up.weight.numel())
            call("pis_convt2x2_prep", up.weight.data_ptr(), t.data_ptr(), up.in_channels, up.out_channels, stream)
        self.convt_ready = True

    def _event(self) -> torch.cuda.Event:
        ev = torch.cuda.Event()
        if torch.cuda.is_current_stream_capturing():
            self.capture_events.append(ev)
        return ev

    def _gbuf(self, name: str, *shape) -> torch.Tensor:
        t = self.gbufs.get(name)
        if t is None:
            t = torch.empty(*shape, dtype=torch.float32, device=self.m.arena.device)
            self.gbufs[name] = t
        return t

    # ---- dropout ------------------------------------------------------------
    def dropout_scales(self, B: int, training: bool, override) -> Dict[str, Optional[torch.Tensor]]:
        """Per-block (B, C) keep-scales. Drawn like ATen's feature_dropout
        (noise.bernoulli_(1-p).div_(1-p), one draw per block in forward order)."""
        out: Dict[str, Optional[torch.Tensor]] = {}
        for name in BLOCK_ORDER:
            blk = self.m.block(name)
            if not training or blk.p <= 0:
                out[name] = None
                continue
            if override is not None and name in override:
                s = override[name].to(device=self.m.arena.device, dtype=torch.float32).contiguous()
            elif blk.p >= 1.0:
                s = torch.zeros(B, blk.conv0.out_channels, device=self.m.arena.device)
            else:
                s = torch.empty(B, blk.conv0.out_channels, device=self.m.arena.device)
                s.bernoulli_(1.0 - blk.p).div_(1.0 - blk.p)
            out[name] = s
        return out

    # ---- kernel helpers ------------------------------------------------------
    def _stream(self):
        return torch.cuda.current_stream().cuda_stream

    def _conv_fwd(self, conv: nn.Conv2d, x: _Buf, y: _Buf, B, H, W, scale, pool: Optional[torch.Tensor] = None):
        flags = PIS_RELU | (PIS_SCALE if scale is not None else 0)
        keep = self.keep.get(id(conv)) if self._keeping else None
        wptr = conv.weight.data_ptr()
        if id(conv) in self.fev:  # its filter transform (or direct split), computed ahead
            ev = self.fev.pop(id(conv))
            if ev is not None:
                torch.cuda.current_stream().wait_event(ev)
            wptr, flags = self.ffilt[id(conv)][3].data_ptr(), flags | PIS_FILTER_READY
        if pool is not None:  # encoder conv1 + MaxPool2d in one call (pooled in the output epilogue)
            call("pis_conv3x3_fwd_pool", x.p, x.ld, wptr, conv.bias.data_ptr(), ptr(scale),
                 y.p, y.ld, B, H, W, conv.in_channels, conv.out_channels, flags, self.ws.data_ptr(), self.ws_bytes,
                 ptr(keep), pool.data_ptr(), self._stream())
            return
        call("pis_conv3x3_fwd_keep", x.p, x.ld, wptr, conv.bias.data_ptr(), ptr(scale),
             y.p, y.ld, B, H, W, conv.in_channels, conv.out_channels, flags, self.ws.data_ptr(), self.ws_bytes,
             ptr(keep), self._stream())

    def _grad_slot(self, p: torch.Tensor) -> Tuple[int, int]:
        return self._offsets[id(p)]

    def _gptr(self, p: torch.Tensor) -> int:
        o, _ = self._offsets[id(p)]
        return self.garena.data_ptr() + 4 * o

    def _ready(self, *params):
        hook = self.m.grad_ready_hook
        if hook is None:
            return
        lo = min(self._offsets[id(p)][0] for p in params)
        hi = max(self._offsets[id(p)][0] + self._offsets[id(p)][1] for p in params)
        hook.on_ready(lo, hi)

    # ---- forward -------------------------------------------------------------
    @torch.no_grad()
    def forward(self, x: torch.Tensor, scales: Dict[str, Optional[torch.Tensor]], keep: bool) -> torch.Tensor:
        m, c = self.m, self.c
        B, _, H, W = x.shape
        self._plan(B, H, W, x.device)
        x = x.contiguous()
        bf = self.bufs
        self._keeping = keep  # only a forward the backward will use may overwrite the kept transforms
        # the side stream is idle during the forward: it transforms every filter of the step there,
        # the forward's in layer order, then the input gradients' (backward order)
        self.fev, self.bev = {}, {}
        self.convt_ready = False
        if keep and self.filter_jobs_d is not None:  # modes 4 / 5: all of them, in two launches
            self._filters_batched()
        elif keep and self.filter_jobs is not None:  # one launch, same stream: no events
            call("pis_conv3x3_filters", ctypes.addressof(self.filter_jobs), len(self.filter_jobs), self._stream())
            self.fev = dict.fromkeys(self.ffilt)
            self.bev = dict.fromkeys(self.bfilt)
        elif keep and self.side is not None:
            if self.ffilt:
                self.fev = self._filters_ahead(self.ffilt, 0, list(self.ffilt))
            if self.bfilt:
                self.bev = self._filters_ahead(self.bfilt, 1, list(reversed(list(self.bfilt))))
        self.x = x
        self.scales = scales
        src = _Buf(x, m.in_channels)
        for l in range(1, 5):
            Hl, Wl, Cl = H >> (l - 1), W >> (l - 1), c << (l - 1)
            blk = m.block(f"enc{l}")
            a = _Buf(bf[f"a{l}"], Cl)
            e = _Buf(bf[f"cat{l}"], 2 * Cl, Cl)         # enc output lives in the concat buffer
            self._conv_fwd(blk.conv0, src, a, B, Hl, Wl, scales[f"enc{l}"])
            self._conv_fwd(blk.conv1, a, e, B, Hl, Wl, None, pool=bf[f"pool{l}"])
            src = _Buf(bf[f"pool{l}"], Cl)
        H5, W5 = H >> 4, W >> 4
        blk = m.bottleneck
        self._conv_fwd(blk.conv0, src, _Buf(bf["b0"], 8 * c), B, H5, W5, scales["bottleneck"])
        self._conv_fwd(blk.conv1, _Buf(bf["b0"], 8 * c), _Buf(bf["b1"], 8 * c), B, H5, W5, None)
        d = _Buf(bf["b1"], 8 * c)
        dC = 8 * c
        for l in (4, 3, 2, 1):
            Hl, Wl, Cl = H >> (l - 1), W >> (l - 1), c << (l - 1)
            up = getattr(m, f"up{l}")
            cat = _Buf(bf[f"cat{l}"], 2 * Cl)
            call("pis_convt2x2_fwd", d.p, d.ld, up.weight.data_ptr(), up.bias.data_ptr(), cat.p, cat.ld,
                 B, Hl // 2, Wl // 2, dC, Cl, self._stream())
            blk = m.block(f"dec{l}")
            d0 = _Buf(bf[f"d0_{l}"], Cl)
            d1 = _Buf(bf[f"d1_{l}"], Cl)
            self._conv_fwd(blk.conv0, cat, d0, B, Hl, Wl, scales[f"dec{l}"])
            self._conv_fwd(blk.conv1, d0, d1, B, Hl, Wl, None)
            d, dC = d1, Cl
        u = bf["u"] if keep else torch.empty(B, 1, H, W, device=x.device)
        z = bf["z"]
        lr, self.loss_request = self.loss_request, None
        lib = _hip.lib()
        if lr is not None and lib.pis_head_loss_fwd_ok(B, H, W, c) and d.ld % 4 == 0:
            # the head + the loss forward in one pass over the head input (forward_with_loss)
            t, prm, sink = lr
            dev = x.device
            terms = torch.empty(_hip.LOSS_NTERMS, dtype=torch.float32, device=dev)
            counts = torch.empty(B, 3, dtype=torch.int32, device=dev)
            scores = torch.empty(B, 2, dtype=torch.float32, device=dev)
            call("pis_head_loss_fwd", d.p, d.ld, m.out_conv.weight.data_ptr(), m.out_conv.bias.data_ptr(),
                 t.data_ptr(), z.data_ptr(), u.data_ptr(), B, H, W, c, ctypes.byref(prm), terms.data_ptr(),
                 counts.data_ptr(), scores.data_ptr(), self.hl_ws.data_ptr(), self.hl_ws.numel() * 4, self._stream())
            sink["terms"], sink["counts"], sink["scores"] = terms, counts, scores
        else:
            call("pis_head_fwd", d.p, d.ld, m.out_conv.weight.data_ptr(), m.out_conv.bias.data_ptr(), z.data_ptr(),
                 u.data_ptr(), B * H * W, c, self._stream())
        m.last_logits = z
        # every forward overwrites the engine's activation buffers: a graph built before it
        # can no longer be backpropagated (its backward raises instead of reading stale data)
        self.generation += 1
        if keep:
            self.u = u
        return u

    # ---- loss backward fused into the head backward ---------------------------
    def can_fuse_loss(self, u: torch.Tensor, generation: int) -> bool:
        return (generation == self.generation and self.pending_head is None and self.W <= 1024
                and u.data_ptr() == self.u.data_ptr())

    @torch.no_grad()
    def fuse_loss_backward(self, t: torch.Tensor, prm, terms: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
        """Run the loss backward and the head backward as one kernel (pis_head_loss_bwd)
        from inside the loss's autograd backward. Returns dL/du (written too, so any
        other consumer of u sees the exact gradient); the U-Net backward recognises
        that tensor and skips its own head step (only the head's dW/db still go into
        the gradient arena, in the arena's accumulate/overwrite mode)."""
        m, c = self.m, self.c
        B, H, W = self.B, self.H, self.W
        st = self._stream()
        d1 = _Buf(self.bufs["d1_1"], c)
        g_d1 = _Buf(self._gbuf("g_d1_1", B, H, W, c), c)
        self.head_scratch = self._gbuf("head_scratch", c + 1)
        hs = self.head_scratch.data_ptr()
        du = torch.empty_like(self.u)
        call("pis_head_loss_bwd", d1.p, d1.ld, m.out_conv.weight.data_ptr(), self.u.data_ptr(), t.data_ptr(),
             du.data_ptr(), B, H, W, c, prm, terms.data_ptr(), g.data_ptr(), g_d1.p, g_d1.ld, hs, hs + 4 * c, 0,
             self.ws.data_ptr(), self.ws_bytes, st)
        self.pending_head = du
        return du

    # ---- backward ------------------------------------------------------------
    def _grad_mode(self) -> str:
        """'overwrite' when every .grad is None (zero_grad(set_to_none=True)),
        'accumulate' when every .grad already views the gradient arena."""
        params = [mod._parameters[pn] for mod, pn, *_ in self.m._entries]
        if all(p.grad is None for p in params):
            return "overwrite"
        g = self.m.grad_arena()
        lo, hi = g.data_ptr(), g.data_ptr() + 4 * g.numel()
        if all(p.grad is not None and lo <= p.grad.data_ptr() < hi for p in params):
            return "accumulate"
        return "scratch"

    @torch.no_grad()
    def backward(self, du: torch.Tensor) -> List[Optional[torch.Tensor]]:
        m, c = self.m, self.c
        B, H, W = self.B, self.H, self.W
        bf = self.bufs
        mode = self._grad_mode()
        self.last_grad_mode = mode
        if mode == "scratch":
            self.garena = torch.zeros_like(m.arena)
        else:
            self.garena = m.grad_arena()
        acc = PIS_ACCUMULATE if mode == "accumulate" else 0
        st = self._stream()
        ws, wsb = self.ws.data_ptr(), self.ws_bytes
        ws2 = self.ws2.data_ptr()
        main = torch.cuda.current_stream()
        side = self.side if self.side is not None else main
        sst = side.cuda_stream
        if side is not main:
            side.wait_stream(main)  # forward activations, kept transforms, a zeroed scratch arena
        # the previous backward ended with main.wait_stream(side): every earlier use of the
        # alternating weight-gradient workspaces is ordered before this point already (and a
        # graph capture must not wait on events recorded outside it)
        self.ws3_free = [None, None]
        if side is main and self.filter_jobs is None:
            self.bev = {}  # serialised A/B mode: each dgrad transforms its own filter
        gb = self._gbuf

        def to_side():
            """Order the side stream after everything enqueued on the main stream so far."""
            if side is not main:
                ev = self._event()
                ev.record(main)
                side.wait_event(ev)

        def ready_on_side(*params):
            with torch.cuda.stream(side):  # DDP buckets all-reduce after their weight gradients
                self._ready(*params)

        # dgrad operands, rebuilt from the current weights. A 3x3 layer whose input gradient runs
        # on the prepared F(4x4,3x3) path reads its original weights (the filter transform rotates
        # them); the others get a flipped copy right before their dgrad.
        flips = {}

        def flipped(conv):
            t = gb(f"flip_{id(conv)}", conv.weight.numel())
            call("pis_conv3x3_flip", conv.weight.data_ptr(), t.data_ptr(), conv.in_channels,
                 conv.out_channels, st)
            return t

        for l in (1, 2, 3, 4):
            up = getattr(m, f"up{l}")
            t = gb(f"prep_up{l}", up.weight.numel())
            if not self.convt_ready:  # (else prepared with the filter operands at the forward's start)
                call("pis_convt2x2_prep", up.weight.data_ptr(), t.data_ptr(), up.in_channels, up.out_channels, st)
            flips[id(up)] = t
        self.convt_ready = False

        lib = _hip.lib()
        nprep = [0]
        enc_convs = {id(cv) for l in (1, 2, 3, 4) for cv in (m.block(f"enc{l}").conv0, m.block(f"enc{l}").conv1)}

        def conv_bwd(conv, x: _Buf, dz: _Buf, dx: Optional[_Buf], Hl, Wl, mask: Optional[_Buf], scale):
            kept = self.keep.get(id(conv))
            prep, wsw, wswb = 0, ws2, wsb
            if dx is not None and kept is not None:
                # one pass over dz for both backward products (main stream): V into the dgrad
                # workspace, E + bias partials into an alternating weight-gradient workspace
                j = nprep[0] & 1
                if self.ws3_free[j] is not None:
                    main.wait_event(self.ws3_free[j])
                prep = lib.pis_conv3x3_bwd_prep(dz.p, dz.ld, B, Hl, Wl, conv.in_channels, conv.out_channels, ws, wsb,
                                                self.ws3[j].data_ptr(), self.ws3_bytes, st)
                if prep < 0:
                    raise RuntimeError(lib.pis_last_error().decode())
                if prep:
                    nprep[0] += 1
                    wsw, wswb = self.ws3[j].data_ptr(), self.ws3_bytes
            def wgrad():
                call("pis_conv3x3_wgrad_keep", x.p, x.ld, dz.p, dz.ld, self._gptr(conv.weight),
                     self._gptr(conv.bias), B, Hl, Wl, conv.in_channels, conv.out_channels,
                     acc | (PIS_WINO_PREPARED if prep else 0), wsw, wswb, ptr(kept), sst)
                if prep and side is not main:
                    ev = self._event()
                    ev.record(side)
                    self.ws3_free[(nprep[0] - 1) & 1] = ev
                ready_on_side(conv.weight, conv.bias)

            def dgrad():
                flags = (PIS_MASK if mask is not None else 0) | (PIS_SCALE if scale is not None else 0)
                if prep:
                    wf, flags = conv.weight.data_ptr(), flags | PIS_WINO_PREPARED | PIS_W_UNFLIPPED
                    if id(conv) in self.bev:  # its rotated filter transform, computed ahead
                        ev = self.bev.pop(id(conv))
                        if ev is not None:
                            main.wait_event(ev)
                        wf, flags = self.bfilt[id(conv)][3].data_ptr(), flags | PIS_FILTER_READY
                elif lib.pis_conv3x3_dgrad_direct(B, Hl, Wl, conv.in_channels, conv.out_channels, dz.ld, wsb):
                    wf, flags = conv.weight.data_ptr(), flags | PIS_W_UNFLIPPED  # the direct kernel splits it
                    if id(conv) in self.bev:  # ... unless its split was computed ahead
                        ev = self.bev.pop(id(conv))
                        if ev is not None:
                            main.wait_event(ev)
                        wf, flags = self.bfilt[id(conv)][3].data_ptr(), flags | PIS_FILTER_READY
                elif id(conv) in self.bev and lib.pis_conv3x3_filter_format(
                        B, Hl, Wl, conv.in_channels, conv.out_channels, 1) == 4:
                    # F(6x6,3x3) input gradient: its transform of the ORIGINAL weights, computed ahead
                    ev = self.bev.pop(id(conv))
                    if ev is not None:
                        main.wait_event(ev)
                    wf, flags = self.bfilt[id(conv)][3].data_ptr(), flags | PIS_W_UNFLIPPED | PIS_FILTER_READY
                else:
                    wf = flipped(conv).data_ptr()
                call("pis_conv3x3_dgrad_ex", dz.p, dz.ld, wf,
                     mask.p if mask is not None else 0, mask.ld if mask is not None else 0, ptr(scale),
                     dx.p, dx.ld, B, Hl, Wl, conv.in_channels, conv.out_channels, flags, ws, wsb, st)

            if (self.fused_wgrad_main == "1" and prep and dx is not None and side is not main
                    and lib.pis_conv3x3_filter_format(B, Hl, Wl, conv.in_channels, conv.out_channels, 1) == 2):
                dgrad()
                call("pis_conv3x3_wgrad_keep", x.p, x.ld, dz.p, dz.ld, self._gptr(conv.weight),
                     self._gptr(conv.bias), B, Hl, Wl, conv.in_channels, conv.out_channels,
                     acc | PIS_WINO_PREPARED, wsw, wswb, ptr(kept), st)
                self.ws3_free[(nprep[0] - 1) & 1] = None  # written and read on the main stream
                if m.grad_ready_hook is not None:
                    to_side()
                    ready_on_side(conv.weight, conv.bias)
                return
            sync = self.side_sync if (prep and dx is not None and side is not main) else "prep"
            on_main = self.direct_wgrad_main == "1" or (self.direct_wgrad_main == "dec" and id(conv) not in enc_convs)
            if (on_main and not prep and dx is not None and side is not main
                    and lib.pis_conv3x3_dgrad_direct(B, Hl, Wl, conv.in_channels, conv.out_channels, dz.ld, wsb)
                    and lib.pis_conv3x3_wgrad_ws(B, Hl, Wl, conv.in_channels, conv.out_channels) <= wsb):
                # a direct layer's weight gradient on the main stream right after its input gradient,
                # in the main workspace: the two MFMA-bound kernels in sequence instead of the weight
                # gradient's one-wave-per-SIMD blocks (497 registers per lane) locking every CU under
                # the main stream's work. Step-neutral (22.37 vs 22.38 ms, profiles/r5_c_*), but each
                # direct kernel then runs at its own rate: the weight gradient 0.23 -> 0.41 of the
                # fp16x3 pipe live, the input gradient 0.35 -> 0.44, the convT input gradients 2.07 ->
                # 1.41 ms per step
                dgrad()
                call("pis_conv3x3_wgrad_keep", x.p, x.ld, dz.p, dz.ld, self._gptr(conv.weight),
                     self._gptr(conv.bias), B, Hl, Wl, conv.in_channels, conv.out_channels, acc, ws, wsb, 0, st)
                if m.grad_ready_hook is not None:  # DDP: the bucket's all-reduce runs from the side
                    to_side()                      # stream, which now waits for this weight gradient
                    ready_on_side(conv.weight, conv.bias)
                return
            if sync == "prep":  # the weight gradient starts as soon as dz's transforms exist
                to_side()
                wgrad()
                if dx is not None:
                    dgrad()
                return
            # the weight gradient (MFMA-bound) starts after the input gradient's contractions
            # ("gemm": overlapping the HBM-bound output transform) or after the whole input
            # gradient ("dgrad"); it only needs dz's transforms, which precede either point
            ev = self._event()
            ev.record(main)
            if sync == "gemm":
                lib.pis_arm_gemm_event(ev.cuda_event)
            dgrad()
            if sync != "gemm" or lib.pis_arm_gemm_event(None):
                ev.record(main)
            side.wait_event(ev)
            wgrad()

        # head: sigmoid backward + 1x1 conv + ReLU backward of dec1.conv1
        d1 = _Buf(bf["d1_1"], c)
        g_d1 = _Buf(gb("g_d1_1", B, H, W, c), c)
        fused, self.pending_head = self.pending_head, None
        if fused is not None and du.data_ptr() == fused.data_ptr():
            # the loss backward already ran the head backward (pis_head_loss_bwd): g_d1 is
            # written and the head's dW/db wait in the scratch; only their arena update is left —
            # weight-gradient work, so on the side stream in its workspace, off the critical path
            hs = self.head_scratch
            to_side()
            hws = ws2 if side is not main else ws
            call("pis_colsum", hs.data_ptr(), c, 1, c, self._gptr(m.out_conv.weight), acc, hws, wsb, sst)
            call("pis_colsum", hs.data_ptr() + 4 * c, 1, 1, 1, self._gptr(m.out_conv.bias), acc, hws, wsb, sst)
            ready_on_side(m.out_conv.weight, m.out_conv.bias)
        else:
            du = du.contiguous()
            call("pis_head_bwd", d1.p, d1.ld, m.out_conv.weight.data_ptr(), du.data_ptr(), self.u.data_ptr(),
                 g_d1.p, g_d1.ld, self._gptr(m.out_conv.weight), self._gptr(m.out_conv.bias), B * H * W, c, acc,
                 ws, wsb, st)
            self._ready(m.out_conv.weight, m.out_conv.bias)

        g_top = g_d1  # dz of dec_l.conv1
        for l in (1, 2, 3, 4):
            Hl, Wl, Cl = H >> (l - 1), W >> (l - 1), c << (l - 1)
            blk = m.block(f"dec{l}")
            d0 = _Buf(bf[f"d0_{l}"], Cl)
            cat = _Buf(bf[f"cat{l}"], 2 * Cl)
            g_d0 = _Buf(gb(f"g_d0_{l}", B, Hl, Wl, Cl), Cl)
            conv_bwd(blk.conv1, d0, g_top, g_d0, Hl, Wl, d0, self.scales[f"dec{l}"])
            g_cat = _Buf(gb(f"g_cat{l}", B, Hl, Wl, 2 * Cl), 2 * Cl)
            conv_bwd(blk.conv0, cat, g_d0, g_cat, Hl, Wl, None, None)
            # transposed conv up_l: its input is dec_{l+1} conv1 output (or bottleneck conv1)
            up = getattr(m, f"up{l}")
            if l == 4:
                xin = _Buf(bf["b1"], 8 * c)
            else:
                xin = _Buf(bf[f"d1_{l + 1}"], up.in_channels)
            Hh, Wh = Hl // 2, Wl // 2
            g_in = _Buf(gb(f"g_upin{l}", B, Hh, Wh, up.in_channels), up.in_channels)
            if str(l) in self.convt_wgrad_main and side is not main:
                call("pis_convt2x2_dgrad", g_cat.p, g_cat.ld, flips[id(up)].data_ptr(), xin.p, xin.ld, g_in.p,
                     g_in.ld, B, Hh, Wh, up.in_channels, up.out_channels, PIS_MASK, st)
                call("pis_convt2x2_wgrad", xin.p, xin.ld, g_cat.p, g_cat.ld, self._gptr(up.weight),
                     self._gptr(up.bias), B, Hh, Wh, up.in_channels, up.out_channels, acc, ws, wsb, st)
                if m.grad_ready_hook is not None:
                    to_side()
                    ready_on_side(up.weight, up.bias)
                g_top = g_in
                continue
            to_side()
            call("pis_convt2x2_wgrad", xin.p, xin.ld, g_cat.p, g_cat.ld, self._gptr(up.weight), self._gptr(up.bias),
                 B, Hh, Wh, up.in_channels, up.out_channels, acc, ws2, wsb, sst)
            ready_on_side(up.weight, up.bias)
            call("pis_convt2x2_dgrad", g_cat.p, g_cat.ld, flips[id(up)].data_ptr(), xin.p, xin.ld, g_in.p, g_in.ld,
                 B, Hh, Wh, up.in_channels, up.out_channels, PIS_MASK, st)
            g_top = g_in
        # bottleneck
        H5, W5 = H >> 4, W >> 4
        blk = m.bottleneck
        b0 = _Buf(bf["b0"], 8 * c)
        g_b0 = _Buf(gb("g_b0", B, H5, W5, 8 * c), 8 * c)
        conv_bwd(blk.conv1, b0, g_top, g_b0, H5, W5, b0, self.scales["bottleneck"])
        g_pool = _Buf(gb("g_pool4", B, H5, W5, 8 * c), 8 * c)
        conv_bwd(blk.conv0, _Buf(bf["pool4"], 8 * c), g_b0, g_pool, H5, W5, None, None)
        # encoder, deepest first
        for l in (4, 3, 2, 1):
            Hl, Wl, Cl = H >> (l - 1), W >> (l - 1), c << (l - 1)
            blk = m.block(f"enc{l}")
            e = _Buf(bf[f"cat{l}"], 2 * Cl, Cl)
            g_skip = _Buf(self.gbufs[f"g_cat{l}"], 2 * Cl, Cl)
            g_e = _Buf(gb(f"g_e{l}", B, Hl, Wl, Cl), Cl)
            call("pis_maxpool2x2_bwd", e.p, e.ld, g_pool.p, g_skip.p, g_skip.ld, g_e.p, g_e.ld, B, Hl, Wl, Cl, st)
            a = _Buf(bf[f"a{l}"], Cl)
            g_a = _Buf(gb(f"g_a{l}", B, Hl, Wl, Cl), Cl)
            conv_bwd(blk.conv1, a, g_e, g_a, Hl, Wl, a, self.scales[f"enc{l}"])
            if l > 1:
                g_pool = _Buf(gb(f"g_pool{l - 1}", B, Hl, Wl, Cl // 2), Cl // 2)
                conv_bwd(blk.conv0, _Buf(bf[f"pool{l - 1}"], Cl // 2), g_a, g_pool, Hl, Wl, None, None)
            elif (side is not main and m.grad_ready_hook is None and self.keep.get(id(blk.conv0)) is None
                  and lib.pis_tune(_hip.PIS_TUNE_LAST_WGRAD_MAIN, -1) != 0
                  and lib.pis_conv3x3_wgrad_ws(B, Hl, Wl, m.in_channels, blk.conv0.out_channels) <= wsb):
                # the step's last weight gradient (enc1.conv0, input channels = the image's): its dz
                # is the main stream's last product and the main stream is idle after it, while the
                # side stream still runs enc1.conv1's weight gradient — so it runs here, in the
                # main stream's workspace (free after enc1.conv1's input gradient), beside that tail
                conv = blk.conv0
                call("pis_conv3x3_wgrad_keep", self.x.data_ptr(), m.in_channels, g_a.p, g_a.ld,
                     self._gptr(conv.weight), self._gptr(conv.bias), B, Hl, Wl, m.in_channels, conv.out_channels,
                     acc, ws, wsb, 0, st)
            else:
                conv_bwd(blk.conv0, _Buf(self.x, m.in_channels), g_a, None, Hl, Wl, None, None)

        if m.grad_ready_hook is not None:
            if mode == "scratch":
                raise RuntimeError("data-parallel gradients need zero_grad() before every backward")
            mark = getattr(m.grad_ready_hook, "mark_backward_done", None)
            if mark is not None:
                mark(main, side)
            with torch.cuda.stream(side):
                m.grad_ready_hook.finish()
        if side is not main:
            main.wait_stream(side)  # the optimizer (and the next forward) see every weight gradient
        if mode == "accumulate":
            return [None] * len(m._entries)
        g = self.garena
        return [_phys_view(g[o:o + n], shape, kind) for _, _, shape, kind, o, n in m._entries]
