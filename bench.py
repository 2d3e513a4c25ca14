"""Benchmark: training images/sec of the PDE-constrained U-Net step on MI355X.

Workload (BASELINE.json configs[1], "C2"): UNet(1,1,64), batch 8 per GPU,
512x512 synthetic disc masks, Stage-II loss
(0.5 Dice + 0.5 BCE + 1e-4 RD(D=5, a=0.5) + 1e-4 PF(eps=0.05)), AdamW
lr=1e-5 (Stage II = 0.1 x 1e-4), wd=1e-5, train mode with Dropout2d.
A step = zero_grad -> forward -> fused loss -> backward (+ RCCL bucketed
all-reduce when N > 1) -> AdamW, inputs already resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...       (one rank per GPU)

With ``--gpus N > 1`` and no torchrun environment (WORLD_SIZE unset), bench.py is
its own launcher: before anything touches the GPU it starts N child processes of
itself with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT
set (one rank per GPU, RCCL), waits for them and exits with the first non-zero
child status. Every rank checks WORLD_SIZE == --gpus and fails otherwise.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import time

import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from physics_informed_image_segmentation_amd import AdamW, DiceBCEPDELoss, UNet  # noqa: E402
from physics_informed_image_segmentation_amd.dataset import disc_sample  # noqa: E402
from physics_informed_image_segmentation_amd.distributed import (GradBucketer, broadcast_parameters,  # noqa: E402
                                                                 env_world, init_from_env)

B, H, W = 8, 512, 512
LOSS_KW = dict(pde_weight=1e-4, phase_field_weight=1e-4, diffusion_coeff=5.0, reaction_threshold=0.5, epsilon=0.05)
LR = 1e-5
# --config: C2 is the headline (BASELINE.json configs[1]); the others are BASELINE's C4 ablation
# variants at C2 size (run_ablation.py R1, the fused loss kernel specialised per gating) and
# C5's per-rank shape (S2 sweep: 1024^2, lambda_RD = 1e-3, no phase field; D does not change the work)
CONFIGS = {
    "c2": (512, dict(LOSS_KW), "C2: UNet(1,1,64) bs=8/GPU 512x512 Stage-II (lambda_RD=lambda_PF=1e-4, D=5, a=0.5, "
                               "eps=0.05) AdamW lr=1e-5"),
    "c4-baseline": (512, dict(pde_weight=0.0, phase_field_weight=0.0), "C4 R1.0: bs=8 512x512, Dice+BCE only"),
    "c4-rd": (512, dict(pde_weight=1e-4, phase_field_weight=0.0, diffusion_coeff=5.0, reaction_threshold=0.5),
              "C4 R1.1: bs=8 512x512, RD only (lambda_RD=1e-4)"),
    "c4-pf": (512, dict(pde_weight=0.0, phase_field_weight=1e-4, epsilon=0.05),
              "C4 R1.2: bs=8 512x512, PF only (lambda_PF=1e-4)"),
    "c4-rdpf": (512, dict(LOSS_KW), "C4 R1.3: bs=8 512x512, RD+PF"),
    "c5": (1024, dict(pde_weight=1e-3, phase_field_weight=0.0, diffusion_coeff=5.0, reaction_threshold=0.5),
           "C5 (per rank): bs=8 1024x1024, S2 RD only (lambda_RD=1e-3, D=5)"),
}


def conv_flops_per_image(H: int, W: int, c: int = 64) -> float:
    """Algorithmic FLOPs of one training image: 2 x MACs x 3
    (fwd, dgrad, wgrad) over every conv / convT, minus the dgrad of enc1.conv0."""
    macs = 0.0
    first = 0.0
    for l in range(1, 5):
        hw = (H >> (l - 1)) * (W >> (l - 1))
        cl = c << (l - 1)
        cin0 = 1 if l == 1 else cl // 2
        m0 = hw * cl * cin0 * 9
        if l == 1:
            first = m0
        macs += m0 + hw * cl * cl * 9                    # enc conv0, conv1
        macs += hw * cl * 2 * cl * 9 + hw * cl * cl * 9  # dec conv0 (2C in), conv1
        cup = 8 * c if l == 4 else 2 * cl
        macs += (hw // 4) * cup * cl * 4                 # convT into level l
    hw5 = (H >> 4) * (W >> 4)
    macs += 2 * hw5 * (8 * c) * (8 * c) * 9              # bottleneck
    macs += H * W * c                                    # head 1x1
    return 2.0 * macs * 3 - 2.0 * first


def wino_gemm_launches(H: int, W: int, B: int, c: int = 64):
    """(T, C, N, planes) of every batched Winograd GEMM launch ("wino_gemm") of one training step: the
    forward and input gradient of each F(4x4,3x3) 3x3 conv (T = B H W / 16 tiles, contraction C,
    N outputs), in no particular order — the 64 / 128-channel contractions into <= 256 outputs run
    the fused contraction + output transform kernel instead (fused_wanted), and enc1.conv0 (Cin = 1) the VALU row kernels (csrc/winograd.hip
    wino_gemm_out_wanted, csrc/igemm.hip wino_wanted_dims)."""
    convs = []
    for l in range(1, 5):
        cl = c << (l - 1)
        hl, wl = H >> (l - 1), W >> (l - 1)
        if l > 1:
            convs.append((hl, wl, cl // 2, cl))          # enc conv0
        convs += [(hl, wl, cl, cl), (hl, wl, 2 * cl, cl), (hl, wl, cl, cl)]  # enc conv1, dec conv0, conv1
    convs += [(H >> 4, W >> 4, 8 * c, 8 * c)] * 2        # bottleneck
    out = []
    for hl, wl, ci, co in convs:
        T = B * (hl // 4) * (wl // 4)
        if wino6_layer(B, hl, wl, ci, co):  # F(6x6,3x3) both ways: 64 planes over the 6 x 6 tile grid
            T6 = B * ((hl + 5) // 6) * ((wl + 5) // 6)
            out += [(T6, ci, co, 64), (T6, co, ci, 64)]
            continue
        out += [(T, C, N, 36) for C, N in ((ci, co), (co, ci))
                if not direct_wanted(hl, wl, C, N) and not fused_wanted(T, C, N)]
    return out


def wino6_layer(B: int, H: int, W: int, Cin: int, Cout: int) -> bool:
    """csrc/igemm.hip wino6_layer (pis_tune key 47 as set now): the layers whose forward and input
    gradient run Winograd F(6x6,3x3)."""
    from physics_informed_image_segmentation_amd import _hip
    return _hip.lib().pis_conv3x3_filter_format(B, H, W, Cin, Cout, 0) == 4


def fused_launches(H: int, W: int, B: int, c: int = 64):
    """(T, C, N, dgrad) of every launch of the fused contraction + output transform
    ("wino_gemm_out") in one training step (the complement of wino_gemm_launches)."""
    convs = []
    for l in range(1, 5):
        cl = c << (l - 1)
        hl, wl = H >> (l - 1), W >> (l - 1)
        if l > 1:
            convs.append((hl, wl, cl // 2, cl))
        convs += [(hl, wl, cl, cl), (hl, wl, 2 * cl, cl), (hl, wl, cl, cl)]
    convs += [(H >> 4, W >> 4, 8 * c, 8 * c)] * 2
    out = []
    for hl, wl, ci, co in convs:
        T = B * (hl // 4) * (wl // 4)
        out += [(T, C, N, dg) for C, N, dg in ((ci, co, 0), (co, ci, 1))
                if not direct_wanted(hl, wl, C, N) and fused_wanted(T, C, N)]
    return out


def fused_bytes(T: int, C: int, N: int, dgrad: int) -> float:
    """Algorithmic HBM bytes of one fused launch: V read (36 fp32 planes of C channels per tile),
    the filter planes read once (fp16x3: 4 B per element), the 4x4 output tile written (16 pixels
    x N fp32 per tile) and, for an input gradient, the ReLU mask of its input read; the pooled
    copy, keep-scales and accumulation reads are not counted."""
    return 4.0 * (36 * T * C + 36 * N * C + 16 * T * N * (2 if dgrad else 1))


# the configuration the committed PMC counters (profiles/pmc_dominant.json) were collected on:
# another --config reports its PMC fields as null instead of these
PMC_CONFIG = "c2"
PMC_NOTE = ("PMC counters (HBM traffic, MFMA busy) are collected on C2 only (profiles/pmc_dominant.json); "
            "null for this config rather than C2's figures")


def pmc_bytes(substr, config=PMC_CONFIG):
    """Launch-weighted HBM bytes per launch of the kernels whose name contains substr (or any of
    a list of substrings), from the committed rocprofv3 --pmc summary (profiles/pmc_dominant.json),
    or None (also for a config the summary was not collected on)."""
    path = os.path.join(HERE, "profiles", "pmc_dominant.json")
    if config != PMC_CONFIG or not os.path.exists(path):
        return None
    with open(path) as f:
        ks = json.load(f).get("kernels", {})
    subs = [substr] if isinstance(substr, str) else list(substr)
    sel = [(v["hbm_bytes_per_launch"], v["launches"]) for k, v in ks.items()
           if any(x in k for x in subs) and "hbm_bytes_per_launch" in v]
    n = sum(c for _, c in sel)
    return sum(b * c for b, c in sel) / n if n else None


def direct_layers(H: int, W: int, c: int = 64):
    """(name, h, w, Cin, Cout, pooled forward, masked input gradient, has an input gradient) of the
    3x3 convs the direct fp16x3 kernels take (csrc/direct.hip direct_h3_wanted, pis_tune key 29 as
    set now); the engine's schedule (unet.py): encoder conv1 forwards are pooled, the input
    gradients of conv1 layers carry the ReLU mask of their input, conv0 ones do not."""
    from physics_informed_image_segmentation_amd import _hip
    mode = _hip.lib().pis_tune(29, -1)

    def wanted(h, w, ci, co):
        if mode == 0 or ci < 16 or h % 8 or w % 32 or ci % 16 or co % 64:
            return False
        lo, hi = min(ci, co), max(ci, co)
        if mode == 3:
            return (h >= 256 and hi <= 256) or (h >= 128 and hi <= 256 and lo <= 128)
        if mode == 4:
            return h >= 128 and hi <= 256
        if mode == 5:
            return h >= 128
        return mode == 2 or (hi <= 128 and h >= 256)

    convs = []
    for l in range(1, 5):
        cl, hl, wl = c << (l - 1), H >> (l - 1), W >> (l - 1)
        cin0 = 1 if l == 1 else cl // 2
        convs += [(f"enc{l}.conv0", hl, wl, cin0, cl, False, False, l > 1),
                  (f"enc{l}.conv1", hl, wl, cl, cl, True, True, True),
                  (f"dec{l}.conv0", hl, wl, 2 * cl, cl, False, False, True),
                  (f"dec{l}.conv1", hl, wl, cl, cl, False, True, True)]
    convs += [("bottleneck.conv0", H >> 4, W >> 4, 8 * c, 8 * c, False, False, True),
              ("bottleneck.conv1", H >> 4, W >> 4, 8 * c, 8 * c, False, True, True)]
    return [cv for cv in convs if wanted(cv[1], cv[2], cv[3], cv[4])]


def direct_role_launches(H: int, W: int, B: int):
    """{hook label: [(FLOP, algorithmic HBM bytes)] per launch} of the direct kernels in one step.
    Bytes: forward x read + y written (+ the pooled copy); input gradient dz read + dx written
    (+ the ReLU mask of the conv's input); weight gradient x + dz read + dW written once (the
    split-K slabs are implementation traffic, visible in the PMC figure, not algorithmic)."""
    out = {"direct_h3_fwd": [], "direct_h3_pool": [], "direct_h3_dgrad": [], "direct_wgrad_h3": []}
    for _, h, w, ci, co, pool, mask, dg in direct_layers(H, W):
        P = B * h * w
        fl = 2.0 * 9 * P * ci * co
        out["direct_h3_pool" if pool else "direct_h3_fwd"].append(
            (fl, 4.0 * P * (ci + co) + (4.0 * P / 4 * co if pool else 0.0)))
        if dg:
            out["direct_h3_dgrad"].append((fl, 4.0 * P * (co + ci) + (4.0 * P * ci if mask else 0.0)))
        out["direct_wgrad_h3"].append((fl, 4.0 * P * (ci + co) + 4.0 * 9 * ci * co))
    return out


def direct_wanted(H: int, W: int, C: int, N: int) -> bool:
    """csrc/direct.hip direct_h3_wanted (pis_tune key 29 as set now): the 3x3 convs (both
    directions) that run the direct fp16x3 kernels instead of a Winograd pipeline."""
    from physics_informed_image_segmentation_amd import _hip
    mode = _hip.lib().pis_tune(29, -1)
    if mode == 0 or H % 8 or W % 32 or C % 16 or N % 64 or C < 16:
        return False
    lo, hi = min(C, N), max(C, N)
    if mode == 3:
        return (H >= 256 and hi <= 256) or (H >= 128 and hi <= 256 and lo <= 128)
    if mode == 4:
        return H >= 128 and hi <= 256
    if mode == 5:
        return H >= 128
    return mode == 2 or (hi <= 128 and H >= 256)


def fused_wanted(T: int, C: int, N: int) -> bool:
    """csrc/winograd.hip wino_gemm_out_wanted: the launches the fused contraction + output
    transform takes instead of the batched GEMM (pis_tune keys 10, 15, 26, 27 as set now)."""
    from physics_informed_image_segmentation_amd import _hip
    tune = _hip.lib().pis_tune
    if tune(15, -1) == 0 or tune(10, -1) < 3 or T % 32 or T < 2 * C:
        return False
    return (C == 64 or (C == 128 and tune(27, -1) != 0)) and (N == 64 or (N % 64 == 0 and N <= 64 << tune(26, -1)))


def gemm_attainable(launches, pipe_peak_tflops: float, hbm_gbs: float = 8000.0):
    """Per launch the roofline time max(FLOP / pipe peak, algorithmic bytes / HBM peak), the
    algorithmic bytes being V read + U read + M written once (36 fp32 planes each). Returns
    (FLOP, bytes, roofline seconds, FLOP-only seconds, bytes-only seconds), summed."""
    fl = by = tmin = tf = tb = 0.0
    for T, C, N, nxi in launches:
        f, b = 2.0 * nxi * T * C * N, 4.0 * nxi * (T * C + N * C + T * N)
        fl, by = fl + f, by + b
        tf, tb = tf + f / (pipe_peak_tflops * 1e12), tb + b / (hbm_gbs * 1e9)
        tmin += max(f / (pipe_peak_tflops * 1e12), b / (hbm_gbs * 1e9))
    return fl, by, tmin, tf, tb


# The dominant kernel of the step (profiles/r1_*_kernel_stats.csv): the batched fp32 MFMA GEMM
# of the Winograd 3x3 convs (forward + input gradient), launched as "wino_gemm" by the C-ABI
# (csrc/winograd.hip) and named gemm_nt_kernel<128, 128> / <128, 64> by rocprofv3.
DOMINANT = "wino_gemm"
DOMINANT_KERNEL = "gemm_nt_kernel<"  # rocprofv3 name stem on the fp32 pipe (key 10 = 2); gemm_nt_h3_ / gemm_nt_x6_ on fp16x3 / bf16x6


def loss_call_bytes(name, a):
    """Algorithmic HBM bytes of the fused-loss C-ABI calls: the loss
    forward reads p and t (8 B/px); the loss backward fused into the head backward reads
    the 64-channel head input, u and t and writes dx and dL/du (2 x 256 + 12 B/px)."""
    if name == "pis_loss_fwd":
        B, H, W = a[2:5]
        return 8.0 * B * H * W
    if name == "pis_head_loss_bwd":
        B, H, W, C = a[6:10]
        return (8.0 * C + 12.0) * B * H * W
    if name == "pis_head_loss_fwd":  # the call: kernel + its one-block finalize launch
        B, H, W, C = a[7:11]
        return (4.0 * C + 12.0) * B * H * W
    return None


# direct-kernel roles: launch-hook label -> (bench key, description, rocprofv3 symbols)
DIRECT_ROLES = {
    "direct_h3_fwd": ("roofline_direct_fwd", "conv3x3_h3_kernel<false, false, false, false> (forward, 8 x 32 px x "
                      "64 ch per block)", ["conv3x3_h3_kernel<false, false, false, false>"]),
    "direct_h3_pool": ("roofline_direct_pool", "conv3x3_h3_kernel<true, false, false, false> (encoder conv1 forward "
                       "with the 2x2 max pool in the epilogue)", ["conv3x3_h3_kernel<true, false, false, false>"]),
    "direct_h3_dgrad": ("roofline_direct_dgrad", "conv3x3_h3_kernel<false, true|false, false, true> (input gradient "
                        "on the original weights; the ReLU-mask rows prefetched where masked)",
                        ["conv3x3_h3_kernel<false, true, false, true>", "conv3x3_h3_kernel<false, false, false, true>"]),
    "direct_wgrad_h3": ("roofline_direct_wgrad", "conv3x3_wgrad_h3r_kernel<2> (weight gradient: 2-row tiles, two "
                        "blocks per CU, split-K slabs; pis_tune(49, 4): the 4-row conv3x3_wgrad_h3_kernel)",
                        ["conv3x3_wgrad_h3r_kernel", "conv3x3_wgrad_h3_kernel"]),
}


class KernelTimer:
    """HIP events recorded on the launch stream right before / after each launch of the
    dominant kernel (pis_set_launch_hook), with the MFMA FLOPs that launch executes."""

    def __init__(self, kernel=DOMINANT):
        self.kernel = kernel
        self.records = []
        self._open = None

    def __call__(self, kernel, phase, stream, flop):
        if kernel != self.kernel:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream())
        if phase == 0:
            self._open = (ev, flop)
        else:
            self.records.append((self._open[0], ev, flop))

    def summary(self):
        torch.cuda.synchronize()
        if not self.records:
            return 0, 0.0, 0.0
        ms = [e0.elapsed_time(e1) for e0, e1, _ in self.records]
        fl = [f for _, _, f in self.records]
        return len(ms), sum(fl) / len(fl), sum(ms) / len(ms)


class LossCallTimer:
    """HIP events around the fused-loss C-ABI calls (call tracer of _hip.call)."""

    def __init__(self):
        self.loss = {}

    def begin(self, name, args):
        nbytes = loss_call_bytes(name, args)
        if nbytes is None:
            return None
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        return (name, e0, e1, nbytes)

    def end(self, tok):
        if tok is not None:
            name, e0, e1, nbytes = tok
            e1.record()
            self.loss.setdefault(name, []).append((e0, e1, nbytes))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, recs in self.loss.items():
            ms = sum(e0.elapsed_time(e1) for e0, e1, _ in recs) / len(recs)
            nbytes = recs[0][2]
            out[name] = (ms, nbytes, nbytes / (ms * 1e-3) / 1e9)
        return out


# kernels whose MFMA-busy fraction the bench line quotes: the GEMM-shaped ones and the fused loss
BUSY_REPORTED = ("gemm_nt", "wgrad_x6", "wgrad_h3", "wino4_gemm_out", "convt_gemm", "convt_h3", "conv3x3_h3",
                 "conv3x3_wgrad", "loss_fwd", "head_loss", "loss_bwd")


def load_pmc(kernel=DOMINANT_KERNEL, config=PMC_CONFIG):
    """Per-launch HBM bytes and MFMA-busy fraction of the dominant kernel from the committed
    rocprofv3 --pmc summary (tools/pmc_summary.py: FETCH_SIZE x2 gfx950 correction +
    WRITE_SIZE; SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); all None for a
    config the summary was not collected on."""
    path = os.path.join(HERE, "profiles", "pmc_dominant.json")
    if config != PMC_CONFIG or not os.path.exists(path):
        return None, None, None
    with open(path) as f:
        d = json.load(f)
    if kernel not in (d.get("dominant_kernel") or ""):
        return None, None, None  # counters were taken on another kernel: report none rather than stale ones
    busy = {k.split("(")[0].replace("void ", ""): v["mfma_busy_frac"] for k, v in d.get("kernels", {}).items()
            if "mfma_busy_frac" in v and any(s in k for s in BUSY_REPORTED)}
    return d.get("hbm_bytes_per_launch"), d.get("mfma_busy_frac"), busy


def host_cpus():
    """(usable CPUs, description) of this process: the affinity mask, capped by the cgroup
    CPU quota when one is set (a container may see every core of the machine in its
    affinity mask but be granted only a share of them)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    n = min(aff, quota) if quota else aff
    return n, {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "cpu_model": model,
               "machine_cpus": os.cpu_count()}


def cpu_baseline(batch: int = 8, steps: int = 3, size: int = 512, loss_kw=None, lr: float = LR):
    """The oracle (stock-PyTorch CPU restatement of the reference step) on the
    host cores: the C2 batch (8 x 512^2, Stage II), 1 warm-up step, median of ``steps``."""
    from oracle import reference_torch as rt
    threads, info = host_cpus()
    torch.set_num_threads(threads)
    img, mask = rt.synthetic_batch(batch, size, size, seed=42)
    torch.manual_seed(42)
    ref = rt.UNetRef(1, 1, 64).train()
    opt = rt.make_adamw(ref, lr=lr)
    kw = dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05) if loss_kw is None else loss_kw
    rt.train_step(ref, opt, img, mask, kw)  # warm-up
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        rt.train_step(ref, opt, img, mask, kw)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    out = {"value": batch / med, "unit": "images/s", "cores": threads, "kind": "port",
           "sample": f"median of {steps} training steps of {batch} images {size}x{size} "
                     f"({'Stage II' if kw.get('rd_w') or kw.get('pf_w') else 'Stage I'}; oracle/reference_torch.py, "
                     f"torch {torch.__version__} CPU, {threads} threads) after 1 warm-up step; step times "
                     + ", ".join(f"{t:.2f}" for t in times) + " s"}
    out.update(info)
    return out


def make_batch(rank: int, device):
    g = torch.Generator().manual_seed(42 + rank)
    imgs, masks = zip(*[disc_sample(H, W, g) for _ in range(B)])
    return torch.stack(imgs).to(device), torch.stack(masks).to(device)


def loss_standalone(u: torch.Tensor, t: torch.Tensor, loss_kw: dict, reps: int = 20):
    """pis_loss_fwd and pis_loss_bwd alone on the step's own probabilities and masks (C2: 2.1 M
    px), timed with HIP events with a 1 GiB buffer READ between reps so p and t come from HBM,
    not the 256 MiB Infinity Cache, and no dirty lines of the flush are written back
    during the timed call; median over reps. Algorithmic bytes: forward
    8 B/px (read p, t), backward 12 B/px (read p, t; write dL/dz)."""
    import ctypes

    from physics_informed_image_segmentation_amd import _hip
    lib = _hip.lib()
    Bn, Hn, Wn = u.shape[0], u.shape[-2], u.shape[-1]
    crit = DiceBCEPDELoss(**loss_kw)
    prm = crit.config().params()
    st = torch.cuda.current_stream().cuda_stream
    terms = torch.empty(8, device=u.device)
    counts = torch.empty(Bn, 3, dtype=torch.int32, device=u.device)
    scores = torch.empty(Bn, 2, device=u.device)
    nws = lib.pis_loss_ws(Bn, Hn, Wn)
    ws = torch.zeros(nws // 4 + 1, device=u.device)
    dz = torch.empty_like(u)
    flush = torch.ones(256 << 20, device=u.device)  # 1 GiB
    sink = torch.empty((), device=u.device)
    calls = {
        "fwd": (lambda: lib.pis_loss_fwd(u.data_ptr(), t.data_ptr(), Bn, Hn, Wn, ctypes.byref(prm), terms.data_ptr(),
                                         counts.data_ptr(), scores.data_ptr(), ws.data_ptr(), nws, st), 8.0),
        "bwd": (lambda: lib.pis_loss_bwd(u.data_ptr(), t.data_ptr(), Bn, Hn, Wn, ctypes.byref(prm), terms.data_ptr(),
                                         0, dz.data_ptr(), 2, st), 12.0),
    }
    def cold_ms(fn):
        ts = []
        for _ in range(reps):
            torch.sum(flush, dim=0, out=sink)  # a READ: evicts with clean lines (no write-back tail)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if fn() != 0:
                raise RuntimeError(lib.pis_last_error().decode())
            e1.record()
            ts.append((e0, e1))
        torch.cuda.synchronize()
        return statistics.median(a.elapsed_time(b) for a, b in ts)

    # the floor at this size: ONE bandwidth-probe launch moving the same bytes (read p, t: forward;
    # + write one float per pixel: backward) under the same protocol, best over its grid sizes
    part = torch.empty(16384, device=u.device)
    probe = {
        "fwd": lambda grid: lib.pis_debug_stream_probe(u.data_ptr(), t.data_ptr(), 0, u.numel(), part.data_ptr(),
                                                       grid, st),
        "bwd": lambda grid: lib.pis_debug_stream_probe(u.data_ptr(), t.data_ptr(), dz.data_ptr(), u.numel(), 0,
                                                       grid, st),
    }
    out = {}
    for name, (fn, bpp) in calls.items():
        ms = cold_ms(fn)
        nbytes = bpp * u.numel()
        gbs = nbytes / (ms * 1e-3) / 1e9
        floor = min((cold_ms(lambda g=g: probe[name](g)), g) for g in (256, 512, 1024, 2048, 4096))
        fgbs = nbytes / (floor[0] * 1e-3) / 1e9
        out[f"pis_loss_{name}_cold"] = {
            "bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
            "bytes_per_call": nbytes, "avg_call_ms": ms,
            "measured": f"standalone, median of {reps}, 1 GiB read between calls",
            "floor": {"kernel": "stream_probe_kernel (one float4 grid-stride launch, the same bytes)", "grid": floor[1],
                      "avg_call_ms": floor[0], "achieved": fgbs, "frac": fgbs / 8000.0,
                      "loss_over_floor": ms / floor[0]}}
    return out


def hbm_probe(device, reps: int = 10) -> dict:
    """The box's attainable streaming rate, for context beside the HBM rooflines (which are priced
    against the 8 TB/s datasheet figure): stream_probe_kernel (a float4 grid-stride loop) reading
    two 256 MiB arrays and writing a third (768 MiB per launch, 2:1 read:write), best over its grid
    sizes, median of ``reps`` launches each. MI355X_MICROARCH.md quotes 6.29 TB/s for a float4 copy."""
    from physics_informed_image_segmentation_amd import _hip
    lib = _hip.lib()
    n = 64 << 20  # floats per array
    a = torch.ones(n, device=device)
    b = torch.ones(n, device=device)
    c = torch.empty(n, device=device)
    st = torch.cuda.current_stream().cuda_stream
    best = None
    for grid in (256, 512, 1024, 2048, 4096, 8192):
        evs = []
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if lib.pis_debug_stream_probe(a.data_ptr(), b.data_ptr(), c.data_ptr(), n, 0, grid, st) != 0:
                raise RuntimeError(lib.pis_last_error().decode())
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        ms = statistics.median(x.elapsed_time(y) for x, y in evs[1:])
        if best is None or ms < best[0]:
            best = (ms, grid)
    gbs = 12.0 * n / (best[0] * 1e-3) / 1e9
    del a, b, c
    return {"kernel": "stream_probe_kernel (read 2 x 256 MiB, write 256 MiB, float4 grid-stride)", "grid": best[1],
            "avg_launch_ms": best[0], "achieved": gbs, "unit": "GB/s", "frac_of_8tbs": gbs / 8000.0}


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch(n: int) -> int:
    """Start ``n`` ranks of this script (one process per GPU) and wait for them. The parent
    never touches the GPU; it only forwards signals and collects exit statuses."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                stop()  # one rank failed: the others would hang in their next collective
        time.sleep(0.2)
    return rc


def dist_summary(bucketer, device, backend):
    """N > 1: what the process group actually formed and how much of the gradient all-reduce the
    backward left exposed: the backend, the world size as formed,
    RCCL's version, the bucket plan, and per rank the mean / worst exposed all-reduce ms over the
    timed steps (GradBucketer.exposed_ms: later stream's last gradient kernel -> all-reduces
    waited for), gathered to every rank (the max over ranks is the figure that bounds the step)."""
    per_step = bucketer.exposed_ms()
    world, rank = dist.get_world_size(), dist.get_rank()
    mine = torch.zeros(2 * world, dtype=torch.float64, device=device if backend == "nccl" else "cpu")
    if per_step:
        mine[rank] = sum(per_step) / len(per_step)
        mine[world + rank] = max(per_step)
    dist.all_reduce(mine, op=dist.ReduceOp.SUM)
    mean_r, worst_r = mine[:world].tolist(), mine[world:].tolist()
    rccl = None
    if dist.get_backend() == "nccl":
        try:
            v = torch.cuda.nccl.version()
            rccl = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception:  # noqa: BLE001 - informational only
            rccl = None
    return {
        "backend": dist.get_backend(), "world_size_formed": world, "rccl_version": rccl,
        "grad_bytes": int(bucketer.model.arena.numel()) * 4, "buckets": len(bucketer.buckets),
        "bucket_bytes": bucketer.bucket_bytes,
        "exposed_allreduce_ms": {"max_over_ranks": max(mean_r), "worst_step_max_over_ranks": max(worst_r),
                                 "mean_per_rank": mean_r, "steps": len(per_step)},
        "measured": "HIP events: after each rank's last gradient kernel on both streams vs after "
                    "GradBucketer.finish() waited for the bucketed all-reduces (per timed step)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c2")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="process-group backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse "
                         "several ranks on one GPU)")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="pis_tune knob for experiments (include/pis_capi.h PIS_TUNE_*); defaults are the measured best")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args.gpus))
    global H, W
    size, loss_kw, workload = CONFIGS[args.config]
    H = W = size
    _, local_rank, world = env_world()
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    ndev = torch.cuda.device_count()  # counts devices without initialising the runtime
    if ndev == 0 or (local_rank >= ndev and args.backend == "nccl"):
        print(f"bench.py: rank {local_rank} has no GPU of its own ({ndev} visible); RCCL needs one GPU per rank",
              file=sys.stderr)
        sys.exit(2)
    device = torch.device("cuda", local_rank % ndev)
    torch.cuda.set_device(device)
    rank, local_rank, world = init_from_env(args.backend)

    if args.tune:
        from physics_informed_image_segmentation_amd import _hip as _h
        for kv in args.tune:
            k, v = (int(z) for z in kv.split("="))
            _h.lib().pis_tune(k, v)
    torch.manual_seed(42)
    model = UNet(1, 1, 64).to(device).train()
    broadcast_parameters(model)
    bucketer = GradBucketer(model) if world > 1 else None
    torch.cuda.manual_seed(42 + rank)  # Dropout2d masks per rank (train() does the same)
    crit = DiceBCEPDELoss(**loss_kw)
    opt = AdamW(model.parameters(), lr=LR, weight_decay=1e-5, grad_scale=1.0 / world)
    x, t = make_batch(rank, device)

    def step():
        opt.zero_grad()
        # u = model(x); loss = crit(u, t) with the head and the loss forward in one kernel
        # (UNet.forward_with_loss: pis_head_loss_fwd), as train_epoch runs it
        _, loss = model.forward_with_loss(x, t, crit)
        loss.backward()
        opt.step()
        return loss

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # roofline of the dominant kernel, live over the timed region: HIP events recorded on the
    # launch stream right around each of its launches (pis_set_launch_hook), and around the
    # fused-loss C-ABI calls (host-side enqueue only; the GPU stays the bottleneck)
    from physics_informed_image_segmentation_amd import _hip
    ktimer, ftimer, ltimer = KernelTimer(), KernelTimer("wino_gemm_out"), LossCallTimer()
    htimer = KernelTimer("head_loss_fwd")  # its hook "flop" carries the launch's algorithmic bytes
    dtimers = {k: KernelTimer(k) for k in DIRECT_ROLES}
    _hip.set_launch_hook(lambda *a: (ktimer(*a), ftimer(*a), htimer(*a), *(tm(*a) for tm in dtimers.values())))
    _hip.set_tracer(ltimer)
    if bucketer is not None:
        bucketer.timing = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rank_ms = None
    if world > 1:
        # every rank's own time (straggling), then the max over ranks for the line
        tt = torch.zeros(world, device=device if args.backend == "nccl" else "cpu", dtype=torch.float64)
        tt[rank] = dt
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        per = [v / args.steps * 1e3 for v in tt.tolist()]
        rank_ms = {"min": min(per), "max": max(per), "per_rank": per,
                   "measured": "each rank's own barrier-to-barrier time / steps; ms_per_step is the max"}
        dt = max(tt.tolist())
    ms = dt / args.steps * 1e3
    imgs_per_s = world * B * args.steps / dt
    dist_info = None
    if bucketer is not None:
        bucketer.timing = False
        dist_info = dist_summary(bucketer, device, args.backend)

    _hip.set_tracer(None)
    _hip.set_launch_hook(None)
    n_launch, flop_per_launch, ms_per_launch = ktimer.summary()
    n_launch //= args.steps
    nf_launch, f_flop, f_ms = ftimer.summary()
    nf_launch //= args.steps
    direct_live = {k: tm.summary() for k, tm in dtimers.items()}
    loss_t = ltimer.summary()
    nh_launch, h_bytes, h_ms = htimer.summary()
    achieved = flop_per_launch / (ms_per_launch * 1e-3) / 1e12
    # the same kernel with the weight gradients serialised on one stream (no concurrent
    # kernel sharing the CUs): one extra instrumented step after the timed region
    eng = model.engine()
    side, eng.side = eng.side, None
    iso, fiso = KernelTimer(), KernelTimer("wino_gemm_out")
    disos = {k: KernelTimer(k) for k in DIRECT_ROLES}
    _hip.set_launch_hook(lambda *a: (iso(*a), fiso(*a), *(tm(*a) for tm in disos.values())))
    step()
    _hip.set_launch_hook(None)
    eng.side = side
    _, iso_flop, iso_ms = iso.summary()
    _, _, fiso_ms = fiso.summary()
    direct_iso = {k: tm.summary() for k, tm in disos.items()}
    # the pipe the dominant kernel runs on. fp32-class GEMMs on the MFMA pipe: fp16x3 (pis_tune
    # key 10 = 4, the default: per-K-step power-of-two tile scales, hi + lo fp16 split, three
    # fp16 MFMAs per fp32 multiply-add) peaks at the dense fp16 MFMA rate (~2.5 PFLOP/s,
    # MI355X_MICROARCH.md / the task's dense figure) / 3 in fp32-equivalent FLOPs; bf16x6 (key 10
    # = 3: six bf16 MFMAs) at / 6; the native fp32 MFMA path (key 10 = 2) at 157.3 TFLOP/s
    mode = _hip.lib().pis_tune(10, -1)
    x6, h3 = mode == 3, mode == 4
    peak = 2500.0 / 3.0 if h3 else 2500.0 / 6.0 if x6 else 157.3
    pipe = ("fp16 MFMA, fp32-class fp16x3 split (per-K-step power-of-two tile scales, hi + lo fp16, 3 fp16 "
            "products per fp32 multiply-add); achieved/peak in fp32-equivalent FLOPs" if h3 else
            "bf16 MFMA, fp32-accurate bf16x6 split (6 bf16 products per fp32 multiply-add); achieved/peak in "
            "fp32-equivalent FLOPs" if x6 else "fp32 MFMA")
    # gemm_nt_h3_bk32_kernel / gemm_nt_x6_bk32_kernel (K % 32 == 0, every C2 layer)
    kname = "gemm_nt_h3_" if h3 else "gemm_nt_x6_" if x6 else DOMINANT_KERNEL
    traffic, mfma_busy, busy_by_kernel = load_pmc(kname, args.config)
    pmc = lambda sub: pmc_bytes(sub, args.config)  # noqa: E731
    # the same launches against BOTH bounds (per launch max of FLOP / pipe peak and algorithmic
    # bytes / 8 TB/s): only valid when the shape list reproduces the launches the hook timed
    gl = wino_gemm_launches(H, W, B)
    g_fl, g_by, g_tmin, g_tf, g_tb = gemm_attainable(gl, peak)
    hbm_view = None
    if len(gl) == n_launch and abs(g_fl / len(gl) - flop_per_launch) <= 1e-6 * flop_per_launch:
        bpl = g_by / len(gl)
        hbm_view = {
            "bytes_per_launch": bpl, "unit": "GB/s", "peak": 8000.0,
            "achieved": bpl / (ms_per_launch * 1e-3) / 1e9, "frac": bpl / (ms_per_launch * 1e-3) / 8e12,
            "isolated_frac": bpl / (iso_ms * 1e-3) / 8e12,
            "step_bytes_s": g_tb, "step_flop_s": g_tf,
            "attainable_frac": g_tmin / (n_launch * ms_per_launch * 1e-3),
            "attainable_frac_isolated": g_tmin / (n_launch * iso_ms * 1e-3),
            "hbm_bound_launches": sum(1 for T, C, N, nxi in gl if 4.0 * nxi * (T * C + N * C + T * N) / 8e12 >
                                      2.0 * nxi * T * C * N / (peak * 1e12)),
            "f6_launches": sum(1 for *_, nxi in gl if nxi == 64),
            "note": "algorithmic bytes = V read + U read + M written once (4 B x 36 planes, 64 for the F(6x6,3x3) "
                    "launches); attainable = "
                    "sum over the step's launches of max(FLOP / pipe peak, bytes / 8 TB/s) / their measured "
                    "time: the GEMMs are mostly HBM-bound (the 36 fp32 M planes)"}
    # the fused contraction + output transform (wino4_gemm_out_x6_kernel): HBM-bound by design
    fl_ = fused_launches(H, W, B)
    fused_roof = None
    if nf_launch and len(fl_) == nf_launch:
        fb = sum(fused_bytes(*u) for u in fl_) / nf_launch
        fused_roof = {
            "bound": "hbm", "kernel": "wino4_gemm_out_x6_kernel<4, 2, 64|128, 4, fp16x3> (wino_gemm_out: the 36 "
                                      "F(4x4,3x3) contractions fused with the output transform, 64 / 128-channel "
                                      "contractions into <= 256 outputs)",
            "achieved": fb / (f_ms * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
            "frac": fb / (f_ms * 1e-3) / 8e12, "traffic": pmc("wino4_gemm_out"),
            "bytes_per_launch": fb, "launches_per_step": nf_launch, "avg_launch_ms": f_ms,
            "flop_per_launch": f_flop, "mfma_tflops": f_flop / (f_ms * 1e-3) / 1e12,
            "bytes": "V read + filter planes read once + output written (+ the input gradient's ReLU mask read)",
            "measured": "live over the timed steps",
            "isolated": {"frac": fb / (fiso_ms * 1e-3) / 8e12 if fiso_ms else None, "avg_launch_ms": fiso_ms,
                         "measured": "one extra step, weight gradients serialised"}}
    # the direct fp16x3 3x3 convolutions (csrc/direct.hip, the shallow layers), one roofline per
    # role — and per kernel symbol (forward, pooled forward, input gradient, weight gradient):
    # MFMA-bound, priced in fp32-equivalent FLOPs (2 x 9 x pixels x C x N per launch) against the
    # fp16x3 pipe, with the algorithmic HBM bytes per launch beside the PMC traffic of the same symbols
    h3_peak = 2500.0 / 3.0
    direct_roofs = {}
    role_launches = direct_role_launches(H, W, B)
    for key, (name, kern, syms) in DIRECT_ROLES.items():
        n_d, fl_d, ms_d = direct_live[key]
        if not n_d:
            continue
        n_d //= args.steps
        _, ifl_d, ims_d = direct_iso[key]
        busy = None
        if busy_by_kernel is not None:
            hits = [v for k, v in busy_by_kernel.items() if any(x in k for x in syms)]
            busy = sum(hits) / len(hits) if hits else None
        lay = role_launches.get(key, [])
        alg = (sum(b for _, b in lay) / len(lay)
               if len(lay) == n_d and abs(sum(f for f, _ in lay) / len(lay) - fl_d) <= 1e-6 * fl_d else None)
        direct_roofs[name] = {
            "bound": "mfma", "kernel": kern, "achieved": fl_d / (ms_d * 1e-3) / 1e12, "peak": h3_peak,
            "unit": "TFLOP/s", "frac": fl_d / (ms_d * 1e-3) / 1e12 / h3_peak, "traffic": pmc(syms),
            "traffic_symbols": syms,
            "pipe": "fp16 MFMA, fp32-class fp16x3 split (3 fp16 products per fp32 multiply-add); fp32-equivalent "
                    "FLOPs of the direct convolution",
            "mfma_busy_frac": busy, "launches_per_step": n_d, "avg_launch_ms": ms_d, "flop_per_launch": fl_d,
            "ms_per_step": n_d * ms_d, "algorithmic_bytes_per_launch": alg,
            "hbm_frac": alg / (ms_d * 1e-3) / 8e12 if alg else None,
            "measured": "live over the timed steps (HIP events on the launch stream)",
            "isolated": {"achieved": ifl_d / (ims_d * 1e-3) / 1e12 if ims_d else None,
                         "frac": ifl_d / (ims_d * 1e-3) / 1e12 / h3_peak if ims_d else None, "avg_launch_ms": ims_d,
                         "measured": "one extra step, weight gradients serialised"}}
    loss_cold = loss_standalone(model.engine().u, t, loss_kw)
    hbm = hbm_probe(device)
    if rank == 0:
        flops = conv_flops_per_image(H, W) * B
        out = {
            "metric": ("training images/sec (512x512, Stage-II RD+PF loss)" if args.config == "c2"
                       else f"training images/sec ({H}x{W}, {args.config})"),
            "value": imgs_per_s, "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32 (fp16x3 split MFMA, power-of-two block scales; direct + Winograd convs)", "data": "synthetic",
            "config": {"workload": workload,
                       "global_batch": B * world, "image_size": [H, W], "parallelism": f"dp{world}"},
            "roofline": None,
            "roofline_gemm": {"bound": "mfma", "kernel": ("gemm_nt_h3_bk32_kernel<128, 128|64>" if h3 else
                                                     "gemm_nt_x6_bk32_kernel<128, 128|64>" if x6 else
                                                     "gemm_nt_kernel<128, 128|64>")
                         + f" ({DOMINANT}: the batched GEMMs of Winograd fwd/dgrad: 36 per F(4x4,3x3) launch, "
                           "64 per F(6x6,3x3) launch)",
                         "achieved": achieved, "peak": peak,
                         "unit": "TFLOP/s", "frac": achieved / peak, "traffic": traffic, "pipe": pipe,
                         "fp32_mfma_peak_frac": achieved / 157.3,
                         # against the round-1/2 bf16x6 pipe roofline (2.5 PF / 6), for continuity
                         "bf16x6_roofline_frac": achieved / (2500.0 / 6.0),
                         # rocprofv3 PMC (profiles/pmc_dominant.json): fraction of SIMD-cycles the
                         # matrix pipe was busy in this kernel, and in the step's other kernels
                         "mfma_busy_frac": mfma_busy, "mfma_busy_by_kernel": busy_by_kernel,
                         "hbm_view": hbm_view,
                         "launches_per_step": n_launch, "avg_launch_ms": ms_per_launch,
                         "flop_per_launch": flop_per_launch,
                         "measured": "live over the timed steps; the input-gradient launches share the GPU "
                                     "with the weight-gradient stream",
                         "isolated": {"achieved": iso_flop / (iso_ms * 1e-3) / 1e12,
                                      "frac": iso_flop / (iso_ms * 1e-3) / 1e12 / peak, "avg_launch_ms": iso_ms,
                                      "measured": "one extra step, weight gradients serialised"}},
            "roofline_fused": fused_roof,
            # direct-convolution FLOPs of the step / step time (Winograd executes fewer)
            "step_tflops_direct_equiv": flops / (ms * 1e-3) / 1e12,
            # north-star HBM figure for the fused loss (live over the timed steps): the backward
            # runs inside the head backward kernel (its reduce_slabs follow-ups inside the
            # events); the forward is the row kernel + its one-block finalize launch
            "roofline_loss": dict({
                name.replace("pis_", "") + "_live": {
                    "bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                    "bytes_per_call": nb, "avg_call_ms": t,
                    "measured": ("live over the timed steps (Infinity-Cache warm)" if name == "pis_loss_fwd" else
                                 "live; the loss backward fused into the head backward: bytes are dominated "
                                 "by the 64-channel head input and its gradient, not by the loss")}
                for name, (t, nb, gbs) in loss_t.items()}, **loss_cold,
                **({"head_loss_fwd_kernel_live": {
                    "bound": "hbm", "achieved": h_bytes / (h_ms * 1e-3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                    "frac": h_bytes / (h_ms * 1e-3) / 8e12, "bytes_per_launch": h_bytes, "avg_launch_ms": h_ms,
                    "launches_per_step": nh_launch // args.steps, "traffic": pmc("head_loss_fwd_kernel"),
                    "kernel": "head_loss_fwd_kernel (the U-Net head's 1x1 conv + sigmoid fused with the whole loss "
                              "forward: Dice / BCE / RD / PF partials and the per-sample counters)",
                    "bytes": "head input read (4 C B/px) + targets read (4 B/px) + z and u written (8 B/px); the "
                             "two halo rows per band re-read from L2 / MALL are not algorithmic",
                    "measured": "live over the timed steps (HIP events on the launch stream, kernel only; its "
                                "one-block finalize launch follows)"}} if nh_launch else {})),
            "final_loss": float(loss.item()),
            # context for the HBM rooflines above (priced against 8 TB/s): this box's streaming rate
            "hbm_probe": hbm,
        }
        for r in (out["roofline_loss"].get("head_loss_fwd_kernel_live"), fused_roof):
            if r:
                r["frac_of_hbm_probe"] = r["achieved"] / hbm["achieved"]
        # the dominant kernel (most GPU time per step) carries the contract's "roofline"; the
        # other of the two conv kernels stays beside it
        g_ms, f_ms_step = n_launch * ms_per_launch, (nf_launch * f_ms if fused_roof else 0.0)
        out["roofline_gemm"]["ms_per_step"] = g_ms
        if fused_roof:
            fused_roof["ms_per_step"] = f_ms_step
        out.update(direct_roofs)
        cands = {"roofline_gemm": g_ms, **({"roofline_fused": f_ms_step} if fused_roof else {}),
                 **{k: v["ms_per_step"] for k, v in direct_roofs.items()}}
        out["roofline_dominant"] = max(cands, key=cands.get)
        out["roofline"] = out[out["roofline_dominant"]]
        if dist_info is not None:
            out["distributed"] = dist_info
            out["ms_per_step_by_rank"] = rank_ms
        if args.config != PMC_CONFIG:
            out["pmc_note"] = PMC_NOTE
        if world == 1 and not args.no_cpu_baseline and args.config == "c2":
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
