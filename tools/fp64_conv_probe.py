"""Times the float64 oracle's convolutions on the GPU (the full-size parity tests' truth runs):
F.conv2d forward + backward in float64 through MIOpen (cudnn enabled) vs torch's native
im2col + GEMM path (torch.backends.cudnn.enabled = False), at the U-Net's C5 shapes (2 images of
1024^2 per chunk). Test tooling only; prints one line per shape and path."""
import time

import torch
import torch.nn.functional as F


def run(B, C, N, H, cudnn, reps=2):
    torch.backends.cudnn.enabled = cudnn
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(B, C, H, H, device="cuda", dtype=torch.float64, generator=g).requires_grad_()
    w = torch.randn(N, C, 3, 3, device="cuda", dtype=torch.float64, generator=g).requires_grad_()
    out = None
    for r in range(reps + 1):
        if r == 1:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        y = F.conv2d(x, w, padding=1)
        gx, gw = torch.autograd.grad(y, (x, w), torch.ones_like(y))
        out = (y, gx, gw)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


if __name__ == "__main__":
    for (B, C, N, H) in [(2, 64, 64, 1024), (2, 128, 128, 512), (2, 512, 512, 128), (2, 1024, 1024, 64)]:
        t1, o1 = run(B, C, N, H, True)
        t0, o0 = run(B, C, N, H, False)
        d = max(float((a - b).abs().max() / b.abs().max()) for a, b in zip(o0, o1))
        print(f"B={B} {C}->{N} {H}^2  miopen {t1 * 1e3:9.1f} ms  native {t0 * 1e3:9.1f} ms  rel diff {d:.2e}",
              flush=True)
