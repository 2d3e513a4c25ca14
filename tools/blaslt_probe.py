"""Probe (analysis tooling): what the vendor fp16 batched GEMM (torch.bmm -> hipBLASLt / rocBLAS)
reaches on the Winograd GEMM shapes of the C2 step, with the fp16x3 product written as ONE GEMM
over a 3x longer contraction ([Ah | Al | Ah] x [Bl | Bh | Bh]^T) — i.e. the rate a pre-split
Winograd pipeline would get from the library. Prints per shape the fp16 TFLOP/s and the
fp32-equivalent rate (/3) next to gemm_nt_h3_bk32_kernel's (the trace's per-launch times).

    python tools/blaslt_probe.py
"""
import time

import torch

# (name, T tiles, C contraction, N outputs) of the C2 step's batched GEMMs (36 batches)
SHAPES = [("enc3.conv1", 8192, 256, 256), ("enc4.conv0", 2048, 256, 512), ("enc4.conv1", 2048, 512, 512),
          ("bottleneck", 512, 512, 512), ("dec4.conv0", 2048, 1024, 512), ("dec4.conv1", 2048, 512, 512),
          ("dec3.conv0", 8192, 512, 256), ("dec3.conv1", 8192, 256, 256), ("dec2.conv0", 32768, 256, 128)]


def bench(f, reps=10):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.device("cuda")
    for name, T, C, N in SHAPES:
        a = torch.randn(36, T, 3 * C, device=dev, dtype=torch.float16)
        b = torch.randn(36, 3 * C, N, device=dev, dtype=torch.float16)
        t = bench(lambda: torch.bmm(a, b))
        fl = 2.0 * 36 * T * 3 * C * N
        # fp32 output variant: fp16 inputs, fp32 accumulation and output via addbmm-free baddbmm on
        # float32 views is not available; report the fp16-output rate (output bytes are half)
        print(f"{name:11s} T={T:6d} C={C:5d} N={N:4d}  {t * 1e6:8.1f} us  fp16 {fl / t / 1e12:7.1f} TF/s  "
              f"fp32-eq {fl / 3 / t / 1e12:6.1f} TF/s", flush=True)
        del a, b
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
