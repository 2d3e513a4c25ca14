"""Time the batched Winograd NT GEMM kernels in isolation (HIP events, interleaved rounds).

The shapes are the C2 (B = 8, 512^2) F(4x4,3x3) GEMMs: 36 batched products
C[xi] (T x N) = V[xi] (T x C) . U[xi]^T, T = 8 H W / 16 tiles.

    python tools/bench_gemm.py [--variants 0,1,2,3] [--rounds 3] [--check]

variants: see pis_debug_gemm_nt in include/pis_capi.h. TF/s are fp32-equivalent.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402

SHAPES = [  # name, H, C (contraction), N (outputs)
    ("enc2.conv1", 256, 128, 128), ("enc3.conv1", 128, 256, 256), ("dec3.conv0", 128, 512, 256),
    ("enc4.conv1", 64, 512, 512), ("dec4.conv0", 64, 1024, 512), ("bottleneck", 32, 512, 512),
    ("dec2.conv0", 256, 256, 128),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--check", action="store_true", help="compare variant outputs with torch fp64")
    ap.add_argument("--dist", default="randn",
                    help="operand values: randn | tiny (A x 1e-9, B x 1e-3: gradient-like) | "
                         "wide (A rows x 10^U(-5,0), B x 1e4)")
    ap.add_argument("--shapes", default="", help="comma-separated shape names (default: all)")
    args = ap.parse_args()
    lib = _hip.lib()
    s = torch.cuda.current_stream().cuda_stream
    variants = [int(v) for v in args.variants.split(",")]
    for name, H, C, N in SHAPES:
        if args.shapes and name not in args.shapes.split(","):
            continue
        T = 8 * H * H // 16
        A = torch.randn(36, T, C, device="cuda")
        Bm = torch.randn(36, N, C, device="cuda")
        if args.dist == "tiny":
            A *= 1e-9
            Bm *= 1e-3
        elif args.dist == "wide":
            A *= 10.0 ** (-5 * torch.rand(36, T, 1, device="cuda"))
            Bm *= 1e4
        Cm = torch.empty(36, T, N, device="cuda")
        bptr = {}
        flop = 2.0 * 36 * T * N * C
        res = {}
        for _ in range(args.rounds):
            for v in variants:
                rc = lib.pis_debug_gemm_nt(A.data_ptr(), bptr.get(v, Bm.data_ptr()), Cm.data_ptr(), T, N, C, 36, v, s)
                if rc != 0:  # shape not covered by this variant
                    res.setdefault(v, []).append(float("inf"))
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(args.reps):
                    lib.pis_debug_gemm_nt(A.data_ptr(), bptr.get(v, Bm.data_ptr()), Cm.data_ptr(), T, N, C, 36, v, s)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault(v, []).append(e0.elapsed_time(e1) / args.reps)
        line = f"{name:11s} T={T:6d} C={C:4d} N={N:4d}"
        for v in variants:
            ms = min(res[v])
            line += f"  v{v}: {ms * 1e3:6.1f} us {flop / ms / 1e9:6.1f} TF/s"
        print(line, flush=True)
        if args.check:
            ref = torch.bmm(A[:2].double(), Bm[:2].double().transpose(1, 2))
            for v in variants:
                if v in (1, 2, 9, 13, 14) or min(res[v]) == float("inf"):
                    continue
                lib.pis_debug_gemm_nt(A.data_ptr(), bptr.get(v, Bm.data_ptr()), Cm.data_ptr(), T, N, C, 36, v, s)
                torch.cuda.synchronize()
                err = ((Cm[:2].double() - ref).norm() / ref.norm()).item()
                print(f"    v{v} rel err {err:.2e}", flush=True)
        del A, Bm, Cm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
