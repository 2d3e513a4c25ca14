"""The F(3x3,4x4) weight gradient's slab sum + output transform (launch_wino_wgrad_out) per C2 layer:
HIP events from the end of the weight-gradient GEMM (launch hook) to the end of the C-ABI call, for
each pis_tune(48) form, interleaved rounds; bytes = 36 x splits x Cout x Cin x 4 read + the 3 x 3
gradient written (read too when accumulating).

    python tools/bench_wgrad_out.py [--variants 0,1] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402

LAYERS = [  # name, H, Cin, Cout (C2, B = 8): the layers whose weight gradient runs F(3x3,4x4)
    ("enc3.conv0", 128, 128, 256), ("enc3.conv1", 128, 256, 256), ("dec3.conv0", 128, 512, 256),
    ("dec3.conv1", 128, 256, 256), ("enc4.conv0", 64, 256, 512), ("enc4.conv1", 64, 512, 512),
    ("dec4.conv0", 64, 1024, 512), ("bott.conv0", 32, 512, 1024), ("bott.conv1", 32, 1024, 1024),
    ("dec2.conv0", 256, 256, 128),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    lib = _hip.lib()
    B = 8
    st = torch.cuda.current_stream().cuda_stream
    evs = []

    def hook(kernel, phase, stream, flop):
        if kernel == "wino_wgrad_gemm" and phase == 1:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            evs.append(ev)

    _hip.set_launch_hook(hook)
    variants = [int(v) for v in args.variants.split(",")]
    tot = {v: 0.0 for v in variants}
    for name, H, cin, cout in LAYERS:
        x = torch.rand(B, H, H, cin, device="cuda")
        dz = torch.randn(B, H, H, cout, device="cuda")
        dw = torch.zeros(cout, 3, 3, cin, device="cuda")
        db = torch.zeros(cout, device="cuda")
        nws = lib.pis_conv3x3_wgrad_ws(B, H, H, cin, cout)
        ws = torch.empty(nws // 4 + 1, device="cuda")
        res = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                prev = lib.pis_tune(48, v)
                try:
                    for _ in range(args.reps):
                        evs.clear()
                        e1 = torch.cuda.Event(enable_timing=True)
                        rc = lib.pis_conv3x3_wgrad(x.data_ptr(), cin, dz.data_ptr(), cout, dw.data_ptr(), db.data_ptr(),
                                                   B, H, H, cin, cout, 8, ws.data_ptr(), nws, st)
                        e1.record()
                        if rc != 0:
                            raise RuntimeError(lib.pis_last_error().decode())
                        torch.cuda.synchronize()
                        if evs:
                            res[v].append(evs[-1].elapsed_time(e1))
                finally:
                    lib.pis_tune(48, prev)
        if not res[variants[0]]:
            print(f"{name:12s} not a Winograd weight gradient", flush=True)
            continue
        line = f"{name:12s}"
        for v in variants:
            ms = statistics.median(res[v])
            tot[v] += ms
            line += f"  v{v}: {ms * 1e3:7.1f} us"
        print(line, flush=True)
        del x, dz, ws
        torch.cuda.empty_cache()
    print("total " + "  ".join(f"v{v}: {tot[v] * 1e3:.1f} us" for v in variants), flush=True)
    _hip.set_launch_hook(None)


if __name__ == "__main__":
    main()
