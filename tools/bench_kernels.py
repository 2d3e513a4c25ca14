"""Per-layer kernel micro-benchmark on the GPU (C2 shapes: B=8, 512^2 input).

Times conv3x3 fwd / dgrad / wgrad through the C-ABI with HIP events, for each
value of one tuning knob (pis_tune key), in interleaved rounds inside one
process (cdna_hip_programming.md §5.4 rule 24). Prints TFLOP/s per layer.

    python tools/bench_kernels.py [--key 4] [--variants 0,1,2] [--rounds 3] [--noload]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from physics_informed_image_segmentation_amd import _hip  # noqa: E402

LAYERS = [  # name, H, Cin, Cout
    ("enc1.conv1", 512, 64, 64), ("dec1.conv0", 512, 128, 64), ("enc2.conv1", 256, 128, 128),
    ("dec2.conv0", 256, 256, 128), ("enc3.conv1", 128, 256, 256), ("dec3.conv0", 128, 512, 256),
    ("enc4.conv1", 64, 512, 512), ("dec4.conv0", 64, 1024, 512), ("bottleneck", 32, 512, 512),
    ("enc2.conv0", 256, 64, 128), ("enc3.conv0", 128, 128, 256), ("enc4.conv0", 64, 256, 512),
]
B = 8
NOLOAD_KEY = 2
UP_LAYERS = [  # name, input H, Cin, Cout (2x2 stride-2 transposed convs)
    ("up1", 256, 128, 64), ("up2", 128, 256, 128), ("up3", 64, 512, 256), ("up4", 32, 512, 512),
]


def timed(fn, reps=3):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--key", type=int, default=4)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--layers", default="")
    ap.add_argument("--ops", default="fwd,dgrad,wgrad")
    ap.add_argument("--noload", action="store_true", help="also time each variant without global loads")
    ap.add_argument("--dbg", default="", help="timing twins: pis_tune key 2 levels to time beside each variant "
                    "(direct kernels: 1 no global loads, 2 no LDS staging, 4 no epilogue; OR-ed)")
    ap.add_argument("--convt", action="store_true", help="time the transposed convs instead")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE", help="fixed knobs for every variant")
    args = ap.parse_args()
    lib = _hip.lib()
    for kv in args.tune:
        k, v = kv.split("=")
        lib.pis_tune(int(k), int(v))
    variants = [int(v) for v in args.variants.split(",")]
    default = lib.pis_tune(args.key, -1)
    s = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda")
    opsel = args.ops.split(",")
    if args.convt:
        return bench_convt(lib, args, variants, default, s, dev, opsel)
    sel = [l for l in LAYERS if not args.layers or l[0] in args.layers.split(",")]
    for name, H, cin, cout in sel:
        x = torch.rand(B, H, H, cin, device=dev)
        dz = torch.randn(B, H, H, cout, device=dev)
        w = torch.randn(cout, 3, 3, cin, device=dev) * 0.05
        bias = torch.randn(cout, device=dev)
        wf = torch.empty(cin * 9 * cout, device=dev)
        lib.pis_conv3x3_flip(w.data_ptr(), wf.data_ptr(), cin, cout, s)
        y = torch.empty(B, H, H, cout, device=dev)
        dx = torch.empty(B, H, H, cin, device=dev)
        nws = 0
        for v in variants:  # the weight-gradient workspace depends on the knob being timed
            pv = lib.pis_tune(args.key, v)
            nws = max(nws, lib.pis_conv3x3_wgrad_ws(B, H, H, cin, cout))
            lib.pis_tune(args.key, pv)
        ws = torch.empty(nws // 4 + 1, device=dev)
        dw = torch.empty(cout * 9 * cin, device=dev)
        db = torch.empty(cout, device=dev)
        prev8 = lib.pis_tune(8, 2)  # workspace for the Winograd path whichever policy / tile is timed
        nwx = 0
        for v in variants:
            pv = lib.pis_tune(args.key, v)
            if args.key != 8:
                nwx = max(nwx, lib.pis_conv3x3_ex_ws(B, H, H, cin, cout))
            lib.pis_tune(args.key, pv)
        nwx = max(nwx, lib.pis_conv3x3_ex_ws(B, H, H, cin, cout))
        lib.pis_tune(8, prev8)
        wsx = torch.empty(max(nwx, 4) // 4 + 1, device=dev)
        flops = 2.0 * B * H * H * cout * cin * 9
        dflags = 0 if name.startswith("dec") and name.endswith("conv0") else 4  # ReLU mask unless a concat input
        ops = {
            "fwd": lambda: lib.pis_conv3x3_fwd_ex(x.data_ptr(), cin, w.data_ptr(), bias.data_ptr(), 0, y.data_ptr(),
                                                  cout, B, H, H, cin, cout, 1, wsx.data_ptr(), nwx, s),
            "dgrad": lambda: lib.pis_conv3x3_dgrad_ex(dz.data_ptr(), cout, wf.data_ptr(), x.data_ptr(), cin, 0,
                                                      dx.data_ptr(), cin, B, H, H, cin, cout, dflags, wsx.data_ptr(),
                                                      nwx, s),
            "wgrad": lambda: lib.pis_conv3x3_wgrad(x.data_ptr(), cin, dz.data_ptr(), cout, dw.data_ptr(),
                                                   db.data_ptr(), B, H, H, cin, cout, 0, ws.data_ptr(), nws, s),
        }
        dbg = [int(d) for d in args.dbg.split(",") if d] or ([1] if args.noload else [])
        vlist = [(v, 0) for v in variants] + [(v, d) for d in dbg for v in variants]
        results = {}
        for _ in range(args.rounds):
            for v, nl in vlist:
                lib.pis_tune(args.key, v)
                lib.pis_tune(NOLOAD_KEY, nl)
                for op in opsel:
                    results.setdefault((op, v, nl), []).append(timed(ops[op]))
        lib.pis_tune(args.key, default)
        lib.pis_tune(NOLOAD_KEY, 0)
        for op in opsel:
            line = f"{name:12s} {op:6s}"
            for v, nl in vlist:
                ms = min(results[(op, v, nl)])
                line += f"  v{v}{f'-d{nl}' if nl else ''}: {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF/s"
            print(line, flush=True)
        del x, dz, w, y, dx, ws, dw
        torch.cuda.empty_cache()


def bench_convt(lib, args, variants, default, s, dev, opsel):
    for name, H, cin, cout in UP_LAYERS:
        x = torch.rand(B, H, H, cin, device=dev)
        dy = torch.randn(B, 2 * H, 2 * H, cout, device=dev)
        w = torch.randn(2, 2, cout, cin, device=dev) * 0.05
        bias = torch.randn(cout, device=dev)
        wc = torch.empty(cin * 4 * cout, device=dev)
        lib.pis_convt2x2_prep(w.data_ptr(), wc.data_ptr(), cin, cout, s)
        y = torch.empty(B, 2 * H, 2 * H, cout, device=dev)
        dx = torch.empty(B, H, H, cin, device=dev)
        nws = lib.pis_convt2x2_wgrad_ws(B, H, H, cin, cout)
        ws = torch.empty(nws // 4 + 1, device=dev)
        dw = torch.empty(4 * cout * cin, device=dev)
        db = torch.empty(cout, device=dev)
        flops = 2.0 * B * H * H * 4 * cout * cin
        ops = {
            "fwd": lambda: lib.pis_convt2x2_fwd(x.data_ptr(), cin, w.data_ptr(), bias.data_ptr(), y.data_ptr(), cout,
                                                B, H, H, cin, cout, s),
            "dgrad": lambda: lib.pis_convt2x2_dgrad(dy.data_ptr(), cout, wc.data_ptr(), x.data_ptr(), cin,
                                                    dx.data_ptr(), cin, B, H, H, cin, cout, 4, s),
            "wgrad": lambda: lib.pis_convt2x2_wgrad(x.data_ptr(), cin, dy.data_ptr(), cout, dw.data_ptr(),
                                                    db.data_ptr(), B, H, H, cin, cout, 0, ws.data_ptr(), nws, s),
        }
        results = {}
        for _ in range(args.rounds):
            for v in variants:
                lib.pis_tune(args.key, v)
                for op in opsel:
                    results.setdefault((op, v), []).append(timed(ops[op]))
        lib.pis_tune(args.key, default)
        for op in opsel:
            line = f"{name:12s} {op:6s}"
            for v in variants:
                ms = min(results[(op, v)])
                line += f"  v{v}: {ms:7.3f} ms {flops / ms / 1e9:6.1f} TF/s"
            print(line, flush=True)


if __name__ == "__main__":
    main()
