"""CPU baselines of SURVEY §8(d) on this host: the oracle (stock-PyTorch CPU restatement of the
reference step, oracle/reference_torch.py) at C1 (B=2, 256^2, Stage I) and C2 (B=8, 512^2,
Stage II), 1 warm-up step + median of 3, on the host's usable CPUs (affinity mask capped by the
cgroup CPU quota). Prints one JSON line per config (for BASELINE.md §2).

    python tools/cpu_baseline.py [--configs c1,c2]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2")
    args = ap.parse_args()
    import importlib.util
    spec = importlib.util.spec_from_file_location("pis_bench", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    cfg = {"c1": dict(batch=2, size=256, loss_kw=dict(), lr=1e-4),
           "c2": dict(batch=8, size=512, loss_kw=dict(rd_w=1e-4, pf_w=1e-4, D=5.0, a=0.5, eps=0.05), lr=1e-5)}
    for name in args.configs.split(","):
        out = bench.cpu_baseline(**cfg[name])
        out["config"] = name
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
