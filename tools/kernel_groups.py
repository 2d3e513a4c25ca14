"""Per-step kernel time by group from a rocprofv3 kernel trace (steps end at the AdamW kernel):
the average over the last K full steps of the summed durations of every kernel whose name
contains a group's pattern, and the launch count.

    python tools/kernel_groups.py gpurun_out/TAG/prof/run_kernel_trace.csv [K] [pattern ...]
"""
import csv
import sys
from collections import defaultdict

DEFAULT = ["reduce_slabs", "reduce_rows_chunk", "conv3x3_wgrad_h3", "gemm_nt_h3_bk32", "wgrad_h3t", "wgrad_x6",
           "conv3x3_h3_kernel", "convt_h3", "wino4_dz2", "wino4_output", "wino4_input", "wino4_wgrad_out",
           "wino4_gemm_out", "maxpool_bwd", "head_loss", "adamw"]


def main(path, k=4, pats=None):
    pats = pats or DEFAULT
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    k = min(k, len(idx) - 1)
    tot, cnt = defaultdict(float), defaultdict(int)
    busy = 0.0
    for s in range(len(idx) - k, len(idx)):
        for r in rows[idx[s - 1] + 1: idx[s] + 1]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            busy += d
            for p in pats:
                if p in r["Kernel_Name"]:
                    tot[p] += d
                    cnt[p] += 1
                    break
    print(f"{'group':24s} {'us/step':>10s} {'launches':>9s}")
    for p in pats:
        print(f"{p:24s} {tot[p] / k:10.1f} {cnt[p] / k:9.1f}")
    print(f"{'all kernels':24s} {busy / k:10.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 4, sys.argv[3:] or None)
