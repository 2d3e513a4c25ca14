"""Per-stream view of the last full training step of a rocprofv3 kernel trace (steps end at the
AdamW kernel): each queue's busy time, the union busy time of the GPU, idle gaps, and the
largest kernels per queue.

    python tools/trace_streams.py gpurun_out/TAG/prof/run_kernel_trace.csv [top]
"""
import csv
import sys
from collections import defaultdict


def main(path, top=12):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # which step from the end (1 = last)
    step = rows[idx[-k - 1] + 1: idx[-k] + 1]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    per_q = defaultdict(list)
    for r in step:
        per_q[r["Queue_Id"]].append(r)
    # union of busy intervals
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
    union, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            union += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    print(f"step span {(t1 - t0) / 1e6:.3f} ms, GPU busy (union) {union / 1e6:.3f} ms")
    for q, rs in sorted(per_q.items(), key=lambda kv: -len(kv[1])):
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
        print(f"queue {q}: {len(rs)} kernels, busy {busy / 1e6:.3f} ms")
        agg = defaultdict(lambda: [0, 0])
        for r in rs:
            k = r["Kernel_Name"].replace("pis::", "").replace("void ", "")[:60]
            agg[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            agg[k][1] += 1
        for k, (ns, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
            print(f"   {ns / 1e6:7.3f} ms  x{n:3d}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
