"""Per-step stream view of a rocprofv3 kernel trace (test/analysis tooling): for the last full
training step (adamw_kernel to adamw_kernel) the step time, the GPU-busy union, the idle gaps, and
per stream the kernel count and busy time; with --list, the main stream's kernels in order with the
gap before each and whether the other stream was running meanwhile.

    python tools/stream_timeline.py run_kernel_trace.csv [--list]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ad = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    seg = rows[ad[-3] + 1:ad[-2] + 1]
    t0, t1 = int(rows[ad[-3]]["End_Timestamp"]), int(rows[ad[-2]]["End_Timestamp"])
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg)
    busy, cur, gaps = 0, None, []
    for a, b in iv:
        if cur is None:
            cur = [a, b]
        elif a <= cur[1]:
            cur[1] = max(cur[1], b)
        else:
            busy += cur[1] - cur[0]
            gaps.append(a - cur[1])
            cur = [a, b]
    busy += cur[1] - cur[0]
    print(f"step {(t1 - t0) / 1e3:.1f} us  GPU busy {busy / 1e3:.1f} us  idle gaps {len(gaps)} "
          f"sum {sum(gaps) / 1e3:.1f} us")
    by = {}
    for r in seg:
        s = by.setdefault(r["Stream_Id"], [0, 0])
        s[0] += 1
        s[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, (n, t) in sorted(by.items()):
        print(f"stream {k}: {n} kernels, {t / 1e3:.1f} us")
    if "--list" in sys.argv:
        main_id = max(by, key=lambda k: by[k][0])
        others = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in seg if r["Stream_Id"] != main_id]
        prev = t0
        for r in seg:
            if r["Stream_Id"] != main_id:
                continue
            a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            ov = sum(max(0, min(b, y) - max(a, x)) for x, y in others)
            nm = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pis::", "")[:56]
            print(f"{(a - prev) / 1e3:6.1f} gap {(b - a) / 1e3:8.1f} us  side-overlap {ov / 1e3:7.1f}  {nm}")
            prev = b


if __name__ == "__main__":
    main()
