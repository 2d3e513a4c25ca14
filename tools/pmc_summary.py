"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE
are collected in separate passes: they do not fit one TCC pass on gfx950).

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a
wide coalesced read on gfx950, so read bytes = 2 x FETCH_SIZE x 1024;
WRITE_SIZE x 1024 is exact for 16-B streaming stores.

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV OUT_JSON [dominant-substring]
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        if not name.startswith("void pis::") and not name.startswith("pis::"):
            continue
        acc[name].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(fetch_csv, write_csv, out_json, dominant="gemm_nt_x6_"):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    table = {}
    for k in sorted(set(f) | set(w)):
        fk = f.get(k, (0.0, 0))[0]
        wk = w.get(k, (0.0, 0))[0]
        table[k] = {"fetch_size_kib": fk, "write_size_kib": wk,
                    "read_bytes_corrected": 2.0 * fk * 1024, "write_bytes": wk * 1024,
                    "hbm_bytes_per_launch": 2.0 * fk * 1024 + wk * 1024,
                    "launches": max(f.get(k, (0, 0))[1], w.get(k, (0, 0))[1])}
    dom = [k for k in table if dominant in k]
    # every instantiation of the dominant kernel, launch-weighted
    nl = sum(table[k]["launches"] for k in dom)
    per_launch = sum(table[k]["hbm_bytes_per_launch"] * table[k]["launches"] for k in dom) / nl if nl else None
    out = {"dominant_kernel": " + ".join(dom) if dom else None,
           "hbm_bytes_per_launch": per_launch,
           "note": "per-launch average over every launch of the kernel in the profiled run; "
                   "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 correction), write = WRITE_SIZE x 1024",
           "kernels": table}
    with open(out_json, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in sorted(table.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  x{v['launches']:<4} {k[:80]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
