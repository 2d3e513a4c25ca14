"""Per-kernel counters from rocprofv3 --pmc passes (one pass per counter group: FETCH_SIZE
and WRITE_SIZE do not fit one TCC pass on gfx950, MI355X_MICROARCH.md §rocprofv3 PMC slots).

Derived, per launch (launch-averaged over every dispatch of the kernel in the run):
  * HBM bytes = 2 x FETCH_SIZE x 1024 + WRITE_SIZE x 1024 (gfx950: FETCH_SIZE reports half the
    bytes of a wide coalesced read; WRITE_SIZE is exact for 16-B stores; §HBM);
  * kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the counter over the 8 XCDs);
  * MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs) — the fraction of SIMD-cycles
    the matrix pipe was busy (the MfmaUtil formula of rocprofiler-sdk's counter_defs.yaml,
    with the XCD sum undone);
  * MFMA-busy check: every bf16 MFMA shape retires 1024 FLOP per busy SIMD-cycle
    (32x32x16: 32 cycles; 16x16x32: 16 cycles) and SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 = bf16
    FLOPs, so busy_from_mops = MOPS_BF16 / 2 (+ MOPS_F32 x 512 / 64 for f32-input MFMAs, 64
    FLOP/cycle) must match the busy counter.

    python tools/pmc_summary.py OUT_JSON DOMINANT_SUBSTRING CSV [CSV ...]
"""
import csv
import json
import sys
from collections import defaultdict

SIMDS = 1024  # 256 CUs x 4 SIMDs
XCDS = 8


def read(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for path in paths:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"]
            if "pis::" not in name and "_ZN3pis" not in name:  # some names arrive mangled
                continue
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: (sum(v) / len(v), len(v)) for c, v in cs.items()} for k, cs in acc.items()}


def derive(cs):
    g = lambda c: cs[c][0] if c in cs else None
    out = {c: v for c, (v, _) in cs.items()}
    out["launches"] = max(n for _, n in cs.values())
    f, w = g("FETCH_SIZE"), g("WRITE_SIZE")
    if f is not None and w is not None:
        out["hbm_bytes_per_launch"] = 2.0 * f * 1024 + w * 1024
    cyc = g("GRBM_GUI_ACTIVE")
    busy = g("SQ_VALU_MFMA_BUSY_CYCLES")
    if cyc:
        out["kernel_cycles"] = cyc / XCDS
        if busy is not None:
            out["mfma_busy_frac"] = busy / (cyc / XCDS * SIMDS)
    bf, f32, f16 = (g("SQ_INSTS_VALU_MFMA_MOPS_BF16"), g("SQ_INSTS_VALU_MFMA_MOPS_F32"),
                    g("SQ_INSTS_VALU_MFMA_MOPS_F16"))
    if bf is not None:
        out["mfma_bf16_flop"] = bf * 512
        if f16 is not None:
            out["mfma_f16_flop"] = f16 * 512
        exp = (bf + (f16 or 0.0)) / 2 + (f32 or 0.0) * 512 / 64
        out["busy_cycles_from_mops"] = exp
        if busy:
            out["busy_check_ratio"] = exp / busy
    return out


def main(out_json, dominant, *csvs):
    table = {k: derive(cs) for k, cs in read(csvs).items()}
    dom = [k for k in table if dominant in k]
    nl = sum(table[k]["launches"] for k in dom)

    def weighted(key):
        ks = [k for k in dom if key in table[k]]
        n = sum(table[k]["launches"] for k in ks)
        return sum(table[k][key] * table[k]["launches"] for k in ks) / n if n else None

    out = {"dominant_kernel": " + ".join(dom) if dom else None, "dominant_launches": nl,
           "hbm_bytes_per_launch": weighted("hbm_bytes_per_launch"),
           "mfma_busy_frac": weighted("mfma_busy_frac"),
           "note": "launch-weighted averages over every dispatch of the kernel in the profiled run; "
                   "read bytes = 2 x FETCH_SIZE x 1024 (gfx950 correction), write = WRITE_SIZE x 1024; "
                   "mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)",
           "kernels": table}
    with open(out_json, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in sorted(table.items(), key=lambda kv: -kv[1].get("kernel_cycles", 0) * kv[1]["launches"]):
        hb = v.get("hbm_bytes_per_launch")
        mb = v.get("mfma_busy_frac")
        print(f"x{v['launches']:<4} {'' if hb is None else f'{hb / 1e6:9.2f} MB':>12} "
              f"{'' if mb is None else f'mfma {mb * 100:5.1f}%':>11}  {k[:90]}")


if __name__ == "__main__":
    main(*sys.argv[1:])
