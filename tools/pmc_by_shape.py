"""MFMA-busy fraction of one kernel's launches grouped by grid size (= layer shape) from a
rocprofv3 --pmc run with SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/gpu_round.sh pmc_mfma):
busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), as tools/pmc_summary.py.

    python tools/pmc_by_shape.py gpurun_out/TAG/pmc_mfma/run_counter_collection.csv gemm_nt_h3_bk32
"""
import csv
import sys
from collections import defaultdict

SIMDS = 1024


def main(path, substr):
    per = defaultdict(dict)  # dispatch -> counters
    meta = {}
    for r in csv.DictReader(open(path)):
        if substr not in r["Kernel_Name"]:
            continue
        d = r["Dispatch_Id"]
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    groups = defaultdict(list)
    for d, c in per.items():
        if "GRBM_GUI_ACTIVE" in c and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            cyc = c["GRBM_GUI_ACTIVE"] / 8
            groups[meta[d][0]].append((c["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS), meta[d][1]))
    print(f"{substr}: MFMA busy by grid size (threads; blocks = threads / 256)")
    for g, v in sorted(groups.items()):
        busy = sum(b * t for b, t in v) / sum(t for _, t in v)
        print(f"  grid {g:>10} ({g // 256:>6} blocks)  launches {len(v):3d}  busy {100 * busy:5.1f} %  "
              f"avg {sum(t for _, t in v) / len(v) / 1e3:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
