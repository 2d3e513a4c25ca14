"""Print the kernel timeline of the last full training step of a rocprofv3
kernel trace (steps are delimited by the AdamW kernel).

    python tools/trace_step.py gpurun_out/prof1/run_kernel_trace.csv [min_us]
"""
import csv
import sys


def main(path, min_us=0.0):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    s, e = idx[-2] + 1, idx[-1] + 1
    step = rows[s:e]
    busy = 0.0
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy += d
        if d >= min_us:
            name = r["Kernel_Name"].replace("pis::", "")[:70]
            print(f"{d:10.1f} us  wg={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']):>7}  "
                  f"vgpr={r['VGPR_Count']:>3}/{r['Accum_VGPR_Count']:>3}  {name}")
    span = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
    print(f"kernels {len(step)}  busy {busy / 1e3:.2f} ms  span {span / 1e3:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.0)
