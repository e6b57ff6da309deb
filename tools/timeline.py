"""Print the kernel timeline of the last bench step from a rocprofv3 kernel_trace.csv.

usage: python3 tools/timeline.py gpurun_out/prof2/.../run_kernel_trace.csv
"""
import csv
import glob
import sys

path = sys.argv[1] if len(sys.argv) > 1 else sorted(glob.glob("gpurun_out/prof2/**/*kernel_trace.csv", recursive=True))[-1]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
first = [i for i, r in enumerate(rows) if "prep_batch" in r["Kernel_Name"]]
s = first[-1] if first else 0
t0 = int(rows[s]["Start_Timestamp"])
for r in rows[s:]:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mim::", "")
    a = (int(r["Start_Timestamp"]) - t0) / 1e3
    b = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{a:9.1f} {b:9.1f} {b - a:8.1f}  {n}")
