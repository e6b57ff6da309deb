"""Sum rocprofv3 counter_collection.csv files per (kernel, counter); print per-dispatch means."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmck"
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
dur = {}
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
        agg[k] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for (kn, cn), v in sorted(agg.items()):
    n = len(disp[(kn, cn)])
    print(f"{kn:40s} {cn:28s} total {v:16.0f}  per-dispatch {v / max(n, 1):14.0f}  ({n} dispatches)")
for f in sorted(glob.glob(f"{root}/p*/run_kernel_trace.csv"))[:1]:
    ds = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        ds[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, v in ds.items():
        print(f"{k:40s} dispatch ms: {', '.join(f'{x:.3f}' for x in v)}")
