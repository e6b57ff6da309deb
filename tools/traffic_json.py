"""HBM traffic per step of the roofline kernels from the round's rocprofv3 PMC passes.

usage: python3 tools/traffic_json.py gpurun_out/prof_round profiles/r01_pmc_traffic.json
Reads pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/ (separate passes of `bench.py --steps 1 --warmup 0`),
doubles FETCH_SIZE (gfx950 tallies 128-B requests at 64 B: MI355X_MICROARCH.md, HBM section) and sums
the launches of one step per kernel family ("ransac_bound" = the MFMA bound kernel of both chunks).
"""
import collections
import csv
import glob
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
FAMILY = {"knn2_i8_kernel": "knn2_i8_kernel", "ransac_bound_mfma_kernel": "ransac_bound",
          "ransac_attempt_kernel": "ransac_attempt", "ransac_check_kernel": "ransac_check"}
per = collections.defaultdict(lambda: {"fetch_size_per_launch": [], "write_size_per_launch": []})
for counter, key, scale in (("FETCH_SIZE", "fetch_size_per_launch", 2), ("WRITE_SIZE", "write_size_per_launch", 1)):
    for f in sorted(glob.glob(f"{src}/pmc_{counter}/**/*counter_collection.csv", recursive=True)):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0].replace("void ", "").strip()
            fam = FAMILY.get(name)
            if fam:
                # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
                per[fam][key].append(float(r["Counter_Value"]) * 1024 * scale)
out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes), "
                 "python3 bench.py --steps 1 --warmup 0 --no-timing (C3, 96 problems)",
       "units": "bytes per launch (counter KiB x 1024); FETCH_SIZE doubled for gfx950 wide reads "
                "(MI355X_MICROARCH.md HBM section)",
       "kernels": {}}
for fam, d in per.items():
    d["hbm_bytes_per_step"] = sum(d["fetch_size_per_launch"]) + sum(d["write_size_per_launch"])
    out["kernels"][fam] = d
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
