"""HBM traffic of the roofline kernels from a round's rocprofv3 PMC passes.

usage: python3 tools/traffic_json.py <dir with pmc_FETCH_SIZE/ pmc_WRITE_SIZE/> <out.json> <config>
The passes run `bench.py --config <config> --inflight 1 ...` (one batch at a time), each counter in a
pass of its own.  FETCH_SIZE is doubled (gfx950 tallies a wide coalesced read's 128-B requests at
64 B: MI355X_MICROARCH.md, HBM section).  Reported per launch (mean over the launches of the run) and
per step (the launches of one step: 1 distance kernel, 2 bound kernels).
"""
import collections
import csv
import glob
import json
import sys

src, dst, config = sys.argv[1], sys.argv[2], sys.argv[3]
FAMILY = {"knn2_i8_kernel": "knn2_i8_kernel", "ransac_bound_mfma_kernel": "ransac_bound",
          "ransac_attempt_kernel": "ransac_attempt", "ransac_check_kernel": "ransac_check"}
PER_STEP = {"knn2_i8_kernel": 1, "ransac_bound": 2, "ransac_attempt": 2, "ransac_check": 2}
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for counter, scale in (("FETCH_SIZE", 2), ("WRITE_SIZE", 1)):
    for f in sorted(glob.glob(f"{src}/pmc_{counter}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0].replace("void ", "").strip()
            fam = FAMILY.get(name)
            if fam:  # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
                vals[fam][counter].append(float(r["Counter_Value"]) * 1024 * scale)
out = {"config": config,
       "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes) of "
                 f"bench.py --config {config} --inflight 1",
       "units": "bytes (counter KiB x 1024); FETCH_SIZE doubled for gfx950 wide reads (MI355X_MICROARCH.md)",
       "kernels": {}}
for fam, d in vals.items():
    f, w = d.get("FETCH_SIZE", []), d.get("WRITE_SIZE", [])
    if not f or not w:
        continue
    per_launch = sum(f) / len(f) + sum(w) / len(w)
    out["kernels"][fam] = {"launches": len(f), "fetch_bytes_per_launch": sum(f) / len(f),
                           "write_bytes_per_launch": sum(w) / len(w), "hbm_bytes_per_launch": per_launch,
                           "hbm_bytes_per_step": per_launch * PER_STEP[fam]}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
