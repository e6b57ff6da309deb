"""Per-kernel average launch duration of a rocprofv3 kernel trace of the default bench, split into
bench.py's phases by launch order: warm-up steps, the K timed steps, the K isolated steps.
usage: prof_window.py <kernel_trace.csv> <bench json log> [kernel-regex ...]"""
import csv
import json
import re
import sys

trace, log = sys.argv[1], sys.argv[2]
pats = sys.argv[3:] or [r"knn2_i8_kernel", r"ransac_bound_mfma_kernel<false>"]
b = json.loads([l for l in open(log) if l.startswith("{")][-1])
K, W = b["steps"], max(b["warmup"], b["config"].get("batches_in_flight", 1))
rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
out = {"trace": trace, "steps": K, "warmup_steps": W}
for p in pats:
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if re.search(p, r["Kernel_Name"])]
    per = len(d) // (W + 2 * K) if d else 0  # launches per step
    if per == 0:
        continue
    timed, iso = d[W * per:(W + K) * per], d[(W + K) * per:(W + 2 * K) * per]
    out[p] = {"launches": len(d), "per_step": per,
              "timed_avg_ms": round(sum(timed) / len(timed), 4), "isolated_avg_ms": round(sum(iso) / len(iso), 4)}
r = b["roofline"]
out["bench_hip_events_ms_per_step"] = {"knn": r["kernel_ms_per_step"]["knn"], "knn_isolated": r["isolated_kernel_ms_per_step"]["knn"],
                                       "score": r["kernel_ms_per_step"]["score"], "score_isolated": r["isolated_kernel_ms_per_step"]["score"]}
print(json.dumps(out, indent=1))
