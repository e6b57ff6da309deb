"""GPU busy fraction from a rocprofv3 kernel trace: the union of kernel intervals over a time window
(default: the whole trace), and the busiest kernels by summed duration.
usage: python tools/busy_frac.py <run_kernel_trace.csv> [t0_frac t1_frac]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
lo, hi = iv[0][0], max(e for _, e, _ in iv)
f0, f1 = (float(sys.argv[2]), float(sys.argv[3])) if len(sys.argv) > 3 else (0.0, 1.0)
w0, w1 = lo + f0 * (hi - lo), lo + f1 * (hi - lo)
busy, cur_s, cur_e = 0, None, None
tot = defaultdict(float)
for s, e, n in iv:
    s, e = max(s, w0), min(e, w1)
    if e <= s:
        continue
    tot[n.replace("(anonymous namespace)::", "").split("(")[0][:50]] += (e - s) / 1e6
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += cur_e - cur_s
print(f"window {(w1 - w0) / 1e6:.2f} ms, GPU busy (union of kernels) {busy / 1e6:.2f} ms = {busy / (w1 - w0):.3f}")
for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:15]:
    print(f"  {n:50s} {t:9.2f} ms")
