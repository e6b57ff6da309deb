"""Busy fraction of the GPU over a pipelined bench run's kernel trace (rocprofv3 --kernel-trace csv).

usage: python tools/trace_busy.py run_kernel_trace.csv [skip_first_fraction]
       python tools/trace_busy.py run_kernel_trace.csv --timed WARMUP STEPS

First form: over the trace window after the first `skip` fraction (warm-up and set-up), the union of
the kernel intervals (time with at least one kernel running) over the window, the summed kernel time
per kernel name (ms) and the gaps' distribution.  Second form: the timed region of a bench.py run
(from the distance kernel of step WARMUP to the refine of step WARMUP + STEPS - 1, counting launches),
its busy union, and for the main kernels the fraction of that region in which at least one launch of
the kernel is running (round 5n: the 32-problem shard against the full C4 batch).  Diagnostic only.
"""
import csv
import sys
from collections import defaultdict


def union(iv):
    tot, cs, ce = 0, None, None
    gaps = []
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
                gaps.append(s - ce)
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot, gaps


def main():
    path = sys.argv[1]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if len(sys.argv) > 2 and sys.argv[2] == "--timed":
        warm, steps = int(sys.argv[3]), int(sys.argv[4])
        knn = [r for r in rows if "knn2_i8_kernel" in r[2]]
        ref = [r for r in rows if "ransac_refine_kernel" in r[2]]
        t0, t1 = knn[warm][0], ref[warm + steps - 1][1]
        sel = [r for r in rows if r[0] >= t0 and r[1] <= t1]
        span = t1 - t0
        busy, _ = union([(s, e) for s, e, _ in sel])
        print(f"timed region {span / 1e6:.2f} ms ({span / 1e6 / steps:.3f} ms per step), busy union {busy / span:.3f}")
        for key in ("knn2_i8_kernel", "ransac_bound_mfma_kernel<false>", "ransac_exact_kernel", "ransac_refine_kernel"):
            iv = [(s, e) for s, e, n in sel if key in n]
            u, _ = union(iv)
            print(f"  {key:34s} running {u / span:.3f} of the region, mean launch {sum(e - s for s, e in iv) / max(len(iv), 1) / 1e6:.3f} ms")
        return
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    w0 = t0 + int(skip * (t1 - t0))
    sel = [(s, e, n) for s, e, n in rows if s >= w0]
    busy, gaps = union([(s, e) for s, e, _ in sel])
    span = max(e for _, e, _ in sel) - sel[0][0]
    per = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in sel:
        k = n.split("(")[0].replace("void ", "")
        per[k] += (e - s) / 1e6
        cnt[k] += 1
    print(f"window {span / 1e6:.3f} ms, busy union {busy / 1e6:.3f} ms ({busy / span:.4f}), kernels {len(sel)}")
    gaps.sort()
    if gaps:
        print(f"gaps {len(gaps)} total {sum(gaps) / 1e6:.3f} ms, median {gaps[len(gaps) // 2] / 1e3:.1f} us, "
              f"max {gaps[-1] / 1e3:.1f} us")
    for k, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{v:10.3f} ms {cnt[k]:6d}  {k}")


if __name__ == "__main__":
    main()
