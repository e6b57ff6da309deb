"""Busy fraction of the GPU over a pipelined bench run's kernel trace (rocprofv3 --kernel-trace csv).

usage: python tools/trace_busy.py run_kernel_trace.csv [skip_first_fraction]

Prints, over the trace window after the first `skip` fraction (warm-up and set-up), the union of the
kernel intervals (time with at least one kernel running) over the window, the summed kernel time per
kernel name (ms) and the gaps' distribution.  Diagnostic only (round 5n: the 32-problem shard).
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t0, t1 = rows[0][0], max(e for _, e, _ in rows)
    w0 = t0 + int(skip * (t1 - t0))
    sel = [(s, e, n) for s, e, n in rows if s >= w0]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = cur_e - sel[0][0]
    per = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n in sel:
        k = n.split("(")[0].replace("void ", "")
        per[k] += (e - s) / 1e6
        cnt[k] += 1
    print(f"window {span / 1e6:.3f} ms, busy union {busy / 1e6:.3f} ms ({busy / span:.4f}), kernels {len(sel)}")
    gaps.sort()
    if gaps:
        tot = sum(gaps)
        print(f"gaps {len(gaps)} total {tot / 1e6:.3f} ms, median {gaps[len(gaps) // 2] / 1e3:.1f} us, "
              f"max {gaps[-1] / 1e3:.1f} us")
    for k, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"{v:10.3f} ms {cnt[k]:6d}  {k}")


if __name__ == "__main__":
    main()
