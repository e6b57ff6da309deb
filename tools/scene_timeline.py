"""Timeline of single scenes from a rocprofv3 kernel trace of `bench.py --config c1img --inflight 1`.

usage: python tools/scene_timeline.py run_kernel_trace.csv [n_last_scenes]

A scene (pipeline.detect_objects) ends with its inlier_gather_kernel; the next scene starts with the
first kernel after it.  For each of the last n scenes: its span, the union of kernel time, the idle
time (no kernel running: host work, synchronisations, launch gaps) and the time by phase (SIFT + resize,
distance + ratio + prep, RANSAC sampler/selection, refine, gather), then the kernel list of the last
scene with start offsets and durations (diagnostic only).
"""
import csv
import sys


def phase(name):
    if "anonymous namespace" in name:
        return "sift"
    if "knn" in name or "ratio" in name or "prep_batch" in name:
        return "match"
    if "refine" in name:
        return "refine"
    if "inlier_gather" in name:
        return "gather"
    if "ransac" in name or "rng_stream" in name:
        return "ransac"
    return "other"


def union(iv):
    tot, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    ends = [i for i, r in enumerate(rows) if "inlier_gather_kernel" in r[2]]
    scenes = []
    for a, b in zip(ends[:-1], ends[1:]):
        scenes.append(rows[a + 1:b + 1])
    for sc in scenes[-n_last:]:
        t0, t1 = sc[0][0], max(e for _, e, _ in sc)
        span = t1 - t0
        busy = union([(s, e) for s, e, _ in sc])
        by = {}
        for s, e, n in sc:
            by.setdefault(phase(n), []).append((s, e))
        parts = ", ".join(f"{k} {union(v) / 1e6:.3f} ({min(s for s, _ in v) - t0:.0f}..{max(e for _, e in v) - t0:.0f} ns)"
                          for k, v in by.items())
        print(f"scene: span {span / 1e6:.3f} ms, kernels busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms, "
              f"{len(sc)} kernels; {parts}")
    sc = scenes[-1]
    t0 = sc[0][0]
    prev_end = t0
    print("\nlast scene, kernel by kernel (start offset us, duration us, gap before us):")
    for s, e, n in sc:
        short = n.replace("mim::(anonymous namespace)::", "sift::").split("(")[0].replace("mim::", "")
        print(f"  {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev_end) / 1e3:8.1f}  {short}")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
