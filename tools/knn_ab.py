"""A/B timing of the distance kernel (one library build per process, MIM_LIB selects it).

C3 shape: 96 problems of 10k x 10k (one batch, one context, HIP events on the library stream: the
kernel's own launch duration, `isolated`), then C5 (50k x 50k, mim_knn2_sets_dev).  The kNN rows of a
few C3 problems and of C5 sample rows are saved by the first run (--save) and compared bit for bit by
the others, so a variant that changes any index or distance is reported.
  python tools/knn_ab.py --tag NAME [--save] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cached(name, make):
    p = f"/tmp/knn_ab_{name}.npz"
    if os.path.exists(p):
        with np.load(p) as z:
            return {k: z[k] for k in z.files}
    d = make()
    np.savez(p, **d)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--save", action="store_true")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--c3-only", action="store_true", help="skip C5 and the parity rows (profiling passes)")
    args = ap.parse_args()
    import torch
    from computervision_objectdetection_featurematching_amd import Matcher, default_params
    from computervision_objectdetection_featurematching_amd._lib import SO_PATH
    from computervision_objectdetection_featurematching_amd.synthetic import make_config_dataset, sift_like

    def mk_c3():
        ds = make_config_dataset("c3", seed=0x5EED0000)
        return {"md": np.stack(ds.model_desc), "mk": np.stack(ds.model_kp), "sd": np.stack(ds.scene_desc),
                "sk": np.stack(ds.scene_kp), "pr": np.array(ds.problems)}

    d = cached("c3", mk_c3)
    dev = torch.device("cuda", 0)
    m = Matcher(0)
    out = {"tag": args.tag, "lib": os.path.basename(SO_PATH)}
    md = [torch.from_numpy(x).to(dev) for x in d["md"]]
    mk = [torch.from_numpy(x).to(dev) for x in d["mk"]]
    sd = [torch.from_numpy(x).to(dev) for x in d["sd"]]
    sk = [torch.from_numpy(x).to(dev) for x in d["sk"]]
    torch.cuda.synchronize()
    prm = default_params(max_iters=50000)
    stream = torch.cuda.ExternalStream(m.stream_handle(), device=dev)

    def step():
        with torch.cuda.stream(stream):
            m.clear_sets()
            q = [m.add_set(a, b) for a, b in zip(md, mk)]
            t = [m.add_set(a, b) for a, b in zip(sd, sk)]
            m.match_batch_async([(q[a], t[b]) for a, b in d["pr"]], prm)
            return q, t

    m.set_timing(False)
    step()
    m.batch_results(len(d["pr"]))
    m.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    res = m.batch_results(len(d["pr"]))
    el = time.perf_counter() - t0
    out["c3_knn_ms"] = round(m.kernel_ms("knn") / args.steps, 4)
    out["c3_kernels"] = {k: round(m.kernel_ms(k) / args.steps, 4) for k in
                         ("ratio", "attempt", "chain", "check", "sample", "score", "cand", "exact", "select", "refine")
                         if m.kernel_ms(k) > 0}
    out["c3_step_ms"] = round(1e3 * el / args.steps, 3)
    out["c3_tops"] = round(2.0 * 1e4 * 1e4 * 128 * 96 / (out["c3_knn_ms"] * 1e-3) / 1e12, 1)
    out["c3_frac"] = round(out["c3_tops"] / 5000.0, 4)
    if args.c3_only:
        m.close()
        print(json.dumps(out), flush=True)
        return
    # kNN rows of a few problems (query set 0 vs scene sets 0..3)
    q, t = step()
    m.batch_results(len(d["pr"]))
    rows = {}
    nq = d["md"].shape[1]
    idx = torch.empty((nq, 2), dtype=torch.int32, device=dev)
    dist = torch.empty((nq, 2), dtype=torch.float32, device=dev)
    for s in range(4):
        with torch.cuda.stream(stream):
            m.knn_sets_dev(q[s % 3], t[s], idx, dist)
        m.synchronize()
        rows[f"c3_{s}_i"] = idx.cpu().numpy().copy()
        rows[f"c3_{s}_d"] = dist.cpu().numpy().copy()
    rows["res"] = res.view(np.uint8).copy()
    m.close()

    # C5: 50k x 50k
    def mk_c5():
        rng = np.random.default_rng(0xC5)
        return {"q": sift_like(rng, 50000), "t": sift_like(rng, 50000)}

    c5 = cached("c5", mk_c5)
    m = Matcher(0)
    stream = torch.cuda.ExternalStream(m.stream_handle(), device=dev)
    qd, td = torch.from_numpy(c5["q"]).to(dev), torch.from_numpy(c5["t"]).to(dev)
    kp = torch.zeros((50000, 2), dtype=torch.float32, device=dev)
    idx = torch.empty((50000, 2), dtype=torch.int32, device=dev)
    dist = torch.empty((50000, 2), dtype=torch.float32, device=dev)
    with torch.cuda.stream(stream):
        qs, ts = m.add_set(qd, kp), m.add_set(td, kp)
        m.knn_sets_dev(qs, ts, idx, dist)
    m.synchronize()
    m.set_timing(True)
    for _ in range(args.steps):
        with torch.cuda.stream(stream):
            m.knn_sets_dev(qs, ts, idx, dist)
    m.synchronize()
    m.batch_results(0)
    out["c5_knn_ms"] = round(m.kernel_ms("knn") / args.steps, 4)
    out["c5_tops"] = round(2.0 * 5e4 * 5e4 * 128 / (out["c5_knn_ms"] * 1e-3) / 1e12, 1)
    out["c5_frac"] = round(out["c5_tops"] / 5000.0, 4)
    rows["c5_i"] = idx.cpu().numpy()[::97].copy()
    rows["c5_d"] = dist.cpu().numpy()[::97].copy()
    m.close()

    ref = "/tmp/knn_ab_ref.npz"
    if args.save:
        np.savez(ref, **rows)
        out["parity"] = "reference saved"
    elif os.path.exists(ref):
        with np.load(ref) as z:
            bad = [k for k in z.files if not np.array_equal(z[k].view(np.uint8), rows[k].view(np.uint8))]
        out["parity"] = "identical" if not bad else f"DIFFERS: {bad}"
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
