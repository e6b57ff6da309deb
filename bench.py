#!/usr/bin/env python3
"""Benchmark: matches+homographies/sec (10k x 10k SIFT, 50k RANSAC iters) — BASELINE.json metric.

One step = one pass of the hot path (knnMatch k=2 + ratio test + findHomography RANSAC + refine +
gates, /root/reference/src/TestsDetector.cpp:58-95) over one batch of problems.  Configs
(BASELINE.json `configs`; `--config`, default c3):
  c3  configs[2]: 3 model descriptor sets x 32 scene sets per GPU, 10,000 x 10,000 128-D SIFT-like
      descriptors per problem, RANSAC maxIters 50,000, conf 0.995, 8 % geometric inliers among 2,000
      planted matches (no early termination: SURVEY.md App. B).  C4 (configs[3]) is this workload
      with --gpus 8: every rank owns its own 32 scenes.
  c2  configs[1]: 1 x 1, 2k x 2k, maxIters 2000.
  c1  configs[0] surrogate: the reference's own shape, one scene = 29 model views x 5 scales = 145
      ragged problems (Nq 100-500, Nt 1k-4k, maxIters 2000); the real data needs SIFT.
  c5  configs[4]: the 50k x 50k dense distance contraction alone (mim_knn2_sets_dev), no RANSAC.
  c1img  configs[0] on the reference's own images (tests/golden/c1_sugar_box.npz): the sugar_box model
      (29 views, SIFT computed once before the timed region as processAllModelsImages does) against one
      test view per step through detectObjects: 5 x (resize + SIFT) on the GPU, the 145 problems as one
      device batch, clustering and boxes on the host (pipeline.detect_objects).
Inputs (descriptors + keypoints) are resident in HBM before the timed region; each step registers
the sets (the i8 layout prep is inside the step) and runs the batch.  Multi-GPU: one process per GPU
(`--gpus N` launches N ranks through torch.distributed.run when WORLD_SIZE is unset), each rank
owns its own scenes (weak scaling, no data-path collective); the per-problem result records are
all-gathered over RCCL at the end of every step.  Twelve scene batches are in flight on one GPU
(--inflight).

Prints ONE JSON line on rank 0 with, besides the contract fields: "roofline" (dominant kernel, HIP
events on the library's stream), "cpu_baseline" (oracle/ restatement on this host's cores, bounded
sample, with a "parity" check of those problems against the GPU records) and "ranks_seen".
`--dry-run` exercises the launcher and the gloo/RCCL record gather without a GPU (CPU test).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_I8_TOPS = 5000.0       # MI355X dense i8 MFMA = 2x dense bf16 2.5 PF (MI355X_MICROARCH.md, no sparsity)
PEAK_F32_VALU_TFLOPS = 157.3  # MI355X fp32 vector (VALU) peak
FLOP_PER_POINT_EVAL = 17      # one fp32 reprojection test of a hypothesis on a point
H_TOL = 1e-4                  # SURVEY.md 8(c) contract item 4 (the GPU tests hold 1e-7)


def pmc_traffic(kernel, config):
    """HBM bytes per step of `kernel` from the newest committed rocprofv3 PMC pass (or None)."""
    for rnd in ("r02", "r01"):
        try:
            with open(os.path.join(ROOT, "profiles", f"{rnd}_pmc_traffic.json")) as f:
                d = json.load(f)
            if d.get("config", "c3") != config:
                continue
            return d["kernels"][kernel]["hbm_bytes_per_step"]
        except (OSError, KeyError, ValueError):
            continue
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=["c1", "c1img", "c2", "c3", "c5"])
    ap.add_argument("--cpu-sample", type=int, default=6,
                    help="problems of the sequential CPU-baseline sample (1 warm-up + the median of the rest; "
                         "0: skip the CPU baseline)")
    ap.add_argument("--cpu-rounds", type=int, default=5, help="timed rounds of the parallel CPU row")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--inflight", type=int, default=0,
                    help="scene batches in flight: one library context + HIP stream each, steps assigned "
                         "round-robin, so a batch's latency-bound RANSAC tail overlaps the next batch's kNN "
                         "(0: 12, c1 3; with GPU_MAX_HW_QUEUES=16 their streams, torch's and RCCL's each get a "
                         "hardware queue)")
    ap.add_argument("--hw-queues", type=int, default=16,
                    help="GPU_MAX_HW_QUEUES for this process and the ranks it launches (set before HIP initialises)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: launch the ranks, gather fake records over gloo, print the JSON line")
    return ap.parse_args()


# ------------------------------------------------------------------------------------------------
# launcher: N ranks of this script, started before anything touches the GPU
# ------------------------------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """`python bench.py --gpus N` without WORLD_SIZE: run N ranks via torch.distributed.run as child
    processes (this process never initialises the GPU) and return the launcher's exit code."""
    argv = [a for a in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def dist_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def dry_run(args):
    """Launcher + process group + record gather on gloo (CPU): what the N-rank bench does around its
    GPU work.  Prints the JSON line with n_gpus / ranks_seen so a CPU test can check the launch."""
    import torch
    import torch.distributed as dist

    from computervision_objectdetection_featurematching_amd import shard
    from computervision_objectdetection_featurematching_amd._lib import RESULT_DTYPE

    rank, world, _ = dist_env()
    if world > 1:
        dist.init_process_group("gloo")
    seen = dist.get_world_size() if world > 1 else 1
    if seen != args.gpus:
        raise SystemExit(f"rank {rank}: process group has {seen} ranks, --gpus {args.gpus}")
    rec = np.zeros(4, RESULT_DTYPE)
    rec["n_good"] = 1000 * rank + np.arange(4)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    g = shard.decode(shard.gather_results(torch.from_numpy(rec.view(np.uint8).copy()), world))
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        assert g.shape == (world, 4) and list(g["n_good"][:, 0]) == [1000 * r for r in range(world)]
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "problems/s", "n_gpus": world,
                          "ranks_seen": seen, "steps": 0, "warmup": 0, "ms_per_step": float(t.item()) * 1e3,
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dry_run": True}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


# ------------------------------------------------------------------------------------------------
# CPU baseline: the oracle (CPU restatement of OpenCV 4.5.4) on this host, plus parity of the sample
# ------------------------------------------------------------------------------------------------
def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """Host threads for the CPU baseline: the GPU box's CPU share (OMP_NUM_THREADS, 16 per GPU there;
    nproc shows the whole machine), else every core this process may run on."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _cmp_problem(o, r, det):
    """First difference between an oracle record and the GPU record/detail of one problem, or None."""
    gq, gt, gm = det
    if int(r["n_good"]) != o["n_good"]:
        return f"n_good {int(r['n_good'])} vs {o['n_good']}"
    if not (np.array_equal(gq, o["good_q"]) and np.array_equal(gt, o["good_t"])):
        return "good-match lists"
    if int(r["status"]) != o["status"] or int(r["n_inl"]) != o["n_inl"] or int(r["iters"]) != o["iters"]:
        return f"status/n_inl/iters {(int(r['status']), int(r['n_inl']), int(r['iters']))} vs " \
               f"{(o['status'], o['n_inl'], o['iters'])}"
    if len(o["mask"]) and not np.array_equal(gm, o["mask"]):
        return "inlier mask"
    Ho = o["H"]
    if np.any(Ho != 0) and np.max(np.abs(r["H"].reshape(3, 3) - Ho) / (np.abs(Ho) + 1e-3)) > H_TOL:
        return "H"
    return None


def cpu_baseline_problems(ds, cfg, gpu_res, gpu_detail, n_sample, rounds):
    """Reference-style leg: problems one after another, kNN on all host cores (OpenCV parallel_for_),
    RANSAC single-threaded (cv::findHomography); 1 warm-up problem, value = 1 / median of the others.
    Parallel leg ("best effort"): one problem per core at once (ctypes releases the GIL), 1 warm-up
    round + `rounds` timed rounds, median.  Every oracle record is compared with the GPU's."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O
    O.build()
    cores = host_cores()
    prm = O.default_params(max_iters=cfg["max_iters"])
    P = ds.problems
    checked, mismatches = {}, []

    def run(i, threads):
        m, s = P[i]
        o = O.match_problem(ds.model_desc[m], ds.model_kp[m], ds.scene_desc[s], ds.scene_kp[s], prm, threads)
        if i not in checked:
            d = _cmp_problem(o, gpu_res[i], gpu_detail(i))
            checked[i] = d
            if d:
                mismatches.append((i, d))
        return o

    ids = [(7 * k) % len(P) for k in range(max(n_sample, 2))]
    times = []
    for i in ids:
        t0 = time.perf_counter()
        run(i, cores)
        times.append(time.perf_counter() - t0)
        log(f"cpu baseline: problem {i} {times[-1]:.2f} s")
    seq = 1.0 / statistics.median(times[1:])
    par_times = []
    with ThreadPoolExecutor(cores) as ex:
        for rnd in range(rounds + 1):
            batch = [(rnd * cores + k) % len(P) for k in range(cores)]
            t0 = time.perf_counter()
            list(ex.map(lambda i: run(i, 1), batch))
            if rnd:
                par_times.append(time.perf_counter() - t0)
            log(f"cpu baseline: parallel round {rnd} {time.perf_counter() - t0:.2f} s")
    par = cores / statistics.median(par_times)
    return {"value": round(seq, 4), "unit": "problems/s", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{len(ids)} problems of the same workload one after another (1 warm-up, median of "
                      f"{len(ids) - 1}): kNN on {cores} threads like OpenCV parallel_for_, RANSAC single-threaded "
                      f"as cv::findHomography; oracle/mim_oracle.c -O3 -ffp-contract=off",
            "parallel": {"value": round(par, 4), "unit": "problems/s", "cores": cores,
                         "sample": f"{cores} problems at once, one per core (kNN and RANSAC single-threaded), "
                                   f"1 warm-up + {rounds} rounds, median"},
            "parity": {"checked": len(checked), "mismatch": len(mismatches),
                       "first": mismatches[0] if mismatches else None}}


def cpu_baseline_knn(q, t, idx_gpu, dist_gpu, n_rows):
    """C5: the oracle's batchDistance(K=2) restatement on all host cores over n_rows query rows of the
    50k set against the full 50k train set (1 warm-up + median of 5), bit-compared with the GPU rows."""
    from oracle import oracle as O
    O.build()
    cores = host_cores()
    rows = np.linspace(0, q.shape[0] - 1, n_rows).astype(np.int64)
    times = []
    mism = 0
    for r in range(6):
        sub = rows[r::6] if r else rows[:max(1, n_rows // 6)]
        t0 = time.perf_counter()
        i_o, d_o = O.knn2(q[sub], t, cores)
        times.append((time.perf_counter() - t0) / len(sub))
        mism += int(np.sum(np.any(i_o != idx_gpu[sub], axis=1) | np.any(d_o.view(np.int32) != dist_gpu[sub].view(np.int32),
                                                                        axis=1)))
    per_row = statistics.median(times[1:])
    ops = 2.0 * t.shape[0] * 128
    return {"value": round(ops / per_row / 1e9, 3), "unit": "GOP/s (distance)", "cores": cores, "kind": "port",
            "cpu_model": cpu_model(),
            "sample": f"{n_rows} query rows x {t.shape[0]} train rows in 6 slices (1 warm-up, median of 5) on "
                      f"{cores} threads, oracle batchDistance restatement",
            "problems_per_s_equiv": round(1.0 / (per_row * q.shape[0]), 6),
            "parity": {"checked": int(n_rows + max(1, n_rows // 6)), "mismatch": mism}}


# ------------------------------------------------------------------------------------------------
def run_c1img(args, rank, world, local):
    """configs[0] on the reference's images, one scene per step (see the module docstring)."""
    import torch
    import torch.distributed as dist

    from computervision_objectdetection_featurematching_amd import Matcher, build
    from computervision_objectdetection_featurematching_amd.pipeline import SCALES, detect_objects, process_model_views

    build.build()
    with np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden", "c1_sugar_box.npz")) as z:
        d = {k: z[k] for k in z.files if not k.startswith("exp/")}
    names = sorted(k[5:] for k in d if k.startswith("view/"))
    scenes = sorted(k[6:] for k in d if k.startswith("scene/"))
    # scenes in flight: one library context (own streams and device copy of the model's sets) per
    # host thread; a scene's host stages and synchronisations overlap the other scenes' GPU work (the
    # C ABI calls release the GIL).  The model (host arrays) is computed once and shared.
    nf = args.inflight if args.inflight > 0 else 12
    ms = [Matcher(local) for _ in range(nf)]
    for mm in ms:  # the scenes overlap each other: one stream per context (12, sampler off: 163 scenes/s
        mm.set_sampler_stream(nf == 1)  # vs 131 with it on, 101 at 3 in flight)
    m = ms[0]
    model = process_model_views(m, "004_sugar_box", [(d[f"view/{n}"], d[f"mask/{n}"]) for n in names])
    models = [model] * nf
    sid = scenes[rank % len(scenes)]
    scene = d[f"scene/{sid}"]
    n_probs = len(SCALES) * len(names)
    for mm, md in zip(ms[1:], models[1:]):
        detect_objects(mm, scene, [md])
    for _ in range(max(args.warmup, 1)):
        run = detect_objects(m, scene, [model], keep=True)
    for mm in ms:
        mm.set_timing(not args.no_timing)
    out_dets = [None] * nf

    def worker(k):
        for _ in range(k, args.steps, nf):
            out_dets[k] = detect_objects(ms[k], scene, [models[k]])

    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(nf)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    list(pool.map(worker, range(nf)))
    torch.cuda.synchronize()
    pool.shutdown()
    dets = out_dets[0]
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=torch.device("cuda", local))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    # SIFT of one 640x480 image alone (the step's dominant stage), timed separately
    ts = []
    for _ in range(5):
        t1 = time.perf_counter()
        m.sift_detect_compute(scene)
        ts.append(time.perf_counter() - t1)
    if rank == 0:
        out = {"metric": "matches+homographies/sec (configs[0]: sugar_box model vs one test view, reference images, "
                         "SIFT + match + RANSAC + boxes)",
               "value": round(world * n_probs * args.steps / el, 3), "unit": "problems/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "f32 SIFT (OpenCV order), i8-MFMA exact-int distances, fp64 DLT/LM, fp32 reprojection",
               "data": "reference images: 29 sugar_box model views + masks, test view " + sid,
               "config": {"workload": f"c1img: detectObjects of one 640x480 scene against {len(names)} views x "
                                      f"{len(SCALES)} scales = {n_probs} problems per step per GPU",
                          "problems_per_gpu": n_probs, "global_batch": world * n_probs, "parallelism": f"dp{world}",
                          "scenes_in_flight": nf},
               "scenes_per_s": round(world * args.steps / el, 3),
               "sift_640x480_ms": round(1e3 * statistics.median(ts), 3),
               "detections_rank0": [list(b) for b, _ in dets],
               "accepted_problems_rank0": int((run.results["status"] == 0).sum())}
        if args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline_c1img(scene, model, run, names)
            out["parity"] = out["cpu_baseline"]["parity"]
        print(json.dumps(out), flush=True)
    for mm in ms:
        mm.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_c1img(scene, model, run, names):
    """The oracle pipeline for the same scene, one core: resize + SIFT per scale, then the 145
    problems (kNN + ratio + RANSAC + refine) one after another; every record compared with the GPU's."""
    from oracle import oracle as O
    from computervision_objectdetection_featurematching_amd.pipeline import SCALES
    O.build()
    t0 = time.perf_counter()
    res, mism = [], 0
    for si, s in enumerate(SCALES):
        sk, sd = O.sift_detect_compute(O.resize_linear_u8(scene, fx=s))
        sxy = np.stack([sk["x"], sk["y"]], 1)
        for vi in range(len(names)):
            k, dd = model.keypoints[vi], model.descriptors[vi]
            o = O.match_problem(dd, np.stack([k["x"], k["y"]], 1), sd, sxy, threads=1)
            g = run.results[si * len(names) + vi]
            same = (o["n_good"], o["n_inl"], o["status"], o["iters"]) == (int(g["n_good"]), int(g["n_inl"]),
                                                                         int(g["status"]), int(g["iters"]))
            same = same and (o["status"] not in (0, 3, 4) or np.array_equal(o["H"].reshape(9), g["H"]))
            mism += not same
            res.append(o)
    el = time.perf_counter() - t0
    n = len(res)
    return {"value": round(n / el, 4), "unit": "problems/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"one scene: 5 x (resize + SIFT) + {n} problems, oracle/sift_oracle.c + oracle/mim_oracle.c "
                      f"single-threaded (-O3 -ffp-contract=off), {el:.1f} s",
            "parity": {"checked": n, "mismatch": mism}}


def main():
    args = parse()
    # HIP hardware queues per process (read at HIP init, inherited by launched ranks): the batches in
    # flight each keep their own stream, and with HIP's default 4 queues streams past the 4th share a
    # queue, serialising unrelated batches (same box: 4 queues / 3 batches 23.0k, 16 / 12 25.9k problems/s)
    # (the GPU box exports GPU_MAX_HW_QUEUES=4, HIP's default: overridden here, not defaulted)
    os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))  # children only: this process never touches the GPU
    if args.dry_run:
        return dry_run(args)
    rank, world, local = dist_env()
    if args.config == "c1img":
        import torch
        import torch.distributed as dist
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return run_c1img(args, rank, world, local)
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    ranks_seen = dist.get_world_size() if world > 1 else 1
    if ranks_seen != args.gpus:
        raise SystemExit(f"rank {rank}: {ranks_seen} ranks in the process group, --gpus {args.gpus}")
    dev = torch.device("cuda", local)

    from computervision_objectdetection_featurematching_amd import Matcher, build, default_params, shard
    from computervision_objectdetection_featurematching_amd._lib import RESULT_DTYPE
    from computervision_objectdetection_featurematching_amd.synthetic import CONFIGS, SEED_BASE, make_config_dataset

    build.build()
    cfg = CONFIGS[args.config]
    knn_only = bool(cfg.get("knn_only"))
    # every rank: the same models, its own scenes (seeded by rank)
    ds = make_config_dataset(args.config, seed=SEED_BASE + 1000 * rank)
    n_probs = len(ds.problems)
    mdesc = [torch.from_numpy(d).to(dev) for d in ds.model_desc]
    mkp = [torch.from_numpy(k).to(dev) for k in ds.model_kp]
    sdesc = [torch.from_numpy(d).to(dev) for d in ds.scene_desc]
    skp = [torch.from_numpy(k).to(dev) for k in ds.scene_kp]
    torch.cuda.synchronize()

    # C3: 12 batches in flight (+11 % over 3, same box); the C1 surrogate's small batches: 3 (12: -40 %)
    # C5: 2 (one contraction's set prep overlaps the other's distance kernel: 2,020 -> 2,696/s)
    nf = args.inflight if args.inflight > 0 else (2 if knn_only else (3 if args.config == "c1" else 12))
    if nf > 1:  # the sampler stream helps one batch alone (+5 %), not batches already overlapping
        os.environ.setdefault("MIM_SAMPLER_STREAM", "0")
    matchers = [Matcher(local) for _ in range(nf)]
    # each context keeps its own non-blocking HIP stream; torch work of a step (the result gather)
    # is ordered on the same stream
    streams = [torch.cuda.ExternalStream(mm.stream_handle(), device=dev) for mm in matchers]
    prm = default_params(max_iters=max(cfg["max_iters"], 1))
    mine = [torch.empty(n_probs * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(nf)]
    nq0 = int(ds.model_desc[0].shape[0])
    knn_idx = [torch.empty((nq0, 2), dtype=torch.int32, device=dev) for _ in range(nf)]  # per context
    knn_dist = [torch.empty((nq0, 2), dtype=torch.float32, device=dev) for _ in range(nf)]
    counter = [0]

    def step():
        k = counter[0] % nf
        counter[0] += 1
        m = matchers[k]
        with torch.cuda.stream(streams[k]):
            m.clear_sets()
            q_ids = [m.add_set(d, kp) for d, kp in zip(mdesc, mkp)]
            t_ids = [m.add_set(d, kp) for d, kp in zip(sdesc, skp)]
            if knn_only:  # C5: the distance contraction + top-2 alone
                m.knn_sets_dev(q_ids[0], t_ids[0], knn_idx[k], knn_dist[k])
                return
            m.match_batch_async([(q_ids[a], t_ids[b]) for a, b in ds.problems], prm)
            m.batch_results_copy_to(mine[k])
            shard.gather_results(mine[k], world)  # RCCL all-gather of the result records

    for mm in matchers:
        mm.set_timing(False)
    for _ in range(max(args.warmup, nf if args.warmup > 0 else 0)):
        step()
    torch.cuda.synchronize()
    # the warm-up output: records (and, for the CPU parity sample, good lists + masks) of context 0
    m0 = matchers[0]
    res = None if knn_only else m0.batch_results(n_probs)

    for mm in matchers:
        mm.set_timing(not args.no_timing)
    kern = {}
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()  # no host wait inside the loop: steps queue back to back on the streams
    t_host = time.perf_counter() - t0  # host enqueue time of the K steps (< el: the GPU is the bound)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    names = ("knn", "ratio") if knn_only else ("knn", "ratio", "attempt", "chain", "check", "sample", "hypo", "score",
                                               "cand", "exact", "select", "refine")
    if not args.no_timing:
        for mm in matchers:
            if knn_only:
                mm.synchronize()
            mm.batch_results(0)  # collects the HIP events of every timed step (outside the timed region)
        for k in names:
            kern[k] = sum(max(mm.kernel_ms(k), 0.0) for mm in matchers)
    # the same kernels without a concurrent batch (one context, steps back to back; not part of `value`)
    iso = {}
    if not args.no_timing and nf > 1:
        for _ in range(args.steps):
            counter[0] = 0  # always context 0
            step()
        torch.cuda.synchronize()
        m0.batch_results(0)
        iso = {k: max(m0.kernel_ms(k), 0.0) / max(args.steps, 1) for k in kern}
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total = world * n_probs * args.steps
    value = total / el

    if rank == 0:
        nq_all = np.array([d.shape[0] for d in ds.model_desc])
        nt_all = np.array([d.shape[0] for d in ds.scene_desc])
        pq = np.array([nq_all[m] for m, _ in ds.problems], np.float64)
        pt = np.array([nt_all[s] for _, s in ds.problems], np.float64)
        knn_flops = float(np.sum(2.0 * pq * pt * 128))
        knn_bytes = float(np.sum(4 * 128 * (pq + pt) + 16 * pq))
        point_evals = 0.0 if knn_only else float(np.sum(res["iters"].astype(np.float64) * res["n_good"]))
        steps = max(args.steps, 1)
        kavg = {k: v / steps for k, v in kern.items()}
        dom = max(kavg, key=kavg.get) if kavg else None
        rooflines = {}
        if kavg.get("knn", 0) > 0:
            ach = knn_flops / (kavg["knn"] * 1e-3) / 1e12
            rooflines["knn"] = {"kernel": "knn2_i8 (distance GEMM on i8 MFMA, exact integer, + top-2 selection), "
                                          "1 launch/step; ops = 2*Nq*Nt*128 integer ops, peak = dense i8",
                                "bound": "mfma",
                                "achieved": round(ach, 2), "peak": PEAK_I8_TOPS, "unit": "TFLOP/s",
                                "frac": round(ach / PEAK_I8_TOPS, 4),
                                "traffic": pmc_traffic("knn2_i8_kernel", args.config),
                                "algorithmic_bytes": knn_bytes,
                                "achieved_hbm_GBs": round(knn_bytes / (kavg["knn"] * 1e-3) / 1e9, 1)}
        if kavg.get("score", 0) > 0:
            ach = FLOP_PER_POINT_EVAL * point_evals / (kavg["score"] * 1e-3) / 1e12
            rooflines["score"] = {"kernel": "ransac_bound (closed-form hypotheses, bounded inlier counts), 2 launches/step",
                                  "bound": "valu", "achieved": round(ach, 2), "peak": PEAK_F32_VALU_TFLOPS,
                                  "unit": "TFLOP/s", "frac": round(ach / PEAK_F32_VALU_TFLOPS, 4),
                                  "traffic": pmc_traffic("ransac_bound", args.config),
                                  "point_evals_per_step": point_evals,
                                  "hypothesis_point_evals_per_s": round(point_evals / (kavg["score"] * 1e-3), 1)}
        roof = None
        if rooflines:
            key = max(rooflines, key=lambda k: kavg.get(k, 0))  # the dominant of the two hot kernels
            roof = dict(rooflines[key])
            roof["dominant_kernel_by_time"] = dom
            roof["kernel_ms_per_step"] = {k: round(v, 3) for k, v in kavg.items()}
            if iso:  # per-kernel times of one batch alone (no overlap with the other in-flight batches)
                roof["isolated_kernel_ms_per_step"] = {k: round(v, 3) for k, v in iso.items()}
                for key2, r in rooflines.items():
                    t_iso = iso.get(key2, 0)
                    if t_iso > 0:
                        r["isolated_achieved"] = round(r["achieved"] * kavg[key2] / t_iso, 2)
                        r["isolated_frac"] = round(r["isolated_achieved"] / r["peak"], 4)
                roof.update({k: v for k, v in rooflines[key].items() if k.startswith("isolated")})
            roof["others"] = {k: v for k, v in rooflines.items() if k != key}
            if nf > 1:
                roof["note"] = (f"achieved/frac: the kernel's HIP-event span in the timed region, where {nf} batches in "
                                "flight share the GPU (its launches overlap the other batches' kernels); "
                                "isolated_*: the same kernel with one batch alone")
        metric = {"c3": "matches+homographies/sec (10k x 10k SIFT, 50k RANSAC iters)",
                  "c2": "matches+homographies/sec (2k x 2k SIFT, 2k RANSAC iters)",
                  "c1": "matches+homographies/sec (C1 surrogate: 29 views x 5 scales, ragged 100-500 x 1k-4k, "
                        "2k RANSAC iters)",
                  "c5": "knnMatch(k=2) problems/sec (50k x 50k SIFT dense distance contraction)"}[args.config]
        if cfg.get("ragged"):
            workload = (f"c1: {len(ds.model_desc)} model views (Nq {nq_all.min()}-{nq_all.max()}) x {len(ds.scene_desc)} "
                        f"scene scales (Nt {nt_all.min()}-{nt_all.max()}) per GPU, maxIters {cfg['max_iters']}")
        elif knn_only:
            workload = f"c5: {cfg['nq']} x {cfg['nt']} descriptors, distance + top-2 only"
        else:
            workload = (f"{args.config}: {cfg['n_models']} models x {cfg['n_scenes']} scenes per GPU, "
                        f"{cfg['nq']}x{cfg['nt']} descriptors, maxIters {cfg['max_iters']}")
        out = {
            "metric": metric, "value": round(value, 3), "unit": "problems/s", "n_gpus": world,
            "ranks_seen": ranks_seen, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1e3 * el / args.steps, 3),
            "host_enqueue_ms_per_step": round(1e3 * t_host / args.steps, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "i8-MFMA exact-int distances (i32 acc)" + ("" if knn_only else
                                                               ", fp64 DLT/Jacobi, fp32 reprojection"),
            "data": "synthetic SIFT-like integer descriptors (seeded)" + ("" if knn_only else
                                                                        ", planted geometric inliers"),
            "config": {"workload": workload, "problems_per_gpu": n_probs, "global_batch": world * n_probs,
                       "parallelism": f"dp{world}", "batches_in_flight": nf,
                       "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])},
        }
        if res is not None:
            out["accepted_problems_rank0"] = int((res["status"] == 0).sum())
            out["stream_short_rank0"] = int((res["status"] == 5).sum())
        if roof:
            out["roofline"] = roof
        if args.cpu_sample > 0:
            if knn_only:
                m0.synchronize()
                out["cpu_baseline"] = cpu_baseline_knn(ds.model_desc[0], ds.scene_desc[0], knn_idx[0].cpu().numpy(),
                                                       knn_dist[0].cpu().numpy(), 96 * args.cpu_sample)
            else:
                def detail(i):
                    return m0.problem_detail(i, int(res["n_good"][i]))
                out["cpu_baseline"] = cpu_baseline_problems(ds, cfg, res, detail, args.cpu_sample, args.cpu_rounds)
            out["parity"] = out["cpu_baseline"]["parity"]
        print(json.dumps(out), flush=True)
    for mm in matchers:
        mm.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
