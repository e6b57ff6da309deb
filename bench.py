#!/usr/bin/env python3
"""Benchmark: matches+homographies/sec (10k x 10k SIFT, 50k RANSAC iters) at 1/2/4/8 GPUs — BASELINE.json metric.

One step = one pass of the hot path (knnMatch k=2 + ratio test + findHomography RANSAC + refine +
gates, /root/reference/src/TestsDetector.cpp:58-95) over one batch of problems.  Configs
(BASELINE.json `configs`; `--config`, default c4):
  c4  configs[3]: ONE global batch of 256 scenes x 1 model descriptor set, 10,000 x 10,000 128-D
      SIFT-like descriptors per problem, RANSAC maxIters 50,000, conf 0.995, 8 % geometric inliers
      among 2,000 planted matches (no early termination: SURVEY.md App. B).  Scene s is seeded by the
      global seed and s alone; rank r owns shard_range(256, N, r) (strong scaling: 256 problems per step
      at N = 1, 32 per GPU at N = 8), the per-problem records are all-gathered over RCCL every step.
  c3  configs[2]: 3 model sets x 32 scene sets per GPU (96 problems), same shapes (weak scaling).
  c2  configs[1]: 1 x 1, 2k x 2k, maxIters 2000.
  c1  configs[0] surrogate: the reference's own shape, one scene = 29 model views x 5 scales = 145
      ragged problems (Nq 100-500, Nt 1k-4k, maxIters 2000).
  c5  configs[4]: the 50k x 50k dense distance contraction alone (mim_knn2_sets_dev), no RANSAC.
  c1img  configs[0] on the reference's own images (tests/golden/c1_sugar_box.npz): the sugar_box model
      (29 views, SIFT computed once before the timed region as processAllModelsImages does) against one
      test view per step through detectObjects: 5 x (resize + SIFT) on the GPU, the 145 problems as one
      device batch, clustering and boxes on the host (pipeline.detect_objects).
  dataset  the reference's whole run on its own data: 3 models (89 views) vs its 30 test images, one
      step = processAllTestImages over the 30 scenes, split round robin over the ranks.
Inputs (descriptors + keypoints) are resident in HBM before the timed region; each step registers
the sets (the i8 layout prep is inside the step) and runs the batch.  Multi-GPU: one process per GPU
(`--gpus N` launches N ranks through torch.distributed.run when WORLD_SIZE is unset).  Twelve scene
batches are in flight on one GPU (--inflight).  The timed region runs with kernel
timing off.

Prints ONE JSON line on rank 0 with, besides the contract fields:
  "roofline": the distance kernel's launch duration from HIP events in an isolated pass after the
      timed region (one batch at a time on one context, so an event pair brackets exactly that
      kernel; `rocprofv3 --kernel-trace --stats` of `--inflight 1` reproduces it), and
      the RANSAC bound kernel as an instruction roofline ("others");
  "cpu_baseline": oracle/ restatement on this host's cores, bounded sample (rank 0, N = 1);
  "parity": oracle records vs GPU records of sampled problems, summed over all ranks;
  "ranks_seen".
`--dry-run` exercises the launcher, the C4 sharding and the gloo/RCCL record gather without a GPU.
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
PEAK_F16_MFMA_TFLOPS = 2500.0  # dense f16 MFMA
# VALU issue peak: 1024 SIMDs x one wave64 fp32 add/fma per 2 cycles (a SIMD-32 retires a wave64 fp32 op in 2
# cycles once two or more waves issue: MI355X_MICROARCH.md cycle-constants table; tools/issue_probe.hip measures
# 1.07-1.21 ns per wave-instruction at 8 waves per SIMD, profiles/r05*_issue_probe.txt) x 2.4 GHz
PEAK_VALU_WAVE_INSTR_PER_S = 1024 * 0.5 * 2.4e9
# ransac_bound_mfma_kernel tile loop, VALU per (point, hypothesis) pair, all fp32 add/sub/fma (round 5: a clamped
# float count instead of the sign bit's v_alignbit): later chunks fma, sub, sub with clamp, add = 4; chunk 1 (the
# first 4,096 iterations, 512 when maxIters <= 4,096) also the lower bound: add (|X'| + |Y'|, shared), then fma,
# sub with clamp, add for each bound = 7
BOUND_VALU_PER_PAIR_C1, BOUND_VALU_PER_PAIR_C2 = 7, 4
BOUND_MFMA_FLOP_PER_PAIR = 96  # 3 v_mfma_f32_32x32x16_f16 per 32 x 32 (point, hypothesis) pairs
# issue model of one SIMD (tools/issue_probe.hip at ~2.0-2.1 GHz, profiles/r05b_issue_probe.txt): a fast fp32
# VALU wave-instruction costs ~1.15 ns, and a v_mfma_f32_32x32x16_f16 takes ~10.5 ns of VALU issue from its SIMD
# (2 MFMAs + 64 fmas run 20-22 ns longer than the 64 fmas alone, at 2 and 4 waves per SIMD, i.e. about 2/3 of the
# MFMA's 32 cycles: the matrix pipe and the VALU do not co-execute on one SIMD beyond that, nor with the roles
# split over two waves, section D)
ISSUE_NS_VALU, ISSUE_NS_MFMA_F16_32 = 1.15, 10.5
H_TOL = 1e-4                  # SURVEY.md 8(c) contract item 4 (the GPU tests hold bit identity)


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC pass (or None)."""
    for name in (f"r06_pmc_traffic_{config}.json", f"r05_pmc_traffic_{config}.json"):  # newest first
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                d = json.load(f)
            if d.get("config", "c3") != config:
                continue
            k = d["kernels"][kernel]
            return k.get("hbm_bytes_per_launch", k.get("hbm_bytes_per_step"))
        except (OSError, KeyError, ValueError):
            continue
    return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=["c1", "c1img", "c2", "c3", "c4", "c5", "dataset"])
    ap.add_argument("--cpu-sample", type=int, default=6,
                    help="problems of the sequential CPU-baseline sample (1 warm-up + the median of the rest; "
                         "0: skip the CPU baseline)")
    ap.add_argument("--cpu-rounds", type=int, default=5, help="timed rounds of the parallel CPU row")
    ap.add_argument("--parity-sample", type=int, default=2,
                    help="problems per rank checked against the oracle when N > 1 (untimed)")
    ap.add_argument("--iso-steps", type=int, default=10,
                    help="steps of the isolated pass (one context, kernel timing on) after the timed region")
    ap.add_argument("--no-timing", action="store_true", help="disable per-kernel HIP events")
    ap.add_argument("--inflight", type=int, default=0,
                    help="scene batches in flight: one library context + HIP stream each, steps assigned "
                         "round-robin, so a batch's latency-bound RANSAC tail overlaps the next batch's kNN "
                         "(0: 16 for the C3/C4 batches and shards, 12 for c1img/dataset scenes, c1 3; with "
                         "GPU_MAX_HW_QUEUES=24 their streams, torch's and RCCL's each get a hardware queue)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="diagnostic (N = 1 only, sharded configs): run rank 0's shard of an N-rank run, the "
                         "per-GPU workload of strong-scaling point N (value = this GPU's rate on it)")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process and the ranks it launches (set before HIP initialises); "
                         "0: 24 for the synthetic batch configs (16 batches in flight), 16 for the scene configs "
                         "c1img/dataset (12 scenes in flight: 24 queues cost the dataset line 15 %, r05v)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (one GPU per rank); gloo = rehearsal of the N-rank path with several "
                         "ranks on one GPU (the record gather through host memory)")
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
    """Launcher + process group + C4 sharding + record gather on gloo (CPU): what the N-rank bench does
    around its GPU work.  Prints the JSON line with n_gpus / ranks_seen and, for a sharded config, the
    scene ids covered by the union of the ranks' shards, so a CPU test can check the launch."""
    import torch
    import torch.distributed as dist

    from computervision_objectdetection_featurematching_amd import shard
    from computervision_objectdetection_featurematching_amd._lib import RESULT_DTYPE
    from computervision_objectdetection_featurematching_amd.synthetic import CONFIGS

    rank, world, _ = dist_env()
    if world > 1:
        dist.init_process_group("gloo")
    seen = dist.get_world_size() if world > 1 else 1
    if seen != args.gpus:
        raise SystemExit(f"rank {rank}: process group has {seen} ranks, --gpus {args.gpus}")
    if args.config == "dataset":  # the real-data split: scenes round robin, detections all-gathered
        mine = list(shard.shard_round_robin(DATASET_SCENES, world, rank))
        parts = shard.gather_objects([(i, [((i, rank, 1, 1), "stub")]) for i in mine], world)
        merged = shard.merge_scene_results(parts, DATASET_SCENES)
        if rank == 0:
            print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "problems/s", "n_gpus": world,
                              "ranks_seen": seen, "steps": 0, "warmup": 0, "ms_per_step": 0.0,
                              "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dry_run": True,
                              "config": {"workload": "dataset", "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])},
                              "scene_ids_covered": sum(d[0][0][0] == i for i, d in enumerate(merged)),
                              "ranks_of_scenes": [d[0][0][1] for d in merged], "global_batch": DATASET_SCENES}),
                  flush=True)
        if world > 1:
            dist.destroy_process_group()
        return
    cfg = CONFIGS.get(args.config, {})
    n_scenes = cfg.get("n_scenes", 4) if cfg.get("sharded") else 4 * world
    ids = shard.shard_range(n_scenes, world, rank) if cfg.get("sharded") else range(4 * rank, 4 * rank + 4)
    # per-rank records of its problems (the scene id in n_good), padded to the largest shard
    per = -(-n_scenes // world)
    rec = np.zeros(per, RESULT_DTYPE)
    rec["n_good"] = -1
    rec["n_good"][:len(ids)] = np.array(list(ids), np.int32)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    g = shard.decode(shard.gather_results(torch.from_numpy(rec.view(np.uint8).copy()), world))
    cnt = torch.tensor([len(ids), 0], dtype=torch.int64)  # the parity sums use the same all-reduce
    if world > 1:
        dist.all_reduce(cnt)
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        got = g["n_good"].ravel()
        got = np.sort(got[got >= 0])
        assert g.shape == (world, per) and np.array_equal(got, np.arange(n_scenes)), got
        assert int(cnt[0]) == n_scenes
        print(json.dumps({"metric": "dry-run", "value": 0.0, "unit": "problems/s", "n_gpus": world,
                          "ranks_seen": seen, "steps": 0, "warmup": 0, "ms_per_step": float(t.item()) * 1e3,
                          "higher_is_better": True, "scaling": "strong" if cfg.get("sharded") else "weak",
                          "vs_baseline": None, "dry_run": True,
                          "config": {"workload": args.config, "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])},
                          "scene_ids_covered": int(len(np.unique(got))), "global_batch": n_scenes}),
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


CORES_NOTE = ("threads = this job's CPU share (OMP_NUM_THREADS: 16 per GPU on the GPU box, whose nproc counts the "
              "whole machine; the box's rules size worker pools to that share, so no all-machine row is run)")


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
            "cpu_model": cpu_model(), "machine_cores": os.cpu_count(), "cores_note": CORES_NOTE,
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
            "cpu_model": cpu_model(), "machine_cores": os.cpu_count(), "cores_note": CORES_NOTE,
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
    # the fixture's 10 sugar_box test views: rank r's steps cycle through its round-robin share
    # (shard_round_robin, as process_all_test_images splits a dataset); the isolated pass, the
    # latency figures and the CPU baseline use the share's first view
    from computervision_objectdetection_featurematching_amd.shard import shard_round_robin
    my_ids = [scenes[i] for i in shard_round_robin(len(scenes), world, rank)] or [scenes[rank % len(scenes)]]
    my_scenes = [d[f"scene/{s}"] for s in my_ids]
    sid = my_ids[0]
    scene = my_scenes[0]
    n_probs = len(SCALES) * len(names)
    for mm, md in zip(ms[1:], models[1:]):
        detect_objects(mm, scene, [md])
    n_warm = max(args.warmup, 1)  # context 0's warm-up steps; contexts 1.. ran one scene each above
    for _ in range(n_warm):
        run = detect_objects(m, scene, [model], keep=True)
    for mm in ms:
        mm.set_timing(not args.no_timing)
    out_dets = [None] * nf

    def worker(k):
        for st in range(k, args.steps, nf):
            out_dets[k] = detect_objects(ms[k], my_scenes[st % len(my_scenes)], [models[k]])

    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(nf)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    list(pool.map(worker, range(nf)))
    torch.cuda.synchronize()
    pool.shutdown()
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
    # single-scene latency (not part of `value`) as the drop-in caller sees it: detectObjects of one scene
    # alone on one context, no keypoints copied out, no per-kernel events; median of the calls
    m.set_sampler_stream(True)
    m.set_timing(False)
    lat, stages = [], {}
    for _ in range(max(args.iso_steps, 5)):
        t1 = time.perf_counter()
        detect_objects(m, scene, [model], stage_ms=stages)
        lat.append(time.perf_counter() - t1)
    scene_ms = 1e3 * statistics.median(lat)
    stages = {k: round(v / len(lat), 3) for k, v in stages.items()}
    # isolated pass (not part of `value`): one scene at a time on one context, kernel timing on — the
    # kernel breakdown and the distance kernel's launch duration
    m.set_timing(True)
    n_iso = max(args.iso_steps, 1)
    names_k = ("knn", "ratio", "attempt", "chain", "check", "sample", "score", "cand", "exact", "select", "refine")
    acc = dict.fromkeys(names_k, 0.0)
    el_iso = 0.0
    for _ in range(n_iso):
        t1 = time.perf_counter()
        run = detect_objects(m, scene, [model], keep=True)
        el_iso += time.perf_counter() - t1
        dets = run.detections
        for k in names_k:  # each scene's batch collects its own events (match_batch -> batch_results)
            acc[k] += max(m.kernel_ms(k), 0.0)
    scene_ms_events = 1e3 * el_iso / n_iso
    iso = {k: v / n_iso for k, v in acc.items() if v > 0}
    nq = np.array([d.shape[0] for d in model.descriptors], np.float64)
    nt = np.array([len(k) for k in run.scene_kp], np.float64)
    knn_ops = float(2.0 * 128 * nq.sum() * nt.sum())  # every (view, scale) pair
    if rank == 0:
        out = {"metric": "matches+homographies/sec (configs[0]: sugar_box model vs one test view, reference images, "
                         "SIFT + match + RANSAC + boxes)",
               "value": round(world * n_probs * args.steps / el, 3), "unit": "problems/s", "n_gpus": world,
               "steps": args.steps, "warmup": n_warm + nf - 1, "ms_per_step": round(1e3 * el / args.steps, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "f32 SIFT (OpenCV order), i8-MFMA exact-int distances, fp64 DLT/LM, fp32 reprojection",
               "data": f"reference images: 29 sugar_box model views + masks, test views {', '.join(my_ids)} (rank 0)",
               "config": {"workload": f"c1img: detectObjects of one 640x480 scene against {len(names)} views x "
                                      f"{len(SCALES)} scales = {n_probs} problems per step per GPU, the steps "
                                      f"cycling through the rank's share of the {len(scenes)} test views",
                          "problems_per_gpu": n_probs, "global_batch": world * n_probs, "parallelism": f"dp{world}",
                          "scenes_in_flight": nf},
               "scenes_per_s": round(world * args.steps / el, 3),
               "sift_640x480_ms": round(1e3 * statistics.median(ts), 3),
               "single_scene_ms": round(scene_ms, 3),
               "single_scene_ms_range": [round(1e3 * min(lat), 3), round(1e3 * max(lat), 3)],
               "single_scene_ms_with_kernel_events": round(scene_ms_events, 3),
               "single_scene_stage_ms": stages,
               "roofline": {"kernel": "knn2_i8_kernel (145 ragged problems of one scene, 1 launch per scene)",
                            "bound": "mfma", "unit": "TFLOP/s", "peak": PEAK_I8_TOPS,
                            "achieved": round(knn_ops / (iso["knn"] * 1e-3) / 1e12, 2),
                            "frac": round(knn_ops / (iso["knn"] * 1e-3) / 1e12 / PEAK_I8_TOPS, 4),
                            "traffic": None, "launch_ms": round(iso["knn"], 4), "ops_per_launch": knn_ops,
                            "timing": "HIP events, isolated pass (one scene at a time, one context)",
                            "kernel_ms_per_scene_isolated": {k: round(v, 4) for k, v in iso.items()},
                            "note": "small problems (Nq ~100-500 x Nt ~1-4k): launch- and latency-bound, the "
                                    "MFMA fraction is not the limiter at this size"},
               "detections_rank0": [list(b) for b, _ in dets], "detections_scene": sid,
               "accepted_problems_rank0": int((run.results["status"] == 0).sum())}
        if args.cpu_sample > 0:
            out["cpu_baseline"] = cpu_baseline_c1img(scene, model, run, names)
            out["parity"] = out["cpu_baseline"]["parity"]
        print(json.dumps(out), flush=True)
    for mm in ms:
        mm.close()


DATASET_SCENES = 30  # tests/golden/dataset_gray.npz: the reference's 30 test images (data/*/test)


def run_dataset(args, rank, world, local):
    """The reference's whole run on its own data (main.cpp:17-33): the 3 objects' 89 model views are
    described once (processAllModelsImages, untimed, as c1img), then one step = processAllTestImages
    over the 30 test images (Output.cpp:19-57: detectObjects of every scene against all 3 models, 445
    problems per scene, plus its results file), the scenes split round robin over the ranks
    (pipeline.process_all_test_images, detections all-gathered every step).  Strong scaling: 30
    scenes per step at any N.  Parity: every scene's detections against the restatement's run
    (tests/golden/dataset_expected.json)."""
    import tempfile

    import torch
    import torch.distributed as dist

    from computervision_objectdetection_featurematching_amd import Matcher, build
    from computervision_objectdetection_featurematching_amd import shard
    from computervision_objectdetection_featurematching_amd.pipeline import (SCALES, process_all_test_images,
                                                                               process_model_views)

    build.build()
    with np.load(os.path.join(ROOT, "tests", "golden", "dataset_gray.npz")) as z:
        imgs = {k: z[k] for k in z.files}
    with open(os.path.join(ROOT, "tests", "golden", "dataset_expected.json")) as f:
        exp = json.load(f)
    objs = sorted({k.split("/")[0] for k in imgs})
    scenes = [(obj, k.split("/")[-1] + "-color", imgs[k]) for obj in objs
              for k in sorted(k for k in imgs if k.startswith(f"{obj}/scene/"))]
    assert len(scenes) == DATASET_SCENES
    mine = list(shard.shard_round_robin(len(scenes), world, rank))
    nf = max(1, min(args.inflight if args.inflight > 0 else 12, len(mine)))
    ms = [Matcher(local) for _ in range(nf)]
    models = []
    for obj in objs:
        views = sorted(k for k in imgs if k.startswith(f"{obj}/view/"))
        models.append(process_model_views(ms[0], obj, [(imgs[k], imgs.get(k.replace("/view/", "/mask/")))
                                                       for k in views]))
    n_views = sum(len(m.descriptors) for m in models)
    per_scene = len(SCALES) * n_views
    out_dir = tempfile.mkdtemp(prefix="mim_dataset_")
    for k, mm in enumerate(ms):  # every context once (code objects, workspaces, the models' sets)
        process_all_test_images(mm, [scenes[mine[k % len(mine)]]], models, tempfile.mkdtemp(prefix="mim_warm_"))
    n_warm = max(args.warmup, 0)
    for _ in range(n_warm):
        process_all_test_images(ms, scenes, models, out_dir, rank=rank, world=world)
    got = None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        got = process_all_test_images(ms, scenes, models, out_dir, rank=rank, world=world)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=torch.device("cuda", local))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        mism = [f"{f}/{s}" for (f, s), d in got.items()
                if [[*b, n] for b, n in d] != exp["scenes"][f"{f}/{s[:-6]}"]["detections"]]
        out = {"metric": "matches+homographies/sec (the reference's dataset: 3 models x 89 views vs its 30 test "
                         "images, SIFT + match + RANSAC + boxes + results files)",
               "value": round(len(scenes) * per_scene * args.steps / el, 3), "unit": "problems/s", "n_gpus": world,
               "steps": args.steps, "warmup": n_warm + nf, "ms_per_step": round(1e3 * el / args.steps, 3),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
               "dtype": "f32 SIFT (OpenCV order), i8-MFMA exact-int distances, fp64 DLT/LM, fp32 reprojection",
               "data": "reference images: 3 objects, 89 model views + masks, 30 test images",
               "config": {"workload": f"dataset: processAllTestImages of {len(scenes)} scenes x {per_scene} problems "
                                      f"(3 models, {n_views} views, {len(SCALES)} scales), scenes round robin over "
                                      f"{world} GPU(s)",
                          "problems_per_step": len(scenes) * per_scene, "scenes_rank0": len(mine),
                          "parallelism": f"dp{world}", "scenes_in_flight": nf},
               "scenes_per_s": round(len(scenes) * args.steps / el, 3),
               "ms_per_scene": round(1e3 * el / (args.steps * len(scenes)), 3),
               "parity": {"checked": len(got), "mismatch": len(mism), "first": mism[:3],
                          "reference": "detections of the restatement's run of the same data "
                                       "(tests/golden/dataset_expected.json; parity vs OpenCV unpinned)"}}
        print(json.dumps(out), flush=True)
    for mm in ms:
        mm.close()


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


def kernel_rooflines(args, ds, res, iso, iso_step_ms, knn_only):
    """Roofline objects from the isolated pass's per-step kernel times (ms)."""
    nq_all = np.array([d.shape[0] for d in ds.model_desc])
    nt_all = np.array([d.shape[0] for d in ds.scene_desc])
    pq = np.array([nq_all[m] for m, _ in ds.problems], np.float64)
    pt = np.array([nt_all[s] for _, s in ds.problems], np.float64)
    knn_ops = float(np.sum(2.0 * pq * pt * 128))
    knn_bytes = float(np.sum(512 * (pq + pt) + 16 * pq))
    t = iso["knn"]
    ach = knn_ops / (t * 1e-3) / 1e12
    # the committed PMC passes profile the config's whole batch on one GPU (bench.py --config C --inflight
    # 1): a shard's smaller launch (N > 1 or --shard-of) has no measured traffic of its own
    from computervision_objectdetection_featurematching_amd.synthetic import CONFIGS
    cfg = CONFIGS.get(args.config, {})
    full = cfg.get("ragged") or not cfg.get("sharded") or len(ds.problems) == cfg["n_scenes"] * cfg["n_models"]
    traffic = pmc_traffic("knn2_i8_kernel", args.config) if full else None
    roof = {"kernel": "knn2_i8_kernel (exact-integer distance contraction on v_mfma_i32_32x32x32_i8 + top-2 "
                      "selection), 1 launch per step",
            "bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_I8_TOPS, "unit": "TFLOP/s",
            "frac": round(ach / PEAK_I8_TOPS, 4),
            "traffic": traffic,
            **({} if full else {"traffic_note": f"PMC traffic is measured on the full {args.config} batch; this "
                                                f"rank's launch holds {len(ds.problems)} problems"}),
            "launch_ms": round(t, 4), "ops_per_launch": knn_ops,
            "ops": "2 * Nq * Nt * 128 integer multiply-adds (i8 operands, i32 accumulate), summed over the batch",
            "algorithmic_bytes_per_launch": knn_bytes,
            "achieved_hbm_GBs": round(knn_bytes / (t * 1e-3) / 1e9, 1),
            "timing": "HIP events on the library stream around the launch, isolated pass: one batch at a time on "
                      "one context after the timed region (rocprofv3 --kernel-trace --stats of --inflight 1 "
                      "reproduces it: profiles/)",
            "isolated_step_ms": round(iso_step_ms, 3),
            "kernel_ms_per_step_isolated": {k: round(v, 4) for k, v in iso.items()}}
    if not knn_only and iso.get("score", 0) > 0:
        it = res["iters"].astype(np.float64)
        c1 = 4096 if args_max_iters(args) > 4096 else 512
        pairs = float(np.sum(it * res["n_good"]))
        pairs1 = float(np.sum(np.minimum(it, c1) * res["n_good"]))
        tb = iso["score"] * 1e-3
        wi = (pairs1 * BOUND_VALU_PER_PAIR_C1 + (pairs - pairs1) * BOUND_VALU_PER_PAIR_C2) / 64.0
        roof["others"] = {"bound": {
            "kernel": "ransac_bound_mfma_kernel (closed-form hypotheses, bounded inlier counts), 2 launches per step",
            "bound": "valu", "unit": "VALU wave-instructions/s",
            "achieved": round(wi / tb, 1), "peak": PEAK_VALU_WAVE_INSTR_PER_S,
            "frac": round(wi / tb / PEAK_VALU_WAVE_INSTR_PER_S, 4),
            "pairs_per_step": pairs, "pairs_chunk1_per_step": pairs1,
            "valu_per_pair": {"chunk1": BOUND_VALU_PER_PAIR_C1, "chunk2": BOUND_VALU_PER_PAIR_C2},
            "floor_ms": round(wi / PEAK_VALU_WAVE_INSTR_PER_S * 1e3, 4), "ms_per_step": round(iso["score"], 4),
            "mfma": {"achieved_TFLOPs": round(pairs * BOUND_MFMA_FLOP_PER_PAIR / tb / 1e12, 1),
                     "peak_TFLOPs": PEAK_F16_MFMA_TFLOPS,
                     "frac": round(pairs * BOUND_MFMA_FLOP_PER_PAIR / tb / 1e12 / PEAK_F16_MFMA_TFLOPS, 4)},
            # the SIMDs' issue time the tile loop needs by the probe's costs (test VALU + MFMA), over the kernel time
            "issue_model": {"valu_ns": ISSUE_NS_VALU, "mfma_ns": ISSUE_NS_MFMA_F16_32,
                            "floor_ms": round((wi * ISSUE_NS_VALU + pairs * 3 / 1024.0 * ISSUE_NS_MFMA_F16_32) / 1024 * 1e-6, 4),
                            "frac": round((wi * ISSUE_NS_VALU + pairs * 3 / 1024.0 * ISSUE_NS_MFMA_F16_32) / 1024 * 1e-9 / tb, 4)},
            "note": "pairs = iterations x good matches of every problem (OpenCV scores every hypothesis on every "
                    "point); VALU peak = 1024 SIMDs x 1 wave64 fp32 instruction per 2 cycles x 2.4 GHz; issue_model: "
                    "the tile loop's test VALU and MFMA priced by tools/issue_probe.hip (per SIMD)"}}
    # consistency: one stream, one batch at a time -> the kernels' durations cannot exceed the step
    worst = max(iso.values()) if iso else 0.0
    total = sum(iso.values())
    if worst > iso_step_ms * 1.02 + 0.02 or total > iso_step_ms * 1.05 + 0.05:
        raise SystemExit(f"bench: isolated kernel times {iso} exceed the isolated step {iso_step_ms:.3f} ms")
    roof["kernel_sum_ms_per_step_isolated"] = round(total, 4)
    return roof


def args_max_iters(args) -> int:
    from computervision_objectdetection_featurematching_amd.synthetic import CONFIGS
    return int(CONFIGS[args.config]["max_iters"])


def parity_sample(ds, cfg, res, detail, ids):
    """Oracle records of problems `ids` (untimed) compared with the GPU's: (checked, mismatches)."""
    from oracle import oracle as O
    O.build()
    prm = O.default_params(max_iters=cfg["max_iters"])
    bad = []
    for i in ids:
        m, s = ds.problems[i]
        o = O.match_problem(ds.model_desc[m], ds.model_kp[m], ds.scene_desc[s], ds.scene_kp[s], prm, host_cores())
        d = _cmp_problem(o, res[i], detail(i))
        if d:
            bad.append((int(i), d))
    return len(ids), bad


def main():
    args = parse()
    # HIP hardware queues per process (read at HIP init, inherited by launched ranks): the batches in
    # flight each keep their own stream, and with HIP's default 4 queues streams past the 4th share a
    # queue, serialising unrelated batches (same box: 4 queues / 3 batches 23.0k, 16 / 12 25.9k problems/s; round 5: 24 / 16, r05p)
    # (the GPU box exports GPU_MAX_HW_QUEUES=4, HIP's default: overridden here, not defaulted)
    if args.hw_queues <= 0:
        args.hw_queues = 16 if args.config in ("c1img", "dataset") else 24
    os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))  # children only: this process never touches the GPU
    if args.dry_run:
        return dry_run(args)
    rank, world, local = dist_env()
    import torch
    import torch.distributed as dist
    if args.dist_backend == "gloo":  # rehearsal: every rank on the visible GPU(s), round robin
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if args.dist_backend == "nccl":
        # RCCL at every N, N = 1 included: the record gather of every step is the same
        # all_gather_into_tensor on the contexts' streams whether 1 or 8 ranks run
        if world == 1:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    elif world > 1:
        dist.init_process_group("gloo")
    try:
        if args.config == "c1img":
            return run_c1img(args, rank, world, local)
        if args.config == "dataset":
            return run_dataset(args, rank, world, local)
        return run_batches(args, rank, world, local)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_batches(args, rank, world, local):
    """The synthetic configs (c1 surrogate, c2-c5): see the module docstring."""
    import torch
    import torch.distributed as dist
    ranks_seen = dist.get_world_size() if dist.is_initialized() else 1
    if ranks_seen != args.gpus:
        raise SystemExit(f"rank {rank}: {ranks_seen} ranks in the process group, --gpus {args.gpus}")
    dev = torch.device("cuda", local)
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")  # where the collectives' tensors live

    from computervision_objectdetection_featurematching_amd import Matcher, build, default_params, shard
    from computervision_objectdetection_featurematching_amd._lib import RESULT_DTYPE
    from computervision_objectdetection_featurematching_amd.synthetic import CONFIGS, SEED_BASE, make_config_dataset

    build.build()
    cfg = CONFIGS[args.config]
    knn_only = bool(cfg.get("knn_only"))
    sharded = bool(cfg.get("sharded"))
    if sharded:  # one global batch: this rank's contiguous block of its scenes (same data at any N)
        # --shard-of N (diagnostic, one process): rank 0's shard of an N-rank run, i.e. the per-GPU
        # workload of the strong-scaling point N; `value` is then this GPU's rate on it
        w_eff = args.shard_of if (args.shard_of > 0 and world == 1) else world
        ids = shard.shard_range(cfg["n_scenes"], w_eff, rank)
        ds = make_config_dataset(args.config, seed=SEED_BASE, scene_ids=ids)
        global_batch = cfg["n_scenes"] * cfg["n_models"] if w_eff == world else len(ids) * cfg["n_models"]
    else:  # every rank: the same models, its own scenes (seeded by rank)
        ds = make_config_dataset(args.config, seed=SEED_BASE + 1000 * rank)
        global_batch = world * len(ds.problems)
    n_probs = len(ds.problems)
    # ranks hold shards differing by at most one scene: records are gathered at the largest size
    n_rec = -(-global_batch // world) if sharded else n_probs
    mdesc = [torch.from_numpy(d).to(dev) for d in ds.model_desc]
    mkp = [torch.from_numpy(k).to(dev) for k in ds.model_kp]
    sdesc = [torch.from_numpy(d).to(dev) for d in ds.scene_desc]
    skp = [torch.from_numpy(k).to(dev) for k in ds.scene_kp]
    torch.cuda.synchronize()

    # C3/C4: 16 batches in flight on 24 hardware queues (12 on 16: -1 % on C4, -2-3 % on its 32-problem
    # shard, profiles/r05o_*, r05p_*; 12 was +11 % over 3); the C1 surrogate's small batches: 3 (12: -40 %)
    # C5: 2 (one contraction's set prep overlaps the other's distance kernel)
    nf = args.inflight if args.inflight > 0 else (2 if knn_only else (3 if args.config == "c1" else 16))
    # one stream per context: the sampler stream helps one batch alone (+5 %), not batches already
    # overlapping; with it off the isolated pass's kernels run one after another on one stream, so
    # their HIP-event durations add up to at most the step (checked in kernel_rooflines)
    os.environ.setdefault("MIM_SAMPLER_STREAM", "0")
    matchers = [Matcher(local) for _ in range(nf)]
    # each context keeps its own non-blocking HIP stream; torch work of a step (the result gather)
    # is ordered on the same stream
    streams = [torch.cuda.ExternalStream(mm.stream_handle(), device=dev) for mm in matchers]
    # diagnostic (MIM_BENCH_PRIO): contexts on torch streams of mixed priority, every `every`-th one high
    prio = os.environ.get("MIM_BENCH_PRIO", "")
    if prio:
        every = int(prio)
        streams = [torch.cuda.Stream(device=dev, priority=-1 if k % every == 0 else 0) for k in range(nf)]
        for mm, st in zip(matchers, streams):
            mm.set_stream(st.cuda_stream)
    prm = default_params(max_iters=max(cfg["max_iters"], 1))
    mine = [torch.zeros(n_rec * RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev) for _ in range(nf)]
    gath = [None] * nf
    nq0 = int(ds.model_desc[0].shape[0])
    knn_idx = [torch.empty((nq0, 2), dtype=torch.int32, device=dev) for _ in range(nf)]  # per context
    knn_dist = [torch.empty((nq0, 2), dtype=torch.float32, device=dev) for _ in range(nf)]
    counter = [0]
    no_gather = os.environ.get("MIM_BENCH_GATHER", "1") == "0"

    def step():
        k = counter[0] % nf
        counter[0] += 1
        m = matchers[k]
        with torch.cuda.stream(streams[k]):
            m.clear_sets()
            q_ids = [m.add_set(d, kp) for d, kp in zip(mdesc, mkp)]
            t_ids = m.add_sets(zip(sdesc, skp))  # the step's scene sets in one library call
            if knn_only:  # C5: the distance contraction + top-2 alone
                m.knn_sets_dev(q_ids[0], t_ids[0], knn_idx[k], knn_dist[k])
                return
            m.match_batch_async([(q_ids[a], t_ids[b]) for a, b in ds.problems], prm)
            m.batch_results_copy_to(mine[k])
            # RCCL all-gather of the result records (gloo rehearsal: through host memory); MIM_BENCH_GATHER=0
            # is a diagnostic that leaves it out (the line then says so and is not a contract line)
            if not no_gather:
                gath[k] = shard.gather_results(mine[k] if cdev.type == "cuda" else mine[k].cpu(), world)

    for mm in matchers:
        mm.set_timing(False)
    n_warm = max(args.warmup, nf if args.warmup > 0 else 0)  # every context once: its first-use allocations
    for _ in range(n_warm):
        step()
    torch.cuda.synchronize()

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
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    total = global_batch * args.steps
    value = total / el
    # the timed region's records as gathered (all ranks): a cut-short RANSAC (RNG stream exhausted,
    # status 5) would have been counted as throughput; batch_results() re-runs such a batch, a device
    # copy cannot, so they are counted here and fail the parity check
    short_timed = 0
    gather_check = None
    if not knn_only:
        # every context's last gathered step: this rank's row must be its own records byte for byte,
        # and the records of all ranks (each rank's shard, without the padding) are summarised
        sizes = ([len(shard.shard_range(global_batch, world, r)) for r in range(world)] if sharded
                 else [n_probs] * world)
        same, n_ctx, st_counts, it_min, it_max = True, 0, {}, None, None
        for k, gk in enumerate(gath):
            if gk is None:
                continue
            n_ctx += 1
            same = same and bool(torch.equal(gk[rank].to(mine[k].device), mine[k]))
            recs = shard.decode(gk)
            short_timed += int((recs["status"] == 5).sum())
            for r in range(world):
                rr = recs[r, :sizes[r]]
                for s, c in zip(*np.unique(rr["status"], return_counts=True)):
                    st_counts[int(s)] = st_counts.get(int(s), 0) + int(c)
                if len(rr):
                    lo, hi = int(rr["iters"].min()), int(rr["iters"].max())
                    it_min = lo if it_min is None else min(it_min, lo)
                    it_max = hi if it_max is None else max(it_max, hi)
        gather_check = {"collective": ("all_gather_into_tensor" if dist.is_initialized() else "identity copy"),
                        "backend": (dist.get_backend() if dist.is_initialized() else None),
                        "world": world, "contexts_checked": n_ctx, "own_row_identical": same,
                        "records": int(sum(st_counts.values())), "status_counts": st_counts,
                        "iters_min": it_min, "iters_max": it_max}

    # ---- isolated pass: one context, one batch at a time, kernel timing on (not part of `value`)
    m0 = matchers[0]
    m0.set_timing(True)
    n_iso = max(args.iso_steps, 1)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(n_iso):
        counter[0] = 0  # always context 0
        step()
    m0.synchronize()
    torch.cuda.synchronize()
    iso_step_ms = 1e3 * (time.perf_counter() - t1) / n_iso
    res = None
    if knn_only:
        m0.batch_results(0)  # collects the HIP events
    else:
        res = m0.batch_results(n_probs)
    names = ("knn", "ratio") if knn_only else ("knn", "ratio", "attempt", "chain", "check", "sample", "hypo", "score",
                                               "cand", "exact", "select", "refine")
    iso = {k: max(m0.kernel_ms(k), 0.0) / n_iso for k in names if m0.kernel_ms(k) > 0}
    roof = kernel_rooflines(args, ds, res, iso, iso_step_ms, knn_only) if rank == 0 else None

    # ---- parity: oracle vs GPU records of sampled problems; the CPU baseline timing on rank 0 at N = 1
    cpu = None
    checked, bad = 0, []
    if knn_only:
        if rank == 0 and args.cpu_sample > 0:
            m0.synchronize()
            cpu = cpu_baseline_knn(ds.model_desc[0], ds.scene_desc[0], knn_idx[0].cpu().numpy(),
                                   knn_dist[0].cpu().numpy(), 96 * args.cpu_sample)
            checked, bad = cpu["parity"]["checked"], [None] * cpu["parity"]["mismatch"]
    else:
        def detail(i):
            return m0.problem_detail(i, int(res["n_good"][i]))
        if rank == 0 and world == 1 and args.cpu_sample > 0:
            cpu = cpu_baseline_problems(ds, cfg, res, detail, args.cpu_sample, args.cpu_rounds)
            checked, bad = cpu["parity"]["checked"], [cpu["parity"]["first"]] * cpu["parity"]["mismatch"]
        elif (world > 1 or args.cpu_sample == 0) and args.parity_sample > 0:
            k = min(args.parity_sample, n_probs)
            checked, bad = parity_sample(ds, cfg, res, detail, [(7 * j + rank) % n_probs for j in range(k)])
    own_differs = int(gather_check is not None and not gather_check["own_row_identical"])
    tot = torch.tensor([checked, len(bad), short_timed, own_differs], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(tot)  # every rank's parity sample and cut-short count

    if rank == 0:
        metric = {"c3": "matches+homographies/sec (10k x 10k SIFT, 50k RANSAC iters)",
                  "c4": "matches+homographies/sec (10k x 10k SIFT, 50k RANSAC iters) at 1/2/4/8 GPUs",
                  "c2": "matches+homographies/sec (2k x 2k SIFT, 2k RANSAC iters)",
                  "c1": "matches+homographies/sec (C1 surrogate: 29 views x 5 scales, ragged 100-500 x 1k-4k, "
                        "2k RANSAC iters)",
                  "c5": "knnMatch(k=2) problems/sec (50k x 50k SIFT dense distance contraction)"}[args.config]
        nq_all = np.array([d.shape[0] for d in ds.model_desc])
        nt_all = np.array([d.shape[0] for d in ds.scene_desc])
        if cfg.get("ragged"):
            workload = (f"c1: {len(ds.model_desc)} model views (Nq {nq_all.min()}-{nq_all.max()}) x {len(ds.scene_desc)} "
                        f"scene scales (Nt {nt_all.min()}-{nt_all.max()}) per GPU, maxIters {cfg['max_iters']}")
        elif knn_only:
            workload = f"c5: {cfg['nq']} x {cfg['nt']} descriptors, distance + top-2 only"
        elif sharded:
            workload = (f"c4: one global batch of {cfg['n_scenes']} scenes x {cfg['n_models']} model set, "
                        f"{cfg['nq']}x{cfg['nt']} descriptors, maxIters {cfg['max_iters']}, scenes sharded over "
                        f"{world} GPU(s) ({n_probs} on rank 0)")
        else:
            workload = (f"{args.config}: {cfg['n_models']} models x {cfg['n_scenes']} scenes per GPU, "
                        f"{cfg['nq']}x{cfg['nt']} descriptors, maxIters {cfg['max_iters']}")
        out = {
            "metric": metric, "value": round(value, 3), "unit": "problems/s", "n_gpus": world,
            "ranks_seen": ranks_seen, "steps": args.steps,
            "warmup": n_warm, "ms_per_step": round(1e3 * el / args.steps, 3),
            "host_enqueue_ms_per_step": round(1e3 * t_host / args.steps, 3), "higher_is_better": True,
            "scaling": "strong" if sharded else "weak", "vs_baseline": None,
            "dtype": "i8-MFMA exact-int distances (i32 acc)" + ("" if knn_only else
                                                               ", fp64 DLT/Jacobi, fp32 reprojection"),
            "data": "synthetic SIFT-like integer descriptors (seeded)" + ("" if knn_only else
                                                                        ", planted geometric inliers"),
            "config": {"workload": workload, "problems_per_gpu": n_probs, "global_batch": global_batch,
                       "parallelism": f"dp{world}", "batches_in_flight": nf, "dist_backend": args.dist_backend,
                       "hw_queues": int(os.environ["GPU_MAX_HW_QUEUES"])},
        }
        if sharded and args.shard_of > 0 and world == 1:
            out["config"]["emulated_shard"] = (f"rank 0's shard of a {args.shard_of}-rank run ({n_probs} problems): "
                                               f"per-GPU rate at that strong-scaling point, not a whole-job value")
        if warm_note := ("" if n_warm == args.warmup else f"--warmup {args.warmup} raised to {n_warm}: every one of "
                                                            f"the {nf} contexts runs once before the timed region"):
            out["warmup_note"] = warm_note
        if res is not None:
            out["accepted_problems_rank0"] = int((res["status"] == 0).sum())
        if roof:
            out["roofline"] = roof
        if cpu is not None:
            out["cpu_baseline"] = cpu
        out["parity"] = {"checked": int(tot[0]), "mismatch": int(tot[1]), "ranks": world,
                         "first": (bad[0] if bad else None),
                         "stream_short_records_timed": int(tot[2]),
                         "reference": "oracle/ restatement of OpenCV 4.5.4 (parity unpinned vs OpenCV itself)"}
        if int(tot[2]):
            out["parity"]["mismatch"] = int(tot[1]) + int(tot[2])
        if gather_check is not None:
            gather_check["ranks_own_row_differs"] = int(tot[3])  # summed over ranks
            out["gather"] = gather_check
        if os.environ.get("MIM_BENCH_GATHER", "1") == "0":
            out["diagnostic"] = "MIM_BENCH_GATHER=0: the per-step record gather left out (not a contract line)"
        print(json.dumps(out), flush=True)
    for mm in matchers:
        mm.close()


if __name__ == "__main__":
    main()
