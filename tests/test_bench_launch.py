"""CPU tests of bench.py's multi-rank launch (`--gpus N` without WORLD_SIZE spawns N ranks through
torch.distributed.run before anything touches a GPU) with the gloo dry-run mode, and of the CPU
baseline's record comparison."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(GLOO_SOCKET_IFNAME="lo", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_spawns_two_ranks():
    d = _run(["--gpus", "2", "--dry-run"])
    assert d["n_gpus"] == 2 and d["ranks_seen"] == 2 and d["dry_run"]


def test_single_rank_dry_run():
    d = _run(["--dry-run"])
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1


def test_hw_queue_defaults_per_config_reach_the_ranks():
    """24 hardware queues for the batch configs, 16 for the scene configs (bench.py main), set before HIP
    starts and inherited by the launched ranks; --hw-queues overrides."""
    assert _run(["--dry-run"])["config"]["hw_queues"] == 24
    assert _run(["--gpus", "2", "--dry-run", "--config", "c4"])["config"]["hw_queues"] == 24
    assert _run(["--gpus", "2", "--dry-run", "--config", "dataset"])["config"]["hw_queues"] == 16
    assert _run(["--dry-run", "--hw-queues", "8"])["config"]["hw_queues"] == 8


def test_cpu_parity_compare_detects_differences():
    sys.path.insert(0, ROOT)
    import bench
    from computervision_objectdetection_featurematching_amd._lib import RESULT_DTYPE
    o = dict(n_good=5, n_inl=4, status=0, iters=7, H=np.eye(3), mask=np.array([1, 1, 0, 1, 1], np.uint8),
             good_q=np.arange(5, dtype=np.int32), good_t=np.arange(5, dtype=np.int32) + 10)
    r = np.zeros(1, RESULT_DTYPE)[0]
    r["n_good"], r["n_inl"], r["status"], r["iters"] = 5, 4, 0, 7
    r["H"] = np.eye(3).ravel()
    det = (o["good_q"].copy(), o["good_t"].copy(), o["mask"].copy())
    assert bench._cmp_problem(o, r, det) is None
    det2 = (det[0], det[1], np.array([1, 1, 1, 1, 1], np.uint8))
    assert bench._cmp_problem(o, r, det2) == "inlier mask"
    r["H"][0] = 1.01
    assert bench._cmp_problem(o, r, det) == "H"


def test_c4_eight_ranks_cover_the_global_batch():
    """C4 (BASELINE configs[3]): 8 gloo ranks each take shard_range(256, 8, r) of the one global scene
    batch; rank 0 checks the gathered shards cover scene ids 0..255 exactly once."""
    d = _run(["--gpus", "8", "--dry-run", "--config", "c4"])
    assert d["n_gpus"] == 8 and d["ranks_seen"] == 8
    assert d["scene_ids_covered"] == 256 and d["global_batch"] == 256 and d["scaling"] == "strong"


def test_c4_shard_data_is_rank_independent():
    """A scene's data depends on its global id only, so any sharding of the C4 batch runs the same problems."""
    sys.path.insert(0, ROOT)
    from computervision_objectdetection_featurematching_amd.shard import shard_range
    from computervision_objectdetection_featurematching_amd.synthetic import make_dataset
    full = make_dataset(1, 8, 200, 700, 60, seed=11)
    for world in (1, 3, 8):
        for r in range(world):
            ids = shard_range(8, world, r)
            part = make_dataset(1, 8, 200, 700, 60, seed=11, scene_ids=ids)
            for j, s in enumerate(ids):
                assert np.array_equal(part.scene_desc[j], full.scene_desc[s])
                assert np.array_equal(part.scene_kp[j], full.scene_kp[s])


def test_dataset_scenes_split_round_robin_over_ranks():
    """The reference's real-data run (bench --config dataset, pipeline.process_all_test_images): its 30
    test images split round robin over 4 gloo ranks (Output.cpp:19-57 processes every scene once), the
    per-scene results all-gathered; rank 0 checks every scene came back once, from rank i mod 4."""
    d = _run(["--gpus", "4", "--dry-run", "--config", "dataset"])
    assert d["n_gpus"] == 4 and d["ranks_seen"] == 4
    assert d["scene_ids_covered"] == 30 and d["global_batch"] == 30
    assert d["ranks_of_scenes"] == [i % 4 for i in range(30)]
