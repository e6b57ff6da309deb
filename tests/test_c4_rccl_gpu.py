"""C4 (BASELINE configs[3]) on the GPU through bench.py's RCCL path, in a fresh child process.

The full 256-scene global batch (10k x 10k descriptors, maxIters 50,000) runs with an RCCL ("nccl")
process group of world 1: `init_process_group("nccl", device_id=...)` and the per-step
`all_gather_into_tensor` of the result records issued on the library contexts' ExternalStreams — the
code an 8-rank run executes, on one MI355X.  Checked (problem independence,
/root/reference/src/TestsDetector.cpp:58-95):
  * every gathered record: status 0 (accepted) and 50,000 iterations (8 % inliers: no early stop);
  * the gathered row of this rank equals the records the library copied out, byte for byte, for
    every context in flight;
  * 8 problems of the batch match the oracle record for record (mask, counts, status, H)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_c4_full_batch_rccl_gather():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "c4", "--steps", "2", "--warmup", "1",
           "--inflight", "2", "--cpu-sample", "0", "--parity-sample", "8", "--iso-steps", "1",
           "--dist-backend", "nccl"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    g = d["gather"]
    assert g["collective"] == "all_gather_into_tensor" and g["backend"] == "nccl", g
    assert g["world"] == 1 and g["contexts_checked"] == 2, g
    assert g["own_row_identical"] and g["ranks_own_row_differs"] == 0, g
    assert g["records"] == 2 * 256, g
    assert g["status_counts"] == {"0": 512}, g
    assert g["iters_min"] == 50000 and g["iters_max"] == 50000, g
    assert d["config"]["global_batch"] == 256 and d["config"]["problems_per_gpu"] == 256
    p = d["parity"]
    assert p["checked"] == 8 and p["mismatch"] == 0, p
    assert p["stream_short_records_timed"] == 0
