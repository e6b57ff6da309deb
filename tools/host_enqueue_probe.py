"""Host-side cost of enqueuing one bench step (no GPU waits): set registration, tables, launches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from computervision_objectdetection_featurematching_amd import Matcher, default_params  # noqa: E402
from computervision_objectdetection_featurematching_amd.synthetic import CONFIGS, SEED_BASE, make_dataset  # noqa: E402

cfg = CONFIGS["c3"]
ds = make_dataset(cfg["n_models"], cfg["n_scenes"], cfg["nq"], cfg["nt"], cfg["n_plant"], seed=SEED_BASE)
dev = torch.device("cuda", 0)
md = [torch.from_numpy(d).to(dev) for d in ds.model_desc]
mk = [torch.from_numpy(k).to(dev) for k in ds.model_kp]
sd = [torch.from_numpy(d).to(dev) for d in ds.scene_desc]
sk = [torch.from_numpy(k).to(dev) for k in ds.scene_kp]
torch.cuda.synchronize()
ms = [Matcher(0), Matcher(0)]
prm = default_params(max_iters=cfg["max_iters"])
for it in range(12):
    m = ms[it % 2]
    t0 = time.perf_counter()
    m.clear_sets()
    q = [m.add_set(d, k) for d, k in zip(md, mk)]
    t1 = time.perf_counter()
    t = [m.add_set(d, k) for d, k in zip(sd, sk)]
    t2 = time.perf_counter()
    m.match_batch_async([(q[a], t[b]) for a, b in ds.problems], prm)
    t3 = time.perf_counter()
    print(f"step {it}: add_set {1e3 * (t2 - t0):.2f} ms, match_batch_async {1e3 * (t3 - t2):.2f} ms", flush=True)
torch.cuda.synchronize()
for m in ms:
    m.close()
