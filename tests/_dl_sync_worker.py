"""Rank body of tests/test_dl_sync_p2p_gpu.py (torch.distributed.run, ranks
sharing the one GPU, gloo bootstrap, device P2P exchanges): H2O DeepLearning
with ``sync_gradients=True``.  Each rank trains on its shard; with world 1 the
worker trains on the two shards' mini-batches interleaved (rank 0's 256 rows,
then rank 1's, per 512-row batch) - the concatenated-batch reference.  Every
step is checked for host-issued collectives; every rank writes one JSON
document (weights, per-step collective counts) to <out_dir>/rank<r>.json."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

from h2omx.frame import Frame  # noqa: E402
from h2omx.frame.distributed import unify_domains  # noqa: E402
from h2omx.models import H2ODeepLearningEstimator  # noqa: E402
from h2omx.models import deeplearning as DLM  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402

M, STEPS, F = 256, 24, 12


def main() -> int:
    out_dir = sys.argv[1]
    comm = Comm.from_env("cuda")
    r, w = comm.rank, comm.world_size
    rng = np.random.default_rng(11)
    n = 2 * M * STEPS
    X = rng.normal(size=(n, F)).astype(np.float32)
    logit = 1.4 * X[:, 0] - X[:, 1] + 0.7 * X[:, 2] * X[:, 3] - 0.5 * np.abs(X[:, 4])
    y = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "b", "a")
    shards = [np.arange(k * n // 2, (k + 1) * n // 2) for k in range(2)]
    if w == 2:
        rows = shards[r]
    else:   # batch k of the 1-rank run = shard 0's batch k, then shard 1's
        rows = np.concatenate([np.concatenate([s[k * M:(k + 1) * M] for s in shards]) for k in range(STEPS)])
    df = pd.DataFrame(X[rows], columns=[f"x{i}" for i in range(F)])
    df["y"] = pd.Categorical(y[rows], categories=["a", "b"])
    c = comm if w > 1 else None
    fr = unify_domains(Frame.from_pandas(df, device=comm.device), c)
    per_step = []
    step0 = DLM._DLTrainer.step

    def step(self):
        before = comm.collective_stats()
        step0(self)
        after = comm.collective_stats()
        host = sum(after[k] - before[k] for k in ("all_reduce_calls", "all_gather_calls", "broadcast_calls"))
        per_step.append({"host": host, "p2p": after["p2p_calls"] - before["p2p_calls"],
                         "graph": self.graph is not None})

    DLM._DLTrainer.step = step
    DLM._DLTrainer.FUSED = False   # the per-op chain on both sides (N ranks cannot take the fused one)
    m = H2ODeepLearningEstimator(hidden=[64, 64], epochs=1, seed=3, mini_batch_size=M * (2 // w),
                                 sync_gradients=True, shuffle_training_data=False, score_each_iteration=False
                                 ).train(y="y", training_frame=fr, comm=c)
    flat = m.net.flat.detach().cpu().numpy()
    res = {"rank": r, "world": w, "p2p": comm.p2p is not None, "steps": per_step,
           "digest": hashlib.sha256(flat.tobytes()).hexdigest(), "w": flat.tolist(),
           "tspi": int(m.train_samples_per_iteration)}
    with open(os.path.join(out_dir, f"rank{r}.json"), "w") as f:
        json.dump(res, f)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
