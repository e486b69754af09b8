"""Rank body of tests/test_p2p_gpu.py::test_p2p_timeout_fails_the_fit (two ranks
sharing the one GPU, gloo bootstrap, one-shot P2P exchanges in the step graph).

H2OMX_FAULT_STALL="1:<tree>:<seconds>" makes rank 1 sleep before enqueueing that
tree, past H2OMX_P2P_TIMEOUT_S: rank 0's exchanges time out on the device, it
aborts the exchanges of every rank, and both ranks' fits must FAIL (PeerLost
through the job, exactly like the watchdog path) instead of returning a model
built on timed-out sums.  Each rank prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from h2omx.models.tree import TreeParams, bin_matrix, compute_edges, train_ensemble  # noqa: E402
from h2omx.parallel.comm import Comm  # noqa: E402
from h2omx.runtime.jobs import JobRegistry  # noqa: E402


def main() -> int:
    from h2omx.models.tree.boost import GpuBooster

    # the test hook is a class attribute (the production step reads no environment)
    GpuBooster.FAULT_STALL_SPEC = os.environ.get("H2OMX_FAULT_STALL")
    comm = Comm.from_env("cuda")
    r, w = comm.rank, comm.world_size
    res = {"rank": r, "p2p": comm.p2p is not None}
    rng = np.random.default_rng(3)
    n, F = 60000, 8
    X = rng.normal(size=(F, n)).astype(np.float32)
    y = (rng.random(n) < 1 / (1 + np.exp(-(X[0] - X[1] * X[2])))).astype(np.float32)
    dev = comm.device
    edges, nvb, nbt = compute_edges(torch.from_numpy(X), 63)
    lo, hi = n * r // w, n * (r + 1) // w
    bm = bin_matrix(torch.from_numpy(X[:, lo:hi]).to(dev), edges, nvb, nbt)
    yd = torch.from_numpy(y[lo:hi]).to(dev)

    def build(job):
        return train_ensemble(bm, yd, dist="bernoulli", ntrees=16, tparams=TreeParams(max_depth=5, min_rows=2),
                              seed=5, comm=comm)

    job = JobRegistry().submit("GBM", "gbm_fault", "Key<Model>", build, sync=True)
    res["job_status"] = job.status
    res["job_exception"] = job.exception
    res["model_returned"] = job.result is not None
    res["comm_failed"] = comm.failed
    print(json.dumps(res), flush=True)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
