"""Rank body of tests/test_p2p_gpu.py (launched by torch.distributed.run, two
ranks sharing the one GPU, gloo for the bootstrap): the one-shot P2P
all-reduce against the exact expected sums, eager and inside a HIP graph."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from h2omx.parallel.comm import Comm  # noqa: E402


def main() -> int:
    comm = Comm.from_env("cuda")
    dev, r, w = comm.device, comm.rank, comm.world_size
    res = {"rank": r, "p2p": comm.p2p is not None, "err": comm.p2p_error}
    if comm.p2p is None:
        print(json.dumps(res), flush=True)
        comm.shutdown()
        return 0
    g = torch.Generator(device="cpu").manual_seed(1234)
    checks = {}
    # int64 histograms of every tree-level size class (odd tails included)
    for n in (1, 2, 3, 7, 255, 4096 * 3 + 5, 28 * 2 * 256 * 8, 31 * 2 * 256 * 32):
        parts = [torch.randint(-2**40, 2**40, (n,), generator=g, dtype=torch.int64) for _ in range(w)]
        x = parts[r].to(dev)
        comm.all_reduce_(x)
        checks[f"i64_{n}"] = bool(torch.equal(x.cpu(), sum(parts)))
    # float64 / float32: rank-order summation, identical on every rank
    for dt in (torch.float64, torch.float32):
        parts = [torch.randn((5003,), generator=g, dtype=dt) for _ in range(w)]
        x = parts[r].to(dev)
        comm.all_reduce_(x)
        want = parts[0].clone()
        for p in parts[1:]:
            want += p
        checks[f"{dt}"] = bool(torch.equal(x.cpu(), want))
        checks[f"{dt}_digest"] = float(x.double().sum())
    # max of int32 (the tree engine's gradient maxima image)
    x = torch.tensor([r, -r, 7 * r, 3], dtype=torch.int32, device=dev)
    comm.all_reduce_(x, "max")
    checks["i32_max"] = x.cpu().tolist() == [w - 1, 0, 7 * (w - 1), 3]
    # captured in a HIP graph and replayed: the epoch advances on the device
    buf = torch.zeros((4099,), dtype=torch.int64, device=dev)
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        graph.capture_begin()
        buf.add_(r + 1)
        comm.all_reduce_(buf)
        graph.capture_end()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    buf.zero_()
    ok = True
    expect = 0
    tri = w * (w + 1) // 2
    for _ in range(5):
        graph.replay()
        torch.cuda.synchronize(dev)
        # every rank adds (rank + 1) to the summed buffer then all-reduces it
        expect = w * expect + tri
        ok &= bool((buf == expect).all())
    checks["graph_replays"] = ok
    comm.p2p.check()
    res["checks"] = checks
    res["p2p_calls"] = comm.stats["p2p_calls"]
    print(json.dumps(res), flush=True)
    comm.shutdown()
    return 0


if __name__ == "__main__":
    sys.exit(main())
