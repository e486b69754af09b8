"""Tree comparison helpers for tests: reachable structure only (GPU tree heaps
keep garbage in unreachable slots; CPU reference trees are compact)."""
import numpy as np


def reachable(tr):
    keep, stack = [], [0]
    while stack:
        i = stack.pop()
        keep.append(i)
        if tr[i]["feat"] >= 0:
            stack += [int(tr[i]["left"]), int(tr[i]["left"]) + 1]
    return sorted(keep)


def same_splits(a, b) -> bool:
    ra, rb = reachable(a), reachable(b)
    return ra == rb and bool((a[ra]["feat"] == b[rb]["feat"]).all())


def frac_same(ta, tb) -> float:
    return float(np.mean([same_splits(a, b) for a, b in zip(ta, tb)]))
