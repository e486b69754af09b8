#!/usr/bin/env python3
"""bench.py with class / module attributes overridden (A/B of the path switches
that are constants in the code):

    python scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.FUSE_FIN=0 -- --rows 1375000 ...
    python scripts/r6/bench_ab.py h2omx.models.tree.engine:HipTreeBuilder.COLMAJOR_EVERY=3 -- scripts/drf_deep_ab.py
"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    args = sys.argv[1:]
    sep = args.index("--") if "--" in args else len(args)
    for spec in args[:sep]:
        target, val = spec.split("=", 1)
        mod, attr = target.split(":")
        obj = importlib.import_module(mod)
        *path, name = attr.split(".")
        for p in path:
            obj = getattr(obj, p)
        cur = getattr(obj, name)
        setattr(obj, name, type(cur)(int(val)) if isinstance(cur, (bool, int)) else type(cur)(val))
    rest = args[sep + 1:]
    # a script path right after "--" runs that script instead of bench.py
    if rest and rest[0].endswith(".py"):
        sys.argv = [os.path.join(ROOT, rest[0]) if not os.path.isabs(rest[0]) else rest[0]] + rest[1:]
    else:
        sys.argv = [os.path.join(ROOT, "bench.py")] + rest
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
