"""Routing between the HIP kernel layer and the CPU reference (the one place
where a host/device choice is made).

``h2omx.ops.*`` contains only device code paths (HIP kernels on the current
stream); ``h2omx.reference.*`` contains only the NumPy/PyTorch CPU
implementations (test oracle, CPU-only deployments such as the kind/iris
config).  Models call ``dense.<op>(tensor, ...)``: the op runs where its first
tensor argument lives, so a GPU run never imports the reference package.
"""
from __future__ import annotations

import importlib

import torch


class _Dispatch:
    def __init__(self, device_module: str, host_module: str):
        self._dev_name, self._host_name = device_module, host_module
        self._dev = self._host = None

    def _device(self):
        if self._dev is None:
            self._dev = importlib.import_module(self._dev_name)
        return self._dev

    def _hostmod(self):
        if self._host is None:
            self._host = importlib.import_module(self._host_name)
        return self._host

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        dev_attr = getattr(self._device(), name)
        if not callable(dev_attr):
            return dev_attr                       # shared constants (FAMILIES, LINKS, ...)

        def call(*args, **kw):
            # device path if ANY tensor argument lives on the GPU (a host tensor in
            # the first position must not route a GPU fit to the NumPy oracle)
            tensors = [a for a in list(args) + list(kw.values()) if isinstance(a, torch.Tensor)]
            for a in args:
                if isinstance(a, (list, tuple)) and a and isinstance(a[0], (list, tuple)) and a[0] \
                        and isinstance(a[0][0], torch.Tensor):
                    tensors.append(a[0][0])
            on_gpu = any(t.is_cuda for t in tensors)
            mod = self._device() if on_gpu else self._hostmod()
            return getattr(mod, name)(*args, **kw)

        call.__name__ = name
        return call


dense = _Dispatch("h2omx.ops.dense", "h2omx.reference.dense")
