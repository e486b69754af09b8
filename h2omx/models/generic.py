"""Generic model (H2O ``H2OGenericEstimator``): import a MOJO zip (exported
by h2omx, see ``h2omx.mojo``) as a scoring model.  ``path`` is a file on the
node; ``model_key`` is the key of an uploaded file (REST ``/3/PostFile``) or
a path registered by ``/3/ImportFiles``."""
from __future__ import annotations

from .base import ModelBuilder


class H2OGenericEstimator(ModelBuilder):
    algo = "generic"
    DEFAULTS = dict(path=None, model_key=None)

    @classmethod
    def from_file(cls, file: str, model_id: str | None = None):
        return cls(path=file, model_id=model_id).train()

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        from ..frame.frame import DKV
        from ..mojo import GenericModel

        self.params.update(kw)
        src = self.params.get("path") or self.params.get("model_key")
        if not src:
            raise ValueError("generic: path or model_key is required")
        data = None
        key = src[len("file://"):] if isinstance(src, str) and src.startswith("file://") else src
        try:
            from ..runtime.ops import _BLOBS

            data = _BLOBS.get(key)
        except ImportError:
            data = None
        if data is None:
            with open(key, "rb") as f:
                data = f.read()
        m = GenericModel(data, self.params.get("model_id"))
        m.comm = comm
        DKV.put(m.model_id, m)
        self.model = m
        return m
