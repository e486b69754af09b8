"""Safe YAML helpers (yaml.safe_load only; never the unsafe loader)."""
from __future__ import annotations

import yaml


def load_all(path: str) -> list:
    with open(path) as f:
        return [d for d in yaml.safe_load_all(f) if d is not None]


def load(path: str):
    with open(path) as f:
        return yaml.safe_load(f)
