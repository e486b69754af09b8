"""Synthetic data generators with the shapes of the BASELINE.json configs.

There is no network access, so the benchmark datasets (HIGGS, Airlines,
...) are replaced by generators that reproduce their *shape*: row/column
counts, column types and value distributions (continuous skewed kinematics,
discrete b-tags, categorical carriers, ...) with a planted nonlinear signal so
AUC is meaningful.  All generation happens on the target device with a
fixed seed, so every rank of a distributed run generates its own shard
without touching the host.
"""
from __future__ import annotations

import math

import torch

HIGGS_COLUMNS = (
    ["lepton_pT", "lepton_eta", "lepton_phi", "missing_energy_magnitude", "missing_energy_phi"]
    + [f"jet{j}_{k}" for j in range(1, 5) for k in ("pt", "eta", "phi", "b_tag")]
    + ["m_jj", "m_jjj", "m_lv", "m_jlv", "m_bb", "m_wbb", "m_wwbb"]
)
assert len(HIGGS_COLUMNS) == 28


def _gen(device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def higgs_like(n: int, seed: int = 42, device="cpu") -> tuple[torch.Tensor, torch.Tensor]:
    """HIGGS-shape synthetic binary classification data.

    Returns (X feature-major float32 [28][n], y float32 [n]).
    """
    dev = torch.device(device)
    g = _gen(dev, seed)
    X = torch.empty((28, n), dtype=torch.float32, device=dev)

    def expo(scale):
        u = torch.rand(n, generator=g, device=dev).clamp_min_(1e-7)
        return -torch.log(u) * scale

    def normal(std=1.0):
        return torch.randn(n, generator=g, device=dev) * std

    def phi():
        return (torch.rand(n, generator=g, device=dev) * 2 - 1) * math.pi

    # a latent "signal-ness" drives correlated shifts in the kinematics
    z = normal()
    X[0] = expo(0.8) + 0.25 * torch.sigmoid(z)
    X[1] = normal(1.0).clamp_(-2.5, 2.5)
    X[2] = phi()
    X[3] = expo(0.9) + 0.15 * z.abs()
    X[4] = phi()
    for j in range(4):
        b = 5 + 4 * j
        X[b] = expo(0.9 - 0.1 * j) + 0.1 * torch.relu(z)
        X[b + 1] = normal(1.0).clamp_(-2.5, 2.5)
        X[b + 2] = phi()
        u = torch.rand(n, generator=g, device=dev)
        X[b + 3] = torch.where(u < 0.55, 0.0, torch.where(u < 0.8, 1.0865, 2.173))
    # high-level invariant masses: log-normal around 1 with signal-dependent peaks
    for k in range(7):
        X[21 + k] = torch.exp(normal(0.35) + 0.12 * z * (1 + 0.3 * k) - 0.05 * k)
    logit = (1.1 * z
             + 0.8 * torch.tanh(X[23] * 2 - 2.0)
             - 0.6 * (X[26] - 1.0) ** 2
             + 0.35 * (X[8] + X[12]) * 0.5
             + 0.3 * torch.cos(X[2] - X[4])
             + 0.25 * X[0] * X[3]
             - 0.3)
    y = (torch.rand(n, generator=g, device=dev) < torch.sigmoid(logit)).float()
    return X, y


def higgs_like_portable(n: int, seed: int = 1) -> tuple[torch.Tensor, torch.Tensor]:
    """HIGGS-shape binary data that every x86 host generates BIT-identically:
    NumPy's PCG64 stream (scalar C) and only IEEE-exact operations (+, -, *,
    /, abs, min / max) in float64, rounded once to float32 - no
    vectorised transcendental (exp / log / sin) whose last bit depends on the
    host's SIMD level.  Used by scripts/precision_parity.py, whose GPU part
    runs on the GPU box and whose fp64-oracle part runs elsewhere: both must
    bin the same values.  Returns (X [28][n] float32 on the CPU, y [n])."""
    import numpy as np

    rng = np.random.Generator(np.random.PCG64(seed))

    def unif():
        return rng.random(n)

    def normal(std=1.0):            # Irwin-Hall: sum of 12 uniforms - 6, added one array at a time
        s = unif()
        for _ in range(11):
            s += unif()
        return (s - 6.0) * std

    def heavy(scale):               # exponential-like tail without a log: u / (1 - u)
        u = unif()
        return np.minimum(u / (1.0 - u + 1e-4), 50.0) * scale

    def angle():
        return (unif() * 2.0 - 1.0) * 3.141592653589793

    def squash(t):                  # rational sigmoid in (-1, 1)
        return t / (1.0 + np.abs(t))

    X = np.empty((28, n), np.float64)
    z = normal()
    X[0] = heavy(0.8) + 0.25 * (0.5 + 0.5 * squash(z))
    X[1] = np.clip(normal(), -2.5, 2.5)
    X[2] = angle()
    X[3] = heavy(0.9) + 0.15 * np.abs(z)
    X[4] = angle()
    for j in range(4):
        b = 5 + 4 * j
        X[b] = heavy(0.9 - 0.1 * j) + 0.1 * np.maximum(z, 0.0)
        X[b + 1] = np.clip(normal(), -2.5, 2.5)
        X[b + 2] = angle()
        u = unif()
        X[b + 3] = np.where(u < 0.55, 0.0, np.where(u < 0.8, 1.0865, 2.173))
    for k in range(7):
        t = normal(0.35) + 0.12 * z * (1 + 0.3 * k) - 0.05 * k
        X[21 + k] = 1.0 + t + 0.5 * t * t          # positive-skewed "mass" around 1
    dphi = X[2] - X[4]
    logit = (1.1 * z + 0.8 * squash(X[23] * 2.0 - 2.0) - 0.6 * (X[26] - 1.0) ** 2
             + 0.175 * (X[8] + X[12]) - 0.3 * np.minimum(np.abs(dphi), 2.0))
    pr = 0.5 + 0.5 * squash(logit)
    y = (unif() < pr).astype(np.float32)
    return torch.from_numpy(X.astype(np.float32)), torch.from_numpy(y)


def airlines_like(n: int, seed: int = 7, device="cpu") -> tuple[torch.Tensor, torch.Tensor]:
    """Airlines-shape (31 columns: dates, carrier/origin/dest codes, times,
    distance) synthetic delay classification; categoricals are integer codes."""
    dev = torch.device(device)
    g = _gen(dev, seed)
    F = 31
    X = torch.empty((F, n), dtype=torch.float32, device=dev)
    X[0] = torch.randint(1987, 2009, (n,), generator=g, device=dev).float()  # Year
    X[1] = torch.randint(1, 13, (n,), generator=g, device=dev).float()       # Month
    X[2] = torch.randint(1, 32, (n,), generator=g, device=dev).float()       # DayofMonth
    X[3] = torch.randint(1, 8, (n,), generator=g, device=dev).float()        # DayOfWeek
    dep = torch.randint(0, 2400, (n,), generator=g, device=dev).float()
    X[4] = dep
    X[5] = (dep + torch.randint(0, 30, (n,), generator=g, device=dev).float()) % 2400
    X[6] = (dep + torch.randint(30, 400, (n,), generator=g, device=dev).float()) % 2400
    X[7] = X[6]
    X[8] = torch.randint(0, 29, (n,), generator=g, device=dev).float()        # carrier code
    X[9] = torch.randint(0, 8000, (n,), generator=g, device=dev).float()      # flight num
    X[10] = torch.randint(0, 5000, (n,), generator=g, device=dev).float()     # tail num
    dist_ = torch.exp(torch.randn(n, generator=g, device=dev) * 0.6 + 6.3)
    X[11] = dist_ / 8.0 + 20
    X[12] = X[11]
    X[13] = dist_ / 8.0
    X[14] = torch.randint(0, 300, (n,), generator=g, device=dev).float()      # origin
    X[15] = torch.randint(0, 300, (n,), generator=g, device=dev).float()      # dest
    X[16] = dist_
    X[17] = torch.randint(0, 30, (n,), generator=g, device=dev).float()
    X[18] = torch.randint(0, 40, (n,), generator=g, device=dev).float()
    for k in range(19, F):
        X[k] = torch.randn(n, generator=g, device=dev)
    hour = torch.div(dep, 100, rounding_mode="floor")
    logit = (0.08 * (hour - 12) + 0.4 * torch.sin(X[1] / 12 * 2 * math.pi) + 0.3 * ((X[8] % 7) == 3).float()
             + 0.0004 * (dist_ - 600) + 0.5 * X[20] * X[21] * 0.3 - 0.2 * (X[3] > 5).float() - 0.3)
    y = (torch.rand(n, generator=g, device=dev) < torch.sigmoid(logit)).float()
    return X, y


def wide_gaussian(n: int, p: int, seed: int = 3, device="cpu", task: str = "binomial"):
    """Dense n x p standard-normal features with a sparse linear + interaction signal
    (AutoML 10M x 100 and DL 50M x 200 configs)."""
    dev = torch.device(device)
    g = _gen(dev, seed)
    X = torch.randn((p, n), generator=g, device=dev)
    beta = torch.zeros(p, device=dev)
    k = min(p, 20)
    beta[:k] = torch.linspace(1.0, -1.0, k, device=dev)
    # the k-term signal as an elementwise sum (no vendor GEMV launch)
    logit = (beta[:k, None] * X[:k]).sum(0) + 0.5 * X[0] * X[1] - 0.4 * torch.relu(X[2]) + 0.3 * torch.sin(2 * X[3])
    if task == "regression":
        y = logit + 0.5 * torch.randn(n, generator=g, device=dev)
        return X, y
    if task.startswith("multinomial"):
        y = torch.bucketize(logit, torch.tensor([-1.0, 0.0, 1.0], device=dev)).float()
        return X, y
    y = (torch.rand(n, generator=g, device=dev) < torch.sigmoid(logit)).float()
    return X, y
