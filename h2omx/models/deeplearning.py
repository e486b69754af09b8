"""Deep Learning (H2O DeepLearning equivalent): a feed-forward MLP trained
with mini-batch back-propagation on the hand-written fp32 MFMA GEMM
(csrc/dense_kernels.hip gemm_kernel, bias + activation fused into the
epilogue), fused softmax-cross-entropy, activation-backward, bias-gradient
and ADADELTA / momentum-SGD update kernels.

Multi-GPU training is synchronous data parallel: every rank runs the same
mini-batch schedule on its shard and the per-layer gradient buckets are
all-reduced asynchronously as back-propagation walks down the layers (RCCL,
one bucket per layer so the last layers' reduction overlaps the earlier
layers' backward GEMMs).  H2O itself averages Hogwild replicas once per
``train_samples_per_iteration``; synchronous gradient
averaging is the MI355X-friendly equivalent and keeps replicas bit-identical.

Parameters follow H2O names.  ``mini_batch_size`` = 1 (H2O's per-row
Hogwild default) maps to a GPU mini-batch of 256 rows (fewer on small frames
so an epoch still has >= 64 updates); any larger value is used as given.
The non-adaptive learning rate is per row, as in H2O.  Supported: activations Rectifier / Tanh / Maxout /
ExpRectifier (+ WithDropout variants), input / hidden dropout, L1 / L2,
ADADELTA (``adaptive_rate``) or SGD with rate annealing and momentum ramp,
classification (softmax), regression (quadratic / absolute / huber loss,
standardized response) and autoencoders with ``anomaly()``.
"""
from __future__ import annotations

import contextlib
import gc
import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame, Vec
from ..backend import dense as D
from ..ops import dense as OD
from ..ops import mlp as OM
from .base import Model, ModelBuilder, ModelCategory
from .glm import DesignInfo

_ACT = {"rectifier": 1, "tanh": 2, "maxout": 3, "exprectifier": 4}


def _act_code(name: str) -> tuple[int, bool]:
    n = name.lower()
    drop = n.endswith("withdropout")
    if drop:
        n = n[: -len("withdropout")]
    if n not in _ACT:
        raise ValueError(f"unsupported activation {name}")
    return _ACT[n], drop


class _Net:
    """Flat parameter / gradient buffers with per-layer views."""

    def __init__(self, sizes, act, dev, gen, scale=1.0, dist="UniformAdaptive"):
        self.sizes = sizes
        self.act = act
        self.layers = []
        shapes = []
        for i in range(len(sizes) - 1):
            fan_in, out = sizes[i], sizes[i + 1]
            width = out * (2 if (act == 3 and i < len(sizes) - 2) else 1)
            shapes.append((width, fan_in))
        total = sum(w * f + w for w, f in shapes)
        self.flat = torch.empty((total,), dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.flat)
        off = 0
        init = torch.empty((total,), dtype=torch.float32)
        for (w, f) in shapes:
            nW = w * f
            if dist.lower() == "uniform":
                bound = scale
                init[off:off + nW].uniform_(-bound, bound, generator=gen)
            elif dist.lower() == "normal":
                init[off:off + nW].normal_(0.0, scale, generator=gen)
            else:  # UniformAdaptive (Glorot)
                bound = math.sqrt(6.0 / (f + w))
                init[off:off + nW].uniform_(-bound, bound, generator=gen)
            init[off + nW: off + nW + w] = 0.0
            self.layers.append((off, w, f))
            off += nW + w
        self.flat.copy_(init.to(dev))

    def W(self, i, buf=None):
        off, w, f = self.layers[i]
        b = self.flat if buf is None else buf
        return b[off: off + w * f].view(w, f)

    def b(self, i, buf=None):
        off, w, f = self.layers[i]
        b = self.flat if buf is None else buf
        return b[off + w * f: off + w * f + w]

    def span(self, i):
        off, w, f = self.layers[i]
        return off, off + w * f + w


def _forward(net: _Net, X, act, train, drop_in, drop_hid, gen_dev, out_act=0, skip_last=False):
    """Returns activations list [X, H1, ..., Z] and the maxout arg masks / dropout
    masks (``skip_last``: stop before the output layer, the caller fuses it)."""
    Hs = [X]
    aux = []
    H = X
    if train and drop_in > 0:
        m = (torch.rand(H.shape, device=H.device, generator=gen_dev) >= drop_in).float() / (1 - drop_in)
        H = H * m
        Hs[0] = H
    L = len(net.layers)
    for i in range(L):
        last = i == L - 1
        W, b = net.W(i), net.b(i)
        if last:
            if skip_last:
                break
            Z = D.gemm(H, W, bias=b, act=out_act, tb=True)
            Hs.append(Z)
            aux.append(None)
            break
        if act == 3:
            Z2 = D.gemm(H, W, bias=b, act=0, tb=True)           # [M][2*out]
            Zv = Z2.view(Z2.shape[0], -1, 2)
            Hn, arg = Zv.max(-1)
            aux.append(arg)
        elif act == 4:
            Z = D.gemm(H, W, bias=b, act=0, tb=True)
            Hn = torch.nn.functional.elu(Z)
            aux.append(None)
        else:
            Hn = D.gemm(H, W, bias=b, act=act, tb=True)
            aux.append(None)
        if train and drop_hid[i] > 0:
            m = (torch.rand(Hn.shape, device=Hn.device, generator=gen_dev) >= drop_hid[i]).float() / (1 - drop_hid[i])
            Hn = Hn * m
            aux[-1] = (aux[-1], m)
        else:
            aux[-1] = (aux[-1], None)
        Hs.append(Hn)
        H = Hn
    return Hs, aux


def _pad8(x: int) -> int:
    return (x + 7) // 8 * 8


class _Bf16Mlp:
    """bf16-operand training step of a Rectifier / Tanh MLP (no maxout, no
    dropout) on the bf16 matrix cores (ops.dense.gemm_bf16_nt: fp32
    accumulation, bias / activation / activation-derivative fused into the
    epilogue, which also writes the transposed bf16 copies the weight
    gradients read).  The fp32 master weights and the optimizer stay in fp32
    (``net.flat``); ``refresh()`` re-derives the bf16 weights after an update.
    All activation buffers are persistent and zero-padded to 8-element rows.
    """

    def __init__(self, net: _Net, act: int, batch: int, dev, out_act: int = 0):
        if act not in (1, 2) or batch % 8:
            raise ValueError("bf16 MLP path needs Rectifier/Tanh and a batch that is a multiple of 8")
        self.net, self.act, self.B, self.out_act = net, act, batch, out_act
        self.L = L = len(net.layers)
        self.shapes = [(w, f) for (_, w, f) in net.layers]
        self.kp = [_pad8(f) for (w, f) in self.shapes]
        self.wp = [_pad8(w) for (w, f) in self.shapes]

        def z(*shape):
            return torch.zeros(shape, dtype=torch.bfloat16, device=dev)

        self.Wb = [z(w, kp) for (w, f), kp in zip(self.shapes, self.kp)]
        self.Wbt = [z(f, wp) for (w, f), wp in zip(self.shapes, self.wp)]
        self.H = [None] + [z(batch, self.kp[i]) for i in range(1, L)]
        # transposed layer inputs carry an extra row of ones: the weight-gradient
        # GEMM then also produces the bias gradient (its last output column)
        self.Ht = [None] + [self.with_ones_row(z(self.shapes[i][1] + 1, batch)) for i in range(1, L)]
        self.logits = torch.zeros((batch, self.shapes[-1][0]), dtype=torch.float32, device=dev)
        self.loss = torch.zeros((1,), dtype=torch.float32, device=dev)
        self.dZ = [z(batch, self.wp[i]) for i in range(L)]
        self.dZt = [z(self.shapes[i][0], batch) for i in range(L)]
        self.Xb = z(batch, self.kp[0])
        self.Xbt = self.with_ones_row(z(self.shapes[0][1] + 1, batch))
        self.refresh()

    @staticmethod
    def with_ones_row(t: torch.Tensor) -> torch.Tensor:
        t[-1].fill_(1.0)
        return t

    def refresh(self) -> None:
        """fp32 master weights -> bf16 [w][kp] and transposed [f][wp] copies (one launch)."""
        D.cvt_bf16_multi([(self.net.W(i), self.Wb[i], self.Wbt[i]) for i in range(self.L)])

    def load_batch(self, xb: torch.Tensor):
        """fp32 [B][d] mini-batch -> bf16 row-major + transposed (ones row kept) staging buffers."""
        D.cvt_bf16(xb, out=self.Xb, out_t=self.Xbt)
        return self.Xb, self.Xbt

    def forward(self, xb: torch.Tensor) -> torch.Tensor:
        """xb: bf16 [B][kp0] (row stride multiple of 8).  Returns fp32 logits [B][K]."""
        H = xb
        for i in range(self.L):
            w, f = self.shapes[i]
            if i == self.L - 1:
                D.gemm_bf16_nt(H, self.Wb[i], self.B, w, self.kp[i], bias=self.net.b(i), act=self.out_act,
                               out_f32=self.logits)
            else:
                D.gemm_bf16_nt(H, self.Wb[i], self.B, w, self.kp[i], bias=self.net.b(i), act=self.act,
                               out_bf16=self.H[i + 1], out_bf16_t=self.Ht[i + 1])
                H = self.H[i + 1]
        return self.logits

    def loss_grad(self, y: torch.Tensor) -> None:
        """Softmax cross-entropy of the last forward's logits: bf16 dZ / dZ^T of the output layer."""
        self.loss.zero_()
        D.softmax_xent_bf16(self.logits, y, self.dZ[self.L - 1], self.dZt[self.L - 1], self.loss)

    def backward(self, dZ: torch.Tensor | None, xbt: torch.Tensor, comm=None, world: int = 1) -> None:
        """dZ: fp32 [B][K] loss gradient of the logits, or None after ``loss_grad``;
        xbt: bf16 [d + 1][>=B] (the batch's inputs transposed, last row ones).
        Writes net.grad (all-reduced when world > 1)."""
        net, B = self.net, self.B
        L = self.L
        if dZ is not None:
            D.cvt_bf16(dZ, out=self.dZ[L - 1], out_t=self.dZt[L - 1])
        handles = []
        for i in range(L - 1, -1, -1):
            w, f = self.shapes[i]
            Hin_t = xbt if i == 0 else self.Ht[i]
            tiles = -(-w // 128) * -(-(f + 1) // 128)
            S = max(1, min(64, 256 // tiles, B // 256))
            D.gemm_bf16_nt(self.dZt[i], Hin_t, w, f + 1, B, out_f32=net.W(i, net.grad), splitk=S,
                           c_last=net.b(i, net.grad))
            if comm is not None and world > 1:
                a, b = net.span(i)
                handles.append(comm.all_reduce_bucket_(net.grad[a:b]))
            if i == 0:
                break
            D.gemm_bf16_nt(self.dZ[i], self.Wbt[i], B, f, self.wp[i], ymask=self.H[i], mask_act=self.act,
                           out_bf16=self.dZ[i - 1], out_bf16_t=self.dZt[i - 1])
        for h in handles:
            h.wait()
        if comm is not None and world > 1:
            net.grad.div_(world)


class _DLTrainer:
    """One rank's mini-batch training loop (H2O DeepLearningTask's role).

    Replica synchronisation when the job spans several GPUs:

    * **model averaging** (default; H2O semantics): each
      rank trains its own replica on its shard for one *iteration* of
      ``train_samples_per_iteration`` samples, then one all-reduce averages the
      weights and the ADADELTA accumulators (H2O averages its
      DeepLearningModelInfo the same way).  ``train_samples_per_iteration``:
      > 0 global samples per iteration, 0 one epoch, -1 every rank's whole shard,
      -2 (default) auto-tuned so that the averaging all-reduce costs
      ``target_ratio_comm_to_comp`` of the compute, timed on the first
      iteration and agreed across ranks.  Over xGMI this turns one 3.6 MB
      all-reduce per 256-row mini-batch into one per iteration.
    * ``sync_gradients=True``: a gradient all-reduce per mini-batch, bucketed
      per layer and overlapped with back-propagation (replicas bit-identical).
    """

    PROBE_STEPS = 32
    # path switches (class attributes; the GPU tests flip them with monkeypatch):
    # bias / output-layer gradient folds inside the ADADELTA kernel (fewer
    # launches), the fused latency-optimised step chain (ops/mlp.py), HIP-graph
    # replay of the update
    FOLD = True
    FUSED = True
    GRAPH = True

    def __init__(self, p_, net, X, Y, act, cls, auto, drop_in, hd, M, steps_per_epoch, comm, gen, gen_dev,
                 n_hidden, backward):
        self.p, self.net, self.X, self.Y = p_, net, X, Y
        self.act, self.cls, self.auto = act, cls, auto
        self.drop_in, self.hd, self.M = drop_in, hd, M
        self.steps_per_epoch = steps_per_epoch
        self.comm = comm
        self.world = comm.world_size if comm is not None else 1
        self.gen, self.gen_dev = gen, gen_dev
        self.backward = backward
        self.adaptive = bool(p_["adaptive_rate"])
        P = net.flat.numel()
        dev = net.flat.device
        self.sync_grad = self.world > 1 and bool(p_.get("sync_gradients"))
        self.avg = self.world > 1 and not self.sync_grad
        if self.avg:
            # weights (+ ADADELTA accumulators) in one buffer: one all-reduce per iteration
            state = torch.zeros(((3 if self.adaptive else 1) * P,), dtype=torch.float32, device=dev)
            state[:P].copy_(net.flat)
            net.flat = state[:P]
            self.state = state
            self.Eg2 = state[P:2 * P] if self.adaptive else torch.zeros_like(net.flat)
            self.Edx2 = state[2 * P:] if self.adaptive else torch.zeros_like(net.flat)
        else:
            self.Eg2 = torch.zeros_like(net.flat)
            self.Edx2 = torch.zeros_like(net.flat)
        self.V = torch.zeros_like(net.flat)
        self.l1, self.l2 = float(p_["l1"]), float(p_["l2"])
        self.loss_kind = str(p_["loss"]).lower()
        self.samples = 0
        self.n_steps = 0
        self.since_sync = 0
        self.perm = None
        self.spi = None      # steps per iteration (model averaging)
        self.graph = None
        self.graph_g = None
        self.pending = 0
        self.idx_buf = None
        self._t0 = None
        if self.avg:
            t = int(p_.get("train_samples_per_iteration", -2))
            if t == 0 or t == -1:
                self.spi = steps_per_epoch
            elif t > 0:
                self.spi = max(1, round(t / (self.world * M)))
        # h2omx extension: precision="bf16" trains Rectifier / Tanh nets without dropout
        # on the bf16 matrix cores (fp32 accumulation, fp32 master weights / optimizer)
        self.mlp = None
        if (str(p_.get("precision", "fp32")).lower() == "bf16" and X.is_cuda and act in (1, 2) and drop_in == 0
                and not any(hd[:n_hidden]) and M % 8 == 0):
            self.mlp = _Bf16Mlp(net, act, M, dev)
        # fp32 small-batch updates (the estimator defaults' 256-row mini-batches) as
        # one chain of latency-optimised launches: forward, loss gradient, backward
        # and ADADELTA (ops/mlp.py).  FUSED = False keeps the per-op path.
        self.fused = None
        classes = net.layers[-1][1]
        regression = not cls and not auto
        if (self.mlp is None and not self.sync_grad and self.FUSED
                and not auto and (cls or self.loss_kind in ("automatic", "quadratic"))
                and OM.FusedMlpStep.supported(net, act, classes, regression, drop_in > 0 or any(hd[:n_hidden]),
                                              self.adaptive, M)):
            self.fused = OM.FusedMlpStep(net, act, M, self.Eg2, self.Edx2, float(p_["rho"]), float(p_["epsilon"]),
                                         self.l2, regression=regression)

    def samples_per_iteration(self) -> int:
        """global samples between replica synchronisations (0: single GPU)"""
        if self.world == 1:
            return 0
        if self.sync_grad:
            return self.world * self.M
        return self.world * self.M * (self.spi or self.steps_per_epoch)

    def graph_eligible(self) -> bool:
        """the whole update replays as one HIP graph: device data, ADADELTA, no
        dropout / L1 / max_w2 / host-issued collectives (host-side state per
        step).  Synchronous gradients qualify when their bucket all-reduces are
        device-side P2P kernels (Comm.all_reduce_bucket_): an N-rank step is then
        one graph replay too."""
        sync_ok = not self.sync_grad or bool(getattr(self.comm, "graph_collectives", False))
        return (self.X.is_cuda and self.adaptive and self.drop_in == 0 and not any(self.hd) and self.l1 == 0
                and not math.isfinite(float(self.p["max_w2"])) and sync_ok
                and self.GRAPH)

    # single-GPU graph replays: GROUP consecutive mini-batches per launch (the
    # inter-graph gap and the per-step index copy paid once per group)
    GROUP = 8

    def step_deferred(self) -> None:
        """step(), possibly held back so GROUP steps replay as one graph;
        readers of the weights call flush() first (the training loop does at
        every scoring point, bench.py inside its timed window)."""
        if self.graph is None or self.world != 1 or self.GROUP <= 1:
            self.flush()
            self.step()
            return
        self.pending += 1
        e_pos = (self.n_steps + self.pending - 1) % self.steps_per_epoch
        if e_pos == self.steps_per_epoch - 1 or self.pending == self.GROUP:
            self.flush()

    def flush(self) -> None:
        k = getattr(self, "pending", 0)
        self.pending = 0
        if k <= 0:
            return
        e_pos = self.n_steps % self.steps_per_epoch
        if k == self.GROUP and e_pos != 0 and e_pos + k <= self.steps_per_epoch:
            self._group_replay(e_pos, k)
        else:
            for _ in range(k):
                self.step()

    def _group_replay(self, e_pos: int, k: int) -> None:
        M = self.M
        if self.graph_g is None:
            self.idx_g = torch.empty((k * M,), dtype=self.idx_buf.dtype, device=self.idx_buf.device)
            self.idx_g.copy_(self.perm[e_pos * M:(e_pos + k) * M])
            g = torch.cuda.CUDAGraph()
            gc_was = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g):
                    # the group's k mini-batches gathered by two launches, not 2 k
                    xg = self.X.index_select(0, self.idx_g)
                    yg = self.Y.index_select(0, self.idx_g) if not self.auto else None
                    for i in range(k):
                        self._body(None, xg[i * M:(i + 1) * M], None if yg is None else yg[i * M:(i + 1) * M])
            finally:
                if gc_was:
                    gc.enable()
            self.graph_g = g
        else:
            self.idx_g.copy_(self.perm[e_pos * M:(e_pos + k) * M])
        self.graph_g.replay()
        self.samples += M * self.world * k
        self.n_steps += k
        self.since_sync += k

    def step(self) -> None:
        p_, M = self.p, self.M
        e_pos = self.n_steps % self.steps_per_epoch
        n = self.X.shape[0]
        if e_pos == 0:
            self.perm = (torch.randperm(n, generator=self.gen).to(self.X.device) if p_["shuffle_training_data"]
                         else torch.arange(n, device=self.X.device))
        idx = self.perm[e_pos * M:(e_pos + 1) * M]
        # small mini-batches are launch-bound (~25 kernels of a few us): after one eager
        # step (workspaces allocated) the update is captured once and replayed with the
        # batch's row ids copied into a fixed index buffer
        if self.graph is not None:
            self.idx_buf.copy_(idx)
            self.graph.replay()
        elif self.n_steps >= 1 and self.graph_eligible():
            self.idx_buf = idx.clone()
            g = torch.cuda.CUDAGraph()
            # no automatic garbage collection while the stream captures: a cyclic
            # earlier model holding a graph (e.g. a tree booster's TreeGraph) would
            # be destroyed mid-capture, which aborts the process
            gc_was = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.graph(g):
                    self._body(self.idx_buf)
            finally:
                if gc_was:
                    gc.enable()
            self.graph = g
            g.replay()
        else:
            self._body(idx)
        self.samples += M * self.world
        self.n_steps += 1
        self.since_sync += 1
        if not self.avg:
            return
        if self.spi is None:
            self._autotune()
        elif self.since_sync >= self.spi:
            self.sync()

    def _body(self, idx, xb=None, yb=None) -> None:
        """one mini-batch update (forward, loss gradient, backward, optimizer) of
        rows ``idx``, or of the pre-gathered batch (xb, yb)"""
        p_, net, M = self.p, self.net, self.M
        if xb is None:
            xb = self.X.index_select(0, idx)
            yb = self.Y.index_select(0, idx) if not self.auto else None
        if self.fused is not None:
            self.fused.step(xb.contiguous(), yb)
            if self.l1 > 0:
                net.flat.sub_(self.l1 * torch.sign(net.flat))
            if math.isfinite(float(p_["max_w2"])):
                H2ODeepLearningEstimator._clip_w2(net, float(p_["max_w2"]))
            return
        mlp = self.mlp
        if mlp is not None:
            xbb, xbt = mlp.load_batch(xb)
            Z = mlp.forward(xbb)
            Hs = aux = None
        else:
            L = len(net.layers)
            fuse = self.cls and not self.auto and OD.out_softmax_ok(xb, net.W(L - 1))
            Hs, aux = _forward(net, xb, self.act, True, self.drop_in, self.hd, self.gen_dev, skip_last=fuse)
            if fuse:   # output layer + softmax cross-entropy gradient in one launch
                Z, dZ = OD.gemm_softmax_xent(Hs[-1], net.W(L - 1), net.b(L - 1), yb)
                Hs.append(Z)
                aux.append(None)
            Z = Hs[-1]
        if self.auto:
            dZ = (Z - xb) * (2.0 / Z.numel())
        elif self.cls and mlp is None and fuse:
            pass
        elif self.cls:
            dZ, _ = D.softmax_xent(Z, yb, with_loss=False)
        else:
            r = Z[:, 0] - yb
            if self.loss_kind == "absolute":
                g = torch.sign(r)
            elif self.loss_kind == "huber":
                delta = float(p_["huber_alpha"])
                g = torch.clamp(r, -delta, delta)
            else:
                g = r
            dZ = (g / r.numel())[:, None].contiguous()
        comm = self.comm if self.sync_grad else None
        folds = None
        if mlp is not None:
            mlp.backward(dZ, xbt, comm, self.world)
        elif self.adaptive and comm is None and net.flat.is_cuda and self.FOLD:
            # the last reductions of the backward (bias-gradient slices, the output
            # layer's split partials) run inside the ADADELTA kernel
            with OD.defer_grad_folds() as folds:
                self.backward(net, Hs, aux, dZ, self.act, comm, self.world)
        else:
            self.backward(net, Hs, aux, dZ, self.act, comm, self.world)
        if self.adaptive and folds:
            OD.adadelta_(net.flat, net.grad, self.Eg2, self.Edx2, float(p_["rho"]), float(p_["epsilon"]), self.l2,
                         folds=folds)
        elif self.adaptive:
            D.adadelta_(net.flat, net.grad, self.Eg2, self.Edx2, float(p_["rho"]), float(p_["epsilon"]), self.l2)
        else:
            # H2O's rate is per row: a mean-gradient step over M rows takes M of them
            done = self.samples + M * self.world
            lr = M * float(p_["rate"]) / (1.0 + float(p_["rate_annealing"]) * done)
            ramp = min(1.0, done / max(float(p_["momentum_ramp"]), 1.0))
            mom = float(p_["momentum_start"]) + (float(p_["momentum_stable"]) - float(p_["momentum_start"])) * ramp
            D.sgd_momentum_(net.flat, net.grad, self.V, lr, mom, self.l2)
        if self.l1 > 0:
            net.flat.sub_(self.l1 * torch.sign(net.flat) * (1.0 if self.adaptive else float(p_["rate"])))
        if math.isfinite(float(p_["max_w2"])):
            H2ODeepLearningEstimator._clip_w2(net, float(p_["max_w2"]))
        if mlp is not None:
            mlp.refresh()

    def _autotune(self) -> None:
        """train_samples_per_iteration = -2: after PROBE_STEPS local steps, time one
        averaging all-reduce against the per-step compute and set the iteration
        length so that the all-reduce is ``target_ratio_comm_to_comp`` of it."""
        import time

        dev = self.X.device
        if self.since_sync == 1:
            _sync_dev(dev)
            self._t0 = time.perf_counter()
            return
        if self.since_sync < min(self.PROBE_STEPS, self.steps_per_epoch) + 1:
            return
        _sync_dev(dev)
        t_step = (time.perf_counter() - self._t0) / (self.since_sync - 1)
        t1 = time.perf_counter()
        self.sync()
        _sync_dev(dev)
        t_ar = time.perf_counter() - t1
        ratio = float(self.p.get("target_ratio_comm_to_comp") or 0.05)
        spi = max(1, math.ceil(t_ar / max(ratio * t_step, 1e-9)))
        spi = float(min(spi, self.steps_per_epoch))
        self.spi = int(self.comm.max_scalar(spi))       # every rank the same schedule

    def sync(self) -> None:
        """model averaging: mean of the replicas' weights (+ ADADELTA state)"""
        if not self.avg or self.since_sync == 0:
            return
        self.comm.all_reduce_(self.state)
        self.state.div_(self.world)
        if self.mlp is not None:
            self.mlp.refresh()
        self.since_sync = 0


def _sync_dev(dev) -> None:
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class DeepLearningModel(Model):
    algo = "deeplearning"
    algo_full_name = "Deep Learning"

    def __init__(self, builder, model_id, design, net, act, y_mean, y_sd, autoencoder):
        super().__init__(builder, model_id)
        self.design = design
        self.net = net
        self.act = act
        self.y_mean, self.y_sd = y_mean, y_sd
        self.autoencoder = autoencoder

    def _rows(self, frame):
        return self.design.transform(self.design.raw_matrix(frame)).T.contiguous()

    def _score(self, X, batch=65536):
        outs = []
        for s in range(0, X.shape[0], batch):
            Hs, _ = _forward(self.net, X[s:s + batch], self.act, False, 0.0, [0.0] * 16, None)
            outs.append(Hs[-1])
        return torch.cat(outs) if outs else torch.zeros((0, self.net.sizes[-1]), device=X.device)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        X = self._rows(frame)
        Z = self._score(X)
        if self.autoencoder:
            return Z.T.contiguous()
        if self.category in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL):
            return torch.softmax(Z, 1).T.contiguous()
        return (Z[:, 0] * self.y_sd + self.y_mean)[None, :]

    def anomaly(self, frame: Frame, per_feature: bool = False) -> Frame:
        """Reconstruction MSE per row (H2O ``anomaly``) for autoencoders."""
        if not self.autoencoder:
            raise ValueError("anomaly() requires an autoencoder model")
        X = self._rows(frame)
        R = self._score(X)
        err = (R - X) ** 2
        if per_feature:
            return Frame([Vec(f"reconstr_{n}.SE", err[:, j], "real") for j, n in enumerate(self.design.names)])
        return Frame([Vec("Reconstruction.MSE", err.mean(1), "real")])

    def predict(self, frame: Frame) -> Frame:
        if self.autoencoder:
            R = self.predict_raw(frame)
            return Frame([Vec(f"reconstr_{n}", R[j], "real") for j, n in enumerate(self.design.names)])
        return super().predict(frame)

    def model_performance(self, frame: Frame | None = None):
        if self.autoencoder:
            if frame is None:
                return self.training_metrics
            X = self._rows(frame)
            return {"MSE": float(((self._score(X) - X) ** 2).mean())}
        return super().model_performance(frame)

    def varimp(self):
        # Gedeon method (H2O's DL variable importance): input weights propagated
        W = [self.net.W(i).detach().abs().double().cpu() for i in range(len(self.net.layers))]
        if self.act == 3:
            W = [w.view(-1, 2, w.shape[1]).max(1).values if i < len(W) - 1 else w for i, w in enumerate(W)]
        imp = None
        for w in W[::-1]:
            r = w / w.sum(1, keepdim=True).clamp_min(1e-30)
            imp = r if imp is None else imp @ r
        v = imp.sum(0).numpy()
        names = self.design.names
        mx = v.max() if v.size and v.max() > 0 else 1.0
        order = np.argsort(-v)
        tot = v.sum() if v.sum() > 0 else 1.0
        return [(names[j], float(v[j]), float(v[j] / mx), float(v[j] / tot)) for j in order]

    def summary(self):
        rows = [{"layer": 1, "units": self.net.sizes[0], "type": "Input"}]
        for i in range(1, len(self.net.sizes)):
            last = i == len(self.net.sizes) - 1
            rows.append({"layer": i + 1, "units": self.net.sizes[i],
                         "type": ("Softmax" if self.category in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL)
                                  else "Linear") if last else self.params["activation"]})
        return {"model_id": self.model_id, "layers": rows, "parameters": int(self.net.flat.numel())}


class H2ODeepLearningEstimator(ModelBuilder):
    algo = "deeplearning"
    DEFAULTS = dict(hidden=[200, 200], epochs=10.0, activation="Rectifier", loss="Automatic",
                    input_dropout_ratio=0.0, hidden_dropout_ratios=None, l1=0.0, l2=0.0,
                    adaptive_rate=True, rho=0.99, epsilon=1e-8, rate=0.005, rate_annealing=1e-6, rate_decay=1.0,
                    momentum_start=0.0, momentum_ramp=1e6, momentum_stable=0.0, nesterov_accelerated_gradient=True,
                    mini_batch_size=1, standardize=True, autoencoder=False,
                    initial_weight_distribution="UniformAdaptive", initial_weight_scale=1.0, max_w2=float("inf"),
                    train_samples_per_iteration=-2, score_training_samples=10000, score_each_iteration=False,
                    stopping_rounds=5, stopping_metric="AUTO", stopping_tolerance=0.0, huber_alpha=0.9,
                    shuffle_training_data=True, reproducible=False, categorical_encoding="AUTO",
                    use_all_factor_levels=True, offset_column=None, balance_classes=False, checkpoint=None,
                    target_ratio_comm_to_comp=0.05, sync_gradients=False, precision="fp32")

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        if self.params.get("autoencoder"):
            y = None
        return super().train(x=x, y=y, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        comm = self.comm
        world = comm.world_size if comm is not None else 1
        dev = train.device
        act, act_drop = _act_code(p_["activation"])
        auto = bool(p_["autoencoder"])
        design = DesignInfo(self.x, self.feature_types, self.feature_domains,
                            use_all_levels=bool(p_["use_all_factor_levels"]))
        Xraw = design.raw_matrix(train)
        design.fit_standardization(Xraw, bool(p_["standardize"]), comm)
        X = design.transform(Xraw).T.contiguous()       # row-major [n][d]
        del Xraw
        n, d = X.shape
        cls = self.category in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL)
        y_mean, y_sd = 0.0, 1.0
        if auto:
            K = d
            Y = None
        elif cls:
            K = len(self.response_domain)
            Y = train.vec(self.y).data.to(torch.int32)
            ok = Y >= 0
            if not bool(ok.all()):
                X, Y = X[ok], Y[ok]
        else:
            K = 1
            Y = train.vec(self.y).as_float()
            ok = ~torch.isnan(Y)
            if not bool(ok.all()):
                X, Y = X[ok], Y[ok]
            st = torch.stack([Y.double().sum(), (Y.double() ** 2).sum(), torch.tensor(float(Y.numel()), device=dev,
                                                                                     dtype=torch.float64)])
            if comm is not None and world > 1:
                comm.all_reduce_(st)
            cnt = max(float(st[2]), 1.0)
            y_mean = float(st[0]) / cnt
            y_sd = math.sqrt(max(float(st[1]) / cnt - y_mean ** 2, 0.0)) or 1.0
            Y = ((Y - y_mean) / y_sd).float()
        n = X.shape[0]
        hidden = list(p_["hidden"])
        sizes = [d] + hidden + [K]
        seed = self._seed()
        gen = torch.Generator().manual_seed(seed)
        net = _Net(sizes, act, dev, gen, float(p_["initial_weight_scale"]), str(p_["initial_weight_distribution"]))
        epochs_done = 0.0
        ck = p_.get("checkpoint")
        if ck:
            # H2O checkpoint: continue training a previous model; `epochs` counts the total
            from ..frame.frame import DKV

            prev = DKV.get(ck) if isinstance(ck, str) else ck
            if not isinstance(prev, DeepLearningModel) or prev.net.sizes != sizes or prev.act != act:
                raise ValueError(f"checkpoint {ck!r} is not a DeepLearning model with the same architecture")
            net.flat.copy_(prev.net.flat.to(dev))
            epochs_done = float(getattr(prev, "epochs_trained", 0.0))
        if comm is not None and world > 1:
            comm.broadcast(net.flat, 0)
        gen_dev = torch.Generator(device=dev).manual_seed(seed + 1000003 * (comm.rank if comm else 0))
        drop_in = float(p_["input_dropout_ratio"] or 0.0)
        hd = p_["hidden_dropout_ratios"]
        if hd is None:
            hd = [0.5 if act_drop else 0.0] * len(hidden)
        hd = list(hd) + [0.0] * 16
        mb = int(p_["mini_batch_size"])
        # per-row Hogwild (H2O default) -> GPU mini-batches; small frames keep
        # >= 64 updates per epoch
        M = (256 if n >= 256 * 64 else max(16, n // 64)) if mb <= 1 else mb
        # every rank runs the same number of steps (synchronous allreduce)
        n_min = n
        if comm is not None and world > 1:
            n_min = int(-comm.max_scalar(-float(n)))
        epochs = max(0.0, float(p_["epochs"]) - epochs_done)
        steps_per_epoch = max(1, n_min // M)
        total_steps = max(1, int(round(epochs * steps_per_epoch))) if epochs > 0 else 0
        model = DeepLearningModel(self, model_id, design, net, act, y_mean, y_sd, auto)
        history = []
        from ..runtime.jobs import current_job
        from .scoring import ScoreKeeper

        keeper = ScoreKeeper(p_["stopping_metric"] if not auto else "mse",
                             self.category if not auto else "Regression", int(p_["stopping_rounds"] or 0),
                             float(p_["stopping_tolerance"]))
        job = current_job()
        score_every = max(1, steps_per_epoch)
        tr = _DLTrainer(p_, net, X, Y, act, cls, auto, drop_in, hd, M, steps_per_epoch, comm, gen, gen_dev,
                        len(hidden), backward=self._backward)
        self._last_trainer = tr
        step = -1
        for step in range(total_steps):
            tr.step_deferred()
            if job is not None:
                job.progress = (step + 1) / total_steps
            if (step + 1) % score_every == 0 or step == total_steps - 1:
                tr.flush()
                tr.sync()     # replicas agree before they are scored
                ent = self._score_entry(model, X, Y, cls, auto, epochs_done + (step + 1) / steps_per_epoch,
                                        tr.samples, comm)
                history.append(ent)
                mk = {"logloss": ent["training_loss"], "MSE": ent["training_loss"],
                      "mean_residual_deviance": ent["training_loss"]}
                stop = keeper.record(ent, mk)
                cancel = 1.0 if (job is not None and job.cancel_requested) else 0.0
                if comm is not None and world > 1:
                    cancel = float(comm.all_reduce_numpy(np.array([cancel]), "max")[0])
                if stop or cancel > 0:
                    break
        tr.flush()
        tr.sync()
        model.train_samples_per_iteration = tr.samples_per_iteration()
        model.scoring_history = history
        model.epochs_trained = epochs_done + (step + 1) / steps_per_epoch if total_steps else epochs_done
        if auto:
            model.training_metrics = {"MSE": history[-1]["training_loss"] if history else float("nan")}
        return model

    @staticmethod
    def _backward(net, Hs, aux, dZ, act, comm, world):
        """Back-propagation into net.grad (gradient buckets all-reduced per layer,
        overlapped with the rest of the backward, when ``comm`` syncs them).
        (A side stream for the weight gradients measured slower inside the step
        graph, profiles/r4/dl/side_stream_ab_r4u.txt, and was removed.)"""
        L = len(net.layers)
        handles = []
        bpart = None   # bias-gradient slices of dZ from the fused activation backward
        # per-layer scratch when the partial sums are folded later (deferred folds)
        layer_ns = OD._GRAD_FOLDS[0] is not None
        # W^T of the layers whose data gradient runs on the x3 GEMM, one launch
        Wts = {}
        if dZ.is_cuda and act in (1, 2):
            xi = [i for i in range(1, L) if aux[i - 1][1] is None and OD.x3_dact_layer(dZ.shape[0], net.W(i), act)]
            if xi:
                Wts = dict(zip(xi, OD.transpose_weights([net.W(i) for i in xi])))
        for i in range(L - 1, -1, -1):
            Hin = Hs[i]
            W = net.W(i)
            if (i == L - 1 and i > 0 and comm is None and act in (1, 2) and aux[i - 1][1] is None
                    and OD.out_backward_ok(dZ, Hin, net.W(i, net.grad), net.b(i, net.grad))):
                # output layer: weight / bias gradients (a pending fold) and dZ_prev in one pass
                with OD.workspace_ns(1000 + i):
                    dZ, bpart = OD.out_backward(dZ, Hin, W, net.W(i, net.grad), net.b(i, net.grad), act)
                continue
            with OD.workspace_ns(1000 + i) if layer_ns else contextlib.nullcontext():
                if bpart is not None:
                    D.wgrad_bias(dZ, Hin, net.W(i, net.grad), net.b(i, net.grad), bpart)   # dW = dZ^T H, db
                elif i == L - 1 and D.out_layer_ok(dZ, Hin):
                    D.out_wgrad(dZ, Hin, net.W(i, net.grad), net.b(i, net.grad))          # few classes: one pass
                else:
                    D.gemm(dZ, Hin, ta=True, out=net.W(i, net.grad))          # dW = dZ^T H
                    D.bias_grad(dZ, out=net.b(i, net.grad))
            if comm is not None and world > 1:
                a, b = net.span(i)
                handles.append(comm.all_reduce_bucket_(net.grad[a:b]))
            if i == 0:
                break
            with OD.workspace_ns(i) if layer_ns else contextlib.nullcontext():
                dZ, bpart = H2ODeepLearningEstimator._dgrad(Hs, aux, dZ, W, act, i, L, Wts.get(i))
        for h in handles:
            h.wait()
        if comm is not None and world > 1:
            net.grad.div_(world)

    @staticmethod
    def _dgrad(Hs, aux, dZ, W, act, i, L, Wt=None):
        """dZ of layer i - 1 from layer i's (dZ, W): (dZ_prev, bias-gradient
        slices or None); ``Wt`` = W^T for the x3 route (OD.transpose_weights)"""
        arg, mask = aux[i - 1]
        if act in (1, 2) and mask is None and i == L - 1 and D.out_layer_ok(dZ, Hs[i]):
            return D.thin_dact(dZ, W, Hs[i], act)
        if act in (1, 2) and mask is None and D.dact_ok(dZ, W):
            # dZ_prev = (dZ W) * act'(H) and its bias-gradient slices in the GEMM epilogue
            if Wt is not None:
                return D.gemm_dact(dZ.contiguous(), W, Hs[i], act, Wt=Wt)
            return D.gemm_dact(dZ.contiguous(), W, Hs[i], act)
        dH = D.gemm(dZ, W)                                            # [M][in]
        if mask is not None:
            dH = dH * mask
        if act == 3:
            g2 = torch.zeros((dH.shape[0], dH.shape[1], 2), device=dH.device)
            g2.scatter_(2, arg[..., None], dH[..., None])
            return g2.view(dH.shape[0], -1), None
        if act == 4:
            Hn = Hs[i]
            return dH * torch.where(Hn > 0, torch.ones_like(Hn), Hn + 1.0), None
        if mask is None:
            return D.act_backward_bias(Hs[i], dH, act)
        return D.act_backward(Hs[i] / mask.clamp_min(1e-30) * (mask > 0), dH, act), None

    @staticmethod
    def _clip_w2(net, max_w2):
        for i in range(len(net.layers)):
            W = net.W(i)
            s = (W * W).sum(1, keepdim=True)
            W.mul_(torch.where(s > max_w2, torch.sqrt(max_w2 / s), torch.ones_like(s)))

    def _score_entry(self, model, X, Y, cls, auto, epoch, samples, comm):
        ns = int(self.params["score_training_samples"] or 0)
        xs = X if ns <= 0 or ns >= X.shape[0] else X[:ns]
        Z = model._score(xs)
        if auto:
            loss = float(((Z - xs) ** 2).mean())
        elif cls:
            ys = Y[: xs.shape[0]].long()
            loss = float(torch.nn.functional.cross_entropy(Z, ys))
        else:
            ys = Y[: xs.shape[0]]
            loss = float(((Z[:, 0] - ys) ** 2).mean()) * model.y_sd ** 2
        if comm is not None and comm.world_size > 1:
            loss = float(comm.all_reduce_numpy(np.array([loss]))[0]) / comm.world_size
        return {"epochs": epoch, "samples": samples, "training_loss": loss,
                ("training_logloss" if cls else "training_mse"): loss}
