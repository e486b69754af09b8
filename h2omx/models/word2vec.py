"""Word2Vec (H2O ``H2OWord2vecEstimator``): skip-gram word embeddings.

Input: a frame whose single string / categorical column holds one token
per row, sentences separated by NA rows (H2O's ``tokenize`` layout).

Training runs on the device that holds the frame: the vocabulary is the
level set filtered by ``min_word_freq`` (counts all-reduced over ranks),
frequent words are sub-sampled with word2vec's ``sent_sample_rate`` rule,
and every epoch builds all (centre, context) pairs inside a window of
``window_size`` (randomly shrunk per centre, as in word2vec) with tensor
ops, then updates the input/output embeddings in shuffled mini-batches
(fused gather -> dot -> sigmoid -> scatter-add).  The output layer uses
negative sampling (5 noise words from the unigram^0.75 distribution);
H2O's default hierarchical softmax (``norm_model="HSM"``) is accepted and
trained with the same negative-sampling objective.  The learning rate decays
linearly from ``init_learning_rate``.  Multi-rank: each rank trains on its
shard and the embeddings are averaged after every epoch (one all-reduce,
H2O's per-iteration model averaging).

``find_synonyms(word, count)`` ranks by cosine similarity;
``transform(frame, aggregate_method)`` returns per-token vectors (``NONE``)
or per-sentence averages (``AVERAGE``); ``to_frame()`` exports the vectors.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..frame.frame import ENUM, Frame, Vec
from .base import Model, ModelBuilder, ModelCategory


class Word2VecModel(Model):
    algo = "word2vec"
    algo_full_name = "Word2Vec"

    def __init__(self, builder, model_id, words, vectors):
        super().__init__(builder, model_id)
        self.words = words                  # vocabulary (list of str)
        self.vectors = vectors              # [V][d] float32 (device of training)
        self.index = {w: i for i, w in enumerate(words)}

    def find_synonyms(self, word: str, count: int = 20) -> dict:
        if word not in self.index:
            return {}
        V = torch.nn.functional.normalize(self.vectors.float(), dim=1)
        sim = V @ V[self.index[word]]
        sim[self.index[word]] = -2.0
        k = min(count, sim.numel() - 1)
        val, idx = torch.topk(sim, k)
        return {self.words[int(i)]: float(v) for v, i in zip(val.cpu(), idx.cpu())}

    def _lookup(self, frame: Frame) -> tuple[torch.Tensor, torch.Tensor]:
        v = frame.vecs[0]
        if v.vtype != ENUM:
            raise ValueError("word2vec transform needs a string / categorical column")
        dom = v.domain or []
        lut = torch.tensor([self.index.get(d, -1) for d in dom] + [-1], dtype=torch.long)
        codes = v.data.long().cpu()
        ids = lut[torch.where(codes >= 0, codes, torch.full_like(codes, len(dom)))]
        return ids.to(self.vectors.device), (codes < 0).to(self.vectors.device)

    def transform(self, frame: Frame, aggregate_method: str = "NONE") -> Frame:
        ids, brk = self._lookup(frame)
        d = self.vectors.shape[1]
        E = torch.cat([self.vectors.float(), torch.full((1, d), float("nan"), device=self.vectors.device)])
        X = E[torch.where(ids >= 0, ids, torch.full_like(ids, E.shape[0] - 1))]    # [n][d]
        if str(aggregate_method).upper() == "AVERAGE":
            sid = torch.cumsum(brk.long(), 0)
            keep = ~brk & (ids >= 0)
            S = int(sid.max()) + 1 if sid.numel() else 0
            sums = torch.zeros((S, d), device=X.device).index_add_(0, sid[keep], X[keep])
            cnt = torch.zeros(S, device=X.device).index_add_(0, sid[keep], torch.ones_like(sid[keep], dtype=torch.float32))
            # sentences = maximal runs of non-NA rows
            starts = torch.unique(sid[~brk])
            A = sums[starts] / cnt[starts].clamp_min(1)[:, None]
            A[cnt[starts] == 0] = float("nan")
            X = A
        return Frame([Vec(f"C{j + 1}", X[:, j].float(), "real") for j in range(d)])

    def to_frame(self) -> Frame:
        d = self.vectors.shape[1]
        vecs = [Vec("Word", torch.arange(len(self.words), dtype=torch.int32), ENUM, list(self.words))]
        vecs += [Vec(f"V{j + 1}", self.vectors[:, j].float().cpu(), "real") for j in range(d)]
        return Frame(vecs)

    def predict_raw(self, frame):
        raise ValueError("word2vec: use transform() / find_synonyms()")

    def model_performance(self, frame=None):
        return self.training_metrics

    def summary(self):
        return {"model_id": self.model_id, "vocab_size": len(self.words), "vec_size": int(self.vectors.shape[1])}


def _apply(W: torch.Tensor, idx: torch.Tensor, grad: torch.Tensor, cap: float = 8.0) -> None:
    """Hogwild-style batched update: a word hit k times in the batch moves by
    its mean gradient times min(k, cap) (plain summed SGD for rare words, no
    blow-up for the few very frequent ones)."""
    u, inv, cnt = torch.unique(idx, return_inverse=True, return_counts=True)
    G = torch.zeros((u.numel(), W.shape[1]), dtype=W.dtype, device=W.device).index_add_(0, inv, grad)
    c = cnt.to(W.dtype)
    W.index_add_(0, u, -G * (c.clamp(max=cap) / c)[:, None])


class H2OWord2vecEstimator(ModelBuilder):
    algo = "word2vec"
    UNSUPERVISED_CATEGORY = ModelCategory.DIMREDUCTION
    DEFAULTS = dict(min_word_freq=5, word_model="SkipGram", norm_model="HSM", vec_size=100, window_size=5,
                    sent_sample_rate=1e-3, init_learning_rate=0.025, epochs=5, pre_trained=None,
                    negative_samples=5, batch_size=4096)

    def train(self, x=None, y=None, training_frame=None, validation_frame=None, comm=None, **kw):
        if training_frame is None and self.params.get("pre_trained") is not None:
            training_frame = self.params["pre_trained"]
        return super().train(x=x, y=None, training_frame=training_frame, validation_frame=validation_frame,
                             comm=comm, **kw)

    def _fit(self, train: Frame, valid, model_id):
        p_ = self.params
        if str(p_["word_model"]).lower() != "skipgram":
            raise ValueError("word2vec: word_model must be 'SkipGram'")
        comm = self.comm
        world = comm.world_size if comm is not None else 1
        pre = p_.get("pre_trained")
        if pre is not None:
            return self._from_pretrained(pre, model_id)
        if len(self.x) != 1 or self.feature_types[self.x[0]] != ENUM:
            raise ValueError("word2vec needs exactly one string / categorical column")
        col = train.vec(self.x[0])
        dom = list(col.domain or [])
        dev = train.device
        codes = col.data.long()
        L = len(dom)
        counts = torch.bincount(codes[codes >= 0], minlength=L).double()
        if world > 1:
            comm.all_reduce_(counts)
        keep = counts >= int(p_["min_word_freq"])
        vocab_codes = torch.nonzero(keep).flatten()
        V = vocab_codes.numel()
        if V == 0:
            raise ValueError("word2vec: no word reaches min_word_freq")
        words = [dom[int(i)] for i in vocab_codes.cpu()]
        remap = torch.full((L + 1,), -1, dtype=torch.long, device=dev)
        remap[vocab_codes.to(dev)] = torch.arange(V, device=dev)
        tok = remap[torch.where(codes >= 0, codes, torch.full_like(codes, L))]     # -1: OOV or break
        brk = codes < 0
        freq = counts[vocab_codes].to(dev)
        total = float(freq.sum())
        d = int(p_["vec_size"])
        seed = self._seed()
        g = torch.Generator(device=dev).manual_seed(seed)
        gcpu = torch.Generator().manual_seed(seed)
        Win = ((torch.rand((V, d), generator=gcpu) - 0.5) / d).to(dev)
        Wout = torch.zeros((V, d), device=dev)
        if world > 1:
            comm.broadcast_(Win, 0)
        noise = freq.pow(0.75)
        noise = (noise / noise.sum()).float()
        s = float(p_["sent_sample_rate"])
        if s > 0:
            fr = freq / total
            keep_p = ((torch.sqrt(fr / s) + 1) * s / fr).clamp(max=1.0).float()
        else:
            keep_p = torch.ones(V, device=dev)
        sid_all = torch.cumsum(brk.long(), 0)
        win = int(p_["window_size"])
        neg = int(p_["negative_samples"])
        B = int(p_["batch_size"])
        epochs = int(p_["epochs"])
        lr0 = float(p_["init_learning_rate"])
        # pair count estimate for the linear learning-rate decay
        n_tok = int((tok >= 0).sum())
        est_pairs = max(1, epochs * n_tok * win)
        done = 0
        hist = []
        for ep in range(epochs):
            ok = tok >= 0
            if s > 0:
                ok &= torch.rand(tok.shape, generator=g, device=dev) < keep_p[tok.clamp_min(0)]
            pos = torch.nonzero(ok).flatten()
            t_ids, t_sid = tok[pos], sid_all[pos]
            m = pos.numel()
            shrink = torch.randint(1, win + 1, (m,), generator=g, device=dev)   # per-centre window
            cs, cx = [], []
            for o in range(1, win + 1):
                if o >= m:
                    break
                same = t_sid[o:] == t_sid[:-o]
                a = torch.nonzero(same & (shrink[:-o] >= o)).flatten()          # centre i, context i+o
                b = torch.nonzero(same & (shrink[o:] >= o)).flatten()           # centre i+o, context i
                cs += [t_ids[a], t_ids[b + o]]
                cx += [t_ids[a + o], t_ids[b]]
            if not cs:
                break
            C = torch.cat(cs)
            X = torch.cat(cx)
            perm = torch.randperm(C.numel(), generator=g, device=dev)
            C, X = C[perm], X[perm]
            loss_sum, loss_n = 0.0, 0
            for b0 in range(0, C.numel(), B):
                c, x = C[b0:b0 + B], X[b0:b0 + B]
                lr = max(lr0 * (1 - done / est_pairs), lr0 * 1e-4)
                done += c.numel()
                nz = torch.multinomial(noise, c.numel() * neg, replacement=True, generator=g).view(-1, neg)
                tgt = torch.cat([x[:, None], nz], 1)                             # [b][1+neg]
                lab = torch.zeros(tgt.shape, device=dev)
                lab[:, 0] = 1.0
                u = Win[c]                                                        # [b][d]
                v = Wout[tgt]                                                     # [b][1+neg][d]
                sc = torch.sigmoid((v * u[:, None, :]).sum(-1))
                gsc = (sc - lab) * lr                                             # [b][1+neg]
                gu = (gsc[..., None] * v).sum(1)
                gv = gsc[..., None] * u[:, None, :]
                _apply(Win, c, gu)
                _apply(Wout, tgt.flatten(), gv.reshape(-1, d))
                if b0 % (64 * B) == 0:
                    l = -(torch.log(sc[:, 0].clamp_min(1e-7)).mean() + torch.log((1 - sc[:, 1:]).clamp_min(1e-7))
                          .sum(1).mean())
                    loss_sum += float(l)
                    loss_n += 1
            if world > 1:
                comm.all_reduce_(Win)
                comm.all_reduce_(Wout)
                Win /= world
                Wout /= world
            hist.append({"epochs": ep + 1, "training_loss": loss_sum / max(loss_n, 1)})
        model = Word2VecModel(self, model_id, words, Win)
        model.scoring_history = hist
        model.training_metrics = {"vocab_size": V, "training_loss": hist[-1]["training_loss"] if hist else float("nan")}
        return model

    def _from_pretrained(self, pre, model_id):
        """H2O ``pre_trained``: a frame with the words in column 0 and vec_size vectors after it."""
        words_v = pre.vecs[0]
        words = [words_v.domain[int(c)] if words_v.vtype == ENUM else str(c) for c in words_v.data.cpu().tolist()]
        M = torch.stack([v.as_float() for v in pre.vecs[1:]], 1).float()
        model = Word2VecModel(self, model_id, words, M)
        model.training_metrics = {"vocab_size": len(words)}
        return model
