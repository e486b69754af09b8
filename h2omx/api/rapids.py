"""Rapids: H2O's frame-expression language (``POST /99/Rapids``), the
subset h2o-py emits for everyday frame munging — column / row slicing,
``asfactor``, arithmetic and comparisons, ``h2o.runif`` (split_frame),
column assignment, cbind / rbind, renaming, reductions and temp-key
management.

Every rank evaluates the expression on its own row shard (element-wise and
slicing ops are shard-local); reductions and categorical domains are
combined with the cluster communicator.
"""
from __future__ import annotations

import math
import re
import uuid

import numpy as np
import torch

from ..frame.distributed import global_nrows, unify_domains
from ..frame.frame import DKV, ENUM, INT, REAL, Frame, Vec

_TOKEN = re.compile(r'\s*(?:(\()|(\))|(\[)|(\])|"((?:[^"\\]|\\.)*)"|\'((?:[^\'\\]|\\.)*)\'|([^\s()\[\]]+))')


class Sym(str):
    pass


def parse(src: str):
    pos = 0
    stack: list[list] = [[]]
    while pos < len(src):
        m = _TOKEN.match(src, pos)
        if not m or m.end() == pos:
            if src[pos:].strip() == "":
                break
            raise ValueError(f"rapids: cannot parse near {src[pos:pos + 20]!r}")
        pos = m.end()
        lp, rp, lb, rb, dq, sq, atom = m.groups()
        if lp or lb:
            stack.append(["__list__"] if lb else [])
        elif rp or rb:
            node = stack.pop()
            if node and node[0] == "__list__":
                node = ("list", node[1:])
            stack[-1].append(node)
        elif dq is not None or sq is not None:
            stack[-1].append((dq if dq is not None else sq).encode().decode("unicode_escape"))
        else:
            stack[-1].append(_atom(atom))
    if len(stack) != 1 or len(stack[0]) != 1:
        raise ValueError("rapids: unbalanced expression")
    return stack[0][0]


def _atom(a: str):
    if a in ("TRUE", "true", "True"):
        return True
    if a in ("FALSE", "false", "False"):
        return False
    if a in ("NA", "NaN", "nan"):
        return float("nan")
    if re.fullmatch(r"[-+]?(\d+\.?\d*|\.\d+)([eE][-+]?\d+)?", a):
        f = float(a)
        return int(f) if f.is_integer() and "." not in a and "e" not in a.lower() else f
    if re.fullmatch(r"\d+:\d+", a):  # span lo:count
        lo, cnt = a.split(":")
        return ("span", int(lo), int(cnt))
    return Sym(a)


class _Ctx:
    def __init__(self, cl):
        self.cl = cl
        self.comm = cl.comm if cl is not None and cl.world_size > 1 else None


def evaluate(src: str, cl=None) -> dict:
    ctx = _Ctx(cl)
    val = _eval(parse(src), ctx)
    if isinstance(val, Frame):
        if val.key not in DKV.keys() or DKV.get(val.key) is not val:
            DKV.put(val.key, val)
        return {"key": {"name": val.key}, "num_rows": global_nrows(val, ctx.comm), "num_cols": val.ncols}
    if isinstance(val, str):
        return {"string": val}
    if isinstance(val, (list, tuple)):
        return {"scalar": [float(v) for v in val]}
    if val is None:
        return {"string": ""}
    return {"scalar": float(val)}


def _frame(v) -> Frame:
    if isinstance(v, Frame):
        return v
    fr = DKV.get(str(v))
    if not isinstance(fr, Frame):
        raise KeyError(f"rapids: frame {v!r} not found")
    return fr


def _idx_list(v, n):
    if isinstance(v, tuple) and v and v[0] == "list":
        out = []
        for x in v[1]:
            if isinstance(x, tuple) and x[0] == "span":
                out += list(range(x[1], x[1] + x[2]))
            else:
                out.append(x)
        return out
    if isinstance(v, tuple) and v[0] == "span":
        return list(range(v[1], v[1] + v[2]))
    return [v]


def _cols(fr: Frame, sel) -> list[int]:
    out = []
    for c in _idx_list(sel, fr.ncols):
        if isinstance(c, str):
            out.append(fr.names.index(str(c)))
        else:
            out.append(int(c) if c >= 0 else fr.ncols + int(c))
    return out


def _new_key():
    return f"rapids_{uuid.uuid4().hex[:10]}"


def _binop(op, a, b):
    def to_t(x, like):
        if isinstance(x, Frame):
            return x.vecs[0].as_float() if x.ncols == 1 else torch.stack([v.as_float() for v in x.vecs])
        return torch.tensor(float(x), device=like.device if like is not None else "cpu")

    fa = a if isinstance(a, Frame) else None
    fb = b if isinstance(b, Frame) else None
    base = fa or fb
    if base is None:
        return _scalar_op(op, float(a), float(b))
    names = base.names
    ta = to_t(a, base.vecs[0].data)
    tb = to_t(b, base.vecs[0].data)
    # enum == "level" comparisons
    if op in ("==", "!=") and isinstance(b, str) and fa is not None and fa.vecs[0].vtype == ENUM:
        dom = fa.vecs[0].domain
        code = dom.index(b) if b in dom else -2
        r = (fa.vecs[0].data == code).float()
        r = torch.where(fa.vecs[0].data < 0, torch.full_like(r, float("nan")), r)
        if op == "!=":
            r = 1 - r
        return Frame([Vec(names[0], r, INT)], key=_new_key())
    r = {"+": lambda: ta + tb, "-": lambda: ta - tb, "*": lambda: ta * tb, "/": lambda: ta / tb,
         "^": lambda: ta ** tb, "%": lambda: torch.remainder(ta, tb), "%%": lambda: torch.remainder(ta, tb),
         "intDiv": lambda: torch.floor(ta / tb),
         "<": lambda: (ta < tb).float(), ">": lambda: (ta > tb).float(), "<=": lambda: (ta <= tb).float(),
         ">=": lambda: (ta >= tb).float(), "==": lambda: (ta == tb).float(), "!=": lambda: (ta != tb).float(),
         "&": lambda: ((ta != 0) & (tb != 0)).float(), "|": lambda: ((ta != 0) | (tb != 0)).float(),
         "&&": lambda: ((ta != 0) & (tb != 0)).float(), "||": lambda: ((ta != 0) | (tb != 0)).float()}[op]()
    nan = torch.isnan(ta) | torch.isnan(tb) if op in ("<", ">", "<=", ">=", "==", "!=") else None
    if nan is not None:
        r = torch.where(nan, torch.full_like(r, float("nan")), r)
    logical = op in ("<", ">", "<=", ">=", "==", "!=", "&", "|", "&&", "||")
    if r.dim() == 1:
        return Frame([Vec(names[0], r.float(), INT if logical else REAL)], key=_new_key())
    return Frame([Vec(n, r[i].float(), INT if logical else REAL) for i, n in enumerate(names)], key=_new_key())


def _scalar_op(op, a, b):
    return {"+": a + b, "-": a - b, "*": a * b, "/": a / b if b else float("nan"), "^": a ** b,
            "<": float(a < b), ">": float(a > b), "<=": float(a <= b), ">=": float(a >= b), "==": float(a == b),
            "!=": float(a != b), "&": float(bool(a) and bool(b)), "|": float(bool(a) or bool(b))}[op]


def _reduce(ctx, fr: Frame, how: str, na_rm=True):
    vals = []
    for v in fr.vecs:
        x = v.as_float().double()
        ok = ~torch.isnan(x)
        xs = x[ok] if na_rm else x
        n = float(xs.numel())
        vals.append([n, float(xs.sum()) if n else 0.0, float((xs * xs).sum()) if n else 0.0,
                     float(xs.min()) if n else math.inf, -float(xs.max()) if n else math.inf])
    a = np.array(vals, np.float64)
    if ctx.comm is not None:
        s = ctx.comm.all_reduce_numpy(np.ascontiguousarray(a[:, :3]))
        m = ctx.comm.all_reduce_numpy(np.ascontiguousarray(a[:, 3:]), "min")
        a = np.concatenate([s, m], 1)
    out = []
    for n, s1, s2, mn, nmx in a:
        if how == "sum":
            out.append(s1)
        elif how == "mean":
            out.append(s1 / n if n else float("nan"))
        elif how in ("sd", "var"):
            var = (s2 - s1 * s1 / n) / (n - 1) if n > 1 else float("nan")
            out.append(math.sqrt(var) if how == "sd" else var)
        elif how == "min":
            out.append(mn)
        elif how == "max":
            out.append(-nmx)
        elif how == "nrow":
            out.append(n)
    return out[0] if len(out) == 1 else out


def _eval(node, ctx):
    if isinstance(node, Sym):
        fr = DKV.get(str(node))
        return fr if fr is not None else str(node)
    if not isinstance(node, list):
        return node
    if not node:
        return None
    op = node[0]
    args = node[1:]
    if isinstance(op, list):  # ((lambda ...)) not supported
        raise ValueError("rapids: lambdas are not supported")
    op = str(op)
    E = lambda a: _eval(a, ctx)  # noqa: E731
    if op in ("tmp=", "assign"):
        key = str(args[0])
        val = E(args[1])
        if isinstance(val, Frame):
            val = Frame(list(val.vecs), key=key)
            DKV.put(key, val)
        return val
    if op == "rm":
        DKV.remove(str(args[0]))
        return 0.0
    if op in ("cols_py", "cols"):
        fr = _frame(E(args[0]))
        return Frame([fr.vecs[i] for i in _cols(fr, args[1])], key=_new_key())
    if op == "rows":
        fr = _frame(E(args[0]))
        sel = args[1]
        if isinstance(sel, list) or isinstance(sel, Sym):
            mask = _frame(E(sel)).vecs[0].as_float()
            return fr.rows(torch.nan_to_num(mask, nan=0.0) != 0)
        idx = torch.tensor([int(i) for i in _idx_list(sel, fr.nrows)], dtype=torch.long)
        return fr.rows(idx)
    if op in ("as.factor", "asfactor"):
        fr = _frame(E(args[0]))
        for c in fr.names:
            fr = fr.asfactor(c)
        fr = unify_domains(fr, ctx.comm)
        return Frame(list(fr.vecs), key=_new_key())
    if op in ("as.numeric", "asnumeric"):
        fr = _frame(E(args[0]))
        return Frame([Vec(v.name, v.as_float(), REAL) for v in fr.vecs], key=_new_key())
    if op == "is.na":
        fr = _frame(E(args[0]))
        return Frame([Vec(v.name, torch.isnan(v.as_float()).float(), INT) for v in fr.vecs], key=_new_key())
    if op in ("!", "not"):
        fr = _frame(E(args[0]))
        return Frame([Vec(v.name, (v.as_float() == 0).float(), INT) for v in fr.vecs], key=_new_key())
    if op in ("+", "-", "*", "/", "^", "%", "%%", "intDiv", "<", ">", "<=", ">=", "==", "!=", "&", "|", "&&", "||"):
        return _binop(op, E(args[0]), E(args[1]))
    if op == "h2o.runif":
        fr = _frame(E(args[0]))
        seed = int(args[1]) if len(args) > 1 and args[1] not in (-1, None) else 12345
        rank = ctx.cl.rank if ctx.cl is not None else 0
        g = torch.Generator().manual_seed(seed + 7919 * rank)
        u = torch.rand(fr.nrows, generator=g, dtype=torch.float64).float().to(fr.device)
        return Frame([Vec("rnd", u, REAL)], key=_new_key())
    if op == "cbind":
        frs = [_frame(E(a)) for a in args]
        vecs = []
        for f in frs:
            vecs += f.vecs
        return Frame(vecs, key=_new_key())
    if op == "rbind":
        from ..runtime.ops import _rbind

        return Frame(list(_rbind([_frame(E(a)) for a in args]).vecs), key=_new_key())
    if op == "colnames=":
        fr = _frame(E(args[0]))
        idx = _cols(fr, args[1])
        names = _idx_list(args[2], len(idx))
        vecs = list(fr.vecs)
        for i, nm in zip(idx, names):
            v = vecs[i]
            vecs[i] = Vec(str(nm), v.data, v.vtype, v.domain)
        return Frame(vecs, key=_new_key())
    if op == ":=":
        dst = _frame(E(args[0]))
        src = E(args[1])
        cols = _cols(dst, args[2]) if not (isinstance(args[2], tuple) and args[2][1] == []) else list(range(dst.ncols))
        vecs = list(dst.vecs)
        if isinstance(src, Frame):
            for j, ci in enumerate(cols):
                sv = src.vecs[min(j, src.ncols - 1)]
                if ci >= len(vecs):
                    vecs.append(Vec(sv.name, sv.data, sv.vtype, sv.domain))
                else:
                    vecs[ci] = Vec(vecs[ci].name, sv.data, sv.vtype, sv.domain)
        else:
            for ci in cols:
                n = dst.nrows
                vecs[ci] = Vec(vecs[ci].name, torch.full((n,), float(src), device=dst.device), REAL)
        return Frame(vecs, key=dst.key)
    if op in ("sum", "mean", "sd", "var", "min", "max"):
        fr = _frame(E(args[0]))
        na_rm = bool(args[1]) if len(args) > 1 else True
        return _reduce(ctx, fr, op, na_rm)
    if op == "nrow":
        return float(global_nrows(_frame(E(args[0])), ctx.comm))
    if op == "ncol":
        return float(_frame(E(args[0])).ncols)
    if op == "dim":
        fr = _frame(E(args[0]))
        return [float(global_nrows(fr, ctx.comm)), float(fr.ncols)]
    if op == "levels":
        fr = _frame(E(args[0]))
        return str(fr.vecs[0].domain)
    if op == "nlevels":
        return float(len(_frame(E(args[0])).vecs[0].domain or []))
    if op in ("abs", "log", "exp", "sqrt", "floor", "ceiling", "round", "sign", "cos", "sin", "tanh"):
        fr = _frame(E(args[0]))
        fn = {"abs": torch.abs, "log": torch.log, "exp": torch.exp, "sqrt": torch.sqrt, "floor": torch.floor,
              "ceiling": torch.ceil, "round": torch.round, "sign": torch.sign, "cos": torch.cos, "sin": torch.sin,
              "tanh": torch.tanh}[op]
        return Frame([Vec(v.name, fn(v.as_float()), REAL) for v in fr.vecs], key=_new_key())
    out = _munge(op, args, E, ctx)
    if out is not _NOT_MUNGE:
        return out
    raise ValueError(f"rapids: unsupported operation {op!r}")


_NOT_MUNGE = object()


def _bool(v, default=False):
    if v is None:
        return default
    if isinstance(v, str):
        return v.lower() in ("true", "1")
    if isinstance(v, tuple) and v and v[0] == "list":
        return [_bool(x) for x in v[1]]
    return bool(v)


def _num_list(v):
    return [float(x) for x in _idx_list(v, 0)] if v is not None else []


def _munge(op, args, E, ctx):
    """h2o-py frame methods (frame/munging.py)."""
    from ..frame import munging as M

    comm = ctx.comm
    if op == "ifelse":
        test = _frame(E(args[0]))
        return Frame(list(M.ifelse(test, E(args[1]), E(args[2])).vecs), key=_new_key())
    if op == "na.omit":
        return Frame(list(M.na_omit(_frame(E(args[0]))).vecs), key=_new_key())
    if op == "cut":
        fr = _frame(E(args[0]))
        labels = [str(x) for x in _idx_list(args[2], 0)] if len(args) > 2 and isinstance(args[2], tuple) and \
            args[2][1] else None
        return Frame(list(M.cut(fr, _num_list(args[1]), labels, _bool(args[3] if len(args) > 3 else False),
                                _bool(args[4] if len(args) > 4 else True),
                                int(args[5]) if len(args) > 5 else 3).vecs), key=_new_key())
    if op == "relevel":
        return Frame(list(M.relevel(_frame(E(args[0])), str(args[1])).vecs), key=_new_key())
    if op == "h2o.random_stratified_split":
        fr = _frame(E(args[0]))
        return Frame(list(M.stratified_split(fr, float(args[1]), int(args[2]) if len(args) > 2 else 42,
                                             comm).vecs), key=_new_key())
    if op == "scale":
        fr = _frame(E(args[0]))
        return Frame(list(M.scale(fr, _bool(args[1], True), _bool(args[2], True), comm).vecs), key=_new_key())
    if op in ("cumsum", "cumprod", "cummin", "cummax"):
        return Frame(list(M.cumulative(_frame(E(args[0])), op, comm).vecs), key=_new_key())
    if op in ("kfold_column", "modulo_kfold_column", "stratified_kfold_column"):
        fr = _frame(E(args[0]))
        how = "modulo" if op == "modulo_kfold_column" else "random"
        seed = int(args[2]) if len(args) > 2 else -1
        return Frame(list(M.kfold_column(fr, int(args[1]), seed, comm, how).vecs), key=_new_key())
    if op == "which":
        return Frame(list(M.which(_frame(E(args[0])), comm).vecs), key=_new_key())
    if op in ("any", "all", "naCnt", "any.na"):
        fr = _frame(E(args[0]))
        vals = []
        for v in fr.vecs:
            x = v.as_float()
            if op == "naCnt":
                vals.append(float(torch.isnan(x).sum()))
            elif op == "any.na":
                vals.append(float(torch.isnan(x).any()))
            elif op == "any":
                vals.append(float((torch.nan_to_num(x, nan=0.0) != 0).any()))
            else:
                vals.append(float(((x != 0) | torch.isnan(x)).all()) if x.numel() else 1.0)
        a = np.array(vals, np.float64)
        if comm is not None:
            a = comm.all_reduce_numpy(a, "sum" if op in ("naCnt", "any", "any.na") else "min")
        if op in ("any", "any.na"):
            return float(a.max() > 0)
        if op == "all":
            return float(a.min() > 0)
        return [float(x) for x in a] if len(a) > 1 else float(a[0])
    if op == "quantile":
        fr = _frame(E(args[0]))
        return Frame(list(M.quantile(fr, _num_list(args[1]), comm).vecs), key=_new_key())
    if op == "h2o.impute":
        fr = _frame(E(args[0]))
        col = int(args[1]) if len(args) > 1 else -1
        method = str(args[2]) if len(args) > 2 else "mean"
        values = _num_list(args[6]) if len(args) > 6 and isinstance(args[6], tuple) and args[6][1] else None
        cols = range(fr.ncols) if col < 0 else [col]
        fills = []
        for c in cols:
            if method.lower() == "mean" and fr.vecs[c].vtype == ENUM:
                method_c = "mode"
            else:
                method_c = method
            fr, f = M.impute(fr, c, method_c, comm, values)
            fills += f
        DKV.put(fr.key, fr)
        return fills if len(fills) > 1 else fills[0]
    if op == "GB":
        fr = _frame(E(args[0]))
        gcols = _cols(fr, args[1])
        rest = args[2:]
        aggs = []
        for i in range(0, len(rest) - 2, 3):
            ci = rest[i + 1]
            ci = fr.names.index(ci) if isinstance(ci, str) and ci in fr.names else int(ci)
            aggs.append((str(rest[i]), ci, str(rest[i + 2])))
        return Frame(list(M.group_by(fr, gcols, aggs, comm).vecs), key=_new_key())
    if op == "unique":
        fr = _frame(E(args[0]))
        return Frame(list(M.unique(fr, comm, _bool(args[1] if len(args) > 1 else False)).vecs), key=_new_key())
    if op == "table":
        frs = [E(a) for a in args if isinstance(E(a), Frame)]
        fr = frs[0] if len(frs) == 1 else Frame(frs[0].vecs + frs[1].vecs)
        return Frame(list(M.table(fr, comm).vecs), key=_new_key())
    if op == "sort":
        fr = _frame(E(args[0]))
        cols = _cols(fr, args[1])
        asc = _bool(args[2]) if len(args) > 2 else None
        asc = asc if isinstance(asc, list) else None
        return Frame(list(M.sort(fr, cols, asc, comm).vecs), key=_new_key())
    if op == "merge":
        left, right = _frame(E(args[0])), _frame(E(args[1]))
        bx = [int(x) for x in _idx_list(args[4], 0)] if len(args) > 4 and isinstance(args[4], tuple) and \
            args[4][1] else None
        by = [int(x) for x in _idx_list(args[5], 0)] if len(args) > 5 and isinstance(args[5], tuple) and \
            args[5][1] else None
        return Frame(list(M.merge(left, right, _bool(args[2]), _bool(args[3]), bx, by, comm).vecs),
                     key=_new_key())
    if op == "setDomain":
        fr = _frame(E(args[0]))
        levels = [str(x) for x in _idx_list(args[2], 0)]
        v = fr.vecs[0]
        if v.vtype != ENUM or len(levels) != len(v.domain or []):
            raise ValueError("setDomain: the new domain must have as many levels as the column")
        return Frame([Vec(v.name, v.data, ENUM, levels)] + list(fr.vecs[1:]), key=_new_key())
    return _NOT_MUNGE
