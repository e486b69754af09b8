"""MOJO export / import (H2O "Model ObJect, Optimized").

A MOJO is a zip with ``model.ini`` (``[info]`` key/values, ``[columns]``,
``[domains]``), ``domains/dNNN.txt`` level files and an algorithm payload,
following H2O-3's genmodel layout:

* tree models (gbm / drf / xgboost): one ``trees/tCC_TTT.bin`` per class CC
  and tree TTT in a compressed pre-order byte encoding.  Every inner node is
  ``nodeType:u8 | colId:u16 | naSplitDir:u8 | splitVal:f32`` followed by the
  left subtree (preceded by its byte size, 1-4 bytes by ``nodeType & 3``) or
  a leaf ``f32`` (``nodeType & 48``), then the right subtree or a leaf ``f32``
  (``nodeType & 192``); a tree that is a single leaf is ``0 | 0xFFFF | f32``.
  Rows go right when ``value >= splitVal``; NAs follow ``naSplitDir`` (2 =
  left, 3 = right).
* glm: coefficients and imputation data in ``model.ini`` (``beta``, ``cats``,
  ``cat_offsets``, ``nums``, ``num_means``, ``family``, ``link``), categorical
  predictors first, intercept last, on the original (de-standardized) scale.
* kmeans: ``center_<i>`` rows on the standardized scale plus
  ``standardize``/``center_mean``/``center_mult``.
* deeplearning: ``neural_network_sizes``, ``activation``, ``norm_sub``,
  ``norm_mul``, ``norm_resp_*`` and ``weight_layer<i>``/``bias_layer<i>``.
* pca, glrm, isotonicregression, coxph, targetencoder, word2vec,
  extendedisolationforest, gam: scalar settings in ``model.ini`` and every
  array (eigenvectors, archetypes, thresholds, coefficients, per-level
  target sums, word vectors, hyperplanes, spline knots / bases, design
  means / scales) as little-endian fp64 ``h2omx/<name>.bin`` with its shape
  in ``h2omx_shape_<name>`` (h2omx's own payload, exact round trip).  pca,
  isotonicregression, coxph and word2vec ALSO carry the entries the genmodel
  readers use (PCAMojoReader: ``k``/``eigenvector_size``/``catOffsets``/
  ``permutation``/``normSub``/``normMul`` + big-endian ``eigenvectors_raw``;
  IsotonicRegressionMojoReader: ``thresholds_x``/``thresholds_y``/
  ``min_x``/``max_x``; CoxPHMojoReader: ``coef``/``x_mean_num``/...;
  Word2VecMojoReader: text ``vocabulary`` + big-endian float ``vectors``), and
  isotonic / word2vec MOJOs that hold only those entries import.  glrm and
  targetencoder also write their genmodel entries (GlrmMojoReader:
  ``ncolA``/``ncolY``/``nrowY``/``cat_offsets``/``norm_sub``/``norm_mul`` +
  text ``losses`` + big-endian ``archetypes``; TargetEncoderMojoReader:
  ``with_blending``/``non_predictors`` + ``feature_engineering/
  target_encoding/encoding_map.ini`` and its NA-presence / column maps), and
  target-encoder MOJOs import from the encoding map alone; extended isolation
  forests write genmodel's per-tree ``trees/tNN.bin`` (node number, ``'N'``
  normal + intercept point or ``'L'`` row count) and import from those.

Binary compatibility with H2O's h2o-genmodel.jar cannot be checked here (no
JVM or jar in the environment): the layout follows the public format as
documented above and is pinned by round-trip tests (export -> import ->
identical predictions) in tests/test_mojo.py — "parity unpinned" against
genmodel itself.  Imported MOJOs become :class:`GenericModel` instances
(H2O's ``Generic`` algo) and score on the GPU through the same kernels.
"""
from __future__ import annotations

import io
import json
import struct
import time
import uuid
import zipfile

import numpy as np
import torch

from ..frame.frame import ENUM, Frame
from ..models.base import Model, ModelCategory

MOJO_VERSIONS = {"gbm": "1.40", "drf": "1.40", "xgboost": "1.00", "glm": "1.00", "kmeans": "1.00",
                 "deeplearning": "1.10", "stackedensemble": "1.01", "pca": "1.00", "glrm": "1.10",
                 "isotonicregression": "1.00", "coxph": "1.00", "targetencoder": "1.00", "word2vec": "1.00",
                 "extendedisolationforest": "1.00", "gam": "1.00", "upliftdrf": "1.40"}
# algorithms whose payload is the h2omx array layout below (design + named arrays)
ARRAY_ALGOS = ("pca", "glrm", "isotonicregression", "coxph", "targetencoder", "word2vec",
               "extendedisolationforest", "gam", "upliftdrf")
NSD_NA_LEFT, NSD_NA_RIGHT = 2, 3


# ---------------------------------------------------------------------------
# tree encoding
# ---------------------------------------------------------------------------
def _encode_tree(tree: np.ndarray, catbits: np.ndarray | None = None, nlev=None) -> bytes:
    """``catbits`` [nodes][8]: left sets of categorical group splits
    (TreeNode.na_left bit 1), written as genmodel bitset splits (nodeType
    equal = 12: ``bitOff:u16 | nBits:u32 | bytes``) holding the levels that go
    RIGHT over the column's domain ``nlev[feat]`` levels (out-of-range levels
    follow the NA direction, as unseen levels do in h2omx)."""
    def enc(i) -> tuple[bytes, bool]:
        nd = tree[i]
        if nd["feat"] < 0:
            return struct.pack("<f", float(nd["value"])), True
        lb, lleaf = enc(int(nd["left"]))
        rb, rleaf = enc(int(nd["left"]) + 1)
        is_cat = (int(nd["na_left"]) & 2) != 0 and catbits is not None
        split = np.nextafter(np.float32(nd["thr"]), np.float32(np.inf))
        node_type = 12 if is_cat else 0
        head_left = b""
        if lleaf:
            node_type |= 48
        else:
            n = len(lb)
            size_bytes = 1 if n < 256 else (2 if n < 65536 else (3 if n < (1 << 24) else 4))
            node_type |= size_bytes - 1
            head_left = n.to_bytes(size_bytes, "little")
        if rleaf:
            node_type |= 192
        nsd = NSD_NA_LEFT if (int(nd["na_left"]) & 1) else NSD_NA_RIGHT
        if is_cat:
            from ..models.tree.structs import bitset_has

            nb = int(nlev[int(nd["feat"])]) if nlev is not None else 256
            nb = max(1, min(nb, 256))
            right = ~bitset_has(catbits[i], np.arange(nb))
            by = np.packbits(right.astype(np.uint8), bitorder="little").tobytes()
            hdr = struct.pack("<BHBHI", node_type, int(nd["feat"]), nsd, 0, nb) + by
        else:
            hdr = struct.pack("<BHBf", node_type, int(nd["feat"]), nsd, float(split))
        return hdr + head_left + lb + rb, False

    body, leaf = enc(0)
    if leaf:
        return struct.pack("<BH", 0, 0xFFFF) + body
    return body


class _TreeCodec:
    """Pre-order tree (de)serialisation with an explicit stack."""

    @staticmethod
    def decode(data: bytes) -> np.ndarray:
        from ..models.tree.structs import TREE_NODE_DTYPE

        feat, left, na_left, thr, value = [], [], [], [], []
        cats = {}       # node -> left-set words of a bitset split

        def new():
            feat.append(-1)
            left.append(-1)
            na_left.append(0)
            thr.append(0.0)
            value.append(0.0)
            return len(feat) - 1

        root = new()
        if struct.unpack_from("<H", data, 1)[0] == 0xFFFF:
            value[root] = struct.unpack_from("<f", data, 3)[0]
        else:
            pos = 0
            # stack entries: node index awaiting decode of an inner node at `pos`,
            # or ("leaf", idx) meaning the next 4 bytes are that leaf's value
            stack = [root]
            while stack:
                top = stack.pop()
                if isinstance(top, tuple):
                    value[top[1]] = struct.unpack_from("<f", data, pos)[0]
                    pos += 4
                    continue
                idx = top
                node_type, col, nsd = struct.unpack_from("<BHB", data, pos)
                lp, rp = new(), new()
                feat[idx], left[idx] = col, lp
                na_left[idx] = 1 if nsd == NSD_NA_LEFT else 0
                equal = node_type & 12
                if equal == 0:
                    split = struct.unpack_from("<f", data, pos + 4)[0]
                    pos += 8
                    thr[idx] = float(np.nextafter(np.float32(split), np.float32(-np.inf)))
                else:
                    # bitset split: the set holds the levels going right; levels
                    # outside [bitoff, bitoff + nbits) follow the NA direction
                    if equal == 8:
                        bitoff, nbits, pos = 0, 32, pos + 4
                    else:
                        bitoff, nbits = struct.unpack_from("<HI", data, pos + 4)
                        pos += 10
                    nby = (nbits + 7) // 8
                    rbits = np.unpackbits(np.frombuffer(data, np.uint8, nby, pos), bitorder="little")[:nbits]
                    pos += nby
                    lv = np.arange(256)
                    inr = (lv >= bitoff) & (lv < bitoff + nbits)
                    rel = np.clip(lv - bitoff, 0, max(nbits - 1, 0))
                    goes_right = np.where(inr, rbits[rel] != 0 if nbits else False, na_left[idx] == 0)
                    from ..models.tree.structs import bitset_words

                    cats[idx] = bitset_words(np.nonzero(~goes_right)[0])
                    na_left[idx] |= 2
                    thr[idx] = float("nan")
                # push right first so the left subtree is decoded next
                stack.append(("leaf", rp) if node_type & 192 else rp)
                if node_type & 48:
                    stack.append(("leaf", lp))
                else:
                    pos += (node_type & 3) + 1
                    stack.append(lp)
        arr = np.zeros(len(feat), TREE_NODE_DTYPE)
        arr["feat"], arr["left"], arr["na_left"] = feat, left, na_left
        arr["thr"], arr["value"] = thr, value
        if cats:
            cb = np.zeros((len(feat), 8), np.uint32)
            for i, w in cats.items():
                cb[i] = w
            return arr, cb
        return arr, None


def encode_tree(tree: np.ndarray, catbits: np.ndarray | None = None, nlev=None) -> bytes:
    return _encode_tree(tree, catbits, nlev)


def decode_tree(data: bytes) -> np.ndarray:
    return _TreeCodec.decode(data)[0]


def decode_tree_cat(data: bytes):
    """(tree records, categorical bitsets [nodes][8] or None)."""
    return _TreeCodec.decode(data)


# ---------------------------------------------------------------------------
# writer
# ---------------------------------------------------------------------------
def _fmt(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (list, tuple, np.ndarray)):
        return "[" + ", ".join(_fmt(x) for x in v) + "]"
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    return str(v)


def _category_name(cat):
    return {ModelCategory.BINOMIAL: "Binomial", ModelCategory.MULTINOMIAL: "Multinomial",
            ModelCategory.REGRESSION: "Regression", ModelCategory.CLUSTERING: "Clustering",
            ModelCategory.DIMREDUCTION: "DimReduction", ModelCategory.ANOMALY: "AnomalyDetection"}.get(cat, str(cat))


def _design_columns(design):
    """DataInfo order: categorical columns first, then numerics."""
    cats = [c for c in design.x if design.types[c] == ENUM]
    nums = [c for c in design.x if design.types[c] != ENUM]
    return cats, nums


def mojo_bytes(model: Model) -> bytes:
    if model.preprocessors:
        raise ValueError(f"{model.model_id}: a model trained behind a preprocessing pipeline (AutoML target "
                         "encoding) has no single-model MOJO; export the TargetEncoder and the model separately")
    algo = model.algo
    info: dict = {}
    files: dict[str, bytes] = {}
    if algo in ("gbm", "drf", "xgboost"):
        columns = list(model.x)
        info.update(_tree_info(model, files))
        cal = getattr(model, "calibration", None)
        if cal is not None and cal["method"] == "PlattScaling":
            # genmodel calibrateClassProbabilities: p1' = logitInv(p1 * beta[0] + beta[1])
            info.update(calib_method="platt", calib_glm_beta=[cal["slope"], cal["intercept"]])
        elif cal is not None and cal["method"] == "IsotonicRegression":
            # step function of the pooled-adjacent-violators fit: p1 clipped to
            # [x_min, x_max], value of the first threshold >= p1 (h2omx entries;
            # genmodel parity of the isotonic calibration block is unpinned)
            info.update(calib_method="isotonic", calib_isotonic_x_min=cal["x_min"])
            _put(files, info, "calib_isotonic_x", np.asarray(cal["x"], np.float64))
            _put(files, info, "calib_isotonic_y", np.asarray(cal["y"], np.float64))
    elif algo == "glm" and (getattr(model, "interaction_spec", None) or model.family == "ordinal"):
        columns, ext = _glm_ext_info(model, files)       # h2omx array payload
        info.update(ext)
    elif algo == "glm":
        cats, nums = _design_columns(model.design)
        columns = cats + nums
        info.update(_glm_info(model, cats, nums))
    elif algo == "kmeans":
        cats, nums = _design_columns(model.design)
        columns = cats + nums
        info.update(_kmeans_info(model, cats, nums))
    elif algo == "deeplearning":
        cats, nums = _design_columns(model.design)
        columns = cats + nums
        info.update(_dl_info(model, cats, nums))
    elif algo == "stackedensemble":
        columns = list(model.x)
        info.update(_se_info(model, files))
    elif algo == "isolationforest":
        columns = list(model.x)
        info.update(_if_info(model, files))
    elif algo in ARRAY_ALGOS:
        columns = list(model.x)
        if algo == "gam":
            # genmodel GAM column order: categorical, numeric, then the gam columns
            cats, nums = _gam_design_columns(model)
            columns = cats + nums + [c for c in model.gam_spec if c not in cats + nums]
        info.update(_array_info(model, files))
    elif algo == "generic":
        return model.raw_mojo
    else:
        raise NotImplementedError(f"MOJO export for {algo}")
    enc = getattr(model, "cat_encoder", None)
    enc_domains = {}
    if enc is not None:
        # frame-transform categorical_encoding: the MOJO takes the ORIGINAL
        # predictors (genmodel applies the scheme named in model.ini); the fitted
        # encoding itself travels as h2omx payload (exact round trip)
        info["categorical_encoding"] = {"onehotexplicit": "OneHotExplicit", "binary": "Binary", "eigen": "Eigen",
                                        "labelencoder": "LabelEncoder", "enumlimited": "EnumLimited",
                                        "sortbyresponse": "SortByResponse"}[enc.scheme]
        files["h2omx/categorical_encoder.json"] = json.dumps(enc.to_json()).encode()
        columns = list(enc.x_in)
        enc_domains = {c: enc.domains.get(c) for c in enc.x_in}
    if model.y is not None and algo not in ("kmeans", "coxph") and not getattr(model, "autoencoder", False):
        columns = columns + [model.y]
    domains = []
    for j, c in enumerate(columns):
        dom = model.response_domain if c == model.y else (enc_domains.get(c) or model.feature_domains.get(c) or (
            model.gam_frame_domains.get(c) if hasattr(model, "gam_frame_domains") else None))
        if dom:
            domains.append((j, dom))
    nclass = len(model.response_domain) if model.response_domain else 1
    cd = getattr(model, "class_dist", None)     # balance_classes: (prior, modelled) class fractions
    head = {
        "h2o_version": "3.46.0.6", "mojo_version": MOJO_VERSIONS.get(algo, "1.00"),
        "license": "Apache License Version 2.0", "algo": algo, "algorithm": getattr(model, "algo_full_name", algo),
        "endianness": "LITTLE_ENDIAN", "category": _category_name(model.category),
        "uuid": str(uuid.uuid4().int & ((1 << 63) - 1)),
        "supervised": model.y is not None, "n_features": len(model.x), "n_classes": nclass,
        "n_columns": len(columns), "n_domains": len(domains), "balance_classes": cd is not None,
        "default_threshold": float((model.training_metrics or {}).get("max_f1_threshold", 0.5) or 0.5),
        "prior_class_distrib": "null" if cd is None else [float(v) for v in cd[0]],
        "model_class_distrib": "null" if cd is None else [float(v) for v in cd[1]],
        "timestamp": time.strftime("%Y-%m-%dT%H:%M:%S"),
        "h2omx_model_id": model.model_id, "response_column": model.y or "",
    }
    if algo == "coxph":
        head["supervised"] = False
        head["category"] = "CoxPH"
    if algo == "upliftdrf":
        head["category"] = "BinomialUplift"
    lines =["[info]"] + [f"{k} = {_fmt(v)}" for k, v in {**head, **info}.items()]
    lines += ["", "[columns]"] + columns + ["", "[domains]"]
    for i, (j, dom) in enumerate(domains):
        lines.append(f"{j}: {len(dom)} d{i:03d}.txt")
        files[f"domains/d{i:03d}.txt"] = ("\n".join(str(d) for d in dom) + "\n").encode()
    files["model.ini"] = ("\n".join(lines) + "\n").encode()
    files["experimental/modelDetails.json"] = json.dumps(_details(model), default=str).encode()
    buf = io.BytesIO()
    with zipfile.ZipFile(buf, "w", zipfile.ZIP_DEFLATED) as z:
        for name in sorted(files):
            z.writestr(name, files[name])
    return buf.getvalue()


def _details(model):
    try:
        from ..api.schemas import model_json

        return model_json(model)
    except Exception:  # noqa: BLE001
        return {"model_id": model.model_id, "algo": model.algo}


def _tree_info(model, files):
    ens = model.ens
    K = ens.K
    nt = ens.ntrees
    nlev = [len(model.feature_domains.get(c) or []) for c in model.x] if ens.catbits is not None else None
    for t in range(nt):
        for k in range(K):
            i = t * K + k
            files[f"trees/t{k:02d}_{t:03d}.bin"] = _encode_tree(
                ens.trees[i], None if ens.catbits is None else ens.catbits[i], nlev)
    dist = {"drf": "AUTO"}.get(model.dist, model.dist)
    return {"n_trees": nt, "n_trees_per_class": K, "init_f": float(ens.init_f[0]) if K == 1 else 0.0,
            "init_f_per_class": [float(x) for x in ens.init_f], "distribution": dist,
            "h2omx_engine_dist": model.dist, "h2omx_average": bool(ens.average),
            "offset_column": model.params.get("offset_column") or "null", "binomial_double_trees": False,
            "link_function": _tree_link(model)}


def _if_info(model, files):
    ens = model.ens
    for t in range(ens.ntrees):
        files[f"trees/t00_{t:03d}.bin"] = _encode_tree(ens.trees[t])
    return {"n_trees": ens.ntrees, "n_trees_per_class": 1, "init_f": 0.0, "init_f_per_class": [0.0],
            "h2omx_engine_dist": "isolation", "h2omx_average": True, "sample_size": int(model.sample_size),
            "min_path_length": float(model.min_path_length), "max_path_length": float(model.max_path_length),
            "output_anomaly_flag": model.threshold is not None,
            "h2omx_threshold": float(model.threshold) if model.threshold is not None else "null"}


def _tree_link(model):
    if model.dist == "drf":
        return "identity"
    if model.category == ModelCategory.BINOMIAL:
        return "logit"
    if model.category == ModelCategory.MULTINOMIAL:
        return "multinomial"
    return "log" if model.dist in ("poisson", "gamma", "tweedie") else "identity"


def _reorder(vec_names, design, cats, nums):
    order = []
    for c in cats + nums:
        order += [i for i, (cc, _) in enumerate(design.spec) if cc == c]
    return order


def _glm_info(model, cats, nums):
    d = model.design
    order = _reorder(d.names, d, cats, nums)
    betas = []
    for k in range(model.beta.shape[0]):
        betas += [float(model.beta[k, i]) for i in order] + [float(model.beta[k, -1])]
    offs = [0]
    for c in cats:
        offs.append(offs[-1] + sum(1 for cc, _ in d.spec if cc == c))
    num_means = [float(d.means[[i for i, (cc, _) in enumerate(d.spec) if cc == c][0]]) for c in nums]
    return {"use_all_factor_levels": bool(d.use_all_levels), "cats": len(cats), "cat_offsets": offs,
            "nums": len(nums), "mean_imputation": True, "num_means": num_means,
            "cat_modes": [0] * len(cats), "h2omx_means": [float(d.means[i]) for i in order], "beta": betas, "family": model.family, "link": model.link,
            "tweedie_link_power": float(model.params.get("tweedie_link_power", 0.0) or 0.0)}


def _glm_ext_info(model, files):
    """GLM with interaction columns and / or the ordinal family: the raw
    source columns, the interaction spec, the design over the augmented
    columns and the standardised coefficients (h2omx array payload)."""
    from ..models.glm_extras import interaction_columns

    spec = getattr(model, "interaction_spec", None) or []
    gen = set(interaction_columns(spec))
    base = [c for c in model.x if c not in gen]
    for _, a, b, _ in spec:
        for c in (a, b):
            if c not in base:
                base.append(c)
    info = {"h2omx_glm_ext": True, "family": model.family, "link": model.link,
            "tweedie_link_power": float(model.params.get("tweedie_link_power", 0.0) or 0.0)}
    # structured settings travel as a JSON entry (model.ini values are flat)
    files["h2omx/glm_ext.json"] = json.dumps({
        "interactions": [list(t) for t in spec],
        "aug_types": {c: [model.feature_types.get(c), model.feature_domains.get(c)] for c in model.x if c in gen},
        "ordinal_thresholds": list(model.stats.get("ordinal_thresholds") or []),
    }).encode()
    _design_info(model.design, info, files)
    _put(files, info, "beta", model.beta_std)
    return base, info


def _kmeans_info(model, cats, nums):
    d = model.design
    order = _reorder(d.names, d, cats, nums)
    out = {"standardize": bool(model.params.get("standardize", True)), "center_num": int(model.centers_std.shape[0]),
           "center_mean": [float(d.center[i]) for i in order], "center_mult": [float(1.0 / d.sds[i]) for i in order],
           "means": [float(d.means[i]) for i in order], "cats": len(cats), "nums": len(nums),
           "use_all_factor_levels": True}
    for i in range(model.centers_std.shape[0]):
        out[f"center_{i}"] = [float(model.centers_std[i, j]) for j in order]
    return out


def _dl_info(model, cats, nums):
    d = model.design
    order = _reorder(d.names, d, cats, nums)
    net = model.net
    out = {"neural_network_sizes": list(net.sizes), "activation": model.params["activation"],
           "norm_sub": [float(d.center[i]) for i in order], "norm_mul": [float(1.0 / d.sds[i]) for i in order],
           "means": [float(d.means[i]) for i in order], "norm_resp_sub": float(model.y_mean),
           "norm_resp_mul": float(1.0 / model.y_sd), "cats": len(cats), "nums": len(nums),
           "use_all_factor_levels": bool(d.use_all_levels), "autoencoder": bool(model.autoencoder),
           "h2omx_act": int(model.act)}
    for i in range(len(net.layers)):
        W = net.W(i).detach().cpu().numpy()
        if i == 0:
            W = W[:, order]
        out[f"weight_layer{i}"] = W.reshape(-1).tolist()
        out[f"weight_shape{i}"] = list(W.shape)
        out[f"bias_layer{i}"] = net.b(i).detach().cpu().numpy().tolist()
    return out


def _se_info(model, files):
    out = {"base_models_num": len(model.base_models), "metalearner": model.metalearner.model_id}
    for i, bm in enumerate(model.base_models):
        files[f"models/{bm.model_id}.zip"] = mojo_bytes(bm)
        out[f"base_model{i}"] = bm.model_id
    files[f"models/{model.metalearner.model_id}.zip"] = mojo_bytes(model.metalearner)
    return out


# ---------------------------------------------------------------------------
# array payload (PCA, GLRM, isotonic, CoxPH, TargetEncoder, Word2Vec, EIF, GAM)
# ---------------------------------------------------------------------------
def _put(files, info, name, arr):
    a = np.ascontiguousarray(np.asarray(arr, dtype="<f8"))
    files[f"h2omx/{name}.bin"] = a.tobytes()
    info[f"h2omx_shape_{name}"] = list(a.shape) if a.ndim else [1]


def _get(z, info, name):
    shape = info[f"h2omx_shape_{name}"]
    shape = shape if isinstance(shape, list) else [shape]
    return np.frombuffer(z.read(f"h2omx/{name}.bin"), dtype="<f8").reshape(shape).copy()


def _design_info(design, info, files, tag="design"):
    info[f"h2omx_{tag}_use_all"] = bool(design.use_all_levels)
    info[f"h2omx_{tag}_x"] = list(design.x)
    _put(files, info, f"{tag}_means", design.means)
    _put(files, info, f"{tag}_sds", design.sds if design.sds is not None else np.ones(len(design.names)))
    _put(files, info, f"{tag}_center", getattr(design, "center", np.zeros(len(design.names))))


def _uplift_genmodel_trees(model, files) -> int:
    """genmodel SharedTree layout of the uplift forest: every tree twice, the
    same splits with the treatment leaf predictions (trees/t00_*) and the
    control ones (trees/t01_*), i.e. two tree classes per group as
    UpliftDrfMojoModel reads them (uplift = mean t00 - mean t01).  Bin splits
    become value thresholds: code <= bin  <=>  x <= edges[f][bin]."""
    from ..models.tree.structs import TREE_NODE_DTYPE

    edges = np.asarray(model.edges, np.float32)
    nvb = np.asarray(model.nvb, np.int64)
    for t, tr in enumerate(model.trees):
        m = len(tr["feat"])
        for k, key in enumerate(("pt", "pc")):
            a = np.zeros(m, TREE_NODE_DTYPE)
            a["feat"], a["left"], a["na_left"] = tr["feat"], tr["left"], tr["na_left"]
            a["bin"] = tr["bin"]
            f = np.maximum(np.asarray(tr["feat"], np.int64), 0)
            b = np.asarray(tr["bin"], np.int64)
            inner = b < nvb[f] - 1
            a["thr"] = np.where(inner, edges[f, np.minimum(b, edges.shape[1] - 1)], np.float32(np.inf))
            a["value"] = np.asarray(tr[key], np.float32)
            files[f"trees/t{k:02d}_{t:03d}.bin"] = _encode_tree(a)
    return len(model.trees)


def _uplift_info(model, info, files):
    nt = _uplift_genmodel_trees(model, files)
    info.update(n_trees=nt, n_trees_per_class=2, n_tree_groups=nt, init_f=0.0, distribution="bernoulli",
                binomial_double_trees=False, default_threshold=0.5)
    for k in ("feat", "bin", "na_left", "left", "pt", "pc"):
        _put(files, info, f"uplift_{k}", np.concatenate([np.asarray(t[k], np.float64) for t in model.trees]))
    _put(files, info, "uplift_tree_sizes", [len(t["feat"]) for t in model.trees])
    _put(files, info, "uplift_edges", np.asarray(model.edges, np.float64))
    _put(files, info, "uplift_nvb", np.asarray(model.nvb, np.float64))
    info.update(nbt=int(model.nbt), treatment_column=model.treatment_column, ntrees=len(model.trees),
                uplift_metric=str(model.params.get("uplift_metric", "AUTO")),
                auuc_type=str(model.params.get("auuc_type", "AUTO")))


def _pca_genmodel(model, info, files):
    """genmodel PCAMojoReader entries next to the h2omx arrays: DataInfo
    counts / offsets, numeric normalisation (normSub subtracted, normMul
    multiplied) and ``eigenvectors_raw`` ([eigenvector_size][k] big-endian
    fp64, java.nio.ByteBuffer order)."""
    d = model.design
    cats, nums = _design_columns(d)
    offs, o = [0], 0
    for c in cats:
        o += len(d.domains[c]) - (0 if d.use_all_levels else 1)
        offs.append(o)
    ev = np.asarray(model.eigenvectors, np.float64)
    ncat_cols = offs[-1]
    cen = np.asarray(model.center, np.float64)
    sc = np.asarray(model.scale, np.float64)
    info.update(use_all_factor_levels=bool(d.use_all_levels), pcaMethod="GramSVD", pca_impl="MTJ_EVD_SYMMMATRIX",
                eigenvector_size=int(ev.shape[0]), ncats=len(cats), nnums=len(nums), catOffsets=offs,
                permutation=[model.x.index(c) for c in cats + nums],
                normSub=cen[ncat_cols:].tolist(), normMul=(1.0 / np.where(sc[ncat_cols:] == 0, 1.0, sc[ncat_cols:])).tolist())
    files["eigenvectors_raw"] = np.ascontiguousarray(ev, dtype=">f8").tobytes()


def _glrm_genmodel(model, info, files):
    """genmodel GlrmMojoReader entries: A / Y / X dimensions, regulariser and
    initialisation, DataInfo layout (categoricals first: ``num_categories``,
    ``cat_offsets``, ``cols_permutation``), the numeric normalisation
    (``norm_sub`` subtracted, ``norm_mul`` multiplied), one loss per original
    column in the text entry ``losses`` and the archetypes as ``archetypes``
    ([nrowY][ncolY] big-endian fp64, java.nio.ByteBuffer order)."""
    d, p = model.design, model.params
    cats, nums = _design_columns(d)
    offs, o = [0], 0
    for c in cats:
        o += len(d.domains[c]) - (0 if d.use_all_levels else 1)
        offs.append(o)
    Y = np.asarray(model.Y, np.float64)
    ncat_cols = offs[-1]
    cen = np.asarray(model.center, np.float64)
    sc = np.asarray(model.scale, np.float64)
    info.update(ncolA=len(d.x), ncolY=int(Y.shape[1]), nrowY=int(Y.shape[0]), regularizationX=str(p["regularization_x"]),
                gammaX=float(p["gamma_x"]), initialization=str(p["init"]), num_categories=len(cats),
                num_numeric=len(nums), cat_offsets=offs, cols_permutation=[d.x.index(c) for c in cats + nums],
                norm_sub=cen[ncat_cols:].tolist(),
                norm_mul=(1.0 / np.where(sc[ncat_cols:] == 0, 1.0, sc[ncat_cols:])).tolist(),
                transposed=False, reverse_transform=True, seed=int(p.get("seed") or -1),
                max_iterations=int(p["max_iterations"]))
    files["losses"] = ("\n".join([str(p["multi_loss"])] * len(cats) + [str(p["loss"])] * len(nums)) + "\n").encode()
    files["archetypes"] = np.ascontiguousarray(Y, dtype=">f8").tobytes()


EIF_NODE, EIF_LEAF = ord("N"), ord("L")


def eif_encode_tree(normals: np.ndarray, offs: np.ndarray, sizes: np.ndarray) -> bytes:
    """One extended-isolation tree in genmodel's CompressedIsolationTree byte
    layout (little-endian): ``int32 p`` (branching-array length), then every
    reachable heap node in index order as ``int32 nodeNumber | u8 type`` and
    for ``'N'`` the normal ``n`` and an intercept point ``p`` (p doubles each;
    a row goes left when ``(x - p) . n <= 0``), for ``'L'`` ``int32 numRows``.
    h2omx stores the offset ``b`` (left when ``x . n <= b``); the point
    ``p = b n / |n|^2`` lies on that hyperplane, so both rules agree."""
    p = normals.shape[1]
    out = [struct.pack("<i", p)]
    stack, nodes = [0], []
    while stack:
        i = stack.pop()
        nodes.append(i)
        if sizes[i] < 0:
            stack += [2 * i + 1, 2 * i + 2]
    for i in sorted(nodes):
        if sizes[i] >= 0:
            out.append(struct.pack("<iBi", i, EIF_LEAF, int(sizes[i])))
        else:
            n = normals[i].astype(np.float64)
            pt = n * (float(offs[i]) / max(float(n @ n), 1e-300))
            out.append(struct.pack("<iB", i, EIF_NODE) + n.astype("<f8").tobytes() + pt.astype("<f8").tobytes())
    return b"".join(out)


def eif_decode_tree(data: bytes, cap: int):
    """Inverse of :func:`eif_encode_tree` into heap arrays (normals [cap][p],
    offsets [cap] with ``b = p . n``, leaf sizes [cap], -1 inner)."""
    (p,) = struct.unpack_from("<i", data, 0)
    normals, offs, sizes = np.zeros((cap, p), np.float32), np.zeros(cap, np.float32), np.full(cap, -1.0, np.float32)
    o = 4
    while o < len(data):
        i, typ = struct.unpack_from("<iB", data, o)
        o += 5
        if typ == EIF_LEAF:
            sizes[i] = struct.unpack_from("<i", data, o)[0]
            o += 4
        else:
            n = np.frombuffer(data, "<f8", p, o)
            pt = np.frombuffer(data, "<f8", p, o + 8 * p)
            normals[i], offs[i] = n, float(pt @ n)
            o += 16 * p
    return normals, offs, sizes


TE_DIR = "feature_engineering/target_encoding/"


def _te_genmodel(model, info, files):
    """genmodel TargetEncoderMojoReader entries: ``with_blending`` /
    ``non_predictors`` key/values, the per-column encoding map
    (``[col]`` sections of ``level = numerator denominator [targetClass]``,
    the NA level last), the NA-presence map and the input -> output column
    mappings.  Multinomial rows carry the class index (1..K-1) as H2O's."""
    p = model.params
    info.update(with_blending=bool(p["blending"]),
                non_predictors=";".join(c for c in (model.y, p.get("fold_column"), p.get("weights_column")) if c))
    enc, na = [], []
    for c in model.columns:
        sums, cnts, _ = model.stats[c]
        s, n = sums.double().numpy(), cnts.double().numpy()
        enc.append(f"[{c}]")
        for lv in range(n.size):
            if n[lv] == 0 and lv == n.size - 1:
                continue        # no NA level seen in training
            if model.classes is None:
                enc.append(f"{lv} = {_fmt(float(s[lv, 0]))} {_fmt(float(n[lv]))}")
            else:
                enc.extend(f"{lv} = {_fmt(float(s[lv, k]))} {_fmt(float(n[lv]))} {k + 1}" for k in range(s.shape[1]))
        na.append(f"{c} = {1 if n[-1] > 0 else 0}")
    files[TE_DIR + "encoding_map.ini"] = ("\n".join(enc) + "\n").encode()
    files[TE_DIR + "te_column_name_to_missing_values_presence.ini"] = ("\n".join(na) + "\n").encode()
    frm = "\n".join(f"[from]\n{c}\n[to]\n{c}" for c in model.columns)
    files[TE_DIR + "input_encoding_columns_map.ini"] = (frm + "\n").encode()
    outs = "\n".join(f"[from]\n{c}\n[to]\n" + "\n".join(n for n in _te_out_names(c, model.classes))
                     for c in model.columns)
    files[TE_DIR + "input_output_columns_map.ini"] = (outs + "\n").encode()


def _te_out_names(col, classes):
    return [f"{col}_te"] if classes is None else [f"{col}_{k}_te" for k in classes]


def _te_from_genmodel(z, info, levels: dict):
    """Per-column (sums [L+1][C], counts [L+1]) and the prior from the genmodel
    encoding map alone (H2O's prior: total numerator / total denominator)."""
    text = z.read(TE_DIR + "encoding_map.ini").decode()
    cols, cur = {}, None
    for line in text.splitlines():
        line = line.strip()
        if not line:
            continue
        if line.startswith("[") and line.endswith("]"):
            cur = line[1:-1]
            cols[cur] = []
            continue
        k, v = line.split("=", 1)
        parts = v.split()
        cols[cur].append((int(k), float(parts[0]), float(parts[1]), int(parts[2]) if len(parts) > 2 else 1))
    C = max((t[3] for rows in cols.values() for t in rows), default=1)
    out, tot_s, tot_n = {}, np.zeros(C), 0.0
    for c, rows in cols.items():
        L = len(levels.get(c) or []) or (max(t[0] for t in rows) if rows else 0)
        s, n = np.zeros((L + 1, C)), np.zeros(L + 1)
        for lv, num, den, tc in rows:
            s[min(lv, L), tc - 1] = num
            n[min(lv, L)] = den
        out[c] = (s, n)
        if not tot_n:
            tot_s, tot_n = s.sum(0), n.sum()
    prior = tot_s / tot_n if tot_n else np.zeros(C)
    return out, prior


def _array_info(model, files):
    info: dict = {}
    a = model.algo
    if a in ("pca", "glrm", "coxph", "extendedisolationforest"):
        _design_info(model.design, info, files)
    if a == "pca":
        _put(files, info, "center", model.center)
        _put(files, info, "scale", model.scale)
        _put(files, info, "eigenvectors", model.eigenvectors)
        info["k"] = int(model.eigenvectors.shape[1])
        _pca_genmodel(model, info, files)
    elif a == "glrm":
        _put(files, info, "center", model.center)
        _put(files, info, "scale", model.scale)
        _put(files, info, "archetypes", model.Y)
        info.update(ncolX=int(model.Y.shape[0]), regularization_x=str(model.params["regularization_x"]),
                    gamma_x=float(model.params["gamma_x"]), h2omx_recon_names=list(model.design.names))
        _glrm_genmodel(model, info, files)
    elif a == "isotonicregression":
        _put(files, info, "thresholds_x", model.thresholds_x)
        _put(files, info, "thresholds_y", model.thresholds_y)
        info["out_of_bounds"] = str(model.params["out_of_bounds"])
        # genmodel IsotonicRegressionMojoReader entries
        tx = np.asarray(model.thresholds_x, np.float64)
        info.update(thresholds_x=tx.tolist(), thresholds_y=np.asarray(model.thresholds_y, np.float64).tolist(),
                    min_x=float(tx.min()) if tx.size else 0.0, max_x=float(tx.max()) if tx.size else 0.0)
    elif a == "upliftdrf":
        _uplift_info(model, info, files)
    elif a == "coxph":
        _put(files, info, "coef", model.beta)
        _put(files, info, "x_mean_num", model.x_mean)
        # genmodel CoxPHMojoReader key/values (numeric predictors)
        info.update(coef=np.asarray(model.beta, np.float64).ravel().tolist(),
                    x_mean_num=np.asarray(model.x_mean, np.float64).ravel().tolist(),
                    x_mean_cat=[], cat_offsets=[0], cats=0, nums=int(np.asarray(model.x_mean).size),
                    use_all_factor_levels=bool(model.design.use_all_levels))
    elif a == "targetencoder":
        info["te_columns"] = list(model.columns)
        info["blending"] = bool(model.params["blending"])
        info["inflection_point"] = float(model.params["inflection_point"])
        info["smoothing"] = float(model.params["smoothing"])
        info["keep_original_categorical_columns"] = bool(model.params["keep_original_categorical_columns"])
        info["h2omx_classes"] = list(model.classes) if model.classes is not None else "null"
        _put(files, info, "prior", model.prior.numpy())
        for i, c in enumerate(model.columns):
            sums, cnts, _ = model.stats[c]
            _put(files, info, f"te_sums_{i}", sums.numpy())
            _put(files, info, f"te_counts_{i}", cnts.numpy())
        _te_genmodel(model, info, files)
    elif a == "word2vec":
        files["h2omx/vocabulary.txt"] = ("\n".join(model.words) + "\n").encode()
        vec = model.vectors.float().cpu().numpy()
        _put(files, info, "vectors", vec)
        info["vec_size"] = int(model.vectors.shape[1])
        info["vocab_size"] = len(model.words)
        # genmodel Word2VecMojoReader entries: text "vocabulary", blob "vectors"
        # (java.nio.ByteBuffer order: big-endian float32, word-major)
        files["vocabulary"] = ("\n".join(model.words) + "\n").encode()
        files["vectors"] = np.ascontiguousarray(vec, dtype=">f4").tobytes()
    elif a == "extendedisolationforest":
        _put(files, info, "normals", model.normals)
        _put(files, info, "offsets", model.offs)
        _put(files, info, "leaf_sizes", model.sizes)
        info.update(limit=int(model.limit), sample_size=int(model.sample_size), ntrees=int(model.normals.shape[0]),
                    extension_level=int(model.params["extension_level"]))
        for t in range(model.normals.shape[0]):
            files[f"trees/t{t:02d}.bin"] = eif_encode_tree(model.normals[t], model.offs[t], model.sizes[t])
    elif a == "gam":
        _design_info(model.design, info, files)
        _put(files, info, "beta", model.beta_std)      # standardised scale (design.transform)
        info.update(family=model.family, link=model.link, gam_columns=list(model.gam_spec),
                    h2omx_glm_x=list(model.x),
                    tweedie_link_power=float(model.params.get("tweedie_link_power", 0.0) or 0.0))
        for i, (c, sp) in enumerate(model.gam_spec.items()):
            _put(files, info, f"gam_knots_{i}", sp["knots"])
            _put(files, info, f"gam_F_{i}", sp["F"])
            _put(files, info, f"gam_Z_{i}", sp["Z"])
            info[f"gam_mean_{i}"] = float(sp["mean"])
        _gam_genmodel(model, info, files)
    return info


def _gam_design_columns(model):
    """(categorical, numeric) non-gam predictors of a GAM, DataInfo order."""
    basis = {f"{c}_cr_{i}" for c, sp in model.gam_spec.items() for i in range(sp["Z"].shape[1])}
    cats, nums = _design_columns(model.design)
    return [c for c in cats if c not in basis], [c for c in nums if c not in basis]


def _gam_genmodel(model, info, files):
    """GamMojoReader-style entries: the GLM part (cats / cat_offsets / nums, NA
    fills, coefficients over [one-hot cats, nums, centred gam basis columns,
    intercept] on the original scale: ``beta_center``; the same with every gam
    column's basis un-centred through Z: ``beta``), the spline settings
    (``gam_columns``, ``num_knots``, ``bs``, the gam columns' NA fills) and
    big-endian float64 blobs ``knots`` (per column, concatenated), ``binvD``
    (B^-1 D, (k-2) x k) and ``zTranspose`` (Z^T, (k-1) x k).  No genmodel jar
    exists here, so byte parity with H2O's GamMojoWriter is unpinned; h2omx
    imports GAM MOJOs from these entries alone (tests/test_mojo_more.py)."""
    d = model.design
    cats, nums = _gam_design_columns(model)
    spec = model.gam_spec
    basis = [f"{c}_cr_{i}" for c, sp in spec.items() for i in range(sp["Z"].shape[1])]
    pos = {n: i for i, n in enumerate(d.names)}
    order = _reorder(d.names, d, cats, nums) + [pos[b] for b in basis]
    beta = np.asarray(model.beta, np.float64).reshape(-1, len(d.names) + 1)
    centre, full = [], []
    for k in range(beta.shape[0]):
        bc = [float(beta[k, i]) for i in order] + [float(beta[k, -1])]
        centre += bc
        nb = len(order) - len(basis)
        row, o = bc[:nb], nb
        for c, sp in spec.items():
            kc = sp["Z"].shape[1]
            row += [float(v) for v in np.asarray(sp["Z"]) @ np.asarray(bc[o:o + kc])]
            o += kc
        full += row + [bc[-1]]
    offs = [0]
    for c in cats:
        offs.append(offs[-1] + sum(1 for cc, _ in d.spec if cc == c))
    num_means = [float(d.means[[i for i, (cc, _) in enumerate(d.spec) if cc == c][0]]) for c in nums]
    # NA categorical: each one-hot column takes its training mean (DesignInfo.transform)
    cat_level_means = [float(d.means[i]) for i in _reorder(d.names, d, cats, [])]
    knots =[np.asarray(sp["knots"], np.float64) for sp in spec.values()]
    info.update({
        "use_all_factor_levels": bool(d.use_all_levels), "cats": len(cats), "cat_offsets": offs, "nums": len(nums),
        "mean_imputation": True, "num_means": num_means, "cat_level_means": cat_level_means,
        "beta_center": centre, "beta": full,
        "beta center length per class": len(order) + 1, "beta length per class": len(full) // beta.shape[0],
        "gam_columns": list(spec), "num_knots": [int(k.size) for k in knots], "bs": [0] * len(spec),
        "num_expanded_gam_columns": int(sum(k.size for k in knots)),
        "num_expanded_gam_columns_center": int(sum(k.size - 1 for k in knots)),
        "gam_col_means": [float(sp["mean"]) for sp in spec.values()]})
    files["knots"] = np.concatenate(knots).astype(">f8").tobytes()
    files["binvD"] = np.concatenate([np.asarray(sp["F"], np.float64)[1:-1].ravel() for sp in spec.values()]
                                    ).astype(">f8").tobytes()
    files["zTranspose"] = np.concatenate([np.asarray(sp["Z"], np.float64).T.ravel() for sp in spec.values()]
                                         ).astype(">f8").tobytes()


def export_mojo(model: Model, path: str) -> str:
    import os

    if os.path.isdir(path):
        path = os.path.join(path, model.model_id + ".zip")
    with open(path, "wb") as f:
        f.write(mojo_bytes(model))
    return path


save_model = export_mojo


# ---------------------------------------------------------------------------
# reader / generic model
# ---------------------------------------------------------------------------
def _parse_value(s: str):
    s = s.strip()
    if s in ("true", "false"):
        return s == "true"
    if s == "null":
        return None
    if s.startswith("["):
        inner = s[1:-1].strip()
        if not inner:
            return []
        return [_parse_value(x) for x in inner.split(",")]
    try:
        return int(s)
    except ValueError:
        pass
    try:
        return float(s)
    except ValueError:
        return s


def read_mojo(data: bytes) -> dict:
    z = zipfile.ZipFile(io.BytesIO(data))
    ini = z.read("model.ini").decode().splitlines()
    info, columns, domains = {}, [], {}
    section = None
    for line in ini:
        line = line.strip()
        if not line:
            continue
        if line.startswith("["):
            section = line.strip("[]")
            continue
        if section == "info":
            k, v = line.split("=", 1)
            info[k.strip()] = _parse_value(v)
        elif section == "columns":
            columns.append(line)
        elif section == "domains":
            j, rest = line.split(":", 1)
            n, fname = rest.split()
            domains[int(j)] = z.read(f"domains/{fname}").decode().splitlines()[: int(n)]
    return {"info": info, "columns": columns, "domains": domains, "zip": z}


class GenericModel(Model):
    """A model imported from a MOJO (H2O ``Generic``); scores on the GPU."""

    algo = "generic"
    algo_full_name = "Import MOJO Model"

    def __init__(self, data: bytes, model_id: str | None = None):
        m = read_mojo(data)
        info, cols, doms = m["info"], m["columns"], m["domains"]
        self.raw_mojo = data
        self.info = info
        self.model_id = model_id or str(info.get("h2omx_model_id") or f"Generic_{uuid.uuid4().hex[:8]}")
        self.params = {"mojo_algo": info["algo"]}
        self.mojo_algo = info["algo"]
        sup = bool(info.get("supervised"))
        self.y = cols[-1] if sup and not info.get("autoencoder") else None
        self.x = cols[:-1] if self.y is not None else list(cols)
        cat = info.get("category", "Regression")
        self.category = {"Binomial": ModelCategory.BINOMIAL, "Multinomial": ModelCategory.MULTINOMIAL,
                         "Clustering": ModelCategory.CLUSTERING, "DimReduction": ModelCategory.DIMREDUCTION,
                         "AnomalyDetection": ModelCategory.ANOMALY}.get(cat, ModelCategory.REGRESSION)
        self.response_domain = doms.get(len(cols) - 1) if self.y is not None else None
        self.feature_domains = {c: doms.get(j) for j, c in enumerate(self.x)}
        self.feature_types = {c: (ENUM if doms.get(j) else "real") for j, c in enumerate(self.x)}
        self.training_metrics = {"max_f1_threshold": info.get("default_threshold", 0.5)}
        self.validation_metrics = self.cross_validation_metrics = None
        self.cross_validation_holdout = None
        self.cv_models, self.scoring_history, self.timings = [], [], {}
        self.run_time_ms = 0
        self.comm = None
        z = m["zip"]
        self.cat_encoder = None
        if "h2omx/categorical_encoder.json" in z.namelist():
            # frame-transform categorical_encoding: original columns in, encoded predictors to the trees
            from ..frame.encoding import CategoricalEncoder

            ce = CategoricalEncoder.from_json(json.loads(z.read("h2omx/categorical_encoder.json")))
            self.cat_encoder = ce
            self.x = list(ce.x_out)
            self.feature_types, self.feature_domains = dict(ce.out_types), dict(ce.out_domains)
        if self.mojo_algo in ("gbm", "drf", "xgboost", "isolationforest"):
            self._load_trees(z, info)
        elif self.mojo_algo == "stackedensemble":
            self.base = [GenericModel(z.read(f"models/{info[f'base_model{i}']}.zip"))
                         for i in range(int(info["base_models_num"]))]
            self.meta = GenericModel(z.read(f"models/{info['metalearner']}.zip"))
        elif self.mojo_algo in ARRAY_ALGOS:
            self._load_arrays(z, info)
        elif info.get("h2omx_glm_ext"):
            self._load_glm_ext(z, info)
        if self.mojo_algo == "coxph":
            self.category = ModelCategory.REGRESSION
        if self.mojo_algo == "upliftdrf":
            self.category = "BinomialUplift"

    def _design(self, z, info, tag="design"):
        from ..models.glm import DesignInfo

        x = info[f"h2omx_{tag}_x"]
        x = x if isinstance(x, list) else [x]
        d = DesignInfo(x, self.feature_types, self.feature_domains, bool(info[f"h2omx_{tag}_use_all"]))
        d.means = _get(z, info, f"{tag}_means")
        d.sds = _get(z, info, f"{tag}_sds")
        d.center = _get(z, info, f"{tag}_center")
        return d

    def _load_glm_ext(self, z, info):
        ext = json.loads(z.read("h2omx/glm_ext.json").decode())
        for c, (t, dom) in ext["aug_types"].items():
            self.feature_types[c] = t
            self.feature_domains[c] = dom
        self.ia_spec = [tuple(t) for t in ext["interactions"]]
        self.ordinal_thresholds = ext["ordinal_thresholds"]
        self.design = self._design(z, info)
        self.arr = {"beta": _get(z, info, "beta")}

    def _load_arrays(self, z, info):
        a = self.mojo_algo
        self.arr = {}
        eif_gm = a == "extendedisolationforest" and "h2omx_shape_normals" not in info
        if eif_gm:
            # H2O-written MOJO: numeric predictors in [columns] order, trees/tNN.bin only
            from ..models.glm import DesignInfo

            self.design = DesignInfo(self.x, self.feature_types, self.feature_domains, False)
            self.design.means = np.zeros(len(self.design.names))
            ss = int(info["sample_size"])
            info.setdefault("limit", int(np.ceil(np.log2(max(ss, 2)))))
            cap = (1 << (int(info["limit"]) + 1)) - 1
            trees = [eif_decode_tree(z.read(f"trees/t{t:02d}.bin"), cap) for t in range(int(info["ntrees"]))]
            for j, nm in enumerate(("normals", "offsets", "leaf_sizes")):
                self.arr[nm] = np.stack([t[j] for t in trees])
        elif a in ("pca", "glrm", "coxph", "extendedisolationforest"):
            self.design = self._design(z, info)
        names = {"pca": ("center", "scale", "eigenvectors"), "glrm": ("center", "scale", "archetypes"),
                 "isotonicregression": ("thresholds_x", "thresholds_y"), "coxph": ("coef", "x_mean_num"),
                 "extendedisolationforest": ("normals", "offsets", "leaf_sizes"), "gam": ("beta",)}.get(a, ())
        for nm in names:
            if f"h2omx_shape_{nm}" not in info and (a in ("isotonicregression", "gam") or eif_gm):
                continue   # H2O-written MOJO: genmodel key/values below
            self.arr[nm] = _get(z, info, nm)
        if a == "isotonicregression" and "thresholds_x" not in self.arr:
            tx, ty = info["thresholds_x"], info["thresholds_y"]
            self.arr["thresholds_x"] = np.asarray(tx if isinstance(tx, list) else [tx], np.float64)
            self.arr["thresholds_y"] = np.asarray(ty if isinstance(ty, list) else [ty], np.float64)
        if a == "targetencoder" and "h2omx_shape_prior" not in info:
            # H2O-written MOJO: the genmodel encoding map alone
            stats, prior = _te_from_genmodel(z, info, self.feature_domains)
            self.te_columns = list(stats)
            self.arr["prior"] = prior
            for i, c in enumerate(self.te_columns):
                self.arr[f"te_sums_{i}"], self.arr[f"te_counts_{i}"] = stats[c]
            info.setdefault("blending", bool(info.get("with_blending", False)))
            info.setdefault("inflection_point", 10.0)
            info.setdefault("smoothing", 20.0)
            if prior.size > 1 and self.response_domain:
                info.setdefault("h2omx_classes", list(self.response_domain)[1:])
        elif a == "targetencoder":
            cols = info["te_columns"]
            self.te_columns = cols if isinstance(cols, list) else [cols]
            self.arr["prior"] = _get(z, info, "prior")
            for i in range(len(self.te_columns)):
                self.arr[f"te_sums_{i}"] = _get(z, info, f"te_sums_{i}")
                self.arr[f"te_counts_{i}"] = _get(z, info, f"te_counts_{i}")
        if a == "upliftdrf" and "h2omx_shape_uplift_feat" not in info:
            # genmodel layout only: treatment (class 0) / control (class 1) trees
            self._load_trees(z, dict(info, h2omx_average=True, h2omx_engine_dist="drf"))
            self.uplift_trees = None
        elif a == "upliftdrf":
            sizes = _get(z, info, "uplift_tree_sizes").astype(np.int64)
            cols = {k: _get(z, info, f"uplift_{k}") for k in ("feat", "bin", "na_left", "left", "pt", "pc")}
            self.uplift_trees, o = [], 0
            for sz in sizes:
                t = {k: v[o:o + sz] for k, v in cols.items()}
                self.uplift_trees.append({"feat": t["feat"].astype(np.int32), "bin": t["bin"].astype(np.int32),
                                          "na_left": t["na_left"].astype(np.int8),
                                          "left": t["left"].astype(np.int32), "pt": t["pt"], "pc": t["pc"]})
                o += int(sz)
            self.arr["edges"] = _get(z, info, "uplift_edges").astype(np.float32)
            self.arr["nvb"] = _get(z, info, "uplift_nvb").astype(np.int64)
        if a == "word2vec":
            if "h2omx_shape_vectors" in info:
                self.words = z.read("h2omx/vocabulary.txt").decode().split("\n")[: int(info["vocab_size"])]
                self.vectors = torch.from_numpy(_get(z, info, "vectors").astype(np.float32))
            else:   # H2O-written MOJO: genmodel text "vocabulary" + big-endian blob "vectors"
                nv, vs = int(info["vocab_size"]), int(info["vec_size"])
                self.words = z.read("vocabulary").decode().split("\n")[:nv]
                vec = np.frombuffer(z.read("vectors"), dtype=">f4", count=nv * vs).reshape(nv, vs)
                self.vectors = torch.from_numpy(vec.astype(np.float32))
        if a == "gam" and "h2omx_design_x" not in info:
            # H2O-layout GAM MOJO: splines from the knots / binvD / zTranspose blobs
            def _lst(v):
                return v if isinstance(v, list) else [v]

            gcols, nk = _lst(info["gam_columns"]), [int(k) for k in _lst(info["num_knots"])]
            gm = [float(v) for v in _lst(info.get("gam_col_means", [0.0] * len(gcols)))]
            kn, bd, zt = (np.frombuffer(z.read(n), dtype=">f8").astype(np.float64)
                          for n in ("knots", "binvD", "zTranspose"))
            self.gam_spec, o1, o2, o3 = {}, 0, 0, 0
            for c, k, mean in zip(gcols, nk, gm):
                F = np.zeros((k, k))
                F[1:-1] = bd[o2:o2 + (k - 2) * k].reshape(k - 2, k)
                self.gam_spec[c] = {"knots": kn[o1:o1 + k].copy(), "F": F,
                                    "Z": zt[o3:o3 + (k - 1) * k].reshape(k - 1, k).T.copy(), "mean": mean}
                o1, o2, o3 = o1 + k, o2 + (k - 2) * k, o3 + (k - 1) * k
                self.feature_types[c] = "real"
            self.gam_genmodel = True
        elif a == "gam":
            dx = info["h2omx_design_x"]
            for n in (dx if isinstance(dx, list) else [dx]):
                self.feature_types.setdefault(n, "real")
                self.feature_domains.setdefault(n, None)
            self.design = self._design(z, info)
            gcols = info["gam_columns"]
            gcols = gcols if isinstance(gcols, list) else [gcols]
            self.gam_spec = {c: {"knots": _get(z, info, f"gam_knots_{i}"), "F": _get(z, info, f"gam_F_{i}"),
                                 "Z": _get(z, info, f"gam_Z_{i}"), "mean": info[f"gam_mean_{i}"]}
                             for i, c in enumerate(gcols)}
            for c in gcols:       # raw gam columns are numeric
                self.feature_types[c] = "real"

    # -- h2omx array payload scoring -------------------------------------------
    def _score_arrays(self, frame: Frame) -> torch.Tensor:
        a = self.mojo_algo
        info = self.info
        frame = self.adapt_frame(frame)
        dev = frame.device
        if a in ("pca", "glrm"):
            Xraw = self.design.raw_matrix(frame)
            c = torch.from_numpy(self.arr["center"]).to(dev, torch.float32)[:, None]
            s_ = torch.from_numpy(self.arr["scale"]).to(dev, torch.float32)[:, None]
            if a == "pca":
                m = torch.from_numpy(self.design.means).to(dev, torch.float32)[:, None]
                X = (torch.where(torch.isnan(Xraw), m.expand_as(Xraw), Xraw) - c) / s_
                V = torch.from_numpy(self.arr["eigenvectors"]).to(dev, torch.float32)
                return V.T @ X
            from ..models.glrm import _solve_x

            A = (Xraw - c) / s_
            mask = ~torch.isnan(A)
            A = torch.where(mask, A, torch.zeros_like(A))
            Y = torch.from_numpy(self.arr["archetypes"]).to(dev, torch.float32)
            Xk = _solve_x(A.contiguous(), mask, Y, {"regularization_x": info["regularization_x"],
                                                    "gamma_x": info["gamma_x"]})
            return (Y.T @ Xk) * s_ + c
        if a == "isotonicregression":
            x = frame.vec(self.x[0]).as_float().double()
            tx = torch.from_numpy(self.arr["thresholds_x"]).to(dev)
            ty = torch.from_numpy(self.arr["thresholds_y"]).to(dev)
            if tx.numel() == 1:
                out = ty[0].expand_as(x).clone()
            else:
                i = torch.searchsorted(tx, x).clamp(1, tx.numel() - 1)
                t = ((x - tx[i - 1]) / (tx[i] - tx[i - 1]).clamp_min(1e-300)).clamp(0, 1)
                out = ty[i - 1] + t * (ty[i] - ty[i - 1])
            if str(info["out_of_bounds"]).lower() == "clip":
                out = torch.where(x < tx[0], ty[0], torch.where(x > tx[-1], ty[-1], out))
            else:
                out = torch.where((x < tx[0]) | (x > tx[-1]), torch.full_like(out, float("nan")), out)
            return torch.where(torch.isnan(x), torch.full_like(out, float("nan")), out).float()[None, :]
        if a == "coxph":
            X = self.design.raw_matrix(frame).double()
            mu = torch.from_numpy(self.arr["x_mean_num"]).to(dev)[:, None]
            X = torch.where(torch.isnan(X), mu.expand_as(X), X)
            b = torch.from_numpy(self.arr["coef"]).to(dev)
            return ((X - mu) * b[:, None]).sum(0).float()[None, :]
        if a == "extendedisolationforest":
            from ..models.extended_isolation_forest import ExtendedIsolationForestModel
            from ..models.isolation_forest import avg_path

            m = ExtendedIsolationForestModel.__new__(ExtendedIsolationForestModel)
            m.design, m.limit = self.design, int(info["limit"])
            m.normals = self.arr["normals"].astype(np.float32)
            m.offs = self.arr["offsets"].astype(np.float32)
            m.sizes = self.arr["leaf_sizes"].astype(np.float32)
            ml = m.mean_length(frame)
            cst = float(avg_path(np.array([int(info["sample_size"])]))[0]) or 1.0
            return torch.stack([torch.pow(2.0, -ml / cst), ml])
        if a == "targetencoder":
            return self._te(frame)
        if a == "glm":                              # interactions / ordinal (h2omx_glm_ext)
            from ..models.glm import _torch_linkinv
            from ..models.glm_extras import apply_interactions, ordinal_probs

            fr = apply_interactions(frame, self.ia_spec)
            Xs = self.design.transform(self.design.raw_matrix(fr)).double()
            p = Xs.shape[0]
            beta = torch.from_numpy(self.arr["beta"]).to(dev).view(-1, p + 1)
            if info["family"] == "ordinal":
                th = torch.tensor(self.ordinal_thresholds, dtype=torch.float64, device=dev)
                return ordinal_probs(Xs, beta[0, :p], th).float()
            eta = beta[:, :p] @ Xs + beta[:, p:p + 1]
            if info["family"] == "multinomial":
                return torch.softmax(eta, 0).float()
            mu = _torch_linkinv(eta[0], info["link"], info.get("tweedie_link_power", 0.0))
            if self.category == ModelCategory.BINOMIAL:
                return torch.stack([1 - mu, mu]).float()
            return mu[None, :].float()
        if a == "upliftdrf" and self.uplift_trees is None:
            m = self.ens.raw_margin(self._matrix(frame)).to(dev).float()   # [2][n]: mean p_t, mean p_c
            return torch.stack([m[0] - m[1], m[0], m[1]])
        if a == "upliftdrf":
            from ..models.tree import bin_matrix
            from ..models.uplift import predict_tree

            nbt = int(info["nbt"])
            bm = bin_matrix(frame.feature_matrix(self.x), self.arr["edges"], self.arr["nvb"], nbt)
            n = frame.nrows
            pt = torch.zeros(n, dtype=torch.float64, device=bm.device)
            pc = torch.zeros_like(pt)
            for tr in self.uplift_trees:
                a_, b_ = predict_tree(tr, bm.codes, n, nbt)
                pt += a_
                pc += b_
            k = max(len(self.uplift_trees), 1)
            pt, pc = (pt / k).float(), (pc / k).float()
            return torch.stack([pt - pc, pt, pc]).to(dev)
        if a == "gam" and getattr(self, "gam_genmodel", False):
            from ..models.gam import cr_basis
            from ..models.glm import _torch_linkinv

            nc, nn = int(info["cats"]), int(info["nums"])
            X = self._matrix(frame).double()
            lm = info.get("cat_level_means", [])
            means = (lm if isinstance(lm, list) else [lm]) + list(info.get("num_means") or [])
            parts = [self._expand(X[: nc + nn], bool(info["use_all_factor_levels"]), means=means or None)]
            for j, (c, sp) in enumerate(self.gam_spec.items()):
                x = X[nc + nn + j]
                x = torch.where(torch.isnan(x), torch.full_like(x, sp["mean"]), x)
                parts.append((cr_basis(x, sp["knots"], sp["F"]) @ torch.from_numpy(sp["Z"]).to(dev)).T)
            Zd = torch.cat(parts)
            beta = torch.tensor(info["beta_center"], dtype=torch.float64, device=dev).view(-1, Zd.shape[0] + 1)
            eta = beta[:, :-1] @ Zd + beta[:, -1:]
            if info["family"] == "multinomial":
                return torch.softmax(eta, 0).float()
            mu = _torch_linkinv(eta[0], info["link"], info.get("tweedie_link_power", 0.0))
            if self.category == ModelCategory.BINOMIAL:
                return torch.stack([1 - mu, mu]).float()
            return mu[None, :].float()
        if a == "gam":
            from ..models.gam import _augment

            aug = _augment(frame, self.gam_spec)
            Xs = self.design.transform(self.design.raw_matrix(aug)).double()
            beta = torch.from_numpy(self.arr["beta"]).to(dev)
            beta = beta.view(-1, Xs.shape[0] + 1)
            eta = beta[:, :-1] @ Xs + beta[:, -1:]
            from ..models.glm import _torch_linkinv

            mu = _torch_linkinv(eta[0], info["link"], info.get("tweedie_link_power", 0.0))
            if self.category == ModelCategory.BINOMIAL:
                return torch.stack([1 - mu, mu]).float()
            return mu[None, :].float()
        raise NotImplementedError(a)

    def predict(self, frame: Frame) -> Frame:
        from ..frame.frame import Vec

        a = self.mojo_algo
        if a == "targetencoder":
            P = self._te(self.adapt_frame(frame))
            cls = self.info.get("h2omx_classes")
            names = [f"{c}_te" if not isinstance(cls, list) else f"{c}_{k}_te"
                     for c in self.te_columns for k in (cls if isinstance(cls, list) else [None])]
            return Frame([Vec(n, P[i], "real") for i, n in enumerate(names)])
        if a == "glrm":
            R = self._score_arrays(frame)
            rn = self.info["h2omx_recon_names"]
            rn = rn if isinstance(rn, list) else [rn]
            return Frame([Vec(f"reconstr_{n}", R[j].float(), "real") for j, n in enumerate(rn)])
        if a == "extendedisolationforest":
            P = self._score_arrays(frame)
            return Frame([Vec("anomaly_score", P[0].float(), "real"), Vec("mean_length", P[1].float(), "real")])
        if a == "coxph":
            return Frame([Vec("lp", self._score_arrays(frame)[0], "real")])
        if a == "word2vec":
            raise ValueError("word2vec MOJO: use transform() / find_synonyms()")
        if a == "upliftdrf":
            P = self._score_arrays(frame)
            return Frame([Vec("uplift_predict", P[0], "real"), Vec("p_y1_with_treatment", P[1], "real"),
                          Vec("p_y1_without_treatment", P[2], "real")])
        fr = super().predict(frame)
        beta = self.info.get("calib_glm_beta")
        if self.info.get("calib_method") == "platt" and isinstance(beta, list) and self.response_domain:
            p1 = fr.vec(self.response_domain[1]).data.double()
            c1 = torch.sigmoid(p1 * float(beta[0]) + float(beta[1])).float()
            fr = Frame(list(fr.vecs) + [Vec("cal_p0", 1.0 - c1, "real"), Vec("cal_p1", c1, "real")])
        elif self.info.get("calib_method") == "isotonic" and self.response_domain:
            from ..models.tree_models import _apply_calibration

            z = read_mojo(self.raw_mojo)["zip"]
            p1 = fr.vec(self.response_domain[1]).data.double()
            cal = {"method": "IsotonicRegression", "x": _get(z, self.info, "calib_isotonic_x").tolist(),
                   "y": _get(z, self.info, "calib_isotonic_y").tolist(),
                   "x_min": float(self.info["calib_isotonic_x_min"])}
            c1 = _apply_calibration(cal, p1).float()
            fr = Frame(list(fr.vecs) + [Vec("cal_p0", 1.0 - c1, "real"), Vec("cal_p1", c1, "real")])
        return fr

    def _te(self, frame: Frame) -> torch.Tensor:
        info = self.info
        dev = frame.device
        prior = torch.from_numpy(self.arr["prior"]).to(dev)
        outs = []
        for i, c in enumerate(self.te_columns):
            sums = torch.from_numpy(self.arr[f"te_sums_{i}"]).to(dev)
            cnts = torch.from_numpy(self.arr[f"te_counts_{i}"]).to(dev)
            L = cnts.numel() - 1
            codes = frame.vec(c).data.long()
            idx = torch.where((codes >= 0) & (codes < L), codes, torch.full_like(codes, L))
            mean = torch.where(cnts[:, None] > 0, sums / cnts.clamp_min(1e-300)[:, None], prior[None, :])
            if info["blending"]:
                lam = 1.0 / (1.0 + torch.exp((info["inflection_point"] - cnts) / max(info["smoothing"], 1e-12)))
                mean = lam[:, None] * mean + (1 - lam[:, None]) * prior[None, :]
            enc = mean[idx]
            enc = torch.where((idx == L)[:, None], prior[None, :].expand_as(enc), enc)
            outs.append(enc.T.float())
        return torch.cat(outs) if outs else torch.zeros((0, frame.nrows), device=dev)

    def find_synonyms(self, word: str, count: int = 20) -> dict:
        from ..models.word2vec import Word2VecModel

        return Word2VecModel.find_synonyms(self._w2v(), word, count)

    def transform(self, frame: Frame, aggregate_method: str = "NONE") -> Frame:
        from ..models.word2vec import Word2VecModel

        return Word2VecModel.transform(self._w2v(), frame, aggregate_method)

    def _w2v(self):
        from ..models.word2vec import Word2VecModel

        w = Word2VecModel.__new__(Word2VecModel)
        w.words, w.vectors = self.words, self.vectors
        w.index = {t: i for i, t in enumerate(self.words)}
        return w

    def _load_trees(self, z, info):
        from ..models.tree.boost import TreeEnsemble

        K, nt = int(info["n_trees_per_class"]), int(info["n_trees"])
        dec = [decode_tree_cat(z.read(f"trees/t{k:02d}_{t:03d}.bin")) for t in range(nt) for k in range(K)]
        trees = [d[0] for d in dec]
        cap = max((len(t) for t in trees), default=1)
        from ..models.tree.structs import TREE_NODE_DTYPE

        arr = np.zeros((len(trees), cap), TREE_NODE_DTYPE)
        arr["feat"] = -1
        for i, t in enumerate(trees):
            arr[i, : len(t)] = t
        catbits = None
        if any(d[1] is not None for d in dec):
            catbits = np.zeros((len(trees), cap, 8), np.uint32)
            for i, d in enumerate(dec):
                if d[1] is not None:
                    catbits[i, : len(d[1])] = d[1]
        init = info.get("init_f_per_class")
        init = np.array(init if isinstance(init, list) else [info.get("init_f", 0.0)] * K, np.float64)
        self.ens = TreeEnsemble(arr, K, str(info.get("h2omx_engine_dist", info.get("distribution"))), init,
                                average=bool(info.get("h2omx_average", False)))
        self.ens.catbits = catbits
        self.link = info.get("link_function", "identity")

    # -- scoring ---------------------------------------------------------------
    def _matrix(self, frame: Frame) -> torch.Tensor:
        rows = []
        for c in self.x:
            v = frame.vec(c)
            dom_model = self.feature_domains.get(c)
            if v.vtype == ENUM and dom_model and list(v.domain) != list(dom_model):
                pos = {s: i for i, s in enumerate(dom_model)}
                lut = torch.tensor([pos.get(s, -1) for s in v.domain] + [-1], dtype=torch.float32,
                                   device=v.data.device)
                codes = v.data.long()
                codes = torch.where(codes < 0, torch.full_like(codes, len(v.domain)), codes)
                f = lut[codes]
                rows.append(torch.where(f < 0, torch.full_like(f, float("nan")), f))
            else:
                rows.append(v.as_float())
        return torch.stack(rows) if rows else torch.zeros((0, frame.nrows), device=frame.device)

    def predict_raw(self, frame: Frame) -> torch.Tensor:
        a = self.mojo_algo
        if a in ARRAY_ALGOS or self.info.get("h2omx_glm_ext"):
            return self._score_arrays(frame)
        X = self._matrix(frame)
        if a == "isolationforest":
            L = self.ens.raw_margin(X)[0].to(X.device)
            lo, hi = float(self.info["min_path_length"]), float(self.info["max_path_length"])
            return torch.stack([(hi - L) / max(hi - lo, 1e-12), L])
        if a in ("gbm", "drf", "xgboost"):
            m = self.ens.raw_margin(X).to(X.device)
            oc = self.info.get("offset_column")
            if oc not in (None, "null", ""):
                # H2O GBM with an offset: margin = init_f + offset + trees, link applied after
                if oc not in frame.names:
                    raise ValueError(f"MOJO was trained with offset_column {oc!r}; the scoring frame lacks it")
                m = m + frame.vec(oc).as_float().to(m.device)[None, :]
            P = self._tree_scores(m)
            if self.info.get("balance_classes") and isinstance(self.info.get("prior_class_distrib"), list):
                # balance_classes models: genmodel's correctProbabilities
                from ..models.tree_models import correct_probabilities

                P = correct_probabilities(P, self.info["prior_class_distrib"], self.info["model_class_distrib"])
            return P
        if a == "glm":
            return self._glm(X)
        if a == "kmeans":
            return self._kmeans(X)
        if a == "deeplearning":
            return self._dl(X)
        if a == "stackedensemble":
            return self._se(frame)
        raise NotImplementedError(a)

    def _tree_scores(self, m: torch.Tensor) -> torch.Tensor:
        if self.mojo_algo == "drf" or self.link == "identity":
            if self.category == ModelCategory.BINOMIAL:
                p1 = m[0].clamp(0, 1)
                return torch.stack([1 - p1, p1])
            if self.category == ModelCategory.MULTINOMIAL:
                mm = m.clamp_min(0)
                return mm / mm.sum(0, keepdim=True).clamp_min(1e-30)
            return m
        if self.link == "logit":
            p1 = torch.sigmoid(m[0])
            return torch.stack([1 - p1, p1])
        if self.link == "multinomial":
            return torch.softmax(m, 0)
        if self.link == "log":
            return torch.exp(m)
        return m

    def _expand(self, X, use_all, means=None, center=None, mult=None):
        """One-hot categoricals (the first ``cats`` columns) + numerics in MOJO
        column order; NAs / unseen levels imputed with the training means."""
        ncat = int(self.info.get("cats", 0))
        parts = []
        for j in range(ncat):
            L = max(len(self.feature_domains[self.x[j]] or []), 1)
            codes = X[j]
            na = torch.isnan(codes)
            ci = torch.where(na, torch.zeros_like(codes), codes).long().clamp(0, L - 1)
            oh = torch.nn.functional.one_hot(ci, L).T.to(X.dtype)
            oh = torch.where(na[None, :], torch.full_like(oh, float("nan")), oh)
            parts.append(oh if use_all else oh[1:])
        parts.append(X[ncat:])
        Z = torch.cat(parts)
        if means is not None:
            mv = torch.tensor(means, dtype=X.dtype, device=X.device)[:, None]
            Z = torch.where(torch.isnan(Z), mv.expand_as(Z), Z)
        if center is not None:
            c = torch.tensor(center, dtype=X.dtype, device=X.device)[:, None]
            m = torch.tensor(mult, dtype=X.dtype, device=X.device)[:, None]
            Z = (Z - c) * m
        return Z

    def _glm(self, X):
        info = self.info
        X = X.double()
        Z = self._expand(X, bool(info["use_all_factor_levels"]), means=info["h2omx_means"])
        beta = torch.tensor(info["beta"], dtype=torch.float64, device=X.device)
        p = Z.shape[0]
        K = beta.numel() // (p + 1)
        B = beta.view(K, p + 1)
        eta = B[:, :p] @ Z + B[:, p:]
        fam, link = info["family"], info["link"]
        if fam == "multinomial":
            return torch.softmax(eta, 0).float()
        from ..models.glm import _torch_linkinv

        mu = _torch_linkinv(eta[0], link, info.get("tweedie_link_power", 0.0))
        if self.category == ModelCategory.BINOMIAL:
            return torch.stack([1 - mu, mu]).float()
        return mu[None, :].float()

    def _kmeans(self, X):
        info = self.info
        Z = self._expand(X.double(), True, means=info["means"], center=info["center_mean"], mult=info["center_mult"])
        C = torch.tensor([info[f"center_{i}"] for i in range(int(info["center_num"]))], dtype=torch.float64,
                         device=X.device)
        d2 = (Z.pow(2).sum(0)[None, :] - 2 * C @ Z + C.pow(2).sum(1)[:, None])
        return d2.argmin(0).float()[None, :]

    def _dl(self, X):
        info = self.info
        Z = self._expand(X.float(), bool(info["use_all_factor_levels"]), means=info["means"],
                         center=info["norm_sub"], mult=info["norm_mul"])
        H = Z.T.contiguous()
        sizes = info["neural_network_sizes"]
        act = int(info.get("h2omx_act", 1))
        L = len(sizes) - 1
        for i in range(L):
            W = torch.tensor(info[f"weight_layer{i}"], dtype=torch.float32, device=X.device).view(
                *info[f"weight_shape{i}"])
            b = torch.tensor(info[f"bias_layer{i}"], dtype=torch.float32, device=X.device)
            H = H @ W.T + b
            if i < L - 1:
                if act == 1:
                    H = torch.relu(H)
                elif act == 2:
                    H = torch.tanh(H)
                elif act == 3:
                    H = H.view(H.shape[0], -1, 2).max(-1).values
                elif act == 4:
                    H = torch.nn.functional.elu(H)
        if info.get("autoencoder"):
            return H.T.contiguous()
        if self.category in (ModelCategory.BINOMIAL, ModelCategory.MULTINOMIAL):
            return torch.softmax(H, 1).T.contiguous()
        return (H[:, 0] / info["norm_resp_mul"] + info["norm_resp_sub"])[None, :]

    def _se(self, frame):
        from ..models.ensemble import level_one_frame

        lvl1 = level_one_frame(self.base, frame, self.category)
        return self.meta.predict_raw(lvl1)


def import_mojo(path: str, model_id: str | None = None) -> GenericModel:
    from ..frame.frame import DKV

    with open(path, "rb") as f:
        m = GenericModel(f.read(), model_id)
    DKV.put(m.model_id, m)
    return m


def load_model(path: str) -> GenericModel:
    return import_mojo(path)
