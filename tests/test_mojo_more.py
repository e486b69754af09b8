"""MOJO round trips (export -> import as Generic -> identical scores) for the
newer estimators (h2omx array payload)."""
import numpy as np
import pandas as pd
import pytest

from h2omx.frame import Frame
from h2omx.models import (H2OCoxProportionalHazardsEstimator, H2OExtendedIsolationForestEstimator,
                          H2OGeneralizedAdditiveEstimator, H2OGeneralizedLowRankEstimator,
                          H2OIsotonicRegressionEstimator, H2OPrincipalComponentAnalysisEstimator,
                          H2OTargetEncoderEstimator, H2OWord2vecEstimator)
from h2omx.mojo import import_mojo


def _df(n=800, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(n, 4))
    df = pd.DataFrame(X, columns=list("abcd"))
    df["g"] = pd.Categorical(rng.choice(list("pqr"), n))
    df["y"] = np.sin(X[:, 0]) + X[:, 1] + 0.1 * rng.normal(size=n)
    df["yb"] = pd.Categorical(np.where(df.y > 0, "t", "f"))
    df["t"] = np.ceil(rng.exponential(np.exp(-0.5 * X[:, 0])) * 10) / 10
    df["ev"] = (rng.random(n) < 0.7).astype(float)
    df.loc[::17, "c"] = np.nan
    return df


def _roundtrip(model, tmp_path):
    path = model.download_mojo(str(tmp_path))
    return import_mojo(path)


def _same(a: Frame, b: Frame, rtol=1e-5, atol=1e-6):
    pa, pb = a.to_pandas(), b.to_pandas()
    assert list(pa.columns) == list(pb.columns)
    np.testing.assert_allclose(pa.to_numpy(dtype=float), pb.to_numpy(dtype=float), rtol=rtol, atol=atol)


@pytest.mark.parametrize("kind", ["pca", "glrm", "isotonic", "coxph", "te", "eif", "gam"])
def test_mojo_roundtrip(kind, tmp_path):
    df = _df()
    fr = Frame.from_pandas(df)
    if kind == "pca":
        m = H2OPrincipalComponentAnalysisEstimator(k=2, transform="STANDARDIZE").train(x=list("abcdg"), training_frame=fr)
    elif kind == "glrm":
        m = H2OGeneralizedLowRankEstimator(k=2, init="SVD", max_iterations=20).train(x=list("abcd"), training_frame=fr)
    elif kind == "isotonic":
        m = H2OIsotonicRegressionEstimator(out_of_bounds="clip").train(x=["a"], y="y", training_frame=fr)
    elif kind == "coxph":
        m = H2OCoxProportionalHazardsEstimator(stop_column="t").train(x=["a", "b", "g"], y="ev", training_frame=fr)
    elif kind == "te":
        m = H2OTargetEncoderEstimator(noise=0.0, blending=True).train(x=["g"], y="yb", training_frame=fr)
    elif kind == "eif":
        m = H2OExtendedIsolationForestEstimator(ntrees=10, extension_level=1, seed=1).train(x=list("abc"),
                                                                                         training_frame=fr)
    else:
        m = H2OGeneralizedAdditiveEstimator(family="gaussian", gam_columns=["a"], num_knots=[6], lambda_=0.0).train(
            x=["a", "b"], y="y", training_frame=fr)
    g = _roundtrip(m, tmp_path)
    if kind == "te":
        got = g.predict(fr)
        exp = m.transform(fr)
        np.testing.assert_allclose(got.to_pandas()["g_te"], exp.to_pandas()["g_te"], rtol=1e-6)
        return
    _same(m.predict(fr), g.predict(fr), rtol=1e-4, atol=1e-5)


def test_word2vec_mojo(tmp_path):
    rng = np.random.default_rng(0)
    toks = []
    for _ in range(500):
        toks += list(rng.choice([f"w{i}" for i in range(10)], size=5)) + [None]
    fr = Frame.from_pandas(pd.DataFrame({"w": toks}))
    m = H2OWord2vecEstimator(vec_size=8, epochs=1, min_word_freq=1, seed=1).train(training_frame=fr)
    g = _roundtrip(m, tmp_path)
    assert g.find_synonyms("w1", 3) == m.find_synonyms("w1", 3)
    _same(m.transform(fr, "AVERAGE"), g.transform(fr, "AVERAGE"))


def test_uplift_mojo(tmp_path):
    from h2omx.models import H2OUpliftRandomForestEstimator

    rng = np.random.default_rng(2)
    n = 3000
    X = rng.normal(size=(n, 3))
    trt = rng.random(n) < 0.5
    p = np.clip(0.3 + 0.1 * X[:, 1] + trt * np.where(X[:, 0] > 0, 0.3, -0.1), 0.02, 0.98)
    df = pd.DataFrame(X, columns=list("abc"))
    df.loc[::13, "b"] = np.nan
    df["trt"] = pd.Categorical(np.where(trt, "treatment", "control"), categories=["control", "treatment"])
    df["y"] = pd.Categorical(np.where(rng.random(n) < p, "1", "0"), categories=["0", "1"])
    fr = Frame.from_pandas(df)
    m = H2OUpliftRandomForestEstimator(ntrees=4, max_depth=4, treatment_column="trt", seed=1).train(
        x=list("abc"), y="y", training_frame=fr)
    g = _roundtrip(m, tmp_path)
    assert g.category == "BinomialUplift"
    _same(g.predict(fr), m.predict(fr))


@pytest.mark.parametrize("kind", ["interactions", "ordinal"])
def test_glm_ext_mojo(kind, tmp_path):
    from h2omx.models import H2OGeneralizedLinearEstimator

    rng = np.random.default_rng(5)
    n = 1500
    df = pd.DataFrame(rng.normal(size=(n, 2)), columns=["a", "b"])
    df["g"] = pd.Categorical(rng.choice(["p", "q", "r"], n))
    if kind == "interactions":
        df["y"] = 1 + df.a * df.b + np.where(df.g == "q", 1.0, -1.0) * df.b + 0.1 * rng.normal(size=n)
        m = H2OGeneralizedLinearEstimator(lambda_=0.0, interaction_pairs=[("a", "b"), ("g", "b")]).train(
            x=["a", "b", "g"], y="y", training_frame=Frame.from_pandas(df))
    else:
        eta = df.a - 0.5 * df.b
        df["y"] = pd.Categorical(np.digitize(eta + rng.logistic(size=n), [-1, 1]).astype(str))
        m = H2OGeneralizedLinearEstimator(family="ordinal", lambda_=0.0).train(x=["a", "b", "g"], y="y",
                                                                               training_frame=Frame.from_pandas(df))
    fr = Frame.from_pandas(df)
    g = _roundtrip(m, tmp_path)
    np.testing.assert_allclose(g.predict_raw(fr).numpy(), m.predict_raw(fr).numpy(), rtol=1e-4, atol=1e-5)


def _genmodel_only(path, out):
    """Copy of a MOJO without h2omx's own payload (h2omx/* entries, h2omx_* keys):
    what an H2O-written MOJO of the same model would hold."""
    import zipfile

    with zipfile.ZipFile(path) as zi, zipfile.ZipFile(out, "w") as zo:
        for n in zi.namelist():
            if n.startswith("h2omx/"):
                continue
            data = zi.read(n)
            if n == "model.ini":
                data = "\n".join(ln for ln in data.decode().split("\n") if not ln.startswith("h2omx_")).encode()
            zo.writestr(n, data)
    return out


def test_genmodel_entries_import_without_h2omx_payload(tmp_path):
    """isotonic regression and word2vec MOJOs carry genmodel's entries
    (thresholds_x/_y key/values; text vocabulary + big-endian vectors blob) and
    import from those alone; PCA's eigenvectors_raw / normalisation match."""
    import zipfile

    df = _df()
    fr = Frame.from_pandas(df)
    m = H2OIsotonicRegressionEstimator(out_of_bounds="clip").train(x=["a"], y="y", training_frame=fr)
    g = import_mojo(_genmodel_only(m.download_mojo(str(tmp_path)), str(tmp_path / "iso_gm.zip")))
    _same(m.predict(fr), g.predict(fr), rtol=1e-6, atol=1e-7)

    rng = np.random.default_rng(0)
    toks = []
    for _ in range(300):
        toks += list(rng.choice([f"w{i}" for i in range(10)], size=5)) + [None]
    wf = Frame.from_pandas(pd.DataFrame({"w": toks}))
    w2v = H2OWord2vecEstimator(vec_size=8, epochs=1, min_word_freq=1, seed=1).train(training_frame=wf)
    g = import_mojo(_genmodel_only(w2v.download_mojo(str(tmp_path)), str(tmp_path / "w2v_gm.zip")))
    _same(w2v.transform(wf, "AVERAGE"), g.transform(wf, "AVERAGE"))

    pca = H2OPrincipalComponentAnalysisEstimator(k=2, transform="STANDARDIZE").train(x=list("abcd"), training_frame=fr)
    with zipfile.ZipFile(pca.download_mojo(str(tmp_path))) as z:
        ini = z.read("model.ini").decode()
        raw = np.frombuffer(z.read("eigenvectors_raw"), dtype=">f8")
    kv = dict(ln.split(" = ", 1) for ln in ini.split("\n") if " = " in ln)
    assert int(kv["k"]) == 2 and int(kv["eigenvector_size"]) == pca.eigenvectors.shape[0]
    np.testing.assert_array_equal(raw.reshape(pca.eigenvectors.shape), pca.eigenvectors)
    norm_mul = np.array([float(v) for v in kv["normMul"].strip("[]").split(",")])
    np.testing.assert_allclose(norm_mul, 1.0 / pca.scale, rtol=1e-12)


@pytest.mark.parametrize("resp", ["yb", "y", "ym"])
def test_target_encoder_genmodel_entries(resp, tmp_path):
    """TargetEncoder MOJOs carry genmodel's encoding map (``[col]`` sections of
    ``level = numerator denominator [class]``), NA-presence and column maps,
    and import from those alone (binomial, regression, multinomial)."""
    import zipfile

    df = _df()
    rng = np.random.default_rng(4)
    df["ym"] = pd.Categorical(rng.choice(["u", "v", "w"], len(df)))
    df.loc[::11, "g"] = np.nan
    fr = Frame.from_pandas(df)
    m = H2OTargetEncoderEstimator(noise=0.0, blending=True).train(x=["g"], y=resp, training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    with zipfile.ZipFile(path) as z:
        enc = z.read("feature_engineering/target_encoding/encoding_map.ini").decode().split("\n")
        na = z.read("feature_engineering/target_encoding/te_column_name_to_missing_values_presence.ini").decode()
    assert enc[0] == "[g]" and na.strip() == "g = 1"
    sums, cnts, _ = m.stats["g"]
    lv, rest = enc[1].split(" = ")
    assert int(lv) == 0 and float(rest.split()[1]) == float(cnts[0])
    g = import_mojo(_genmodel_only(path, str(tmp_path / "te_gm.zip")))
    got, exp = g.predict(fr).to_pandas(), m.transform(fr).to_pandas()
    te_cols = [c for c in got.columns if c.endswith("_te")]
    assert te_cols and all(c in exp.columns for c in te_cols)
    np.testing.assert_allclose(got[te_cols].to_numpy(float), exp[te_cols].to_numpy(float), rtol=1e-9, atol=1e-12)


def test_glrm_genmodel_entries(tmp_path):
    """GLRM MOJOs carry GlrmMojoReader's dimensions, DataInfo layout, losses
    text and the big-endian archetypes blob."""
    import zipfile

    fr = Frame.from_pandas(_df())
    m = H2OGeneralizedLowRankEstimator(k=2, init="SVD", max_iterations=20).train(x=list("abcdg"), training_frame=fr)
    with zipfile.ZipFile(m.download_mojo(str(tmp_path))) as z:
        ini = z.read("model.ini").decode()
        Y = np.frombuffer(z.read("archetypes"), dtype=">f8")
        losses = z.read("losses").decode().split()
    kv = dict(ln.split(" = ", 1) for ln in ini.split("\n") if " = " in ln)
    assert (int(kv["nrowY"]), int(kv["ncolY"])) == m.Y.shape and int(kv["ncolA"]) == 5
    np.testing.assert_array_equal(Y.reshape(m.Y.shape), m.Y)
    assert int(kv["num_categories"]) == 1 and kv["cat_offsets"] == f"[0, {m.Y.shape[1] - 4}]"
    assert losses == ["Categorical"] + ["Quadratic"] * 4


def test_eif_genmodel_trees(tmp_path):
    """Extended isolation forest MOJOs carry one genmodel tree blob per tree
    (trees/tNN.bin: node number, 'N' normal + intercept point / 'L' row count)
    and score identically when imported from those blobs alone."""
    df = _df()
    fr = Frame.from_pandas(df[list("abd")])
    m = H2OExtendedIsolationForestEstimator(ntrees=8, extension_level=2, seed=3).train(training_frame=fr)
    g = import_mojo(_genmodel_only(m.download_mojo(str(tmp_path)), str(tmp_path / "eif_gm.zip")))
    assert "h2omx_shape_normals" not in g.info
    _same(m.predict(fr), g.predict(fr), rtol=1e-5, atol=1e-6)


def test_uplift_genmodel_trees(tmp_path):
    """Uplift DRF MOJOs carry the forest in genmodel's SharedTree layout
    (trees/t00_* treatment, trees/t01_* control leaf predictions, threshold
    splits) and score identically when imported from those trees alone."""
    from h2omx.models import H2OUpliftRandomForestEstimator

    rng = np.random.default_rng(5)
    n = 2500
    X = rng.normal(size=(n, 3))
    trt = rng.random(n) < 0.5
    p = np.clip(0.3 + 0.1 * X[:, 1] + trt * np.where(X[:, 0] > 0, 0.3, -0.1), 0.02, 0.98)
    df = pd.DataFrame(X, columns=list("abc"))
    df.loc[::11, "a"] = np.nan
    df["trt"] = pd.Categorical(np.where(trt, "treatment", "control"), categories=["control", "treatment"])
    df["y"] = pd.Categorical(np.where(rng.random(n) < p, "1", "0"), categories=["0", "1"])
    fr = Frame.from_pandas(df)
    m = H2OUpliftRandomForestEstimator(ntrees=5, max_depth=4, treatment_column="trt", seed=2).train(
        x=list("abc"), y="y", training_frame=fr)
    g = import_mojo(_genmodel_only(m.download_mojo(str(tmp_path)), str(tmp_path / "uplift_gm.zip")))
    assert "h2omx_shape_uplift_feat" not in g.info and int(g.info["n_trees_per_class"]) == 2
    _same(g.predict(fr), m.predict(fr), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("family", ["gaussian", "binomial"])
def test_gam_genmodel_entries(family, tmp_path):
    """GAM MOJOs carry GamMojoReader-style entries (cats / nums / NA fills,
    centred and un-centred coefficients, gam_columns / num_knots / bs and the
    big-endian knots / binvD / zTranspose blobs) and score identically when
    imported from those alone (categorical + NA predictors, two gam columns)."""
    import zipfile

    df = _df()
    df.loc[::13, "g"] = np.nan
    df.loc[::7, "a"] = np.nan
    fr = Frame.from_pandas(df)
    y = "y" if family == "gaussian" else "yb"
    m = H2OGeneralizedAdditiveEstimator(family=family, gam_columns=["a", "c"], num_knots=[6, 5], lambda_=0.0).train(
        x=["a", "b", "c", "g"], y=y, training_frame=fr)
    path = m.download_mojo(str(tmp_path))
    with zipfile.ZipFile(path) as z:
        ini = z.read("model.ini").decode()
        knots = np.frombuffer(z.read("knots"), dtype=">f8")
        zt = np.frombuffer(z.read("zTranspose"), dtype=">f8")
    kv = dict(ln.split(" = ", 1) for ln in ini.split("\n") if " = " in ln)
    assert kv["num_knots"] == "[6, 5]" and int(kv["cats"]) == 1 and int(kv["nums"]) == 1
    np.testing.assert_array_equal(knots[:6], m.gam_spec["a"]["knots"])
    np.testing.assert_array_equal(zt[:30].reshape(5, 6), m.gam_spec["a"]["Z"].T)
    g = import_mojo(_genmodel_only(path, str(tmp_path / "gam_gm.zip")))
    assert getattr(g, "gam_genmodel", False)
    np.testing.assert_allclose(g.predict_raw(fr).numpy(), m.predict_raw(fr).numpy(), rtol=1e-4, atol=1e-5)
